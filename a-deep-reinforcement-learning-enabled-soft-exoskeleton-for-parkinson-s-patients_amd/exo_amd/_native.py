"""ctypes binding of libexo_amd.so (include/exo_amd.h).

The library is the MI355X product path.  It is loaded AFTER torch so that it
binds to the HIP runtime torch already loaded (both carry the SONAME
libamdhip64.so.7), which makes torch streams and device pointers valid in it.
There is no CPU fallback: if the library is missing or no GPU is present the
env/replay classes raise.
"""
import ctypes
import os
import subprocess

import torch  # noqa: F401  (must be imported before the HIP library is loaded)

HERE = os.path.dirname(os.path.abspath(__file__))
PKG_ROOT = os.path.dirname(HERE)
LIB_PATH = os.path.join(HERE, "_lib", os.environ.get("EXO_AMD_LIB", "libexo_amd.so"))
CSRC = os.path.join(PKG_ROOT, "csrc")

EXO_OK = 0
ERRORS = {-22: "EINVAL", -12: "ENOMEM", -5: "EDEVICE", -34: "ERANGE"}

c_int32, c_double, c_void_p, c_uint64 = ctypes.c_int32, ctypes.c_double, ctypes.c_void_p, ctypes.c_uint64
c_long = ctypes.c_long
P = ctypes.POINTER


class LapTreeDesc(ctypes.Structure):
    _fields_ = [("tree", c_void_p), ("max_priority", c_void_p), ("n_strata", c_int32), ("capacity", c_int32),
                ("cap", c_int32)]


class LapStorageDesc(ctypes.Structure):
    _fields_ = [("state", c_void_p), ("action", c_void_p), ("next_state", c_void_p), ("reward", c_void_p),
                ("not_done", c_void_p), ("state_dim", c_int32), ("action_dim", c_int32), ("ptr", c_void_p),
                ("size", c_void_p)]


class ExoEnvConfig(ctypes.Structure):
    """exo_env_config: the constructor arguments of ExoskeletonEnv_train
    (Environment/Exoskeleton_env.py:38-48)."""
    _fields_ = [("motion", c_int32), ("tremor_sequence", c_int32 * 7),
                ("tremor_amplitude_range", c_double * 2), ("first_harmonics_interval", c_double * 2),
                ("second_harmonics_interval", c_double * 2), ("max_force_shoulder", c_double),
                ("max_force_elbow", c_double), ("dr_actuator_end_pos_shift", c_double),
                ("dr_actuator_range", c_double), ("matrix_noise_fraction", c_double)]


class ExoMbParams(ctypes.Structure):
    """exo_mb_params: constants of the multibody stepSimulation (include/exo_amd.h)."""
    _fields_ = [(n, c_double) for n in ("gravity", "kp", "kd", "motor_impulse", "passive_impulse", "limit_impulse",
                                        "erp", "lin_damp", "ang_damp", "max_vel")] + [("iters", c_int32)]


class TD7FLin(ctypes.Structure):
    """td7f_lin (include/exo_amd.h)."""
    _fields_ = [("wf", c_void_p), ("wb", c_void_p), ("b", c_void_p), ("n_out", c_int32), ("n_in", c_int32),
                ("ksf", c_int32), ("ksb", c_int32), ("w", c_void_p), ("ldw", ctypes.c_int64)]


class TD7FPackJob(ctypes.Structure):
    """td7f_pack_job (include/exo_amd.h)."""
    _fields_ = [("w", c_void_p), ("ld", ctypes.c_int64), ("n_out", c_int32), ("n_in", c_int32), ("wf", c_void_p),
                ("wb", c_void_p), ("ksf", c_int32), ("ntf", c_int32), ("ksb", c_int32), ("ntb", c_int32)]


class TD7FNoise(ctypes.Structure):
    """td7f_noise (include/exo_amd.h)."""
    _fields_ = [("seed", c_uint64), ("tag", ctypes.c_uint32), ("pad0", ctypes.c_uint32), ("counter", c_void_p),
                ("ticket", c_void_p), ("sigma", c_void_p), ("sigma_dec", ctypes.c_float), ("clip", ctypes.c_float),
                ("scale", ctypes.c_float), ("pad1", c_int32), ("z", c_void_p),
                ("dec_count", c_void_p)]


class TD7FXT(ctypes.Structure):
    """td7f_xt (include/exo_amd.h)."""
    _fields_ = [("x", c_void_p), ("dp", c_void_p), ("part", c_void_p)]


class TD7FActorBufs(ctypes.Structure):
    """td7f_actor_bufs (include/exo_amd.h)."""
    _fields_ = [("act_out", c_void_p), ("zsa_out", c_void_p), ("h0", c_void_p), ("mean0", c_void_p),
                ("ya", c_void_p * 2), ("yz", c_void_p * 2), ("yc", c_void_p * 2), ("da", c_void_p),
                ("dzsa", c_void_p)]


class TD7FWgJob(ctypes.Structure):
    """td7f_wg_job (include/exo_amd.h)."""
    _fields_ = [("dp", c_void_p), ("x", c_void_p), ("part", c_void_p), ("dw", c_void_p), ("db", c_void_p),
                ("n", c_int32), ("k", c_int32), ("row_tiles", c_int32)]


class TD7FWgAdam(ctypes.Structure):
    """td7f_wg_adam (include/exo_amd.h)."""
    _fields_ = [("opt", c_int32), ("w_off", ctypes.c_int64), ("b_off", ctypes.c_int64), ("wf", c_void_p),
                ("wb", c_void_p), ("ksf", c_int32), ("ksb", c_int32)]


EXPORTS = {
    "exo_create": (c_int32, [P(ExoEnvConfig), c_int32, P(c_double), P(c_int32), c_int32, c_int32, c_uint64, c_int32,
                             P(c_void_p)]),
    "exo_reset": (c_int32, [c_void_p, c_void_p, c_void_p, c_void_p]),
    "exo_reset_from_draws": (c_int32, [c_void_p, P(c_int32), c_int32, P(c_double), c_void_p, c_void_p]),
    "exo_step": (c_int32, [c_void_p] * 8),
    "exo_num_envs": (c_int32, [c_void_p]),
    "exo_episode_length": (c_int32, [c_void_p, c_int32, P(c_int32)]),
    "exo_tremor_host": (c_int32, [c_void_p, c_int32, P(c_double)]),
    "exo_original_joint_angles_host": (c_int32, [c_void_p, c_int32, P(c_double)]),
    "exo_episode_host": (c_int32, [c_void_p, c_int32, P(c_double), P(c_double), P(c_double), P(c_double),
                                   P(c_double)]),
    "exo_get_state_host": (c_int32, [c_void_p, c_int32, P(c_double)]),
    "exo_set_state_host": (c_int32, [c_void_p, c_int32, P(c_double)]),
    "exo_set_seed": (c_int32, [c_void_p, c_uint64]),
    "exo_set_step_variant": (c_int32, [c_void_p, c_int32]),
    "exo_set_step_budget": (c_int32, [c_void_p, c_int32]),
    "exo_step_carry": (c_int32, [c_void_p] * 9),
    "exo_budget_advance": (c_int32, [c_void_p] * 6),
    "exo_episode_advance": (c_int32, [c_void_p] * 7),
    "exo_multibody_default_params": (None, [P(ExoMbParams)]),
    "exo_set_physics": (c_int32, [c_void_p, c_int32, P(ExoMbParams)]),
    "exo_multibody_advance": (c_int32, [c_void_p, c_void_p, c_void_p, c_void_p]),
    "exo_get_multibody_state_host": (c_int32, [c_void_p, c_int32, P(c_double), P(c_double)]),
    "exo_set_multibody_state_host": (c_int32, [c_void_p, c_int32, P(c_double), P(c_double)]),
    "exo_last_error": (ctypes.c_char_p, [c_void_p]),
    "exo_destroy": (None, [c_void_p]),
    "exo_tremor_metrics": (c_int32, [c_void_p, c_void_p, c_void_p, c_double, c_double, c_double, c_int32, c_void_p,
                                     c_void_p, c_void_p]),
    "exo_set_tremor_model": (c_int32, [c_void_p, c_void_p, c_int32]),
    "exo_set_step_clock": (c_int32, [c_void_p, c_void_p, c_void_p]),
    "exo_active_advance": (c_int32, [c_void_p, c_int32, c_int32, c_void_p, c_void_p, c_void_p, c_void_p]),
    "exo_active_advance_score": (c_int32, [c_void_p, c_int32, c_int32, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                                           c_void_p]),
    "exo_eval_metrics": (c_int32, [c_void_p, c_void_p, c_void_p, c_double, c_double, c_void_p, c_void_p]),
    "lap_tree_floats": (c_int32, [c_int32, c_int32]),
    "lap_init": (c_int32, [c_void_p, c_void_p]),
    "lap_add": (c_int32, [c_void_p, c_void_p, c_void_p, c_int32, c_void_p]),
    "lap_sample": (c_int32, [c_void_p, c_void_p, c_void_p, c_int32, c_void_p, c_void_p]),
    "lap_update": (c_int32, [c_void_p, c_void_p, c_void_p, c_int32, c_void_p]),
    "lap_reset_max": (c_int32, [c_void_p, c_void_p]),
    "lap_totals": (c_int32, [c_void_p, c_void_p, c_void_p]),
    "exo_stream_ballast": (c_int32, [c_int32]),
    "td7_dense_set_xl": (c_int32, [c_int32]),
    "exo_graph_branch_bound": (c_int32, [c_void_p, c_void_p]),
    "lap_store_batch": (c_int32, [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                                  c_void_p, ctypes.c_float, c_int32, c_void_p, c_void_p]),
    "lap_store_batch_ref": (c_int32, [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                                      c_void_p, c_void_p, c_void_p, ctypes.c_float, c_int32, c_void_p, c_void_p]),
    "lap_store_batch_ref_fused": (c_int32, [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                                            c_void_p, c_void_p, c_void_p, ctypes.c_float, c_int32, c_void_p,
                                            c_void_p]),
    "lap_store_batch_ref_fused_adv": (c_int32, [c_void_p] * 10 + [ctypes.c_float, c_int32, c_void_p, c_void_p,
                                                                 c_int32, c_void_p, c_void_p, c_void_p, c_void_p]),
    "lap_ref_plan": (c_int32, [c_void_p, c_void_p, c_void_p, c_int32, c_int32, c_void_p, c_void_p, ctypes.c_int64,
                               c_void_p, c_void_p, c_void_p]),
    "lap_ref_step": (c_int32, [c_void_p, c_void_p, c_void_p, c_int32, c_int32, c_void_p, c_int32, c_void_p, c_void_p]
                     + [c_void_p] * 5 + [ctypes.c_float, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p]),
    "lap_ref_commit": (c_int32, [c_void_p, c_void_p, c_void_p, c_void_p, c_int32, c_int32, c_void_p, ctypes.c_int64,
                                 c_void_p]),
    "lap_update_sample_rng": (c_int32, [c_void_p, c_void_p, c_void_p, c_void_p, c_int32, ctypes.c_uint64,
                                        ctypes.c_uint32, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                                        c_void_p, c_void_p, c_void_p]),
    "lap_update_sample_idx": (c_int32, [c_void_p, c_void_p, c_void_p, c_void_p, c_int32, ctypes.c_uint64,
                                        ctypes.c_uint32, c_void_p, c_void_p, c_void_p, c_void_p]),
    "lap_gather_rows": (c_int32, [c_void_p, c_void_p, c_int32, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                                  c_void_p, c_void_p]),
    "lap_update_sample_td": (c_int32, [c_void_p, c_void_p, c_void_p, c_void_p, ctypes.c_float, ctypes.c_float,
                                       c_void_p, c_int32, ctypes.c_uint64, ctypes.c_uint32, c_void_p, c_void_p,
                                       c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p]),
    "lap_sample_gather_rng": (c_int32, [c_void_p, c_void_p, ctypes.c_uint64, ctypes.c_uint32, c_void_p, c_void_p,
                                        c_int32, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                                        c_void_p]),
    "lap_sample_gather": (c_int32, [c_void_p, c_void_p, c_void_p, c_int32, c_void_p, c_void_p, c_void_p, c_void_p,
                                    c_void_p, c_void_p, c_void_p]),
    "td7_adam_step": (c_int32, [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, ctypes.c_int64,
                                ctypes.c_float, ctypes.c_float, ctypes.c_float, ctypes.c_float, ctypes.c_float,
                                ctypes.c_float, c_void_p]),
    "td7_q_target": (c_int32, [c_void_p, c_long, c_long, c_void_p, c_void_p, ctypes.c_float, c_void_p, c_void_p,
                               c_void_p, c_void_p, c_void_p, c_int32, c_void_p]),
    "td7_critic_loss": (c_int32, [c_void_p, c_long, c_long, c_void_p, c_void_p, c_void_p, c_void_p, ctypes.c_float,
                                  ctypes.c_float, c_int32, c_void_p]),
    "td7_critic_loss_strided": (c_int32, [c_void_p, c_long, c_long, c_void_p, c_void_p, c_void_p, c_void_p, c_long,
                                          c_long, ctypes.c_float, ctypes.c_float, c_int32, c_void_p]),
    "td7_noisy_action": (c_int32, [c_void_p, c_void_p, c_void_p, ctypes.c_float, ctypes.c_float, ctypes.c_float,
                                   c_void_p, c_int32, c_void_p]),
    "td7_mse_fwd": (c_int32, [c_void_p, c_void_p, ctypes.c_int64, c_void_p, c_void_p, c_void_p]),
    "td7_mse_bwd": (c_int32, [c_void_p, c_void_p, c_void_p, ctypes.c_int64, c_void_p, c_void_p]),
    "td7_avgl1norm_fwd": (c_int32, [c_void_p, c_void_p, c_void_p, c_int32, c_int32, ctypes.c_float, c_void_p]),
    "td7_avgl1norm_fwd_h": (c_int32, [c_void_p, c_void_p, c_void_p, c_int32, c_int32, ctypes.c_float, c_int32,
                                      c_void_p]),
    "td7_avgl1norm_bwd": (c_int32, [c_void_p, c_void_p, c_void_p, c_void_p, c_int32, c_int32, ctypes.c_float,
                                    c_void_p]),
    "td7_dense_fwd": (c_int32, [c_void_p, c_long, c_long, c_void_p, c_void_p, c_void_p, c_long, c_long,
                                c_int32, c_int32, c_int32, c_int32, c_int32, c_void_p]),
    "td7_dense_bwd_data": (c_int32, [c_void_p, c_long, c_long, c_void_p, c_long, c_long, c_void_p, c_void_p,
                                     c_long, c_long, c_int32, c_int32, c_int32, c_int32, c_int32, c_int32,
                                     c_void_p]),
    "td7_dense_bwd_data_cols": (c_int32, [c_void_p, c_long, c_long, c_void_p, c_long, c_long, c_void_p, c_void_p,
                                          c_long, c_long, c_int32, c_int32, c_int32, c_int32, c_int32, c_int32, c_int32,
                                          c_int32, c_void_p]),
    "td7_dense_fwd_cat": (c_int32, [c_int32, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                                    c_long, c_long, c_int32, c_int32, c_int32, c_int32, c_void_p]),
    "td7_dense_fwd_w16": (c_int32, [c_void_p, c_long, c_long, c_void_p, c_void_p, c_void_p, c_long, c_long,
                                    c_int32, c_int32, c_int32, c_int32, c_int32, c_void_p, c_void_p]),
    "td7_dense_fwd_cat_w16": (c_int32, [c_int32, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                                        c_void_p, c_long, c_long, c_int32, c_int32, c_int32, c_int32, c_void_p,
                                        c_void_p]),
    "td7_dense_fwd_h": (c_int32, [c_void_p, c_void_p, c_long, c_long, c_void_p, c_void_p, c_void_p, c_void_p,
                                  c_long, c_long, c_int32, c_int32, c_int32, c_int32, c_int32, c_void_p, c_void_p]),
    "td7_dense_fwd_cat_h": (c_int32, [c_int32, c_void_p, c_int32, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                                      c_void_p, c_long, c_long, c_int32, c_int32, c_int32, c_int32, c_void_p,
                                      c_void_p]),
    "td7_dense_bwd_weight_cat": (c_int32, [c_void_p, c_long, c_long, c_void_p, c_long, c_long, c_int32, c_void_p,
                                           c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_int32, c_int32, c_int32,
                                           c_int32, c_void_p]),
    "td7_adam_step_multi": (c_int32, [c_int32, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                                      c_void_p, c_void_p, c_int32, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                                      c_void_p]),
    "td7_dense_fwd_norm": (c_int32, [c_void_p, c_long, c_long, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                                     c_long, c_long, c_int32, c_int32, c_int32, c_int32, c_int32, ctypes.c_float,
                                     c_void_p]),
    "td7_dense_fwd_norm_cat": (c_int32, [c_int32, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                                         c_void_p, c_void_p, c_long, c_long, c_int32, c_int32, c_int32, c_int32,
                                         ctypes.c_float, c_void_p]),
    "td7_noisy_action_rng": (c_int32, [c_void_p, ctypes.c_uint64, ctypes.c_uint32, c_void_p, c_void_p, c_void_p,
                                       ctypes.c_float, ctypes.c_float, ctypes.c_float, c_void_p, c_int32, c_void_p,
                                       c_void_p]),
    "td7_dense_bwd_weight": (c_int32, [c_void_p, c_long, c_long, c_void_p, c_long, c_long, c_void_p, c_long,
                                       c_long, c_void_p, c_void_p, c_int32, c_int32, c_int32, c_int32, c_int32,
                                       c_void_p]),
    "td7f_pack": (c_int32, [c_int32, c_int32, P(TD7FPackJob), c_void_p]),
    "td7f_adam_pack": (c_int32, [c_int32, c_int32, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                                 c_void_p, c_void_p, c_void_p, c_int32, c_void_p, c_void_p, c_void_p, c_void_p,
                                 c_int32, P(TD7FPackJob), c_void_p, c_void_p, c_void_p]),
    "td7f_probe": (c_int32, [c_int32]),
    "td7f_select": (c_int32, [c_int32, P(c_int32), P(TD7FLin), P(TD7FLin), c_void_p, c_int32, P(TD7FNoise), c_void_p,
                              c_int32, c_int32, c_void_p]),
    "td7f_select_part": (c_int32, [c_int32, P(c_int32), P(TD7FLin), P(TD7FLin), c_void_p, c_int32, P(TD7FNoise),
                                   c_void_p, c_int32, c_int32, c_void_p, c_int32, c_void_p]),
    "td7f_target": (c_int32, [c_int32, P(c_int32), P(TD7FLin), P(TD7FLin), P(TD7FLin), c_void_p, c_int32,
                              P(TD7FNoise), c_void_p, c_void_p, c_void_p]),
    "td7f_fixed": (c_int32, [c_int32, P(c_int32), P(TD7FLin), c_void_p, c_void_p, c_int32, c_void_p, c_void_p,
                             c_void_p]),
    "td7f_critic": (c_int32, [c_int32, P(c_int32), P(TD7FLin)] + [c_void_p] * 7 + [ctypes.c_float]
                    + [c_void_p] * 4 + [c_int32] * 3 + [c_void_p] * 4 + [P(TD7FXT), ctypes.c_int64, c_void_p]),
    "td7f_critic_phase": (c_int32, [c_int32, c_int32, P(c_int32), P(TD7FLin)] + [c_void_p] * 7 + [ctypes.c_float]
                          + [c_void_p] * 4 + [c_int32] * 3 + [c_void_p] * 4
                          + [P(TD7FXT), ctypes.c_int64, c_void_p, c_void_p, c_void_p, c_void_p]),
    "td7f_encoder": (c_int32, [c_int32, P(c_int32), P(TD7FLin), c_void_p, c_void_p, c_void_p, c_int32, P(c_void_p),
                               P(TD7FXT), ctypes.c_int64, c_void_p, c_void_p, c_void_p]),
    "td7f_actor": (c_int32, [c_int32, c_int32, P(c_int32), P(TD7FLin), P(TD7FLin), P(TD7FLin), c_void_p, c_void_p,
                             c_int32, P(TD7FActorBufs), P(TD7FXT), ctypes.c_int64, c_void_p]),
    "td7f_wgrad": (c_int32, [c_int32, c_int32, P(TD7FWgJob), ctypes.c_int64, c_int32, c_void_p, c_void_p, c_int32,
                             ctypes.c_float, ctypes.c_float, c_void_p]),
    "td7f_wgrad_adam": (c_int32, [c_int32, c_int32, P(TD7FWgJob), ctypes.c_int64, c_int32, c_void_p, c_void_p,
                                  c_int32, ctypes.c_float, ctypes.c_float, c_int32, c_void_p, c_void_p, c_void_p,
                                  c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, P(TD7FWgAdam), c_void_p,
                                  c_void_p]),
}

_lib = None


def build(force=False):
    """Compile csrc/*.hip for gfx950 into exo_amd/_lib/libexo_amd.so."""
    if force:
        subprocess.run(["make", "-s", "-C", CSRC, "clean"], check=True)
    subprocess.run(["make", "-s", "-j4", "-C", CSRC], check=True)


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise ImportError(f"{LIB_PATH} is missing: build it with `make -C {CSRC}` (hipcc, gfx950)")
        L = ctypes.CDLL(LIB_PATH)
        for name, (res, args) in EXPORTS.items():
            fn = getattr(L, name)
            fn.restype, fn.argtypes = res, args
        _lib = L
    return _lib


def check(rc, what, ctx=None):
    if rc != EXO_OK:
        msg = ""
        if ctx is not None:
            m = lib().exo_last_error(ctx)
            msg = m.decode() if m else ""
        raise RuntimeError(f"{what} failed: {ERRORS.get(rc, rc)} {msg}")


def require_gpu(device):
    if not torch.cuda.is_available():
        raise RuntimeError("exo_amd runs on an MI355X (HIP) device; no GPU is visible and there is no CPU fallback")
    dev = torch.device(device if device is not None else "cuda")
    if dev.type != "cuda":
        raise RuntimeError(f"exo_amd tensors live on the GPU, got device {dev}")
    if dev.index is None:
        dev = torch.device("cuda", torch.cuda.current_device())
    return dev


def stream_ptr(device):
    return ctypes.c_void_p(torch.cuda.current_stream(device).cuda_stream)


def ptr(t):
    return ctypes.c_void_p(t.data_ptr()) if t is not None else None
