/*
 * exo_amd.h -- C ABI of the MI355X-native exoskeleton environment and LAP
 * replay kernels (libexo_amd.so, built for gfx950).
 *
 * The reference (TomasDelaney/A-Deep-Reinforcement-Learning-Enabled-Soft-
 * Exoskeleton-for-Parkinson-s-Patients) is pure Python and has no FFI; the
 * entry points below are what its Python call sites would bind through
 * ctypes.  Each one cites the reference interface it replaces (path:line).
 * INTEGRATION.md shows the ctypes binding.
 *
 * Conventions
 *   - All functions return 0 on success, a negative errno-style code
 *     otherwise (EXO_E*); nothing throws across the ABI.  exo_last_error()
 *     returns a message for the last failing call on that context.
 *   - Buffers named *_dev are DEVICE pointers (e.g. torch tensor data_ptr()).
 *     Buffers named *_host are host pointers.  `stream` is a hipStream_t
 *     (NULL = default stream).  Work is stream ordered; only the *_host
 *     read-back helpers synchronise.
 *   - One context per device.  Calls on one context are not thread safe.
 */
#ifndef EXO_AMD_H
#define EXO_AMD_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define EXO_OK 0
#define EXO_EINVAL (-22)
#define EXO_ENOMEM (-12)
#define EXO_EDEVICE (-5)
#define EXO_ERANGE (-34)

#define EXO_OBS_DIM 80  /* Exoskeleton_env.py:99-111 */
#define EXO_ACT_DIM 7   /* Exoskeleton_env.py:74 */
#define EXO_INFO_DIM 40 /* Exoskeleton_env.py:464-469: 5 x [7] + 5 reward terms */
#define EXO_STATE_DOUBLES 53

/* Number of unit-uniform draws one reset consumes for an episode of length L
 * (the np.random call order of Exoskeleton_env.py:198-217). */
#define EXO_DRAWS_PER_EPISODE(L) (208 + 8 * (L))

/* Constructor arguments of ExoskeletonEnv_train.__init__
 * (Environment/Exoskeleton_env.py:38-48); one per env, so domain-randomisation
 * sweeps can vary them per env. */
typedef struct {
    int32_t motion;                      /* reference_motion_file_num (index into the motion table) */
    int32_t tremor_sequence[7];          /* 0/1 per joint axis */
    double tremor_amplitude_range[2];
    double first_harmonics_interval[2];
    double second_harmonics_interval[2];
    double max_force_shoulder;
    double max_force_elbow;
    double dr_actuator_end_pos_shift;
    double dr_actuator_range;
    double matrix_noise_fraction;
} exo_env_config;

typedef struct exo_ctx exo_ctx;

/* Replaces ExoskeletonEnv_train.__init__ (Exoskeleton_env.py:38-175) for n_envs
 * envs at once, including the constructor's initialize_movement() (:172).
 * motion_angles_host: [n_motions][5][max_len] degrees, columns elbow_y,
 * elbow_z, shoulder_x, shoulder_y, shoulder_z (read_txt_env.py:109-113).
 * Draws for every reset come from Philox4x32-10 keyed by (seed, env, episode). */
int exo_create(const exo_env_config *cfgs_host, int32_t n_envs, const double *motion_angles_host,
               const int32_t *motion_lengths_host, int32_t n_motions, int32_t max_len, uint64_t seed,
               int32_t device, exo_ctx **out);

/* Replaces ExoskeletonEnv_train.reset() (Exoskeleton_env.py:473-478 ->
 * initialize_movement :193-254) for every env whose mask byte is non-zero
 * (mask_dev NULL = all envs).  Writes the reset observation of those envs. */
int exo_reset(exo_ctx *ctx, const uint8_t *mask_dev, float *obs_dev, void *stream);

/* Parity hook: reset the listed envs from explicit draw streams instead of
 * Philox.  draws_host holds n rows of EXO_DRAWS_PER_EPISODE(max_len) doubles;
 * row k feeds env env_ids_host[k] (only its first 208+8L entries are read). */
int exo_reset_from_draws(exo_ctx *ctx, const int32_t *env_ids_host, int32_t n, const double *draws_host,
                         float *obs_dev, void *stream);

/* Replaces ExoskeletonEnv_train.step(action) (Exoskeleton_env.py:368-471) for
 * all envs.  act_dev [N][7] in [-1,1]; obs_dev [N][80]; rew_dev [N]; done_dev
 * [N]; info_dev [N][40] or NULL.  Envs whose active byte is 0 (active_dev
 * non-NULL), or that already reached the end of their motion, are skipped and
 * their outputs left untouched (the training script steps only envs that are
 * not done: Exoskeleton_agent_train.py:139-141). */
int exo_step(exo_ctx *ctx, const float *act_dev, float *obs_dev, float *rew_dev, uint8_t *done_dev,
             float *info_dev, const uint8_t *active_dev, void *stream);

/* Accessors mirroring return_max_length (:577), return_generated_tremor_data
 * (:572-575) and return_original_joint_angles (:580-592). */
int32_t exo_num_envs(const exo_ctx *ctx);
int exo_episode_length(const exo_ctx *ctx, int32_t env, int32_t *L_out);
int exo_tremor_host(exo_ctx *ctx, int32_t env, double *tremor_out /* [7][L] */);
int exo_original_joint_angles_host(exo_ctx *ctx, int32_t env, double *out7);

/* Episode constants of one env: dense D and S (49 each), dense I^-1 (49),
 * dummy shift (42), max_output_shoulder, max_output_elbow. */
int exo_episode_host(exo_ctx *ctx, int32_t env, double *D49, double *S49, double *Iinv49, double *shift42,
                     double *maxSE2);

/* Checkpoint/inspection of one env's carried state (EXO_STATE_DOUBLES doubles):
 * [0] counts, [1..5] joint positions, [6..11] cached reference positions,
 * [12..32] position vectors, [33..39] prev action, [40..46] second prev action,
 * [47] max_output_shoulder, [48] max_output_elbow, [49] episode index, [50] L, [51] motion,
 * [52] steps that violated the joint ranges of check_movement_boundaries (:594-605). */
int exo_get_state_host(exo_ctx *ctx, int32_t env, double *out);
int exo_set_state_host(exo_ctx *ctx, int32_t env, const double *in);

/* Kernel variant of exo_step: EXO_STEP_LANES = one lane per ODE solve (best
 * throughput at large N), EXO_STEP_ROWS = 16 lanes per env, one joint row per
 * lane (lowest latency at small N), EXO_STEP_AUTO (default) = ROWS for
 * N <= 16384, EXO_STEP_ROWS_SHARED = ROWS packed 32 envs per 512-thread
 * workgroup (half the CUs at 4,096 envs: for a GPU shared with concurrent
 * kernels, the training loop).  All compute the same step. */
#define EXO_STEP_AUTO 0
#define EXO_STEP_LANES 1
#define EXO_STEP_ROWS 2
#define EXO_STEP_ROWS_SHARED 3
int exo_set_step_variant(exo_ctx *ctx, int32_t variant);

/* Budgeted step (no reference counterpart; BASELINE configs[3]'s stiff
 * domain-randomised envs): with budget > 0 each launch of exo_step runs at most
 * `budget` RK45 step attempts per ODE solve (Utilities/calculate_joint_angles.py:
 * 5-22); a solve left unfinished keeps its exact solver state on the device and
 * continues in the next launch, and its env starts no new step until both
 * solves of its step are done (the step's observation, reward and done were
 * already written when it started: they never depend on the solves).  Every
 * env's trajectory is the unbudgeted one.  Row-parallel kernels only (ROWS /
 * ROWS_SHARED / AUTO at N <= 16384), idealised physics only.  budget 0
 * restores unbudgeted launches (refused while a solve is pending). */
int exo_set_step_budget(exo_ctx *ctx, int32_t budget);
/* exo_step with, in budget mode, the current observation buffer obs_cur_dev
 * [N][80] (may be NULL): an env resuming a pending solve copies its row into
 * obs_dev, so alternating observation buffers stay current. */
int exo_step_carry(exo_ctx *ctx, const float *act_dev, float *obs_dev, float *rew_dev, uint8_t *done_dev,
                   float *info_dev, const uint8_t *active_dev, const float *obs_cur_dev, void *stream);
/* Budget mode's step mask on the device: active_dev[e] = the env will start a
 * step in the next launch (episode not over, no pending solve), *count_dev
 * (int32) their number, *remaining_dev (int32) the envs not finished (episode
 * not over or a solve pending: 0 = the round is over), *steps_total_dev (int64,
 * may be NULL) += the previous *count_dev (the envs the last launch stepped).
 * One workgroup, graph-capturable. */
int exo_budget_advance(exo_ctx *ctx, uint8_t *active_dev, int32_t *count_dev, int32_t *remaining_dev,
                       int64_t *steps_total_dev, void *stream);

/* Auto-reset episodes (the vectorised trainer's asynchronous mode): after a
 * step launch, every env whose episode is over (its done step was taken and,
 * with a step budget, that step's solve is complete) is reset in place --
 * exo_reset for those envs, its observation written into obs_dev (the buffer
 * the step just wrote) -- and the mask of the next launch is written: every
 * env, except (step budget) one whose solve is pending.
 * count_dev = that mask's population, steps_total_dev (int64, optional) += the
 * previous *count_dev (the envs the last launch stepped).  reset_ws_dev:
 * int32 [N + 1] workspace (the envs reset, their number at [N]).  Replaces the
 * training script's per-round reset (Simulation/Exoskeleton_agent_train.py:
 * 111-113) with a per-env one, as a vectorised env's auto-reset. */
int exo_episode_advance(exo_ctx *c, uint8_t *active_dev, int32_t *count_dev, int32_t *reset_ws_dev,
                        int64_t *steps_total_dev, float *obs_dev, void *stream);

/* Step clock (measurement; no reference counterpart): with clock_dev non-NULL
 * (3 device uint64), every later exo_step -- eager or captured into a graph --
 * brackets its launches with two one-lane kernels on its stream that read the
 * device wall clock; clock_dev[1] accumulates the bracketed ticks and
 * clock_dev[2] counts the steps.  *ticks_per_ms (if non-NULL) receives the
 * clock rate.  NULL turns it off for later launches. */
int exo_set_step_clock(exo_ctx *ctx, unsigned long long *clock_dev, double *ticks_per_ms);

/* Tremor model of later resets (diagnostic; the default is the shipped code):
 * jmax7 = joint_max_values before the magnitude (generate_parkinson_tremor.py:59;
 * NULL = the shipped {2.5, 5, 10, 5, 5, 0.5, 0.5}), sign_mode = how
 * np.random.choice([-1, 1], L) (:70) applies: EXO_TREMOR_SIGN_PER_SAMPLE (the
 * shipped code), EXO_TREMOR_SIGN_PER_AXIS (the axis's first sign draw for
 * every sample), EXO_TREMOR_SIGN_NONE.  The draw stream is unchanged.  Used
 * to test which code revision produced the authors' Evaluation_logs (their
 * per-env blocks print max torques of exactly {10, 5, 2.5, 5} on axes 0-3). */
#define EXO_TREMOR_SIGN_PER_SAMPLE 0
#define EXO_TREMOR_SIGN_PER_AXIS 1
#define EXO_TREMOR_SIGN_NONE 2
int exo_set_tremor_model(exo_ctx *ctx, const double *jmax7, int32_t sign_mode);

/* ------------------------------------------------------------------------
 * Physics of stepSimulation (Exoskeleton_env.py:433, Bullet 3.2.5 -- absent
 * here).  EXO_PHYS_IDEAL (default): the idealised position motors of
 * SURVEY.md A.2 (each revolute joint moves 10 % of the way to its target,
 * clamped to the URDF limits; prismatic anchors stay at 0).
 * EXO_PHYS_MULTIBODY: the btMultiBody pipeline on the 19-joint URDF tree --
 * Featherstone forward dynamics (gravity, link damping, gyroscopic terms), the
 * joint motors and violated joint limits as rows of a joint-space projected
 * Gauss-Seidel impulse solve, semi-implicit Euler (csrc/exo_multibody.hip,
 * oracle/multibody.c).  The constants are Bullet
 * defaults from its documentation, not measured against pybullet.
 * ---------------------------------------------------------------------- */
#define EXO_PHYS_IDEAL 0
#define EXO_PHYS_MULTIBODY 1
typedef struct {
    double gravity;         /* m/s^2 along -z (setGravity, :116) */
    double kp, kd;          /* POSITION_CONTROL gains of the revolute motors (sim:115-117 defaults 0.1, 1) */
    double motor_impulse;   /* max impulse of the revolute motors (force 1e5 x dt) */
    double passive_impulse; /* max impulse of the prismatic joints' default velocity motors (1) */
    double limit_impulse;   /* max impulse of a joint-limit row (100) */
    double erp;             /* limit error reduction (0.2) */
    double lin_damp, ang_damp; /* btMultiBody link damping (0.04, 0.04) */
    double max_vel;         /* max joint velocity (100) */
    int32_t iters;          /* solver sweeps (numSolverIterations, 50) */
} exo_mb_params;
void exo_multibody_default_params(exo_mb_params *out);
/* Select the physics (params NULL = defaults).  Switching to MULTIBODY starts
 * from the current arm pose at rest with the k-links at 0. */
int exo_set_physics(exo_ctx *ctx, int32_t mode, const exo_mb_params *params);
/* One multibody stepSimulation alone for the envs with mask byte != 0 (NULL =
 * all), POSITION_CONTROL targets targets_dev [5][N] (rad, joints 0..4). */
int exo_multibody_advance(exo_ctx *ctx, const double *targets_dev, const uint8_t *mask_dev, void *stream);
/* Joint positions / velocities of the 19 URDF joints (pybullet link order). */
int exo_get_multibody_state_host(exo_ctx *ctx, int32_t env, double *q19, double *qd19);
int exo_set_multibody_state_host(exo_ctx *ctx, int32_t env, const double *q19, const double *qd19);

/* Re-key the Philox draw streams of later resets (ExoskeletonEnv_train.seed, :189-191). */
int exo_set_seed(exo_ctx *ctx, uint64_t seed);

const char *exo_last_error(const exo_ctx *ctx);
void exo_destroy(exo_ctx *ctx);

/* Tremor-suppression statistics of Simulation/Exoskeleton_agent_train.py:149-200
 * for every env the last exo_step advanced (stepped_dev[i] != 0; NULL = all),
 * read from that step's info rows (info_dev [N][40]):
 *   metrics_dev [N][16] (written): torque reduction per axis (7, percent,
 *     nan_to_num), amplitude reduction per axis (7), end-effector amplitude
 *     change (1; DH FK of Utilities/calculate_arm_end_effector_points.py:18-50
 *     on the IMU angles with the suppressed / unsuppressed tremor amplitudes),
 *     any-nonzero flag (1); with disregard != 0 positive values are zeroed
 *     (:186-191); the rows of envs not stepped are zeros (:201-203);
 *   counters_dev [N][6] (accumulated): tremor_when_reduction[0..1],
 *     tremor_reduction_in_episode, tremor_when_ampl_reduction[0..1],
 *     tremor_ampl_total_reduction_ep (last negative value). */
int exo_tremor_metrics(exo_ctx *c, const float *info_dev, const uint8_t *stepped_dev, double humerus_length,
                       double forearm_length, double hand_length, int32_t disregard, float *metrics_dev,
                       float *counters_dev, void *stream);

/* The evaluation script's statistics (Simulation/Evaluate_control_performance.py:
 * 192-260: reductions over |ref + 1e-10|, SFE/SAA amplitudes swapped before the
 * DH FK, torque counters over the env's tremor axes with <= 0) for every env
 * the last exo_step advanced; counters_dev [N][5] accumulate:
 *   steps with every tremor axis suppressed (tremor_when_reduction[i, 1]),
 *   steps with any tremor axis suppressed (tremor_reduction_in_episode[i]),
 *   steps with end-effector amplitude change < 0 / >= 0
 *     (tremor_when_ampl_reduction[i, 1] / [i, 0]),
 *   the sum of the negative changes (for the episode mean over non-zero
 *     entries of tremor_ampl_total_reduction_full_ep, :262). */
/* The synchronous-episode trainer's active mask on the device
 * (Simulation/Exoskeleton_agent_train.py:123-125): *k_dev (int64) advances by
 * one, saturating at rows - 1, and row *k_dev of table_dev [rows][n] (uint8)
 * is copied to active_dev [n]; count_dev (int32, may be NULL) receives the
 * number of active envs of that row -- the number of select_action calls the
 * script makes at that step (:125-128).  Graph-capturable, no host sync. */
int exo_active_advance(const uint8_t *table_dev, int32_t rows, int32_t n, int64_t *k_dev, uint8_t *active_dev,
                       int32_t *count_dev, void *stream);
/* exo_active_advance that first adds this step's rewards into the episode
 * scores of the envs active under the mask it replaces:
 * score_dev[e] (float64) += active_dev[e] ? reward_dev[e] (float32) : 0.0
 * (Simulation/Exoskeleton_agent_train.py:144 `score[i] += reward`), one launch
 * instead of torch's where + add_. */
int exo_active_advance_score(const uint8_t *table_dev, int32_t rows, int32_t n, int64_t *k_dev, uint8_t *active_dev,
                             int32_t *count_dev, const float *reward_dev, double *score_dev, void *stream);

int exo_eval_metrics(exo_ctx *c, const float *info_dev, const uint8_t *stepped_dev, double humerus_length,
                     double forearm_length, float *counters_dev, void *stream);

/* ------------------------------------------------------------------------
 * LAP prioritised replay (Agent/TD7_buffer_multi_agent.py:5-120), one
 * sum tree per stratum (the reference keeps one priority row per env,
 * :41, and samples batch_size rows from each, :75-85).
 * ---------------------------------------------------------------------- */
/* Caller-owned sum trees: tree[n_strata][2*cap] fp32 (cap = capacity rounded
 * up to a power of two; node 1 of a stratum is its total, leaf i -- the
 * reference's self.priority[s, i] -- is node cap + i) and one fp32
 * max_priority scalar.  Both are device memory (e.g. torch tensors). */
typedef struct {
    float *tree;
    float *max_priority;
    int32_t n_strata;
    int32_t capacity; /* max_size per stratum (:19) */
    int32_t cap;      /* power of two >= capacity */
} lap_tree_desc;

/* floats needed for the trees of n_strata x capacity (= n_strata * 2 * cap). */
int32_t lap_tree_floats(int32_t n_strata, int32_t capacity);

/* zero every tree, max_priority = 1 (LAP.__init__ / reset_buffer, :39-45, :133-137). */
int lap_init(const lap_tree_desc *t, void *stream);

/* LAP.add (:49-63) for n items: stratum_dev[n], slot_dev[n] (slot < 0: skip);
 * every item gets the current max_priority. */
int lap_add(const lap_tree_desc *t, const int32_t *stratum_dev, const int32_t *slot_dev, int32_t n, void *stream);

/* LAP.sample (:65-85): for every stratum s, batch indices
 * idx = searchsorted_left(cumsum(p[s, :size[s]]), u * sum) for the
 * per-stratum uniforms u_dev[s][batch].  size_dev[n_strata] (int32).
 * Writes idx_dev[s][batch] (int32, within-stratum slot). */
int lap_sample(const lap_tree_desc *t, const float *u_dev, const int32_t *size_dev, int32_t batch, int32_t *idx_dev,
               void *stream);

/* LAP.update_priority (:113-117): p[s, idx[s][b]] = prio[s*batch+b] (the last
 * occurrence wins for duplicate indices, as the reference's CPU index_put),
 * then max_priority = max(max_priority, max(prio)). */
int lap_update(const lap_tree_desc *t, const int32_t *idx_dev, const float *prio_dev, int32_t batch, void *stream);

/* LAP.reset_max_priority (:119-120): max_priority = max over all leaves. */
int lap_reset_max(const lap_tree_desc *t, void *stream);

/* Total priority of each stratum (root of its tree) -> out_dev[n_strata]. */
int lap_totals(const lap_tree_desc *t, float *out_dev, void *stream);

/* Transition storage of the LAP buffer: [n_strata][capacity + 1][dim] fp32
 * (row `capacity` of every stratum is a trash row for inactive envs), and
 * the device ring pointer / size of every stratum. */
typedef struct {
    float *state, *action, *next_state, *reward, *not_done;
    int32_t state_dim, action_dim;
    int32_t *ptr, *size;
} lap_storage_desc;

/* LAP.add (:49-63) for one vectorised env step of n envs: env i, when
 * active[i] (NULL = all), goes to stratum strata[i] at the next ring slot
 * (env order within a stratum), with priority max_priority; stores
 * action/action_scale and not_done = 1 - done.  row_ws: n int32 scratch. */
int lap_store_batch(const lap_tree_desc *t, const lap_storage_desc *st, const float *state_dev,
                    const float *action_dev, const float *next_state_dev, const float *reward_dev,
                    const uint8_t *done_dev, const int32_t *strata_dev, const uint8_t *active_dev, float action_scale,
                    int32_t n, int32_t *row_ws_dev, void *stream);

/* LAP.add (Agent/TD7_buffer_multi_agent.py:49-63) called once per active env
 * of one vectorised step, in env order -- the training script's per-env loop
 * (Simulation/Exoskeleton_agent_train.py:139-142) -- with the reference's
 * SHARED pointer: ref_dev = int64 {ptr, count, size} (zero = a fresh buffer),
 * the c-th add writes slot ptr + #{multiples of n_strata in [count, c)} of
 * stratum strata[i] (env 0's first transition one slot behind, overwrites when
 * envs are done: the later add wins), every stratum's sampling size set to the
 * shared size.  Same stored values as lap_store_batch.  ws_dev: 3n int32
 * scratch. */
int lap_store_batch_ref(const lap_tree_desc *t, const lap_storage_desc *st, int64_t *ref_dev,
                        const float *state_dev, const float *action_dev, const float *next_state_dev,
                        const float *reward_dev, const uint8_t *done_dev, const int32_t *strata_dev,
                        const uint8_t *active_dev, float action_scale, int32_t n, int32_t *ws_dev, void *stream);

/* lap_store_batch_ref as ONE launch (the same stored rows, leaves, sums,
 * pointer and sizes, bit for bit): grid n_strata x (copy parts); the last
 * workgroup out advances ref_dev.  ticket_dev: one uint32, zero at the first
 * call, left zero. */
int lap_store_batch_ref_fused(const lap_tree_desc *t, const lap_storage_desc *st, int64_t *ref_dev,
                              const float *state_dev, const float *action_dev, const float *next_state_dev,
                              const float *reward_dev, const uint8_t *done_dev, const int32_t *strata_dev,
                              const uint8_t *active_dev, float action_scale, int32_t n, uint32_t *ticket_dev,
                              void *stream);

/* lap_store_batch_ref_fused plus the training loop's mask advance in the same
 * launch (the reference-schedule rollout step, Simulation/
 * Exoskeleton_agent_train.py:123-144): once every workgroup has read the
 * step's mask, the last one out adds the step's rewards into the episode
 * scores where the mask is set (score_dev, float64 [N], optional), advances
 * the device step counter *k_dev = min(*k_dev + 1, rows - 1) and copies row
 * *k_dev of the mask table (uint8 [rows][N]) into active (and its population
 * into *count_dev, optional) -- exo_active_advance_score's arithmetic. */
int lap_store_batch_ref_fused_adv(const lap_tree_desc *t, const lap_storage_desc *st, int64_t *ref_dev,
                                  const float *state, const float *action, const float *next_state,
                                  const float *reward, const uint8_t *done, const int32_t *strata, uint8_t *active,
                                  float action_scale, int32_t n, uint32_t *ticket_dev, const uint8_t *table,
                                  int32_t rows, int64_t *k_dev, int32_t *count_dev, double *score_dev, void *stream);

/* The reference-schedule rollout's inserts planned per episode round (r05;
 * the same rows, leaves, sums, pointer and sizes as calling
 * lap_store_batch_ref_fused_adv at every step, bit for bit, provided the tree
 * is not read before lap_ref_commit -- the rollout trains nothing):
 * lap_ref_plan: for the mask table rows [0, rows) of the round (uint8
 * [rows][n], table_dev, the envs running at each step) and offs_dev (int64
 * [rows]: the adds before each step, i.e. the exclusive prefix sums of the
 * rows' active counts; total = all the round's adds), plan_dev[k][e] = the
 * slot env e's step-k add writes, -1 when it is inactive or a later add of
 * its slot group has its stratum (overwritten).  add_ws_dev: total int32.
 * ref_dev is read (the pointer at the round start), not changed. */
int lap_ref_plan(const lap_tree_desc *t, const int64_t *ref_dev, const uint8_t *table_dev, int32_t rows, int32_t n,
                 const int32_t *strata_dev, const int64_t *offs_dev, int64_t total, int32_t *add_ws_dev,
                 int32_t *plan_dev, void *stream);
/* One rollout step of a planned round: every env with plan[k][e] >= 0 stores
 * its transition there (action / action_scale, not_done = 1 - done); then
 * score_dev[e] += reward where active[e] (optional), active = table row k + 1
 * (saturating at rows - 1), *count_dev = counts_table_dev[k + 1] (optional).
 * k = kk_dev[par]; the launch writes k + 1 into kk_dev[par ^ 1] and *k_dev
 * (optional), so consecutive steps alternate par. */
int lap_ref_step(const lap_tree_desc *t, const lap_storage_desc *st, const int32_t *plan_dev, int32_t rows,
                 int32_t n, int64_t *kk_dev, int32_t par, int64_t *k_dev, const int32_t *strata_dev,
                 const float *state, const float *action, const float *next_state, const float *reward,
                 const uint8_t *done, float action_scale, const uint8_t *table_dev, uint8_t *active_dev,
                 int32_t *count_dev, const int32_t *counts_table_dev, double *score_dev, void *stream);
/* The end of a planned round: the leaves of every planned slot set to
 * max_priority, the round's ring span recomputed in every stratum, the shared
 * pointer {ptr, count, size} advanced by the round's `total` adds and every
 * stratum's sampling size set. */
int lap_ref_commit(const lap_tree_desc *t, const lap_storage_desc *st, int64_t *ref_dev, const int32_t *plan_dev,
                   int32_t rows, int32_t n, const int32_t *strata_dev, int64_t total, void *stream);

/* LAP.sample (:65-111): batch draws per stratum (u_dev [n_strata][batch]),
 * indices -> idx_dev [n_strata][batch], the sampled rows gathered into
 * out_* [n_strata * batch][dim] (stratum-major). */
int lap_sample_gather(const lap_tree_desc *t, const lap_storage_desc *st, const float *u_dev, int32_t batch,
                      int32_t *idx_dev, float *out_state, float *out_action, float *out_next_state,
                      float *out_reward, float *out_not_done, void *stream);
/* LAP.update_priority (:113-117) followed by the next LAP.sample (:65-111)
 * as ONE launch: the priorities prio_dev of the draws idx_in_dev, then the
 * next batch drawn and gathered exactly as lap_sample_gather_rng (same
 * counter stream) into idx_dev / out_*.  batch <= 1024. */
int lap_update_sample_rng(const lap_tree_desc *t, const lap_storage_desc *st, const int32_t *idx_in_dev,
                          const float *prio_dev, int32_t batch, uint64_t seed, uint32_t tag,
                          unsigned long long *counter_dev, uint32_t *ticket_dev, int32_t *idx_dev, float *out_state,
                          float *out_action, float *out_next_state, float *out_reward, float *out_not_done,
                          void *stream);

/* lap_update_sample_rng in two launches (r05): the priority update and the
 * next sample's indices (idx_out [n_strata][batch]), then the rows of those
 * indices gathered from the storage -- so a caller can start the first once the
 * tree is current (this step's inserts ranked) and the second once the rows
 * are (its copies done).  Together bit-identical to lap_update_sample_rng
 * (TD7_buffer_multi_agent.py:113-117, then :65-111). */
int lap_update_sample_idx(const lap_tree_desc *t, const lap_storage_desc *st, const int32_t *idx_in,
                          const float *prio, int32_t batch, uint64_t seed, uint32_t tag, unsigned long long *counter,
                          uint32_t *ticket, int32_t *idx_out, void *stream);
int lap_gather_rows(const lap_tree_desc *t, const lap_storage_desc *st, int32_t batch, const int32_t *idx,
                    float *out_state, float *out_action, float *out_next_state, float *out_reward,
                    float *out_not_done, void *stream);
/* lap_update_sample_rng with the priorities computed in the launch from the
 * critic pass's |td| of both heads (td [B][2], B = n_strata x batch):
 * prio = max(|td0|, |td1|, min_priority)^alpha (TD7_multi_agent.py:259, the
 * expression td7f_wgrad writes), also stored in prio_out if non-NULL -- the
 * priority update then depends on the critic pass only, not on the weight
 * gradients that follow it.  Bit-identical to td7f_wgrad's priorities +
 * lap_update_sample_rng. */
int lap_update_sample_td(const lap_tree_desc *t, const lap_storage_desc *st, const int32_t *idx_in, const float *td,
                         float alpha, float min_priority, float *prio_out, int32_t batch, uint64_t seed, uint32_t tag,
                         unsigned long long *counter, uint32_t *ticket, int32_t *idx_out, float *out_state,
                         float *out_action, float *out_next_state, float *out_reward, float *out_not_done,
                         void *stream);
/* lap_sample_gather with the uniforms drawn inside the kernel (Philox4x32-10,
 * key seed, counter words (draw index, call, tag)); *counter_dev (the call
 * number) advances by one per launch, ticket_dev: one uint32, zero at the first
 * call, left zero.  Graph-replay safe: no host value changes between calls. */
int lap_sample_gather_rng(const lap_tree_desc *t, const lap_storage_desc *st, uint64_t seed, uint32_t tag,
                          unsigned long long *counter_dev, uint32_t *ticket_dev, int32_t batch, int32_t *idx_dev,
                          float *out_state, float *out_action, float *out_next_state, float *out_reward,
                          float *out_not_done, void *stream);

/* ------------------------------------------------------------------------
 * Fused TD7 net pieces (Agent/TD7_multi_agent.py:53-54, AvgL1Norm).
 * ---------------------------------------------------------------------- */
/* y = x / max(mean|x|, eps) per row; mean_out[rows] keeps mean|x| for backward. */
int td7_avgl1norm_fwd(const float *x_dev, float *y_dev, float *mean_out_dev, int32_t rows, int32_t cols, float eps,
                      void *stream);
/* The same with y as 16-bit values (prec 1 = bf16, 2 = fp16 bits, RNE) for an
 * inference chain whose next layer rounds its input to that type (bit-identical,
 * half the bytes); mean_out may be null; 256 < cols <= 1,024, else EXO_ERANGE. */
int td7_avgl1norm_fwd_h(const float *x_dev, uint16_t *y16_dev, float *mean_out_dev, int32_t rows, int32_t cols,
                        float eps, int32_t prec, void *stream);
/* gradient of the above w.r.t. x given dL/dy. */
int td7_avgl1norm_bwd(const float *x_dev, const float *mean_dev, const float *gy_dev, float *gx_dev, int32_t rows,
                      int32_t cols, float eps, void *stream);

/* torch.optim.Adam step (Agent/TD7_multi_agent.py:165-170, weight_decay) over a
 * flat buffer of n parameters: g *= grad_scale; g += wd p; m, v, p updated in
 * place.  *step_dev (float, the optimiser's step count) is read by every
 * workgroup and advanced by the last one (ticket_dev: one uint32, zero at
 * the first call, left zero by every call). */
int td7_adam_step(float *p_dev, const float *g_dev, float *m_dev, float *v_dev, float *step_dev, uint32_t *ticket_dev,
                  int64_t n, float lr, float beta1, float beta2, float eps, float weight_decay, float grad_scale,
                  void *stream);

/* nopt FlatAdam steps (each: flat p / m / v buffers, device step count,
 * hyper-parameters) in ONE launch, the gradients read from nseg separate
 * tensors: segment k is g[k][0 .. n[k]) for the parameters at flat offset
 * off[k] of optimiser opt[k] (a parameter without gradient has no segment and
 * is skipped, as torch.optim.Adam skips it).  grad_scale 1.  The steps of all
 * optimisers advance by one; ticket_dev as td7_adam_step (its own, one uint32). */
#define TD7_ADAM_MAX_OPT 3
#define TD7_ADAM_MAX_SEG 40
int td7_adam_step_multi(int32_t nopt, float *const *p_dev, float *const *m_dev, float *const *v_dev,
                        float *const *step_dev, const float *lr, const float *beta1, const float *beta2,
                        const float *eps, const float *weight_decay, int32_t nseg, const float *const *g_dev,
                        const int64_t *off, const int32_t *n, const int32_t *opt, uint32_t *ticket_dev, void *stream);

/* Critic target (Agent/TD7_multi_agent.py:240-246): out[b] = reward[b] +
 * not_done[b] * discount * clamp(min(qt[b][0], qt[b][1]), *min_target,
 * *max_target); *run_max / *run_min take the batch max / min.  qt element
 * (b, h) at qt_dev[b*qs_b + h*qs_h]. */
int td7_q_target(const float *qt_dev, long qs_b, long qs_h, const float *reward_dev, const float *not_done_dev,
                 float discount, const float *min_target_dev, const float *max_target_dev, float *run_max_dev,
                 float *run_min_dev, float *out_dev, int32_t batch, void *stream);
/* Critic loss (:257-262): loss = mean_b sum_h LAP_huber(|q[b][h] - q_target[b]|),
 * priority[b] = max(max_h td, min_priority)^alpha, dq [batch][2] = dloss/dq. */
int td7_critic_loss(const float *q_dev, long qs_b, long qs_h, const float *q_target_dev, float *loss_dev,
                    float *priority_dev, float *dq_dev, float alpha, float min_priority, int32_t batch, void *stream);
/* td7_critic_loss with dloss/dQ written at dq[b*dqs_b + head*dqs_h] (the
 * layout of the critic's output view, so the backward needs no copy). */
int td7_critic_loss_strided(const float *q_dev, long qs_b, long qs_h, const float *q_target_dev, float *loss_dev,
                            float *priority_dev, float *dq_dev, long dqs_b, long dqs_h, float alpha,
                            float min_priority, int32_t batch, void *stream);

/* out = clamp(a + c(noise * *sigma), -1, 1) * scale over n values, c = clamp to
 * +-clip when clip > 0; then *sigma -= sigma_dec.  The exploration noise of
 * select_action (TD7_multi_agent_Pink_noise.py:209-228, batched) and the
 * target policy smoothing of the critic target (TD7_multi_agent.py:236-238). */
int td7_noisy_action(const float *a_dev, const float *noise_dev, float *sigma_dev, float sigma_dec, float clip,
                     float scale, float *out_dev, int32_t n, void *stream);
/* td7_noisy_action with the noise drawn in the kernel: element 2j+t is normal t
 * (Box-Muller) of Philox4x32-10 block (j, call, tag) under key seed, call =
 * *counter_dev, which advances by one per launch (graph-replay safe);
 * ticket_dev: one uint32, zero at the first call, left zero.  dec_count_dev
 * (int32, may be NULL): sigma -= sigma_dec * *dec_count_dev instead of
 * sigma_dec -- one decrement per select_action call of the script, i.e. per
 * ACTIVE env (TD7_multi_agent.py:207, Exoskeleton_agent_train.py:125-128). */
int td7_noisy_action_rng(const float *a_dev, uint64_t seed, uint32_t tag, unsigned long long *counter_dev,
                         uint32_t *ticket_dev, float *sigma_dev, float sigma_dec, float clip, float scale,
                         float *out_dev, int32_t n, const int32_t *dec_count_dev, void *stream);
/* F.mse_loss (encoder loss, TD7_multi_agent.py:226): *loss = mean (x - y)^2;
 * backward dx = 2 (x - y) / n * (*g).  ws_dev: TD7_MSE_WS floats, zeroed once
 * by the caller (block partials + a ticket the kernel leaves at zero); one
 * workspace per stream. */
#define TD7_MSE_WS 257
int td7_mse_fwd(const float *x_dev, const float *y_dev, int64_t n, float *loss_dev, float *ws_dev, void *stream);
int td7_mse_bwd(const float *x_dev, const float *y_dev, const float *g_dev, int64_t n, float *dx_dev, void *stream);

/* ------------------------------------------------------------------------
 * Fused dense layers of the TD7 nets on fp32 MFMA (csrc/td7_dense.hip).
 * Each replaces one nn.Linear + activation of Agent/TD7_multi_agent.py:61-140
 * (forward) and its autograd backward.  act: 0 none, 1 relu, 2 elu, 3 tanh.
 * G groups (the critic's Q heads, :120-127) run in one launch; strides are in
 * floats; every row has unit column stride.
 * ---------------------------------------------------------------------- */
/* Y[g] = act(X[g] W[g]^T + b[g]); X [G][M][K] (xsg = 0: one X for all
 * groups), W [G][N][K] contiguous, b [G][N] or NULL, Y [G][M][N]. */
int td7_dense_fwd(const float *x_dev, long xsg, long ldx, const float *w_dev, const float *b_dev, float *y_dev,
                  long ysg, long ldy, int32_t groups, int32_t m, int32_t n, int32_t k, int32_t act, void *stream);
/* dX = (dY * act'(Y)) W per group, or summed over the groups when
 * shared_input != 0 (X was shared); act' is taken from the saved output Y. */
int td7_dense_bwd_data(const float *dy_dev, long dysg, long lddy, const float *y_dev, long ysg, long ldy,
                       const float *w_dev, float *dx_dev, long dxsg, long lddx, int32_t groups, int32_t shared_input,
                       int32_t m, int32_t n, int32_t k, int32_t act, void *stream);
/* td7_dense_fwd of a concatenated input X = [X_0 | ... | X_{nseg-1}] read in
 * place (the reference's Linear(torch.cat([...], 1)), Agent/TD7_multi_agent.py:
 * 70, 104, 126-129): segment s is xs[s], [G][M][widths[s]] with group stride
 * xsg[s] (0 = shared by the groups) and row stride ldx[s]; K = sum of widths.
 * nseg <= 4, interior widths multiples of 4, the last >= 4 (else EXO_EINVAL). */
int td7_dense_fwd_cat(int32_t nseg, const float *const *xs_dev, const long *xsg, const long *ldx,
                      const int32_t *widths, const float *w_dev, const float *b_dev, float *y_dev, long ysg, long ldy,
                      int32_t groups, int32_t m, int32_t n, int32_t act, void *stream);
/* td7_dense_fwd / td7_dense_fwd_cat (the same Linear + activation of
 * Agent/TD7_multi_agent.py:61-140) with W also given rounded to the MFMA
 * operand type (w16_dev: bf16 / fp16 bits, [G][N][K] contiguous, may be null):
 * the large-layer kernel loads it instead of rounding the fp32 W per slice --
 * bit-identical results. */
int td7_dense_fwd_w16(const float *x_dev, long xsg, long ldx, const float *w_dev, const float *b_dev, float *y_dev,
                      long ysg, long ldy, int32_t groups, int32_t m, int32_t n, int32_t k, int32_t act,
                      const uint16_t *w16_dev, void *stream);
int td7_dense_fwd_cat_w16(int32_t nseg, const float *const *xs_dev, const long *xsg, const long *ldx,
                          const int32_t *widths, const float *w_dev, const float *b_dev, float *y_dev, long ysg,
                          long ldy, int32_t groups, int32_t m, int32_t n, int32_t act, const uint16_t *w16_dev,
                          void *stream);
/* The same Linear + activation on an inference chain (select_action,
 * TD7_multi_agent.py:192-209 / Pink :209-228; no backward): X (x16_dev) and /
 * or Y (y16_dev) as 16-bit values of the MFMA operand type -- exactly what the
 * consumer rounds its operand to, so a chain is bit-identical with half the
 * activation bytes; the fp32 pointer of a 16-bit operand is null.  Only where
 * the large-layer kernels run (r05: the 256 x 256-tile kernels for 16-bit X
 * and W at >= 256 such tiles -- summed in another order than the 128 x 256
 * kernel the fp32 chain takes there, so within fp32 tolerance rather than
 * bit-identical) or, for a 16-bit X with an fp32 Y, where the fp32 path takes
 * the small-tile kernel (a narrow head: bit-identical): EXO_ERANGE otherwise
 * (the caller falls back to fp32).  w16_dev required. */
int td7_dense_fwd_h(const float *x_dev, const uint16_t *x16_dev, long xsg, long ldx, const float *w_dev,
                    const float *b_dev, float *y_dev, uint16_t *y16_dev, long ysg, long ldy, int32_t groups, int32_t m,
                    int32_t n, int32_t k, int32_t act, const uint16_t *w16_dev, void *stream);
/* The 256 x 256-tile forward kernel of td7_dense_fwd_h / _cat_h (no
 * reference counterpart: kernel selection for same-process A/Bs): 0 the
 * 128 x 256 big kernel, 1 dense_fwd_xl_kernel, 2 dense_fwd_xl8_kernel (two
 * 64-deep LDS-DMA slices); the environment's EXO_FWD_XL is the default.
 * Returns the previous setting or EXO_EINVAL. */
int td7_dense_set_xl(int32_t variant);
/* td7_dense_fwd_cat_h: xs16 = 1 takes every segment as 16-bit values (the
 * AvgL1Norm outputs of td7_avgl1norm_fwd_h), 0 as fp32. */
int td7_dense_fwd_cat_h(int32_t nseg, const void *const *xs_dev, int32_t xs16, const long *xsg, const long *ldx,
                        const int32_t *widths, const float *w_dev, const float *b_dev, uint16_t *y16_dev, long ysg,
                        long ldy, int32_t groups, int32_t m, int32_t n, int32_t act, const uint16_t *w16_dev,
                        void *stream);

/* y = AvgL1Norm(X W^T + b) per output row (Agent/TD7_multi_agent.py:53-54
 * after a Linear without activation, :61 / :103 / :126), N <= 320: one launch
 * for td7_dense_fwd + td7_avgl1norm_fwd.  Layout as td7_dense_fwd; h_dev
 * (pre-norm, y's layout) and mean_dev ([G][M], the raw mean |h| of
 * td7_avgl1norm_fwd) are written when non-null.  prec: MFMA operand precision
 * (0 fp32, 1 bf16, 2 fp16). */
int td7_dense_fwd_norm(const float *x_dev, long xsg, long ldx, const float *w_dev, const float *b_dev, float *y_dev,
                       float *h_dev, float *mean_dev, long ysg, long ldy, int32_t groups, int32_t m, int32_t n,
                       int32_t k, int32_t prec, float eps, void *stream);
/* td7_dense_fwd_norm of a concatenated input (td7_dense_fwd_cat's segments). */
int td7_dense_fwd_norm_cat(int32_t nseg, const float *const *xs_dev, const long *xsg, const long *ldx,
                           const int32_t *widths, const float *w_dev, const float *b_dev, float *y_dev, float *h_dev,
                           float *mean_dev, long ysg, long ldy, int32_t groups, int32_t m, int32_t n, int32_t prec,
                           float eps, void *stream);

/* td7_dense_bwd_weight of a layer whose input is given by segments (the
 * layout of td7_dense_fwd_cat); N >= 4. */
int td7_dense_bwd_weight_cat(const float *dy_dev, long dysg, long lddy, const float *y_dev, long ysg, long ldy,
                             int32_t nseg, const float *const *xs_dev, const long *xsg, const long *ldx,
                             const int32_t *widths, float *dw_dev, float *db_dev, int32_t groups, int32_t m, int32_t n,
                             int32_t act, void *stream);

/* The same for the input columns [c0, c1) only (the slice of a concatenated
 * input that requires a gradient, e.g. the critic's q part, :123-126); the
 * other columns of dX are not written. */
int td7_dense_bwd_data_cols(const float *dy_dev, long dysg, long lddy, const float *y_dev, long ysg, long ldy,
                            const float *w_dev, float *dx_dev, long dxsg, long lddx, int32_t groups,
                            int32_t shared_input, int32_t m, int32_t n, int32_t k, int32_t c0, int32_t c1, int32_t act,
                            void *stream);
/* dW[g] = (dY * act'(Y))^T X  [G][N][K]; db[g] = its column sums [G][N] (db may be NULL). */
int td7_dense_bwd_weight(const float *dy_dev, long dysg, long lddy, const float *y_dev, long ysg, long ldy,
                         const float *x_dev, long xsg, long ldx, float *dw_dev, float *db_dev, int32_t groups,
                         int32_t m, int32_t n, int32_t k, int32_t act, void *stream);

/* ---------------------------------------------------------------------------
 * Row-tile-fused TD7 networks (csrc/td7_fused.hip), bf16 / fp16 / fp32 MFMA
 * operands (prec 1 / 2 / 3).  One workgroup owns 16 (select: 32) rows and runs
 * a whole network pass of Agent/TD7_multi_agent.py on them with the
 * activations in LDS; weights are read from packed copies in the operand type
 * (td7f_pack, refreshed after every optimiser step / target copy).  Widths:
 * hidden <= 320, inputs <= 1,008.  A k-step is 32 inputs of a 16-bit operand
 * or 16 of an fp32 one (64 bytes per row either way): "kd" below. */
#define TD7F_PD 5          /* k-steps of weight loads in flight; packed k-steps are multiples of it */
#define TD7F_MAX_PACK 32

/* One nn.Linear: packed operands + fp32 bias.  ksf = k-steps of the forward
 * operand (ceil(n_in/kd) rounded up to TD7F_PD), ksb = k-steps of the dX
 * operand (ceil(n_out/kd) rounded up to TD7F_PD). */
typedef struct {
    const void *wf;
    const void *wb;
    const float *b;
    int32_t n_out, n_in, ksf, ksb;
    const float *w; /* fp32 master weight [n_out][n_in] (row stride ldw): the thin (<= 16 wide) products */
    int64_t ldw;
} td7f_lin;

/* Pack one fp32 weight [n_out][n_in] (row stride ld floats) into the forward
 * operand wf (ntf tiles x ksf k-steps x 64 lanes x 16 B) and, when wb is not
 * NULL, the dX operand wb (ntb tiles x ksb k-steps x 64 x 16 B); zero padded. */
typedef struct {
    const float *w;
    int64_t ld;
    int32_t n_out, n_in;
    void *wf;
    void *wb;
    int32_t ksf, ntf, ksb, ntb;
} td7f_pack_job;

/* In-kernel Gaussian noise of td7_noisy_action_rng (same stream, same element
 * order): out = clamp(a + c(z * sigma), -1, 1) * scale, then sigma -= sigma_dec
 * and the call counter advances (last workgroup out, ticket).  z non-NULL:
 * the standard normals are given (z[row * A + c], td7_noisy_action) and the
 * counter is left alone. */
typedef struct {
    uint64_t seed;
    uint32_t tag, pad0;
    unsigned long long *counter;
    uint32_t *ticket;
    float *sigma;
    float sigma_dec, clip, scale;
    int32_t pad1;
    const float *z;
    const int32_t *dec_count; /* non-NULL: sigma -= sigma_dec * *dec_count (td7_noisy_action_rng) */
} td7f_noise;

/* Activation codes of the three nets: act[0] encoder, act[1] actor, act[2] critic (1 relu, 2 elu). */
int td7f_pack(int32_t prec, int32_t njobs, const td7f_pack_job *jobs, void *stream);
/* td7_adam_step_multi (same arguments, same results bit for bit) fused with
 * td7f_pack of the weights it changes: job q packs the fp32 weight jobs[q].w,
 * a contiguous [n_out][n_in] block (ld == n_in) inside segment job_seg[q] of
 * its optimiser, from the updated values.  A segment is covered exactly by its
 * jobs or by none (EXO_EINVAL otherwise).  The optimiser step of
 * Agent/TD7_multi_agent.py:253-255 / :277 followed by the repack the fused
 * passes need, as one launch. */
#define TD7F_MAX_ADAM_PACK 16
int td7f_adam_pack(int32_t prec, int32_t nopt, float *const *p_dev, float *const *m_dev, float *const *v_dev,
                   float *const *step_dev, const float *lr, const float *beta1, const float *beta2, const float *eps,
                   const float *weight_decay, int32_t nseg, const float *const *g_dev, const int64_t *off,
                   const int32_t *n, const int32_t *opt, int32_t njobs, const td7f_pack_job *jobs,
                   const int32_t *job_seg, uint32_t *ticket_dev, void *stream);
/* Plan-only mode for the calling host thread (on != 0): every td7f_* pass
 * below validates its arguments and its shared-memory plan and returns without
 * launching (EXO_EINVAL when a network shape's images do not fit one
 * workgroup's LDS).  The host side probes each pass once when it builds the
 * fused passes for a learner (TD7_multi_agent.py:148-190, Agent.__init__) and
 * keeps the per-layer kernels for a shape the fused plan cannot hold. */
int td7f_probe(int32_t on);
/* Agent.select_action_batch (TD7_multi_agent.py:192-209 batched): actor(obs,
 * fixed_encoder.zs(obs)) + Gaussian exploration noise -> act_out [n][A].
 * enc: zs1..zs3, actor: l0..l3.  wg_cap > 0 (16-row tiles): at most that
 * many workgroups per launch, the tiles in back-to-back launches (same
 * results; the noise state advances once); 0: one launch.  The environment
 * variable EXO_SELECT_WG_CAP, when set, overrides wg_cap (experiments).
 * rt: rows per tile in units of 16 -- 0 picks (32 above 8,192 rows), 1 or 2
 * asks (16-bit operands; fp32 always 16); EXO_SELECT_RT overrides. */
int td7f_select(int32_t prec, const int32_t *act, const td7f_lin *enc, const td7f_lin *actor, const float *obs_dev,
                int32_t n, const td7f_noise *noise, float *act_out_dev, int32_t wg_cap, int32_t rt, void *stream);
/* td7f_select in two launches (r06): mode 1 computes fixed_encoder.zs(obs)
 * (TD7_multi_agent.py:93-97) and stores its normalised rows, in the operand
 * type, to zs_img_dev [n][zs_dim] (noise and act_out unused, the noise state
 * untouched); mode 2 runs the actor (:72-77) and the exploration noise from
 * that image.  Mode 1 then mode 2 with the same rt == td7f_select bit for
 * bit; the zs half needs only the fixed encoder, so a training loop can run
 * it before the actor step.  zs_dim <= 512, zs_dim and actor l0's width
 * even at 16-bit operands. */
int td7f_select_part(int32_t prec, const int32_t *act, const td7f_lin *enc, const td7f_lin *actor,
                     const float *obs_dev, int32_t n, const td7f_noise *noise, float *act_out_dev, int32_t wg_cap,
                     int32_t rt, void *zs_img_dev, int32_t mode, void *stream);
/* The critic target chain (TD7_multi_agent.py:233-241): fixed_target_zs(s'),
 * next_action = actor_target(s', zs) + clipped noise, fixed_target_zsa and both
 * heads of critic_target -> qt_dev [B][2].  tenc: zs1..zs3, zsa1..zsa3;
 * tcritic: [layer][head] (8).  tgt_img_dev: [B][round_up(2 zs_dim + A, 8)]
 * scratch in the operand type ([zsa | zs | next_action] per row). */
int td7f_target(int32_t prec, const int32_t *act, const td7f_lin *tenc, const td7f_lin *tactor,
                const td7f_lin *tcritic, const float *next_state_dev, int32_t B, const td7f_noise *noise,
                void *tgt_img_dev, float *qt_dev, void *stream);
/* fixed_zs = fixed_encoder.zs(state), fixed_zsa = fixed_encoder.zsa(fixed_zs,
 * action) (TD7_multi_agent.py:248-249) -> fp32 [B][zs_dim] each. */
int td7f_fixed(int32_t prec, const int32_t *act, const td7f_lin *fenc, const float *state_dev,
               const float *action_dev, int32_t B, float *zs_dev, float *zsa_dev, void *stream);

/* The gradient passes (csrc/td7_fused_train.hip).  Each leaves, per trained
 * layer, the transposed operands of its weight gradient (operand type) -- the
 * layer input X^T [round_up(n_in, 64)][ld] and dP^T = (dY act'(Y))^T
 * [round_up(n_out, 64)][ld] (x 1024 at fp16), ld = the batch padded to 256,
 * stored in 1 KiB MFMA-fragment blocks of 16 operand rows x kd batch rows
 * (csrc/td7_fused.h blk8 / blk4), padding zero -- and fp32 column sums of dP per 16-row tile (part
 * [ceil(B/16)][n_out]); td7f_wgrad turns them into dW and db. */
typedef struct {
    void *x;
    void *dp;
    float *part;
} td7f_xt;
/* Critic update (TD7_multi_agent.py:241-262): Q_target from the target heads
 * qt_dev [B][2] (clamp to [*lo, *hi], running bounds *run_max / *run_min
 * updated), both heads of the critic on [s, a] and [q | zsa | zs], |Q - Q_target|
 * -> td_dev [B][2] (the LAP priorities), the LAP-Huber gradient and the dX
 * chain of every layer.  critic: [layer][head] (8), with dX operands.  q_dev
 * (may be NULL): the Q values; y1/y2: [2][B][hdim] fp32 scratch.  xt: [layer][head]. */
int td7f_critic(int32_t prec, const int32_t *act, const td7f_lin *critic, const float *s_dev, const float *a_dev,
                const float *zs_dev, const float *zsa_dev, const float *qt_dev, const float *reward_dev,
                const float *not_done_dev, float discount, const float *lo_dev, const float *hi_dev,
                float *run_max_dev, float *run_min_dev, int32_t B, int32_t state_dim, int32_t action_dim,
                float *td_dev, float *q_dev, float *y1_dev, float *y2_dev, const td7f_xt *xt, int64_t ld,
                void *stream);
/* td7f_critic in two launches (the same results bit for bit): phase 1 the
 * critic forward (it needs only the batch and the fixed embeddings, so the
 * trainer runs it beside the target chain), storing Q, the pre-norm q0
 * output and the row means into q_ws [2][Bp], h0_ws [2][Bp][hdim], mean_ws
 * [2][Bp] (Bp = B rounded up to 16); phase 2 the loss from qt and the whole
 * backward from that state.  phase 0 = td7f_critic (workspaces unused). */
int td7f_critic_phase(int32_t phase, int32_t prec, const int32_t *act, const td7f_lin *critic, const float *s_dev,
                      const float *a_dev, const float *zs_dev, const float *zsa_dev, const float *qt_dev,
                      const float *reward_dev, const float *not_done_dev, float discount, const float *lo_dev,
                      const float *hi_dev, float *run_max_dev, float *run_min_dev, int32_t B, int32_t state_dim,
                      int32_t action_dim, float *td_dev, float *q_dev, float *y1_dev, float *y2_dev,
                      const td7f_xt *xt, int64_t ld, float *q_ws, float *h0_ws, float *mean_ws, void *stream);
/* Encoder update (TD7_multi_agent.py:219-228): zs(s') (no grad), zs(s),
 * zsa(zs, a), d mse / d pred and the dX chain of all six layers.  y: four
 * [B][enc_hdim] fp32 scratch buffers (zs1, zs2, zsa1, zsa2 activations).
 * nz_ws / flag_ws (both or neither): zs(s') on its own workgroup row --
 * nz_ws [ceil(B/16)*16][zs_dim] fp32 scratch, flag_ws [ceil(B/16)] int32,
 * zero at the first call and left zero. */
int td7f_encoder(int32_t prec, const int32_t *act, const td7f_lin *enc, const float *s_dev, const float *a_dev,
                 const float *ns_dev, int32_t B, float *const *y, const td7f_xt *xt, int64_t ld, float *nz_ws,
                 int32_t *flag_ws, void *stream);
/* Actor update (TD7_multi_agent.py:266-277) in three launches: phase 0 actor(s,
 * fixed_zs) and fixed_encoder.zsa of it; phase 1 the (updated) critic on them and
 * d(-mean Q) back to the action and zsa inputs per head; phase 2 the fixed zsa
 * backward to the action, tanh' and the actor's dX chain (xt: the 4 actor layers). */
typedef struct {
    float *act_out;  /* [B][A] */
    float *zsa_out;  /* [B][zs_dim] */
    float *h0;       /* [B][actor_hdim] pre-norm l0 output */
    float *mean0;    /* [B] */
    float *ya[2];    /* actor l1 / l2 activations [B][actor_hdim] */
    float *yz[2];    /* fixed zsa1 / zsa2 activations [B][enc_hdim] */
    float *yc[2];    /* critic l1 / l2 activations [2][B][critic_hdim] */
    float *da;       /* [2][B][A] */
    float *dzsa;     /* [2][B][zs_dim] */
} td7f_actor_bufs;
int td7f_actor(int32_t prec, int32_t phase, const int32_t *act, const td7f_lin *actor, const td7f_lin *fenc,
               const td7f_lin *critic, const float *s_dev, const float *zs_dev, int32_t B,
               const td7f_actor_bufs *bufs, const td7f_xt *xt, int64_t ld, void *stream);
/* dW = dP^T X / gs -> dw [n][k] (fp32, row stride k) and db = the column
 * partials summed over row_tiles (when db is not NULL), for njobs layers in one
 * launch; rows = the reduction length (multiple of 32).  prio_dev not NULL:
 * also the LAP priorities max(td0, td1, min_priority)^alpha (TD7_multi_agent.py:262). */
#define TD7F_MAX_WG 16
typedef struct {
    const void *dp;
    const void *x;
    const float *part;
    float *dw;
    float *db;
    int32_t n, k, row_tiles;
} td7f_wg_job;
int td7f_wgrad(int32_t prec, int32_t njobs, const td7f_wg_job *jobs, int64_t ld, int32_t rows, const float *td_dev,
               float *prio_dev, int32_t B, float alpha, float min_priority, void *stream);
/* Where job q's layer lives in its optimiser: W[0][0] and b[0] at flat offsets
 * w_off / b_off of optimiser opt's p / m / v; its packed operands (td7f_pack_job). */
typedef struct {
    int32_t opt;
    int64_t w_off, b_off;
    void *wf;
    void *wb;
    int32_t ksf, ksb;
} td7f_wg_adam;
/* td7f_wgrad followed by the optimiser step of every weight and bias the jobs
 * differentiate (every job needs db) and the repack of the updated weights,
 * in one launch: dw / db are still written, and p / m / v, the step counts
 * (nopt FlatAdams, td7_adam_step_multi's arguments) and the packed operands end
 * bit-identical to td7f_wgrad + td7_adam_step_multi + td7f_pack.  The weight
 * gradients, optimiser step and repack of TD7_multi_agent.py:253-255 / :275-277
 * as one node of the update's dependency chain; the caller makes sure the jobs
 * cover every parameter of the optimisers (torch's Adam steps all of them). */
int td7f_wgrad_adam(int32_t prec, int32_t njobs, const td7f_wg_job *jobs, int64_t ld, int32_t rows,
                    const float *td_dev, float *prio_dev, int32_t B, float alpha, float min_priority, int32_t nopt,
                    float *const *p_dev, float *const *m_dev, float *const *v_dev, float *const *step_dev,
                    const float *lr, const float *beta1, const float *beta2, const float *eps,
                    const float *weight_decay, const td7f_wg_adam *adam, uint32_t *ticket_dev, void *stream);

/* ---------------------------------------------------------- HIP runtime
 * No reference counterpart: a workaround for the ROCm 7.0 graph-launch defect
 * ("The graph-replay crash").  Creates n non-blocking streams on
 * the current device and keeps them for the life of the process, so that the
 * streams released by destroyed graph execs are replaced on the least-loaded
 * hardware queues.  Returns the number of ballast streams held (>= 0) or
 * EXO_E*.  exo_amd.graphs.release_graphs calls it after destroying execs. */
int exo_stream_ballast(int32_t n);
/* 1 + the sum over the nodes of a captured hipGraph_t of (dependents - 1): an
 * upper bound on its parallel branches, i.e. on the streams its exec owns
 * (diagnostic for the ballast count). */
int exo_graph_branch_bound(void *graph, int32_t *out);

#ifdef __cplusplus
}
#endif
#endif /* EXO_AMD_H */
