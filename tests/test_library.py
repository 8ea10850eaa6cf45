"""libexo_amd.so builds for gfx950, loads, and exports every symbol that
include/exo_amd.h declares.  No device calls (CPU-only container)."""
import ctypes
import os
import re
import subprocess

import pytest

from helpers import PKG, REPO

HEADER = os.path.join(REPO, "include", "exo_amd.h")
LIB = os.path.join(PKG, "exo_amd", "_lib", "libexo_amd.so")


def declared_functions():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    names = re.findall(r"^[A-Za-z_][\w\s\*]*?\b((?:exo|lap)_\w+)\s*\(", src, flags=re.M)
    return sorted(set(names))


@pytest.fixture(scope="module")
def lib():
    subprocess.run(["make", "-s", "-j4", "-C", os.path.join(PKG, "csrc")], check=True)
    return ctypes.CDLL(LIB)


def test_header_declares_the_boundary():
    names = declared_functions()
    for required in ["exo_create", "exo_reset", "exo_reset_from_draws", "exo_step", "exo_destroy", "exo_last_error",
                     "exo_get_state_host", "exo_set_state_host", "lap_init", "lap_add", "lap_sample", "lap_update",
                     "lap_reset_max"]:
        assert required in names


def test_library_exports_every_declared_symbol(lib):
    out = subprocess.run(["nm", "-D", "--defined-only", LIB], capture_output=True, text=True, check=True).stdout
    exported = set(re.findall(r"\sT\s(\w+)", out))
    missing = [n for n in declared_functions() if n not in exported]
    assert not missing, missing
    for n in declared_functions():
        getattr(lib, n)


def test_code_object_targets_gfx950(lib):
    blob = open(LIB, "rb").read()
    assert b"amdgcn-amd-amdhsa--gfx950" in blob
    assert b"exo_step_kernel" in blob and b"lap_sample_kernel" in blob


def test_python_binding_signatures_cover_the_header():
    import exo_amd._native as nat
    assert set(declared_functions()) <= set(nat.EXPORTS), set(declared_functions()) - set(nat.EXPORTS)


def test_product_refuses_to_run_without_gpu():
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    from exo_amd import VecExoskeletonEnv
    with pytest.raises(RuntimeError, match="no CPU fallback"):
        VecExoskeletonEnv(8)
