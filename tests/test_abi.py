"""The C-ABI library: it loads (after torch, sharing its HIP runtime), exports
every entry point include/mgx.h declares, and rejects invalid configurations
with the reference's error meaning -- all without touching a GPU."""
import ctypes
import os
import re
import subprocess

import pytest

from conftest import ROOT

HDR = os.path.join(ROOT, "include", "mgx.h")
LIB = os.path.join(ROOT, "minigrid-rl_amd", "mgx", "libmgx.so")


def declared():
    src = open(HDR).read()
    return sorted(set(re.findall(r"^\s*(?:mgx_status|int64_t|int|const char \*)\s*(mgx_\w+)\s*\(", src, re.M)))


def test_header_declares_expected_api():
    from mgx import _lib
    assert set(declared()) == set(_lib.EXPORTS)


@pytest.fixture(scope="module")
def lib():
    if not os.path.exists(LIB):
        subprocess.check_call(["make", "-s", "-C", os.path.join(ROOT, "minigrid-rl_amd")])
    from mgx import _lib
    return _lib.load()


def test_library_exports_every_declared_symbol(lib):
    out = subprocess.check_output(["nm", "-D", "--defined-only", LIB]).decode()
    syms = {ln.split()[-1] for ln in out.splitlines() if " T " in ln}
    missing = [s for s in declared() if s not in syms]
    assert not missing, missing
    for s in declared():
        assert getattr(lib, s) is not None


def test_library_is_gfx950_code_object():
    blob = open(LIB, "rb").read()
    assert b"amdgcn-amd-amdhsa--gfx950" in blob   # the embedded code-object bundle target


def test_invalid_configs_rejected_without_gpu(lib):
    from mgx import _lib
    P = _lib.PROBLEMS
    bad = [dict(problem=99), dict(size=3), dict(n_envs=0), dict(obstacles=1, percent_obstacles=1.5),
           dict(mission=3), dict(num_objects=19), dict(n_stack=0),
           # room too small for everything place_obj must place: the reference never returns
           dict(problem=P["full"], size=7), dict(problem=P["gtg"], size=5, num_objects=8),
           dict(problem=P["mov"], size=5, num_objects=7, obstacles=1, percent_obstacles=0.3),
           dict(problem=P["drp"], num_objects=25)]
    for kw in bad:
        c = _lib.MgxConfig(problem=0, mission=5, size=8, num_objects=4, see_through_walls=1, n_stack=4,
                           n_envs=64, base_seed=42)
        for k, v in kw.items():
            setattr(c, k, v)
        h = ctypes.c_void_p()
        st = lib.mgx_create(ctypes.byref(c), 0, ctypes.byref(h))
        assert st == 1, (kw, st)        # MGX_ERR_INVALID, before any HIP call
        assert lib.mgx_last_error()


def test_mission_text_table(lib):
    from mgx import _lib
    assert _lib.mission_text(3) == "go to goal"
    # cmd | colour-name << 2 | type-slot << 5
    assert _lib.mission_text(0 | (0 << 2) | (0 << 5)) == "go to blue door"
    assert _lib.mission_text(2 | (5 << 2) | (3 << 5)) == "pick up yellow box"
    assert _lib.mission_text(1 | (3 << 2) | (0 << 5)) == "toggle purple door"
    assert _lib.mission_text(128) == "drop"
    assert [_lib.mission_text(129 + d) for d in range(4)] == ["move left", "move right", "move up", "move down"]


def test_random_actions_rejects_bad_arguments_without_gpu(lib):
    """mgx_random_actions (ABI 7) refuses an empty batch, a null buffer / counter and n_actions outside
    [1, 65536] with MGX_ERR_INVALID before any HIP call."""
    dummy = ctypes.c_void_p(0x1000)                     # never dereferenced: the checks come first
    for out, count, na, ctr in [(dummy, 0, 7, dummy), (dummy, -5, 7, dummy), (None, 16, 7, dummy),
                                (dummy, 16, 7, None), (dummy, 16, 0, dummy), (dummy, 16, 65537, dummy)]:
        st = lib.mgx_random_actions(out, count, na, ctypes.c_uint64(1), ctr, None)
        assert st == 1, (count, na, st)                  # MGX_ERR_INVALID
        assert b"mgx_random_actions" in lib.mgx_last_error()
