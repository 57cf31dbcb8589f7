"""The engine's episode generator (minigrid-rl_amd/csrc/mgx_device.h: reset_env and everything under it)
compiled for the HOST (tests/host_gen, -DMGX_HOST_SIM, one env after the other) against the C oracle:
consecutive episodes of every env -- the seeded first reset, then resets continuing both RNG streams (the
oracle steps 'done', which ends every episode) -- must have the same grid, agent, mission target and id,
MT19937 cursor, PCG64 state and abandoned-attempt count.  A CPU check of the draw order for refill-kernel
changes in seconds; the kernels themselves are pinned by the -m gpu tests.  Test infrastructure only."""
import ctypes
import os
import subprocess

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
SRC = os.path.join(HERE, "host_gen", "gen_host.cpp")
HDRS = [os.path.join(ROOT, "minigrid-rl_amd", "csrc", h) for h in ("mgx_device.h", "mgx_diag.h")] + \
       [os.path.join(HERE, "host_gen", "host_sim.h")]
LIB = os.path.join(HERE, "host_gen", "libgen_host.so")


def _lib():
    if not os.path.exists(LIB) or any(os.path.getmtime(LIB) < os.path.getmtime(p) for p in [SRC] + HDRS):
        subprocess.check_call(["g++", "-O2", "-std=c++17", "-ffp-contract=off", "-shared", "-fPIC", "-DMGX_HOST_SIM",
                               "-I", os.path.join(HERE, "host_gen"), "-I", os.path.join(ROOT, "minigrid-rl_amd", "csrc"),
                               "-o", LIB, SRC])
    L = ctypes.CDLL(LIB)
    P = ctypes.c_void_p
    L.hg_run.argtypes = [ctypes.c_int] * 7 + [ctypes.c_int64, ctypes.c_int] + [P] * 6
    return L


def _p(a):
    return a.ctypes.data_as(ctypes.c_void_p)


def encode(codes, S):
    """engine cell codes [..., S*S] (y*S + x) -> the dump layout [..., S(x), S(y), 4]"""
    c = codes.reshape(codes.shape[:-1] + (S, S)).swapaxes(-1, -2).astype(np.int32)   # [.., x, y]
    t, col, aux = c & 15, (c >> 4) & 7, c >> 7
    state = np.where(t == 4, 1 + aux, 0)
    box_key = ((t == 7) & (aux == 1)).astype(np.int32)
    t = np.where(t == 11, 4, t)
    return np.stack([t, col, state, box_key], -1).astype(np.uint8)


PROBLEMS = {"multi": 0, "full": 1, "gto": 2, "gtg": 3, "opn": 4, "pkp": 5, "drp": 6, "mov": 7}
CASES = [("multi", 5, 8, 0, 0), ("multi", None, 8, 0, 0), ("multi", 1, 16, 0, 0), ("multi", 2, 11, 0, 0),
         ("multi", None, 8, 1, 0), ("multi", 0, 16, 1, 0), ("multi", None, 11, 0, 0), ("pkp", None, 8, 0, 0),
         ("gtg", None, 8, 0, 0), ("multi", None, 8, 0, 4), ("gtg", None, 8, 0, 1), ("mov", None, 8, 0, 2),
         ("full", None, 11, 0, 0), ("pkp", None, 11, 0, 3), ("opn", None, 16, 0, 0)]


@pytest.mark.parametrize("problem,mission,size,ado,nobst", CASES,
                         ids=["%s_%s_s%d_ado%d_obst%d" % c for c in CASES])
def test_host_generator_matches_oracle(problem, mission, size, ado, nobst):
    import oracle as O
    from mgx._lib import mission_tokens
    n, E, seed = 64, 24, 42
    S = size
    pct = 0.05 if nobst == 0 else nobst / float((size - 2) ** 2) + 1e-9
    n_obst = int(np.floor((size - 2) ** 2 * pct)) if nobst else 0
    L = _lib()
    grids = np.zeros((n, E, S * S), np.uint8)
    agent = np.zeros((n, E, 3), np.uint8)
    target = np.zeros((n, E, 4), np.uint8)
    cursor = np.zeros((n, E), np.int64)
    pcg = np.zeros((n, E, 4), np.uint64)
    ll = np.zeros((n, E), np.int32)
    err = L.hg_run(PROBLEMS[problem], -1 if mission is None else mission, S, 4, ado, n_obst, n, seed, E,
                   _p(grids), _p(agent), _p(target), _p(cursor), _p(pcg), _p(ll))
    assert err == 0, err
    ov = O.OracleVec(problem, mission, S, 4, n, seed, all_doors_open=bool(ado), obstacles=bool(nobst),
                     percent_obstacles=pct)
    r = ov.reset()
    tok = mission_tokens()
    g = encode(grids, S)
    for k in range(E):
        d = ov.dump()
        assert np.array_equal(g[:, k], d["grid"]), ("grid", k)
        assert np.array_equal(agent[:, k], d["agent"]), ("agent", k)
        assert np.array_equal(target[:, k, :3], d["target"]), ("target", k)
        assert np.array_equal(cursor[:, k], d["mtwords"]), ("mt cursor", k)
        assert np.array_equal(pcg[:, k, 0], d["pcg"][:, 0]) and np.array_equal(pcg[:, k, 1], d["pcg"][:, 1]), ("pcg", k)
        assert np.array_equal(pcg[:, k, 2], d["pcg"][:, 4]) and np.array_equal(pcg[:, k, 3], d["pcg"][:, 5]), ("pcg buf", k)
        assert np.array_equal(tok[target[:, k, 3]], r["mission"] if k == 0 else o["r_mission"]), ("mission", k)
        assert np.array_equal(ll[:, k], r["livelock"] if k == 0 else o["livelock"]), ("livelock", k)
        o = ov.step(np.full(n, 6, np.int32))                  # 'done': ends every episode, auto-reset
        assert (o["terminated"] | o["truncated"]).all()
