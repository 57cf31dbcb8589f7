"""Shared trajectory comparison against the golden fixtures (tests/golden/traj).

A fixture holds, per step t and env i, the reference's raw obs (image HWC,
direction, mission tokens), reward (fp64), terminated/truncated, the post-step
env state, and -- where the env finished -- the new episode's obs/state and
RNG positions.  `compare(source, fixture)` drives any source (the C oracle or
the HIP engine) with the fixture's actions and returns the first mismatch.
"""
import glob
import os

import numpy as np

from conftest import GOLDEN

STATE_KEYS = ("agent", "carrying", "step_count", "grid")


def fixtures():
    return sorted(glob.glob(os.path.join(GOLDEN, "traj", "*.npz")))


def fixture_cfg(d):
    S, n, T, seed, mission, nobj = [int(x) for x in d["meta"]]
    flags = [int(x) for x in d["env_flags"]] if "env_flags" in d else [1, 0]
    stw, obst = flags[0], flags[1]
    ado = flags[2] if len(flags) > 2 else 0          # all_doors_open (third flag, added in round 2)
    manual = flags[3] if len(flags) > 3 else 0       # PlaygroundEnv(manual=True) (fourth flag, round 3)
    pct = float(d["percent_obstacles"]) if "percent_obstacles" in d else 0.05
    cfg = dict(problem=str(d["problem"]), mission=None if mission < 0 else mission, size=S,
               num_objects=nobj, n_envs=n, seed=seed, see_through_walls=bool(stw), obstacles=bool(obst),
               percent_obstacles=pct, all_doors_open=bool(ado))
    if manual:
        cfg["manual"] = True
    return cfg, T


def _eq(a, b):
    a = np.asarray(a)
    b = np.asarray(b)
    if a.dtype.kind == "f":
        return np.array_equal(a, b, equal_nan=True)
    return np.array_equal(a, b)


def compare(src, d, T=None, check_state=True):
    """src: object with reset() -> dict(image HWC [n,7,7,3], dir [n], mission [n,32], livelock [n]),
    step(actions) -> dict(image, dir, mission, reward f64, terminated, truncated,
                          r_image, r_dir, r_mission, livelock) and dump() -> state dict.
    Returns None when identical, else a message."""
    _, T_all = fixture_cfg(d)
    T = T_all if T is None else min(T, T_all)
    r = src.reset()
    st = src.dump() if check_state else None
    checks = [("image", r["image"], d["reset0_image"]), ("dir", r["dir"], d["reset0_dir"]),
              ("mission", r["mission"], d["reset0_mission"]), ("livelock", r["livelock"], d["reset0_livelock"])]
    if check_state:
        checks += [("grid", st["grid"], d["reset0_grid"]), ("agent", st["agent"], d["reset0_agent"]),
                   ("mtwords", st["mtwords"], d["reset0_mtwords"]), ("pcg", st["pcg"], d["reset0_pcg"]),
                   ("target", st["target"], d["reset0_target"])]
    for name, a, b in checks:
        if not _eq(a, b):
            return "first reset: %s differs (envs %s)" % (name, _diff_envs(a, b))
    for t in range(T):
        o = src.step(d["actions"][t].astype(np.int32))
        done = (d["terminated"][t] | d["truncated"][t]).astype(bool)
        checks = [(k, o[k], d[k][t]) for k in ("image", "dir", "mission", "reward", "terminated", "truncated")]
        checks += [("r_" + k, o["r_" + k][done], d["r_" + k][t][done]) for k in ("image", "dir", "mission")]
        checks.append(("livelock", o["livelock"], d["livelock"][t]))
        if check_state:
            st = src.dump()
            nd = ~done
            checks += [(k, st[k][nd], d[k][t][nd]) for k in STATE_KEYS]
            checks += [("mission_done", st["mission_done"], d["mission_done"][t]),
                       ("stored_reward", st["stored_reward"], d["stored_reward"][t]),
                       ("r_grid", st["grid"][done], d["r_grid"][t][done]),
                       ("r_agent", st["agent"][done], d["r_agent"][t][done]),
                       ("r_mtwords", st["mtwords"][done], d["r_mtwords"][t][done]),
                       ("r_pcg", st["pcg"][done], d["r_pcg"][t][done]),
                       ("r_target", st["target"][done], d["r_target"][t][done])]
        for name, a, b in checks:
            if not _eq(a, b):
                return "t=%d: %s differs" % (t, name)
    return None


def _diff_envs(a, b):
    a = np.asarray(a)
    b = np.asarray(b)
    if a.shape != b.shape:
        return "shape %s vs %s" % (a.shape, b.shape)
    m = (a != b).reshape(a.shape[0], -1).any(1)
    return np.nonzero(m)[0][:8].tolist()


class OracleSource:
    """The C oracle behind the compare() protocol."""

    def __init__(self, cfg):
        import oracle as O
        self.v = O.OracleVec(cfg["problem"], cfg["mission"], cfg["size"], cfg["num_objects"], cfg["n_envs"],
                             cfg["seed"], see_through_walls=cfg.get("see_through_walls", True),
                             obstacles=cfg.get("obstacles", False),
                             percent_obstacles=cfg.get("percent_obstacles", 0.05),
                             all_doors_open=cfg.get("all_doors_open", False), manual=cfg.get("manual", False))

    def reset(self):
        return self.v.reset()

    def step(self, a):
        return self.v.step(a)

    def dump(self):
        return self.v.dump()
