"""Generate the golden fixtures under tests/golden/ by EXECUTING THE REFERENCE.

Runs only in the build container (needs /root/reference).  The reference's own
`src/custom_env.py` + `src/environment.py` (make_env -> TokenizeVocabWrapper ->
Discrete2BoxWrapper) run unchanged on the clean-room minigrid/gymnasium
restatement in oracle/refshim (parity for that 3P layer is *unpinned*, see
DESIGN.md §Oracle).  The SB3 layer (SubprocVecEnv auto-reset, Monitor,
VecTransposeImage, VecFrameStack, DictRolloutBuffer GAE) is restated here from
SB3 2.x semantics -- also unpinned.

SubprocVecEnv semantics: every worker process runs
`random.seed(cfg.seed)` in PlaygroundEnv.__init__ (custom_env.py:82), so each
env owns an MT19937 seeded 42.  We reproduce this by giving env i its own
`random.Random(42)` and binding the reference module's imported `choice` /
`randint` (custom_env.py:4) to it around every call into env i.  Env i is
first reset with seed 42+i (make_vec_env(seed=42) / VecEnv.seed), later resets
are unseeded (PCG64 stream continues).

Usage:  python tests/golden/make_golden.py  [--quick]
"""
import argparse
import os
import random
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "oracle", "refshim"))

from loader import load_reference, make_cfg  # noqa: E402

# Live-lock policy (engine-defined; the reference would hang):
# a reset *attempt* may consume at most LIVELOCK_WORDS MT words.  The attempt
# that would draw word LIVELOCK_WORDS+1 is abandoned (exactly LIVELOCK_WORDS
# words consumed, PCG64 left where it is) and reset is re-run unseeded with
# both streams continuing.  Must equal MGX_LIVELOCK_WORDS in include/mgx.h.
LIVELOCK_WORDS = 4096


class LivelockError(RuntimeError):
    pass


class CountingRandom(random.Random):
    """random.Random whose 32-bit word consumption is counted.

    Overriding getrandbits keeps CPython's `_randbelow_with_getrandbits`
    (Random.__init_subclass__), i.e. identical draws to the stock generator.
    """

    def __init__(self, seed):
        self.words = 0
        self.reset_start = 0
        super().__init__(seed)

    def getrandbits(self, k):
        assert 0 < k <= 32
        if self.words - self.reset_start >= LIVELOCK_WORDS:
            raise LivelockError("reset attempt would exceed %d MT words" % LIVELOCK_WORDS)
        self.words += 1
        return super().getrandbits(k)


TYPE_IDX = {"empty": 1, "wall": 2, "door": 4, "key": 5, "ball": 6, "box": 7, "goal": 8, "lava": 9}


def encode_cell(v):
    """(type, colour, state, contains) of one world object (None -> empty)."""
    if v is None:
        return (1, 0, 0, 0)
    t, c, s = v.encode()
    contains = 0
    if v.type == "box" and v.contains is not None:
        contains = 1
    return (t, c, s, contains)


def encode_grid(grid):
    S = grid.width
    out = np.zeros((S, S, 4), np.uint8)   # [x][y][4]
    for x in range(S):
        for y in range(S):
            out[x, y] = encode_cell(grid.get(x, y))
    return out


def pcg_state(env):
    st = env.unwrapped.np_random.bit_generator.state
    s, inc = st["state"]["state"], st["state"]["inc"]
    m = (1 << 64) - 1
    return np.array([s >> 64, s & m, inc >> 64, inc & m, st["has_uint32"], st["uinteger"]],
                    dtype=np.uint64)


class RefVec:
    """N reference envs with SubprocVecEnv-style private MT streams."""

    def __init__(self, cfg, n, manual=False):
        self.ce, self.envm = load_reference()
        self.cfg = cfg
        self.n = n
        self.rngs = []
        self.envs = []
        for i in range(n):
            rng = CountingRandom(cfg.seed)
            self.rngs.append(rng)
            with self._bind(i):
                if manual:
                    # PlaygroundEnv(manual=True) -- make_env(manual=True)'s env (environment.py:12); the
                    # observation wrappers of the training path (TokenizeVocab + Discrete2Box, :22,29)
                    # instead of LLMDescriptionWrapper, so the fixture has the usual layout
                    env = self.ce.PlaygroundEnv(render_mode=None, cfg=cfg, manual=True)
                    env = self.envm.Discrete2BoxWrapper(self.envm.TokenizeVocabWrapper(env))
                    self.envs.append(env)
                else:
                    self.envs.append(self.envm.make_env("custom", None, cfg=cfg, manual=False))

    class _Bind:
        def __init__(self, outer, i):
            self.o, self.i = outer, i

        def __enter__(self):
            rng = self.o.rngs[self.i] if self.i < len(self.o.rngs) else None
            if rng is not None:
                self.o.ce.choice = rng.choice
                self.o.ce.randint = rng.randint

        def __exit__(self, *a):
            return False

    def _bind(self, i):
        return RefVec._Bind(self, i)

    def reset_env(self, i, seed=None):
        """Returns (obs, n_livelocked_attempts)."""
        rng = self.rngs[i]
        n_ll = 0
        while True:
            rng.reset_start = rng.words
            try:
                with self._bind(i):
                    obs, _ = self.envs[i].reset(seed=seed if n_ll == 0 else None)
                return obs, n_ll
            except LivelockError:
                n_ll += 1
                if n_ll > 1000:
                    raise

    def step_env(self, i, a):
        with self._bind(i):
            return self.envs[i].step(int(a))


def env_state(env):
    u = env.unwrapped
    ax, ay = (int(u.agent_pos[0]), int(u.agent_pos[1]))
    carry = encode_cell(u.carrying) if u.carrying is not None else (0, 0, 0, 0)
    rew = np.nan if u.reward is None else float(u.reward)
    return ax, ay, int(u.agent_dir), carry, int(u.step_count), int(bool(u.mission_done)), rew


def target_info(env):
    u = env.unwrapped
    tp = u.target_pos
    tx, ty = (255, 255) if tp is None else (int(tp[0]), int(tp[1]))
    ta = 255 if u.target_action is None else int(u.target_action)
    return tx, ty, ta


def run_config(name, cfg, n, T, seed_actions=1234, manual=False):
    S = cfg.env.size
    vec = RefVec(cfg, n, manual=manual)
    acts = np.random.default_rng(seed_actions).integers(0, 7, (T, n)).astype(np.int8)
    d = {}

    def alloc(key, shape, dtype, fill=0):
        d[key] = np.full(shape, fill, dtype)

    # per-reset records: index 0 = first reset, then one per (t, env) done
    alloc("reset0_image", (n, 7, 7, 3), np.uint8)
    alloc("reset0_dir", (n,), np.uint8)
    alloc("reset0_mission", (n, 32), np.uint8)
    alloc("reset0_grid", (n, S, S, 4), np.uint8)
    alloc("reset0_agent", (n, 3), np.uint8)
    alloc("reset0_target", (n, 3), np.uint8)
    alloc("reset0_mtwords", (n,), np.int64)
    alloc("reset0_pcg", (n, 6), np.uint64)
    for k, shape, dt in [
        ("image", (T, n, 7, 7, 3), np.uint8), ("dir", (T, n), np.uint8),
        ("mission", (T, n, 32), np.uint8), ("reward", (T, n), np.float64),
        ("terminated", (T, n), np.uint8), ("truncated", (T, n), np.uint8),
        ("agent", (T, n, 3), np.uint8), ("carrying", (T, n, 4), np.uint8),
        ("step_count", (T, n), np.int32), ("mission_done", (T, n), np.uint8),
        ("stored_reward", (T, n), np.float64), ("grid", (T, n, S, S, 4), np.uint8),
        ("r_image", (T, n, 7, 7, 3), np.uint8), ("r_dir", (T, n), np.uint8),
        ("r_mission", (T, n, 32), np.uint8), ("r_grid", (T, n, S, S, 4), np.uint8),
        ("r_agent", (T, n, 3), np.uint8), ("r_target", (T, n, 3), np.uint8),
        ("r_mtwords", (T, n), np.int64), ("r_pcg", (T, n, 6), np.uint64),
        ("livelock", (T, n), np.int32),
    ]:
        alloc(k, shape, dt)

    def dir_of(obs):
        return int(np.argmax(obs["direction"]))

    def rec_reset(prefix, idx, i, obs):
        env = vec.envs[i]
        u = env.unwrapped
        d[prefix + "image"][idx] = obs["image"]
        d[prefix + "dir"][idx] = dir_of(obs)
        d[prefix + "mission"][idx] = obs["mission"].astype(np.uint8)
        d[prefix + "grid"][idx] = encode_grid(u.grid)
        d[prefix + "agent"][idx] = (int(u.agent_pos[0]), int(u.agent_pos[1]), int(u.agent_dir))
        d[prefix + "target"][idx] = target_info(env)
        d[prefix + "mtwords"][idx] = vec.rngs[i].words
        d[prefix + "pcg"][idx] = pcg_state(env)

    alloc("reset0_livelock", (n,), np.int32)
    # PlaygroundEnv.llm_description of every reset (LLMDescriptionWrapper, environment.py:152-195):
    # (t, env, text) in reset order, t = -1 for the first reset
    descs = []
    for i in range(n):
        obs, nll = vec.reset_env(i, seed=cfg.seed + i)
        rec_reset("reset0_", i, i, obs)
        d["reset0_livelock"][i] = nll
        descs.append((-1, i, vec.envs[i].unwrapped.llm_description))
    missions = {}
    for t in range(T):
        for i in range(n):
            obs, r, term, trunc, _ = vec.step_env(i, acts[t, i])
            u = vec.envs[i].unwrapped
            missions[u.mission] = obs["mission"].astype(np.uint8)
            d["image"][t, i] = obs["image"]
            d["dir"][t, i] = dir_of(obs)
            d["mission"][t, i] = obs["mission"].astype(np.uint8)
            d["reward"][t, i] = float(r)
            d["terminated"][t, i] = bool(term)
            d["truncated"][t, i] = bool(trunc)
            ax, ay, adir, carry, sc, md, srew = env_state(vec.envs[i])
            d["agent"][t, i] = (ax, ay, adir)
            d["carrying"][t, i] = carry
            d["step_count"][t, i] = sc
            d["mission_done"][t, i] = md
            d["stored_reward"][t, i] = srew
            d["grid"][t, i] = encode_grid(u.grid)
            if term or trunc:
                obs2, nll = vec.reset_env(i)
                d["livelock"][t, i] = nll
                rec_reset("r_", (t, i), i, obs2)
                descs.append((t, i, vec.envs[i].unwrapped.llm_description))
    d["actions"] = acts
    d["desc_t"] = np.array([x[0] for x in descs], np.int32)
    d["desc_env"] = np.array([x[1] for x in descs], np.int32)
    d["desc_text"] = np.array([x[2] for x in descs])
    d["meta"] = np.array([S, n, T, cfg.seed, -1 if cfg.env.mission is None else cfg.env.mission,
                          cfg.env.num_objects], np.int64)
    d["problem"] = np.array(cfg.env.problem)
    d["env_flags"] = np.array([int(bool(cfg.env.see_through_walls)), int(bool(cfg.env.obstacles)),
                               int(bool(cfg.env.all_doors_open)), int(bool(manual))], np.int64)
    d["percent_obstacles"] = np.array(float(cfg.env.percent_obstacles), np.float64)
    names = sorted(missions)
    d["mission_names"] = np.array(names)
    d["mission_tokens"] = np.stack([missions[k] for k in names]) if names else np.zeros((0, 32), np.uint8)
    return d


CONFIGS = []
for m, tag in [(5, "gtg"), (0, "gto"), (2, "pkp"), (1, "tgl"), (None, "all")]:
    for S in (8, 11, 16):
        CONFIGS.append(("multi_%s_s%d" % (tag, S), dict(problem="multi", mission=m, size=S)))
for p in ("gtg", "gto", "pkp", "opn", "drp", "mov", "full"):
    CONFIGS.append(("single_%s_s8" % p, dict(problem=p, mission=None, size=8)))
# env features no shipped config enables (single.yaml:26-28): obstacles (custom_env.py:155-172)
# and see_through_walls=False (minigrid process_vis), alone and together
CONFIGS += [
    ("single_full_s11", dict(problem="full", mission=None, size=11)),
    ("single_mov_s16", dict(problem="mov", mission=None, size=16)),
    ("obst_single_gtg_s8", dict(problem="gtg", mission=None, size=8, obstacles=True)),
    ("obst_single_mov_s11", dict(problem="mov", mission=None, size=11, obstacles=True, percent_obstacles=0.2)),
    ("obst_multi_all_s8", dict(problem="multi", mission=None, size=8, obstacles=True)),
    ("obst_multi_all_s16", dict(problem="multi", mission=None, size=16, obstacles=True)),
    ("novis_multi_all_s8", dict(problem="multi", mission=None, size=8, see_through_walls=False)),
    ("novis_single_gto_s11", dict(problem="gto", mission=None, size=11, see_through_walls=False, num_objects=12)),
    ("novis_obst_multi_tgl_s16", dict(problem="multi", mission=1, size=16, see_through_walls=False,
                                      obstacles=True, percent_obstacles=0.1)),
    # crowded rooms (8 objects; the reference itself raises IndexError once locked doors have
    # taken enough of the 18 (type, colour) choices, e.g. at 18 objects)
    ("multi_all_s11_o8", dict(problem="multi", mission=None, size=11, num_objects=8)),
    # all_doors_open=True (shipped by distilling.yaml:27 and moe.yaml:23): no `locked` draw, an extra
    # `is_open` draw per door (custom_env.py:637-649, 882-928, 1326-...), open doors see-through /
    # passable / toggled shut.  2-, 3- and 4-room layouts come from the multi problems' randint(2,4).
    ("ado_multi_all_s8", dict(problem="multi", mission=None, size=8, all_doors_open=True)),
    ("ado_multi_all_s11", dict(problem="multi", mission=None, size=11, all_doors_open=True)),
    ("ado_multi_tgl_s16", dict(problem="multi", mission=1, size=16, all_doors_open=True)),
    ("ado_multi_gtg_s8", dict(problem="multi", mission=5, size=8, all_doors_open=True)),
    ("ado_single_opn_s8", dict(problem="opn", mission=None, size=8, all_doors_open=True)),
    # manual=True (make_env(manual=True), the LLMDescriptionWrapper / GUI path): a premature 'done'
    # is a no-op (custom_env.py:319-328), so episodes end only on goal / lava / completed missions /
    # the time limit
    ("manual_multi_all_s8", dict(problem="multi", mission=None, size=8, manual=True)),
    ("manual_multi_pkp_s11", dict(problem="multi", mission=2, size=11, manual=True)),
]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=16)
    ap.add_argument("--T", type=int, default=512)
    ap.add_argument("--only", default=None)
    args = ap.parse_args()
    out_dir = os.path.join(HERE, "traj")
    os.makedirs(out_dir, exist_ok=True)
    for name, kw in CONFIGS:
        if args.only and args.only not in name:
            continue
        t0 = time.time()
        kw = dict(kw)
        manual = kw.pop("manual", False)
        cfg = make_cfg(**kw)
        d = run_config(name, cfg, args.n, args.T, manual=manual)
        np.savez_compressed(os.path.join(out_dir, name + ".npz"), **d)
        print("%-22s %6.1fs resets=%d livelocks=%d" % (
            name, time.time() - t0, int((d["terminated"] | d["truncated"]).sum()),
            int(d["livelock"].sum() + d["reset0_livelock"].sum())), flush=True)


if __name__ == "__main__":
    main()
