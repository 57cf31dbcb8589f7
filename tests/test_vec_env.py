"""MgxVecEnv (the SB3 VecEnv drop-in, mgx/vec_env.py) against a VecEnv built
from the C oracle + the numpy SB3 layer: obs, rewards, dones and every info
field (terminal_observation, TimeLimit.truncated, Monitor episode r/l), plus
SB3's reset semantics (first reset seeded, later resets unseeded unless
VecEnv.seed() was called; mission_done / stored reward persist, Q2)."""
import numpy as np
import pytest

torch = pytest.importorskip("torch")

pytestmark = pytest.mark.gpu


class OracleVecEnv:
    """SubprocVecEnv(Monitor(make_env)) + VecTransposeImage + VecFrameStack, restated."""

    def __init__(self, n, n_stack, **kw):
        import oracle as O
        self.O = O
        self.v = O.OracleVec(n_envs=n, **kw)
        self.fs = O.FrameStackOracle(n, n_stack)
        self.n = n
        self.ep_len = np.zeros(n, np.int64)

    def _raw(self, img, d, m):
        O = self.O
        return dict(image=O.vec_transpose_image(img), direction=O.one_hot_dir(d), mission=m.astype(np.int64))

    def reset(self, seed="init"):
        r = self.v.reset(seed)
        self.ep_len[:] = 0
        return self.fs.reset(self._raw(r["image"], r["dir"], r["mission"]))

    def step(self, actions):
        o = self.v.step(actions)
        done = (o["terminated"] | o["truncated"]).astype(bool)
        self.ep_len += 1
        cur = self._raw(np.where(done[:, None, None, None], o["r_image"], o["image"]),
                        np.where(done, o["r_dir"], o["dir"]), np.where(done[:, None], o["r_mission"], o["mission"]))
        obs, term = self.fs.step(cur, done, self._raw(o["image"], o["dir"], o["mission"]))
        infos = [{} for _ in range(self.n)]
        for i in np.nonzero(done)[0]:
            infos[i] = {"TimeLimit.truncated": bool(o["truncated"][i] and not o["terminated"][i]),
                        "terminal_observation": {k: v[i] for k, v in term.items()},
                        "episode": {"r": round(float(o["reward"][i]), 6), "l": int(self.ep_len[i])}}
        self.ep_len[done] = 0
        return obs, o["reward"].astype(np.float32), done, infos


def _same_obs(a, b):
    return all(np.array_equal(np.asarray(a[k]).astype(np.int64), np.asarray(b[k]).astype(np.int64)) for k in b)


@pytest.mark.parametrize("problem,mission,size,n_stack", [("multi", 5, 8, 4), ("multi", None, 11, 4),
                                                          ("pkp", 2, 8, 3)])
def test_vec_env_matches_sb3_stack(problem, mission, size, n_stack):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from mgx import MgxVecEnv
    n, T = 256, 160
    kw = dict(problem=problem, mission=mission, size=size, num_objects=4, seed=42)
    ref = OracleVecEnv(n, n_stack, **kw)
    env = MgxVecEnv(n, n_frames_stack=n_stack, **kw)
    assert env.num_envs == n and env.action_space.n == 7
    assert env.observation_space["image"].shape == (3 * n_stack, 7, 7)
    rng = np.random.default_rng(17)

    def run(steps):
        for t in range(steps):
            a = rng.integers(0, 7, n)
            o1, r1, d1, i1 = env.step(a)
            o2, r2, d2, i2 = ref.step(a.astype(np.int32))
            assert _same_obs(o1, o2), t
            assert np.array_equal(r1, r2) and r1.dtype == np.float32, t
            assert np.array_equal(d1, d2) and d1.dtype == bool, t
            for i in np.nonzero(d2)[0]:
                assert i1[i]["TimeLimit.truncated"] == i2[i]["TimeLimit.truncated"], (t, i)
                assert _same_obs(i1[i]["terminal_observation"], i2[i]["terminal_observation"]), (t, i)
                assert i1[i]["episode"]["r"] == i2[i]["episode"]["r"], (t, i)
                assert i1[i]["episode"]["l"] == i2[i]["episode"]["l"], (t, i)
            assert all(not x for j, x in enumerate(i1) if not d1[j])

    assert _same_obs(env.reset(), ref.reset())
    run(T)
    # a later VecEnv.reset() is unseeded: both streams continue from the current episode
    assert _same_obs(env.reset(), ref.reset(None))
    run(40)
    # VecEnv.seed(s) -> the next reset re-seeds PCG64 with s + i; MT continues
    seeds = env.seed(1000)
    assert seeds[:2] == [1000, 1001]
    assert _same_obs(env.reset(), ref.reset(1000))
    run(40)
    a, b = env.engine.dump_state(), ref.v.dump()
    for k in ("grid", "agent", "mission_done", "mtwords", "pcg"):
        assert np.array_equal(a[k], b[k]), k
    env.close()


class TransposeStack:
    """src/ppo.py:125-126 restated over a raw VecEnv: VecTransposeImage (image HWC -> CHW, the
    infos' terminal_observation too), then VecFrameStack(n_stack, 'first') (roll, zero done
    envs' stacks, re-stack terminal_observation) -- SB3 2.x semantics, unpinned."""

    def __init__(self, venv, n_stack):
        import oracle as O
        self.O, self.venv = O, venv
        self.fs = O.FrameStackOracle(venv.num_envs, n_stack)
        self.num_envs = venv.num_envs

    def _t(self, obs):
        return dict(image=self.O.vec_transpose_image(obs["image"]), direction=obs["direction"],
                    mission=obs["mission"].astype(np.int64))

    def reset(self):
        return self.fs.reset(self._t(self.venv.reset()))

    def step(self, a):
        o, r, d, infos = self.venv.step(a)
        cur = self._t(o)
        term_frames = {k: np.zeros_like(v) for k, v in cur.items()}
        for i in np.nonzero(d)[0]:
            t = self._t({k: np.asarray(v)[None] for k, v in infos[i]["terminal_observation"].items()})
            for k in t:
                term_frames[k][i] = t[k][0]
        obs, term = self.fs.step(cur, d, term_frames)
        for i in np.nonzero(d)[0]:
            infos[i] = dict(infos[i])
            infos[i]["terminal_observation"] = {k: v[i] for k, v in term.items()}
        return obs, r, d, infos


@pytest.mark.parametrize("problem,mission,size,n_stack", [("multi", 5, 8, 4), ("multi", None, 11, 2)])
def test_raw_mode_under_sb3_wrappers_matches_reference_stack(problem, mission, size, n_stack):
    """MgxVecEnv(raw=True) -- the drop-in for make_vec_env alone (ppo.py:118-122) -- hands out the
    wrapped env's own observation (image HWC (7,7,3), one-hot direction, int64 tokens) and raw
    terminal observations, so the reference's unchanged lines 124-126 stack it: that chain must
    equal the SubprocVecEnv + VecTransposeImage + VecFrameStack restatement over the C oracle in
    every obs, reward, done and info."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from mgx import MgxVecEnv
    n, T = 192, 160
    kw = dict(problem=problem, mission=mission, size=size, num_objects=4, seed=42)
    ref = OracleVecEnv(n, n_stack, **kw)
    raw = MgxVecEnv(n, raw=True, **kw)
    sp = raw.observation_space
    assert sp["image"].shape == (7, 7, 3) and sp["direction"].shape == (4,) and sp["mission"].shape == (32,)
    env = TransposeStack(raw, n_stack)
    assert _same_obs(env.reset(), ref.reset())
    rng = np.random.default_rng(23)
    for t in range(T):
        a = rng.integers(0, 7, n)
        o1, r1, d1, i1 = env.step(a)
        o2, r2, d2, i2 = ref.step(a.astype(np.int32))
        assert _same_obs(o1, o2), t
        assert np.array_equal(r1, r2) and np.array_equal(d1, d2), t
        for i in np.nonzero(d2)[0]:
            assert i1[i]["TimeLimit.truncated"] == i2[i]["TimeLimit.truncated"], (t, i)
            assert _same_obs(i1[i]["terminal_observation"], i2[i]["terminal_observation"]), (t, i)
            assert i1[i]["episode"]["l"] == i2[i]["episode"]["l"], (t, i)
    raw.close()


@pytest.mark.parametrize("n_frames_stack,recurrent", [(1, False), (4, True)])
def test_raw_mode_direction_is_discrete_without_discrete2box(n_frames_stack, recurrent):
    """make_env adds Discrete2BoxWrapper only when n_frames_stack > 1 and not recurrent
    (environment.py:28-29): otherwise the raw env's direction is MiniGridEnv's Discrete(4), an int per
    env -- obs and terminal_observation -- equal to the C oracle's agent direction."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import oracle as O
    from mgx import MgxVecEnv
    n, T = 128, 96
    kw = dict(problem="multi", mission=None, size=8, num_objects=4, seed=42)
    ref = O.OracleVec(n_envs=n, **kw)
    env = MgxVecEnv(n, raw=True, n_frames_stack=n_frames_stack, recurrent=recurrent, **kw)
    sp = env.observation_space["direction"]
    assert getattr(sp, "n", None) == 4 and tuple(sp.shape) == ()
    o = env.reset()
    r = ref.reset()
    assert o["direction"].shape == (n,) and o["direction"].dtype == np.int64
    assert np.array_equal(o["direction"], r["dir"]) and np.array_equal(o["image"], r["image"])
    rng = np.random.default_rng(31)
    for t in range(T):
        a = rng.integers(0, 7, n)
        o, rew, d, infos = env.step(a)
        w = ref.step(a.astype(np.int32))
        done = (w["terminated"] | w["truncated"]).astype(bool)
        assert np.array_equal(d, done), t
        assert np.array_equal(o["direction"], np.where(done, w["r_dir"], w["dir"])), t
        assert np.array_equal(o["image"], np.where(done[:, None, None, None], w["r_image"], w["image"])), t
        for i in np.nonzero(done)[0]:
            to = infos[i]["terminal_observation"]
            assert int(to["direction"]) == int(w["dir"][i]) and np.array_equal(to["image"], w["image"][i]), (t, i)
    env.close()
