"""ctypes front-end for the C oracle (oracle/mgx_oracle.c) + numpy restatement
of the SB3 layer (VecTransposeImage, VecFrameStack, GAE, per-minibatch
advantage normalisation).

TEST INFRASTRUCTURE / CHECKER ONLY -- imported by tests/, by
__graft_entry__.smoke() and by bench.py's cpu_baseline leg, never by the
product package.

SB3 semantics restated here (not vendored by the reference, unpinned;
SURVEY.md A.5 / A.9):
  * VecTransposeImage: image (7,7,3)[vx][vy][c] -> (3,7,7)[c][vx][vy]
  * VecFrameStack(n, 'first'): per key, roll left by C along axis 1, zero the
    stacks of done envs (after saving the terminal stack), write newest last.
  * DictRolloutBuffer.compute_returns_and_advantage: fp32 GAE, op order
    delta = ((r + (g*nv)*nnt) - V);  last = delta + (c*nnt)*last.
"""
import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "libmgx_oracle.so")

PROBLEMS = {"multi": 0, "full": 1, "gto": 2, "gtg": 3, "opn": 4, "pkp": 5, "drp": 6, "mov": 7}
LIVELOCK_WORDS = 4096   # == MGX_LIVELOCK_WORDS (include/mgx.h)

_lib = None


def build():
    subprocess.check_call(["make", "-s", "-C", HERE])


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH) or (
                os.path.getmtime(LIB_PATH) < os.path.getmtime(os.path.join(HERE, "mgx_oracle.c"))):
            build()
        L = ctypes.CDLL(LIB_PATH)
        P = ctypes.c_void_p
        L.orc_create.restype = P
        L.orc_create.argtypes = [ctypes.c_int] * 6 + [ctypes.c_int64, ctypes.c_int64, ctypes.c_int,
                                                      ctypes.c_int, ctypes.c_int, ctypes.c_double]
        L.orc_destroy.argtypes = [P]
        L.orc_set_manual.argtypes = [P, ctypes.c_int]
        L.orc_reset.argtypes = [P, ctypes.c_int64, ctypes.c_int64, P, P, P, P]
        L.orc_reset_ex.argtypes = [P, ctypes.c_int, ctypes.c_int64, ctypes.c_int64, P, P, P, P]
        L.orc_step.argtypes = [P] * 12
        L.orc_dump.argtypes = [P] * 10
        L.orc_bench.argtypes = [P, ctypes.c_int64, ctypes.c_uint64]
        L.orc_bench.restype = ctypes.c_int64
        L.orc_mission.restype = ctypes.c_char_p
        L.orc_mission.argtypes = [P, ctypes.c_int]
        L.orc_mt_words.argtypes = [ctypes.c_uint64, ctypes.c_int, P]
        L.orc_pcg_seed_state.argtypes = [ctypes.c_uint64, P]
        L.orc_pcg_integers.argtypes = [ctypes.c_uint64, ctypes.c_int, P, P, P]
        _lib = L
    return _lib


def _p(a):
    return None if a is None else a.ctypes.data_as(ctypes.c_void_p)


class OracleVec:
    """N independent reference-semantics envs (SubprocVecEnv seeding)."""

    def __init__(self, problem="multi", mission=5, size=8, num_objects=4, n_envs=16,
                 seed=42, index_offset=0, all_doors_open=False,
                 livelock_words=LIVELOCK_WORDS, see_through_walls=True, obstacles=False,
                 percent_obstacles=0.05, manual=False):
        self.L = lib()
        self.n, self.S, self.seed, self.offset = n_envs, size, seed, index_offset
        m = -1 if mission is None else int(mission)
        self.h = self.L.orc_create(PROBLEMS[problem], m, size, num_objects, int(all_doors_open),
                                   n_envs, seed, index_offset, livelock_words, int(see_through_walls),
                                   int(obstacles), float(percent_obstacles))
        if not self.h:
            raise ValueError("orc_create failed")
        if manual:
            self.L.orc_set_manual(self.h, 1)

    def close(self):
        if self.h:
            self.L.orc_destroy(self.h)
            self.h = None

    __del__ = close

    def _obs_bufs(self):
        n = self.n
        return (np.zeros((n, 7, 7, 3), np.uint8), np.zeros(n, np.uint8), np.zeros((n, 32), np.uint8))

    def reset(self, seed="init"):
        """VecEnv.reset(): seed="init" -> the configured seed; an int -> that seed
        (after VecEnv.seed); None -> unseeded (streams continue)."""
        img, d, m = self._obs_bufs()
        ll = np.zeros(self.n, np.int32)
        sd = self.seed if seed == "init" else (0 if seed is None else int(seed))
        self.L.orc_reset_ex(self.h, int(seed is not None), sd, self.offset, _p(img), _p(d), _p(m), _p(ll))
        return dict(image=img, dir=d, mission=m, livelock=ll)

    def step(self, actions):
        a = np.ascontiguousarray(actions, dtype=np.int32)
        assert a.shape == (self.n,)
        img, d, m = self._obs_bufs()
        rimg, rd, rm = self._obs_bufs()
        rew = np.zeros(self.n, np.float64)
        term = np.zeros(self.n, np.uint8)
        trunc = np.zeros(self.n, np.uint8)
        ll = np.zeros(self.n, np.int32)
        self.L.orc_step(self.h, _p(a), _p(img), _p(d), _p(m), _p(rew), _p(term), _p(trunc),
                        _p(rimg), _p(rd), _p(rm), _p(ll))
        return dict(image=img, dir=d, mission=m, reward=rew, terminated=term, truncated=trunc,
                    r_image=rimg, r_dir=rd, r_mission=rm, livelock=ll)

    def bench(self, steps, seed=1234):
        """`steps` random-action vectorised steps in C (orc_bench; CPU baseline leg) -> resets."""
        return int(self.L.orc_bench(self.h, int(steps), int(seed)))

    def dump(self):
        n, S = self.n, self.S
        out = dict(grid=np.zeros((n, S, S, 4), np.uint8), agent=np.zeros((n, 3), np.uint8),
                   carrying=np.zeros((n, 4), np.uint8), step_count=np.zeros(n, np.int32),
                   mission_done=np.zeros(n, np.uint8), stored_reward=np.zeros(n, np.float64),
                   mtwords=np.zeros(n, np.int64), pcg=np.zeros((n, 6), np.uint64),
                   target=np.zeros((n, 3), np.uint8))
        self.L.orc_dump(self.h, *[_p(out[k]) for k in (
            "grid", "agent", "carrying", "step_count", "mission_done", "stored_reward",
            "mtwords", "pcg", "target")])
        return out

    def mission(self, i):
        return self.L.orc_mission(self.h, i).decode()


# ------------------------------- RNG KAT hooks ---------------------------
def mt_words(seed, n):
    out = np.zeros(n, np.uint32)
    lib().orc_mt_words(seed, n, _p(out))
    return out


def pcg_seed_state(seed):
    out = np.zeros(4, np.uint64)
    lib().orc_pcg_seed_state(seed, _p(out))
    return out


def pcg_integers(seed, lo, hi):
    lo = np.ascontiguousarray(lo, np.int64)
    hi = np.ascontiguousarray(hi, np.int64)
    out = np.zeros(len(lo), np.int64)
    lib().orc_pcg_integers(seed, len(lo), _p(lo), _p(hi), _p(out))
    return out


# ------------------------------- SB3 layer --------------------------------
def vec_transpose_image(img_hwc):
    """(..., 7, 7, 3) [vx][vy][c] -> (..., 3, 7, 7)."""
    return np.ascontiguousarray(np.moveaxis(img_hwc, -1, -3))


def one_hot_dir(d):
    out = np.zeros(d.shape + (4,), np.uint8)
    np.put_along_axis(out, d[..., None].astype(np.int64), 1, axis=-1)
    return out


class FrameStackOracle:
    """VecFrameStack(n_stack, channels_order='first') over the dict obs
    {'image': (N,3,7,7) u8, 'direction': (N,4) u8, 'mission': (N,32) int64}."""

    def __init__(self, n_envs, n_stack=4):
        self.n, self.k = n_envs, n_stack
        self.stack = {
            "image": np.zeros((n_envs, 3 * n_stack, 7, 7), np.uint8),
            "direction": np.zeros((n_envs, 4 * n_stack), np.uint8),
            "mission": np.zeros((n_envs, 32 * n_stack), np.int64),
        }

    def reset(self, obs):
        for key, v in obs.items():
            s = self.stack[key]
            c = v.shape[1]
            s[...] = 0
            s[:, -c:] = v
        return {k: v.copy() for k, v in self.stack.items()}

    def step(self, obs, dones, terminal_obs):
        """obs = VecEnv obs (new-episode obs where done); terminal_obs = the
        env's final frame per key (read where done).  Returns
        (stacked_obs, terminal_stacked_obs) -- the latter valid where done."""
        term = {}
        for key, v in obs.items():
            s = self.stack[key]
            c = v.shape[1]
            s[...] = np.roll(s, shift=-c, axis=1)
            term[key] = np.concatenate([s[:, :-c], terminal_obs[key]], axis=1)
            s[dones] = 0
            s[:, -c:] = v
        return {k: v.copy() for k, v in self.stack.items()}, term


def gae(rewards, values, episode_starts, last_values, last_dones, gamma, gae_lambda):
    """DictRolloutBuffer.compute_returns_and_advantage, fp32 op order."""
    T, N = rewards.shape
    g = np.float32(gamma)
    c = np.float32(gamma * gae_lambda)
    adv = np.zeros((T, N), np.float32)
    last = np.zeros(N, np.float32)
    for t in range(T - 1, -1, -1):
        if t == T - 1:
            nnt = np.float32(1.0) - last_dones.astype(np.float32)
            nv = last_values.astype(np.float32)
        else:
            nnt = np.float32(1.0) - episode_starts[t + 1].astype(np.float32)
            nv = values[t + 1]
        delta = ((rewards[t] + (g * nv) * nnt) - values[t]).astype(np.float32)
        last = (delta + (c * nnt) * last).astype(np.float32)
        adv[t] = last
    ret = (adv + values).astype(np.float32)
    return adv, ret


def _splitmix64(x):
    """splitmix64 over a numpy uint64 array (mod 2^64)."""
    with np.errstate(over="ignore"):
        z = x + np.uint64(0x9E3779B97F4A7C15)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        return z ^ (z >> np.uint64(31))


def random_actions_ref(count, seed, counter, n_actions=7):
    """Restatement of mgx_random_actions (include/mgx.h, ABI 7): the synthetic random policy's actions of the launch
    that reads counter value `counter` -- no reference counterpart beyond env.action_space.sample() (uniform)."""
    with np.errstate(over="ignore"):
        key = _splitmix64(np.uint64(seed) + np.uint64(counter) * np.uint64(0x9E3779B97F4A7C15))
        i = np.arange(count, dtype=np.uint64)
        h = _splitmix64(key ^ (i * np.uint64(0xD1B54A32D192ED03)))
        return (((h >> np.uint64(32)) * np.uint64(n_actions)) >> np.uint64(32)).astype(np.int32)
