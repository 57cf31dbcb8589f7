"""MgxEngine: device-resident vectorised PlaygroundEnv (torch tensors in, torch
tensors out, no host round trip).

Mirrors the reference's env construction (`make_vec_env(make_env, n_envs,
seed, SubprocVecEnv)` + `VecTransposeImage` + `VecFrameStack(n_stack,
'first')`, src/ppo.py:118-126) behind one object whose `step` is one kernel
launch (libmgx `mgx_step`).  Observation tensors are updated IN PLACE every
step (the stacks roll); clone them if you keep them across steps.
"""
import ctypes

import torch

from . import _lib

_P = ctypes.c_void_p


def _ptr(t):
    return None if t is None else ctypes.c_void_p(t.data_ptr())


class MgxEngine:
    def __init__(self, problem="multi", mission=5, size=8, num_objects=4, n_envs=65536, seed=42,
                 env_index_offset=0, n_stack=4, all_doors_open=False, see_through_walls=True,
                 obstacles=False, percent_obstacles=0.05, terminal_mode="truncated", mission_dtype=torch.int64,
                 device="cuda", livelock_words=0, mt_table_words=0, reward64=False, ring_depth=0,
                 refill_every=0, refill_cap=0, manual=False):
        self.L = _lib.load()
        if not torch.cuda.is_available():
            raise _lib.MgxError("MgxEngine needs a GPU (no CPU fallback by design)")
        self.device = torch.device(device)
        if self.device.index is None:
            self.device = torch.device("cuda", torch.cuda.current_device())
        if problem not in _lib.PROBLEMS:
            raise ValueError("Invalid problem type given: %s" % problem)
        self.n = int(n_envs)
        self.size = int(size)
        self.n_stack = int(n_stack)
        self.seed = int(seed)
        self.env_index_offset = int(env_index_offset)
        cfg = _lib.MgxConfig()
        cfg.problem = _lib.PROBLEMS[problem]
        cfg.mission = -1 if mission is None else int(mission)
        cfg.size = self.size
        cfg.num_objects = int(num_objects)
        cfg.see_through_walls = int(bool(see_through_walls))
        cfg.all_doors_open = int(bool(all_doors_open))
        cfg.obstacles = int(bool(obstacles))
        cfg.percent_obstacles = float(percent_obstacles)
        cfg.n_stack = self.n_stack
        cfg.n_envs = self.n
        cfg.base_seed = self.seed
        cfg.env_index_offset = self.env_index_offset
        cfg.livelock_words = int(livelock_words)
        cfg.terminal_mode = _lib.TERMINAL[terminal_mode]
        cfg.mission_int64 = 1 if mission_dtype == torch.int64 else 0
        cfg.mt_table_words = int(mt_table_words)
        cfg.ring_depth = int(ring_depth)
        cfg.refill_every = int(refill_every)
        cfg.refill_cap = int(refill_cap)
        cfg.manual = int(bool(manual))
        self.manual = bool(manual)
        self.terminal_mode = terminal_mode
        self.mission_dtype = torch.int64 if cfg.mission_int64 else torch.uint8
        h = _P()
        _lib.check(self.L.mgx_create(ctypes.byref(cfg), self.device.index, ctypes.byref(h)), "mgx_create")
        self.h = h
        eff = _lib.MgxConfig()
        _lib.check(self.L.mgx_get_config(h, ctypes.byref(eff)), "mgx_get_config")
        self.ring_depth = int(eff.ring_depth)          # 0 = no ring (inline resets)
        self.refill_every = int(eff.refill_every)      # K: steps per refill epoch
        self.calls = 0                                 # mgx_step calls since the last reset()
        n, k, dev = self.n, self.n_stack, self.device
        self.obs = dict(image=torch.zeros((n, 3 * k, 7, 7), dtype=torch.uint8, device=dev),
                        direction=torch.zeros((n, 4 * k), dtype=torch.uint8, device=dev),
                        mission=torch.zeros((n, 32 * k), dtype=self.mission_dtype, device=dev))
        if terminal_mode != "none":
            self.terminal_obs = {kk: torch.zeros_like(v) for kk, v in self.obs.items()}
        else:
            self.terminal_obs = None
        self.reward = torch.zeros(n, dtype=torch.float32, device=dev)
        self.reward64 = torch.zeros(n, dtype=torch.float64, device=dev) if reward64 else None
        self.terminated = torch.zeros(n, dtype=torch.bool, device=dev)
        self.truncated = torch.zeros(n, dtype=torch.bool, device=dev)
        self.done = torch.zeros(n, dtype=torch.bool, device=dev)
        self.ep_return = torch.zeros(n, dtype=torch.float32, device=dev)
        self.ep_len = torch.zeros(n, dtype=torch.int32, device=dev)
        self.livelock = torch.zeros(n, dtype=torch.int32, device=dev)
        self._obs_c = _lib.MgxObs(_ptr(self.obs["image"]), _ptr(self.obs["direction"]), _ptr(self.obs["mission"]))
        so = _lib.MgxStepOut()
        so.obs = self._obs_c
        if self.terminal_obs is not None:
            so.terminal = _lib.MgxObs(_ptr(self.terminal_obs["image"]), _ptr(self.terminal_obs["direction"]),
                                      _ptr(self.terminal_obs["mission"]))
        so.reward_dev = _ptr(self.reward)
        so.reward64_dev = _ptr(self.reward64)
        so.terminated_dev = _ptr(self.terminated)
        so.truncated_dev = _ptr(self.truncated)
        so.done_dev = _ptr(self.done)
        so.ep_return_dev = _ptr(self.ep_return)
        so.ep_len_dev = _ptr(self.ep_len)
        so.livelock_dev = _ptr(self.livelock)
        self._step_out = so

    # ------------------------------------------------------------------
    def _stream(self):
        return ctypes.c_void_p(torch.cuda.current_stream(self.device).cuda_stream)

    def set_seed(self, seed):
        """VecEnv.seed: the next reset() seeds env i's PCG64 with seed + env_index_offset + i."""
        _lib.check(self.L.mgx_set_seed(self.h, int(seed)), "mgx_set_seed")
        self.seed = int(seed)

    def reset(self):
        """Seeded reset of every env: env i <- seed + env_index_offset + i (MT cursor 0)."""
        _lib.check(self.L.mgx_reset(self.h, ctypes.byref(self._obs_c), _ptr(self.livelock), self._stream()),
                   "mgx_reset")
        self.calls = 0
        return self.obs

    def step(self, actions):
        """actions: int32/int64 device tensor [N].  Returns the in-place obs dict;
        reward/terminated/truncated/done/ep_return/ep_len are attributes."""
        if actions.device != self.device or actions.dtype not in (torch.int32, torch.int64) \
                or actions.shape != (self.n,) or not actions.is_contiguous():
            raise ValueError("actions must be a contiguous int32/int64 [%d] tensor on %s" % (self.n, self.device))
        _lib.check(self.L.mgx_step(self.h, _ptr(actions), actions.element_size(), ctypes.byref(self._step_out),
                                   self._stream()), "mgx_step")
        self.calls += 1
        return self.obs

    def step_into(self, actions, reward=None, done=None):
        """step() with the per-step reward (f32 [N]) and done (u8/bool [N]) outputs written to the
        given device tensors instead of the engine's own -- e.g. row t of a [T, N] rollout buffer,
        so a captured graph of T steps fills the buffer without copies."""
        so = self._step_out
        if reward is not None or done is not None:
            so = _lib.MgxStepOut.from_buffer_copy(self._step_out)
            for t, name, dt in ((reward, "reward_dev", (torch.float32,)), (done, "done_dev", (torch.uint8, torch.bool))):
                if t is None:
                    continue
                if t.device != self.device or t.dtype not in dt or t.numel() != self.n or not t.is_contiguous():
                    raise ValueError("%s output must be a contiguous %s [%d] tensor on %s" % (name, dt, self.n, self.device))
                setattr(so, name, t.data_ptr())
        if actions.device != self.device or actions.dtype not in (torch.int32, torch.int64) \
                or actions.shape != (self.n,) or not actions.is_contiguous():
            raise ValueError("actions must be a contiguous int32/int64 [%d] tensor on %s" % (self.n, self.device))
        _lib.check(self.L.mgx_step(self.h, _ptr(actions), actions.element_size(), ctypes.byref(so), self._stream()),
                   "mgx_step")
        self.calls += 1
        return self.obs

    def epoch_boundary(self, call=None):
        """True if step call number `call` (default: the next one) starts a refill epoch: it joins
        the previous epoch's refill and forks the next (include/mgx.h, mgx_step)."""
        c = self.calls if call is None else call
        return self.ring_depth > 0 and c % self.refill_every == 0

    def enable_clock(self, slots=4096):
        """Device kernel clocks (mgx_set_clock, ABI 6): every workgroup of every launch of the step kernels
        (class 0: mgx_step, mgx_step_compact, mgx_rollout_compact) and of the refill (class 1) records its start
        and end on the device -- so a launch inside a replayed hipGraph is timed where it runs.  Set before
        capturing graphs (kernel parameters are captured).  `slots`: launches recorded per class."""
        words = int(self.L.mgx_clock_words(self.h, int(slots)))
        if words <= 0:
            raise ValueError("bad clock slots")
        self.clock = torch.zeros(words, dtype=torch.int64, device=self.device)
        khz = ctypes.c_int(0)
        _lib.check(self.L.mgx_set_clock(self.h, _ptr(self.clock), int(slots), ctypes.byref(khz)), "mgx_set_clock")
        self.clock_slots, self.clock_khz = int(slots), int(khz.value)
        self._clock_blocks, off = [], 0
        for c in range(_lib.CLOCK_CLASSES):
            g = int(self.L.mgx_clock_groups(self.h, c))
            self._clock_blocks.append((off, g))
            off += g * (1 + 2 * self.clock_slots)
        return self.clock

    def clock_rewind(self):
        """Forget every recorded launch (counters and records to zero), e.g. after a warm-up, so that the slots
        hold the launches that follow.  Call with no kernel of this engine in flight (synchronises first)."""
        torch.cuda.synchronize(self.device)
        self.clock.zero_()
        torch.cuda.synchronize(self.device)

    def clock_launches(self, cls=0):
        """Launches of kernel class `cls` so far (synchronises)."""
        torch.cuda.synchronize(self.device)
        off, g = self._clock_blocks[cls]
        return int(self.clock[off]) if g > 0 else 0

    def rollout_clock_class(self):
        """The clock class of this engine's fused rollout launches: 3 for the 32-env blocks at S = 16, else 0 (the
        step kernels' class; include/mgx.h MGX_CLOCK_CLASSES)."""
        return 3 if self._clock_blocks[3][1] > 0 else 0

    def clock_spans_us(self, cls, first, last):
        """Durations (us) of launches [first, last) of kernel class `cls`: min workgroup start to max workgroup
        end of each launch (synchronises)."""
        torch.cuda.synchronize(self.device)
        off, g = self._clock_blocks[cls]
        last = min(last, self.clock_slots)
        if last <= first:
            return []
        rec = self.clock[off + g:off + g * (1 + 2 * self.clock_slots)].view(self.clock_slots, g, 2)[first:last]
        # (a launch with a smaller grid than the class's largest leaves its other records zero: not a start)
        start = torch.where(rec[:, :, 0] > 0, rec[:, :, 0], torch.iinfo(torch.int64).max).min(1).values
        span = rec[:, :, 1].max(1).values - start                               # (ticks < 2^63: signed is fine)
        return [float(x) * 1e3 / self.clock_khz for x in span.cpu().tolist()]

    def join(self):
        """Make the current stream wait for the in-flight episode refill (mgx_join)."""
        _lib.check(self.L.mgx_join(self.h, self._stream()), "mgx_join")

    def poll_error(self):
        bits = ctypes.c_uint32()
        _lib.check(self.L.mgx_poll_error(self.h, self._stream(), ctypes.byref(bits)), "mgx_poll_error")
        if bits.value:
            msgs = [m for b, m in _lib.DEVERR.items() if bits.value & b]
            raise _lib.MgxError("device error: " + "; ".join(msgs))

    def stats(self):
        out = (ctypes.c_uint64 * 8)()
        _lib.check(self.L.mgx_stats(self.h, self._stream(), out), "mgx_stats")
        return dict(steps=int(out[0]), resets=int(out[1]), livelocks=int(out[2]), max_mt_cursor=int(out[3]),
                    queued=int(out[4]), refill_launches=int(out[5]), calls=int(out[6]), mt_generated=int(out[7]))

    def set_random_policy(self, seed=0, enable=True):
        """The fused rollout's own random policy (mgx_set_random_policy): CompactBuffer.rollout(t, None) then draws
        each launch's [K, N] actions on the device -- mgx_random_actions' draws at counter c = the launches since
        this call (`random_launches` counts them on the host)."""
        _lib.check(self.L.mgx_set_random_policy(self.h, 1 if enable else 0, ctypes.c_uint64(seed & (2 ** 64 - 1))),
                   "mgx_set_random_policy")
        self.random_policy = (seed & (2 ** 64 - 1)) if enable else None
        self.random_launches = 0

    def ring_levels(self):
        """Episodes queued in each env's ring now (mgx_ring_levels: (tail - head) mod 2^16), a numpy u16 [N]
        (synchronises; measurement only)."""
        import numpy as np
        out = np.zeros(self.n, np.uint16)
        _lib.check(self.L.mgx_ring_levels(self.h, self._stream(), out.ctypes.data_as(_P)), "mgx_ring_levels")
        return out

    def debug_counters(self, n=32):
        """Raw diagnostic counters (section clocks of the stamp builds)."""
        out = (ctypes.c_uint64 * n)()
        _lib.check(self.L.mgx_debug_counters(self.h, self._stream(), out, n), "mgx_debug_counters")
        return [int(v) for v in out]

    def dump_state(self):
        import numpy as np
        n, S = self.n, self.size
        out = dict(grid=np.zeros((n, S, S, 4), np.uint8), agent=np.zeros((n, 3), np.uint8),
                   carrying=np.zeros((n, 4), np.uint8), step_count=np.zeros(n, np.int32),
                   mission_done=np.zeros(n, np.uint8), stored_reward=np.zeros(n, np.float64),
                   mtwords=np.zeros(n, np.int64), pcg=np.zeros((n, 6), np.uint64),
                   target=np.zeros((n, 3), np.uint8), mission_id=np.zeros(n, np.uint8))
        args = [out[k].ctypes.data_as(_P) for k in ("grid", "agent", "carrying", "step_count", "mission_done",
                                                     "stored_reward", "mtwords", "pcg", "target", "mission_id")]
        _lib.check(self.L.mgx_dump_state(self.h, self._stream(), *args), "mgx_dump_state")
        return out

    def close(self):
        if getattr(self, "h", None):
            torch.cuda.synchronize(self.device)
            self.L.mgx_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


_HOST_WAIT = {"auto": 0x0, "spin": 0x1, "yield": 0x2}     # hipDeviceSchedule* (hip_runtime_api.h)
_HIP = None


def _hip():
    """The HIP runtime torch loaded (libamdhip64 of torch/lib, else the system one)."""
    global _HIP
    if _HIP is None:
        import os
        path = os.path.join(os.path.dirname(torch.__file__), "lib", "libamdhip64.so")
        _HIP = ctypes.CDLL(path if os.path.exists(path) else "libamdhip64.so")
        _HIP.hipGraphLaunch.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
        _HIP.hipGraphLaunch.restype = ctypes.c_int
    return _HIP


def graph_launch(graph, stream):
    """Launch an instantiated torch.cuda.CUDAGraph on `stream` with hipGraphLaunch directly: the same work as
    graph.replay() without its per-call bookkeeping (device guards, capture checks, RNG-offset updates --
    ~9 us of host time before the launch, HIP API trace of bench.py).  Only for graphs that captured no torch
    random-number op (whose Philox offsets replay() advances): the engine's rollouts, GAE and gathers qualify."""
    rc = _hip().hipGraphLaunch(ctypes.c_void_p(graph.raw_cuda_graph_exec()), ctypes.c_void_p(stream.cuda_stream))
    if rc != 0:
        raise _lib.MgxError("hipGraphLaunch failed: hipError %d" % rc)


def set_host_wait(mode, device=None):
    """How the calling process's host threads wait for `device` (hipSetDeviceFlags): "spin" polls the
    completion signal (lowest latency from the last kernel's end to `synchronize()` returning, one busy
    core while waiting), "yield" sleeps on it, "auto" is HIP's default (yield unless there are more HIP
    contexts than logical CPUs).  A collector that synchronises once per rollout (the reference's
    `collect_rollouts` reads the rewards back every step) pays the sleeping wait's wake-up on every
    sync.  Call before the first GPU work on `device`; raises if the runtime refuses the flags."""
    if mode not in _HOST_WAIT:
        raise ValueError("host wait mode must be one of %s" % sorted(_HOST_WAIT))
    hip = _hip()                                     # the runtime torch loaded
    dev = device if isinstance(device, int) else (torch.device(device).index or 0) if device is not None else 0
    for fn, arg in (("hipSetDevice", dev), ("hipSetDeviceFlags", _HOST_WAIT[mode])):
        rc = getattr(hip, fn)(ctypes.c_int(arg) if fn == "hipSetDevice" else ctypes.c_uint(arg))
        if rc != 0:
            raise _lib.MgxError("%s(%d) failed: hipError %d" % (fn, arg, rc))


def _check_stats(stats, device=None):
    """The adv-stat triple: f64, >= 3 elements, contiguous, on `device` (the kernel adds to stats[0..2])."""
    if stats is None:
        return
    if stats.dtype != torch.float64 or stats.numel() < 3 or not stats.is_contiguous() or not stats.is_cuda \
            or (device is not None and stats.device != torch.device(device)):
        raise ValueError("stats must be a contiguous f64 tensor of >= 3 elements on %s" % (device or "the GPU"))


def _scratch_for(stats, scratch):
    _check_stats(stats)
    if scratch is None:
        return _stats_scratch(stats)
    if stats is None or scratch.dtype != torch.float64 or not scratch.is_contiguous() \
            or scratch.numel() < _lib.GAE_SCRATCH_WORDS or scratch.device != stats.device:
        raise ValueError("scratch must be a contiguous f64 tensor of >= %d elements on the stats' device"
                         % _lib.GAE_SCRATCH_WORDS)
    return scratch


def _stats_scratch(stats):
    """The adv-stat shard scratch (include/mgx.h, MGX_GAE_SCRATCH_WORDS) of this `stats` tensor on the
    calling stream: GAE calls on different streams (e.g. two collectors) never share partial sums; calls on
    one stream are ordered.  The scratches live on the stats tensor itself, so they are freed with it (a
    module-level cache keyed by stream handle kept one per stream handle for the life of the process)."""
    if stats is None:
        return None
    assert stats.dtype == torch.float64 and stats.numel() >= 3 and stats.is_contiguous()
    per = stats.__dict__.setdefault("_mgx_scratch", {})
    key = torch.cuda.current_stream(stats.device).cuda_stream
    buf = per.get(key)
    if buf is None:
        buf = torch.zeros(_lib.GAE_SCRATCH_WORDS, dtype=torch.float64, device=stats.device)
        per[key] = buf
    return buf


def gae(rewards, values, episode_starts, last_values, last_dones, gamma, gae_lambda, stats=None, scratch=None):
    """DictRolloutBuffer.compute_returns_and_advantage on device (libmgx mgx_gae).

    rewards/values/episode_starts: f32 [T, N]; last_values f32 [N]; last_dones bool/u8 [N].
    Returns (advantages, returns) f32 [T, N].  `stats` (f64 [3] tensor, optional)
    accumulates (sum A, sum A^2, count); `scratch` (f64 [MGX_GAE_SCRATCH_WORDS], zeroed, optional) the
    caller's shard partials (default: one per stats tensor and stream)."""
    L = _lib.load()
    T, N = rewards.shape
    for t in (rewards, values, episode_starts):
        assert t.dtype == torch.float32 and t.is_contiguous() and t.shape == (T, N)
    lv = last_values.reshape(N).float().contiguous()
    ld = last_dones.reshape(N).to(torch.uint8).contiguous()
    adv = torch.empty_like(rewards)
    ret = torch.empty_like(rewards)
    gl = float(torch.tensor(gamma * gae_lambda, dtype=torch.float64).float())   # f32(gamma*lambda in fp64)
    stream = ctypes.c_void_p(torch.cuda.current_stream(rewards.device).cuda_stream)
    _lib.check(L.mgx_gae(_ptr(rewards), _ptr(values), _ptr(episode_starts), _ptr(lv), _ptr(ld), T, N,
                         ctypes.c_float(gamma), ctypes.c_float(gl), _ptr(adv), _ptr(ret), _ptr(stats),
                         _ptr(_scratch_for(stats, scratch)), stream), "mgx_gae")
    return adv, ret


def random_actions(out, counter, seed=0, n_actions=7):
    """A random policy's actions for a whole batch (libmgx mgx_random_actions): fills the contiguous int32 device
    tensor `out` with uniform draws on {0..n_actions-1} from a counter-based hash of (seed, counter[0], index), then
    advances counter[0] by one ON THE DEVICE -- the launch can be captured in a hipGraph and draws fresh actions at
    every replay (no host bookkeeping, unlike torch's Philox offsets).  `counter`: a zeroed int64 device tensor of 2
    words, one per stream of launches that must not overlap.  Host restatement: oracle.random_actions_ref."""
    L = _lib.load()
    assert out.dtype == torch.int32 and out.is_contiguous() and out.is_cuda
    assert counter.dtype == torch.int64 and counter.numel() >= 2 and counter.device == out.device
    stream = ctypes.c_void_p(torch.cuda.current_stream(out.device).cuda_stream)
    _lib.check(L.mgx_random_actions(_ptr(out), out.numel(), int(n_actions), ctypes.c_uint64(seed & (2 ** 64 - 1)),
                                    _ptr(counter), stream), "mgx_random_actions")
    return out


def gae_dones(rewards, values, dones, last_values, gamma, gae_lambda, stats=None, out=None, scratch=None):
    """GAE over the compact rollout layout (libmgx mgx_gae_dones): dones u8/bool [T, N] is
    the `done` of step t, i.e. SB3's episode_starts shifted by one plus last_dones.
    Returns (advantages, returns) f32 [T, N] (written into `out` if given)."""
    L = _lib.load()
    T, N = rewards.shape
    for t in (rewards, values):
        assert t.dtype == torch.float32 and t.is_contiguous() and t.shape == (T, N)
    assert dones.shape == (T, N) and dones.is_contiguous() and dones.element_size() == 1
    lv = last_values.reshape(N).float().contiguous()
    adv, ret = out if out is not None else (torch.empty_like(rewards), torch.empty_like(rewards))
    gl = float(torch.tensor(gamma * gae_lambda, dtype=torch.float64).float())
    stream = ctypes.c_void_p(torch.cuda.current_stream(rewards.device).cuda_stream)
    _lib.check(L.mgx_gae_dones(_ptr(rewards), _ptr(values), _ptr(dones), _ptr(lv), T, N, ctypes.c_float(gamma),
                               ctypes.c_float(gl), _ptr(adv), _ptr(ret), _ptr(stats), _ptr(_scratch_for(stats, scratch)),
                               stream), "mgx_gae_dones")
    return adv, ret
