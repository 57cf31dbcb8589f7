"""Compact rollout layout: the engine writes each observation as
one 148-B row (direction + [c][vx][vy] frame) plus a mission-id byte straight into a
[rows, N] device buffer (mgx_step_compact), and mgx_gather rebuilds SB3's stacked
observation (VecTransposeImage + VecFrameStack(n_stack), src/ppo.py:124-126) for any set
of (t, env) samples -- optionally already as the policy's float input (preprocess_obs).

Per env-step the buffer holds 150 B instead of the stacked 588 + 16 + 128..1024 B, and no
stack is rolled per step.  Row layout of a rollout of T steps with H = n_stack - 1 history
rows (the previous rollout's last observations):

    row H + t   observation t (t = 0..T; row H + T is the observation after the last step)
    starts[r]   1 if row r is an episode's first observation (= `done` of the step before)

so GAE's per-step dones are starts[H+1 : H+T+1] (mgx_gae_dones).  carry_over() copies the last H + 1
rows to the front for the next rollout.

ring=True (the bench's and the collector's layout, round 5): the buffer is a ring of m blocks of T rows
(m = 1 + ceil((H + 1) / T)); rollout c writes its observations 1..T into block c mod m, and its observation
0 and history rows are the previous rollouts' last rows, read in place (mgx_gather_ring wraps the walk
back) -- carry_over() only advances the block, no rows move:

    row(t) = (b*T + t - 1) mod R,  b = c mod m,  R = m*T;  dones = starts[b*T : b*T + T]"""
import ctypes

import torch

from . import _lib
from .engine import _ptr

ROW = 148


class CompactBuffer:
    """Device rollout storage for T steps of an MgxEngine's N envs in the compact layout."""

    def __init__(self, engine, T, device=None, ring=False):
        self.engine = engine
        self.T, self.N, self.K = int(T), engine.n, engine.n_stack
        self.H = self.K - 1
        self.ring = bool(ring)
        self.c = 0                                            # rollouts started (ring: block c % m)
        if self.ring:
            self.blocks = 1 + -(-(self.H + 1) // self.T)
            R = self.blocks * self.T
        else:
            self.blocks = 0
            R = self.T + self.H + 1
        self.R = R
        dev = device or engine.device
        u8 = dict(dtype=torch.uint8, device=dev)
        self.rows = torch.zeros((R, self.N, ROW), **u8)
        self.mids = torch.zeros((R, self.N), **u8)
        self.starts = torch.ones((R, self.N), **u8)          # history rows: "start" blocks older frames
        self.terminal_rows = torch.zeros((self.N, ROW), **u8)
        f32 = dict(dtype=torch.float32, device=dev)
        self.rewards = torch.zeros((self.T, self.N), **f32)
        self.terminated = torch.zeros((self.T, self.N), **u8)
        self.truncated = torch.zeros((self.T, self.N), **u8)
        self._out = _lib.MgxCompactOut()
        self._arange = torch.arange(self.N, device=dev, dtype=torch.int64)

    def row(self, t):
        """Buffer row of observation t (an int or an integer tensor) of the current rollout."""
        if self.ring:
            return (self.block * self.T + t - 1) % self.R
        return self.H + t

    @property
    def block(self):
        return self.c % self.blocks if self.ring else 0

    def index(self, t, env):
        """Flat gather index (row * N + env) of observation t of `env`."""
        return self.row(t) * self.N + env

    @property
    def dones(self):
        """u8 [T, N]: done of step t (= start flag of observation t+1)."""
        if self.ring:
            b = self.block * self.T
            return self.starts[b:b + self.T]
        return self.starts[self.H + 1:self.H + 1 + self.T]

    def observe(self, t=0):
        """Write every env's current observation as observation t (after a reset), start = 1."""
        r = self.row(t)
        e = self.engine
        _lib.check(e.L.mgx_observe_compact(e.h, _ptr(self.rows[r]), _ptr(self.mids[r]), e._stream()),
                   "mgx_observe_compact")
        self.starts[r].fill_(1)

    def step(self, t, actions):
        """Step every env with `actions`; the new observation becomes observation t+1."""
        e = self.engine
        if actions.device != e.device or actions.dtype not in (torch.int32, torch.int64) \
                or actions.shape != (self.N,) or not actions.is_contiguous():
            raise ValueError("actions must be a contiguous int32/int64 [%d] tensor on %s" % (self.N, e.device))
        r = self.row(t + 1)
        o = self._out
        o.row_dev = self.rows[r].data_ptr()
        o.mission_id_dev = self.mids[r].data_ptr()
        o.terminal_row_dev = self.terminal_rows.data_ptr()
        o.reward_dev = self.rewards[t].data_ptr()
        o.reward64_dev = None if e.reward64 is None else e.reward64.data_ptr()
        o.terminated_dev = self.terminated[t].data_ptr()
        o.truncated_dev = self.truncated[t].data_ptr()
        o.done_dev = self.starts[r].data_ptr()
        o.ep_return_dev = e.ep_return.data_ptr()
        o.ep_len_dev = e.ep_len.data_ptr()
        o.livelock_dev = e.livelock.data_ptr()
        _lib.check(e.L.mgx_step_compact(e.h, _ptr(actions), actions.element_size(), ctypes.byref(o), e._stream()),
                   "mgx_step_compact")
        e.calls += 1

    def rollout(self, t, actions, gae=None, K=None):
        """K = len(actions) steps in ONE launch (mgx_rollout_compact): actions int32 [K, N] known up
        front (a random-action or scripted rollout) -- or None with `K` given, after
        engine.set_random_policy(seed): the launch draws its own uniform actions on the device
        (mgx_random_actions' draws at the engine's random-launch counter); observations t+1 .. t+K, rewards / dones of
        steps t .. t+K-1 -- the same as K step() calls, bit for bit.  The K steps must lie within one
        refill epoch of the engine.
        gae: dict(values f32 [K, N], last_values f32 [N], gamma, gae_lambda, out=(adv, ret) f32 [K, N],
        stats=f64 [3] or None, scratch=None) -- also the GAE of these K steps, fused into the launch
        (mgx_rollout_compact_gae): gae_dones(rewards[t:t+K], values, dones of the K steps, ...) bit for bit."""
        self.rollout_launcher(t, actions, gae, K)()

    def rollout_launcher(self, t, actions, gae=None, K=None):
        """rollout(t, actions, gae, K) prepared for the CURRENT ring block and not launched: the returned callable
        issues it with the ctypes arguments built here, once -- one C call per launch (bench.py --launch eager: the
        timed region's launches without a graph's launch latency).  The tensors it writes are this buffer's; those
        it reads (actions, GAE inputs) must stay alive and in place."""
        e = self.engine
        if actions is None:
            if getattr(e, "random_policy", None) is None or K is None:
                raise ValueError("rollout without actions needs engine.set_random_policy(seed) and K")
            K = int(K)
        else:
            K = int(actions.shape[0])
            if actions.device != e.device or actions.dtype != torch.int32 or tuple(actions.shape) != (K, self.N) \
                    or not actions.is_contiguous():
                raise ValueError("actions must be a contiguous int32 [K, %d] tensor on %s" % (self.N, e.device))
        if t < 0 or t + K > self.T:
            raise ValueError("steps %d..%d outside the buffer's %d" % (t, t + K - 1, self.T))
        r = self.row(t + 1)
        o = _lib.MgxRolloutOut()
        o.rows_dev = self.rows[r].data_ptr()
        o.mission_ids_dev = self.mids[r].data_ptr()
        o.terminal_row_dev = self.terminal_rows.data_ptr()
        o.rewards_dev = self.rewards[t].data_ptr()
        o.rewards64_dev = None
        o.terminated_dev = self.terminated[t].data_ptr()
        o.truncated_dev = self.truncated[t].data_ptr()
        o.dones_dev = self.starts[r].data_ptr()
        o.ep_return_dev = e.ep_return.data_ptr()
        o.ep_len_dev = e.ep_len.data_ptr()
        o.livelock_dev = e.livelock.data_ptr()
        ap = _ptr(actions)
        L, h = e.L, e.h
        if gae is None:
            g, keep = None, (actions,)
        else:
            from .engine import _scratch_for
            v, lv = gae["values"], gae["last_values"].reshape(self.N).float().contiguous()
            adv, ret = gae["out"]
            for x in (v, adv, ret):
                if x.dtype != torch.float32 or tuple(x.shape) != (K, self.N) or not x.is_contiguous() \
                        or x.device != e.device:
                    raise ValueError("GAE values / advantages / returns must be contiguous f32 [%d, %d]" % (K, self.N))
            if lv.device != e.device:
                raise ValueError("GAE last_values must be on %s" % e.device)
            stats = gae.get("stats")
            from .engine import _check_stats
            _check_stats(stats, e.device)
            g = _lib.MgxGaeArgs()
            g.values_dev, g.last_values_dev = v.data_ptr(), lv.data_ptr()
            g.gamma = float(gae["gamma"])
            g.gamma_lambda = float(torch.tensor(gae["gamma"] * gae["gae_lambda"], dtype=torch.float64).float())
            g.advantages_dev, g.returns_dev = adv.data_ptr(), ret.data_ptr()
            g.adv_stats_dev = stats.data_ptr() if stats is not None else None
            sc = _scratch_for(stats, gae.get("scratch")) if stats is not None else None
            g.stats_scratch_dev = sc.data_ptr() if sc is not None else None
            keep = (actions, v, lv, adv, ret, stats, sc)
        o_ref = ctypes.byref(o)
        g_ref = ctypes.byref(g) if g is not None else None

        def launch(stream=None):
            _keep = (o, g, keep)                             # noqa: F841  (the structs and inputs outlive the call)
            st = stream if stream is not None else e._stream()
            if g_ref is None:
                _lib.check(L.mgx_rollout_compact(h, ap, K, o_ref, st), "mgx_rollout_compact")
            else:
                _lib.check(L.mgx_rollout_compact_gae(h, ap, K, o_ref, g_ref, st), "mgx_rollout_compact_gae")
            e.calls += K
            if actions is None:
                e.random_launches += 1
        return launch

    def carry_over(self):
        """Start the next rollout: its history rows and observation 0 are this one's last rows (ring: read in
        place, only the block advances)."""
        self.c += 1
        if self.ring:
            return
        src = slice(self.T, self.T + self.H + 1)
        for a in (self.rows, self.mids, self.starts):
            a[:self.H + 1].copy_(a[src].clone() if self.T < self.H + 1 else a[src])

    def gather(self, index, terminal=False, f32=True, out=None):
        """Stacked observations of flat buffer indices `index` (i64 [B] = row * N + env, see index()):
        dict(image [B, 3K, 7, 7], direction [B, 4K] (f32 = policy input, else u8), mission u8 [B, 32K]).
        terminal=True: the stacked terminal_observation of the step that left row index."""
        e = self.engine
        B = index.numel()
        K = self.K
        if out is None:
            ft = torch.float32 if f32 else torch.uint8
            out = dict(image=torch.empty((B, 3 * K, 7, 7), dtype=ft, device=e.device),
                       direction=torch.empty((B, 4 * K), dtype=ft, device=e.device),
                       mission=torch.empty((B, 32 * K), dtype=torch.uint8, device=e.device))
        idx = index.to(torch.int64).contiguous()
        _lib.check(e.L.mgx_gather_ring(e.h, _ptr(self.rows), _ptr(self.mids), _ptr(self.starts), self.N,
                                       self.R if self.ring else 0, _ptr(idx), B,
                                  _ptr(self.terminal_rows) if terminal else None,
                                  _ptr(out["image"]), int(out["image"].dtype == torch.float32),
                                  _ptr(out["direction"]), int(out["direction"].dtype == torch.float32),
                                  _ptr(out["mission"]), e._stream()), "mgx_gather")
        return out

    def gather_step(self, t, terminal=False, f32=True, out=None, envs=None):
        """Stacked observation t of every env (or of `envs`)."""
        ix = self._arange if envs is None else envs.to(torch.int64)
        return self.gather(self.index(t, ix), terminal=terminal, f32=f32, out=out)
