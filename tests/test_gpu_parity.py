"""HIP engine parity (needs an MI355X): libmgx through its C ABI against
  (1) the golden fixtures made by executing the reference (every config,
      every step, every state field, every RNG position),
  (2) the SB3-layer oracle (VecTransposeImage + VecFrameStack + terminal obs),
  (3) the C oracle at 1,024 envs (bit-exact transitions),
  (4) the GAE oracle (bit-exact fp32),
  (5) size-independent properties at the BASELINE size (65,536 envs).
"""
import numpy as np
import pytest

import trajcheck as TC

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")


def _need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


class EngineSource:
    """libmgx behind trajcheck's compare() protocol (raw frames recovered from
    the stacked, transposed observation)."""

    def __init__(self, cfg, n_stack=4, mission_dtype=None, ring_depth=0, refill_every=0):
        from mgx import MgxEngine
        kw = dict(cfg)
        self.n = kw.pop("n_envs")
        self.e = MgxEngine(n_envs=self.n, n_stack=n_stack, terminal_mode="all", reward64=True,
                           mission_dtype=mission_dtype or torch.int64, ring_depth=ring_depth,
                           refill_every=refill_every, **kw)
        self.fs = None

    @staticmethod
    def newest(obs):
        img = obs["image"][:, -3:].permute(0, 2, 3, 1).contiguous().cpu().numpy()
        d = obs["direction"][:, -4:].argmax(1).to(torch.uint8).cpu().numpy()
        m = obs["mission"][:, -32:].to(torch.uint8).cpu().numpy()
        return img, d, m

    def reset(self):
        obs = self.e.reset()
        img, d, m = self.newest(obs)
        return dict(image=img, dir=d, mission=m, livelock=self.e.livelock.cpu().numpy())

    def step(self, a):
        obs = self.e.step(torch.as_tensor(a, device=self.e.device))
        done = self.e.done.cpu().numpy()
        img, d, m = self.newest(obs)
        timg, td, tm = self.newest(self.e.terminal_obs)
        dd = done.astype(bool)
        return dict(image=np.where(dd[:, None, None, None], timg, img), dir=np.where(dd, td, d),
                    mission=np.where(dd[:, None], tm, m), reward=self.e.reward64.cpu().numpy(),
                    terminated=self.e.terminated.cpu().numpy().astype(np.uint8),
                    truncated=self.e.truncated.cpu().numpy().astype(np.uint8),
                    r_image=img, r_dir=d, r_mission=m, livelock=self.e.livelock.cpu().numpy())

    def dump(self):
        return self.e.dump_state()


class CompactSource:
    """libmgx's COMPACT layout -- mgx_step_compact, the kernel bench.py times -- behind
    trajcheck's compare() protocol.  Each step writes one 148-B observation row (byte 0
    direction, bytes 1..147 the [c][vx][vy] frame) + a mission-id byte into a CompactBuffer of
    T rows (carried over when full, as the collector does); where an episode ended the buffer
    row is the new episode's first observation and the terminal row (terminal_mode 'all') the
    finished one's final frame, whose mission id is the previous row's (include/mgx.h)."""

    def __init__(self, cfg, T=64, ring_depth=0, refill_every=0, terminal_mode="all", n_stack=4):
        from mgx import MgxEngine
        from mgx._lib import mission_tokens
        from mgx.compact import CompactBuffer
        kw = dict(cfg)
        self.n = kw.pop("n_envs")
        self.e = MgxEngine(n_envs=self.n, n_stack=n_stack, terminal_mode=terminal_mode, reward64=True,
                           mission_dtype=torch.uint8, ring_depth=ring_depth, refill_every=refill_every, **kw)
        self.buf = CompactBuffer(self.e, T)
        self.tok = torch.as_tensor(mission_tokens(), device=self.e.device)
        self.t = 0

    @staticmethod
    def decode(rows):
        """u8 [n, 148] device rows -> (image HWC [n, 7, 7, 3], direction [n]) on the host."""
        img = rows[:, 1:].reshape(-1, 3, 7, 7).permute(0, 2, 3, 1).contiguous().cpu().numpy()
        return img, rows[:, 0].cpu().numpy()

    def tokens(self, mids):
        return self.tok[mids.long()].cpu().numpy()

    def reset(self):
        self.e.reset()
        self.buf.observe(0)
        self.t = 0
        r = self.buf.row(0)
        img, d = self.decode(self.buf.rows[r])
        return dict(image=img, dir=d, mission=self.tokens(self.buf.mids[r]), livelock=self.e.livelock.cpu().numpy())

    def step(self, a):
        if self.t == self.buf.T:
            self.buf.carry_over()
            self.t = 0
        t = self.t
        self.buf.step(t, torch.as_tensor(np.ascontiguousarray(a), device=self.e.device))
        self.t += 1
        r = self.buf.row(t + 1)
        dd = self.buf.starts[r].cpu().numpy().astype(bool)
        img, d = self.decode(self.buf.rows[r])
        timg, td = self.decode(self.buf.terminal_rows)
        m, tm = self.tokens(self.buf.mids[r]), self.tokens(self.buf.mids[r - 1])
        return dict(image=np.where(dd[:, None, None, None], timg, img), dir=np.where(dd, td, d),
                    mission=np.where(dd[:, None], tm, m), reward=self.e.reward64.cpu().numpy(),
                    terminated=self.buf.terminated[t].cpu().numpy(), truncated=self.buf.truncated[t].cpu().numpy(),
                    r_image=img, r_dir=d, r_mission=m, livelock=self.e.livelock.cpu().numpy(),
                    reward32=self.buf.rewards[t].cpu().numpy())

    def dump(self):
        return self.e.dump_state()


FIXTURES = TC.fixtures()


@pytest.mark.parametrize("kw", [dict(problem="full", size=7), dict(problem="gtg", size=5, num_objects=8),
                                dict(problem="mov", size=5, num_objects=7, obstacles=True, percent_obstacles=0.3),
                                dict(problem="multi", mission=3), dict(problem="opn", num_objects=13),
                                dict(problem="nope")])
def test_unsatisfiable_or_invalid_configs_are_rejected(kw):
    """Configs on which the reference raises (ValueError / AssertionError) or never returns
    (place_obj over a room with too few free cells) are refused at create time."""
    _need_gpu()
    from mgx import MgxEngine
    from mgx._lib import MgxError
    with pytest.raises((MgxError, ValueError)):
        MgxEngine(n_envs=64, **kw)


@pytest.mark.parametrize("layout", ["sb3", "compact"])
@pytest.mark.parametrize("path", FIXTURES, ids=lambda p: p.split("/")[-1][:-4])
def test_engine_matches_reference_fixture(path, layout):
    """Every reference fixture (every step, every state field, every RNG position) through both
    observation layouts: the SB3 stacks (mgx_step, the VecEnv drop-in) and the compact rows
    (mgx_step_compact, the kernel the headline bench times)."""
    _need_gpu()
    d = dict(np.load(path))
    cfg, T = TC.fixture_cfg(d)
    src = EngineSource(cfg) if layout == "sb3" else CompactSource(cfg)
    msg = TC.compare(src, d)
    src.e.poll_error()
    assert msg is None, msg


@pytest.mark.parametrize("name", ["multi_all_s8", "multi_gtg_s8", "multi_tgl_s16", "single_pkp_s8",
                                  "single_full_s8", "obst_single_mov_s11", "novis_obst_multi_tgl_s16",
                                  "ado_multi_all_s11"])
@pytest.mark.parametrize("ring", [(-1, 0, "sb3"), (2, 1, "sb3"), (4, 2, "sb3"), (8, 3, "sb3"), (2, 1, "compact"),
                                  (8, 3, "compact")],
                         ids=["inline", "ring2", "ring4", "ring8_every3", "compact_ring2", "compact_ring8_every3"])
def test_engine_reset_paths_match_fixture(name, ring):
    """Same fixtures through the other reset paths: episodes generated inline in
    the step kernel (no ring) and small rings refilled at different cadences (the compact
    layout needs the ring)."""
    _need_gpu()
    d = dict(np.load(TC.GOLDEN + "/traj/%s.npz" % name))
    cfg, T = TC.fixture_cfg(d)
    if ring[2] == "sb3":
        src = EngineSource(cfg, ring_depth=ring[0], refill_every=ring[1])
    else:
        src = CompactSource(cfg, T=37, ring_depth=ring[0], refill_every=ring[1])
    msg = TC.compare(src, d)
    src.e.poll_error()
    assert msg is None, msg


@pytest.mark.parametrize("name,n_stack,mdt", [("multi_all_s8", 4, "i64"), ("multi_pkp_s11", 3, "u8"),
                                              ("multi_tgl_s16", 1, "i64"), ("novis_multi_all_s8", 4, "i64"),
                                              ("novis_single_gto_s11", 2, "u8")])
def test_frame_stack_and_terminal_obs_match_sb3_layer(name, n_stack, mdt):
    """Full stacked observation + stacked terminal_observation every step vs the
    numpy VecTransposeImage/VecFrameStack restatement fed with the fixture."""
    _need_gpu()
    import oracle as O
    d = dict(np.load(TC.GOLDEN + "/traj/%s.npz" % name))
    cfg, T = TC.fixture_cfg(d)
    n = cfg["n_envs"]
    src = EngineSource(cfg, n_stack=n_stack, mission_dtype=torch.int64 if mdt == "i64" else torch.uint8)
    fs = O.FrameStackOracle(n, n_stack)

    def raw(img, dr, mi):
        return dict(image=O.vec_transpose_image(img), direction=O.one_hot_dir(dr), mission=mi.astype(np.int64))

    want = fs.reset(raw(d["reset0_image"], d["reset0_dir"], d["reset0_mission"]))
    obs = src.e.reset()

    def same(got, want):
        return all(np.array_equal(got[k].to(torch.int64).cpu().numpy(), want[k].astype(np.int64)) for k in want)

    assert same(obs, want)
    for t in range(min(T, 200)):
        done = (d["terminated"][t] | d["truncated"][t]).astype(bool)
        step_obs = raw(np.where(done[:, None, None, None], d["r_image"][t], d["image"][t]),
                       np.where(done, d["r_dir"][t], d["dir"][t]),
                       np.where(done[:, None], d["r_mission"][t], d["mission"][t]))
        term_frame = raw(d["image"][t], d["dir"][t], d["mission"][t])
        want, want_term = fs.step(step_obs, done, term_frame)
        obs = src.e.step(torch.as_tensor(d["actions"][t].astype(np.int64), device=src.e.device))
        assert same(obs, want), "t=%d stacked obs" % t
        if done.any():
            for k in want_term:
                got = src.e.terminal_obs[k].to(torch.int64).cpu().numpy()[done]
                assert np.array_equal(got, want_term[k][done].astype(np.int64)), "t=%d terminal %s" % (t, k)
    src.e.poll_error()


@pytest.mark.parametrize("problem,mission,size,ado", [("multi", 5, 8, 0), ("multi", None, 8, 0), ("multi", 2, 8, 0),
                                                      ("multi", None, 16, 0), ("multi", 1, 16, 0), ("gto", None, 8, 0),
                                                      ("multi", None, 8, 1), ("multi", 1, 16, 1),
                                                      ("multi", None, 11, 0)])   # (testing.yaml's size: the 11x11 evals)
def test_engine_matches_oracle_1024_envs(problem, mission, size, ado):
    """Bit-exact transitions vs the C oracle at 1,024 envs x 256 random steps
    (global env index offset 4096 exercises sharded seeding).  ado: all_doors_open=True
    (distilling.yaml:27, moe.yaml:23)."""
    _need_gpu()
    import oracle as O
    from mgx import MgxEngine
    n, T, off = 1024, 256, 4096
    ov = O.OracleVec(problem, mission, size, 4, n, 42, index_offset=off, all_doors_open=bool(ado))
    eng = MgxEngine(problem=problem, mission=mission, size=size, n_envs=n, env_index_offset=off, n_stack=4,
                    terminal_mode="all", reward64=True, all_doors_open=bool(ado))
    r = ov.reset()
    obs = eng.reset()
    img, dr, mi = EngineSource.newest(obs)
    assert np.array_equal(img, r["image"]) and np.array_equal(dr, r["dir"]) and np.array_equal(mi, r["mission"])
    acts = np.random.default_rng(99).integers(0, 7, (T, n))
    for t in range(T):
        o = ov.step(acts[t])
        obs = eng.step(torch.as_tensor(acts[t], device=eng.device))
        done = eng.done.cpu().numpy().astype(bool)
        assert np.array_equal(done, (o["terminated"] | o["truncated"]).astype(bool)), t
        assert np.array_equal(eng.reward64.cpu().numpy(), o["reward"]), t
        assert np.array_equal(eng.reward.cpu().numpy(), o["reward"].astype(np.float32)), t
        img, dr, mi = EngineSource.newest(obs)
        timg, tdr, tmi = EngineSource.newest(eng.terminal_obs)
        assert np.array_equal(np.where(done[:, None, None, None], timg, img), o["image"]), t
        assert np.array_equal(img[done], o["r_image"][done]), t
        assert np.array_equal(np.where(done, tdr, dr), o["dir"]), t
        assert np.array_equal(np.where(done[:, None], tmi, mi), o["mission"]), t
        assert np.array_equal(eng.livelock.cpu().numpy()[done], o["livelock"][done]), t
    a, b = eng.dump_state(), ov.dump()
    for k in ("grid", "agent", "carrying", "step_count", "mission_done", "mtwords", "pcg", "target"):
        assert np.array_equal(a[k], b[k]), k
    assert np.array_equal(a["stored_reward"], b["stored_reward"], equal_nan=True)
    eng.poll_error()


@pytest.mark.parametrize("problem,mission,size,nobj", [("multi", None, 8, 8), ("multi", None, 11, 8),
                                                       ("full", None, 8, 0), ("gtg", None, 8, 24)])
def test_engine_matches_oracle_object_capacity(problem, mission, size, nobj):
    """The generator's per-lane object list is sized per config (mgx_create: obj_cap).  At large
    object counts (single room: the most the 8x8 room holds; multi: crowded rooms, pinned by the
    multi_all_s11_o8 reference fixture) transitions stay bit-exact vs the C oracle and no error bit
    is raised (512 envs x 128 random steps)."""
    _need_gpu()
    import oracle as O
    from mgx import MgxEngine
    n, T = 512, 128
    ov = O.OracleVec(problem, mission, size, nobj, n, 42)
    eng = MgxEngine(problem=problem, mission=mission, size=size, num_objects=nobj, n_envs=n, n_stack=4,
                    terminal_mode="all", reward64=True)
    r = ov.reset()
    obs = eng.reset()
    img, dr, mi = EngineSource.newest(obs)
    assert np.array_equal(img, r["image"]) and np.array_equal(mi, r["mission"])
    acts = np.random.default_rng(7).integers(0, 7, (T, n))
    for t in range(T):
        o = ov.step(acts[t])
        obs = eng.step(torch.as_tensor(acts[t], device=eng.device))
        done = eng.done.cpu().numpy().astype(bool)
        assert np.array_equal(done, (o["terminated"] | o["truncated"]).astype(bool)), t
        assert np.array_equal(eng.reward64.cpu().numpy(), o["reward"]), t
        img, dr, mi = EngineSource.newest(obs)
        timg, tdr, tmi = EngineSource.newest(eng.terminal_obs)
        assert np.array_equal(np.where(done[:, None, None, None], timg, img), o["image"]), t
        assert np.array_equal(np.where(done[:, None], tmi, mi), o["mission"]), t
    a, b = eng.dump_state(), ov.dump()
    for k in ("grid", "agent", "mtwords", "pcg", "target"):
        assert np.array_equal(a[k], b[k]), k
    eng.poll_error()


def test_objects_exhausted_is_reported():
    """multi with 18 objects: once locked doors have taken their keys (and key boxes) out of the 18
    (type, colour) choices, the reference's `choice(obj_choice)` raises IndexError
    (custom_env.py:1236).  The engine must report it (MGX_DEVERR_OBJECTS), never go on silently."""
    _need_gpu()
    from mgx import MgxEngine, MgxError
    eng = MgxEngine(problem="multi", mission=None, size=11, num_objects=18, n_envs=512)
    eng.reset()
    with pytest.raises(MgxError, match="object list exhausted"):
        for _ in range(64):
            eng.step(torch.full((512,), 6, dtype=torch.int32, device=eng.device))   # 'done': reset every step
        eng.poll_error()


@pytest.mark.parametrize("T,N", [(1, 300), (7, 513), (64, 4099), (1024, 1000)])
def test_gae_bit_exact(T, N):
    """mgx_gae (SB3 f32 episode_starts + last_dones) and mgx_gae_dones (compact u8 dones of each
    step) against the numpy GAE: advantages and returns bit-exact; the f64 stats triple
    (sum A, sum A^2, n) that feeds the cross-rank advantage normalisation."""
    _need_gpu()
    import oracle as O
    from mgx import gae, gae_dones
    rng = np.random.default_rng(5 + T)
    r = rng.standard_normal((T, N)).astype(np.float32)
    v = rng.standard_normal((T, N)).astype(np.float32)
    dones = rng.random((T, N)) < 0.15
    es = np.zeros((T, N), np.float32)                 # episode_starts[t] = dones[t-1]
    es[1:] = dones[:-1]
    es[0] = rng.random(N) < 0.5
    lv = rng.standard_normal(N).astype(np.float32)
    ld = dones[-1]
    g, lam = 0.8108071290665859, 0.9452281119742252
    want_a, want_r = O.gae(r, v, es, lv, ld, g, lam)
    dev = torch.device("cuda")
    tt = lambda x: torch.tensor(x, device=dev)       # noqa: E731
    st = torch.zeros(3, dtype=torch.float64, device=dev)
    a, ret = gae(tt(r), tt(v), tt(es), tt(lv), tt(ld), g, lam, stats=st)
    assert np.array_equal(a.cpu().numpy(), want_a)
    assert np.array_equal(ret.cpu().numpy(), want_r)
    s = st.cpu().numpy()
    w = want_a.astype(np.float64)
    assert s[2] == T * N
    assert abs(s[0] - w.sum()) <= 1e-9 * np.abs(w).sum() + 1e-9
    assert abs(s[1] - (w * w).sum()) <= 1e-9 * (w * w).sum()
    st2 = torch.zeros(3, dtype=torch.float64, device=dev)
    a2, ret2 = gae_dones(tt(r), tt(v), tt(dones.astype(np.uint8)), tt(lv), g, lam, stats=st2)
    assert np.array_equal(a2.cpu().numpy(), want_a)
    assert np.array_equal(ret2.cpu().numpy(), want_r)
    assert np.allclose(st2.cpu().numpy(), s, rtol=1e-12, atol=1e-9)


FULL_SIZE = [("multi", 5, 8, 65536, 64),       # BASELINE config 2 (1 GPU)
             ("multi", None, 8, 32768, 64),    # config 4, one GPU's shard of 262,144
             ("multi", 1, 16, 131072, 24)]     # config 5, one GPU's shard of 1,048,576


@pytest.mark.parametrize("layout", ["sb3", "compact"])
@pytest.mark.parametrize("problem,mission,size,n,T", FULL_SIZE, ids=["cfg2_65536", "cfg4_32768", "cfg5_131072"])
def test_full_size_matches_oracle(problem, mission, size, n, T, layout):
    """Every env at the BASELINE per-GPU sizes against the C oracle, in both observation layouts
    (compact = the kernel the headline bench times): per step the done flags, the f64 and f32
    rewards, the terminated / truncated flags, the final frame of every env (the terminal frame
    where done), the new episode's first frame and mission where done; after T steps every env's
    full state (grid, agent, carrying, step count, mission flags, stored reward, MT cursor,
    PCG64 state, target)."""
    _need_gpu()
    import oracle as O
    ov = O.OracleVec(problem, mission, size, 4, n, 42)
    cfg = dict(problem=problem, mission=mission, size=size, n_envs=n)
    src = EngineSource(cfg) if layout == "sb3" else CompactSource(cfg, T=T)
    r = ov.reset()
    g = src.reset()
    assert np.array_equal(g["image"], r["image"]) and np.array_equal(g["mission"], r["mission"])
    assert np.array_equal(g["dir"], r["dir"])
    acts = np.random.default_rng(2024).integers(0, 7, (T, n)).astype(np.int32)
    for t in range(T):
        o = ov.step(acts[t])
        s = src.step(acts[t])
        done = (o["terminated"] | o["truncated"]).astype(bool)
        for k in ("terminated", "truncated", "reward", "image", "dir", "mission"):
            assert np.array_equal(np.asarray(s[k]).astype(o[k].dtype), o[k]), (t, k)
        if layout == "compact":
            assert np.array_equal(s["reward32"], o["reward"].astype(np.float32)), t
        for k in ("r_image", "r_dir", "r_mission"):
            assert np.array_equal(s[k][done], o[k][done]), (t, k)
    eng = src.e
    a, b = eng.dump_state(), ov.dump()
    for k in ("grid", "agent", "carrying", "step_count", "mission_done", "mtwords", "pcg", "target"):
        assert np.array_equal(a[k], b[k]), k
    assert np.array_equal(a["stored_reward"], b["stored_reward"], equal_nan=True)
    eng.poll_error()


@pytest.mark.parametrize("layout", ["fused", "fused_gae", "compact"])
@pytest.mark.parametrize("n", [8192, 65536])
def test_bench_shape_graph_matches_oracle(n, layout):
    """The exact shape bench.py times -- the driver's `--steps 20` line: GTG 8x8, terminal_mode
    'truncated', refill epoch E = 20 = horizon H, the compact buffer as a ring of two 20-row blocks (round 5:
    the carry-over is a block advance, no copy) and so two hipGraphs, one per block, each holding the
    carry-over, the steps, mgx_gae_dones with the adv-stat triple and mgx_join -- replayed in turn 4 times
    with new actions in their static buffer.  `fused` (the headline): ONE mgx_rollout_compact launch of the 20 steps (it
    forks the epoch's refill); `fused_gae`: the same launch with the GAE fused in (mgx_rollout_compact_gae,
    the bench's graph at E = H); `compact`: 20 mgx_step_compact launches (the per-step line).  Every
    replay: each step's observation rows, mission ids, dones, terminated / truncated flags and f32
    rewards vs the C oracle, the terminal row of every env that was truncated, GAE advantages /
    returns bit-exact vs numpy and the (sum A, sum A^2, n) triple; at the end every env's state."""
    _need_gpu()
    import oracle as O
    from mgx import MgxEngine, gae_dones
    from mgx._lib import mission_tokens
    from mgx.compact import CompactBuffer
    E, W, reps = 20, 200, 4                       # W: eager warm-up steps (10 refill epochs)
    ov = O.OracleVec("multi", 5, 8, 4, n, 42)
    eng = MgxEngine(problem="multi", mission=5, size=8, n_envs=n, n_stack=4, terminal_mode="truncated",
                    refill_every=E)
    assert eng.refill_every == E
    dev = eng.device
    buf = CompactBuffer(eng, E, ring=True)
    tok = mission_tokens()
    rng = np.random.default_rng(77)
    acts = rng.integers(0, 7, (W + reps * E, n)).astype(np.int32)
    ov.reset()
    eng.reset()
    buf.observe(0)
    fused = layout in ("fused", "fused_gae")        # fused_gae: the driver's graph, GAE in the rollout launch
    for t in range(0, W, E if fused else 1):
        if t and t % E == 0:
            buf.carry_over()
        if fused:
            buf.rollout(0, torch.as_tensor(acts[t:t + E], device=dev))
            for j in range(E):
                ov.step(acts[t + j])
        else:
            buf.step(t % E, torch.as_tensor(acts[t], device=dev))
            ov.step(acts[t])
    eng.join()
    torch.cuda.synchronize()
    vals = torch.as_tensor(rng.standard_normal((E, n)).astype(np.float32), device=dev)
    last_v = torch.as_tensor(rng.standard_normal(n).astype(np.float32), device=dev)
    adv, ret = torch.empty((E, n), device=dev), torch.empty((E, n), device=dev)
    st = torch.zeros(3, dtype=torch.float64, device=dev)
    static = torch.zeros((E, n), dtype=torch.int32, device=dev)
    gamma, lam = 0.8108071290665859, 0.9452281119742252
    s = torch.cuda.Stream()
    c0, graphs = buf.c, []
    with torch.cuda.stream(s):
        for _ in range(buf.blocks):                 # one graph per ring block, as bench.py captures them
            gr = torch.cuda.CUDAGraph()
            gr.capture_begin()
            st.zero_()
            buf.carry_over()
            if layout == "fused_gae":
                buf.rollout(0, static, gae=dict(values=vals, last_values=last_v, gamma=gamma, gae_lambda=lam,
                                                out=(adv, ret), stats=st))
            elif fused:
                buf.rollout(0, static)
            else:
                for j in range(E):
                    buf.step(j, static[j])
            if layout != "fused_gae":
                gae_dones(buf.rewards, vals, buf.dones, last_v, gamma, lam, stats=st, out=(adv, ret))
            eng.join()
            gr.capture_end()
            graphs.append(gr)
    torch.cuda.synchronize()
    assert buf.blocks == 2
    for r in range(reps):
        static.copy_(torch.as_tensor(acts[W + r * E:W + (r + 1) * E], device=dev))
        graphs[r % buf.blocks].replay()
        torch.cuda.synchronize()
        b0 = ((c0 + r % buf.blocks + 1) % buf.blocks) * E      # the block this replay wrote: obs j+1 at b0 + j
        rows = buf.rows.cpu().numpy()
        mids = buf.mids.cpu().numpy()
        starts = buf.starts.cpu().numpy().astype(bool)
        rew = buf.rewards.cpu().numpy()
        trm, trc = buf.terminated.cpu().numpy(), buf.truncated.cpu().numpy()
        t_img = np.zeros((n, 7, 7, 3), np.uint8)
        t_has = np.zeros(n, bool)
        for j in range(E):
            o = ov.step(acts[W + r * E + j])
            done = (o["terminated"] | o["truncated"]).astype(bool)
            row = rows[b0 + j]
            img = row[:, 1:].reshape(n, 3, 7, 7).transpose(0, 2, 3, 1)
            want_img = np.where(done[:, None, None, None], o["r_image"], o["image"])
            assert np.array_equal(img, want_img), (r, j, "image")
            assert np.array_equal(row[:, 0], np.where(done, o["r_dir"], o["dir"])), (r, j, "dir")
            assert np.array_equal(tok[mids[b0 + j]], np.where(done[:, None], o["r_mission"], o["mission"])), (r, j)
            assert np.array_equal(starts[b0 + j], done), (r, j, "done")
            assert np.array_equal(trm[j], o["terminated"]) and np.array_equal(trc[j], o["truncated"]), (r, j)
            assert np.array_equal(rew[j], o["reward"].astype(np.float32)), (r, j, "reward")
            tr = o["truncated"].astype(bool) & ~o["terminated"].astype(bool)
            t_img[tr] = o["image"][tr]
            t_has |= tr
        trows = buf.terminal_rows.cpu().numpy()
        got_t = trows[:, 1:].reshape(n, 3, 7, 7).transpose(0, 2, 3, 1)
        assert np.array_equal(got_t[t_has], t_img[t_has]), (r, "terminal rows")
        dn = starts[b0:b0 + E]
        es = np.zeros((E, n), np.float32)
        es[1:] = dn[:-1]
        want_a, want_r = O.gae(rew, vals.cpu().numpy(), es, last_v.cpu().numpy(), dn[-1], gamma, lam)
        assert np.array_equal(adv.cpu().numpy(), want_a), r
        assert np.array_equal(ret.cpu().numpy(), want_r), r
        sv = st.cpu().numpy()
        w = want_a.astype(np.float64)
        assert sv[2] == E * n and abs(sv[0] - w.sum()) <= 1e-9 * np.abs(w).sum() + 1e-9, (r, sv)
        assert abs(sv[1] - (w * w).sum()) <= 1e-9 * (w * w).sum(), (r, sv)
    a, b = eng.dump_state(), ov.dump()
    for k in ("grid", "agent", "carrying", "step_count", "mission_done", "mtwords", "pcg", "target"):
        assert np.array_equal(a[k], b[k]), k
    assert np.array_equal(a["stored_reward"], b["stored_reward"], equal_nan=True)
    eng.poll_error()


def test_refill_accounting():
    """mgx_stats: pre-generated episodes queued in the rings.  mgx_reset fills every ring to D
    (less abandoned attempts);
    each epoch the refill tops the rings up so that >= K stay queued at its join,
    never more than D; episodes produced in an epoch = resets consumed + change of the queue.
    Production follows consumption (the wave's mean, rounded up): over 40 epochs the queue
    settles below D and the refill produces what the steps consumed."""
    _need_gpu()
    from mgx import MgxEngine
    n = 4096
    eng = MgxEngine(problem="multi", mission=None, size=8, n_envs=n, terminal_mode="none")
    eng.reset()
    K, D = eng.refill_every, eng.ring_depth
    st = eng.stats()
    # to D, less the attempts abandoned on the way (each costs its lane one episode of the fill)
    assert 0.97 * D * n <= st["queued"] <= D * n and st["refill_launches"] == 1 and st["calls"] == 0
    g = torch.Generator(device="cuda")
    g.manual_seed(5)
    first = st
    for epoch in range(40):
        prev = st
        for _ in range(K):
            eng.step(torch.randint(0, 7, (n,), device="cuda", generator=g, dtype=torch.int32))
        st = eng.stats()
        assert n * K <= st["queued"] <= n * D, (epoch, st)
        produced = (st["resets"] - prev["resets"]) + (st["queued"] - prev["queued"])
        assert produced >= 0 and st["resets"] - prev["resets"] > 0, (epoch, st, prev)
        assert st["refill_launches"] == 2 + epoch and st["calls"] == K * (epoch + 1)
    consumed = st["resets"] - first["resets"]
    produced = consumed + st["queued"] - first["queued"]
    assert st["queued"] < D * n and produced > 0.9 * consumed, (st, first)
    eng.poll_error()


@pytest.mark.parametrize("n,terminal_mode", [(77, "all"), (130, "truncated")])
def test_ragged_block_full_stacks_match_oracle(n, terminal_mode):
    """A partial last workgroup (n not a multiple of 64, rows not a multiple of 4
    dwords): full stacked observation and stacked terminal_observation every step,
    against the C oracle + the numpy VecFrameStack restatement."""
    _need_gpu()
    import oracle as O
    from mgx import MgxEngine
    T = 160
    ov = O.OracleVec("multi", None, 8, 4, n, 42)
    fs = O.FrameStackOracle(n, 4)
    eng = MgxEngine(problem="multi", mission=None, size=8, n_envs=n, n_stack=4, terminal_mode=terminal_mode)

    def raw(img, dr, mi):
        return dict(image=O.vec_transpose_image(img), direction=O.one_hot_dir(dr), mission=mi.astype(np.int64))

    r = ov.reset()
    want = fs.reset(raw(r["image"], r["dir"], r["mission"]))
    obs = eng.reset()
    for k in want:
        assert np.array_equal(obs[k].to(torch.int64).cpu().numpy(), want[k].astype(np.int64)), k
    rng = np.random.default_rng(7)
    n_term = 0
    for t in range(T):
        a = rng.integers(0, 7 if terminal_mode == "all" else 6, n)   # no 'done' -> truncations
        o = ov.step(a.astype(np.int32))
        done = (o["terminated"] | o["truncated"]).astype(bool)
        cur = raw(np.where(done[:, None, None, None], o["r_image"], o["image"]), np.where(done, o["r_dir"], o["dir"]),
                  np.where(done[:, None], o["r_mission"], o["mission"]))
        want, want_term = fs.step(cur, done, raw(o["image"], o["dir"], o["mission"]))
        obs = eng.step(torch.as_tensor(a, device=eng.device))
        for k in want:
            assert np.array_equal(obs[k].to(torch.int64).cpu().numpy(), want[k].astype(np.int64)), (t, k)
        sel = done if terminal_mode == "all" else (o["truncated"].astype(bool) & ~o["terminated"].astype(bool))
        if sel.any():
            n_term += int(sel.sum())
            for k in want_term:
                got = eng.terminal_obs[k].to(torch.int64).cpu().numpy()[sel]
                assert np.array_equal(got, want_term[k][sel].astype(np.int64)), (t, k)
    assert n_term > 0
    eng.poll_error()


@pytest.mark.parametrize("ring", [(0, 0, 0), (16, 4, 1), (8, 4, -1)], ids=["default", "d16_k4_cap1", "d8_k4_fill"])
def test_ring_never_runs_dry_under_max_consumption(ring):
    """Every env resets every step ('done' action: one episode per step, the most a
    step can consume) -- the refill's production rule must keep every ring non-empty
    (no MGX_DEVERR_RING_EMPTY) and the stream must stay bit-exact with the oracle."""
    _need_gpu()
    import oracle as O
    from mgx import MgxEngine
    n, T = 512, 160
    ov = O.OracleVec("multi", None, 8, 4, n, 42)
    eng = MgxEngine(problem="multi", mission=None, size=8, n_envs=n, terminal_mode="none",
                    ring_depth=ring[0], refill_every=ring[1], refill_cap=ring[2])
    ov.reset()
    eng.reset()
    rng = np.random.default_rng(3)
    for t in range(T):
        a = np.full(n, 6) if t % 40 < 30 else rng.integers(0, 7, n)   # bursts of 'done', then random
        o = ov.step(a.astype(np.int32))
        obs = eng.step(torch.as_tensor(a, device=eng.device))
        img, dr, mi = EngineSource.newest(obs)
        done = (o["terminated"] | o["truncated"]).astype(bool)
        assert np.array_equal(img, np.where(done[:, None, None, None], o["r_image"], o["image"])), t
    eng.poll_error()            # raises on MGX_DEVERR_RING_EMPTY
    a_, b_ = eng.dump_state(), ov.dump()
    for k in ("grid", "agent", "mtwords", "pcg"):
        assert np.array_equal(a_[k], b_[k]), k


@pytest.mark.parametrize("ring_depth", [0, -1], ids=["ring", "inline"])
def test_mt_stream_outlives_its_ring(ring_depth):
    """The shared MT19937(42) stream (custom_env.py:82, one CPython `random` per env) never runs
    out: the device holds a ring of it (mt_table_words = 2^18 -> 32,768 groups = 327,680 words) and
    mgx_mt_slide_kernel keeps generating the stream on the device ahead of the furthest cursor,
    over the groups no env can read again.  GTG 8x8, 1,024 envs stepped until the stream generated
    is several ring lengths (the live cursors spread over ~200 k words by then -- what the ring
    must hold), with an unseeded VecEnv.reset() in the middle (both streams continue from each
    env's current episode, so its cursor must still be in the ring): transitions bit-exact vs the
    C oracle (per-env CPython MT state), every RNG position equal at the end, no
    MGX_DEVERR_MT_TABLE."""
    _need_gpu()
    import oracle as O
    from mgx import MgxEngine
    n = 1024
    T = 48000 if ring_depth == 0 else 24000
    ov = O.OracleVec("multi", 5, 8, 4, n, 42)
    eng = MgxEngine(problem="multi", mission=5, size=8, n_envs=n, n_stack=4, terminal_mode="none", reward64=True,
                    mt_table_words=1 << 18, ring_depth=ring_depth)
    ring_words = 32768 * 10
    ov.reset()
    eng.reset()
    rng = np.random.default_rng(31)
    acts = torch.as_tensor(rng.integers(0, 7, (T, n)).astype(np.int32), device=eng.device)
    acts_h = acts.cpu().numpy()
    for t in range(T):
        if t == T // 2:
            r = ov.reset(seed=None)
            obs = eng.reset()
            img, dr, mi = EngineSource.newest(obs)
            assert np.array_equal(img, r["image"]) and np.array_equal(mi, r["mission"]), "reset at %d" % t
        o = ov.step(acts_h[t])
        obs = eng.step(acts[t])
        if t % 200 == 0 or t == T - 1:
            done = eng.done.cpu().numpy().astype(bool)
            assert np.array_equal(done, (o["terminated"] | o["truncated"]).astype(bool)), t
            assert np.array_equal(eng.reward64.cpu().numpy(), o["reward"]), t
            img, _, mi = EngineSource.newest(obs)
            assert np.array_equal(img, np.where(done[:, None, None, None], o["r_image"], o["image"])), t
    eng.poll_error()                         # raises on MGX_DEVERR_MT_TABLE
    a, b = eng.dump_state(), ov.dump()
    for k in ("grid", "agent", "carrying", "step_count", "mission_done", "mtwords", "pcg", "target"):
        assert np.array_equal(a[k], b[k]), k
    st = eng.stats()
    assert st["mt_generated"] > (2 if ring_depth == 0 else 1) * ring_words, st   # the ring was rewritten
    assert a["mtwords"].max() - a["mtwords"].min() < ring_words


def test_gae_stats_of_overlapping_streams_stay_apart():
    """Two GAE calls with advantage statistics in flight at once on two streams (two collectors):
    each stream's partial sums go through its own shard scratch (include/mgx.h,
    MGX_GAE_SCRATCH_WORDS), so each triple is its own rollout's."""
    _need_gpu()
    import oracle as O
    from mgx import gae_dones
    dev = torch.device("cuda")
    g, lam = 0.8108071290665859, 0.9452281119742252
    rng = np.random.default_rng(41)
    T, N = 256, 65536
    data = []
    for k in range(2):
        r = rng.standard_normal((T, N)).astype(np.float32) * (1 + 3 * k)
        v = rng.standard_normal((T, N)).astype(np.float32)
        d = (rng.random((T, N)) < 0.15).astype(np.uint8)
        lv = rng.standard_normal(N).astype(np.float32)
        data.append((r, v, d, lv))
    streams = [torch.cuda.Stream(), torch.cuda.Stream()]
    dev_data = [tuple(torch.as_tensor(x, device=dev) for x in dd) for dd in data]
    stats = [torch.zeros(3, dtype=torch.float64, device=dev) for _ in range(2)]
    torch.cuda.synchronize()
    outs = []
    for rep in range(3):
        for k in range(2):
            with torch.cuda.stream(streams[k]):
                r, v, d, lv = dev_data[k]
                outs.append(gae_dones(r, v, d, lv, g, lam, stats=stats[k]))
    torch.cuda.synchronize()
    for k in range(2):
        r, v, d, lv = data[k]
        es = np.zeros((T, N), np.float32)
        es[1:] = d[:-1]
        want_a, _ = O.gae(r, v, es, lv, d[-1], g, lam)
        w = want_a.astype(np.float64)
        s = stats[k].cpu().numpy()
        assert s[2] == 3 * T * N, s
        assert abs(s[0] - 3 * w.sum()) <= 1e-9 * 3 * np.abs(w).sum() + 1e-9, (k, s)
        assert abs(s[1] - 3 * (w * w).sum()) <= 1e-9 * 3 * (w * w).sum(), (k, s)
