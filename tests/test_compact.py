"""Compact rollout layout (mgx_step_compact + mgx_gather, mgx/compact.py) against the SB3
layout the engine materialises (mgx_step): two engines of the same config and seed stepped in
lockstep; every step, the stacked observation and the stacked terminal_observation rebuilt by
the gather kernel must equal the engine's materialised stacks bit for bit (which are pinned to
the reference fixtures by test_gpu_parity.py), and the f32 gather must equal torch's
preprocess_obs of them (image / 255 on the same device)."""
import numpy as np
import pytest

torch = pytest.importorskip("torch")

pytestmark = pytest.mark.gpu


def _need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


CASES = [dict(problem="multi", mission=5, size=8, n=4000, n_stack=4),      # BASELINE config 2's GTG
         dict(problem="multi", mission=None, size=8, n=200, n_stack=4),
         dict(problem="multi", mission=1, size=16, n=130, n_stack=4, see_through_walls=False),
         dict(problem="multi", mission=2, size=11, n=77, n_stack=3, all_doors_open=True),
         dict(problem="pkp", mission=None, size=8, n=64, n_stack=1)]


@pytest.mark.parametrize("case", CASES, ids=lambda c: "%s_%s_s%d_n%d_k%d" % (
    c["problem"], c["mission"], c["size"], c["n"], c["n_stack"]))
def test_gathered_stacks_equal_materialised_stacks(case):
    _need_gpu()
    from mgx import MgxEngine
    from mgx.compact import CompactBuffer
    from mgx.policy import preprocess
    kw = dict(case)
    n, k = kw.pop("n"), kw.pop("n_stack")
    T = 96
    ref = MgxEngine(n_envs=n, n_stack=k, terminal_mode="all", mission_dtype=torch.uint8, reward64=True, **kw)
    cmp_ = MgxEngine(n_envs=n, n_stack=k, terminal_mode="all", mission_dtype=torch.uint8, reward64=True, **kw)
    buf = CompactBuffer(cmp_, T)
    obs = ref.reset()
    cmp_.reset()
    buf.observe(0)
    g = buf.gather_step(0, f32=False)
    for key in ("image", "direction", "mission"):
        assert torch.equal(g[key], obs[key]), key
    rng = np.random.default_rng(11)
    n_done = 0
    for t in range(T):
        # bursts of 'done' make episodes start inside every stack position
        a = np.full(n, 6) if t % 23 == 5 else rng.integers(0, 7, n)
        act = torch.as_tensor(a, device=ref.device)
        obs = ref.step(act)
        buf.step(t, act)
        assert torch.equal(buf.rewards[t], ref.reward), t
        assert torch.equal(buf.dones[t].bool(), ref.done), t
        assert torch.equal(buf.terminated[t].bool(), ref.terminated), t
        g = buf.gather_step(t + 1, f32=False)
        for key in ("image", "direction", "mission"):
            assert torch.equal(g[key], obs[key]), (t, key)
        d = ref.done.nonzero().flatten()
        if d.numel():
            n_done += d.numel()
            gt = buf.gather_step(t, terminal=True, f32=False, envs=d)
            for key in ("image", "direction", "mission"):
                assert torch.equal(gt[key], ref.terminal_obs[key][d]), (t, key)
        if t % 16 == 0:
            gf = buf.gather_step(t + 1, f32=True)
            want = preprocess(obs)
            assert torch.equal(gf["image"], want["image"]), t
            assert torch.equal(gf["direction"], want["direction"]), t
    assert n_done > n
    ref.poll_error()
    cmp_.poll_error()
    a_, b_ = ref.dump_state(), cmp_.dump_state()
    for key in ("grid", "agent", "mtwords", "pcg"):
        assert np.array_equal(a_[key], b_[key]), key


@pytest.mark.parametrize("ring,T,rolls", [(False, 8, 2), (True, 8, 4), (True, 2, 7), (True, 3, 5)],
                         ids=["copy_T8", "ring_T8", "ring_T2", "ring_T3"])
def test_carry_over_and_minibatch_gather(ring, T, rolls):
    """Rollouts of T steps with the buffer carried over: any (t, env) sample of every rollout after the
    first, in a random minibatch order, gathers the stack the SB3 engine showed at that step (the history
    rows bridge the rollout boundary).  ring=True (the bench's and the collector's layout): the history rows
    are read in place through mgx_gather_ring, the ring wraps several times (T = 2 and 3 < n_stack: the
    history reaches two blocks back), and the terminal stacks of the finished episodes are checked too."""
    _need_gpu()
    from mgx import MgxEngine
    from mgx.compact import CompactBuffer
    n = 96
    ref = MgxEngine(problem="multi", mission=None, size=8, n_envs=n, mission_dtype=torch.uint8, terminal_mode="all")
    cmp_ = MgxEngine(problem="multi", mission=None, size=8, n_envs=n, mission_dtype=torch.uint8, terminal_mode="all")
    buf = CompactBuffer(cmp_, T, ring=ring)
    ref.reset()
    cmp_.reset()
    buf.observe(0)
    g = torch.Generator(device="cuda")
    g.manual_seed(3)
    for roll in range(rolls):
        if roll:
            buf.carry_over()
        seen = []
        for t in range(T):
            seen.append({k: v.clone() for k, v in ref.obs.items()})
            a = torch.randint(0, 7, (n,), device="cuda", generator=g)
            if t % 5 == 4:
                a[: n // 3] = 6                                  # bursts of 'done'
            ref.step(a)
            buf.step(t, a)
            assert torch.equal(buf.dones[t].bool(), ref.done), (roll, t)
            d = ref.done.nonzero().flatten()
            if d.numel():
                gt = buf.gather_step(t, terminal=True, f32=False, envs=d)
                for key in ("image", "direction", "mission"):
                    assert torch.equal(gt[key], ref.terminal_obs[key][d]), (roll, t, key)
        if roll == 0:
            continue
        perm = torch.randperm(n * T, device="cuda")            # env-major flat index (swap_and_flatten)
        env, t_ = perm // T, perm % T
        got = buf.gather(buf.index(t_, env), f32=False)
        for key in ("image", "direction", "mission"):
            want = torch.stack([seen[int(tt)][key][int(ee)] for tt, ee in zip(t_.tolist(), env.tolist())])
            assert torch.equal(got[key], want), (roll, key)


def test_graph_replays_equal_eager_steps():
    """Refill epochs captured in hipGraphs (whole epochs ending in mgx_join, as bench.py does: the
    join of each epoch sits at the next epoch's fork, include/mgx.h) replay the same transitions as
    eager steps: two engines of one config and seed, one stepped eagerly, one by replaying a graph
    of E steps with the actions copied into its static buffer; rows, rewards, dones and the final
    engine state must be equal."""
    _need_gpu()
    from mgx import MgxEngine
    from mgx.compact import CompactBuffer
    n, E, reps = 256, 8, 6
    kw = dict(problem="multi", mission=None, size=8, n_envs=n, refill_every=E)
    eager, graphed = MgxEngine(**kw), MgxEngine(**kw)
    be, bg = CompactBuffer(eager, E), CompactBuffer(graphed, E)
    eager.reset(); graphed.reset()
    be.observe(0); bg.observe(0)
    rng = np.random.default_rng(5)
    acts = [torch.as_tensor(rng.integers(0, 7, (E, n)), device=eager.device, dtype=torch.int32) for _ in range(reps)]
    static = torch.zeros((E, n), device=graphed.device, dtype=torch.int32)
    torch.cuda.synchronize()
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        gr = torch.cuda.CUDAGraph()
        gr.capture_begin()
        for j in range(E):
            bg.step(j, static[j])
        graphed.join()
        gr.capture_end()
    torch.cuda.synchronize()
    for r in range(reps):
        if r:
            be.carry_over(); bg.carry_over()
        for j in range(E):
            be.step(j, acts[r][j])
        static.copy_(acts[r])
        gr.replay()
        torch.cuda.synchronize()
        assert torch.equal(be.rows, bg.rows), r
        assert torch.equal(be.rewards, bg.rewards), r
        assert torch.equal(be.starts, bg.starts), r
    de, dg = eager.dump_state(), graphed.dump_state()
    for k in de:
        a, b = np.asarray(de[k]), np.asarray(dg[k])
        assert np.array_equal(a, b, equal_nan=a.dtype.kind == "f"), k      # None is stored as NaN


GATHER_FIXTURES = [("multi_all_s8", 4), ("multi_gtg_s8", 4), ("multi_pkp_s11", 3), ("multi_tgl_s16", 4),
                   ("novis_multi_all_s8", 2), ("manual_multi_all_s8", 4)]


@pytest.mark.parametrize("name,n_stack", GATHER_FIXTURES, ids=[f[0] + "_k%d" % f[1] for f in GATHER_FIXTURES])
def test_gather_matches_framestack_oracle_on_fixtures(name, n_stack):
    """mgx_gather pinned directly to the reference fixtures through the restated SB3 layer
    (O.FrameStackOracle = VecTransposeImage + VecFrameStack(n_stack, 'first') over the fixture's own
    per-step observations): the engine steps the fixture's actions in the compact layout; after every
    step the gathered stack of every env (u8 and f32 = u8 * (1/255), SB3 preprocess_obs) and, where the
    env finished, the gathered terminal stack (terminal row + older rows) equal the oracle's stack and
    terminal_observation stack; at the end one random-order minibatch gather over every (t, env) of the
    rollout equals the stacks recorded along the way."""
    _need_gpu()
    import os
    import oracle as O
    import trajcheck as TC
    from mgx import MgxEngine
    from mgx.compact import CompactBuffer
    d = dict(np.load(os.path.join(os.path.dirname(TC.__file__), "golden", "traj", name + ".npz")))
    cfg, T = TC.fixture_cfg(d)
    T = min(T, 256)
    kw = dict(cfg)
    n = kw.pop("n_envs")
    eng = MgxEngine(n_envs=n, n_stack=n_stack, terminal_mode="all", mission_dtype=torch.uint8, **kw)
    buf = CompactBuffer(eng, T)
    fs = O.FrameStackOracle(n, n_stack)

    def raw(img, dr, ms):
        return dict(image=O.vec_transpose_image(img), direction=O.one_hot_dir(dr), mission=ms.astype(np.int64))

    def check(g, want, f32, tag):
        if f32:
            assert np.array_equal(g["image"].cpu().numpy(), want["image"].astype(np.float32) * np.float32(1.0 / 255.0)), tag
            assert np.array_equal(g["direction"].cpu().numpy(), want["direction"].astype(np.float32)), tag
        else:
            assert np.array_equal(g["image"].cpu().numpy(), want["image"]), tag
            assert np.array_equal(g["direction"].cpu().numpy(), want["direction"]), tag
        assert np.array_equal(g["mission"].cpu().numpy().astype(np.int64), want["mission"]), tag

    eng.reset()
    buf.observe(0)
    stacks = [fs.reset(raw(d["reset0_image"], d["reset0_dir"], d["reset0_mission"]))]
    check(buf.gather_step(0, f32=False), stacks[0], False, "reset")
    n_term = 0
    for t in range(T):
        buf.step(t, torch.as_tensor(d["actions"][t].astype(np.int32), device=eng.device))
        done = (d["terminated"][t] | d["truncated"][t]).astype(bool)
        cur = raw(np.where(done[:, None, None, None], d["r_image"][t], d["image"][t]),
                  np.where(done, d["r_dir"][t], d["dir"][t]), np.where(done[:, None], d["r_mission"][t], d["mission"][t]))
        st, term = fs.step(cur, done, raw(d["image"][t], d["dir"][t], d["mission"][t]))
        stacks.append(st)
        check(buf.gather_step(t + 1, f32=bool(t % 2)), st, bool(t % 2), ("obs", t))
        if done.any():
            envs = np.nonzero(done)[0]
            n_term += envs.size
            g = buf.gather_step(t, terminal=True, f32=bool(t % 3 == 0), envs=torch.as_tensor(envs, device=eng.device))
            check(g, {k: v[envs] for k, v in term.items()}, bool(t % 3 == 0), ("terminal", t))
    assert n_term > 0
    eng.poll_error()
    gen = torch.Generator(device="cpu")
    gen.manual_seed(5)
    perm = torch.randperm((T + 1) * n, generator=gen)
    tt, ee = (perm // n).numpy(), (perm % n).numpy()
    g = buf.gather(torch.as_tensor((buf.H + tt) * n + ee, device=eng.device), f32=False)
    want = {k: np.stack([stacks[a][k][b] for a, b in zip(tt, ee)]) for k in ("image", "direction", "mission")}
    check(g, want, False, "minibatch")
