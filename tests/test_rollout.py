"""The fused rollout (mgx_rollout_compact: K compact steps in one launch, mgx/compact.py
CompactBuffer.rollout) against the per-step kernel and the C oracle: every step's observation row,
mission id, reward, done / terminated / truncated flags, the terminal rows, the counters and the
engine state after every chunk must equal K mgx_step_compact calls bit for bit (which are pinned to
the reference fixtures, test_gpu_parity.py), and the C oracle directly at BASELINE sizes."""
import numpy as np
import pytest

import trajcheck as TC

torch = pytest.importorskip("torch")

pytestmark = pytest.mark.gpu


def _need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


def _engines(kw, n, **ekw):
    from mgx import MgxEngine
    from mgx.compact import CompactBuffer
    a = MgxEngine(n_envs=n, terminal_mode="all", mission_dtype=torch.uint8, reward64=False, **kw, **ekw)
    b = MgxEngine(n_envs=n, terminal_mode="all", mission_dtype=torch.uint8, reward64=False, **kw, **ekw)
    return a, b


CASES = [dict(problem="multi", mission=5, size=8, n=4096),                     # config 2's GTG
         dict(problem="multi", mission=None, size=8, n=1000),                  # ragged last workgroup
         dict(problem="multi", mission=1, size=16, n=300),
         dict(problem="multi", mission=1, size=16, n=130, see_through_walls=False),
         dict(problem="multi", mission=2, size=11, n=257, all_doors_open=True),
         dict(problem="mov", mission=None, size=8, n=200),                     # 'move' target ranges
         dict(problem="multi", mission=None, size=8, n=512, manual=True)]


@pytest.mark.parametrize("case", CASES, ids=lambda c: "_".join("%s%s" % (k[:3], v) for k, v in c.items()))
@pytest.mark.parametrize("chunks", [(32,), (5, 11, 16)], ids=["epoch", "split"])
def test_rollout_equals_per_step(case, chunks):
    """Two engines of one config and seed: one steps per call (mgx_step_compact), the other runs the
    same actions in fused chunks (a whole refill epoch, or an epoch split 5 + 11 + 16) -- over
    several epochs with the buffer carried over, every output and the final state equal."""
    _need_gpu()
    from mgx.compact import CompactBuffer
    kw = dict(case)
    n = kw.pop("n")
    E = 32
    ref, fus = _engines(kw, n, refill_every=E)
    assert ref.refill_every == E and sum(chunks) == E
    T = 2 * E
    br, bf = CompactBuffer(ref, T), CompactBuffer(fus, T)
    ref.reset(); fus.reset()
    br.observe(0); bf.observe(0)
    g = torch.Generator(device=ref.device)
    g.manual_seed(9)
    for rollout in range(3):
        if rollout:
            br.carry_over(); bf.carry_over()
        acts = torch.randint(0, 7, (T, n), device=ref.device, generator=g, dtype=torch.int32)
        if rollout == 1:
            acts[3:9] = 6                                     # bursts of 'done': pops on consecutive steps
        t = 0
        while t < T:
            for k in chunks:
                bf.rollout(t, acts[t:t + k].contiguous())
                for j in range(k):
                    br.step(t + j, acts[t + j])
                t += k
                assert torch.equal(br.terminal_rows, bf.terminal_rows), (rollout, t)
        for name in ("rows", "mids", "starts", "rewards", "terminated", "truncated"):
            assert torch.equal(getattr(br, name), getattr(bf, name)), (rollout, name)
        for name in ("ep_return", "ep_len", "livelock"):
            assert torch.equal(getattr(ref, name), getattr(fus, name)), (rollout, name)
    ref.poll_error()
    fus.poll_error()
    a, b = ref.dump_state(), fus.dump_state()
    for k in a:
        assert np.array_equal(np.asarray(a[k]), np.asarray(b[k]), equal_nan=True), k
    sa, sb = ref.stats(), fus.stats()
    # ('queued' may differ: the refill reads each ring head once, at its start, concurrently with the
    # steps -- per-step calls may already have advanced some heads, the fused kernel writes them at its
    # end; both keep >= K episodes queued at every join, DESIGN §4.3.  What is produced -- and so the
    # producer-side max MT cursor -- is a prefix of the same episode sequence either way; the
    # consumed episodes are the same.)
    for k in ("steps", "resets", "livelocks", "calls"):
        assert sa[k] == sb[k], (k, sa, sb)
    assert sb["queued"] >= E * n, sb


def test_rollout_bursts_of_pops():
    """Over 640 steps with 'done' on 3 of 4 actions every env pops > 300 episodes (pops on most
    consecutive steps, the staged ring episodes cycling through both LDS buffers).  Fused chunks equal
    per-step calls bit for bit.  (Ring positions are u16 since round 3: test_ring_positions_wrap_u16
    runs them past 65,535 -> 0.)"""
    _need_gpu()
    from mgx.compact import CompactBuffer
    n, E, T = 512, 32, 64
    ref, fus = _engines(dict(problem="multi", mission=5, size=8), n, refill_every=E)
    br, bf = CompactBuffer(ref, T), CompactBuffer(fus, T)
    ref.reset(); fus.reset()
    br.observe(0); bf.observe(0)
    g = torch.Generator(device=ref.device)
    g.manual_seed(77)
    for rollout in range(10):
        if rollout:
            br.carry_over(); bf.carry_over()
        acts = torch.randint(0, 7, (T, n), device=ref.device, generator=g, dtype=torch.int32)
        acts = torch.where(torch.rand((T, n), device=ref.device, generator=g) < 0.75, 6, acts).to(torch.int32)
        for t in range(0, T, E):
            bf.rollout(t, acts[t:t + E].contiguous())
            for j in range(E):
                br.step(t + j, acts[t + j])
        for name in ("rows", "mids", "starts", "rewards", "terminated", "truncated"):
            assert torch.equal(getattr(br, name), getattr(bf, name)), (rollout, name)
        assert torch.equal(br.terminal_rows, bf.terminal_rows), rollout
    ref.poll_error()
    fus.poll_error()
    a, b = ref.dump_state(), fus.dump_state()
    for k in a:
        assert np.array_equal(np.asarray(a[k]), np.asarray(b[k]), equal_nan=True), k
    sa, sb = ref.stats(), fus.stats()
    assert sa["resets"] == sb["resets"] > 300 * n, (sa, sb)


def test_ring_positions_wrap_u16():
    """Ring positions (head, tail, pub, pubn, seen) are u16 counters mod 2^16 (rpos_t): with 'done' on
    97 % of the actions, 64 envs pop > 65,536 episodes each over 69,120 steps, so every position passes
    65,535 -> 0 -- the (rpos_t)(pub - head) levels, the refill's `tail - head` and `head - seen`, and the
    `head & (D - 1)` slots across the wrap.  Fused chunks (one launch per 64-step epoch) equal per-step
    calls bit for bit at every chunk; at the end both engines' states equal the C oracle's."""
    _need_gpu()
    import oracle as O
    from mgx.compact import CompactBuffer
    n, E = 64, 64
    nchunk = 1080
    ref, fus = _engines(dict(problem="multi", mission=5, size=8), n, refill_every=E)
    ov = O.OracleVec("multi", 5, 8, 4, n, 42)
    br, bf = CompactBuffer(ref, E), CompactBuffer(fus, E)
    ref.reset(); fus.reset(); ov.reset()
    br.observe(0); bf.observe(0)
    rng = np.random.default_rng(65536)
    acts = np.where(rng.random((nchunk * E, n)) < 0.97, 6, rng.integers(0, 7, (nchunk * E, n))).astype(np.int32)
    ad = torch.as_tensor(acts, device=ref.device)
    for c in range(nchunk):
        if c:
            br.carry_over(); bf.carry_over()
        bf.rollout(0, ad[c * E:(c + 1) * E])
        for j in range(E):
            br.step(j, ad[c * E + j])
        if c % 8 == 7 or c == nchunk - 1:
            for name in ("rows", "mids", "starts", "rewards", "terminated", "truncated"):
                assert torch.equal(getattr(br, name), getattr(bf, name)), (c, name)
            assert torch.equal(br.terminal_rows, bf.terminal_rows), c
    for t in range(nchunk * E):
        ov.step(acts[t])
    ref.poll_error()
    fus.poll_error()
    sa, sb = ref.stats(), fus.stats()
    assert sa["resets"] == sb["resets"] > 65600 * n, (sa, sb)
    want = ov.dump()
    for eng in (ref, fus):
        got = eng.dump_state()
        for k in ("grid", "agent", "carrying", "step_count", "mission_done", "mtwords", "pcg", "target"):
            assert np.array_equal(got[k], want[k]), k
        assert np.array_equal(got["stored_reward"], want["stored_reward"], equal_nan=True)


@pytest.mark.parametrize("problem,mission,size,n,T,offset", [("multi", 5, 8, 65536, 64, 0),
                                                               ("multi", None, 8, 32768, 64, 32768),
                                                               ("multi", 1, 16, 131072, 32, 0)],
                         ids=["cfg2_65536", "cfg4_32768_rank1", "cfg5_131072"])
def test_rollout_full_size_matches_oracle(problem, mission, size, n, T, offset):
    """BASELINE per-GPU sizes: the fused rollout of T steps (whole refill epochs) against the C
    oracle -- every env's row, done flag and f32 reward at every step, then every env's state.
    cfg4_32768_rank1 is rank 1's shard of config 4 (ALL mixed 8x8, env_index_offset = 32,768: envs
    seeded 42 + 32,768 + i), what ranks 1-7 of the 8-GPU bench run."""
    _need_gpu()
    import oracle as O
    from mgx import MgxEngine
    from mgx._lib import mission_tokens
    from mgx.compact import CompactBuffer
    E = 32
    ov = O.OracleVec(problem, mission, size, 4, n, 42, index_offset=offset)
    eng = MgxEngine(problem=problem, mission=mission, size=size, n_envs=n, terminal_mode="truncated",
                    mission_dtype=torch.uint8, refill_every=E, env_index_offset=offset)
    buf = CompactBuffer(eng, T)
    tok = mission_tokens()
    ov.reset()
    eng.reset()
    buf.observe(0)
    acts = np.random.default_rng(2024).integers(0, 7, (T, n)).astype(np.int32)
    ad = torch.as_tensor(acts, device=eng.device)
    for t in range(0, T, E):
        buf.rollout(t, ad[t:t + E].contiguous())
    torch.cuda.synchronize()
    rows, mids = buf.rows.cpu().numpy(), buf.mids.cpu().numpy()
    starts, rew = buf.starts.cpu().numpy().astype(bool), buf.rewards.cpu().numpy()
    H = buf.H
    for t in range(T):
        o = ov.step(acts[t])
        done = (o["terminated"] | o["truncated"]).astype(bool)
        r = rows[H + 1 + t]
        img = r[:, 1:].reshape(n, 3, 7, 7).transpose(0, 2, 3, 1)
        assert np.array_equal(starts[H + 1 + t], done), t
        assert np.array_equal(img, np.where(done[:, None, None, None], o["r_image"], o["image"])), t
        assert np.array_equal(r[:, 0], np.where(done, o["r_dir"], o["dir"])), t
        assert np.array_equal(tok[mids[H + 1 + t]], np.where(done[:, None], o["r_mission"], o["mission"])), t
        assert np.array_equal(rew[t], o["reward"].astype(np.float32)), t
    a, b = eng.dump_state(), ov.dump()
    for k in ("grid", "agent", "carrying", "step_count", "mission_done", "mtwords", "pcg", "target"):
        assert np.array_equal(a[k], b[k]), k
    assert np.array_equal(a["stored_reward"], b["stored_reward"], equal_nan=True)
    eng.poll_error()


@pytest.mark.parametrize("path", TC.fixtures(), ids=lambda p: p.split("/")[-1][:-4])
def test_rollout_matches_reference_fixture(path):
    """Every reference fixture through the fused rollout in whole epochs of 16 steps: each step's
    observation (the terminal frame where the episode ended, from the terminal row of that chunk when
    it is the env's last ending in it), reward, flags and new-episode observation; at every chunk end
    the env state."""
    _need_gpu()
    from mgx import MgxEngine
    from mgx._lib import mission_tokens
    from mgx.compact import CompactBuffer
    d = dict(np.load(path))
    cfg, T = TC.fixture_cfg(d)
    kw = dict(cfg)
    n = kw.pop("n_envs")
    E = 16
    eng = MgxEngine(n_envs=n, terminal_mode="all", mission_dtype=torch.uint8, refill_every=E, **kw)
    buf = CompactBuffer(eng, T)
    tok = mission_tokens()
    eng.reset()
    buf.observe(0)
    H = buf.H
    r0 = buf.rows[H].cpu().numpy()
    assert np.array_equal(r0[:, 1:].reshape(n, 3, 7, 7).transpose(0, 2, 3, 1), d["reset0_image"])
    acts = torch.as_tensor(d["actions"].astype(np.int32), device=eng.device)
    for c in range(T // E):
        t0 = c * E
        buf.rollout(t0, acts[t0:t0 + E].contiguous())
        torch.cuda.synchronize()
        rows, mids = buf.rows.cpu().numpy(), buf.mids.cpu().numpy()
        starts, rew = buf.starts.cpu().numpy().astype(bool), buf.rewards.cpu().numpy()
        trm, trc = buf.terminated.cpu().numpy(), buf.truncated.cpu().numpy()
        trows = buf.terminal_rows.cpu().numpy()
        last_end = np.full(n, -1)
        for t in range(t0, t0 + E):
            done = (d["terminated"][t] | d["truncated"][t]).astype(bool)
            last_end[done] = t
            r = rows[H + 1 + t]
            img = r[:, 1:].reshape(n, 3, 7, 7).transpose(0, 2, 3, 1)
            assert np.array_equal(starts[H + 1 + t], done), t
            assert np.array_equal(trm[t], d["terminated"][t]) and np.array_equal(trc[t], d["truncated"][t]), t
            assert np.array_equal(rew[t], d["reward"][t].astype(np.float32)), t
            assert np.array_equal(img[~done], d["image"][t][~done]), t
            assert np.array_equal(img[done], d["r_image"][t][done]), t
            assert np.array_equal(r[~done, 0], d["dir"][t][~done]) and np.array_equal(r[done, 0], d["r_dir"][t][done]), t
            assert np.array_equal(tok[mids[H + 1 + t]][~done], d["mission"][t][~done]), t
            assert np.array_equal(tok[mids[H + 1 + t]][done], d["r_mission"][t][done]), t
        for i in np.nonzero(last_end >= 0)[0]:                      # the chunk's last terminal row per env
            t = last_end[i]
            got = trows[i, 1:].reshape(3, 7, 7).transpose(1, 2, 0)
            assert np.array_equal(got, d["image"][t][i]) and trows[i, 0] == d["dir"][t][i], (t, i)
        st = eng.dump_state()
        t = t0 + E - 1
        done = (d["terminated"][t] | d["truncated"][t]).astype(bool)
        for k in TC.STATE_KEYS:
            assert np.array_equal(st[k][~done], d[k][t][~done]), (t, k)
        for k in ("grid", "agent", "mtwords", "pcg", "target"):
            assert np.array_equal(st[k][done], d["r_" + k][t][done]), (t, k)
        assert np.array_equal(st["mission_done"], d["mission_done"][t]), t
        assert np.array_equal(st["stored_reward"], d["stored_reward"][t], equal_nan=True), t
    eng.poll_error()


def test_rollout_rejects_chunks_across_epochs():
    _need_gpu()
    from mgx import MgxEngine, MgxError
    from mgx.compact import CompactBuffer
    eng = MgxEngine(problem="multi", mission=5, size=8, n_envs=128, refill_every=16, mission_dtype=torch.uint8)
    buf = CompactBuffer(eng, 64)
    eng.reset()
    buf.observe(0)
    a = torch.zeros((64, 128), dtype=torch.int32, device=eng.device)
    buf.rollout(0, a[:10].contiguous())
    with pytest.raises(MgxError, match="refill epoch"):
        buf.rollout(10, a[10:20].contiguous())          # 10 + 10 > 16
    buf.rollout(10, a[10:16].contiguous())
    buf.rollout(16, a[16:32].contiguous())
    eng.poll_error()


@pytest.mark.parametrize("layout", ["fused", "compact"])
@pytest.mark.parametrize("problem,mission,size,n", [("multi", 5, 8, 4096), ("multi", None, 8, 2048), ("multi", 1, 16, 1024)],
                         ids=["cfg2", "cfg4", "cfg5"])
def test_shards_equal_slices_of_one_engine(problem, mission, size, n, layout):
    """Multi-GPU sharding: rank r owns global envs [r*n, (r+1)*n) through env_index_offset.
    Two shard engines (offsets 0 and n) against ONE engine of 2n envs, same actions: every output row,
    mission id, reward, done / terminated / truncated flag, terminal row and counter, and every env's state
    at the end, is the matching slice of the single engine's, bit for bit -- in the fused rollout (the
    bench's headline launch) and per step (the PPO path)."""
    _need_gpu()
    from mgx import MgxEngine
    from mgx.compact import CompactBuffer
    E, T, rolls = 32, 64, 3
    kw = dict(problem=problem, mission=mission, size=size, terminal_mode="all", mission_dtype=torch.uint8,
              refill_every=E)
    whole = MgxEngine(n_envs=2 * n, **kw)
    shards = [MgxEngine(n_envs=n, env_index_offset=r * n, **kw) for r in range(2)]
    bw = CompactBuffer(whole, T)
    bs = [CompactBuffer(s, T) for s in shards]
    for e, b in [(whole, bw)] + list(zip(shards, bs)):
        e.reset()
        b.observe(0)
    g = torch.Generator(device=whole.device)
    g.manual_seed(4242)
    for roll in range(rolls):
        if roll:
            for b in [bw] + bs:
                b.carry_over()
        acts = torch.randint(0, 7, (T, 2 * n), device=whole.device, generator=g, dtype=torch.int32)
        for t in range(0, T, E):
            chunk = acts[t:t + E]
            if layout == "fused":
                bw.rollout(t, chunk.contiguous())
                for r in range(2):
                    bs[r].rollout(t, chunk[:, r * n:(r + 1) * n].contiguous())
            else:
                for j in range(E):
                    bw.step(t + j, chunk[j])
                    for r in range(2):
                        bs[r].step(t + j, chunk[j, r * n:(r + 1) * n].contiguous())
        for name in ("rows", "mids", "starts", "rewards", "terminated", "truncated"):
            w = getattr(bw, name)
            for r in range(2):
                assert torch.equal(getattr(bs[r], name), w[:, r * n:(r + 1) * n]), (roll, name, r)
        for r in range(2):
            assert torch.equal(bs[r].terminal_rows, bw.terminal_rows[r * n:(r + 1) * n]), (roll, r)
            for name in ("ep_return", "ep_len", "livelock"):
                assert torch.equal(getattr(shards[r], name), getattr(whole, name)[r * n:(r + 1) * n]), (roll, name)
    whole.poll_error()
    a = whole.dump_state()
    tot = 0
    for r in range(2):
        shards[r].poll_error()
        b = shards[r].dump_state()
        for k in a:
            assert np.array_equal(np.asarray(b[k]), np.asarray(a[k])[r * n:(r + 1) * n], equal_nan=True), (r, k)
        tot += shards[r].stats()["resets"]
    assert tot == whole.stats()["resets"]


def test_kernel_clock_records_every_launch():
    """mgx_set_clock (the bench's roofline timer): every step-kernel launch (fused rollout or per step) and
    every refill launch records one span on the device, graph replays included; each span is positive and
    lies inside the HIP-event window around its launches; clocked and unclocked engines step identically."""
    _need_gpu()
    from mgx import MgxEngine
    from mgx.compact import CompactBuffer
    n, E = 4096, 16
    kw = dict(problem="multi", mission=5, size=8, n_envs=n, refill_every=E, mission_dtype=torch.uint8)
    a, b = MgxEngine(**kw), MgxEngine(**kw)
    a.enable_clock(slots=64)
    ba, bb = CompactBuffer(a, E, ring=True), CompactBuffer(b, E, ring=True)
    a.reset(); b.reset()
    assert a.clock_launches(1) == 1                          # mgx_reset's synchronous fill
    ba.observe(0); bb.observe(0)
    acts = torch.randint(0, 7, (3 * E, n), device=a.device, dtype=torch.int32)
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ev0.record()
    ba.rollout(0, acts[:E]); bb.rollout(0, acts[:E])
    ev1.record()
    for t in range(E):                                       # a second epoch, one launch per step
        ba.step(t, acts[E + t]); bb.step(t, acts[E + t])
    a.join()                                                 # (no dependency across the capture)
    torch.cuda.synchronize()
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        g = torch.cuda.CUDAGraph()
        g.capture_begin()
        ba.rollout(0, acts[2 * E:])
        a.join()
        g.capture_end()
    g.replay()
    for t in range(E):
        bb.step(t, acts[2 * E + t])
    a.join()
    torch.cuda.synchronize()
    assert a.clock_launches(0) == 1 + E + 1
    assert a.clock_launches(1) == 1 + 3
    spans = a.clock_spans_us(0, 0, a.clock_launches(0))
    assert all(0 < x < 1e5 for x in spans), spans
    assert spans[0] <= ev0.elapsed_time(ev1) * 1e3 + 1.0, (spans[0], ev0.elapsed_time(ev1))
    assert all(0 < x < 1e6 for x in a.clock_spans_us(1, 0, 4))
    assert torch.equal(ba.rows, bb.rows) and torch.equal(ba.starts, bb.starts)
    sa, sb = a.dump_state(), b.dump_state()
    for k in ("grid", "agent", "mtwords", "pcg"):
        assert np.array_equal(sa[k], sb[k]), k


@pytest.mark.gpu
def test_kernel_clock_classes_keep_their_grids_at_s16():
    """at S = 16 the fused rollout runs 32-env blocks (twice the step kernels' grid); it records into a clock
    class of its own (3), so per-step launches (class 0) and rollout launches on one engine never mix grids."""
    _need_gpu()
    from mgx import MgxEngine
    from mgx.compact import CompactBuffer
    n, E = 1024, 8
    eng = MgxEngine(problem="multi", mission=1, size=16, n_envs=n, refill_every=E, mission_dtype=torch.uint8)
    eng.enable_clock(slots=16)
    assert eng.rollout_clock_class() == 3
    cb = CompactBuffer(eng, E, ring=True)
    eng.reset()
    cb.observe(0)
    acts = torch.randint(0, 7, (3 * E, n), device=eng.device, dtype=torch.int32)
    cb.rollout(0, acts[:E])
    for t in range(E):
        cb.step(t, acts[E + t])
    cb.carry_over()
    cb.rollout(0, acts[2 * E:])
    eng.join()
    torch.cuda.synchronize()
    assert eng.clock_launches(0) == E and eng.clock_launches(3) == 2
    for cls, k in ((0, E), (3, 2)):
        spans = eng.clock_spans_us(cls, 0, k)
        assert len(spans) == k and all(0 < x < 1e5 for x in spans), (cls, spans)
    eng.poll_error()
