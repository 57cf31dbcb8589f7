"""The synthetic random policy (mgx_random_actions, ABI 7) and the ring-level diagnostic (mgx_ring_levels).

bench.py's graphs draw every replay's actions with mgx_random_actions (round 6): replaying one fixed slice of actions
(rounds 2-5) gave each env a persistent consumption rate and drained the rings of the envs whose slice held many
'done' actions (tools/diag_ring_levels.py).  CPU: the host restatement (oracle.random_actions_ref) is uniform and
changes with the counter.  GPU: the kernel equals the restatement bit for bit, advances its counter on the device
(also inside a replayed hipGraph), and the rings of a long fresh-action rollout stay far above the invariant's floor."""
import numpy as np
import pytest
import torch

import oracle as O


def test_reference_draws_are_uniform_and_fresh_per_counter():
    n = 7 * 100_000
    a = O.random_actions_ref(n, 4321, 0)
    b = O.random_actions_ref(n, 4321, 1)
    assert a.dtype == np.int32 and a.min() == 0 and a.max() == 6
    for x in (a, b):
        cnt = np.bincount(x, minlength=7)
        chi2 = float(((cnt - n / 7) ** 2 / (n / 7)).sum())
        assert chi2 < 30.0, chi2                        # 6 dof: p ~ 4e-5
    assert (a == b).mean() < 0.2                        # a new counter is a new draw (1/7 agree by chance)
    assert np.array_equal(O.random_actions_ref(1000, 4321, 5), O.random_actions_ref(1000, 4321, 5))
    c = O.random_actions_ref(1000, 17, 0, n_actions=3)
    assert set(np.unique(c)) <= {0, 1, 2}


@pytest.mark.gpu
def test_random_actions_match_reference_and_advance():
    from mgx import random_actions
    dev = torch.device("cuda", 0)
    n = 65536 * 20 + 13                                  # ragged: not a multiple of the block
    out = torch.empty(n, dtype=torch.int32, device=dev)
    ctr = torch.zeros(2, dtype=torch.int64, device=dev)
    for c in range(3):
        random_actions(out, ctr, seed=4321)
        torch.cuda.synchronize()
        assert np.array_equal(out.cpu().numpy(), O.random_actions_ref(n, 4321, c)), c
        assert int(ctr[0]) == c + 1 and int(ctr[1]) == 0
    small = torch.empty(5, dtype=torch.int32, device=dev)
    random_actions(small, ctr, seed=9, n_actions=3)
    assert np.array_equal(small.cpu().numpy(), O.random_actions_ref(5, 9, 3, n_actions=3))


@pytest.mark.gpu
@pytest.mark.parametrize("n_actions", [1, 2, 65536])
def test_random_actions_extreme_action_counts(n_actions):
    """n_actions at the ABI's bounds: 1 (every draw 0), 2, and 65,536 -- equal to the host restatement."""
    from mgx import random_actions
    dev = torch.device("cuda", 0)
    out = torch.empty(4097, dtype=torch.int32, device=dev)
    ctr = torch.zeros(2, dtype=torch.int64, device=dev)
    random_actions(out, ctr, seed=2024, n_actions=n_actions)
    got = out.cpu().numpy()
    assert np.array_equal(got, O.random_actions_ref(4097, 2024, 0, n_actions=n_actions))
    assert got.min() >= 0 and got.max() < n_actions
    if n_actions == 1:
        assert not got.any()


@pytest.mark.gpu
def test_random_actions_fresh_in_graph_replays():
    from mgx import random_actions
    dev = torch.device("cuda", 0)
    n = 4096
    out = torch.empty(n, dtype=torch.int32, device=dev)
    ctr = torch.zeros(2, dtype=torch.int64, device=dev)
    s = torch.cuda.Stream(dev)
    with torch.cuda.stream(s):
        g = torch.cuda.CUDAGraph()
        g.capture_begin()
        random_actions(out, ctr, seed=77)
        g.capture_end()
    torch.cuda.synchronize()
    ctr.zero_()
    for c in range(4):
        g.replay()
        torch.cuda.synchronize()
        assert np.array_equal(out.cpu().numpy(), O.random_actions_ref(n, 77, c)), c


@pytest.mark.gpu
def test_ring_levels_stay_off_the_floor_with_fresh_actions():
    """4,096 envs, 20-step fused epochs, 200 epochs of fresh random actions: every ring level stays within (2K, D],
    the levels sum to mgx_stats' queued count, and production keeps up with consumption."""
    from mgx import MgxEngine, random_actions
    from mgx.compact import CompactBuffer
    dev = torch.device("cuda", 0)
    n, E = 4096, 20
    eng = MgxEngine(problem="multi", mission=5, size=8, n_envs=n, terminal_mode="truncated", refill_every=E,
                    mission_dtype=torch.uint8, device=dev)
    cbuf = CompactBuffer(eng, E, ring=True)
    acts = torch.empty((E, n), dtype=torch.int32, device=dev)
    ctr = torch.zeros(2, dtype=torch.int64, device=dev)
    eng.reset()
    cbuf.observe(0)
    D = eng.ring_depth
    lv0 = eng.ring_levels()
    # mgx_reset fills every ring to D, less the attempts it abandoned (live-locks cost the fill one episode each)
    assert lv0.max() == D and lv0.min() >= D - 24, (lv0.min(), lv0.max())
    s0 = eng.stats()
    for _ in range(200):
        random_actions(acts, ctr, seed=4321)
        cbuf.carry_over()
        cbuf.rollout(0, acts)
    eng.join()
    torch.cuda.synchronize()
    eng.poll_error()
    lv = eng.ring_levels().astype(np.int64)
    s1 = eng.stats()
    assert int(lv.sum()) == s1["queued"]
    assert lv.min() > 2 * E and lv.max() <= D, (lv.min(), lv.max())
    cons = s1["resets"] - s0["resets"]
    prod = cons + s1["queued"] - s0["queued"]
    assert cons > 0.12 * n * 200 * E                     # a random policy resets ~0.146 envs per step
    assert prod > cons - n * 3 * E                       # the rings started full: production follows consumption
    assert lv.mean() > D - 80, lv.mean()                 # the levels' mean deficit settles at ~25-30 (D = 512)


@pytest.mark.gpu
@pytest.mark.parametrize("cfg", [dict(mission=5, size=8, n=1000), dict(mission=1, size=16, n=520)],
                         ids=["gtg8_ragged", "tgl16_epb32"])
def test_rollout_random_policy_equals_explicit_actions(cfg):
    """mgx_set_random_policy: three fused launches that draw their own actions give the same rows, rewards, dones
    and final state, bit for bit, as the same launches fed mgx_random_actions' draws (the host restatement) at
    counters 0, 1, 2."""
    from mgx import MgxEngine
    from mgx.compact import CompactBuffer
    dev = torch.device("cuda", 0)
    n, E, seed = cfg["n"], 16, 987654321
    kw = dict(problem="multi", mission=cfg["mission"], size=cfg["size"], n_envs=n, terminal_mode="truncated",
              refill_every=E, mission_dtype=torch.uint8, device=dev)
    a, b = MgxEngine(**kw), MgxEngine(**kw)
    b.set_random_policy(seed)
    bufs = [CompactBuffer(x, E, ring=True) for x in (a, b)]
    for x, cb in zip((a, b), bufs):
        x.reset()
        cb.observe(0)
    for c in range(3):
        acts = torch.as_tensor(O.random_actions_ref(E * n, seed, c).reshape(E, n), device=dev)
        for cb in bufs:
            cb.carry_over()
        bufs[0].rollout(0, acts)
        bufs[1].rollout(0, None, K=E)
        torch.cuda.synchronize()
        for name in ("rows", "mids", "rewards", "starts", "terminated", "truncated", "terminal_rows"):
            assert torch.equal(getattr(bufs[0], name), getattr(bufs[1], name)), (c, name)
    for x in (a, b):
        x.join()
        x.poll_error()
    sa, sb = a.dump_state(), b.dump_state()
    for k in sa:
        assert np.array_equal(sa[k], sb[k], equal_nan=sa[k].dtype.kind == "f"), k
    assert b.random_launches == 3
