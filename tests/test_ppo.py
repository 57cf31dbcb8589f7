"""PPO layer (mgx/policy.py, mgx/ppo.py) against restatements of the
reference's policy (src/policies.py) and of SB3's collect_rollouts / PPO.train
(SB3 is not installed: parity with SB3 itself is unpinned).

CPU: policy structure and init, mission-feature cache, the training step vs
an SB3-shaped loop (swap_and_flatten order, per-minibatch normalisation,
clipping), data-parallel training over gloo with world size 2.
GPU: the device-resident rollout collector vs the SB3 host loop driven
through MgxVecEnv (same policy, same torch RNG)."""
import copy
import os
import socket

import numpy as np
import pytest

torch = pytest.importorskip("torch")

from mgx.policy import ActorCriticPolicy, preprocess  # noqa: E402
from mgx.ppo import PPOConfig, RolloutBuffer, Trainer  # noqa: E402


def _rand_obs(n, n_stack=4, seed=0):
    g = torch.Generator().manual_seed(seed)
    return dict(image=torch.randint(0, 11, (n, 3 * n_stack, 7, 7), dtype=torch.uint8, generator=g),
                direction=torch.randint(0, 2, (n, 4 * n_stack), dtype=torch.uint8, generator=g),
                mission=torch.randint(0, 32, (n, 32 * n_stack), dtype=torch.uint8, generator=g))


def test_policy_structure_and_init():
    torch.manual_seed(0)
    p = ActorCriticPolicy()
    fe = p.features_extractor
    assert fe.features_dim == 16 + 64 + 128
    assert list(fe.extractors.keys()) == ["direction", "image", "mission"]
    conv0 = fe.extractors["image"][0]
    assert conv0.in_channels == 12 and conv0.out_channels == 16           # 3 * n_frames_stack
    assert fe.extractors["direction"][0].in_features == 16                # 4 * n_frames_stack
    assert fe.extractors["mission"][0].num_embeddings == 32               # Embedding is not widened
    gru = fe.extractors["mission"][1]
    assert gru.hidden_size == 128 and gru.batch_first
    for m in p.modules():                                                 # init_weights (policies.py:245-255)
        if isinstance(m, torch.nn.Linear):
            assert torch.allclose(m.weight.pow(2).sum(1), torch.ones(m.out_features), atol=1e-5)
            assert torch.all(m.bias == 0)
    w = conv0.weight.reshape(16, -1)
    assert torch.allclose(w @ w.t(), 2.0 * torch.eye(16), atol=1e-4)      # orthogonal, gain sqrt(2)
    assert p.optimizer.defaults["eps"] == 1e-8
    a, v, lp = p(_rand_obs(7))
    assert a.shape == (7,) and v.shape == (7,) and lp.shape == (7,)
    assert int(a.max()) < 7


def test_mission_cache_same_features_and_grads():
    torch.manual_seed(1)
    p = ActorCriticPolicy()
    q = ActorCriticPolicy(mission_cache=True)
    q.load_state_dict(p.state_dict())
    obs = _rand_obs(64, seed=3)
    obs["mission"][10:40] = obs["mission"][5]                              # many repeated rows
    obs["mission"][50:] = 0
    acts = torch.randint(0, 7, (64,))
    v1, l1, e1 = p.evaluate_actions(obs, acts)
    v2, l2, e2 = q.evaluate_actions(obs, acts)
    assert torch.allclose(v1, v2, atol=1e-6) and torch.allclose(l1, l2, atol=1e-6)
    (v1.sum() + l1.sum()).backward()
    (v2.sum() + l2.sum()).backward()
    for (n1, a), (_, b) in zip(p.named_parameters(), q.named_parameters()):
        assert torch.allclose(a.grad, b.grad, atol=1e-5, rtol=1e-4), n1


@pytest.mark.gpu
def test_mission_cache_same_features_and_grads_gpu_large_batch():
    """The same equality on the GPU at 40,000 rows: the uncached path splits the GRU batch into
    8,192-row chunks (MIOpen's RNN refuses 16,384 rows; CustomExtractor.gru_chunk) and the cached
    path runs the distinct rows only (padded to a power of two, chunked the same way); fp32
    tolerance 1e-5 on features, rtol 1e-3 on summed gradients (summation order differs)."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    torch.manual_seed(1)
    p = ActorCriticPolicy().cuda()
    q = ActorCriticPolicy(mission_cache=True).cuda()
    q.load_state_dict(p.state_dict())
    n = 40000
    obs = {k: v.cuda() for k, v in _rand_obs(n, seed=4).items()}
    # stacks drawn from 4,000 mission rows (>8,192 distinct stacks), a third with zero-filled older frames
    lib = torch.randint(0, 32, (4000, 32), dtype=torch.uint8, device="cuda")
    pick = torch.randint(0, 4000, (n, 4), device="cuda")   # > 8,192 distinct stacks: cache path chunks too
    m = lib[pick].reshape(n, 128)
    m[: n // 3, :64] = 0
    obs["mission"] = m
    assert p.features_extractor.gru_chunk < n
    pre = preprocess(obs)
    f1 = p.features_extractor(pre)
    f2 = q.features_extractor(pre)
    assert torch.allclose(f1, f2, atol=1e-5, rtol=1e-5)
    acts = torch.randint(0, 7, (n,), device="cuda")
    v1, l1, _ = p.evaluate_actions(obs, acts)
    v2, l2, _ = q.evaluate_actions(obs, acts)
    (v1.sum() + l1.sum()).backward()
    (v2.sum() + l2.sum()).backward()
    for (n1, a), (_, b) in zip(p.named_parameters(), q.named_parameters()):
        assert torch.allclose(a.grad, b.grad, atol=1e-3, rtol=1e-3), n1


def _fill_buffer(T, N, seed):
    g = torch.Generator().manual_seed(seed)
    buf = RolloutBuffer(T, N, 4, "cpu")
    for t in range(T):
        o = _rand_obs(N, seed=seed * 1000 + t)
        buf.image[t], buf.direction[t], buf.mission[t] = o["image"], o["direction"], o["mission"]
    buf.actions.copy_(torch.randint(0, 7, (T, N), generator=g))
    buf.values.copy_(torch.randn((T, N), generator=g))
    buf.log_probs.copy_(-torch.rand((T, N), generator=g) * 2)
    buf.advantages = torch.randn((T, N), generator=g)
    buf.returns = buf.advantages + buf.values
    a = buf.advantages.double()
    buf.adv_stats.copy_(torch.tensor([a.sum(), (a * a).sum(), float(a.numel())], dtype=torch.float64))
    return buf


def _sb3_train(policy, buf, cfg, perms, lr):
    """PPO.train as SB3 2.x writes it, over swap_and_flatten'ed buffer arrays."""
    def flat(x):   # [T, N, ...] -> [N*T, ...] env-major (RolloutBuffer.swap_and_flatten)
        return x.transpose(0, 1).reshape((x.shape[0] * x.shape[1],) + tuple(x.shape[2:]))
    obs_all = {k: flat(getattr(buf, k)) for k in ("image", "direction", "mission")}
    A, V, LP, ADV, RET = (flat(x) for x in (buf.actions, buf.values, buf.log_probs, buf.advantages, buf.returns))
    for g in policy.optimizer.param_groups:
        g["lr"] = lr
    for perm in perms:
        for s in range(0, perm.numel(), cfg.batch_size):
            idx = perm[s:s + cfg.batch_size]
            values, log_prob, entropy = policy.evaluate_actions({k: v[idx] for k, v in obs_all.items()}, A[idx])
            adv = ADV[idx]
            adv = (adv - adv.mean()) / (adv.std() + 1e-8)
            ratio = torch.exp(log_prob - LP[idx])
            policy_loss = -torch.min(adv * ratio, adv * torch.clamp(ratio, 1 - cfg.clip_range, 1 + cfg.clip_range)).mean()
            vp = V[idx] + torch.clamp(values - V[idx], -cfg.clip_range_vf, cfg.clip_range_vf)
            value_loss = torch.nn.functional.mse_loss(RET[idx], vp)
            loss = policy_loss + cfg.ent_coef * -torch.mean(entropy) + cfg.vf_coef * value_loss
            policy.optimizer.zero_grad()
            loss.backward()
            torch.nn.utils.clip_grad_norm_(policy.parameters(), cfg.max_grad_norm)
            policy.optimizer.step()


def test_train_step_matches_sb3_restatement():
    torch.manual_seed(2)
    cfg = PPOConfig(batch_size=32, n_epochs=2)
    T, N = 8, 12
    buf = _fill_buffer(T, N, 5)
    p = ActorCriticPolicy(optim_eps=cfg.optim_eps)
    q = copy.deepcopy(p)
    q.optimizer = torch.optim.Adam(q.parameters(), lr=3e-4, eps=cfg.optim_eps)
    perms = [torch.randperm(T * N, generator=torch.Generator().manual_seed(k)) for k in range(cfg.n_epochs)]
    it = iter(perms)
    tr = Trainer(p, cfg)
    progress = 0.37
    st = tr.train(buf, progress, perm_fn=lambda n: next(it))
    lr = max(progress * cfg.initial_learning_rate, cfg.final_learning_rate)
    assert st["lr"] == lr
    _sb3_train(q, buf, cfg, perms, lr)
    for (n1, a), (_, b) in zip(p.named_parameters(), q.named_parameters()):
        assert torch.allclose(a, b, atol=1e-6, rtol=1e-5), n1


def test_linear_schedule():
    from mgx.ppo import linear_schedule
    f = linear_schedule(3e-4, 3e-6)
    assert f(1.0) == 3e-4 and f(0.5) == 1.5e-4 and f(0.001) == 3e-6


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _dp_worker(rank, world, port, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.distributed.init_process_group("gloo", rank=rank, world_size=world)
    try:
        torch.manual_seed(100 + rank)                       # different init: learn() broadcasts rank 0's
        cfg = PPOConfig(batch_size=16, n_epochs=1)
        p = ActorCriticPolicy()
        for prm in p.parameters():
            torch.distributed.broadcast(prm.data, 0)
        buf = _fill_buffer(4, 8, 10 + rank)                 # each rank: its own env shard
        tr = Trainer(p, cfg, group=torch.distributed.group.WORLD)
        mean, std, s = tr.global_adv_stats(buf)
        tr.train(buf, 1.0, perm_fn=lambda n: torch.randperm(n, generator=torch.Generator().manual_seed(7)))
        flat = torch.cat([x.detach().reshape(-1) for x in p.parameters()])
        gathered = [torch.zeros_like(flat) for _ in range(world)]
        torch.distributed.all_gather(gathered, flat)
        out[rank] = dict(same=all(torch.equal(gathered[0], g) for g in gathered), mean=float(mean),
                         std=float(std), n=float(s[2]))
    finally:
        torch.distributed.destroy_process_group()


def test_data_parallel_gloo_world2():
    """Two ranks, each its own shard: one all-reduce of the advantage stats per
    rollout and one gradient all-reduce per optimiser step keep the replicas
    identical, and the global stats equal those of the concatenated shards."""
    import torch.multiprocessing as mp
    mgr = mp.Manager()
    out = mgr.dict()
    port = _free_port()
    mp.spawn(_dp_worker, args=(2, port, out), nprocs=2, join=True)
    a = torch.cat([_fill_buffer(4, 8, 10 + r).advantages.reshape(-1).double() for r in range(2)])
    for r in range(2):
        assert out[r]["same"]
        assert out[r]["n"] == a.numel()
        assert abs(out[r]["mean"] - float(a.mean())) < 1e-12
        assert abs(out[r]["std"] - float(a.std())) < 1e-9


# ------------------------------------------------------------------------ GPU
@pytest.mark.gpu
@pytest.mark.parametrize("env_kw,T", [(dict(problem="gtg", mission=5, size=6, num_objects=2), 48),
                                      (dict(problem="multi", mission=2, size=8, num_objects=4), 80)],
                         ids=["gtg6", "pkp8_config3"])
def test_rollout_collector_matches_sb3_loop(env_kw, T):
    """The device-resident collector (SB3 stacked layout) against SB3's collect_rollouts loop
    driven through the MgxVecEnv drop-in, on a small single-room case and on BASELINE config
    3's workload (multi / 'pick up' / 8x8; T=80 > max_steps so truncation bootstraps occur)."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import oracle as O
    from mgx import MgxEngine, MgxVecEnv
    from mgx.ppo import RolloutCollector
    n = 96
    cfg = PPOConfig(n_envs=n, horizon=T, env=env_kw, layout="sb3")
    torch.manual_seed(0)
    pol = ActorCriticPolicy().cuda()
    with torch.no_grad():
        pol.action_net.bias[6] = -30.0       # rarely 'done': episodes end on the goal or by truncation
    # device-resident collector
    eng = MgxEngine(n_envs=n, n_stack=4, terminal_mode="truncated", mission_dtype=torch.uint8, **env_kw)
    col = RolloutCollector(eng, pol, cfg)
    col.start()
    torch.manual_seed(1234)
    buf = col.collect()
    # SB3-shaped host loop over the VecEnv drop-in
    vec = MgxVecEnv(n, n_frames_stack=4, **env_kw)
    last_obs = vec.reset()
    last_starts = np.ones(n, bool)
    torch.manual_seed(1234)
    R = np.zeros((T, n), np.float32)
    ES = np.zeros((T, n), np.float32)
    V = np.zeros((T, n), np.float32)
    n_boot = 0
    with torch.no_grad():
        for t in range(T):
            obs_t = {k: torch.as_tensor(v).cuda() for k, v in last_obs.items()}
            for k in ("image", "direction", "mission"):
                assert torch.equal(obs_t[k].to(torch.int64), getattr(buf, k)[t].to(torch.int64)), (t, k)
            actions, values, log_probs = pol(obs_t)
            assert torch.equal(actions, buf.actions[t]), t
            new_obs, rewards, dones, infos = vec.step(actions.cpu().numpy())
            for idx, done in enumerate(dones):
                if done and infos[idx].get("terminal_observation") is not None and \
                        infos[idx].get("TimeLimit.truncated", False):
                    tob = {k: torch.as_tensor(v[None]).cuda() for k, v in infos[idx]["terminal_observation"].items()}
                    terminal_value = pol.predict_values(tob)[0]
                    rewards[idx] += cfg.gamma * terminal_value
                    n_boot += 1
            R[t], ES[t], V[t] = rewards, last_starts, values.cpu().numpy()
            last_obs, last_starts = new_obs, dones
        last_values = pol.predict_values({k: torch.as_tensor(v).cuda() for k, v in last_obs.items()})
    assert n_boot > 0, "no truncation exercised"
    assert np.array_equal(ES, buf.episode_starts.cpu().numpy())
    assert np.array_equal(V, buf.values.cpu().numpy())
    # bootstrap values: batch-1 vs batched GEMM -> tolerance on the bootstrapped entries only
    np.testing.assert_allclose(buf.rewards.cpu().numpy(), R, rtol=1e-6, atol=1e-6)
    want_a, want_r = O.gae(R, V, ES, last_values.cpu().numpy(), last_starts, cfg.gamma, cfg.gae_lambda)
    np.testing.assert_allclose(buf.advantages.cpu().numpy(), want_a, rtol=1e-5, atol=1e-5)
    np.testing.assert_allclose(buf.returns.cpu().numpy(), want_r, rtol=1e-5, atol=1e-5)
    eng.poll_error()


@pytest.mark.gpu
def test_compact_collector_equals_sb3_layout_collector():
    """CompactRolloutCollector (compact rows + mgx_gather into the policy's f32 input +
    mgx_gae_dones) against RolloutCollector (materialised SB3 stacks + mgx_gae) on config 3's
    workload, two rollouts (the second starts from carried-over history rows): same policy,
    same torch RNG -> the same actions, values, rewards (with truncation bootstraps), advantages
    and returns; then one PPO update from each buffer gives the same weights (minibatches
    gathered vs indexed)."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from mgx import MgxEngine
    from mgx.ppo import CompactRolloutCollector, RolloutCollector
    n, T = 256, 72
    env_kw = dict(problem="multi", mission=2, size=8, num_objects=4)
    torch.manual_seed(0)
    pol_a = ActorCriticPolicy().cuda()
    with torch.no_grad():
        pol_a.action_net.bias[6] = -30.0                     # rarely 'done': truncations happen
    pol_b = copy.deepcopy(pol_a)
    pol_b.optimizer = torch.optim.Adam(pol_b.parameters(), lr=3e-4, eps=1e-8)
    pol_b.optimizer.load_state_dict(pol_a.optimizer.state_dict())
    mk = lambda: MgxEngine(n_envs=n, n_stack=4, terminal_mode="truncated", mission_dtype=torch.uint8,  # noqa: E731
                           **env_kw)
    ca = RolloutCollector(mk(), pol_a, PPOConfig(n_envs=n, horizon=T, env=env_kw, layout="sb3"))
    cb = CompactRolloutCollector(mk(), pol_b, PPOConfig(n_envs=n, horizon=T, env=env_kw))
    ca.start()
    cb.start()
    for roll in range(2):
        torch.manual_seed(77 + roll)
        ba = ca.collect()
        torch.manual_seed(77 + roll)
        bb = cb.collect()
        assert torch.equal(ba.actions, bb.actions), roll
        assert torch.equal(ba.values, bb.values), roll
        assert torch.equal(ba.episode_starts[1:], bb.buf.dones[:-1].float()), roll
        assert bool((bb.buf.truncated.bool() & ~bb.buf.terminated.bool()).any())
        torch.testing.assert_close(ba.rewards, bb.rewards, rtol=1e-6, atol=1e-6)
        torch.testing.assert_close(ba.advantages, bb.advantages, rtol=1e-5, atol=1e-5)
        torch.testing.assert_close(ba.returns, bb.returns, rtol=1e-5, atol=1e-5)
    cfg = PPOConfig(n_envs=n, horizon=T, batch_size=4608, n_epochs=1)
    perm = torch.randperm(n * T, device="cuda", generator=torch.Generator(device="cuda").manual_seed(5))
    Trainer(pol_a, cfg).train(ba, 1.0, perm_fn=lambda _: perm)
    Trainer(pol_b, cfg).train(bb, 1.0, perm_fn=lambda _: perm)
    for (name, a), (_, b) in zip(pol_a.named_parameters(), pol_b.named_parameters()):
        torch.testing.assert_close(a, b, rtol=1e-4, atol=1e-5, msg=name)


def test_conv2d_gemm_equals_conv2d():
    from mgx.policy import Conv2dGemm
    torch.manual_seed(4)
    Conv2dGemm.enabled = True
    for cin, cout, k in ((12, 16, 2), (16, 32, 2), (32, 64, 2)):
        ref = torch.nn.Conv2d(cin, cout, [k, k])
        mine = Conv2dGemm(cin, cout, [k, k])
        mine.load_state_dict(ref.state_dict())
        x = torch.randn(5, cin, 7 if cin == 12 else 3, 7 if cin == 12 else 3, requires_grad=True)
        x2 = x.detach().clone().requires_grad_(True)
        y1, y2 = ref(x), mine(x2)
        assert torch.allclose(y1, y2, atol=1e-5)
        y1.square().sum().backward()
        y2.square().sum().backward()
        assert torch.allclose(x.grad, x2.grad, atol=1e-4)
        assert torch.allclose(ref.weight.grad, mine.weight.grad, atol=1e-4)
    Conv2dGemm.enabled = False
