"""evaluate_policy / EvalCallback (mgx/evaluation.py) against a
restatement of SB3 2.x `evaluate_policy` driving the C oracle with the same
deterministic policy.  The policy is a pure function of the newest frame
(image byte sum + 3 * direction, mod 7), so both sides act identically and the
episode reward/length lists must match exactly, in order."""
import numpy as np
import pytest

torch = pytest.importorskip("torch")


def hash_action_np(img_hwc, d):
    return ((img_hwc.reshape(len(d), -1).astype(np.int64).sum(1) + 3 * d.astype(np.int64)) % 7).astype(np.int32)


def sb3_evaluate_policy_oracle(cfg, n_eval_episodes):
    """stable_baselines3.common.evaluation.evaluate_policy (Monitor-wrapped VecEnv,
    deterministic) over oracle.OracleVec; returns (episode_rewards, episode_lengths)."""
    import oracle as O
    v = O.OracleVec(**cfg)
    n = v.n
    counts = np.zeros(n, int)
    targets = np.array([(n_eval_episodes + i) // n for i in range(n)], int)
    cur_len = np.zeros(n, int)
    r = v.reset()
    img, d = r["image"], r["dir"]
    rewards, lengths = [], []
    while (counts < targets).any():
        o = v.step(hash_action_np(img, d))
        done = (o["terminated"] | o["truncated"]).astype(bool)
        cur_len += 1
        for i in range(n):
            if counts[i] < targets[i] and done[i]:
                rewards.append(round(float(o["reward"][i]), 6))   # Monitor info["episode"]["r"]
                lengths.append(int(cur_len[i]))
                counts[i] += 1
            if done[i]:
                cur_len[i] = 0
        img = np.where(done[:, None, None, None], o["r_image"], o["image"])
        d = np.where(done, o["r_dir"], o["dir"])
    return rewards, lengths


def test_oracle_restatement_counts_episodes():
    cfg = dict(problem="multi", mission=None, size=8, num_objects=4, n_envs=8, seed=42)
    rw, ln = sb3_evaluate_policy_oracle(cfg, 21)
    assert len(rw) == len(ln) == 21
    assert all(1 <= x <= 64 for x in ln)


@pytest.mark.gpu
@pytest.mark.parametrize("n_eval", [5, 16, 37])
@pytest.mark.parametrize("problem,mission,size", [("multi", None, 8), ("pkp", None, 8), ("multi", 1, 11)])
def test_evaluate_policy_matches_sb3_restatement(n_eval, problem, mission, size):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from mgx import MgxEngine, evaluate_policy
    cfg = dict(problem=problem, mission=mission, size=size, num_objects=4, n_envs=16, seed=42)
    want_r, want_l = sb3_evaluate_policy_oracle(cfg, n_eval)
    eng = MgxEngine(problem=problem, mission=mission, size=size, n_envs=16, seed=42, reward64=True,
                    device="cuda:0")

    def policy(obs):
        img = obs["image"][:, -3:].to(torch.int64).sum((1, 2, 3))
        d = obs["direction"][:, -4:].argmax(1)
        return ((img + 3 * d) % 7).to(torch.int32).contiguous()

    got_r, got_l = evaluate_policy(policy, eng, n_eval_episodes=n_eval, return_episode_rewards=True)
    assert got_l == want_l
    assert got_r == want_r
    mean, std = evaluate_policy(policy, MgxEngine(problem=problem, mission=mission, size=size, n_envs=16,
                                                  seed=42, reward64=True, device="cuda:0"), n_eval)
    assert mean == float(np.mean(want_r)) and std == float(np.std(want_r))
    eng.poll_error()


@pytest.mark.gpu
def test_eval_callback_keeps_best_model(tmp_path):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from mgx import EvalCallback, MgxEngine
    from mgx.policy import ActorCriticPolicy
    pol = ActorCriticPolicy(n_stack=4).cuda()
    ev = MgxEngine(problem="multi", mission=2, size=8, n_envs=64, seed=7, reward64=True, device="cuda:0")
    cb = EvalCallback(ev, best_model_save_path=str(tmp_path), eval_freq=2, n_eval_episodes=8)
    for k in range(4):
        cb.on_step(pol, 64 * (k + 1))
    assert len(cb.evaluations) == 2
    assert (tmp_path / "best_model.pt").exists()
    sd = torch.load(tmp_path / "best_model.pt", weights_only=True)
    assert set(sd) == set(pol.state_dict())


@pytest.mark.gpu
def test_learn_with_callback_and_final_evaluation():
    """learn(..., callback=EvalCallback, evaluate=True): src/ppo.py:143-165 end to end."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from mgx import EvalCallback, MgxEngine
    from mgx.ppo import PPOConfig, learn
    cfg = PPOConfig(n_envs=256, horizon=16, batch_size=1024, n_epochs=1, n_eval_episodes=20,
                    env=dict(problem="multi", mission=2, size=8, num_objects=4))
    ev = MgxEngine(problem="multi", mission=2, size=8, n_envs=32, seed=43, reward64=True, device="cuda:0")
    cb = EvalCallback(ev, eval_freq=8, n_eval_episodes=10)
    pol, hist, eng = learn(cfg, total_timesteps=2 * 256 * 16, callback=cb, evaluate=True)
    assert len(hist) == 2 and len(cb.evaluations) == 4
    assert np.isfinite(hist[-1]["mean_reward"]) and 0.0 <= hist[-1]["mean_reward"] <= 1.0


@pytest.mark.gpu
def test_learn_stops_when_callback_returns_false():
    """SB3 early stop: EvalCallback(callback_on_new_best=StopTrainingOnRewardThreshold(t)) makes
    on_step return False at the first evaluation that reaches t; collect_rollouts returns at once
    and learn() ends (no further rollout or update)."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from mgx import EvalCallback, MgxEngine, StopTrainingOnRewardThreshold
    from mgx.ppo import PPOConfig, learn
    cfg = PPOConfig(n_envs=256, horizon=16, batch_size=1024, n_epochs=1,
                    env=dict(problem="multi", mission=2, size=8, num_objects=4))
    ev = MgxEngine(problem="multi", mission=2, size=8, n_envs=32, seed=43, reward64=True, device="cuda:0")
    cb = EvalCallback(ev, eval_freq=8, n_eval_episodes=10,
                      callback_on_new_best=StopTrainingOnRewardThreshold(-1.0))   # any reward >= -1 stops
    pol, hist, eng = learn(cfg, total_timesteps=4 * 256 * 16, callback=cb)
    assert len(cb.evaluations) == 1          # stopped at the first evaluation (step 8 of rollout 0)
    assert len(hist) == 0                    # the interrupted rollout is not trained on


def protocol_oracle(cfg, n_episodes):
    """src/ppo.py:185-230 `test()` restated over the C oracle: one env seeded cfg.seed (DummyVecEnv), per
    episode vec_env.reset() (unseeded after the first, both streams continuing from the env's auto-reset
    episode) and the deterministic hash policy until done; -> [(reward, length, mission text, doors)]."""
    import oracle as O
    v = O.OracleVec(n_envs=1, **cfg)
    out = []
    for i in range(n_episodes):
        r = v.reset() if i == 0 else v.reset(seed=None)
        doors = int((v.dump()["grid"][0, :, :, 0] == 4).sum())
        text = v.mission(0)
        img, d = r["image"], r["dir"]
        total, length = 0.0, 0
        while True:
            o = v.step(hash_action_np(img, d))
            length += 1
            total += float(o["reward"][0])
            if o["terminated"][0] or o["truncated"][0]:
                break
            img, d = o["image"], o["dir"]
        out.append((total, length, text, doors))
    return out


def test_protocol_restatement_varies_the_cell():
    """The reference's benchmark protocol draws a different (mission, rooms) cell per episode -- the single
    MT19937 stream advances across episodes -- whereas the first episode of N fresh envs seeded alike is ONE
    cell (every env's CPython random is MT19937(seed), custom_env.py:82)."""
    from mgx.evaluation import task_of
    cfg = dict(problem="multi", mission=None, size=8, num_objects=4, seed=42)
    eps = protocol_oracle(cfg, 120)
    assert {task_of(e[2]) for e in eps} == {"GTG", "GTO", "PKP", "TGL"}            # every task
    assert {e[3] for e in eps} == {1, 3, 4}                                          # 2, 3 and 4 rooms
    import oracle as O
    v = O.OracleVec(n_envs=64, **cfg)
    v.reset()
    assert len({task_of(v.mission(i)) for i in range(64)}) == 1                     # the flawed protocol: one
    assert len({int((g[:, :, 0] == 4).sum()) for g in v.dump()["grid"]}) == 1       # task, one room count


@pytest.mark.gpu
@pytest.mark.parametrize("problem,mission,size", [("multi", None, 8), ("multi", 2, 8), ("multi", 1, 11)])
def test_evaluate_test_protocol_matches_oracle(problem, mission, size):
    """mgx.evaluate_test_protocol (one env, reset per episode, the MT stream advancing) = the restated
    test() over the C oracle, episode by episode: reward, length, mission and room count."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from mgx import MgxEngine, evaluate_test_protocol
    cfg = dict(problem=problem, mission=mission, size=size, num_objects=4, seed=42)
    want = protocol_oracle(cfg, 40)
    eng = MgxEngine(problem=problem, mission=mission, size=size, n_envs=1, seed=42, reward64=True,
                    terminal_mode="none", mission_dtype=torch.uint8, device="cuda:0")

    def policy(obs):
        img = obs["image"][:, -3:].to(torch.int64).sum((1, 2, 3))
        d = obs["direction"][:, -4:].argmax(1)
        return ((img + 3 * d) % 7).to(torch.int32).contiguous()

    got = evaluate_test_protocol(policy, eng, 40)
    rooms = {1: 2, 3: 3, 4: 4}
    for g, w in zip(got, want):
        assert (g["reward"], g["length"], g["mission"]) == (w[0], w[1], w[2])
        assert g["rooms"] == rooms[w[3]]
    eng.poll_error()
