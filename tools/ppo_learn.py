"""BASELINE config 3 learning evidence: PPO (mgx.ppo.learn: the reference's PPO(CustomPPOPolicy,
vec_env).learn restated over the engine) on PKP 8x8 (or --mission), then the success rate over 1,000
deterministic episodes under the reference's test() protocol (README.md:54-65 "Benchmark (1k ep)": one env
seeded 42, sequential episodes; success = the episode paid a reward, i.e. the mission was completed; the
reference reports PKP 57%).

The reference trains 16 envs x horizon 1024 with minibatch 256 (algorithm/ppo.yaml); at 65,536 envs
the same update count per sample would take 16,384 optimiser steps per 16-step rollout, so this run
keeps the reference's ratio of optimiser steps per rollout (4 epochs x 64 minibatches) with larger
minibatches -- stated in the output, a knob that changes optimisation (SURVEY.md §7 hard part 5).

  python tools/ppo_learn.py [--timesteps 1e8] [--n-envs 65536] [--horizon 16] [--batch-size 16384]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "minigrid-rl_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402


def success_rate(policy, env_kw, n_episodes, seed=42):
    """README.md:54-65's success rate under the reference's own test() protocol (src/ppo.py:185-230; round 5,
    ADVICE r4): ONE env seeded `seed`, `n_episodes` sequential deterministic episodes, the MT19937 stream advancing
    -- tools/eval_protocol.py's column.  (Round 4 ran one episode on each of N fresh envs: every env's first episode
    draws the same mission and room count, one (task, rooms) cell.)  policy None: uniform random actions."""
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    from eval_protocol import protocol_column
    if policy is None:
        g = torch.Generator(device="cuda")
        g.manual_seed(seed)
        model = lambda obs: torch.randint(0, 7, (obs["image"].shape[0],), device="cuda", generator=g)   # noqa: E731
    else:
        policy.train(False)
        model = policy
    col = protocol_column(model, env_kw.get("mission"), n_episodes, env_kw.get("size", 8), seed)
    return dict(col["overall"], per_task=col["per_task"], per_cell=col["per_cell"])


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--timesteps", type=float, default=1e8)
    ap.add_argument("--n-envs", type=int, default=65536)
    ap.add_argument("--horizon", type=int, default=16)
    ap.add_argument("--batch-size", type=int, default=16384)
    ap.add_argument("--epochs", type=int, default=4)
    ap.add_argument("--lr0", type=float, default=1e-3)        # README.md:19-51 first-stage schedule (pkp0)
    ap.add_argument("--lr1", type=float, default=3e-5)
    ap.add_argument("--mission", default="2", help="2 PKP, 5 GTG, 0 GTO, 1 TGL, None = ALL (the mixed-task config 4)")
    ap.add_argument("--size", type=int, default=8)
    ap.add_argument("--eval-episodes", type=int, default=1000)
    ap.add_argument("--out", default=None)
    ap.add_argument("--max-seconds", type=float, default=0, help="stop training after this long (then evaluate)")
    ap.add_argument("--progress", default=None, help="append one JSON line per rollout here")
    ap.add_argument("--save", default=None, help="checkpoint (policy, optimizer, timesteps, curve) written here")
    ap.add_argument("--resume", default=None, help="continue the run saved here (--timesteps stays the total)")
    ap.add_argument("--no-eval", action="store_true", help="skip the evaluation (an intermediate segment)")
    args = ap.parse_args()
    from mgx.ppo import PPOConfig, learn
    mission = None if args.mission == "None" else int(args.mission)
    env_kw = dict(problem="multi", mission=mission, size=args.size, num_objects=4)
    cfg = PPOConfig(n_envs=args.n_envs, horizon=args.horizon, batch_size=args.batch_size, n_epochs=args.epochs,
                    initial_learning_rate=args.lr0, final_learning_rate=args.lr1, env=env_kw)
    t0 = t_seg = time.perf_counter()
    curve, init, prior_s, segment = [], None, 0.0, 0
    if args.resume:                                    # our own checkpoint: tensors, ints and lists only
        ck = torch.load(args.resume, map_location="cuda", weights_only=True)
        curve, prior_s, segment = ck["curve"], float(ck["train_seconds"]), int(ck["segment"]) + 1
        init = {"policy": ck["policy"], "optimizer": ck["optimizer"], "timesteps": int(ck["timesteps"]),
                "seed_offset": 1000003 * segment}
        t0 -= prior_s

    class Stop:                                        # SB3-style callback: False ends learn()
        def on_step(self, policy, num_timesteps):
            # --max-seconds bounds this segment (a resumed run's earlier segments are not counted)
            return not (args.max_seconds and time.perf_counter() - t_seg > args.max_seconds)

    def log(st):
        if "timesteps" in st:
            curve.append({k: st[k] for k in ("timesteps", "ep_rew_mean", "ep_len_mean", "lr", "kl", "clipfrac")})
            curve[-1]["seconds"] = time.perf_counter() - t0
            if args.progress:
                with open(args.progress, "a") as f:
                    f.write(json.dumps(curve[-1]) + "\n")
            if len(curve) % 10 == 1:
                print("t=%.0fs %s" % (time.perf_counter() - t0, json.dumps(curve[-1])), file=sys.stderr, flush=True)
    random_eval = None if args.no_eval else success_rate(None, env_kw, args.eval_episodes)
    t_start = time.perf_counter()
    pol, hist, eng = learn(cfg, int(args.timesteps), log=log, callback=Stop(), init=init)
    train_s = prior_s + time.perf_counter() - t_start
    eng.close()
    steps_done = hist[-1]["timesteps"] if hist else (init or {}).get("timesteps", 0)
    if args.save:
        torch.save({"policy": pol.state_dict(), "optimizer": pol.optimizer.state_dict(), "timesteps": steps_done,
                    "curve": curve, "train_seconds": train_s, "segment": segment}, args.save)
    if args.no_eval:
        print(json.dumps({"segment": segment, "timesteps": steps_done, "train_seconds": train_s,
                          "last": curve[-1] if curve else None}))
        return
    ev = success_rate(pol, env_kw, args.eval_episodes)
    names = {2: "PKP", 5: "GTG", 0: "GTO", 1: "TGL", None: "ALL"}
    # README.md:54-65's table: the model evaluated on every task (columns GTG GTO PKP TGL ALL)
    per_task = {names[m]: success_rate(pol, dict(env_kw, mission=m), args.eval_episodes)
                for m in (5, 0, 2, 1)} if mission is None else None
    out = {"what": "PPO (mgx.ppo.learn) on %s, then the reference's test() protocol: one env seeded 42, %d "
                   "sequential deterministic episodes (tools/eval_protocol.py)" % (names.get(mission, "mission %s" % mission),
                                                                                   args.eval_episodes),
           "eval_per_task": per_task,
           "config": {"env": env_kw, "n_envs": cfg.n_envs, "horizon": cfg.horizon, "batch_size": cfg.batch_size,
                      "n_epochs": cfg.n_epochs, "optimizer_steps_per_rollout": cfg.n_epochs * cfg.n_envs *
                      cfg.horizon // cfg.batch_size, "lr": [cfg.initial_learning_rate, cfg.final_learning_rate],
                      "other_hyperparameters": "algorithm/ppo.yaml (gamma, gae_lambda, clip ranges, ent/vf coef, "
                                               "max_grad_norm)"},
           "timesteps": steps_done, "rollouts": len(curve), "segments": segment + 1, "train_seconds": train_s,
           "env_steps_per_s_incl_training": steps_done / train_s if train_s else None,
           "eval": ev, "eval_random_policy": random_eval,
           "reference": ("README.md:65 PPO ALL model: GTG 75%, GTO 65%, PKP 59%, TGL 58%, ALL 65% (1k episodes; trained "
                         "through the all0..all6 curriculum, README.md:40-46; size and training steps unstated)"
                         if mission is None else
                         {5: "README.md:59 PPO GTG model: GTG 86%, ALL 19%", 0: "README.md:60 PPO GTO model: GTO 72%, ALL 17%",
                          2: "README.md:61 PPO PKP model: PKP 57%, ALL 26%", 1: "README.md:63 PPO TGL model: TGL 47%, ALL 27%"
                          }.get(mission, "") + " (1k episodes; size and training steps unstated)"),
           "curve": curve[::max(1, len(curve) // 40)]}
    print(json.dumps(out))
    if args.out:
        with open(args.out, "w") as f:
            json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
