"""Learning-parity evidence under the reference's own benchmark protocol: the policy of a
tools/ppo_learn.py checkpoint evaluated exactly as src/ppo.py:185-230 `test()` does -- ONE env seeded 42
(make_vec_env n_envs=1, DummyVecEnv), 1,000 sequential deterministic episodes, each started by vec_env.reset()
with the single MT19937 stream advancing (mgx.evaluate_test_protocol) -- per task column of README.md:54-65
(GTG / GTO / PKP / TGL / ALL) plus the success per (task, room count) cell and the cell histogram.  The same
columns under round 4's method (N fresh envs, each one episode: ONE (mission, rooms) cell) are reported
beside it for comparison.

  python tools/eval_protocol.py --ckpt gpurun_out/all_ck3.pt --out profiles/r05_eval_all.json [--size 8]
  python tools/eval_protocol.py --random --out ...      (uniform random actions: the reference point)
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "minigrid-rl_amd"))

import torch  # noqa: E402

COLUMNS = (("GTG", 5), ("GTO", 0), ("PKP", 2), ("TGL", 1), ("ALL", None))


def protocol_column(model, mission, episodes=1000, size=8, seed=42, dev=None):
    """One README.md:54-65 column under test(): a 1-env engine seeded `seed`, `episodes` sequential deterministic
    episodes (mgx.evaluate_test_protocol), summarised per task and per (task, room count) cell."""
    from mgx import MgxEngine, evaluate_test_protocol
    from mgx.evaluation import summarize_episodes
    eng = MgxEngine(problem="multi", mission=mission, size=size, num_objects=4, n_envs=1, seed=seed, n_stack=4,
                    terminal_mode="none", reward64=True, mission_dtype=torch.uint8, device=dev or "cuda")
    try:
        def progress(k):                                  # (a line a minute or so: a silent GPU run looks hung)
            if k % 100 == 0:
                print("  %d / %d episodes" % (k, episodes), file=sys.stderr, flush=True)
        return summarize_episodes(evaluate_test_protocol(model, eng, episodes, deterministic=True, progress=progress))
    finally:
        eng.close()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ckpt", default=None)
    ap.add_argument("--random", action="store_true")
    ap.add_argument("--episodes", type=int, default=1000)
    ap.add_argument("--size", type=int, default=8)
    ap.add_argument("--seed", type=int, default=42, help="cfg.seed (testing.yaml: 42)")
    ap.add_argument("--columns", default="GTG,GTO,PKP,TGL,ALL")
    ap.add_argument("--fresh", type=int, default=1, help="also round 4's fresh-engine method, for comparison")
    ap.add_argument("--out", default=None)
    args = ap.parse_args()
    from mgx import MgxEngine, evaluate_policy
    from mgx.policy import ActorCriticPolicy
    dev = torch.device("cuda:0")
    ck = None
    if args.random:
        g = torch.Generator(device=dev)
        g.manual_seed(args.seed)
        model = lambda obs: torch.randint(0, 7, (obs["image"].shape[0],), device=dev, generator=g)   # noqa: E731
    else:
        ck = torch.load(args.ckpt, map_location="cuda", weights_only=True)
        model = ActorCriticPolicy(n_stack=4).to(dev)
        model.load_state_dict(ck["policy"])
        model.train(False)
    want = set(args.columns.split(","))
    out = {"what": "README.md:54-65 'Benchmark (1k ep)' under the reference's test() protocol (src/ppo.py:185-230): "
                   "one env, seed %d, %d sequential deterministic episodes, vec_env.reset() per episode (the MT19937 "
                   "stream advancing), success = the episode paid a reward" % (args.seed, args.episodes),
           "policy": "uniform random" if args.random else {"checkpoint": os.path.relpath(args.ckpt, ROOT),
                                                          "timesteps": int(ck["timesteps"]),
                                                          "train_seconds": float(ck["train_seconds"])},
           "env": {"problem": "multi", "size": args.size, "num_objects": 4}, "columns": {}}
    for name, mission in COLUMNS:
        if name not in want:
            continue
        t0 = time.perf_counter()
        col = protocol_column(model, mission, args.episodes, args.size, args.seed, dev)
        col["seconds"] = round(time.perf_counter() - t0, 1)
        if args.fresh:
            # round 4's method: n_envs = episodes fresh envs, one episode each (one (mission, rooms) cell)
            e2 = MgxEngine(problem="multi", mission=mission, size=args.size, num_objects=4, n_envs=args.episodes,
                           seed=4242, n_stack=4, terminal_mode="none", reward64=True, mission_dtype=torch.uint8,
                           device=dev)
            rw, ln = evaluate_policy(model, e2, args.episodes, deterministic=True, return_episode_rewards=True)
            e2.close()
            col["round4_fresh_engine_method"] = {"success_rate": sum(r > 0 for r in rw) / len(rw),
                                                 "mean_length": sum(ln) / len(ln)}
        out["columns"][name] = col
        print("%s: %.3f success over %d episodes (%d cells) %.0fs" % (
            name, col["overall"]["success_rate"], col["overall"]["episodes"], len(col["per_cell"]), col["seconds"]),
            file=sys.stderr, flush=True)
    print(json.dumps({k: (v["overall"]["success_rate"] if isinstance(v, dict) and "overall" in v else v)
                      for k, v in out["columns"].items()}))
    if args.out:
        with open(args.out, "w") as f:
            json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
