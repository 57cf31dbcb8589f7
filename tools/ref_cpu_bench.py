"""Times the REFERENCE's own env on this host's CPU: src/custom_env.py + src/environment.py
(make_env -> PlaygroundEnv -> TokenizeVocabWrapper -> Discrete2BoxWrapper), executed unchanged
from /root/reference on the clean-room minigrid / gymnasium restatement in oracle/refshim (the
3P layer the reference imports but does not vendor; its speed is that restatement's, written in
the same object-per-cell style as minigrid).  One process, one env (BASELINE configs[0]: GTG
8x8), uniform random actions, SubprocVecEnv-style auto-reset on terminated | truncated.

Build container only (needs /root/reference); the GPU box never runs it.  The reference would
hang on an unsatisfiable placement: resets run under make_golden.py's
live-lock cap (a counting getrandbits override -- a few hundred ns per MT draw).

  python tools/ref_cpu_bench.py [--seconds 20] [--out profiles/r03_reference_cpu.json]
"""
import argparse
import json
import os
import platform
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))
sys.path.insert(0, os.path.join(ROOT, "oracle", "refshim"))


def cpu_model():
    for ln in open("/proc/cpuinfo"):
        if ln.startswith("model name"):
            return ln.split(":", 1)[1].strip()
    return platform.processor() or "unknown"


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--seconds", type=float, default=20.0)
    ap.add_argument("--problem", default="multi")
    ap.add_argument("--mission", type=int, default=5)
    ap.add_argument("--size", type=int, default=8)
    ap.add_argument("--out", default=None)
    args = ap.parse_args()
    import make_golden as MG
    from loader import make_cfg
    cfg = make_cfg(problem=args.problem, mission=args.mission, size=args.size)
    vec = MG.RefVec(cfg, 1)
    rng = np.random.default_rng(1234)
    vec.reset_env(0, seed=cfg.seed)
    steps = resets = 0
    t0 = time.perf_counter()
    t_end = t0 + args.seconds
    while True:
        acts = rng.integers(0, 7, 1024)
        for a in acts:
            _, _, term, trunc, _ = vec.step_env(0, a)
            steps += 1
            if term or trunc:
                vec.reset_env(0)
                resets += 1
        if time.perf_counter() >= t_end:
            break
    dt = time.perf_counter() - t0
    out = {"what": "reference custom_env.py + environment.py wrappers (unchanged source, refshim 3P layer), "
                   "1 process x 1 env, random actions, auto-reset",
           "config": "%s/%s %dx%d (BASELINE configs[0])" % (args.problem, args.mission, args.size, args.size),
           "env_steps": steps, "resets": resets, "seconds": dt, "env_steps_per_s": steps / dt,
           "us_per_step": dt / steps * 1e6, "cores": 1,
           "host": {"cpu": cpu_model(), "logical_cpus": os.cpu_count(), "affinity": len(os.sched_getaffinity(0)),
                    "python": platform.python_version(), "machine": "build container (no GPU)"}}
    print(json.dumps(out))
    if args.out:
        with open(args.out, "w") as f:
            json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
