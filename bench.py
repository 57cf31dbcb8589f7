"""bench.py -- env-steps/s of the MI355X MiniGrid engine (BASELINE config 2).

Workload (one "step" = one vectorised step of the whole per-GPU batch:
PlaygroundEnv.step + gen_obs + the two wrappers + SubprocVecEnv auto-reset, the
new observation written into the rollout buffer in the compact layout -- one
148-B row + mission id per env; the collector's stacked VecFrameStack(4) input
is rebuilt from rows by `mgx_gather`, bit-exact with the materialised stacks,
tests/test_compact.py).  The actions of this random-action rollout are known up
front, so the headline runs each refill epoch's steps in one launch
(`mgx_rollout_compact`, bit-exact with per-step calls, tests/test_rollout.py).
At N=1 the same workload is also timed with one launch per step
(`mgx_step_compact`: the path a policy in the loop takes) as `compact_layout`
and with the materialised SB3 stacks (`mgx_step`: VecTransposeImage +
VecFrameStack roll per step, the MgxVecEnv drop-in) as `sb3_layout`):
  multi / mission 5 ('go to goal', GTG) / 8x8 / num_objects 4 / 65,536 envs per
  GPU, uniform random actions on {0..6} (pre-generated on device for all
  warmup+timed steps, so inputs are resident in HBM), seed 42, env global
  index i seeded 42+i (rank r owns [r*N, (r+1)*N)) -> weak scaling.

The timed region pays for every reset it consumes: it is a whole number of
refill epochs (the episode generator's launches are inside it; `window` reports
episodes produced vs consumed), and every `horizon` steps it runs GAE over the
rewards/dones the steps wrote (mgx_gae_dones, synthetic values) and, for N>1,
the one all-reduce of the (sum A, sum A^2, n) advantage statistics (RCCL).

Prints ONE JSON line (rank 0).  `roofline` prices the kernel that runs the steps
(mgx_rollout_kernel in the fused headline, mgx_step_kernel per step) with
SURVEY.md §8(d)'s algorithmic bytes
  B_alg = 334*steps + (3*S^2 + 208)*resets     (per step: one step of all N envs)
divided by its average duration per step, measured live with HIP events on the
launch stream: fused, one event pair around each epoch's launch (the epoch's refill
beside it); per step, around each run of consecutive mgx_step calls that neither
fork nor join a refill epoch (those launches still run concurrently with that
epoch's refill, as in the timed region);
`traffic` is the rocprofv3 PMC figure committed under profiles/.  `gae` times
mgx_gae_dones alone at the horizon and at T=1024 (17 B per element).
`cpu_baseline` times the C port of the env (oracle/) on this host's cores.

  python bench.py [--gpus N] [--steps K] [--warmup W]
  (N>1: python -m torch.distributed.run --nproc-per-node N bench.py --gpus N ...)

  python bench.py --workload ppo [--steps K] [--warmup W]
  BASELINE config 3: the full PPO loop (PKP 8x8, 65,536 envs/GPU, PyTorch policy,
  device-resident rollout + train); a "step" is one PPO iteration (collect
  `--horizon` env steps + n_epochs of minibatch training); value = env-steps/s.
"""
import argparse
import ctypes
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "minigrid-rl_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

METRIC = "env-steps/sec at 65k parallel envs, 1/2/4/8 MI355X; % HBM roofline"
PEAK_HBM_GBPS = 8000.0          # MI355X HBM3E spec (MI355X_MICROARCH.md)
B_STEP = 334                    # per env-step algorithmic bytes


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=None, help="timed steps (rollout 2048; ppo: PPO iterations, 4)")
    ap.add_argument("--warmup", type=int, default=None, help="untimed steps (rollout 128; ppo: 1)")
    ap.add_argument("--n-envs", type=int, default=65536, help="envs per GPU")
    ap.add_argument("--problem", default="multi")
    ap.add_argument("--mission", default="5")
    ap.add_argument("--size", type=int, default=8)
    ap.add_argument("--n-stack", type=int, default=4)
    ap.add_argument("--cpu-seconds", type=float, default=10.0, help="CPU baseline sample budget (0 = skip)")
    ap.add_argument("--graph", type=int, default=1, help="replay the timed steps from a hipGraph")
    ap.add_argument("--probe", type=int, default=256, help="eager steps timed per launch for the roofline")
    ap.add_argument("--workload", default="rollout", choices=["rollout", "ppo"])
    ap.add_argument("--gae-fused", type=int, default=1,
                    help="fused layout with one launch per horizon (E = H): 1 = GAE in the rollout launch "
                         "(mgx_rollout_compact_gae; round 5: +2 %% on the driver's line over the separate kernels, "
                         "which cost two more launches on the rollout's branch of the graph); 0 = a separate "
                         "mgx_gae_dones launch + its fold")
    ap.add_argument("--refill-every", type=int, default=0, help="steps per refill epoch (0 = engine default, D/4)")
    ap.add_argument("--warmup-ms", type=float, default=0.0,
                    help="rollout: untimed graph replays continue until the warm-up has run this long (0: one "
                         "replay of each graph, the rings still nearly full: see --steady-ms)")
    ap.add_argument("--steady-ms", type=float, default=400.0,
                    help="rollout: after everything else, this much more of untimed replays, then the same "
                         "steps timed again -> `steady_state` beside the headline (0: skip)")
    ap.add_argument("--steady-steps", type=int, default=20480,
                    help="rollout: untimed graph replays continue until this many steps after mgx_reset, so that the "
                         "timed region sits in the rings' steady state (round 6; 0: one replay of each graph)")
    ap.add_argument("--min-warmup", type=int, default=256,
                    help="rollout: the warm-up is at least this many steps (whole refill epochs)")
    ap.add_argument("--refill-cap", type=int, default=0, help="extra episodes per env per epoch (0 = engine default)")
    ap.add_argument("--ring-depth", type=int, default=0, help="episode ring depth (0 = engine default)")
    ap.add_argument("--config", type=int, default=2, choices=[2, 4, 5],
                    help="BASELINE.json config preset (per-GPU share): 2 GTG 8x8 65,536 envs; "
                         "4 ALL mixed 8x8 32,768 envs (256k over 8 GPUs); 5 TGL 16x16 131,072 envs (1M over 8)")
    ap.add_argument("--horizon", type=int, default=None,
                    help="env steps per rollout (rollout: GAE + adv-stat reduction cadence, default the "
                         "largest whole-epoch divisor of --steps up to 1024; ppo: default 16)")
    ap.add_argument("--batch-size", type=int, default=65536, help="ppo: minibatch size")
    ap.add_argument("--epochs", type=int, default=4, help="ppo: n_epochs")
    ap.add_argument("--eval-episodes", type=int, default=100,
                    help="ppo: deterministic evaluate_policy episodes after the timed iterations (0: none)")
    ap.add_argument("--host-wait", default="spin", choices=["auto", "spin", "yield"],
                    help="how the host waits for the GPU (mgx.engine.set_host_wait: hipSetDeviceFlags); spin: "
                         "the synchronize() that closes the region returns ~10-20 us sooner after the last kernel "
                         "(round 5: +3 %% on the driver's 20-step line), one busy host core per rank")
    ap.add_argument("--graph-launch", default="torch", choices=["raw", "torch"],
                    help="timed graph replays: torch's CUDAGraph.replay(), or hipGraphLaunch on the graph exec "
                         "(mgx.engine.graph_launch: without replay()'s ~9 us of host bookkeeping; round 5 A/B: "
                         "no difference on the driver's line, 6.04-6.18 vs 5.95-6.23 x 10^9)")
    ap.add_argument("--launch", default="graph", choices=["graph", "eager"],
                    help="fused layout, one launch per horizon: each timed chunk as a captured hipGraph replay, or as "
                         "ONE prepared C call (rollout + refill fork + GAE, ctypes arguments built once) + mgx_join")
    ap.add_argument("--mark-region", type=int, default=0,
                    help="a torch.cuda._sleep kernel right before and after the timed region (kernel-trace marker for "
                         "tools/trace_window.py; outside the region)")
    ap.add_argument("--both-layouts", type=int, default=1, help="rollout, N=1: also time the other layouts")
    ap.add_argument("--layout", default=None, choices=["compact", "sb3", "fused"],
                    help="observation storage: compact rows + mgx_gather from one launch per refill epoch "
                         "(fused: mgx_rollout_compact, actions known up front; the rollout default when the "
                         "timed steps are whole epochs), the same rows from one launch per step "
                         "(mgx_step_compact; the ppo default) or the materialised SB3 stacks (mgx_step, the "
                         "VecEnv drop-in's)")
    args = ap.parse_args()
    presets = {2: dict(mission="5", size=8, n_envs=65536), 4: dict(mission="None", size=8, n_envs=32768),
               5: dict(mission="1", size=16, n_envs=131072)}
    for k, v in presets[args.config].items():          # a preset fills what was not given explicitly
        if getattr(args, k) == ap.get_default(k):
            setattr(args, k, v)
    ppo = args.workload == "ppo"
    if args.steps is None:
        args.steps = 4 if ppo else 2048
    if args.warmup is None:
        args.warmup = 1 if ppo else 128
    if ppo and args.horizon is None:
        args.horizon = 16
    if args.layout is None:
        # rollout: the fused launch per refill epoch (the actions of a random-action rollout are known
        # up front); it needs the timed steps to be whole epochs (pick_epoch), else one launch per step
        args.layout = "compact" if ppo or pick_epoch(args.steps, args.ring_depth or 512) is None else "fused"
    return args


def _cpu_leg(problem, mission, size, n, seconds, seed, q=None):
    """One CPU-baseline process: the C port (oracle/mgx_oracle.c, orc_bench) stepping `n` envs
    with random actions for about `seconds`; returns (env_steps, seconds)."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as O
    v = O.OracleVec(problem, mission, size, 4, n, 42)
    v.reset()
    steps = max(1, 20000 // n)
    t0 = time.perf_counter()
    v.bench(steps, seed)                                   # calibration run (counted)
    done = steps
    dt = time.perf_counter() - t0
    steps = max(1, int(done * (seconds - dt) / max(dt, 1e-6)))
    v.bench(steps, seed + 1)
    done += steps
    out = (n * done, time.perf_counter() - t0)
    if q is not None:
        q.put(out)
    return out


def cpu_baseline(args, seconds):
    """SURVEY.md 8(d) CPU baseline, timed on this host BEFORE the GPU is touched: the C port of
    the reference-shaped env (oracle/, object grid + literal slice/rotate/encode per step,
    random actions, auto-reset) in three legs of about `seconds` each:
      all-cores  P processes, one env each (the SubprocVecEnv analogue, ppo.py:121),
                 P = this process's CPU share (affinity, at most 16 on a shared GPU box);
      1 thread   1 process stepping 1,024 envs of the same config;
      config 1   1 process, 1 env, GTG 8x8 (BASELINE configs[0])."""
    import multiprocessing as mp
    mission = None if args.mission == "None" else int(args.mission)
    affinity = len(os.sched_getaffinity(0))
    P = max(1, min(affinity, 16))
    ctx = mp.get_context("fork")                           # no GPU state exists yet in this process
    q = ctx.Queue()
    procs = [ctx.Process(target=_cpu_leg, args=(args.problem, mission, args.size, 1, seconds, 7 + i, q))
             for i in range(P)]
    for pr in procs:
        pr.start()
    res = [q.get() for _ in procs]
    for pr in procs:
        pr.join()
    all_cores = sum(r[0] for r in res) / max(r[1] for r in res)
    s1, t1 = _cpu_leg(args.problem, mission, args.size, 1024, seconds, 3)
    c1, tc1 = _cpu_leg("multi", 5, 8, 1, seconds, 5)
    return dict(value=all_cores, unit="env-steps/s", cores=P, kind="port",
                sample="C port of the reference env (oracle/mgx_oracle.c orc_bench: object grid, slice+rotate+"
                       "encode per step, tokenised mission, auto-reset), random actions, same config as the GPU "
                       "line; %d processes x 1 env x %.1fs; host: %s" % (P, seconds, _cpu_model()),
                affinity_cpus=affinity, cpu_count=os.cpu_count(),
                cap_note="P = min(affinity, 16): the reference's SubprocVecEnv runs n_envs = 16 workers "
                         "(algorithm/ppo.yaml:4), and a shared GPU box grants 16 CPUs per GPU",
                reference_python=_reference_cpu(),
                # every logical CPU of the host: not run -- a GPU box grants one GPU's job 16 CPUs and
                # asks that worker pools stay within that share -- so priced from the measured per-process rate (the
                # P processes run one env each, independently: the rate scales with processes up to the share)
                all_affinity_extrapolated={"value": all_cores / P * affinity, "processes": affinity,
                                           "note": "measured per-process rate x %d logical CPUs; NOT measured (the "
                                                   "box's CPU share is 16)" % affinity},
                legs={"all_cores": {"value": all_cores, "processes": P, "envs_per_process": 1},
                      "one_thread": {"value": s1 / t1, "processes": 1, "envs": 1024, "seconds": t1},
                      "config1_gtg8_1env": {"value": c1 / tc1, "processes": 1, "envs": 1, "seconds": tc1}})


def _reference_cpu():
    """The reference's own Python env timed by tools/ref_cpu_bench.py (custom_env.py + environment.py
    wrappers, unchanged, 1 process x 1 env, GTG 8x8).  /root/reference exists only in the build
    container, so this leg is recorded there (profiles/r03_reference_cpu.json names that host) and
    reported here as recorded, not re-timed on the GPU box."""
    path = os.path.join(ROOT, "profiles", "r03_reference_cpu.json")
    try:
        r = json.load(open(path))
    except (OSError, ValueError):
        return None
    return {"value": r["env_steps_per_s"], "unit": "env-steps/s", "us_per_step": r["us_per_step"], "cores": 1,
            "kind": "reference", "config": r["config"], "host": r["host"],
            "source": "profiles/r03_reference_cpu.json (tools/ref_cpu_bench.py, build container)"}


def _workload_name(args, mission, n, world):
    key = (args.problem, mission, args.size)
    if key == ("multi", 5, 8):
        return "GTG 8x8 random-action rollout, %d envs/GPU (BASELINE config 2)" % n
    if key == ("multi", None, 8):
        return "ALL mixed-task 8x8 random-action rollout, %d envs/GPU, %d total (BASELINE config 4)" % (n, n * world)
    if key == ("multi", 1, 16):
        return "TGL 16x16 random-action rollout, %d envs/GPU, %d total (BASELINE config 5)" % (n, n * world)
    return "%s/%s %dx%d random-action rollout, %d envs/GPU" % (args.problem, mission, args.size, args.size, n)


def _cpu_model():
    try:
        for ln in open("/proc/cpuinfo"):
            if ln.startswith("model name"):
                return ln.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def _allreduce(t, op):
    """all_reduce on the backend's device (RCCL: GPU tensors; gloo rehearsal: CPU)."""
    if dist.get_backend() == "gloo":
        c = t.cpu()
        dist.all_reduce(c, op=op)
        return c.to(t.device)
    dist.all_reduce(t, op=op)
    return t


def main_ppo(args, world, rank, local, dev, ranks_seen=1):
    """BASELINE config 3: PPO(CustomPPOPolicy) on PKP 8x8 with the engine (mgx/ppo.py)."""
    from mgx.policy import ActorCriticPolicy
    from mgx.ppo import PPOConfig, Trainer, make_collector
    from mgx import MgxEngine
    mission = None if args.mission == "None" else int(args.mission)
    if args.mission == "5" and args.problem == "multi":
        mission = 2                                   # config 3 is PKP ('pick up')
    n = args.n_envs
    cfg = PPOConfig(n_envs=n, horizon=args.horizon, batch_size=args.batch_size, n_epochs=args.epochs,
                    env=dict(problem=args.problem, mission=mission, size=args.size, num_objects=4),
                    layout=args.layout)
    torch.manual_seed(cfg.seed + rank)
    eng = MgxEngine(n_envs=n, seed=cfg.seed, env_index_offset=rank * n, n_stack=cfg.n_frames_stack,
                    terminal_mode="truncated", mission_dtype=torch.uint8, device=dev, **cfg.env)
    pol = ActorCriticPolicy(n_stack=cfg.n_frames_stack, optim_eps=cfg.optim_eps, lr=cfg.initial_learning_rate,
                            mission_cache=cfg.mission_cache).to(dev)
    group = dist.group.WORLD if world > 1 else None
    if group is not None:
        for p_ in pol.parameters():
            dist.broadcast(p_.data, 0)
    col = make_collector(eng, pol, cfg)
    tr = Trainer(pol, cfg, group)
    if rank == 0:                       # heartbeat: the first iteration compiles MIOpen kernels for minutes
        import threading
        t_start = time.perf_counter()

        def beat():
            while True:
                time.sleep(30)
                print("ppo: running, %.0fs" % (time.perf_counter() - t_start), file=sys.stderr, flush=True)
        threading.Thread(target=beat, daemon=True).start()
    col.start()
    K, W = args.steps, args.warmup
    total = (K + W) * n * cfg.horizon * world

    def iteration():
        t0 = time.perf_counter()
        buf = col.collect()
        torch.cuda.synchronize(dev)
        t1 = time.perf_counter()
        tr.global_adv_stats(buf)
        tr.train(buf, 1.0 - float(col.num_timesteps * world) / total)
        torch.cuda.synchronize(dev)
        return t1 - t0, time.perf_counter() - t1

    for i in range(W):
        a, b = iteration()
        if rank == 0:
            print("ppo warmup %d: collect %.3fs train %.3fs" % (i, a, b), file=sys.stderr, flush=True)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    tc = tt = 0.0
    for i in range(K):
        a, b = iteration()
        tc += a
        tt += b
        if rank == 0:
            print("ppo iter %d: collect %.3fs train %.3fs" % (i, a, b), file=sys.stderr, flush=True)
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    wall = torch.tensor([time.perf_counter() - t0], dtype=torch.float64, device=dev)
    if world > 1:
        wall = _allreduce(wall, dist.ReduceOp.MAX)
    eng.poll_error()
    wall = float(wall[0])
    ev = None
    if rank == 0 and args.eval_episodes > 0:          # untimed: learning evidence for the trained policy
        ev = _ppo_success(pol, cfg.env, args.eval_episodes, dev)
        ev["after"] = {"ppo_iterations": K + W, "env_steps": (K + W) * n * cfg.horizon * world,
                       "optimizer_steps": (K + W) * cfg.n_epochs * max(1, n * world * cfg.horizon // cfg.batch_size)}
    if rank == 0:
        print(json.dumps({
            "metric": "PPO env-steps/sec (rollout + train), PKP 8x8, 65k envs/GPU",
            "value": K * n * cfg.horizon * world / wall, "unit": "env-steps/s", "n_gpus": world, "steps": K,
            "warmup": W,
            "warmup_requested": args.warmup, "ms_per_step": wall * 1e3 / K, "higher_is_better": True, "scaling": "weak",
            "vs_baseline": None, "dtype": "u8 env / fp32 policy",
            "data": "synthetic (policy-sampled actions; env i seeded 42+i; random-init policy)",
            "config": {"workload": "PKP 8x8 full PPO loop, %d envs/GPU (BASELINE config 3)" % n,
                       "problem": args.problem, "mission": mission, "size": args.size, "envs_per_gpu": n,
                       "horizon": cfg.horizon, "batch_size": cfg.batch_size, "n_epochs": cfg.n_epochs,
                       "minibatches_per_epoch": n * world * cfg.horizon // cfg.batch_size // world,
                       "mission_cache": cfg.mission_cache, "layout": cfg.layout,
                       "parallelism": "env-sharded dp%d" % world, "host_wait": getattr(args, "host_wait_applied", "auto")},
            "phases_s_per_iter": {"collect": tc / K, "train": tt / K},
            "eval": ev,
            "roofline": None,
            "ranks_seen": ranks_seen, "dist_backend": dist.get_backend() if world > 1 else None,
        }), flush=True)
    if world > 1:
        dist.destroy_process_group()


def _ppo_success(pol, env_kw, episodes, dev):
    """evaluate_policy (mgx/evaluation.py, SB3's semantics) over `episodes` deterministic episodes
    on a fresh engine (seed 4242): success = an episode that paid a reward (README.md:54-65's
    "Benchmark (1k ep)" column; the reference quotes 57 % for its PKP model)."""
    from mgx import MgxEngine, evaluate_policy
    eng = MgxEngine(n_envs=episodes, seed=4242, n_stack=4, terminal_mode="none", reward64=True,
                    mission_dtype=torch.uint8, device=dev, **env_kw)
    was = pol.training
    pol.train(False)
    t0 = time.perf_counter()
    rews, lens = evaluate_policy(pol, eng, episodes, deterministic=True, return_episode_rewards=True)
    pol.train(was)
    eng.close()
    r = np.asarray(rews)
    return {"episodes": int(r.size), "deterministic": True, "success_rate": float((r > 0).mean()),
            "mean_reward": float(r.mean()), "mean_length": float(np.mean(lens)),
            "seconds": round(time.perf_counter() - t0, 3)}


def _rocprof_kernel_avg(path, kernel):
    """Average duration (us) of `kernel` (name substring) in a rocprofv3 --stats kernel_stats.csv, or None."""
    import csv
    try:
        rows = list(csv.DictReader(open(path)))
    except OSError:
        return None
    for r in rows:
        if kernel in r.get("Name", ""):
            return {"avg_us": float(r["AverageNs"]) / 1e3, "calls": int(r["Calls"]),
                    "source": os.path.relpath(path, ROOT)}
    return None


def _rocprof_trace_timed_avg(path, kernel, first, count):
    """Average duration (us) of launches [first, first + count) of `kernel` (name substring, in start order) in a
    committed rocprofv3 kernel trace (.csv.gz) of this same command: the timed region's launches (after the
    warm-up's, the untimed graph replay's), or None."""
    import csv
    import gzip
    try:
        rows = [r for r in csv.DictReader(gzip.open(path, "rt")) if kernel in r.get("Kernel_Name", "")]
    except OSError:
        return None
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    sel = rows[first:first + count]
    if len(sel) != count or count == 0:
        return None
    return sum(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in sel) / 1e3 / count


def _profile_dir():
    """(profiles/<round>_pmc directory whose manifest.json names the libmgx.so this process loaded, its
    hash): committed rocprof figures are reported only for the build they were collected with."""
    import glob
    import hashlib
    from mgx import _lib
    try:
        sha = hashlib.sha256(open(_lib.LIB_PATH, "rb").read()).hexdigest()[:16]
    except OSError:
        return None, None
    for man in sorted(glob.glob(os.path.join(ROOT, "profiles", "r*_pmc", "manifest.json")), reverse=True):
        try:
            if json.load(open(man)).get("lib_sha16") == sha:
                return os.path.dirname(man), sha
        except (OSError, ValueError):
            continue
    return None, sha


class _PreparedChunk:
    """--launch eager: one horizon chunk as a prepared C call + its join, replayed like a graph (same cyclic block
    order: each replay advances the ring buffer to the block it was prepared for)."""

    def __init__(self, cbuf, block, fn, eng, stream_ptr):
        self.cbuf, self.block, self.fn, self.eng, self.sp = cbuf, block, fn, eng, stream_ptr

    def replay(self):
        self.cbuf.carry_over()
        assert self.cbuf.block == self.block, "prepared chunks must be replayed in cyclic order"
        self.fn(self.sp)
        if self.eng.L.mgx_join(self.eng.h, self.sp) != 0:
            raise RuntimeError("mgx_join failed")


def pick_epoch(K, D=512):
    """Refill epoch E (mgx refill_every) so that the K timed steps are whole epochs: the largest
    divisor of K in [8, min(64, D/4)] (at D/2 the ring invariant 2E <= D makes every epoch refill the
    rings to full, so each wave runs as many rounds as its busiest lane consumed; at <= D/4 the
    production cap bounds them); K < 8 -> E = K.  None when K has no such divisor (then E = D/4
    and the timed region ends with mgx_join, paying for the whole last epoch's refill)."""
    for E in range(min(64, D // 4), 7, -1):
        if K % E == 0:
            return E
    return K if K < 8 else None


def pick_horizon(K, E, req):
    """Rollout horizon H (GAE + advantage-stat all-reduce every H steps): a multiple of E that
    divides K, at most 1,024 (algorithm/ppo.yaml:30 n_steps); `req` if it qualifies."""
    if req and K % req == 0 and (E is None or req % E == 0):
        return req
    best = None
    for H in range(1, min(K, 1024) + 1):
        if K % H == 0 and (E is None or H % E == 0):
            best = H
    return best or K


def gae_probe(dev, n, T, reps=20):
    """Average duration of mgx_gae_dones over [T, n] (HIP events on the launch stream)."""
    from mgx import gae_dones
    g = torch.Generator(device=dev)
    g.manual_seed(77)
    r = torch.randn((T, n), device=dev, generator=g)
    v = torch.randn((T, n), device=dev, generator=g)
    d = (torch.rand((T, n), device=dev, generator=g) < 0.14).to(torch.uint8)
    lv = torch.randn(n, device=dev, generator=g)
    out = (torch.empty_like(r), torch.empty_like(r))
    st = torch.zeros(3, dtype=torch.float64, device=dev)
    for _ in range(3):
        gae_dones(r, v, d, lv, 0.8108071290665859, 0.9452281119742252, stats=st, out=out)
    stream = torch.cuda.current_stream(dev)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(stream)
    for _ in range(reps):
        gae_dones(r, v, d, lv, 0.8108071290665859, 0.9452281119742252, stats=st, out=out)
    e1.record(stream)
    torch.cuda.synchronize(dev)
    us = e0.elapsed_time(e1) * 1e3 / reps
    b = 17.0 * T * n                                  # r 4 + v 4 + done 1 + adv 4 + ret 4
    del r, v, d, out
    return {"T": T, "N": n, "avg_launch_us": us, "alg_bytes": b, "achieved": b / us / 1e3,
            "frac": b / us / 1e3 / PEAK_HBM_GBPS, "unit": "GB/s"}


def measure_rollout(args, layout, world, rank, dev):
    """One rollout measurement (the timed region of the module docstring) on a fresh engine;
    returns the JSON dict on rank 0."""
    from mgx import MgxEngine, gae_dones
    n = args.n_envs
    mission = None if args.mission == "None" else int(args.mission)
    K = args.steps
    D = args.ring_depth or 512
    E = args.refill_every or pick_epoch(K, D)
    aligned = E is not None and K % E == 0
    eng = MgxEngine(problem=args.problem, mission=mission, size=args.size, n_envs=n, seed=42,
                    env_index_offset=rank * n, n_stack=args.n_stack, terminal_mode="truncated", device=dev,
                    refill_every=E or 0, refill_cap=args.refill_cap, ring_depth=args.ring_depth)
    E = eng.refill_every
    H = pick_horizon(K, E if aligned else None, args.horizon or 0)
    # warm-up: whole refill epochs, and at least --min-warmup (256) steps.  mgx_reset fills every ring
    # to D, so production follows consumption from the first epoch; but every env starts its first
    # episode at step 0, and the reset rate (what the refill pays for) settles only after a few
    # max_steps (64 at S = 8): a window right after the reset would see fewer resets than steady state
    W = -(-max(args.warmup, args.min_warmup, 1) // E) * E
    # device kernel clocks (mgx_set_clock): every step-kernel and refill launch records its own span, so the
    # roofline prices the kernel's launches INSIDE the timed graph replays (set before any capture)
    per0 = E if layout == "fused" and aligned else 1
    eng.enable_clock(slots=(W + 3 * K + args.probe) // per0 + 64)     # every step-kernel launch of this run
    g = torch.Generator(device=dev)
    g.manual_seed(1234 + rank)
    P = args.probe
    actions = torch.randint(0, 7, (W + K + P, n), device=dev, generator=g, dtype=torch.int32)
    # rollout storage the steps write directly (compact layout): reward f32 and done u8 per step;
    # values are synthetic (the rollout bench has no policy); GAE + the (sum A, sum A^2, n)
    # all-reduce run once per horizon inside the timed region
    fused = layout == "fused"
    compact = layout in ("compact", "fused")
    assert not fused or (aligned and H % E == 0), "fused rollouts need whole refill epochs"
    cbuf = None
    if compact:
        # compact layout: each step writes its observation row, reward and done straight into the
        # rollout buffer (mgx_step_compact); GAE reads the buffer's rewards and dones
        from mgx.compact import CompactBuffer
        # ring layout: a horizon's history rows are the previous horizon's last rows, read in place -- the
        # per-horizon carry-over is a block advance, not a copy (every timed horizon pays for what
        # a steady-state horizon costs, and no copy exists outside the graphs)
        cbuf = CompactBuffer(eng, H, ring=True)
        rew, dones = cbuf.rewards, cbuf.dones
    else:
        rew = torch.zeros((H, n), dtype=torch.float32, device=dev)
        dones = torch.zeros((H, n), dtype=torch.uint8, device=dev)
    vals = torch.randn((H, n), device=dev, generator=g)
    last_v = torch.randn(n, device=dev, generator=g)
    adv, ret = torch.empty_like(rew), torch.empty_like(rew)
    nchunks = K // H
    # the (sum A, sum A^2, n) triple of each horizon chunk is accumulated by GAE straight into its row of
    # `hist` (which the N>1 all-reduce reads), through a shard scratch allocated here -- outside the
    # captured graphs, so they hold neither a zero-fill nor a copy of the triple
    hist = torch.zeros((nchunks, 3), dtype=torch.float64, device=dev)
    from mgx import _lib as _L
    scratch = torch.zeros(_L.GAE_SCRATCH_WORDS, dtype=torch.float64, device=dev)
    gamma, lam = 0.8108071290665859, 0.9452281119742252
    eng.reset()
    stream = torch.cuda.current_stream(dev)
    t_warm0 = time.perf_counter()
    if compact:
        cbuf.observe(0)
        for t in range(0, W, E if fused else 1):
            if t and t % H == 0:
                cbuf.carry_over()
            if fused:
                cbuf.rollout(t % H, actions[t:t + E])
            else:
                cbuf.step(t % H, actions[t])
        cbuf.carry_over()
    else:
        for t in range(W):
            eng.step(actions[t])
    eng.join()                                           # the warm-up's last refill: joined outside the
    torch.cuda.synchronize(dev)                          # captures (no cross-capture dependency)
    assert eng.calls % E == 0                            # the timed region starts on an epoch boundary

    def chunk(c, acts=None, device_policy=False):
        # acts: the chunk's [H, n] actions (a graph's own buffer, refreshed between replays), else the table's slice;
        # device_policy: the fused launches draw their own actions (mgx_set_random_policy), nothing is read
        if acts is None and not device_policy:
            acts = actions[W + c * H:W + c * H + H]
        if compact:
            cbuf.carry_over()                            # every horizon starts a rollout (ring: no copy)
            if fused and E == H and args.gae_fused:      # one launch for the horizon, its GAE fused in
                cbuf.rollout(0, None if device_policy else acts[0:E], K=E, gae=dict(
                    values=vals, last_values=last_v, gamma=gamma, gae_lambda=lam, out=(adv, ret), stats=hist[c],
                    scratch=scratch))
            elif fused:                                  # one launch per refill epoch
                for j in range(0, H, E):
                    cbuf.rollout(j, None if device_policy else acts[j:j + E], K=E)
            else:
                for j in range(H):
                    cbuf.step(j, acts[j])
        else:
            for j in range(H):
                eng.step_into(acts[j], reward=rew[j], done=dones[j])
        if not (fused and E == H and args.gae_fused):
            gae_dones(rew, vals, cbuf.dones if compact else dones, last_v, gamma, lam, stats=hist[c], scratch=scratch,
                      out=(adv, ret))                    # (ring: this horizon's block of start flags)
        eng.join()                                       # the epoch's refill (it ran beside GAE): the
                                                         # chunk's graph is self-contained, and the region
                                                         # pays for every refill it forked

    graphs = []
    replay_cycles = 1                                    # untimed replays of the graph set (warm-up)
    forks0 = eng.stats()["refill_launches"]
    # ring buffer: graph c writes block (c0 + c + 1) % m; replayed in cyclic order, the graphs continue the
    # block sequence only if there is a multiple of m of them (one 20-step chunk -> two graphs, alternating)
    ng = nchunks
    if compact and args.graph:
        m = cbuf.blocks
        ng = -(-nchunks // m) * m
    steps_since_reset = W
    if args.graph:
        # one hipGraph per horizon chunk (launch-bound loop -> one replay each); a chunk is whole
        # refill epochs, so each graph holds its forks and joins (self-contained capture).
        # FRESH ACTIONS EVERY REPLAY (round 6), uniform on {0..6}.  Rounds 2-5 replayed one fixed slice of actions in every replay,
        # so env i repeated the same H actions forever: an env whose slice held 6-7 'done' actions consumed 6-7
        # episodes per 20-step epoch, every epoch, against a production cap of ~3 -- its ring drained to the 2K
        # floor within ~100 epochs and its wave then ran need-driven rounds (6-13) every epoch.  That, not the
        # engine, was round 5's "steady-state drain" (tools/diag_ring_levels.py: fixed vs fresh actions).
        # The draws: counter-based hashes whose counters live on the device (not torch's Philox: replay() would add two
        # offset-fill launches and its bookkeeping before every graph launch, ~20 us of the 20-step window in the
        # rocprofv3 trace, and a raw hipGraphLaunch would repeat them).  Fused layout: the rollout launches draw their
        # own actions in the DMA wave that would have loaded them (mgx_set_random_policy) -- no kernel, no buffer, no
        # action byte read.  A separate draw kernel beside the rollout and the refill measured ruinous (round 6: its
        # 1,024 workgroups found slots only between theirs, lingered 120 us and slowed both by ~40 %).  Per-step
        # layouts: mgx_random_actions redraws the graph's own buffer after its steps, on the steps' stream.
        from mgx import random_actions
        act_ctr = torch.zeros(2, dtype=torch.int64, device=dev)
        act_seed = 4321 + rank
        if fused:
            eng.set_random_policy(act_seed)
            abuf = [None] * ng
        else:
            abuf = [actions[W + (c % nchunks) * H:W + (c % nchunks) * H + H].clone() for c in range(ng)]
        s = torch.cuda.Stream(dev)
        if args.launch == "eager" and fused and E == H and args.gae_fused:
            # --launch eager: no graph -- each chunk is ONE prepared C call (mgx_rollout_compact_gae: the epoch's refill
            # fork, the MT slide, the rollout, the GAE fold) + mgx_join, its ctypes arguments built here once
            # (CompactBuffer.rollout_launcher); the "graphs" below replay them in the same cyclic block order
            sp = ctypes.c_void_p(stream.cuda_stream)
            for c in range(ng):
                cbuf.carry_over()
                fn = cbuf.rollout_launcher(0, None, K=E, gae=dict(
                    values=vals, last_values=last_v, gamma=gamma, gae_lambda=lam, out=(adv, ret),
                    stats=hist[c % nchunks], scratch=scratch))
                graphs.append(_PreparedChunk(cbuf, cbuf.block, fn, eng, sp))
        else:
            with torch.cuda.stream(s):
                for c in range(ng):
                    gr = torch.cuda.CUDAGraph()
                    gr.capture_begin()
                    chunk(c % nchunks, abuf[c], device_policy=fused)
                    if not fused:                        # this graph's next actions, after its steps read them
                        random_actions(abuf[c], act_ctr, seed=act_seed)
                    gr.capture_end()
                    graphs.append(gr)
        # one untimed replay of each graph (more warm-up steps: every graph is whole refill epochs
        # ending in a join): the first launch of an instantiated graph pays its upload, ~0.1 ms
        # that a 20-step window would otherwise count as 5 us per step
        for gr in graphs:
            gr.replay()
        torch.cuda.synchronize(dev)
        steps_since_reset += ng * H
        # then whole cycles of untimed replays (in cyclic order: each graph's actions are drawn by the one before
        # it) until the rings have reached their steady state -- >= --steady-steps steps after mgx_reset (round 6:
        # the timed region no longer sits in the first few hundred steps, when every ring is still nearly full) --
        # and the GPU has been busy for --warmup-ms
        while steps_since_reset < args.steady_steps or (time.perf_counter() - t_warm0) * 1e3 < args.warmup_ms:
            for _ in range(16):
                for gr in graphs:
                    gr.replay()
                steps_since_reset += ng * H
                replay_cycles += 1
            torch.cuda.synchronize(dev)
    eng.clock_rewind()                                   # (the slots then hold the region's and the probe's launches)
    st0 = eng.stats()
    # refill launches inside the timed region: the forks the steps enqueued (captured once in the
    # graphs, replayed once each; eagerly, counted as they run)
    forks = (st0["refill_launches"] - forks0) * nchunks // len(graphs) if graphs else None
    hist.zero_()                                         # (the untimed replays accumulated into it)
    scls = eng.rollout_clock_class() if fused else 0     # (S = 16 fused: the 32-env blocks' own class)
    clk0 = (eng.clock_launches(scls), eng.clock_launches(1), eng.clock_launches(2))   # launch counts at the region's start
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    ev0 = torch.cuda.Event(enable_timing=True)
    ev1 = torch.cuda.Event(enable_timing=True)
    ev0.record(stream)                                   # (HIP events are created at their first record:
    ev1.record(stream)                                   # not inside the region)
    torch.cuda.synchronize(dev)
    from mgx.engine import graph_launch
    raw = args.graph_launch == "raw"
    if args.mark_region and hasattr(torch.cuda, "_sleep"):
        torch.cuda._sleep(1000)                          # trace marker (tools/trace_window.py): the region follows
        torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    ev0.record(stream)
    for c in range(nchunks):
        if graphs:
            if raw:
                graph_launch(graphs[c], stream)
            else:
                graphs[c].replay()
        else:
            chunk(c)
        if world > 1:                                    # the one exchange per rollout
            hist[c].copy_(_allreduce(hist[c], dist.ReduceOp.SUM))
    ev1.record(stream)
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    wall = time.perf_counter() - t0
    if args.mark_region and hasattr(torch.cuda, "_sleep"):
        torch.cuda._sleep(1000)                          # trace marker: the region ended
        torch.cuda.synchronize(dev)
    gpu_ms = ev0.elapsed_time(ev1)
    clk1 = (eng.clock_launches(scls), eng.clock_launches(1), eng.clock_launches(2))
    timed_step_us = eng.clock_spans_us(scls, clk0[0], clk1[0])   # the timed region's own kernel launches
    timed_refill_us = eng.clock_spans_us(1, clk0[1], clk1[1])
    timed_slide_us = eng.clock_spans_us(2, clk0[2], clk1[2])
    st1 = eng.stats()
    eng.poll_error()
    # roofline probe: per-launch duration of mgx_step_kernel (HIP events on its stream) in the
    # timed region's regime.  Whole refill epochs; each window is an epoch's launches after its
    # first (the first joins the previous epoch's refill and forks the next), bracketed by one
    # event pair, so the per-launch figure is kernel time plus the back-to-back dispatch gap, with
    # the refill beside the steps for as long as it runs (an event pair around every launch would
    # keep consecutive launches from overlapping at all).
    windows, cur = [], None
    if fused:
        # one window per launch (one refill epoch of E steps); the previous epoch's refill is joined
        # before the window opens, so the window holds the epoch's fork and the kernel.  A spin kernel
        # first keeps the GPU busy while the host enqueues every window (round 4: without it each window
        # also held the host's time to enqueue the refill ahead of the rollout, ~19 us per launch)
        if hasattr(torch.cuda, "_sleep"):
            torch.cuda._sleep(int((P // E) * 60e-6 * 2.4e9))
        for t in range(0, P - P % E, E):
            eng.join()
            w = [torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True), E]
            w[0].record(stream)
            cbuf.rollout(t % H, actions[W + K + t:W + K + t + E])
            w[1].record(stream)
            windows.append(w)
        P = 0

    def probe_step(t):
        if compact:
            cbuf.step(t % H, actions[W + K + t])   # rows are overwritten: timing only
        else:
            eng.step(actions[W + K + t])
    # the host enqueues the probe's launches one by one (~15 us of Python per step, about the
    # kernel's own time): a spin kernel first keeps the GPU busy until they are all queued, so
    # the windows time back-to-back launches, not the host
    if hasattr(torch.cuda, "_sleep"):
        torch.cuda._sleep(int(P * 40e-6 * 2.4e9))
    for t in range(P):
        if eng.epoch_boundary():
            if cur is not None:
                cur[1].record(stream)
                windows.append(cur)
                cur = None
            probe_step(t)
            continue
        if cur is None:
            cur = [torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True), 0]
            cur[0].record(stream)
        probe_step(t)
        cur[2] += 1
    if cur is not None:
        cur[1].record(stream)
        windows.append(cur)
    eng.join()
    torch.cuda.synchronize(dev)
    eng.poll_error()
    probe_us = []
    for a0, a1, cnt in windows:
        probe_us += [a0.elapsed_time(a1) * 1e3 / cnt] * cnt
    per = E if fused else 1                              # steps per step-kernel launch
    step_us = sum(timed_step_us) / len(timed_step_us) / per if timed_step_us else float("nan")
    refill_us = sum(timed_refill_us) / len(timed_refill_us) if timed_refill_us else float("nan")
    elapsed = torch.tensor([wall, gpu_ms / 1e3, step_us, refill_us], dtype=torch.float64, device=dev)
    steps_done = torch.tensor([float(st1["steps"] - st0["steps"]), float(st1["resets"] - st0["resets"])],
                              dtype=torch.float64, device=dev)
    if world > 1:
        elapsed = _allreduce(elapsed, dist.ReduceOp.MAX)
        steps_done = _allreduce(steps_done, dist.ReduceOp.SUM)
    wall_max, gpu_max = float(elapsed[0]), float(elapsed[1])
    step_us_max, refill_us_max = float(elapsed[2]), float(elapsed[3])
    total_env_steps, total_resets = float(steps_done[0]), float(steps_done[1])
    assert int(total_env_steps) == n * K * world, (total_env_steps, n * K * world)
    hs = hist.cpu().numpy()
    assert abs(hs[:, 2].sum() - float(H) * n * world * nchunks) < 0.5, hs    # every chunk's GAE ran
    gae_h = gae_probe(dev, n, H)
    gae_1k = gae_probe(dev, n, 1024) if H != 1024 else gae_h
    # Steady state (round 5, reported beside the headline, N = 1): the same graphs after --steady-ms more of
    # untimed replays, then several timed replays.  The region above follows mgx_reset by a few hundred steps, when
    # every ring is still nearly full; over thousands of steps a few rings drain to the 2K floor and their waves
    # run need-driven rounds every epoch -- the slowest wave sets the refill launch.
    # A second window much later (round 5: N = 1 only; round 6: every world size, barrier + max over ranks): the graphs
    # replayed on, in cyclic order from where the region stopped, for --steady-ms more, then whole cycles timed.  The
    # headline region itself already follows >= --steady-steps steps of warm-up; this checks that the line holds.
    steady = None
    if graphs and args.steady_ms > 0 and layout == args.layout:
        gi = nchunks % len(graphs)                       # the next graph in the cyclic order
        t_s = time.perf_counter()
        cyc = 0
        while (time.perf_counter() - t_s) * 1e3 < args.steady_ms:
            for _ in range(len(graphs)):
                graphs[gi].replay()
                gi = (gi + 1) % len(graphs)
            torch.cuda.synchronize(dev)
            cyc += 1
        nrep = len(graphs) * max(1, -(-200 // (len(graphs) * H)))   # whole cycles, >= 200 steps
        sa = eng.stats()
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize(dev)
        t0s = time.perf_counter()
        for k in range(nrep):
            graphs[gi].replay()
            if world > 1:
                hist[gi % nchunks].copy_(_allreduce(hist[gi % nchunks], dist.ReduceOp.SUM))
            gi = (gi + 1) % len(graphs)
        torch.cuda.synchronize(dev)
        if world > 1:
            dist.barrier()
        wall_s = time.perf_counter() - t0s
        sb = eng.stats()
        tot = torch.tensor([wall_s, float((sb["resets"] - sa["resets"]) + (sb["queued"] - sa["queued"])),
                            float(sb["resets"] - sa["resets"])], dtype=torch.float64, device=dev)
        if world > 1:
            wmax = _allreduce(tot[:1].clone(), dist.ReduceOp.MAX)
            pc = _allreduce(tot[1:].clone(), dist.ReduceOp.SUM)
            tot = torch.cat([wmax.to(dev), pc.to(dev)])
        wall_s, prod_s, cons_s = float(tot[0]), float(tot[1]), float(tot[2])
        steady = {"value": n * world * H * nrep / wall_s, "ms_per_step": wall_s * 1e3 / (H * nrep),
                  "timed_steps": H * nrep,
                  "after_steps": steps_since_reset + K + cyc * len(graphs) * H,
                  "produced_over_consumed": prod_s / max(cons_s, 1),
                  "ratio_to_value": None,
                  "note": "the region's graphs replayed %d more cycles (%.0f ms) untimed, in cyclic order, then %d "
                          "replays (whole cycles) timed, barrier + max over ranks" % (cyc, args.steady_ms, nrep)}
    if rank == 0:
        probe_s = (sum(probe_us) / len(probe_us)) * 1e-6 if probe_us else None
        resets_per_launch = (st1["resets"] - st0["resets"]) / K
        dev_policy = fused and bool(graphs)              # the timed launches draw their own actions: no action byte
        b_alg = (B_STEP - (1 if dev_policy else 0)) * n + (3 * args.size ** 2 + 208) * resets_per_launch
        gae_in = fused and E == H and args.gae_fused
        if gae_in:                                       # the launch also runs GAE over its steps: SURVEY 8(d)'s
            b_alg += 17 * n                              # 17 B per element (r, v, done, adv, ret), per step
        # THE roofline duration: the kernel's own launches inside the timed region, per step, from the device
        # clock (first workgroup start -> last workgroup end of each launch; the max over ranks)
        per_launch_s = step_us_max * 1e-6
        achieved = b_alg / per_launch_s / 1e9
        prof_dir, lib_sha = _profile_dir()
        traffic, traffic_src = None, None
        spl = per
        if prof_dir is not None:
            # rocprofv3 PMC HBM bytes of this kernel at this config AND launch shape (a fused launch of E steps
            # moves per step what E steps share: the PMC file must have steps_per_launch == E), committed under
            # profiles/<round>_pmc/ for THIS build (manifest.json: the libmgx.so hash it was collected with)
            import glob
            for pmc_file in sorted(glob.glob(os.path.join(prof_dir, "pmc_[0-9]_%s*.json" % layout))):
                try:
                    pmc = json.load(open(pmc_file))
                except (OSError, ValueError):
                    continue
                if (pmc.get("n_envs") == n and pmc.get("size") == args.size and pmc.get("mission") == mission
                        and pmc.get("steps_per_launch", 1) == spl):
                    traffic = pmc.get("hbm_bytes_per_launch")
                    if traffic is not None:              # per step (a fused launch holds several)
                        traffic = traffic / spl
                        traffic_src = os.path.relpath(pmc_file, ROOT)
                    break
        kname = "mgx_rollout_kernel" if fused else ("mgx_step_kernel<int, true" if compact else "mgx_step_kernel<int, false")
        kstat = None
        if prof_dir is not None:
            # the same kernel's average duration from the committed rocprofv3 kernel stats of this exact command
            # shape (kernel_stats_<cfg>_<layout>_e<E>.csv), and over the timed region's launches alone from the
            # committed kernel trace of the same command (kernel_trace_*.csv.gz): the cross-check of the device clock
            kstat = _rocprof_kernel_avg(os.path.join(prof_dir, "kernel_stats_%d_%s_e%d.csv" % (
                args.config, layout, spl if fused else E)), kname)
            t_avg = _rocprof_trace_timed_avg(os.path.join(prof_dir, "kernel_trace_%d_%s_e%d.csv.gz" % (
                args.config, layout, spl if fused else E)), kname, steps_since_reset // per, K // per)
            if kstat is not None and t_avg is not None:
                kstat["timed_avg_us"] = t_avg
        produced = (st1["resets"] - st0["resets"]) + (st1["queued"] - st0["queued"])
        consumed = st1["resets"] - st0["resets"]
        refill_launches = forks if forks is not None else st1["refill_launches"] - st0["refill_launches"]
        # the refill (episode generator) inside the timed region: SURVEY §8(d) 400 B per episode produced
        refill = None
        if timed_refill_us:
            b_ref = 400.0 * produced / max(refill_launches, 1)
            refill = {"launches": len(timed_refill_us), "avg_launch_us": refill_us_max,
                      "steps_per_launch": E, "episodes_per_launch": produced / max(refill_launches, 1),
                      "alg_bytes_per_launch": b_ref, "achieved": b_ref / refill_us_max / 1e3,
                      "frac": b_ref / refill_us_max / 1e3 / PEAK_HBM_GBPS, "unit": "GB/s",
                      "slide_avg_launch_us": (sum(timed_slide_us) / len(timed_slide_us)) if timed_slide_us else None,
                      "note": "mgx_refill kernel launches of the timed region (device clock, beside the rollout); "
                              "slide: the MT slide that follows each refill on its stream (rank 0)"}
        # VecFrameStack image + direction roll (reported separately); the compact layout rolls nothing
        stack_bytes = 0 if compact else n * (441 + 588 + 12 + 16)
        out = {
            "metric": METRIC,
            "value": total_env_steps / wall_max,
            "unit": "env-steps/s",
            "n_gpus": world,
            "steps": K,
            "warmup": steps_since_reset,                 # eager warm-up + the graphs' untimed replays
            "warmup_requested": args.warmup,
            "warmup_note": "warm-up raised to >= %d steps in whole refill epochs, then untimed replays of the "
                           "graphs in cyclic order (%d cycles) until >= %d steps after mgx_reset (--steady-steps; "
                           "--warmup-ms %.0f): the timed region sits in the rings' steady state, not in the first "
                           "few hundred steps after the reset filled every ring; every replay draws fresh random "
                           "actions for the next one" % (args.min_warmup, replay_cycles, args.steady_steps,
                                                         args.warmup_ms),
            "steps_after_reset": steps_since_reset,
            "ms_per_step": wall_max * 1e3 / K,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u8",
            "data": "synthetic (uniform random actions on {0..6}: seed 1234+rank for the eager warm-up, then drawn "
                    "afresh inside the graphs at every replay (mgx_random_actions, seed 4321+rank); env i seeded 42+i; "
                    "synthetic values for GAE)",
            "config": {"workload": _workload_name(args, mission, n, world) + (
                           " [fused rollout: one launch per %d-step refill epoch, observation rows into the rollout "
                           "buffer]" % E if fused else
                           " [compact layout: observation rows into the rollout buffer]" if compact else ""),
                       "problem": args.problem, "mission": mission, "size": args.size, "num_objects": 4,
                       "envs_per_gpu": n, "n_stack": args.n_stack, "parallelism": "env-sharded dp%d" % world,
                       "hipgraph": bool(graphs) and not isinstance(graphs[0], _PreparedChunk),
                       "launch": ("prepared C call per chunk" if graphs and isinstance(graphs[0], _PreparedChunk)
                                  else "hipGraph per chunk" if graphs else "python per step"), "refill_every": E, "horizon": H, "layout": layout,
                       "host_wait": getattr(args, "host_wait_applied", "auto"),
                       "graph_launch": ("hipGraphLaunch" if args.graph_launch == "raw" else "CUDAGraph.replay")
                       if graphs else None,
                       "timed": "%d steps = %d whole refill epochs%s; GAE + adv-stat %s every %d steps%s" % (
                           K, K // E, "" if aligned else " + a joined partial one",
                           "all-reduce (%s)" % dist.get_backend() if world > 1 else "accumulation", H,
                           " (fused into the rollout launch: mgx_rollout_compact_gae)" if fused and E == H and args.gae_fused
                           else "")},
            # every episode the timed steps consumed is paid for by a refill inside the region; when the region
            # (one 20-step refill epoch on the driver's line) produced fewer than it consumed, value_resets_paid
            # prices the shortfall in at the region's own production rate
            "value_resets_paid": total_env_steps / wall_max * min(1.0, produced / max(consumed, 1)),
            "window": {"refill_launches": refill_launches, "episodes_produced": produced,
                       "episodes_consumed": consumed, "produced_over_consumed": produced / max(consumed, 1),
                       "gae_launches": nchunks, "graphs": len(graphs),
                       "carry_over": "ring rows (no copy)" if compact else None},
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": PEAK_HBM_GBPS, "unit": "GB/s",
                         "frac": achieved / PEAK_HBM_GBPS, "traffic": traffic, "traffic_source": traffic_src,
                         "kernel": ("mgx_rollout_kernel<false> (fused: %d steps per launch%s; per-step figures = "
                                    "launch / %d)" % (E, ", GAE epilogue: B_alg + 17 B per env-step" if gae_in else "",
                                                      E) if fused else
                                    "mgx_step_kernel<int, true[, 8]> (compact)" if compact else
                                    "mgx_step_kernel<int, false[, 8]> (SB3 stacks)"),
                         "avg_launch_us": per_launch_s * 1e6,
                         "timing": "device clock (mgx_set_clock): the kernel's %d launches inside the timed region, "
                                   "first workgroup start to last workgroup end, per step; max over ranks"
                                   % len(timed_step_us),
                         "timed_launches": len(timed_step_us),
                         "probe_avg_launch_us": probe_s * 1e6 if probe_s else None,
                         "probe_frac": (b_alg / probe_s / 1e9 / PEAK_HBM_GBPS) if probe_s else None,
                         "probe_note": "HIP events around eager probe launches after the region (rollout dispatched "
                                       "first, previous refill joined): not the timed region's regime",
                         "refill": refill,
                         "build": lib_sha,
                         "rocprof": None if kstat is None else {
                             "source": kstat["source"], "avg_launch_us": kstat["avg_us"] / spl,
                             "frac": b_alg / (kstat["avg_us"] / spl * 1e-6) / 1e9 / PEAK_HBM_GBPS,
                             "note": "the committed rocprofv3 --stats average of the same kernel at this config and "
                                     "launch shape, collected with this build (per step; all its launches: warm-up, "
                                     "graph replays, probe), B_alg of this run",
                             "timed_avg_us": (kstat["timed_avg_us"] / spl) if "timed_avg_us" in kstat else None,
                             "timed_frac": (b_alg / (kstat["timed_avg_us"] / spl * 1e-6) / 1e9 / PEAK_HBM_GBPS)
                             if "timed_avg_us" in kstat else None,
                             "timed_note": "the timed region's launches alone (committed kernel trace of the same "
                                           "command, per step)"},
                         "probe_launches": len(probe_us),
                         "step_pipeline_us": float(gpu_ms) * 1e3 / K,
                         "alg_bytes_per_launch": b_alg, "resets_per_launch": resets_per_launch,
                         # the same duration priced with the PMC bytes instead of B_alg: the fused kernel
                         # moves less than B_alg (grids and env state stay in LDS for the whole epoch)
                         "traffic_frac": (traffic / per_launch_s / 1e9 / PEAK_HBM_GBPS) if traffic else None,
                         "stack_bytes_per_launch": stack_bytes,
                         "achieved_incl_stack": (b_alg + stack_bytes) / per_launch_s / 1e9},
            "gae": {"horizon": gae_h, "T1024": gae_1k},
            "steady_state": dict(steady, ratio_to_value=steady["value"] / (total_env_steps / wall_max))
                            if steady else None,
            "gpu_time_ms": gpu_max * 1e3,
        }
        return out
    return None


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    cpu = None
    if args.workload == "rollout" and args.cpu_seconds > 0 and world == 1:
        cpu = cpu_baseline(args, args.cpu_seconds)      # before any GPU call (forks workers)
    # one process per GPU; `local % device_count` only matters for a rehearsal of the
    # N>1 path with more ranks than GPUs (MGX_DIST_BACKEND=gloo: RCCL refuses shared GPUs)
    ndev = torch.cuda.device_count()
    gpu = local % max(ndev, 1)
    backend = os.environ.get("MGX_DIST_BACKEND", "nccl")
    args.host_wait_applied = "auto"
    if args.host_wait != "auto":
        from mgx import MgxError
        from mgx.engine import set_host_wait
        try:
            set_host_wait(args.host_wait, gpu)          # before the first GPU work of this process
            args.host_wait_applied = args.host_wait
        except MgxError as ex:                          # (the line is still printed; it says which wait it ran)
            print("bench: host wait %s refused (%s); HIP's default" % (args.host_wait, ex), file=sys.stderr)
    if world > 1:
        os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", gpu))
        else:
            dist.init_process_group(backend)
    torch.cuda.set_device(gpu)
    dev = torch.device("cuda", gpu)
    ranks_seen = 1
    if world > 1:                                     # the collective itself counts the ranks it joined
        ones = _allreduce(torch.ones(1, dtype=torch.float64, device=dev), dist.ReduceOp.SUM)
        ranks_seen = int(round(float(ones[0])))
    if args.workload == "ppo":
        return main_ppo(args, world, rank, local, dev, ranks_seen)
    out = measure_rollout(args, args.layout, world, rank, dev)
    if world == 1 and args.both_layouts:
        # the other observation layouts on the same workload, reported beside the headline: one launch
        # per step (compact rows: the path a policy in the loop takes) and the materialised SB3 stacks
        # (the MgxVecEnv drop-in's)
        for other in [l for l in ("compact", "sb3") if l != args.layout]:
            torch.cuda.empty_cache()
            o2 = measure_rollout(args, other, world, rank, dev)
            out[other + "_layout"] = {k: o2[k] for k in ("value", "ms_per_step", "roofline", "window")}
    if rank == 0:
        out["ranks_seen"] = ranks_seen
        out["dist_backend"] = dist.get_backend() if world > 1 else None
        if cpu is not None:
            out["cpu_baseline"] = cpu
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
