"""bench.py's timed-region rules (CPU): the refill epoch divides the timed steps and stays within
D/4, the horizon is whole epochs dividing the steps (<= 1,024, ppo.yaml's n_steps)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import bench  # noqa: E402


def test_pick_epoch():
    assert bench.pick_epoch(2048) == 64          # D/4 at D = 256
    assert bench.pick_epoch(20) == 20            # the driver's --steps 20
    assert bench.pick_epoch(96) == 48
    assert bench.pick_epoch(5) == 5              # K < 8: one epoch
    assert bench.pick_epoch(67) is None          # prime > 64: joined partial epoch
    for K in (20, 64, 100, 2048, 4096):
        E = bench.pick_epoch(K)
        assert K % E == 0 and 8 <= E <= 64


def test_pick_horizon():
    assert bench.pick_horizon(2048, 32, 0) == 1024
    assert bench.pick_horizon(20, 20, 0) == 20
    assert bench.pick_horizon(4096, 32, 256) == 256   # requested and valid
    assert bench.pick_horizon(4096, 32, 100) == 1024  # invalid request -> default
    for K, E in ((2048, 32), (96, 32), (20, 20), (640, 32)):
        H = bench.pick_horizon(K, E, 0)
        assert K % H == 0 and H % E == 0 and H <= 1024


def test_committed_profiles_reproduce_the_driver_line_roofline():
    """profiles/r04_pmc holds, for the driver's command (config 2, fused, 20-step epochs), the rocprofv3
    kernel stats, the kernel trace and the FETCH / WRITE passes that bench.py reads back: the rollout
    kernel's average launch, the timed region's launch (after 13 warm-up epochs and the graph's untimed
    replay) and the PMC bytes per launch of the same launch shape."""
    import json
    d = os.path.join(bench.ROOT, "profiles", "r04_pmc")
    st = bench._rocprof_kernel_avg(os.path.join(d, "kernel_stats_2_fused_e20.csv"), "mgx_rollout_kernel")
    assert st is not None and st["calls"] >= 15 and 80.0 < st["avg_us"] < 250.0
    W, K, E = 260, 20, 20                      # bench's warm-up (>= 256, whole epochs), timed steps, epoch
    t = bench._rocprof_trace_timed_avg(os.path.join(d, "kernel_trace_2_fused_e20.csv.gz"), "mgx_rollout_kernel",
                                       (W + K) // E, K // E)
    assert t is not None and 80.0 < t < 300.0
    pmc = json.load(open(os.path.join(d, "pmc_2_fused_e20.json")))
    assert pmc["steps_per_launch"] == 20 and pmc["n_envs"] == 65536 and pmc["mission"] == 5
    # the rows (148 B), mission ids, rewards and flags the launch writes: >= 20 x 65,536 x 158 B
    assert pmc["write_bytes_per_launch"] >= 20 * 65536 * 158
    # a window of launches outside the trace is refused, not averaged
    assert bench._rocprof_trace_timed_avg(os.path.join(d, "kernel_trace_2_fused_e20.csv.gz"),
                                          "mgx_rollout_kernel", 10 ** 6, 1) is None


def test_host_wait_modes_and_defaults():
    """bench.py's defaults (round 5): spin-waiting host, GAE fused into the rollout launch; an unknown wait mode
    is refused before anything touches the HIP runtime."""
    import pytest
    sys.argv = ["bench.py"]
    a = bench.parse()
    assert a.host_wait == "spin" and a.gae_fused == 1
    sys.path.insert(0, os.path.join(bench.ROOT, "minigrid-rl_amd"))
    from mgx.engine import set_host_wait
    with pytest.raises(ValueError):
        set_host_wait("busy")
