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
