"""The C oracle (oracle/mgx_oracle.c) against the golden fixtures produced by
executing the reference's own custom_env.py / environment.py
(tests/golden/make_golden.py).  Bit-exact: obs, rewards (fp64), flags, full
grid + agent state after every step, RNG stream positions after every reset,
live-lock retry counts."""
import numpy as np
import pytest

import trajcheck as TC

FIXTURES = TC.fixtures()


def test_fixtures_present():
    assert len(FIXTURES) == 37


@pytest.mark.parametrize("path", FIXTURES, ids=lambda p: p.split("/")[-1][:-4])
def test_oracle_matches_reference_fixture(path):
    d = dict(np.load(path))
    cfg, T = TC.fixture_cfg(d)
    msg = TC.compare(TC.OracleSource(cfg), d)
    assert msg is None, msg


def test_fixture_covers_quirks():
    """The fixtures exercise the paths that matter: live-locks (S=8), truncation,
    mission completion with stored reward, goal termination."""
    tot_ll = tot_trunc = tot_goal = tot_stored = 0
    for p in FIXTURES:
        d = dict(np.load(p))
        tot_ll += int(d["livelock"].sum() + d["reset0_livelock"].sum())
        tot_trunc += int(d["truncated"].sum())
        tot_goal += int(((d["reward"] > 0) & (d["terminated"] == 1)).sum())
        tot_stored += int(np.isfinite(d["stored_reward"]).sum())
    assert tot_ll > 0 and tot_goal > 0 and tot_stored > 0
