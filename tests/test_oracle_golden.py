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
    assert len(FIXTURES) == 39


def test_manual_fixtures_hold_premature_dones():
    """The manual=True fixtures (PlaygroundEnv(manual=True), custom_env.py:319-328) contain 'done'
    actions that end nothing (mission not complete) and 'done' actions that end a completed
    mission with its stored reward."""
    for name in ("manual_multi_all_s8", "manual_multi_pkp_s11"):
        d = dict(np.load(TC.GOLDEN + "/traj/%s.npz" % name))
        a, term = d["actions"], d["terminated"]
        assert ((a == 6) & (term == 0)).sum() > 100, name
        assert ((a == 6) & (term == 1) & (d["reward"] > 0)).sum() > 0, name


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
