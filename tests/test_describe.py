"""LLMDescriptionWrapper / PlaygroundEnv.llm_description (environment.py:152-195, custom_env.py's
generators) against the reference: every fixture records the llm_description text of every reset
the reference made (tests/golden/make_golden.py runs the reference); the engine, driven by the
same actions in the inline reset mode, must rebuild each of them from its scene record."""
import numpy as np
import pytest

import trajcheck as TC

torch = pytest.importorskip("torch")


def test_mission_tokens_vocab():
    from mgx.describe import MSN_LEN, VOCAB, mission_tokens
    assert VOCAB[:6] == [" ", "\n", "-", ":", ",", "."] and VOCAB[6] == "a" and len(VOCAB) == 32
    t = mission_tokens("The scene contains:\nMission: go to goal")
    assert t.shape == (MSN_LEN,) and t.dtype == np.int64
    assert list(t[:4]) == [VOCAB.index("t"), VOCAB.index("h"), VOCAB.index("e"), 0] and t[40:].sum() == 0


@pytest.mark.gpu
@pytest.mark.parametrize("path", [p for p in TC.fixtures()], ids=lambda p: p.split("/")[-1][:-4])
def test_llm_description_matches_reference(path):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from mgx import MgxEngine
    from mgx.describe import LLMDescriptionWrapper
    d = dict(np.load(path))
    if "desc_text" not in d:
        pytest.skip("fixture without descriptions")
    cfg, T = TC.fixture_cfg(d)
    kw = dict(cfg)
    n = kw.pop("n_envs")
    problem = kw["problem"]
    eng = MgxEngine(n_envs=n, ring_depth=-1, terminal_mode="none", **kw)
    if kw.get("manual"):
        # the wrapper's own path: make_env(manual=True) -> PlaygroundEnv(manual=True), where a
        # premature 'done' ends nothing (custom_env.py:325)
        wrap = LLMDescriptionWrapper(eng, problem)
        describe = wrap.description
    else:
        from mgx.describe import llm_description, scene
        with pytest.raises(Exception, match="manual=True"):
            LLMDescriptionWrapper(eng, problem)
        describe = lambda i: llm_description(scene(eng, i), problem)     # noqa: E731
    eng.reset()
    want = {}
    for t, i, txt in zip(d["desc_t"], d["desc_env"], d["desc_text"]):
        want.setdefault(int(t), {})[int(i)] = str(txt)
    T = min(T, 200)
    for i in range(n):
        assert describe(i) == want[-1][i], ("first reset", i)
    checked = n
    for t in range(T):
        eng.step(torch.as_tensor(d["actions"][t].astype(np.int32), device=eng.device))
        for i, txt in want.get(t, {}).items():
            assert describe(i) == txt, (t, i)
            checked += 1
    assert checked > n
    eng.poll_error()


def test_llm_description_formatting_from_a_record():
    """The formatter on a hand-made 2-room scene record: the layout and door lines, then per room
    robot / door keys / goal / objects in placement order (custom_env.py:617-725)."""
    from mgx.describe import KEYFLAG, llm_description
    S = 8
    grid = np.full((S, S), 1, np.uint8)
    grid[3, 4] = 4 | (4 << 4) | 0x80                                   # locked door at x=4, y=3
    objs = [dict(type=4, color=5, x=4, y=3, key=False),                # yellow door
            dict(type=8, color=15, x=6, y=2, key=False),               # goal, right room
            dict(type=7, color=5, x=2, y=5, key=True),                 # key box for the door, left room
            dict(type=6, color=0, x=1, y=1, key=False),                # blue ball, left
            dict(type=5, color=3, x=5, y=6, key=False)]                # purple key, right
    sc = dict(objs=objs, agent=(2, 2, 0), mission_id=3, grid=grid, size=S)
    assert llm_description(sc, "multi") == (
        "The scene contains:\nTwo rooms. Left and right.\n"
        "There is a locked yellow door between the rooms\n"
        "Left room contains:\n- robot\n- yellow box\n- blue ball\n"
        "Right room contains:\n- goal\n- purple key\nMission: ")
    assert KEYFLAG == 1 << 24
    single = dict(objs=[dict(type=6, color=1, x=1, y=1, key=False), dict(type=8, color=15, x=2, y=2, key=False)],
                  agent=(3, 3, 0), mission_id=3, grid=grid, size=S)
    assert llm_description(single, "gtg").endswith("- green ball\n- goal\nMission: ")
    assert llm_description(single, "drp").endswith("- green ball\nMission: ")     # the drop map's quirk
