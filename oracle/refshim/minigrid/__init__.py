"""Clean-room restatement of the minigrid API surface used by the reference
(`src/custom_env.py:6-11`, `src/environment.py:3`).

TEST INFRASTRUCTURE ONLY: lets `tests/golden/make_golden.py` execute the
reference's own `custom_env.py` unchanged.  minigrid is not installed here and
is unpinned in the reference (`requirements.txt:9`); the semantics below are
restated from the public minigrid 2.x/3.x sources (SURVEY.md Appendix A, items
marked (R)) and are therefore *parity unpinned* at this boundary.
"""
