"""RNG known-answer tests: the oracle's MT19937 / SeedSequence / PCG64 /
Generator.integers restatements against the REAL CPython `random` and numpy
of this image (these two are pinned, unlike minigrid/SB3)."""
import random

import numpy as np

import oracle as O


def test_mt19937_matches_cpython_random():
    for seed in (0, 1, 42, 2**31 + 5, 2**40 + 3):
        r = random.Random(seed)
        ref = np.array([r.getrandbits(32) for _ in range(2000)], np.uint32)
        assert np.array_equal(O.mt_words(seed, 2000), ref), seed


def test_randbelow_rule():
    """_randbelow(n) == getrandbits(bit_length(n)) rejection, one word per draw."""
    r = random.Random(42)
    words = O.mt_words(42, 5000)
    i = 0
    for n in [2, 3, 4, 6, 5, 18, 17, 1, 25, 7] * 30:
        k = n.bit_length()
        while True:
            v = int(words[i]) >> (32 - k)
            i += 1
            if v < n:
                break
        assert r.randrange(n) == v


def test_pcg64_seeding_matches_numpy():
    for seed in [0, 1, 42, 43, 57, 1000, 65535 + 42, 2**32 + 7, 2**40 + 42]:
        st = np.random.PCG64(np.random.SeedSequence(seed)).state["state"]
        m = (1 << 64) - 1
        want = [st["state"] >> 64, st["state"] & m, st["inc"] >> 64, st["inc"] & m]
        assert [int(x) for x in O.pcg_seed_state(seed)] == want, seed


def test_generator_integers_matches_numpy():
    rng = np.random.default_rng(7)
    lo = rng.integers(0, 5, 3000)
    hi = lo + rng.integers(1, 40, 3000)
    for seed in (42, 43, 1234):
        g = np.random.Generator(np.random.PCG64(np.random.SeedSequence(seed)))
        ref = np.array([g.integers(int(a), int(b)) for a, b in zip(lo, hi)], np.int64)
        assert np.array_equal(O.pcg_integers(seed, lo, hi), ref), seed
