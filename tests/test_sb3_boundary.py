"""The SB3 boundary of the VecEnv drop-in (src/ppo.py:118-136), checked on the declared spaces
without a GPU.  stable_baselines3 is not importable here, so SB3's BaseAlgorithm._wrap_env and
the VecTransposeImage / VecFrameStack space transforms are RESTATED from SB3 2.x below: this
boundary is parity unpinned.

_wrap_env(env) does two things to the env the reference hands PPO (ppo.py:134-136):
  1. anything that is not an SB3 VecEnv is wrapped in DummyVecEnv;
  2. for every image space (uint8 Box, 3 dims, bounds 0..255) that is not channels-first
     (argmin(shape) != 0), VecTransposeImage is applied -- unless the chain already holds one
     (is_vecenv_wrapped(env, VecTransposeImage)).
"""
import numpy as np

from mgx import vec_env as V
from mgx.spaces import make_spaces


def is_image_space(space):
    return (len(space.shape) == 3 and np.dtype(space.dtype) == np.uint8 and bool(np.all(space.low == 0))
            and bool(np.all(space.high == 255)))


def channels_first(space):
    return int(np.argmin(space.shape)) == 0


def wrap_env_transposes(obs_space, chain):
    """Keys _wrap_env would transpose (again) for a wrapper chain (outermost first)."""
    if "VecTransposeImage" in chain:
        return []
    return [k for k, s in obs_space.items() if is_image_space(s) and not channels_first(s)]


class _Box:
    def __init__(self, shape, dtype, low, high):
        self.shape, self.dtype = tuple(shape), np.dtype(dtype)
        self.low, self.high = np.full(self.shape, low, self.dtype), np.full(self.shape, high, self.dtype)


def transpose_space(space):                     # VecTransposeImage.transpose_space: (H, W, C) -> (C, H, W)
    h, w, c = space.shape
    return _Box((c, h, w), space.dtype, 0, 255)


def stack_space(space, n):                      # VecFrameStack(n, 'first'): repeat along axis 0
    return _Box((space.shape[0] * n,) + tuple(space.shape[1:]), space.dtype, space.low.min(), space.high.max())


def test_raw_mode_survives_ppo_wrap_env_after_the_reference_wrappers():
    """Raw mode + the reference's own lines 124-126: the chain holds a VecTransposeImage, so
    _wrap_env adds nothing, and the spaces PPO sees equal the fused mode's (what the engine's
    collectors use)."""
    raw, act = make_spaces(1, raw=True)
    assert raw["image"].shape == (7, 7, 3) and raw["mission"].dtype == np.int64 and act.n == 7
    # ppo.py:125-126
    img = stack_space(transpose_space(raw["image"]), 4)
    stacked = {"image": img, "direction": stack_space(raw["direction"], 4), "mission": stack_space(raw["mission"], 4)}
    assert wrap_env_transposes(stacked, ["VecFrameStack", "VecTransposeImage", "MgxVecEnv"]) == []
    fused, _ = make_spaces(4)
    for k in ("image", "direction", "mission"):
        assert tuple(fused[k].shape) == stacked[k].shape, k
        assert np.dtype(fused[k].dtype) == stacked[k].dtype, k
    # n_frames_stack == 1 (line 124 false): the raw (7,7,3) image is transposed by _wrap_env itself,
    # exactly as the reference's own make_vec_env envs would be
    assert wrap_env_transposes(raw, ["MgxVecEnv"]) == ["image"]


def test_fused_mode_is_not_for_sb3_wrap_env():
    """Fused mode's (12,7,7) image has its smallest dimension at index 1: _wrap_env, finding no
    VecTransposeImage in the chain, would transpose it to (7,12,7).  That is why raw mode is the
    SB3 drop-in and the module docstring says so."""
    fused, _ = make_spaces(4)
    assert wrap_env_transposes(fused, ["MgxVecEnv"]) == ["image"]
    assert "raw mode" in V.__doc__


def test_vec_env_subclasses_sb3_vecenv_when_importable():
    """_wrap_env's first check: MgxVecEnv is an SB3 VecEnv whenever SB3 is importable (no
    DummyVecEnv around it); without SB3 it duck-types the same methods."""
    assert V.MgxVecEnv.__mro__[1] is V._VecEnvBase
    assert V.HAVE_SB3 == (V._VecEnvBase is not object)
    for m in ("reset", "step_async", "step_wait", "step", "seed", "close", "get_attr", "set_attr", "env_method",
              "env_is_wrapped", "get_images", "render"):
        assert callable(getattr(V.MgxVecEnv, m)), m


def test_raw_direction_space_follows_make_env():
    """environment.py:28-29: Discrete2BoxWrapper (one-hot Box(4,)) only when n_frames_stack > 1 and not
    recurrent; otherwise MiniGridEnv's own Discrete(4)."""
    box, _ = make_spaces(1, raw=True)
    assert tuple(box["direction"].shape) == (4,)
    disc, _ = make_spaces(1, raw=True, dir_one_hot=False)
    assert disc["direction"].n == 4 and tuple(disc["direction"].shape) == ()


def test_dummy_vec_env_semantics_warn():
    """ppo.py:121 picks DummyVecEnv outside single-run mode; its envs share one process-global MT19937
    stream, which the engine does not interleave: asking for it with n_envs > 1 warns (before the
    engine, so this runs without a GPU too)."""
    import pytest
    with pytest.warns(RuntimeWarning, match="DummyVecEnv"):
        try:
            V.MgxVecEnv(4, vec_env_cls="dummy")
        except Exception as e:                      # no GPU here: the engine itself refuses after the warning
            assert "GPU" in str(e) or "device" in str(e).lower(), e
    with pytest.raises(ValueError):
        V.MgxVecEnv(4, vec_env_cls="forked")
