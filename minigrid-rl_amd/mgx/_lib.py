"""ctypes binding of libmgx.so (the C ABI declared in include/mgx.h).

This is the reference-side binding a Python caller uses; no torch types cross
the ABI (device pointers are plain integers).  torch MUST be imported before
the library is loaded so that libmgx binds to the HIP runtime torch already
loaded (both carry SONAME libamdhip64.so.7) -- one runtime per process.
"""
import ctypes
import os

import torch  # noqa: F401  (see module docstring: load order matters)

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("MGX_LIB_PATH", os.path.join(HERE, "libmgx.so"))   # override: diagnostic builds

MGX_OK = 0
GAE_SCRATCH_WORDS = 512  # == MGX_GAE_SCRATCH_WORDS (include/mgx.h)
ABI_VERSION = 7        # == MGX_ABI_VERSION (include/mgx.h)
PROBLEMS = {"multi": 0, "full": 1, "gto": 2, "gtg": 3, "opn": 4, "pkp": 5, "drp": 6, "mov": 7}
TERMINAL = {"none": 0, "truncated": 1, "all": 2}
DEVERR = {1: "MT19937 ring: a cursor left the window of the stream the device holds", 2: "action outside 0..6 (ValueError: Unknown action)",
          4: "PCG64 rejection loop bound exceeded", 8: "object list exhausted (AssertionError / IndexError in the reference)",
          16: "episode ring ran dry (engine invariant broken)"}

# Every entry point include/mgx.h declares (checked by tests/test_abi.py).
EXPORTS = ("mgx_last_error", "mgx_abi_version", "mgx_create", "mgx_destroy", "mgx_reset", "mgx_step",
           "mgx_join", "mgx_get_config", "mgx_set_seed", "mgx_gae", "mgx_gae_dones", "mgx_poll_error", "mgx_stats", "mgx_debug_counters", "mgx_dump_state", "mgx_mission_text",
           "mgx_step_compact", "mgx_rollout_compact", "mgx_rollout_compact_gae", "mgx_observe_compact", "mgx_gather",
           "mgx_gather_ring", "mgx_scene", "mgx_set_clock", "mgx_clock_words", "mgx_clock_groups",
           "mgx_ring_levels", "mgx_random_actions", "mgx_set_random_policy")
CLOCK_CLASSES = 4   # == MGX_CLOCK_CLASSES (include/mgx.h)


class MgxConfig(ctypes.Structure):
    _fields_ = [
        ("problem", ctypes.c_int32), ("mission", ctypes.c_int32), ("size", ctypes.c_int32),
        ("num_objects", ctypes.c_int32), ("see_through_walls", ctypes.c_int32),
        ("all_doors_open", ctypes.c_int32), ("obstacles", ctypes.c_int32), ("n_stack", ctypes.c_int32),
        ("n_envs", ctypes.c_int64), ("base_seed", ctypes.c_int64), ("env_index_offset", ctypes.c_int64),
        ("livelock_words", ctypes.c_int32), ("terminal_mode", ctypes.c_int32),
        ("mission_int64", ctypes.c_int32), ("refill_cap", ctypes.c_int32), ("mt_table_words", ctypes.c_int64),
        ("ring_depth", ctypes.c_int32), ("refill_every", ctypes.c_int32),
        ("percent_obstacles", ctypes.c_double), ("manual", ctypes.c_int32), ("reserved0", ctypes.c_int32),
    ]


class MgxObs(ctypes.Structure):
    _fields_ = [("image_dev", ctypes.c_void_p), ("direction_dev", ctypes.c_void_p),
                ("mission_dev", ctypes.c_void_p)]


class MgxStepOut(ctypes.Structure):
    _fields_ = [
        ("obs", MgxObs), ("terminal", MgxObs),
        ("reward_dev", ctypes.c_void_p), ("reward64_dev", ctypes.c_void_p),
        ("terminated_dev", ctypes.c_void_p), ("truncated_dev", ctypes.c_void_p), ("done_dev", ctypes.c_void_p),
        ("ep_return_dev", ctypes.c_void_p), ("ep_len_dev", ctypes.c_void_p), ("livelock_dev", ctypes.c_void_p),
    ]


class MgxCompactOut(ctypes.Structure):
    _fields_ = [
        ("row_dev", ctypes.c_void_p), ("mission_id_dev", ctypes.c_void_p), ("terminal_row_dev", ctypes.c_void_p),
        ("reward_dev", ctypes.c_void_p), ("reward64_dev", ctypes.c_void_p),
        ("terminated_dev", ctypes.c_void_p), ("truncated_dev", ctypes.c_void_p), ("done_dev", ctypes.c_void_p),
        ("ep_return_dev", ctypes.c_void_p), ("ep_len_dev", ctypes.c_void_p), ("livelock_dev", ctypes.c_void_p),
    ]


class MgxRolloutOut(ctypes.Structure):
    _fields_ = [
        ("rows_dev", ctypes.c_void_p), ("mission_ids_dev", ctypes.c_void_p), ("terminal_row_dev", ctypes.c_void_p),
        ("rewards_dev", ctypes.c_void_p), ("rewards64_dev", ctypes.c_void_p), ("terminated_dev", ctypes.c_void_p),
        ("truncated_dev", ctypes.c_void_p), ("dones_dev", ctypes.c_void_p), ("ep_return_dev", ctypes.c_void_p),
        ("ep_len_dev", ctypes.c_void_p), ("livelock_dev", ctypes.c_void_p),
    ]


class MgxGaeArgs(ctypes.Structure):
    _fields_ = [
        ("values_dev", ctypes.c_void_p), ("last_values_dev", ctypes.c_void_p), ("gamma", ctypes.c_float),
        ("gamma_lambda", ctypes.c_float), ("advantages_dev", ctypes.c_void_p), ("returns_dev", ctypes.c_void_p),
        ("adv_stats_dev", ctypes.c_void_p), ("stats_scratch_dev", ctypes.c_void_p),
    ]


class MgxError(RuntimeError):
    pass


_lib = None


def load():
    """Load libmgx.so; fails loudly when the HIP extension has not been built."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise MgxError("libmgx.so not found at %s -- run `python __graft_entry__.py build` "
                       "(the engine has no CPU fallback)" % LIB_PATH)
    L = ctypes.CDLL(LIB_PATH)
    P, I, I64 = ctypes.c_void_p, ctypes.c_int, ctypes.c_int64
    L.mgx_last_error.restype = ctypes.c_char_p
    L.mgx_abi_version.restype = I
    L.mgx_create.argtypes = [ctypes.POINTER(MgxConfig), I, ctypes.POINTER(P)]
    L.mgx_destroy.argtypes = [P]
    L.mgx_reset.argtypes = [P, ctypes.POINTER(MgxObs), P, P]
    L.mgx_step.argtypes = [P, P, I, ctypes.POINTER(MgxStepOut), P]
    L.mgx_join.argtypes = [P, P]
    L.mgx_set_seed.argtypes = [P, I64]
    L.mgx_get_config.argtypes = [P, ctypes.POINTER(MgxConfig)]
    L.mgx_gae.argtypes = [P, P, P, P, P, I64, I64, ctypes.c_float, ctypes.c_float, P, P, P, P, P]
    L.mgx_gae_dones.argtypes = [P, P, P, P, I64, I64, ctypes.c_float, ctypes.c_float, P, P, P, P, P]
    L.mgx_poll_error.argtypes = [P, P, ctypes.POINTER(ctypes.c_uint32)]
    L.mgx_stats.argtypes = [P, P, ctypes.POINTER(ctypes.c_uint64)]
    L.mgx_ring_levels.argtypes = [P, P, P]
    L.mgx_random_actions.argtypes = [P, I64, I, ctypes.c_uint64, P, P]
    L.mgx_set_random_policy.argtypes = [P, I, ctypes.c_uint64]
    L.mgx_debug_counters.argtypes = [P, P, ctypes.POINTER(ctypes.c_uint64), ctypes.c_int]
    L.mgx_dump_state.argtypes = [P, P] + [P] * 10
    L.mgx_mission_text.argtypes = [I, ctypes.c_char_p, ctypes.c_size_t]
    L.mgx_step_compact.argtypes = [P, P, I, ctypes.POINTER(MgxCompactOut), P]
    L.mgx_observe_compact.argtypes = [P, P, P, P]
    L.mgx_rollout_compact.argtypes = [P, P, I, ctypes.POINTER(MgxRolloutOut), P]
    L.mgx_rollout_compact_gae.argtypes = [P, P, I, ctypes.POINTER(MgxRolloutOut), ctypes.POINTER(MgxGaeArgs), P]
    L.mgx_gather.argtypes = [P, P, P, P, I64, P, I64, P, P, I, P, I, P, P]
    L.mgx_gather_ring.argtypes = [P, P, P, P, I64, I64, P, I64, P, P, I, P, I, P, P]
    L.mgx_set_clock.argtypes = [P, P, I, ctypes.POINTER(I)]
    L.mgx_clock_words.argtypes = [P, I]
    L.mgx_clock_words.restype = I64
    L.mgx_clock_groups.argtypes = [P, I]
    L.mgx_scene.argtypes = [P, I64, ctypes.POINTER(ctypes.c_uint32), P]
    for name in EXPORTS:
        getattr(L, name).restype = getattr(L, name).restype or I
    if L.mgx_abi_version() != ABI_VERSION:
        raise MgxError("libmgx ABI mismatch")
    _lib = L
    return L


def check(status, what=""):
    if status != MGX_OK:
        raise MgxError("%s failed (status %d): %s" % (what, status, load().mgx_last_error().decode()))


def mission_text(mission_id):
    buf = ctypes.create_string_buffer(64)
    check(load().mgx_mission_text(int(mission_id), buf, 64), "mgx_mission_text")
    return buf.value.decode()


# TokenizeVocabWrapper's vocabulary (environment.py:75-81): ' ' '\n' '-' ':' ',' '.' then a..z
_VOCAB = {c: i for i, c in enumerate(" \n-:,." + "abcdefghijklmnopqrstuvwxyz")}


def tokenize(text):
    """TokenizeVocabWrapper.observation (environment.py:91-112): lower-cased mission text ->
    32 vocabulary indices, zero-padded."""
    out = [0] * 32
    for i, c in enumerate(text.lower()[:32]):
        out[i] = _VOCAB.get(c, 0)
    return out


def mission_tokens():
    """u8 [256][32]: the tokens of every mission id (rows of unused ids are zeros) -- what the
    engine's compact rows carry as one mission-id byte."""
    import numpy as np
    tab = np.zeros((256, 32), np.uint8)
    buf = ctypes.create_string_buffer(64)
    L = load()
    for mid in range(256):
        if L.mgx_mission_text(mid, buf, 64) == MGX_OK:
            tab[mid] = tokenize(buf.value.decode())
    return tab
