"""ctypes binding of the HIP C-ABI (include/othello.h -> lib/libsubproc_amd_hip.so).

There is no CPU fallback: if the library is missing or fails to load, every
product entry point raises :class:`OthelloLibraryError`.
"""
import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "lib", "libsubproc_amd_hip.so")
HEADER = os.path.join(os.path.dirname(_HERE), "include", "othello.h")

OTH_OK = 0
OTH_EINVAL = -1000
BLACK, WHITE, PASS = 1, 2, 64
HIST_BINS = 133
MOVES_STRIDE = 128
POS_STRIDE = 129
BOOK_LINE = 67
N_FEATURES = 10
POLICY_RANDOM, POLICY_GREEDY, POLICY_EVAL = 0, 1, 2
EVAL_PHASES, EVAL_FEATURES, EVAL_WEIGHTS = 4, 9, 36
TD_KEY_BITS = 43
TD_SKEY_BITS = 36         # include/othello.h packed update words: the sort key's bits
TD_PACK_TURN_SHIFT = 36
TD_PACK_VALUE_SHIFT = 56
TD_FIT_BLOCKS, TD_FIT_COLS = 1024, 64

# name -> (restype, argtypes); must match include/othello.h exactly
_P, _I64, _U64, _I = ctypes.c_void_p, ctypes.c_int64, ctypes.c_uint64, ctypes.c_int
SIGNATURES = {
    "oth_version": (ctypes.c_char_p, []),
    "oth_reset": (_I, [_P, _P, _P, _I64, _P]),
    "oth_legal": (_I, [_P, _P, _P, _I64, _P]),
    "oth_step": (_I, [_P, _P, _P, _P, _P, _P, _P, _P, _P, _I64, _P]),
    "oth_result": (_I, [_P, _P, _P, _P, _P, _I64, _P]),
    "oth_hands": (_I, [_P, _P, _P, _P, _P, _P, _P, _I64, _P]),
    "oth_rollout": (_I, [_P, _P, _U64, _U64, _I, _I, _P, _P, _P, _P, _P, _P, _I64, _P]),
    "oth_sample_midgame": (_I, [_U64, _U64, _P, _P, _P, _P, _I64, _P]),
    "oth_replay": (_I, [_P, _P, _P, _P, _P, _P, _P, _I64, _P]),
    "oth_replay_rows": (_I, [_P, _P, _P, _P, _P, _P, _P, _P, _I64, _P]),
    "oth_book_text": (_I, [_P, _P, _I64, _P, _P]),
    "oth_book_parse": (_I, [_P, _I64, _P, _P, _I64, _P]),
    "oth_features": (_I, [_P, _P, _P, _I64, _P]),
    "oth_rollout_eval": (_I, [_P, _P, _U64, _U64, _I, _P, _P, _P, _P, _P, _P, _P, _I64, _P]),
    "oth_rollout_match": (_I, [_P, _P, _U64, _U64, _I, _P, _P, _P, _P, _P, _P, _P, _P, _I64, _P]),
    "oth_rollout_runner": (_I, [_P, _P, _U64, _U64, _I, _P, _P, _I, _I, _I, _P, _P, _P, _P, _P, _P, _P, _I64, _P]),
    "oth_eval": (_I, [_P, _P, _P, _P, _I64, _P]),
    "oth_td_updates": (_I, [_P, _P, _P, _P, _P, _P, _I64, _P]),
    "oth_td_updates_rows": (_I, [_P, _P, _P, _P, _P, _P, _P, _I64, _P]),
    "oth_td_updates_records": (_I, [_P, _P, _P, _P, _P, _P, _I64, _P]),
    "oth_td_ema": (_I, [_P, _P, _P, ctypes.c_double, ctypes.c_double, _P, _I64, _P]),
    "oth_td_new_before": (_I, [_P, _I64, _P, _P, _P, _P]),
    "oth_td_segments": (_I, [_P, _I64, _I64, _P, _P, _P, _P, _P, _P, _P]),
    "oth_td_segments_words": (_I, [_P, _P, _I64, _I64, _P, _P, _P, _P, _P, _P, _P, _P]),
    "oth_td_ema_split": (_I, [_P, _P, _P, ctypes.c_double, ctypes.c_double, _P, _I64, _I64, _P, _I64, _I64, _P, _P,
                              _P]),
    "oth_td_sort_pairs": (_I, [_P, _P, _P, _P, _I64, _P, _P, _P]),
    "oth_rollout_grid": (_I, [_I, _I64]),
    "oth_td_updates_packed": (_I, [_P, _P, _P, _P, _P, _I64, _P]),
    "oth_td_sort_packed": (_I, [_P, _P, _I64, _P, _P, _P]),
    "oth_td_sort_unpack": (_I, [_P, _P, _P, _P, _I64, _P, _P, _P]),
    "oth_td_unpack": (_I, [_P, _P, _P, _P, _I64, _P]),
    "oth_td_word_errors": (_I, [_P, _I, _P]),
    "oth_td_merge": (_I, [_P, _P, _I64, _P, _P, _P, _I64, _P, _P, _P, _P, _P]),
    "oth_td_lookup": (_I, [_P, _P, _I64, _P, _I64, _P, _P, _P, _P, _P]),
    "oth_td_lookup_dev": (_I, [_P, _P, _I64, _P, _I64, _P, _P, _P, _P, _P, _P]),
    "oth_td_merge_after_lookup": (_I, [_P, _P, _I64, _P, _P, _P, _I64, _P, _P, _P, _P]),
    "oth_td_fit_moments": (_I, [_P, _P, _I64, _P, _P, _P]),
}


class OthelloLibraryError(RuntimeError):
    pass


class OthelloCallError(RuntimeError):
    pass


_lib = None


def load():
    """Load the HIP library (once).  torch is imported first so that the HIP
    runtime the library binds to (soname libamdhip64.so.7) is the one torch
    already loaded: device pointers and hipStream_t handles from torch are then
    valid in the library."""
    global _lib
    if _lib is not None:
        return _lib
    import torch  # noqa: F401  (runtime sharing, see docstring)

    if not os.path.exists(LIB_PATH):
        raise OthelloLibraryError(
            f"{LIB_PATH} not found: build it with `python -c 'import __graft_entry__ as g; g.build()'` "
            "(hipcc --offload-arch=gfx950). There is no CPU fallback.")
    try:
        lib = ctypes.CDLL(LIB_PATH)
    except OSError as e:
        raise OthelloLibraryError(f"cannot load {LIB_PATH}: {e}") from e
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    _lib = lib
    return lib


def check(status, what):
    if status != OTH_OK:
        if status == OTH_EINVAL:
            raise OthelloCallError(f"{what}: invalid argument (OTH_EINVAL)")
        raise OthelloCallError(f"{what}: HIP error {-status}")


def version():
    return load().oth_version().decode()


def library_sha16(path=None):
    """First 16 hex digits of the SHA-256 of the HIP library file: the build
    identity that bench lines and profile digests are stamped with (the build
    is deterministic: the same sources and flags give the same file)."""
    import hashlib

    with open(path or LIB_PATH, "rb") as f:
        return hashlib.sha256(f.read()).hexdigest()[:16]
