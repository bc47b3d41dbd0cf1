"""Linear-eval weights of the progress/position/moves learner.

The learner (progress_position_moves_learn.py) fits, per disc-count shard
(0..16, 17..32, 33..48, 49..64 -- its ``__get_fit_parameters_shards``, 112-113),
a linear model of the TD value on the 9 non-phase ``counts()`` features
(n_puttable_for, region mask counts a..h; parameter_progress_position_moves_learn.py:5-17),
scales the coefficients to max |w| = 127 (180-181) and stores them as 36
integers (196-203).  ``paramgen.py`` writes them for the engine as bytes:
a header byte, the 36 values as two's-complement int8, and a trailing 0
(paramgen.py:5-19).

This module holds that table as an int8 array [4, 9] -- the layout
``oth_eval`` / ``oth_rollout_eval`` take -- and reads/writes the paramgen
file format.
"""
import numpy as np

from ._lib import EVAL_FEATURES, EVAL_PHASES, EVAL_WEIGHTS

# ProgressPositionMovesParameter.default_value() (parameter_progress_position_moves_learn.py:30-36)
DEFAULT_WEIGHTS = np.array([
    [100, 99, -1, -1, -1, -1, 3, 8, 20],
    [75, 99, 2, -5, 7, 6, 4, 5, 5],
    [25, 99, 2, -5, -7, -6, 4, 5, 5],
    [1, 100, 50, 30, 30, 30, 30, 30, 30],
], dtype=np.int8)

# ProgressPositionMovesParameter.header() (parameter_progress_position_moves_learn.py:27-28),
# the first value read_parameters returns (progress_position_moves_learn.py:217)
HEADER = 2

# learner shard bounds (inclusive), row k of the table
SHARDS = ((0, 16), (17, 32), (33, 48), (49, 64))


def shard_of(discs):
    """Row of the table used for a position with `discs` discs (p_min <= d <= p_max)."""
    for k, (lo, hi) in enumerate(SHARDS):
        if lo <= discs <= hi:
            return k
    raise ValueError(f"disc count {discs} outside 0..64")


def as_weights(w):
    """Validate/convert to a C-contiguous int8 [4, 9] array."""
    a = np.asarray(w)
    if a.shape == (EVAL_WEIGHTS,):
        a = a.reshape(EVAL_PHASES, EVAL_FEATURES)
    if a.shape != (EVAL_PHASES, EVAL_FEATURES):
        raise ValueError(f"weights must have shape ({EVAL_PHASES}, {EVAL_FEATURES}) or ({EVAL_WEIGHTS},)")
    if a.dtype != np.int8:
        if np.any(a < -128) or np.any(a > 127):
            raise ValueError("weights must fit in int8")
        a = a.astype(np.int8)
    return np.ascontiguousarray(a)


def from_learner_params(params):
    """Weights from ``read_parameters()``'s tuple: (header, 36 values)."""
    params = list(params)
    if len(params) != EVAL_WEIGHTS + 1:
        raise ValueError(f"expected header + {EVAL_WEIGHTS} values, got {len(params)}")
    return as_weights([int(x) for x in params[1:]])


def from_coef(coef):
    """The learner's scaling of fitted coefficients to stored parameters
    (progress_position_moves_learn.py:180-181, 200): per shard, coef * 127 /
    max|coef|, then int() (truncation toward zero).  A shard whose coefficients
    are all 0 (the learner would divide by zero) stays 0."""
    coef = np.asarray(coef, np.float64)
    out = np.zeros(coef.shape, np.int8)
    for k, row in enumerate(coef):
        mx = max(abs(float(q)) for q in row)
        if mx > 0:
            out[k] = [int(float(q) * (127 / mx)) for q in row]
    return as_weights(out)


def encode(weights, header=HEADER):
    """paramgen.write_data bytes (paramgen.py:12-19): header, the 36 weights
    as unsigned bytes (conv_num: negative -> 256 + v), trailing 0."""
    w = as_weights(weights).reshape(-1)
    return bytes([header & 0xFF]) + w.view(np.uint8).tobytes() + b"\x00"


def decode(data):
    """Inverse of :func:`encode`: (header, int8 [4, 9])."""
    data = bytes(data)
    if len(data) != EVAL_WEIGHTS + 2:
        raise ValueError(f"paramgen file must be {EVAL_WEIGHTS + 2} bytes, got {len(data)}")
    if data[-1] != 0:
        raise ValueError("paramgen file must end with a 0 byte")
    w = np.frombuffer(data[1:-1], dtype=np.uint8).view(np.int8).reshape(EVAL_PHASES, EVAL_FEATURES)
    return data[0], w.copy()


def write_paramgen(path, weights, header=HEADER):
    with open(path, "wb") as f:
        f.write(encode(weights, header))


def read_paramgen(path):
    with open(path, "rb") as f:
        return decode(f.read())
