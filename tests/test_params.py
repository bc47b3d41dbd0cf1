"""Eval weights and the paramgen file format (host logic, CPU)."""
import numpy as np
import pytest

from golden_io import load_npz
from subproc_amd import params


def test_default_weights_are_the_reference_default_value():
    # eval_values.npz holds ProgressPositionMovesParameter().default_value() as
    # gen_golden.py read it from the reference module
    np.testing.assert_array_equal(params.DEFAULT_WEIGHTS, load_npz("eval_values.npz")["weights_default"])


def test_paramgen_round_trip_and_layout():
    w = load_npz("eval_values.npz")["weights_rand"]
    data = params.encode(w)
    # paramgen.write_data: header, conv_num(v) = 256 + v for v < 0, trailing 0
    assert len(data) == 38 and data[0] == 2 and data[-1] == 0
    assert list(data[1:-1]) == [v + 256 if v < 0 else v for v in w.reshape(-1).tolist()]
    header, back = params.decode(data)
    assert header == 2
    np.testing.assert_array_equal(back, w)


def test_paramgen_file(tmp_path):
    path = tmp_path / "param.bin"
    params.write_paramgen(path, params.DEFAULT_WEIGHTS)
    header, w = params.read_paramgen(path)
    assert header == params.HEADER
    np.testing.assert_array_equal(w, params.DEFAULT_WEIGHTS)


def test_from_learner_params():
    # read_parameters() returns (header, 36 ints) (progress_position_moves_learn.py:211-224)
    flat = [2] + params.DEFAULT_WEIGHTS.reshape(-1).tolist()
    np.testing.assert_array_equal(params.from_learner_params(flat), params.DEFAULT_WEIGHTS)
    with pytest.raises(ValueError):
        params.from_learner_params(flat[:-1])


def test_shards_and_validation():
    assert [params.shard_of(d) for d in (0, 16, 17, 32, 33, 48, 49, 64)] == [0, 0, 1, 1, 2, 2, 3, 3]
    with pytest.raises(ValueError):
        params.shard_of(65)
    with pytest.raises(ValueError):
        params.as_weights(np.zeros((3, 9)))
    with pytest.raises(ValueError):
        params.as_weights(np.full((4, 9), 200))
    with pytest.raises(ValueError):
        params.decode(b"\x02" + bytes(36) + b"\x01")


def test_from_coef_is_the_learners_scaling():
    coef = np.array([[0.5, -2.0, 0.25, 0.0, 1.0, -1.0, 0.125, 1.999, -0.001],
                     [0.0] * 9,
                     [3.0, 1.5, -3.0, 0.3, 0.1, 2.9, -2.9, 1.0, 0.01],
                     [1e-3, 2e-3, -4e-3, 0, 0, 0, 0, 0, 1e-3]])
    got = params.from_coef(coef)
    for k, row in enumerate(coef):
        mx = max(abs(q) for q in row)
        want = [int(q * (127 / mx)) for q in row] if mx else [0] * 9  # coef = 127/max|coef|; int(i*coef)
        assert got[k].tolist() == want
    assert got[0][1] == -127 and got[2][0] == 127
