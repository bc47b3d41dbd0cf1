"""TD state map on the GPU: oth_td_updates + stable sort +
oth_td_ema must reproduce the learner's float64 values bit-exactly."""
import numpy as np
import pytest
import torch

import oracle
from golden_io import load_npz
from subproc_amd import ops, td

pytestmark = pytest.mark.gpu
DEV = "cuda"


def test_state_map_matches_reference_fixture_and_batches_compose():
    z = load_npz("rollout_random.npz")
    f = load_npz("td_state.npz")
    want = {h: float(v) for h, v in zip(f["hash"].tolist(), f["value"])}
    moves = torch.from_numpy(z["moves"]).to(DEV)
    plies = torch.from_numpy(z["plies"]).to(DEV)
    pos = ops.replay(moves, plies)
    sm = td.StateMap(DEV)
    assert sm.update(pos.boards, plies) == int(2 * (z["plies"].astype(np.int64) + 1).sum())
    assert sm.items() == want
    # the same books in three batches
    sm2 = td.StateMap(DEV)
    for lo, hi in ((0, 1), (1, 100), (100, 256)):
        sm2.update(pos.boards[lo:hi].contiguous(), plies[lo:hi].contiguous())
    assert sm2.items() == want
    # the packed-rows replay (oth_replay_rows + oth_td_updates_rows), and via GameBooks
    sm3 = td.StateMap(DEV)
    pk = ops.replay_rows(moves, plies)
    assert sm3.update(pk.boards, plies, pk.row_off) == int(2 * (z["plies"].astype(np.int64) + 1).sum())
    assert sm3.items() == want
    sm5 = td.StateMap(DEV)  # round 5: offsets from the replay's own row offsets, no host read
    assert sm5.update_rows(pk, plies) == int(2 * (z["plies"].astype(np.int64) + 1).sum())
    assert sm5.items() == want
    from subproc_amd.books import GameBooks
    sm4 = td.StateMap(DEV)
    sm4.update_from_books(GameBooks(moves, plies))
    assert sm4.items() == want
    k = next(iter(want))
    assert sm.get(tuple(int(x) for x in k.split(":"))) == want[k]
    assert sm.get((64, 0, 0, 0, 0, 0, 0, 0, 0, 0)) == 0.0


def test_state_map_at_scale_vs_oracle():
    """4096 random + 1024 greedy games (greedy ones start mid-game-like sequences
    of repeated keys) against the Python restatement over the C oracle."""
    r1 = ops.rollout(4096, 17, 0, "random", record_moves=True, device=DEV)
    r2 = ops.rollout(1024, 18, 0, "greedy", 10, record_moves=True, device=DEV)
    sm = td.StateMap(DEV)
    store = {}
    for r in (r1, r2):
        pos = ops.replay(r.moves, r.plies)
        sm.update(pos.boards, r.plies)
        store = oracle.td_state_map(ops.to_numpy_u64(pos.boards), r.plies.cpu().numpy(), store)
    got = {td.key_to_counts(k): v for k, v in zip(sm.keys.cpu().tolist(), sm.values.cpu().tolist())}
    assert got == store
    assert torch.all(sm.keys[1:] > sm.keys[:-1])  # table stays sorted and unique
    sm2 = td.StateMap(DEV)  # the packed rows (StateMap.update_rows), bit for bit the same table
    for r in (r1, r2):
        sm2.update_rows(ops.replay_rows(r.moves, r.plies), r.plies)
    assert torch.equal(sm2.keys, sm.keys) and torch.equal(sm2.values.view(torch.int64), sm.values.view(torch.int64))


@pytest.mark.parametrize("long_min,spec_warm", [(None, None), (48, None), (1024, None), (48, "1"), (1024, "3")])
def test_td_ema_zero_states_in_long_segments(long_min, spec_warm, monkeypatch):
    """oth_td_ema speculates that no state in a 16-update chunk is exactly 0 and
    redoes the chunk otherwise: plant exact zero states (a = 0.5, x = -v) at
    chunk starts, middles and ends of long segments and compare with the
    sequential rule in Python floats.  With long_min, oth_td_ema_split runs
    the segments at least that long on a whole wave each (LDS stages of 512
    values: lengths around multiples of the stage), those at least 3 warm-ups
    long split into parts over many waves (warm-up 86 at a = 0.5).  A
    warm-up of 1 or 3 values (OTH_TD_SPEC_WARM) makes most guesses miss: the
    rerun passes."""
    from subproc_amd import _lib
    if spec_warm is not None:
        monkeypatch.setenv("OTH_TD_SPEC_WARM", spec_warm)
    a, oma = 0.5, 0.5
    rng = np.random.default_rng(11)
    lengths = [1, 5, 47, 48, 49, 63, 64, 100, 511, 512, 513, 1000, 1023, 1024, 1025, 2048, 4099, 12345]
    vals, seg, want = [], [0], []
    for L in lengths:
        v = 0.0 if L % 2 else 0.25
        init_v = v
        zero_at = set(rng.choice(L, size=min(L, 9), replace=False).tolist()) | {15, 16, 47, 48}
        for k in range(L):
            x = float(rng.normal())
            if k in zero_at and v != 0.0:
                x = -v  # v * 0.5 + (-v) * 0.5 == 0 exactly
            vals.append(x)
            v = x if v == 0.0 else v * oma + x * a
        seg.append(len(vals))
        want.append((init_v, v))
    init = torch.tensor([w[0] for w in want], dtype=torch.float64, device=DEV)
    dv = torch.tensor(vals, dtype=torch.float64, device=DEV)
    ds = torch.tensor(seg, dtype=torch.int64, device=DEV)
    out = torch.empty(len(lengths), dtype=torch.float64, device=DEV)
    lib = _lib.load()
    st = torch.cuda.current_stream().cuda_stream
    if long_min is None:
        _lib.check(lib.oth_td_ema(dv.data_ptr(), ds.data_ptr(), init.data_ptr(), a, oma, out.data_ptr(),
                                  len(lengths), st), "oth_td_ema")
    else:
        li = torch.tensor([i for i, L in enumerate(lengths) if L >= long_min][::-1], dtype=torch.int64, device=DEV)
        td._with_scratch(lib.oth_td_ema_split, (dv.data_ptr(), ds.data_ptr(), init.data_ptr(), a, oma,
                                                out.data_ptr(), len(lengths), long_min, li.data_ptr(), li.numel(),
                                                dv.numel()), st, DEV, "oth_td_ema_split")
    assert out.cpu().tolist() == [w[1] for w in want]


@pytest.mark.parametrize("kind,short", [("normal", False), ("constant", False), ("sparse", False), ("normal", True)])
def test_td_ema_split_speculation_learner_rate(kind, short):
    """Long segments at the learner's rate (a = 0.03, warm-up 1,942 values: 4/3
    of the 2^-64 contraction length) split into parts of 1,040 (600,001 values:
    577 parts over 10 one-wave work items; 5,825 values stay on one lane, 5,826
    are split): the result is the sequential rule's, bit for bit,
    whether the lanes' guesses converge (random targets), sit on a fixed
    point of the rounding (a constant target) or run through exact zeros
    (mostly-zero targets: draws).  short: n_values far below seg_off[n_seg]
    (ADVICE r4), so the scratch holds the parts of the first keys only; the
    keys that do not fit run unsplit, same results, nothing written past it."""
    from subproc_amd import _lib
    a = 0.03
    oma = 1 - a
    rng = np.random.default_rng({"normal": 5, "constant": 6, "sparse": 7}[kind])
    lengths = [5825, 5826, 9000, 70001, 200003, 600001]
    vals, seg, want = [], [0], []
    for L in lengths:
        if kind == "normal":
            xs = rng.normal(size=L) * 0.01
        elif kind == "constant":
            xs = np.full(L, 0.1234567)
        else:
            xs = np.where(rng.random(L) < 0.9, 0.0, rng.normal(size=L))
        v = 0.0
        for x in xs.tolist():
            vals.append(x)
            v = x if v == 0.0 else v * oma + x * a
        seg.append(len(vals))
        want.append(v)
    dv = torch.tensor(vals, dtype=torch.float64, device=DEV)
    ds = torch.tensor(seg, dtype=torch.int64, device=DEV)
    init = torch.zeros(len(lengths), dtype=torch.float64, device=DEV)
    out = torch.empty(len(lengths), dtype=torch.float64, device=DEV)
    li = torch.arange(len(lengths), dtype=torch.int64, device=DEV)
    lib = _lib.load()
    td._with_scratch(lib.oth_td_ema_split, (dv.data_ptr(), ds.data_ptr(), init.data_ptr(), a, oma, out.data_ptr(),
                                            len(lengths), 1024, li.data_ptr(), li.numel(),
                                            10_000 if short else dv.numel()),
                     torch.cuda.current_stream().cuda_stream, DEV, "oth_td_ema_split")
    assert out.cpu().tolist() == want


def test_fit_on_device_matches_sklearn():
    from sklearn import linear_model
    from subproc_amd import params

    r = ops.rollout(8192, 23, 0, "random", record_moves=True, device=DEV)
    sm = td.StateMap(DEV)
    sm.update(ops.replay(r.moves, r.plies).boards, r.plies)
    coef, icpt, n = sm.fit()
    c = td.unpack_counts(sm.keys).cpu().numpy()
    y = sm.values.cpu().numpy()
    for k, (lo, hi) in enumerate(td.SHARDS):
        m = (c[:, 0] >= lo) & (c[:, 0] <= hi)
        assert m.sum() == n[k]
        lr = linear_model.LinearRegression(fit_intercept=True).fit(c[m, 1:].astype(np.float64), y[m])
        np.testing.assert_allclose(coef[k], lr.coef_, rtol=1e-6, atol=1e-9)  # float64 normal equations vs SVD
    w = params.from_coef(coef)
    assert w.dtype == np.int8 and np.abs(w).max() == 127


_EMA_PROBE = r"""
import sys, numpy as np, torch
sys.path.insert(0, sys.argv[1])
from subproc_amd import _lib, td
a, oma = 0.03, 0.97
rng = np.random.default_rng(9)
lengths = [1, 47, 48, 600, 5825, 5826, 9000, 70001]
vals, seg = [], [0]
for L in lengths:
    vals += (rng.normal(size=L) * 0.01).tolist()
    seg.append(len(vals))
dv = torch.tensor(vals, dtype=torch.float64, device="cuda")
ds = torch.tensor(seg, dtype=torch.int64, device="cuda")
init = torch.full((len(lengths),), 0.5, dtype=torch.float64, device="cuda")
out = torch.empty(len(lengths), dtype=torch.float64, device="cuda")
li = torch.tensor([i for i, L in enumerate(lengths) if L >= 48], dtype=torch.int64, device="cuda")
td._with_scratch(_lib.load().oth_td_ema_split, (dv.data_ptr(), ds.data_ptr(), init.data_ptr(), a, oma,
                                                out.data_ptr(), len(lengths), 48, li.data_ptr(), li.numel(),
                                                dv.numel()), torch.cuda.current_stream().cuda_stream, "cuda", "ema")
want = []
for k, L in enumerate(lengths):
    v = 0.5
    for x in vals[seg[k]:seg[k + 1]]:
        v = x if v == 0.0 else v * oma + x * a
    want.append(v)
assert out.cpu().tolist() == want, "EMA differs"
print("ok")
"""


@pytest.mark.parametrize("env", [{"OTH_TD_EMA_FORK": "1"}, {"OTH_TD_EMA_MERGED": "0"}, {}])
def test_td_ema_split_launch_variants(env):
    """oth_td_ema_split's launch schedules, each read once per process from the
    environment, in a child process: the side-stream fork (OTH_TD_EMA_FORK=1,
    opt-in), the long keys and split-key parts as separate launches
    (OTH_TD_EMA_MERGED=0), and the default (one launch for both).  Short,
    long, unsplit-long and split keys in one call, bit for bit the sequential
    rule at the learner's rate."""
    import os
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    r = subprocess.run([sys.executable, "-c", _EMA_PROBE, root], env={**os.environ, **env}, capture_output=True,
                       text=True, timeout=110)
    assert r.returncode == 0 and r.stdout.strip().endswith("ok"), r.stdout + r.stderr
