"""Tensor-level batched Othello ops on the MI355X (one call = one HIP launch).

Every function takes/returns torch tensors resident on a ROCm device and calls
the C-ABI of include/othello.h on torch's current stream.  Bitboards are
``(n, 2)`` ``torch.int64`` tensors holding the uint64 bit patterns
``[black, white]`` (torch has no general uint64 arithmetic; the bits are what
matter, see :func:`to_numpy_u64`).  There is no CPU fallback: CPU tensors or a
missing library raise.

Reference mapping (board.py line numbers):
  reset   -> Board.__init__            22-27
  legal   -> Board.puttables           46-52   (n_puttable_for = popcount)
  step    -> Board.put_s / put         161-209
  result  -> n_black / n_white / is_game_over 37-58 + game_runner.py:194-199
  hands   -> Board.hands_for_direc     124-139 (any origin, all 8 directions)
  rollout -> GameRunner.play_a_game loop   game_runner.py:165-201
  evaluate -> linear eval of the learner's counts() features
"""
import ctypes
from collections import namedtuple

import numpy as np
import torch

from . import _lib
from ._lib import (BLACK, BOOK_LINE, HIST_BINS, MOVES_STRIDE, N_FEATURES, PASS, POLICY_EVAL, POLICY_GREEDY,
                   POLICY_RANDOM, POS_STRIDE, WHITE, check)
from .params import DEFAULT_WEIGHTS, as_weights

StepResult = namedtuple("StepResult", "boards turn flips legal_next ret")
Result = namedtuple("Result", "n_black n_white diff terminal")
RolloutResult = namedtuple("RolloutResult", "final_boards diff plies moves hist")
Positions = namedtuple("Positions", "boards turn nturn move")
Replay = namedtuple("Replay", "boards turn end")
ReplayRows = namedtuple("ReplayRows", "boards turn end row_off")

_POLICIES = {"random": POLICY_RANDOM, "greedy": POLICY_GREEDY, "eval": POLICY_EVAL, POLICY_RANDOM: POLICY_RANDOM,
             POLICY_GREEDY: POLICY_GREEDY, POLICY_EVAL: POLICY_EVAL}


def _weights_ptr(weights):
    """Host int8[36] buffer for oth_eval / oth_rollout_eval (copied into the launch)."""
    w = as_weights(DEFAULT_WEIGHTS if weights is None else weights)
    return (ctypes.c_int8 * w.size).from_buffer_copy(w.tobytes())


def _stream():
    return ctypes_stream(torch.cuda.current_stream())


def ctypes_stream(s):
    return s.cuda_stream  # hipStream_t as an integer handle


def _dev(t, name, dtype, shape=None, device=None):
    if not isinstance(t, torch.Tensor):
        raise TypeError(f"{name}: expected a torch.Tensor")
    if t.device.type != "cuda":
        raise ValueError(f"{name}: tensor must be on a ROCm device (got {t.device}); there is no CPU path")
    if device is not None and t.device != device:
        raise ValueError(f"{name}: tensor is on {t.device}, expected {device} (all arguments on one device)")
    if t.dtype != dtype:
        raise TypeError(f"{name}: expected dtype {dtype}, got {t.dtype}")
    if not t.is_contiguous():
        raise ValueError(f"{name}: tensor must be contiguous")
    if shape is not None and tuple(t.shape) != tuple(shape):
        raise ValueError(f"{name}: expected shape {tuple(shape)}, got {tuple(t.shape)}")
    return t.data_ptr()


def _opt(t, name, dtype, shape, device=None):
    return None if t is None else _dev(t, name, dtype, shape, device)


def _n(boards):
    if boards.dim() != 2 or boards.shape[1] != 2:
        raise ValueError(f"boards: expected shape (n, 2), got {tuple(boards.shape)}")
    return boards.shape[0]


def _device(device):
    d = torch.device(device)
    if d.type != "cuda":
        raise ValueError(f"device must be a ROCm device, got {d}")
    if d.index is None:  # "cuda" -> the current device, so it compares equal to tensors' devices
        d = torch.device("cuda", torch.cuda.current_device())
    return d


# ---------------------------------------------------------------------------
def reset(n, device="cuda"):
    """n games at the opening position: (boards (n,2) int64, turn (n,) uint8, nturn (n,) uint8)."""
    d = _device(device)
    boards = torch.empty((n, 2), dtype=torch.int64, device=d)
    turn = torch.empty(n, dtype=torch.uint8, device=d)
    nturn = torch.empty(n, dtype=torch.uint8, device=d)
    with torch.cuda.device(d):
        check(_lib.load().oth_reset(boards.data_ptr(), turn.data_ptr(), nturn.data_ptr(), n, _stream()), "oth_reset")
    return boards, turn, nturn


def legal(boards, turn, out=None):
    """Legal-move bitboard of the side to move (Board.puttables as a mask)."""
    n = _n(boards)
    pb = _dev(boards, "boards", torch.int64)
    pt = _dev(turn, "turn", torch.uint8, (n,), boards.device)
    if out is None:
        out = torch.empty(n, dtype=torch.int64, device=boards.device)
    po = _dev(out, "out", torch.int64, (n,), boards.device)
    with torch.cuda.device(boards.device):
        check(_lib.load().oth_legal(pb, pt, po, n, _stream()), "oth_legal")
    return out


def step(boards, turn, move, nturn=None, inplace=False, want_flips=True, want_legal=True):
    """One Board.put_s per game on integer move codes (0..63 square, 64 pass).

    Returns StepResult(boards, turn, flips, legal_next, ret) with ret exactly as
    board.py: -1 illegal (state unchanged), 0 pass, n >= 1 discs flipped.
    ``nturn`` (uint8, optional) is incremented in place where ret >= 0.
    ``inplace=True`` writes the new boards/turn into the input tensors.
    """
    n = _n(boards)
    pb = _dev(boards, "boards", torch.int64)
    pt = _dev(turn, "turn", torch.uint8, (n,), boards.device)
    pm = _dev(move, "move", torch.uint8, (n,), boards.device)
    pn = _opt(nturn, "nturn", torch.uint8, (n,), boards.device)
    dev = boards.device
    bo = boards if inplace else torch.empty_like(boards)
    to = turn if inplace else torch.empty_like(turn)
    fl = torch.empty(n, dtype=torch.int64, device=dev) if want_flips else None
    ln = torch.empty(n, dtype=torch.int64, device=dev) if want_legal else None
    ret = torch.empty(n, dtype=torch.int8, device=dev)
    with torch.cuda.device(dev):
        check(_lib.load().oth_step(pb, pt, pm, bo.data_ptr(), to.data_ptr(), None if fl is None else fl.data_ptr(),
                                   None if ln is None else ln.data_ptr(), ret.data_ptr(), pn, n, _stream()),
              "oth_step")
    return StepResult(bo, to, fl, ln, ret)


def result(boards):
    """Result(n_black, n_white, diff = n_black - n_white, terminal = is_game_over())."""
    n = _n(boards)
    pb = _dev(boards, "boards", torch.int64)
    dev = boards.device
    nb = torch.empty(n, dtype=torch.uint8, device=dev)
    nw = torch.empty(n, dtype=torch.uint8, device=dev)
    df = torch.empty(n, dtype=torch.int8, device=dev)
    te = torch.empty(n, dtype=torch.uint8, device=dev)
    with torch.cuda.device(dev):
        check(_lib.load().oth_result(pb, nb.data_ptr(), nw.data_ptr(), df.data_ptr(), te.data_ptr(), n, _stream()),
              "oth_result")
    return Result(nb, nw, df, te)


def hands(own, hostile, x, y, dx, dy):
    """len(Board.hands_for_direc((dx, dy), piece, x, y)) (board.py:124-139) per
    item, for any origin and direction (int64: off-board origins included);
    own[i] / hostile[i] = squares holding the piece / hostile(piece).  The
    returned squares are (x + k*dx, y + k*dy), k = 1..count: (n,) uint8."""
    n = own.shape[0]
    po = _dev(own, "own", torch.int64, (n,))
    ph = _dev(hostile, "hostile", torch.int64, (n,), own.device)
    pc = [_dev(v, nm, torch.int64, (n,), own.device) for v, nm in ((x, "x"), (y, "y"), (dx, "dx"), (dy, "dy"))]
    out = torch.empty(n, dtype=torch.uint8, device=own.device)
    with torch.cuda.device(own.device):
        check(_lib.load().oth_hands(po, ph, *pc, out.data_ptr(), n, _stream()), "oth_hands")
    return out


_WORK = {}


def work_word(device=None):
    """The rollout work word of torch's current stream on `device` (one zeroed
    device uint64 per (device, stream), include/othello.h oth_rollout): a
    launch finds it at 0 and leaves it at 0, so launches ordered on one stream
    share it and launches on different streams never do."""
    d = _device("cuda" if device is None else device)
    with torch.cuda.device(d):
        key = (d.index, torch.cuda.current_stream().cuda_stream)
        w = _WORK.get(key)
        if w is None:
            w = torch.zeros(1, dtype=torch.int64, device=d)  # zeroed on this stream, before any launch on it
            _WORK[key] = w
    return w


def rollout(n, seed, game_id0=0, policy="random", n_random=10, start=None, start_turn=None, record_moves=False,
            hist=None, device="cuda", want_boards=True, want_diff=True, want_plies=True, weights=None,
            weights_white=None, work=None):
    """Play n games to terminal on the GPU (one lane per game).

    Game i uses the RNG stream of global id game_id0 + i, so results do not
    depend on how games are split over launches or GPUs.  ``hist`` (int64[133])
    is accumulated into if given (zero it yourself), else a fresh zeroed one is
    returned: [0..128] diff+64, 129 black wins, 130 white wins, 131 draws,
    132 total plies (= env-steps).

    Policies: "random"; "greedy" (minimise the opponent's mobility) and "eval"
    (maximise the mover's linear eval under ``weights``, int8 [4, 9], default
    params.DEFAULT_WEIGHTS) after ``n_random`` random plies.  With
    ``weights_white`` the eval policy is a match: Black plays ``weights``,
    White plays ``weights_white`` (oth_rollout_match).

    ``work`` (int64 (1,) device tensor, 0 at the launch) is the launch's batch
    counter; default: the current stream's :func:`work_word`.  Under graph
    capture ``work`` is required: a replay runs on the replaying stream, so
    every captured launch needs a word of its own, zeroed before the capture
    (graphs replayed concurrently must not share one).
    """
    if policy not in _POLICIES:
        raise ValueError(f"policy must be 'random', 'greedy' or 'eval', got {policy!r}")
    capturing = torch.cuda.is_current_stream_capturing()
    if work is None and capturing:
        raise RuntimeError("ops.rollout under graph capture needs an explicit work word: an int64 (1,) device "
                           "tensor zeroed before the capture, one per captured launch")
    d = _device(device) if start is None else start.device
    ps = pst = None
    if start is not None:
        if _n(start) != n:
            raise ValueError("start must have n rows")
        ps = _dev(start, "start", torch.int64)
        pst = _opt(start_turn, "start_turn", torch.uint8, (n,), start.device)
    fb = torch.empty((n, 2), dtype=torch.int64, device=d) if want_boards else None
    df = torch.empty(n, dtype=torch.int8, device=d) if want_diff else None
    pl = torch.empty(n, dtype=torch.uint8, device=d) if want_plies else None
    mv = torch.empty((n, MOVES_STRIDE), dtype=torch.uint8, device=d) if record_moves else None
    if hist is None:
        hist = torch.zeros(HIST_BINS, dtype=torch.int64, device=d)
    ph = _dev(hist, "hist", torch.int64, (HIST_BINS,), d)
    if _POLICIES[policy] != POLICY_EVAL and (weights is not None or weights_white is not None):
        raise ValueError("weights apply to policy 'eval' only")
    w = work_word(d) if work is None else work
    pw = _dev(w, "work", torch.int64, (1,), d)

    def ptr(t):
        return None if t is None else t.data_ptr()

    with torch.cuda.device(d):
        seed64 = seed & (2**64 - 1)
        if _POLICIES[policy] == POLICY_EVAL and weights_white is not None:
            rc, what = _lib.load().oth_rollout_match(ps, pst, seed64, game_id0, n_random, _weights_ptr(weights),
                                                     _weights_ptr(weights_white), ptr(fb), ptr(df), ptr(pl), ptr(mv),
                                                     ph, pw, n, _stream()), "oth_rollout_match"
        elif _POLICIES[policy] == POLICY_EVAL:
            rc, what = _lib.load().oth_rollout_eval(ps, pst, seed64, game_id0, n_random, _weights_ptr(weights),
                                                    ptr(fb), ptr(df), ptr(pl), ptr(mv), ph, pw, n,
                                                    _stream()), "oth_rollout_eval"
        else:
            rc, what = _lib.load().oth_rollout(ps, pst, seed64, game_id0, _POLICIES[policy], n_random, ptr(fb),
                                               ptr(df), ptr(pl), ptr(mv), ph, pw, n, _stream()), "oth_rollout"
        if rc != _lib.OTH_OK:
            # a failed launch leaves the counter unknown (include/othello.h): the
            # stream's default word is dropped (the next call makes a fresh zeroed
            # one); a caller's word is reset eagerly, never as a captured node
            if work is None:
                _WORK.pop((d.index, torch.cuda.current_stream().cuda_stream), None)
            elif not capturing:
                w.zero_()
        check(rc, what)
    return RolloutResult(fb, df, pl, mv, hist)


_SIDE = {}


def _side_streams(d, k):
    """k side streams of device d, created once and reused (rollout_batches)."""
    have = _SIDE.setdefault(d.index, [])
    while len(have) < k:
        have.append(torch.cuda.Stream(d))
    return have[:k]


ROLLOUT_MERGE_GAMES = 1 << 24  # rollout_batches merges batches into launches of up to this many games


def rollout_batches(n, steps, seed, game_id0=0, policy="random", n_random=10, hist=None, device="cuda", streams=2,
                    want_boards=False, want_diff=False, want_plies=False, weights=None, merge=True):
    """`steps` batches of `n` games each, pipelined: batch s plays global ids
    [game_id0 + s*n, +n).  Consecutive batches are merged into launches of up
    to max(n, ROLLOUT_MERGE_GAMES) games (merge=False: one launch per batch),
    and the launches are issued round-robin on `streams` HIP streams (torch's
    current stream and streams - 1 side streams, each with its own work
    word), so the last batches of one launch share the CUs with the first
    batches of the next instead of leaving them idle (batch
    tail): ten batches of 1M games run as one launch of 10M, with one launch
    tail where ten launches had ten.  The result equals ``rollout(n * steps, seed, game_id0,
    ...)`` game for game whatever the launches: every game keeps the RNG
    stream of its global id, and the launches add into one histogram (device
    atomics).  Outputs, if asked for, are (n * steps, ...) in game-id order.
    On return the current stream is ordered after every launch; nothing is
    synchronised with the host.
    """
    if policy not in _POLICIES:
        raise ValueError(f"policy must be 'random', 'greedy' or 'eval', got {policy!r}")
    if steps < 1 or n < 0 or streams < 1:
        raise ValueError("rollout_batches: steps >= 1, n >= 0 and streams >= 1")
    if torch.cuda.is_current_stream_capturing():
        raise RuntimeError("rollout_batches issues on side streams: capture ops.rollout launches instead")
    d = _device(device)
    pid = _POLICIES[policy]
    if pid != POLICY_EVAL and weights is not None:
        raise ValueError("weights apply to policy 'eval' only")
    total = n * steps
    fb = torch.empty((total, 2), dtype=torch.int64, device=d) if want_boards else None
    df = torch.empty(total, dtype=torch.int8, device=d) if want_diff else None
    pl = torch.empty(total, dtype=torch.uint8, device=d) if want_plies else None
    if hist is None:
        hist = torch.zeros(HIST_BINS, dtype=torch.int64, device=d)
    ph = _dev(hist, "hist", torch.int64, (HIST_BINS,), d)
    lib = _lib.load()
    wp = _weights_ptr(weights) if pid == POLICY_EVAL else None
    with torch.cuda.device(d):
        main = torch.cuda.current_stream()
        side = _side_streams(d, streams - 1)
        sts = [main] + side
        fork = torch.cuda.Event()
        fork.record(main)
        for st in side:
            st.wait_event(fork)
        # one work word per stream (0 before and after each launch on it): the
        # streams' cached words, as ops.rollout uses them
        works = []
        for st in sts:
            with torch.cuda.stream(st):
                works.append(work_word(d))
        per = 1  # batches per launch
        if merge and n > 0:
            per = max(1, min(steps, ROLLOUT_MERGE_GAMES // n))
        for L, s0 in enumerate(range(0, steps, per)):
            i = L % len(sts)
            st, w = sts[i], works[i]
            g0 = game_id0 + s0 * n
            m = min(per, steps - s0) * n  # this launch's games

            def part(t, k=1):
                return None if t is None else t.data_ptr() + s0 * n * k * t.element_size()

            if pid == POLICY_EVAL:
                rc = lib.oth_rollout_eval(None, None, seed & (2**64 - 1), g0, n_random, wp, part(fb, 2), part(df),
                                          part(pl), None, ph, w.data_ptr(), m, st.cuda_stream)
            else:
                rc = lib.oth_rollout(None, None, seed & (2**64 - 1), g0, pid, n_random, part(fb, 2), part(df),
                                     part(pl), None, ph, w.data_ptr(), m, st.cuda_stream)
            if rc != _lib.OTH_OK:  # the failed launch's word is unknown: drop it (ops.rollout does the same)
                _WORK.pop((d.index, st.cuda_stream), None)
            check(rc, "oth_rollout (rollout_batches launch %d)" % L)
        for st in side:  # the caller's stream waits for every launch
            e = torch.cuda.Event()
            e.record(st)
            main.wait_event(e)
        for t in (fb, df, pl, hist):
            if t is not None:
                for st in side:
                    t.record_stream(st)
    return RolloutResult(fb, df, pl, None, hist)


RunnerResult = namedtuple("RunnerResult", "final_boards diff plies moves hist a_black")


def rollout_runner(n, seed, game_id0=0, policy="eval", weights_a=None, weights_b=None, n_rand_a=0, n_rand_b=0,
                   swap_colours=False, start=None, start_turn=None, record_moves=False, hist=None, device="cuda",
                   work=None):
    """n GameRunner matches between player A and player B on the GPU
    (oth_rollout_runner, include/othello.h): both play ``policy`` ("greedy",
    or "eval" with tables ``weights_a`` / ``weights_b``, default
    params.DEFAULT_WEIGHTS), each places min(n_rand, 10) random moves by
    go_for's coin (game_runner.py:115-150), and with ``swap_colours`` each game
    draws who plays Black (subproc.do_match's proc_randomize_black_white).
    Game i is global id game_id0 + i.  ``a_black`` (n,) uint8: 1 where A
    played Black; diff / hist / final boards are by colour."""
    if policy not in ("greedy", "eval"):
        raise ValueError(f"policy must be 'greedy' or 'eval', got {policy!r}")
    if work is None and torch.cuda.is_current_stream_capturing():
        raise RuntimeError("ops.rollout_runner under graph capture needs an explicit work word")
    d = _device(device) if start is None else start.device
    ps = pst = None
    if start is not None:
        if _n(start) != n:
            raise ValueError("start must have n rows")
        ps = _dev(start, "start", torch.int64)
        pst = _opt(start_turn, "start_turn", torch.uint8, (n,), start.device)
    fb = torch.empty((n, 2), dtype=torch.int64, device=d)
    df = torch.empty(n, dtype=torch.int8, device=d)
    pl = torch.empty(n, dtype=torch.uint8, device=d)
    ab = torch.empty(n, dtype=torch.uint8, device=d)
    mv = torch.empty((n, MOVES_STRIDE), dtype=torch.uint8, device=d) if record_moves else None
    if hist is None:
        hist = torch.zeros(HIST_BINS, dtype=torch.int64, device=d)
    ph = _dev(hist, "hist", torch.int64, (HIST_BINS,), d)
    w = work_word(d) if work is None else work
    pw = _dev(w, "work", torch.int64, (1,), d)
    with torch.cuda.device(d):
        rc = _lib.load().oth_rollout_runner(ps, pst, seed & (2**64 - 1), game_id0, _POLICIES[policy],
                                            _weights_ptr(weights_a), _weights_ptr(weights_b), int(n_rand_a),
                                            int(n_rand_b), int(bool(swap_colours)), ab.data_ptr(), fb.data_ptr(),
                                            df.data_ptr(), pl.data_ptr(), None if mv is None else mv.data_ptr(), ph,
                                            pw, n, _stream())
        if rc != _lib.OTH_OK:  # as ops.rollout: drop the stream's default word, reset a caller's eagerly
            if work is None:
                _WORK.pop((d.index, torch.cuda.current_stream().cuda_stream), None)
            elif not torch.cuda.is_current_stream_capturing():
                w.zero_()
        check(rc, "oth_rollout_runner")
    return RunnerResult(fb, df, pl, mv, hist, ab)


def sample_midgame(n, seed, index0=0, device="cuda"):
    """Synthetic reachable mid-game positions + one random legal move each (config 2 inputs)."""
    d = _device(device)
    b = torch.empty((n, 2), dtype=torch.int64, device=d)
    t = torch.empty(n, dtype=torch.uint8, device=d)
    nt = torch.empty(n, dtype=torch.uint8, device=d)
    m = torch.empty(n, dtype=torch.uint8, device=d)
    with torch.cuda.device(d):
        check(_lib.load().oth_sample_midgame(seed & (2**64 - 1), index0, b.data_ptr(), t.data_ptr(), nt.data_ptr(),
                                             m.data_ptr(), n, _stream()), "oth_sample_midgame")
    return Positions(b, t, nt, m)


def replay(moves, plies, start=None, start_turn=None):
    """Every recorded position of n games (GameRunner records the board after
    Board() and after each put_s, game_runner.py:169-184).  Returns Replay with
    boards (n, 129, 2) int64, turn (n, 129) uint8, end (n, 129) uint8 =
    is_game_over(); game i's positions are rows 0..plies[i] (later rows: boards 0,
    turn 0, end 0)."""
    n = moves.shape[0]
    pm = _dev(moves, "moves", torch.uint8, (n, MOVES_STRIDE))
    pp = _dev(plies, "plies", torch.uint8, (n,), moves.device)
    ps = _opt(start, "start", torch.int64, (n, 2), moves.device)
    pst = _opt(start_turn, "start_turn", torch.uint8, (n,), moves.device)
    dev = moves.device
    # every row is written by the kernel (rows past plies as 0): no fill pass
    b = torch.empty((n, POS_STRIDE, 2), dtype=torch.int64, device=dev)
    t = torch.empty((n, POS_STRIDE), dtype=torch.uint8, device=dev)
    e = torch.empty((n, POS_STRIDE), dtype=torch.uint8, device=dev)
    with torch.cuda.device(dev):
        check(_lib.load().oth_replay(ps, pst, pm, pp, b.data_ptr(), t.data_ptr(), e.data_ptr(), n, _stream()),
              "oth_replay")
    return Replay(b, t, e)


def row_offsets(plies):
    """Exclusive prefix sum of min(plies, 128) + 1 (int64, on plies' device):
    the first row of each game in an oth_replay_rows table; also returns the
    total row count (one host sync)."""
    cnt = plies.long().clamp(max=MOVES_STRIDE) + 1
    ends = torch.cumsum(cnt, 0)
    total = int(ends[-1]) if ends.numel() else 0
    return (ends - cnt).contiguous(), total


def replay_rows(moves, plies, start=None, start_turn=None):
    """ops.replay into packed rows (oth_replay_rows): game i's recorded
    positions are rows row_off[i] .. row_off[i] + plies[i] of boards (R, 2)
    int64, turn (R,) and end (R,) uint8, R = sum(plies + 1) -- only the rows
    GameRunner records, about half of the strided table of random games."""
    n = moves.shape[0]
    pm = _dev(moves, "moves", torch.uint8, (n, MOVES_STRIDE))
    pp = _dev(plies, "plies", torch.uint8, (n,), moves.device)
    ps = _opt(start, "start", torch.int64, (n, 2), moves.device)
    pst = _opt(start_turn, "start_turn", torch.uint8, (n,), moves.device)
    dev = moves.device
    row_off, total = row_offsets(plies)
    b = torch.empty((total, 2), dtype=torch.int64, device=dev)
    t = torch.empty(total, dtype=torch.uint8, device=dev)
    e = torch.empty(total, dtype=torch.uint8, device=dev)
    with torch.cuda.device(dev):
        check(_lib.load().oth_replay_rows(ps, pst, pm, pp, row_off.data_ptr(), b.data_ptr(), t.data_ptr(),
                                          e.data_ptr(), n, _stream()), "oth_replay_rows")
    return ReplayRows(b, t, e, row_off)


def book_text(boards, turn):
    """serialize_str() + newline of each position (board.py:214-243), concatenated:
    a uint8 tensor of n * 67 bytes on the device."""
    n = _n(boards)
    pb = _dev(boards, "boards", torch.int64)
    pt = _dev(turn, "turn", torch.uint8, (n,), boards.device)
    out = torch.empty(n * BOOK_LINE, dtype=torch.uint8, device=boards.device)
    with torch.cuda.device(boards.device):
        check(_lib.load().oth_book_text(pb, pt, n, out.data_ptr(), _stream()), "oth_book_text")
    return out


def book_parse(text, n, stride=64, want_turn=False):
    """Board strings back into bitboards (oth_book_parse): ``text`` a uint8
    device tensor holding n strings of 64 chars at a stride of ``stride``
    bytes (64 packed; 67 = OTH_BOOK_LINE for serialize_str lines).  Returns
    (boards (n, 2) int64, turn (n,) uint8 or None); ``want_turn`` parses the
    side after each board's space (needs stride >= 66)."""
    if not isinstance(text, torch.Tensor) or text.dtype != torch.uint8 or text.dim() != 1:
        raise TypeError("text: expected a 1-D uint8 tensor")
    if stride < 64 or (want_turn and stride < 66):
        raise ValueError("stride must be >= 64 (>= 66 to parse the side)")
    if n < 0 or (n > 0 and text.numel() < (n - 1) * stride + (66 if want_turn else 64)):
        raise ValueError(f"text holds fewer than {n} strings at stride {stride}")
    pt = _dev(text, "text", torch.uint8)
    dev = text.device
    b = torch.empty((n, 2), dtype=torch.int64, device=dev)
    t = torch.empty(n, dtype=torch.uint8, device=dev) if want_turn else None
    with torch.cuda.device(dev):
        check(_lib.load().oth_book_parse(pt, stride, b.data_ptr(), None if t is None else t.data_ptr(), n, _stream()),
              "oth_book_parse")
    return b, t


def features(boards, side):
    """counts() of parameter_progress_position_moves_learn.py:5-17 per position
    for side 1 ('O' = Black) / 2 ('X' = White): (n, 10) uint8 =
    (64 - n_empty, n_puttable_for(side), 8 region mask_counts)."""
    n = _n(boards)
    pb = _dev(boards, "boards", torch.int64)
    ps = _dev(side, "side", torch.uint8, (n,), boards.device)
    out = torch.empty((n, N_FEATURES), dtype=torch.uint8, device=boards.device)
    with torch.cuda.device(boards.device):
        check(_lib.load().oth_features(pb, ps, out.data_ptr(), n, _stream()), "oth_features")
    return out


def evaluate(boards, side, weights=None):
    """Linear eval of each position from side 1 ('O') / 2 ('X')'s view: int32
    (n,) = sum_j W[shard(discs)][j] * counts()[1+j] (include/othello.h oth_eval;
    the model progress_position_moves_learn.py:160-184 fits)."""
    n = _n(boards)
    pb = _dev(boards, "boards", torch.int64)
    ps = _dev(side, "side", torch.uint8, (n,), boards.device)
    out = torch.empty(n, dtype=torch.int32, device=boards.device)
    with torch.cuda.device(boards.device):
        check(_lib.load().oth_eval(pb, ps, _weights_ptr(weights), out.data_ptr(), n, _stream()), "oth_eval")
    return out


# ---------------------------------------------------------------------------
# host <-> device conversion helpers (uint64 bit patterns)
# ---------------------------------------------------------------------------
def to_numpy_u64(t):
    """Device/host int64 tensor -> numpy uint64 array with the same bits."""
    return t.detach().cpu().numpy().view(np.uint64)


def from_numpy_u64(a, device="cuda"):
    """numpy uint64 array -> int64 tensor with the same bits on `device`."""
    a = np.ascontiguousarray(a, dtype=np.uint64)
    return torch.from_numpy(a.view(np.int64).copy()).to(device)


__all__ = ["reset", "legal", "step", "result", "hands", "rollout", "work_word", "sample_midgame", "replay",
           "book_text", "features", "evaluate", "to_numpy_u64", "from_numpy_u64",
           "StepResult", "Result", "RolloutResult", "Positions", "Replay", "BLACK", "WHITE", "PASS", "HIST_BINS"]
