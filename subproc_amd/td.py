"""TD state map of the progress/position/moves learner on the GPU.

ProgressPositionMovesLearn keeps, per ``counts()`` hash, an exponentially
averaged TD target in the parameter store, one Redis round trip per position and
side (progress_position_moves_learn.py:37-62):

    for book in books:                    # learn_books order; each book terminal-first
        last_turn, v_O = terminal nturn, n_black - n_white (v_X = -v_O)
        for record in book:               # terminal -> opening
            for side, value in (('O', v_O), ('X', v_X)):
                new = value * l ** (last_turn - turn)
                v[key] = new if v[key] == 0 else v[key] * (1 - a) + new * a

Here the whole batch runs on the device:
  1. ``oth_td_updates_packed`` (HIP) emits the ordered update stream from an
     ``oth_replay`` / ``oth_replay_rows`` position table, one uint64 word per
     (position, side): the packed counts() key, the terminal's disc
     difference and the turns left, from which the value is recomputed
     exactly (``oth_td_unpack``);
  2. ``oth_td_sort_packed`` (rocPRIM keys-only radix sort over the words' 43
     key bits) sorts them by key, stably: each key's updates stay in stream
     order (books read from records take ``oth_td_updates_records`` and the
     (key, value) pair sort ``oth_td_sort_pairs``);
  3. ``oth_td_ema_split`` (HIP) replays each key's updates in order in
     float64 with separate multiply and add, so every value is bit-identical
     to the Python learner's (a key with at least LONG_MIN updates gets a
     whole wavefront; the longest are split over its lanes from verified
     warm-up guesses);
  4. ``oth_td_lookup`` (before 3: each key's state before the batch) and
     ``oth_td_merge`` (after it: the results into the device-resident,
     key-sorted table) are HIP merge paths over the table and the batch's
     keys.
Batches applied one after another equal one batch of all their books.
Values are kept as float64 (the Python learner's float, before any store
round trip).  ``StateMap.fit`` runs the learner's regression step
(fit_parameter, progress_position_moves_learn.py:160-184) over every state of
a shard on the device instead of a random 50,000-state sample; Redis and the
pyres fan-out stay out of scope.
"""
import ctypes
import os

import numpy as np
import torch

from . import _lib
from ._lib import POS_STRIDE, check
from .params import SHARDS

A = 0.03       # ProgressPositionMovesLearn.a  (progress_position_moves_learn.py:22)
LAMBDA = 0.90  # ProgressPositionMovesLearn.l  (progress_position_moves_learn.py:24)
# the lookup queued ahead of the host's read of the segment counts (round 5);
# OTH_TD_LOOKUP_AHEAD=0 reads them first (tools/diag A/Bs only)
_LOOKUP_AHEAD = os.environ.get("OTH_TD_LOOKUP_AHEAD", "1") != "0"
# the merge reads the lookup's merge-path splits (round 5); OTH_TD_MERGE_SPLITS=0
# searches again (oth_td_merge; A/Bs only)
_MERGE_SPLITS_FROM_LOOKUP = os.environ.get("OTH_TD_MERGE_SPLITS", "1") != "0"
LONG_MIN = 48  # updates per key from which oth_td_ema_split runs the key on a whole wave
# include/othello.h OTH_TD_KEY layout: each field as wide as its largest value
# (discs 0..64, moves 0..63, region counts up to the region sizes 4, 8, 4, 8,
# 8, 16, 4, 12)
_SHIFTS = (36, 30, 27, 23, 20, 16, 12, 7, 4, 0)
_WIDTH = (7, 6, 3, 4, 3, 4, 4, 5, 3, 4)


def lam_pow_table(lam=LAMBDA):
    """l ** k for k = 0..128 as CPython computes it (the learner's own pow)."""
    return [lam ** k for k in range(POS_STRIDE)]


def counts_to_key(c):
    """Pack a counts() 10-tuple (include/othello.h OTH_TD_KEY_BITS layout)."""
    k = 0
    for v, s, w in zip(c, _SHIFTS, _WIDTH):
        if not 0 <= int(v) < (1 << w):
            raise ValueError(f"counts value {v} out of range")
        k |= int(v) << s
    return k


def key_to_counts(k):
    k = int(k)
    return tuple((k >> s) & ((1 << w) - 1) for s, w in zip(_SHIFTS, _WIDTH))


# include/othello.h OTH_TD_SKEY (the packed words' 36-bit sort key): (discs,
# moves) numbered along the triangle moves <= 64 - discs, the region counts as
# mixed-radix digits of bases region size + 1; (pair, region a) << 22 | (b..h)
_SKEY_BASES = (5, 9, 5, 9, 9, 17, 5, 13)
_SKEY_LOW = 22
SKEY_LIMIT = (2145 * 5) << _SKEY_LOW  # the skeys lie below it (not every value below is one)
_TRI = np.array([65 * d - d * (d - 1) // 2 for d in range(66)], np.int64)


def counts_to_skey(c):
    """A counts() 10-tuple's OTH_TD_SKEY (same order as counts_to_key)."""
    d, m = int(c[0]), int(c[1])
    if not (0 <= d <= 64 and 0 <= m <= 64 - d):
        raise ValueError(f"counts ({d}, {m}) outside moves <= 64 - discs")
    for v, b in zip(c[2:], _SKEY_BASES):
        if not 0 <= int(v) < b:
            raise ValueError(f"region count {v} out of range")
    low = 0
    for v, b in zip(c[3:], _SKEY_BASES[1:]):
        low = low * b + int(v)
    return (((65 * d - d * (d - 1) // 2 + m) * 5 + int(c[2])) << _SKEY_LOW) | low


def skeys_to_keys(s):
    """OTH_TD_SKEY values -> OTH_TD_KEY values (numpy, vectorised)."""
    s = np.asarray(s, dtype=np.int64)
    pair, ra = np.divmod(s >> _SKEY_LOW, 5)
    low = s & ((1 << _SKEY_LOW) - 1)
    d = np.searchsorted(_TRI, pair, side="right") - 1
    key = (d << _SHIFTS[0]) | ((pair - _TRI[d]) << _SHIFTS[1]) | (ra << _SHIFTS[2])
    for b, sh in zip(reversed(_SKEY_BASES[1:]), reversed(_SHIFTS[3:])):
        low, v = np.divmod(low, b)
        key |= v << sh
    return key


def skey_to_counts(s):
    return key_to_counts(int(skeys_to_keys(np.array([int(s)]))[0]))


def unpack_counts(keys):
    """Packed keys (device int64 tensor) -> (n, 10) int64 counts() tuples."""
    cols = [(keys >> s) & ((1 << w) - 1) for s, w in zip(_SHIFTS, _WIDTH)]
    return torch.stack(cols, 1)


def hash_string(k):
    """ProgressPositionMovesParameter.hash_from_book format (parameter_progress_position_moves_learn.py:47-49)."""
    return ":".join(str(v) for v in key_to_counts(k))


def records_plan(books, lam=LAMBDA):
    """The host half of StateMap.update_from_records: the board strings of
    every record in processing order, and per record the row of its book's
    terminal record (int64), its index (int32) into a table (float64) of
    l ** (last_turn - turn) over the distinct exponents, each power computed
    as the learner computes it (a CPython float power, 46)."""
    strings, expo, term = [], [], []
    for _book_id, book, _meta in books:
        last_turn = int(book[0]["turn"])
        t0 = len(strings)
        for rec in book:
            strings.append(rec["book"])
            expo.append(last_turn - int(rec["turn"]))
            term.append(t0)
    uniq = sorted(set(expo))
    slot = {k: i for i, k in enumerate(uniq)}
    return (strings, np.array(term, np.int64), np.array([slot[k] for k in expo], np.int32),
            np.array([lam ** k for k in uniq], np.float64))


def _with_scratch(fn, args, stream, device, what):
    """Call a TD entry point that takes caller scratch (temp, temp_bytes): its
    size query, the scratch from torch's caching allocator, the call."""
    tb = ctypes.c_size_t(0)
    check(fn(*args, None, ctypes.byref(tb), stream), what + " (size query)")
    temp = torch.empty(max(tb.value, 1), dtype=torch.uint8, device=device)
    check(fn(*args, temp.data_ptr(), ctypes.byref(tb), stream), what)
    return temp


def word_errors(device="cuda", reset=True):
    """The number of packed update words with a turn_left past the lam_pow
    table that the TD readers (unpack, sort_unpack, segments_words) met on
    `device` since the last reset (include/othello.h oth_td_word_errors): 0
    unless a word array was corrupted or did not come from
    oth_td_updates_packed.  Synchronizes the current stream."""
    d = torch.device(device)
    with torch.cuda.device(d):
        out = ctypes.c_uint64(0)
        check(_lib.load().oth_td_word_errors(ctypes.byref(out), int(bool(reset)),
                                              torch.cuda.current_stream(d).cuda_stream), "oth_td_word_errors")
    return int(out.value)


class StateMap:
    """Device-resident 'param:state:*' table: sorted int64 keys + float64 values."""

    def __init__(self, device="cuda", a=A, lam=LAMBDA):
        d = torch.device(device)
        if d.type == "cuda" and d.index is None:
            d = torch.device("cuda", torch.cuda.current_device())
        self.device = d
        self.a = a
        self.lam = lam
        self.keys = torch.empty(0, dtype=torch.int64, device=self.device)
        self.values = torch.empty(0, dtype=torch.float64, device=self.device)
        self._lam_pow = torch.tensor(lam_pow_table(lam), dtype=torch.float64, device=self.device)

    def __len__(self):
        return int(self.keys.numel())

    def update(self, pos_boards, plies, row_off=None):
        """Apply the books of n games: pos_boards (n, 129, 2) int64 as ops.replay
        returns it, or the packed (R, 2) rows of ops.replay_rows with their
        ``row_off``; plies (n,) uint8.  Returns the number of updates applied."""
        n = plies.shape[0]
        if row_off is None:
            if pos_boards.shape != (n, POS_STRIDE, 2) or pos_boards.dtype != torch.int64:
                raise ValueError("pos_boards must be an (n, 129, 2) int64 replay table")
        elif pos_boards.dim() != 2 or pos_boards.shape[1] != 2 or pos_boards.dtype != torch.int64 or \
                row_off.shape != (n,) or row_off.dtype != torch.int64 or row_off.device != self.device:
            raise ValueError("packed rows: pos_boards (R, 2) int64 and row_off (n,) int64 on the map's device")
        if plies.dtype != torch.uint8 or pos_boards.device != self.device or plies.device != self.device:
            raise ValueError("plies must be uint8; both on the map's device")
        if n == 0:
            return 0
        cnt = 2 * (plies.long().clamp(max=POS_STRIDE - 1) + 1)
        ends = torch.cumsum(cnt, 0)
        base = (ends - cnt).contiguous()
        return self._update_packed(pos_boards, plies, row_off, base, int(ends[-1]))

    def update_rows(self, rows, plies):
        """update() over the packed rows of ops.replay_rows(moves, plies) (a
        ReplayRows: game g's rows start at row_off[g], the games' rows
        contiguous and in order, min(plies, 128) + 1 each): the update
        offsets are twice the row offsets and the total twice the row count,
        so no device-to-host read precedes the update kernel (round 5)."""
        n = plies.shape[0]
        b, off = rows.boards, rows.row_off
        if b.dim() != 2 or b.shape[1] != 2 or b.dtype != torch.int64 or off.shape != (n,) or \
                off.dtype != torch.int64 or plies.dtype != torch.uint8 or \
                not (b.device == off.device == plies.device == self.device):
            raise ValueError("rows: ops.replay_rows of these plies on the map's device")
        if n == 0:
            return 0
        return self._update_packed(b, plies, off, (2 * off).contiguous(), 2 * b.shape[0])

    def _update_packed(self, pos_boards, plies, row_off, base, total):
        n = plies.shape[0]
        lib = _lib.load()
        stream = torch.cuda.current_stream(self.device).cuda_stream
        with torch.cuda.device(self.device):
            # the update stream as packed words (skey | turn_left | value_side):
            # half the bytes of (key, value) pairs through the sort
            words = torch.empty(total, dtype=torch.int64, device=self.device)
            check(lib.oth_td_updates_packed(pos_boards.contiguous().data_ptr(),
                                            None if row_off is None else row_off.contiguous().data_ptr(),
                                            plies.contiguous().data_ptr(), base.data_ptr(), words.data_ptr(), n,
                                            stream), "oth_td_updates_packed")
            # a keys-only sort of the words by their skey bits (the payload rides
            # along), then the segments straight from the sorted words, which
            # also writes each update's value (oth_td_segments_words: no
            # separate unpack into a keys array and a values array)
            sorted_words = torch.empty_like(words)
            _with_scratch(lib.oth_td_sort_packed, (words.data_ptr(), sorted_words.data_ptr(), total), stream,
                          self.device, "oth_td_sort_packed")
            del words
            sv = torch.empty(total, dtype=torch.float64, device=self.device)
            segs = self._segments(sorted_words, sv)
            del sorted_words
        self._apply_segments(sv, *segs)
        return total

    def update_from_records(self, books):
        """learn_and_update_batch's state-map half (progress_position_moves_learn.py:94-96
        -> __update_state_for_a_book, 37-62) over books as replearn.learn_books
        hands them over (replearn.py:27-46), from any source: ``books`` =
        [(book_id, records, meta), ...], each record a dict with 'book' (the
        board string) and 'turn', the terminal record first.  Every record is
        applied in the given order, sides 'O' then 'X', with its own
        l ** (last_turn - turn) (gaps, repeats and any order of turns as the
        reference has them); the board strings are parsed on the GPU
        (books.parse_book_strings) and the updates built by
        oth_td_updates_records.  A book without records raises IndexError, a
        malformed turn ValueError, as in the reference.  Returns the number of
        updates applied."""
        from .books import parse_book_strings
        strings, term, lam_idx, lam_pow = records_plan(books, self.lam)
        if not strings:
            return 0
        rows = parse_book_strings(strings, self.device)
        lam_pow = torch.from_numpy(lam_pow).to(self.device)
        lam_idx = torch.from_numpy(lam_idx).to(self.device)
        term_row = torch.from_numpy(term).to(self.device)
        total = 2 * len(strings)
        keys = torch.empty(total, dtype=torch.int64, device=self.device)
        vals = torch.empty(total, dtype=torch.float64, device=self.device)
        with torch.cuda.device(self.device):
            check(_lib.load().oth_td_updates_records(rows.data_ptr(), term_row.data_ptr(), lam_idx.data_ptr(),
                                                     lam_pow.data_ptr(), keys.data_ptr(), vals.data_ptr(),
                                                     len(strings), torch.cuda.current_stream(self.device).cuda_stream),
                  "oth_td_updates_records")
        self._apply(keys, vals)
        return total

    def _apply(self, keys, vals):
        """The batch's ordered (key, value) update stream into the table:
        stable sort by key, each key's EMA in stream order, merge."""
        total = keys.numel()
        lib = _lib.load()
        stream = torch.cuda.current_stream(self.device).cuda_stream
        with torch.cuda.device(self.device):
            sk, sv = torch.empty_like(keys), torch.empty_like(vals)
            _with_scratch(lib.oth_td_sort_pairs, (keys.data_ptr(), vals.data_ptr(), sk.data_ptr(), sv.data_ptr(),
                                                  total), stream, self.device, "oth_td_sort_pairs")
        self._apply_sorted(sk, sv)

    def _apply_sorted(self, sk, sv):
        """The key-sorted update stream (equal keys in stream order) into the
        table: each key's EMA in stream order, then the merge."""
        with torch.cuda.device(self.device):
            segs = self._segments(sk, None)
        self._apply_segments(sv, *segs)

    def _segments(self, sorted_in, values):
        """The sorted stream's segments in one pass pair: from keys
        (oth_td_segments), or (values given) from the sorted packed words, the
        values written as a side effect (oth_td_segments_words).  Returns
        (ukeys, seg_off, long_idx, counts) sized for every update; counts =
        (the device pair (n keys, n long keys), its pinned host copy, the
        copy's event), not yet waited for: _apply_segments queues the lookup
        behind the segments pass before the host reads them."""
        lib = _lib.load()
        stream = torch.cuda.current_stream(self.device).cuda_stream
        n = sorted_in.numel()
        seg_off = torch.empty(n + 1, dtype=torch.int64, device=self.device)
        ukeys = torch.empty(n, dtype=torch.int64, device=self.device)
        long_idx = torch.empty(n, dtype=torch.int64, device=self.device)
        cnt = torch.empty(2, dtype=torch.int64, device=self.device)
        if values is None:
            _with_scratch(lib.oth_td_segments, (sorted_in.data_ptr(), n, LONG_MIN, seg_off.data_ptr(),
                                                ukeys.data_ptr(), long_idx.data_ptr(), cnt.data_ptr()), stream,
                          self.device, "oth_td_segments")
        else:
            _with_scratch(lib.oth_td_segments_words, (sorted_in.data_ptr(), self._lam_pow.data_ptr(), n, LONG_MIN,
                                                      seg_off.data_ptr(), ukeys.data_ptr(), long_idx.data_ptr(),
                                                      cnt.data_ptr(), values.data_ptr()), stream, self.device,
                          "oth_td_segments_words")
        host = torch.empty(2, dtype=torch.int64, pin_memory=True)
        host.copy_(cnt, non_blocking=True)
        ev = torch.cuda.Event()
        ev.record()
        return ukeys, seg_off, long_idx, (cnt, host, ev)

    def _apply_segments(self, sv, ukeys, seg_off, long_idx, counts):
        """Each key's EMA in stream order over its segment of sv, then the merge."""
        cnt, host, ev = counts
        if not _LOOKUP_AHEAD:  # A/B (OTH_TD_LOOKUP_AHEAD=0): the host reads the counts first
            ev.synchronize()
        lib = _lib.load()
        stream = torch.cuda.current_stream(self.device).cuda_stream
        with torch.cuda.device(self.device):
            pending = None
            if len(self):
                # the lookup queued before the host reads the key count: it
                # takes the count from the device (oth_td_lookup_dev), so the
                # host's read below overlaps it (round 5: the read and the
                # Python after it left the GPU idle ~50 us per batch)
                # sized for every update, not the distinct keys (unknown yet):
                # ~9 B per update, ~290 MB at a 32M-update batch, short-lived
                # and recycled batch to batch by torch's caching allocator --
                # the memory price of queuing the lookup early
                n_max = ukeys.numel()
                init = torch.empty(n_max, dtype=torch.float64, device=self.device)
                is_new = torch.empty(n_max, dtype=torch.uint8, device=self.device)
                # (its scratch, the merge path's splits, is the merge's too:
                # oth_td_merge_after_lookup)
                lk_temp = _with_scratch(lib.oth_td_lookup_dev, (self.keys.data_ptr(), self.values.data_ptr(),
                                                                len(self), ukeys.data_ptr(), n_max, cnt.data_ptr(),
                                                                init.data_ptr(), is_new.data_ptr()),
                                        stream, self.device, "oth_td_lookup_dev")
            ev.synchronize()  # the counts' copy, queued before the lookup
            n_upd, n_long = host.tolist()
            ukeys, seg_off, long_idx = ukeys[:n_upd], seg_off[:n_upd + 1], long_idx[:n_long]
            if len(self):
                init, is_new = init[:n_upd], is_new[:n_upd]
                # the merge's sizes before the EMA: the host reads the new-key
                # count while the EMA runs (round 5; a stream sync after the
                # EMA left the GPU idle while the host sized and launched the
                # merge)
                pending = self._new_before(is_new, lib, stream) + (lk_temp,)
            else:
                init = torch.zeros(n_upd, dtype=torch.float64, device=self.device)
            out = torch.empty_like(init)
            # keys with many updates (the opening and the first plies of every
            # game) are each run by a whole wavefront, the longest split into
            # parts over many (oth_td_ema_split)
            _with_scratch(lib.oth_td_ema_split, (sv.data_ptr(), seg_off.data_ptr(), init.data_ptr(), self.a,
                                                 1 - self.a, out.data_ptr(), ukeys.numel(), LONG_MIN,
                                                 long_idx.data_ptr(), long_idx.numel(), sv.numel()),
                          stream, self.device, "oth_td_ema_split")
            if pending is None:  # (a copy: ukeys is a view of an n-entry buffer)
                self.keys, self.values = ukeys.clone(), out
            else:
                self._merge(pending, ukeys, out, lib, stream)

    def _new_before(self, is_new, lib, stream):
        """new_before[j] = batch keys before j that are new (oth_td_new_before),
        and its total copied to pinned host memory behind an event."""
        n_upd = is_new.numel()
        new_before = torch.empty(n_upd + 1, dtype=torch.int64, device=self.device)
        _with_scratch(lib.oth_td_new_before, (is_new.data_ptr(), n_upd, new_before.data_ptr()), stream, self.device,
                      "oth_td_new_before")
        host = torch.empty(1, dtype=torch.int64, pin_memory=True)
        host.copy_(new_before[-1:], non_blocking=True)
        ev = torch.cuda.Event()
        ev.record()
        return new_before, host, ev

    def _merge(self, pending, ukeys, out, lib, stream):
        """The batch's keys (sorted, unique) into the key-sorted table:
        oth_td_merge (HIP merge path) writes the sorted union, placing every
        element by rank; new_before[j] = batch keys before j that are absent
        from the table (pending: _new_before's result)."""
        new_before, host, ev, lk_temp = pending
        n_old, n_upd = len(self), ukeys.numel()
        ev.synchronize()
        n_new = int(host[0])
        keys = torch.empty(n_old + n_new, dtype=torch.int64, device=self.device)
        vals = torch.empty(n_old + n_new, dtype=torch.float64, device=self.device)
        if _MERGE_SPLITS_FROM_LOOKUP:  # the lookup's splits (same tiles): no second search
            check(lib.oth_td_merge_after_lookup(self.keys.data_ptr(), self.values.data_ptr(), n_old, ukeys.data_ptr(),
                                                out.data_ptr(), new_before.data_ptr(), n_upd, keys.data_ptr(),
                                                vals.data_ptr(), lk_temp.data_ptr(), stream),
                  "oth_td_merge_after_lookup")
        else:
            _with_scratch(lib.oth_td_merge, (self.keys.data_ptr(), self.values.data_ptr(), n_old, ukeys.data_ptr(),
                                             out.data_ptr(), new_before.data_ptr(), n_upd, keys.data_ptr(),
                                             vals.data_ptr()), stream, self.device, "oth_td_merge")
        self.keys, self.values = keys, vals

    def update_from_books(self, books):
        """Apply a subproc_amd.books.GameBooks batch."""
        return self.update_rows(books.pos, books.plies)

    def get(self, counts):
        """Value for a counts() tuple, 0.0 if absent (a fresh key reads as 0, 53-56)."""
        k = torch.tensor([counts_to_key(counts)], dtype=torch.int64, device=self.device)
        if not len(self):
            return 0.0
        i = int(torch.searchsorted(self.keys, k).clamp(max=len(self) - 1))
        return float(self.values[i]) if int(self.keys[i]) == int(k) else 0.0

    def items(self):
        """{hash_from_book string: value} on the host."""
        return {hash_string(k): v for k, v in zip(self.keys.cpu().tolist(), self.values.cpu().tolist())}

    def fit(self, shards=SHARDS):
        """The learner's per-shard regression (fit_parameter,
        progress_position_moves_learn.py:160-184: LinearRegression with an
        intercept of the state value on counts()[1:], states whose counts()[0]
        lies in the shard) over EVERY state of the map, not a random sample.
        Normal equations of the centred data, accumulated in float64 on the
        device over the shard's contiguous range of the table by
        oth_td_fit_moments (two passes: means, then centred cross products),
        solved (minimum norm) on the host.  Returns float64 arrays
        coef (len(shards), 9), intercept (len(shards),), n (len(shards),)."""
        # the table is key-sorted and the phase is the key's top field: each
        # shard is one contiguous range of it
        lib = _lib.load()
        stream = torch.cuda.current_stream(self.device).cuda_stream
        edges = torch.tensor([[lo << _SHIFTS[0], (hi + 1) << _SHIFTS[0]] for lo, hi in shards], dtype=torch.int64,
                             device=self.device)
        ranges = torch.searchsorted(self.keys, edges.flatten()).view(-1, 2).cpu().tolist()
        partials = torch.empty((_lib.TD_FIT_BLOCKS, _lib.TD_FIT_COLS), dtype=torch.float64, device=self.device)
        coef = np.zeros((len(shards), 9))
        icpt = np.zeros(len(shards))
        nk = np.zeros(len(shards), np.int64)
        for k, (s, e) in enumerate(ranges):
            nk[k] = e - s
            if nk[k] == 0:
                continue
            kp, vp = self.keys[s:e], self.values[s:e]
            with torch.cuda.device(self.device):
                check(lib.oth_td_fit_moments(kp.data_ptr(), vp.data_ptr(), e - s, None, partials.data_ptr(), stream),
                      "oth_td_fit_moments")
                m1 = partials[:, :11].sum(0)
                mean = torch.cat([m1[1:10], m1[10:11]]) / m1[0]
                check(lib.oth_td_fit_moments(kp.data_ptr(), vp.data_ptr(), e - s, mean.data_ptr(),
                                             partials.data_ptr(), stream), "oth_td_fit_moments")
                m2 = partials[:, :54].sum(0).cpu().numpy()
            A = np.zeros((9, 9))
            A[np.triu_indices(9)] = m2[:45]
            A = A + np.triu(A, 1).T
            mean = mean.cpu().numpy()
            coef[k] = np.linalg.lstsq(A, m2[45:54], rcond=None)[0]
            icpt[k] = float(mean[9]) - float(mean[:9] @ coef[k])
        return coef, icpt, nk
