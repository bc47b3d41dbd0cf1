/*
 * othello_cpu_abi.c — libothello_cpu.so: the C-ABI of include/othello.h built
 * for the HOST on top of the parity oracle (othello_oracle.c).
 *
 * TEST INFRASTRUCTURE ONLY.  SURVEY.md §8(b)/(c) ask for a CPU build of the
 * same header that gives identical results, so parity can be checked at the
 * ABI itself: tests call the same entry points with the same arguments on this
 * library (host pointers) and on libsubproc_amd_hip.so (device pointers) and
 * compare.  The product package never loads this library.
 *
 * Differences from the HIP library, by design:
 *   - every pointer is HOST memory; `stream` is ignored (calls are synchronous);
 *   - OpenMP over all host threads where the oracle parallelises.
 */
#include <stdint.h>
#include <string.h>

#include "../include/othello.h"

/* the oracle's exported functions (othello_oracle.c) */
int oracle_reset(uint64_t* boards, uint8_t* turn, uint8_t* nturn, int64_t n);
int oracle_legal(const uint64_t* boards, const uint8_t* turn, uint64_t* legal, int64_t n);
int oracle_step(const uint64_t* boards_in, const uint8_t* turn_in, const uint8_t* move, uint64_t* boards_out,
                uint8_t* turn_out, uint64_t* flips, uint64_t* legal_next, int8_t* ret, uint8_t* nturn, int64_t n);
int oracle_result(const uint64_t* boards, uint8_t* n_black, uint8_t* n_white, int8_t* diff, uint8_t* terminal,
                  int64_t n);
int oracle_rollout(const uint64_t* start, const uint8_t* start_turn, uint64_t seed, uint64_t game_id0, int policy,
                   int n_random, uint64_t* final_boards, int8_t* diff, uint8_t* plies, uint8_t* moves,
                   int64_t* hist, int64_t n, int n_threads, const int8_t* weights, const int8_t* weights_white);
int oracle_sample_midgame(uint64_t seed, uint64_t index0, uint64_t* boards, uint8_t* turn, uint8_t* nturn,
                          uint8_t* move, int64_t n);
int oracle_rollout_runner(const uint64_t* start, const uint8_t* start_turn, uint64_t seed, uint64_t game_id0,
                          int policy, const int8_t* weights_a, const int8_t* weights_b, int n_rand_a, int n_rand_b,
                          int swap, uint8_t* a_black, uint64_t* final_boards, int8_t* diff, uint8_t* plies,
                          uint8_t* moves, int64_t* hist, int64_t n, int n_threads);
int oracle_features(const uint64_t* boards, const uint8_t* side, uint8_t* out, int64_t n);
int oracle_eval(const uint64_t* boards, const uint8_t* side, const int8_t* weights, int32_t* out, int64_t n);
int oracle_replay(const uint64_t* start, const uint8_t* start_turn, const uint8_t* moves, const uint8_t* plies,
                  uint64_t* pos, uint8_t* pos_turn, uint8_t* pos_end, int64_t n);

int oracle_hands(const uint64_t* boards, const uint8_t* piece, const int64_t* x, const int64_t* y, const int64_t* dx,
                 const int64_t* dy, uint8_t* count, int64_t n);

const char* oth_version(void) { return "subproc_amd-cpu 0.1.0 host (oracle)"; }

int oth_reset(uint64_t* boards, uint8_t* turn, uint8_t* nturn, int64_t n, void* stream) {
    (void)stream;
    if (n < 0 || (n > 0 && !boards)) return OTH_EINVAL;
    return oracle_reset(boards, turn, nturn, n);
}

int oth_legal(const uint64_t* boards, const uint8_t* turn, uint64_t* legal, int64_t n, void* stream) {
    (void)stream;
    if (n < 0 || (n > 0 && (!boards || !turn || !legal))) return OTH_EINVAL;
    return oracle_legal(boards, turn, legal, n);
}

int oth_step(const uint64_t* boards_in, const uint8_t* turn_in, const uint8_t* move, uint64_t* boards_out,
             uint8_t* turn_out, uint64_t* flips, uint64_t* legal_next, int8_t* ret, uint8_t* nturn, int64_t n,
             void* stream) {
    (void)stream;
    if (n < 0 || (n > 0 && (!boards_in || !turn_in || !move))) return OTH_EINVAL;
    return oracle_step(boards_in, turn_in, move, boards_out, turn_out, flips, legal_next, ret, nturn, n);
}

int oth_result(const uint64_t* boards, uint8_t* n_black, uint8_t* n_white, int8_t* diff, uint8_t* terminal,
               int64_t n, void* stream) {
    (void)stream;
    if (n < 0 || (n > 0 && !boards)) return OTH_EINVAL;
    return oracle_result(boards, n_black, n_white, diff, terminal, n);
}

/* own -> White squares, hostile -> Black squares, then the scan of piece White
 * (hostile(White) = Black): the same question on a board the oracle holds */
int oth_hands(const uint64_t* own, const uint64_t* hostile, const int64_t* x, const int64_t* y, const int64_t* dx,
              const int64_t* dy, uint8_t* count, int64_t n, void* stream) {
    (void)stream;
    if (n < 0 || (n > 0 && (!own || !hostile || !x || !y || !dx || !dy || !count))) return OTH_EINVAL;
    for (int64_t i = 0; i < n; i++) {
        const uint64_t b[2] = {hostile[i], own[i] & ~hostile[i]};
        const uint8_t piece = OTH_WHITE;
        oracle_hands(b, &piece, x + i, y + i, dx + i, dy + i, count + i, 1);
    }
    return OTH_OK;
}

/* `work` is the GPU launch's batch counter: checked, otherwise unused here */
int oth_rollout(const uint64_t* start, const uint8_t* start_turn, uint64_t seed, uint64_t game_id0, int policy,
                int n_random, uint64_t* final_boards, int8_t* diff, uint8_t* plies, uint8_t* moves, int64_t* hist,
                uint64_t* work, int64_t n, void* stream) {
    (void)stream;
    if (n < 0 || !work || (policy != OTH_POLICY_RANDOM && policy != OTH_POLICY_GREEDY)) return OTH_EINVAL;
    if (n == 0) return OTH_OK;
    return oracle_rollout(start, start_turn, seed, game_id0, policy, n_random, final_boards, diff, plies, moves, hist,
                          n, 0, NULL, NULL);
}

int oth_rollout_eval(const uint64_t* start, const uint8_t* start_turn, uint64_t seed, uint64_t game_id0,
                     int n_random, const int8_t* weights, uint64_t* final_boards, int8_t* diff, uint8_t* plies,
                     uint8_t* moves, int64_t* hist, uint64_t* work, int64_t n, void* stream) {
    (void)stream;
    if (n < 0 || !weights || !work) return OTH_EINVAL;
    if (n == 0) return OTH_OK;
    return oracle_rollout(start, start_turn, seed, game_id0, OTH_POLICY_EVAL, n_random, final_boards, diff, plies,
                          moves, hist, n, 0, weights, NULL);
}

int oth_rollout_match(const uint64_t* start, const uint8_t* start_turn, uint64_t seed, uint64_t game_id0,
                      int n_random, const int8_t* weights_black, const int8_t* weights_white, uint64_t* final_boards,
                      int8_t* diff, uint8_t* plies, uint8_t* moves, int64_t* hist, uint64_t* work, int64_t n,
                      void* stream) {
    (void)stream;
    if (n < 0 || !weights_black || !weights_white || !work) return OTH_EINVAL;
    if (n == 0) return OTH_OK;
    return oracle_rollout(start, start_turn, seed, game_id0, OTH_POLICY_EVAL, n_random, final_boards, diff, plies,
                          moves, hist, n, 0, weights_black, weights_white);
}

int oth_rollout_runner(const uint64_t* start, const uint8_t* start_turn, uint64_t seed, uint64_t game_id0, int policy,
                       const int8_t* weights_a, const int8_t* weights_b, int n_rand_a, int n_rand_b, int swap_colours,
                       uint8_t* a_black, uint64_t* final_boards, int8_t* diff, uint8_t* plies, uint8_t* moves,
                       int64_t* hist, uint64_t* work, int64_t n, void* stream) {
    (void)stream;
    if (n < 0 || !work || (policy != OTH_POLICY_GREEDY && policy != OTH_POLICY_EVAL) ||
        (policy == OTH_POLICY_EVAL && (!weights_a || !weights_b)) || n_rand_a < 0 || n_rand_b < 0)
        return OTH_EINVAL;
    if (n == 0) return OTH_OK;
    return oracle_rollout_runner(start, start_turn, seed, game_id0, policy, weights_a, weights_b, n_rand_a, n_rand_b,
                                 swap_colours, a_black, final_boards, diff, plies, moves, hist, n, 0);
}

int oth_sample_midgame(uint64_t seed, uint64_t index0, uint64_t* boards, uint8_t* turn, uint8_t* nturn,
                       uint8_t* move, int64_t n, void* stream) {
    (void)stream;
    if (n < 0 || (n > 0 && (!boards || !turn || !move))) return OTH_EINVAL;
    return oracle_sample_midgame(seed, index0, boards, turn, nturn, move, n);
}

int oth_replay(const uint64_t* start, const uint8_t* start_turn, const uint8_t* moves, const uint8_t* plies,
               uint64_t* pos_boards, uint8_t* pos_turn, uint8_t* pos_end, int64_t n, void* stream) {
    (void)stream;
    if (n < 0 || (n > 0 && (!moves || !plies || !pos_boards))) return OTH_EINVAL;
    return oracle_replay(start, start_turn, moves, plies, pos_boards, pos_turn, pos_end, n);
}

/* the packed-rows layout: the oracle's strided replay of one game at a time,
 * its rows 0..plies copied to row_off[i] */
int oth_replay_rows(const uint64_t* start, const uint8_t* start_turn, const uint8_t* moves, const uint8_t* plies,
                    const int64_t* row_off, uint64_t* pos_boards, uint8_t* pos_turn, uint8_t* pos_end, int64_t n,
                    void* stream) {
    (void)stream;
    if (n < 0 || (n > 0 && (!moves || !plies || !row_off || !pos_boards))) return OTH_EINVAL;
    uint64_t b[2 * OTH_POS_STRIDE];
    uint8_t t[OTH_POS_STRIDE], e[OTH_POS_STRIDE];
    for (int64_t i = 0; i < n; i++) {
        int rc = oracle_replay(start ? start + 2 * i : NULL, start_turn ? start_turn + i : NULL,
                               moves + i * OTH_MOVES_STRIDE, plies + i, b, t, e, 1);
        if (rc != OTH_OK) return rc;
        const int np = plies[i] < OTH_MOVES_STRIDE ? plies[i] : OTH_MOVES_STRIDE;
        for (int p = 0; p <= np; p++) {
            pos_boards[2 * (row_off[i] + p)] = b[2 * p];
            pos_boards[2 * (row_off[i] + p) + 1] = b[2 * p + 1];
            if (pos_turn) pos_turn[row_off[i] + p] = t[p];
            if (pos_end) pos_end[row_off[i] + p] = e[p];
        }
    }
    return OTH_OK;
}

/* serialize_str (board.py:214-243) + '\n': 64 chars row-major, 'O' black,
 * 'X' white, '-' empty, then ' ' and the side to move ('O', 'X', or '-'). */
int oth_book_text(const uint64_t* boards, const uint8_t* turn, int64_t n, char* out, void* stream) {
    (void)stream;
    if (n < 0 || (n > 0 && (!boards || !turn || !out))) return OTH_EINVAL;
    for (int64_t i = 0; i < n; i++) {
        char* line = out + i * OTH_BOOK_LINE;
        const uint64_t bl = boards[2 * i], wh = boards[2 * i + 1];
        for (int sq = 0; sq < 64; sq++) line[sq] = (bl >> sq & 1) ? 'O' : ((wh >> sq & 1) ? 'X' : '-');
        line[64] = ' ';
        line[65] = turn[i] == OTH_BLACK ? 'O' : (turn[i] == OTH_WHITE ? 'X' : '-');
        line[66] = '\n';
    }
    return OTH_OK;
}

/* Board.deserialize of each 64-char string onto a fresh Board, one char at a
 * time (board.py:253-258): 'O' Black, 'X' White, anything else Empty */
int oth_book_parse(const char* text, int64_t stride, uint64_t* boards, uint8_t* turn, int64_t n, void* stream) {
    (void)stream;
    if (n < 0 || stride < 64 || (turn && stride < 66) || (n > 0 && (!text || !boards))) return OTH_EINVAL;
    for (int64_t i = 0; i < n; i++) {
        const char* s = text + i * stride;
        uint64_t bl = 0, wh = 0;
        for (int sq = 0; sq < 64; sq++) {
            if (s[sq] == 'O') bl |= 1ull << sq;
            else if (s[sq] == 'X') wh |= 1ull << sq;
        }
        boards[2 * i] = bl;
        boards[2 * i + 1] = wh;
        if (turn) turn[i] = s[65] == 'O' ? OTH_BLACK : (s[65] == 'X' ? OTH_WHITE : 0);
    }
    return OTH_OK;
}

int oth_features(const uint64_t* boards, const uint8_t* side, uint8_t* out, int64_t n, void* stream) {
    (void)stream;
    if (n < 0 || (n > 0 && (!boards || !side || !out))) return OTH_EINVAL;
    return oracle_features(boards, side, out, n);
}

/* TD update stream over the oracle's counts() (see include/othello.h) */
static int64_t td_key(const uint8_t f[10]) {
    static const int shift[10] = {36, 30, 27, 23, 20, 16, 12, 7, 4, 0};  /* include/othello.h OTH_TD_KEY layout */
    int64_t k = 0;
    for (int i = 0; i < 10; i++) k |= (int64_t)f[i] << shift[i];
    return k;
}

/* the packed words' sort key, include/othello.h OTH_TD_SKEY: (discs, moves)
 * numbered row by row of the triangle moves <= 64 - discs, then the regions as
 * mixed-radix digits (bases: region sizes + 1), a most significant; the
 * number split as (pair, a) << 22 | (b..h) */
static const uint64_t skey_base[8] = {5, 9, 5, 9, 9, 17, 5, 13};
static uint64_t td_skey(const uint8_t f[10]) {
    uint64_t pair = 0;
    for (int d = 0; d < f[0]; d++) pair += (uint64_t)(65 - d);
    pair += f[1];
    uint64_t low = 0, scale = 1;
    for (int i = 7; i >= 1; i--) {
        low += (uint64_t)f[2 + i] * scale;
        scale *= skey_base[i];
    }
    return ((pair * skey_base[0] + f[2]) << 22) | low;
}
static int64_t td_key_of_skey(uint64_t s) {
    uint64_t high = s >> 22, low = s & ((1ull << 22) - 1);
    uint8_t f[10];
    uint64_t pair = high / skey_base[0];
    f[2] = (uint8_t)(high % skey_base[0]);
    int d = 0;
    while (pair >= (uint64_t)(65 - d)) pair -= (uint64_t)(65 - d++);
    f[0] = (uint8_t)d;
    f[1] = (uint8_t)pair;
    for (int i = 7; i >= 1; i--) {
        f[2 + i] = (uint8_t)(low % skey_base[i]);
        low /= skey_base[i];
    }
    return td_key(f);
}

static int td_updates_any(const uint64_t* pos_boards, const int64_t* row_off, const uint8_t* plies,
                          const int64_t* base, const double* lam_pow, int64_t* keys, double* values, int64_t n) {
    for (int64_t g = 0; g < n; g++) {
        const uint64_t* row = pos_boards + (row_off ? row_off[g] : g * OTH_POS_STRIDE) * 2;
        const int np = plies[g] < OTH_MOVES_STRIDE ? plies[g] : OTH_MOVES_STRIDE;
        int8_t d;
        oracle_result(row + 2 * np, NULL, NULL, &d, NULL, 1);
        for (int p = 0; p <= np; p++) {
            uint8_t f[2][10];
            const uint8_t sides[2] = {OTH_BLACK, OTH_WHITE};
            const uint64_t b2[4] = {row[2 * p], row[2 * p + 1], row[2 * p], row[2 * p + 1]};
            oracle_features(b2, sides, &f[0][0], 2);
            const int64_t j = base[g] + 2 * (int64_t)(np - p);
            keys[j] = td_key(f[0]);
            values[j] = (double)d * lam_pow[np - p];
            keys[j + 1] = td_key(f[1]);
            values[j + 1] = (double)(-d) * lam_pow[np - p];
        }
    }
    return OTH_OK;
}

int oth_rollout_grid(int policy, int64_t n) {
    if (n < 0 || policy < OTH_POLICY_RANDOM || policy > OTH_POLICY_EVAL) return OTH_EINVAL;
    return 1;
}

int oth_td_updates(const uint64_t* pos_boards, const uint8_t* plies, const int64_t* base, const double* lam_pow,
                   int64_t* keys, double* values, int64_t n, void* stream) {
    (void)stream;
    if (n < 0 || (n > 0 && (!pos_boards || !plies || !base || !lam_pow || !keys || !values))) return OTH_EINVAL;
    return td_updates_any(pos_boards, NULL, plies, base, lam_pow, keys, values, n);
}

int oth_td_updates_rows(const uint64_t* pos_boards, const int64_t* row_off, const uint8_t* plies, const int64_t* base,
                        const double* lam_pow, int64_t* keys, double* values, int64_t n, void* stream) {
    (void)stream;
    if (n < 0 || (n > 0 && (!pos_boards || !row_off || !plies || !base || !lam_pow || !keys || !values)))
        return OTH_EINVAL;
    return td_updates_any(pos_boards, row_off, plies, base, lam_pow, keys, values, n);
}

/* packed words: the same updates, (value_side + 64) << 56 | turn_left << 36 | OTH_TD_SKEY */
int oth_td_updates_packed(const uint64_t* pos_boards, const int64_t* row_off, const uint8_t* plies,
                          const int64_t* base, uint64_t* words, int64_t n, void* stream) {
    (void)stream;
    if (n < 0 || (n > 0 && (!pos_boards || !plies || !base || !words))) return OTH_EINVAL;
    for (int64_t g = 0; g < n; g++) {
        const uint64_t* row = pos_boards + (row_off ? row_off[g] : g * OTH_POS_STRIDE) * 2;
        const int np = plies[g] < OTH_MOVES_STRIDE ? plies[g] : OTH_MOVES_STRIDE;
        int8_t d;
        oracle_result(row + 2 * np, NULL, NULL, &d, NULL, 1);
        for (int p = 0; p <= np; p++) {
            uint8_t f[2][10];
            const uint8_t sides[2] = {OTH_BLACK, OTH_WHITE};
            const uint64_t b2[4] = {row[2 * p], row[2 * p + 1], row[2 * p], row[2 * p + 1]};
            oracle_features(b2, sides, &f[0][0], 2);
            const int64_t j = base[g] + 2 * (int64_t)(np - p);
            const uint64_t tl = (uint64_t)(np - p);
            const uint64_t t = tl << OTH_TD_PACK_TURN_SHIFT;
            words[j] = ((uint64_t)(d + 64) << OTH_TD_PACK_VALUE_SHIFT) | t | td_skey(f[0]);
            words[j + 1] = ((uint64_t)(64 - d) << OTH_TD_PACK_VALUE_SHIFT) | t | td_skey(f[1]);
        }
    }
    return OTH_OK;
}

/* turn_left as a lam_pow index, clamped to the table and counted when out of
 * range (as the GPU build) */
static uint64_t g_td_bad_words;
static uint64_t td_turn_idx(uint64_t w) {
    const uint64_t t = (w >> OTH_TD_PACK_TURN_SHIFT) & OTH_TD_PACK_TURN_MASK;
    if (t < OTH_POS_STRIDE) return t;
    g_td_bad_words++;
    return OTH_POS_STRIDE - 1;
}

int oth_td_word_errors(uint64_t* count, int reset, void* stream) {
    (void)stream;
    if (!count) return OTH_EINVAL;
    *count = g_td_bad_words;
    if (reset) g_td_bad_words = 0;
    return OTH_OK;
}

int oth_td_unpack(const uint64_t* words, const double* lam_pow, int64_t* keys, double* values, int64_t n,
                  void* stream) {
    (void)stream;
    if (n < 0 || (n > 0 && (!words || !lam_pow || !keys || !values))) return OTH_EINVAL;
    for (int64_t i = 0; i < n; i++) {
        keys[i] = td_key_of_skey(words[i] & ((1ull << OTH_TD_SKEY_BITS) - 1));
        values[i] = (double)((int)(words[i] >> OTH_TD_PACK_VALUE_SHIFT) - 64) *
                    lam_pow[td_turn_idx(words[i])];
    }
    return OTH_OK;
}

int oth_td_updates_records(const uint64_t* rows, const int64_t* term_row, const int32_t* lam_idx,
                           const double* lam_pow, int64_t* keys, double* values, int64_t n_rows, void* stream) {
    (void)stream;
    if (n_rows < 0 || (n_rows > 0 && (!rows || !term_row || !lam_idx || !lam_pow || !keys || !values)))
        return OTH_EINVAL;
    for (int64_t r = 0; r < n_rows; r++) {
        int8_t d;
        oracle_result(rows + 2 * term_row[r], NULL, NULL, &d, NULL, 1);
        uint8_t f[2][10];
        const uint8_t sides[2] = {OTH_BLACK, OTH_WHITE};
        const uint64_t b2[4] = {rows[2 * r], rows[2 * r + 1], rows[2 * r], rows[2 * r + 1]};
        oracle_features(b2, sides, &f[0][0], 2);
        const double lam = lam_pow[lam_idx[r]];
        keys[2 * r] = td_key(f[0]);
        values[2 * r] = (double)d * lam;
        keys[2 * r + 1] = td_key(f[1]);
        values[2 * r + 1] = (double)(-d) * lam;
    }
    return OTH_OK;
}

int oth_td_ema(const double* values, const int64_t* seg_off, const double* init, double a, double one_minus_a,
               double* out, int64_t n_seg, void* stream) {
    (void)stream;
    if (n_seg < 0 || (n_seg > 0 && (!values || !seg_off || !out))) return OTH_EINVAL;
    for (int64_t s = 0; s < n_seg; s++) {
        double v = init ? init[s] : 0.0;
        for (int64_t i = seg_off[s]; i < seg_off[s + 1]; i++) {
            const double x = values[i];
            if (v == 0.0) {
                v = x;
            } else {
                const double t1 = v * one_minus_a, t2 = x * a;
                v = t1 + t2;
            }
        }
        out[s] = v;
    }
    return OTH_OK;
}

int oth_td_ema_split(const double* values, const int64_t* seg_off, const double* init, double a,
                     double one_minus_a, double* out, int64_t n_seg, int64_t long_min, const int64_t* long_idx,
                     int64_t n_long, int64_t n_values, void* temp, size_t* temp_bytes, void* stream) {
    /* the split only changes how the GPU schedules segments: every segment in
       order here, no scratch */
    if (long_min < 1 || n_long < 0 || n_values < 0 || !temp_bytes || (n_long > 0 && !long_idx)) return OTH_EINVAL;
    if (!temp) {
        *temp_bytes = 0;
        return OTH_OK;
    }
    return oth_td_ema(values, seg_off, init, a, one_minus_a, out, n_seg, stream);
}

int oth_td_new_before(const uint8_t* is_new, int64_t n, int64_t* new_before, void* temp, size_t* temp_bytes,
                      void* stream) {
    (void)stream;
    if (n < 0 || !temp_bytes) return OTH_EINVAL;
    if (!temp) {
        *temp_bytes = 0;
        return OTH_OK;
    }
    if (!new_before || (n > 0 && !is_new)) return OTH_EINVAL;
    int64_t c = 0;
    for (int64_t j = 0; j < n; j++) {
        new_before[j] = c;
        c += is_new[j] != 0;
    }
    new_before[n] = c;
    return OTH_OK;
}

/* the segments of a key-sorted stream: starts in order, long ones in order
   (the GPU lists those in any order) */
int oth_td_segments(const int64_t* keys, int64_t n, int64_t long_min, int64_t* seg_off, int64_t* ukeys,
                    int64_t* long_idx, int64_t* counts, void* temp, size_t* temp_bytes, void* stream) {
    (void)stream;
    if (n < 0 || long_min < 1 || !temp_bytes) return OTH_EINVAL;
    if (!temp) {
        *temp_bytes = 0;
        return OTH_OK;
    }
    if (!seg_off || !counts || (n > 0 && (!keys || !ukeys || !long_idx))) return OTH_EINVAL;
    int64_t m = 0, nl = 0;
    for (int64_t i = 0; i < n; i++)
        if (i == 0 || keys[i] != keys[i - 1]) {
            seg_off[m] = i;
            ukeys[m++] = keys[i];
        }
    seg_off[m] = n;
    for (int64_t j = 0; j < m; j++)
        if (seg_off[j + 1] - seg_off[j] >= long_min) long_idx[nl++] = j;
    counts[0] = m;
    counts[1] = nl;
    return OTH_OK;
}

/* the segments of the sorted words' keys (temp: the keys, n int64), and the
 * words' values by oth_td_unpack */
int oth_td_segments_words(const uint64_t* words, const double* lam_pow, int64_t n, int64_t long_min, int64_t* seg_off,
                          int64_t* ukeys, int64_t* long_idx, int64_t* counts, double* values, void* temp,
                          size_t* temp_bytes, void* stream) {
    if (n < 0 || long_min < 1 || !temp_bytes) return OTH_EINVAL;
    const size_t need = (size_t)(n > 0 ? n : 1) * sizeof(int64_t);
    if (!temp) {
        *temp_bytes = need;
        return OTH_OK;
    }
    if (*temp_bytes < need || !seg_off || !counts || (n > 0 && (!words || !lam_pow || !ukeys || !long_idx || !values)))
        return OTH_EINVAL;
    int64_t* keys = (int64_t*)temp;
    size_t none = 0;
    int rc = oth_td_unpack(words, lam_pow, keys, values, n, stream);
    if (rc == OTH_OK) rc = oth_td_segments(keys, n, long_min, seg_off, ukeys, long_idx, counts, keys, &none, stream);
    return rc;
}

/* stable sort of (key, value) pairs by key: bottom-up merge sort of the pair
 * indices (temp holds 2 * n int64 indices), then a gather */
int oth_td_sort_pairs(const int64_t* keys_in, const double* vals_in, int64_t* keys_out, double* vals_out, int64_t n,
                      void* temp, size_t* temp_bytes, void* stream) {
    (void)stream;
    if (n < 0 || !temp_bytes) return OTH_EINVAL;
    const size_t need = (size_t)(n > 0 ? n : 1) * 2 * sizeof(int64_t);
    if (!temp) {
        *temp_bytes = need;
        return OTH_OK;
    }
    if (*temp_bytes < need || (n > 0 && (!keys_in || !vals_in || !keys_out || !vals_out))) return OTH_EINVAL;
    int64_t* a = (int64_t*)temp;
    int64_t* b = a + n;
    for (int64_t i = 0; i < n; i++) a[i] = i;
    for (int64_t w = 1; w < n; w *= 2) {
        for (int64_t lo = 0; lo < n; lo += 2 * w) {
            const int64_t mid = lo + w < n ? lo + w : n, hi = lo + 2 * w < n ? lo + 2 * w : n;
            int64_t i = lo, j = mid, k = lo;
            while (i < mid && j < hi) b[k++] = keys_in[a[j]] < keys_in[a[i]] ? a[j++] : a[i++]; /* ties: left first */
            while (i < mid) b[k++] = a[i++];
            while (j < hi) b[k++] = a[j++];
        }
        int64_t* t = a;
        a = b;
        b = t;
    }
    for (int64_t i = 0; i < n; i++) {
        keys_out[i] = keys_in[a[i]];
        vals_out[i] = vals_in[a[i]];
    }
    return OTH_OK;
}

/* stable sort of packed words by their key bits: the pairs' merge sort over
 * the words' low OTH_TD_SKEY_BITS with the words as the payload */
#define KEY_MASK ((1ull << OTH_TD_SKEY_BITS) - 1)
int oth_td_sort_packed(const uint64_t* words_in, uint64_t* words_out, int64_t n, void* temp, size_t* temp_bytes,
                       void* stream) {
    (void)stream;
    if (n < 0 || !temp_bytes) return OTH_EINVAL;
    const size_t need = (size_t)(n > 0 ? n : 1) * 2 * sizeof(int64_t);
    if (!temp) {
        *temp_bytes = need;
        return OTH_OK;
    }
    if (*temp_bytes < need || (n > 0 && (!words_in || !words_out))) return OTH_EINVAL;
    int64_t* a = (int64_t*)temp;
    int64_t* b = a + n;
    for (int64_t i = 0; i < n; i++) a[i] = i;
    for (int64_t w = 1; w < n; w *= 2) {
        for (int64_t lo = 0; lo < n; lo += 2 * w) {
            const int64_t mid = lo + w < n ? lo + w : n, hi = lo + 2 * w < n ? lo + 2 * w : n;
            int64_t i = lo, j = mid, k = lo;
            while (i < mid && j < hi)
                b[k++] = (words_in[a[j]] & KEY_MASK) < (words_in[a[i]] & KEY_MASK) ? a[j++] : a[i++];
            while (i < mid) b[k++] = a[i++];
            while (j < hi) b[k++] = a[j++];
        }
        int64_t* t = a;
        a = b;
        b = t;
    }
    for (int64_t i = 0; i < n; i++) words_out[i] = words_in[a[i]];
    return OTH_OK;
}

/* the sort, then the unpack of the sorted words (temp: the sort's scratch
 * plus the sorted words) */
int oth_td_sort_unpack(const uint64_t* words_in, const double* lam_pow, int64_t* keys, double* values, int64_t n,
                       void* temp, size_t* temp_bytes, void* stream) {
    if (n < 0 || !temp_bytes) return OTH_EINVAL;
    size_t sort_bytes = 0;
    oth_td_sort_packed(NULL, NULL, n, NULL, &sort_bytes, stream);
    const size_t need = sort_bytes + (size_t)(n > 0 ? n : 1) * sizeof(uint64_t);
    if (!temp) {
        *temp_bytes = need;
        return OTH_OK;
    }
    if (*temp_bytes < need || (n > 0 && (!words_in || !lam_pow || !keys || !values || (const void*)words_in == (const void*)keys)))
        return OTH_EINVAL;
    uint64_t* sorted = (uint64_t*)((char*)temp + sort_bytes);
    int rc = oth_td_sort_packed(words_in, sorted, n, temp, &sort_bytes, stream);
    if (rc != OTH_OK) return rc;
    return oth_td_unpack(sorted, lam_pow, keys, values, n, stream);
}

/* the regression sums in one row (the other rows zero): same contract */
int oth_td_fit_moments(const int64_t* keys, const double* values, int64_t n, const double* mean, double* partials,
                       void* stream) {
    (void)stream;
    if (n < 0 || !partials || (n > 0 && (!keys || !values))) return OTH_EINVAL;
    memset(partials, 0, sizeof(double) * OTH_TD_FIT_BLOCKS * OTH_TD_FIT_COLS);
    for (int64_t i = 0; i < n; i++) {
        double x[9];
        /* counts()[1..9] of the key (include/othello.h OTH_TD_KEY layout) */
        static const int shift[9] = {30, 27, 23, 20, 16, 12, 7, 4, 0}, width[9] = {6, 3, 4, 3, 4, 4, 5, 3, 4};
        for (int f = 0; f < 9; f++) x[f] = (double)((keys[i] >> shift[f]) & ((1 << width[f]) - 1));
        if (!mean) {
            partials[0] += 1.0;
            for (int f = 0; f < 9; f++) partials[1 + f] += x[f];
            partials[10] += values[i];
        } else {
            for (int f = 0; f < 9; f++) x[f] -= mean[f];
            const double y = values[i] - mean[9];
            int q = 0;
            for (int f = 0; f < 9; f++)
                for (int g = f; g < 9; g++) partials[q++] += x[f] * x[g];
            for (int f = 0; f < 9; f++) partials[45 + f] += x[f] * y;
        }
    }
    return OTH_OK;
}

/* each batch key in the table by a two-pointer walk */
int oth_td_lookup(const int64_t* old_keys, const double* old_vals, int64_t n_old, const int64_t* upd_keys,
                  int64_t n_upd, double* init, uint8_t* is_new, void* temp, size_t* temp_bytes, void* stream) {
    (void)stream;
    if (n_old < 0 || n_upd < 0 || !temp_bytes) return OTH_EINVAL;
    if (!temp) { /* size query: the two-pointer walk needs no scratch */
        *temp_bytes = 0;
        return OTH_OK;
    }
    if ((n_old > 0 && (!old_keys || !old_vals)) || (n_upd > 0 && (!upd_keys || !init || !is_new)))
        return OTH_EINVAL;
    int64_t i = 0;
    for (int64_t j = 0; j < n_upd; j++) {
        while (i < n_old && old_keys[i] < upd_keys[j]) i++;
        const int hit = i < n_old && old_keys[i] == upd_keys[j];
        init[j] = hit ? old_vals[i] : 0.0;
        is_new[j] = (uint8_t)!hit;
    }
    return OTH_OK;
}

/* the host merge needs no splits: lookup_temp is only checked for presence */
int oth_td_merge_after_lookup(const int64_t* old_keys, const double* old_vals, int64_t n_old, const int64_t* upd_keys,
                              const double* upd_vals, const int64_t* new_before, int64_t n_upd, int64_t* out_keys,
                              double* out_vals, const void* lookup_temp, void* stream) {
    size_t zero = 0;
    if (n_upd > 0 && !lookup_temp) return OTH_EINVAL;
    return oth_td_merge(old_keys, old_vals, n_old, upd_keys, upd_vals, new_before, n_upd, out_keys, out_vals,
                        (void*)&zero, &zero, stream);
}

/* the count from (host) memory, clamped as the GPU build clamps it */
int oth_td_lookup_dev(const int64_t* old_keys, const double* old_vals, int64_t n_old, const int64_t* upd_keys,
                      int64_t n_upd_max, const int64_t* n_upd_dev, double* init, uint8_t* is_new, void* temp,
                      size_t* temp_bytes, void* stream) {
    if (n_upd_max < 0 || (temp && n_upd_max > 0 && !n_upd_dev)) return OTH_EINVAL;
    int64_t n = n_upd_max;
    if (temp && n_upd_dev) n = *n_upd_dev < 0 ? 0 : (*n_upd_dev > n_upd_max ? n_upd_max : *n_upd_dev);
    return oth_td_lookup(old_keys, old_vals, n_old, upd_keys, n, init, is_new, temp, temp_bytes, stream);
}

/* the sorted union, batch values winning (two-pointer merge; new_before is
 * the GPU kernel's placement input and is only bounds-checked here) */
int oth_td_merge(const int64_t* old_keys, const double* old_vals, int64_t n_old, const int64_t* upd_keys,
                 const double* upd_vals, const int64_t* new_before, int64_t n_upd, int64_t* out_keys,
                 double* out_vals, void* temp, size_t* temp_bytes, void* stream) {
    (void)stream;
    if (n_old < 0 || n_upd < 0 || !temp_bytes) return OTH_EINVAL;
    if (!temp) { /* size query: the two-pointer merge needs no scratch */
        *temp_bytes = 0;
        return OTH_OK;
    }
    if ((n_old > 0 && (!old_keys || !old_vals)) ||
        (n_upd > 0 && (!upd_keys || !upd_vals || !new_before)) || (n_old + n_upd > 0 && (!out_keys || !out_vals)))
        return OTH_EINVAL;
    const int64_t n_out = n_old + (n_upd > 0 ? new_before[n_upd] : 0);
    int64_t i = 0, j = 0, k = 0;
    while ((i < n_old || j < n_upd) && k < n_out) {
        if (j >= n_upd || (i < n_old && old_keys[i] < upd_keys[j])) {
            out_keys[k] = old_keys[i];
            out_vals[k++] = old_vals[i++];
        } else {
            if (i < n_old && old_keys[i] == upd_keys[j]) i++;
            out_keys[k] = upd_keys[j];
            out_vals[k++] = upd_vals[j++];
        }
    }
    return (i < n_old || j < n_upd || k != n_out) ? OTH_EINVAL : OTH_OK;
}

int oth_eval(const uint64_t* boards, const uint8_t* side, const int8_t* weights, int32_t* out, int64_t n,
             void* stream) {
    (void)stream;
    if (n < 0 || !weights || (n > 0 && (!boards || !side || !out))) return OTH_EINVAL;
    return oracle_eval(boards, side, weights, out, n);
}
