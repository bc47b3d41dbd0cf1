/*
 * othello.h — C-ABI of the MI355X-native batched Othello environment
 * (libsubproc_amd_hip.so, built from subproc_amd/csrc/othello.hip for gfx950).
 *
 * The reference (ysnrkdm/subproc) has no FFI: its step path is the Python
 * class board.Board (board.py:20-262), imported as a module by
 * game_runner.py:3, learn_base.py:1 and parameter.py:2.  Each entry point
 * below is the batched replacement of one group of Board methods; the Python
 * facade subproc_amd/board.py restores the exact method-level API on top of it
 * (INTEGRATION.md shows the ctypes binding).
 *
 * Conventions:
 *   board   = 2 x uint64 per game, [black, white] (colour-absolute), array (n,2)
 *             bit sq = x + 8*y, x = file a..h, y = rank 1..8   (board.py:74-81)
 *   turn    = uint8, 1 = Black, 2 = White                         (board.py:3-7);
 *             0 = Empty (deserialize with a side string other than 'O'/'X',
 *             board.py:245-262), any other value = a piece no square holds
 *   move    = uint8 code, 0..63 = square, 64 = pass ('PS')      (board.py:192-209)
 *   legal   = uint64 bitboard; LSB-first order == puttables() row-major order
 *
 * Ownership / errors / threading:
 *   - every pointer is DEVICE memory owned by the caller (e.g. torch tensors);
 *     the library keeps no device state (the rollouts' work counter is a
 *     word the caller passes in, see oth_rollout) and allocates nothing:
 *     the TD calls that need scratch (oth_td_sort_pairs, oth_td_lookup,
 *     oth_td_merge) take it from the caller, with a size query;
 *   - calls are asynchronous on `stream` (a hipStream_t; NULL = default stream)
 *     and thread-safe on distinct streams; they may be captured in a hipGraph;
 *   - return value: OTH_OK (0), OTH_EINVAL (invalid argument, nothing launched),
 *     or -(hipError_t) of the failed launch.  Per-game semantics (illegal
 *     move ...) are reported in `ret`, never as a status.
 */
#ifndef SUBPROC_AMD_OTHELLO_H
#define SUBPROC_AMD_OTHELLO_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define OTH_OK 0
#define OTH_EINVAL (-1000)

#define OTH_BLACK 1
#define OTH_WHITE 2
#define OTH_PASS 64
#define OTH_HIST_BINS 133   /* [0..128] diff+64, 129 black wins, 130 white wins, 131 draws, 132 total plies */
#define OTH_MOVES_STRIDE 128 /* bytes per game in the optional rollout move record */
#define OTH_POS_STRIDE 129   /* positions per game in a replay (start + one per recorded move) */
#define OTH_BOOK_LINE 67     /* bytes per serialize_str() line incl. '\n' */
#define OTH_FEATURES 10      /* features per position of oth_features */

#define OTH_POLICY_RANDOM 0
#define OTH_POLICY_GREEDY 1  /* 1-ply minimise opponent mobility, ties -> lowest square */
#define OTH_POLICY_EVAL 2    /* 1-ply maximise the mover's linear eval (oth_eval), ties -> lowest square */

/* Linear evaluation weights: int8 [OTH_EVAL_PHASES][OTH_EVAL_FEATURES], row k
 * for positions whose disc count lies in learner shard k = (0..16, 17..32,
 * 33..48, 49..64) (progress_position_moves_learn.py:112-113), columns = the 9
 * non-phase counts() features (n_puttable_for, region masks a..h).  This is the
 * table ProgressPositionMovesLearn stores and paramgen.py writes (header byte,
 * 36 int8, trailing 0; paramgen.py:5-19). */
#define OTH_EVAL_PHASES 4
#define OTH_EVAL_FEATURES 9
#define OTH_EVAL_WEIGHTS 36

/* Library version string ("subproc_amd <semver> gfx950"). */
const char* oth_version(void);

/* Board.__init__ (board.py:22-27) for n games: opening position, turn = Black,
 * nturn = 0.  turn / nturn may be NULL. */
int oth_reset(uint64_t* boards, uint8_t* turn, uint8_t* nturn, int64_t n, void* stream);

/* Board.puttables(turn) (board.py:46-52) as a bitmask per game;
 * Board.n_puttable_for (54-55) = popcount.  turn 0 (Empty) -> puttables(Empty):
 * empty squares from which a run of Black discs ends on an empty square
 * (hostile(Empty) = Black, 155-159); any other turn outside {1,2} -> 0. */
int oth_legal(const uint64_t* boards, const uint8_t* turn, uint64_t* legal, int64_t n, void* stream);

/* Board.put_s (board.py:192-209) on integer move codes, one step per game:
 *   move == 64            -> ret 0, turn toggles (accepted even with legal moves)
 *   move 0..63, legal     -> ret = number of flipped discs (>= 1), board updated, turn toggles
 *   move 0..63, occupied or flips nothing -> ret -1, board and turn unchanged
 *   move > 64             -> ret -1, unchanged  (board.py raises IndexError for
 *                            'a9'/'i1', the strings no code 0..64 stands for)
 * "Toggles" is board.py's rule: Black -> White, anything else -> Black.  With
 * turn 0 (Empty) a move flips the Black runs that end on an empty square to
 * Empty (the origin stays empty); with any other turn outside {1,2} no move
 * flips anything (only a pass is accepted).
 * Outputs: boards_out (n,2), turn_out, flips (discs that changed, origin excluded),
 * legal_next = puttables(turn_out) on boards_out, ret.  Any output may be NULL.
 * boards_out may alias boards_in and turn_out may alias turn_in (in-place step).
 * nturn (may be NULL) is incremented in place where ret >= 0 (board.py:203-204);
 * it is a byte and wraps mod 256, where board.py's int does not (a game to its
 * end makes at most 60 placements plus its passes; only a caller that keeps
 * passing on purpose reaches 256).  The Board facade keeps nturn as an int. */
int oth_step(const uint64_t* boards_in, const uint8_t* turn_in, const uint8_t* move,
             uint64_t* boards_out, uint8_t* turn_out, uint64_t* flips, uint64_t* legal_next,
             int8_t* ret, uint8_t* nturn, int64_t n, void* stream);

/* n_black / n_white (board.py:37-41), diff = n_black - n_white (game_runner.py:194-199,
 * no empty-square bonus), terminal = is_game_over() (board.py:57-58).  Any output may be NULL. */
int oth_result(const uint64_t* boards, uint8_t* n_black, uint8_t* n_white, int8_t* diff,
               uint8_t* terminal, int64_t n, void* stream);

/* Board.hands_for_direc (board.py:124-139) from any origin (x[i], y[i]) along
 * any direction (dx[i], dy[i]) -- on the board, next to it or anywhere --
 * with own[i] = the squares holding the piece and hostile[i] = the squares
 * holding hostile(piece) (155-159).  count[i] = the length of the returned
 * list; its entries are the squares (x + k*dx, y + k*dy) for k = 1..count[i].
 * Off-board origins are what Python's list indexing lets Board.put /
 * is_puttable_at reach (x = -1 is file h for the emptiness test while the scan
 * starts at x = -1); a run of 8 hostile squares is kept without a closing
 * piece, as board.py's 8-step loop does. */
int oth_hands(const uint64_t* own, const uint64_t* hostile, const int64_t* x, const int64_t* y, const int64_t* dx,
              const int64_t* dy, uint8_t* count, int64_t n, void* stream);

/* Play n independent games to terminal (game_runner.py:165-201 loop, engines
 * replaced by `policy`; a side without a legal move passes).
 *   start / start_turn : (n,2) / (n) start positions; NULL = opening, Black to
 *                        move; a start_turn other than 2 (White) is Black
 *   seed, game_id0     : game i uses the RNG stream of global game id game_id0 + i
 *                         -> results independent of batch split / GPU count
 *   policy, n_random   : OTH_POLICY_RANDOM, or OTH_POLICY_GREEDY whose first
 *                        n_random plies are random
 * Outputs (each may be NULL): final_boards (n,2), diff (n), plies (n) = env-steps
 * incl. passes, moves (n * OTH_MOVES_STRIDE, 255-padded move codes),
 * hist (OTH_HIST_BINS int64, ACCUMULATED: caller zeroes it).
 *   work : ONE device uint64 owned by the caller (required): the launch's
 *          batch counter.  It must be 0 when the launch starts; the launch
 *          leaves it 0 when it completes.  So a word zeroed once serves any
 *          number of launches ordered on one stream (or replays of a graph),
 *          and launches that may run concurrently need distinct words.  After
 *          a failed or aborted launch, zero it again. */
int oth_rollout(const uint64_t* start, const uint8_t* start_turn, uint64_t seed, uint64_t game_id0,
                int policy, int n_random, uint64_t* final_boards, int8_t* diff, uint8_t* plies,
                uint8_t* moves, int64_t* hist, uint64_t* work, int64_t n, void* stream);

/* Launch geometry (diagnostic, no launch): the number of 256-thread blocks a
 * rollout of n games with `policy` launches on the current device -- its
 * resident-block count, at most one block per 256 games -- or OTH_EINVAL for
 * an unknown policy.  The CPU build returns 1. */
int oth_rollout_grid(int policy, int64_t n);

/* oth_rollout with the eval policy: after n_random random plies, each mover
 * plays the legal move whose child maximises oth_eval(child, mover) under
 * `weights` (HOST pointer to OTH_EVAL_WEIGHTS int8, copied into the launch, so
 * the caller may reuse it as soon as the call returns).  Other arguments and
 * outputs as oth_rollout. */
int oth_rollout_eval(const uint64_t* start, const uint8_t* start_turn, uint64_t seed, uint64_t game_id0,
                     int n_random, const int8_t* weights, uint64_t* final_boards, int8_t* diff, uint8_t* plies,
                     uint8_t* moves, int64_t* hist, uint64_t* work, int64_t n, void* stream);

/* A match between two eval tables (the GPU counterpart of GameRunner playing
 * engine A as Black against engine B as White, game_runner.py:154-201): as
 * oth_rollout_eval, but Black's moves use weights_black and White's moves
 * weights_white (both HOST pointers to OTH_EVAL_WEIGHTS int8, copied into the
 * launch).  oth_rollout_eval(w) == oth_rollout_match(w, w). */
int oth_rollout_match(const uint64_t* start, const uint8_t* start_turn, uint64_t seed, uint64_t game_id0,
                      int n_random, const int8_t* weights_black, const int8_t* weights_white, uint64_t* final_boards,
                      int8_t* diff, uint8_t* plies, uint8_t* moves, int64_t* hist, uint64_t* work, int64_t n,
                      void* stream);

/* Synthetic reachable mid-game positions for the step benchmark (config 2):
 * position index0+j is a random-policy playout of 10..49 plies from the opening
 * at which the mover has >= 1 legal move, plus that mover's random legal move
 * (DESIGN.md §Synthetic mid-game positions).  nturn may be NULL. */
int oth_sample_midgame(uint64_t seed, uint64_t index0, uint64_t* boards, uint8_t* turn,
                       uint8_t* nturn, uint8_t* move, int64_t n, void* stream);

/* ---- SURVEY.md §8f "next" rows ------------------------------------------ */

/* GameRunner's match schedule (game_runner.py:104-201 as subproc.do_match,
 * subproc.py:15-39, runs it) for n games between player A and player B, both
 * playing `policy`: OTH_POLICY_GREEDY, or OTH_POLICY_EVAL with the eval
 * tables weights_a / weights_b (HOST pointers, OTH_EVAL_WEIGHTS int8 each;
 * unused by greedy).  Per game, on its counter RNG stream:
 *  - colours: with swap_colours != 0 the first draw c = pick(2), and A plays
 *    White iff c == 1 (do_match's randrange(2), proc_randomize_black_white);
 *    otherwise A plays Black (proc_a is the black engine, 28-35);
 *  - random moves: each player starts with min(n_rand, 10) random moves to
 *    place (n_rand_a / n_rand_b = proc_n_rand_hands_for_a / _b; GameRunner
 *    caps the budget at N_RAND_HAND_UNTIL, 115-119).  On each of its turns --
 *    a placement or a pass -- a player with budget r > 0 draws c = pick(r);
 *    c == 0 and at least one legal move: it plays the legal move of index
 *    pick(#legal) in puttables order and r -= 1 (go_for, 133-150); otherwise
 *    it plays its policy's move, or passes.
 * a_black (n bytes, may be NULL) receives 1 where A played Black.  Everything
 * else as oth_rollout_match (diff, hist and final boards are by colour). */
int oth_rollout_runner(const uint64_t* start, const uint8_t* start_turn, uint64_t seed, uint64_t game_id0, int policy,
                       const int8_t* weights_a, const int8_t* weights_b, int n_rand_a, int n_rand_b, int swap_colours,
                       uint8_t* a_black, uint64_t* final_boards, int8_t* diff, uint8_t* plies, uint8_t* moves,
                       int64_t* hist, uint64_t* work, int64_t n, void* stream);

/* Book emitter, step 1: replay recorded move codes (a rollout's `moves`
 * record, or any put_s code list) into every recorded position, as
 * GameRunner records them (game_runner.py:169-184: after Board() and after each
 * put_s, put_s semantics incl. ignored illegal moves).  Game i's position p
 * (0 <= p <= plies[i], plies capped at OTH_MOVES_STRIDE) goes to row
 * i*OTH_POS_STRIDE + p of pos_boards (rows, 2 x u64), pos_turn and pos_end
 * (is_game_over(), board.py:57-58; game_recorder.py:111).  start/start_turn
 * NULL = opening.  pos_turn / pos_end may be NULL.  Every row of a game's
 * stride is written: rows past plies[i] are 0 in pos_boards, pos_turn and
 * pos_end. */
int oth_replay(const uint64_t* start, const uint8_t* start_turn, const uint8_t* moves, const uint8_t* plies,
               uint64_t* pos_boards, uint8_t* pos_turn, uint8_t* pos_end, int64_t n, void* stream);

/* oth_replay into packed rows: game i's position p (0 <= p <= plies[i], plies
 * capped at OTH_MOVES_STRIDE) goes to row row_off[i] + p of pos_boards,
 * pos_turn and pos_end, and only those rows are written -- the useful bytes,
 * about half of the strided table for random games.  row_off (device, n int64)
 * must be the exclusive prefix sum of min(plies[i], OTH_MOVES_STRIDE) + 1, so
 * the rows of all games are one contiguous range of row_off[n-1] +
 * min(plies[n-1], OTH_MOVES_STRIDE) + 1 rows (oth_book_text serialises them in
 * one call).  Other offsets are the caller's risk where rows overlap; games
 * with disjoint rows in any order are written correctly (a block whose games'
 * rows do not form one short range writes its bytes directly). */
int oth_replay_rows(const uint64_t* start, const uint8_t* start_turn, const uint8_t* moves, const uint8_t* plies,
                    const int64_t* row_off, uint64_t* pos_boards, uint8_t* pos_turn, uint8_t* pos_end, int64_t n,
                    void* stream);

/* Book emitter, step 2: serialize_str() (board.py:214-243: 64 chars O/X/-,
 * ' ', side O/X/-) + '\n' for n consecutive positions, concatenated into
 * out[n * OTH_BOOK_LINE] -- the body of FlatFileRecorder's file
 * (game_recorder.py:67-76). */
int oth_book_text(const uint64_t* boards, const uint8_t* turn, int64_t n, char* out, void* stream);

/* Book ingest, the reader's side of the same format (game_reader.py:60-75 /
 * replearn.learn_books, replearn.py:27-46): the board strings of n records --
 * 64 chars at text + i*stride, char k for square (k % 8, k / 8) -- into
 * boards[i] = {black, white} as Board.deserialize sets them on a fresh Board
 * (board.py:253-258 with turn_from_string, 245-251: 'O' Black, 'X' White, any
 * other byte Empty).  stride >= 64: 64 for packed strings, OTH_BOOK_LINE for
 * the serialize_str lines of a FlatFileRecorder file (game_recorder.py:67-76).
 * turn (may be NULL; needs stride >= 66) receives turn_from_string of byte 65,
 * the side after the board's space.  Replaces the per-record
 * board_from_a_book (parameter.py:5-8) of the learner. */
int oth_book_parse(const char* text, int64_t stride, uint64_t* boards, uint8_t* turn, int64_t n, void* stream);

/* Learner features: counts() of parameter_progress_position_moves_learn.py:5-17
 * for side[i] in {1 = 'O', 2 = 'X'}: out[i*10 + 0] = 64 - n_empty,
 * [1] = n_puttable_for(side), [2..9] = mask_count(side, region mask a..h). */
int oth_features(const uint64_t* boards, const uint8_t* side, uint8_t* out, int64_t n, void* stream);

/* Linear evaluation from side[i]'s view: out[i] = sum_j W[k][j] * counts()[1+j],
 * k = learner shard of counts()[0] (see OTH_EVAL_WEIGHTS) -- the model
 * ProgressPositionMovesLearn.fit_parameter fits (progress_position_moves_learn.py:160-184;
 * its intercept is not stored, so none is added).  weights: HOST pointer,
 * OTH_EVAL_WEIGHTS int8, copied into the launch. */
int oth_eval(const uint64_t* boards, const uint8_t* side, const int8_t* weights, int32_t* out, int64_t n,
             void* stream);

/* TD state map of ProgressPositionMovesLearn (progress_position_moves_learn.py:37-62),
 * step 1: the ordered update stream of n games.  Game g's recorded positions
 * (an oth_replay layout: row g*OTH_POS_STRIDE + p, p = 0..plies[g]) are visited
 * as learn_books orders a book (sorted by turn, reversed: terminal first,
 * replearn.py:36-38) and __update_state_for_a_book walks it (sides 'O' then
 * 'X'): update j = base[g] + 2*(plies[g] - p) + (0 for 'O', 1 for 'X') gets
 *   keys[j]   = OTH_TD_KEY(counts(position p, side))      (hash_from_book)
 *   values[j] = (double)value_side * lam_pow[plies[g] - p]   (value * l ** turn_left)
 * with value_O = n_black - n_white of the terminal position and value_X its
 * negation (41-42).  base (n, exclusive prefix sum of 2*(plies+1)) and lam_pow
 * (OTH_POS_STRIDE doubles, lam_pow[k] = l ** k as the host computes it) are
 * device arrays. */
#define OTH_TD_KEY_BITS 43
/* packed counts() key, each field as wide as its largest value: discs (0..64,
 * 7 bits) << 36 | moves (0..63, 6 bits) << 30 | the regions a..h (sizes 4, 8,
 * 4, 8, 8, 16, 4, 12: 3, 4, 3, 4, 4, 5, 3, 4 bits) at bits 27, 23, 20, 16,
 * 12, 7, 4, 0.  Integer order == tuple order; 43 bits are 5 radix passes of
 * the sort where the round-3 layout's 54 (5 bits per region) were 6. */
int oth_td_updates(const uint64_t* pos_boards, const uint8_t* plies, const int64_t* base, const double* lam_pow,
                   int64_t* keys, double* values, int64_t n, void* stream);
/* oth_td_updates over an oth_replay_rows table: game g's position p is row
 * row_off[g] + p (device, n int64). */
int oth_td_updates_rows(const uint64_t* pos_boards, const int64_t* row_off, const uint8_t* plies, const int64_t* base,
                        const double* lam_pow, int64_t* keys, double* values, int64_t n, void* stream);

/* oth_td_updates over book records in the learner's own order
 * (learn_and_update_batch -> __update_state_for_a_book,
 * progress_position_moves_learn.py:37-62, 94-96), for books from any source:
 * row r of rows (record boards, e.g. from oth_book_parse; books concatenated in
 * batch order, each book's records as given, terminal record first) is update
 * pair 2r ('O') and 2r + 1 ('X'):
 *   keys[2r + s]   = OTH_TD_KEY(counts(row r, side s))
 *   values[2r + s] = (double)value_s(rows[term_row[r]]) * lam_pow[lam_idx[r]]
 * term_row[r]: the row of r's book's first record (book[0], whose board gives
 * value_O = n_black - n_white and value_X = -value_O); lam_pow[lam_idx[r]]:
 * l ** (last_turn - turn) of the record, from the caller's table. */
int oth_td_updates_records(const uint64_t* rows, const int64_t* term_row, const int32_t* lam_idx,
                           const double* lam_pow, int64_t* keys, double* values, int64_t n_rows, void* stream);

/* TD state map, step 2: segment s (updates seg_off[s] .. seg_off[s+1]-1 of one
 * key, in stream order) starts from init[s] and applies, in order,
 *   v = (v == 0) ? x : v * one_minus_a + x * a          (58-61; no fused multiply-add)
 * out[s] = final v.  All arrays are device memory. */
int oth_td_ema(const double* values, const int64_t* seg_off, const double* init, double a, double one_minus_a,
               double* out, int64_t n_seg, void* stream);

/* oth_td_ema with the long segments split off: segments of length >= long_min
 * are each run by a whole wavefront, the others one per thread as in
 * oth_td_ema.  Such a wave runs a segment on one lane from LDS stages or, if
 * the rule contracts (|1 - a| < 1) and the segment is long enough, as parts
 * of ~1,000 updates on many waves from warm-up guesses of each part's start
 * state, each guess verified bit for bit and a part rerun when its guess
 * missed.  long_idx (device, n_long entries) must list every segment of
 * length >= long_min, in any order, each once; a segment that long missing
 * from it is left unwritten.  n_values = seg_off[n_seg], the length of
 * values; it sizes the split's scratch, and a smaller n_values only makes
 * the keys whose parts do not fit run unsplit (sequentially, same result;
 * nothing is written past the scratch).  temp / temp_bytes: device scratch of the split (its plan, the
 * parts' guesses and end states), the caller's; temp == NULL is a size query
 * (*temp_bytes receives the size for these n_long and n_values, nothing else
 * happens), otherwise *temp_bytes is the size of temp.  Same results as
 * oth_td_ema, bit for bit.  With OTH_TD_EMA_FORK=1 in the environment
 * (off by default) the long and split segments run on two high-priority
 * side streams of the device (created on first use, kept for the process)
 * beside the short segments' kernel on `stream`: they wait for what
 * `stream` had queued before the call, and `stream` waits for them before
 * anything queued after it, so to the caller the call is still ordered on
 * `stream` alone. */
int oth_td_ema_split(const double* values, const int64_t* seg_off, const double* init, double a,
                     double one_minus_a, double* out, int64_t n_seg, int64_t long_min, const int64_t* long_idx,
                     int64_t n_long, int64_t n_values, void* temp, size_t* temp_bytes, void* stream);

/* Packed updates (the GPU books' path, StateMap.update): the update stream
 * of oth_td_updates / oth_td_updates_rows (row_off NULL: the strided table)
 * with each update as one uint64 word,
 *   (value_side + 64) << 56 | turn_left << 36 | OTH_TD_SKEY,
 * turn_left = min(plies[g], OTH_MOVES_STRIDE) - p (0..128; the clamp
 * oth_td_updates applies too), value_side = +-(n_black - n_white) of
 * the terminal: the value is value_side * lam_pow[turn_left], exactly the
 * double oth_td_updates writes, and oth_td_unpack recomputes it.  Half the
 * bytes of a (key, value) pair, and the grouping sort becomes a keys-only
 * sort of these words by their low OTH_TD_SKEY_BITS (oth_td_sort_packed):
 * the payload rides along in the word's top bits.
 * OTH_TD_SKEY (round 5; round 4's words held the OTH_TD_KEY itself in 43
 * bits): the same counts() tuple numbered in an order-preserving mixed radix
 * of 36 bits, so the sort takes four radix passes of 9 bits, not five.  With
 * d discs, m moves (m <= 64 - d) and region counts r_a..r_h,
 *   OTH_TD_SKEY = ((tri(d) + m) * 5 + r_a) << 22
 *               | ((((((r_b * 5 + r_c) * 9 + r_d) * 9 + r_e) * 17 + r_f) * 5 + r_g) * 13 + r_h),
 *   tri(d) = 65 d - d (d - 1) / 2
 * (the region digits' bases are the region sizes + 1).  Skey order == key
 * order; the entry points that hand keys back (oth_td_unpack,
 * oth_td_sort_unpack, oth_td_segments_words) convert to OTH_TD_KEY. */
#define OTH_TD_SKEY_BITS 36
#define OTH_TD_PACK_TURN_SHIFT 36
#define OTH_TD_PACK_TURN_MASK 0xFFFFFu
#define OTH_TD_PACK_VALUE_SHIFT 56
int oth_td_updates_packed(const uint64_t* pos_boards, const int64_t* row_off, const uint8_t* plies,
                          const int64_t* base, uint64_t* words, int64_t n, void* stream);
/* Stable sort of n packed words by bits 0..OTH_TD_SKEY_BITS-1 (the skey):
 * equal keys keep their stream order; words_out distinct from words_in.
 * temp / temp_bytes as oth_td_sort_pairs.  (rocPRIM's onesweep radix sort,
 * 4 passes of 9 bits: the one vendor kernel of the library, DESIGN.md.) */
int oth_td_sort_packed(const uint64_t* words_in, uint64_t* words_out, int64_t n, void* temp, size_t* temp_bytes,
                       void* stream);
/* oth_td_sort_packed followed by oth_td_unpack in one: the sorted words'
 * keys and values (keys[i] = the OTH_TD_KEY of the i-th sorted word's skey,
 * values[i] = value_side * lam_pow[turn_left]), the last radix pass writing
 * them directly.  keys distinct from words_in.  temp / temp_bytes as
 * oth_td_sort_pairs (round 5). */
int oth_td_sort_unpack(const uint64_t* words_in, const double* lam_pow, int64_t* keys, double* values, int64_t n,
                       void* temp, size_t* temp_bytes, void* stream);
/* The segments of a key-sorted update stream (what StateMap.update groups
 * by): counts[0] = n_seg, the number of distinct keys; seg_off[0..n_seg] the
 * offsets of their runs (seg_off[j] = first index of key j, seg_off[n_seg]
 * = n); ukeys[0..n_seg) the keys; long_idx[0..counts[1]) the indices j of
 * the segments of >= long_min updates, in increasing order (what
 * oth_td_ema_split takes).  seg_off holds n + 1 entries, ukeys and long_idx
 * n (capacities: the counts are known only after the call); counts (2
 * int64) is device memory, like the rest.  temp / temp_bytes as
 * oth_td_sort_pairs.  Replaces torch's unique_consecutive + cumsum +
 * nonzero (and their two host syncs). */
int oth_td_segments(const int64_t* keys, int64_t n, int64_t long_min, int64_t* seg_off, int64_t* ukeys,
                    int64_t* long_idx, int64_t* counts, void* temp, size_t* temp_bytes, void* stream);
/* oth_td_segments over the skey-sorted packed words themselves (each read as
 * its low OTH_TD_SKEY_BITS; ukeys receives OTH_TD_KEY values), also
 * writing values[i] = value_side * lam_pow[turn_left] of word i
 * (oth_td_unpack's rule), so a sorted word stream needs no unpack pass: the keys array oth_td_segments reads is never
 * formed (round 5).  values: n doubles (device); the rest as oth_td_segments. */
int oth_td_segments_words(const uint64_t* words, const double* lam_pow, int64_t n, int64_t long_min, int64_t* seg_off,
                          int64_t* ukeys, int64_t* long_idx, int64_t* counts, double* values, void* temp,
                          size_t* temp_bytes, void* stream);

/* new_before[j] = the number of nonzero is_new[0..j) for j = 0..n (n + 1
 * entries, device): oth_td_merge's new_before from oth_td_lookup's is_new.
 * temp / temp_bytes as oth_td_sort_pairs. */
int oth_td_new_before(const uint8_t* is_new, int64_t n, int64_t* new_before, void* temp, size_t* temp_bytes,
                      void* stream);

/* Packed words -> keys[i] = the OTH_TD_KEY of the word's skey and values[i] =
 * value_side * lam_pow[turn_left] (lam_pow: OTH_POS_STRIDE doubles, device).
 * Every entry point that reads a word's turn_left (this one,
 * oth_td_sort_unpack, oth_td_segments_words) clamps it to OTH_POS_STRIDE - 1,
 * so words not made by oth_td_updates_packed never read past lam_pow. */
int oth_td_unpack(const uint64_t* words, const double* lam_pow, int64_t* keys, double* values, int64_t n,
                  void* stream);

/* The number of packed words whose turn_left exceeded the lam_pow table
 * (clamped, as above) that oth_td_unpack, oth_td_sort_unpack and
 * oth_td_segments_words have read on the current device since the last reset
 * (a device-side counter): 0 for every word array oth_td_updates_packed
 * wrote.  *count (host memory) receives it once the work queued on `stream`
 * so far is done (the call synchronizes the stream); reset != 0 zeroes it. */
int oth_td_word_errors(uint64_t* count, int reset, void* stream);

/* The grouping sort between oth_td_updates and oth_td_ema: the n (key, value)
 * pairs of the update stream into key order, stable (a key's values keep
 * their stream order), keys_out/vals_out distinct from the inputs.  Keys must
 * be OTH_TD_KEY values (non-negative, below 2^OTH_TD_KEY_BITS).  temp == NULL
 * is a size query: *temp_bytes receives the scratch size (device memory, the
 * caller's) for n pairs and nothing else happens; otherwise *temp_bytes is the
 * size of temp.  Replaces the sort of the updates in learner order by key that
 * __update_state_for_a_book's per-key EMA implies (37-62). */
int oth_td_sort_pairs(const int64_t* keys_in, const double* vals_in, int64_t* keys_out, double* vals_out, int64_t n,
                      void* temp, size_t* temp_bytes, void* stream);

/* Sums for the learner's regression (fit_parameter,
 * progress_position_moves_learn.py:160-184) over n states of one shard, keys
 * (OTH_TD_KEY values) and values: x = counts()[1..9] of the key, y = value.
 * mean == NULL (pass 1): row r of partials gets, for its share of the states,
 *   [0] n, [1..9] sum x, [10] sum y.
 * mean = (mean x[0..8], mean y) (pass 2): row r gets
 *   [0..44] sum (x - mean x)(x - mean x)^T, upper triangle row by row,
 *   [45..53] sum (x - mean x)(y - mean y).
 * partials: OTH_TD_FIT_BLOCKS rows of OTH_TD_FIT_COLS doubles (device); the
 * first 11 (pass 1) or 54 (pass 2) entries of every row are written, and the
 * sum of the rows (in any fixed order) is the result. */
#define OTH_TD_FIT_BLOCKS 1024
#define OTH_TD_FIT_COLS 64
int oth_td_fit_moments(const int64_t* keys, const double* values, int64_t n, const double* mean,
                       double* partials, void* stream);

/* The batch's keys in the table: old_keys (n_old, unique, ascending) with
 * old_vals, upd_keys (n_upd, unique, ascending).  init[j] = the table value of
 * upd_keys[j], 0.0 if absent (a fresh key reads as 0, 53-56); is_new[j] = 1
 * if absent, else 0 (its cumsum is oth_td_merge's new_before).
 * temp / temp_bytes: device scratch for the merge path's tile splits, as
 * oth_td_sort_pairs: temp == NULL is a size query (*temp_bytes is set from
 * n_old and n_upd alone; nothing is read or launched); otherwise *temp_bytes
 * must be at least that size (any non-NULL temp when it is 0).  The library
 * allocates nothing. */
int oth_td_lookup(const int64_t* old_keys, const double* old_vals, int64_t n_old, const int64_t* upd_keys,
                  int64_t n_upd, double* init, uint8_t* is_new, void* temp, size_t* temp_bytes, void* stream);
/* oth_td_lookup with the batch's key count read from device memory when the
 * call runs on the stream: *n_upd_dev (one int64, device; clamped to
 * [0, n_upd_max]) is n_upd, e.g. the counts[0] that oth_td_segments(_words)
 * wrote just before, so the lookup can be queued behind the segments pass
 * before the host has read that count (round 5: the host's read then
 * overlaps the lookup).  Scratch (size query from n_old and n_upd_max) and
 * the arrays are sized for n_upd_max; init / is_new past the count are left
 * as they were.  Same results as oth_td_lookup with n_upd = *n_upd_dev. */
int oth_td_lookup_dev(const int64_t* old_keys, const double* old_vals, int64_t n_old, const int64_t* upd_keys,
                      int64_t n_upd_max, const int64_t* n_upd_dev, double* init, uint8_t* is_new, void* temp,
                      size_t* temp_bytes, void* stream);

/* The batch's results into the table: old_keys (n_old, unique, ascending) with
 * old_vals, and upd_keys (n_upd, unique, ascending) with their new values
 * upd_vals, merged into out_keys / out_vals, ascending; a key in both lists
 * appears once, with its upd value.  new_before (n_upd + 1 entries) counts
 * the batch keys absent from the table: new_before[j] = how many of
 * upd_keys[0..j) are not in old_keys.  The output has n_old +
 * new_before[n_upd] entries and must not overlap the inputs.  Keys are
 * OTH_TD_KEY values.  This is the store write of every updated key
 * (progress_position_moves_learn.py:58-62) for a whole batch.
 * new_before must be the exclusive cumsum of oth_td_lookup's is_new for the
 * same two key lists: for any other array the GPU build's output is undefined
 * (slots may stay unwritten), while the host build returns OTH_EINVAL.
 * temp / temp_bytes: as oth_td_lookup's (its own size query). */
int oth_td_merge(const int64_t* old_keys, const double* old_vals, int64_t n_old, const int64_t* upd_keys,
                 const double* upd_vals, const int64_t* new_before, int64_t n_upd, int64_t* out_keys,
                 double* out_vals, void* temp, size_t* temp_bytes, void* stream);
/* oth_td_merge without its own scratch: lookup_temp is the temp of an
 * oth_td_lookup / oth_td_lookup_dev call over the same old_keys and
 * upd_keys (for _dev, with *n_upd_dev == n_upd), queued before this call
 * and not reused since.  The lookup and the merge cut the merged sequence
 * into the same tiles, so the lookup's scratch already holds the merge path's
 * splits: the GPU build reads them instead of searching again (round 5).
 * The host build ignores lookup_temp.  Same output as oth_td_merge. */
int oth_td_merge_after_lookup(const int64_t* old_keys, const double* old_vals, int64_t n_old, const int64_t* upd_keys,
                              const double* upd_vals, const int64_t* new_before, int64_t n_upd, int64_t* out_keys,
                              double* out_vals, const void* lookup_temp, void* stream);

#ifdef __cplusplus
}
#endif

#endif /* SUBPROC_AMD_OTHELLO_H */
