/*
 * othello_oracle.c — CPU restatement of ysnrkdm/subproc board.py (the parity
 * ORACLE).  TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke()
 * and bench.py's cpu_baseline leg, never by the product path (subproc_amd/).
 *
 * Pinned against the reference: tests/test_oracle.py checks every function here
 * against the tests/golden fixtures, which tests/golden/gen_golden.py produced by running
 * the real /root/reference/board.py (SURVEY.md §8c shim).
 *
 * Deliberately NOT a bitboard implementation: it follows board.py's own
 * algorithm — an 8x8 mailbox ``board[y][x]`` scanned ray by ray from every
 * cell — so the GPU's Kogge-Stone bitboards are checked against an independent
 * formulation.  Bitboards appear only at the API boundary (sq = x + 8*y,
 * SURVEY.md §8 conventions: board.py:74-81 mask_count defines the bit order).
 *
 * API mirrors include/othello.h with host pointers, prefix ``oracle_`` and no
 * stream argument.
 */
#include <stdint.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

enum { Empty = 0, Black = 1, White = 2 };  /* board.py:3-7 */
#define PASS_CODE 64
#define HIST_BINS 133
#define MOVES_STRIDE 128

/* DIRECS, board.py:9-17 — order LU, U, RU, L, R, LD, D, RD */
static const int DIRECS[8][2] = {{-1, -1}, {0, -1}, {1, -1}, {-1, 0}, {1, 0}, {-1, 1}, {0, 1}, {1, 1}};

typedef struct {
    int8_t b[8][8]; /* board[y][x], board.py:23 */
    int turn;       /* board.py:26 */
    int nturn;      /* board.py:27 */
} Board;

/* board.py:265-266 */
static int is_within_board(int x, int y) { return 0 <= x && x < 8 && 0 <= y && y < 8; }

/* board.py:155-159 */
static int hostile(int piece) { return piece == Black ? White : Black; }

/* board.py:22-27 */
static void board_init(Board* s) {
    memset(s->b, Empty, sizeof s->b);
    s->b[3][3] = s->b[4][4] = White;
    s->b[3][4] = s->b[4][3] = Black;
    s->turn = Black;
    s->nturn = 0;
}

static void board_from_bits(Board* s, uint64_t bl, uint64_t wh, int turn) {
    for (int y = 0; y < 8; y++)
        for (int x = 0; x < 8; x++) {
            int sq = x + 8 * y;
            s->b[y][x] = (bl >> sq & 1) ? Black : (wh >> sq & 1) ? White : Empty;
        }
    s->turn = turn;
    s->nturn = 0;
}

static void board_to_bits(const Board* s, uint64_t* bl, uint64_t* wh) {
    uint64_t B = 0, W = 0;
    for (int y = 0; y < 8; y++)
        for (int x = 0; x < 8; x++) {
            if (s->b[y][x] == Black) B |= 1ull << (x + 8 * y);
            else if (s->b[y][x] == White) W |= 1ull << (x + 8 * y);
        }
    *bl = B;
    *wh = W;
}

/* hands_for_direc, board.py:124-139: hostile discs along one ray that end in
 * an own disc; empty/edge discards the ray.  Writes squares to out, returns count. */
static int hands_for_direc(const Board* s, int d, int piece, int x, int y, int out[8][2]) {
    int n = 0, h = hostile(piece);
    for (int i = 1; i < 9; i++) {
        int nx = x + i * DIRECS[d][0], ny = y + i * DIRECS[d][1];
        if (is_within_board(nx, ny) && s->b[ny][nx] == h) {
            out[n][0] = nx;
            out[n][1] = ny;
            n++;
        } else if (is_within_board(nx, ny) && s->b[ny][nx] == piece) {
            break;
        } else {
            n = 0;
            break;
        }
    }
    return n;
}

/* is_puttable_at, board.py:141-149 */
static int is_puttable_at(const Board* s, int piece, int x, int y) {
    if (s->b[y][x] != Empty) return 0;
    int tmp[8][2], n = 0;
    for (int d = 0; d < 8; d++) n += hands_for_direc(s, d, piece, x, y, tmp);
    return n > 0;
}

/* puttables, board.py:46-52, as a bitmask; row-major scan order == LSB-first */
static uint64_t puttables(const Board* s, int piece) {
    uint64_t m = 0;
    for (int y = 0; y < 8; y++)
        for (int x = 0; x < 8; x++)
            if (is_puttable_at(s, piece, x, y)) m |= 1ull << (x + 8 * y);
    return m;
}

static int popcount64(uint64_t m) { return __builtin_popcountll(m); }

/* n_puttable_for, board.py:54-55 */
static int n_puttable_for(const Board* s, int piece) { return popcount64(puttables(s, piece)); }

/* is_game_over, board.py:57-58 (short-circuit kept) */
static int is_game_over(const Board* s) { return n_puttable_for(s, Black) == 0 && n_puttable_for(s, White) == 0; }

/* put, board.py:161-174: returns total flipped count, 0 = illegal (no change) */
static int put(Board* s, int piece, int x, int y) {
    if (s->b[y][x] != Empty) return 0;
    int count = 0, hands[8][2];
    for (int d = 0; d < 8; d++) {
        int n = hands_for_direc(s, d, piece, x, y, hands);
        if (n) {
            for (int k = 0; k < n; k++) s->b[hands[k][1]][hands[k][0]] = (int8_t)piece; /* set_hands 151-153 */
            count += n;
            s->b[y][x] = (int8_t)piece;
        }
    }
    return count;
}

/* put_s, board.py:192-209, on the integer move code (0..63 = x+8y, 64 = 'PS').
 * Codes > 64 correspond to no string board.py accepts without IndexError;
 * the C-ABI contract returns -1 for them. */
static int put_code(Board* s, int code) {
    int out = -1;
    if (code == PASS_CODE) {
        out = 0;
    } else if (code >= 0 && code < 64) {
        out = put(s, s->turn, code % 8, code / 8);
        if (out == 0) out = -1;
    }
    if (out >= 0) {
        s->nturn += 1;
        s->turn = (s->turn == Black) ? White : Black;
    }
    return out;
}

static int n_of(const Board* s, int c) {
    int n = 0; /* count_over_board, board.py:29-44 */
    for (int y = 0; y < 8; y++)
        for (int x = 0; x < 8; x++) n += s->b[y][x] == c;
    return n;
}

/* ------------------------------------------------------------------------ */
/* RNG spec (Python twin in tests/golden/gen_golden.py)      */
/* ------------------------------------------------------------------------ */
#define GOLDEN64 0x9E3779B97F4A7C15ull
static uint64_t mix64(uint64_t z) {
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}
static uint64_t seed_state(uint64_t seed) { return mix64(seed + GOLDEN64); }
static uint64_t game_key(uint64_t S, uint64_t g) { return mix64(S + g * GOLDEN64); }
/* per-game draw stream: 32-bit LCG, state0 = lo32(key), increment = hi32(key) | 1 */
#define LCG_MUL 0x915F77F5u
typedef struct { uint32_t state, inc; } GameRng;
static GameRng rng_init(uint64_t key) { GameRng r = {(uint32_t)key, (uint32_t)(key >> 32) | 1u}; return r; }
static uint32_t rng_draw(GameRng* r) { r->state = r->state * LCG_MUL + r->inc; return r->state; }
static int rng_pick(GameRng* r, int n) { return (int)(((uint64_t)rng_draw(r) * (uint64_t)n) >> 32); }

/* k-th entry of puttables() (row-major list), as a square code */
static int kth_square(uint64_t legal, int k) {
    for (int sq = 0; sq < 64; sq++)
        if (legal >> sq & 1) {
            if (k == 0) return sq;
            k--;
        }
    return -1;
}

/* ------------------------------------------------------------------------ */
/* exported API                                                             */
/* ------------------------------------------------------------------------ */
int oracle_reset(uint64_t* boards, uint8_t* turn, uint8_t* nturn, int64_t n) {
    Board s;
    board_init(&s);
    uint64_t bl, wh;
    board_to_bits(&s, &bl, &wh);
    for (int64_t i = 0; i < n; i++) {
        boards[2 * i] = bl;
        boards[2 * i + 1] = wh;
        if (turn) turn[i] = (uint8_t)s.turn;
        if (nturn) nturn[i] = (uint8_t)s.nturn;
    }
    return 0;
}

int oracle_legal(const uint64_t* boards, const uint8_t* turn, uint64_t* legal, int64_t n) {
#pragma omp parallel for schedule(static)
    for (int64_t i = 0; i < n; i++) {
        Board s;
        board_from_bits(&s, boards[2 * i], boards[2 * i + 1], turn[i]);
        legal[i] = puttables(&s, turn[i]); /* any piece value, as board.py (Empty: hostile = Black) */
    }
    return 0;
}

int oracle_step(const uint64_t* boards_in, const uint8_t* turn_in, const uint8_t* move, uint64_t* boards_out,
                uint8_t* turn_out, uint64_t* flips, uint64_t* legal_next, int8_t* ret, uint8_t* nturn, int64_t n) {
#pragma omp parallel for schedule(static)
    for (int64_t i = 0; i < n; i++) {
        Board s;
        uint64_t b0 = boards_in[2 * i], w0 = boards_in[2 * i + 1];
        int t = turn_in[i];
        board_from_bits(&s, b0, w0, t);
        int r = put_code(&s, move[i]); /* any side to move, as board.py */
        uint64_t bl, wh;
        board_to_bits(&s, &bl, &wh);
        if (boards_out) {
            boards_out[2 * i] = bl;
            boards_out[2 * i + 1] = wh;
        }
        if (turn_out) turn_out[i] = (uint8_t)s.turn;
        /* flipped discs = squares that changed (origin excluded) */
        if (flips) flips[i] = ((b0 ^ bl) | (w0 ^ wh)) & ~(move[i] < 64 ? 1ull << move[i] : 0ull);
        if (legal_next) legal_next[i] = puttables(&s, s.turn);
        if (ret) ret[i] = (int8_t)r;
        if (nturn && r >= 0) nturn[i] = (uint8_t)(nturn[i] + 1); /* board.py:203-204 */
    }
    return 0;
}

int oracle_result(const uint64_t* boards, uint8_t* n_black, uint8_t* n_white, int8_t* diff, uint8_t* terminal,
                  int64_t n) {
#pragma omp parallel for schedule(static)
    for (int64_t i = 0; i < n; i++) {
        Board s;
        board_from_bits(&s, boards[2 * i], boards[2 * i + 1], Black);
        int nb = n_of(&s, Black), nw = n_of(&s, White);
        if (n_black) n_black[i] = (uint8_t)nb;
        if (n_white) n_white[i] = (uint8_t)nw;
        if (diff) diff[i] = (int8_t)(nb - nw); /* game_runner.py:194-199 rule, no empty bonus */
        if (terminal) terminal[i] = (uint8_t)is_game_over(&s);
    }
    return 0;
}

/* mask_count, board.py:74-81 */
static int mask_count(const Board* s, int color, uint64_t mask) {
    int ret = 0;
    for (int i = 0; i < 8; i++)
        for (int j = 0; j < 8; j++)
            if (((mask >> (j + i * 8)) & 1) && s->b[i][j] == color) ret++;
    return ret;
}

/* counts(), parameter_progress_position_moves_learn.py:5-17 for side t (1 = 'O', 2 = 'X') */
static void counts(const Board* s, int t, int o[10]) {
    static const uint64_t masks[8] = {0x8100000000000081ull, 0x4281000000008142ull, 0x0042000000004200ull,
                                      0x2400810000810024ull, 0x1800008181000018ull, 0x003C424242423C00ull,
                                      0x0000240000240000ull, 0x0000183C3C180000ull};
    o[0] = 64 - n_of(s, Empty);
    o[1] = n_puttable_for(s, t); /* any piece value, as board.py (Empty: hostile = Black) */
    for (int k = 0; k < 8; k++) o[2 + k] = mask_count(s, t, masks[k]);
}

/* linear eval of the learner's model: weights row = shard of counts()[0]
 * (0..16, 17..32, 33..48, 49..64: progress_position_moves_learn.py:112-113),
 * columns = counts()[1..9] (fit in progress_position_moves_learn.py:160-184) */
static int eval_of(const Board* s, int t, const int8_t* w) {
    int o[10];
    counts(s, t, o);
    int shard = o[0] <= 16 ? 0 : o[0] <= 32 ? 1 : o[0] <= 48 ? 2 : 3;
    int v = 0;
    for (int j = 0; j < 9; j++) v += (int)w[shard * 9 + j] * o[1 + j];
    return v;
}

/* GameRunner's match schedule (game_runner.py:104-152, subproc.py:15-39;
 * include/othello.h oth_rollout_runner): NULL = the plain rollouts' rule (the
 * first n_random plies random for both sides). */
typedef struct {
    int n_rand_a, n_rand_b; /* proc_n_rand_hands_for_a / _b */
    int swap;               /* proc_randomize_black_white */
    const int8_t *w_a, *w_b;
} Runner;

/* One game to terminal from s, game_runner.py:165-201 loop with the build's
 * policies: a side with no move passes ('PS').  With a
 * runner schedule: the colour draw first (subproc.py:28-32), then on each turn
 * of a player with random budget left a coin pick(budget); 0 with a legal move
 * plays puttables[pick(#legal)] and spends one (go_for, game_runner.py:133-150).
 * *a_black (runner only) = 1 where player A played Black. */
static int play_game(Board* s, uint64_t key, int policy, int n_random, const int8_t* w, const int8_t* w_white,
                     uint8_t* moves, const Runner* run, uint8_t* a_black) {
    int ply = 0;
    GameRng rng = rng_init(key);
    int rem[3] = {0, 0, 0}; /* random budget left, by colour (Black = 1, White = 2) */
    if (run) {
        int ab = 1;
        if (run->swap && rng_pick(&rng, 2) == 1) ab = 0; /* do_match swapped proc_a and proc_b */
        int ra = run->n_rand_a < 10 ? run->n_rand_a : 10, rb = run->n_rand_b < 10 ? run->n_rand_b : 10;
        rem[Black] = ab ? ra : rb;
        rem[White] = ab ? rb : ra;
        w = ab ? run->w_a : run->w_b;       /* Black's table */
        w_white = ab ? run->w_b : run->w_a; /* White's table */
        if (a_black) *a_black = (uint8_t)ab;
    }
    while (!is_game_over(s)) {
        uint64_t legal = puttables(s, s->turn);
        int code;
        int coin_random = 0;
        if (run && (s->turn == Black || s->turn == White) && rem[s->turn] > 0 &&
            rng_pick(&rng, rem[s->turn]) == 0 && legal) {
            coin_random = 1;
            rem[s->turn]--;
        }
        if (!legal) {
            code = PASS_CODE;
        } else if (coin_random || (!run && (policy == 0 || ply < n_random))) {
            code = kth_square(legal, rng_pick(&rng, popcount64(legal)));
        } else if (policy == 1) { /* greedy: minimise the opponent's mobility */
            int best = -1, bestv = 1 << 30;
            for (int sq = 0; sq < 64; sq++) {
                if (!(legal >> sq & 1)) continue;
                Board c = *s;
                put_code(&c, sq);
                int v = n_puttable_for(&c, hostile(s->turn));
                if (v < bestv) { bestv = v; best = sq; }
            }
            code = best;
        } else { /* eval: maximise the mover's linear eval of the child */
            int best = -1, bestv = -(1 << 30);
            for (int sq = 0; sq < 64; sq++) {
                if (!(legal >> sq & 1)) continue;
                Board c = *s;
                put_code(&c, sq);
                int v = eval_of(&c, s->turn, s->turn == White ? w_white : w);
                if (v > bestv) { bestv = v; best = sq; }
            }
            code = best;
        }
        int r = put_code(s, code);
        (void)r;
        if (moves && ply < MOVES_STRIDE) moves[ply] = (uint8_t)code;
        ply++;
    }
    return ply;
}

/* policy 0 random, 1 greedy, 2 eval (weights: int8[36], used by policy 2 only;
 * weights_white NULL = White uses `weights` too, else White's table: a match) */
static int rollout_any(const uint64_t* start, const uint8_t* start_turn, uint64_t seed, uint64_t game_id0,
                       int policy, int n_random, uint64_t* final_boards, int8_t* diff, uint8_t* plies,
                       uint8_t* moves, int64_t* hist, int64_t n, int n_threads, const int8_t* weights,
                       const int8_t* weights_white, const Runner* run, uint8_t* a_black);

int oracle_rollout(const uint64_t* start, const uint8_t* start_turn, uint64_t seed, uint64_t game_id0, int policy,
                   int n_random, uint64_t* final_boards, int8_t* diff, uint8_t* plies, uint8_t* moves,
                   int64_t* hist, int64_t n, int n_threads, const int8_t* weights, const int8_t* weights_white) {
    return rollout_any(start, start_turn, seed, game_id0, policy, n_random, final_boards, diff, plies, moves, hist,
                       n, n_threads, weights, weights_white, 0, 0);
}

/* GameRunner matches (oth_rollout_runner): policy 1 greedy or 2 eval for both
 * players, A's and B's eval tables, random budgets and colour swap */
int oracle_rollout_runner(const uint64_t* start, const uint8_t* start_turn, uint64_t seed, uint64_t game_id0,
                          int policy, const int8_t* weights_a, const int8_t* weights_b, int n_rand_a, int n_rand_b,
                          int swap, uint8_t* a_black, uint64_t* final_boards, int8_t* diff, uint8_t* plies,
                          uint8_t* moves, int64_t* hist, int64_t n, int n_threads) {
    if ((policy != 1 && policy != 2) || (policy == 2 && (!weights_a || !weights_b)) || n_rand_a < 0 || n_rand_b < 0)
        return -1;
    Runner run = {n_rand_a, n_rand_b, swap != 0, weights_a, weights_b};
    return rollout_any(start, start_turn, seed, game_id0, policy, 0, final_boards, diff, plies, moves, hist, n,
                       n_threads, weights_a, weights_b, &run, a_black);
}

static int rollout_any(const uint64_t* start, const uint8_t* start_turn, uint64_t seed, uint64_t game_id0,
                       int policy, int n_random, uint64_t* final_boards, int8_t* diff, uint8_t* plies,
                       uint8_t* moves, int64_t* hist, int64_t n, int n_threads, const int8_t* weights,
                       const int8_t* weights_white, const Runner* run, uint8_t* a_black) {
    if (policy == 2 && !weights) return -1;
    if (!weights_white) weights_white = weights;
    uint64_t S = seed_state(seed);
    int64_t h[HIST_BINS];
    memset(h, 0, sizeof h);
#ifdef _OPENMP
    if (n_threads <= 0) n_threads = omp_get_max_threads();
#pragma omp parallel num_threads(n_threads)
#endif
    {
        int64_t hl[HIST_BINS];
        memset(hl, 0, sizeof hl);
#pragma omp for schedule(dynamic, 64)
        for (int64_t i = 0; i < n; i++) {
            Board s;
            /* the build's rollouts start with Black or White to move (include/othello.h) */
            if (start)
                board_from_bits(&s, start[2 * i], start[2 * i + 1],
                                start_turn && start_turn[i] == White ? White : Black);
            else board_init(&s);
            if (moves) memset(moves + i * MOVES_STRIDE, 255, MOVES_STRIDE);
            int p = play_game(&s, game_key(S, game_id0 + (uint64_t)i), policy, n_random, weights, weights_white,
                              moves ? moves + i * MOVES_STRIDE : 0, run, a_black ? a_black + i : 0);
            int d = n_of(&s, Black) - n_of(&s, White);
            uint64_t bl, wh;
            board_to_bits(&s, &bl, &wh);
            if (final_boards) {
                final_boards[2 * i] = bl;
                final_boards[2 * i + 1] = wh;
            }
            if (diff) diff[i] = (int8_t)d;
            if (plies) plies[i] = (uint8_t)p;
            hl[d + 64]++;
            hl[d > 0 ? 129 : d < 0 ? 130 : 131]++;
            hl[132] += p;
        }
#pragma omp critical
        for (int k = 0; k < HIST_BINS; k++) h[k] += hl[k];
    }
    if (hist)
        for (int k = 0; k < HIST_BINS; k++) hist[k] += h[k];
    return 0;
}

/* the games of explicit global ids (a strided sample of a large launch): game
 * j is the game oracle_rollout plays as id ids[j], from the opening */
int oracle_rollout_ids(const uint64_t* ids, int64_t n, uint64_t seed, int policy, int n_random,
                       const int8_t* weights, const int8_t* weights_white, uint64_t* final_boards, int8_t* diff,
                       uint8_t* plies) {
    if (policy == 2 && !weights) return -1;
    if (!weights_white) weights_white = weights;
    uint64_t S = seed_state(seed);
#pragma omp parallel for schedule(dynamic, 16)
    for (int64_t j = 0; j < n; j++) {
        Board s;
        board_init(&s);
        int p = play_game(&s, game_key(S, ids[j]), policy, n_random, weights, weights_white, 0, 0, 0);
        board_to_bits(&s, &final_boards[2 * j], &final_boards[2 * j + 1]);
        diff[j] = (int8_t)(n_of(&s, Black) - n_of(&s, White));
        plies[j] = (uint8_t)p;
    }
    return 0;
}

/* Synthetic mid-game position generator for the config-2 step benchmark
 * (DESIGN.md §Synthetic mid-game positions; Python twin in gen_golden.py). */
int oracle_sample_midgame(uint64_t seed, uint64_t index0, uint64_t* boards, uint8_t* turn, uint8_t* nturn,
                          uint8_t* move, int64_t n) {
    uint64_t S = seed_state(seed);
#pragma omp parallel for schedule(dynamic, 64)
    for (int64_t j = 0; j < n; j++) {
        uint64_t i = index0 + (uint64_t)j;
        for (uint64_t attempt = 0;; attempt++) {
            GameRng rng = rng_init(game_key(S, i ^ (attempt << 48)));
            int target = 10 + rng_pick(&rng, 40); /* the first draw picks the stopping ply */
            Board s;
            board_init(&s);
            int ply = 0, ok = 0;
            while (!is_game_over(&s)) {
                uint64_t legal = puttables(&s, s.turn);
                if (ply >= target && legal) { ok = 1; break; }
                int code = legal ? kth_square(legal, rng_pick(&rng, popcount64(legal))) : PASS_CODE;
                put_code(&s, code);
                ply++;
            }
            if (ok) {
                uint64_t legal = puttables(&s, s.turn);
                board_to_bits(&s, &boards[2 * j], &boards[2 * j + 1]);
                turn[j] = (uint8_t)s.turn;
                if (nturn) nturn[j] = (uint8_t)ply;
                move[j] = (uint8_t)kth_square(legal, rng_pick(&rng, popcount64(legal)));
                break;
            }
        }
    }
    return 0;
}

/* counts(), parameter_progress_position_moves_learn.py:5-17 (side 1 = 'O', 2 = 'X') */
int oracle_features(const uint64_t* boards, const uint8_t* side, uint8_t* out, int64_t n) {
#pragma omp parallel for schedule(static)
    for (int64_t i = 0; i < n; i++) {
        Board s;
        board_from_bits(&s, boards[2 * i], boards[2 * i + 1], side[i]);
        int o[10];
        counts(&s, side[i], o);
        for (int k = 0; k < 10; k++) out[i * 10 + k] = (uint8_t)o[k];
    }
    return 0;
}

/* the learner's linear eval from side[i]'s view (eval_of) */
int oracle_eval(const uint64_t* boards, const uint8_t* side, const int8_t* weights, int32_t* out, int64_t n) {
#pragma omp parallel for schedule(static)
    for (int64_t i = 0; i < n; i++) {
        Board s;
        board_from_bits(&s, boards[2 * i], boards[2 * i + 1], side[i]);
        out[i] = eval_of(&s, side[i], weights);
    }
    return 0;
}

/* recorded positions of a move list, game_runner.py:169-184 (put_s semantics) */
int oracle_replay(const uint64_t* start, const uint8_t* start_turn, const uint8_t* moves, const uint8_t* plies,
                  uint64_t* pos, uint8_t* pos_turn, uint8_t* pos_end, int64_t n) {
#pragma omp parallel for schedule(dynamic, 64)
    for (int64_t i = 0; i < n; i++) {
        Board s;
        if (start) board_from_bits(&s, start[2 * i], start[2 * i + 1], start_turn ? start_turn[i] : Black);
        else board_init(&s);
        int np = plies[i] < MOVES_STRIDE ? plies[i] : MOVES_STRIDE;
        /* rows past plies: board, turn and end 0 (include/othello.h oth_replay) */
        for (int p = np + 1; p <= MOVES_STRIDE; p++) {
            pos[2 * (i * (MOVES_STRIDE + 1) + p)] = 0;
            pos[2 * (i * (MOVES_STRIDE + 1) + p) + 1] = 0;
            if (pos_turn) pos_turn[i * (MOVES_STRIDE + 1) + p] = 0;
            if (pos_end) pos_end[i * (MOVES_STRIDE + 1) + p] = 0;
        }
        for (int p = 0;; p++) {
            int64_t r = i * (MOVES_STRIDE + 1) + p;
            board_to_bits(&s, &pos[2 * r], &pos[2 * r + 1]);
            if (pos_turn) pos_turn[r] = (uint8_t)s.turn;
            if (pos_end) pos_end[r] = (uint8_t)is_game_over(&s);
            if (p == np) break;
            put_code(&s, moves[i * MOVES_STRIDE + p]);
        }
    }
    return 0;
}

/* one step of a scan from coordinate c along d: false if it leaves the board
 * (an overflowing coordinate is far off it) */
static int step_on(int64_t c, int64_t d, int k, int64_t* out) {
    int64_t t;
    return !__builtin_mul_overflow(d, (int64_t)k, &t) && !__builtin_add_overflow(c, t, out) && *out >= 0 && *out < 8;
}

/* hands_for_direc (board.py:124-139) for any direc (dx, dy), piece and origin:
 * the length of the returned list (its squares are steps 1..len) */
static int hands_any(const Board* s, int64_t dx, int64_t dy, int piece, int64_t x, int64_t y) {
    int n = 0, h = hostile(piece);
    for (int i = 1; i < 9; i++) {
        int64_t nx, ny;
        int on = step_on(x, dx, i, &nx) && step_on(y, dy, i, &ny);
        if (on && s->b[ny][nx] == h) {
            n++;
        } else if (on && s->b[ny][nx] == piece) {
            break;
        } else {
            n = 0;
            break;
        }
    }
    return n;
}

int oracle_hands(const uint64_t* boards, const uint8_t* piece, const int64_t* x, const int64_t* y, const int64_t* dx,
                 const int64_t* dy, uint8_t* count, int64_t n) {
    for (int64_t i = 0; i < n; i++) {
        Board s;
        board_from_bits(&s, boards[2 * i], boards[2 * i + 1], Black);
        count[i] = (uint8_t)hands_any(&s, dx[i], dy[i], piece[i], x[i], y[i]);
    }
    return 0;
}

/* RNG known answers for the fixture check */
uint64_t oracle_game_key(uint64_t seed, uint64_t g) { return game_key(seed_state(seed), g); }
uint32_t oracle_rng_draws(uint64_t key, uint32_t count) {
    GameRng r = rng_init(key);
    uint32_t v = 0;
    for (uint32_t i = 0; i < count; i++) v = rng_draw(&r);
    return v; /* the count-th draw */
}
