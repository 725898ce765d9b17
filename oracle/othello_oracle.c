/*
 * oracle/othello_oracle.c -- CPU restatement of the reference rules engine.
 *
 * TEST INFRASTRUCTURE ONLY.  This file is the *checker*: it is linked by
 * tests/, by __graft_entry__.smoke() and by bench.py's cpu_baseline leg, and by
 * nothing in the product path (gymothelloenv_amd/ never loads it).
 *
 * It restates, scalar and cell-by-cell, the algorithm of the reference's
 * OthelloBaseEnv (othello.py:217-501) -- the per-cell 8-direction ray walk of
 * get_num_killed_enemy / get_possible_actions, update_board's flips, step()'s
 * pass / double-pass / sudden-death / reward logic -- plus the two scripted
 * policies the configs use (simple_policies.py:37-41 Random, :69-92 Greedy)
 * and util.make_state (util.py:48-74).  Each function cites the reference line
 * it follows.  Pinned by the tests/golden fixtures (generated from the reference itself
 * by tests/golden/gen_golden.py) in tests/test_oracle_golden.py.
 *
 * State exchange format (shared with the HIP library, include/othello_mi355x.h):
 *   boards[e*2W + 0..W-1]   black discs, bit a = row*N+col in word a/64
 *   boards[e*2W + W..2W-1]  white discs
 *   meta[e]   bit0 white-to-move, bit1 terminated, bits2-3 winner
 *             (0 none/draw, 1 white, 2 black), bits8-15 random-opening plies left
 *   legal[e*W ..]           possible_moves (may be stale, exactly as the reference)
 */
#include <stdint.h>
#include <string.h>

#define BLACK_DISK (-1) /* othello.py:10 */
#define NO_DISK 0       /* othello.py:11 */
#define WHITE_DISK 1    /* othello.py:12 */
#define MAXN 16
#define MAXW 4

#define F_SUDDEN_DEATH 1u
#define F_DISK_REWARD 2u
#define F_AUTO_RESET 4u

#define M_TURN_WHITE 1u
#define M_TERMINATED 2u
#define M_WINNER_SHIFT 2
#define M_RAND_SHIFT 8

typedef struct {
    int n;
    int sudden_death;
    int disk_reward;
    int8_t board[MAXN * MAXN];
    int turn;
    int winner;
    int terminated;
    int nmoves;
    int moves[MAXN * MAXN];
    int rand_left;
} oenv;

static int nwords(int n) { return (n * n + 63) / 64; }

/* othello.py:256-263 */
static void reset_board(oenv *e) {
    int c = e->n / 2;
    memset(e->board, 0, sizeof(e->board));
    e->board[(c - 1) * e->n + (c - 1)] = WHITE_DISK;
    e->board[c * e->n + c] = WHITE_DISK;
    e->board[c * e->n + (c - 1)] = BLACK_DISK;
    e->board[(c - 1) * e->n + c] = BLACK_DISK;
}

/* othello.py:273-311.  `me` plays the role of WHITE_DISK after the reference's
 * canonicalising negation (othello.py:316-319, 395-396): own = me, enemy = -me. */
static int num_killed_enemy(const oenv *e, const int8_t *board, int me, int x, int y, int dx, int dy) {
    int n = e->n;
    int nx = x + dx, ny = y + dy, cnt = 0;
    if (nx < 0 || nx >= n || ny < 0 || ny >= n || board[nx * n + ny] != -me) return 0;
    while (0 <= nx && nx < n && 0 <= ny && ny < n && board[nx * n + ny] == -me) {
        nx += dx;
        ny += dy;
        cnt++;
    }
    if (nx < 0 || nx >= n || ny < 0 || ny >= n || board[nx * n + ny] != me) return 0;
    return cnt;
}

/* othello.py:313-343: ascending list of empty cells with a capturing ray. */
static int possible_actions(const oenv *e, const int8_t *board, int me, int *out) {
    static const int D[8][2] = {{1, 1}, {1, 0}, {1, -1}, {0, 1}, {0, -1}, {-1, 1}, {-1, 0}, {-1, -1}};
    int n = e->n, cnt = 0;
    for (int r = 0; r < n; r++)
        for (int c = 0; c < n; c++) {
            if (board[r * n + c] != NO_DISK) continue;
            for (int d = 0; d < 8; d++)
                if (num_killed_enemy(e, board, me, r, c, D[d][0], D[d][1])) {
                    out[cnt++] = r * n + c;
                    break;
                }
        }
    return cnt;
}

/* othello.py:464-466 */
static void set_player_turn(oenv *e, int turn) {
    e->turn = turn;
    e->nmoves = possible_actions(e, e->board, turn, e->moves);
}

/* othello.py:265-271 */
static void env_reset(oenv *e) {
    reset_board(e);
    e->turn = BLACK_DISK;
    e->winner = NO_DISK;
    e->terminated = 0;
    e->nmoves = possible_actions(e, e->board, e->turn, e->moves);
}

/* othello.py:468-471 */
static void count_disks(const oenv *e, int *white, int *black) {
    int w = 0, b = 0;
    for (int i = 0; i < e->n * e->n; i++) {
        w += e->board[i] == WHITE_DISK;
        b += e->board[i] == BLACK_DISK;
    }
    *white = w;
    *black = b;
}

/* othello.py:473-501 */
static int determine_winner(oenv *e, int sudden_death) {
    e->terminated = 1;
    if (sudden_death) return e->turn == WHITE_DISK ? BLACK_DISK : WHITE_DISK;
    int w, b;
    count_disks(e, &w, &b);
    if (w > b) return WHITE_DISK;
    if (b > w) return BLACK_DISK;
    return NO_DISK;
}

/* othello.py:391-410: flip every capped ray from (x, y), then place the disc. */
static void update_board(oenv *e, int action) {
    int n = e->n, x = action / n, y = action % n, me = e->turn;
    for (int dx = -1; dx <= 1; dx++)
        for (int dy = -1; dy <= 1; dy++) {
            if (dx == 0 && dy == 0) continue;
            int k = num_killed_enemy(e, e->board, me, x, y, dx, dy);
            for (int i = 0; i < k; i++) e->board[(x + (i + 1) * dx) * n + (y + (i + 1) * dy)] = (int8_t)me;
        }
    e->board[x * n + y] = (int8_t)me;
}

static int in_moves(const oenv *e, int action) {
    for (int i = 0; i < e->nmoves; i++)
        if (e->moves[i] == action) return 1;
    return 0;
}

/* othello.py:412-462.  Returns 0 and fills reward and done, or -1 where the
 * reference raises ValueError('Game has terminated!') (othello.py:415-416). */
static int env_step(oenv *e, int action, int *reward, int *done) {
    if (e->terminated) return -1;
    int invalid = !in_moves(e, action); /* othello.py:417 (covers <0 and >=N*N) */
    if (!invalid) update_board(e, action);
    int vacant = 0;
    for (int i = 0; i < e->n * e->n; i++) vacant += e->board[i] == NO_DISK;
    int sudden = invalid && e->sudden_death;
    int dn = sudden || vacant == 0;
    int cur = e->turn;
    if (dn) {
        e->winner = determine_winner(e, sudden); /* turn / possible_moves left stale */
    } else {
        set_player_turn(e, -e->turn);
        if (e->nmoves == 0) {
            set_player_turn(e, -e->turn);
            if (e->nmoves == 0) e->winner = determine_winner(e, 0);
        }
    }
    int r = 0;
    if (e->terminated) {
        if (e->disk_reward) {
            if (sudden) {
                r = -(e->n * e->n);
            } else {
                int w, b;
                count_disks(e, &w, &b);
                if (cur == WHITE_DISK) {
                    r = w - b;
                    if (b == 0) r = e->n * e->n;
                } else {
                    r = b - w;
                    if (w == 0) r = e->n * e->n;
                }
            }
        } else {
            r = e->winner * cur;
        }
    }
    *reward = r;
    *done = e->terminated;
    return 0;
}

/* simple_policies.py:69-92: simulate every legal move on a fresh copy
 * (copy_env :12-18, set_board_state / set_player_turn / step / count_disks)
 * and keep the first move with the largest own-disc count (np.argmax). */
static int greedy_action(const oenv *e) {
    oenv sim;
    int best = -1, best_cnt = -1;
    for (int i = 0; i < e->nmoves; i++) {
        int mv = e->moves[i], r, d, w, b;
        sim = *e;
        sim.terminated = 0;
        sim.winner = NO_DISK;
        set_player_turn(&sim, e->turn);
        env_step(&sim, mv, &r, &d);
        count_disks(&sim, &w, &b);
        int own = e->turn == WHITE_DISK ? w : b;
        if (own > best_cnt) {
            best_cnt = own;
            best = mv;
        }
    }
    return best;
}

static int maximin_search(const oenv *e, int depth, int max_depth, int perspective, int my, int *move);

/* the move of a deterministic scripted policy: 1 GreedyPolicy, 2.. MaxiMinPolicy(policy - 1), any depth */
static int policy_move(const oenv *e, int policy) {
    int mv;
    if (policy == 1) return greedy_action(e);
    maximin_search(e, 0, policy - 1, e->turn, e->turn, &mv);
    return mv;
}

/* ---------------- Philox4x32-10 (the device RNG's specification) ---------------- */
static void philox(uint32_t key0, uint32_t key1, uint32_t c[4]) {
    for (int r = 0; r < 10; r++) {
        uint64_t p0 = (uint64_t)0xD2511F53u * c[0];
        uint64_t p1 = (uint64_t)0xCD9E8D57u * c[2];
        uint32_t n0 = (uint32_t)(p1 >> 32) ^ c[1] ^ key0;
        uint32_t n1 = (uint32_t)p1;
        uint32_t n2 = (uint32_t)(p0 >> 32) ^ c[3] ^ key1;
        uint32_t n3 = (uint32_t)p0;
        c[0] = n0; c[1] = n1; c[2] = n2; c[3] = n3;
        key0 += 0x9E3779B9u;
        key1 += 0xBB67AE85u;
    }
}


/* ---------------- bitboard exchange ---------------- */
static void load(oenv *e, int n, uint32_t flags, const uint64_t *bd, uint16_t meta, const uint64_t *lg) {
    int W = nwords(n);
    e->n = n;
    e->sudden_death = (flags & F_SUDDEN_DEATH) != 0;
    e->disk_reward = (flags & F_DISK_REWARD) != 0;
    for (int a = 0; a < n * n; a++) {
        int b = (int)((bd[a / 64] >> (a % 64)) & 1u), w = (int)((bd[W + a / 64] >> (a % 64)) & 1u);
        e->board[a] = (int8_t)(w ? WHITE_DISK : (b ? BLACK_DISK : NO_DISK));
    }
    e->turn = (meta & M_TURN_WHITE) ? WHITE_DISK : BLACK_DISK;
    e->terminated = (meta & M_TERMINATED) != 0;
    int wc = (meta >> M_WINNER_SHIFT) & 3;
    e->winner = wc == 1 ? WHITE_DISK : (wc == 2 ? BLACK_DISK : NO_DISK);
    e->rand_left = meta >> M_RAND_SHIFT;
    e->nmoves = 0;
    for (int a = 0; a < n * n; a++)
        if ((lg[a / 64] >> (a % 64)) & 1u) e->moves[e->nmoves++] = a;
}

static void store(const oenv *e, uint64_t *bd, uint16_t *meta, uint64_t *lg) {
    int n = e->n, W = nwords(n);
    memset(bd, 0, sizeof(uint64_t) * 2 * W);
    memset(lg, 0, sizeof(uint64_t) * W);
    for (int a = 0; a < n * n; a++) {
        if (e->board[a] == BLACK_DISK) bd[a / 64] |= 1ull << (a % 64);
        if (e->board[a] == WHITE_DISK) bd[W + a / 64] |= 1ull << (a % 64);
    }
    for (int i = 0; i < e->nmoves; i++) lg[e->moves[i] / 64] |= 1ull << (e->moves[i] % 64);
    uint16_t m = 0;
    if (e->turn == WHITE_DISK) m |= M_TURN_WHITE;
    if (e->terminated) m |= M_TERMINATED;
    m |= (uint16_t)((e->winner == WHITE_DISK ? 1 : (e->winner == BLACK_DISK ? 2 : 0)) << M_WINNER_SHIFT);
    m |= (uint16_t)((e->rand_left & 0xff) << M_RAND_SHIFT);
    *meta = m;
}

/* ---------------- exported batch API (ctypes, oracle/oracle.py) ---------------- */
int oracle_nwords(int n) { return nwords(n); }

/* OthelloBaseEnv.reset (othello.py:265-271) for E envs. */
void oracle_reset_batch(int n, int E, uint64_t *boards, uint16_t *meta, uint64_t *legal) {
    int W = nwords(n);
    oenv e;
    memset(&e, 0, sizeof(e));
    e.n = n;
    env_reset(&e);
    for (int i = 0; i < E; i++) store(&e, boards + (size_t)i * 2 * W, meta + i, legal + (size_t)i * W);
}

/* get_possible_actions(board) (othello.py:313-343) for canonical boards given as
 * (mover, opponent) bitboards: mover plays the reference's WHITE_DISK role. */
void oracle_legal_batch(int n, int E, const uint64_t *mover, const uint64_t *opp, uint64_t *out) {
    int W = nwords(n);
    oenv e;
    memset(&e, 0, sizeof(e));
    e.n = n;
    int moves[MAXN * MAXN];
    for (int i = 0; i < E; i++) {
        for (int a = 0; a < n * n; a++) {
            int m = (int)((mover[(size_t)i * W + a / 64] >> (a % 64)) & 1u);
            int o = (int)((opp[(size_t)i * W + a / 64] >> (a % 64)) & 1u);
            e.board[a] = (int8_t)(m ? WHITE_DISK : (o ? BLACK_DISK : NO_DISK));
        }
        int k = possible_actions(&e, e.board, WHITE_DISK, moves);
        memset(out + (size_t)i * W, 0, sizeof(uint64_t) * W);
        for (int j = 0; j < k; j++) out[(size_t)i * W + moves[j] / 64] |= 1ull << (moves[j] % 64);
    }
}

/* update_board (othello.py:391-410) alone for E envs: the side to move (meta
 * bit 0) flips every capped ray from square actions[i] in [0, N*N) and puts its
 * disc on it, whatever the square held; meta and possible_moves are untouched
 * (only boards is written). */
void oracle_update_board_batch(int n, int E, uint64_t *boards, const uint16_t *meta, const int32_t *actions) {
    int W = nwords(n);
    uint64_t lg[MAXW], lg_out[MAXW];
    uint16_t m_out;
    memset(lg, 0, sizeof(lg));
    oenv e;
    for (int i = 0; i < E; i++) {
        memset(&e, 0, sizeof(e));
        load(&e, n, 0, boards + (size_t)i * 2 * W, meta[i], lg);
        update_board(&e, actions[i]);
        store(&e, boards + (size_t)i * 2 * W, &m_out, lg_out);
    }
}

/* OthelloBaseEnv.step (othello.py:412-462) for E envs with external actions.
 * A terminated env is left unchanged and reports done=1, reward=0 (the batched
 * stand-in for the reference's ValueError); with F_AUTO_RESET an env that
 * terminates is reset after its outputs are written (random-opening length
 * drawn with purpose 1 at ply `ply`).  Games that end are tallied into wdl
 * (may be NULL).  Returns the number of envs stepped while already terminated. */
static int opening_plies(uint64_t seed, uint32_t id, uint64_t ply, uint32_t purpose, int initial_rand_steps);

int oracle_step_batch(int n, uint32_t flags, uint64_t seed, uint32_t id_base, uint64_t ply, int initial_rand_steps,
                      int E, uint64_t *boards, uint16_t *meta, uint64_t *legal, const int32_t *actions,
                      int32_t *rewards, uint8_t *dones, int64_t *wdl) {
    int W = nwords(n), errs = 0;
    oenv e;
    for (int i = 0; i < E; i++) {
        uint64_t *bd = boards + (size_t)i * 2 * W, *lg = legal + (size_t)i * W;
        load(&e, n, flags, bd, meta[i], lg);
        int r = 0, d = 1;
        if (env_step(&e, actions[i], &r, &d) < 0) {
            errs++;
            r = 0;
            d = 1;
        } else if (d) {
            if (wdl) wdl[e.winner == BLACK_DISK ? 0 : (e.winner == NO_DISK ? 1 : 2)]++;
            if (flags & F_AUTO_RESET) {
                env_reset(&e);
                e.rand_left = initial_rand_steps > 0
                                  ? opening_plies(seed, id_base + (uint32_t)i, ply, 1, initial_rand_steps)
                                  : 0;
            }
        }
        rewards[i] = r;
        dones[i] = (uint8_t)d;
        store(&e, bd, meta + i, lg);
    }
    return errs;
}

/* RandomPolicy.get_action (simple_policies.py:37-41) with the device RNG:
 * index k = floor(u32 * len / 2^32) into the ascending possible_moves list;
 * u = word (ply % 4) of the Philox block with counter ply / 4. */
static int random_action(const oenv *e, uint64_t seed, uint32_t id, uint64_t ply) {
    if (e->nmoves == 0) return -1; /* no legal move: the invalid path, as on the device */
    uint32_t c[4] = {id, (uint32_t)(ply >> 2), (uint32_t)(ply >> 34), 0};
    philox((uint32_t)seed, (uint32_t)(seed >> 32), c);
    uint32_t u = c[ply & 3];
    int k = (int)(((uint64_t)u * (uint64_t)e->nmoves) >> 32);
    return e->moves[k];
}

/* The opening-length word: murmur3's 32-bit finaliser on a key of (seed, purpose),
 * then the ply, then the env id -- the device's opening_draw (bitboard.hpp). */
static uint32_t fmix32(uint32_t h) {
    h ^= h >> 16;
    h *= 0x85EBCA6Bu;
    h ^= h >> 13;
    h *= 0xC2B2AE35u;
    h ^= h >> 16;
    return h;
}
static uint32_t opening_draw(uint64_t seed, uint32_t id, uint64_t ply, uint32_t purpose) {
    uint32_t key = fmix32((uint32_t)seed ^ fmix32((uint32_t)(seed >> 32) ^ purpose * 0x7FEB352Du));
    uint32_t c = fmix32(key ^ (uint32_t)ply ^ (uint32_t)(ply >> 32) * 0x9E3779B9u);
    return fmix32(c ^ id);
}

static int opening_plies(uint64_t seed, uint32_t id, uint64_t ply, uint32_t purpose, int initial_rand_steps) {
    /* SimpleOthelloEnv.reset: randint(0, k//2 + 1) * 2 (othello.py:62-63), the word
     * from opening_draw (Philox drew it up to round 5) */
    uint32_t u = opening_draw(seed, id, ply, purpose);
    return (int)(((uint64_t)u * (uint64_t)(initial_rand_steps / 2 + 1)) >> 32) * 2;
}

/* Explicit reset with a random-opening draw (purpose 2), as oth_reset. */
void oracle_reset_openings(int n, int E, uint64_t seed, uint32_t id_base, uint64_t ply, int initial_rand_steps,
                           uint64_t *boards, uint16_t *meta, uint64_t *legal) {
    int W = nwords(n);
    oenv e;
    memset(&e, 0, sizeof(e));
    e.n = n;
    for (int i = 0; i < E; i++) {
        env_reset(&e);
        e.rand_left = initial_rand_steps > 0 ? opening_plies(seed, id_base + (uint32_t)i, ply, 2, initial_rand_steps) : 0;
        store(&e, boards + (size_t)i * 2 * W, meta + i, legal + (size_t)i * W);
    }
}

/* On-device-policy rollout semantics (oth_step_policy): `plies` plies over E
 * envs.  policy 0 = random, 1 = greedy, d + 1 = maximin depth d.  Global ply index g = ply0 + p.
 * actions/rewards/dones are [plies][E] (NULL to skip); wdl[3] accumulates
 * {black wins, draws, white wins} over games that end in this call. */
int oracle_rollout(int n, uint32_t flags, int policy, int initial_rand_steps, uint64_t seed, uint32_t id_base,
                   uint64_t ply0, int E, int plies, uint64_t *boards, uint16_t *meta, uint64_t *legal,
                   int32_t *actions, int32_t *rewards, uint8_t *dones, int64_t *wdl) {
    int W = nwords(n);
    oenv e;
    for (int i = 0; i < E; i++) {
        uint64_t *bd = boards + (size_t)i * 2 * W, *lg = legal + (size_t)i * W;
        uint32_t id = id_base + (uint32_t)i;
        load(&e, n, flags, bd, meta[i], lg);
        for (int p = 0; p < plies; p++) {
            uint64_t g = ply0 + (uint64_t)p;
            size_t o = (size_t)p * E + i;
            int a = -1, r = 0, d = 1;
            if (!e.terminated) {
                if (policy == 0 || e.rand_left > 0) {
                    a = random_action(&e, seed, id, g);
                    if (e.rand_left > 0) e.rand_left--;
                } else {
                    a = policy_move(&e, policy);
                }
                env_step(&e, a, &r, &d);
                if (d) {
                    if (wdl) wdl[e.winner == BLACK_DISK ? 0 : (e.winner == NO_DISK ? 1 : 2)]++;
                    if (flags & F_AUTO_RESET) {
                        env_reset(&e);
                        e.rand_left = initial_rand_steps > 0 ? opening_plies(seed, id, g, 1, initial_rand_steps) : 0;
                    }
                }
            }
            if (actions) actions[o] = a;
            if (rewards) rewards[o] = r;
            if (dones) dones[o] = (uint8_t)d;
        }
        store(&e, bd, meta + i, lg);
    }
    return 0;
}

/* GreedyPolicy.get_action for E positions given in the exchange format. */
void oracle_greedy_batch(int n, int E, const uint64_t *boards, const uint16_t *meta, const uint64_t *legal,
                         int32_t *out) {
    int W = nwords(n);
    oenv e;
    for (int i = 0; i < E; i++) {
        load(&e, n, 0, boards + (size_t)i * 2 * W, meta[i], legal + (size_t)i * W);
        out[i] = e.nmoves ? greedy_action(&e) : -1;
    }
}

/* Recompute possible_moves for the side to move (set_player_turn, othello.py:464-466). */
void oracle_recompute_legal(int n, int E, const uint64_t *boards, const uint16_t *meta, uint64_t *legal) {
    int W = nwords(n);
    oenv e;
    uint64_t zero[MAXW] = {0};
    for (int i = 0; i < E; i++) {
        load(&e, n, 0, boards + (size_t)i * 2 * W, meta[i], zero);
        set_player_turn(&e, e.turn);
        uint64_t bd[2 * MAXW];
        uint16_t m;
        store(&e, bd, &m, legal + (size_t)i * W);
    }
}

/* count_disks (othello.py:468-471) of every board: out[2i] = white, out[2i+1] = black. */
void oracle_count_disks_batch(int n, int E, const uint64_t *boards, const uint16_t *meta, int32_t *out) {
    int W = nwords(n);
    oenv e;
    uint64_t zero[MAXW] = {0};
    for (int i = 0; i < E; i++) {
        int w, b;
        load(&e, n, 0, boards + (size_t)i * 2 * W, meta[i], zero);
        count_disks(&e, &w, &b);
        out[2 * (size_t)i] = w;
        out[2 * (size_t)i + 1] = b;
    }
}

/* get_observation (othello.py:363-378) as int8 (E, [2,] N, N) and
 * util.make_state (util.py:48-74) as float32 (E, 4, N, N). */
void oracle_observe(int n, int E, const uint64_t *boards, const uint16_t *meta, const uint64_t *legal,
                    int8_t *obs, int8_t *obs2, float *make_state) {
    int W = nwords(n), nn = n * n;
    oenv e;
    for (int i = 0; i < E; i++) {
        load(&e, n, 0, boards + (size_t)i * 2 * W, meta[i], legal + (size_t)i * W);
        int sign = e.turn == WHITE_DISK ? 1 : -1;
        for (int a = 0; a < nn; a++) {
            int v = e.board[a] * sign;
            if (obs) obs[(size_t)i * nn + a] = (int8_t)v;
            if (obs2) {
                obs2[(size_t)i * 2 * nn + a] = (int8_t)v;
                obs2[(size_t)i * 2 * nn + nn + a] = (int8_t)in_moves(&e, a);
            }
            if (make_state) {
                float *s = make_state + (size_t)i * 4 * nn;
                s[a] = e.board[a] == BLACK_DISK;
                s[nn + a] = e.board[a] == WHITE_DISK;
                s[2 * nn + a] = e.turn == WHITE_DISK;
                s[3 * nn + a] = (e.nmoves > 1) && in_moves(&e, a); /* util.py:55 quirk */
            }
        }
    }
}

/* ---------------- OthelloEnv with an embedded opponent (othello.py:151-200) ---------------- */
#define VS_PLIES_PER_CALL 256u

/* while the game runs and it is not the protagonist's turn, the opponent moves
 * (othello.py:190-199); `openings` applies the rand_step_cnt override (:191-194),
 * which the opponent's reply inside reset() does not (:165-169). */
static void opponent_reply(oenv *e, int prot, int openings, int policy, uint64_t seed, uint32_t id, uint64_t gbase,
                           uint32_t *j, int *r, int *d) {
    while (!e->terminated && e->turn != prot) {
        uint64_t g = gbase + (*j)++; /* ply j of the call */
        int a;
        if (policy == 0 || (openings && e->rand_left > 0))
            a = random_action(e, seed, id, g);
        else
            a = policy_move(e, policy);
        if (openings && e->rand_left > 0) e->rand_left--;
        env_step(e, a, r, d);
    }
}

static void reset_vs(oenv *e, int prot, int policy, uint64_t seed, uint32_t id, uint64_t call, uint32_t purpose,
                     int initial_rand_steps, uint32_t *j) {
    int r, d;
    env_reset(e);
    e->rand_left = initial_rand_steps > 0 ? opening_plies(seed, id, call, purpose, initial_rand_steps) : 0;
    opponent_reply(e, prot, 0, policy, seed, id, call * VS_PLIES_PER_CALL, j, &r, &d);
}

/* OthelloEnv.reset (othello.py:151-174) for E envs; prot int8[E] (+1/-1) or NULL = white. */
void oracle_reset_vs(int n, uint32_t flags, int policy, int initial_rand_steps, uint64_t seed, uint32_t id_base,
                     uint64_t call, int E, const int8_t *prot, uint64_t *boards, uint16_t *meta, uint64_t *legal) {
    int W = nwords(n);
    oenv e;
    memset(&e, 0, sizeof(e));
    e.n = n;
    e.sudden_death = (flags & F_SUDDEN_DEATH) != 0;
    e.disk_reward = (flags & F_DISK_REWARD) != 0;
    for (int i = 0; i < E; i++) {
        uint32_t j = 0;
        reset_vs(&e, prot ? prot[i] : WHITE_DISK, policy, seed, id_base + (uint32_t)i, call, 2, initial_rand_steps, &j);
        store(&e, boards + (size_t)i * 2 * W, meta + i, legal + (size_t)i * W);
    }
}

/* OthelloEnv.step (othello.py:176-200) for E envs: rewards from the
 * protagonist's view (negated after an opponent ply, :200). */
void oracle_step_vs(int n, uint32_t flags, int policy, int initial_rand_steps, uint64_t seed, uint32_t id_base,
                    uint64_t call, int E, const int8_t *prot, const int32_t *actions, uint64_t *boards,
                    uint16_t *meta, uint64_t *legal, int32_t *rewards, uint8_t *dones, int32_t *plies,
                    int64_t *wdl) {
    int W = nwords(n);
    oenv e;
    for (int i = 0; i < E; i++) {
        uint64_t *bd = boards + (size_t)i * 2 * W, *lg = legal + (size_t)i * W;
        uint32_t id = id_base + (uint32_t)i, j = 0;
        int p = prot ? prot[i] : WHITE_DISK;
        uint64_t gbase = call * VS_PLIES_PER_CALL;
        load(&e, n, flags, bd, meta[i], lg);
        int r = 0, d = 1, np = 0;
        if (!e.terminated) {
            d = 0;
            opponent_reply(&e, p, 1, policy, seed, id, gbase, &j, &r, &d);
            if (!e.terminated) {
                int a = actions[i];
                uint64_t g = gbase + j++;
                if (e.rand_left > 0) { /* :179-182 */
                    a = random_action(&e, seed, id, g);
                    e.rand_left--;
                }
                env_step(&e, a, &r, &d);
                if (!d) {
                    opponent_reply(&e, p, 1, policy, seed, id, gbase, &j, &r, &d);
                    r = -r;
                }
            } else {
                r = -r;
            }
            np = (int)j;
            if (d) {
                if (wdl) wdl[e.winner == BLACK_DISK ? 0 : (e.winner == NO_DISK ? 1 : 2)]++;
                if (flags & F_AUTO_RESET) reset_vs(&e, p, policy, seed, id, call, 1, initial_rand_steps, &j);
            }
        }
        store(&e, bd, meta + i, lg);
        if (rewards) rewards[i] = r;
        if (dones) dones[i] = (uint8_t)d;
        if (plies) plies[i] = np;
    }
}

/* ---------------- MaxiMinPolicy (simple_policies.py:98-163) ---------------- */
/* search() restated with the reference's simulation: for each legal move a
 * fresh copy gets the board (set_board_state), the turn (set_player_turn), the
 * move (step); if the opponent must pass, the turn is forced to the opponent
 * anyway (set_player_turn(-perspective), :139-144), whose empty move list then
 * ends the branch.  Leaves count the searching side's discs; ties keep the
 * first move (np.argmax / np.argmin). */
static int maximin_search(const oenv *e, int depth, int max_depth, int perspective, int my, int *move) {
    if (e->terminated || depth >= max_depth || e->nmoves == 0) {
        int w, b;
        count_disks(e, &w, &b);
        *move = -1;
        return my == WHITE_DISK ? w : b;
    }
    int best = 0, best_move = -1, have = 0;
    for (int i = 0; i < e->nmoves; i++) {
        oenv c = *e; /* copy_env + reset + set_board_state(...) */
        int r, d, mv;
        c.terminated = 0;
        c.winner = NO_DISK;
        set_player_turn(&c, perspective);
        env_step(&c, e->moves[i], &r, &d);
        if (!c.terminated && c.turn == perspective) set_player_turn(&c, -perspective);
        int cnt = maximin_search(&c, depth + 1, max_depth, -perspective, my, &mv);
        if (!have || (perspective == my ? cnt > best : cnt < best)) {
            best = cnt;
            best_move = e->moves[i];
            have = 1;
        }
    }
    *move = best_move;
    return best;
}

/* MaxiMinPolicy(depth).get_action for E positions (exchange format). */
void oracle_maximin_batch(int n, int depth, int E, const uint64_t *boards, const uint16_t *meta,
                          const uint64_t *legal, int32_t *out) {
    int W = nwords(n);
    oenv e;
    for (int i = 0; i < E; i++) {
        int mv;
        load(&e, n, F_SUDDEN_DEATH, boards + (size_t)i * 2 * W, meta[i], legal + (size_t)i * W);
        maximin_search(&e, 0, depth, e.turn, e.turn, &mv);
        out[i] = mv;
    }
}
