// ply.hpp -- the single-ply kernel of one-word boards (N <= 8): one launch =
// one OthelloBaseEnv.step (othello.py:412-462) of every board, with the state
// read from and written back to HBM.  Two sources of the move:
//   PLY_ACTIONS  the caller's device actions (oth_step: the north-star
//                step(action) path, any action, legal or not);
//   PLY_RANDOM   RandomPolicy.get_action (simple_policies.py:37-41) from the
//                Philox stream (oth_step_policy(RANDOM, n_plies = 1)).
// Results are identical to k_step / k_play (the generic kernels); the shape is
// built for a launch that moves every board once:
//   * every load a lane needs (board, possible_moves, flags, action, the
//     wave's W/D/L slot) is issued first and unconditionally (lanes past E load
//     board E - 1 and store nothing), so one memory latency is paid, not two;
//   * update_board's flips are capped runs along the eight rays of the square
//     (the nearest non-opponent square, one 3-input op per dword for the cap
//     test): about 90 VALU against about 260 for Kogge-Stone runs from the
//     square; the rays are computed (small launches) or read from the up half
//     of the handle's ray table staged in LDS by one 8-byte load per thread
//     issued before the boards' loads (large launches);
//   * the reset position's possible_moves is a compile-time constant;
//   * the W/D/L tally is per wave: three ballots, and lane 0 adds their counts
//     to the wave's own slot with plain stores (read with the board loads) --
//     no LDS, no barrier, no atomics.
#pragma once

#include "device.hpp"

namespace oth_dev {

constexpr int PLY_ACTIONS = 0, PLY_RANDOM = 1;

// Where the flips' rays come from (a template parameter of the single-ply kernels):
//   RAYS_MATH  computed per move, no table, no LDS, no barrier (+32 VALU: faster
//              where one wave per SIMD runs a latency-bound chain, 65,536
//              boards 3.37 -> 3.11 us per ply against the whole table in LDS;
//              profiles/r03/ab/ab_blocks.jsonl)
//   RAYS_HALF  the four up directions of the handle's table staged in LDS, 8
//              bytes per thread; a turned down ray of square a is the up ray of
//              square NN-1-a (RayMath below).  Against the whole table (16 bytes
//              per thread): 262,144 boards 5.79 -> 5.45 us per ply, 1,048,576
//              13.32 -> 13.12 (profiles/r03/ply/ab_half_table.jsonl)
//   RAYS_PAIR  computed, split over a lane pair holding the same board (k_sample_step2):
//              lane 0 runs the four up directions, lane 1 the four down ones on the
//              turned board, and the pair ORs the two halves through DPP
constexpr int RAYS_MATH = 2, RAYS_HALF = 3, RAYS_PAIR = 4;
#ifndef OTH_PLY_MATH_MAX_E
#define OTH_PLY_MATH_MAX_E 65536  // single-ply launches of at most this many boards compute their rays
#endif

// RayMath (the rays of a square without a table) is in device.hpp.

// The run one direction flips: the ray's squares before its nearest
// non-opponent square y0 (the lowest set bit of y = ray & ~O; all of them
// opponent discs), kept iff y0 holds an own disc.  y - 1 keeps y's higher bits,
// which are not opponent squares, so ray & O & (y - 1) is exactly that run (the
// whole ray when y == 0, then uncapped).
__device__ __forceinline__ uint64_t capped_run(uint64_t ray, uint64_t P, uint64_t O) {
    const uint64_t y = ray & ~O;
    const uint64_t ym = y - 1ull;
    const uint64_t run = and3_64(ray, O, ym);
    // y0 if it is an own disc (y & ~(y - 1) & P): one v_bitop3_b32 per dword (the
    // backend rewrites a plain ~(y - 1) as -y: six ops)
    const uint64_t cap = andn_and_64(y, ym, P);
    return cap ? run : 0ull;
}


// update_board's flips (othello.py:391-410) for a move on square a: the four
// directions toward higher squares on the board, the four toward lower ones on
// the board turned by 180 degrees (OneWord::turn180), where they point to
// higher squares too.  r = rays + a, the table of fill_rays<N, true>.
template <int N, int RAYS>
__device__ __forceinline__ uint64_t flips_rays(uint64_t P, uint64_t O, const uint64_t* __restrict__ r, int a,
                                               int h = 0) {
    if constexpr (RAYS == RAYS_PAIR) {  // lane h of a pair: up (h = 0) or turned down (h = 1) half
        const uint32_t s0 = (uint32_t)a & 63u, c0 = s0 % N;
        const bool dn = h != 0;
        const uint64_t Pt = OneWord<N>::turn180(P), Ot = OneWord<N>::turn180(O);
        const uint64_t Pl = dn ? Pt : P, Ol = dn ? Ot : O;
        uint64_t ray[4];
        RayMath<N>::up(dn ? RayMath<N>::turned(s0) : s0, dn ? N - 1 - c0 : c0, ray);
        uint64_t f = 0;
#pragma unroll
        for (int d = 0; d < 4; ++d) f |= capped_run(ray[d], Pl, Ol);
        const uint64_t ft = OneWord<N>::turn180(f);
        f = dn ? ft : f;
        const uint32_t lo = (uint32_t)f, hi = (uint32_t)(f >> 32);  // the partner's half: quad_perm [1,0,3,2]
        const uint32_t plo = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)lo, 0xB1, 0xF, 0xF, false);
        const uint32_t phi = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)hi, 0xB1, 0xF, 0xF, false);
        return f | ((uint64_t)phi << 32 | plo);
    }
    uint64_t ray[8];
    if constexpr (RAYS == RAYS_MATH) {  // the turned rays are the up rays of square NN-1-a, column N-1-c
        const uint32_t s = (uint32_t)a & 63u, c = s % N;
        RayMath<N>::up(s, c, ray);
        RayMath<N>::up(RayMath<N>::turned(s), N - 1 - c, ray + 4);
    } else {
        static_assert(RAYS == RAYS_HALF || RAYS == RAYS_PAIR, "ray source");  // (PAIR returned above)
        const uint64_t* rt = r - (a & 63) + ((N * N - 1 - (a & 63)) & 63);  // (in the table for any a)
#pragma unroll
        for (int d = 0; d < 4; ++d) {
            ray[d] = r[64 * d];
            ray[4 + d] = rt[64 * d];
        }
    }
    uint64_t f = 0, g = 0;
#pragma unroll
    for (int d = 0; d < 4; ++d) f |= capped_run(ray[d], P, O);
    const uint64_t Pt = OneWord<N>::turn180(P), Ot = OneWord<N>::turn180(O);
#pragma unroll
    for (int d = 4; d < 8; ++d) g |= capped_run(ray[d], Pt, Ot);
    return f | OneWord<N>::turn180(g);
}


// get_possible_actions (othello.py:313-343) split over a lane pair holding the
// same board: each lane scans two of the four axes -- lane 0 E/W and S/N, lane
// 1 the two diagonals -- with the same code (per-lane shift amounts and
// propagator masks in registers: a 64-bit shift by a VGPR amount is one
// v_lshl*_b64 like a constant one), and the pair ORs its halves through DPP.
// Kogge-Stone doubling 1 + 1 + 2 + 2 covers the longest run (N - 2 <= 6).
struct PairAxes {
    uint32_t s0, s1;  // the lane's two axis steps
    uint64_t m0, m1;  // their propagator masks (inner columns, or the board for S/N)
};
template <int N>
__device__ __forceinline__ PairAxes pair_axes(int h) {
    constexpr uint64_t BD = Geo<N>::BOARD.w[0], IN = Geo<N>::INNER.w[0];
    return h ? PairAxes{N + 1u, N - 1u, IN, IN} : PairAxes{1u, (uint32_t)N, IN, BD};
}
__device__ __forceinline__ uint64_t and_or_64(uint64_t a, uint64_t b, uint64_t c) {  // (a & b) | c
    const uint32_t lo = __builtin_amdgcn_bitop3_b32((uint32_t)a, (uint32_t)b, (uint32_t)c, 0xEA);
    const uint32_t hi = __builtin_amdgcn_bitop3_b32((uint32_t)(a >> 32), (uint32_t)(b >> 32), (uint32_t)(c >> 32), 0xEA);
    return ((uint64_t)hi << 32) | lo;
}
// squares one step past the fills of the mover P through p1, both directions of step s
__device__ __forceinline__ uint64_t axis_var(uint64_t P, uint64_t p1, uint32_t s) {
    const uint64_t p2 = p1 & (p1 << s);
    uint64_t x = (P << s) & p1;
    x = and_or_64(p1, x << s, x);
    x = and_or_64(p2, x << (2 * s), x);
    x = and_or_64(p2, x << (2 * s), x);
    const uint64_t up = x << s;
    const uint64_t p2m = p2 >> s;
    x = (P >> s) & p1;
    x = and_or_64(p1, x >> s, x);
    x = and_or_64(p2m, x >> (2 * s), x);
    x = and_or_64(p2m, x >> (2 * s), x);
    return up | (x >> s);
}
__device__ __forceinline__ uint64_t pair_or(uint64_t x) {  // x | the partner lane's x (quad_perm [1,0,3,2])
    const uint32_t lo = (uint32_t)x, hi = (uint32_t)(x >> 32);
    const uint32_t plo = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)lo, 0xB1, 0xF, 0xF, false);
    const uint32_t phi = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)hi, 0xB1, 0xF, 0xF, false);
    return x | ((uint64_t)phi << 32 | plo);
}
template <int N>
__device__ __forceinline__ uint64_t legal_pair(uint64_t P, uint64_t O, const PairAxes& ax) {
    constexpr uint64_t BD = Geo<N>::BOARD.w[0];
    const uint64_t L = axis_var(P, O & ax.m0, ax.s0) | axis_var(P, O & ax.m1, ax.s1);
    return pair_or(L) & ~(P | O) & BD;
}
// the side to move's possible_moves after a ply: one lane's whole scan, or the pair's split one
template <int N, int RAYS>
__device__ __forceinline__ uint64_t scan1(uint64_t P, uint64_t O, const PairAxes& ax) {
    if constexpr (RAYS == RAYS_PAIR) {
        return legal_pair<N>(P, O, ax);
    } else {
        uint64_t t[8];  // (the fills are not used: the flips come from the rays)
        return OneWord<N>::legal(P, O, t);
    }
}

// OthelloBaseEnv.step (othello.py:412-462) on a one-word board held as
// (black B, white Wt, possible_moves L, meta m): step_lane + finish_step's
// decisions, branch-free except the pass re-scan (taken by the wave only when
// one of its lanes passes).  valid: the action is in possible_moves (`a` in
// [0, N*N) then).  Returns reward / done / winner (0 unless the game ended).
// RAYS_PAIR: lane h of a pair holding the same board (the flips and the
// legal scans split over the pair; every result is the same on both lanes).
// KEEP (one lane per board): the next mover's eight fills (OneWord::legal's t)
// into tk, for a greedy pick that follows without a scan of its own.
template <int N, int RAYS = RAYS_MATH, bool KEEP = false>
__device__ __forceinline__ void step1(uint64_t& B, uint64_t& Wt, uint64_t& L, uint32_t& m, int a, bool valid,
                                      uint32_t flags, const uint64_t* __restrict__ rays, int& reward, int& done,
                                      int& winner, int h = 0, uint64_t* tk = nullptr) {
    constexpr uint64_t BD = Geo<N>::BOARD.w[0];
    constexpr int NN = N * N;
    const bool tw = (m & M_TURN_WHITE) != 0;
    uint64_t P = tw ? Wt : B, O = tw ? B : Wt;
    const uint64_t mv = valid ? 1ull << a : 0ull;                          // update_board (:391-410)
    const uint64_t f = flips_rays<N, RAYS>(P, O, rays + (a & 63), a, h) & (0ull - (uint64_t)valid);
    P |= f | mv;
    O &= ~f;
    const bool full = (P | O) == BD;                                        // :425-426
    const bool sudden = !valid && (flags & OTH_SUDDEN_DEATH);              // :427
    const bool stale = sudden || full;  // :431-433: turn and possible_moves stay as they were
    const PairAxes ax = pair_axes<N>(h);
    uint64_t nl;
    if constexpr (KEEP) nl = OneWord<N>::legal(O, P, tk);                  // :436
    else nl = scan1<N, RAYS>(O, P, ax);
    const bool opp_pass = nl == 0;
    if (opp_pass && !stale) {                                               // :437-440
        if constexpr (KEEP) nl = OneWord<N>::legal(P, O, tk);
        else nl = scan1<N, RAYS>(P, O, ax);
    }
    const bool term = stale || (opp_pass && nl == 0);                       // :441-442
    const int pc = popc64(P), oc = popc64(O);
    const int cur = tw ? WHITE_DISK : BLACK_DISK;
    const int by_count = pc > oc ? cur : (pc < oc ? -cur : NO_DISK);       // determine_winner (:486-501)
    winner = term ? (sudden ? -cur : by_count) : NO_DISK;                   // :475-485
    L = stale ? L : nl;
    Wt = tw ? P : O;
    B = tw ? O : P;
    const bool new_tw = (!stale && !opp_pass) ? !tw : tw;
    int r = 0;  // :444-461
    if (flags & OTH_DISK_REWARD) r = sudden ? -NN : (oc == 0 ? NN : pc - oc);
    else r = winner * cur;
    reward = term ? r : 0;
    done = term ? 1 : 0;
    const uint32_t wcode = winner == WHITE_DISK ? 1u : (winner == BLACK_DISK ? 2u : 0u);
    m = (m & 0xff00u) | (new_tw ? M_TURN_WHITE : 0u) | (term ? M_TERMINATED | (wcode << M_WINNER_SHIFT) : 0u);
}

// One ply of every board, one lane per board, 256 threads per block (128 or 64:
// ±0 to +4 % at 65,536 and 1,048,576 boards, also with computed rays at every
// size; profiles/r04/e/ab_block.jsonl).  Two boards per lane (the second
// board's loads in flight while the first is stepped and stored) measured
// slower again in round 4: 262,144 boards 5.79 -> 6.14 us per ply, 1,048,576
// 12.82 -> 13.33 (profiles/r04/f/ab_bpl2.jsonl).  A lane pair per board (the
// flips and the legal scans split over the pair as in k_sample_step2: twice
// the waves, each lane's stream shorter) measured slower at 65,536 boards:
// oth_step 2.94 -> 3.22 us per graphed ply, one random ply 3.24 -> 3.66
// (profiles/r04/a/ab_ply.jsonl).  More boards per lane (all
// their loads issued first, each group stepped as its own loads return, the
// stores after the last group) measured slower at 262,144 and 1,048,576 boards
// (2 per lane +2-6 %, 4 per lane +5-17 %), and so did a grid-stride loop with
// the next group's loads issued before the current group's work (1,048,576
// boards: 15.4 -> 16.2 us per ply) and one streaming the next group into LDS by
// global_load_lds while the current one computes (15.1 -> 16.8 us with 16
// waves per CU, 18.5 with 8).
template <int N, int SRC, int RAYS>
__device__ __forceinline__ void ply_body(uint64_t* __restrict__ boards, uint16_t* __restrict__ meta,
                                         uint64_t* __restrict__ legal, int E, uint32_t flags,
                                         int32_t* __restrict__ actions, int32_t* __restrict__ rewards,
                                         uint8_t* __restrict__ dones, unsigned long long* __restrict__ wdl,
                                         const uint64_t* __restrict__ rays_g, Rng rng, uint64_t ply) {
    static_assert(Geo<N>::W == 1, "one-word boards");
    constexpr int NN = N * N;
    constexpr int TABLE = RAYS == RAYS_HALF ? 4 * 64 : 0;  // words staged in LDS
    // the large launches store nontemporally (streaming, no L2 allocation): 262,144
    // boards 5.85 -> 5.50 us per ply, 1,048,576 13.32 -> 12.78; the small ones gain
    // nothing from it (profiles/r03/nt/)
    constexpr bool NT = RAYS == RAYS_HALF;
    static_assert(TABLE == 0 || TABLE == BLOCK, "one 8-byte piece of the table per thread");
    __shared__ __attribute__((aligned(16))) uint64_t rays[TABLE ? TABLE : 1];
    ply += *rng.ply_off;  // graph-region offset (oth_graph_end); 0 eagerly
    const int t = blockIdx.x * BLOCK + threadIdx.x;
    const bool mine = t < E;
    const int e = mine ? t : E - 1;
    // every load first, none behind a branch: the ray table's piece first of
    // all (the wave then waits only for it before its LDS store), the board's
    // loads (lanes past E load board E - 1 and store nothing), the wave's slot
    uint64_t rh;
    if constexpr (TABLE) rh = rays_g[threadIdx.x];  // the four up directions: the table's first half
    const ulonglong2 bw = reinterpret_cast<const ulonglong2*>(boards)[e];
    uint64_t L = legal[e];
    uint32_t m = meta[e];
    int a = 0;
    if constexpr (SRC == PLY_ACTIONS) a = actions[e];
    WaveSlot slot(wdl, t, E);
    if constexpr (TABLE) {
        rays[threadIdx.x] = rh;
        __syncthreads();
    }
    const uint32_t id = rng.id_base + (uint32_t)e;
    uint64_t B = bw.x, Wt = bw.y;
    const bool was_term = (m & M_TERMINATED) != 0;
    bool valid;
    if constexpr (SRC == PLY_RANDOM) {
        // RandomPolicy: possible_moves[randint(len)] (k_play's pick); -1 without a move
        const uint32_t u = action_draw(rng.seed, id, ply);
        const int n = popc64(L);
        a = n ? select64(L, scale_index(u, n)) : -1;
        a = was_term ? -1 : a;  // k_play: a terminated board reports action -1
        valid = a >= 0;
        if (!was_term && (m >> M_RAND_SHIFT) > 0) m -= 1u << M_RAND_SHIFT;  // a random-opening ply used up
    } else {
        valid = (unsigned)a < (unsigned)NN && ((L >> (a & 63)) & 1ull);  // `action not in possible_moves` (:417)
    }
    int r, d, win;
    step1<N, RAYS>(B, Wt, L, m, a, valid, flags, rays, r, d, win);
    if (was_term) {  // reference: ValueError (othello.py:415-416); batched: a no-op reporting done
        r = 0;       // (the state is not stored back)
        d = 1;
    }
    const bool ended = mine && d && !was_term;
    if (ended && (flags & OTH_AUTO_RESET)) {  // reset (othello.py:256-271), black to move
        B = Start<N>::BLACK.w[0];
        Wt = Start<N>::WHITE.w[0];
        constexpr uint64_t START_MOVES = start_moves<N>();  // constant-evaluated
        L = START_MOVES;
        uint32_t rl = 0;
        if (rng.init_rand > 0)
            rl = (uint32_t)scale_index(opening_draw(rng.seed, id, ply, RNG_OPENING_AUTO), rng.init_rand / 2 + 1) * 2u;
        m = (rl & 0xffu) << M_RAND_SHIFT;
    }
    if (mine) {
        if (!was_term) {
            ulonglong2 o;
            o.x = B;
            o.y = Wt;
            if (NT) {
                __builtin_nontemporal_store(o.x, &boards[2 * (size_t)e]);
                __builtin_nontemporal_store(o.y, &boards[2 * (size_t)e + 1]);
                __builtin_nontemporal_store(L, &legal[e]);
                __builtin_nontemporal_store((uint16_t)m, &meta[e]);
            } else {
                reinterpret_cast<ulonglong2*>(boards)[e] = o;
                legal[e] = L;
                meta[e] = (uint16_t)m;
            }
        }
        if constexpr (SRC == PLY_RANDOM)
            if (actions) actions[e] = a;
        if (NT) {  // (dones, half a line a wave, through L2 instead: +-0 at 1,048,576; profiles/r04/d/)
            if (rewards) __builtin_nontemporal_store(r, &rewards[e]);
            if (dones) __builtin_nontemporal_store((uint8_t)d, &dones[e]);
        } else {
            if (rewards) rewards[e] = r;
            if (dones) dones[e] = (uint8_t)d;
        }
    }
    slot.count(ended && win == BLACK_DISK, ended && win == NO_DISK, ended && win == WHITE_DISK);
    slot.flush();
}

// oth_step on one-word boards (no register bound: 64 VGPRs forced a spill,
// whose scratch traffic cost 16 B per board)
template <int N, int RAYS>
__global__ __launch_bounds__(BLOCK) void k_ply_step(uint64_t* __restrict__ boards, uint16_t* __restrict__ meta,
                                                    uint64_t* __restrict__ legal, int E, uint32_t flags,
                                                    const int32_t* __restrict__ actions, int32_t* __restrict__ rewards,
                                                    uint8_t* __restrict__ dones, unsigned long long* __restrict__ wdl,
                                                    const uint64_t* __restrict__ rays, Rng rng, uint64_t ply) {
    ply_body<N, PLY_ACTIONS, RAYS>(boards, meta, legal, E, flags, const_cast<int32_t*>(actions), rewards, dones, wdl,
                                   rays, rng, ply);
}

// oth_step_observe on one-word boards: OthelloBaseEnv.step (othello.py:412-462)
// with the caller's actions and the returned get_observation() (:462) -- or any
// oth_observe layout and dtype -- in one launch: the wave steps its BPW boards
// (LPB lanes per board: one lane with computed rays, or a lane pair splitting
// the flips and the scans as k_sample_step2), stores the state, then streams
// the boards' observations from registers (obs_tail: the state as the step --
// and an auto-reset -- left it, exactly what oth_observe after oth_step reads,
// without reading it back).  BPW < 64 / LPB leaves lanes idle during the step
// (they step a copy of the wave's last board and store nothing) and gives the
// store stream more waves per SIMD: at 65,536 boards the observation's store
// loop wants four waves per SIMD (k_observe_w's 16 boards per wave), the step
// one (k_ply_step).
// Lane pairs with 32 boards per wave measured best at 65,536 8x8 boards (graphed,
// us per ply; profiles/r05/a/ab_step_obs.json): int64 board 10.94 (one lane, 16
// boards per wave) / 10.85 (one lane, 64) / 10.88 (pairs, 32); f32 make_state
// 13.86 / 16.50 / 13.40; the two-launch form 13.01 / 16.20, the observation
// alone 9.67 / 12.63, the step alone 3.04.
#ifndef OTH_SO_LPB
#define OTH_SO_LPB 2  // lanes per board of k_ply_step_obs
#endif
#ifndef OTH_SO_BPW
#define OTH_SO_BPW 32  // boards per wave of k_ply_step_obs
#endif
template <int N, int LPB, int BPW>
__global__ __launch_bounds__(BLOCK) void k_ply_step_obs(uint64_t* __restrict__ boards, uint16_t* __restrict__ meta,
                                                        uint64_t* __restrict__ legal, int E, uint32_t flags,
                                                        const int32_t* __restrict__ actions,
                                                        int32_t* __restrict__ rewards, uint8_t* __restrict__ dones,
                                                        unsigned long long* __restrict__ wdl, Rng rng, uint64_t ply,
                                                        int layout, int dtype, void* __restrict__ obs) {
    static_assert(Geo<N>::W == 1, "one-word boards");
    static_assert((LPB == 1 || LPB == 2) && LPB * BPW <= 64 && BPW >= 16, "lanes per board, boards per wave");
    // (BPW >= 16: ceil(E / BPW) waves fit the handle's ceil(4E / 64) W/D/L slots)
    constexpr int NN = N * N;
    constexpr int RAYS = LPB == 2 ? RAYS_PAIR : RAYS_MATH;
    ply += *rng.ply_off;  // graph-region offset (oth_graph_end); 0 eagerly
    const int lane = threadIdx.x & 63;
    const int wave = (int)(((long long)blockIdx.x * BLOCK + threadIdx.x) >> 6);
    const long long e0 = (long long)wave * BPW;
    if (e0 >= E) return;  // wave-uniform
    const int nb = (int)(E - e0 < BPW ? E - e0 : BPW);
    const int kb = lane / LPB, h = lane % LPB;
    const bool mine = kb < nb;                                 // lanes past the wave's boards (or past
    const int e = (int)e0 + (mine ? kb : nb - 1);              // BPW) step a copy of its last one
    const ulonglong2 bw = reinterpret_cast<const ulonglong2*>(boards)[e];
    uint64_t L = legal[e];
    uint32_t m = meta[e];
    const int a = actions[e];
    WaveSlot slot(wdl, wave);  // (ceil(E / BPW) <= the handle's ceil(4E / 64) slots for BPW >= 16)
    const uint32_t id = rng.id_base + (uint32_t)e;
    uint64_t B = bw.x, Wt = bw.y;
    const bool was_term = (m & M_TERMINATED) != 0;
    const bool valid = (unsigned)a < (unsigned)NN && ((L >> (a & 63)) & 1ull);  // (:417)
    int r, d, win;
    const uint64_t L0 = L;
    const uint32_t m0 = m;
    step1<N, RAYS>(B, Wt, L, m, a, valid, flags, nullptr, r, d, win, h);
    if (was_term) {  // a no-op reporting done (othello.py:415-416): the state stays as it was
        r = 0;
        d = 1;
        B = bw.x;
        Wt = bw.y;
        L = L0;
        m = m0;
    }
    const bool ended = mine && d && !was_term;
    if (ended && (flags & OTH_AUTO_RESET)) {  // reset (othello.py:256-271), black to move
        B = Start<N>::BLACK.w[0];
        Wt = Start<N>::WHITE.w[0];
        constexpr uint64_t START_MOVES = start_moves<N>();
        L = START_MOVES;
        uint32_t rl = 0;
        if (rng.init_rand > 0)
            rl = (uint32_t)scale_index(opening_draw(rng.seed, id, ply, RNG_OPENING_AUTO), rng.init_rand / 2 + 1) * 2u;
        m = (rl & 0xffu) << M_RAND_SHIFT;
    }
    if (mine && h == 0) {
        if (!was_term) {
            reinterpret_cast<ulonglong2*>(boards)[e] = ulonglong2{B, Wt};
            legal[e] = L;
            meta[e] = (uint16_t)m;
        }
        if (rewards) rewards[e] = r;
        if (dones) dones[e] = (uint8_t)d;
    }
    const bool h0 = h == 0;
    slot.count(h0 && ended && win == BLACK_DISK, h0 && ended && win == NO_DISK, h0 && ended && win == WHITE_DISK);
    slot.flush();
    const uint64_t ob[1] = {B}, ow[1] = {Wt}, ol[1] = {L};
    obs_tail<N, BPW, LPB>(layout, dtype, obs, e0, ob, ow, ol, m, nb);
}

// oth_step_policy(RANDOM, 1 ply) on one-word boards
template <int N, int RAYS>
__global__ __launch_bounds__(BLOCK) void k_ply_rand(uint64_t* __restrict__ boards, uint16_t* __restrict__ meta,
                                                    uint64_t* __restrict__ legal, int E, uint32_t flags,
                                                    int32_t* __restrict__ actions, int32_t* __restrict__ rewards,
                                                    uint8_t* __restrict__ dones, unsigned long long* __restrict__ wdl,
                                                    const uint64_t* __restrict__ rays, Rng rng, uint64_t ply) {
    ply_body<N, PLY_RANDOM, RAYS>(boards, meta, legal, E, flags, actions, rewards, dones, wdl, rays, rng, ply);
}

// OthelloEnv.step (othello.py:176-200) on one-word boards against a random or
// greedy opponent: k_step_vs's control flow (device.hpp: the opponent's replies
// before and after the protagonist's ply, random-opening plies, the reward
// negated after opponent plies, the W/D/L tallies, the auto-reset with the
// opponent's opening reply) with every ply through step1 (computed rays,
// branch-free but for the pass re-scan) on the board held as four registers
// instead of the generic Lane / Solo engine.  Results are identical.
template <int N, int POLICY>
__global__ __launch_bounds__(BLOCK) void k_step_vs1(uint64_t* __restrict__ boards, uint16_t* __restrict__ meta,
                                                    uint64_t* __restrict__ legal, int E, uint32_t flags,
                                                    const int32_t* __restrict__ actions,
                                                    const int8_t* __restrict__ prot, int32_t* __restrict__ rewards,
                                                    uint8_t* __restrict__ dones, int32_t* __restrict__ plies_out,
                                                    unsigned long long* __restrict__ wdl,
                                                    unsigned long long* __restrict__ wdl_vs, Rng rng, uint64_t call,
                                                    int obs_layout, int obs_dtype, void* __restrict__ obs) {
    static_assert(Geo<N>::W == 1, "one-word boards");
    static_assert(POLICY == OTH_POLICY_RANDOM || POLICY == OTH_POLICY_GREEDY, "random or greedy opponent");
    constexpr int NN = N * N;
    __shared__ uint64_t no_table[1];  // step1's ray table argument (RAYS_MATH reads none)
    call += *rng.ply_off;  // graph-region offset (oth_graph_end); 0 eagerly
    const int e = blockIdx.x * BLOCK + threadIdx.x;
    // per-wave W/D/L slots (ballots, no LDS, no barrier: the waves of a block end
    // after different numbers of opponent plies), read with the first loads
    WaveSlot slot(wdl, e, E), slot_vs(wdl_vs, e, E);
    uint32_t cb = 0, cd = 0, cw = 0, pw_n = 0, pd_n = 0, pl_n = 0;
    uint64_t B = 0, Wt = 0, L = 0;  // the board after the call (the observation tail's)
    uint32_t m = 0;
    if (e < E) {
        const uint32_t id = rng.id_base + (uint32_t)e;
        const bool pw = prot ? prot[e] == WHITE_DISK : true;
        const uint64_t gbase = call * VS_PLIES_PER_CALL;
        const ulonglong2 bw = reinterpret_cast<const ulonglong2*>(boards)[e];
        B = bw.x;
        Wt = bw.y;
        L = legal[e];
        m = meta[e];
        int act = actions[e];
        uint32_t j = 0;
        int r = 0, d = 1, win = NO_DISK, plies = 0;
        // greedy: the side to move's fills, carried from the scan of the ply before
        // (step1<KEEP>) so that a greedy pick needs no scan of its own
        constexpr bool KEEP = POLICY == OTH_POLICY_GREEDY;
        uint64_t t[8];
        bool have_t = false;
        // one ply of the side to move: a (any square; the invalid path when it is not
        // in possible_moves, as step_lane)
        auto ply = [&](int a) __attribute__((always_inline)) {
            const bool valid = (unsigned)a < (unsigned)NN && ((L >> (a & 63)) & 1ull);
            step1<N, RAYS_MATH, KEEP>(B, Wt, L, m, a, valid, flags, no_table, r, d, win, 0, t);
            have_t = true;
        };
        // (keeping the Philox block across a chain of opponent plies instead of
        // action_draw's block per ply measured +-0: 15.20 -> 15.09 us per call with a
        // random opponent, 15.03 -> 15.08 greedy; profiles/r04/vs/ab_vs_block.jsonl)
        auto random_pick = [&](uint64_t g) __attribute__((always_inline)) {  // random_action: -1 without a move
            const int n = popc64(L);
            return n ? select64(L, scale_index(action_draw(rng.seed, id, g), n)) : -1;
        };
        // opponent_reply: the opponent moves while it is to move and the game is on
        auto reply = [&](bool openings) __attribute__((always_inline)) {
            while (!(m & M_TERMINATED) && (((m & M_TURN_WHITE) != 0) != pw)) {
                const uint32_t rl = m >> M_RAND_SHIFT;
                const uint64_t g = gbase + j++;
                int a;
                if (POLICY == OTH_POLICY_RANDOM || (openings && rl > 0)) {
                    a = random_pick(g);
                } else {  // GreedyPolicy from the mover's fills (greedy_action)
                    if (!have_t) {
                        const bool tw = (m & M_TURN_WHITE) != 0;
                        (void)OneWord<N>::legal(tw ? Wt : B, tw ? B : Wt, t);
                        have_t = true;
                    }
                    a = OneWord<N>::greedy(t, L);
                }
                if (openings && rl > 0) m -= 1u << M_RAND_SHIFT;
                ply(a);
            }
        };
        if (!(m & M_TERMINATED)) {
            d = 0;
            reply(true);  // the protagonist must be to move (othello.py:177): else the opponent replies first
            if (!(m & M_TERMINATED)) {
                const uint32_t rl = m >> M_RAND_SHIFT;
                const uint64_t g = gbase + j++;
                if (rl > 0) {  // opening ply: the protagonist's action is replaced too (:179-182)
                    act = random_pick(g);
                    m -= 1u << M_RAND_SHIFT;
                }
                ply(act);
                if (!d) {
                    reply(true);
                    r = -r;  // :200
                }
            } else {
                r = -r;
            }
            plies = (int)j;
            if (d) {
                cb = win == BLACK_DISK;
                cd = win == NO_DISK;
                cw = win == WHITE_DISK;
                const int pcol = pw ? WHITE_DISK : BLACK_DISK;  // run.py:100-130's count
                pw_n = win == pcol;
                pd_n = win == NO_DISK;
                pl_n = win == -pcol;
                if (flags & OTH_AUTO_RESET) {  // reset_vs_lane: reset, then the opponent's opening reply
                    B = Start<N>::BLACK.w[0];
                    Wt = Start<N>::WHITE.w[0];
                    constexpr uint64_t START_MOVES = start_moves<N>();
                    L = START_MOVES;
                    uint32_t rl = 0;
                    if (rng.init_rand > 0)
                        rl = (uint32_t)scale_index(opening_draw(rng.seed, id, call, RNG_OPENING_AUTO),
                                                   rng.init_rand / 2 + 1) * 2u;
                    m = (rl & 0xffu) << M_RAND_SHIFT;
                    if constexpr (KEEP) {  // the start position's fills (black to move)
                        constexpr StartFills<N> SF = start_fills<N>();
#pragma unroll
                        for (int k = 0; k < 8; ++k) t[k] = SF.t[k];
                        have_t = true;
                    }
                    const int rs = r, ds = d, ws = win;  // (the reply's reward / done are not
                    reply(false);                         // reported, as in reset_vs_lane)
                    r = rs, d = ds, win = ws;
                }
            }
        }
        reinterpret_cast<ulonglong2*>(boards)[e] = ulonglong2{B, Wt};
        legal[e] = L;
        meta[e] = (uint16_t)m;
        if (rewards) rewards[e] = r;
        if (dones) dones[e] = (uint8_t)d;
        if (plies_out) plies_out[e] = plies;
    }
    slot.count(cb != 0, cd != 0, cw != 0);
    slot.flush();
    slot_vs.count(pw_n != 0, pd_n != 0, pl_n != 0);
    slot_vs.flush();
    // oth_step_vs_observe: the wave's 64 boards' observations, the protagonist to move
    const long long e0 = e - (int)(threadIdx.x & 63);
    const uint64_t ob[1] = {B}, ow[1] = {Wt}, ol[1] = {L};
    obs_tail<N, 64, 1>(obs_layout, obs_dtype, obs, e0, ob, ow, ol, m, (int)(E - e0 < 64 ? E - e0 : 64));
}

// oth_create: the handle's tables in device memory: the ray table (fill_rays<N,
// true>'s 8 x 64 words) and the sel8 table (256 words, sel8_word) after it
template <int N>
__global__ __launch_bounds__(BLOCK) void k_fill_rays(uint64_t* __restrict__ rays) {
    fill_rays<N, true, false>(rays);
    for (int i = threadIdx.x; i < 256; i += BLOCK) rays[8 * 64 + i] = sel8_word((uint32_t)i);
}

}  // namespace oth_dev
