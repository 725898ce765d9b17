// device.hpp -- HIP/CDNA4 device code of the vectorised Othello rules engine:
// per-lane board state, the rule engines (Solo / Rays / Fills / Quartet), policies and
// every __global__ kernel template.  Included by kernels_n.hip (compiled once
// per board size N, so the templates build in parallel) and by capi.hip.
//

// One board per lane.  A board is two W-word bitboards (black, white) held in
// VGPRs; legal moves and flips are Kogge-Stone occluded fills (bitboard.hpp).
// The reference's per-step Python work -- get_possible_actions'
// N*N*8 ray walks (othello.py:313-343), update_board (:391-410), step's
// pass / double-pass / sudden-death / reward logic (:412-462) -- becomes a few
// hundred integer VALU ops per lane.  No MFMA: the work is bit manipulation.
//
// HBM layout (exchange format, see the header): boards [E][2W] u64 (a lane
// reads 16W contiguous bytes: dwordx4 loads), meta [E] u16, legal [E][W] u64;
// per-ply outputs are [ply][E] so every store instruction is coalesced.
#pragma once
#include <hip/hip_runtime.h>

#include <stdio.h>
#include <string.h>

#include <new>
#include <string>
#include <type_traits>

#include "bitboard.hpp"
#include "masked.hpp"
#include "othello_mi355x.h"

using namespace oth;

#ifndef OTH_BLOCK
#define OTH_BLOCK 256
#endif
#ifndef OTH_SS_QUAD_MAX_E
#define OTH_SS_QUAD_MAX_E 16384  // oth_sample_step on lane quads up to this many boards: 4 lanes each fill at most 1,024 waves (one per SIMD)
#endif
#ifndef OTH_SS_PAIR_W_MAX_E
#define OTH_SS_PAIR_W_MAX_E 32768  // two-word boards whose rows are not float4-aligned: lane pairs up to this many boards
#endif

namespace oth_dev {

constexpr int BLOCK = OTH_BLOCK;
constexpr uint32_t M_TURN_WHITE = 1u;
constexpr uint32_t M_TERMINATED = 2u;
constexpr int M_WINNER_SHIFT = 2;
constexpr int M_RAND_SHIFT = 8;
constexpr int BLACK_DISK = -1, NO_DISK = 0, WHITE_DISK = 1;  // othello.py:10-12

// Philox "purpose" word: which decision a draw feeds.
constexpr uint32_t RNG_ACTION = 0, RNG_OPENING_AUTO = 1, RNG_OPENING_RESET = 2;

template <int N>
struct Start {  // _reset_board (othello.py:256-263): W at (c-1,c-1),(c,c); B at (c,c-1),(c-1,c)
    static constexpr int W = Geo<N>::W;
    static constexpr int C = N / 2;
    static constexpr BB<W> make(int a0, int a1) {
        BB<W> b{};
        for (int i = 0; i < W; ++i) b.w[i] = 0;
        b.w[a0 / 64] |= 1ull << (a0 % 64);
        b.w[a1 / 64] |= 1ull << (a1 % 64);
        return b;
    }
    static constexpr BB<W> BLACK = make(C * N + (C - 1), (C - 1) * N + C);
    static constexpr BB<W> WHITE = make((C - 1) * N + (C - 1), C * N + C);
};

// black's possible_moves on the reset board (_reset_board + get_possible_actions,
// othello.py:256-263, 313-343), by a compile-time ray walk
template <int N>
constexpr uint64_t start_moves() {
    static_assert(Geo<N>::W == 1, "one-word boards");
    const uint64_t B = Start<N>::BLACK.w[0], Wt = Start<N>::WHITE.w[0];
    uint64_t L = 0;
    for (int a = 0; a < N * N; ++a) {
        if (((B | Wt) >> a) & 1ull) continue;
        for (int dr = -1; dr <= 1; ++dr)
            for (int dc = -1; dc <= 1; ++dc) {
                if (!dr && !dc) continue;
                int r = a / N + dr, c = a % N + dc, run = 0;
                while (r >= 0 && r < N && c >= 0 && c < N && ((Wt >> (r * N + c)) & 1ull)) {
                    r += dr;
                    c += dc;
                    ++run;
                }
                if (run > 0 && r >= 0 && r < N && c >= 0 && c < N && ((B >> (r * N + c)) & 1ull)) L |= 1ull << a;
            }
    }
    return L;
}

// the Fills engine's eight fills on the reset board, black to move (what
// OneWord::legal stores in t for the start position), by the same ray walk:
// t[d] = opponent discs from which going along ray direction d (E, S, SE, SW,
// W, N, NW, NE) through opponent discs -- of the inner columns, except on the
// vertical axis, as the scan's propagators -- ends on an own disc
template <int N>
struct StartFills {
    uint64_t t[8];
};
template <int N>
constexpr StartFills<N> start_fills() {
    static_assert(Geo<N>::W == 1, "one-word boards");
    const uint64_t P = Start<N>::BLACK.w[0], O = Start<N>::WHITE.w[0], IN = Geo<N>::INNER.w[0];
    constexpr int DR[8] = {0, 1, 1, 1, 0, -1, -1, -1}, DC[8] = {1, 0, 1, -1, -1, 0, -1, 1};
    StartFills<N> f{};
    for (int d = 0; d < 8; ++d) {
        const uint64_t p1 = DC[d] == 0 ? O : (O & IN);
        f.t[d] = 0;
        for (int a = 0; a < N * N; ++a) {
            if (!((p1 >> a) & 1ull)) continue;
            int r = a / N + DR[d], c = a % N + DC[d];
            while (r >= 0 && r < N && c >= 0 && c < N && ((p1 >> (r * N + c)) & 1ull)) {
                r += DR[d];
                c += DC[d];
            }
            if (r >= 0 && r < N && c >= 0 && c < N && ((P >> (r * N + c)) & 1ull)) f.t[d] |= 1ull << a;
        }
    }
    return f;
}

template <int N>
struct Lane {
    static constexpr int W = Geo<N>::W;
    BB<W> black, white, legal;
    uint32_t meta;
};

template <int N>
__device__ __forceinline__ void load_lane(Lane<N>& s, const uint64_t* __restrict__ boards,
                                          const uint16_t* __restrict__ meta, const uint64_t* __restrict__ legal,
                                          int e) {
    constexpr int W = Geo<N>::W;
    const ulonglong2* bp = reinterpret_cast<const ulonglong2*>(boards) + (size_t)e * W;
    uint64_t tmp[2 * W];
#pragma unroll
    for (int i = 0; i < W; ++i) {
        ulonglong2 v = bp[i];
        tmp[2 * i] = v.x;
        tmp[2 * i + 1] = v.y;
    }
#pragma unroll
    for (int i = 0; i < W; ++i) {
        s.black.w[i] = tmp[i];
        s.white.w[i] = tmp[W + i];
        s.legal.w[i] = legal[(size_t)e * W + i];
    }
    s.meta = meta[e];
}

template <int N>
__device__ __forceinline__ void store_lane(const Lane<N>& s, uint64_t* __restrict__ boards,
                                           uint16_t* __restrict__ meta, uint64_t* __restrict__ legal, int e) {
    constexpr int W = Geo<N>::W;
    uint64_t tmp[2 * W];
#pragma unroll
    for (int i = 0; i < W; ++i) {
        tmp[i] = s.black.w[i];
        tmp[W + i] = s.white.w[i];
    }
    ulonglong2* bp = reinterpret_cast<ulonglong2*>(boards) + (size_t)e * W;
#pragma unroll
    for (int i = 0; i < W; ++i) {
        ulonglong2 v;
        v.x = tmp[2 * i];
        v.y = tmp[2 * i + 1];
        bp[i] = v;
        legal[(size_t)e * W + i] = s.legal.w[i];
    }
    meta[e] = (uint16_t)s.meta;
}

// ---------------------------------------------------------------------------
// Engines: who computes legal moves and flips for a lane.
//   Solo<N>: one lane per board, all 8 directions (any N).
//   Fills<N> / FillsW<N>: flips from LDS ray tables and the legal scan's fills.
//   Quartet<N>: four lanes per board (N <= 8): each lane of the quad scans
//            one axis and the parts are or-ed through DPP quad_perm steps.
// ---------------------------------------------------------------------------
template <int N>
struct Solo {
    static constexpr int LANES = 1;
    static constexpr int RAY_WORDS = 0;
    __device__ __forceinline__ Solo(int, const uint64_t*) {}
    __device__ __forceinline__ BB<Geo<N>::W> legal(const BB<Geo<N>::W>& P, const BB<Geo<N>::W>& O) const {
        if constexpr (Geo<N>::W == 1) {  // the dword-pair scan (fills unused, so dead)
            uint64_t t[8];
            BB<1> r;
            r.w[0] = OneWord<N>::legal(P.w[0], O.w[0], t);
            return r;
        }
        return legal_moves<N>(P, O);
    }
    __device__ __forceinline__ BB<Geo<N>::W> flip(const BB<Geo<N>::W>& P, const BB<Geo<N>::W>& O, int a) const {
        return flips<N>(P, O, square<Geo<N>::W>(a));
    }
    __device__ __forceinline__ void prime(const Lane<N>&) const {}
    __device__ __forceinline__ bool leader() const { return true; }
};

// Ray tables for one-word boards: rays[d*64 + sq] = the squares strictly beyond
// sq in direction d, up to the edge.  d 0..3 point to higher squares (E, S, SE,
// SW), d 4..7 to lower ones (W, N, NW, NE).  Built in LDS once per launch.
// Steps (row, col) of direction d: RAY_DR = {0, 1, 1, 1, 0, -1, -1, -1},
// RAY_DC = {1, 0, 1, -1, -1, 0, -1, 1} (nibbles of the immediates in fill_rays).

// TURNED: the tables of the directions toward lower squares (d >= 4) hold
// their rays on the board turned by 180 degrees (square s -> N*N-1-s), still
// indexed by the unturned square (Fills).
template <int N, bool TURNED = false, bool SYNC = true>
__device__ __forceinline__ void fill_rays(uint64_t* rays) {
    for (int i = threadIdx.x; i < 8 * 64; i += BLOCK) {
        const int d = i >> 6, sq = i & 63;
        uint64_t r = 0;
        if (sq < N * N) {
            // RAY_DR / RAY_DC as sign-extended nibbles: no constant-memory loads
            const int dr = __builtin_amdgcn_sbfe((int)0xFFF01110u, 4 * d, 4);
            const int dc = __builtin_amdgcn_sbfe((int)0x1F0FF101u, 4 * d, 4);
            int row = sq / N + dr, col = sq % N + dc;
            while (row >= 0 && row < N && col >= 0 && col < N) {
                const int s2 = row * N + col;
                r |= 1ull << ((TURNED && d >= 4) ? N * N - 1 - s2 : s2);
                row += dr;
                col += dc;
            }
        }
        rays[i] = r;
    }
    if (SYNC) __syncthreads();
}

// Without a table: the rays of square s toward higher squares (E, S, SE, SW)
// as one shifted constant each -- the ray from square 0 (or row 0's squares
// 1 .. N-1 for E) moved to s -- with the squares that wrapped past the board's
// right (E, SE) or left (SW) edge masked off by column.
template <int N>
struct RayMath {
    static constexpr uint64_t sum_steps(int step, int k0, int k1) {
        uint64_t x = 0;
        for (int k = k0; k <= k1; ++k) x |= 1ull << (k * step);
        return x;
    }
    static constexpr uint64_t BD = Geo<N>::BOARD.w[0];
    static constexpr uint64_t ROW1 = sum_steps(N, 0, N - 1);      // column 0 of every row
    static constexpr uint64_t EAST = ((1ull << N) - 1) & ~1ull;    // squares 1 .. N-1 of row 0
    static constexpr uint64_t COL = sum_steps(N, 1, N - 1);       // S from square 0
    static constexpr uint64_t DIAG = sum_steps(N + 1, 1, N - 1);  // SE from square 0
    static constexpr uint64_t ANTI = sum_steps(N - 1, 1, N - 1);  // SW from square N-1, moved to square 0
    // square s of the board turned by 180 degrees, for any s < 64: an invalid
    // action's square may lie past N*N - 1 on boards of N < 8, so the result is
    // kept below 64 (every shift count of up() stays defined; the caller masks
    // the flips of an invalid action)
    __device__ __forceinline__ static uint32_t turned(uint32_t s) {
        return N == 8 ? N * N - 1 - s : (N * N - 1 - s) & 63u;
    }
    __device__ __forceinline__ static void up(uint32_t s, uint32_t c, uint64_t* ray) {
        const uint32_t row = (1u << N) - 1u;
        const uint64_t gt = ROW1 * (uint64_t)((row << (c + 1)) & row);  // columns > c of every row
        const uint64_t lt = ROW1 * (uint64_t)((1u << c) - 1u);           // columns < c
        ray[0] = (EAST << s) & gt;
        ray[1] = (COL << s) & BD;
        ray[2] = (DIAG << s) & gt & BD;
        ray[3] = (ANTI << s) & lt & BD;
    }
};

// Fills<N>: flips from the ray tables and the legal scan's fills.  legal_moves' axis scans
// compute, for the side to move, the fills t(dir) = opponent discs reachable
// from an own disc through contiguous opponent discs stepping in direction dir
// (the scan shifts them once more onto the empty squares).  Kept in registers
// until the next ply, they answer update_board's capping test: along ray d
// from the played square a, the run to flip is the contiguous part of ray_d(a)
// inside t(-d) -- every square of t(-d) on that run is already capped by an
// own disc further along d.  So per direction: nearest square of the ray NOT
// in t(-d), and the ray squares before it; no test against the own discs.
// The fills are valid for the board they were computed on: every path that
// changes the side to move computes them (legal() in step_lane), and k_play
// primes them after loading or resetting a board.
template <int N>
struct Fills {
    static_assert(Geo<N>::W == 1, "fills engine is for one-word boards (N <= 8)");
    static constexpr int LANES = 1;
    static constexpr int RAY_WORDS = 8 * 64;
    static constexpr int STEPS = Pro<N, 0, 1>::STEPS;
    static constexpr uint64_t BD = Geo<N>::BOARD.w[0], IN = Geo<N>::INNER.w[0];
    const uint64_t* rays;
    // t[d] = the fill to use for ray direction d (rays: E, S, SE, SW, W, N, NW, NE):
    // up directions (+S) use the -S fill, down directions the +S fill
    mutable uint64_t t[8];
    __device__ __forceinline__ Fills(int, const uint64_t* lds) : rays(lds) {}

    // get_possible_actions for mover P, keeping the fills: the axis-paired scan
    // on dwords (bitboard.hpp OneWord: v_bitop3 / v_and_or, carry-chain horizontal axis)
    __device__ __forceinline__ BB<1> legal(const BB<1>& Pb, const BB<1>& Ob) const {
        BB<1> r;
        r.w[0] = OneWord<N>::legal(Pb.w[0], Ob.w[0], t);
        return r;
    }
    // FIRST: the eight ray loads issued together before the runs (a scheduling
    // barrier after them), one LDS round trip instead of the two the backend's
    // interleaving left: greedy 100-ply launches 1.296 -> 1.264 us per ply, 6x6
    // random 0.791 -> 0.775, but 8x8 random 0.685 -> 0.689 (profiles/r06/t, u),
    // so k_play_rand asks for it except at 8x8 random play
    template <bool FIRST = false>
    __device__ __forceinline__ BB<1> flip(const BB<1>&, const BB<1>&, int a) const {
        const uint64_t* r = rays + a;
        // (the rays computed by RayMath instead of read from the LDS table: 8x8
        // 0.671 -> 0.696 us per ply, greedy +2.8 %, 6x6 +3.3 %: +38 VALU per ply cost
        // more than the LDS round trip they remove; profiles/r04/fm/ab.jsonl)
        uint64_t rr[8];
        if constexpr (FIRST) {
#pragma unroll
            for (int d = 0; d < 8; ++d) rr[d] = r[64 * d];
            __builtin_amdgcn_sched_barrier(0);
        }
        auto ray_of = [&](int d) __attribute__((always_inline)) { return FIRST ? rr[d] : r[64 * d]; };
        uint64_t f = 0;
#pragma unroll
        for (int d = 0; d < 4; ++d) {  // toward higher squares: cap = lowest ray square outside the fill
            const uint64_t ray = ray_of(d);
            const uint64_t y = ray & ~t[d];
            // ray & ((y & -y) - 1) == ray & t & (y - 1): one 3-input AND per dword
            f |= and3_64(ray, t[d], y - 1ull);
        }
        // toward lower squares on the board turned by 180 degrees (square s ->
        // NN-1-s, OneWord::turn180): the ray runs toward higher squares there,
        // so the same lowest-bit form applies to the turned fill; one turn of
        // the or-ed runs at the end.  The turned rays are tabled under the
        // unturned square (the same address as the other four)
        uint64_t g = 0;
#pragma unroll
        for (int d = 4; d < 8; ++d) {
            const uint64_t ray = ray_of(d);
            const uint64_t tt = OneWord<N>::turn180(t[d]);
            const uint64_t y = ray & ~tt;
            g |= and3_64(ray, tt, y - 1ull);
        }
        f |= OneWord<N>::turn180(g);
        BB<1> out;
        out.w[0] = f;
        return out;
    }
    // GreedyPolicy from the fills of the side to move (bitboard.hpp OneWord::greedy)
    __device__ __forceinline__ int greedy(const BB<1>& legal) const { return OneWord<N>::greedy(t, legal.w[0]); }
    // recompute the fills for the side to move (after a load or a reset)
    __device__ __forceinline__ void prime(const Lane<N>& s) const {
        const bool tw = (s.meta & M_TURN_WHITE) != 0;
        (void)legal(pick(tw, s.white, s.black), pick(tw, s.black, s.white));
    }
    __device__ __forceinline__ bool leader() const { return true; }
};

// FillsW<N>: the Fills engine for multi-word boards (N >= 9): the legal scan
// keeps its eight fills (legal_moves_fills) and update_board's flips come from
// them and a ray table of BB<W> entries in LDS (flips_fills), without the
// Kogge-Stone run and capping test per direction.
template <int N>
struct FillsW {
    static constexpr int W = Geo<N>::W;
    static constexpr int LANES = 1;
    static constexpr int RAY_WORDS = 8 * N * N * W;
    const BB<W>* rays;
    mutable BB<W> t[8];
    __device__ __forceinline__ FillsW(int, const uint64_t* lds) : rays(reinterpret_cast<const BB<W>*>(lds)) {}
    __device__ __forceinline__ BB<W> legal(const BB<W>& P, const BB<W>& O) const {
        return legal_moves_fills<N>(P, O, t);
    }
    __device__ __forceinline__ BB<W> flip(const BB<W>&, const BB<W>&, int a) const {
        return flips_fills<N>(rays, t, a);
    }
    __device__ __forceinline__ void prime(const Lane<N>& s) const {
        const bool tw = (s.meta & M_TURN_WHITE) != 0;
        BB<W> P, O;  // word-wise selects: a select of the two members' addresses puts the lane in scratch
#pragma unroll
        for (int i = 0; i < W; ++i) {
            P.w[i] = tw ? s.white.w[i] : s.black.w[i];
            O.w[i] = tw ? s.black.w[i] : s.white.w[i];
        }
        (void)legal(P, O);
    }
    __device__ __forceinline__ bool leader() const { return true; }
    __device__ static void fill(uint64_t* lds) {
        BB<W>* r = reinterpret_cast<BB<W>*>(lds);
        for (int i = threadIdx.x; i < 8 * N * N; i += BLOCK) r[i] = ray_from<N>(i / (N * N), i % (N * N));
        __syncthreads();
    }
};

// does the engine read the ray tables of the directions toward lower squares turned?
template <typename Eng>
struct turned_rays : std::false_type {};
template <int N>
struct turned_rays<Fills<N>> : std::true_type {};

template <typename Eng>
struct is_fills_w : std::false_type {};
template <int N>
struct is_fills_w<FillsW<N>> : std::true_type {};


// Quartet<N>: four lanes per board (N <= 8, one word), lanes 4k..4k+3 of a DPP
// quad: lane q scans one axis (E/W, S/N, SE/NW, SW/NE) and computes the flips
// of its two ray directions (q toward higher squares, q + 4 toward lower);
// the four parts are or-ed through quad_perm [1,0,3,2] and [2,3,0,1].  Every
// decision of step_lane is taken on the or-ed (quad-uniform) masks, so the four
// lanes always follow the same branches and the DPP steps never read an
// inactive lane.
template <int N>
struct Quartet {
    static_assert(Geo<N>::W == 1, "Quartet engine is for one-word boards (N <= 8)");
    static constexpr int LANES = 4;
    static constexpr int RAY_WORDS = 8 * 64;
    static constexpr uint64_t BD = Geo<N>::BOARD.w[0], IN = Geo<N>::INNER.w[0];
    const uint64_t* rays;  // this lane's "up" table; its "down" table is 4 * 64 words further
    uint32_t sh;           // axis shift: 1, N, N + 1, N - 1
    uint64_t pm;           // propagator mask: the vertical axis may pass edge columns
    int q;
    __device__ __forceinline__ Quartet(int lane_q, const uint64_t* lds) : q(lane_q) {
        rays = lds + 64 * lane_q;
        sh = lane_q == 0 ? 1u : (lane_q == 1 ? (uint32_t)N : (lane_q == 2 ? N + 1u : N - 1u));
        pm = lane_q == 1 ? BD : IN;
    }
    static constexpr int STEPS = Pro<N, 0, 1>::STEPS;
    // legal_moves along one axis (+s and -s) with a per-lane shift amount
    __device__ __forceinline__ static void axis(uint64_t P, uint64_t p1, uint32_t s, uint64_t& L) {
        uint64_t p2 = 0, p4 = 0;
        if constexpr (STEPS > 1) p2 = p1 & (p1 << s);
        if constexpr (STEPS > 2) p4 = p2 & (p2 << (2 * s));
        uint64_t t = (P << s) & p1;
        t |= p1 & (t << s);
        if constexpr (STEPS > 1) t |= p2 & (t << (2 * s));
        if constexpr (STEPS > 2) t |= p4 & (t << (4 * s));
        L |= t << s;
        t = (P >> s) & p1;
        t |= p1 & (t >> s);
        if constexpr (STEPS > 1) t |= (p2 >> s) & (t >> (2 * s));
        if constexpr (STEPS > 2) t |= (p4 >> (3 * s)) & (t >> (4 * s));
        L |= t >> s;
    }
    __device__ __forceinline__ static uint32_t quad_or32(uint32_t x) {
        x |= (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0xB1, 0xF, 0xF, false);
        return x | (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0x4E, 0xF, 0xF, false);
    }
    __device__ __forceinline__ static uint64_t quad_or(uint64_t x) {
        return ((uint64_t)quad_or32((uint32_t)(x >> 32)) << 32) | quad_or32((uint32_t)x);
    }
    __device__ __forceinline__ BB<1> legal(const BB<1>& Pb, const BB<1>& Ob) const {
        const uint64_t P = Pb.w[0], O = Ob.w[0];
        uint64_t L = 0;
        axis(P, O & pm, sh, L);
        BB<1> r;
        r.w[0] = quad_or(L) & ~(P | O) & BD;
        return r;
    }
    __device__ __forceinline__ BB<1> flip(const BB<1>& Pb, const BB<1>& Ob, int a) const {
        const uint64_t P = Pb.w[0], nO = ~Ob.w[0];
        uint64_t f;
        {  // toward higher squares: the nearest non-opponent square is the lowest set bit
            const uint64_t ray = rays[a];
            const uint64_t x = ray & nO;
            const uint64_t fb = x & (0ull - x);
            f = (fb & P) ? (ray & (fb - 1ull)) : 0ull;
        }
        {  // toward lower squares: the highest set bit
            const uint64_t ray = rays[4 * 64 + a];
            const uint64_t x = ray & nO;
            const uint64_t hb = x ? (0x8000000000000000ull >> __clzll(x)) : 0ull;
            f |= (hb & P) ? (ray & (0ull - (hb << 1))) : 0ull;
        }
        BB<1> out;
        out.w[0] = quad_or(f);
        return out;
    }
    __device__ __forceinline__ void prime(const Lane<N>&) const {}
    __device__ __forceinline__ bool leader() const { return q == 0; }
};

// OthelloBaseEnv.reset (othello.py:265-271); rand_left = SimpleOthelloEnv's
// random-opening length randint(0, k//2+1)*2 (othello.py:62-63) from Philox.
template <int N>
__device__ __forceinline__ void reset_lane(Lane<N>& s, uint64_t seed, uint32_t id, uint64_t ply, uint32_t purpose,
                                           int init_rand) {
    s.black = Start<N>::BLACK;
    s.white = Start<N>::WHITE;
    s.legal = legal_moves<N>(s.black, s.white);  // black moves first (othello.py:267)
    uint32_t rl = 0;
    if (init_rand > 0) rl = (uint32_t)scale_index(opening_draw(seed, id, ply, purpose), init_rand / 2 + 1) * 2u;
    s.meta = (rl & 0xffu) << M_RAND_SHIFT;
}

// The rest of OthelloBaseEnv.step after update_board (othello.py:425-462):
// full board / sudden death, the opponent's legal moves, pass and double pass,
// winner and reward.  P / O are the mover's / opponent's discs after the move.
template <int N, typename Eng>
__device__ __forceinline__ void finish_step(Lane<N>& s, bool tw, bool valid, const BB<Geo<N>::W>& P,
                                            const BB<Geo<N>::W>& O, uint32_t flags, int& reward, int& done,
                                            int& winner, const Eng& eng) {
    constexpr int W = Geo<N>::W;
    constexpr int NN = N * N;
    const bool full = !any(~(P | O) & Geo<N>::BOARD);                       // :425-426
    const bool sudden = !valid && (flags & OTH_SUDDEN_DEATH);              // :427
    const int pc = popcount(P), oc = popcount(O);
    const int cur = tw ? WHITE_DISK : BLACK_DISK;
    const int by_count = pc > oc ? cur : (pc < oc ? -cur : NO_DISK);       // determine_winner (:486-501)
    bool term = false, new_tw = tw;
    if (sudden || full) {  // :431-433 -- turn and possible_moves stay stale
        term = true;
        winner = sudden ? -cur : by_count;  // :475-485
    } else {               // :436-442
        const BB<W> om = eng.legal(O, P);
        const bool opp_pass = !any(om);
        BB<W> nl = om;
        if (opp_pass) nl = eng.legal(P, O);
        s.legal = nl;
        if (!opp_pass) {
            new_tw = !tw;
        } else if (!any(nl)) {  // nobody can move
            term = true;
            winner = by_count;
        }
    }
    s.white = pick(tw, P, O);  // word-wise: a store through a selected member address puts the lane in scratch
    s.black = pick(tw, O, P);
    int r = 0;  // :444-461
    if (term) {
        if (flags & OTH_DISK_REWARD) {
            r = sudden ? -NN : (oc == 0 ? NN : pc - oc);
        } else {
            r = winner * cur;
        }
    }
    const uint32_t wcode = winner == WHITE_DISK ? 1u : (winner == BLACK_DISK ? 2u : 0u);
    s.meta = (s.meta & 0xff00u) | (new_tw ? M_TURN_WHITE : 0u) | (term ? M_TERMINATED : 0u) |
             (term ? (wcode << M_WINNER_SHIFT) : 0u);
    reward = r;
    done = term ? 1 : 0;
}

// OthelloBaseEnv.step (othello.py:412-462) for one lane.  Returns the winner
// code (0 none) through `winner` when the game ends on this ply.
// PICKED: `a` is a policy's pick from s.legal, or -1 when s.legal is empty, so
// validity is a >= 0 and the flip is computed without a branch and masked.
template <int N, typename Eng, bool PICKED = false>
__device__ __forceinline__ void step_lane(Lane<N>& s, int a, uint32_t flags, int& reward, int& done, int& winner,
                                          const Eng& eng) {
    constexpr int W = Geo<N>::W;
    constexpr int NN = N * N;
    winner = NO_DISK;
    if (s.meta & M_TERMINATED) {  // reference: ValueError (othello.py:415-416)
        reward = 0;
        done = 1;
        return;
    }
    const bool tw = (s.meta & M_TURN_WHITE) != 0;
    BB<W> P = pick(tw, s.white, s.black);
    BB<W> O = pick(tw, s.black, s.white);
    if constexpr (PICKED && Eng::RAY_WORDS > 0 && W == 1) {
        const bool valid = a >= 0;
        const uint64_t m = valid ? 1ull << (a & 63) : 0ull;
        const uint64_t f = eng.flip(P, O, a & 63).w[0] & (0ull - (uint64_t)valid);
        P.w[0] |= f | m;
        O.w[0] &= ~(f | m);
        finish_step<N>(s, tw, valid, P, O, flags, reward, done, winner, eng);
        return;
    }
    const bool valid = a >= 0 && a < NN && test(s.legal, a);  // `action not in possible_moves` (:417)
    if (valid) {                                               // update_board (:391-410)
        const BB<W> m = square<W>(a);
        const BB<W> f = eng.flip(P, O, a);
        P |= f | m;
        O = O & ~(f | m);
    }
    finish_step<N>(s, tw, valid, P, O, flags, reward, done, winner, eng);
}

// RandomPolicy.get_action (simple_policies.py:37-41): possible_moves[randint(len)]
// with u = the ply's 32-bit draw.
template <int N>
__device__ __forceinline__ int random_action(const Lane<N>& s, uint32_t u) {
    const int n = popcount(s.legal);
    return select_bit(s.legal, scale_index(u, n));
}

// GreedyPolicy.get_action (simple_policies.py:69-92): the move that leaves the
// mover the most discs = the most flips; np.argmax keeps the first (lowest
// square) of equal counts.
template <int N, typename Eng>
__device__ __forceinline__ int greedy_action(const Lane<N>& s, const Eng& eng) {
    static_assert(Eng::LANES == 1, "greedy runs one lane per board");
    // every square's flip count on bit planes, no loop over the candidates
    if constexpr (std::is_same<Eng, Fills<N>>::value) {
        return eng.greedy(s.legal);  // the fills of the side to move are carried from the last scan
    } else if constexpr (Geo<N>::W == 1) {
        const bool tw = (s.meta & M_TURN_WHITE) != 0;
        uint64_t t[8];
        (void)OneWord<N>::legal(tw ? s.white.w[0] : s.black.w[0], tw ? s.black.w[0] : s.white.w[0], t);
        return OneWord<N>::greedy(t, s.legal.w[0]);
    } else if constexpr (is_fills_w<Eng>::value) {  // multi-word boards: the same planes on BB<W> (PlanesW)
        return PlanesW<N>::greedy(eng.t, s.legal);  // fills carried from the last scan
    } else {
        const bool tw = (s.meta & M_TURN_WHITE) != 0;
        BB<Geo<N>::W> t[8];
        (void)legal_moves_fills<N>(pick(tw, s.white, s.black), pick(tw, s.black, s.white), t);
        return PlanesW<N>::greedy(t, s.legal);
    }
}

// MaxiMinPolicy(depth).get_action (simple_policies.py:98-163).  P is the side to
// move at this node, O the other side; the root mover's ("my") discs are P at
// even levels and O at odd ones.  A child is a leaf when the search depth is
// reached, the board is full, or the side to reply has no move: the
// reference then either ends the game (double pass) or forces the turn to
// that side anyway (:139-144), whose empty move list ends the branch
// (:117-126) -- either way the leaf value is my disc count.  Ties keep the
// first (lowest) square: np.argmax / np.argmin (:152-154).  The depth is a
// template parameter, so the recursion unrolls into straight-line levels.
template <int N, int D, int LVL>
__device__ int maximin_node(const BB<Geo<N>::W>& P, const BB<Geo<N>::W>& O, const BB<Geo<N>::W>& L, int& move) {
    constexpr int W = Geo<N>::W;
    constexpr bool MINE = (LVL % 2) == 0;
    int best = MINE ? -1 : 0x7fffffff;
    move = -1;
#pragma unroll
    for (int i = 0; i < W; ++i) {
        uint64_t x = L.w[i];
        while (x) {
            const int b = __builtin_ctzll(x);
            x &= x - 1;
            BB<W> m = zero<W>();
            m.w[i] = 1ull << b;
            const BB<W> f = flips<N>(P, O, m);
            const BB<W> P2 = P | f | m;
            const BB<W> O2 = O & ~(f | m);
            int v = popcount(MINE ? P2 : O2);
            if constexpr (LVL + 2 == D) {
                // the child is the last level: its value is the mover's best flip
                // count over its moves (bit planes, no loop): my discs after the
                // child's move are O2 + flips + 1 when I move there, P2 - flips otherwise
                if (any(~(P2 | O2) & Geo<N>::BOARD)) {
                    BB<W> t2[8];
                    const BB<W> L2 = legal_moves_fills<N>(O2, P2, t2);
                    if (any(L2)) {
                        const int mf = PlanesW<N>::max_flips(t2, L2);
                        v = ((LVL + 1) % 2 == 0) ? popcount(O2) + 1 + mf : popcount(P2) - mf;
                    }
                }
            } else if constexpr (LVL + 1 < D) {
                if (any(~(P2 | O2) & Geo<N>::BOARD)) {
                    const BB<W> L2 = legal_moves<N>(O2, P2);
                    if (any(L2)) {
                        int unused;
                        v = maximin_node<N, D, LVL + 1>(O2, P2, L2, unused);
                    }
                }
            }
            if (MINE ? v > best : v < best) {
                best = v;
                move = 64 * i + b;
            }
        }
    }
    return best;
}

// MaxiMinPolicy(D).get_action for a runtime depth D (the OTH_POLICY_MAXIMIN_DEEP
// launches, D >= 4; maximin_node's rules): the reference's recursion
// (simple_policies.py:111-155) as a depth-first walk over an explicit stack,
// one level per search depth -- level l moves the root's side at even l and
// holds (mover, other, moves not yet tried, best value, move being tried).
// The level above the leaves takes its value from the greedy planes' maximum
// flip count, as maximin_node does.  -1 without a move (the reference's None).
template <int N>
__device__ int maximin_search(const BB<Geo<N>::W>& P0, const BB<Geo<N>::W>& O0, const BB<Geo<N>::W>& L0, int D) {
    constexpr int W = Geo<N>::W;
    constexpr int MAXD = OTH_MAXIMIN_MAX_DEPTH;
    BB<W> SP[MAXD], SO[MAXD], SR[MAXD];
    int SV[MAXD], SM[MAXD];
    if (!any(L0)) return -1;
    int best_move = -1, l = 0;
    SP[0] = P0;
    SO[0] = O0;
    SR[0] = L0;
    SV[0] = -1;
    for (;;) {
        if (!any(SR[l])) {  // every move of level l tried: its value goes to the level above
            if (l == 0) break;
            const int v = SV[l];
            --l;
            if ((l & 1) == 0 ? v > SV[l] : v < SV[l]) {  // np.argmax / np.argmin: the first of equals
                SV[l] = v;
                if (l == 0) best_move = SM[l];
            }
            continue;
        }
        // the lowest untried move of level l (possible_moves ascending)
        BB<W> R = SR[l], m = zero<W>();
        int b = -1;
#pragma unroll
        for (int i = W - 1; i >= 0; --i)
            if (R.w[i]) b = 64 * i + ctz64(R.w[i]);
#pragma unroll
        for (int i = 0; i < W; ++i) {
            m.w[i] = (b >> 6) == i ? 1ull << (b & 63) : 0ull;
            R.w[i] &= ~m.w[i];
        }
        SR[l] = R;
        SM[l] = b;
        const BB<W> P = SP[l], O = SO[l];
        const BB<W> f = flips<N>(P, O, m);
        const BB<W> P2 = P | f | m;
        const BB<W> O2 = O & ~(f | m);
        const bool mine = (l & 1) == 0;
        int v = popcount(mine ? P2 : O2);  // a leaf: my disc count (:117-126)
        bool leaf = true;
        if (l + 1 < D && any(~(P2 | O2) & Geo<N>::BOARD)) {
            BB<W> t2[8];
            const BB<W> L2 = legal_moves_fills<N>(O2, P2, t2);
            if (any(L2)) {  // no reply: the game ends or the turn is forced back to a side without moves
                if (l + 2 == D) {  // the child's moves end the search: its best from the planes
                    const int mf = PlanesW<N>::max_flips(t2, L2);
                    v = ((l + 1) & 1) == 0 ? popcount(O2) + 1 + mf : popcount(P2) - mf;
                } else {
                    ++l;
                    SP[l] = O2;
                    SO[l] = P2;
                    SR[l] = L2;
                    SV[l] = (l & 1) == 0 ? -1 : 0x7fffffff;
                    leaf = false;
                }
            }
        }
        if (leaf && (mine ? v > SV[l] : v < SV[l])) {
            SV[l] = v;
            if (l == 0) best_move = b;
        }
    }
    return best_move;
}

template <int N, int D>
__device__ __forceinline__ int maximin_action(const Lane<N>& s) {
    const bool tw = (s.meta & M_TURN_WHITE) != 0;
    int move;
    maximin_node<N, D, 0>(pick(tw, s.white, s.black), pick(tw, s.black, s.white), s.legal, move);
    return move;
}

// The move of a deterministic scripted policy (everything but RANDOM); depth:
// the search depth of OTH_POLICY_MAXIMIN_DEEP (Rng::depth).
constexpr int OTH_POLICY_MAXIMIN_DEEP = 0x100;  // launcher-internal: MaxiMin of a runtime depth >= 4
template <int N, int POLICY, typename Eng>
__device__ __forceinline__ int policy_action(const Lane<N>& s, const Eng& eng, int depth = 0) {
    if constexpr (POLICY == OTH_POLICY_GREEDY) {
        return greedy_action<N>(s, eng);
    } else if constexpr (POLICY == OTH_POLICY_MAXIMIN2) {
        return maximin_action<N, 2>(s);
    } else if constexpr (POLICY == OTH_POLICY_MAXIMIN3) {
        return maximin_action<N, 3>(s);
    } else if constexpr (POLICY == OTH_POLICY_MAXIMIN_DEEP) {
        const bool tw = (s.meta & M_TURN_WHITE) != 0;
        return maximin_search<N>(pick(tw, s.white, s.black), pick(tw, s.black, s.white), s.legal, depth);
    } else {
        return -1;
    }
}

__device__ __forceinline__ uint32_t wave_sum(uint32_t v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}

// Add this block's finished games {black wins, draws, white wins} to its own
// slot wdl[blockIdx.x][0..2].  One slot per block: no atomics, no contention
// (launches on a stream are ordered, and block b of every launch owns slot b);
// oth_counts sums the slots.  Every thread of the block must call this.
__device__ __forceinline__ void tally(unsigned long long* wdl, uint32_t b, uint32_t d, uint32_t w) {
    b = wave_sum(b);
    d = wave_sum(d);
    w = wave_sum(w);
    __shared__ uint32_t part[BLOCK / 64][3];
    const int wave = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 0) {
        part[wave][0] = b;
        part[wave][1] = d;
        part[wave][2] = w;
    }
    __syncthreads();
    if (threadIdx.x == 0 && wdl) {
        uint32_t sb = 0, sd = 0, sw = 0;
#pragma unroll
        for (int i = 0; i < BLOCK / 64; ++i) {
            sb += part[i][0];
            sd += part[i][1];
            sw += part[i][2];
        }
        if (sb | sd | sw) {
            unsigned long long* slot = wdl + 4 * (size_t)blockIdx.x;
            // only this block touches its slot: uncontended atomics without a
            // return value are posted, so the block does not wait for the slot's
            // read (the read-modify-write cost one memory round trip per launch)
            if (sb) atomicAdd(slot + 0, (unsigned long long)sb);
            if (sd) atomicAdd(slot + 1, (unsigned long long)sd);
            if (sw) atomicAdd(slot + 2, (unsigned long long)sw);
        }
    }
}

// A launch's draw context (and the search depth of OTH_POLICY_MAXIMIN_DEEP launches).
struct Rng {
    uint64_t seed;
    uint32_t id_base;
    int init_rand;
    const uint64_t* ply_off;  // device offset of the ply counter: slot 0 (= 0) eagerly, a graph region's slot under capture
    int depth;                // MaxiMinPolicy(depth) for OTH_POLICY_MAXIMIN_DEEP (depth >= 4)
};

template <int N>
__global__ __launch_bounds__(BLOCK) void k_reset(uint64_t* __restrict__ boards, uint16_t* __restrict__ meta,
                                                 uint64_t* __restrict__ legal, int E,
                                                 const uint8_t* __restrict__ mask, Rng rng, uint64_t ply) {
    ply += *rng.ply_off;  // graph-region offset (oth_graph_end); 0 eagerly
    const int e = blockIdx.x * BLOCK + threadIdx.x;
    if (e >= E) return;
    if (mask && !mask[e]) return;
    Lane<N> s;
    reset_lane<N>(s, rng.seed, rng.id_base + (uint32_t)e, ply, RNG_OPENING_RESET, rng.init_rand);
    store_lane<N>(s, boards, meta, legal, e);
}

// oth_step: external actions, one ply.
// Per-wave W/D/L slot of a single-ply launch: slot w of the handle's
// [nslots][4] array belongs to wave w of the grid (nslots = ceil(4E / 64) covers
// every wave of a grid of up to four lanes per board; a wave past E reads the
// last live wave's slot and never writes).  The wave's counts accumulate in SGPRs over its boards (three
// ballots per group of 64) and lane 0 adds them with plain stores at the end.
// Launches on a stream are ordered, so the read at a launch's start sees every
// earlier launch's adds.
struct WaveSlot {
    unsigned long long* p;
    unsigned long long v0, v1, v2;
    uint32_t nb = 0, nd = 0, nw = 0;
    __device__ __forceinline__ WaveSlot(unsigned long long* wdl, int t, int E) : WaveSlot(wdl, min(t >> 6, (E - 1) >> 6)) {}
    // slot `wave` (the caller's wave index, clamped to its last live wave)
    __device__ __forceinline__ explicit WaveSlot(unsigned long long* wdl, int wave) {
        // wave-uniform: the slot is read by scalar loads into SGPRs (the values
        // live through the whole kernel; written back by lane 0's vector stores)
        const int w = __builtin_amdgcn_readfirstlane(wave);
        p = wdl + 4 * (size_t)w;
        const ulonglong2 a = *reinterpret_cast<const ulonglong2*>(p);
        v0 = a.x;
        v1 = a.y;
        v2 = p[2];
    }
    // {black wins, draws, white wins} of this wave's lanes (0 / 1 each)
    __device__ __forceinline__ void count(bool b, bool d, bool w) {
        nb += (uint32_t)__popcll(__ballot(b));
        nd += (uint32_t)__popcll(__ballot(d));
        nw += (uint32_t)__popcll(__ballot(w));
    }
    __device__ __forceinline__ void flush() const {
        if ((nb | nd | nw) && (threadIdx.x & 63) == 0) {
            ulonglong2 a;
            a.x = v0 + nb;
            a.y = v1 + nd;
            *reinterpret_cast<ulonglong2*>(p) = a;
            p[2] = v2 + nw;
        }
    }
};

template <int N>
__global__ __launch_bounds__(BLOCK) void k_step(uint64_t* __restrict__ boards, uint16_t* __restrict__ meta,
                                                uint64_t* __restrict__ legal, int E, uint32_t flags,
                                                const int32_t* __restrict__ actions, int32_t* __restrict__ rewards,
                                                uint8_t* __restrict__ dones, unsigned long long* __restrict__ wdl,
                                                Rng rng, uint64_t ply) {
    ply += *rng.ply_off;  // graph-region offset (oth_graph_end); 0 eagerly
    const int e = blockIdx.x * BLOCK + threadIdx.x;
    uint32_t cb = 0, cd = 0, cw = 0;
    WaveSlot slot(wdl, e, E);
    if (e < E) {
        Lane<N> s;
        load_lane<N>(s, boards, meta, legal, e);
        const int a = actions[e];  // with the board's loads, not behind the terminated test
        const bool was_term = (s.meta & M_TERMINATED) != 0;
        int r, d, win;
        step_lane<N>(s, a, flags, r, d, win, Solo<N>(0, nullptr));
        if (d && !was_term) {
            cb = win == BLACK_DISK;
            cd = win == NO_DISK;
            cw = win == WHITE_DISK;
            if (flags & OTH_AUTO_RESET)
                reset_lane<N>(s, rng.seed, rng.id_base + (uint32_t)e, ply, RNG_OPENING_AUTO, rng.init_rand);
        }
        store_lane<N>(s, boards, meta, legal, e);
        if (rewards) rewards[e] = r;
        if (dones) dones[e] = (uint8_t)d;
    }
    slot.count(cb != 0, cd != 0, cw != 0);
    slot.flush();
}

// oth_step_policy: `plies` plies of on-device play with the board kept in
// registers between plies; per-ply outputs stored [ply][E].  Eng::LANES lanes
// per board (Eng::LANES); only the group's leader lane stores.
// REC: all three per-ply outputs requested (stores without per-pointer branches,
// so the ply's tail stays one basic block the scheduler can interleave).
template <int N, int POLICY, typename Eng, bool REC>
__global__ __launch_bounds__(BLOCK) void k_play(uint64_t* __restrict__ boards, uint16_t* __restrict__ meta,
                                                uint64_t* __restrict__ legal, int E, uint32_t flags, int plies,
                                                int32_t* __restrict__ actions, int32_t* __restrict__ rewards,
                                                uint8_t* __restrict__ dones, unsigned long long* __restrict__ wdl,
                                                Rng rng, uint64_t ply0) {
    ply0 += *rng.ply_off;  // graph-region offset (oth_graph_end); 0 eagerly
    __shared__ __attribute__((aligned(16))) uint64_t lds_rays[Eng::RAY_WORDS > 0 ? Eng::RAY_WORDS : 1];
    if constexpr (is_fills_w<Eng>::value) Eng::fill(lds_rays);
    else if constexpr (Eng::RAY_WORDS > 0) fill_rays<N, turned_rays<Eng>::value>(lds_rays);
    const int gt = blockIdx.x * BLOCK + threadIdx.x;
    const int e = gt / Eng::LANES;
    const Eng eng(gt % Eng::LANES, lds_rays);
    const bool lead = eng.leader();
    uint32_t cb = 0, cd = 0, cw = 0;
    if (e < E) {
        const uint32_t id = rng.id_base + (uint32_t)e;
        Lane<N> s;
        load_lane<N>(s, boards, meta, legal, e);
        eng.prime(s);
        int32_t* act_p = actions + e;
        int32_t* rew_p = rewards + e;
        uint8_t* done_p = dones + e;
        // one ply; u_rand = the random policy's 32-bit draw for this ply
        auto ply = [&](int p, uint32_t u_rand) __attribute__((always_inline)) {
            const uint64_t g = ply0 + (uint64_t)p;
            const size_t o = (size_t)p * (size_t)E + (size_t)e;
            int a = -1, r = 0, d = 1, win = NO_DISK;
            if (!(s.meta & M_TERMINATED)) {
                const uint32_t rl = s.meta >> M_RAND_SHIFT;
                if (POLICY == OTH_POLICY_RANDOM || rl > 0) {
                    const uint32_t u = POLICY == OTH_POLICY_RANDOM ? u_rand : action_draw(rng.seed, id, g);
                    a = random_action<N>(s, u);
                    if (rl > 0) s.meta -= 1u << M_RAND_SHIFT;
                } else {
                    a = policy_action<N, POLICY>(s, eng, rng.depth);
                }
                step_lane<N, Eng, true>(s, a, flags, r, d, win, eng);  // a: a pick from s.legal
                if (d) {
                    cb += win == BLACK_DISK;
                    cd += win == NO_DISK;
                    cw += win == WHITE_DISK;
                    if (flags & OTH_AUTO_RESET) {
                        reset_lane<N>(s, rng.seed, id, g, RNG_OPENING_AUTO, rng.init_rand);
                        eng.prime(s);
                    }
                }
            }
            if (lead) {
                if constexpr (REC) {  // running pointers: one 64-bit add each per ply
                    *act_p = a;
                    *rew_p = r;
                    *done_p = (uint8_t)d;
                    act_p += E;
                    rew_p += E;
                    done_p += E;
                } else {
                    if (actions) actions[o] = a;
                    if (rewards) rewards[o] = r;
                    if (dones) dones[o] = (uint8_t)d;
                }
            }
        };
        if constexpr (POLICY == OTH_POLICY_RANDOM) {
            // Philox block g/4 gives plies 4k..4k+3 their words x, y, z, w: four
            // plies unrolled per block once g is 4-aligned (g is uniform, so
            // these branches are scalar); single plies before and after
            int p = 0;
            while (p < plies) {
                const uint64_t g = ply0 + (uint64_t)p;
                const U4 d4 = philox4(rng.seed, id, g >> 2, RNG_ACTION);
                if ((g & 3) == 0 && p + 4 <= plies) {
                    ply(p, d4.x);
                    ply(p + 1, d4.y);
                    ply(p + 2, d4.z);
                    ply(p + 3, d4.w);
                    p += 4;
                } else {
                    ply(p, pick4(d4, (uint32_t)(g & 3)));
                    ++p;
                }
            }
        } else {  // scripted policies draw only on random-opening plies (action_draw inside ply)
            for (int p = 0; p < plies; ++p) ply(p, 0u);
        }
        if (lead) store_lane<N>(s, boards, meta, legal, e);
    }
    if (!lead) cb = cd = cw = 0;
    tally(wdl, cb, cd, cw);
}

// k_play_rand: oth_step_policy(RANDOM) on one-word boards with auto-reset and
// every per-ply output stored -- the benchmark configuration -- with the
// same results as k_play<N, RANDOM, Fills<N>, true>, restructured for one
// wave per SIMD, where every VALU instruction of every path a lane of the
// wave takes is paid by the whole wave:
//   * the board is held as (mover, opponent) plus the side-to-move bit, so a
//     ply swaps two words once instead of selecting mover / opponent from
//     (black, white) and writing them back (othello.py:412-462 flips the
//     `player_turn`, not the board);
//   * with auto-reset no board is terminated at a ply's start, so there is no
//     per-ply "terminated?" branch and no branch-join copies of the carried
//     fills (a wave holding a board loaded terminated runs k_play's body);
//   * the opponent's legal scan runs unconditionally (on a full board it
//     finds nothing: no empty square); only a pass re-scans, in place.
// The random pick is always legal, so sudden death never triggers here.
// POLICY GREEDY (k_play_rand<N, GREEDY>): GreedyPolicy's move from the bit
// planes of the carried fills (simple_policies.py:69-92), a random move while
// random-opening plies remain (SimpleOthelloEnv, othello.py:60-79).
// OPEN: some board of the wave may have random-opening plies left (the
// handle's initial_rand_steps > 0, or a board loaded with some); without, the
// opening bookkeeping is compiled out.
struct NoFill {
    __device__ __forceinline__ void operator()() const {}
};


// the terminal ply's reward: the disk difference (disk_reward, othello.py:446-459)
// or the sign.  By a mask on the uniform flag: as `if (flags & ...)` the backend
// made a scalar branch of it inside the terminal block (multi-word play: one per
// ply the block runs, ~40-80 cycles to a lone wave)
__device__ __forceinline__ int term_reward(uint32_t flags, int disk, int sg) {
    const uint32_t m = 0u - (uint32_t)((flags & OTH_DISK_REWARD) != 0u);
    return (int)__builtin_amdgcn_bitop3_b32(m, (uint32_t)disk, (uint32_t)sg, 0xCA);
}

// black wins / draws / white wins from play_rand_fast's (sum of black's signs, games, decided games)
__device__ __forceinline__ void tally_from_signs(uint32_t s, uint32_t g, uint32_t z, uint32_t& cb, uint32_t& cd,
                                                 uint32_t& cw) {
    cb += (z + s) >> 1;
    cw += (z - s) >> 1;
    cd += g - z;
}
// FILL: independent work (the next Philox block) run after the opponent's scan
// and pinned there, so that it shares the ply's first scheduling region with the
// pick, the ray-table loads, the flips and the scan
template <int N, int POLICY = OTH_POLICY_RANDOM, bool OPEN = true, typename Eng = Fills<N>, typename FILL = NoFill>
__device__ __forceinline__ void play_rand_fast(uint64_t& M, uint64_t& O, uint64_t& L, uint32_t& meta,
                                               const Eng& eng, uint32_t u, uint32_t flags, const Rng& rng,
                                               uint32_t id, uint64_t g, int& a, int& r, int& d, uint32_t& cb,
                                               uint32_t& cd, uint32_t& cw, const FILL& fill = FILL{},
                                               const uint8_t* sel8 = nullptr) {
    constexpr uint64_t BD = Geo<N>::BOARD.w[0];
    constexpr int NN = N * N;
    // the k-th legal square, the bit inside its byte from the 2-KiB LDS table
    auto pick = [&](uint32_t draw) __attribute__((always_inline)) {
        const int k = scale_index(draw, popc64(L));
        return select64_tab(L, k, sel8);
    };
    if constexpr (POLICY == OTH_POLICY_RANDOM) {
        a = pick(u);  // RandomPolicy (simple_policies.py:37-41); L != 0
    } else if constexpr (OPEN) {
        // a random-opening ply draws u = action_draw(seed, id, g), from the caller's block
        // both computed and selected: as two exec-masked branches the wave ran both on
        // most plies (some board of the 64 in its opening) with the pick's LDS round
        // trip exposed between them; selected, the greedy planes' independent work
        // hides it: config 3 at 65,536 boards 1.378 -> 1.318 us per ply (100-ply
        // launches), 1.744 -> 1.697 (10-ply; profiles/r06/f)
        const int ap = pick(u), ag = OneWord<N>::greedy(eng.t, L);
        a = (meta & 0xff00u) ? ap : ag;
    } else {
        a = OneWord<N>::greedy(eng.t, L);
    }
    if constexpr (OPEN) meta -= (meta & 0xff00u) ? (1u << M_RAND_SHIFT) : 0u;  // a random-opening ply used up
    const uint64_t m = 1ull << a;
    BB<1> dummy;
    dummy.w[0] = 0;
    constexpr bool RAYS_FIRST = POLICY != OTH_POLICY_RANDOM || N != 8;
    uint64_t f;  // update_board (othello.py:391-410)
    if constexpr (std::is_same<Eng, Fills<N>>::value) f = eng.template flip<RAYS_FIRST>(dummy, dummy, a).w[0];
    else f = eng.flip(dummy, dummy, a).w[0];
    const uint64_t Mn = M | f | m, On = O & ~f;
    const bool full = (Mn | On) == BD;  // :425-426
    if constexpr (POLICY == OTH_POLICY_RANDOM) {
        // random play: a full board ends the game and auto-resets (othello.py:256-271)
        // before the scan, which then runs on the start position (black to move)
        // instead of the full board, where it would find nothing: the reset's
        // possible_moves and fills come from it and the terminal block holds no reset
        // moves; only a double pass (inside the pass block) resets explicitly.  8x8
        // 0.678 -> 0.675 us per ply, 6x6 -1.6 %; for greedy play it measured 3 % slower
        // (the scan waits on the full-board select), so greedy keeps the reset in the
        // terminal block (profiles/r04/g/ab_term.jsonl)
        constexpr uint64_t B0 = Start<N>::BLACK.w[0], W0 = Start<N>::WHITE.w[0];
        BB<1> pb, ob;
        pb.w[0] = full ? B0 : On;
        ob.w[0] = full ? W0 : Mn;
        uint64_t Ln = eng.legal(pb, ob).w[0];  // the next mover's possible_moves (:436), fills kept in eng.t
        fill();
        const bool pass = Ln == 0;  // never on the start position
        bool term = full;
        M = pb.w[0];
        O = ob.w[0];
        if (pass) {  // :437-440: the mover moves again (fills recomputed for the mover)
            pb.w[0] = Mn;
            ob.w[0] = On;
            Ln = eng.legal(pb, ob).w[0];
            M = Mn;
            O = On;
            if (Ln == 0) {  // nobody can move (:441-442): reset
                term = true;
                M = B0;
                O = W0;
                constexpr uint64_t START_MOVES = start_moves<N>();
                constexpr StartFills<N> SF = start_fills<N>();
                Ln = START_MOVES;
#pragma unroll
                for (int k = 0; k < 8; ++k) eng.t[k] = SF.t[k];
            }
        }
        L = Ln;
        const uint32_t mover = meta;
        meta ^= pass ? 0u : M_TURN_WHITE;
        r = 0;
        d = term ? 1 : 0;
        if (term) {
            const int pc = popc64(Mn), oc = popc64(On), df = pc - oc;
            const int sg = sign_i32(df);  // the mover's result
            r = term_reward(flags, oc == 0 ? NN : df, sg);  // :446-459 / winner * player_turn
            // the tally as (cb, cd, cw) = (sum of black's signs, games, decided games),
            // turned into wins / draws / wins by tally_from_signs: three adds, no selects
            const int mw = -(int)(mover & M_TURN_WHITE);  // 0 black, -1 white
            const int sb = (sg ^ mw) - mw;                // black's result
            cb += (uint32_t)sb;
            cd += 1u;
            cw += (uint32_t)__mul24(sb, sb);
            uint32_t rl = 0;
            if (rng.init_rand > 0)
                rl = (uint32_t)scale_index(opening_draw(rng.seed, id, g, RNG_OPENING_AUTO), rng.init_rand / 2 + 1) * 2u;
            meta = (rl & 0xffu) << M_RAND_SHIFT;
        }
    } else {
        BB<1> pb, ob;
        pb.w[0] = On;
        ob.w[0] = Mn;
        uint64_t Ln = eng.legal(pb, ob).w[0];  // the opponent's possible_moves (:436), fills kept in eng.t
        fill();
        const bool pass = Ln == 0 && !full;
        if (pass) {  // :437-440: the mover moves again (fills recomputed for the mover)
            pb.w[0] = Mn;
            ob.w[0] = On;
            Ln = eng.legal(pb, ob).w[0];
        }
        const bool term = full || Ln == 0;  // full board or nobody can move (:441-442)
        // (M, O) := (next mover, its opponent).  Alternating the two words' roles
        // statically from ply to ply instead (no selects; a pass swapping them in its
        // own exec-masked block) measured 2.3 % slower; per-ply outputs through buffer descriptors (no 64-bit
        // address VALU) 2.3 % slower too, their descriptor SALU in the same issue stream
        // (profiles/r03/st/)
        const bool swap = !pass && !full;
        M = swap ? On : Mn;
        O = swap ? Mn : On;
        L = Ln;
        meta ^= swap ? M_TURN_WHITE : 0u;
        r = 0;
        d = term ? 1 : 0;
        if (term) {
            const int pc = popc64(Mn), oc = popc64(On), df = pc - oc;
            const int sg = sign_i32(df);  // the mover's result
            r = term_reward(flags, oc == 0 ? NN : df, sg);  // :446-459 / winner * player_turn
            // the tally as (cb, cd, cw) = (sum of black's signs, games, decided games),
            // turned into wins / draws / wins by tally_from_signs: three adds, no selects
            const int m = -(int)(meta & M_TURN_WHITE);  // the mover (the turn is not passed on): 0 black, -1 white
            const int sb = (sg ^ m) - m;                // black's result
            cb += (uint32_t)sb;
            cd += 1u;
            cw += (uint32_t)__mul24(sb, sb);
            // auto-reset (othello.py:256-271): black to move from the start position
            M = Start<N>::BLACK.w[0];
            O = Start<N>::WHITE.w[0];
            constexpr uint64_t START_MOVES = start_moves<N>();  // constant-evaluated
            constexpr StartFills<N> SF = start_fills<N>();
            L = START_MOVES;
#pragma unroll
            for (int k = 0; k < 8; ++k) eng.t[k] = SF.t[k];
            uint32_t rl = 0;
            if (rng.init_rand > 0)
                rl = (uint32_t)scale_index(opening_draw(rng.seed, id, g, RNG_OPENING_AUTO), rng.init_rand / 2 + 1) * 2u;
            meta = (rl & 0xffu) << M_RAND_SHIFT;
        }
    }
}

// tables: the handle's ray + sel8 tables (oth_env::rays, k_fill_rays), copied into
// LDS by one 16-byte and one 8-byte load per thread, issued with the board's loads
// (against building them per block: greedy 10-ply launches 1.85 -> 1.80 us per
// ply, random 100-ply 0.679 -> 0.678; profiles/r04/b/)
template <int N, int POLICY = OTH_POLICY_RANDOM>
__global__ __launch_bounds__(BLOCK) void k_play_rand(uint64_t* __restrict__ boards, uint16_t* __restrict__ meta,
                                                     uint64_t* __restrict__ legal, int E, uint32_t flags, int plies,
                                                     int32_t* __restrict__ actions, int32_t* __restrict__ rewards,
                                                     uint8_t* __restrict__ dones,
                                                     unsigned long long* __restrict__ wdl, Rng rng, uint64_t ply0,
                                                     const uint64_t* __restrict__ tables) {
    static_assert(Geo<N>::W == 1, "one-word boards");
    static_assert(BLOCK == 256 && Fills<N>::RAY_WORDS == 2 * BLOCK, "two ray words and one sel8 word a thread");
    ply0 += *rng.ply_off;  // graph-region offset (oth_graph_end); 0 eagerly
    __shared__ __attribute__((aligned(16))) uint64_t lds_rays[Fills<N>::RAY_WORDS];
    __shared__ __attribute__((aligned(16))) uint64_t lds_sel[256];
    const uint8_t* sel8 = reinterpret_cast<const uint8_t*>(lds_sel);
    const int e = blockIdx.x * BLOCK + threadIdx.x;
    Lane<N> s;
    const ulonglong2 tr = reinterpret_cast<const ulonglong2*>(tables)[threadIdx.x];
    const uint64_t ts = tables[Fills<N>::RAY_WORDS + threadIdx.x];
    if (e < E) load_lane<N>(s, boards, meta, legal, e);
    reinterpret_cast<ulonglong2*>(lds_rays)[threadIdx.x] = tr;
    lds_sel[threadIdx.x] = ts;
    __syncthreads();
    uint32_t cb = 0, cd = 0, cw = 0;
    if (e < E) {
        const uint32_t id = rng.id_base + (uint32_t)e;
        const Fills<N> eng(0, lds_rays);
        const bool tw0 = (s.meta & M_TURN_WHITE) != 0;
        uint64_t M = tw0 ? s.white.w[0] : s.black.w[0];
        uint64_t O = tw0 ? s.black.w[0] : s.white.w[0];
        uint64_t L = s.legal.w[0];
        uint32_t mt = s.meta & (0xff00u | M_TURN_WHITE);
        eng.prime(s);
        // a board loaded terminated stays so (k_play's semantics), and a live board
        // loaded with no possible move takes the invalid path (othello.py:417-427,
        // possible_moves == [] before a reset, :242); such a wave is rare
        // (set_state) and takes the generic loop below.  Inside the fast loop no
        // live board has L == 0: a pass re-scans, a double pass terminates and
        // auto-resets.
        const bool slow = __any((s.meta & M_TERMINATED) != 0 || L == 0);
        int32_t* act_p = actions + e;
        int32_t* rew_p = rewards + e;
        uint8_t* done_p = dones + e;
        uint32_t t0 = 0, t1 = 0, t2 = 0;  // play_rand_fast's tally (tally_from_signs)
        auto fast = [&](auto OPENC) __attribute__((always_inline)) {
        constexpr bool OPEN = decltype(OPENC)::value;
        auto ply = [&](int p, uint32_t u, const auto& fill) __attribute__((always_inline)) {
            int a, r, d;
            play_rand_fast<N, POLICY, OPEN>(M, O, L, mt, eng, u, flags, rng, id, ply0 + (uint64_t)p, a, r, d, t0, t1,
                                            t2, fill, sel8);
            // the trajectory rows are written once: streaming stores (+0.9 % at 65,536
            // boards, +0.7 % at 131,072; profiles/r03/nt/).  Row stores at a scalar
            // (SGPR) row base and a constant lane offset -- 3 VALU fewer per ply, 32 SALU
            // more per 4-ply group -- measured 0.674 -> 0.709 us per ply (the lone wave's
            // issue slots: profiles/r04/c/ab_saddr.jsonl), so the running pointers stay
            __builtin_nontemporal_store(a, act_p);
            __builtin_nontemporal_store(r, rew_p);
            __builtin_nontemporal_store((uint8_t)d, done_p);
            act_p += E;
            rew_p += E;
            done_p += E;
        };
        const NoFill nofill;
        if constexpr (POLICY != OTH_POLICY_RANDOM) {  // scripted policy: draws only on opening plies
            if constexpr (OPEN) {
                // an opening ply's draw is word g % 4 of Philox block g / 4 (action_draw's
                // value).  Plies in groups of four from a multiple of 4, as random play
                // does: the group's block computed at its start and its words taken
                // statically, instead of a per-ply test for a new block and a per-ply
                // word choice (both scalar branches, ~40-80 cycles each to a lone wave):
                // config 3 at 65,536 boards, 100-ply launches 1.315 -> 1.256-1.263 us per
                // ply (profiles/r06/j, k).  (The auto-reset's opening-length draw in block form
                // measured 3-4 % slower: a wave's greedy games run almost in step, so
                // few plies see a game end, profiles/r04/oblk/.)
                int p = 0;
                // plies [p, q) inside one group: its block once, the words by pick4
                auto partial = [&](int q) __attribute__((always_inline)) {
                    const U4 blk = philox4(rng.seed, id, (ply0 + (uint64_t)p) >> 2, RNG_ACTION);
                    for (; p < q; ++p) ply(p, pick4(blk, (uint32_t)((ply0 + (uint64_t)p) & 3)), nofill);
                };
                const int head = (int)((4u - (uint32_t)(ply0 & 3)) & 3u);
                if (head > 0) partial(head < plies ? head : plies);
                while (p + 4 <= plies) {
                    const U4 blk = philox4(rng.seed, id, (ply0 + (uint64_t)p) >> 2, RNG_ACTION);
                    ply(p, blk.x, nofill);
                    ply(p + 1, blk.y, nofill);
                    ply(p + 2, blk.z, nofill);
                    ply(p + 3, blk.w, nofill);
                    p += 4;
                }
                if (p < plies) partial(plies);
            } else {
                for (int p = 0; p < plies; ++p) ply(p, 0u, nofill);
            }
            return;
        }
        int p = 0;
            // Philox block g/4 serves plies 4k..4k+3 (g uniform: scalar branches).
            // The next block is computed in the current group's first ply, after its
            // opponent scan and pinned there (FILL), where its independent VALU
            // work shares the ply's scheduling region (profiles/r02/fi/).
            while (p < plies && ((ply0 + (uint64_t)p) & 3) != 0) {
                const uint64_t g = ply0 + (uint64_t)p;
                ply(p, pick4(philox4(rng.seed, id, g >> 2, RNG_ACTION), (uint32_t)(g & 3)), nofill);
                ++p;
            }
            if (p + 4 <= plies) {
                U4 cur = philox4(rng.seed, id, (ply0 + (uint64_t)p) >> 2, RNG_ACTION);
                while (p + 4 <= plies) {
                    U4 nxt;  // (one unused block after the last group)
                    const uint64_t nb = ((ply0 + (uint64_t)p) >> 2) + 1;
                    ply(p, cur.x, [&]() __attribute__((always_inline)) {
                        nxt = philox4(rng.seed, id, nb, RNG_ACTION);
                        asm volatile("" : "+v"(nxt.x), "+v"(nxt.y), "+v"(nxt.z), "+v"(nxt.w));
                    });
                    ply(p + 1, cur.y, nofill);
                    ply(p + 2, cur.z, nofill);
                    ply(p + 3, cur.w, nofill);
                    cur = nxt;
                    p += 4;
                }
            }
            while (p < plies) {
                const uint64_t g = ply0 + (uint64_t)p;
                ply(p, pick4(philox4(rng.seed, id, g >> 2, RNG_ACTION), (uint32_t)(g & 3)), nofill);
                ++p;
            }
        };
        if (!slow) {
            // no opening bookkeeping when no board of the wave can have opening plies
            if (rng.init_rand == 0 && !__any((mt & 0xff00u) != 0)) fast(std::false_type{});
            else fast(std::true_type{});
            tally_from_signs(t0, t1, t2, cb, cd, cw);
            const bool tw = (mt & M_TURN_WHITE) != 0;
            s.white.w[0] = tw ? M : O;
            s.black.w[0] = tw ? O : M;
            s.legal.w[0] = L;
            s.meta = mt;
        } else {
            for (int p = 0; p < plies; ++p) {
                const uint64_t g = ply0 + (uint64_t)p;
                int a = -1, r = 0, d = 1, win = NO_DISK;
                if (!(s.meta & M_TERMINATED)) {
                    if (POLICY == OTH_POLICY_RANDOM || (s.meta >> M_RAND_SHIFT) > 0)
                        a = random_action<N>(s, action_draw(rng.seed, id, g));
                    else
                        a = policy_action<N, POLICY>(s, eng);
                    if ((s.meta >> M_RAND_SHIFT) > 0) s.meta -= 1u << M_RAND_SHIFT;
                    step_lane<N, Fills<N>, true>(s, a, flags, r, d, win, eng);
                    if (d) {
                        cb += win == BLACK_DISK;
                        cd += win == NO_DISK;
                        cw += win == WHITE_DISK;
                        reset_lane<N>(s, rng.seed, id, g, RNG_OPENING_AUTO, rng.init_rand);
                        eng.prime(s);
                    }
                }
                actions[(size_t)p * E + e] = a;
                rewards[(size_t)p * E + e] = r;
                dones[(size_t)p * E + e] = (uint8_t)d;
            }
        }
        store_lane<N>(s, boards, meta, legal, e);
    }
    tally(wdl, cb, cd, cw);
}

// play_rand_fast for multi-word boards (N >= 9, the FillsW engine): the same
// (mover, opponent) form with BB<W> words; every multi-word select is word by
// word (a selected member address puts the lane in scratch).
template <int N, bool OPEN = true, typename FILL = NoFill>
__device__ __forceinline__ void play_rand_fast_w(BB<Geo<N>::W>& M, BB<Geo<N>::W>& O, BB<Geo<N>::W>& L,
                                                 uint32_t& meta, const FillsW<N>& eng, uint32_t u, uint32_t flags,
                                                 const Rng& rng, uint32_t id, uint64_t g, int& a, int& r, int& d,
                                                 uint32_t& cb, uint32_t& cd, uint32_t& cw, const uint8_t* sel8,
                                                 const FILL& fill = FILL{}) {
    constexpr int W = Geo<N>::W;
    constexpr int NN = N * N;
    a = select_bit_tab(L, scale_index(u, popcount(L)), sel8);  // RandomPolicy (simple_policies.py:37-41); L != 0
    if constexpr (OPEN) meta -= (meta & 0xff00u) ? (1u << M_RAND_SHIFT) : 0u;
    const BB<W> m = square<W>(a);
    const BB<W> f = eng.flip(M, O, a);  // update_board (othello.py:391-410)
    const BB<W> Mn = M | f | m, On = O & ~f;
    const bool full = !any(~(Mn | On) & Geo<N>::BOARD);  // :425-426
    // a full board resets before the scan, as in play_rand_fast: the next mover's
    // scan runs on the start position, and only a double pass scans it again
    // (10x10: 1.692 -> 1.689 us per ply, profiles/r04/g/ab_term.jsonl)
    BB<W> nM, nO;
#pragma unroll
    for (int i = 0; i < W; ++i) {
        nM.w[i] = full ? Start<N>::BLACK.w[i] : On.w[i];
        nO.w[i] = full ? Start<N>::WHITE.w[i] : Mn.w[i];
    }
    BB<W> Ln = eng.legal(nM, nO);  // the next mover's possible_moves (:436)
    fill();
    const bool pass = !any(Ln);  // never on the start position
    bool term = full;
    M = nM;
    O = nO;
    if (pass) {  // :437-440
        Ln = eng.legal(Mn, On);
        M = Mn;
        O = On;
        if (!any(Ln)) {  // nobody can move (:441-442): reset
            term = true;
            M = Start<N>::BLACK;
            O = Start<N>::WHITE;
            Ln = eng.legal(M, O);
        }
    }
    L = Ln;
    const uint32_t mover = meta;
    meta ^= pass ? 0u : M_TURN_WHITE;
    r = 0;
    d = term ? 1 : 0;
    if (term) {
        const int pc = popcount(Mn), oc = popcount(On), df = pc - oc;
        const int sg = sign_i32(df);  // the mover's result
        r = term_reward(flags, oc == 0 ? NN : df, sg);  // :446-459 / winner * player_turn
        const int mw = -(int)(mover & M_TURN_WHITE);  // (cb, cd, cw) as in play_rand_fast
        const int sb = (sg ^ mw) - mw;
        cb += (uint32_t)sb;
        cd += 1u;
        cw += (uint32_t)__mul24(sb, sb);
        uint32_t rl = 0;
        if constexpr (OPEN) {  // (without: no opening plies and none drawn, the scalar branch compiled out)
            if (rng.init_rand > 0)
                rl = (uint32_t)scale_index(opening_draw(rng.seed, id, g, RNG_OPENING_AUTO), rng.init_rand / 2 + 1) * 2u;
        }
        meta = (rl & 0xffu) << M_RAND_SHIFT;
    }
}

// k_play_rand for multi-word boards (config 5's 10x10 and every N >= 9).
template <int N>
__global__ __launch_bounds__(BLOCK) void k_play_rand_w(uint64_t* __restrict__ boards, uint16_t* __restrict__ meta,
                                                       uint64_t* __restrict__ legal, int E, uint32_t flags, int plies,
                                                       int32_t* __restrict__ actions, int32_t* __restrict__ rewards,
                                                       uint8_t* __restrict__ dones,
                                                       unsigned long long* __restrict__ wdl, Rng rng, uint64_t ply0) {
    constexpr int W = Geo<N>::W;
    static_assert(W > 1, "multi-word boards");
    ply0 += *rng.ply_off;  // graph-region offset (oth_graph_end); 0 eagerly
    __shared__ __attribute__((aligned(16))) uint64_t lds_rays[FillsW<N>::RAY_WORDS];
    __shared__ __attribute__((aligned(16))) uint64_t lds_sel[256];
    for (int i = threadIdx.x; i < 256; i += BLOCK) lds_sel[i] = sel8_word((uint32_t)i);
    const uint8_t* sel8 = reinterpret_cast<const uint8_t*>(lds_sel);
    FillsW<N>::fill(lds_rays);  // (its barrier covers lds_sel)
    const int e = blockIdx.x * BLOCK + threadIdx.x;
    uint32_t cb = 0, cd = 0, cw = 0;
    if (e < E) {
        const uint32_t id = rng.id_base + (uint32_t)e;
        const FillsW<N> eng(0, lds_rays);
        Lane<N> s;
        load_lane<N>(s, boards, meta, legal, e);
        const bool tw0 = (s.meta & M_TURN_WHITE) != 0;
        BB<W> M, O, L = s.legal;
#pragma unroll
        for (int i = 0; i < W; ++i) {
            M.w[i] = tw0 ? s.white.w[i] : s.black.w[i];
            O.w[i] = tw0 ? s.black.w[i] : s.white.w[i];
        }
        uint32_t mt = s.meta & (0xff00u | M_TURN_WHITE);
        eng.prime(s);
        const bool slow = __any((s.meta & M_TERMINATED) != 0 || !any(L));  // as k_play_rand
        int32_t* act_p = actions + e;
        int32_t* rew_p = rewards + e;
        uint8_t* done_p = dones + e;
        uint32_t t0 = 0, t1 = 0, t2 = 0;  // play_rand_fast_w's tally (tally_from_signs)
        // OPEN: some board of the wave may have or draw random-opening plies; without,
        // the opening bookkeeping and the reset's opening draw are compiled out
        auto fast = [&](auto OPENC) __attribute__((always_inline)) {
            constexpr bool OPEN = decltype(OPENC)::value;
            auto ply = [&](uint64_t g, uint32_t u, const auto& fill) __attribute__((always_inline)) {
                int a, r, d;
                play_rand_fast_w<N, OPEN>(M, O, L, mt, eng, u, flags, rng, id, g, a, r, d, t0, t1, t2, sel8, fill);
                *act_p = a;
                *rew_p = r;
                *done_p = (uint8_t)d;
                act_p += E;
                rew_p += E;
                done_p += E;
            };
            // Philox block g/4 serves plies 4k..4k+3 (g uniform: scalar branches).
            // Two-word boards compute the next block in the current group's first ply
            // (as k_play_rand: 10x10 +5 %); boards of 3+ words, already past 256 VGPRs,
            // at each group's start (the pipelined form: 12x12 -4 %)
            const NoFill nofill;
            int p = 0;
            if constexpr (W > 2) {
                while (p < plies) {
                    const uint64_t g = ply0 + (uint64_t)p;
                    const U4 d4 = philox4(rng.seed, id, g >> 2, RNG_ACTION);
                    if ((g & 3) == 0 && p + 4 <= plies) {
                        ply(g, d4.x, nofill);
                        ply(g + 1, d4.y, nofill);
                        ply(g + 2, d4.z, nofill);
                        ply(g + 3, d4.w, nofill);
                        p += 4;
                    } else {
                        ply(g, pick4(d4, (uint32_t)(g & 3)), nofill);
                        ++p;
                    }
                }
            } else {
                while (p < plies && ((ply0 + (uint64_t)p) & 3) != 0) {
                    const uint64_t g = ply0 + (uint64_t)p;
                    ply(g, pick4(philox4(rng.seed, id, g >> 2, RNG_ACTION), (uint32_t)(g & 3)), nofill);
                    ++p;
                }
                if (p + 4 <= plies) {
                    U4 cur = philox4(rng.seed, id, (ply0 + (uint64_t)p) >> 2, RNG_ACTION);
                    while (p + 4 <= plies) {
                        const uint64_t g = ply0 + (uint64_t)p;
                        U4 nxt;  // (one unused block after the last group)
                        ply(g, cur.x, [&]() __attribute__((always_inline)) {
                            nxt = philox4(rng.seed, id, (g >> 2) + 1, RNG_ACTION);
                            asm volatile("" : "+v"(nxt.x), "+v"(nxt.y), "+v"(nxt.z), "+v"(nxt.w));
                        });
                        ply(g + 1, cur.y, nofill);
                        ply(g + 2, cur.z, nofill);
                        ply(g + 3, cur.w, nofill);
                        cur = nxt;
                        p += 4;
                    }
                }
                while (p < plies) {
                    const uint64_t g = ply0 + (uint64_t)p;
                    ply(g, pick4(philox4(rng.seed, id, g >> 2, RNG_ACTION), (uint32_t)(g & 3)), nofill);
                    ++p;
                }
            }
        };
        if (!slow) {
            // (one loop for both: 10x10 without openings 1.422 -> 1.447 us per ply, profiles/r06/n)
            if (rng.init_rand == 0 && !__any((mt & 0xff00u) != 0)) fast(std::false_type{});
            else fast(std::true_type{});
            tally_from_signs(t0, t1, t2, cb, cd, cw);
            const bool tw = (mt & M_TURN_WHITE) != 0;
#pragma unroll
            for (int i = 0; i < W; ++i) {
                s.white.w[i] = tw ? M.w[i] : O.w[i];
                s.black.w[i] = tw ? O.w[i] : M.w[i];
            }
            s.legal = L;
            s.meta = mt;
        } else {
            for (int p = 0; p < plies; ++p) {
                const uint64_t g = ply0 + (uint64_t)p;
                int a = -1, r = 0, d = 1, win = NO_DISK;
                if (!(s.meta & M_TERMINATED)) {
                    a = random_action<N>(s, action_draw(rng.seed, id, g));
                    if ((s.meta >> M_RAND_SHIFT) > 0) s.meta -= 1u << M_RAND_SHIFT;
                    step_lane<N, FillsW<N>, true>(s, a, flags, r, d, win, eng);
                    if (d) {
                        cb += win == BLACK_DISK;
                        cd += win == NO_DISK;
                        cw += win == WHITE_DISK;
                        reset_lane<N>(s, rng.seed, id, g, RNG_OPENING_AUTO, rng.init_rand);
                        eng.prime(s);
                    }
                }
                act_p[(size_t)p * E] = a;
                rew_p[(size_t)p * E] = r;
                done_p[(size_t)p * E] = (uint8_t)d;
            }
        }
        store_lane<N>(s, boards, meta, legal, e);
    }
    tally(wdl, cb, cd, cw);
}


// ---------------------------------------------------------------------------
// OthelloEnv semantics on the device (othello.py:151-200): the protagonist
// steps with the caller's action, then the embedded opponent (random or greedy,
// on device) replies until it is the protagonist's turn again; the reward of
// a game the opponent's ply ends is negated (:200).  Random-opening plies
// (SimpleOthelloEnv / OthelloEnv rand_step_cnt, :179-182, :191-194) replace
// both sides' moves by random ones; the opponent's reply inside reset() uses
// the policy directly (:165-174).  Draws: ply j of call c uses
// action_draw(seed, id, c * 256 + j).
// ---------------------------------------------------------------------------
constexpr uint64_t VS_PLIES_PER_CALL = 256;

template <int N, int POLICY>
__device__ __forceinline__ void opponent_reply(Lane<N>& s, bool prot_white, bool openings, uint32_t flags,
                                               const Rng& rng, uint32_t id, uint64_t gbase, uint32_t& j, int& r,
                                               int& d, int& win) {
    const Solo<N> eng(0, nullptr);
    while (!(s.meta & M_TERMINATED) && (((s.meta & M_TURN_WHITE) != 0) != prot_white)) {
        const uint32_t rl = s.meta >> M_RAND_SHIFT;
        const uint64_t g = gbase + j++;  // ply j of the call
        int a;
        if (POLICY == OTH_POLICY_RANDOM || (openings && rl > 0)) {
            a = random_action<N>(s, action_draw(rng.seed, id, g));
        } else {
            a = policy_action<N, POLICY>(s, eng, rng.depth);
        }
        if (openings && rl > 0) s.meta -= 1u << M_RAND_SHIFT;
        step_lane<N>(s, a, flags, r, d, win, eng);
    }
}

template <int N, int POLICY>
__device__ __forceinline__ void reset_vs_lane(Lane<N>& s, bool prot_white, uint32_t flags, const Rng& rng,
                                              uint32_t id, uint64_t call, uint32_t purpose, uint32_t& j) {
    reset_lane<N>(s, rng.seed, id, call, purpose, rng.init_rand);
    int r, d, win;
    opponent_reply<N, POLICY>(s, prot_white, false, flags, rng, id, call * VS_PLIES_PER_CALL, j, r, d, win);
}

template <int N, int POLICY>
__global__ __launch_bounds__(BLOCK) void k_reset_vs(uint64_t* __restrict__ boards, uint16_t* __restrict__ meta,
                                                    uint64_t* __restrict__ legal, int E, uint32_t flags,
                                                    const int8_t* __restrict__ prot, const uint8_t* __restrict__ mask,
                                                    Rng rng, uint64_t call) {
    call += *rng.ply_off;  // graph-region offset (oth_graph_end); 0 eagerly
    const int e = blockIdx.x * BLOCK + threadIdx.x;
    if (e >= E) return;
    if (mask && !mask[e]) return;
    const bool pw = prot ? prot[e] == WHITE_DISK : true;
    Lane<N> s;
    uint32_t j = 0;
    reset_vs_lane<N, POLICY>(s, pw, flags, rng, rng.id_base + (uint32_t)e, call, RNG_OPENING_RESET, j);
    store_lane<N>(s, boards, meta, legal, e);
}

template <int N, int POLICY>
__global__ __launch_bounds__(BLOCK) void k_step_vs(uint64_t* __restrict__ boards, uint16_t* __restrict__ meta,
                                                   uint64_t* __restrict__ legal, int E, uint32_t flags,
                                                   const int32_t* __restrict__ actions, const int8_t* __restrict__ prot,
                                                   int32_t* __restrict__ rewards, uint8_t* __restrict__ dones,
                                                   int32_t* __restrict__ plies_out,
                                                   unsigned long long* __restrict__ wdl,
                                                   unsigned long long* __restrict__ wdl_vs, Rng rng, uint64_t call) {
    call += *rng.ply_off;  // graph-region offset (oth_graph_end); 0 eagerly
    const int e = blockIdx.x * BLOCK + threadIdx.x;
    uint32_t cb = 0, cd = 0, cw = 0, pw_n = 0, pd_n = 0, pl_n = 0;
    if (e < E) {
        const uint32_t id = rng.id_base + (uint32_t)e;
        const bool pw = prot ? prot[e] == WHITE_DISK : true;
        const uint64_t gbase = call * VS_PLIES_PER_CALL;
        Lane<N> s;
        load_lane<N>(s, boards, meta, legal, e);
        uint32_t j = 0;
        int r = 0, d = 1, win = NO_DISK, plies = 0;
        if (!(s.meta & M_TERMINATED)) {
            const Solo<N> eng(0, nullptr);
            d = 0;
            // the protagonist must be to move (OthelloEnv.step asserts it, othello.py:177);
            // if not, the opponent replies first, as OthelloEnv.reset does
            opponent_reply<N, POLICY>(s, pw, true, flags, rng, id, gbase, j, r, d, win);
            if (!(s.meta & M_TERMINATED)) {
                int a = actions[e];
                const uint32_t rl = s.meta >> M_RAND_SHIFT;
                const uint64_t g = gbase + j++;
                if (rl > 0) {  // opening ply: the protagonist's action is replaced too (:179-182)
                    a = random_action<N>(s, action_draw(rng.seed, id, g));
                    s.meta -= 1u << M_RAND_SHIFT;
                }
                step_lane<N>(s, a, flags, r, d, win, eng);
                if (!d) {
                    opponent_reply<N, POLICY>(s, pw, true, flags, rng, id, gbase, j, r, d, win);
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
                // the harnesses' count from the protagonist's final reward (run.py:100-130:
                // its sign is the protagonist's result in both reward modes)
                const int pcol = pw ? WHITE_DISK : BLACK_DISK;
                pw_n = win == pcol;
                pd_n = win == NO_DISK;
                pl_n = win == -pcol;
                if (flags & OTH_AUTO_RESET) reset_vs_lane<N, POLICY>(s, pw, flags, rng, id, call, RNG_OPENING_AUTO, j);
            }
        }
        store_lane<N>(s, boards, meta, legal, e);
        if (rewards) rewards[e] = r;
        if (dones) dones[e] = (uint8_t)d;
        if (plies_out) plies_out[e] = plies;
    }
    tally(wdl, cb, cd, cw);
    tally(wdl_vs, pw_n, pd_n, pl_n);
}

template <int N>
__global__ __launch_bounds__(BLOCK) void k_legal_moves(const uint64_t* __restrict__ mover,
                                                       const uint64_t* __restrict__ opp, uint64_t* __restrict__ out,
                                                       int n) {
    constexpr int W = Geo<N>::W;
    const int e = blockIdx.x * BLOCK + threadIdx.x;
    if (e >= n) return;
    BB<W> P, O;
#pragma unroll
    for (int i = 0; i < W; ++i) {
        P.w[i] = mover[(size_t)e * W + i] & Geo<N>::BOARD.w[i];
        O.w[i] = opp[(size_t)e * W + i] & Geo<N>::BOARD.w[i] & ~P.w[i];
    }
    const BB<W> L = legal_moves<N>(P, O);
#pragma unroll
    for (int i = 0; i < W; ++i) out[(size_t)e * W + i] = L.w[i];
}

template <int N, int POLICY>
__global__ __launch_bounds__(BLOCK) void k_policy_actions(const uint64_t* __restrict__ boards,
                                                          const uint16_t* __restrict__ meta,
                                                          const uint64_t* __restrict__ legal, int E,
                                                          int32_t* __restrict__ out, int depth) {
    const int e = blockIdx.x * BLOCK + threadIdx.x;
    if (e >= E) return;
    Lane<N> s;
    load_lane<N>(s, boards, meta, legal, e);
    out[e] = policy_action<N, POLICY>(s, Solo<N>(0, nullptr), depth);
}

template <int N>
__global__ __launch_bounds__(BLOCK) void k_set_turn(const uint64_t* __restrict__ boards, uint16_t* __restrict__ meta,
                                                    uint64_t* __restrict__ legal, int E, int turn,
                                                    const uint8_t* __restrict__ mask) {
    constexpr int W = Geo<N>::W;
    const int e = blockIdx.x * BLOCK + threadIdx.x;
    if (e >= E) return;
    if (mask && !mask[e]) return;
    BB<W> b, w;
#pragma unroll
    for (int i = 0; i < W; ++i) {
        b.w[i] = boards[(size_t)e * 2 * W + i];
        w.w[i] = boards[(size_t)e * 2 * W + W + i];
    }
    const BB<W> L = turn == WHITE_DISK ? legal_moves<N>(w, b) : legal_moves<N>(b, w);
#pragma unroll
    for (int i = 0; i < W; ++i) legal[(size_t)e * W + i] = L.w[i];
    meta[e] = (uint16_t)((meta[e] & ~M_TURN_WHITE) | (turn == WHITE_DISK ? M_TURN_WHITE : 0u));
}

template <int N>
__global__ __launch_bounds__(BLOCK) void k_count(const uint64_t* __restrict__ boards, int E,
                                                 int32_t* __restrict__ out) {
    constexpr int W = Geo<N>::W;
    const int e = blockIdx.x * BLOCK + threadIdx.x;
    if (e >= E) return;
    int b = 0, w = 0;
#pragma unroll
    for (int i = 0; i < W; ++i) {
        b += popc64(boards[(size_t)e * 2 * W + i]);
        w += popc64(boards[(size_t)e * 2 * W + W + i]);
    }
    out[2 * (size_t)e] = w;
    out[2 * (size_t)e + 1] = b;
}

// A bfloat16 observation element (OTH_BF16).  The observations hold -1, 0 and
// +1 only, each exact in bfloat16: 0xBF80, 0x0000, 0x3F80.
struct obs_bf16 {
    uint16_t bits;
    obs_bf16() = default;
    __host__ __device__ explicit obs_bf16(int v) : bits(v == 0 ? 0u : (v > 0 ? 0x3F80u : 0xBF80u)) {}
};
static_assert(sizeof(obs_bf16) == 2, "a bfloat16");

template <typename T>
__device__ __forceinline__ void put(void* out, size_t i, int v) {
    reinterpret_cast<T*>(out)[i] = (T)v;
}

// One thread per output element, (E, planes, N, N) row-major: coalesced stores.
template <int N>
__global__ __launch_bounds__(BLOCK) void k_observe(const uint64_t* __restrict__ boards,
                                                   const uint16_t* __restrict__ meta,
                                                   const uint64_t* __restrict__ legal, int E, int layout, int dtype,
                                                   void* __restrict__ out) {
    constexpr int W = Geo<N>::W;
    constexpr int NN = N * N;
    const int planes = layout == OTH_OBS_BOARD_LEGAL ? 2 : (layout == OTH_OBS_MAKE_STATE ? 4 : 1);
    const size_t total = (size_t)E * planes * NN;
    for (size_t i = (size_t)blockIdx.x * BLOCK + threadIdx.x; i < total; i += (size_t)gridDim.x * BLOCK) {
        const int a = (int)(i % NN);
        const size_t rest = i / NN;
        const int plane = (int)(rest % planes);
        const size_t e = rest / planes;
        const int wi = a / 64, bi = a % 64;
        const int isb = (int)((boards[e * 2 * W + wi] >> bi) & 1u);
        const int isw = (int)((boards[e * 2 * W + W + wi] >> bi) & 1u);
        const uint32_t m = meta[e];
        const bool tw = (m & M_TURN_WHITE) != 0;
        int v;
        if (layout == OTH_OBS_ABSOLUTE) {
            v = isw - isb;
        } else if (layout == OTH_OBS_LEGAL) {
            v = (int)((legal[e * W + wi] >> bi) & 1u);
        } else if (layout == OTH_OBS_MAKE_STATE) {
            if (plane == 0) {
                v = isb;
            } else if (plane == 1) {
                v = isw;
            } else if (plane == 2) {
                v = tw ? 1 : 0;
            } else {  // util.py:55: the legal plane only when >= 2 moves
                int cnt = 0;
#pragma unroll
                for (int k = 0; k < W; ++k) cnt += popc64(legal[e * W + k]);
                v = cnt > 1 ? (int)((legal[e * W + wi] >> bi) & 1u) : 0;
            }
        } else {
            if (plane == 0) {
                v = tw ? (isw - isb) : (isb - isw);  // othello.py:364-369
            } else {
                v = (int)((legal[e * W + wi] >> bi) & 1u);
            }
        }
        switch (dtype) {
            case OTH_I8: put<int8_t>(out, i, v); break;
            case OTH_I32: put<int32_t>(out, i, v); break;
            case OTH_I64: put<int64_t>(out, i, v); break;
            case OTH_F32: put<float>(out, i, v); break;
            case OTH_BF16: put<obs_bf16>(out, i, v); break;
            default: put<double>(out, i, v); break;
        }
    }
}

// A quad of 4 consecutive squares of one plane as one vector store (16 B for
// f32 / i32, 8 B for bf16, 4 B for i8, 2 x 16 B for the 8-byte types): k_observe_w's unit
// (the 8-byte types take pairs of squares instead, OTH_OBS_PAIR8).
// (as streaming stores: 65,536 boards 2-3 % slower, 1,048,576 int64 boards 104 -> 250 us;
// profiles/r04/d/ab_obs_nt.jsonl)
template <typename T>
__device__ __forceinline__ void put_quad(T* out, uint32_t q, int v0, int v1, int v2, int v3) {
    if constexpr (sizeof(T) == 1) {
        const uint32_t x = (uint32_t)(uint8_t)(int8_t)v0 | ((uint32_t)(uint8_t)(int8_t)v1 << 8) |
                           ((uint32_t)(uint8_t)(int8_t)v2 << 16) | ((uint32_t)(uint8_t)(int8_t)v3 << 24);
        reinterpret_cast<uint32_t*>(out)[q] = x;
    } else if constexpr (sizeof(T) == 2) {
        uint2 x;
        x.x = (uint32_t)T(v0).bits | ((uint32_t)T(v1).bits << 16);
        x.y = (uint32_t)T(v2).bits | ((uint32_t)T(v3).bits << 16);
        reinterpret_cast<uint2*>(out)[q] = x;
    } else if constexpr (sizeof(T) == 4) {
        using V4 = typename std::conditional<std::is_same<T, float>::value, float4, int4>::type;
        V4 x;
        x.x = (T)v0;
        x.y = (T)v1;
        x.z = (T)v2;
        x.w = (T)v3;
        reinterpret_cast<V4*>(out)[q] = x;
    } else {
        using V2 = typename std::conditional<std::is_same<T, double>::value, double2, longlong2>::type;
        V2 a, b;
        a.x = (T)v0;
        a.y = (T)v1;
        b.x = (T)v2;
        b.y = (T)v3;
        reinterpret_cast<V2*>(out)[2 * (size_t)q] = a;
        reinterpret_cast<V2*>(out)[2 * (size_t)q + 1] = b;
    }
}

// S one- or two-byte observation elements of one unit (+1 where pos, -1 where
// neg, 0 elsewhere: bit j of the masks is square j of the unit) as ONE store of
// S * sizeof(T) bytes.  Each dword spreads 4 bits into bytes (bit i of x < 16
// lands in byte i of x * 0x204081 & 0x01010101) or 2 bits into halves (x * 0x8001
// & 0x10001), then scales: 0xFF (int8 -1), 0x3F80 / 0xBF80 (bf16 +1 / -1).
template <typename T, int S>
__device__ __forceinline__ void put_narrow(T* out, uint32_t g, uint32_t pos, uint32_t neg) {
    static_assert(sizeof(T) <= 2 && (S * sizeof(T)) % 4 == 0 && S * sizeof(T) <= 16, "one store of 4 to 16 bytes");
    constexpr int D = (int)(S * sizeof(T) / 4);
    uint32_t d[D];
#pragma unroll
    for (int k = 0; k < D; ++k) {
        if constexpr (sizeof(T) == 1) {
            const uint32_t p = (pos >> (4 * k)) & 0xFu, n = (neg >> (4 * k)) & 0xFu;
            d[k] = ((p * 0x204081u) & 0x01010101u) | (((n * 0x204081u) & 0x01010101u) * 0xFFu);
        } else {
            const uint32_t p = (pos >> (2 * k)) & 3u, n = (neg >> (2 * k)) & 3u;
            d[k] = ((p * 0x8001u) & 0x10001u) * 0x3F80u | ((n * 0x8001u) & 0x10001u) * 0xBF80u;
        }
    }
    if constexpr (D == 4) {
        reinterpret_cast<uint4*>(out)[g] = make_uint4(d[0], d[1], d[2], d[3]);
    } else if constexpr (D == 2) {
        reinterpret_cast<uint2*>(out)[g] = make_uint2(d[0], d[1]);
    } else {
        reinterpret_cast<uint32_t*>(out)[g] = d[0];
    }
}

#ifndef OTH_OBS_PAIR8
// 8-byte observations by pairs of squares, one 16-B store per lane (1 KiB
// contiguous per store instruction) instead of quads in two 16-B stores (each
// instruction half of a 2-KiB span): oth_step_observe with its int64 board at
// 65,536 8x8 boards 11.05 -> 8.80 us per graphed ply (torch's fill_ of the same
// tensor: 8.95; profiles/r05/i/ab_step_obs.json)
#define OTH_OBS_PAIR8 1
#endif
// obs_stream's squares per lane and store for NN squares of esize-byte elements
// (below), and the byte alignment the output needs for them
__host__ __device__ constexpr int obs_unit(int NN, int esize) {
    return esize == 8 ? (OTH_OBS_PAIR8 ? 2 : 4) : (NN % (16 / esize) == 0 ? 16 / esize : 4);
}
__host__ __device__ constexpr int obs_align(int NN, int esize) {
    return obs_unit(NN, esize) * esize > 4 * esize ? obs_unit(NN, esize) * esize : 4 * esize;
}
template <int LAYOUT>
constexpr int obs_planes() {
    return LAYOUT == OTH_OBS_BOARD_LEGAL ? 2 : (LAYOUT == OTH_OBS_MAKE_STATE ? 4 : 1);
}
template <int LAYOUT>
constexpr bool obs_needs_legal() {
    return LAYOUT == OTH_OBS_BOARD_LEGAL || LAYOUT == OTH_OBS_MAKE_STATE || LAYOUT == OTH_OBS_LEGAL;
}
// the board facts the observation needs beside its words: bit 0 white to move,
// bit 1 more than one legal move (util.py:55's make_state condition)
template <int W>
__device__ __forceinline__ uint32_t obs_flags(uint32_t m, const uint64_t (&lw)[W]) {
    int cnt = 0;
#pragma unroll
    for (int k = 0; k < W; ++k) cnt += popc64(lw[k]);
    return ((m & M_TURN_WHITE) ? 1u : 0u) | (cnt > 1 ? 2u : 0u);
}

// The observation (E, planes, N, N) of nb <= BPW consecutive boards whose words
// the wave holds -- board kb's black / white / possible_moves words and its
// obs_flags in lane kb * LS (LS lanes per board) -- streamed into their
// contiguous output region `base` (nb x planes x N*N/4 quads), one 64-quad
// vector store per step, each lane taking the words of the board its quad
// belongs to from that board's lane (ds_bpermute).  Every lane of the wave
// must take part (ds_bpermute reads an inactive source lane as 0).  Used by
// k_observe_w (the boards loaded from HBM) and by the step kernels' fused
// observation (oth_step_observe / oth_sample_step_observe: the boards as the
// step left them in registers).
template <int N, int LAYOUT, typename T, int BPW, int LS = 1>
__device__ __forceinline__ void obs_stream(const uint64_t (&bw)[Geo<N>::W], const uint64_t (&ww)[Geo<N>::W],
                                           const uint64_t (&lw)[Geo<N>::W], uint32_t fl, int nb,
                                           T* __restrict__ base) {
    static_assert(BPW * LS <= 64, "the wave holds its boards");
    constexpr int W = Geo<N>::W;
    constexpr int NN = N * N;
    static_assert(NN % 4 == 0, "quads of squares");
    constexpr int Q = NN / 4;
    constexpr int PQ = obs_planes<LAYOUT>() * Q;  // quads per board
    constexpr bool NEED_L = obs_needs_legal<LAYOUT>();
    const int lane = threadIdx.x & 63;
    const int total = nb * PQ;
    auto fetch = [&](const uint64_t (&x)[W], int kb, int wi) __attribute__((always_inline)) {
        uint64_t r = 0;
#pragma unroll
        for (int k = 0; k < W; ++k) {
            const uint64_t y = (uint64_t)__shfl((unsigned long long)x[k], kb * LS);
            r = wi == k ? y : r;
        }
        return r;
    };
    // every lane takes part in every step (ds_bpermute reads an inactive source lane
    // as 0): the last step's lanes past the region clamp their quad and skip the store.
    // Measured and not kept (1,048,576 boards, make_state f32; a plain torch fill of the
    // same tensor: 155 us, ours 219): the waves starting their regions at different
    // steps 217.8 -> 225.8 us; boards dealt to the waves with the grid's stride (the
    // resident waves store into one window) 219.6 -> 264.3; the step's board words by
    // v_readlane 218.9 -> 217.5 (and +-0 again on the branch-free body below); the loop
    // unrolled by 4 +-0 (by 2 / 4 on the branch-free body: +-0, profiles/r04/obs/ab_unroll_bf.jsonl); 128 / 256 boards per wave (every wave resident at once, all
    // loads first) 218.8 -> 216.6 / 234.4, and at 262,144 boards 46.5 -> 57.6 / 110.3
    // (profiles/r04/obs/)
    // S squares per lane and store: 16 bytes a lane where a plane divides into such
    // units -- 16 squares of int8, 8 of bf16, quads of the 4-byte types, and for the
    // 8-byte types under OTH_OBS_PAIR8 pairs (one 16-B store per lane, so each store
    // instruction writes 1 KiB contiguous instead of two half-filled 2-KiB spans) --
    // else quads.  One- and two-byte units are packed from their bit masks
    // (put_narrow): at 65,536 8x8 boards the learners' fused ply with its make_state
    // 15.43 -> 10.03 us per graphed ply in int8 (quads: a 4-B store per lane; the
    // sample-step alone 6.2), 17.25 -> 13.34 in bf16; k_observe_w make_state int8
    // 9.54 -> 5.36 us, 1,048,576 boards 86.6 -> 50.0 (profiles/r06/e)
    constexpr int S = obs_unit(NN, (int)sizeof(T));
    constexpr bool NARROW = sizeof(T) <= 2;
    constexpr uint32_t UQ = (uint32_t)(NN / S), UB = (uint32_t)obs_planes<LAYOUT>() * UQ;  // units per plane / board
    constexpr uint32_t SM = (1u << S) - 1u;
    const int totalu = nb * (int)UB;
    (void)total;
    for (int g0 = 0; g0 < totalu; g0 += 64) {
        const uint32_t g = (uint32_t)(g0 + lane < totalu ? g0 + lane : totalu - 1);
        const uint32_t kb = g / UB, rr = g - kb * UB;
        const uint32_t plane = rr / UQ, q = rr - plane * UQ;
        const uint32_t a0 = S * q, wi = a0 / 64, bi = a0 % 64;  // S | 64: a unit never straddles words
        // (a probe storing values made from g alone, nothing fetched: k_observe_w at 65,536 /
        // 1,048,576 boards, make_state f32 13.1 -> 12.5 / 208.7 -> 187.3 us, int64 board
        // 7.9 -> 7.8 / 100.5 -> 89.8; profiles/r05/l/ab_obs_cst.jsonl)
        const uint64_t xb = fetch(bw, (int)kb, (int)wi), xw = fetch(ww, (int)kb, (int)wi);
        const uint32_t flk = (uint32_t)__shfl((int)fl, (int)kb * LS);
        const bool tw = (flk & 1u) != 0;
        uint64_t xl = 0;
        if constexpr (NEED_L) xl = fetch(lw, (int)kb, (int)wi);
        // the lanes of one store cover several planes: each lane's plane word is
        // picked by masks, not branches (the compiler had made the plane choice
        // branches, so the wave ran every plane's path in turn with exec-mask SALU
        // between them): make_state f32 at 65,536 / 262,144 / 1,048,576 boards
        // 13.75 -> 12.79 / 46.6 -> 41.5 / 219.8 -> 208.3 us, int64 board 1,048,576
        // 104.7 -> 102.4 (profiles/r04/obs/ab_branchfree.jsonl)
        if constexpr (NARROW) {  // +1 where pos, -1 where neg, packed a dword at a time
            uint32_t pos, neg = 0u;
            if constexpr (LAYOUT == OTH_OBS_LEGAL) {
                pos = (uint32_t)(xl >> bi) & SM;
            } else if constexpr (LAYOUT == OTH_OBS_ABSOLUTE) {
                pos = (uint32_t)(xw >> bi) & SM;
                neg = (uint32_t)(xb >> bi) & SM;
            } else if constexpr (LAYOUT == OTH_OBS_MAKE_STATE) {
                const uint64_t m0 = 0ull - (uint64_t)(plane == 0u), m1 = 0ull - (uint64_t)(plane == 1u);
                const uint64_t m2 = 0ull - (uint64_t)(plane == 2u && tw), m3 = 0ull - (uint64_t)(plane == 3u && (flk & 2u));
                pos = (uint32_t)(((xb & m0) | (xw & m1) | (xl & m3) | m2) >> bi) & SM;
            } else {
                const uint64_t xm = tw ? xw : xb, xo = tw ? xb : xw;
                const bool p1 = plane != 0u;
                pos = (uint32_t)((p1 ? xl : xm) >> bi) & SM;
                neg = p1 ? 0u : (uint32_t)(xo >> bi) & SM;
            }
            if (g0 + lane < totalu) put_narrow<T, S>(base, g, pos, neg);
            continue;
        }
        int v[4] = {0, 0, 0, 0};
        if constexpr (LAYOUT == OTH_OBS_LEGAL) {  // possible_moves
            const uint32_t nl = (uint32_t)(xl >> bi) & SM;
#pragma unroll
            for (int j = 0; j < S; ++j) v[j] = (int)((nl >> j) & 1u);
        } else if constexpr (LAYOUT == OTH_OBS_ABSOLUTE) {  // othello.py:257
            const uint32_t nbk = (uint32_t)(xb >> bi) & SM, nwk = (uint32_t)(xw >> bi) & SM;
#pragma unroll
            for (int j = 0; j < S; ++j) v[j] = (int)((nwk >> j) & 1u) - (int)((nbk >> j) & 1u);
        } else if constexpr (LAYOUT == OTH_OBS_MAKE_STATE) {  // util.py:48-74
            const uint64_t m0 = 0ull - (uint64_t)(plane == 0u), m1 = 0ull - (uint64_t)(plane == 1u);
            const uint64_t m2 = 0ull - (uint64_t)(plane == 2u && tw), m3 = 0ull - (uint64_t)(plane == 3u && (flk & 2u));
            const uint32_t bits = (uint32_t)(((xb & m0) | (xw & m1) | (xl & m3) | m2) >> bi) & SM;
#pragma unroll
            for (int j = 0; j < S; ++j) v[j] = (int)((bits >> j) & 1u);
        } else {  // othello.py:363-376: mover +1, opponent -1; plane 1 the legal squares
            const uint64_t xm = tw ? xw : xb, xo = tw ? xb : xw;
            const uint32_t mv = (uint32_t)(xm >> bi) & SM, op = (uint32_t)(xo >> bi) & SM;
            const uint32_t nl = (uint32_t)(xl >> bi) & SM;
            const bool p1 = plane != 0u;
#pragma unroll
            for (int j = 0; j < S; ++j) {
                const int b = (int)((mv >> j) & 1u) - (int)((op >> j) & 1u);
                v[j] = p1 ? (int)((nl >> j) & 1u) : b;
            }
        }
        if (g0 + lane < totalu) {
            if constexpr (S == 2) {
                using V2 = typename std::conditional<std::is_same<T, double>::value, double2, longlong2>::type;
                V2 x;
                x.x = (T)v[0];
                x.y = (T)v[1];
                reinterpret_cast<V2*>(base)[g] = x;
            } else {
                put_quad<T>(base, g, v[0], v[1], v[2], v[3]);
            }
        }
    }
}

// k_observe_w: the same values as k_observe, one wave per BPW consecutive
// boards.  Each lane loads one board (coalesced), then the wave streams the
// boards' output region (obs_stream).  One board per wave (round 2's
// k_observe_q, each wave waiting on its own board's loads before one 1-KiB
// store) reached 2.6 TB/s for make_state f32 at 1,048,576 boards; one wave's
// loads feeding 64 boards' stores, 5.0 (a plain fill: 6.9).  BPW boards per wave:
// 16 below 262,144 boards (four times the waves of 64, each streaming a quarter
// of the region, so the store streams start sooner and more of them are in
// flight); from there 64, and once the output exceeds 384 MiB as many as fill
// about 4 KiB of output (launch_observe_w: make_state f32 at 1,048,576 boards
// 5.3 -> 6.0 TB/s with 4 boards a wave).
template <int N, int LAYOUT, typename T, int BPW = 64>
__global__ __launch_bounds__(BLOCK) void k_observe_w(const uint64_t* __restrict__ boards,
                                                     const uint16_t* __restrict__ meta,
                                                     const uint64_t* __restrict__ legal, int E, T* __restrict__ out) {
    static_assert(BPW == 4 || BPW == 8 || BPW == 16 || BPW == 32 || BPW == 64, "boards per wave");
    constexpr int W = Geo<N>::W;
    constexpr int PQ = obs_planes<LAYOUT>() * N * N / 4;  // quads per board
    const int lane = threadIdx.x & 63;
    const long long e0 = ((long long)blockIdx.x * BLOCK + threadIdx.x - lane) / 64 * BPW;  // the wave's first board
    if (e0 >= E) return;                                                                 // wave-uniform
    const long long e = lane < BPW ? e0 + lane : E;  // lanes past BPW load nothing
    uint64_t bw[W], ww[W], lw[W];
    uint32_t fl = 0;
#pragma unroll
    for (int k = 0; k < W; ++k) bw[k] = ww[k] = lw[k] = 0;
    if (e < E) {
#pragma unroll
        for (int k = 0; k < W; ++k) {
            bw[k] = boards[(size_t)e * 2 * W + k];
            ww[k] = boards[(size_t)e * 2 * W + W + k];
            if constexpr (obs_needs_legal<LAYOUT>()) lw[k] = legal[(size_t)e * W + k];
        }
        fl = obs_flags<W>(meta[e], lw);
    }
    const int nb = (int)(E - e0 < BPW ? E - e0 : BPW);
    obs_stream<N, LAYOUT, T, BPW, 1>(bw, ww, lw, fl, nb, out + (size_t)e0 * PQ * 4);
}

// The fused observation of the step kernels (oth_step_observe,
// oth_sample_step_observe): obs_stream for a runtime layout and dtype (kernel
// arguments, so the switch is a scalar branch taken once per wave), into the
// region of the wave's first board e0.  layout < 0: no observation.  Only
// N*N % 4 == 0 (the quad stores); the C ABI takes two launches for other N.
template <int N, int BPW, int LS>
__device__ __forceinline__ void obs_tail(int layout, int dtype, void* __restrict__ out, long long e0,
                                         const uint64_t (&bw)[Geo<N>::W], const uint64_t (&ww)[Geo<N>::W],
                                         const uint64_t (&lw)[Geo<N>::W], uint32_t m, int nb) {
    if constexpr ((N * N) % 4 == 0) {
        if (layout < 0 || nb <= 0) return;
        const uint32_t fl = obs_flags<Geo<N>::W>(m, lw);
        auto by_type = [&](auto LC) __attribute__((always_inline)) {
            constexpr int LAY = decltype(LC)::value;
            constexpr size_t PER = (size_t)obs_planes<LAY>() * N * N;  // elements per board
            switch (dtype) {
                case OTH_I8:
                    obs_stream<N, LAY, int8_t, BPW, LS>(bw, ww, lw, fl, nb, (int8_t*)out + e0 * PER);
                    break;
                case OTH_I32:
                    obs_stream<N, LAY, int32_t, BPW, LS>(bw, ww, lw, fl, nb, (int32_t*)out + e0 * PER);
                    break;
                case OTH_I64:
                    obs_stream<N, LAY, long long, BPW, LS>(bw, ww, lw, fl, nb, (long long*)out + e0 * PER);
                    break;
                case OTH_F32:
                    obs_stream<N, LAY, float, BPW, LS>(bw, ww, lw, fl, nb, (float*)out + e0 * PER);
                    break;
                case OTH_BF16:
                    obs_stream<N, LAY, obs_bf16, BPW, LS>(bw, ww, lw, fl, nb, (obs_bf16*)out + e0 * PER);
                    break;
                default:
                    obs_stream<N, LAY, double, BPW, LS>(bw, ww, lw, fl, nb, (double*)out + e0 * PER);
                    break;
            }
        };
        switch (layout) {
            case OTH_OBS_BOARD: by_type(std::integral_constant<int, OTH_OBS_BOARD>{}); break;
            case OTH_OBS_BOARD_LEGAL: by_type(std::integral_constant<int, OTH_OBS_BOARD_LEGAL>{}); break;
            case OTH_OBS_MAKE_STATE: by_type(std::integral_constant<int, OTH_OBS_MAKE_STATE>{}); break;
            case OTH_OBS_ABSOLUTE: by_type(std::integral_constant<int, OTH_OBS_ABSOLUTE>{}); break;
            default: by_type(std::integral_constant<int, OTH_OBS_LEGAL>{}); break;
        }
    }
}

// oth_step_sync: one board -- the single-board drop-in classes (BASELINE config
// 1) -- stepped with a host action passed by value, then its whole record
// (oth_record: state, reward / done, count_disks, GreedyPolicy's move,
// get_observation and board_state) written into mapped host memory by the same
// launch, the sequence number last behind a system-scope fence, so the host
// can read the record as soon as that number lands.  One wave: every lane
// holds the board (the step is tiny), lane 0 stores the state back, the lanes
// write the squares of the observation planes.
template <int N>
__global__ __launch_bounds__(64) void k_record(uint64_t* __restrict__ boards, uint16_t* __restrict__ meta,
                                               uint64_t* __restrict__ legal, int board, int step, int action,
                                               uint32_t flags, int planes, unsigned long long* __restrict__ wdl,
                                               Rng rng, uint64_t ply, oth_record* __restrict__ rec, uint32_t seq) {
    constexpr int W = Geo<N>::W, NN = N * N;
    static_assert(W <= OTH_RECORD_MAX_WORDS && NN <= OTH_RECORD_MAX_SQUARES, "record capacity");
    ply += *rng.ply_off;
    const int lane = threadIdx.x;
    WaveSlot slot(wdl, board >> 6);
    Lane<N> s;
    load_lane<N>(s, boards, meta, legal, board);
    int r = 0, d = 0, win = NO_DISK;
    bool ended = false;
    if (step & 1) {
        const bool was_term = (s.meta & M_TERMINATED) != 0;
        step_lane<N>(s, action, flags, r, d, win, Solo<N>(0, nullptr));
        ended = d && !was_term;
        if (ended && (flags & OTH_AUTO_RESET))
            reset_lane<N>(s, rng.seed, rng.id_base + (uint32_t)board, ply, RNG_OPENING_AUTO, rng.init_rand);
        if (lane == 0 && !was_term) store_lane<N>(s, boards, meta, legal, board);
    }
    slot.count(lane == 0 && ended && win == BLACK_DISK, lane == 0 && ended && win == NO_DISK,
               lane == 0 && ended && win == WHITE_DISK);
    slot.flush();
    const bool tw = (s.meta & M_TURN_WHITE) != 0;
    const int sign = tw ? 1 : -1;  // othello.py:364-369: mover +1
    for (int a = lane; a < NN; a += 64) {
        const int isb = (int)((s.black.w[a / 64] >> (a % 64)) & 1u), isw = (int)((s.white.w[a / 64] >> (a % 64)) & 1u);
        rec->board_state[a] = (int8_t)(isw - isb);
        rec->obs[a] = (int8_t)((isw - isb) * sign);
        if (planes == 2) rec->obs[NN + a] = (int8_t)((s.legal.w[a / 64] >> (a % 64)) & 1u);
    }
    if (lane == 0) {
#pragma unroll
        for (int i = 0; i < W; ++i) {
            rec->black[i] = s.black.w[i];
            rec->white[i] = s.white.w[i];
            rec->legal[i] = s.legal.w[i];
        }
        rec->meta = (uint16_t)s.meta;
        rec->done = (uint8_t)d;
        rec->planes = (uint8_t)planes;
        rec->reward = r;
        rec->white_cnt = popcount(s.white);
        rec->black_cnt = popcount(s.black);
        // (one lane's bit-plane flip counts: the bare call 8.96 -> 8.43 us without them, so only on request)
        rec->greedy = !(step & OTH_RECORD_GREEDY) ? OTH_RECORD_NO_GREEDY
                                                  : (popcount(s.legal) ? greedy_action<N>(s, Solo<N>(0, nullptr)) : -1);
    }
    __threadfence_system();  // every lane's record bytes before the sequence number
    __syncthreads();
    if (lane == 0) {
        __threadfence_system();
        *reinterpret_cast<volatile uint32_t*>(&rec->seq) = seq;
    }
}

}  // namespace oth_dev
