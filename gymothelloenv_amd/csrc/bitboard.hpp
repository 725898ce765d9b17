// bitboard.hpp -- W-word bitboards for an N x N Othello board (4 <= N <= 16).
//
// Square a = row * N + col (othello.py:392-393) lives in word a / 64, bit a % 64.
// W = ceil(N*N / 64): 1 word for N <= 8, 2 for N <= 11, 3 for N <= 13, 4 for N <= 16.
// Everything here is constexpr / __forceinline__ and fully unrolled on the
// compile-time N, so a board is 2W VGPR pairs and every mask is an immediate.
//
// The 8-direction ray scan of the reference (get_num_killed_enemy,
// othello.py:273-311, driven per empty cell by get_possible_actions,
// othello.py:313-343) becomes, per direction, a Kogge-Stone occluded fill:
// a shift of the mover's discs through contiguous opponent discs in
// log2(N) doubling steps, then one more shift onto an empty square.
#pragma once
#include <stdint.h>
#include <type_traits>

#ifndef OTH_OPENING_PHILOX
#define OTH_OPENING_PHILOX 0  // opening-length draws by Philox (round-5 spec; A/B timing arm, round 6)
#endif

#if defined(__HIPCC__)
#define OTH_HD __host__ __device__ __forceinline__
#else
#define OTH_HD inline
#endif

namespace oth {

template <int W>
struct BB {
    uint64_t w[W];
};

template <int W>
OTH_HD BB<W> operator|(const BB<W>& a, const BB<W>& b) {
    BB<W> r;
#pragma unroll
    for (int i = 0; i < W; ++i) r.w[i] = a.w[i] | b.w[i];
    return r;
}
template <int W>
OTH_HD BB<W> operator&(const BB<W>& a, const BB<W>& b) {
    BB<W> r;
#pragma unroll
    for (int i = 0; i < W; ++i) r.w[i] = a.w[i] & b.w[i];
    return r;
}
template <int W>
OTH_HD BB<W> operator^(const BB<W>& a, const BB<W>& b) {
    BB<W> r;
#pragma unroll
    for (int i = 0; i < W; ++i) r.w[i] = a.w[i] ^ b.w[i];
    return r;
}
template <int W>
OTH_HD BB<W> operator~(const BB<W>& a) {
    BB<W> r;
#pragma unroll
    for (int i = 0; i < W; ++i) r.w[i] = ~a.w[i];
    return r;
}
template <int W>
OTH_HD BB<W>& operator|=(BB<W>& a, const BB<W>& b) {
    a = a | b;
    return a;
}
template <int W>
OTH_HD BB<W>& operator&=(BB<W>& a, const BB<W>& b) {
    a = a & b;
    return a;
}
// c ? a : b word by word (a select of two structs' addresses can force them into scratch)
template <int W>
OTH_HD BB<W> pick(bool c, const BB<W>& a, const BB<W>& b) {
    BB<W> r;
#pragma unroll
    for (int i = 0; i < W; ++i) r.w[i] = c ? a.w[i] : b.w[i];
    return r;
}

template <int W>
OTH_HD bool any(const BB<W>& a) {
    uint64_t x = 0;
#pragma unroll
    for (int i = 0; i < W; ++i) x |= a.w[i];
    return x != 0;
}
template <int W>
OTH_HD BB<W> zero() {
    BB<W> r;
#pragma unroll
    for (int i = 0; i < W; ++i) r.w[i] = 0;
    return r;
}
// all-ones if c else all-zeros, branch-free
template <int W>
OTH_HD BB<W> select_if(bool c, const BB<W>& a) {
    const uint64_t m = 0ull - (uint64_t)c;
    BB<W> r;
#pragma unroll
    for (int i = 0; i < W; ++i) r.w[i] = a.w[i] & m;
    return r;
}
template <int W>
OTH_HD BB<W> square(int a) {  // single-bit board; a outside [0, 64W) -> empty
    BB<W> r;
#pragma unroll
    for (int i = 0; i < W; ++i) r.w[i] = (a >= 64 * i && a < 64 * i + 64) ? (1ull << (a - 64 * i)) : 0ull;
    return r;
}
template <int W>
OTH_HD bool test(const BB<W>& b, int a) {
    bool r = false;
#pragma unroll
    for (int i = 0; i < W; ++i)
        if (a >= 64 * i && a < 64 * i + 64) r = (b.w[i] >> (a - 64 * i)) & 1u;
    return r;
}

OTH_HD int popc64(uint64_t x) {
#if defined(__HIP_DEVICE_COMPILE__)
    // two 32-bit counts (one v_bcnt_u32_b32 chain) as an i32: compares of counts
    // stay 32-bit (__popcll's i64 count put 64-bit compares into the select)
    return __popc((uint32_t)x) + __popc((uint32_t)(x >> 32));
#else
    return __builtin_popcountll(x);
#endif
}
// -1, 0 or +1: one v_med3_i32 on the device (LLVM turns min(max(x, -1), 1) of a
// difference into two compares and two selects)
OTH_HD int sign_i32(int x) {
#if defined(__HIP_DEVICE_COMPILE__)
    int r;
    asm("v_med3_i32 %0, %1, -1, 1" : "=v"(r) : "v"(x));
    return r;
#else
    return x > 0 ? 1 : (x < 0 ? -1 : 0);
#endif
}
OTH_HD int ctz64(uint64_t x) {  // x != 0
    return __builtin_ctzll(x);
}
OTH_HD int clz64(uint64_t x) {  // x != 0
#if defined(__HIP_DEVICE_COMPILE__)
    return __clzll(x);
#else
    return __builtin_clzll(x);
#endif
}
// Bit reversal of a 64-bit word (bit a -> bit 63 - a): two v_bfrev_b32 on the device.
OTH_HD uint64_t rev64(uint64_t x) {
#if defined(__HIP_DEVICE_COMPILE__) || defined(__clang__)
    return __builtin_bitreverse64(x);
#else
    x = __builtin_bswap64(x);
    x = ((x >> 4) & 0x0F0F0F0F0F0F0F0Full) | ((x & 0x0F0F0F0F0F0F0F0Full) << 4);
    x = ((x >> 2) & 0x3333333333333333ull) | ((x & 0x3333333333333333ull) << 2);
    return ((x >> 1) & 0x5555555555555555ull) | ((x & 0x5555555555555555ull) << 1);
#endif
}
template <int W>
OTH_HD int popcount(const BB<W>& a) {
    int c = 0;
#pragma unroll
    for (int i = 0; i < W; ++i) c += popc64(a.w[i]);
    return c;
}


// Logical shift of the whole W-word board by S bits (S > 0 toward higher squares).
template <int W, int S>
OTH_HD BB<W> shift(const BB<W>& x) {
    if constexpr (S == 0) {
        return x;
    } else if constexpr (S > 0) {
        constexpr int q = S / 64, s = S % 64;
        BB<W> r;
#pragma unroll
        for (int i = 0; i < W; ++i) {
            uint64_t v = 0;
            if (i - q >= 0) v = s ? (x.w[i - q] << s) : x.w[i - q];
            if (s && i - q - 1 >= 0) v |= x.w[i - q - 1] >> (64 - s);
            r.w[i] = v;
        }
        return r;
    } else {
        constexpr int T = -S, q = T / 64, s = T % 64;
        BB<W> r;
#pragma unroll
        for (int i = 0; i < W; ++i) {
            uint64_t v = 0;
            if (i + q < W) v = s ? (x.w[i + q] >> s) : x.w[i + q];
            if (s && i + q + 1 < W) v |= x.w[i + q + 1] << (64 - s);
            r.w[i] = v;
        }
        return r;
    }
}

// A one-word board as two dwords.  hipcc splits 64-bit logic into 32-bit halves
// only after instruction selection, so `(a & b) | c` on uint64_t becomes four
// VALU ops; on explicit dwords it becomes v_and_or_b32 / gfx950's 3-input
// v_bitop3_b32 per half.  Constant shifts stay one v_lshl*_b64 (sh below).
struct U2 {
    uint32_t lo, hi;
};
OTH_HD U2 u2(uint64_t v) { return U2{(uint32_t)v, (uint32_t)(v >> 32)}; }
OTH_HD uint64_t u64(U2 v) { return ((uint64_t)v.hi << 32) | v.lo; }
OTH_HD U2 operator&(U2 a, U2 b) { return U2{a.lo & b.lo, a.hi & b.hi}; }
OTH_HD U2 operator|(U2 a, U2 b) { return U2{a.lo | b.lo, a.hi | b.hi}; }
OTH_HD U2 operator~(U2 a) { return U2{~a.lo, ~a.hi}; }
OTH_HD U2 operator^(U2 a, U2 b) { return U2{a.lo ^ b.lo, a.hi ^ b.hi}; }
OTH_HD bool any(U2 a) { return (a.lo | a.hi) != 0u; }
template <int S>  // S > 0: toward higher squares; S < 0: toward lower squares
OTH_HD U2 sh(U2 x) {
    static_assert(S > -64 && S < 64, "shift within one word");
#if defined(__HIP_DEVICE_COMPILE__)
    // A shift by 1..31 as ONE v_lshl*_b64 (inline asm: the backend splits a 64-bit
    // shift of a value used as dwords back into v_lshlrev_b32 + v_alignbit_b32).
    // With one wave per SIMD an independent 64-bit shift issues in ~6.6 cycles,
    // the dword pair in ~11.5 (profiles/r01/ubench_valu.json): k_play_rand 8x8
    // 0.769 -> 0.720 us per ply (profiles/r03/sh64).  Constants still fold.
    if constexpr (S != 0 && S > -32 && S < 32) {
        const uint64_t v = u64(x);
        if (!__builtin_constant_p(v)) {
            uint64_t r;
            if constexpr (S > 0) asm("v_lshlrev_b64 %0, %2, %1" : "=v"(r) : "v"(v), "n"(S));
            else asm("v_lshrrev_b64 %0, %2, %1" : "=v"(r) : "v"(v), "n"(-S));
            return u2(r);
        }
    }
#endif
    if constexpr (S == 0) {
        return x;
    } else if constexpr (S >= 32) {
        return U2{0u, x.lo << (S - 32)};
    } else if constexpr (S > 0) {
        return U2{x.lo << S, (x.hi << S) | (x.lo >> (32 - S))};  // v_alignbit_b32
    } else if constexpr (S <= -32) {
        return U2{x.hi >> (-S - 32), 0u};
    } else {
        return U2{(x.lo >> -S) | (x.hi << (32 + S)), x.hi >> -S};
    }
}

// (a & b) | c per dword: one v_and_or_b32 each (spelled out: with 64-bit
// shifts in the chain the combiner refactors the first step into or + and)
OTH_HD U2 and_or(U2 a, U2 b, U2 c) {
#if defined(__HIP_DEVICE_COMPILE__)
    if (!__builtin_constant_p(u64(a) ^ u64(b) ^ u64(c)))
        return U2{(uint32_t)__builtin_amdgcn_bitop3_b32(a.lo, b.lo, c.lo, 0xEA),
                  (uint32_t)__builtin_amdgcn_bitop3_b32(a.hi, b.hi, c.hi, 0xEA)};
#endif
    return (a & b) | c;
}

// constant shift of a plain 64-bit word (OneWord::greedy's run lengths)
template <int S>
OTH_HD uint64_t sh(uint64_t x) {
    static_assert(S > -64 && S < 64, "shift within one word");
    if constexpr (S >= 0) return x << S;
    else return x >> -S;
}
OTH_HD bool any(uint64_t a) { return a != 0ull; }
// sh<S> of a plain word whose halves feed 3-input dword ops: kept ONE v_lshl*_b64
// for |S| < 32 (the backend would split it into v_lshlrev_b32 + v_alignbit_b32, as
// for U2's sh); |S| >= 32 is a dword move
template <int S>
OTH_HD uint64_t sh64(uint64_t x) {
#if defined(__HIP_DEVICE_COMPILE__)
    if constexpr (S != 0 && S > -32 && S < 32) {
        if (!__builtin_constant_p(x)) {
            uint64_t r;
            if constexpr (S > 0) asm("v_lshlrev_b64 %0, %2, %1" : "=v"(r) : "v"(x), "n"(S));
            else asm("v_lshrrev_b64 %0, %2, %1" : "=v"(r) : "v"(x), "n"(-S));
            return r;
        }
    }
#endif
    return sh<S>(x);
}

// a ^ b ^ c and majority(a, b, c): symmetric, so the builtin's operand order does not matter
OTH_HD uint64_t xor3_64(uint64_t a, uint64_t b, uint64_t c) {
#if defined(__HIP_DEVICE_COMPILE__)
    const uint32_t lo = __builtin_amdgcn_bitop3_b32((uint32_t)a, (uint32_t)b, (uint32_t)c, 0x96);
    const uint32_t hi = __builtin_amdgcn_bitop3_b32((uint32_t)(a >> 32), (uint32_t)(b >> 32), (uint32_t)(c >> 32), 0x96);
    return ((uint64_t)hi << 32) | lo;
#else
    return a ^ b ^ c;
#endif
}
OTH_HD uint64_t and3_64(uint64_t a, uint64_t b, uint64_t c) {
#if defined(__HIP_DEVICE_COMPILE__)
    const uint32_t lo = __builtin_amdgcn_bitop3_b32((uint32_t)a, (uint32_t)b, (uint32_t)c, 0x80);
    const uint32_t hi = __builtin_amdgcn_bitop3_b32((uint32_t)(a >> 32), (uint32_t)(b >> 32), (uint32_t)(c >> 32), 0x80);
    return ((uint64_t)hi << 32) | lo;
#else
    return a & b & c;
#endif
}
// a & ~b & c (the lowest set bit of y restricted to c, as (y, y - 1, c)): one 3-input op per dword
OTH_HD uint64_t andn_and_64(uint64_t a, uint64_t b, uint64_t c) {
#if defined(__HIP_DEVICE_COMPILE__)
    const uint32_t lo = __builtin_amdgcn_bitop3_b32((uint32_t)a, (uint32_t)b, (uint32_t)c, 0x20);
    const uint32_t hi = __builtin_amdgcn_bitop3_b32((uint32_t)(a >> 32), (uint32_t)(b >> 32), (uint32_t)(c >> 32), 0x20);
    return ((uint64_t)hi << 32) | lo;
#else
    return a & ~b & c;
#endif
}
OTH_HD uint64_t maj3_64(uint64_t a, uint64_t b, uint64_t c) {
#if defined(__HIP_DEVICE_COMPILE__)
    const uint32_t lo = __builtin_amdgcn_bitop3_b32((uint32_t)a, (uint32_t)b, (uint32_t)c, 0xE8);
    const uint32_t hi = __builtin_amdgcn_bitop3_b32((uint32_t)(a >> 32), (uint32_t)(b >> 32), (uint32_t)(c >> 32), 0xE8);
    return ((uint64_t)hi << 32) | lo;
#else
    return (a & b) | (c & (a | b));
#endif
}
// c ? x : y bit by bit: one 3-input op per dword
OTH_HD uint64_t sel_64(uint64_t c, uint64_t x, uint64_t y) {
#if defined(__HIP_DEVICE_COMPILE__)
    const uint32_t lo = __builtin_amdgcn_bitop3_b32((uint32_t)c, (uint32_t)x, (uint32_t)y, 0xCA);
    const uint32_t hi = __builtin_amdgcn_bitop3_b32((uint32_t)(c >> 32), (uint32_t)(x >> 32), (uint32_t)(y >> 32), 0xCA);
    return ((uint64_t)hi << 32) | lo;
#else
    return (c & x) | (~c & y);
#endif
}
// a | b | c: one 3-input op per dword
OTH_HD uint64_t or3_64(uint64_t a, uint64_t b, uint64_t c) {
#if defined(__HIP_DEVICE_COMPILE__)
    const uint32_t lo = __builtin_amdgcn_bitop3_b32((uint32_t)a, (uint32_t)b, (uint32_t)c, 0xFE);
    const uint32_t hi = __builtin_amdgcn_bitop3_b32((uint32_t)(a >> 32), (uint32_t)(b >> 32), (uint32_t)(c >> 32), 0xFE);
    return ((uint64_t)hi << 32) | lo;
#else
    return a | b | c;
#endif
}

template <int N>
struct Geo {
    static constexpr int NN = N * N;
    static constexpr int W = (NN + 63) / 64;
    static constexpr int MAXRUN = N - 2;  // longest capturable opponent run

    // bit a set iff square a is on the board and pred(col) holds
    template <int COLSKIP>
    static constexpr BB<W> make_mask() {
        BB<W> m{};
        for (int i = 0; i < W; ++i) m.w[i] = 0;
        for (int a = 0; a < NN; ++a)
            if (COLSKIP < 0 || a % N != COLSKIP) m.w[a / 64] |= 1ull << (a % 64);
        return m;
    }
    static constexpr BB<W> BOARD = make_mask<-1>();
    static constexpr BB<W> NOT_COL0 = make_mask<0>();
    static constexpr BB<W> NOT_COLN1 = make_mask<N - 1>();
    static constexpr BB<W> make_inner() {
        BB<W> m{};
        for (int i = 0; i < W; ++i) m.w[i] = 0;
        for (int a = 0; a < NN; ++a)
            if (a % N != 0 && a % N != N - 1) m.w[a / 64] |= 1ull << (a % 64);
        return m;
    }
    static constexpr BB<W> INNER = make_inner();  // board minus the two edge columns

    // A move one step in direction (DR, DC) = shift by DR*N+DC, then drop the
    // squares that wrapped around a board edge (or fell off the last word).
    template <int DC>
    static constexpr BB<W> dst_mask() {
        return DC > 0 ? NOT_COL0 : (DC < 0 ? NOT_COLN1 : BOARD);
    }
};

// (a & b) | c (the multi-word Kogge-Stone step; one-word and dword scans use U2 / DW)
template <int W>
OTH_HD BB<W> and_or(const BB<W>& a, const BB<W>& b, const BB<W>& c) {
    return (a & b) | c;
}

// Propagators of one direction for the discs O: pro[k] holds the squares x with
// x, x-S, ..., x-(2^k - 1)S all in O & dst_mask (Kogge-Stone doubling).  They
// depend only on O, so one set serves every ray cast through O in that direction.
template <int N, int DR, int DC>
struct Pro {
    static constexpr int W = Geo<N>::W;
    static constexpr int S = DR * N + DC;
    static constexpr int STEPS = Geo<N>::MAXRUN > 8 ? 4 : (Geo<N>::MAXRUN > 4 ? 3 : (Geo<N>::MAXRUN > 2 ? 2 : 1));
    // the last step reuses the previous propagator when that covers N - 2 (see legal_axis)
    static constexpr bool R3 = STEPS == 3 && Geo<N>::MAXRUN <= 6;
    static constexpr bool R4 = STEPS == 4 && Geo<N>::MAXRUN <= 12;
    BB<W> p1, p2, p4, p8;
    OTH_HD explicit Pro(const BB<W>& O) {
        p1 = O & Geo<N>::template dst_mask<DC>();
        if constexpr (STEPS > 1) p2 = p1 & shift<W, S>(p1);
        if constexpr (STEPS > 2 && !R3) p4 = p2 & shift<W, 2 * S>(p2);
        if constexpr (STEPS > 3 && !R4) p8 = p4 & shift<W, 4 * S>(p4);
    }
    // Extend `t` (opponent squares next to the generator) through the
    // contiguous opponent run along the direction (runs up to N - 2 long).
    OTH_HD BB<W> fill(BB<W> t) const {
        t = and_or(p1, shift<W, S>(t), t);
        if constexpr (STEPS > 1) t = and_or(p2, shift<W, 2 * S>(t), t);
        if constexpr (STEPS > 2) {
            if constexpr (R3) t = and_or(p2, shift<W, 2 * S>(t), t);
            else t = and_or(p4, shift<W, 4 * S>(t), t);
        }
        if constexpr (STEPS > 3) {
            if constexpr (R4) t = and_or(p4, shift<W, 4 * S>(t), t);
            else t = and_or(p8, shift<W, 8 * S>(t), t);
        }
        return t;
    }
    // squares of the run starting one step from the generator g
    OTH_HD BB<W> run_from(const BB<W>& g) const { return fill(shift<W, S>(g) & p1); }
};

// Both directions of one axis (shift S > 0 and -S) for the mover P against the
// propagator p1 (opponent discs that a run may pass through).  For the
// horizontal and diagonal axes p1 excludes the two edge columns: a run can
// never continue through an edge-column disc along those axes, and with t kept
// inside the inner columns no shift of t can wrap around a row, so no
// per-shift edge masks are needed.  The -S doubling chain is the +S chain
// shifted: p2-(y) = p2+(y+S), p4-(y) = p4+(y+3S), p8-(y) = p8+(y+7S).
template <int N, int S>
OTH_HD void legal_axis(const BB<Geo<N>::W>& P, const BB<Geo<N>::W>& p1, BB<Geo<N>::W>& L, BB<Geo<N>::W>& tplus,
                       BB<Geo<N>::W>& tminus) {
    constexpr int W = Geo<N>::W;
    constexpr int STEPS = Pro<N, 0, 1>::STEPS;
    // The last doubling step may reuse the previous propagator when that still
    // covers the longest run: 1 + 1 + 2 + 2 = 6 >= N - 2 for N <= 8, and
    // 1 + 1 + 2 + 4 + 4 = 12 >= N - 2 for N <= 14 (one propagator fewer per axis).
    constexpr bool R3 = STEPS == 3 && Geo<N>::MAXRUN <= 6;
    constexpr bool R4 = STEPS == 4 && Geo<N>::MAXRUN <= 12;
    BB<W> p2, p4, p8;
    if constexpr (STEPS > 1) p2 = p1 & shift<W, S>(p1);
    if constexpr (STEPS > 2 && !R3) p4 = p2 & shift<W, 2 * S>(p2);
    if constexpr (STEPS > 3 && !R4) p8 = p4 & shift<W, 4 * S>(p4);
    {  // +S
        BB<W> t = shift<W, S>(P) & p1;
        t |= p1 & shift<W, S>(t);
        if constexpr (STEPS > 1) t |= p2 & shift<W, 2 * S>(t);
        if constexpr (STEPS > 2) {
            if constexpr (R3) t |= p2 & shift<W, 2 * S>(t);
            else t |= p4 & shift<W, 4 * S>(t);
        }
        if constexpr (STEPS > 3) {
            if constexpr (R4) t |= p4 & shift<W, 4 * S>(t);
            else t |= p8 & shift<W, 8 * S>(t);
        }
        tplus = t;
        L |= shift<W, S>(t);
    }
    {  // -S
        BB<W> t = shift<W, -S>(P) & p1;
        t |= p1 & shift<W, -S>(t);
        BB<W> p2m, p4m;
        if constexpr (STEPS > 1) {
            p2m = shift<W, -S>(p2);
            t |= p2m & shift<W, -2 * S>(t);
        }
        if constexpr (STEPS > 2) {
            if constexpr (R3) {
                t |= p2m & shift<W, -2 * S>(t);
            } else {
                p4m = shift<W, -3 * S>(p4);
                t |= p4m & shift<W, -4 * S>(t);
            }
        }
        if constexpr (STEPS > 3) {
            if constexpr (R4) t |= p4m & shift<W, -4 * S>(t);
            else t |= shift<W, -7 * S>(p8) & shift<W, -8 * S>(t);
        }
        tminus = t;
        L |= shift<W, -S>(t);
    }
}
template <int N, int S>
OTH_HD void legal_axis(const BB<Geo<N>::W>& P, const BB<Geo<N>::W>& p1, BB<Geo<N>::W>& L) {
    BB<Geo<N>::W> tp, tm;  // fills not kept
    legal_axis<N, S>(P, p1, L, tp, tm);
}

// get_possible_actions (othello.py:313-343) as a mask: empty squares from
// which some direction holds >= 1 opponent disc followed by an own disc.
// Written as rays cast FROM the mover's discs; the set of (square, direction)
// pairs it accepts is the same as the reference's per-cell scan.
// Multi-word boards (W = 2..4) scan on dwords (legal_moves_fills_dw), both
// here and in legal_moves_fills.
template <int N>
OTH_HD BB<Geo<N>::W> legal_moves_fills_dw(const BB<Geo<N>::W>& Pb, const BB<Geo<N>::W>& Ob, BB<Geo<N>::W> t[8]);

template <int N>
OTH_HD BB<Geo<N>::W> legal_moves(const BB<Geo<N>::W>& P, const BB<Geo<N>::W>& O) {
    if constexpr (Geo<N>::W >= 2) {
        BB<Geo<N>::W> t[8];  // the fills are dead here
        return legal_moves_fills_dw<N>(P, O, t);
    }
    auto L = zero<Geo<N>::W>();
    const auto pin = O & Geo<N>::INNER;
    legal_axis<N, 1>(P, pin, L);      // E / W
    legal_axis<N, N>(P, O, L);        // S / N
    legal_axis<N, N + 1>(P, pin, L);  // SE / NW
    legal_axis<N, N - 1>(P, pin, L);  // SW / NE
    return L & ~(P | O) & Geo<N>::BOARD;
}

// legal_moves that keeps the eight fills (any W): t[d] = the opponent discs
// from which an own disc is reached going along ray direction d through
// opponent discs only (d = 0..3: E, S, SE, SW toward higher squares; 4..7: W,
// N, NW, NE).  The scan stepping +S from the own discs yields the fill of
// direction -S and vice versa.
template <int N>
OTH_HD BB<Geo<N>::W> legal_moves_fills(const BB<Geo<N>::W>& P, const BB<Geo<N>::W>& O, BB<Geo<N>::W> t[8]) {
    if constexpr (Geo<N>::W >= 2) return legal_moves_fills_dw<N>(P, O, t);
    auto L = zero<Geo<N>::W>();
    const auto pin = O & Geo<N>::INNER;
    legal_axis<N, 1>(P, pin, L, t[4], t[0]);      // W / E
    legal_axis<N, N>(P, O, L, t[5], t[1]);        // N / S
    legal_axis<N, N + 1>(P, pin, L, t[6], t[2]);  // NW / SE
    legal_axis<N, N - 1>(P, pin, L, t[7], t[3]);  // NE / SW
    return L & ~(P | O) & Geo<N>::BOARD;
}

// Multi-word boards (N = 9..16) on dwords (DW<2W>): legal_axis's arithmetic
// with every multi-word shift as one v_lshlrev / v_alignbit per dword (a
// funnel shift across the dword boundary) instead of 64-bit shifts plus the
// cross-word carries, and and-or pairs as v_and_or_b32 / v_bitop3_b32.
template <int K>
struct DW {
    uint32_t d[K];
};
template <int W>
OTH_HD DW<2 * W> to_dw(const BB<W>& b) {
    DW<2 * W> q;
#pragma unroll
    for (int i = 0; i < W; ++i) {
        q.d[2 * i] = (uint32_t)b.w[i];
        q.d[2 * i + 1] = (uint32_t)(b.w[i] >> 32);
    }
    return q;
}
template <int K>
OTH_HD BB<K / 2> to_bb(const DW<K>& q) {
    BB<K / 2> b;
#pragma unroll
    for (int i = 0; i < K / 2; ++i) b.w[i] = ((uint64_t)q.d[2 * i + 1] << 32) | q.d[2 * i];
    return b;
}
template <int K>
OTH_HD DW<K> operator&(const DW<K>& a, const DW<K>& b) {
    DW<K> r;
#pragma unroll
    for (int i = 0; i < K; ++i) r.d[i] = a.d[i] & b.d[i];
    return r;
}
template <int K>
OTH_HD DW<K> operator|(const DW<K>& a, const DW<K>& b) {
    DW<K> r;
#pragma unroll
    for (int i = 0; i < K; ++i) r.d[i] = a.d[i] | b.d[i];
    return r;
}
template <int K>
OTH_HD DW<K> operator~(const DW<K>& a) {
    DW<K> r;
#pragma unroll
    for (int i = 0; i < K; ++i) r.d[i] = ~a.d[i];
    return r;
}
// (hi:lo) >> c, low dword (c in 1..31)
OTH_HD uint32_t funnel_hd(uint32_t hi, uint32_t lo, uint32_t c) {
#if defined(__HIP_DEVICE_COMPILE__)
    return __builtin_amdgcn_alignbit(hi, lo, c);
#else
    return (uint32_t)((((uint64_t)hi << 32) | lo) >> c);
#endif
}
template <int S, int K>  // S > 0: toward higher squares
OTH_HD DW<K> sh(const DW<K>& x) {
    DW<K> y;
    if constexpr (S >= 0) {
        constexpr int q = S / 32, r = S % 32;
#pragma unroll
        for (int i = 0; i < K; ++i) {
            const int src = i - q;
            if (src < 0) y.d[i] = 0u;
            else if (r == 0) y.d[i] = x.d[src];
            else if (src == 0) y.d[i] = x.d[0] << r;
            else y.d[i] = funnel_hd(x.d[src], x.d[src - 1], 32 - r);
        }
    } else {
        constexpr int q = (-S) / 32, r = (-S) % 32;
#pragma unroll
        for (int i = 0; i < K; ++i) {
            const int src = i + q;
            if (src > K - 1) y.d[i] = 0u;
            else if (r == 0) y.d[i] = x.d[src];
            else if (src == K - 1) y.d[i] = x.d[K - 1] >> r;
            else y.d[i] = funnel_hd(x.d[src + 1], x.d[src], r);
        }
    }
    return y;
}

// a + b and y - 1 on K dwords, the carry / borrow passed along (v_add_co_u32 /
// v_sub_co_u32, then v_addc_co_u32 / v_subb_co_u32 per dword)
template <int K>
OTH_HD DW<K> add_dw(const DW<K>& a, const DW<K>& b) {
    DW<K> r;
    uint32_t c = 0;
#pragma unroll
    for (int i = 0; i < K; ++i) {
#if defined(__clang__)
        r.d[i] = __builtin_addc(a.d[i], b.d[i], c, &c);
#else
        const uint64_t x = (uint64_t)a.d[i] + b.d[i] + c;
        r.d[i] = (uint32_t)x;
        c = (uint32_t)(x >> 32);
#endif
    }
    return r;
}
template <int K>
OTH_HD DW<K> dec_dw(const DW<K>& y) {
    DW<K> r;
    uint32_t b = 0;
#pragma unroll
    for (int i = 0; i < K; ++i) {
#if defined(__clang__)
        r.d[i] = __builtin_subc(y.d[i], i == 0 ? 1u : 0u, b, &b);
#else
        const uint64_t x = (uint64_t)y.d[i] - (i == 0 ? 1u : 0u) - b;
        r.d[i] = (uint32_t)x;
        b = (uint32_t)(x >> 63);
#endif
    }
    return r;
}
OTH_HD uint32_t rev32(uint32_t x) {
#if defined(__clang__)
    return __builtin_bitreverse32(x);
#else
    return (uint32_t)(rev64(x) >> 32);
#endif
}
// Square a -> NN - 1 - a (the board turned by 180 degrees: rows stay rows,
// reversed; an involution) on K dwords: the dwords bit-reversed in reverse
// order (v_bfrev_b32), then moved down past the 32K - NN unused bits.
template <int N, int K>
OTH_HD DW<K> turn_dw(const DW<K>& x) {
    static_assert(32 * K >= N * N && 32 * K - N * N < 64, "the board's words");
    DW<K> r;
#pragma unroll
    for (int j = 0; j < K; ++j) r.d[j] = rev32(x.d[K - 1 - j]);
    return sh<-(32 * K - N * N)>(r);
}

// legal_axis on dwords (the same steps, propagators and reuse)
template <int N, int S, int K = 2 * Geo<N>::W>
OTH_HD void legal_axis_dw(const DW<K>& P, const DW<K>& p1, DW<K>& L, DW<K>& tplus, DW<K>& tminus) {
    constexpr int STEPS = Pro<N, 0, 1>::STEPS;
    constexpr bool R3 = STEPS == 3 && Geo<N>::MAXRUN <= 6;
    constexpr bool R4 = STEPS == 4 && Geo<N>::MAXRUN <= 12;
    DW<K> p2{}, p4{}, p8{};
    if constexpr (STEPS > 1) p2 = p1 & sh<S>(p1);
    if constexpr (STEPS > 2 && !R3) p4 = p2 & sh<2 * S>(p2);
    if constexpr (STEPS > 3 && !R4) p8 = p4 & sh<4 * S>(p4);
    {
        DW<K> t = sh<S>(P) & p1;
        t = (p1 & sh<S>(t)) | t;
        if constexpr (STEPS > 1) t = (p2 & sh<2 * S>(t)) | t;
        if constexpr (STEPS > 2) {
            if constexpr (R3) t = (p2 & sh<2 * S>(t)) | t;
            else t = (p4 & sh<4 * S>(t)) | t;
        }
        if constexpr (STEPS > 3) {
            if constexpr (R4) t = (p4 & sh<4 * S>(t)) | t;
            else t = (p8 & sh<8 * S>(t)) | t;
        }
        tplus = t;
        L = L | sh<S>(t);
    }
    {
        DW<K> t = sh<-S>(P) & p1;
        t = (p1 & sh<-S>(t)) | t;
        DW<K> p2m{}, p4m{};
        if constexpr (STEPS > 1) {
            p2m = sh<-S>(p2);
            t = (p2m & sh<-2 * S>(t)) | t;
        }
        if constexpr (STEPS > 2) {
            if constexpr (R3) {
                t = (p2m & sh<-2 * S>(t)) | t;
            } else {
                p4m = sh<-3 * S>(p4);
                t = (p4m & sh<-4 * S>(t)) | t;
            }
        }
        if constexpr (STEPS > 3) {
            if constexpr (R4) t = (p4m & sh<-4 * S>(t)) | t;
            else t = (sh<-7 * S>(p8) & sh<-8 * S>(t)) | t;
        }
        tminus = t;
        L = L | sh<-S>(t);
    }
}

// The horizontal axis of legal_axis_dw by carries (OneWord::axis_h on K dwords):
// stepping +1 from an own disc through a run of inner-column opponent discs is
// the carry chain of (P << 1) + pin, which clears the run and sets the square
// past it, so that fill is pin & ~((P << 1) + pin) -- a shift, a K-dword add
// and an and-not per dword instead of the Kogge-Stone chain and its
// propagators; stepping -1 is the same on the board turned by 180 degrees
// (turn_dw).  No carry crosses a row: pin holds no edge-column square.
template <int N, int K>
OTH_HD void axis_h_dw(const DW<K>& P, const DW<K>& pin, DW<K>& L, DW<K>& tplus, DW<K>& tminus) {
    const DW<K> fe = pin & ~add_dw(sh<1>(P), pin);
    const DW<K> rpin = turn_dw<N>(pin);
    const DW<K> fw = turn_dw<N>(rpin & ~add_dw(sh<1>(turn_dw<N>(P)), rpin));
    tplus = fe;
    tminus = fw;
    L = L | sh<1>(fe) | sh<-1>(fw);
}

// legal_moves_fills for multi-word boards on dwords (fills returned as words)
template <int N>
OTH_HD BB<Geo<N>::W> legal_moves_fills_dw(const BB<Geo<N>::W>& Pb, const BB<Geo<N>::W>& Ob, BB<Geo<N>::W> t[8]) {
    constexpr int W = Geo<N>::W, K = 2 * W;
    static_assert(W >= 2, "multi-word boards");
    const DW<K> P = to_dw<W>(Pb), O = to_dw<W>(Ob), pin = O & to_dw<W>(Geo<N>::INNER);
    DW<K> L{}, f[8];
    axis_h_dw<N>(P, pin, L, f[4], f[0]);  // 10x10 random play: 1.632 -> 1.536 us per ply (profiles/r06/d)
    legal_axis_dw<N, N>(P, O, L, f[5], f[1]);
    legal_axis_dw<N, N + 1>(P, pin, L, f[6], f[2]);
    legal_axis_dw<N, N - 1>(P, pin, L, f[7], f[3]);
#pragma unroll
    for (int d = 0; d < 8; ++d) t[d] = to_bb<K>(f[d]);
    return to_bb<K>(L & ~(P | O) & to_dw<W>(Geo<N>::BOARD));
}

// update_board's flips (othello.py:391-410) from the fills of the side to
// move (t[d]: the opponent discs from which an own disc is reached going along
// d) and the ray table rays[d * N*N + a] (the squares strictly beyond a in
// direction d), on dwords: along each ray direction d toward higher squares the
// run is ray & t[d] & (y - 1) with y = ray & ~t[d] (y - 1 a K-dword decrement:
// its lowest set bit, the first ray square outside the fill, cleared and every
// bit below it set); toward lower squares the same on the board turned by 180
// degrees, where the ray of d from a is the ray of the opposite direction d - 4
// from NN - 1 - a (the table's "up" half) and the fill is turn_dw(t[d]); the
// four turned runs are turned back once.  No count-leading-zeros, no per-word
// found / carry selects (round 5's word-by-word form with a lowest / highest set
// bit per word: 10x10 random play 1.588 -> 1.536 us per ply, profiles/r06/d).
template <int N>
OTH_HD BB<Geo<N>::W> flips_fills(const BB<Geo<N>::W>* rays, const BB<Geo<N>::W> t[8], int a) {
    constexpr int W = Geo<N>::W, K = 2 * W, NN = N * N;
    DW<K> up{}, dn{};
    const int ta = NN - 1 - a;
#pragma unroll
    for (int d = 0; d < 4; ++d) {
        const DW<K> ray = to_dw<W>(rays[d * NN + a]), td = to_dw<W>(t[d]);
        const DW<K> run = ray & td & dec_dw(ray & ~td);
        up = up | run;
    }
#pragma unroll
    for (int d = 4; d < 8; ++d) {
        const DW<K> ray = to_dw<W>(rays[(d - 4) * NN + ta]), td = turn_dw<N>(to_dw<W>(t[d]));
        const DW<K> run = ray & td & dec_dw(ray & ~td);
        dn = dn | run;
    }
    return to_bb<K>(up | turn_dw<N>(dn));
}

// GreedyPolicy on bit planes for any W (OneWord::greedy's algorithm on BB<W>):
// per direction the run length of every square from the fills as K-bit
// planes, the eight summed, the argmax narrowed plane by plane from the top.
template <int N>
struct PlanesW {
    static constexpr int W = Geo<N>::W;
    static constexpr int R = N - 2;  // longest run
    static constexpr int bits(int v) { return v < 2 ? 1 : 1 + bits(v / 2); }
    static constexpr int K = bits(R);      // planes of one run length
    static constexpr int T = bits(8 * R);  // planes of the sum over the 8 directions
    static constexpr int hi_of(int j) { return j >= 8 ? 8 : (j >= 4 ? 4 : (j >= 2 ? 2 : 1)); }

    // A[j] = {a : a + S, ..., a + jS all in the fill} (nested): A[1] = the fill
    // stepped back once; A[j] = A[hi] & (A[j - hi] stepped back hi times), hi the
    // largest power of two below j (A[2h] = A[h] & A[h] stepped back h).  Off-board
    // squares a shift reaches never come back: every shift of one direction goes
    // the same way.
    template <int S, int J>
    static OTH_HD void fill_A(BB<W>* A) {
        if constexpr (J <= R) {
            constexpr int H = hi_of(J);
            if constexpr (H == J) A[J] = A[H / 2] & shift<W, -(H / 2) * S>(A[H / 2]);
            else A[J] = A[H] & shift<W, -H * S>(A[J - H]);
            fill_A<S, J + 1>(A);
        }
    }
    // run length of every square along step S as K bit planes: bit k = XOR of
    // the A[j] with j a multiple of 2^k
    template <int S>
    static OTH_HD void run_len(const BB<W>& fill, BB<W>* out) {
        BB<W> A[R + 1];
        A[0] = zero<W>();
        A[1] = shift<W, -S>(fill);
        fill_A<S, 2>(A);
#pragma unroll
        for (int k = 0; k < K; ++k) {
            BB<W> b = zero<W>();
#pragma unroll
            for (int j = 1 << k; j <= R; j += 1 << k) b = b ^ A[j];
            out[k] = b;
        }
    }
    // out[0..NO) = a[0..NA) + b[0..NB) (ripple carry, carries past NO dropped)
    template <int NA, int NB, int NO>
    static OTH_HD void add(const BB<W>* a, const BB<W>* b, BB<W>* out) {
        BB<W> c = zero<W>();
#pragma unroll
        for (int i = 0; i < NO; ++i) {
            const BB<W> x = i < NA ? a[i] : zero<W>(), y = i < NB ? b[i] : zero<W>();
            out[i] = x ^ y ^ c;
            c = (x & y) | (c & (x | y));
        }
    }
    static constexpr int min_(int a, int b) { return a < b ? a : b; }
    // the candidates of `legal` with the largest flip count (narrowed plane by
    // plane from the top) and that count
    static OTH_HD BB<W> argmax_set(const BB<W> t[8], const BB<W>& legal, int& count) {
        constexpr int K1 = min_(K + 1, T), K2 = min_(K + 2, T);
        BB<W> n[8][K];
        run_len<1>(t[0], n[0]);
        run_len<N>(t[1], n[1]);
        run_len<N + 1>(t[2], n[2]);
        run_len<N - 1>(t[3], n[3]);
        run_len<-1>(t[4], n[4]);
        run_len<-N>(t[5], n[5]);
        run_len<-N - 1>(t[6], n[6]);
        run_len<-N + 1>(t[7], n[7]);
        BB<W> s1[4][K1], s2[2][K2], tot[T];
#pragma unroll
        for (int i = 0; i < 4; ++i) add<K, K, K1>(n[2 * i], n[2 * i + 1], s1[i]);
        add<K1, K1, K2>(s1[0], s1[1], s2[0]);
        add<K1, K1, K2>(s1[2], s1[3], s2[1]);
        add<K2, K2, T>(s2[0], s2[1], tot);
        BB<W> cand = legal;
        int c = 0;
#pragma unroll
        for (int i = T - 1; i >= 0; --i) {
            const BB<W> h = cand & tot[i];
            const bool hit = any(h);
            cand = pick(hit, h, cand);
            c |= hit ? 1 << i : 0;
        }
        count = c;
        return cand;
    }
    // GreedyPolicy.get_action (simple_policies.py:69-92): the candidate of
    // `legal` flipping the most discs, the lowest of equal counts; -1 without one
    static OTH_HD int greedy(const BB<W> t[8], const BB<W>& legal) {
        int unused;
        const BB<W> cand = argmax_set(t, legal, unused);
        int res = -1;
#pragma unroll
        for (int i = W - 1; i >= 0; --i)
            if (cand.w[i]) res = 64 * i + ctz64(cand.w[i]);
        return res;
    }
    // the largest flip count among the candidates of `legal` (0 without one)
    static OTH_HD int max_flips(const BB<W> t[8], const BB<W>& legal) {
        int count;
        (void)argmax_set(t, legal, count);
        return count;
    }
};

// ray table of fills_flips: rays[d * N*N + sq] for the eight directions
template <int N>
OTH_HD BB<Geo<N>::W> ray_from(int d, int sq) {
    // d: E, S, SE, SW, W, N, NW, NE (no tables: a runtime-indexed local array would live in scratch)
    const int dr = d == 0 || d == 4 ? 0 : (d < 4 ? 1 : -1);
    const int dc = d == 1 || d == 5 ? 0 : (d == 0 || d == 2 || d == 7 ? 1 : -1);
    auto r = zero<Geo<N>::W>();
    int row = sq / N + dr, col = sq % N + dc;
    while (row >= 0 && row < N && col >= 0 && col < N) {
        const int b = row * N + col;
#pragma unroll
        for (int i = 0; i < Geo<N>::W; ++i) r.w[i] |= (b / 64 == i) ? 1ull << (b % 64) : 0ull;  // no dynamic word index
        row += dr;
        col += dc;
    }
    return r;
}

template <int N, int DR, int DC>
OTH_HD void flips_dir(const BB<Geo<N>::W>& P, const BB<Geo<N>::W>& O, const BB<Geo<N>::W>& m,
                      BB<Geo<N>::W>& f) {
    constexpr int W = Geo<N>::W;
    const Pro<N, DR, DC> pro(O);
    const BB<W> t = pro.run_from(m);
    const bool capped = any(shift<W, DR * N + DC>(t) & (P & Geo<N>::template dst_mask<DC>()));
    f = and_or(t, select_if(capped, ~zero<W>()), f);
}

// update_board's flips (othello.py:391-410): for each direction, the run of
// opponent discs starting next to the move, kept only if capped by an own disc.
template <int N>
OTH_HD BB<Geo<N>::W> flips(const BB<Geo<N>::W>& P, const BB<Geo<N>::W>& O, const BB<Geo<N>::W>& m) {
    auto f = zero<Geo<N>::W>();
    flips_dir<N, 0, 1>(P, O, m, f);
    flips_dir<N, 0, -1>(P, O, m, f);
    flips_dir<N, 1, 0>(P, O, m, f);
    flips_dir<N, -1, 0>(P, O, m, f);
    flips_dir<N, 1, 1>(P, O, m, f);
    flips_dir<N, 1, -1>(P, O, m, f);
    flips_dir<N, -1, 1>(P, O, m, f);
    flips_dir<N, -1, -1>(P, O, m, f);
    return f;
}

// ---------------------------------------------------------------------------
// One-word boards (N <= 8) on dword pairs (U2): the legal scan that keeps its
// per-direction fills, and GreedyPolicy's flip count of every square at once.
// Ray directions d = 0..7: E, S, SE, SW (toward higher squares), W, N, NW, NE;
// t[d] = the fill of ray direction d: opponent discs from which an own disc is
// reached going along d through opponent discs only.  The run a move on square
// a flips along d is the contiguous part of ray d from a inside t[d].

template <int N>
struct OneWord {
    static_assert(Geo<N>::W == 1, "one-word boards (N <= 8)");
    static constexpr int STEPS = Pro<N, 0, 1>::STEPS;
    static_assert(STEPS <= 3 && Geo<N>::MAXRUN <= 6, "1 + 1 + 2 + 2 doubling covers the longest run");
    static constexpr uint64_t BD = Geo<N>::BOARD.w[0], IN = Geo<N>::INNER.w[0];

    // One axis (+S and -S) of legal_moves for the mover P through the
    // propagator p1: or-s the squares one step past each fill into L and
    // returns the fills (tplus: reached stepping +S from an own disc, the
    // fill of ray direction -S; tminus likewise).  The last doubling step
    // reuses p2 (runs are at most N - 2 <= 6 long).
    template <int S>
    static OTH_HD void axis(U2 P, U2 p1, U2& L, U2& tplus, U2& tminus) {
        U2 p2{0u, 0u};
        if constexpr (STEPS > 1) p2 = p1 & sh<S>(p1);
        U2 x = sh<S>(P) & p1;
        x = and_or(p1, sh<S>(x), x);
        if constexpr (STEPS > 1) x = and_or(p2, sh<2 * S>(x), x);
        if constexpr (STEPS > 2) x = and_or(p2, sh<2 * S>(x), x);
        tplus = x;
        L = L | sh<S>(x);
        const U2 p2m = sh<-S>(p2);
        x = sh<-S>(P) & p1;
        x = and_or(p1, sh<-S>(x), x);
        if constexpr (STEPS > 1) x = and_or(p2m, sh<-2 * S>(x), x);
        if constexpr (STEPS > 2) x = and_or(p2m, sh<-2 * S>(x), x);
        tminus = x;
        L = L | sh<-S>(x);
    }
    // Square a -> square NN-1-a: the board turned by 180 degrees (a row stays
    // a row, reversed), an involution on the board's NN bits.
    static OTH_HD uint64_t turn180(uint64_t x) { return rev64(x) >> (64 - N * N); }

    // The horizontal axis by carries: stepping +1 from an own
    // disc through a run of opponent discs of the inner columns is a carry
    // chain of (P << 1) + pin, which clears the run and sets the square past
    // it, so the fill is pin & ~((P << 1) + pin) -- one v_lshl_add_u64 and an
    // and-not instead of the doubling steps (no carry crosses a row: pin has
    // no edge-column square).  Stepping -1 is the same on the board turned by
    // 180 degrees.  tplus / tminus as in axis<1>.
    static OTH_HD void axis_h(uint64_t P, uint64_t pin, U2& L, U2& tplus, U2& tminus) {
        const uint64_t fe = pin & ~((P << 1) + pin);
        const uint64_t rpin = turn180(pin);
        const uint64_t fw = turn180(rpin & ~((turn180(P) << 1) + rpin));
        tplus = u2(fe);
        tminus = u2(fw);
        L = L | u2((fe << 1) | (fw >> 1));
    }

    // get_possible_actions (othello.py:313-343) for the mover P against O,
    // with the eight fills stored in t.
    static OTH_HD uint64_t legal(uint64_t Pw, uint64_t Ow, uint64_t t[8]) {
        const U2 P = u2(Pw), O = u2(Ow), pin = O & u2(IN);
        U2 L{0u, 0u}, f[8];
        axis_h(Pw, Ow & IN, L, f[4], f[0]);
        axis<N>(P, O, L, f[5], f[1]);
        axis<N + 1>(P, pin, L, f[6], f[2]);
        axis<N - 1>(P, pin, L, f[7], f[3]);
#pragma unroll
        for (int d = 0; d < 8; ++d) t[d] = u64(f[d]);
        return u64(L & ~(P | O) & u2(BD));
    }

    // out[0..NO) = a[0..NA) + b[0..NB) on bit planes (ripple carry, carries past NO
    // dropped): a half adder, then one 3-input op per dword for each sum and carry
    template <int NA, int NB, int NO>
    static OTH_HD void add_planes(const uint64_t* a, const uint64_t* b, uint64_t* out) {
        uint64_t c = 0;
#pragma unroll
        for (int i = 0; i < NO; ++i) {
            const uint64_t x = i < NA ? a[i] : 0ull, y = i < NB ? b[i] : 0ull;
            if (i == 0) {
                out[i] = x ^ y;
                c = x & y;
            } else {
                out[i] = xor3_64(x, y, c);
                c = maj3_64(x, y, c);
            }
        }
    }
    // The run length of every square along ray direction S -- how many of
    // a + S, a + 2S, ... lie in T before the first that does not (at most N - 2
    // for a fill) -- in binary (out[2], out[1], out[0]), by doubling a window:
    // L2 = min(r, 2) from T at a + S and a + 2S, L4 = L2 + [L2 = 2] L2(a + 2S),
    // L8 = L4 + [L4 = 4] L4(a + 4S): 6 shifts and 7 two- or three-input ops per
    // dword (20 VALU at 8x8, against 24 for the nested thermometer A_j =
    // {a : a + S, ..., a + jS all in T}, j = 1..6, and its binary code).  A
    // window is read past the square only when every square before it lies in
    // T; a horizontal or diagonal fill holds no edge-column square, so no
    // window that counts reads across a row's end.
    template <int S>
    static OTH_HD void run_bin(uint64_t T, uint64_t out[3]) {
        constexpr int R = N - 2;
        static_assert(R >= 2 && R <= 6, "N = 4 .. 8");
        const uint64_t x1 = sh64<-S>(T), y = sh64<-S>(x1);
        const uint64_t b1 = x1 & y, b0 = x1 & ~y;  // L2 = 2 b1 + b0
        if constexpr (R == 2) {
            out[0] = b0;
            out[1] = b1;
            out[2] = 0;
            return;
        }
        const uint64_t b1s = sh64<-2 * S>(b1), b0s = sh64<-2 * S>(b0);
        const uint64_t c2 = b1 & b1s, c1 = b1 & ~b1s, c0 = sel_64(b1, b0s, b0);  // L4
        if constexpr (R <= 4) {
            out[0] = c0;
            out[1] = c1;
            out[2] = c2;
            return;
        }
        const uint64_t c1s = sh64<-4 * S>(c1), c0s = sh64<-4 * S>(c0);
        out[0] = sel_64(c2, c0s, c0);  // L8 (a window of 8 would be a run past the board: never used)
        out[1] = sel_64(c2, c1s, c1);
        out[2] = c2;
    }
    // tot[0..5) = a[0] + a[1] + a[2] + a[3] for four 3-bit numbers on bit planes
    // (carry-save: full adders column by column, 18 three-input ops per dword
    // against 20 for the adder tree add_planes builds)
    static OTH_HD void sum4_planes(const uint64_t a[4][3], uint64_t tot[5]) {
        const uint64_t p = xor3_64(a[0][0], a[1][0], a[2][0]), cA = maj3_64(a[0][0], a[1][0], a[2][0]);
        tot[0] = p ^ a[3][0];
        const uint64_t cB = p & a[3][0];
        const uint64_t q1 = xor3_64(a[0][1], a[1][1], a[2][1]), cC = maj3_64(a[0][1], a[1][1], a[2][1]);
        const uint64_t q2 = xor3_64(a[3][1], cA, cB), cD = maj3_64(a[3][1], cA, cB);
        tot[1] = q1 ^ q2;
        const uint64_t cE = q1 & q2;
        const uint64_t r1 = xor3_64(a[0][2], a[1][2], a[2][2]), cF = maj3_64(a[0][2], a[1][2], a[2][2]);
        const uint64_t r2 = xor3_64(a[3][2], cC, cD), cG = maj3_64(a[3][2], cC, cD);
        tot[2] = xor3_64(r1, r2, cE);
        const uint64_t cH = maj3_64(r1, r2, cE);
        tot[3] = xor3_64(cF, cG, cH);
        tot[4] = maj3_64(cF, cG, cH);
    }
    // GreedyPolicy.get_action (simple_policies.py:69-92): the candidate (a
    // square of `legal`) flipping the most discs, the lowest of equal counts
    // (np.argmax); -1 without candidates.  The eight run lengths are summed on
    // bit planes (at most 18 flips on a board of N <= 8: 5 planes), then the
    // largest total among the candidates is found plane by plane from the top.
    // Opposite directions are added first: both runs lie on one line through
    // the square, between two own discs, so their sum is at most N - 2 <= 6 and
    // stays 3 bits (no carry out of the first adders); the four axis sums meet
    // in sum4_planes.  Round 6: 331 -> 264 VALU for this function in k_play_rand
    // <8, GREEDY> (run_bin's doubling instead of the nested thermometer
    // A_1..A_6, the carry-save sum); config 3, 65,536 boards, 100-ply launches
    // 1.458 -> 1.377 us per ply on one box (profiles/r06/a).
    // The planes are plain 64-bit words: on dword pairs (U2) the gfx950 backend
    // miscompiled them inside k_play ("A compiler hazard";
    // tests/test_gpu_hazards.py pins the position).
    static OTH_HD int greedy(const uint64_t t[8], uint64_t legal) {
        static_assert(N - 2 <= 7, "an axis' two runs fit 3 bits");
        uint64_t n[8][3], tot[5];
        run_bin<1>(t[0], n[0]);
        run_bin<N>(t[1], n[1]);
        run_bin<N + 1>(t[2], n[2]);
        run_bin<N - 1>(t[3], n[3]);
        run_bin<-1>(t[4], n[4]);
        run_bin<-N>(t[5], n[5]);
        run_bin<-N - 1>(t[6], n[6]);
        run_bin<-N + 1>(t[7], n[7]);
        uint64_t s3[4][3];
#pragma unroll
        for (int i = 0; i < 4; ++i) add_planes<3, 3, 3>(n[i], n[i + 4], s3[i]);  // d and its opposite d + 4
        sum4_planes(s3, tot);
        uint64_t cand = legal;
#pragma unroll
        for (int i = 4; i >= 0; --i) {
            const uint64_t h = cand & tot[i];
            cand = h ? h : cand;
        }
        return cand ? __builtin_ctzll(cand) : -1;
    }
};

// Position of the j-th set bit (j < popcount) of every 4-bit value v, 2 bits
// per (v, j) at bit offset 2 * (4 v + j): two 64-bit constants.
constexpr uint64_t sel4_table(int half) {
    uint64_t t = 0;
    for (int v = 8 * half; v < 8 * half + 8; ++v) {
        int j = 0;
        for (int b = 0; b < 4; ++b)
            if ((v >> b) & 1) {
                t |= (uint64_t)b << (2 * (4 * (v - 8 * half) + j));
                ++j;
            }
    }
    return t;
}

// Index of the k-th (0-based, ascending) set bit of a non-zero word, k < popcount.
// Shallow form for one wave per SIMD: the 32-bit half by the low word's count,
// the byte by comparing k with the three byte-prefix counts at once, the nibble
// by one count, the bit from a 128-bit table.
OTH_HD int select64(uint64_t x, int k) {
    const uint32_t lo = (uint32_t)x;
    const int c = popc64(lo);
    const bool up = k >= c;
    const uint32_t v = up ? (uint32_t)(x >> 32) : lo;
    const int kk = up ? k - c : k;
    const int q1 = popc64(v & 0xFFu), q2 = popc64(v & 0xFFFFu), q3 = popc64(v & 0xFFFFFFu);
    const bool m1 = q1 <= kk, m2 = q2 <= kk, m3 = q3 <= kk;
    const int b = (int)m1 + (int)m2 + (int)m3;  // prefix counts grow with the byte index
    const int qb = m3 ? q3 : (m2 ? q2 : (m1 ? q1 : 0));
    const uint32_t byte = (v >> (8 * b)) & 0xFFu;
    const int kb = kk - qb;
    const int cn = popc64(byte & 0xFu);
    const bool un = kb >= cn;
    const uint32_t nib = un ? byte >> 4 : byte & 0xFu;
    const int kn = un ? kb - cn : kb;
    constexpr uint64_t T0 = sel4_table(0), T1 = sel4_table(1);
    const uint64_t t = (nib & 8u) ? T1 : T0;
    const int bit = (int)((t >> (2 * (4 * (nib & 7u) + kn))) & 3u);
    return (up ? 32 : 0) + 8 * b + (un ? 4 : 0) + bit;
}
// The same select with the bit inside the byte read from a table (sel8: the
// set-bit positions of every byte value, ascending, one byte each -- 2 KiB in
// LDS, sel8_word): one ds_read_u8 in place of the nibble step's ~18 VALU.
OTH_HD constexpr uint64_t sel8_word(uint32_t v) {
    uint64_t w = 0;
    int j = 0;
    for (int b = 0; b < 8; ++b)
        if ((v >> b) & 1u) {
            w |= (uint64_t)b << (8 * j);
            ++j;
        }
    return w;
}
OTH_HD int select64_tab(uint64_t x, int k, const uint8_t* sel8) {
    const uint32_t lo = (uint32_t)x;
    const int c = popc64(lo);
    const bool up = k >= c;
    const uint32_t v = up ? (uint32_t)(x >> 32) : lo;
    const int kk = up ? k - c : k;
    const int q1 = popc64(v & 0xFFu), q2 = popc64(v & 0xFFFFu), q3 = popc64(v & 0xFFFFFFu);
    const bool m1 = q1 <= kk, m2 = q2 <= kk, m3 = q3 <= kk;
    const int b = (int)m1 + (int)m2 + (int)m3;
    const int qb = m3 ? q3 : (m2 ? q2 : (m1 ? q1 : 0));
#if defined(__HIP_DEVICE_COMPILE__)
    const uint32_t byte = __builtin_amdgcn_ubfe(v, 8u * (uint32_t)b, 8u);  // v_bfe_u32
#else
    const uint32_t byte = (v >> (8 * b)) & 0xFFu;
#endif
    return (up ? 32 : 0) + 8 * b + sel8[8 * byte + (uint32_t)(kk - qb)];
}
// select_bit with select64_tab inside the word (k < popcount: a pick from a
// non-empty mask), without branches: the word holding the k-th set bit picked by
// selects on the words' prefix counts, then ONE select64_tab.  A word-by-word
// loop compiles to an exec-masked region per word, each run whenever some lane
// of the wave picks in that word (two-word random play ran both on almost every
// ply): 10x10 random play 1.540 -> 1.437 us per ply (profiles/r06/e).
template <int W>
OTH_HD int select_bit_tab(const BB<W>& b, int k, const uint8_t* sel8) {
    uint64_t x = b.w[0];
    int kk = k, base = 0, pre = 0;
#pragma unroll
    for (int i = 1; i < W; ++i) {
        pre += popc64(b.w[i - 1]);
        const bool up = k >= pre;
        x = up ? b.w[i] : x;
        kk = up ? k - pre : kk;
        base = up ? 64 * i : base;
    }
    return base + select64_tab(x, kk, sel8);
}
template <int W>
OTH_HD int select_bit(const BB<W>& b, int k) {
    if constexpr (W == 1) {  // branch-free: -1 when k >= popcount (no legal move)
        const int s = select64(b.w[0], k);
        return k < popc64(b.w[0]) ? s : -1;
    }
    int res = -1;
    bool found = false;
#pragma unroll
    for (int i = 0; i < W; ++i) {
        int c = popc64(b.w[i]);
        if (!found && k < c) {
            res = 64 * i + select64(b.w[i], k);
            found = true;
        }
        if (!found) k -= c;
    }
    return res;
}

// Philox4x32-10 (Salmon et al., SC'11): the env RNG.  Counter = {env id,
// ply lo, ply hi, purpose}, key = seed.  Stateless, so results do not depend on
// how envs are sharded over GPUs or batched over launches.
struct U4 {
    uint32_t x, y, z, w;
};
// a ^ b ^ c; round r of philox4 takes the 3-input form (one v_bitop3_b32; the
// backend emits two v_xor_b32) only from round 2 on,
// where every operand but the key varies per lane (rounds 0 and 1 keep their
// uniform parts on the scalar unit)
template <int R>
OTH_HD uint32_t philox_xor(uint32_t a, uint32_t b, uint32_t c) {
#if defined(__HIP_DEVICE_COMPILE__)
    if constexpr (R >= 2) return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);
#endif
    return a ^ b ^ c;
}
template <int R>
OTH_HD void philox_round(uint32_t& c0, uint32_t& c1, uint32_t& c2, uint32_t& c3, uint32_t k0, uint32_t k1) {
    const uint64_t p0 = (uint64_t)0xD2511F53u * c0;
    const uint64_t p1 = (uint64_t)0xCD9E8D57u * c2;
    const uint32_t n0 = philox_xor<R>((uint32_t)(p1 >> 32), c1, k0);
    const uint32_t n1 = (uint32_t)p1;
    const uint32_t n2 = philox_xor<R>((uint32_t)(p0 >> 32), c3, k1);
    const uint32_t n3 = (uint32_t)p0;
    c0 = n0;
    c1 = n1;
    c2 = n2;
    c3 = n3;
}
OTH_HD U4 philox4(uint64_t seed, uint32_t id, uint64_t ctr, uint32_t purpose) {
    uint32_t k0 = (uint32_t)seed, k1 = (uint32_t)(seed >> 32);
    uint32_t c0 = id, c1 = (uint32_t)ctr, c2 = (uint32_t)(ctr >> 32), c3 = purpose;
    constexpr uint32_t W0 = 0x9E3779B9u, W1 = 0xBB67AE85u;
    philox_round<0>(c0, c1, c2, c3, k0, k1);
    philox_round<1>(c0, c1, c2, c3, k0 + W0, k1 + W1);
    philox_round<2>(c0, c1, c2, c3, k0 + 2 * W0, k1 + 2 * W1);
    philox_round<3>(c0, c1, c2, c3, k0 + 3 * W0, k1 + 3 * W1);
    philox_round<4>(c0, c1, c2, c3, k0 + 4 * W0, k1 + 4 * W1);
    philox_round<5>(c0, c1, c2, c3, k0 + 5 * W0, k1 + 5 * W1);
    philox_round<6>(c0, c1, c2, c3, k0 + 6 * W0, k1 + 6 * W1);
    philox_round<7>(c0, c1, c2, c3, k0 + 7 * W0, k1 + 7 * W1);
    philox_round<8>(c0, c1, c2, c3, k0 + 8 * W0, k1 + 8 * W1);
    philox_round<9>(c0, c1, c2, c3, k0 + 9 * W0, k1 + 9 * W1);
    return U4{c0, c1, c2, c3};
}
OTH_HD uint32_t philox_x(uint64_t seed, uint32_t id, uint64_t ply, uint32_t purpose) {
    return philox4(seed, id, ply, purpose).x;
}
// The random-opening length draw (SimpleOthelloEnv.reset's randint, othello.py:62-63,
// at a reset or an auto-reset): one 32-bit word from (seed, env id, ply, purpose) by
// murmur3's 32-bit finaliser: a key from the seed and the purpose, then the ply (both
// wave-uniform: scalar work), then the env id: 5-7 VALU a lane, where a Philox4x32-10
// evaluation was ~40 with 16-19 v_mad_u64_u32.  The terminal block that draws it runs
// on most of a wave's plies (some board of 64 ends a game): config 3 at 65,536 boards,
// 100-ply launches -3.9 % with a cheap draw in its place (profiles/r06/aa).  A choice
// among init_rand / 2 + 1 <= 6 lengths needs the top bits well mixed, which fmix32's
// avalanche gives; the action and sampling draws stay Philox.
OTH_HD uint32_t fmix32(uint32_t h) {
    h ^= h >> 16;
    h *= 0x85EBCA6Bu;
    h ^= h >> 13;
    h *= 0xC2B2AE35u;
    h ^= h >> 16;
    return h;
}
OTH_HD uint32_t opening_draw(uint64_t seed, uint32_t id, uint64_t ply, uint32_t purpose) {
#if OTH_OPENING_PHILOX  // A/B timing arm only (other values: the oracle follows the hash)
    return philox_x(seed, id, ply, purpose);
#else
    // the key depends on the seed and the purpose alone (loop-invariant: hoisted out
    // of the play loops), the ply enters once, the env id last
    const uint32_t key = fmix32((uint32_t)seed ^ fmix32((uint32_t)(seed >> 32) ^ purpose * 0x7FEB352Du));
    const uint32_t c = fmix32(key ^ (uint32_t)ply ^ (uint32_t)(ply >> 32) * 0x9E3779B9u);
    return fmix32(c ^ id);
#endif
}
OTH_HD uint32_t pick4(const U4& u, uint32_t j) {
#if defined(__HIP_DEVICE_COMPILE__)
    // by masks: on a wave-uniform j (a ply counter) the select chain became a tree
    // of scalar branches, ~40-80 cycles each to a lone wave
    const uint32_t m0 = 0u - (uint32_t)(j == 0), m1 = 0u - (uint32_t)(j == 1), m2 = 0u - (uint32_t)(j == 2);
    return (u.x & m0) | (u.y & m1) | (u.z & m2) | (u.w & ~(m0 | m1 | m2));
#else
    return j == 0 ? u.x : (j == 1 ? u.y : (j == 2 ? u.z : u.w));
#endif
}
// The random-move draw of ply g: word g % 4 of the block counter g / 4, so one
// Philox evaluation serves four consecutive plies of a board.
OTH_HD uint32_t action_draw(uint64_t seed, uint32_t id, uint64_t g) {
    return pick4(philox4(seed, id, g >> 2, 0), (uint32_t)(g & 3));
}

// floor(u * n / 2^32): uniform index in [0, n) (RandomPolicy, simple_policies.py:39).
OTH_HD int scale_index(uint32_t u, int n) {
#if defined(__HIP_DEVICE_COMPILE__)
    return (int)__umulhi(u, (uint32_t)n);  // a 32-bit result: the callers' compares stay 32-bit
#else
    return (int)(((uint64_t)u * (uint64_t)n) >> 32);
#endif
}

}  // namespace oth
