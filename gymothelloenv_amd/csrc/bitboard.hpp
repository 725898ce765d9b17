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
    return __popcll(x);
#else
    return __builtin_popcountll(x);
#endif
}
template <int W>
OTH_HD int popcount(const BB<W>& a) {
    int c = 0;
#pragma unroll
    for (int i = 0; i < W; ++i) c += popc64(a.w[i]);
    return c;
}

#ifndef OTH_SHIFT32
#define OTH_SHIFT32 0
#endif

#if defined(__HIP_DEVICE_COMPILE__)
// ({hi, lo} >> c)[31:0]: one full-rate VALU op (v_alignbit_b32)
__device__ __forceinline__ uint32_t funnel(uint32_t hi, uint32_t lo, uint32_t c) {
    return __builtin_amdgcn_alignbit(hi, lo, c);
}
#endif

// Logical shift of the whole W-word board by S bits (S > 0 toward higher squares).
template <int W, int S>
OTH_HD BB<W> shift(const BB<W>& x) {
#if defined(__HIP_DEVICE_COMPILE__) && OTH_SHIFT32
    // On the device the board is handled as 2W dwords: each output dword is one
    // funnel shift of two input dwords (v_alignbit_b32), instead of 64-bit
    // shifts (v_lshlrev_b64 / v_lshrrev_b64) plus or-combines.
    if constexpr (S != 0) {
        constexpr int D = 2 * W;
        uint32_t v[D], r[D];
#pragma unroll
        for (int i = 0; i < W; ++i) {
            v[2 * i] = (uint32_t)x.w[i];
            v[2 * i + 1] = (uint32_t)(x.w[i] >> 32);
        }
        if constexpr (S > 0) {
            constexpr int q = S / 32, s = S % 32;
#pragma unroll
            for (int i = 0; i < D; ++i) {
                if (i - q < 0) {
                    r[i] = 0;
                } else if (s == 0) {
                    r[i] = v[i - q];
                } else if (i - q - 1 < 0) {
                    r[i] = v[i - q] << s;
                } else {
                    r[i] = funnel(v[i - q], v[i - q - 1], 32 - s);
                }
            }
        } else {
            constexpr int T = -S, q = T / 32, s = T % 32;
#pragma unroll
            for (int i = 0; i < D; ++i) {
                if (i + q >= D) {
                    r[i] = 0;
                } else if (s == 0) {
                    r[i] = v[i + q];
                } else if (i + q + 1 >= D) {
                    r[i] = v[i + q] >> s;
                } else {
                    r[i] = funnel(v[i + q + 1], v[i + q], s);
                }
            }
        }
        BB<W> out;
#pragma unroll
        for (int i = 0; i < W; ++i) out.w[i] = ((uint64_t)r[2 * i + 1] << 32) | r[2 * i];
        return out;
    }
#endif
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

#ifndef OTH_PROP_REUSE
#define OTH_PROP_REUSE 1  // last doubling step reuses the previous propagator where it covers N - 2
#endif

#ifndef OTH_ANDOR
#define OTH_ANDOR 0
#endif

// (a & b) | c.  hipcc does not fuse 64-bit and/or pairs into v_and_or_b32
// (it does for 32-bit values), so on the device each 32-bit half is one
// explicit v_and_or_b32: 2 VALU ops per word instead of 4.
template <int W>
OTH_HD BB<W> and_or(const BB<W>& a, const BB<W>& b, const BB<W>& c) {
#if defined(__HIP_DEVICE_COMPILE__) && OTH_ANDOR
    BB<W> r;
#pragma unroll
    for (int i = 0; i < W; ++i) {
        uint32_t lo, hi;
        asm("v_and_or_b32 %0, %1, %2, %3" : "=v"(lo) : "v"((uint32_t)a.w[i]), "v"((uint32_t)b.w[i]),
            "v"((uint32_t)c.w[i]));
        asm("v_and_or_b32 %0, %1, %2, %3" : "=v"(hi) : "v"((uint32_t)(a.w[i] >> 32)),
            "v"((uint32_t)(b.w[i] >> 32)), "v"((uint32_t)(c.w[i] >> 32)));
        r.w[i] = ((uint64_t)hi << 32) | lo;
    }
    return r;
#else
    return (a & b) | c;
#endif
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
    static constexpr bool R3 = OTH_PROP_REUSE && STEPS == 3 && Geo<N>::MAXRUN <= 6;
    static constexpr bool R4 = OTH_PROP_REUSE && STEPS == 4 && Geo<N>::MAXRUN <= 12;
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

// Legal squares for the mover P along one direction, or-ed into L (unmasked
// by emptiness; legal_moves applies that once).
template <int N, int DR, int DC>
OTH_HD void legal_dir(const BB<Geo<N>::W>& P, const BB<Geo<N>::W>& O, BB<Geo<N>::W>& L) {
    constexpr int W = Geo<N>::W;
    const Pro<N, DR, DC> pro(O);
    const BB<W> t = pro.run_from(P);
    L = and_or(shift<W, DR * N + DC>(t), Geo<N>::template dst_mask<DC>(), L);
}

#ifndef OTH_AXIS_LEGAL
#define OTH_AXIS_LEGAL 1
#endif

// Both directions of one axis (shift S > 0 and -S) for the mover P against the
// propagator p1 (opponent discs that a run may pass through).  For the
// horizontal and diagonal axes p1 excludes the two edge columns: a run can
// never continue through an edge-column disc along those axes, and with t kept
// inside the inner columns no shift of t can wrap around a row, so no
// per-shift edge masks are needed.  The -S doubling chain is the +S chain
// shifted: p2-(y) = p2+(y+S), p4-(y) = p4+(y+3S), p8-(y) = p8+(y+7S).
template <int N, int S>
OTH_HD void legal_axis(const BB<Geo<N>::W>& P, const BB<Geo<N>::W>& p1, BB<Geo<N>::W>& L) {
    constexpr int W = Geo<N>::W;
    constexpr int STEPS = Pro<N, 0, 1>::STEPS;
    // The last doubling step may reuse the previous propagator when that still
    // covers the longest run: 1 + 1 + 2 + 2 = 6 >= N - 2 for N <= 8, and
    // 1 + 1 + 2 + 4 + 4 = 12 >= N - 2 for N <= 14 (one propagator fewer per axis).
    constexpr bool R3 = OTH_PROP_REUSE && STEPS == 3 && Geo<N>::MAXRUN <= 6;
    constexpr bool R4 = OTH_PROP_REUSE && STEPS == 4 && Geo<N>::MAXRUN <= 12;
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
        L |= shift<W, -S>(t);
    }
}

// get_possible_actions (othello.py:313-343) as a mask: empty squares from
// which some direction holds >= 1 opponent disc followed by an own disc.
// Written as rays cast FROM the mover's discs; the set of (square, direction)
// pairs it accepts is the same as the reference's per-cell scan.
template <int N>
OTH_HD BB<Geo<N>::W> legal_moves(const BB<Geo<N>::W>& P, const BB<Geo<N>::W>& O) {
    auto L = zero<Geo<N>::W>();
#if OTH_AXIS_LEGAL
    const auto pin = O & Geo<N>::INNER;
    legal_axis<N, 1>(P, pin, L);      // E / W
    legal_axis<N, N>(P, O, L);        // S / N
    legal_axis<N, N + 1>(P, pin, L);  // SE / NW
    legal_axis<N, N - 1>(P, pin, L);  // SW / NE
#else
    legal_dir<N, 0, 1>(P, O, L);
    legal_dir<N, 0, -1>(P, O, L);
    legal_dir<N, 1, 0>(P, O, L);
    legal_dir<N, -1, 0>(P, O, L);
    legal_dir<N, 1, 1>(P, O, L);
    legal_dir<N, 1, -1>(P, O, L);
    legal_dir<N, -1, 1>(P, O, L);
    legal_dir<N, -1, -1>(P, O, L);
#endif
    return L & ~(P | O) & Geo<N>::BOARD;
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

#ifndef OTH_SELECT
#define OTH_SELECT 2  // 1: six-level binary search; 2: byte prefix counts compared in parallel + nibble table
#endif

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
#if OTH_SELECT == 2
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
#else
OTH_HD int select64(uint64_t x, int k) {
    int pos = 0;
    uint32_t lo = (uint32_t)x;
    int c = popc64(lo);
    uint32_t v = lo;
    if (k >= c) {
        k -= c;
        v = (uint32_t)(x >> 32);
        pos = 32;
    }
#pragma unroll
    for (int width = 16; width >= 1; width >>= 1) {
        uint32_t low = v & ((1u << width) - 1u);
        int cl = popc64(low);
        if (k >= cl) {
            k -= cl;
            v >>= width;
            pos += width;
        } else {
            v = low;
        }
    }
    return pos;
}
#endif

template <int W>
OTH_HD int select_bit(const BB<W>& b, int k) {
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
OTH_HD U4 philox4(uint64_t seed, uint32_t id, uint64_t ctr, uint32_t purpose) {
    uint32_t k0 = (uint32_t)seed, k1 = (uint32_t)(seed >> 32);
    uint32_t c0 = id, c1 = (uint32_t)ctr, c2 = (uint32_t)(ctr >> 32), c3 = purpose;
#pragma unroll
    for (int r = 0; r < 10; ++r) {
        uint64_t p0 = (uint64_t)0xD2511F53u * c0;
        uint64_t p1 = (uint64_t)0xCD9E8D57u * c2;
        uint32_t n0 = (uint32_t)(p1 >> 32) ^ c1 ^ k0;
        uint32_t n1 = (uint32_t)p1;
        uint32_t n2 = (uint32_t)(p0 >> 32) ^ c3 ^ k1;
        uint32_t n3 = (uint32_t)p0;
        c0 = n0;
        c1 = n1;
        c2 = n2;
        c3 = n3;
        k0 += 0x9E3779B9u;
        k1 += 0xBB67AE85u;
    }
    return U4{c0, c1, c2, c3};
}
OTH_HD uint32_t philox_x(uint64_t seed, uint32_t id, uint64_t ply, uint32_t purpose) {
    return philox4(seed, id, ply, purpose).x;
}
OTH_HD uint32_t pick4(const U4& u, uint32_t j) { return j == 0 ? u.x : (j == 1 ? u.y : (j == 2 ? u.z : u.w)); }
// The random-move draw of ply g: word g % 4 of the block counter g / 4, so one
// Philox evaluation serves four consecutive plies of a board.
OTH_HD uint32_t action_draw(uint64_t seed, uint32_t id, uint64_t g) {
    return pick4(philox4(seed, id, g >> 2, 0), (uint32_t)(g & 3));
}

// floor(u * n / 2^32): uniform index in [0, n) (RandomPolicy, simple_policies.py:39).
OTH_HD int scale_index(uint32_t u, int n) { return (int)(((uint64_t)u * (uint64_t)n) >> 32); }

}  // namespace oth
