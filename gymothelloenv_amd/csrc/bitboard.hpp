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

    // A move one step in direction (DR, DC) = shift by DR*N+DC, then drop the
    // squares that wrapped around a board edge (or fell off the last word).
    template <int DC>
    static constexpr BB<W> dst_mask() {
        return DC > 0 ? NOT_COL0 : (DC < 0 ? NOT_COLN1 : BOARD);
    }
};

template <int N, int DR, int DC>
OTH_HD BB<Geo<N>::W> step_dir(const BB<Geo<N>::W>& x) {
    constexpr int W = Geo<N>::W;
    return shift<W, DR * N + DC>(x) & Geo<N>::template dst_mask<DC>();
}

// Extend `t` (a set of opponent squares adjacent, in direction D, to the
// generator) through the contiguous opponent discs O along D: Kogge-Stone
// doubling over propagator pro = O & dst_mask, enough steps for run N-2.
template <int N, int DR, int DC>
OTH_HD BB<Geo<N>::W> run_fill(BB<Geo<N>::W> t, const BB<Geo<N>::W>& O) {
    constexpr int W = Geo<N>::W;
    constexpr int S = DR * N + DC;
    BB<W> pro = O & Geo<N>::template dst_mask<DC>();
    t |= pro & shift<W, S>(t);  // runs of length <= 2
    if constexpr (Geo<N>::MAXRUN > 2) {
        pro &= shift<W, S>(pro);
        t |= pro & shift<W, 2 * S>(t);  // <= 4
    }
    if constexpr (Geo<N>::MAXRUN > 4) {
        pro &= shift<W, 2 * S>(pro);
        t |= pro & shift<W, 4 * S>(t);  // <= 8
    }
    if constexpr (Geo<N>::MAXRUN > 8) {
        pro &= shift<W, 4 * S>(pro);
        t |= pro & shift<W, 8 * S>(t);  // <= 16
    }
    return t;
}

// Legal squares for the side owning P against O, along one direction.
template <int N, int DR, int DC>
OTH_HD BB<Geo<N>::W> legal_dir(const BB<Geo<N>::W>& P, const BB<Geo<N>::W>& O) {
    auto t = step_dir<N, DR, DC>(P) & O;
    t = run_fill<N, DR, DC>(t, O);
    return step_dir<N, DR, DC>(t);
}

// get_possible_actions (othello.py:313-343) as a mask: empty squares from
// which some direction holds >= 1 opponent disc followed by an own disc.
// Written as rays cast FROM the mover's discs; the set of (square, direction)
// pairs it accepts is the same as the reference's per-cell scan.
template <int N>
OTH_HD BB<Geo<N>::W> legal_moves(const BB<Geo<N>::W>& P, const BB<Geo<N>::W>& O) {
    auto L = legal_dir<N, 0, 1>(P, O);
    L |= legal_dir<N, 0, -1>(P, O);
    L |= legal_dir<N, 1, 0>(P, O);
    L |= legal_dir<N, -1, 0>(P, O);
    L |= legal_dir<N, 1, 1>(P, O);
    L |= legal_dir<N, 1, -1>(P, O);
    L |= legal_dir<N, -1, 1>(P, O);
    L |= legal_dir<N, -1, -1>(P, O);
    return L & ~(P | O) & Geo<N>::BOARD;
}

template <int N, int DR, int DC>
OTH_HD BB<Geo<N>::W> flips_dir(const BB<Geo<N>::W>& P, const BB<Geo<N>::W>& O, const BB<Geo<N>::W>& m) {
    auto t = step_dir<N, DR, DC>(m) & O;
    t = run_fill<N, DR, DC>(t, O);
    return select_if(any(step_dir<N, DR, DC>(t) & P), t);
}

// update_board's flips (othello.py:391-410): for each direction, the run of
// opponent discs starting next to the move, kept only if capped by an own disc.
template <int N>
OTH_HD BB<Geo<N>::W> flips(const BB<Geo<N>::W>& P, const BB<Geo<N>::W>& O, const BB<Geo<N>::W>& m) {
    auto f = flips_dir<N, 0, 1>(P, O, m);
    f |= flips_dir<N, 0, -1>(P, O, m);
    f |= flips_dir<N, 1, 0>(P, O, m);
    f |= flips_dir<N, -1, 0>(P, O, m);
    f |= flips_dir<N, 1, 1>(P, O, m);
    f |= flips_dir<N, 1, -1>(P, O, m);
    f |= flips_dir<N, -1, 1>(P, O, m);
    f |= flips_dir<N, -1, -1>(P, O, m);
    return f;
}

// Index of the k-th (0-based, ascending) set bit of a non-zero word, k < popcount.
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
OTH_HD uint32_t philox_x(uint64_t seed, uint32_t id, uint64_t ply, uint32_t purpose) {
    uint32_t k0 = (uint32_t)seed, k1 = (uint32_t)(seed >> 32);
    uint32_t c0 = id, c1 = (uint32_t)ply, c2 = (uint32_t)(ply >> 32), c3 = purpose;
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
    return c0;
}

// floor(u * n / 2^32): uniform index in [0, n) (RandomPolicy, simple_policies.py:39).
OTH_HD int scale_index(uint32_t u, int n) { return (int)(((uint64_t)u * (uint64_t)n) >> 32); }

}  // namespace oth
