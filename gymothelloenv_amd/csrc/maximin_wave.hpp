// maximin_wave.hpp -- MaxiMinPolicy(D).get_action (simple_policies.py:98-163)
// for D >= 3 with one WAVE per board instead of one lane walking the whole tree.
// The search's first two levels are spread over the wave's lanes: the root's
// moves i (the searching side's) and each one's replies j (the other side's)
// form a list of (i, j) pairs; lane k takes pairs k, k + 64, ... and values each
// with maximin_search's rules over the D - 2 levels below it (maximin_value).
// The reply level takes the minimum over j (the value, not the move, is what the
// root uses: ties at that level do not matter), the root the first maximum over
// i in ascending square order (np.argmax).  A root move whose child is a leaf --
// the board full, or the other side without a move -- is valued as the search
// values a leaf: the searching side's disc count.  Results are identical to
// maximin_search (tested); the wave runs the slowest of its lanes' subtrees, and
// the subtrees of one board are alike in depth, where one lane per board makes
// the wave wait for its deepest board's whole tree.
#pragma once

#include "device.hpp"

#ifndef OTH_MM_NESTED_MAX_E
// launches of at most this many boards at depth >= 4 take the nested subtrees
// (maximin_node: 342 VGPRs, one wave per SIMD); larger launches and depth 3 the
// explicit stack (maximin_value), whose lower register count keeps more boards'
// waves resident.  8x8, nested against the explicit stack: depth 4 at 1,024 /
// 4,096 / 16,384 / 65,536 boards 189 / 434 / 1,363 / 4,951 us against 252 / 515 /
// 1,347 / 4,570; depth 5 at 256 / 4,096 boards 2.51 / 7.17 ms against 3.52 / 8.51;
// one board at depth 6 36.1 against 48.8 ms (profiles/r05/i, profiles/r05/j)
#define OTH_MM_NESTED_MAX_E 8192
#endif

namespace oth_dev {

// maximin_search's best VALUE at a node whose mover is the searching side (its
// level 0), D >= 1 levels below; L0 non-empty.  The same walk as maximin_search.
template <int N>
__device__ int maximin_value(const BB<Geo<N>::W>& P0, const BB<Geo<N>::W>& O0, const BB<Geo<N>::W>& L0, int D) {
    constexpr int W = Geo<N>::W;
    constexpr int MAXD = OTH_MAXIMIN_MAX_DEPTH;
    BB<W> SP[MAXD], SO[MAXD], SR[MAXD];
    int SV[MAXD];
    int l = 0;
    SP[0] = P0;
    SO[0] = O0;
    SR[0] = L0;
    SV[0] = -1;
    for (;;) {
        if (!any(SR[l])) {
            if (l == 0) break;
            const int v = SV[l];
            --l;
            if ((l & 1) == 0 ? v > SV[l] : v < SV[l]) SV[l] = v;
            continue;
        }
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
        const BB<W> P = SP[l], O = SO[l];
        const BB<W> f = flips<N>(P, O, m);
        const BB<W> P2 = P | f | m;
        const BB<W> O2 = O & ~(f | m);
        const bool mine = (l & 1) == 0;
        int v = popcount(mine ? P2 : O2);
        bool leaf = true;
        if (l + 1 < D && any(~(P2 | O2) & Geo<N>::BOARD)) {
            BB<W> t2[8];
            const BB<W> L2 = legal_moves_fills<N>(O2, P2, t2);
            if (any(L2)) {
                if (l + 2 == D) {
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
        if (leaf && (mine ? v > SV[l] : v < SV[l])) SV[l] = v;
    }
    return SV[0];
}

// maximin_value for a subtree depth known only at run time: boards of up to two
// words take maximin_node's compile-time recursion (each level's state in
// registers) for depths 2..8, instead of maximin_value's explicit stack, whose
// dynamically indexed levels live in scratch memory
static_assert(OTH_MAXIMIN_MAX_DEPTH - 2 <= 8, "subtree_value's compile-time depths");
template <int N, bool NESTED>
__device__ __forceinline__ int subtree_value(const BB<Geo<N>::W>& P, const BB<Geo<N>::W>& O,
                                             const BB<Geo<N>::W>& L, int D) {
    if constexpr (NESTED && Geo<N>::W <= 2) {
        int unused;
        switch (D) {
            case 2: return maximin_node<N, 2, 0>(P, O, L, unused);  // (D >= 2: depth 3 ends at the planes)
            case 3: return maximin_node<N, 3, 0>(P, O, L, unused);
            case 4: return maximin_node<N, 4, 0>(P, O, L, unused);
            case 5: return maximin_node<N, 5, 0>(P, O, L, unused);
            case 6: return maximin_node<N, 6, 0>(P, O, L, unused);
            case 7: return maximin_node<N, 7, 0>(P, O, L, unused);
            default: return maximin_node<N, 8, 0>(P, O, L, unused);  // (D <= OTH_MAXIMIN_MAX_DEPTH - 2 = 8)
        }
    } else {
        return maximin_value<N>(P, O, L, D);
    }
}

// the k-th (0-based, ascending) set square of a multi-word mask
template <int W>
__device__ __forceinline__ BB<W> kth_square(const BB<W>& x, int k) {
    BB<W> m = zero<W>();
#pragma unroll
    for (int i = 0; i < W; ++i) {
        const int c = popc64(x.w[i]);
        if (k >= 0 && k < c) m.w[i] = 1ull << select64(x.w[i], k);
        k -= c;
    }
    return m;
}
template <int W>
__device__ __forceinline__ int square_of(const BB<W>& m) {
    int b = -1;
#pragma unroll
    for (int i = W - 1; i >= 0; --i)
        if (m.w[i]) b = 64 * i + ctz64(m.w[i]);
    return b;
}

constexpr int MW_MAX_ROOT = 64;  // root moves held per board (more: one lane searches alone)

// One board per wave (block = one wave), depth D >= 3.
template <int N, bool NESTED>
__global__ __launch_bounds__(64) void k_maximin_wave(const uint64_t* __restrict__ boards,
                                                     const uint16_t* __restrict__ meta,
                                                     const uint64_t* __restrict__ legal, int E,
                                                     int32_t* __restrict__ out, int D) {
    constexpr int W = Geo<N>::W;
    __shared__ BB<W> cP[MW_MAX_ROOT], cO[MW_MAX_ROOT], cL[MW_MAX_ROOT];  // each root child: (mine, theirs, replies)
    __shared__ int first[MW_MAX_ROOT + 1];  // prefix counts of the replies
    __shared__ int leafv[MW_MAX_ROOT], minv[MW_MAX_ROOT], sq[MW_MAX_ROOT];
    const int e = blockIdx.x;
    const int lane = threadIdx.x;
    if (e >= E) return;  // (block-uniform)
    Lane<N> s;
    load_lane<N>(s, boards, meta, legal, e);
    const bool tw = (s.meta & M_TURN_WHITE) != 0;
    const BB<W> P = pick(tw, s.white, s.black), O = pick(tw, s.black, s.white);
    const int n0 = popcount(s.legal);
    if (n0 == 0) {
        if (lane == 0) out[e] = -1;  // the reference's None
        return;
    }
    if (n0 > MW_MAX_ROOT) {  // (no position of N <= 16 found with this many moves; kept exact anyway)
        if (lane == 0) out[e] = maximin_search<N>(P, O, s.legal, D);
        return;
    }
    // the root's children, one lane each
    if (lane < n0) {
        const BB<W> m = kth_square<W>(s.legal, lane);
        const BB<W> f = flips<N>(P, O, m);
        const BB<W> P2 = P | f | m, O2 = O & ~(f | m);
        int nrep = 0;
        BB<W> L2 = zero<W>();
        if (any(~(P2 | O2) & Geo<N>::BOARD)) {  // (1 < D always here)
            L2 = legal_moves<N>(O2, P2);
            nrep = popcount(L2);
        }
        cP[lane] = P2;
        cO[lane] = O2;
        cL[lane] = L2;
        leafv[lane] = popcount(P2);  // a leaf child: my disc count (:117-126)
        minv[lane] = 0x7fffffff;
        sq[lane] = square_of<W>(m);
        first[lane + 1] = nrep;
    }
    __syncthreads();
    if (lane == 0) {
        first[0] = 0;
        for (int i = 0; i < n0; ++i) first[i + 1] += first[i];
    }
    __syncthreads();
    const int total = first[n0];
    for (int p = lane; p < total; p += 64) {
        int i = 0;
        while (first[i + 1] <= p) ++i;
        const int j = p - first[i];
        // level 1: the other side (cO) plays its j-th reply
        const BB<W> Pm = cP[i], Po = cO[i];
        const BB<W> m = kth_square<W>(cL[i], j);
        const BB<W> f = flips<N>(Po, Pm, m);
        const BB<W> Q = Po | f | m;      // theirs after the reply
        const BB<W> R = Pm & ~(f | m);   // mine
        int v = popcount(R);             // a leaf at level 1: my disc count
        if (2 < D && any(~(Q | R) & Geo<N>::BOARD)) {
            BB<W> t3[8];
            const BB<W> L3 = legal_moves_fills<N>(R, Q, t3);
            if (any(L3)) {
                if (D == 3) v = popcount(R) + 1 + PlanesW<N>::max_flips(t3, L3);  // maximin_search's last level
                else v = subtree_value<N, NESTED>(R, Q, L3, D - 2);
            }
        }
        atomicMin(&minv[i], v);
    }
    __syncthreads();
    if (lane == 0) {  // np.argmax over the root's moves in ascending order: the first maximum
        int best = -1, move = -1;
        for (int i = 0; i < n0; ++i) {
            const int v = first[i + 1] > first[i] ? minv[i] : leafv[i];
            if (v > best) {
                best = v;
                move = sq[i];
            }
        }
        out[e] = move;
    }
}

}  // namespace oth_dev
