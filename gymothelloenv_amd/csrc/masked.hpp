// masked.hpp -- the masked categorical's device code,
// shared by k_masked (masked.hip) and the fused sample-and-step kernel
// (device.hpp k_sample_step): both run exactly these instructions per board,
// so the fused path's samples, log-probs and entropies are bit-identical to
// oth_sample_actions followed by oth_step.
//
// Replaces the per-sample Python loops of
//   model.py:60-99    Policy.act: FixedCategorical(logits=x[i][possible_moves[i]])
//                     .sample() / .mode(), action = possible_moves[i][idx],
//                     log_prob; no legal move -> action 0, log_prob 0 (:69-71)
//   model.py:156-178  Policy.evaluate_actions: log_prob of the stored action
//                     among the stored choices; 0 if none or not a choice (:165)
//   ppo.py:228-298    PPO.get_action / get_test_action: softmax restricted to
//                     possible_moves, renormalised, np.random.choice
// Floating point (fp32), so parity is to the reference's fixtures and a numpy
// fp64 restatement within tolerance (tests/test_gpu_masked.py).
//
// Layout: G lanes per board (MS_G = 4 up to two 64-square chunks, 16
// beyond); lane l holds blocks of 4 squares 4G*bi + 4l .. +3 (dwordx4 loads
// when the rows are 16-byte aligned: each load instruction covers 16G
// contiguous bytes of a board), with the legal bits of the same squares, and
// every cross-lane step is a DPP quad_perm / row op inside the group (no LDS,
// no barriers).  Per square: select, max, exp, add, fma, cdf add, compare;
// the per-board work (Philox, reductions, stores) is shared by G lanes.
#pragma once
#include <hip/hip_runtime.h>
#include <float.h>
#include <math.h>

#include "bitboard.hpp"
#include "othello_mi355x.h"

namespace oth_ms {

constexpr int MS_G = 4;    // lanes per board up to 128 squares (16 beyond)
constexpr int MS_BPR = 1;  // boards per lane group of one-chunk boards (loads of all of them issued first)

constexpr int MS_BLOCK = 256;
constexpr uint32_t RNG_SAMPLE = 3;  // Philox purpose word of the sampler's uniforms
constexpr int NONE = 0x7fffffff;

typedef float f32x4 __attribute__((ext_vector_type(4)));

template <int CTRL>
__device__ __forceinline__ float dpp(float x) {
    return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(x), CTRL, 0xF, 0xF, false));
}
template <int CTRL>
__device__ __forceinline__ int dpp(int x) {
    return __builtin_amdgcn_update_dpp(0, x, CTRL, 0xF, 0xF, false);
}

// Cross-lane steps over a group of G lanes (4, 8 or 16 lanes of one DPP row).
// All-reduce: quad_perm [1,0,3,2], [2,3,0,1], then row_half_mirror, row_mirror.
template <int G>
struct Grp {
    static_assert(G == 4 || G == 8 || G == 16, "groups of 4, 8 or 16 lanes");
    template <typename T, typename Op>
    __device__ __forceinline__ static T reduce(T v, Op op) {
        v = op(v, dpp<0xB1>(v));
        v = op(v, dpp<0x4E>(v));
        if constexpr (G >= 8) v = op(v, dpp<0x141>(v));
        if constexpr (G == 16) v = op(v, dpp<0x140>(v));
        return v;
    }
    __device__ __forceinline__ static float max(float v) {
        return reduce(v, [](float a, float b) { return fmaxf(a, b); });
    }
    __device__ __forceinline__ static float sum(float v) {
        return reduce(v, [](float a, float b) { return a + b; });
    }
    __device__ __forceinline__ static int min(int v) {
        return reduce(v, [](int a, int b) { return ::min(a, b); });
    }
    __device__ __forceinline__ static int max(int v) {
        return reduce(v, [](int a, int b) { return ::max(a, b); });
    }
    // Exclusive prefix sum over the group's lanes (lane l gets lanes 0..l-1):
    // row_shr 1, 2, 4, 8 within the row.  A lane whose shifted-in value comes
    // from below its group drops it with an AND mask, not a select: a select
    // lets the compiler move the DPP read under an exec mask, and DPP then
    // reads the disabled source lanes as 0.
    __device__ __forceinline__ static float excl_scan(float v, int l) {
        v += masked(dpp<0x111>(v), l >= 1);
        v += masked(dpp<0x112>(v), l >= 2);
        if constexpr (G >= 8) v += masked(dpp<0x114>(v), l >= 4);
        if constexpr (G == 16) v += dpp<0x118>(v);  // lanes 0..7 of the row read 0
        return masked(dpp<0x111>(v), l >= 1);
    }
    __device__ __forceinline__ static float masked(float v, bool keep) {
        return __uint_as_float(__float_as_uint(v) & (keep ? ~0u : 0u));
    }
};

// One board as seen by one lane of its group: NB = CH * 16/G blocks of 4
// squares; block bi of lane l is squares 4G*bi + 4l .. 4G*bi + 4l + 3, so a
// dwordx4 load instruction covers 16G contiguous bytes of every board.
template <int CH, int G>
struct Slot {
    static constexpr int NB = CH * (16 / G);
    int e;
    bool live;
    uint64_t words[CH];  // the board's legal words
    uint32_t nib[NB];    // legal bits of the lane's blocks (squares past N*N cleared)
    float x[NB][4];
};

template <int CH, int G, bool VEC>
__device__ __forceinline__ void load_slot(Slot<CH, G>& b, int l, int NN, const float* __restrict__ logits,
                                          long long ld, const uint64_t* __restrict__ legal) {
    constexpr int NB = Slot<CH, G>::NB;
    const float* row = logits + (size_t)b.e * (size_t)ld;
#pragma unroll
    for (int c = 0; c < CH; ++c) b.words[c] = legal[(size_t)b.e * CH + c];
#pragma unroll
    for (int bi = 0; bi < NB; ++bi) {
        const int sq = 4 * G * bi + 4 * l;
        const int rem = NN - sq;  // squares of this block inside the board
        const uint32_t inside = rem >= 4 ? 0xFu : (rem > 0 ? (1u << rem) - 1u : 0u);
        b.nib[bi] = (uint32_t)(b.words[sq >> 6] >> (sq & 63)) & inside;
        if constexpr (VEC) {  // N*N % 4 == 0: a block is all inside or all outside
            f32x4 v = {0.f, 0.f, 0.f, 0.f};
            if (sq < NN) v = *reinterpret_cast<const f32x4*>(row + sq);
            b.x[bi][0] = v.x;
            b.x[bi][1] = v.y;
            b.x[bi][2] = v.z;
            b.x[bi][3] = v.w;
        } else {
#pragma unroll
            for (int j = 0; j < 4; ++j) b.x[bi][j] = sq + j < NN ? row[sq + j] : 0.f;
        }
    }
}

// x where the square is legal (bit j of the block's nibble), -inf elsewhere:
// a sign-extended bitfield (v_bfe_i32) and a bitfield select (v_bfi_b32).
__device__ __forceinline__ float legal_or_ninf(uint32_t nib, int j, float x) {
    const uint32_t mk = (uint32_t)__builtin_amdgcn_sbfe((int)nib, j, 1);  // all ones when legal
    return __uint_as_float((mk & __float_as_uint(x)) | (~mk & 0xff800000u));
}
// Maxima on raw v_max3_f32 / v_max_f32: fmaxf of a value the compiler cannot
// prove canonical (a loaded logit, a bitfield select) costs a quieting
// v_max_f32 x, x per operand in IEEE mode; logits are never signalling NaNs.
__device__ __forceinline__ float vmax3(float a, float b, float c) {
    float r;
    asm("v_max3_f32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
    return r;
}
__device__ __forceinline__ float vmax2(float a, float b) {
    float r;
    asm("v_max_f32 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
    return r;
}
// max of v[0..K) (exact in any order): a tree of three-input maxima
template <int K>
__device__ __forceinline__ float max_reduce(float* v) {
#pragma unroll
    for (int w = K; w > 1; w = (w + 2) / 3) {
#pragma unroll
        for (int i = 0; 3 * i < w; ++i) {
            const int k = 3 * i;
            v[i] = k + 2 < w ? vmax3(v[k], v[k + 1], v[k + 2]) : (k + 1 < w ? vmax2(v[k], v[k + 1]) : v[k]);
        }
    }
    return v[0];
}

// exp(x - max).  (Folding the shift into fma(x, log2 e, -max log2 e) saves an
// instruction but leaves exp(0) for the largest logit off 1 by the rounding
// of max * log2 e, so a lone legal move got a log-prob of +1e-7: not used.)
__device__ __forceinline__ float exp_shifted(float x, float max_shift) { return __expf(x - max_shift); }

// The group's result for one board (every lane of the group holds it).
struct Pick {
    int a;      // sampled / mode / given action
    float lp;   // log-prob of a among the legal squares (0 if a is not one)
    float ent;  // entropy (masked, or unmasked with FULL)
};

// a_in: the evaluated action (OTH_MASKED_EVAL); want_lp: compute the log-prob
// (one extra logits read); want_ent: compute the (masked) entropy.
template <int CH, int G, bool FULL>
__device__ __forceinline__ Pick finish_slot(Slot<CH, G>& b, int l, int NN, const float* __restrict__ logits,
                                            long long ld, const float* __restrict__ uniforms, uint64_t seed,
                                            uint32_t id_base, uint64_t counter, int mode, int a_in, bool want_lp,
                                            bool want_ent) {
    constexpr int NB = Slot<CH, G>::NB;
    const int e = b.e;
    // OTH_MASKED_FULL_ENTROPY: entropy of the unmasked categorical over all N*N
    // squares (Policy.evaluate_actions' dist.entropy(), model.py:175)
    float full_ent = 0.f;
    if constexpr (FULL) {
        float fm = -INFINITY;
#pragma unroll
        for (int bi = 0; bi < NB; ++bi)
#pragma unroll
            for (int j = 0; j < 4; ++j)
                if (4 * G * bi + 4 * l + j < NN) fm = fmaxf(fm, b.x[bi][j]);
        fm = Grp<G>::max(fm);
        float fs = 0.f, fsx = 0.f;
#pragma unroll
        for (int bi = 0; bi < NB; ++bi)
#pragma unroll
            for (int j = 0; j < 4; ++j)
                if (4 * G * bi + 4 * l + j < NN) {
                    const float d = b.x[bi][j] - fm;
                    const float q = __expf(d);
                    fs += q;
                    fsx = fmaf(q, d, fsx);
                }
        fs = Grp<G>::sum(fs);
        fsx = Grp<G>::sum(fsx);
        full_ent = __logf(fs) - fsx / fs;
    }
    // illegal squares -> -inf: they drop out of the max and get p = exp(-inf) = 0
    float mb[NB * 4];
#pragma unroll
    for (int bi = 0; bi < NB; ++bi)
#pragma unroll
        for (int j = 0; j < 4; ++j) mb[4 * bi + j] = b.x[bi][j] = legal_or_ninf(b.nib[bi], j, b.x[bi][j]);
    float m = Grp<G>::max(max_reduce<NB * 4>(mb));
    const bool any = m != -INFINITY;
    const float ms = any ? m : 0.f;
    // p = exp(x - max); tot = sum p; SX = sum p (x - max) (illegal: 0 * -FLT_MAX = 0)
    float p[NB][4], loc[NB];
    float s = 0.f, sx = 0.f;
#pragma unroll
    for (int bi = 0; bi < NB; ++bi) {
        loc[bi] = 0.f;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            p[bi][j] = exp_shifted(b.x[bi][j], ms);
            loc[bi] += p[bi][j];
        }
        s += loc[bi];
    }
    if (want_ent) {
#pragma unroll
        for (int bi = 0; bi < NB; ++bi)
#pragma unroll
            for (int j = 0; j < 4; ++j) sx = fmaf(p[bi][j], vmax2(b.x[bi][j] - ms, -FLT_MAX), sx);
    }
    const float tot = Grp<G>::sum(s);
    const float SX = want_ent ? Grp<G>::sum(sx) : 0.f;
    const float logS = __logf(tot);

    int a;
    if (mode == OTH_MASKED_EVAL) {
        a = a_in;
    } else {
        int cand = NONE;
        if (mode == OTH_MASKED_MODE) {  // Categorical.mode: first (lowest) square of the largest logit
#pragma unroll
            for (int bi = NB - 1; bi >= 0; --bi)
#pragma unroll
                for (int j = 3; j >= 0; --j)
                    if (b.x[bi][j] == m) cand = 4 * G * bi + 4 * l + j;
        } else {  // sample: first legal square whose cumulative mass exceeds u * total (np.random.choice)
            float u;
            if (uniforms) {
                u = uniforms[e];
            } else {
                u = (float)(oth::philox_x(seed, id_base + (uint32_t)e, counter, RNG_SAMPLE) >> 8) * 0x1p-24f;
            }
            const float target = u * tot;
            float carry = 0.f;  // mass of the blocks before bi (all lanes)
#pragma unroll
            for (int bi = 0; bi < NB; ++bi) {
                float cdf = carry + Grp<G>::excl_scan(loc[bi], l);
                // squares of the block with cdf <= target form a prefix (cdf is monotone in the block)
                uint32_t below = 0;
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    cdf += p[bi][j];
                    below += cdf <= target ? 1u : 0u;
                }
                const uint32_t hit = b.nib[bi] & (0xFu << below);
                if (cand == NONE && hit) cand = 4 * G * bi + 4 * l + __builtin_ctz(hit);
                if (bi + 1 < NB) carry += Grp<G>::sum(loc[bi]);
            }
        }
        cand = Grp<G>::min(cand);
        if (cand == NONE && any) {  // u * total rounded up to the total: the last legal square
            int last = -1;
#pragma unroll
            for (int bi = 0; bi < NB; ++bi)
                if (b.nib[bi]) last = 4 * G * bi + 4 * l + 31 - __builtin_clz(b.nib[bi]);
            cand = Grp<G>::max(last);
        }
        a = any ? cand : 0;  // model.py:69-71: no legal move -> action 0
    }
    Pick out;
    out.a = a;
    bool choice = false;
#pragma unroll
    for (int c = 0; c < CH; ++c)
        if (a >= 64 * c && a < 64 * c + 64 && a < NN) choice = (b.words[c] >> (a - 64 * c)) & 1ull;
    out.lp = (choice && want_lp) ? logits[(size_t)e * (size_t)ld + a] - m - logS : 0.f;
    out.ent = FULL ? full_ent : ((any && want_ent) ? logS - SX / tot : 0.f);
    return out;
}

// The same arithmetic for ONE board computed by ONE lane: the G lanes of
// finish_slot become an index l, and every cross-lane step is restated in
// the order the DPP steps combine values -- the group sum as the butterfly
// tree (v0+v1)+(v2+v3) (per quad, then quads the same way for G = 16), the
// exclusive scan as its row_shr 1, 2 (, 4, 8) steps -- so the result is
// bit-identical to finish_slot's (tests/test_gpu_masked.py checks it through
// oth_sample_step).  One lane per board keeps 64 boards in a wave, so the
// instruction count per board is a quarter of the grouped form's when one
// wave per SIMD does the sampling (the fused sample-and-step kernel).
template <int G>
__device__ __forceinline__ float tree_sum(const float* v) {
    float q[G / 4];
#pragma unroll
    for (int k = 0; k < G / 4; ++k) q[k] = (v[4 * k] + v[4 * k + 1]) + (v[4 * k + 2] + v[4 * k + 3]);
    if constexpr (G == 4) return q[0];
    else return (q[0] + q[1]) + (q[2] + q[3]);
}

template <int G>
__device__ __forceinline__ void excl_scan_lanes(const float* a, float* r) {
    float v[G];
#pragma unroll
    for (int l = 0; l < G; ++l) v[l] = a[l];
#pragma unroll
    for (int d = 1; d < G; d *= 2) {  // row_shr d: lane l adds lane l-d's value from before the step
        float w[G];
#pragma unroll
        for (int l = 0; l < G; ++l) w[l] = l >= d ? v[l] + v[l - d] : v[l];
#pragma unroll
        for (int l = 0; l < G; ++l) v[l] = w[l];
    }
    r[0] = 0.f;
#pragma unroll
    for (int l = 1; l < G; ++l) r[l] = v[l - 1];
}

template <int CH, int G, bool VEC, bool FULL>
__device__ __forceinline__ Pick sample_lane(int e, int NN, const float* __restrict__ logits, long long ld,
                                            const uint64_t* __restrict__ legal, const float* __restrict__ uniforms,
                                            uint64_t seed, uint32_t id_base, uint64_t counter, int mode, int a_in,
                                            bool want_lp, bool want_ent) {
    constexpr int NB = CH * (16 / G);
    const float* row = logits + (size_t)e * (size_t)ld;
    uint64_t words[CH];
#pragma unroll
    for (int c = 0; c < CH; ++c) words[c] = legal[(size_t)e * CH + c];
    float x[G][NB][4];
    uint32_t nib[G][NB];
#pragma unroll
    for (int bi = 0; bi < NB; ++bi)
#pragma unroll
        for (int l = 0; l < G; ++l) {
            const int sq = 4 * G * bi + 4 * l;
            const int rem = NN - sq;
            const uint32_t inside = rem >= 4 ? 0xFu : (rem > 0 ? (1u << rem) - 1u : 0u);
            nib[l][bi] = (uint32_t)(words[sq >> 6] >> (sq & 63)) & inside;
            if constexpr (VEC) {
                f32x4 v = {0.f, 0.f, 0.f, 0.f};
                if (sq < NN) v = *reinterpret_cast<const f32x4*>(row + sq);
                x[l][bi][0] = v.x;
                x[l][bi][1] = v.y;
                x[l][bi][2] = v.z;
                x[l][bi][3] = v.w;
            } else {
#pragma unroll
                for (int j = 0; j < 4; ++j) x[l][bi][j] = sq + j < NN ? row[sq + j] : 0.f;
            }
        }
    float full_ent = 0.f;
    if constexpr (FULL) {
        float fm = -INFINITY;
#pragma unroll
        for (int l = 0; l < G; ++l)
#pragma unroll
            for (int bi = 0; bi < NB; ++bi)
#pragma unroll
                for (int j = 0; j < 4; ++j)
                    if (4 * G * bi + 4 * l + j < NN) fm = fmaxf(fm, x[l][bi][j]);
        float fs[G], fsx[G];
#pragma unroll
        for (int l = 0; l < G; ++l) {
            fs[l] = 0.f;
            fsx[l] = 0.f;
#pragma unroll
            for (int bi = 0; bi < NB; ++bi)
#pragma unroll
                for (int j = 0; j < 4; ++j)
                    if (4 * G * bi + 4 * l + j < NN) {
                        const float d = x[l][bi][j] - fm;
                        const float q = __expf(d);
                        fs[l] += q;
                        fsx[l] = fmaf(q, d, fsx[l]);
                    }
        }
        const float FS = tree_sum<G>(fs), FSX = tree_sum<G>(fsx);
        full_ent = __logf(FS) - FSX / FS;
    }
    float ml[G * NB * 4];  // a shallow tree instead of one long max chain (the max is exact)
#pragma unroll
    for (int l = 0; l < G; ++l)
#pragma unroll
        for (int bi = 0; bi < NB; ++bi)
#pragma unroll
            for (int j = 0; j < 4; ++j)
                ml[(l * NB + bi) * 4 + j] = x[l][bi][j] = legal_or_ninf(nib[l][bi], j, x[l][bi][j]);
    const float m = max_reduce<G * NB * 4>(ml);
    const bool any = m != -INFINITY;
    const float ms = any ? m : 0.f;
    float p[G][NB][4], loc[G][NB], s[G], sx[G];
#pragma unroll
    for (int l = 0; l < G; ++l) {
        s[l] = 0.f;
        sx[l] = 0.f;
#pragma unroll
        for (int bi = 0; bi < NB; ++bi) {
            loc[l][bi] = 0.f;
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                p[l][bi][j] = exp_shifted(x[l][bi][j], ms);
                loc[l][bi] += p[l][bi][j];
            }
            s[l] += loc[l][bi];
        }
    }
    if (want_ent) {
#pragma unroll
        for (int l = 0; l < G; ++l)
#pragma unroll
            for (int bi = 0; bi < NB; ++bi)
#pragma unroll
                for (int j = 0; j < 4; ++j) sx[l] = fmaf(p[l][bi][j], vmax2(x[l][bi][j] - ms, -FLT_MAX), sx[l]);
    }
    const float tot = tree_sum<G>(s);
    const float SX = want_ent ? tree_sum<G>(sx) : 0.f;
    const float logS = __logf(tot);
    int a;
    if (mode == OTH_MASKED_EVAL) {
        a = a_in;
    } else {
        int cand = NONE;
        if (mode == OTH_MASKED_MODE) {  // the lowest square of the largest legal logit
#pragma unroll
            for (int bi = NB - 1; bi >= 0; --bi)
#pragma unroll
                for (int l = G - 1; l >= 0; --l)
#pragma unroll
                    for (int j = 3; j >= 0; --j)
                        if (x[l][bi][j] == m) cand = 4 * G * bi + 4 * l + j;
        } else {
            float u;
            if (uniforms) u = uniforms[e];
            else u = (float)(oth::philox_x(seed, id_base + (uint32_t)e, counter, RNG_SAMPLE) >> 8) * 0x1p-24f;
            const float target = u * tot;
            float carry = 0.f;
            int cl[G];
#pragma unroll
            for (int l = 0; l < G; ++l) cl[l] = NONE;
#pragma unroll
            for (int bi = 0; bi < NB; ++bi) {
                float lb[G], scan[G];
#pragma unroll
                for (int l = 0; l < G; ++l) lb[l] = loc[l][bi];
                excl_scan_lanes<G>(lb, scan);
#pragma unroll
                for (int l = 0; l < G; ++l) {
                    float cdf = carry + scan[l];
                    uint32_t below = 0;
#pragma unroll
                    for (int j = 0; j < 4; ++j) {
                        cdf += p[l][bi][j];
                        below += cdf <= target ? 1u : 0u;
                    }
                    const uint32_t hit = nib[l][bi] & (0xFu << below);
                    if (cl[l] == NONE && hit) cl[l] = 4 * G * bi + 4 * l + __builtin_ctz(hit);
                }
                if (bi + 1 < NB) carry += tree_sum<G>(lb);
            }
#pragma unroll
            for (int l = 0; l < G; ++l) cand = ::min(cand, cl[l]);
        }
        if (cand == NONE && any) {  // u * total rounded up to the total: the last legal square
            int last = -1;
#pragma unroll
            for (int bi = 0; bi < NB; ++bi)
#pragma unroll
                for (int l = 0; l < G; ++l)
                    if (nib[l][bi]) last = ::max(last, 4 * G * bi + 4 * l + 31 - __builtin_clz(nib[l][bi]));
            cand = last;
        }
        a = any ? cand : 0;
    }
    Pick out;
    out.a = a;
    bool choice = false;
#pragma unroll
    for (int c = 0; c < CH; ++c)
        if (a >= 64 * c && a < 64 * c + 64 && a < NN) choice = (words[c] >> (a - 64 * c)) & 1ull;
    out.lp = (choice && want_lp) ? logits[(size_t)e * (size_t)ld + a] - m - logS : 0.f;
    out.ent = FULL ? full_ent : ((any && want_ent) ? logS - SX / tot : 0.f);
    return out;
}

// The same arithmetic for ONE board computed by a PAIR of lanes (lanes 2k,
// 2k+1; h = 0, 1): lane h restates the group's lanes 2h and 2h+1 of G = 4
// (one-word boards) and the pair exchanges partial results through DPP
// quad_perm [1,0,3,2].  Every combination is the one finish_slot's DPP steps
// make -- the sum (v0+v1)+(v2+v3) is lane 0's v0+v1 plus lane 1's v2+v3 (an
// IEEE add is commutative), the exclusive scan of a block is computed whole
// on both lanes from the four lane values -- so the pick is bit-identical to
// sample_lane's and k_masked's.  Both lanes return the same Pick.  The caller
// keeps every branch around the call pair-uniform (DPP reads the partner).
// The logits rows of a wave's 32 boards (8x8, 16 quads a row) staged through
// LDS for sample_pair: lane i loads quads i, i+64, ... of the 32 consecutive
// rows (each load instruction 1 KiB of consecutive rows when ld == 64), all
// eight loads issued before the first write; quad q = 4bi + 2h + k of row r
// goes to slot 18r + 9h + 2bi + k, so lane (r, h) reads its eight quads at
// 18r + 9h + 0..7 and the sixteen lanes of a ds_read_b128 phase hit sixteen
// distinct bank quads (2r + 9h mod 16).  load_pair_rows issues the loads,
// store_pair_rows writes them and returns the lane's eight quads.
constexpr int PAIR_ROW = 18;  // quads per staged row
__device__ __forceinline__ void load_pair_rows(f32x4 (&v)[8], long long e0, int E, const float* __restrict__ logits,
                                               long long ld, int lane) {
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        const int c = k * 64 + lane, r = c >> 4, q = c & 15;
        const long long row = e0 + r < E ? e0 + r : E - 1;  // clamped, not branched: the loads stay in flight together
        v[k] = *reinterpret_cast<const f32x4*>(logits + (size_t)row * (size_t)ld + 4 * q);
    }
}
__device__ __forceinline__ const f32x4* store_pair_rows(f32x4* ws, const f32x4 (&v)[8], int lane) {
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        const int c = k * 64 + lane, r = c >> 4, q = c & 15;
        ws[r * PAIR_ROW + ((q >> 1) & 1) * 9 + ((q >> 2) << 1) + (q & 1)] = v[k];
    }
    // a wave reads only what it wrote: LDS operations of one wave complete in order
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    return ws + (lane >> 1) * PAIR_ROW + (lane & 1) * 9;
}

__device__ __forceinline__ float pair_swapf(float x) { return dpp<0xB1>(x); }
__device__ __forceinline__ int pair_swapi(int x) { return dpp<0xB1>(x); }

template <int CH, bool VEC, bool FULL, bool STAGED = false>
__device__ __forceinline__ Pick sample_pair(int e, int h, int NN, const float* __restrict__ logits, long long ld,
                                            const uint64_t (&words)[CH], const float* __restrict__ uniforms,
                                            uint64_t seed, uint32_t id_base, uint64_t counter, int mode,
                                            bool want_lp, bool want_ent, const f32x4* staged = nullptr) {
    static_assert(CH <= 2, "k_masked's four lanes per board cover up to 128 squares");
    constexpr int G = 4, NB = 4 * CH, H = 2;  // the lane's group lanes l = 2h + k, k = 0, 1
    const float* row = logits + (size_t)e * (size_t)ld;
    float x[H][NB][4];
    uint32_t nib[H][NB];
#pragma unroll
    for (int bi = 0; bi < NB; ++bi)
#pragma unroll
        for (int k = 0; k < H; ++k) {
            const int sq = 4 * G * bi + 4 * (2 * h + k);
            const int rem = NN - sq;
            const uint32_t inside = rem >= 4 ? 0xFu : (rem > 0 ? (1u << rem) - 1u : 0u);
            nib[k][bi] = (uint32_t)(words[sq >> 6] >> (sq & 63)) & inside;
            if constexpr (VEC) {
                f32x4 v = {0.f, 0.f, 0.f, 0.f};
                if constexpr (STAGED) v = staged[2 * bi + k];  // (8x8: every block inside)
                else if (sq < NN) v = *reinterpret_cast<const f32x4*>(row + sq);
                x[k][bi][0] = v.x;
                x[k][bi][1] = v.y;
                x[k][bi][2] = v.z;
                x[k][bi][3] = v.w;
            } else {
#pragma unroll
                for (int j = 0; j < 4; ++j) x[k][bi][j] = sq + j < NN ? row[sq + j] : 0.f;
            }
        }
    float full_ent = 0.f;
    if constexpr (FULL) {
        float fm = -INFINITY;
#pragma unroll
        for (int k = 0; k < H; ++k)
#pragma unroll
            for (int bi = 0; bi < NB; ++bi)
#pragma unroll
                for (int j = 0; j < 4; ++j)
                    if (4 * G * bi + 4 * (2 * h + k) + j < NN) fm = fmaxf(fm, x[k][bi][j]);
        fm = fmaxf(fm, pair_swapf(fm));
        float fs[H], fsx[H];
#pragma unroll
        for (int k = 0; k < H; ++k) {
            fs[k] = 0.f;
            fsx[k] = 0.f;
#pragma unroll
            for (int bi = 0; bi < NB; ++bi)
#pragma unroll
                for (int j = 0; j < 4; ++j)
                    if (4 * G * bi + 4 * (2 * h + k) + j < NN) {
                        const float d = x[k][bi][j] - fm;
                        const float q = __expf(d);
                        fs[k] += q;
                        fsx[k] = fmaf(q, d, fsx[k]);
                    }
        }
        const float qs = fs[0] + fs[1], qx = fsx[0] + fsx[1];
        const float FS = qs + pair_swapf(qs), FSX = qx + pair_swapf(qx);
        full_ent = __logf(FS) - FSX / FS;
    }
    float ml[H * NB * 4];
#pragma unroll
    for (int k = 0; k < H; ++k)
#pragma unroll
        for (int bi = 0; bi < NB; ++bi)
#pragma unroll
            for (int j = 0; j < 4; ++j) ml[(k * NB + bi) * 4 + j] = x[k][bi][j] = legal_or_ninf(nib[k][bi], j, x[k][bi][j]);
    float m = max_reduce<H * NB * 4>(ml);
    m = vmax2(m, pair_swapf(m));
    const bool any = m != -INFINITY;
    const float ms = any ? m : 0.f;
    float p[H][NB][4], loc[H][NB], sl[H], sx[H];
#pragma unroll
    for (int k = 0; k < H; ++k) {
        sl[k] = 0.f;
        sx[k] = 0.f;
#pragma unroll
        for (int bi = 0; bi < NB; ++bi) {
            loc[k][bi] = 0.f;
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                p[k][bi][j] = exp_shifted(x[k][bi][j], ms);
                loc[k][bi] += p[k][bi][j];
            }
            sl[k] += loc[k][bi];
        }
    }
    if (want_ent) {
#pragma unroll
        for (int k = 0; k < H; ++k)
#pragma unroll
            for (int bi = 0; bi < NB; ++bi)
#pragma unroll
                for (int j = 0; j < 4; ++j) sx[k] = fmaf(p[k][bi][j], vmax2(x[k][bi][j] - ms, -FLT_MAX), sx[k]);
    }
    const float q = sl[0] + sl[1];
    const float tot = q + pair_swapf(q);
    float SX = 0.f;
    if (want_ent) {
        const float qx = sx[0] + sx[1];
        SX = qx + pair_swapf(qx);
    }
    const float logS = __logf(tot);
    int a;
    if (mode == OTH_MASKED_EVAL) {
        a = 0;
    } else {
        int cand = NONE;
        if (mode == OTH_MASKED_MODE) {  // the lowest square of the largest legal logit
#pragma unroll
            for (int bi = NB - 1; bi >= 0; --bi)
#pragma unroll
                for (int k = H - 1; k >= 0; --k)
#pragma unroll
                    for (int j = 3; j >= 0; --j)
                        if (x[k][bi][j] == m) cand = 4 * G * bi + 4 * (2 * h + k) + j;
        } else {
            float u;
            if (uniforms) u = uniforms[e];
            else u = (float)(oth::philox_x(seed, id_base + (uint32_t)e, counter, RNG_SAMPLE) >> 8) * 0x1p-24f;
            const float target = u * tot;
            float carry = 0.f;
            int cl[H] = {NONE, NONE};
#pragma unroll
            for (int bi = 0; bi < NB; ++bi) {
                const float o0 = pair_swapf(loc[0][bi]), o1 = pair_swapf(loc[1][bi]);
                float v[G], scan[G];
                v[0] = h ? o0 : loc[0][bi];
                v[1] = h ? o1 : loc[1][bi];
                v[2] = h ? loc[0][bi] : o0;
                v[3] = h ? loc[1][bi] : o1;
                excl_scan_lanes<G>(v, scan);
#pragma unroll
                for (int k = 0; k < H; ++k) {
                    float cdf = carry + (h ? scan[2 + k] : scan[k]);
                    uint32_t below = 0;
#pragma unroll
                    for (int j = 0; j < 4; ++j) {
                        cdf += p[k][bi][j];
                        below += cdf <= target ? 1u : 0u;
                    }
                    const uint32_t hit = nib[k][bi] & (0xFu << below);
                    if (cl[k] == NONE && hit) cl[k] = 4 * G * bi + 4 * (2 * h + k) + __builtin_ctz(hit);
                }
                if (bi + 1 < NB) carry += tree_sum<G>(v);
            }
            cand = ::min(cl[0], cl[1]);
        }
        cand = ::min(cand, pair_swapi(cand));
        if (cand == NONE && any) {  // u * total rounded up to the total: the last legal square
            int last = -1;
#pragma unroll
            for (int bi = 0; bi < NB; ++bi)
#pragma unroll
                for (int k = 0; k < H; ++k)
                    if (nib[k][bi]) last = ::max(last, 4 * G * bi + 4 * (2 * h + k) + 31 - __builtin_clz(nib[k][bi]));
            cand = ::max(last, pair_swapi(last));
        }
        a = any ? cand : 0;
    }
    Pick out;
    out.a = a;
    bool choice = false;
#pragma unroll
    for (int c = 0; c < CH; ++c)
        if (a >= 64 * c && a < 64 * c + 64 && a < NN) choice = (words[c] >> (a - 64 * c)) & 1ull;
    out.lp = (choice && want_lp) ? logits[(size_t)e * (size_t)ld + a] - m - logS : 0.f;
    out.ent = FULL ? full_ent : ((any && want_ent) ? logS - SX / tot : 0.f);
    return out;
}

}  // namespace oth_ms
