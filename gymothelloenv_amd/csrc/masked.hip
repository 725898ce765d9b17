// masked.hip -- masked categorical over each board's legal squares (SURVEY.md
// §8(f)#3): the policy-head side of the vector env.  Replaces the per-sample
// Python loops of
//   model.py:60-99    Policy.act: FixedCategorical(logits=x[i][possible_moves[i]])
//                     .sample() / .mode(), action = possible_moves[i][idx],
//                     log_prob; no legal move -> action 0, log_prob 0 (:69-71)
//   model.py:156-178  Policy.evaluate_actions: log_prob of the stored action
//                     among the stored choices; 0 if none or not a choice (:165)
//   ppo.py:228-298    PPO.get_action / get_test_action: softmax restricted to
//                     possible_moves, renormalised, np.random.choice
// with one launch over E boards.  Floating point (fp32), so parity is to a
// torch fp32 / numpy fp64 restatement within tolerance (tests/test_gpu_masked.py).
//
// Layout: G lanes per board (OTH_MS_G up to two 64-square chunks, 16
// beyond); lane l holds blocks of 4 squares 4G*bi + 4l .. +3 (dwordx4 loads
// when the rows are 16-byte aligned: each load instruction covers 16G
// contiguous bytes of a board), with the legal bits of the same squares, and
// every cross-lane step is a DPP quad_perm / row op inside the group (no LDS,
// no barriers).  Per square: select, max, exp, add, fma, cdf add, compare;
// the per-board work (Philox, reductions, stores) is shared by G lanes.
// HBM bound: 4 N^2 B of logits + 8W B of legal per board in, 12 B out.
#include <hip/hip_runtime.h>
#include <float.h>
#include <math.h>

#include "bitboard.hpp"
#include "launch.hpp"

#ifndef OTH_MS_BPR
#define OTH_MS_BPR 1  // boards per lane group, loads of all of them issued first
#endif
#ifndef OTH_MS_G
#define OTH_MS_G 4  // lanes per board up to 128 squares (16 beyond)
#endif
#ifndef OTH_MS_NT
#define OTH_MS_NT 0  // 1: non-temporal logits loads (measured -27 % bandwidth)
#endif

namespace {

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
            if (sq < NN) {
#if OTH_MS_NT
                v = __builtin_nontemporal_load(reinterpret_cast<const f32x4*>(row + sq));
#else
                v = *reinterpret_cast<const f32x4*>(row + sq);
#endif
            }
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

template <int CH, int G, bool FULL>
__device__ __forceinline__ void finish_slot(Slot<CH, G>& b, int l, int NN, const float* __restrict__ logits,
                                            long long ld, const float* __restrict__ uniforms, uint64_t seed,
                                            uint32_t id_base, uint64_t counter, int mode,
                                            int32_t* __restrict__ actions, float* __restrict__ log_probs,
                                            float* __restrict__ entropy) {
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
    float m = -INFINITY;
#pragma unroll
    for (int bi = 0; bi < NB; ++bi)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            b.x[bi][j] = ((b.nib[bi] >> j) & 1u) ? b.x[bi][j] : -INFINITY;
            m = fmaxf(m, b.x[bi][j]);
        }
    m = Grp<G>::max(m);
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
            const float d = b.x[bi][j] - ms;
            p[bi][j] = __expf(d);
            loc[bi] += p[bi][j];
            sx = fmaf(p[bi][j], fmaxf(d, -FLT_MAX), sx);
        }
        s += loc[bi];
    }
    const float tot = Grp<G>::sum(s);
    const float SX = Grp<G>::sum(sx);
    const float logS = __logf(tot);

    int a;
    if (mode == OTH_MASKED_EVAL) {
        a = actions[e];
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
    if (b.live && l == 0) {
        bool choice = false;
#pragma unroll
        for (int c = 0; c < CH; ++c)
            if (a >= 64 * c && a < 64 * c + 64 && a < NN) choice = (b.words[c] >> (a - 64 * c)) & 1ull;
        if (mode != OTH_MASKED_EVAL) actions[e] = a;
        if (log_probs) log_probs[e] = choice ? logits[(size_t)e * (size_t)ld + a] - m - logS : 0.f;
        if (entropy) entropy[e] = FULL ? full_ent : (any ? logS - SX / tot : 0.f);
    }
}

// BPR boards per lane group: group r of the grid owns boards r*BPR .. r*BPR + BPR - 1.
template <int CH, int G, bool VEC, int BPR, bool FULL>
__global__ __launch_bounds__(MS_BLOCK) void k_masked(int E, int NN, const float* __restrict__ logits, long long ld,
                                                     const uint64_t* __restrict__ legal,
                                                     const float* __restrict__ uniforms, uint64_t seed,
                                                     uint32_t id_base, uint64_t counter,
                                                     const uint64_t* __restrict__ counter_off, int mode,
                                                     int32_t* __restrict__ actions, float* __restrict__ log_probs,
                                                     float* __restrict__ entropy) {
    if (counter_off) counter += *counter_off;  // graph-region offset (oth_graph_end); 0 eagerly
    const long long t = (long long)blockIdx.x * MS_BLOCK + threadIdx.x;
    const int l = (int)(t % G);
    Slot<CH, G> b[BPR];
#pragma unroll
    for (int k = 0; k < BPR; ++k) {
        const long long e = (t / G) * BPR + k;
        b[k].live = e < E;
        b[k].e = b[k].live ? (int)e : E - 1;  // dead groups still take part in the DPP steps
        load_slot<CH, G, VEC>(b[k], l, NN, logits, ld, legal);
    }
#pragma unroll
    for (int k = 0; k < BPR; ++k)
        finish_slot<CH, G, FULL>(b[k], l, NN, logits, ld, uniforms, seed, id_base, counter, mode, actions, log_probs,
                           entropy);
}

template <int CH, int G, int BPR, bool FULL>
void launch_one(bool vec, int E, hipStream_t st, int NN, const float* logits, long long ld, const uint64_t* legal,
               const float* uniforms, uint64_t seed, uint32_t id_base, uint64_t counter, const uint64_t* counter_off,
               int mode, int32_t* actions, float* log_probs, float* entropy) {
    const long long groups = ((long long)E + BPR - 1) / BPR;
    const int grid = (int)((groups * G + MS_BLOCK - 1) / MS_BLOCK);
    if (vec)
        hipLaunchKernelGGL((k_masked<CH, G, true, BPR, FULL>), dim3(grid), dim3(MS_BLOCK), 0, st, E, NN, logits, ld,
                           legal, uniforms, seed, id_base, counter, counter_off, mode, actions, log_probs, entropy);
    else
        hipLaunchKernelGGL((k_masked<CH, G, false, BPR, FULL>), dim3(grid), dim3(MS_BLOCK), 0, st, E, NN, logits, ld,
                           legal, uniforms, seed, id_base, counter, counter_off, mode, actions, log_probs, entropy);
}

template <int CH, int G, int BPR>
void launch_ch(bool vec, int E, hipStream_t st, int NN, const float* logits, long long ld, const uint64_t* legal,
               const float* uniforms, uint64_t seed, uint32_t id_base, uint64_t counter, const uint64_t* counter_off,
               int mode, int32_t* actions, float* log_probs, float* entropy) {
    const int base = mode & 3;
    if (mode & OTH_MASKED_FULL_ENTROPY)
        launch_one<CH, G, BPR, true>(vec, E, st, NN, logits, ld, legal, uniforms, seed, id_base, counter, counter_off,
                                     base, actions, log_probs, entropy);
    else
        launch_one<CH, G, BPR, false>(vec, E, st, NN, logits, ld, legal, uniforms, seed, id_base, counter,
                                      counter_off, base, actions, log_probs, entropy);
}

}  // namespace

namespace oth_host {

int launch_masked(int n_board, int E, const float* logits, long long ld, const uint64_t* legal, const float* uniforms,
                  uint64_t seed, uint32_t id_base, uint64_t counter, const uint64_t* counter_off, int mode,
                  int32_t* actions, float* log_probs, float* entropy, hipStream_t st) {
    const int NN = n_board * n_board;
    const int CH = (NN + 63) / 64;
    const bool vec = (NN % 4 == 0) && (ld % 4 == 0) && (((uintptr_t)logits & 15u) == 0);
#define OTH_MS_ARGS \
    vec, E, st, NN, logits, ld, legal, uniforms, seed, id_base, counter, counter_off, mode, actions, log_probs, entropy
    switch (CH) {  // OTH_MS_G lanes per board up to 128 squares, 16 beyond (registers)
        case 1: launch_ch<1, OTH_MS_G, OTH_MS_BPR>(OTH_MS_ARGS); break;
        case 2: launch_ch<2, OTH_MS_G, 1>(OTH_MS_ARGS); break;
        case 3: launch_ch<3, 16, 1>(OTH_MS_ARGS); break;
        default: launch_ch<4, 16, 1>(OTH_MS_ARGS); break;
    }
#undef OTH_MS_ARGS
    return after_launch("oth_masked_sample");
}

}  // namespace oth_host
