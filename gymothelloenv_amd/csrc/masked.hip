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
// Layout: 16 lanes (one DPP row) per board, lane l holding squares
// 64c + 4l .. 64c + 4l + 3 of chunk c (c < W = ceil(N*N / 64)): one dwordx4
// load per chunk when the logits rows are 16-byte aligned, the square's legal
// bit is nibble l of legal word c, and every reduction / scan is 4 DPP steps
// inside the row (no LDS, no barriers).  HBM bound: 4 N^2 B of logits + 8W B
// of legal per board in, 12 B out.
#include <hip/hip_runtime.h>
#include <math.h>

#include "bitboard.hpp"
#include "launch.hpp"

namespace {

constexpr int MS_BLOCK = 256;
constexpr uint32_t RNG_SAMPLE = 3;  // Philox purpose word of the sampler's uniforms

template <int CTRL>
__device__ __forceinline__ float dppf(float x) {
    return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(x), CTRL, 0xF, 0xF, false));
}
template <int CTRL>
__device__ __forceinline__ int dppi(int x) {
    return __builtin_amdgcn_update_dpp(0, x, CTRL, 0xF, 0xF, false);
}
// all-reduce inside a 16-lane row: quad_perm [1,0,3,2], [2,3,0,1], row_half_mirror, row_mirror
__device__ __forceinline__ float row_max(float v) {
    v = fmaxf(v, dppf<0xB1>(v));
    v = fmaxf(v, dppf<0x4E>(v));
    v = fmaxf(v, dppf<0x141>(v));
    return fmaxf(v, dppf<0x140>(v));
}
__device__ __forceinline__ float row_sum(float v) {
    v += dppf<0xB1>(v);
    v += dppf<0x4E>(v);
    v += dppf<0x141>(v);
    return v + dppf<0x140>(v);
}
__device__ __forceinline__ int row_min(int v) {
    v = min(v, dppi<0xB1>(v));
    v = min(v, dppi<0x4E>(v));
    v = min(v, dppi<0x141>(v));
    return min(v, dppi<0x140>(v));
}
__device__ __forceinline__ int row_maxi(int v) {
    v = max(v, dppi<0xB1>(v));
    v = max(v, dppi<0x4E>(v));
    v = max(v, dppi<0x141>(v));
    return max(v, dppi<0x140>(v));
}
// exclusive prefix sum inside the row (row_shr 1, 2, 4, 8; lanes without a
// source read 0), then shift by one lane
__device__ __forceinline__ float row_excl_scan(float v) {
    v += dppf<0x111>(v);
    v += dppf<0x112>(v);
    v += dppf<0x114>(v);
    v += dppf<0x118>(v);
    return dppf<0x111>(v);
}

constexpr int NONE = 0x7fffffff;

template <int CH, bool VEC>
__global__ __launch_bounds__(MS_BLOCK) void k_masked(int E, int NN, const float* __restrict__ logits, long long ld,
                                                     const uint64_t* __restrict__ legal,
                                                     const float* __restrict__ uniforms, uint64_t seed,
                                                     uint32_t id_base, uint64_t counter, int mode,
                                                     int32_t* __restrict__ actions, float* __restrict__ log_probs,
                                                     float* __restrict__ entropy) {
    const long long t = (long long)blockIdx.x * MS_BLOCK + threadIdx.x;
    const int l = (int)(t & 15);
    const bool live = (t >> 4) < E;
    const int e = live ? (int)(t >> 4) : E - 1;  // dead lanes still take part in the row's DPP steps
    const float* row = logits + (size_t)e * (size_t)ld;
    float x[CH][4];
    uint32_t nib[CH];
    float m = -INFINITY;
#pragma unroll
    for (int c = 0; c < CH; ++c) {
        const int sq0 = 64 * c + 4 * l;
        nib[c] = (uint32_t)(legal[(size_t)e * CH + c] >> (4 * l)) & 0xFu;
        if constexpr (VEC) {
            float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
            if (sq0 < NN) v = *reinterpret_cast<const float4*>(row + sq0);
            x[c][0] = v.x;
            x[c][1] = v.y;
            x[c][2] = v.z;
            x[c][3] = v.w;
        } else {
#pragma unroll
            for (int j = 0; j < 4; ++j) x[c][j] = sq0 + j < NN ? row[sq0 + j] : 0.f;
        }
#pragma unroll
        for (int j = 0; j < 4; ++j)
            if ((nib[c] >> j) & 1u) m = fmaxf(m, x[c][j]);
    }
    m = row_max(m);
    // p_i = exp(x_i - max) on legal squares; S = sum p, SX = sum p (x - max)
    float p[CH][4], loc[CH];
    float s = 0.f, sx = 0.f;
#pragma unroll
    for (int c = 0; c < CH; ++c) {
        loc[c] = 0.f;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const bool ok = (nib[c] >> j) & 1u;
            const float d = ok ? x[c][j] - m : 0.f;
            p[c][j] = ok ? __expf(d) : 0.f;
            loc[c] += p[c][j];
            sx += p[c][j] * d;
        }
        s += loc[c];
    }
    const float S = row_sum(s);
    const float SX = row_sum(sx);
    const bool any = S > 0.f;
    const float logS = __logf(S);

    int a;
    if (mode == OTH_MASKED_EVAL) {
        a = actions[e];
    } else {
        int cand = NONE;
        if (mode == OTH_MASKED_MODE) {  // Categorical.mode: first (lowest) square of the largest logit
#pragma unroll
            for (int c = CH - 1; c >= 0; --c)
#pragma unroll
                for (int j = 3; j >= 0; --j)
                    if (((nib[c] >> j) & 1u) && x[c][j] == m) cand = 64 * c + 4 * l + j;
        } else {  // sample: first square whose cumulative mass exceeds u * S (np.random.choice)
            float u;
            if (uniforms) {
                u = uniforms[e];
            } else {
                u = (float)(oth::philox_x(seed, id_base + (uint32_t)e, counter, RNG_SAMPLE) >> 8) * 0x1p-24f;
            }
            const float target = u * S;
            float carry = 0.f;
#pragma unroll
            for (int c = 0; c < CH; ++c) {
                float cdf = carry + row_excl_scan(loc[c]);
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    cdf += p[c][j];
                    if (cand == NONE && ((nib[c] >> j) & 1u) && cdf > target) cand = 64 * c + 4 * l + j;
                }
                if (CH > 1) carry += row_sum(loc[c]);
            }
        }
        cand = row_min(cand);
        if (cand == NONE && any) {  // u * S rounded up to the total: the last legal square
            int last = -1;
#pragma unroll
            for (int c = 0; c < CH; ++c)
#pragma unroll
                for (int j = 0; j < 4; ++j)
                    if ((nib[c] >> j) & 1u) last = 64 * c + 4 * l + j;
            cand = row_maxi(last);
        }
        a = any ? cand : 0;  // model.py:69-71: no legal move -> action 0
    }
    // the lane holding square a writes the outputs (lane 0 when a is not a legal square)
    bool owner = false;
    float xa = 0.f;
#pragma unroll
    for (int c = 0; c < CH; ++c)
#pragma unroll
        for (int j = 0; j < 4; ++j)
            if (((nib[c] >> j) & 1u) && a == 64 * c + 4 * l + j) {
                owner = true;
                xa = x[c][j];
            }
    const bool is_choice = row_maxi(owner ? 1 : 0) != 0;
    const bool writer = is_choice ? owner : (l == 0);
    if (live && writer) {
        if (mode != OTH_MASKED_EVAL) actions[e] = a;
        if (log_probs) log_probs[e] = is_choice ? xa - m - logS : 0.f;
        if (entropy) entropy[e] = any ? logS - SX / S : 0.f;
    }
}

template <int CH>
void launch_ch(bool vec, int grid, hipStream_t st, int E, int NN, const float* logits, long long ld,
               const uint64_t* legal, const float* uniforms, uint64_t seed, uint32_t id_base, uint64_t counter,
               int mode, int32_t* actions, float* log_probs, float* entropy) {
    if (vec)
        hipLaunchKernelGGL((k_masked<CH, true>), dim3(grid), dim3(MS_BLOCK), 0, st, E, NN, logits, ld, legal, uniforms,
                           seed, id_base, counter, mode, actions, log_probs, entropy);
    else
        hipLaunchKernelGGL((k_masked<CH, false>), dim3(grid), dim3(MS_BLOCK), 0, st, E, NN, logits, ld, legal,
                           uniforms, seed, id_base, counter, mode, actions, log_probs, entropy);
}

}  // namespace

namespace oth_host {

int launch_masked(int n_board, int E, const float* logits, long long ld, const uint64_t* legal, const float* uniforms,
                  uint64_t seed, uint32_t id_base, uint64_t counter, int mode, int32_t* actions, float* log_probs,
                  float* entropy, hipStream_t st) {
    const int NN = n_board * n_board;
    const int CH = (NN + 63) / 64;
    const bool vec = (NN % 4 == 0) && (ld % 4 == 0) && (((uintptr_t)logits & 15u) == 0);
    const int grid = (int)(((long long)E * 16 + MS_BLOCK - 1) / MS_BLOCK);
    switch (CH) {
        case 1: launch_ch<1>(vec, grid, st, E, NN, logits, ld, legal, uniforms, seed, id_base, counter, mode, actions, log_probs, entropy); break;
        case 2: launch_ch<2>(vec, grid, st, E, NN, logits, ld, legal, uniforms, seed, id_base, counter, mode, actions, log_probs, entropy); break;
        case 3: launch_ch<3>(vec, grid, st, E, NN, logits, ld, legal, uniforms, seed, id_base, counter, mode, actions, log_probs, entropy); break;
        default: launch_ch<4>(vec, grid, st, E, NN, logits, ld, legal, uniforms, seed, id_base, counter, mode, actions, log_probs, entropy); break;
    }
    return after_launch("oth_masked_sample");
}

}  // namespace oth_host
