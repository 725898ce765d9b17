// masked.hip -- k_masked: the masked categorical over each board's legal
// squares as one launch over n boards, the C ABI's
// oth_masked_sample / oth_sample_actions.  The per-board device code is in
// masked.hpp (shared with the fused sample-and-step kernel).
// HBM bound: 4 N^2 B of logits + 8W B of legal per board in, 12 B out.
#include <hip/hip_runtime.h>
#include <float.h>
#include <math.h>

#include "launch.hpp"
#include "masked.hpp"

namespace {

using namespace oth_ms;

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
    for (int k = 0; k < BPR; ++k) {
        const int e = b[k].e;
        const Pick pk = finish_slot<CH, G, FULL>(b[k], l, NN, logits, ld, uniforms, seed, id_base, counter, mode,
                                                 mode == OTH_MASKED_EVAL ? actions[e] : 0, log_probs != nullptr,
                                                 entropy != nullptr);
        if (b[k].live && l == 0) {
            if (mode != OTH_MASKED_EVAL) actions[e] = pk.a;
            if (log_probs) log_probs[e] = pk.lp;
            if (entropy) entropy[e] = pk.ent;
        }
    }
}

template <int CH, int G, int BPR, bool FULL>
void launch_one(bool vec, int E, hipStream_t st, int NN, const float* logits, long long ld, const uint64_t* legal,
               const float* uniforms, uint64_t seed, uint32_t id_base, uint64_t counter, const uint64_t* counter_off,
               int mode, int32_t* actions, float* log_probs, float* entropy) {
    const long long groups = ((long long)E + BPR - 1) / BPR;
    const int grid = (int)((groups * G + MS_BLOCK - 1) / MS_BLOCK);
    if (vec)
        oth_host::launch_k((k_masked<CH, G, true, BPR, FULL>), dim3(grid), dim3(MS_BLOCK), 0, st, E, NN, logits, ld,
                 legal, uniforms, seed, id_base, counter, counter_off, mode, actions, log_probs, entropy);
    else
        oth_host::launch_k((k_masked<CH, G, false, BPR, FULL>), dim3(grid), dim3(MS_BLOCK), 0, st, E, NN, logits, ld,
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
    switch (CH) {  // MS_G lanes per board up to 128 squares, 16 beyond (registers)
        case 1: launch_ch<1, oth_ms::MS_G, oth_ms::MS_BPR>(OTH_MS_ARGS); break;
        case 2: launch_ch<2, oth_ms::MS_G, 1>(OTH_MS_ARGS); break;
        case 3: launch_ch<3, 16, 1>(OTH_MS_ARGS); break;
        default: launch_ch<4, 16, 1>(OTH_MS_ARGS); break;
    }
#undef OTH_MS_ARGS
    return after_launch("oth_masked_sample");
}

}  // namespace oth_host
