// launch.hpp -- host side shared by capi.hip and the per-board-size kernel
// translation units (kernels_n.hip): the handle layout, error reporting, and
// the launcher templates, one explicit instantiation per N in kernels_n.hip.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <tuple>
#include <utility>

#include "othello_mi355x.h"

// one-word boards: oth_env::rays holds the 8 x 64-word ray table, then the sel8 table
constexpr int RAY_TABLE_WORDS = 8 * 64, SEL8_WORDS = 256, TABLE_WORDS = RAY_TABLE_WORDS + SEL8_WORDS;

struct oth_env {
    int32_t E;
    int32_t n;
    int32_t W;
    uint32_t flags;
    uint64_t seed;
    uint32_t id_base;
    int32_t init_rand;
    int32_t device;
    uint64_t ply;
    uint64_t* boards;
    uint16_t* meta;
    uint64_t* legal;
    unsigned long long* wdl;     // [nslots][4] per-block W/D/L slots by colour (tally)
    unsigned long long* wdl_vs;  // [nslots][4] per-block {protagonist wins, draws, losses} of oth_step_vs
    int32_t nslots;
    // Philox counter offsets (HIP-graph regions, oth_graph_begin/_end):
    // device [OTH_GRAPH_SLOTS][2] = (ply, sample) offsets; slot 0 serves eager
    // launches and stays 0, slot k > 0 belongs to graph region k, whose
    // captured counters start at k << OTH_GRAPH_COUNTER_SHIFT and whose offset
    // moves on by what one replay consumed.
    uint64_t* ctr_slots;
    const uint64_t* cur_off;  // the slot launches read now (slot 0 outside a region)
    int32_t graph_slot;       // open region (0: none)
    uint64_t slots_used;      // bit k: slot k belongs to a captured graph (bit 0, eager, always set)
    uint64_t ply_saved;       // eager ply counter while a region is open
    uint64_t* rays;           // one-word boards: the 8 x 64 ray table (fill_rays<N, true>) then the 256-word
                              // sel8 table (TABLE_WORDS), read by the single-ply kernels and k_play_rand
    oth_record* rec_host;     // oth_step_sync's record: mapped pinned host memory (allocated on first use)
    oth_record* rec_dev;      // its device address
    uint32_t rec_seq;         // the last record's sequence number
};

namespace oth_host {

// error reporting (capi.hip): set the thread's oth_last_error() and return the code
int fail(int code, const char* msg);
int hip_fail(hipError_t err, const char* where);
// the status of the launches since the last after_launch (hipGetLastError too)
int after_launch(const char* what);
void note_launch(hipError_t err);

// Every kernel launch of the C ABI: hipLaunchKernel on the kernel's host stub with
// the arguments converted to the kernel's parameter types, its status kept for
// after_launch.  From C, oth_step costs 3.04 us per call this way against 3.79
// through hipLaunchKernelGGL (same box, tools/launch_cost.hip; profiles/r04/lc/).
template <typename... P, typename... A>
inline void launch_k(void (*k)(P...), dim3 grid, dim3 block, size_t shmem, hipStream_t st, A&&... a) {
    static_assert(sizeof...(P) == sizeof...(A), "one argument per kernel parameter");
    std::tuple<P...> args{static_cast<P>(std::forward<A>(a))...};
    std::apply([&](auto&... x) {
        void* ptrs[] = {static_cast<void*>(&x)...};
        note_launch(hipLaunchKernel(reinterpret_cast<const void*>(k), grid, block, ptrs, shmem, st));
    }, args);
}

// masked categorical (masked.hip), any board size
int launch_masked(int n_board, int E, const float* logits, long long ld, const uint64_t* legal, const float* uniforms,
                  uint64_t seed, uint32_t id_base, uint64_t counter, const uint64_t* counter_off, int mode,
                  int32_t* actions, float* log_probs, float* entropy, hipStream_t st);

// one set per board size N (kernels_n.hip instantiates them)
template <int N> int launch_reset(oth_env* env, const uint8_t* mask, hipStream_t st);
template <int N>
int launch_step(oth_env* env, const int32_t* actions, int32_t* rewards, uint8_t* dones, uint64_t ply,
                hipStream_t st);
template <int N>
int launch_play(oth_env* env, int policy, int n_plies, int32_t* actions, int32_t* rewards, uint8_t* dones,
                uint64_t ply0, hipStream_t st);
template <int N>
int launch_reset_vs(oth_env* env, int policy, const int8_t* prot, const uint8_t* mask, uint64_t call,
                    hipStream_t st);
template <int N>
int launch_step_vs(oth_env* env, int policy, const int32_t* actions, const int8_t* prot, int32_t* rewards,
                   uint8_t* dones, int32_t* plies, uint64_t call, int obs_layout, int obs_dtype, void* obs,
                   hipStream_t st);
template <int N>
int launch_step_observe(oth_env* env, const int32_t* actions, int32_t* rewards, uint8_t* dones, int layout, int dtype,
                        void* obs, uint64_t ply, hipStream_t st);
// obs: NULL, or the observation (layout, dtype) of the boards after the step (oth_sample_step_observe)
template <int N>
int launch_sample_step(oth_env* env, const float* logits, long long ld, const float* uniforms, uint64_t counter,
                       int mode, int32_t* actions, float* log_probs, float* entropy, int32_t* rewards, uint8_t* dones,
                       uint64_t ply, int obs_layout, int obs_dtype, void* obs, hipStream_t st);
template <int N> int launch_policy_actions(oth_env* env, int policy, int32_t* out, hipStream_t st);
template <int N>
int launch_legal_moves(int n, const uint64_t* mover, const uint64_t* opp, uint64_t* out, hipStream_t st);
template <int N> int launch_observe(oth_env* env, int layout, int dtype, void* out, hipStream_t st);
template <int N> int launch_set_turn(oth_env* env, int turn, const uint8_t* mask, hipStream_t st);
template <int N> int launch_count(oth_env* env, int32_t* out, hipStream_t st);
template <int N> int launch_fill_rays(oth_env* env, hipStream_t st);
template <int N>
int launch_record(oth_env* env, int board, int step, int action, int planes, uint64_t ply, hipStream_t st);
// k_play_rand (one-word boards, random and greedy) and k_play_rand_w (two-word boards,
// random) in play_rand_n.hip, N = 4..11, with its own scheduler flags
template <int N, int POL>
void launch_play_rand(oth_env* env, int n_plies, int32_t* actions, int32_t* rewards, uint8_t* dones, uint64_t ply0,
                      hipStream_t st);

}  // namespace oth_host
