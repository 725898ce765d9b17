// kernels_n.hip -- kernel launchers for ONE board size, compiled once per N
// (-DOTH_N=4 .. 16) so the 13 template sets build in parallel.
#include <type_traits>

#include "device.hpp"
#include "launch.hpp"
#include "maximin_wave.hpp"
#include "ply.hpp"
#include "sample_step.hpp"

#ifndef OTH_N
#error "compile with -DOTH_N=<board size>"
#endif

using namespace oth;
using namespace oth_dev;

namespace oth_host {
namespace {

int grid_for(long long work) { return (int)((work + BLOCK - 1) / BLOCK); }

// policy: an OTH_POLICY_* id; MaxiMin of depth >= 4 reads its depth from the Rng
Rng rng_of(const oth_env* env, int policy = OTH_POLICY_RANDOM) {
    const int depth = policy >= OTH_POLICY_MAXIMIN1 ? policy - OTH_POLICY_MAXIMIN1 + 1 : 0;
    return Rng{env->seed, env->id_base, env->init_rand, env->cur_off, depth};
}

// Compile-time policy for a runtime id (OTH_POLICY_*); MAXIMIN1 is GREEDY
// (same move: simple_policies.py:111-155 at depth 1 is GreedyPolicy's argmax).
template <typename Fn>
int with_policy(int policy, Fn&& fn) {
    switch (policy) {
        case OTH_POLICY_RANDOM: return fn(std::integral_constant<int, OTH_POLICY_RANDOM>{});
        case OTH_POLICY_GREEDY:
        case OTH_POLICY_MAXIMIN1: return fn(std::integral_constant<int, OTH_POLICY_GREEDY>{});
        case OTH_POLICY_MAXIMIN2: return fn(std::integral_constant<int, OTH_POLICY_MAXIMIN2>{});
        case OTH_POLICY_MAXIMIN3: return fn(std::integral_constant<int, OTH_POLICY_MAXIMIN3>{});
        default:
            if (policy > OTH_POLICY_MAXIMIN3 && policy <= OTH_POLICY_LAST)  // depth 4 .. OTH_MAXIMIN_MAX_DEPTH
                return fn(std::integral_constant<int, OTH_POLICY_MAXIMIN_DEEP>{});
            return fail(OTH_EINVAL, "unknown policy");
    }
}

// the step kernels' fused observation (obs_tail): none, or a layout / dtype / output
struct ObsOut {
    int layout = -1;
    int dtype = 0;
    void* out = nullptr;
};
// obs_tail's quad stores need N*N % 4 == 0 and an output aligned to 4 elements
template <int N>
bool obs_fusable(int dtype, const void* out) {
    static const int esize[6] = {1, 4, 8, 4, 8, 2};
    return (N * N) % 4 == 0 && dtype >= OTH_I8 && dtype <= OTH_BF16 &&
           (uintptr_t)out % obs_align(N * N, esize[dtype]) == 0;
}

}  // namespace

template <int N>
int launch_reset(oth_env* env, const uint8_t* mask, hipStream_t st) {
    launch_k(k_reset<N>, dim3(grid_for(env->E)), dim3(BLOCK), 0, st, env->boards, env->meta, env->legal,
             env->E, mask, rng_of(env), env->ply);
    return after_launch("oth_reset");
}

// oth_create for one-word boards: the single-ply kernels' ray table
template <int N>
int launch_fill_rays(oth_env* env, hipStream_t st) {
    if constexpr (Geo<N>::W == 1) {
        launch_k(k_fill_rays<N>, dim3(1), dim3(BLOCK), 0, st, env->rays);
        return after_launch("oth_create: ray table");
    }
    return OTH_OK;
}

template <int N>
int launch_step(oth_env* env, const int32_t* actions, int32_t* rewards, uint8_t* dones, uint64_t ply,
                hipStream_t st) {
    if constexpr (Geo<N>::W == 1) {  // the single-ply kernel (ply.hpp)
        if (env->E <= OTH_PLY_MATH_MAX_E)
            launch_k((k_ply_step<N, RAYS_MATH>), dim3(grid_for(env->E)), dim3(BLOCK), 0, st, env->boards,
                     env->meta, env->legal, env->E, env->flags, actions, rewards, dones, env->wdl, env->rays,
                     rng_of(env), ply);
        else
            launch_k((k_ply_step<N, RAYS_HALF>), dim3(grid_for(env->E)), dim3(BLOCK), 0, st,
                     env->boards, env->meta, env->legal, env->E, env->flags, actions, rewards, dones,
                     env->wdl, env->rays, rng_of(env), ply);
        return after_launch("oth_step");
    }
    launch_k(k_step<N>, dim3(grid_for(env->E)), dim3(BLOCK), 0, st, env->boards, env->meta, env->legal,
             env->E, env->flags, actions, rewards, dones, env->wdl, rng_of(env), ply);
    return after_launch("oth_step");
}

// from this many boards oth_step_observe takes k_observe_w's large-launch shape (one
// lane per board, 64 boards a wave) instead of lane pairs: at 1,048,576 8x8 boards
// the pairs' launch took 125.4 us with the int64 board against 116 for the two
// launches (profiles/r05/d/step/times.jsonl)
#ifndef OTH_SO_LARGE_E
#define OTH_SO_LARGE_E 262144
#endif
// (the two launches instead from 262,144 boards, with k_observe_w's 4-KiB waves,
// at 1,048,576 8x8 boards: the step with its int64 board 112.6 -> 115.2 us, with
// make_state f32 216.6 -> 209.0, the learners' ply with make_state 268.7 -> 290.2;
// profiles/r05/m)
// oth_step_observe: one-word boards step and observe in one launch (k_ply_step_obs,
// ply.hpp); other sizes, or an output the quad stores cannot write, take
// oth_step's kernel and then oth_observe's
template <int N>
int launch_step_observe(oth_env* env, const int32_t* actions, int32_t* rewards, uint8_t* dones, int layout, int dtype,
                        void* obs, uint64_t ply, hipStream_t st) {
    if constexpr (Geo<N>::W == 1 && (N * N) % 4 == 0) {
        if (obs_fusable<N>(dtype, obs)) {
            if (env->E < OTH_SO_LARGE_E) {
                constexpr int BPW = OTH_SO_BPW;
                const long long waves = ((long long)env->E + BPW - 1) / BPW;
                launch_k((k_ply_step_obs<N, OTH_SO_LPB, BPW>), dim3(grid_for(waves * 64)), dim3(BLOCK), 0, st,
                         env->boards, env->meta, env->legal, env->E, env->flags, actions, rewards, dones, env->wdl,
                         rng_of(env), ply, layout, dtype, obs);
            } else {  // one lane per board, 64 boards a wave
                const long long waves = ((long long)env->E + 63) / 64;
                launch_k((k_ply_step_obs<N, 1, 64>), dim3(grid_for(waves * 64)), dim3(BLOCK), 0, st, env->boards,
                         env->meta, env->legal, env->E, env->flags, actions, rewards, dones, env->wdl, rng_of(env),
                         ply, layout, dtype, obs);
            }
            return after_launch("oth_step_observe");
        }
    }
    const int rc = launch_step<N>(env, actions, rewards, dones, ply, st);
    if (rc) return rc;
    return launch_observe<N>(env, layout, dtype, obs, st);
}

// k_play with the REC specialisation where all per-ply outputs are stored
// (random / greedy only, to bound the number of maximin instantiations).
template <int N, int POL, typename Eng>
void launch_k_play(int lanes_per_board, oth_env* env, int policy, int n_plies, int32_t* actions, int32_t* rewards,
                   uint8_t* dones, uint64_t ply0, hipStream_t st) {
    const dim3 grid(grid_for((long long)lanes_per_board * env->E)), block(BLOCK);
    if constexpr (POL == OTH_POLICY_RANDOM && Geo<N>::W == 1) {
        if (n_plies == 1) {  // one ply per launch: the single-ply kernel (ply.hpp), any flags
            if (env->E <= OTH_PLY_MATH_MAX_E)
                launch_k((k_ply_rand<N, RAYS_MATH>), dim3(grid_for(env->E)), block, 0, st, env->boards,
                         env->meta, env->legal, env->E, env->flags, actions, rewards, dones, env->wdl,
                         env->rays, rng_of(env), ply0);
            else
                launch_k((k_ply_rand<N, RAYS_HALF>), dim3(grid_for(env->E)), block, 0, st,
                         env->boards, env->meta, env->legal, env->E, env->flags, actions, rewards, dones,
                         env->wdl, env->rays, rng_of(env), ply0);
            return;
        }
    }
    if constexpr (POL == OTH_POLICY_RANDOM && std::is_same<Eng, Fills<N>>::value) {
        if (actions && rewards && dones && (env->flags & OTH_AUTO_RESET)) {
            launch_play_rand<N, OTH_POLICY_RANDOM>(env, n_plies, actions, rewards, dones, ply0, st);  // play_rand_n.hip
            return;
        }
    }
    if constexpr (POL == OTH_POLICY_GREEDY && std::is_same<Eng, Fills<N>>::value) {
        if (actions && rewards && dones && (env->flags & OTH_AUTO_RESET)) {
            launch_play_rand<N, OTH_POLICY_GREEDY>(env, n_plies, actions, rewards, dones, ply0, st);  // play_rand_n.hip
            return;
        }
    }
    if constexpr (POL == OTH_POLICY_RANDOM && std::is_same<Eng, FillsW<N>>::value) {
        if (actions && rewards && dones && (env->flags & OTH_AUTO_RESET)) {
            if constexpr (Geo<N>::W == 2)  // the max-ILP unit (play_rand_n.hip): 10x10 +5 %, 12x12 -4 %
                launch_play_rand<N, OTH_POLICY_RANDOM>(env, n_plies, actions, rewards, dones, ply0, st);
            else
                launch_k((k_play_rand_w<N>), grid, block, 0, st, env->boards, env->meta, env->legal, env->E,
                         env->flags, n_plies, actions, rewards, dones, env->wdl, rng_of(env, policy), ply0);
            return;
        }
    }
    if constexpr (POL == OTH_POLICY_RANDOM || POL == OTH_POLICY_GREEDY) {
        if (actions && rewards && dones) {
            launch_k((k_play<N, POL, Eng, true>), grid, block, 0, st, env->boards, env->meta, env->legal,
                     env->E, env->flags, n_plies, actions, rewards, dones, env->wdl, rng_of(env, policy), ply0);
            return;
        }
    }
    launch_k((k_play<N, POL, Eng, false>), grid, block, 0, st, env->boards, env->meta, env->legal, env->E,
             env->flags, n_plies, actions, rewards, dones, env->wdl, rng_of(env, policy), ply0);
}

template <int N>
int launch_play(oth_env* env, int policy, int n_plies, int32_t* actions, int32_t* rewards, uint8_t* dones,
                uint64_t ply0, hipStream_t st) {
    return with_policy(policy, [&](auto PC) {
        constexpr int POL = decltype(PC)::value;
        // random and greedy play: the fills engines (flips from the legal scan's
        // fills and a ray table in LDS; FillsW's BB<W> table of 16x16 boards is 64 KiB);
        // MaxiMin: Kogge-Stone flips (Solo) inside its search
        if constexpr (Geo<N>::W == 1 && (POL == OTH_POLICY_RANDOM || POL == OTH_POLICY_GREEDY)) {
            launch_k_play<N, POL, Fills<N>>(1, env, policy, n_plies, actions, rewards, dones, ply0, st);
        } else if constexpr (Geo<N>::W > 1 && (POL == OTH_POLICY_RANDOM || POL == OTH_POLICY_GREEDY)) {
            launch_k_play<N, POL, FillsW<N>>(1, env, policy, n_plies, actions, rewards, dones, ply0, st);
        } else {
            launch_k_play<N, POL, Solo<N>>(1, env, policy, n_plies, actions, rewards, dones, ply0, st);
        }
        return after_launch("oth_step_policy");
    });
}

// with the observation tail: lane quads (16 boards a wave, the store loop's best
// shape) up to this many boards.  8x8, make_state f32, graphed: 32,768 boards
// 14.27 -> 12.34 us per ply on quads; 65,536 17.37 -> 17.85 (profiles/r05/c/ab_ss_obs*.json)
#ifndef OTH_SSO_QUAD_MAX_E
#define OTH_SSO_QUAD_MAX_E 32768
#endif
template <int N, int G, bool VEC, bool FULL>
void launch_ss(oth_env* env, const float* logits, long long ld, const float* uniforms, uint64_t counter, int mode,
               int32_t* actions, float* log_probs, float* entropy, int32_t* rewards, uint8_t* dones, uint64_t ply,
               const ObsOut& ob, hipStream_t st) {
    // lane quads (k_sample_step4) while the quads fill at most one wave per SIMD: latency-bound sizes,
    // where a quarter of the per-lane instruction stream wins (8x8, E = 3001: 5.67 -> 4.83 us per ply);
    // beyond, the quads' duplicated step work loses to pairs (65,536: 7.02 -> 7.45)
    // (the tally slots oth_create sizes cover the quads' grid: one slot per block)
    if constexpr (Geo<N>::W == 1) {
        const long long quad_max = ob.out ? OTH_SSO_QUAD_MAX_E : OTH_SS_QUAD_MAX_E;
        if (env->E <= quad_max && grid_for(4LL * env->E) <= env->nslots) {
            launch_k((k_sample_step4<N, VEC, FULL>), dim3(grid_for(4LL * env->E)), dim3(BLOCK), 0, st,
                     env->boards, env->meta, env->legal, env->E, env->flags, logits, ld, uniforms, counter,
                     mode, actions, log_probs, entropy, rewards, dones, env->wdl, rng_of(env), ply, ob.layout, ob.dtype,
                     ob.out);
            return;
        }
    }
    // lane pairs (k_sample_step2) for 7x7 and 8x8: 8x8 7.77 -> 7.22 us per ply graphed (-8.5 % with
    // log-probs); 6x6 loses (5.1 -> 6.0: the one-lane form folds the squares past N*N away)
    // two-word boards (9x9 .. 11x11): pairs for float4-aligned rows (10x10: 11.62 -> 11.42 us at 65,536
    // boards) and up to OTH_SS_PAIR_W_MAX_E boards otherwise (9x9 / 11x11 at 16,384: -14 / -20 %; at
    // 65,536 the pairs' scalar loads lose 9 %); 10x10 at 777 .. 32,768 boards: -20 .. -25 %
    constexpr bool PAIR1 = Geo<N>::W == 1 && N >= 7;
    constexpr bool PAIR2 = Geo<N>::W == 2;
    if constexpr (PAIR1 || PAIR2) {
        if (PAIR1 || VEC || env->E <= OTH_SS_PAIR_W_MAX_E) {
            launch_k((k_sample_step2<N, VEC, FULL>), dim3(grid_for(2LL * env->E)), dim3(BLOCK), 0, st,
                     env->boards, env->meta, env->legal, env->E, env->flags, logits, ld, uniforms, counter,
                     mode, actions, log_probs, entropy, rewards, dones, env->wdl, rng_of(env), ply, ob.layout, ob.dtype,
                     ob.out);
            return;
        }
    }
    // one lane samples one board (oth_ms::sample_lane) for boards of <= 2 words
    constexpr bool ONE = Geo<N>::W <= 2;
    const long long lanes = ONE ? (long long)env->E : ((long long)env->E + G - 1) / G * G;
    launch_k((k_sample_step<N, G, VEC, FULL, ONE>), dim3(grid_for(lanes)), dim3(BLOCK), 0, st, env->boards,
             env->meta, env->legal, env->E, env->flags, logits, ld, uniforms, counter, mode, actions,
             log_probs, entropy, rewards, dones, env->wdl, rng_of(env), ply, ob.layout, ob.dtype, ob.out);
}

// the sampler's lanes per board: k_masked's choice for the board's word count
// (launch_masked), so the arithmetic is the same instruction for instruction
template <int N>
int launch_sample_step(oth_env* env, const float* logits, long long ld, const float* uniforms, uint64_t counter,
                       int mode, int32_t* actions, float* log_probs, float* entropy, int32_t* rewards, uint8_t* dones,
                       uint64_t ply, int obs_layout, int obs_dtype, void* obs, hipStream_t st) {
    constexpr int G = Geo<N>::W <= 2 ? oth_ms::MS_G : 16;
    const bool vec = ((N * N) % 4 == 0) && (ld % 4 == 0) && (((uintptr_t)logits & 15u) == 0);
    const bool full = (mode & OTH_MASKED_FULL_ENTROPY) != 0;
    const int base = mode & 3;
    // the observation from the step kernel's registers where its quad stores can
    // write `obs`; else a k_observe launch after it (the same values)
    const bool fuse = obs && obs_fusable<N>(obs_dtype, obs);
    const ObsOut ob = fuse ? ObsOut{obs_layout, obs_dtype, obs} : ObsOut{};
    if (vec) {
        if (full) launch_ss<N, G, true, true>(env, logits, ld, uniforms, counter, base, actions, log_probs, entropy,
                                              rewards, dones, ply, ob, st);
        else launch_ss<N, G, true, false>(env, logits, ld, uniforms, counter, base, actions, log_probs, entropy,
                                          rewards, dones, ply, ob, st);
    } else {
        if (full) launch_ss<N, G, false, true>(env, logits, ld, uniforms, counter, base, actions, log_probs,
                                               entropy, rewards, dones, ply, ob, st);
        else launch_ss<N, G, false, false>(env, logits, ld, uniforms, counter, base, actions, log_probs, entropy,
                                           rewards, dones, ply, ob, st);
    }
    const int rc = after_launch("oth_sample_step");
    if (rc || !obs || fuse) return rc;
    return launch_observe<N>(env, obs_layout, obs_dtype, obs, st);
}

template <int N>
int launch_reset_vs(oth_env* env, int policy, const int8_t* prot, const uint8_t* mask, uint64_t call,
                    hipStream_t st) {
    return with_policy(policy, [&](auto PC) {
        constexpr int POL = decltype(PC)::value;
        launch_k((k_reset_vs<N, POL>), dim3(grid_for(env->E)), dim3(BLOCK), 0, st, env->boards, env->meta,
                 env->legal, env->E, env->flags, prot, mask, rng_of(env, policy), call);
        return after_launch("oth_reset_vs");
    });
}

// obs: NULL, or the observation (layout, dtype) of the boards after the call
// (oth_step_vs_observe): from k_step_vs1's registers where its quad stores can
// write it, else a k_observe launch after the call's kernel
template <int N>
int launch_step_vs(oth_env* env, int policy, const int32_t* actions, const int8_t* prot, int32_t* rewards,
                   uint8_t* dones, int32_t* plies, uint64_t call, int obs_layout, int obs_dtype, void* obs,
                   hipStream_t st) {
    return with_policy(policy, [&](auto PC) {
        constexpr int POL = decltype(PC)::value;
        bool fused = false;
        // one-word boards against a random or greedy opponent: k_step_vs1 (ply.hpp;
        // 65,536 8x8 boards 16-19 % less per call, profiles/r04/vs/)
        if constexpr (Geo<N>::W == 1 && (POL == OTH_POLICY_RANDOM || POL == OTH_POLICY_GREEDY)) {
            fused = obs && obs_fusable<N>(obs_dtype, obs);
            const ObsOut ob = fused ? ObsOut{obs_layout, obs_dtype, obs} : ObsOut{};
            launch_k((k_step_vs1<N, POL>), dim3(grid_for(env->E)), dim3(BLOCK), 0, st, env->boards,
                     env->meta, env->legal, env->E, env->flags, actions, prot, rewards, dones, plies,
                     env->wdl, env->wdl_vs, rng_of(env, policy), call, ob.layout, ob.dtype, ob.out);
        } else {
            launch_k((k_step_vs<N, POL>), dim3(grid_for(env->E)), dim3(BLOCK), 0, st, env->boards,
                     env->meta, env->legal, env->E, env->flags, actions, prot, rewards, dones, plies,
                     env->wdl, env->wdl_vs, rng_of(env, policy), call);
        }
        const int rc = after_launch("oth_step_vs");
        if (rc || !obs || fused) return rc;
        return launch_observe<N>(env, obs_layout, obs_dtype, obs, st);
    });
}

// MaxiMin of depth >= 3: one wave per board (k_maximin_wave, maximin_wave.hpp;
// against one lane per board, 65,536 8x8 boards: depth 3 786 -> 348 us, depth 4
// 19.9 -> 4.7 ms; profiles/r05/b/ab_maximin.jsonl); greedy and MaxiMin-2: one
// lane per board

template <int N>
int launch_policy_actions(oth_env* env, int policy, int32_t* out, hipStream_t st) {
    return with_policy(policy, [&](auto PC) {
        constexpr int POL = decltype(PC)::value;
        if constexpr (POL == OTH_POLICY_MAXIMIN3 || POL == OTH_POLICY_MAXIMIN_DEEP) {
            const int depth = POL == OTH_POLICY_MAXIMIN3 ? 3 : rng_of(env, policy).depth;
            constexpr bool NEST = Geo<N>::W <= 2;  // (boards of 3+ words: maximin_value either way)
            auto k = depth >= 4 && env->E <= OTH_MM_NESTED_MAX_E ? k_maximin_wave<N, NEST> : k_maximin_wave<N, false>;
            launch_k(k, dim3(env->E), dim3(64), 0, st, env->boards, env->meta, env->legal, env->E, out, depth);
        }
        else if constexpr (POL != OTH_POLICY_RANDOM)
            launch_k((k_policy_actions<N, POL>), dim3(grid_for(env->E)), dim3(BLOCK), 0, st, env->boards,
                     env->meta, env->legal, env->E, out, rng_of(env, policy).depth);
        return after_launch("oth_policy_actions");
    });
}

template <int N>
int launch_legal_moves(int n, const uint64_t* mover, const uint64_t* opp, uint64_t* out, hipStream_t st) {
    launch_k(k_legal_moves<N>, dim3(grid_for(n)), dim3(BLOCK), 0, st, mover, opp, out, n);
    return after_launch("oth_legal_moves");
}

// observations of fewer boards: 16 boards per wave (k_observe_w; make_state f32 at
// 65,536 boards 29.3 -> 13.8 us, int64 board 9.9 -> 9.6; 8 or 4 boards per wave:
// 13.1 / 13.2 and 9.7 / 9.9 us, profiles/r04/b/ab_obs.jsonl)
#ifndef OTH_OBS_SMALL_E
#define OTH_OBS_SMALL_E 262144
#endif
// from OTH_OBS_SMALL_E boards 64 boards a wave; once the output exceeds
// OTH_OBS_REGION_MIN_BYTES, as many boards per wave (4..64) as fill about
// OTH_OBS_LARGE_REGION bytes of output.  8x8, graphed, 64 boards a wave against
// 4-KiB regions (profiles/r05/s/ab_obs_sweep.jsonl): int64 board at 262,144 /
// 524,288 / 1,048,576 / 2,097,152 boards (139 / 278 / 556 / 1,112 MB) 22.3 /
// 42.6 / 99.4 / 208.0 us against 23.6 / 50.8 / 94.2 / 187.5; make_state f32
// (275 / 550 / 1,101 / 2,202 MB) 42.7 / 101.2 / 209.1 / 422.4 against 51.9 /
// 93.9 / 182.5 / 363.0 (torch's fill_ of the same tensors: 25.2 / 43.3 / 83.0 /
// 161.4 and 39.6 / 80.3 / 158.2 / 314.4).  Regions of 2 / 8 / 16 KiB and 64
// boards a wave in strided 4-KiB chunks lost at 1,048,576 (profiles/r05/l, m, s)
#ifndef OTH_OBS_REGION_MIN_BYTES
#define OTH_OBS_REGION_MIN_BYTES (384ll << 20)
#endif
#ifndef OTH_OBS_LARGE_REGION
#define OTH_OBS_LARGE_REGION 4096
#endif
template <int N, int LAYOUT, typename T>
constexpr int obs_large_bpw() {
    constexpr int want = OTH_OBS_LARGE_REGION / (obs_planes<LAYOUT>() * N * N * (int)sizeof(T));
    return want >= 64 ? 64 : (want >= 32 ? 32 : (want >= 16 ? 16 : (want >= 8 ? 8 : 4)));
}

// one wave per BPW boards (k_observe_w), vector stores of 4 squares: N*N % 4 == 0
// BPW0: boards per wave, or 0 for the layout's 4-KiB regions (obs_large_bpw)
template <int N, typename T, int BPW0>
void launch_observe_bpw(oth_env* env, int layout, T* o, hipStream_t st) {
    auto go = [&](auto LC) {
        constexpr int LAY = decltype(LC)::value;
        constexpr int BPW = BPW0 ? BPW0 : obs_large_bpw<N, LAY, T>();
        const dim3 gw(grid_for(((long long)env->E + BPW - 1) / BPW * 64));
        launch_k((k_observe_w<N, LAY, T, BPW>), gw, dim3(BLOCK), 0, st, env->boards, env->meta, env->legal, env->E,
                 o);
    };
    switch (layout) {
        case OTH_OBS_BOARD: go(std::integral_constant<int, OTH_OBS_BOARD>{}); break;
        case OTH_OBS_BOARD_LEGAL: go(std::integral_constant<int, OTH_OBS_BOARD_LEGAL>{}); break;
        case OTH_OBS_MAKE_STATE: go(std::integral_constant<int, OTH_OBS_MAKE_STATE>{}); break;
        case OTH_OBS_ABSOLUTE: go(std::integral_constant<int, OTH_OBS_ABSOLUTE>{}); break;
        default: go(std::integral_constant<int, OTH_OBS_LEGAL>{}); break;
    }
}
template <int N, typename T>
void launch_observe_w(oth_env* env, int layout, void* out, hipStream_t st) {
    T* o = static_cast<T*>(out);
    const int planes = layout == OTH_OBS_BOARD_LEGAL ? 2 : (layout == OTH_OBS_MAKE_STATE ? 4 : 1);
    const long long bytes = (long long)env->E * planes * N * N * (long long)sizeof(T);
    if (env->E < OTH_OBS_SMALL_E) launch_observe_bpw<N, T, 16>(env, layout, o, st);
    else if (bytes <= OTH_OBS_REGION_MIN_BYTES) launch_observe_bpw<N, T, 64>(env, layout, o, st);
    else launch_observe_bpw<N, T, 0>(env, layout, o, st);
}

template <int N>
int launch_observe(oth_env* env, int layout, int dtype, void* out, hipStream_t st) {
    const int planes = layout == OTH_OBS_BOARD_LEGAL ? 2 : (layout == OTH_OBS_MAKE_STATE ? 4 : 1);
    const long long total = (long long)env->E * planes * N * N;
    static const int esize[6] = {1, 4, 8, 4, 8, 2};
    if constexpr ((N * N) % 4 == 0) {
        // vector stores need a 4-element-aligned base and 32-bit quad indices
        if (dtype >= OTH_I8 && dtype <= OTH_BF16 && (uintptr_t)out % obs_align(N * N, esize[dtype]) == 0 &&
            total / 4 < (1ll << 31)) {
            switch (dtype) {
                case OTH_I8: launch_observe_w<N, int8_t>(env, layout, out, st); break;
                case OTH_I32: launch_observe_w<N, int32_t>(env, layout, out, st); break;
                case OTH_I64: launch_observe_w<N, long long>(env, layout, out, st); break;
                case OTH_F32: launch_observe_w<N, float>(env, layout, out, st); break;
                case OTH_BF16: launch_observe_w<N, obs_bf16>(env, layout, out, st); break;
                default: launch_observe_w<N, double>(env, layout, out, st); break;
            }
            return after_launch("oth_observe");
        }
    }
    int grid = grid_for(total);
    if (grid > 65536) grid = 65536;
    launch_k(k_observe<N>, dim3(grid), dim3(BLOCK), 0, st, env->boards, env->meta, env->legal, env->E,
             layout, dtype, out);
    return after_launch("oth_observe");
}

// oth_step_sync: one wave steps / records one board into the mapped host record
template <int N>
int launch_record(oth_env* env, int board, int step, int action, int planes, uint64_t ply, hipStream_t st) {
    launch_k(k_record<N>, dim3(1), dim3(64), 0, st, env->boards, env->meta, env->legal, board, step, action,
             env->flags, planes, env->wdl, rng_of(env), ply, env->rec_dev, env->rec_seq);
    return after_launch("oth_step_sync");
}

template <int N>
int launch_set_turn(oth_env* env, int turn, const uint8_t* mask, hipStream_t st) {
    launch_k(k_set_turn<N>, dim3(grid_for(env->E)), dim3(BLOCK), 0, st, env->boards, env->meta, env->legal,
             env->E, turn, mask);
    return after_launch("oth_set_player_turn");
}

template <int N>
int launch_count(oth_env* env, int32_t* out, hipStream_t st) {
    launch_k(k_count<N>, dim3(grid_for(env->E)), dim3(BLOCK), 0, st, env->boards, env->E, out);
    return after_launch("oth_count_disks");
}

template int launch_reset<OTH_N>(oth_env*, const uint8_t*, hipStream_t);
template int launch_step<OTH_N>(oth_env*, const int32_t*, int32_t*, uint8_t*, uint64_t, hipStream_t);
template int launch_play<OTH_N>(oth_env*, int, int, int32_t*, int32_t*, uint8_t*, uint64_t, hipStream_t);
template int launch_reset_vs<OTH_N>(oth_env*, int, const int8_t*, const uint8_t*, uint64_t, hipStream_t);
template int launch_step_vs<OTH_N>(oth_env*, int, const int32_t*, const int8_t*, int32_t*, uint8_t*, int32_t*,
                                   uint64_t, int, int, void*, hipStream_t);
template int launch_sample_step<OTH_N>(oth_env*, const float*, long long, const float*, uint64_t, int, int32_t*,
                                       float*, float*, int32_t*, uint8_t*, uint64_t, int, int, void*, hipStream_t);
template int launch_step_observe<OTH_N>(oth_env*, const int32_t*, int32_t*, uint8_t*, int, int, void*, uint64_t,
                                        hipStream_t);
template int launch_policy_actions<OTH_N>(oth_env*, int, int32_t*, hipStream_t);
template int launch_legal_moves<OTH_N>(int, const uint64_t*, const uint64_t*, uint64_t*, hipStream_t);
template int launch_observe<OTH_N>(oth_env*, int, int, void*, hipStream_t);
template int launch_set_turn<OTH_N>(oth_env*, int, const uint8_t*, hipStream_t);
template int launch_count<OTH_N>(oth_env*, int32_t*, hipStream_t);
template int launch_fill_rays<OTH_N>(oth_env*, hipStream_t);
template int launch_record<OTH_N>(oth_env*, int, int, int, int, uint64_t, hipStream_t);

}  // namespace oth_host
