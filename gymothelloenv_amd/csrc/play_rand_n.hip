// play_rand_n.hip -- k_play_rand (the restructured random / greedy play of
// one-word boards, the bench kernel) and k_play_rand_w (random play of
// multi-word boards) in a translation unit of their own per board size
// (-DOTH_N=4 .. 16), compiled with the max-ILP machine scheduler
// (build.py PLAY_FLAGS: -mllvm -amdgpu-sched-strategy=max-ilp).  At 65,536
// boards each SIMD runs one wave, so what the schedule hides of the dependent
// chains counts and occupancy does not: 8x8 0.779 -> 0.762 us per ply with
// the next Philox block pinned in the group's first ply (profiles/r02/fi/).  The same flag on the whole library costs
// the fused sample-and-step kernel 4 %, hence the separate unit.
#include "device.hpp"
#include "launch.hpp"

#ifndef OTH_N
#error "compile with -DOTH_N=<board size>"
#endif

using namespace oth;
using namespace oth_dev;

namespace oth_host {

template <int N, int POL>
void launch_play_rand(oth_env* env, int n_plies, int32_t* actions, int32_t* rewards, uint8_t* dones, uint64_t ply0,
                      hipStream_t st) {
    const dim3 grid((unsigned)(((long long)env->E + BLOCK - 1) / BLOCK)), block(BLOCK);
    const Rng rng{env->seed, env->id_base, env->init_rand, env->cur_off};
    // (greedy play on lane pairs, k_play_greedy2, measured 7 % slower and was removed:
    // git show 53fb080:gymothelloenv_amd/csrc/pair_play.hpp)
    if constexpr (Geo<N>::W == 1)
        launch_k((k_play_rand<N, POL>), grid, block, 0, st, env->boards, env->meta, env->legal, env->E,
                 env->flags, n_plies, actions, rewards, dones, env->wdl, rng, ply0, env->rays);
    else  // random play only (k_play_rand_w)
        launch_k((k_play_rand_w<N>), grid, block, 0, st, env->boards, env->meta, env->legal, env->E,
                 env->flags, n_plies, actions, rewards, dones, env->wdl, rng, ply0);
}

template void launch_play_rand<OTH_N, OTH_POLICY_RANDOM>(oth_env*, int, int32_t*, int32_t*, uint8_t*, uint64_t,
                                                         hipStream_t);
#if OTH_N <= 8
template void launch_play_rand<OTH_N, OTH_POLICY_GREEDY>(oth_env*, int, int32_t*, int32_t*, uint8_t*, uint64_t,
                                                         hipStream_t);
#endif

}  // namespace oth_host
