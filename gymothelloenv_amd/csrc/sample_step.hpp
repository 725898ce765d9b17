// sample_step.hpp -- oth_sample_step: the learners' per-ply loop in one launch
// (the masked categorical of masked.hpp, then OthelloBaseEnv.step), in three
// lane layouts.  Included after ply.hpp, whose one-lane step (step1) the pair
// layout uses.
#pragma once

#include "device.hpp"
#include "ply.hpp"

// (the observation tail at the end of the three kernels costs nothing when unused:
// 65,536 8x8 boards 5.99 -> 6.03 us per graphed ply, profiles/r05/b/ab_ss_tail.json)

namespace oth_dev {

// oth_sample_step: the learners' per-ply loop in one launch -- the masked
// categorical over each board's possible_moves (Policy.act, model.py:60-99;
// PPO.get_action, ppo.py:228-262) immediately followed by OthelloBaseEnv.step
// (othello.py:412-462) with the sampled action.  The sampling runs the very
// code of k_masked (masked.hpp) with its G lanes per board: lane group g
// samples its G boards g*G .. g*G+G-1 one after the other and lane l keeps
// board g*G+l's pick, which is the board it then steps (one lane per board,
// as k_step).  So the results are bit-identical to oth_sample_actions +
// oth_step, with one launch and no actions round trip through memory.
// ONE (boards of up to two words): each lane samples its own board with
// oth_ms::sample_lane, the group's arithmetic restated for one lane.
template <int N, int G, bool VEC, bool FULL, bool ONE>
__global__ __launch_bounds__(BLOCK) void k_sample_step(uint64_t* __restrict__ boards, uint16_t* __restrict__ meta,
                                                       uint64_t* __restrict__ legal, int E, uint32_t flags,
                                                       const float* __restrict__ logits, long long ld,
                                                       const float* __restrict__ uniforms, uint64_t counter, int mode,
                                                       int32_t* __restrict__ actions, float* __restrict__ log_probs,
                                                       float* __restrict__ entropy, int32_t* __restrict__ rewards,
                                                       uint8_t* __restrict__ dones,
                                                       unsigned long long* __restrict__ wdl, Rng rng, uint64_t ply,
                                                       int obs_layout, int obs_dtype, void* __restrict__ obs) {
    constexpr int NN = N * N;
    constexpr int CH = Geo<N>::W;
    ply += rng.ply_off[0];      // graph-region offsets (oth_graph_end); 0 eagerly
    counter += rng.ply_off[1];  // the sample counter's, as k_masked
    const long long t = (long long)blockIdx.x * BLOCK + threadIdx.x;
    const int l = (int)(t % G);
    const long long g0 = (t / G) * G;
    const bool mine_live = t < E;
    WaveSlot slot(wdl, (int)t, E);
    // the board this lane steps: its loads are issued before the sampling, so
    // they are in flight while the group samples
    Lane<N> s;
    if (mine_live) load_lane<N>(s, boards, meta, legal, (int)t);
    oth_ms::Pick mine{0, 0.f, 0.f};
    if constexpr (ONE) {  // one lane per board: the group's arithmetic restated per lane (oth_ms::sample_lane)
        if (mine_live)
            mine = oth_ms::sample_lane<CH, G, VEC, FULL>((int)t, NN, logits, ld, legal, uniforms, rng.seed,
                                                         rng.id_base, counter, mode, 0, log_probs != nullptr,
                                                         entropy != nullptr);
    } else {
    constexpr int BATCH = G < 4 ? G : 4;  // boards whose logits loads are issued together
#pragma unroll 1
    for (int k0 = 0; k0 < G; k0 += BATCH) {
        oth_ms::Slot<CH, G> b[BATCH];
#pragma unroll
        for (int k = 0; k < BATCH; ++k) {
            const long long eb = g0 + k0 + k;
            b[k].live = eb < E;
            b[k].e = b[k].live ? (int)eb : E - 1;  // dead boards still take part in the group's DPP steps
            oth_ms::load_slot<CH, G, VEC>(b[k], l, NN, logits, ld, legal);
        }
#pragma unroll
        for (int k = 0; k < BATCH; ++k) {
            const oth_ms::Pick pk = oth_ms::finish_slot<CH, G, FULL>(b[k], l, NN, logits, ld, uniforms, rng.seed,
                                                                     rng.id_base, counter, mode, 0,
                                                                     log_probs != nullptr, entropy != nullptr);
            if (k0 + k == l) mine = pk;
        }
    }
    }
    uint32_t cb = 0, cd = 0, cw = 0;
    if (mine_live) {
        const int e = (int)t;
        actions[e] = mine.a;
        if (log_probs) log_probs[e] = mine.lp;
        if (entropy) entropy[e] = mine.ent;
        const bool was_term = (s.meta & M_TERMINATED) != 0;
        int r, d, win;
        step_lane<N>(s, mine.a, flags, r, d, win, Solo<N>(0, nullptr));
        if (d && !was_term) {
            cb = win == BLACK_DISK;
            cd = win == NO_DISK;
            cw = win == WHITE_DISK;
            if (flags & OTH_AUTO_RESET)
                reset_lane<N>(s, rng.seed, rng.id_base + (uint32_t)e, ply, RNG_OPENING_AUTO, rng.init_rand);
        }
        store_lane<N>(s, boards, meta, legal, e);
        if (rewards) rewards[e] = r;
        if (dones) dones[e] = (uint8_t)d;
    }
    slot.count(cb != 0, cd != 0, cw != 0);
    slot.flush();
    // oth_sample_step_observe: the wave's 64 boards' observations (lane = board)
    const long long e0 = t - (threadIdx.x & 63);
    obs_tail<N, 64, 1>(obs_layout, obs_dtype, obs, e0, s.black.w, s.white.w, s.legal.w, s.meta,
                       (int)(E - e0 < 64 ? E - e0 : 64));
}

// k_sample_step on lane pairs (boards of one or two words): the pair samples
// its board with oth_ms::sample_pair (bit-identical to the one-lane form), then
// both lanes step it (the same inputs, so they agree): one-word boards with
// step1 (ply.hpp: capped runs from computed rays -- no ray table, no LDS, no
// barrier -- each lane of the pair running four of the eight directions and the
// pair OR-ing the halves through DPP), two-word boards with the Solo engine.  Twice the waves of
// k_sample_step for the same boards, so two waves share each SIMD at 65,536
// boards: the loads of one hide behind the other's VALU work, and the pair
// halves the per-lane sampling.  The W/D/L tally goes to per-wave slots
// (ballots): no block barrier anywhere in the launch.
template <int N, bool VEC, bool FULL>
__global__ __launch_bounds__(BLOCK) void k_sample_step2(uint64_t* __restrict__ boards, uint16_t* __restrict__ meta,
                                                        uint64_t* __restrict__ legal, int E, uint32_t flags,
                                                        const float* __restrict__ logits, long long ld,
                                                        const float* __restrict__ uniforms, uint64_t counter,
                                                        int mode, int32_t* __restrict__ actions,
                                                        float* __restrict__ log_probs, float* __restrict__ entropy,
                                                        int32_t* __restrict__ rewards, uint8_t* __restrict__ dones,
                                                        unsigned long long* __restrict__ wdl, Rng rng, uint64_t ply,
                                                        int obs_layout, int obs_dtype, void* __restrict__ obs) {
    constexpr int W = Geo<N>::W;
    static_assert(W <= 2 && oth_ms::MS_G == 4, "lane pairs restate k_masked's four lanes of boards of <= 2 words");
    constexpr int NN = N * N;
    ply += rng.ply_off[0];      // graph-region offsets (oth_graph_end); 0 eagerly
    counter += rng.ply_off[1];  // the sample counter's, as k_masked
    const long long gt = (long long)blockIdx.x * BLOCK + threadIdx.x;
    const int e = (int)(gt >> 1), h = (int)(gt & 1);
    uint32_t cb = 0, cd = 0, cw = 0;
    Lane<N> s;  // the board's loads are issued first, in flight with the logits loads
    if (e < E) load_lane<N>(s, boards, meta, legal, e);
    // wave w of the grid owns slot w (2E lanes; the handle holds ceil(4E / 64) slots)
    WaveSlot slot(wdl, (int)min(gt >> 6, (2LL * E - 1) >> 6));
    auto board = [&](auto STAGEDC, const oth_ms::f32x4* staged) __attribute__((always_inline)) {
        if (e >= E) return;  // pair-uniform: both lanes of a pair share e
        const oth_ms::Pick pk = oth_ms::sample_pair<W, VEC, FULL, decltype(STAGEDC)::value>(
            e, h, NN, logits, ld, s.legal.w, uniforms, rng.seed, rng.id_base, counter, mode, log_probs != nullptr,
            entropy != nullptr, staged);
        const bool was_term = (s.meta & M_TERMINATED) != 0;
        int r = 0, d = 0, win = NO_DISK;
        if constexpr (W == 1) {
            uint64_t B = s.black.w[0], Wt = s.white.w[0], L = s.legal.w[0];
            uint32_t m = s.meta;
            const int a = pk.a;
            const bool valid = (unsigned)a < (unsigned)NN && ((L >> (a & 63)) & 1ull);
            // the flips split over the pair (RAYS_PAIR: lane 0 the up half, lane 1 the down
            // half): 65,536 8x8 boards 5.86 -> 5.64 us per graphed ply, 7x7 5.83 -> 5.65
            step1<N, RAYS_PAIR>(B, Wt, L, m, a, valid, flags, nullptr, r, d, win, h);
            if (was_term) {  // a no-op reporting done (othello.py:415-416)
                r = 0;
                d = 1;
            } else {
                s.black.w[0] = B;
                s.white.w[0] = Wt;
                s.legal.w[0] = L;
                s.meta = m;
            }
        } else {
            step_lane<N>(s, pk.a, flags, r, d, win, Solo<N>(0, nullptr));
        }
        if (d && !was_term) {
            if (h == 0) {
                cb = win == BLACK_DISK;
                cd = win == NO_DISK;
                cw = win == WHITE_DISK;
            }
            if (flags & OTH_AUTO_RESET)
                reset_lane<N>(s, rng.seed, rng.id_base + (uint32_t)e, ply, RNG_OPENING_AUTO, rng.init_rand);
        }
        if (h == 0) {
            actions[e] = pk.a;
            if (log_probs) log_probs[e] = pk.lp;
            if (entropy) entropy[e] = pk.ent;
            store_lane<N>(s, boards, meta, legal, e);
            if (rewards) rewards[e] = r;
            if (dones) dones[e] = (uint8_t)d;
        }
    };
    if constexpr (VEC && N == 8) {  // the wave's 32 rows through LDS: coalesced loads
        __shared__ oth_ms::f32x4 stage[(BLOCK / 64) * 32 * oth_ms::PAIR_ROW];
        const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
        oth_ms::f32x4 v[8];
        oth_ms::load_pair_rows(v, (gt - lane) >> 1, E, logits, ld, lane);
        // (store_pair_rows syncs the wave: each wave reads back only its own rows)
        const oth_ms::f32x4* rows = oth_ms::store_pair_rows(stage + wv * 32 * oth_ms::PAIR_ROW, v, lane);
        board(std::true_type{}, rows);
    } else {
        board(std::false_type{}, nullptr);
    }
    slot.count(cb != 0, cd != 0, cw != 0);  // (h == 0 lanes only)
    slot.flush();
    // oth_sample_step_observe: the wave's 32 boards' observations (both lanes of a
    // pair hold the board as stepped and reset)
    const long long e0 = (gt - (threadIdx.x & 63)) >> 1;
    obs_tail<N, 32, 2>(obs_layout, obs_dtype, obs, e0, s.black.w, s.white.w, s.legal.w, s.meta,
                       (int)(E - e0 < 32 ? E - e0 : 32));
}

// k_sample_step on lane quads (one-word boards): the quad IS k_masked's group
// of G = 4 lanes for the board (load_slot / finish_slot, the same code, so the
// pick is k_masked's), then steps it with the Quartet engine.  Four times the
// waves of the one-lane form: each lane's instruction stream is a quarter of
// the sampling and of the scans, and four waves share each SIMD.
template <int N, bool VEC, bool FULL>
__global__ __launch_bounds__(BLOCK) void k_sample_step4(uint64_t* __restrict__ boards, uint16_t* __restrict__ meta,
                                                        uint64_t* __restrict__ legal, int E, uint32_t flags,
                                                        const float* __restrict__ logits, long long ld,
                                                        const float* __restrict__ uniforms, uint64_t counter,
                                                        int mode, int32_t* __restrict__ actions,
                                                        float* __restrict__ log_probs, float* __restrict__ entropy,
                                                        int32_t* __restrict__ rewards, uint8_t* __restrict__ dones,
                                                        unsigned long long* __restrict__ wdl, Rng rng, uint64_t ply,
                                                        int obs_layout, int obs_dtype, void* __restrict__ obs) {
    static_assert(Geo<N>::W == 1 && oth_ms::MS_G == 4, "lane quads are k_masked's four lanes of one-word boards");
    constexpr int NN = N * N;
    ply += rng.ply_off[0];      // graph-region offsets (oth_graph_end); 0 eagerly
    counter += rng.ply_off[1];  // the sample counter's, as k_masked
    __shared__ __attribute__((aligned(16))) uint64_t lds_rays[Quartet<N>::RAY_WORDS];
    const long long gt = (long long)blockIdx.x * BLOCK + threadIdx.x;
    const int e = (int)(gt >> 2), q = (int)(gt & 3);
    const Quartet<N> eng(q, lds_rays);
    uint32_t cb = 0, cd = 0, cw = 0;
    WaveSlot slot(wdl, (int)min(gt >> 6, (4LL * E - 1) >> 6));  // 4E lanes: ceil(4E / 64) slots
    Lane<N> s;  // the board's and the logits' loads are issued before the ray tables are built
    oth_ms::Slot<1, 4> b;
    b.e = e;
    b.live = e < E;
    if (e < E) {
        load_lane<N>(s, boards, meta, legal, e);
        oth_ms::load_slot<1, 4, VEC>(b, q, NN, logits, ld, legal);
    }
    fill_rays<N, false>(lds_rays);
    if (e < E) {  // quad-uniform: the four lanes of a quad share e
        const oth_ms::Pick pk = oth_ms::finish_slot<1, 4, FULL>(b, q, NN, logits, ld, uniforms, rng.seed, rng.id_base,
                                                                counter, mode, 0, log_probs != nullptr,
                                                                entropy != nullptr);
        const bool was_term = (s.meta & M_TERMINATED) != 0;
        int r, d, win;
        step_lane<N>(s, pk.a, flags, r, d, win, eng);
        if (d && !was_term) {
            if (q == 0) {
                cb = win == BLACK_DISK;
                cd = win == NO_DISK;
                cw = win == WHITE_DISK;
            }
            if (flags & OTH_AUTO_RESET)
                reset_lane<N>(s, rng.seed, rng.id_base + (uint32_t)e, ply, RNG_OPENING_AUTO, rng.init_rand);
        }
        if (q == 0) {
            actions[e] = pk.a;
            if (log_probs) log_probs[e] = pk.lp;
            if (entropy) entropy[e] = pk.ent;
            store_lane<N>(s, boards, meta, legal, e);
            if (rewards) rewards[e] = r;
            if (dones) dones[e] = (uint8_t)d;
        }
    }
    slot.count(cb != 0, cd != 0, cw != 0);  // (q == 0 lanes only)
    slot.flush();
    // oth_sample_step_observe: the wave's 16 boards' observations (the quad's four
    // lanes hold the board as stepped and reset)
    const long long e0 = (gt - (threadIdx.x & 63)) >> 2;
    obs_tail<N, 16, 4>(obs_layout, obs_dtype, obs, e0, s.black.w, s.white.w, s.legal.w, s.meta,
                       (int)(E - e0 < 16 ? E - e0 : 16));
}

}  // namespace oth_dev
