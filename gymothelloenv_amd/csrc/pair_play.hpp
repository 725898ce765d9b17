// pair_play.hpp -- k_play_greedy2: greedy play (config 3: GreedyPolicy,
// simple_policies.py:69-92, after SimpleOthelloEnv's random openings,
// othello.py:60-79) of one-word boards on lane PAIRS, the results identical to
// k_play_rand<N, GREEDY>.  Both lanes of a pair hold the board; lane h owns two
// of the four axes -- h = 0 E/W and S/N, h = 1 SE/NW and SW/NE -- and does for
// them, with per-lane shift amounts in registers (one instruction stream for
// both lanes):
//   * the legal scan and its four fills (the pair ORs the moves through DPP);
//   * update_board's flips along its four rays from the LDS ray table (OR-ed);
//   * GreedyPolicy's flip counts: the run lengths of its four directions on bit
//     planes and their sum (4 planes), the partner's sum added through DPP (the
//     totals are exact integers: any order of the adds gives k_play_rand's).
// k_play_rand<8, GREEDY> issues about 567 VALU per wave and ply from one wave per
// SIMD at 65,536 boards, of which the flip counts are about 330: split, each
// lane's stream is shorter and two waves share each SIMD.
#pragma once

#include "device.hpp"
#include "ply.hpp"

namespace oth_dev {

template <int N>
struct PairGreedy {
    static_assert(Geo<N>::W == 1, "one-word boards");
    static constexpr uint64_t BD = Geo<N>::BOARD.w[0], IN = Geo<N>::INNER.w[0];
    const uint64_t* up;    // LDS ray table rows of this lane's up directions 2h, 2h + 1 (Fills' layout)
    const uint64_t* down;  // and of its turned down directions 4 + 2h, 5 + 2h
    uint32_t s0, s1;       // the lane's axis steps: h = 0: 1, N; h = 1: N + 1, N - 1
    uint64_t m1;           // axis 1's propagator mask (S/N: the whole board)
    mutable uint64_t tu[2], td[2];  // fills of ray directions 2h + j (up) and 4 + 2h + j (down)

    __device__ __forceinline__ PairGreedy(int h, const uint64_t* lds) {
        up = lds + 128 * h;
        down = lds + 256 + 128 * h;
        s0 = h ? N + 1u : 1u;
        s1 = h ? N - 1u : (uint32_t)N;
        m1 = h ? IN : BD;
    }
    // one axis of step s through propagator p1: the squares one step past the
    // fills (both directions), the fill reached stepping +s (ray direction -s:
    // a down fill) and -s (ray direction +s: an up fill); 1 + 1 + 2 + 2 doubling
    __device__ __forceinline__ static uint64_t axis(uint64_t P, uint64_t p1, uint32_t s, uint64_t& tdn,
                                                    uint64_t& tup) {
        const uint64_t p2 = p1 & (p1 << s);
        uint64_t x = (P << s) & p1;
        x = and_or_64(p1, x << s, x);
        x = and_or_64(p2, x << (2 * s), x);
        x = and_or_64(p2, x << (2 * s), x);
        tdn = x;
        const uint64_t l = x << s;
        const uint64_t p2m = p2 >> s;
        x = (P >> s) & p1;
        x = and_or_64(p1, x >> s, x);
        x = and_or_64(p2m, x >> (2 * s), x);
        x = and_or_64(p2m, x >> (2 * s), x);
        tup = x;
        return l | (x >> s);
    }
    // get_possible_actions (othello.py:313-343) for the mover P; the lane's fills kept
    __device__ __forceinline__ uint64_t legal(uint64_t P, uint64_t O) const {
        const uint64_t L = axis(P, O & IN, s0, td[0], tu[0]) | axis(P, O & m1, s1, td[1], tu[1]);
        return pair_or(L) & ~(P | O) & BD;
    }
    // update_board's flips (othello.py:391-410) from square a (Fills::flip's form)
    __device__ __forceinline__ uint64_t flip(int a) const {
        uint64_t f = 0, g = 0;
#pragma unroll
        for (int j = 0; j < 2; ++j) {
            const uint64_t ray = up[64 * j + a], t = tu[j];
            f |= and3_64(ray, t, (ray & ~t) - 1ull);
        }
#pragma unroll
        for (int j = 0; j < 2; ++j) {
            const uint64_t ray = down[64 * j + a], tt = OneWord<N>::turn180(td[j]);
            g |= and3_64(ray, tt, (ray & ~tt) - 1ull);
        }
        return pair_or(f | OneWord<N>::turn180(g));
    }
    // OneWord::run_len for a step s held in a register: toward higher squares
    // (UP) the sets shift down, toward lower squares up
    template <bool UP>
    __device__ __forceinline__ static void run_len(uint64_t T, uint32_t s, uint64_t out[3]) {
        constexpr int R = N - 2;
        auto sh = [&](uint64_t x, uint32_t k) __attribute__((always_inline)) { return UP ? x >> k : x << k; };
        const uint64_t A1 = sh(T, s);
        uint64_t A2 = 0, A3 = 0, A4 = 0, A5 = 0, A6 = 0;
        if constexpr (R >= 2) A2 = A1 & sh(A1, s);
        if constexpr (R >= 3) A3 = A2 & sh(A1, 2 * s);
        if constexpr (R >= 4) A4 = A2 & sh(A2, 2 * s);
        if constexpr (R >= 5) A5 = A4 & sh(A1, 4 * s);
        if constexpr (R >= 6) A6 = A4 & sh(A2, 4 * s);
        out[0] = xor3_64(xor3_64(A1, A2, A3), A4, A5) ^ A6;
        out[1] = (A2 ^ A4) | A6;
        out[2] = A4;
    }
    // GreedyPolicy.get_action (simple_policies.py:69-92) for the side to move:
    // the lane's two axes' flip counts (4 planes), the partner's added (5
    // planes), the largest total among the candidates plane by plane, lowest
    // square on ties (np.argmax); -1 without candidates
    __device__ __forceinline__ int greedy(uint64_t legal) const {
        uint64_t n[4][3], s3[2][3], s4[4], q[4], tot[5];
        run_len<true>(tu[0], s0, n[0]);
        run_len<false>(td[0], s0, n[1]);
        run_len<true>(tu[1], s1, n[2]);
        run_len<false>(td[1], s1, n[3]);
        OneWord<N>::template add_planes<3, 3, 3>(n[0], n[1], s3[0]);  // an axis' two runs: <= N - 2, 3 bits
        OneWord<N>::template add_planes<3, 3, 3>(n[2], n[3], s3[1]);
        OneWord<N>::template add_planes<3, 3, 4>(s3[0], s3[1], s4);
#pragma unroll
        for (int i = 0; i < 4; ++i) {  // the partner's planes (quad_perm [1,0,3,2])
            const uint32_t lo = (uint32_t)s4[i], hi = (uint32_t)(s4[i] >> 32);
            const uint32_t plo = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)lo, 0xB1, 0xF, 0xF, false);
            const uint32_t phi = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)hi, 0xB1, 0xF, 0xF, false);
            q[i] = ((uint64_t)phi << 32) | plo;
        }
        OneWord<N>::template add_planes<4, 4, 5>(s4, q, tot);
        uint64_t cand = legal;
#pragma unroll
        for (int i = 4; i >= 0; --i) {
            const uint64_t hh = cand & tot[i];
            cand = hh ? hh : cand;
        }
        return cand ? __builtin_ctzll(cand) : -1;
    }
};

// k_play_rand<N, GREEDY> on lane pairs: the same plies, draws and outputs (both
// lanes of a pair store the same values to the same addresses).
template <int N>
__global__ __launch_bounds__(BLOCK) void k_play_greedy2(uint64_t* __restrict__ boards, uint16_t* __restrict__ meta,
                                                        uint64_t* __restrict__ legal, int E, uint32_t flags,
                                                        int plies, int32_t* __restrict__ actions,
                                                        int32_t* __restrict__ rewards, uint8_t* __restrict__ dones,
                                                        unsigned long long* __restrict__ wdl, Rng rng, uint64_t ply0,
                                                        const uint64_t* __restrict__ tables) {
    static_assert(Geo<N>::W == 1, "one-word boards");
    static_assert(BLOCK == 256 && Fills<N>::RAY_WORDS == 2 * BLOCK, "two ray words and one sel8 word a thread");
    constexpr uint64_t BD = Geo<N>::BOARD.w[0];
    constexpr int NN = N * N;
    ply0 += *rng.ply_off;  // graph-region offset (oth_graph_end); 0 eagerly
    __shared__ __attribute__((aligned(16))) uint64_t lds_rays[Fills<N>::RAY_WORDS];
    __shared__ __attribute__((aligned(16))) uint64_t lds_sel[256];
    const uint8_t* sel8 = reinterpret_cast<const uint8_t*>(lds_sel);
    const int gt = blockIdx.x * BLOCK + threadIdx.x;
    const int e = gt >> 1, h = gt & 1;
    Lane<N> s;
    const ulonglong2 tr = reinterpret_cast<const ulonglong2*>(tables)[threadIdx.x];
    const uint64_t ts = tables[Fills<N>::RAY_WORDS + threadIdx.x];
    if (e < E) load_lane<N>(s, boards, meta, legal, e);
    reinterpret_cast<ulonglong2*>(lds_rays)[threadIdx.x] = tr;
    lds_sel[threadIdx.x] = ts;
    __syncthreads();
    uint32_t cb = 0, cd = 0, cw = 0;
    if (e < E) {  // pair-uniform
        const uint32_t id = rng.id_base + (uint32_t)e;
        const bool tw0 = (s.meta & M_TURN_WHITE) != 0;
        uint64_t M = tw0 ? s.white.w[0] : s.black.w[0];
        uint64_t O = tw0 ? s.black.w[0] : s.white.w[0];
        uint64_t L = s.legal.w[0];
        uint32_t mt = s.meta & (0xff00u | M_TURN_WHITE);
        const bool slow = __any((s.meta & M_TERMINATED) != 0 || L == 0);
        if (!slow) {
            const PairGreedy<N> eng(h, lds_rays);
            (void)eng.legal(M, O);  // the mover's fills
            // the start position's fills of this lane's directions (the auto-reset's)
            constexpr StartFills<N> SF = start_fills<N>();
            const uint64_t st_u0 = h ? SF.t[2] : SF.t[0], st_u1 = h ? SF.t[3] : SF.t[1];
            const uint64_t st_d0 = h ? SF.t[6] : SF.t[4], st_d1 = h ? SF.t[7] : SF.t[5];
            int32_t* act_p = actions + e;
            int32_t* rew_p = rewards + e;
            uint8_t* done_p = dones + e;
            uint32_t t0 = 0, t1 = 0, t2 = 0;  // (sum of black's signs, games, decided games)
            auto ply = [&](int p, uint32_t u, bool open) __attribute__((always_inline)) {
                const uint64_t g = ply0 + (uint64_t)p;
                int a;
                if (open && (mt & 0xff00u)) a = select64_tab(L, scale_index(u, popc64(L)), sel8);
                else a = eng.greedy(L);
                if (open) mt -= (mt & 0xff00u) ? (1u << M_RAND_SHIFT) : 0u;  // a random-opening ply used up
                const uint64_t m = 1ull << a;
                const uint64_t f = eng.flip(a);  // update_board (othello.py:391-410)
                const uint64_t Mn = M | f | m, On = O & ~f;
                const bool full = (Mn | On) == BD;  // :425-426
                uint64_t Ln = eng.legal(On, Mn);    // the opponent's possible_moves (:436)
                const bool pass = Ln == 0 && !full;
                if (pass) Ln = eng.legal(Mn, On);  // :437-440 (pair-uniform)
                const bool term = full || Ln == 0;
                const bool swap = !pass && !full;
                M = swap ? On : Mn;
                O = swap ? Mn : On;
                L = Ln;
                mt ^= swap ? M_TURN_WHITE : 0u;
                int r = 0;
                if (term) {
                    const int pc = popc64(Mn), oc = popc64(On), df = pc - oc;
                    const int sg = sign_i32(df);
                    if (flags & OTH_DISK_REWARD) r = oc == 0 ? NN : df;  // :446-459
                    else r = sg;
                    const int mw = -(int)(mt & M_TURN_WHITE);  // the mover (the turn is not passed on)
                    const int sb = (sg ^ mw) - mw;
                    t0 += (uint32_t)sb;
                    t1 += 1u;
                    t2 += (uint32_t)__mul24(sb, sb);
                    M = Start<N>::BLACK.w[0];  // auto-reset (othello.py:256-271)
                    O = Start<N>::WHITE.w[0];
                    constexpr uint64_t START_MOVES = start_moves<N>();
                    L = START_MOVES;
                    eng.tu[0] = st_u0;
                    eng.tu[1] = st_u1;
                    eng.td[0] = st_d0;
                    eng.td[1] = st_d1;
                    uint32_t rl = 0;
                    if (rng.init_rand > 0)
                        rl = (uint32_t)scale_index(philox_x(rng.seed, id, g, RNG_OPENING_AUTO), rng.init_rand / 2 + 1) *
                             2u;
                    mt = (rl & 0xffu) << M_RAND_SHIFT;
                }
                __builtin_nontemporal_store(a, act_p);
                __builtin_nontemporal_store(r, rew_p);
                __builtin_nontemporal_store((uint8_t)(term ? 1 : 0), done_p);
                act_p += E;
                rew_p += E;
                done_p += E;
            };
            if (rng.init_rand == 0 && !__any((mt & 0xff00u) != 0)) {
                for (int p = 0; p < plies; ++p) ply(p, 0u, false);
            } else {
                // opening plies draw word g % 4 of Philox block g / 4 (action_draw's value),
                // the block computed at the group's first ply some board of the wave needs it
                U4 blk{0u, 0u, 0u, 0u};
                uint64_t held = ~0ull;
                for (int p = 0; p < plies; ++p) {
                    const uint64_t g = ply0 + (uint64_t)p;
                    if ((g >> 2) != held && __any((mt & 0xff00u) != 0)) {
                        blk = philox4(rng.seed, id, g >> 2, RNG_ACTION);
                        held = g >> 2;
                    }
                    ply(p, pick4(blk, (uint32_t)(g & 3)), true);
                }
            }
            if (h == 0) tally_from_signs(t0, t1, t2, cb, cd, cw);
            const bool tw = (mt & M_TURN_WHITE) != 0;
            s.white.w[0] = tw ? M : O;
            s.black.w[0] = tw ? O : M;
            s.legal.w[0] = L;
            s.meta = mt;
        } else if (h == 0) {  // a board loaded terminated, or live without a move: k_play's loop
            const Fills<N> eng(0, lds_rays);
            eng.prime(s);
            for (int p = 0; p < plies; ++p) {
                const uint64_t g = ply0 + (uint64_t)p;
                int a = -1, r = 0, d = 1, win = NO_DISK;
                if (!(s.meta & M_TERMINATED)) {
                    if ((s.meta >> M_RAND_SHIFT) > 0)
                        a = random_action<N>(s, action_draw(rng.seed, id, g));
                    else
                        a = policy_action<N, OTH_POLICY_GREEDY>(s, eng);
                    if ((s.meta >> M_RAND_SHIFT) > 0) s.meta -= 1u << M_RAND_SHIFT;
                    step_lane<N, Fills<N>, true>(s, a, flags, r, d, win, eng);
                    if (d) {
                        cb += win == BLACK_DISK;
                        cd += win == NO_DISK;
                        cw += win == WHITE_DISK;
                        reset_lane<N>(s, rng.seed, id, g, RNG_OPENING_AUTO, rng.init_rand);
                        eng.prime(s);
                    }
                }
                actions[(size_t)p * E + e] = a;
                rewards[(size_t)p * E + e] = r;
                dones[(size_t)p * E + e] = (uint8_t)d;
            }
        }
        if (h == 0) store_lane<N>(s, boards, meta, legal, e);
    }
    tally(wdl, cb, cd, cw);
}

}  // namespace oth_dev
