// oracle/cpu_bitboard.cpp -- the "best CPU" baseline of SURVEY.md §8(d).
//
// TEST / BENCH INFRASTRUCTURE ONLY (bench.py's cpu_baseline leg and tests/):
// the product path never loads it.  Random play (RandomPolicy,
// simple_policies.py:37-41, with the device's Philox stream) over E boards in
// the exchange format, stepped with bitboards on the host: the same shift/mask
// rules templates the kernels use (gymothelloenv_amd/csrc/bitboard.hpp, built
// here by g++) in place of the reference's per-cell ray walk
// (othello.py:273-343).  Step semantics follow othello.py:412-462 for a legal
// move (a random pick is always legal): flip, full-board terminal, pass,
// double pass, winner by counts; finished games auto-reset (oth_step_policy
// with OTH_AUTO_RESET, no random openings).  tests/test_cpu_baseline.py checks
// its actions, rewards, dones and final state against the scalar oracle.
#include <stdint.h>
#include <string.h>

#include "../gymothelloenv_amd/csrc/bitboard.hpp"

using namespace oth;

namespace {

template <int N>
int64_t rollout_n(uint64_t seed, uint32_t id_base, uint64_t ply0, int E, int plies, uint64_t* boards,
                  uint16_t* meta, uint64_t* legal, int32_t* actions, int32_t* rewards, uint8_t* dones,
                  int64_t* wdl) {
    constexpr int W = Geo<N>::W;
    const BB<W> full = Geo<N>::BOARD;
    int64_t steps = 0;
    for (int i = 0; i < E; ++i) {
        const uint32_t id = id_base + (uint32_t)i;
        BB<W> blk, wht, L;
        for (int k = 0; k < W; ++k) {
            blk.w[k] = boards[(size_t)i * 2 * W + k];
            wht.w[k] = boards[(size_t)i * 2 * W + W + k];
            L.w[k] = legal[(size_t)i * W + k];
        }
        bool white = meta[i] & 1u, term = (meta[i] >> 1) & 1u;
        int winner = (meta[i] >> 2) & 3;
        for (int p = 0; p < plies; ++p) {
            const uint64_t g = ply0 + (uint64_t)p;
            int a = -1, r = 0, d = 1;
            if (!term) {
                ++steps;
                const int cnt = popcount(L);
                a = select_bit(L, scale_index(action_draw(seed, id, g), cnt));
                BB<W>& M = white ? wht : blk;
                BB<W>& O = white ? blk : wht;
                const BB<W> m = square<W>(a);
                const BB<W> f = flips<N>(M, O, m);
                M = M | f | m;
                O = O & ~f;
                bool done = !any(full & ~(M | O));
                if (!done) {
                    const BB<W> L2 = legal_moves<N>(O, M);
                    if (any(L2)) {
                        white = !white;
                        L = L2;
                    } else {
                        L = legal_moves<N>(M, O);  // pass: the mover moves again
                        done = !any(L);
                    }
                }
                d = done;
                if (done) {
                    const int nb = popcount(blk), nw = popcount(wht);
                    winner = nw > nb ? 1 : (nb > nw ? 2 : 0);  // othello.py:473-501
                    // reward = winner * mover; `white` is still the mover on both terminal paths
                    const int wv = winner == 1 ? 1 : (winner == 2 ? -1 : 0);
                    r = wv * (white ? 1 : -1);
                    wdl[winner == 2 ? 0 : (winner == 0 ? 1 : 2)]++;
                    // auto-reset (othello.py:256-271)
                    blk = zero<W>();
                    wht = zero<W>();
                    const int c = N / 2;
                    wht = wht | square<W>((c - 1) * N + (c - 1)) | square<W>(c * N + c);
                    blk = blk | square<W>(c * N + (c - 1)) | square<W>((c - 1) * N + c);
                    white = false;
                    winner = 0;
                    L = legal_moves<N>(blk, wht);
                }
            }
            if (actions) actions[(size_t)p * E + i] = a;
            if (rewards) rewards[(size_t)p * E + i] = r;
            if (dones) dones[(size_t)p * E + i] = (uint8_t)d;
        }
        for (int k = 0; k < W; ++k) {
            boards[(size_t)i * 2 * W + k] = blk.w[k];
            boards[(size_t)i * 2 * W + W + k] = wht.w[k];
            legal[(size_t)i * W + k] = L.w[k];
        }
        meta[i] = (uint16_t)((white ? 1u : 0u) | (term ? 2u : 0u) | ((unsigned)winner << 2));
    }
    return steps;
}

}  // namespace

extern "C" {
// Returns the number of env-steps taken (plies applied to live boards).
int64_t cpu_bb_rollout(int n, uint64_t seed, uint32_t id_base, uint64_t ply0, int E, int plies, uint64_t* boards,
                       uint16_t* meta, uint64_t* legal, int32_t* actions, int32_t* rewards, uint8_t* dones,
                       int64_t* wdl) {
#define OTH_CASE(K) \
    case K: return rollout_n<K>(seed, id_base, ply0, E, plies, boards, meta, legal, actions, rewards, dones, wdl);
    switch (n) {
        OTH_CASE(4) OTH_CASE(5) OTH_CASE(6) OTH_CASE(7) OTH_CASE(8) OTH_CASE(9) OTH_CASE(10)
        OTH_CASE(11) OTH_CASE(12) OTH_CASE(13) OTH_CASE(14) OTH_CASE(15) OTH_CASE(16)
        default: return -1;
    }
#undef OTH_CASE
}
}
