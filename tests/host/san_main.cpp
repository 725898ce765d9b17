// Sanitizer driver (host code only): the oracle (oracle/othello_oracle.c) and
// the bitboard CPU engine (oracle/cpu_bitboard.cpp, i.e. bitboard.hpp on the
// host) built with -fsanitize=address,undefined into one executable and driven
// through every exported entry point for N = 4..16, including invalid and
// out-of-range actions, terminal boards and boards with no recorded moves.
// Built and run by tests/test_sanitizers.py.  Exit 0 = clean and consistent.
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <vector>

extern "C" {
int oracle_nwords(int n);
void oracle_reset_batch(int n, int E, uint64_t* boards, uint16_t* meta, uint64_t* legal);
void oracle_legal_batch(int n, int E, const uint64_t* mover, const uint64_t* opp, uint64_t* out);
int oracle_step_batch(int n, uint32_t flags, uint64_t seed, uint32_t id_base, uint64_t ply, int irs, int E,
                      uint64_t* boards, uint16_t* meta, uint64_t* legal, const int32_t* actions, int32_t* rewards,
                      uint8_t* dones, int64_t* wdl);
void oracle_reset_openings(int n, int E, uint64_t seed, uint32_t id_base, uint64_t ply, int irs, uint64_t* boards,
                           uint16_t* meta, uint64_t* legal);
int oracle_rollout(int n, uint32_t flags, int policy, int irs, uint64_t seed, uint32_t id_base, uint64_t ply0, int E,
                   int plies, uint64_t* boards, uint16_t* meta, uint64_t* legal, int32_t* actions, int32_t* rewards,
                   uint8_t* dones, int64_t* wdl);
void oracle_greedy_batch(int n, int E, const uint64_t* boards, const uint16_t* meta, const uint64_t* legal,
                         int32_t* out);
void oracle_recompute_legal(int n, int E, const uint64_t* boards, const uint16_t* meta, uint64_t* legal);
void oracle_observe(int n, int E, const uint64_t* boards, const uint16_t* meta, const uint64_t* legal, int8_t* obs,
                    int8_t* obs2, float* ms);
void oracle_maximin_batch(int n, int depth, int E, const uint64_t* boards, const uint16_t* meta,
                          const uint64_t* legal, int32_t* out);
void oracle_reset_vs(int n, uint32_t flags, int policy, int irs, uint64_t seed, uint32_t id_base, uint64_t call,
                     int E, const int8_t* prot, uint64_t* boards, uint16_t* meta, uint64_t* legal);
void oracle_step_vs(int n, uint32_t flags, int policy, int irs, uint64_t seed, uint32_t id_base, uint64_t call, int E,
                    const int8_t* prot, const int32_t* actions, uint64_t* boards, uint16_t* meta, uint64_t* legal,
                    int32_t* rewards, uint8_t* dones, int32_t* plies, int64_t* wdl);
int64_t cpu_bb_rollout(int n, uint64_t seed, uint32_t id_base, uint64_t ply0, int E, int plies, uint64_t* boards,
                       uint16_t* meta, uint64_t* legal, int32_t* actions, int32_t* rewards, uint8_t* dones,
                       int64_t* wdl);
}

#define CHECK(c)                                                    \
    do {                                                            \
        if (!(c)) {                                                 \
            fprintf(stderr, "FAILED %s at line %d (n=%d)\n", #c, __LINE__, n); \
            return 1;                                               \
        }                                                           \
    } while (0)

static uint32_t rng = 12345u;
static uint32_t next_u32() {
    rng ^= rng << 13;
    rng ^= rng >> 17;
    rng ^= rng << 5;
    return rng;
}

static int run_size(int n) {
    const int W = oracle_nwords(n), E = 64, NN = n * n;
    std::vector<uint64_t> b(E * 2 * W), l(E * W), b2, l2;
    std::vector<uint16_t> m(E), m2;
    std::vector<int32_t> a(E), r(E), pl(E), acts(E * 40), rews(E * 40), acts2(E * 40), rews2(E * 40);
    std::vector<uint8_t> d(E), dn(E * 40), dn2(E * 40);
    int64_t wdl[3] = {0, 0, 0}, wdl2[3] = {0, 0, 0};
    // random play: oracle vs bitboard engine
    oracle_reset_batch(n, E, b.data(), m.data(), l.data());
    b2 = b, m2 = m, l2 = l;
    oracle_rollout(n, 5u, 0, 0, 9, 0, 0, E, 40, b.data(), m.data(), l.data(), acts.data(), rews.data(), dn.data(),
                   wdl);
    cpu_bb_rollout(n, 9, 0, 0, E, 40, b2.data(), m2.data(), l2.data(), acts2.data(), rews2.data(), dn2.data(), wdl2);
    CHECK(acts == acts2 && rews == rews2 && dn == dn2 && b == b2 && m == m2 && l == l2);
    CHECK(wdl[0] == wdl2[0] && wdl[1] == wdl2[1] && wdl[2] == wdl2[2]);
    // external actions incl. invalid and out-of-range, every flag combination
    for (uint32_t flags = 0; flags < 8; ++flags) {
        oracle_reset_openings(n, E, 1, 0, 0, 6, b.data(), m.data(), l.data());
        for (int p = 0; p < 3 * NN; ++p) {
            for (int i = 0; i < E; ++i) {
                const uint32_t u = next_u32();
                a[i] = (u & 7) == 0 ? (int32_t)(u % (NN + 20)) - 10 : (int32_t)(u % NN);
            }
            oracle_step_batch(n, flags, 1, 0, p, 6, E, b.data(), m.data(), l.data(), a.data(), r.data(), d.data(),
                              wdl);
        }
    }
    // scripted policies, observations, stateless legal moves
    oracle_reset_openings(n, E, 2, 0, 0, 10, b.data(), m.data(), l.data());
    oracle_rollout(n, 5u, 1, 10, 2, 0, 0, E, 12, b.data(), m.data(), l.data(), nullptr, nullptr, nullptr, wdl);
    oracle_greedy_batch(n, E, b.data(), m.data(), l.data(), a.data());
    if (n <= 8) oracle_maximin_batch(n, 2, E, b.data(), m.data(), l.data(), a.data());
    oracle_recompute_legal(n, E, b.data(), m.data(), l2.data());
    std::vector<int8_t> obs(E * NN), obs2(E * 2 * NN);
    std::vector<float> ms(E * 4 * NN);
    oracle_observe(n, E, b.data(), m.data(), l.data(), obs.data(), obs2.data(), ms.data());
    std::vector<uint64_t> mv(E * W), op(E * W), out(E * W);
    for (int i = 0; i < E; ++i)
        for (int w = 0; w < W; ++w) {
            mv[i * W + w] = b[i * 2 * W + w];
            op[i * W + w] = b[i * 2 * W + W + w];
        }
    oracle_legal_batch(n, E, mv.data(), op.data(), out.data());
    // boards with no recorded moves take the invalid path (no stale read)
    std::fill(l.begin(), l.end(), 0ull);
    oracle_rollout(n, 1u, 0, 0, 3, 0, 0, E, 1, b.data(), m.data(), l.data(), a.data(), r.data(), d.data(), wdl);
    for (int i = 0; i < E; ++i) CHECK(a[i] == -1);
    // OthelloEnv with an embedded opponent
    std::vector<int8_t> prot(E);
    for (int i = 0; i < E; ++i) prot[i] = (i & 1) ? 1 : -1;
    for (int pol = 0; pol <= (n <= 8 ? 2 : 1); ++pol) {
        oracle_reset_vs(n, 5u, pol, 4, 7, 0, 0, E, prot.data(), b.data(), m.data(), l.data());
        for (int p = 1; p < NN; ++p) {
            for (int i = 0; i < E; ++i) a[i] = (int32_t)(next_u32() % NN);
            oracle_step_vs(n, 4u, pol, 4, 7, 0, p, E, prot.data(), a.data(), b.data(), m.data(), l.data(), r.data(),
                           d.data(), pl.data(), wdl);
        }
    }
    return 0;
}

int main() {
    for (int n = 4; n <= 16; ++n) {
        if (run_size(n)) return 1;
    }
    printf("sanitized oracle + bitboard engine: N = 4..16 clean\n");
    return 0;
}
