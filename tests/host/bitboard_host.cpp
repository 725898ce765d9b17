// Host build of csrc/bitboard.hpp (the same templates the kernels use) for CPU
// tests: legal_moves<N> / flips<N> / select_bit / philox4 and the one-word
// fills scan + bit-plane greedy (OneWord<N>) exported with C linkage.
// Built by tests/test_bitboard_host.py with g++; test infrastructure only.
#include <stdint.h>
#include <string.h>

#include "../../gymothelloenv_amd/csrc/bitboard.hpp"

using namespace oth;

template <int N>
static void legal_n(int E, const uint64_t* mover, const uint64_t* opp, uint64_t* out) {
    constexpr int W = Geo<N>::W;
    for (int e = 0; e < E; ++e) {
        BB<W> P, O;
        for (int i = 0; i < W; ++i) {
            P.w[i] = mover[e * W + i];
            O.w[i] = opp[e * W + i];
        }
        BB<W> L = legal_moves<N>(P, O);
        memcpy(out + e * W, L.w, sizeof(L.w));
    }
}

template <int N>
static void flips_n(int E, const uint64_t* mover, const uint64_t* opp, const int32_t* sq, uint64_t* out) {
    constexpr int W = Geo<N>::W;
    for (int e = 0; e < E; ++e) {
        BB<W> P, O;
        for (int i = 0; i < W; ++i) {
            P.w[i] = mover[e * W + i];
            O.w[i] = opp[e * W + i];
        }
        BB<W> f = flips<N>(P, O, square<W>(sq[e]));
        memcpy(out + e * W, f.w, sizeof(f.w));
    }
}

template <int N>
static void legal_fills_n(int E, const uint64_t* mover, const uint64_t* opp, uint64_t* out, uint64_t* fills) {
    for (int e = 0; e < E; ++e) out[e] = OneWord<N>::legal(mover[e], opp[e], fills + 8 * e);
}

template <int N>
static void greedy_planes_n(int E, const uint64_t* mover, const uint64_t* opp, const uint64_t* legal, int32_t* out) {
    for (int e = 0; e < E; ++e) {
        uint64_t t[8];
        (void)OneWord<N>::legal(mover[e], opp[e], t);
        out[e] = OneWord<N>::greedy(t, legal[e]);
    }
}

// legal_moves_fills + flips_fills (the multi-word fills engine) from every
// square a with legal[a] set: out[e * W * NN + a * W ..] = the flips (0 elsewhere)
template <int N>
static void fills_flips_n(int E, const uint64_t* mover, const uint64_t* opp, uint64_t* legal, uint64_t* out) {
    constexpr int W = Geo<N>::W;
    constexpr int NN = N * N;
    static BB<W> rays[8 * NN];
    for (int d = 0; d < 8; ++d)
        for (int a = 0; a < NN; ++a) rays[d * NN + a] = ray_from<N>(d, a);
    for (int e = 0; e < E; ++e) {
        BB<W> P, O, t[8];
        for (int i = 0; i < W; ++i) {
            P.w[i] = mover[e * W + i];
            O.w[i] = opp[e * W + i];
        }
        const BB<W> L = legal_moves_fills<N>(P, O, t);
        memcpy(legal + e * W, L.w, sizeof(L.w));
        for (int a = 0; a < NN; ++a) {
            BB<W> f = zero<W>();
            if ((L.w[a / 64] >> (a % 64)) & 1u) f = flips_fills<N>(rays, t, a);
            memcpy(out + ((size_t)e * NN + a) * W, f.w, sizeof(f.w));
        }
    }
}

// PlanesW<N>::greedy from legal_moves_fills (multi-word GreedyPolicy on bit planes)
template <int N>
static void greedy_planes_w_n(int E, const uint64_t* mover, const uint64_t* opp, const uint64_t* legal, int32_t* out) {
    constexpr int W = Geo<N>::W;
    for (int e = 0; e < E; ++e) {
        BB<W> P, O, L, t[8];
        for (int i = 0; i < W; ++i) {
            P.w[i] = mover[e * W + i];
            O.w[i] = opp[e * W + i];
            L.w[i] = legal[e * W + i];
        }
        (void)legal_moves_fills<N>(P, O, t);
        out[e] = PlanesW<N>::greedy(t, L);
        out[E + e] = PlanesW<N>::max_flips(t, L);
    }
}


#define DISPATCH8(fn, ...)                 \
    switch (n) {                           \
        case 4: fn<4>(__VA_ARGS__); break; \
        case 5: fn<5>(__VA_ARGS__); break; \
        case 6: fn<6>(__VA_ARGS__); break; \
        case 7: fn<7>(__VA_ARGS__); break; \
        case 8: fn<8>(__VA_ARGS__); break; \
        default: return -1;                \
    }

#define DISPATCH(fn, ...)                \
    switch (n) {                         \
        case 4: fn<4>(__VA_ARGS__); break;   \
        case 5: fn<5>(__VA_ARGS__); break;   \
        case 6: fn<6>(__VA_ARGS__); break;   \
        case 7: fn<7>(__VA_ARGS__); break;   \
        case 8: fn<8>(__VA_ARGS__); break;   \
        case 9: fn<9>(__VA_ARGS__); break;   \
        case 10: fn<10>(__VA_ARGS__); break; \
        case 11: fn<11>(__VA_ARGS__); break; \
        case 12: fn<12>(__VA_ARGS__); break; \
        case 13: fn<13>(__VA_ARGS__); break; \
        case 14: fn<14>(__VA_ARGS__); break; \
        case 15: fn<15>(__VA_ARGS__); break; \
        case 16: fn<16>(__VA_ARGS__); break; \
        default: return -1;              \
    }

extern "C" {
int host_legal(int n, int E, const uint64_t* mover, const uint64_t* opp, uint64_t* out) {
    DISPATCH(legal_n, E, mover, opp, out);
    return 0;
}
int host_flips(int n, int E, const uint64_t* mover, const uint64_t* opp, const int32_t* sq, uint64_t* out) {
    DISPATCH(flips_n, E, mover, opp, sq, out);
    return 0;
}
int host_fills_flips(int n, int E, const uint64_t* mover, const uint64_t* opp, uint64_t* legal, uint64_t* out) {
    DISPATCH(fills_flips_n, E, mover, opp, legal, out);
    return 0;
}
int host_greedy_planes_w(int n, int E, const uint64_t* mover, const uint64_t* opp, const uint64_t* legal,
                         int32_t* out) {
    DISPATCH(greedy_planes_w_n, E, mover, opp, legal, out);
    return 0;
}
int host_legal_fills(int n, int E, const uint64_t* mover, const uint64_t* opp, uint64_t* out, uint64_t* fills) {
    DISPATCH8(legal_fills_n, E, mover, opp, out, fills);
    return 0;
}
int host_greedy_planes(int n, int E, const uint64_t* mover, const uint64_t* opp, const uint64_t* legal, int32_t* out) {
    DISPATCH8(greedy_planes_n, E, mover, opp, legal, out);
    return 0;
}
int host_select(uint64_t x, int k) { return select64(x, k); }
// select64_tab with the sel8 table as k_play_rand stages it in LDS
int host_select_tab(uint64_t x, int k) {
    static uint64_t tab[256];
    static bool init = false;
    if (!init) {
        for (int i = 0; i < 256; ++i) tab[i] = sel8_word((uint32_t)i);
        init = true;
    }
    return select64_tab(x, k, reinterpret_cast<const uint8_t*>(tab));
}
// select_bit_tab (the multi-word branch-free random pick) on W = 2..4 words
int host_select_tab_w(const uint64_t* words, int W, int k) {
    static uint64_t tab[256];
    static bool init = false;
    if (!init) {
        for (int i = 0; i < 256; ++i) tab[i] = sel8_word((uint32_t)i);
        init = true;
    }
    const uint8_t* t = reinterpret_cast<const uint8_t*>(tab);
    BB<4> b;
    for (int i = 0; i < 4; ++i) b.w[i] = i < W ? words[i] : 0;
    if (W == 2) return select_bit_tab<2>(*reinterpret_cast<const BB<2>*>(b.w), k, t);
    if (W == 3) return select_bit_tab<3>(*reinterpret_cast<const BB<3>*>(b.w), k, t);
    return select_bit_tab<4>(b, k, t);
}
void host_philox4(uint64_t seed, uint32_t id, uint64_t ctr, uint32_t purpose, uint32_t* out) {
    U4 u = philox4(seed, id, ctr, purpose);
    out[0] = u.x;
    out[1] = u.y;
    out[2] = u.z;
    out[3] = u.w;
}
}
