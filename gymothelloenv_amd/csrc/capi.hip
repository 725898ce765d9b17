// capi.hip -- the C ABI declared in include/othello_mi355x.h: argument checks,
// handle lifetime, error reporting and dispatch on the board size to the
// per-N launchers (kernels_n.hip).
#include <hip/hip_runtime.h>

#include <stdio.h>
#include <string.h>

#include <new>
#include <string>
#include <type_traits>

#include "device.hpp"
#include "launch.hpp"

using namespace oth;
using namespace oth_dev;
using namespace oth_host;

namespace oth_host {

thread_local std::string g_last_error;

int fail(int code, const char* msg) {
    g_last_error = msg;
    return code;
}

int hip_fail(hipError_t err, const char* where) {
    char buf[256];
    snprintf(buf, sizeof(buf), "%s: %s", where, hipGetErrorString(err));
    g_last_error = buf;
    return OTH_EHIP;
}

namespace {
thread_local hipError_t g_launch_err = hipSuccess;  // the first failed launch since after_launch
}

void note_launch(hipError_t err) {
    if (err != hipSuccess && g_launch_err == hipSuccess) g_launch_err = err;
}

int after_launch(const char* what) {
    hipError_t err = g_launch_err;
    g_launch_err = hipSuccess;
    const hipError_t last = hipGetLastError();  // (and clears HIP's own sticky status)
    if (err == hipSuccess) err = last;
    if (err != hipSuccess) return hip_fail(err, what);
    return OTH_OK;
}

}  // namespace oth_host

namespace {

#define OTH_HIP(call)                                         \
    do {                                                      \
        hipError_t err_ = (call);                             \
        if (err_ != hipSuccess) return hip_fail(err_, #call); \
    } while (0)

template <typename Fn>
int with_n(int n, Fn&& fn) {
    switch (n) {
        case 4: return fn(std::integral_constant<int, 4>{});
        case 5: return fn(std::integral_constant<int, 5>{});
        case 6: return fn(std::integral_constant<int, 6>{});
        case 7: return fn(std::integral_constant<int, 7>{});
        case 8: return fn(std::integral_constant<int, 8>{});
        case 9: return fn(std::integral_constant<int, 9>{});
        case 10: return fn(std::integral_constant<int, 10>{});
        case 11: return fn(std::integral_constant<int, 11>{});
        case 12: return fn(std::integral_constant<int, 12>{});
        case 13: return fn(std::integral_constant<int, 13>{});
        case 14: return fn(std::integral_constant<int, 14>{});
        case 15: return fn(std::integral_constant<int, 15>{});
        case 16: return fn(std::integral_constant<int, 16>{});
        default: return fail(OTH_EINVAL, "board_size must be in [4, 16]");
    }
}

int use_device(const oth_env* env) {
    int cur = -1;
    OTH_HIP(hipGetDevice(&cur));
    if (cur != env->device) OTH_HIP(hipSetDevice(env->device));
    return OTH_OK;
}

#define OTH_CHECK_ENV(env)                                    \
    do {                                                      \
        if (!(env)) return fail(OTH_EINVAL, "NULL oth_env");  \
        int rc_ = use_device(env);                            \
        if (rc_) return rc_;                                  \
    } while (0)

// oth_counts: sum the per-block slots into out[3] (int64); optionally zero them.
__global__ __launch_bounds__(256) void k_reduce_wdl(unsigned long long* __restrict__ wdl, int nslots,
                                                   int64_t* __restrict__ out, int reset) {
    __shared__ unsigned long long acc[256][3];
    unsigned long long b = 0, d = 0, w = 0;
    for (int i = threadIdx.x; i < nslots; i += 256) {
        b += wdl[4 * (size_t)i];
        d += wdl[4 * (size_t)i + 1];
        w += wdl[4 * (size_t)i + 2];
        if (reset) {
            wdl[4 * (size_t)i] = 0;
            wdl[4 * (size_t)i + 1] = 0;
            wdl[4 * (size_t)i + 2] = 0;
        }
    }
    acc[threadIdx.x][0] = b;
    acc[threadIdx.x][1] = d;
    acc[threadIdx.x][2] = w;
    __syncthreads();
    for (int s = 128; s > 0; s >>= 1) {
        if ((int)threadIdx.x < s) {
            acc[threadIdx.x][0] += acc[threadIdx.x + s][0];
            acc[threadIdx.x][1] += acc[threadIdx.x + s][1];
            acc[threadIdx.x][2] += acc[threadIdx.x + s][2];
        }
        __syncthreads();
    }
    if (threadIdx.x < 3) out[threadIdx.x] = (int64_t)acc[0][threadIdx.x];
}

// The leaves of one MaxiMin(d) search from a position with e empty squares:
// `root` moves at the root, then at most min(b, e - j) at level j, since every
// level places a disc (simple_policies.py:138) and a full board ends the game
// (:117-121); b = max(2, N*N / 6) moves per position (8x8 middle games: ~10).
double search_leaves(int d, int e, double root, double b) {
    double leaves = 1.0;
    for (int j = 0; j < d && j < e; ++j) {
        const double moves = j == 0 ? root : (b < e - j ? b : (double)(e - j));
        if (moves <= 0.0) break;  // no move: the search stops here (:120)
        leaves *= moves;
    }
    return leaves;
}

enum MaximinCall { MM_POLICY, MM_STEP_VS, MM_RESET_VS };

// MaxiMin searches of depth >= 3 are refused above OTH_MAXIMIN_LEAF_BUDGET
// estimated leaves per call.  First E x b^d x `searches` (the searches one board
// runs in the call: plies of oth_step_policy, opponent replies of the _vs calls);
// above the budget, the boards are read and each live board's search bounded by
// its own position (search_leaves: its empty squares, and its possible_moves at
// the root of a policy call), so late-game boards are searched at any depth the
// budget allows -- one 8x8 board with 10 empty squares at depth 10 is <= 10!
// leaves, where the position-blind estimate says 1.9e10.
int maximin_budget(const oth_env* env, int policy, double searches, MaximinCall call, hipStream_t st) {
    if (policy < OTH_POLICY_MAXIMIN(3) || policy > OTH_POLICY_LAST) return OTH_OK;
    const int d = policy - OTH_POLICY_MAXIMIN1 + 1, nn = env->n * env->n;
    const double b = nn / 6.0 > 2.0 ? nn / 6.0 : 2.0;
    double leaves = (double)env->E * searches;
    for (int i = 0; i < d; ++i) leaves *= b;
    if (leaves <= OTH_MAXIMIN_LEAF_BUDGET) return OTH_OK;
    const char* why = "";
    hipStreamCaptureStatus cap = hipStreamCaptureStatusNone;
    if (call == MM_RESET_VS) {
        why = " (reset_vs searches from the start position)";
    } else if (hipStreamIsCapturing(st, &cap) != hipSuccess || cap != hipStreamCaptureStatusNone) {
        why = " (during a stream capture the boards cannot be read for a position-aware estimate)";
    } else {
        const size_t E = (size_t)env->E, W = (size_t)env->W;
        uint64_t* bd = new (std::nothrow) uint64_t[E * 3 * W];
        uint16_t* meta = new (std::nothrow) uint16_t[E];
        if (!bd || !meta) {
            delete[] bd;
            delete[] meta;
            return fail(OTH_ENOMEM, "maximin budget: host allocation failed");
        }
        uint64_t* lg = bd + E * 2 * W;
        hipError_t err = hipMemcpyAsync(bd, env->boards, E * 2 * W * 8, hipMemcpyDeviceToHost, st);
        if (err == hipSuccess) err = hipMemcpyAsync(lg, env->legal, E * W * 8, hipMemcpyDeviceToHost, st);
        if (err == hipSuccess) err = hipMemcpyAsync(meta, env->meta, E * 2, hipMemcpyDeviceToHost, st);
        if (err == hipSuccess) err = hipStreamSynchronize(st);
        if (err != hipSuccess) {
            delete[] bd;
            delete[] meta;
            return hip_fail(err, "maximin budget: reading the boards");
        }
        // with auto-reset a board that ends is searched again from the start position
        const bool resets = (env->flags & OTH_AUTO_RESET) != 0;
        leaves = 0.0;
        for (size_t i = 0; i < E; ++i) {
            const bool done = (meta[i] & 2) != 0;
            if (done && !resets) continue;  // terminated: no search
            int discs = 0, moves = 0;
            for (size_t w = 0; w < 2 * W; ++w) discs += __builtin_popcountll(bd[i * 2 * W + w]);
            for (size_t w = 0; w < W; ++w) moves += __builtin_popcountll(lg[i * W + w]);
            const int e = nn - discs, later = resets && nn - 4 > e ? nn - 4 : e;
            const double rest = search_leaves(d, later, b < later ? b : (double)later, b);
            if (call == MM_POLICY && !done)  // the first search from this position, later plies from <= `later` empties
                leaves += search_leaves(d, e, (double)moves, b) + (searches - 1.0) * rest;
            else  // the opponent's replies after the protagonist's move (or searches after a reset)
                leaves += searches * rest;
        }
        delete[] bd;
        delete[] meta;
        if (leaves <= OTH_MAXIMIN_LEAF_BUDGET) return OTH_OK;
        why = " (bounded by each board's empty squares)";
    }
    char msg[320];
    snprintf(msg, sizeof(msg), "MaxiMin depth %d over %d boards of %dx%d (x%.0f searches) is ~%.1e leaves%s, above the "
             "budget of %.1e per call: split the boards over calls or search shallower", d, env->E, env->n, env->n,
             searches, leaves, why, (double)OTH_MAXIMIN_LEAF_BUDGET);
    return fail(OTH_EINVAL, msg);
}

}  // namespace

extern "C" {

const char* oth_last_error(void) { return g_last_error.c_str(); }

#ifndef OTH_SRC_HASH
#define OTH_SRC_HASH "0000000000000000000000000000000000000000000000000000000000000000"
#endif
// build.py passes the SHA-256 of the sources and flags; the loader compares it
// with the tree's sources (gymothelloenv_amd/build.py: embedded_hash)
const char* oth_version(void) { return "othello_mi355x 0.2 (gfx950) oth-src-sha256:" OTH_SRC_HASH; }

int oth_create(int32_t n_envs, int32_t board_size, uint32_t flags, uint64_t seed, uint32_t env_id_base,
               int32_t initial_rand_steps, int32_t device, oth_env** out) {
    if (!out) return fail(OTH_EINVAL, "out is NULL");
    *out = nullptr;
    if (n_envs <= 0) return fail(OTH_EINVAL, "n_envs must be > 0");
    const int n = board_size < 4 ? 4 : board_size;  // othello.py:230
    if (n > 16) return fail(OTH_EINVAL, "board_size must be <= 16");
    if (initial_rand_steps < 0 || initial_rand_steps > 255)
        return fail(OTH_EINVAL, "initial_rand_steps must be in [0, 255]");
    if (flags & ~7u) return fail(OTH_EINVAL, "unknown flag bits");
    OTH_HIP(hipSetDevice(device));
    oth_env* env = new (std::nothrow) oth_env();
    if (!env) return fail(OTH_ENOMEM, "host allocation failed");
    env->E = n_envs;
    env->n = n;
    env->W = (n * n + 63) / 64;
    env->flags = flags;
    env->seed = seed;
    env->id_base = env_id_base;
    env->init_rand = initial_rand_steps;
    env->device = device;
    env->ply = 0;
    const size_t E = (size_t)n_envs, W = (size_t)env->W;
    hipError_t err = hipMalloc((void**)&env->boards, E * 2 * W * sizeof(uint64_t));
    if (err == hipSuccess) err = hipMalloc((void**)&env->meta, ((E * sizeof(uint16_t) + 15) / 16) * 16);
    if (err == hipSuccess) err = hipMalloc((void**)&env->legal, E * W * sizeof(uint64_t));
    // one W/D/L slot per wave of the widest single-ply grid (k_sample_step4: 4 lanes per board) -- also
    // more than the per-block slots of every multi-ply launch
    env->nslots = (int32_t)((4 * (int64_t)E + 63) / 64);
    const size_t slot_bytes = (size_t)env->nslots * 4 * sizeof(unsigned long long);
    if (err == hipSuccess) err = hipMalloc((void**)&env->wdl, slot_bytes);
    if (err == hipSuccess) err = hipMemset(env->wdl, 0, slot_bytes);
    if (err == hipSuccess) err = hipMalloc((void**)&env->wdl_vs, slot_bytes);
    if (err == hipSuccess) err = hipMemset(env->wdl_vs, 0, slot_bytes);
    const size_t ctr_bytes = (size_t)OTH_GRAPH_SLOTS * 2 * sizeof(uint64_t);
    if (err == hipSuccess) err = hipMalloc((void**)&env->ctr_slots, ctr_bytes);
    if (err == hipSuccess) err = hipMemset(env->ctr_slots, 0, ctr_bytes);
    if (err == hipSuccess && env->W == 1) err = hipMalloc((void**)&env->rays, TABLE_WORDS * sizeof(uint64_t));
    env->cur_off = env->ctr_slots;
    env->graph_slot = 0;
    env->slots_used = 1;
    if (err != hipSuccess) {
        oth_destroy(env);
        return hip_fail(err, "oth_create: allocation");
    }
    int rc = with_n(n, [&](auto NC) { return launch_fill_rays<decltype(NC)::value>(env, nullptr); });
    if (rc == OTH_OK) rc = oth_reset(env, nullptr, nullptr);
    if (rc == OTH_OK) {
        err = hipStreamSynchronize(nullptr);
        if (err != hipSuccess) rc = hip_fail(err, "oth_create: reset");
    }
    if (rc != OTH_OK) {
        oth_destroy(env);
        return rc;
    }
    *out = env;
    return OTH_OK;
}

int oth_destroy(oth_env* env) {
    if (!env) return OTH_OK;
    (void)hipSetDevice(env->device);
    if (env->boards) (void)hipFree(env->boards);
    if (env->meta) (void)hipFree(env->meta);
    if (env->legal) (void)hipFree(env->legal);
    if (env->wdl) (void)hipFree(env->wdl);
    if (env->wdl_vs) (void)hipFree(env->wdl_vs);
    if (env->ctr_slots) (void)hipFree(env->ctr_slots);
    if (env->rays) (void)hipFree(env->rays);
    if (env->rec_host) (void)hipHostFree(env->rec_host);
    delete env;
    return OTH_OK;
}

int oth_reset(oth_env* env, const uint8_t* mask, oth_stream_t stream) {
    OTH_CHECK_ENV(env);
    return with_n(env->n, [&](auto NC) { return launch_reset<decltype(NC)::value>(env, mask, (hipStream_t)stream); });
}

int oth_step(oth_env* env, const int32_t* actions, int32_t* rewards, uint8_t* dones, oth_stream_t stream) {
    OTH_CHECK_ENV(env);
    if (!actions) return fail(OTH_EINVAL, "actions is NULL");
    const uint64_t ply = env->ply++;
    return with_n(env->n, [&](auto NC) {
        return launch_step<decltype(NC)::value>(env, actions, rewards, dones, ply, (hipStream_t)stream);
    });
}

int oth_step_observe(oth_env* env, const int32_t* actions, int32_t* rewards, uint8_t* dones, int32_t layout,
                     int32_t dtype, void* obs, oth_stream_t stream) {
    OTH_CHECK_ENV(env);
    if (!actions || !obs) return fail(OTH_EINVAL, "actions / obs is NULL");
    if (layout < OTH_OBS_BOARD || layout > OTH_OBS_LEGAL) return fail(OTH_EINVAL, "unknown layout");
    if (dtype < OTH_I8 || dtype > OTH_BF16) return fail(OTH_EINVAL, "unknown dtype");
    const uint64_t ply = env->ply++;
    return with_n(env->n, [&](auto NC) {
        return launch_step_observe<decltype(NC)::value>(env, actions, rewards, dones, layout, dtype, obs, ply,
                                                        (hipStream_t)stream);
    });
}

int oth_step_sync(oth_env* env, int32_t board, int32_t step, int32_t action, int32_t layout, const oth_record** out,
                  oth_stream_t stream) {
    OTH_CHECK_ENV(env);
    if (!out) return fail(OTH_EINVAL, "out is NULL");
    if (board < 0 || board >= env->E) return fail(OTH_EINVAL, "board out of range");
    if (layout != OTH_OBS_BOARD && layout != OTH_OBS_BOARD_LEGAL)
        return fail(OTH_EINVAL, "layout must be OTH_OBS_BOARD or OTH_OBS_BOARD_LEGAL");
    hipStreamCaptureStatus cap = hipStreamCaptureStatusNone;
    OTH_HIP(hipStreamIsCapturing((hipStream_t)stream, &cap));
    if (cap != hipStreamCaptureStatusNone)  // it waits for its record: never inside a graph capture
        return fail(OTH_EINVAL, "oth_step_sync waits for its result and cannot run during a stream capture");
    if (!env->rec_host) {  // mapped, coherent pinned host memory: the kernel's stores land in it directly
        void* h = nullptr;
        OTH_HIP(hipHostMalloc(&h, sizeof(oth_record), hipHostMallocMapped | hipHostMallocCoherent));
        memset(h, 0, sizeof(oth_record));
        void* d = nullptr;
        const hipError_t err = hipHostGetDevicePointer(&d, h, 0);
        if (err != hipSuccess) {
            (void)hipHostFree(h);
            return hip_fail(err, "oth_step_sync: hipHostGetDevicePointer");
        }
        env->rec_host = static_cast<oth_record*>(h);
        env->rec_dev = static_cast<oth_record*>(d);
        env->rec_seq = 0;
    }
    const uint32_t seq = ++env->rec_seq;
    const uint64_t ply = (step & 1) ? env->ply++ : env->ply;
    const int rc = with_n(env->n, [&](auto NC) {
        return launch_record<decltype(NC)::value>(env, board, step & (1 | OTH_RECORD_GREEDY), action,
                                                  layout == OTH_OBS_BOARD_LEGAL ? 2 : 1, ply, (hipStream_t)stream);
    });
    if (rc) return rc;
    // wait for the sequence number (the kernel writes it last, behind a system-scope
    // fence): no runtime synchronisation on the path; after a bounded spin the
    // stream is synchronised instead, which also reports a failed kernel
    const volatile uint32_t* sp = &env->rec_host->seq;
    for (int i = 0; i < (1 << 22); ++i) {
        if (*sp == seq) {
            __atomic_thread_fence(__ATOMIC_ACQUIRE);
            *out = env->rec_host;
            return OTH_OK;
        }
        __builtin_ia32_pause();
    }
    OTH_HIP(hipStreamSynchronize((hipStream_t)stream));
    if (*sp != seq) return fail(OTH_EHIP, "oth_step_sync: the record did not arrive");
    __atomic_thread_fence(__ATOMIC_ACQUIRE);
    *out = env->rec_host;
    return OTH_OK;
}

int oth_step_policy(oth_env* env, int32_t policy, int32_t n_plies, int32_t* actions, int32_t* rewards,
                    uint8_t* dones, oth_stream_t stream) {
    OTH_CHECK_ENV(env);
    if (n_plies < 0) return fail(OTH_EINVAL, "n_plies must be >= 0");
    if (policy < OTH_POLICY_RANDOM || policy > OTH_POLICY_LAST) return fail(OTH_EINVAL, "unknown policy");
    if (n_plies == 0) return OTH_OK;
    if (int rc = maximin_budget(env, policy, (double)n_plies, MM_POLICY, (hipStream_t)stream)) return rc;
    const uint64_t ply0 = env->ply;
    env->ply += (uint64_t)n_plies;
    return with_n(env->n, [&](auto NC) {
        return launch_play<decltype(NC)::value>(env, policy, n_plies, actions, rewards, dones, ply0,
                                                (hipStream_t)stream);
    });
}

int oth_reset_vs(oth_env* env, int32_t opponent_policy, const int8_t* protagonist, const uint8_t* mask,
                 oth_stream_t stream) {
    OTH_CHECK_ENV(env);
    if (opponent_policy < OTH_POLICY_RANDOM || opponent_policy > OTH_POLICY_LAST)
        return fail(OTH_EINVAL, "unknown opponent policy");
    if (int rc = maximin_budget(env, opponent_policy, 2.0, MM_RESET_VS, (hipStream_t)stream)) return rc;
    const uint64_t call = env->ply++;
    return with_n(env->n, [&](auto NC) {
        return launch_reset_vs<decltype(NC)::value>(env, opponent_policy, protagonist, mask, call,
                                                    (hipStream_t)stream);
    });
}

int oth_step_vs(oth_env* env, int32_t opponent_policy, const int32_t* actions, const int8_t* protagonist,
                int32_t* rewards, uint8_t* dones, int32_t* plies, oth_stream_t stream) {
    OTH_CHECK_ENV(env);
    if (!actions) return fail(OTH_EINVAL, "actions is NULL");
    if (opponent_policy < OTH_POLICY_RANDOM || opponent_policy > OTH_POLICY_LAST)
        return fail(OTH_EINVAL, "unknown opponent policy");
    if (int rc = maximin_budget(env, opponent_policy, 2.0, MM_STEP_VS, (hipStream_t)stream)) return rc;
    const uint64_t call = env->ply++;
    return with_n(env->n, [&](auto NC) {
        return launch_step_vs<decltype(NC)::value>(env, opponent_policy, actions, protagonist, rewards, dones,
                                                   plies, call, -1, 0, nullptr, (hipStream_t)stream);
    });
}

int oth_step_vs_observe(oth_env* env, int32_t opponent_policy, const int32_t* actions, const int8_t* protagonist,
                        int32_t* rewards, uint8_t* dones, int32_t* plies, int32_t layout, int32_t dtype, void* obs,
                        oth_stream_t stream) {
    OTH_CHECK_ENV(env);
    if (!actions || !obs) return fail(OTH_EINVAL, "actions / obs is NULL");
    if (opponent_policy < OTH_POLICY_RANDOM || opponent_policy > OTH_POLICY_LAST)
        return fail(OTH_EINVAL, "unknown opponent policy");
    if (layout < OTH_OBS_BOARD || layout > OTH_OBS_LEGAL) return fail(OTH_EINVAL, "unknown layout");
    if (dtype < OTH_I8 || dtype > OTH_BF16) return fail(OTH_EINVAL, "unknown dtype");
    if (int rc = maximin_budget(env, opponent_policy, 2.0, MM_STEP_VS, (hipStream_t)stream)) return rc;
    const uint64_t call = env->ply++;
    return with_n(env->n, [&](auto NC) {
        return launch_step_vs<decltype(NC)::value>(env, opponent_policy, actions, protagonist, rewards, dones,
                                                   plies, call, layout, dtype, obs, (hipStream_t)stream);
    });
}

int oth_policy_actions(oth_env* env, int32_t policy, int32_t* out, oth_stream_t stream) {
    OTH_CHECK_ENV(env);
    if (!out) return fail(OTH_EINVAL, "out is NULL");
    if (policy < OTH_POLICY_GREEDY || policy > OTH_POLICY_LAST)
        return fail(OTH_EINVAL, "policy must be greedy or maximin (depth 1 .. OTH_MAXIMIN_MAX_DEPTH)");
    if (int rc = maximin_budget(env, policy, 1.0, MM_POLICY, (hipStream_t)stream)) return rc;
    return with_n(env->n, [&](auto NC) {
        return launch_policy_actions<decltype(NC)::value>(env, policy, out, (hipStream_t)stream);
    });
}

int oth_greedy_actions(oth_env* env, int32_t* out, oth_stream_t stream) {
    return oth_policy_actions(env, OTH_POLICY_GREEDY, out, stream);
}

int oth_legal(oth_env* env, uint64_t* out, oth_stream_t stream) {
    OTH_CHECK_ENV(env);
    if (!out) return fail(OTH_EINVAL, "out is NULL");
    OTH_HIP(hipMemcpyAsync(out, env->legal, (size_t)env->E * env->W * sizeof(uint64_t), hipMemcpyDeviceToDevice,
                           (hipStream_t)stream));
    return OTH_OK;
}

int oth_legal_moves(int32_t board_size, int32_t n, const uint64_t* mover, const uint64_t* opp, uint64_t* out,
                    oth_stream_t stream) {
    if (n < 0 || (n > 0 && (!mover || !opp || !out))) return fail(OTH_EINVAL, "bad arguments");
    if (n == 0) return OTH_OK;
    const int bs = board_size < 4 ? 4 : board_size;
    return with_n(bs, [&](auto NC) {
        return launch_legal_moves<decltype(NC)::value>(n, mover, opp, out, (hipStream_t)stream);
    });
}


int oth_masked_sample(int32_t board_size, int32_t n, const float* logits, int64_t ld, const uint64_t* legal,
                      const float* uniforms, uint64_t seed, uint32_t id_base, uint64_t counter, int32_t mode,
                      int32_t* actions, float* log_probs, float* entropy, oth_stream_t stream) {
    const int bs = board_size < 4 ? 4 : board_size;
    if (bs > 16) return fail(OTH_EINVAL, "board_size must be <= 16");
    if ((mode & ~OTH_MASKED_FULL_ENTROPY) < OTH_MASKED_SAMPLE || (mode & ~OTH_MASKED_FULL_ENTROPY) > OTH_MASKED_EVAL)
        return fail(OTH_EINVAL, "unknown mode");
    if (n < 0 || (n > 0 && (!logits || !legal || !actions))) return fail(OTH_EINVAL, "bad arguments");
    if (ld < (int64_t)bs * bs) return fail(OTH_EINVAL, "ld < board_size^2");
    if (n == 0) return OTH_OK;
    return launch_masked(bs, n, logits, (long long)ld, legal, uniforms, seed, id_base, counter, nullptr, mode, actions,
                         log_probs, entropy, (hipStream_t)stream);
}

int oth_sample_actions(oth_env* env, const float* logits, int64_t ld, const float* uniforms, uint64_t counter,
                       int32_t mode, int32_t* actions, float* log_probs, float* entropy, oth_stream_t stream) {
    OTH_CHECK_ENV(env);
    if (!logits || !actions) return fail(OTH_EINVAL, "logits / actions is NULL");
    if ((mode & ~OTH_MASKED_FULL_ENTROPY) < OTH_MASKED_SAMPLE || (mode & ~OTH_MASKED_FULL_ENTROPY) > OTH_MASKED_EVAL)
        return fail(OTH_EINVAL, "unknown mode");
    if (ld < (int64_t)env->n * env->n) return fail(OTH_EINVAL, "ld < N*N");
    return launch_masked(env->n, env->E, logits, (long long)ld, env->legal, uniforms, env->seed, env->id_base, counter,
                         env->cur_off + 1, mode, actions, log_probs, entropy, (hipStream_t)stream);
}

int oth_sample_step(oth_env* env, const float* logits, int64_t ld, const float* uniforms, uint64_t counter,
                    int32_t mode, int32_t* actions, float* log_probs, float* entropy, int32_t* rewards, uint8_t* dones,
                    oth_stream_t stream) {
    OTH_CHECK_ENV(env);
    if (!logits || !actions) return fail(OTH_EINVAL, "logits / actions is NULL");
    const int base = mode & ~OTH_MASKED_FULL_ENTROPY;
    if (base != OTH_MASKED_SAMPLE && base != OTH_MASKED_MODE) return fail(OTH_EINVAL, "mode must be SAMPLE or MODE");
    if (ld < (int64_t)env->n * env->n) return fail(OTH_EINVAL, "ld < N*N");
    const uint64_t ply = env->ply++;
    return with_n(env->n, [&](auto NC) {
        return launch_sample_step<decltype(NC)::value>(env, logits, (long long)ld, uniforms, counter, mode, actions,
                                                       log_probs, entropy, rewards, dones, ply, -1, 0, nullptr,
                                                       (hipStream_t)stream);
    });
}

int oth_sample_step_observe(oth_env* env, const float* logits, int64_t ld, const float* uniforms, uint64_t counter,
                            int32_t mode, int32_t* actions, float* log_probs, float* entropy, int32_t* rewards,
                            uint8_t* dones, int32_t layout, int32_t dtype, void* obs, oth_stream_t stream) {
    OTH_CHECK_ENV(env);
    if (!logits || !actions || !obs) return fail(OTH_EINVAL, "logits / actions / obs is NULL");
    const int base = mode & ~OTH_MASKED_FULL_ENTROPY;
    if (base != OTH_MASKED_SAMPLE && base != OTH_MASKED_MODE) return fail(OTH_EINVAL, "mode must be SAMPLE or MODE");
    if (ld < (int64_t)env->n * env->n) return fail(OTH_EINVAL, "ld < N*N");
    if (layout < OTH_OBS_BOARD || layout > OTH_OBS_LEGAL) return fail(OTH_EINVAL, "unknown layout");
    if (dtype < OTH_I8 || dtype > OTH_BF16) return fail(OTH_EINVAL, "unknown dtype");
    const uint64_t ply = env->ply++;
    return with_n(env->n, [&](auto NC) {
        return launch_sample_step<decltype(NC)::value>(env, logits, (long long)ld, uniforms, counter, mode, actions,
                                                       log_probs, entropy, rewards, dones, ply, layout, dtype, obs,
                                                       (hipStream_t)stream);
    });
}

// A graph region's offsets move on by what one replay consumed (enqueued as
// the region's last node, so every replay advances them).
__global__ void k_graph_advance(uint64_t* __restrict__ off, uint64_t d_ply, uint64_t d_sample) {
    if (threadIdx.x == 0 && blockIdx.x == 0) {
        off[0] += d_ply;
        off[1] += d_sample;
    }
}

int oth_graph_begin(oth_env* env, int32_t* slot) {
    if (!env || !slot) return fail(OTH_EINVAL, "NULL argument");
    if (env->graph_slot) return fail(OTH_EINVAL, "a graph region is already open on this handle");
    if (env->slots_used == ~0ull)
        return fail(OTH_EINVAL, "no graph counter slot left on this handle (oth_graph_release frees one)");
    const int k = __builtin_ctzll(~env->slots_used);  // the lowest free slot
    env->slots_used |= 1ull << k;
    env->graph_slot = k;
    env->ply_saved = env->ply;
    env->ply = (uint64_t)k << OTH_GRAPH_COUNTER_SHIFT;
    env->cur_off = env->ctr_slots + 2 * k;
    *slot = k;
    return OTH_OK;
}

int oth_graph_end(oth_env* env, uint64_t d_sample, int32_t enqueue, uint64_t* d_ply, oth_stream_t stream) {
    if (!env) return fail(OTH_EINVAL, "NULL oth_env");
    if (!env->graph_slot) return fail(OTH_EINVAL, "no graph region is open on this handle");
    const int k = env->graph_slot;
    const uint64_t dp = env->ply - ((uint64_t)k << OTH_GRAPH_COUNTER_SHIFT);
    env->ply = env->ply_saved;  // eager counting resumes where it was
    env->cur_off = env->ctr_slots;
    env->graph_slot = 0;
    if (d_ply) *d_ply = dp;
    if (!enqueue) return OTH_OK;
    OTH_CHECK_ENV(env);
    launch_k(k_graph_advance, dim3(1), dim3(64), 0, (hipStream_t)stream, env->ctr_slots + 2 * k, dp,
             d_sample);
    return oth_host::after_launch("oth_graph_end");
}

// A released slot keeps its device offsets: a later region on it draws past
// every counter the earlier graph drew, so ranges stay disjoint even if that
// graph is still replayed.
int oth_graph_release(oth_env* env, int32_t slot) {
    if (!env) return fail(OTH_EINVAL, "NULL oth_env");
    if (slot <= 0 || slot >= OTH_GRAPH_SLOTS) return fail(OTH_EINVAL, "slot out of range");
    if (slot == env->graph_slot) return fail(OTH_EINVAL, "the slot's graph region is still open");
    env->slots_used &= ~(1ull << slot);
    return OTH_OK;
}

int oth_graph_offsets(const oth_env* env, int32_t slot, uint64_t* out) {
    OTH_CHECK_ENV(env);
    if (!out) return fail(OTH_EINVAL, "out is NULL");
    if (slot < 0 || slot >= OTH_GRAPH_SLOTS) return fail(OTH_EINVAL, "slot out of range");
    OTH_HIP(hipDeviceSynchronize());
    OTH_HIP(hipMemcpy(out, env->ctr_slots + 2 * slot, 2 * sizeof(uint64_t), hipMemcpyDeviceToHost));
    return OTH_OK;
}

int oth_observe(oth_env* env, int32_t layout, int32_t dtype, void* out, oth_stream_t stream) {
    OTH_CHECK_ENV(env);
    if (!out) return fail(OTH_EINVAL, "out is NULL");
    if (layout < OTH_OBS_BOARD || layout > OTH_OBS_LEGAL) return fail(OTH_EINVAL, "unknown layout");
    if (dtype < OTH_I8 || dtype > OTH_BF16) return fail(OTH_EINVAL, "unknown dtype");
    return with_n(env->n, [&](auto NC) {
        return launch_observe<decltype(NC)::value>(env, layout, dtype, out, (hipStream_t)stream);
    });
}

int oth_get_state(oth_env* env, uint64_t* boards, uint16_t* meta, uint64_t* legal, oth_stream_t stream) {
    OTH_CHECK_ENV(env);
    const size_t E = (size_t)env->E, W = (size_t)env->W;
    hipStream_t s = (hipStream_t)stream;
    if (boards) OTH_HIP(hipMemcpyAsync(boards, env->boards, E * 2 * W * 8, hipMemcpyDefault, s));
    if (meta) OTH_HIP(hipMemcpyAsync(meta, env->meta, E * 2, hipMemcpyDefault, s));
    if (legal) OTH_HIP(hipMemcpyAsync(legal, env->legal, E * W * 8, hipMemcpyDefault, s));
    return OTH_OK;
}

int oth_set_state(oth_env* env, const uint64_t* boards, const uint16_t* meta, const uint64_t* legal,
                  oth_stream_t stream) {
    OTH_CHECK_ENV(env);
    const size_t E = (size_t)env->E, W = (size_t)env->W;
    hipStream_t s = (hipStream_t)stream;
    if (boards) OTH_HIP(hipMemcpyAsync(env->boards, boards, E * 2 * W * 8, hipMemcpyDefault, s));
    if (meta) OTH_HIP(hipMemcpyAsync(env->meta, meta, E * 2, hipMemcpyDefault, s));
    if (legal) OTH_HIP(hipMemcpyAsync(env->legal, legal, E * W * 8, hipMemcpyDefault, s));
    return OTH_OK;
}

int oth_set_player_turn(oth_env* env, int32_t turn, const uint8_t* mask, oth_stream_t stream) {
    OTH_CHECK_ENV(env);
    if (turn != WHITE_DISK && turn != BLACK_DISK) return fail(OTH_EINVAL, "turn must be +1 or -1");
    return with_n(env->n, [&](auto NC) {
        return launch_set_turn<decltype(NC)::value>(env, turn, mask, (hipStream_t)stream);
    });
}

int oth_count_disks(oth_env* env, int32_t* out, oth_stream_t stream) {
    OTH_CHECK_ENV(env);
    if (!out) return fail(OTH_EINVAL, "out is NULL");
    return with_n(env->n, [&](auto NC) { return launch_count<decltype(NC)::value>(env, out, (hipStream_t)stream); });
}

int oth_counts(oth_env* env, int64_t* out, int32_t reset, oth_stream_t stream) {
    OTH_CHECK_ENV(env);
    if (!out) return fail(OTH_EINVAL, "out is NULL");
    hipStream_t s = (hipStream_t)stream;
    launch_k(k_reduce_wdl, dim3(1), dim3(256), 0, s, env->wdl, env->nslots, out, reset ? 1 : 0);
    return after_launch("oth_counts");
}

int oth_counts_vs(oth_env* env, int64_t* out, int32_t reset, oth_stream_t stream) {
    OTH_CHECK_ENV(env);
    if (!out) return fail(OTH_EINVAL, "out is NULL");
    launch_k(k_reduce_wdl, dim3(1), dim3(256), 0, (hipStream_t)stream, env->wdl_vs, env->nslots, out,
             reset ? 1 : 0);
    return after_launch("oth_counts_vs");
}

uint64_t oth_ply_counter(const oth_env* env) { return env ? env->ply : 0; }

int oth_set_ply_counter(oth_env* env, uint64_t ply) {
    if (!env) return fail(OTH_EINVAL, "NULL oth_env");
    if (env->graph_slot) return fail(OTH_EINVAL, "cannot set the ply counter inside a graph region");
    env->ply = ply;  // host only: graph regions keep their own counter ranges
    return OTH_OK;
}

int oth_shape(const oth_env* env, int32_t* n_envs, int32_t* board_size, int32_t* words) {
    if (!env) return fail(OTH_EINVAL, "NULL oth_env");
    if (n_envs) *n_envs = env->E;
    if (board_size) *board_size = env->n;
    if (words) *words = env->W;
    return OTH_OK;
}

}  // extern "C"
