// Micro-benchmark, round 6: what a lone wave (one per SIMD, the 65,536-board
// configs) pays per three-input VALU op, and whether that depends on the
// operand kinds (VGPR / SGPR / inline constant) or on the VGPR banks (reg % 4)
// of its sources.  Explicit registers, eight independent destinations per
// group, 64 ops per loop iteration.  Build + run on the GPU box:
//   hipcc --offload-arch=gfx950 -O3 -o /tmp/ub3 tools/ubench_valu3.hip && /tmp/ub3
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#define CLOB                                                                                                          \
    "v8", "v9", "v10", "v11", "v12", "v13", "v14", "v15", "v16", "v17", "v18", "v19", "v20", "v21", "v22", "v23",    \
        "v24", "v25", "v26", "v27", "v28", "v29", "v30", "v31", "v32", "v33", "v34", "v35", "v36", "v37", "v38",     \
        "v39", "v40", "v41", "v42", "v43", "v44", "v45", "v46", "v47", "v48", "v49", "v50", "v51", "v52", "v53",     \
        "v54", "v55", "s40", "s41"

// eight independent ops, destination i = its first source, the other sources fixed
#define G8(fmt) fmt(8) fmt(12) fmt(16) fmt(20) fmt(24) fmt(28) fmt(32) fmt(36)
#define G8B(fmt) fmt(8) fmt(9) fmt(10) fmt(11) fmt(24) fmt(25) fmt(26) fmt(27)

#define INIT                                                                                                          \
    "v_mov_b32 v8, %1\n v_mov_b32 v9, %1\n v_mov_b32 v10, %1\n v_mov_b32 v11, %1\n v_mov_b32 v12, %1\n"              \
    " v_mov_b32 v13, %1\n v_mov_b32 v14, %1\n v_mov_b32 v15, %1\n v_mov_b32 v16, %1\n v_mov_b32 v17, %1\n"           \
    " v_mov_b32 v18, %1\n v_mov_b32 v19, %1\n v_mov_b32 v20, %1\n v_mov_b32 v21, %1\n v_mov_b32 v22, %1\n"           \
    " v_mov_b32 v23, %1\n v_mov_b32 v24, %1\n v_mov_b32 v25, %1\n v_mov_b32 v26, %1\n v_mov_b32 v27, %1\n"           \
    " v_mov_b32 v28, %1\n v_mov_b32 v29, %1\n v_mov_b32 v30, %1\n v_mov_b32 v31, %1\n v_mov_b32 v32, %1\n"           \
    " v_mov_b32 v33, %1\n v_mov_b32 v34, %1\n v_mov_b32 v35, %1\n v_mov_b32 v36, %1\n v_mov_b32 v37, %1\n"           \
    " v_mov_b32 v38, %1\n v_mov_b32 v39, %1\n v_mov_b32 v40, %1\n v_mov_b32 v41, %1\n v_mov_b32 v42, %1\n"           \
    " v_mov_b32 v43, %1\n v_mov_b32 v44, %1\n v_mov_b32 v45, %1\n v_mov_b32 v46, %1\n v_mov_b32 v47, %1\n"           \
    " v_mov_b32 v48, %1\n v_mov_b32 v49, %1\n v_mov_b32 v50, %1\n v_mov_b32 v51, %1\n v_mov_b32 v52, %1\n"           \
    " v_mov_b32 v53, %1\n v_mov_b32 v54, %1\n v_mov_b32 v55, %1\n s_mov_b32 s40, 0x5555\n s_mov_b32 s41, 0\n"

#define KERNEL(name, body)                                                                                            \
    __global__ void name(uint32_t* out, int iters) {                                                                 \
        uint32_t r;                                                                                                   \
        const uint32_t seed = threadIdx.x * 2654435761u + 1u;                                                        \
        asm volatile(INIT : "=v"(r) : "v"(seed) : CLOB);                                                             \
        for (int i = 0; i < iters; ++i) asm volatile(body body body body body body body body : : : CLOB);            \
        asm volatile("v_xor_b32 %0, v8, v12\n v_or3_b32 %0, %0, v16, v20\n v_or3_b32 %0, %0, v24, v28\n"           \
                     " v_or3_b32 %0, %0, v32, v36\n v_or3_b32 %0, %0, v9, v10\n v_or3_b32 %0, %0, v11, v25\n"     \
                     " v_or3_b32 %0, %0, v26, v27"                                                                   \
                     : "=v"(r) : : CLOB);                                                                             \
        out[blockIdx.x * blockDim.x + threadIdx.x] = r;                                                               \
    }

#define S(x) #x
// two-input references
#define AND2(d) "v_and_b32 v" S(d) ", v" S(d) ", v41\n"
#define AND2S(d) "v_and_b32_e64 v" S(d) ", v" S(d) ", s40\n"
// three VGPR sources: banks (d, 1, 2) distinct vs (d, d, d) all bank 0 (d = 8, 12, ... is bank 0)
#define B3_DIST(d) "v_bitop3_b32 v" S(d) ", v" S(d) ", v41, v46 bitop3:0xca\n"
#define B3_SAME(d) "v_bitop3_b32 v" S(d) ", v" S(d) ", v40, v44 bitop3:0xca\n"
// one source an SGPR / an inline constant
#define B3_SGPR(d) "v_bitop3_b32 v" S(d) ", v" S(d) ", v41, s40 bitop3:0xca\n"
#define BFI_C0(d) "v_bfi_b32 v" S(d) ", v41, 0, v" S(d) "\n"
#define BFI_V(d) "v_bfi_b32 v" S(d) ", v41, v46, v" S(d) "\n"
#define ANDOR(d) "v_and_or_b32 v" S(d) ", v" S(d) ", v41, v46\n"
#define XOR3(d) "v_or3_b32 v" S(d) ", v" S(d) ", v41, v46\n"
#define ALIGN(d) "v_alignbit_b32 v" S(d) ", v" S(d) ", v41, 7\n"
#define ALIGNV(d) "v_alignbit_b32 v" S(d) ", v" S(d) ", v41, v46\n"
#define CND(d) "v_cndmask_b32 v" S(d) ", v" S(d) ", v41, vcc\n"
// banks of a two-input op: (0, 1) vs (0, 0)
#define AND2_SAME(d) "v_and_b32 v" S(d) ", v" S(d) ", v40\n"
// 3 VGPR sources where two are the same register
#define B3_DUP(d) "v_bitop3_b32 v" S(d) ", v" S(d) ", v41, v41 bitop3:0xca\n"

KERNEL(k_and2, G8(AND2))
KERNEL(k_and2s, G8(AND2S))
KERNEL(k_and2_same, G8(AND2_SAME))
KERNEL(k_b3_dist, G8(B3_DIST))
KERNEL(k_b3_same, G8(B3_SAME))
KERNEL(k_b3_sgpr, G8(B3_SGPR))
KERNEL(k_b3_dup, G8(B3_DUP))
KERNEL(k_bfi_c0, G8(BFI_C0))
KERNEL(k_bfi_v, G8(BFI_V))
KERNEL(k_andor, G8(ANDOR))
KERNEL(k_xor3, G8(XOR3))
KERNEL(k_align, G8(ALIGN))
KERNEL(k_alignv, G8(ALIGNV))
KERNEL(k_cnd, G8(CND))
// 64-bit ops on pairs v[8:9], v[12:13], ...
#define P8(fmt) fmt(8, 9) fmt(12, 13) fmt(16, 17) fmt(20, 21) fmt(24, 25) fmt(28, 29) fmt(32, 33) fmt(36, 37)
#define SHLP(a, b) "v_lshlrev_b64 v[" S(a) ":" S(b) "], 9, v[" S(a) ":" S(b) "]\n"
#define LADDP(a, b) "v_lshl_add_u64 v[" S(a) ":" S(b) "], v[" S(a) ":" S(b) "], 1, v[46:47]\n"
#define ADDCP(a, b) "v_add_co_u32 v" S(a) ", vcc, v" S(a) ", v46\n v_addc_co_u32 v" S(b) ", vcc, v" S(b) ", v47, vcc\n"
KERNEL(k_shl64, P8(SHLP))
KERNEL(k_lshladd, P8(LADDP))
KERNEL(k_addc, P8(ADDCP))
// mixes in the proportions of the greedy move: per 3 ops, one 64-bit shift, one 2-input, one 3-input
#define MIX(a, b) "v_lshlrev_b64 v[" S(a) ":" S(b) "], 9, v[" S(a) ":" S(b) "]\n v_and_b32 v" S(b) ", v" S(b) ", v41\n"
KERNEL(k_mix_shl_and, P8(MIX))

// the lone wave's issue interval: destination banks and op mixes
#define G16(fmt) fmt(8) fmt(9) fmt(10) fmt(11) fmt(12) fmt(13) fmt(14) fmt(15) fmt(16) fmt(17) fmt(18) fmt(19) fmt(20) fmt(21) fmt(22) fmt(23)
#define B3_DISTB(d) "v_bitop3_b32 v" S(d) ", v" S(d) ", v49, v50 bitop3:0xca\n"
#define AND2B(d) "v_and_b32 v" S(d) ", v" S(d) ", v49\n"
#define ALT(a, b) "v_and_b32 v" S(a) ", v" S(a) ", v41\n v_bitop3_b32 v" S(b) ", v" S(b) ", v41, v46 bitop3:0xca\n"
#define DEP_B3(d) "v_bitop3_b32 v8, v8, v41, v46 bitop3:0xca\n"
#define DEP_AND(d) "v_and_b32 v8, v8, v41\n"
KERNEL(k_and2_b, G8B(AND2B))
KERNEL(k_b3_b, G8B(B3_DISTB))
KERNEL(k_and2_16, G16(AND2B))
KERNEL(k_alt, P8(ALT))
KERNEL(k_dep_b3, G8(DEP_B3))
KERNEL(k_dep_and, G8(DEP_AND))
// the cost of a branch to a lone wave: 128 independent ops per loop iteration
// (G16 x 8) plus one extra branch per 16 ops, taken or not
#define BODY16 G16(AND2B)
#define KB(name, br) \
    __global__ void name(uint32_t* out, int iters) { \
        uint32_t r; \
        const uint32_t seed = threadIdx.x * 2654435761u + 1u; \
        asm volatile(INIT : "=v"(r) : "v"(seed) : CLOB); \
        for (int i = 0; i < iters; ++i) \
            asm volatile(BODY16 br BODY16 br BODY16 br BODY16 br BODY16 br BODY16 br BODY16 br BODY16 br : : : CLOB, "scc"); \
        asm volatile("v_xor_b32 %0, v8, v12\n v_or3_b32 %0, %0, v16, v20" : "=v"(r) : : CLOB); \
        out[blockIdx.x * blockDim.x + threadIdx.x] = r; \
    }
KB(k_br_none, "")
KB(k_br_taken, "s_branch 1f\n1:\n")
KB(k_br_scc_taken, "s_cmp_eq_u32 0, 0\n s_cbranch_scc1 1f\n1:\n")
KB(k_br_scc_not, "s_cmp_eq_u32 0, 1\n s_cbranch_scc1 1f\n1:\n")
KB(k_br_execz_not, "s_cbranch_execz 1f\n1:\n")
KB(k_salu2, "s_cmp_eq_u32 0, 1\n s_nop 0\n")
// 256 ops per iteration: the loop's own branch amortised further
#define KL(name) \
    __global__ void name(uint32_t* out, int iters) { \
        uint32_t r; \
        const uint32_t seed = threadIdx.x * 2654435761u + 1u; \
        asm volatile(INIT : "=v"(r) : "v"(seed) : CLOB); \
        for (int i = 0; i < iters; ++i) \
            asm volatile(BODY16 BODY16 BODY16 BODY16 BODY16 BODY16 BODY16 BODY16 BODY16 BODY16 BODY16 BODY16 BODY16 BODY16 BODY16 BODY16 : : : CLOB); \
        asm volatile("v_xor_b32 %0, v8, v12\n v_or3_b32 %0, %0, v16, v20" : "=v"(r) : : CLOB); \
        out[blockIdx.x * blockDim.x + threadIdx.x] = r; \
    }
KL(k_and2_256)

typedef void (*K)(uint32_t*, int);

static float run(K k, int waves_per_simd, int iters, uint32_t* buf) {
    const int blocks = 256 * waves_per_simd;  // 256-thread blocks: 4 waves each = 1 per SIMD of a CU
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    hipLaunchKernelGGL(k, dim3(blocks), dim3(256), 0, 0, buf, iters);
    (void)hipEventRecord(a, 0);
    hipLaunchKernelGGL(k, dim3(blocks), dim3(256), 0, 0, buf, iters);
    (void)hipEventRecord(b, 0);
    (void)hipEventSynchronize(b);
    float ms = 0;
    (void)hipEventElapsedTime(&ms, a, b);
    return ms;
}

int main() {
    uint32_t* buf;
    if (hipMalloc(&buf, 256 * 16 * 256 * 4) != hipSuccess) return 1;
    const int iters = 2000;
    struct {
        const char* name;
        K k;
        int ops;
    } ks[] = {{"v_and_b32 (v, v) banks 0,1", k_and2, 64},
              {"v_and_b32 (v, s)", k_and2s, 64},
              {"v_and_b32 (v, v) banks 0,0", k_and2_same, 64},
              {"v_bitop3_b32 (v, v, v) banks 0,1,2", k_b3_dist, 64},
              {"v_bitop3_b32 (v, v, v) banks 0,0,0", k_b3_same, 64},
              {"v_bitop3_b32 (v, v, s)", k_b3_sgpr, 64},
              {"v_bitop3_b32 (v, v, v) two the same register", k_b3_dup, 64},
              {"v_bfi_b32 (v, 0, v)", k_bfi_c0, 64},
              {"v_bfi_b32 (v, v, v)", k_bfi_v, 64},
              {"v_and_or_b32 (v, v, v)", k_andor, 64},
              {"v_or3_b32 (v, v, v)", k_xor3, 64},
              {"v_alignbit_b32 (v, v, 7)", k_align, 64},
              {"v_alignbit_b32 (v, v, v)", k_alignv, 64},
              {"v_cndmask_b32 (v, v, vcc)", k_cnd, 64},
              {"v_lshlrev_b64", k_shl64, 64},
              {"v_lshl_add_u64", k_lshladd, 64},
              {"v_add_co_u32 + v_addc_co_u32 pairs (per op)", k_addc, 128},
              {"v_lshlrev_b64 + v_and_b32 pairs (per op)", k_mix_shl_and, 128},
              {"v_and_b32 (v, v) destinations in banks 0-3", k_and2_b, 64},
              {"v_bitop3_b32 (v, v, v) destinations in banks 0-3", k_b3_b, 64},
              {"v_and_b32 (v, v) 16 independent chains, banks 0-3", k_and2_16, 128},
              {"v_and_b32 / v_bitop3_b32 alternating (per op)", k_alt, 128},
              {"v_bitop3_b32 dependent chain", k_dep_b3, 64},
              {"v_and_b32 dependent chain", k_dep_and, 64},
              {"v_and_b32 16 chains, 128 ops an iteration", k_br_none, 128},
              {"the same + 8 taken s_branch an iteration (per v_and)", k_br_taken, 128},
              {"the same + 8 taken s_cbranch_scc1 (per v_and)", k_br_scc_taken, 128},
              {"the same + 8 not-taken s_cbranch_scc1 (per v_and)", k_br_scc_not, 128},
              {"the same + 8 not-taken s_cbranch_execz (per v_and)", k_br_execz_not, 128},
              {"the same + 8 s_cmp + s_nop (per v_and)", k_salu2, 128},
              {"v_and_b32 16 chains, 256 ops an iteration", k_and2_256, 256}};
    printf("{\"clock_note\": \"cycles assume 2.4 GHz\", \"results\": [\n");
    bool first = true;
    for (auto& t : ks)
        for (int w : {1, 2}) {
            float ms = run(t.k, w, iters, buf);
            double ns_per_op = ms * 1e6 / ((double)iters * t.ops);  // per wave-op on one SIMD
            printf("%s{\"op\": \"%s\", \"waves_per_simd\": %d, \"cycles_per_wave_op\": %.3f}", first ? "" : ",\n",
                   t.name, w, ns_per_op / w * 2.4);
            first = false;
        }
    printf("\n]}\n");
    return 0;
}
