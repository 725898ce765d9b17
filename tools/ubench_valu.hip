// Micro-benchmark: issue cost and dependent latency of the VALU ops the Othello
// kernels are made of (64-bit shifts, 32-bit and/or, v_and_or, cndmask), at one
// and at several waves per SIMD.  Build + run on the GPU box:
//   hipcc --offload-arch=gfx950 -O3 -o /tmp/ubench tools/ubench_valu.hip && /tmp/ubench
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#define REP8(x) x x x x x x x x
#define REP64(x) REP8(REP8(x))

// dependent chain: each op consumes the previous result
__global__ void dep_shl64(uint64_t* out, int iters) {
    uint64_t x = threadIdx.x + 1;
    for (int i = 0; i < iters; ++i) { REP64(asm volatile("v_lshlrev_b64 %0, 1, %0" : "+v"(x));) }
    out[blockIdx.x * blockDim.x + threadIdx.x] = x;
}
__global__ void dep_and32(uint64_t* out, int iters) {
    uint32_t x = threadIdx.x + 1, y = 0xfffffffe;
    for (int i = 0; i < iters; ++i) { REP64(asm volatile("v_and_b32 %0, %0, %1" : "+v"(x) : "v"(y));) }
    out[blockIdx.x * blockDim.x + threadIdx.x] = x;
}
// independent streams: 8 registers round-robin
#define IND8(op) \
    asm volatile(op " %0, 1, %0" : "+v"(a0)); asm volatile(op " %0, 1, %0" : "+v"(a1)); \
    asm volatile(op " %0, 1, %0" : "+v"(a2)); asm volatile(op " %0, 1, %0" : "+v"(a3)); \
    asm volatile(op " %0, 1, %0" : "+v"(a4)); asm volatile(op " %0, 1, %0" : "+v"(a5)); \
    asm volatile(op " %0, 1, %0" : "+v"(a6)); asm volatile(op " %0, 1, %0" : "+v"(a7));
__global__ void ind_shl64(uint64_t* out, int iters) {
    uint64_t a0 = 1, a1 = 2, a2 = 3, a3 = 4, a4 = 5, a5 = 6, a6 = 7, a7 = threadIdx.x;
    for (int i = 0; i < iters; ++i) { REP8(IND8("v_lshlrev_b64")) }
    out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
}
#define IND8A \
    asm volatile("v_and_b32 %0, %0, %1" : "+v"(a0) : "v"(m)); asm volatile("v_and_b32 %0, %0, %1" : "+v"(a1) : "v"(m)); \
    asm volatile("v_and_b32 %0, %0, %1" : "+v"(a2) : "v"(m)); asm volatile("v_and_b32 %0, %0, %1" : "+v"(a3) : "v"(m)); \
    asm volatile("v_and_b32 %0, %0, %1" : "+v"(a4) : "v"(m)); asm volatile("v_and_b32 %0, %0, %1" : "+v"(a5) : "v"(m)); \
    asm volatile("v_and_b32 %0, %0, %1" : "+v"(a6) : "v"(m)); asm volatile("v_and_b32 %0, %0, %1" : "+v"(a7) : "v"(m));
__global__ void ind_and32(uint64_t* out, int iters) {
    uint32_t a0 = 1, a1 = 2, a2 = 3, a3 = 4, a4 = 5, a5 = 6, a6 = 7, a7 = threadIdx.x, m = 0xffffffff;
    for (int i = 0; i < iters; ++i) { REP8(IND8A) }
    out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
}
#define IND8O(op) \
    asm volatile(op " %0, %0, %1, %2" : "+v"(a0) : "v"(m), "v"(c)); asm volatile(op " %0, %0, %1, %2" : "+v"(a1) : "v"(m), "v"(c)); \
    asm volatile(op " %0, %0, %1, %2" : "+v"(a2) : "v"(m), "v"(c)); asm volatile(op " %0, %0, %1, %2" : "+v"(a3) : "v"(m), "v"(c)); \
    asm volatile(op " %0, %0, %1, %2" : "+v"(a4) : "v"(m), "v"(c)); asm volatile(op " %0, %0, %1, %2" : "+v"(a5) : "v"(m), "v"(c)); \
    asm volatile(op " %0, %0, %1, %2" : "+v"(a6) : "v"(m), "v"(c)); asm volatile(op " %0, %0, %1, %2" : "+v"(a7) : "v"(m), "v"(c));
__global__ void ind_andor32(uint64_t* out, int iters) {
    uint32_t a0 = 1, a1 = 2, a2 = 3, a3 = 4, a4 = 5, a5 = 6, a6 = 7, a7 = threadIdx.x, m = 0xffffffff, c = 0;
    for (int i = 0; i < iters; ++i) { REP8(IND8O("v_and_or_b32")) }
    out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
}

// same as ind_and32 / ind_shl64 but only the low 32 lanes of each wave active
__global__ void half_and32(uint64_t* out, int iters) {
    if ((threadIdx.x & 63) >= 32) return;
    uint32_t a0 = 1, a1 = 2, a2 = 3, a3 = 4, a4 = 5, a5 = 6, a6 = 7, a7 = threadIdx.x, m = 0xffffffff;
    for (int i = 0; i < iters; ++i) { REP8(IND8A) }
    out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
}
__global__ void half_dep_and32(uint64_t* out, int iters) {
    if ((threadIdx.x & 63) >= 32) return;
    uint32_t x = threadIdx.x + 1, y = 0xfffffffe;
    for (int i = 0; i < iters; ++i) { REP64(asm volatile("v_and_b32 %0, %0, %1" : "+v"(x) : "v"(y));) }
    out[blockIdx.x * blockDim.x + threadIdx.x] = x;
}
__global__ void half_shl64(uint64_t* out, int iters) {
    if ((threadIdx.x & 63) >= 32) return;
    uint64_t a0 = 1, a1 = 2, a2 = 3, a3 = 4, a4 = 5, a5 = 6, a6 = 7, a7 = threadIdx.x;
    for (int i = 0; i < iters; ++i) { REP8(IND8("v_lshlrev_b64")) }
    out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
}

// multi-pass candidates (round 4): 32-bit multiplies (byte broadcasts of RayMath,
// scale_index), the 32x32->64 multiply-add of Philox, and the full-rate ops that
// could stand in for them (v_perm_b32 byte broadcast, v_mul_u32_u24)
#define IND8X(op)                                                                                       \
    asm volatile(op " %0, %0, %1" : "+v"(a0) : "v"(m)); asm volatile(op " %0, %0, %1" : "+v"(a1) : "v"(m)); \
    asm volatile(op " %0, %0, %1" : "+v"(a2) : "v"(m)); asm volatile(op " %0, %0, %1" : "+v"(a3) : "v"(m)); \
    asm volatile(op " %0, %0, %1" : "+v"(a4) : "v"(m)); asm volatile(op " %0, %0, %1" : "+v"(a5) : "v"(m)); \
    asm volatile(op " %0, %0, %1" : "+v"(a6) : "v"(m)); asm volatile(op " %0, %0, %1" : "+v"(a7) : "v"(m));
#define IND_KERNEL2(name, op)                                                                    \
    __global__ void name(uint64_t* out, int iters) {                                             \
        uint32_t a0 = 1, a1 = 2, a2 = 3, a3 = 4, a4 = 5, a5 = 6, a6 = 7, a7 = threadIdx.x, m = 3; \
        for (int i = 0; i < iters; ++i) { REP8(IND8X(op)) }                                      \
        out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;      \
    }
IND_KERNEL2(ind_mullo, "v_mul_lo_u32")
IND_KERNEL2(ind_mulhi, "v_mul_hi_u32")
IND_KERNEL2(ind_mul24, "v_mul_u32_u24")
IND_KERNEL2(ind_bcnt, "v_bcnt_u32_b32")
__global__ void ind_perm(uint64_t* out, int iters) {
    uint32_t a0 = 1, a1 = 2, a2 = 3, a3 = 4, a4 = 5, a5 = 6, a6 = 7, a7 = threadIdx.x, m = 0x04040404u, c = 0;
    for (int i = 0; i < iters; ++i) { REP8(IND8O("v_perm_b32")) }
    out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
}
#define MAD1(o, a) asm volatile("v_mad_u64_u32 %0, %1, %2, %3, 0" : "=v"(o), "=s"(sc) : "v"(a), "v"(m));
__global__ void ind_mad64(uint64_t* out, int iters) {
    uint32_t a0 = 1, a1 = 2, a2 = 3, a3 = 4, a4 = 5, a5 = 6, a6 = 7, a7 = threadIdx.x, m = 0xD2511F53u;
    uint64_t o0 = 0, o1 = 0, o2 = 0, o3 = 0, o4 = 0, o5 = 0, o6 = 0, o7 = 0, sc;
    for (int i = 0; i < iters; ++i) {
        REP8(MAD1(o0, a0) MAD1(o1, a1) MAD1(o2, a2) MAD1(o3, a3) MAD1(o4, a4) MAD1(o5, a5) MAD1(o6, a6) MAD1(o7, a7))
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = o0 ^ o1 ^ o2 ^ o3 ^ o4 ^ o5 ^ o6 ^ o7;
}

typedef void (*K)(uint64_t*, int);

static float run(K k, int waves_per_simd, int iters, uint64_t* buf) {
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
    uint64_t* buf;
    if (hipMalloc(&buf, 256 * 16 * 256 * 8) != hipSuccess) return 1;
    const int iters = 2000;
    struct { const char* name; K k; int ops_per_iter; } ks[] = {
        {"dep v_lshlrev_b64", dep_shl64, 64}, {"dep v_and_b32", dep_and32, 64},
        {"ind v_lshlrev_b64", ind_shl64, 64}, {"ind v_and_b32", ind_and32, 64},
        {"ind v_and_or_b32", ind_andor32, 64}, {"half-wave ind v_and_b32", half_and32, 64},
        {"half-wave dep v_and_b32", half_dep_and32, 64}, {"half-wave ind v_lshlrev_b64", half_shl64, 64},
        {"ind v_mul_lo_u32", ind_mullo, 64}, {"ind v_mul_hi_u32", ind_mulhi, 64}, {"ind v_mul_u32_u24", ind_mul24, 64},
        {"ind v_bcnt_u32_b32", ind_bcnt, 64}, {"ind v_perm_b32", ind_perm, 64}, {"ind v_mad_u64_u32", ind_mad64, 64}};
    printf("{\"clock_note\": \"cycles assume 2.4 GHz\", \"results\": [\n");
    bool first = true;
    for (auto& t : ks)
        for (int w : {1, 2, 4}) {
            float ms = run(t.k, w, iters, buf);
            double ns_per_op = ms * 1e6 / ((double)iters * t.ops_per_iter);  // per wave-op on one SIMD (w waves share it)
            printf("%s{\"op\": \"%s\", \"waves_per_simd\": %d, \"ns_per_wave_op_per_simd\": %.4f, \"cycles_per_wave_op\": %.3f}",
                   first ? "" : ",\n", t.name, w, ns_per_op / w, ns_per_op / w * 2.4);
            first = false;
        }
    printf("\n]}\n");
    return 0;
}
