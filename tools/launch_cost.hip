// launch_cost.hip -- host cost of one kernel launch on this box, without Python:
//   empty     hipLaunchKernelGGL of an empty kernel (65,536 threads), back to back
//   oth_step  the C ABI's oth_step (liboth_mi355x.so, dlopen) on 65,536 8x8 boards
//             with device actions of a fixed legal-or-not pattern (any action is a
//             valid input), back to back
// Each: host wall time per call over K calls (the launch path), and the time
// to drain the queue after the last call.
//   hipcc --offload-arch=gfx950 -O2 -o tools/launch_cost tools/launch_cost.hip -ldl
//   tools/launch_cost gymothelloenv_amd/liboth_mi355x.so
#include <dlfcn.h>
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#include <chrono>

__global__ void k_empty(int* p) {
    if (p && threadIdx.x == 1024) p[0] = 1;
}

typedef int (*create_fn)(int32_t, int32_t, uint32_t, uint64_t, uint32_t, int32_t, int32_t, void**);
typedef int (*step_fn)(void*, const int32_t*, int32_t*, uint8_t*, void*);
typedef int (*destroy_fn)(void*);

static double now_us() {
    return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

int main(int argc, char** argv) {
    const int K = 2000, E = 65536;
    if (hipSetDevice(0) != hipSuccess) return 2;
    hipStream_t st;
    if (hipStreamCreate(&st) != hipSuccess) return 2;
    for (int i = 0; i < 100; ++i) hipLaunchKernelGGL(k_empty, dim3(E / 256), dim3(256), 0, st, nullptr);
    if (hipStreamSynchronize(st) != hipSuccess) return 2;
    double t0 = now_us();
    for (int i = 0; i < K; ++i) hipLaunchKernelGGL(k_empty, dim3(E / 256), dim3(256), 0, st, nullptr);
    double t1 = now_us();
    if (hipStreamSynchronize(st) != hipSuccess) return 2;
    double t2 = now_us();
    printf("{\"case\": \"empty\", \"host_us_per_launch\": %.3f, \"drain_us\": %.1f, \"total_us_per_launch\": %.3f}\n",
           (t1 - t0) / K, t2 - t1, (t2 - t0) / K);
    // the host calls around a launch in the C ABI: hipGetDevice (use_device) and
    // hipGetLastError (after_launch), and hipLaunchKernel returning its status
    {
        int dev = 0;
        double a0 = now_us();
        for (int i = 0; i < K; ++i) (void)hipGetDevice(&dev);
        double a1 = now_us();
        for (int i = 0; i < K; ++i) (void)hipGetLastError();
        double a2 = now_us();
        void* kargs[] = {nullptr};
        int* nullp = nullptr;
        kargs[0] = &nullp;
        for (int i = 0; i < K; ++i)
            (void)hipLaunchKernel((const void*)k_empty, dim3(E / 256), dim3(256), kargs, 0, st);
        double a3 = now_us();
        if (hipStreamSynchronize(st) != hipSuccess) return 2;
        for (int i = 0; i < K; ++i) {
            hipLaunchKernelGGL(k_empty, dim3(E / 256), dim3(256), 0, st, nullptr);
            (void)hipGetLastError();
        }
        double a4 = now_us();
        if (hipStreamSynchronize(st) != hipSuccess) return 2;
        printf("{\"case\": \"host_calls\", \"hipGetDevice_us\": %.3f, \"hipGetLastError_us\": %.3f, "
               "\"hipLaunchKernel_us\": %.3f, \"launchGGL_plus_getlasterror_us\": %.3f}\n",
               (a1 - a0) / K, (a2 - a1) / K, (a3 - a2) / K, (a4 - a3) / K);
    }
    if (argc < 2) return 0;
    void* so = dlopen(argv[1], RTLD_NOW);
    if (!so) {
        printf("dlopen failed: %s\n", dlerror());
        return 1;
    }
    create_fn create = (create_fn)dlsym(so, "oth_create");
    step_fn step = (step_fn)dlsym(so, "oth_step");
    destroy_fn destroy = (destroy_fn)dlsym(so, "oth_destroy");
    void* h = nullptr;
    if (!create || !step || !destroy || create(E, 8, 1 | 4, 7, 0, 0, 0, &h) != 0) return 1;
    int32_t *a, *r;
    uint8_t* d;
    if (hipMalloc(&a, E * 4) != hipSuccess || hipMalloc(&r, E * 4) != hipSuccess || hipMalloc(&d, E) != hipSuccess)
        return 2;
    if (hipMemset(a, 0x13, E * 4) != hipSuccess) return 2;  // square 0x13131313: out of range, the invalid path
    for (int i = 0; i < 100; ++i) step(h, a, r, d, st);
    if (hipStreamSynchronize(st) != hipSuccess) return 2;
    t0 = now_us();
    for (int i = 0; i < K; ++i) step(h, a, r, d, st);
    t1 = now_us();
    if (hipStreamSynchronize(st) != hipSuccess) return 2;
    t2 = now_us();
    printf("{\"case\": \"oth_step\", \"host_us_per_launch\": %.3f, \"drain_us\": %.1f, \"total_us_per_launch\": %.3f}\n",
           (t1 - t0) / K, t2 - t1, (t2 - t0) / K);
    destroy(h);
    (void)hipFree(a);
    (void)hipFree(r);
    (void)hipFree(d);
    return 0;
}
