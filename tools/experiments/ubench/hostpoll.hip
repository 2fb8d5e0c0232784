// Can a running kernel see a host store to pinned host memory?  (diagnostic, not the product)
// One wave polls a word of a hipHostMalloc'd buffer that the host sets 20 ms after the launch, for
// several allocation flags and load forms, with a 2-s timeout on the device's real-time counter.
// Build: hipcc -O3 --offload-arch=gfx950 -o hostpoll hostpoll.hip
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>
#include <thread>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e_), __LINE__); return 1; } } while (0)

__device__ __forceinline__ unsigned long long rt_now() {
    unsigned long long t;
    asm volatile("s_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
    return t;
}

template <int MODE>
__global__ void k_poll(unsigned long long* word, unsigned long long* out) {
    const unsigned long long t0 = rt_now();
    unsigned long long v = 0, it = 0, t = t0;
    for (;; ++it) {
        if (MODE == 0) v = __hip_atomic_load(word, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM);
        else if (MODE == 1) v = __hip_atomic_load(word, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        else v = *(volatile unsigned long long*)word;
        t = rt_now();
        if (v != 0 || t - t0 > 200000000ull) break;
        __builtin_amdgcn_s_sleep(10);
    }
    if (threadIdx.x == 0) {
        out[0] = v;
        out[1] = it;
        out[2] = t - t0;
    }
}

int main() {
    const unsigned flags[3] = {hipHostMallocCoherent | hipHostMallocMapped, hipHostMallocMapped, hipHostMallocDefault};
    const char* fname[3] = {"coherent|mapped", "mapped", "default"};
    for (int f = 0; f < 3; ++f) {
        for (int mode = 0; mode < 3; ++mode) {
            unsigned long long *h, *d, *out;
            CK(hipHostMalloc((void**)&h, 64, flags[f]));
            CK(hipHostGetDevicePointer((void**)&d, h, 0));
            CK(hipHostMalloc((void**)&out, 64, hipHostMallocDefault));
            h[0] = 0;
            out[0] = out[1] = out[2] = 0;
            if (mode == 0) hipLaunchKernelGGL(k_poll<0>, dim3(1), dim3(64), 0, 0, d, out);
            else if (mode == 1) hipLaunchKernelGGL(k_poll<1>, dim3(1), dim3(64), 0, 0, d, out);
            else hipLaunchKernelGGL(k_poll<2>, dim3(1), dim3(64), 0, 0, d, out);
            std::this_thread::sleep_for(std::chrono::milliseconds(20));
            __atomic_store_n(&h[0], 7ull, __ATOMIC_RELEASE);
            CK(hipDeviceSynchronize());
            printf("%-16s load=%s  seen=%llu  polls=%llu  after %.1f ms (dev %p host %p)\n", fname[f],
                   mode == 0 ? "sys-acquire" : mode == 1 ? "sys-relaxed" : "volatile", out[0], out[1],
                   out[2] / 1e5, (void*)d, (void*)h);
            CK(hipHostFree(h));
            CK(hipHostFree(out));
        }
    }
    return 0;
}
