// Device -> pinned host bandwidth: the copy engine (hipMemcpyAsync D2H) against a kernel storing
// 16-B nontemporal words straight into the pinned buffer (what the read-ahead's window kernels
// do), for the sizes a masks walk moves (640 KB = one packed 20k chunk, 5 MB = an 8-chunk window,
// 64 MB).  hipcc --offload-arch=gfx950 -O3 -o tools/ubench_d2h tools/ubench_d2h.hip
#include <hip/hip_runtime.h>
#include <stdio.h>

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

__global__ void __launch_bounds__(256) store_kernel(u32x4 *dst, size_t n16) {
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n16; i += (size_t)gridDim.x * blockDim.x) {
        const u32x4 v = {(unsigned)i, 1u, 2u, 3u};
        __builtin_nontemporal_store(v, dst + i);
    }
}

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e_)); return 1; } } while (0)

int main() {
    const size_t maxb = 64ull << 20;
    void *dev = nullptr, *host = nullptr;
    CK(hipMalloc(&dev, maxb));
    CK(hipHostMalloc(&host, maxb, hipHostMallocDefault));
    CK(hipMemset(dev, 1, maxb));
    hipStream_t s;
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    const size_t sizes[] = {640u << 10, 5u << 20, 64u << 20};
    for (size_t bytes : sizes) {
        const int reps = (int)(std::max<size_t>(1, (2048ull << 20) / bytes));
        for (int form = 0; form < 2; ++form) {
            for (int warm = 0; warm < 2; ++warm) {
                CK(hipEventRecord(a, s));
                for (int r = 0; r < reps; ++r) {
                    if (form == 0)
                        CK(hipMemcpyAsync(host, dev, bytes, hipMemcpyDeviceToHost, s));
                    else
                        hipLaunchKernelGGL(store_kernel, dim3(1024), dim3(256), 0, s, (u32x4 *)host, bytes / 16);
                }
                CK(hipEventRecord(b, s));
                CK(hipEventSynchronize(b));
                float ms = 0;
                CK(hipEventElapsedTime(&ms, a, b));
                if (warm)
                    printf("%-14s %8zu KB x %5d: %7.1f GB/s (%.1f us each)\n", form ? "kernel stores" : "hipMemcpy D2H",
                           bytes >> 10, reps, bytes * (double)reps / (ms * 1e-3) / 1e9, ms * 1e3 / reps);
            }
        }
    }
    return 0;
}
