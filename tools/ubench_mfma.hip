// Diagnostic: fp4 MFMA (32x32x64 f8f6f4) issue rate alone and with VALU
// expansion work interleaved (the planned bit->fp4 path), per SIMD.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>
typedef int v8i __attribute__((ext_vector_type(8)));
typedef float v16f __attribute__((ext_vector_type(16)));

template <int NVALU>
__global__ void __launch_bounds__(256) kern(float *out, int iters, uint32_t seed) {
    v16f acc0 = {0}, acc1 = {0}, acc2 = {0}, acc3 = {0};
    uint32_t x = seed ^ (threadIdx.x * 0x9E3779B9u), y = x * 3u;
    v8i b = {(int)(x * 5), (int)(x * 7), (int)(x * 11), (int)(x * 13), 0, 0, 0, 0};
    for (int it = 0; it < iters; ++it) {
        v8i a0, a1;
        // NVALU bitwise ops producing the A operands (like the bit->fp4 expansion)
        a0[0] = x & 0x22222222u; a0[1] = x & 0x11111111u; a0[2] = y & 0x22222222u; a0[3] = y & 0x11111111u;
        a1[0] = x & 0xAAAAAAAAu; a1[1] = (x << 1) & 0xAAAAAAAAu; a1[2] = y & 0xAAAAAAAAu; a1[3] = (y << 1) & 0xAAAAAAAAu;
        a0[4] = a0[5] = a0[6] = a0[7] = 0; a1[4] = a1[5] = a1[6] = a1[7] = 0;
        if (NVALU == 0) { a0 = b; a1 = b; }
        acc0 = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(a0, b, acc0, 4, 4, 0, 127, 0, 127);
        acc1 = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(a1, b, acc1, 4, 4, 0, 127, 0, 127);
        x = x * 1664525u + 1013904223u;  // keep x/y changing (adds: fast ops)
        y = y + x;
        acc2 = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(b, a0, acc2, 4, 4, 0, 127, 0, 127);
        acc3 = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(b, a1, acc3, 4, 4, 0, 127, 0, 127);
    }
    float s = 0;
    for (int i = 0; i < 16; ++i) s += acc0[i] + acc1[i] + acc2[i] + acc3[i];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

template <int V>
void run(const char *name, int wps) {
    int blocks = 256 * wps, iters = 20000;
    float *out; (void)hipMalloc(&out, blocks * 256 * 4);
    hipEvent_t e0, e1; (void)hipEventCreate(&e0); (void)hipEventCreate(&e1);
    kern<V><<<blocks, 256>>>(out, 10, 1);
    (void)hipEventRecord(e0);
    kern<V><<<blocks, 256>>>(out, iters, 1);
    (void)hipEventRecord(e1); (void)hipEventSynchronize(e1);
    float ms; (void)hipEventElapsedTime(&ms, e0, e1);
    double mfma = (double)blocks * 4 * iters * 4;
    double macs = mfma * 32 * 32 * 64;
    printf("%-34s waves/SIMD=%d %8.3f ms  %.1f cyc/MFMA/SIMD @2.4GHz  %.2f P fp4-MAC/s\n", name, wps, ms,
           ms * 1e-3 * 2.4e9 * 1024 / mfma, macs / (ms * 1e-3) / 1e15);
    (void)hipFree(out);
}

int main() {
    for (int w : {1, 2, 4}) { run<0>("fp4 mfma only", w); run<1>("fp4 mfma + 10 VALU per 2 MFMA", w); }
    return 0;
}
