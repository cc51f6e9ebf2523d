// Diagnostic: the fp4 block-scaled MFMA alone (v_mfma_scale_f32_32x32x64_f8f6f4, 2 waves per
// SIMD, operands that change every iteration with the batched kernel's nibble density: random
// bits under the 0xA / 0x2 / 0x1 masks of tools/ubench_mfma_shapes.hip), launched back to back
// for `seconds` so the package power can be polled beside it.  Prints the MFMAs issued and the
// time: energy per MFMA = mean package power x time / MFMAs.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

typedef int v8i __attribute__((ext_vector_type(8)));
typedef float v16f __attribute__((ext_vector_type(16)));

__global__ void __launch_bounds__(256) kern(float *out, int iters, uint32_t seed) {
    uint32_t x = seed ^ (threadIdx.x * 0x9E3779B9u), y = x * 3u + blockIdx.x;
    v16f acc0 = {0}, acc1 = {0}, acc2 = {0}, acc3 = {0};
    for (int it = 0; it < iters; ++it) {
        v8i a0 = {(int)(x & 0xAAAAAAAAu), (int)((x << 1) & 0xAAAAAAAAu), (int)(y & 0xAAAAAAAAu),
                  (int)((y << 1) & 0xAAAAAAAAu), 0, 0, 0, 0};
        v8i a1 = {(int)(x & 0x22222222u), (int)(x & 0x11111111u), (int)(y & 0x22222222u), (int)(y & 0x11111111u),
                  0, 0, 0, 0};
        acc0 = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(a0, a1, acc0, 4, 4, 0, 127, 0, 127);
        acc1 = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(a1, a0, acc1, 4, 4, 0, 127, 0, 127);
        x = x * 1664525u + 1013904223u;
        y = y + x;
        acc2 = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(a0, a0, acc2, 4, 4, 0, 127, 0, 127);
        acc3 = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(a1, a1, acc3, 4, 4, 0, 127, 0, 127);
    }
    float s = 0.f;
    for (int i = 0; i < 16; ++i) s += acc0[i] + acc1[i] + acc2[i] + acc3[i];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

int main(int argc, char **argv) {
    const double seconds = argc > 1 ? atof(argv[1]) : 10.0;
    const int blocks = 256 * 2, iters = 200000;  // 2 waves per SIMD; ~30 ms per launch
    float *out;
    if (hipMalloc(&out, blocks * 256 * 4) != hipSuccess) return 1;
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    kern<<<blocks, 256>>>(out, iters, 1);
    (void)hipDeviceSynchronize();
    (void)hipEventRecord(e0);
    int launches = 0;
    float ms = 0;
    while (ms < seconds * 1e3) {
        for (int i = 0; i < 16; ++i, ++launches) kern<<<blocks, 256>>>(out, iters, 7 + launches);
        (void)hipEventRecord(e1);
        (void)hipEventSynchronize(e1);
        (void)hipEventElapsedTime(&ms, e0, e1);
    }
    const double mfma = (double)launches * blocks * 4 * (double)iters * 4;
    printf("mfma_alone launches %d  seconds %.3f  mfma %.6e  rate %.4e MFMA/s  %.3f P fp4-MAC/s\n", launches, ms * 1e-3,
           mfma, mfma / (ms * 1e-3), mfma * 65536 / (ms * 1e-3) / 1e15);
    (void)hipFree(out);
    return 0;
}
