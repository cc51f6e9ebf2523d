// Diagnostic: fp4 block-scaled MFMA, 32x32x64 vs 16x16x128, on operands that
// change every iteration (random bits, as in the batched search), at 1/2/4
// waves per SIMD.  Reports the sustained fp4 MAC rate and the in-kernel clock
// (delta s_memtime / delta s_memrealtime x 100 MHz, median over workgroups) —
// MI355X_MICROARCH.md item (6) of the DVFS notes.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#include <algorithm>
#include <vector>

typedef int v8i __attribute__((ext_vector_type(8)));
typedef float v16f __attribute__((ext_vector_type(16)));
typedef float v4f __attribute__((ext_vector_type(4)));

// SHAPE 32: 4 x 32x32x64 per iteration; SHAPE 16: 8 x 16x16x128 (same MACs)
template <int SHAPE, bool ZERO>
__global__ void __launch_bounds__(256) kern(float *out, double *clk, int iters, uint32_t seed) {
    uint32_t x = seed ^ (threadIdx.x * 0x9E3779B9u), y = x * 3u + blockIdx.x;
    if (ZERO) x = y = 0;
    const uint64_t t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
    float s = 0.f;
    if (SHAPE == 32) {
        v16f acc0 = {0}, acc1 = {0}, acc2 = {0}, acc3 = {0};
        for (int it = 0; it < iters; ++it) {
            v8i a0 = {(int)(x & 0xAAAAAAAAu), (int)((x << 1) & 0xAAAAAAAAu), (int)(y & 0xAAAAAAAAu),
                      (int)((y << 1) & 0xAAAAAAAAu), 0, 0, 0, 0};
            v8i a1 = {(int)(x & 0x22222222u), (int)(x & 0x11111111u), (int)(y & 0x22222222u),
                      (int)(y & 0x11111111u), 0, 0, 0, 0};
            acc0 = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(a0, a1, acc0, 4, 4, 0, 127, 0, 127);
            acc1 = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(a1, a0, acc1, 4, 4, 0, 127, 0, 127);
            if (!ZERO) { x = x * 1664525u + 1013904223u; y = y + x; }
            acc2 = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(a0, a0, acc2, 4, 4, 0, 127, 0, 127);
            acc3 = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(a1, a1, acc3, 4, 4, 0, 127, 0, 127);
        }
        for (int i = 0; i < 16; ++i) s += acc0[i] + acc1[i] + acc2[i] + acc3[i];
    } else {
        v4f acc[8];
        for (int j = 0; j < 8; ++j) acc[j] = v4f{0, 0, 0, 0};
        for (int it = 0; it < iters; ++it) {
            v8i a0 = {(int)(x & 0xAAAAAAAAu), (int)((x << 1) & 0xAAAAAAAAu), (int)(y & 0xAAAAAAAAu),
                      (int)((y << 1) & 0xAAAAAAAAu), 0, 0, 0, 0};
            v8i a1 = {(int)(x & 0x22222222u), (int)(x & 0x11111111u), (int)(y & 0x22222222u),
                      (int)(y & 0x11111111u), 0, 0, 0, 0};
            acc[0] = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(a0, a1, acc[0], 4, 4, 0, 127, 0, 127);
            acc[1] = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(a1, a0, acc[1], 4, 4, 0, 127, 0, 127);
            acc[2] = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(a0, a0, acc[2], 4, 4, 0, 127, 0, 127);
            acc[3] = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(a1, a1, acc[3], 4, 4, 0, 127, 0, 127);
            if (!ZERO) { x = x * 1664525u + 1013904223u; y = y + x; }
            acc[4] = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(a0, a1, acc[4], 4, 4, 0, 127, 0, 127);
            acc[5] = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(a1, a0, acc[5], 4, 4, 0, 127, 0, 127);
            acc[6] = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(a0, a0, acc[6], 4, 4, 0, 127, 0, 127);
            acc[7] = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(a1, a1, acc[7], 4, 4, 0, 127, 0, 127);
        }
        for (int j = 0; j < 8; ++j) s += acc[j][0] + acc[j][1] + acc[j][2] + acc[j][3];
    }
    const uint64_t t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
    if (threadIdx.x == 0) clk[blockIdx.x] = (double)(t1 - t0) / (double)(r1 - r0) * 100e6;
}

template <int SHAPE, bool ZERO>
void run(int wps) {
    const int blocks = 256 * wps, iters = 20000;
    float *out;
    double *clk;
    (void)hipMalloc(&out, blocks * 256 * 4);
    (void)hipMalloc(&clk, blocks * 8);
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    for (int i = 0; i < 3; ++i) kern<SHAPE, ZERO><<<blocks, 256>>>(out, clk, iters, 1 + i);  // warm, clocks settle
    (void)hipEventRecord(e0);
    const int reps = 3;
    for (int i = 0; i < reps; ++i) kern<SHAPE, ZERO><<<blocks, 256>>>(out, clk, iters, 7 + i);
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    float ms;
    (void)hipEventElapsedTime(&ms, e0, e1);
    ms /= reps;
    std::vector<double> c(blocks);
    (void)hipMemcpy(c.data(), clk, blocks * 8, hipMemcpyDeviceToHost);
    std::nth_element(c.begin(), c.begin() + blocks / 2, c.end());
    const double ghz = c[blocks / 2] / 1e9;
    const double macs = (double)blocks * 4 * iters * 4 * 65536;  // 4 waves per block, 4 x 32x32x64 per iter
    const double mfma_per_simd = (double)blocks * 4 * iters * (SHAPE == 32 ? 4 : 8) / 1024;
    printf("fp4 %dx%dx%-3d %s waves/SIMD=%d %8.3f ms  %.2f P fp4-MAC/s  clock %.2f GHz  %.1f cyc/MFMA at that clock\n",
           SHAPE, SHAPE, SHAPE == 32 ? 64 : 128, ZERO ? "zero  " : "random", wps, ms, macs / (ms * 1e-3) / 1e15, ghz,
           ms * 1e-3 * ghz * 1e9 / mfma_per_simd);
    (void)hipFree(out);
    (void)hipFree(clk);
}

int main() {
    for (int w : {1, 2, 4}) {
        run<32, false>(w);
        run<16, false>(w);
    }
    run<32, true>(2);
    run<16, true>(2);
    return 0;
}
