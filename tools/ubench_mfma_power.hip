// Diagnostic: the fp4 block-scaled MFMA (v_mfma_scale_f32_32x32x64_f8f6f4, 2 waves per SIMD) launched
// back to back for `seconds` so the package power can be polled beside it.  Prints the MFMAs issued and
// the time: energy per MFMA = mean package power x time / MFMAs.
//
// mode 0: the MFMA alone — 4 accumulators, operands that change every iteration with the batched
//         kernel's nibble density (random bits under the 0xA / 0x2 / 0x1 masks), 2 operand registers.
// mode 1: the batched kernel's MFMA sequence fed from LDS — per 64-bit chunk 2 queries x 2 tiles x
//         (den, encode) = 8 MFMAs on 8 accumulators, the 4 query and 4 template fragments of every chunk
//         read from a 64-KB LDS table of expanded random fragments (ds_read_b128, lane-linear) — no HBM,
//         no L2, no expansion VALU: what the MFMA costs on the kernel's own operand sequence.
// mode 2: mode 1 with the template fragments expanded from compact random words in registers by the
//         kernel's VALU (8 v_and + 2 shifts per chunk and tile) instead of read from LDS.
// mode 3: mode 1 with the template operands held constant (only the query
//         fragments change per chunk): how much of the MFMA energy is operand toggling.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

typedef int v8i __attribute__((ext_vector_type(8)));
typedef float v16f __attribute__((ext_vector_type(16)));

__device__ __forceinline__ v16f mma(const v8i &a, const v8i &b, const v16f &c) {
    return __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(a, b, c, 4, 4, 0, 127, 0, 127);
}

__global__ void __launch_bounds__(256) kern0(float *out, int iters, uint32_t seed) {
    uint32_t x = seed ^ (threadIdx.x * 0x9E3779B9u), y = x * 3u + blockIdx.x;
    v16f acc0 = {0}, acc1 = {0}, acc2 = {0}, acc3 = {0};
    for (int it = 0; it < iters; ++it) {
        v8i a0 = {(int)(x & 0xAAAAAAAAu), (int)((x << 1) & 0xAAAAAAAAu), (int)(y & 0xAAAAAAAAu),
                  (int)((y << 1) & 0xAAAAAAAAu), 0, 0, 0, 0};
        v8i a1 = {(int)(x & 0x22222222u), (int)(x & 0x11111111u), (int)(y & 0x22222222u), (int)(y & 0x11111111u),
                  0, 0, 0, 0};
        acc0 = mma(a0, a1, acc0);
        acc1 = mma(a1, a0, acc1);
        x = x * 1664525u + 1013904223u;
        y = y + x;
        acc2 = mma(a0, a0, acc2);
        acc3 = mma(a1, a1, acc3);
    }
    float s = 0.f;
    for (int i = 0; i < 16; ++i) s += acc0[i] + acc1[i] + acc2[i] + acc3[i];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

__device__ __forceinline__ uint32_t hash(uint32_t x) {
    x ^= x >> 16;
    x *= 0x7feb352du;
    x ^= x >> 15;
    x *= 0x846ca68bu;
    return x ^ (x >> 16);
}

// LDS table: kFr fragments of 64 lanes x 16 B (expanded fp4 den or encode dwords of random bits)
constexpr int kFr = 64;  // 64 KB
template <int MODE>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(2, 2))) kern1(float *out, int iters, uint32_t seed) {
    __shared__ uint4 tab[kFr][64];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    for (int f = w; f < kFr; f += 4) {
        const uint32_t x = hash(seed + f * 64 + lane), y = hash(x + 0x51u);
        tab[f][lane] = (f & 1) ? make_uint4(x & 0xAAAAAAAAu, (x << 1) & 0xAAAAAAAAu, y & 0xAAAAAAAAu,
                                            (y << 1) & 0xAAAAAAAAu)
                               : make_uint4(x & 0x22222222u, x & 0x11111111u, y & 0x22222222u, y & 0x11111111u);
    }
    __syncthreads();
    v16f den[2][2], enc[2][2];
    for (int q = 0; q < 2; ++q)
        for (int t = 0; t < 2; ++t)
            for (int i = 0; i < 16; ++i) den[q][t][i] = enc[q][t][i] = 0.f;
    uint32_t bx[2] = {hash(seed ^ threadIdx.x), hash(seed + threadIdx.x * 7u)}, by[2] = {bx[1] * 3u, bx[0] + 11u};
    int c0 = (blockIdx.x * 5 + w * 3) & (kFr / 8 - 1);
    for (int it = 0; it < iters; ++it) {
        // chunk it: query fragments from rows 8c..8c+3, template fragments 8c+4..8c+7 (den even, encode odd)
        const int c = (c0 + it) & (kFr / 8 - 1);
        const uint4 ad0 = tab[8 * c + 0][lane], ae0 = tab[8 * c + 1][lane];
        const uint4 ad1 = tab[8 * c + 2][lane], ae1 = tab[8 * c + 3][lane];
        v8i bd[2], be[2];
        if (MODE == 2) {
#pragma unroll
            for (int t = 0; t < 2; ++t) {
                bd[t] = v8i{(int)(bx[t] & 0x22222222u), (int)(bx[t] & 0x11111111u), (int)(by[t] & 0x22222222u),
                            (int)(by[t] & 0x11111111u), 0, 0, 0, 0};
                be[t] = v8i{(int)(bx[t] & 0xAAAAAAAAu), (int)((bx[t] << 1) & 0xAAAAAAAAu), (int)(by[t] & 0xAAAAAAAAu),
                            (int)((by[t] << 1) & 0xAAAAAAAAu), 0, 0, 0, 0};
                bx[t] = bx[t] * 1664525u + 1013904223u;
                by[t] ^= bx[t];
            }
        } else {
            const int cb = MODE == 3 ? (c & ~7) : c;
#pragma unroll
            for (int t = 0; t < 2; ++t) {
                const uint4 d = tab[8 * cb + 4 + 2 * t][lane], e = tab[8 * cb + 5 + 2 * t][lane];
                bd[t] = v8i{(int)d.x, (int)d.y, (int)d.z, (int)d.w, 0, 0, 0, 0};
                be[t] = v8i{(int)e.x, (int)e.y, (int)e.z, (int)e.w, 0, 0, 0, 0};
            }
        }
        const uint4 ad[2] = {ad0, ad1}, ae[2] = {ae0, ae1};
#pragma unroll
        for (int q = 0; q < 2; ++q) {
            const v8i a_d = {(int)ad[q].x, (int)ad[q].y, (int)ad[q].z, (int)ad[q].w, 0, 0, 0, 0};
            const v8i a_e = {(int)ae[q].x, (int)ae[q].y, (int)ae[q].z, (int)ae[q].w, 0, 0, 0, 0};
#pragma unroll
            for (int t = 0; t < 2; ++t) den[q][t] = mma(a_d, bd[t], den[q][t]);
#pragma unroll
            for (int t = 0; t < 2; ++t) enc[q][t] = mma(a_e, be[t], enc[q][t]);
        }
    }
    float s = 0.f;
    for (int q = 0; q < 2; ++q)
        for (int t = 0; t < 2; ++t)
            for (int i = 0; i < 16; ++i) s += den[q][t][i] - enc[q][t][i];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

int main(int argc, char **argv) {
    const double seconds = argc > 1 ? atof(argv[1]) : 10.0;
    const int mode = argc > 2 ? atoi(argv[2]) : 0;
    const int blocks = 256 * 2;  // 2 waves per SIMD (4-wave blocks, 2 per CU); ~30 ms per launch
    const int iters = mode == 0 ? 200000 : 100000;
    const double mfma_per_iter = mode == 0 ? 4 : 8;
    float *out;
    if (hipMalloc(&out, blocks * 256 * 4) != hipSuccess) return 1;
    auto launch = [&](uint32_t s) {
        if (mode == 0) kern0<<<blocks, 256>>>(out, iters, s);
        else if (mode == 1) kern1<1><<<blocks, 256>>>(out, iters, s);
        else if (mode == 2) kern1<2><<<blocks, 256>>>(out, iters, s);
        else kern1<3><<<blocks, 256>>>(out, iters, s);
    };
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    launch(1);
    if (hipDeviceSynchronize() != hipSuccess) return 1;
    (void)hipEventRecord(e0);
    int launches = 0;
    float ms = 0;
    while (ms < seconds * 1e3) {
        for (int i = 0; i < 16; ++i, ++launches) launch(7 + launches);
        (void)hipEventRecord(e1);
        (void)hipEventSynchronize(e1);
        (void)hipEventElapsedTime(&ms, e0, e1);
    }
    const double mfma = (double)launches * blocks * 4 * (double)iters * mfma_per_iter;
    printf("mfma_mode%d launches %d  seconds %.3f  mfma %.6e  rate %.4e MFMA/s  %.3f P fp4-MAC/s\n", mode, launches,
           ms * 1e-3, mfma, mfma / (ms * 1e-3), mfma * 65536 / (ms * 1e-3) / 1e15);
    (void)hipFree(out);
    return 0;
}
