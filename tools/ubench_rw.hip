// Micro-benchmark (diagnostic only): what a small write stream costs a read
// stream shaped like the masks engine's (masks_mfma_kernel, MASKS_OUT): each
// wave owns groups of 4 tiles (4 x 50 KB read as 50 K-steps of 4 x 1 KB) and
// writes 7936 B of [u16;31] rows per group (62 B per 1600-B record).  Modes:
//   0 read only
//   1 burst: the group's 496 16-B words stored (nt) at the end of the group
//   2 burst, plain stores
//   3 trickle: the previous group's words stored over the first 8 steps
//   4 spread: ~10 words per step over the 50 steps of the next group
//   5 slotted: the group's words held (as in 3) and stored only inside chip-wide write windows of
//     the constant-rate clock (s_memrealtime, 100 MHz: W of every P ticks), so every wave's writes
//     fall in the same short bursts; a wave still holding words when its next group ends stores them
// All modes read the same bytes; modes 1-4 write the same bytes.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

constexpr int kT = 4, kSteps = 50, kWords = 496;  // 16-B output words per group

template <int MODE>
__global__ void __launch_bounds__(256, 2) rw_kernel(const uint4 *__restrict__ src, uint64_t groups,
                                                     uint4 *__restrict__ dst, uint32_t *out, uint32_t P = 0,
                                                     uint32_t W = 0) {
    const int lane = threadIdx.x & 63;
    const uint64_t wave = (uint64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    const uint64_t nwaves = (uint64_t)gridDim.x * 4;
    uint32_t acc = 0;
    u32x4 pend[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) pend[i] = u32x4{0, 0, 0, 0};
    uint64_t prev = ~0ull;
    bool held = false;  // mode 5: words of group `prev` not stored yet
    auto store_held = [&] {
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            const int i = k * 64 + lane;
            if (i < kWords) __builtin_nontemporal_store(pend[k], (u32x4 *)(dst + prev * kWords + i));
        }
        held = false;
    };
    for (uint64_t g = wave; g < groups; g += nwaves) {
        if (MODE == 5 && held) store_held();  // no window came during the whole group
        const uint4 *base = src + g * kT * 3200;  // 4 tiles of 3200 uint4 (51 200 B)
#pragma unroll 2
        for (int s = 0; s < kSteps; ++s) {
            u32x4 v[kT];
#pragma unroll
            for (int t = 0; t < kT; ++t) v[t] = __builtin_nontemporal_load((const u32x4 *)(base + t * 3200 + s * 64 + lane));
#pragma unroll
            for (int t = 0; t < kT; ++t) acc += v[t].x ^ v[t].y ^ v[t].z ^ v[t].w;
            if (MODE == 3 && prev != ~0ull && s < 8) {
                const int i = s * 64 + lane;
                if (i < kWords) __builtin_nontemporal_store(pend[0], (u32x4 *)(dst + prev * kWords + i));
#pragma unroll
                for (int k = 0; k < 7; ++k) pend[k] = pend[k + 1];
            }
            if (MODE == 5 && held && (uint32_t)(__builtin_amdgcn_s_memrealtime() % P) < W) store_held();
            if (MODE == 4 && prev != ~0ull && lane < 10) {
                const int i = s * 10 + lane;
                if (i < kWords) __builtin_nontemporal_store(u32x4{acc, 0, 0, 0}, (u32x4 *)(dst + prev * kWords + i));
            }
        }
        if (MODE == 1 || MODE == 2) {
            for (int i = lane; i < kWords; i += 64) {
                const u32x4 w = {acc, (uint32_t)i, 0, 0};
                if (MODE == 1)
                    __builtin_nontemporal_store(w, (u32x4 *)(dst + g * kWords + i));
                else
                    *(u32x4 *)(dst + g * kWords + i) = w;
            }
        }
        if (MODE == 3 || MODE == 5) {
#pragma unroll
            for (int k = 0; k < 8; ++k) pend[k] = u32x4{acc, (uint32_t)k, 0, 0};
            held = MODE == 5;
        }
        prev = g;
    }
    if (MODE == 3 && prev != ~0ull) {
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            const int i = k * 64 + lane;
            if (i < kWords) __builtin_nontemporal_store(pend[k], (u32x4 *)(dst + prev * kWords + i));
        }
    }
    if (MODE == 5 && held) store_held();
    if (MODE == 4 && prev != ~0ull && lane < 10)
        for (int i = lane; i < kWords; i += 10) dst[prev * kWords + i] = make_uint4(acc, 0, 0, 0);
    if (acc == 0x12345678u) out[0] = acc;
}

template <int MODE>
void run(const uint4 *src, uint64_t groups, uint4 *dst, uint32_t *out, int bpc, uint32_t P = 0, uint32_t W = 0) {
    const int grid = 256 * bpc;
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    for (int i = 0; i < 2; ++i) hipLaunchKernelGGL((rw_kernel<MODE>), grid, 256, 0, 0, src, groups, dst, out, P, W);
    const int reps = 20;
    (void)hipEventRecord(e0);
    for (int i = 0; i < reps; ++i) hipLaunchKernelGGL((rw_kernel<MODE>), grid, 256, 0, 0, src, groups, dst, out, P, W);
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    float ms = 0;
    (void)hipEventElapsedTime(&ms, e0, e1);
    ms /= reps;
    const double rb = (double)groups * kT * 51200, wb = MODE ? (double)groups * kWords * 16 : 0;
    printf("mode %d  blocks/CU %d  P %4u W %3u  %7.3f ms  read %6.0f GB/s  read+write %6.0f GB/s\n", MODE, bpc, P, W,
           ms, rb / (ms * 1e-3) / 1e9, (rb + wb) / (ms * 1e-3) / 1e9);
}

int main() {
    const uint64_t groups = 78125;  // 10M records
    const uint64_t rbytes = groups * kT * 51200, wbytes = groups * kWords * 16;
    uint4 *src, *dst;
    uint32_t *out;
    if (hipMalloc(&src, rbytes) != hipSuccess || hipMalloc(&dst, wbytes) != hipSuccess ||
        hipMalloc(&out, 64) != hipSuccess) {
        printf("alloc failed\n");
        return 1;
    }
    (void)hipMemset(src, 0x5A, rbytes);
    (void)hipMemset(dst, 0, wbytes);
    (void)hipDeviceSynchronize();
    for (int rep = 0; rep < 2; ++rep)
        for (int bpc : {2}) {
            run<0>(src, groups, dst, out, bpc);
            run<1>(src, groups, dst, out, bpc);
            run<3>(src, groups, dst, out, bpc);
            for (uint32_t P : {500u, 1000u, 2000u, 4000u})
                for (uint32_t W : {P / 20, P / 10, P / 5}) run<5>(src, groups, dst, out, bpc, P, W);
        }
    (void)hipFree(src);
    (void)hipFree(dst);
    (void)hipFree(out);
    return 0;
}
