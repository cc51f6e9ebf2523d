// Micro-benchmark (diagnostic only): VALU issue rate of the masked-Hamming
// inner step on gfx950, registers only (no memory), plus the in-kernel clock.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>

#define REP8(X) X(0) X(1) X(2) X(3) X(4) X(5) X(6) X(7)

template <int V>
__global__ void __launch_bounds__(256) kern(uint32_t *out, int iters, uint32_t s0, uint32_t s1, unsigned long long *clk) {
    uint32_t a[8], b[8];
    uint32_t em = threadIdx.x * 0x9E3779B9u, ep = em ^ 0x5555u;
    for (int i = 0; i < 8; ++i) { a[i] = i; b[i] = 2 * i; }
    unsigned long long t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
    for (int it = 0; it < iters; ++it) {
#define STEP(r) { uint32_t m, x; \
   if (V == 0) asm volatile("v_and_b32 %0, %4, %5\n\tv_bitop3_b32 %1, %6, %7, %0 bitop3:0x28\n\tv_bcnt_u32_b32 %2, %0, %2\n\tv_bcnt_u32_b32 %3, %1, %3" : "=&v"(m), "=&v"(x), "+v"(a[r]), "+v"(b[r]) : "s"(s0 + r), "v"(em), "s"(s1), "v"(ep)); \
   if (V == 1) asm volatile("v_and_b32 %0, %4, %5\n\tv_bitop3_b32 %1, %6, %7, %0 bitop3:0x28\n\tv_add_u32 %2, %0, %2\n\tv_add_u32 %3, %1, %3" : "=&v"(m), "=&v"(x), "+v"(a[r]), "+v"(b[r]) : "s"(s0 + r), "v"(em), "s"(s1), "v"(ep)); \
   if (V == 2) asm volatile("v_bcnt_u32_b32 %2, %4, %2\n\tv_bcnt_u32_b32 %3, %5, %3\n\tv_bcnt_u32_b32 %2, %6, %2\n\tv_bcnt_u32_b32 %3, %7, %3" : "=&v"(m), "=&v"(x), "+v"(a[r]), "+v"(b[r]) : "s"(s0 + r), "v"(em), "s"(s1), "v"(ep)); \
   if (V == 3) asm volatile("v_and_b32 %2, %4, %5\n\tv_and_b32 %3, %6, %7\n\tv_xor_b32 %2, %4, %2\n\tv_xor_b32 %3, %6, %3" : "=&v"(m), "=&v"(x), "+v"(a[r]), "+v"(b[r]) : "s"(s0 + r), "v"(em), "s"(s1), "v"(ep)); \
   if (V == 4) asm volatile("v_bitop3_b32 %2, %4, %5, %2 bitop3:0x28\n\tv_bitop3_b32 %3, %6, %7, %3 bitop3:0x28\n\tv_bitop3_b32 %2, %4, %5, %2 bitop3:0x28\n\tv_bitop3_b32 %3, %6, %7, %3 bitop3:0x28" : "=&v"(m), "=&v"(x), "+v"(a[r]), "+v"(b[r]) : "s"(s0 + r), "v"(em), "s"(s1), "v"(ep)); \
   if (V == 5) asm volatile("v_pk_mad_u16 %2, %5, %4, %2\n\tv_pk_mad_u16 %3, %7, %6, %3\n\tv_pk_mad_u16 %2, %5, %4, %2\n\tv_pk_mad_u16 %3, %7, %6, %3" : "=&v"(m), "=&v"(x), "+v"(a[r]), "+v"(b[r]) : "s"(s0 + r), "v"(em), "s"(s1), "v"(ep)); \
 }
        REP8(STEP)
    }
    unsigned long long t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
    uint32_t acc = 0;
    for (int i = 0; i < 8; ++i) acc += a[i] + b[i];
    out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
    if (threadIdx.x == 0) { clk[2 * blockIdx.x] = t1 - t0; clk[2 * blockIdx.x + 1] = r1 - r0; }
}

template <int V>
void run(const char *name, int waves_per_simd) {
    const int blocks = 256 * waves_per_simd;  // 256-thread blocks: 4 waves, 1 per SIMD
    const int iters = 20000;
    uint32_t *out; unsigned long long *clk;
    hipMalloc(&out, blocks * 256 * 4);
    hipMalloc(&clk, blocks * 16);
    hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
    kern<V><<<blocks, 256>>>(out, 100, 1, 2, clk);
    hipEventRecord(e0);
    kern<V><<<blocks, 256>>>(out, iters, 1, 2, clk);
    hipEventRecord(e1); hipEventSynchronize(e1);
    float ms; hipEventElapsedTime(&ms, e0, e1);
    unsigned long long h[2]; hipMemcpy(h, clk, 16, hipMemcpyDeviceToHost);
    double insts = (double)blocks * 4 /*waves*/ * iters * 8 * 4;  // wave-instructions
    double lane_ops = insts * 64;
    double ghz = (double)h[0] / ((double)h[1] / 100e6) / 1e9;
    // per-SIMD cycles per wave-instruction at the measured clock
    double cyc_per_inst = (ms * 1e-3) * ghz * 1e9 * 1024 / insts;
    printf("%-28s waves/SIMD=%d  %8.3f ms  %7.2f T lane-ops/s  clock %.2f GHz  %.2f SIMD-cycles/wave-inst\n", name,
           waves_per_simd, ms, lane_ops / (ms * 1e-3) / 1e12, ghz, cyc_per_inst);
    hipFree(out); hipFree(clk);
}

int main() {
    for (int w : {1, 2, 4, 8}) {
        run<0>("and+bitop3+2bcnt (hot step)", w);
        run<1>("and+bitop3+2add", w);
        run<2>("4x bcnt", w);
        run<3>("and/xor x4", w);
        run<4>("4x bitop3", w);
        run<5>("4x pk_mad_u16", w);
    }
    return 0;
}
