// Diagnostic: issue cost of individual VALU ops on gfx950 (8 waves/SIMD, 4
// independent dependency chains per wave), SIMD-cycles per wave-instruction.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>

#define OPS(X) \
  X(v_add_u32, "v_add_u32 %0, %1, %0") \
  X(v_and_b32, "v_and_b32 %0, %1, %0") \
  X(v_bcnt, "v_bcnt_u32_b32 %0, %1, %0") \
  X(v_pk_mad_u16, "v_pk_mad_u16 %0, %1, %2, %0") \
  X(v_dot2_u32_u16, "v_dot2_u32_u16 %0, %1, %2, %0") \
  X(v_dot4_i32_i8, "v_dot4_i32_i8 %0, %1, %2, %0") \
  X(v_dot8_i32_i4, "v_dot8_i32_i4 %0, %1, %2, %0") \
  X(v_mad_u32_u24, "v_mad_u32_u24 %0, %1, %2, %0") \
  X(v_mul_u32_u24, "v_mul_u32_u24 %0, %1, %0") \
  X(v_add3_u32, "v_add3_u32 %0, %1, %2, %0") \
  X(v_and_or_b32, "v_and_or_b32 %0, %1, %2, %0") \
  X(v_lshl_or_b32, "v_lshl_or_b32 %0, %1, 3, %0") \
  X(v_perm_b32, "v_perm_b32 %0, %1, %2, %0") \
  X(v_pk_add_u16, "v_pk_add_u16 %0, %1, %0") \
  X(v_pk_mul_lo_u16, "v_pk_mul_lo_u16 %0, %1, %0") \
  X(v_lshlrev_b32, "v_lshlrev_b32 %0, 1, %0") \
  X(v_bfi_b32, "v_bfi_b32 %0, %1, %2, %0") \
  X(v_cndmask_b32, "v_cndmask_b32 %0, %1, %0, vcc") \
  X(v_fma_f32, "v_fma_f32 %0, %1, %2, %0") \
  X(v_xor_b32, "v_xor_b32 %0, %1, %0") \
  X(v_mov_b32, "v_mov_b32 %0, %1")

#define KERN(name, txt) \
__global__ void __launch_bounds__(256) k_##name(uint32_t *out, int iters) { \
    uint32_t a0 = threadIdx.x, a1 = a0 * 3, a2 = a0 * 5, a3 = a0 * 7, b = a0 ^ 0x1234567u, c = a0 * 0x9E3779B9u; \
    typedef float v2f __attribute__((ext_vector_type(2))); (void)sizeof(v2f); \
    for (int it = 0; it < iters; ++it) { \
        _Pragma("unroll") for (int u = 0; u < 8; ++u) { \
        asm volatile(txt : "+v"(a0) : "v"(b), "v"(c)); asm volatile(txt : "+v"(a1) : "v"(b), "v"(c)); \
        asm volatile(txt : "+v"(a2) : "v"(b), "v"(c)); asm volatile(txt : "+v"(a3) : "v"(b), "v"(c)); } \
    } \
    out[blockIdx.x * 256 + threadIdx.x] = a0 + a1 + a2 + a3; }
OPS(KERN)
#define KERN64(name, txt)
__global__ void __launch_bounds__(256) k_pkfma(uint32_t *out, int iters) {
    typedef float v2f __attribute__((ext_vector_type(2)));
    v2f a0 = {1.f * threadIdx.x, 2.f}, a1 = a0 * 2.f, a2 = a0 * 3.f, a3 = a0 * 4.f, b = {0.5f, 0.25f}, c = {1.f, 1.f};
    for (int it = 0; it < iters; ++it) {
        _Pragma("unroll") for (int u = 0; u < 8; ++u) {
        asm volatile("v_pk_fma_f32 %0, %1, %2, %0" : "+v"(a0) : "v"(b), "v"(c)); asm volatile("v_pk_fma_f32 %0, %1, %2, %0" : "+v"(a1) : "v"(b), "v"(c));
        asm volatile("v_pk_fma_f32 %0, %1, %2, %0" : "+v"(a2) : "v"(b), "v"(c)); asm volatile("v_pk_fma_f32 %0, %1, %2, %0" : "+v"(a3) : "v"(b), "v"(c)); }
    }
    out[blockIdx.x * 256 + threadIdx.x] = (uint32_t)(a0.x + a1.x + a2.x + a3.x);
}

template <class F>
void run(const char *name, F kern) {
    const int wps = 8, blocks = 256 * wps, iters = 4000;
    uint32_t *out; (void)hipMalloc(&out, blocks * 256 * 4);
    hipEvent_t e0, e1; (void)hipEventCreate(&e0); (void)hipEventCreate(&e1);
    hipLaunchKernelGGL(kern, dim3(blocks), dim3(256), 0, 0, out, 10);
    (void)hipEventRecord(e0);
    hipLaunchKernelGGL(kern, dim3(blocks), dim3(256), 0, 0, out, iters);
    (void)hipEventRecord(e1); (void)hipEventSynchronize(e1);
    float ms; (void)hipEventElapsedTime(&ms, e0, e1);
    double insts = (double)blocks * 4 * iters * 32;
    printf("%-18s %.2f SIMD-cycles/wave-inst @2.4GHz\n", name, ms * 1e-3 * 2.4e9 * 1024 / insts);
    (void)hipFree(out);
}

int main() {
#define RUN(name, txt) run(#name, k_##name);
    OPS(RUN)
    run("v_pk_fma_f32(v2)", k_pkfma);
    return 0;
}
