// iris_resolver.hip — the resolver's combine + decode + argmin, fused on the GPU.
//
// Reference: src/main.rs:597-621.  For every entry i the resolver sums the
// participants' [u16;31] shares with wrapping adds (:603-607), decodes with
// decode_distance (src/lib.rs:97-107: uneq = (den - num) / 2 in u16, value
// uneq as f64 / den as f64, fold(INF, f64::min)), then keeps the first entry
// with a strictly smaller distance (:616-621).
//
// Exactness: uneq <= 32767 and den <= 65535, so fractions compare exactly by
// u32 cross-multiplication; distinct fractions are distinct f64 values, so the
// exact order is the reference's f64 order.  den = 0 gives NaN or +inf in the
// reference, which never wins a f64::min or a strict <; here it is "no
// candidate".  The winner's f64 is computed once with IEEE division.
#include <hip/hip_runtime.h>

#include "iris_device.hpp"

namespace iris {

constexpr int kMaxParts = 8;
constexpr int kWaveRows = 64;

struct ResolverArgs {
    const uint16_t *shares[kMaxParts];
    uint32_t parts;
};

typedef unsigned short u16x8 __attribute__((ext_vector_type(8)));

// One wave's 64 rows of a [n][31] u16 array as 16-B words: 64 rows = 3968 B =
// 248 words, 16-B aligned when the array is (row0 is a multiple of 64).  Word
// i of the wave's block -> lane i % 64, slot i / 64 (4 slots).  Words past the
// end of the array are read element-wise (zero beyond it).
__device__ __forceinline__ u16x8 load_word(const uint16_t *__restrict__ src, uint64_t e0, uint64_t ne, uint32_t i,
                                           bool aligned) {
    const uint64_t e = (uint64_t)i * 8;
    if (aligned && e + 8 <= ne) {
        // read once: nontemporal loads (the plain-load stream tops out lower, measured in
        // profiles/r01_ubench_read_stream_warm.txt: tools/ubench_stream.hip)
        return __builtin_nontemporal_load((const u16x8 *)(src + e0 + e));
    }
    u16x8 v = {0, 0, 0, 0, 0, 0, 0, 0};
#pragma unroll
    for (int j = 0; j < 8; ++j)
        if (e + j < ne) v[j] = src[e0 + e + j];
    return v;
}

constexpr int kWords = kWaveRows * kRot * 2 / 16;  // 248
constexpr int kSlots = (kWords + 63) / 64;         // 4

__global__ void __launch_bounds__(256) resolver_kernel(ResolverArgs a, const uint16_t *__restrict__ denoms,
                                                       uint64_t n, double *__restrict__ dist_out,
                                                       Partial *__restrict__ partials) {
    __shared__ __attribute__((aligned(16))) uint16_t sh_num[kWaveSlots][kWaveRows * kRot + 8];
    __shared__ __attribute__((aligned(16))) uint16_t sh_den[kWaveSlots][kWaveRows * kRot + 8];
    __shared__ Partial sh_best[kWaveSlots];
    const int lane = threadIdx.x & 63, ws = threadIdx.x >> 6;
    const uint64_t row0 = ((uint64_t)blockIdx.x * kWaveSlots + ws) * kWaveRows;
    const uint64_t rows = row0 < n ? ((n - row0) < kWaveRows ? n - row0 : kWaveRows) : 0;
    const uint64_t e0 = row0 * kRot, ne = rows * kRot;
    bool aligned = ((uintptr_t)denoms & 15) == 0;
    for (uint32_t p = 0; p < a.parts; ++p) aligned &= ((uintptr_t)a.shares[p] & 15) == 0;
    Partial c;
    c.num = 0;
    c.den = 0;
    c.rot = 0;
    c.pad = 0;
    c.idx = row0 + lane;
    // wrapping sum of the shares (src/main.rs:603-607) in packed u16 lanes, all loads issued up front
    u16x8 num[kSlots], den[kSlots];
#pragma unroll
    for (int sl = 0; sl < kSlots; ++sl) {
        const uint32_t i = lane + 64 * sl;
        if (i < kWords) {
            den[sl] = load_word(denoms, e0, ne, i, aligned);
            num[sl] = load_word(a.shares[0], e0, ne, i, aligned);
        }
    }
    for (uint32_t p = 1; p < a.parts; ++p)
#pragma unroll
        for (int sl = 0; sl < kSlots; ++sl) {
            const uint32_t i = lane + 64 * sl;
            if (i < kWords) num[sl] += load_word(a.shares[p], e0, ne, i, aligned);
        }
#pragma unroll
    for (int sl = 0; sl < kSlots; ++sl) {
        const uint32_t i = lane + 64 * sl;
        if (i < kWords) {
            *(u16x8 *)&sh_num[ws][8 * i] = num[sl];
            *(u16x8 *)&sh_den[ws][8 * i] = den[sl];
        }
    }
    __syncthreads();
    if ((uint64_t)lane < rows) {
        const uint16_t *nr = sh_num[ws] + lane * kRot, *dr = sh_den[ws] + lane * kRot;
#pragma unroll
        for (int k = 0; k < kRot; ++k) {
            const uint32_t d = dr[k];
            const uint32_t u = (uint16_t)(d - nr[k]) >> 1;  // src/lib.rs:104
            if (d != 0 && (c.den == 0 || u * c.den < c.num * d)) {
                c.num = u;
                c.den = d;
                c.rot = k;
            }
        }
        if (dist_out) dist_out[row0 + lane] = c.den ? (double)c.num / (double)c.den : __builtin_inf();
    }
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) {
        const Partial o = partial_shfl_xor(c, off);
        if (partial_better_dev(o, c)) c = o;
    }
    if (lane == 0) sh_best[ws] = c;
    __syncthreads();
    if (threadIdx.x == 0) {
        Partial b = sh_best[0];
        for (int w = 1; w < kWaveSlots; ++w)
            if (partial_better_dev(sh_best[w], b)) b = sh_best[w];
        partials[blockIdx.x] = b;
    }
}

uint32_t resolver_partials(uint64_t n) {
    return (uint32_t)((n + kWaveRows * kWaveSlots - 1) / (kWaveRows * kWaveSlots));
}

int launch_resolver(void *stream, const uint16_t *const *shares, uint32_t parts, const uint16_t *denoms, uint64_t n,
                    double *dist_out, Partial *partials) {
    if (n == 0) return 0;
    if (parts == 0 || parts > (uint32_t)kMaxParts) return -1;
    ResolverArgs a{};
    for (uint32_t p = 0; p < parts; ++p) a.shares[p] = shares[p];
    a.parts = parts;
    hipLaunchKernelGGL(resolver_kernel, dim3(resolver_partials(n)), dim3(256), 0, (hipStream_t)stream, a, denoms, n,
                       dist_out, partials);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

}  // namespace iris
