// iris_query.hip — per-engine query preparation on the device.
//
// An engine holds the 31 rotated copies of its query (k = 0..30 <-> r = k - 15,
// DistanceEngine::new / MasksEngine::new, src/lib.rs:33-40, 60-67) in the
// layouts its kernels read: the SGPR tables of the LANES kernels and the MFMA
// A-fragments of the TILES kernels (iris_internal.hpp).  Built here from the
// query alone, so creating an engine costs one small upload and one launch
// (the host builders in iris_host.cpp, bit by bit, took ~3.5 ms per template
// query — as long as the 10M-template search itself).  Template and mask
// queries travel in the kernel arguments, so those engines cost one launch.  The host builders stay
// as the reference the device tables are tested against
// (iris_debug_query_tables, tests/test_gpu_query.py).
#include <hip/hip_runtime.h>
#include <string.h>

#include "iris_internal.hpp"

namespace iris {

// dword w of rot(b, r): bit i is b's bit at row i / 200, column (i % 200 - r)
// mod 200 (Bits::rotated, src/bits.rs:18-29; |r| <= 15).  b: 400 dwords in LDS.
// Word-level: the 32 output bits split into at most four runs of consecutive
// source bits (a row boundary and the column wrap), each one funnel shift.
__device__ __forceinline__ uint32_t rot_dword(const uint32_t *b, int r, int w) {
    uint32_t x = 0;
    int t = 0, i = 32 * w;
    while (t < 32) {
        const int row = i / IRIS_COLS, col = i - row * IRIS_COLS;
        int sc = col - r;
        sc += sc < 0 ? IRIS_COLS : 0;
        sc -= sc >= IRIS_COLS ? IRIS_COLS : 0;
        const int len = min(32 - t, min(IRIS_COLS - col, IRIS_COLS - sc));
        const int src = row * IRIS_COLS + sc, d = src >> 5;
        const uint64_t win = (uint64_t)b[d] | ((uint64_t)(d + 1 < kPlaneDwords ? b[d + 1] : 0u) << 32);
        const uint32_t bits = (uint32_t)(win >> (src & 31)) & (len == 32 ? 0xFFFFFFFFu : ((1u << len) - 1u));
        x |= bits << t;
        t += len;
        i += len;
    }
    return x;
}

// The query travels by value in the kernel arguments (3200 B of the 4 KB
// kernarg segment): creating an engine is one launch, no separate upload.
struct TemplateArg {
    uint32_t pattern[kPlaneDwords], mask[kPlaneDwords];
};
struct MaskArg {
    uint32_t mask[kPlaneDwords];
};

__global__ void __launch_bounds__(256) query_template_kernel(const TemplateArg q, uint32_t *__restrict__ tab,
                                                             uint4 *__restrict__ frag) {
    __shared__ uint32_t sp[kPlaneDwords], sm[kPlaneDwords];
    for (int i = threadIdx.x; i < kPlaneDwords; i += blockDim.x) {
        sp[i] = q.pattern[i];
        sm[i] = q.mask[i];
    }
    __syncthreads();
    const int idx = blockIdx.x * blockDim.x + threadIdx.x;
    if (idx >= kPlaneDwords * 32) return;
    const int k = idx & 31, w = idx >> 5;
    uint32_t mw = 0, pw = 0;
    if (k < kRot) {
        mw = rot_dword(sm, k - 15, w);
        pw = rot_dword(sp, k - 15, w);
    }
    *(uint2 *)&tab[w * kTemplateTabStride + 2 * k] = make_uint2(mw, pw);
    uint32_t f[4] = {0, 0, 0, 0};
#pragma unroll
    for (int j = 0; j < 32; ++j) {
        const int b = frag_bit(j);
        const uint32_t code = ((mw >> b) & 1u) ? (((pw >> b) & 1u) ? 0xAu : 0x2u) : 0u;
        f[j >> 3] |= code << (4 * (j & 7));
    }
    const int c = w >> 1, h = w & 1;
    frag[c * 64 + k + 32 * h] = make_uint4(f[0], f[1], f[2], f[3]);
}

// MASKS: table [w*32 + k] = mask_k dword w; compact fragments dword
// [((c/4)*64 + k + 32h) * 4 + c%4] bit 4 (j%8) + {2,1,0,3}[j/8] = bit
// mask_frag_bit(j) of dword w = 2c + h (build_masks_table / build_masks_frags).
__global__ void __launch_bounds__(256) query_masks_kernel(const MaskArg qmask, uint32_t *__restrict__ tab,
                                                          uint32_t *__restrict__ frag) {
    __shared__ uint32_t sm[kPlaneDwords];
    for (int i = threadIdx.x; i < kPlaneDwords; i += blockDim.x) sm[i] = qmask.mask[i];
    __syncthreads();
    const int idx = blockIdx.x * blockDim.x + threadIdx.x;
    if (idx >= kPlaneDwords * 32) return;
    const int k = idx & 31, w = idx >> 5;
    const uint32_t x = k < kRot ? rot_dword(sm, k - 15, w) : 0u;
    tab[w * kSlotTabStride + k] = x;
    uint32_t f = 0;
#pragma unroll
    for (int j = 0; j < 32; ++j) {
        const int bitpos = (j >> 3) == 3 ? 3 : 2 - (j >> 3);  // {2, 1, 0, 3}[j / 8]
        f |= ((x >> mask_frag_bit(j)) & 1u) << (4 * (j & 7) + bitpos);
    }
    const int c = w >> 1, h = w & 1;
    frag[((c >> 2) * 64 + k + 32 * h) * 4 + (c & 3)] = f;
}

// SHARES (one workgroup per row k): table [d*32 + k] = rot_k[2d] | rot_k[2d+1] << 16;
// i8 fragments: element e = 32c + 16h + j of row k at byte
// ((2c)*64 + k + 32h)*16 + j (low byte ^ 0x80) and ((2c+1)*64 + k + 32h)*16 + j
// (high byte ^ 0x80); row 31 all ones; after the fragments the 32 int2 row
// sums of the biased bytes (row 31: 0) — build_shares_table / build_shares_frags.
__global__ void __launch_bounds__(256) query_shares_kernel(const uint16_t *__restrict__ q, uint32_t *__restrict__ tab,
                                                           uint32_t *__restrict__ frag) {
    __shared__ uint16_t sq[IRIS_BITS];
    __shared__ int red[2][8];
    for (int i = threadIdx.x; i < IRIS_BITS / 2; i += blockDim.x) ((uint32_t *)sq)[i] = ((const uint32_t *)q)[i];
    __syncthreads();
    const int k = blockIdx.x, r = k - 15;
    int slo = 0, shi = 0;
    // thread item: 4 consecutive elements e = 4i .. 4i+3 (same chunk c, half h)
    for (int i = threadIdx.x; i < IRIS_BITS / 4; i += blockDim.x) {
        uint32_t lo = 0x01010101u, hi = 0x01010101u;
        uint32_t v[4] = {0, 0, 0, 0};
        if (k < kRot) {
            lo = 0;
            hi = 0;
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                const int e = 4 * i + u, row = e / IRIS_COLS, col = e - row * IRIS_COLS;
                int sc = col - r;
                sc += sc < 0 ? IRIS_COLS : 0;
                sc -= sc >= IRIS_COLS ? IRIS_COLS : 0;
                v[u] = sq[row * IRIS_COLS + sc];
                const uint32_t bl = (v[u] & 0xFFu) ^ 0x80u, bh = (v[u] >> 8) ^ 0x80u;
                lo |= bl << (8 * u);
                hi |= bh << (8 * u);
                slo += (int8_t)bl;
                shi += (int8_t)bh;
            }
        }
        tab[(2 * i) * kSlotTabStride + k] = v[0] | (v[1] << 16);
        tab[(2 * i + 1) * kSlotTabStride + k] = v[2] | (v[3] << 16);
        const int e = 4 * i, c = e >> 5, h = (e >> 4) & 1, j = e & 15;
        frag[((2 * c) * 64 + k + 32 * h) * 4 + (j >> 2)] = lo;
        frag[((2 * c + 1) * 64 + k + 32 * h) * 4 + (j >> 2)] = hi;
    }
    // workgroup sums of the biased bytes
    for (int off = 32; off >= 1; off >>= 1) {
        slo += __shfl_xor(slo, off);
        shi += __shfl_xor(shi, off);
    }
    if ((threadIdx.x & 63) == 0) {
        red[0][threadIdx.x >> 6] = slo;
        red[1][threadIdx.x >> 6] = shi;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        int a = 0, b = 0;
        for (int wv = 0; wv < (int)(blockDim.x >> 6); ++wv) {
            a += red[0][wv];
            b += red[1][wv];
        }
        int32_t *qsum = (int32_t *)(frag + 4 * kShareFragUint4);
        qsum[2 * k] = a;
        qsum[2 * k + 1] = b;
    }
}

// Batched-query tiles (iris_batch.hip's A operand): query i's 31 rotated copies
// as records 0..30 of a TILES template tile, record 31 zero (build_query_tile).
// One workgroup per query; queries nq .. nqp-1 are zero tiles.
__global__ void __launch_bounds__(256) query_tiles_kernel(const iris_template_t *__restrict__ queries, uint32_t nq,
                                                          uint4 *__restrict__ tiles) {
    __shared__ uint32_t sp[kPlaneDwords], sm[kPlaneDwords];
    const uint32_t qi = blockIdx.x;
    uint4 *tile = tiles + (size_t)qi * kPlaneGroups * 64;
    if (qi >= nq) {
        for (int i = threadIdx.x; i < kPlaneGroups * 64; i += blockDim.x) tile[i] = make_uint4(0, 0, 0, 0);
        return;
    }
    for (int i = threadIdx.x; i < kPlaneDwords; i += blockDim.x) {
        sp[i] = ((const uint32_t *)queries[qi].pattern)[i];
        sm[i] = ((const uint32_t *)queries[qi].mask)[i];
    }
    __syncthreads();
    for (int i = threadIdx.x; i < kPlaneGroups * 64; i += blockDim.x) {
        const int g = i >> 6, L = i & 63, k = L & 31, h = L >> 5;
        uint4 v = make_uint4(0, 0, 0, 0);
        if (k < kRot) {
            const uint32_t em0 = rot_dword(sm, k - 15, 4 * g + h), ep0 = rot_dword(sp, k - 15, 4 * g + h);
            const uint32_t em1 = rot_dword(sm, k - 15, 4 * g + 2 + h), ep1 = rot_dword(sp, k - 15, 4 * g + 2 + h);
            v = make_uint4(xpack(em0 & 0xFFFFu, ep0 & 0xFFFFu), xpack(em0 >> 16, ep0 >> 16),
                           xpack(em1 & 0xFFFFu, ep1 & 0xFFFFu), xpack(em1 >> 16, ep1 >> 16));
        }
        tile[i] = v;
    }
}

// q / qmask: HOST pointers (copied into the kernel arguments at launch)
int launch_query_template(void *stream, const void *q, uint32_t *tab, uint32_t *frag) {
    TemplateArg a;
    memcpy(a.pattern, ((const iris_template_t *)q)->pattern, sizeof(a.pattern));
    memcpy(a.mask, ((const iris_template_t *)q)->mask, sizeof(a.mask));
    hipLaunchKernelGGL(query_template_kernel, dim3(kPlaneDwords * 32 / 256), dim3(256), 0, (hipStream_t)stream, a,
                       tab, (uint4 *)frag);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

int launch_query_masks(void *stream, const void *qmask, uint32_t *tab, uint32_t *frag) {
    MaskArg a;
    memcpy(a.mask, qmask, sizeof(a.mask));
    hipLaunchKernelGGL(query_masks_kernel, dim3(kPlaneDwords * 32 / 256), dim3(256), 0, (hipStream_t)stream, a, tab,
                       frag);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

int launch_query_shares(void *stream, const void *q, uint32_t *tab, uint32_t *frag) {
    hipLaunchKernelGGL(query_shares_kernel, dim3(32), dim3(256), 0, (hipStream_t)stream, (const uint16_t *)q, tab,
                       frag);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

int launch_query_tiles(void *stream, const void *queries, uint32_t nq, uint32_t nqp, uint32_t *tiles) {
    if (nqp == 0) return 0;
    hipLaunchKernelGGL(query_tiles_kernel, dim3(nqp), dim3(256), 0, (hipStream_t)stream,
                       (const iris_template_t *)queries, nq, (uint4 *)tiles);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

}  // namespace iris
