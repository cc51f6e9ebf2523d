// iris_batch.hip — many queries x 31 rotations x N templates (BASELINE configs[2]).
//
// The fp4 formulation of iris_mfma.hip turns a query batch into a GEMM with
// M = 32 rows per query (31 rotations + a zero row), N = templates, K = 12800
// bits, two products (den, encode) per K.  Neither operand fits on chip for
// 1024 queries x 10M templates, so it is tiled like a GEMM:
//
//   workgroup (8 waves) = 4 queries x 8 template tiles (256 templates)
//   wave w              = query (w & 3) x tiles 4 (w >> 2) .. +3  (128 f32 acc)
//   K-step              = 4 chunks of 64 bits, double-buffered in LDS:
//                         A 4 queries x 4 chunks x 64 lanes x 8 B  (8 KB)
//                         B 8 tiles   x 4 chunks x 64 lanes x 8 B  (16 KB)
//
// A (queries) is stored like a template tile: the 31 rotated copies of a query
// packed with xpack (iris_internal.hpp) as records 0..30 of a TILES tile, so
// one expansion routine turns either side into fp4 operands.  Workgroups
// sharing a query group walk the template N-groups with a stride, and all
// query groups walk the same N-groups at once, so a template tile is fetched
// from HBM about once per XCD and re-read from L2 by the other query groups.
// Per query the kernel keeps a running best (exact fraction, lowest index),
// one partial per (query, workgroup), reduced by reduce_kernel per query.
#include <hip/hip_runtime.h>

#include "iris_internal.hpp"

namespace iris {

typedef int v8i __attribute__((ext_vector_type(8)));
typedef float v16f __attribute__((ext_vector_type(16)));

constexpr int BQ = 4;                     // queries per workgroup
constexpr int BT = 8;                     // template tiles per N-group
constexpr int WT = 4;                     // tiles per wave
constexpr int KSTEP = 4;                  // chunks per K-step
constexpr int NSTEPS = kPlaneDwords / 2 / KSTEP;  // 50
constexpr int kTileU4 = kPlaneGroups * 64;        // 6400 uint4 per tile

__device__ __forceinline__ v16f mfma4(const v8i &a, const v8i &b, const v16f &c) {
    return __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(a, b, c, 4, 4, 0, 127, 0, 127);
}

__device__ __forceinline__ bool b_better(const Partial &a, const Partial &b) {
    if (a.den == 0) return false;
    if (b.den == 0) return true;
    const uint32_t l = a.num * b.den, r = b.num * a.den;
    if (l != r) return l < r;
    return a.idx < b.idx;
}

__device__ __forceinline__ Partial b_shfl(const Partial &c, int off) {
    Partial o;
    o.num = __shfl_xor(c.num, off);
    o.den = __shfl_xor(c.den, off);
    o.rot = __shfl_xor(c.rot, off);
    o.pad = 0;
    const uint32_t lo = __shfl_xor((uint32_t)c.idx, off), hi = __shfl_xor((uint32_t)(c.idx >> 32), off);
    o.idx = ((uint64_t)hi << 32) | lo;
    return o;
}

__global__ void __launch_bounds__(512, 1)
    batch_kernel(const uint4 *__restrict__ db, const uint4 *__restrict__ qtiles, uint64_t tile0, uint64_t ntiles,
                 uint64_t first, uint64_t end, uint32_t nqg, uint32_t G, Partial *__restrict__ partials) {
    __shared__ uint2 sA[2][BQ][KSTEP][64];
    __shared__ uint2 sB[2][BT][KSTEP][64];
    __shared__ Partial sP[8];

    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const uint32_t qg = blockIdx.x % nqg, gi = blockIdx.x / nqg;
    const int wq = w & 3, wsub = (w >> 2) * WT;
    const uint64_t ngroups = (ntiles + BT - 1) / BT;

    // loader roles: A: query (tid >> 7), chunk pair (tid >> 6) & 1, lane; B: tile (tid >> 6), lane, both pairs
    const uint4 *qsrc = qtiles + (uint64_t)(qg * BQ + (tid >> 7)) * kTileU4 + ((tid >> 6) & 1) * 64 + lane;
    const int lb_t = tid >> 6;

    Partial best;
    best.num = 0;
    best.den = 0;
    best.rot = 0;
    best.pad = 0;
    best.idx = ~0ull;

    for (uint64_t ng = gi; ng < ngroups; ng += G) {
        const uint64_t trel = ng * BT + lb_t;
        const uint4 *bsrc = db + (tile0 + (trel < ntiles ? trel : ntiles - 1)) * (uint64_t)kTileU4 + lane;
        v16f den[WT], s[WT];
#pragma unroll
        for (int t = 0; t < WT; ++t)
#pragma unroll
            for (int i = 0; i < 16; ++i) {
                den[t][i] = 0.f;
                s[t][i] = 0.f;
            }
        uint4 ra, rb0, rb1;
        auto gload = [&](int step) {  // chunk pairs 2*step, 2*step+1
            ra = qsrc[(2 * step) * 64];
            rb0 = bsrc[(2 * step) * 64];
            rb1 = bsrc[(2 * step + 1) * 64];
        };
        auto lstore = [&](int buf) {
            const int qa = tid >> 7, gp = (tid >> 6) & 1;
            sA[buf][qa][2 * gp][lane] = make_uint2(ra.x, ra.y);
            sA[buf][qa][2 * gp + 1][lane] = make_uint2(ra.z, ra.w);
            sB[buf][lb_t][0][lane] = make_uint2(rb0.x, rb0.y);
            sB[buf][lb_t][1][lane] = make_uint2(rb0.z, rb0.w);
            sB[buf][lb_t][2][lane] = make_uint2(rb1.x, rb1.y);
            sB[buf][lb_t][3][lane] = make_uint2(rb1.z, rb1.w);
        };
        gload(0);
        lstore(0);
        __syncthreads();
#pragma unroll 1
        for (int st = 0; st < NSTEPS; ++st) {
            const int buf = st & 1;
            if (st + 1 < NSTEPS) gload(st + 1);
#pragma unroll
            for (int c = 0; c < KSTEP; ++c) {
                const uint2 a = sA[buf][wq][c][lane];
                const v8i aden = {(int)(a.x & 0x22222222u), (int)((a.x & 0x11111111u) << 2), (int)(a.y & 0x22222222u),
                                  (int)((a.y & 0x11111111u) << 2), 0, 0, 0, 0};
                const v8i aenc = {(int)(a.x & 0xAAAAAAAAu), (int)((a.x << 1) & 0xAAAAAAAAu), (int)(a.y & 0xAAAAAAAAu),
                                  (int)((a.y << 1) & 0xAAAAAAAAu), 0, 0, 0, 0};
#pragma unroll
                for (int t = 0; t < WT; ++t) {
                    const uint2 b = sB[buf][wsub + t][c][lane];
                    const v8i bden = {(int)(b.x & 0x22222222u), (int)(b.x & 0x11111111u), (int)(b.y & 0x22222222u),
                                      (int)(b.y & 0x11111111u), 0, 0, 0, 0};
                    const v8i benc = {(int)(b.x & 0xAAAAAAAAu), (int)((b.x << 1) & 0xAAAAAAAAu),
                                      (int)(b.y & 0xAAAAAAAAu), (int)((b.y << 1) & 0xAAAAAAAAu), 0, 0, 0, 0};
                    den[t] = mfma4(aden, bden, den[t]);
                    s[t] = mfma4(aenc, benc, s[t]);
                }
            }
            if (st + 1 < NSTEPS) lstore(buf ^ 1);
            __syncthreads();
        }
        // per template: min over the 16 rows of this lane, then the partner half
        const int h = lane >> 5;
#pragma unroll
        for (int t = 0; t < WT; ++t) {
            uint32_t bn = 0, bd = 0;
            int br = 0;
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int k = (r & 3) + 8 * (r >> 2) + 4 * h;
                const uint32_t dd = (uint32_t)den[t][r];
                const uint32_t nn = (uint32_t)(((int)dd - (int)s[t][r]) >> 1);
                if (k < kRot && dd != 0 && (bd == 0 || nn * bd < bn * dd)) {
                    bn = nn;
                    bd = dd;
                    br = k;
                }
            }
            const uint32_t pn = __shfl_xor(bn, 32), pd = __shfl_xor(bd, 32);
            const int pr = __shfl_xor(br, 32);
            if (pd != 0 && (bd == 0 || pn * bd < bn * pd || (pn * bd == bn * pd && pr < br))) {
                bn = pn;
                bd = pd;
                br = pr;
            }
            const uint64_t trel2 = ng * BT + wsub + t;
            const uint64_t tg = (tile0 + trel2) * 32 + (lane & 31);
            const bool valid = trel2 < ntiles && tg >= first && tg < end;
            Partial c;
            c.num = bn;
            c.den = valid ? bd : 0;
            c.rot = br;
            c.pad = 0;
            c.idx = tg - first;
            if (b_better(c, best)) best = c;
        }
    }
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) {
        const Partial o = b_shfl(best, off);
        if (b_better(o, best)) best = o;
    }
    if (lane == 0) sP[w] = best;
    __syncthreads();
    if (tid < BQ) {
        Partial b = sP[tid];
        if (b_better(sP[tid + 4], b)) b = sP[tid + 4];
        partials[(uint64_t)(qg * BQ + tid) * G + gi] = b;
    }
}

// one workgroup per query: reduce its G partials
__global__ void __launch_bounds__(256) batch_reduce_kernel(const Partial *__restrict__ partials, uint32_t G,
                                                           Partial *__restrict__ out) {
    const uint32_t q = blockIdx.x;
    Partial c;
    c.num = 0;
    c.den = 0;
    c.rot = 0;
    c.pad = 0;
    c.idx = ~0ull;
    for (uint32_t i = threadIdx.x; i < G; i += blockDim.x) {
        const Partial p = partials[(uint64_t)q * G + i];
        if (b_better(p, c)) c = p;
    }
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) {
        const Partial o = b_shfl(c, off);
        if (b_better(o, c)) c = o;
    }
    __shared__ Partial sh[4];
    if ((threadIdx.x & 63) == 0) sh[threadIdx.x >> 6] = c;
    __syncthreads();
    if (threadIdx.x == 0) {
        Partial b = sh[0];
        for (int i = 1; i < 4; ++i)
            if (b_better(sh[i], b)) b = sh[i];
        out[q] = b;
    }
}

BatchGeometry batch_geometry(LaunchRange r, uint32_t nq) {
    BatchGeometry g;
    g.tile0 = r.first / 32;
    const uint64_t tile1 = (r.first + r.n + 31) / 32;
    g.ntiles = tile1 - g.tile0;
    g.nqg = (nq + BQ - 1) / BQ;
    const uint64_t ngroups = (g.ntiles + BT - 1) / BT;
    uint64_t G = (512 + g.nqg - 1) / g.nqg;  // ~2 workgroups per CU in total
    if (G > ngroups) G = ngroups ? ngroups : 1;
    g.G = (uint32_t)G;
    return g;
}

int launch_batch(void *stream, const void *db, const void *qtiles, LaunchRange r, const BatchGeometry &g,
                 Partial *partials, Partial *out) {
    if (r.n == 0) return 0;
    hipLaunchKernelGGL(batch_kernel, dim3(g.nqg * g.G), dim3(512), 0, (hipStream_t)stream, (const uint4 *)db,
                       (const uint4 *)qtiles, g.tile0, g.ntiles, r.first, r.first + r.n, g.nqg, g.G, partials);
    if (hipGetLastError() != hipSuccess) return -1;
    hipLaunchKernelGGL(batch_reduce_kernel, dim3(g.nqg * BQ), dim3(256), 0, (hipStream_t)stream, partials, g.G, out);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

}  // namespace iris
