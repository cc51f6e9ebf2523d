// iris_mfma.hip — Template masked Hamming on the gfx950 matrix cores (fp4).
//
// Why MFMA for bit work: on gfx950 the integer VALU ops this path needs
// (v_bcnt, v_bitop3) issue at 16 lanes/clk, so the XOR+AND+popcount form is
// capped near 39 T lane-ops/s = ~11 ms per 10M templates (35 % of the HBM
// roofline; tools/ubench_ops.hip).  The same numbers are an
// exact integer matrix product:
//
//   den[k][t] = sum_b qm_k[b] * em_t[b]                       (jointly valid bits)
//   S  [k][t] = sum_b enc(q_k)[b] * enc(e_t)[b],  enc in {0,+1,-1}  (src/lib.rs:16-26)
//   num       = (den - S) / 2                                 (src/lib.rs:134-163 identity)
//
// with M = 32 rotation rows (k = 0..30 + a zero row), N = 32 templates per
// tile, K = 12800 bits: v_mfma_scale_f32_32x32x64_f8f6f4 with e2m1 operands.
// Every product is 0 or +-1 and every sum is an integer <= 12800 < 2^24, so the
// f32 accumulation is exact whatever the internal order.
//
// Operands: the 31 rotated query copies are precomputed once per engine as
// fp4 A-fragments (iris_host.cpp, 400 KB, L2-resident).  The template side
// is streamed from HBM once in the TILES layout (iris_internal.hpp), whose
// interleaved dwords turn into fp4 B-fragments with four v_and + two
// shift-and per dword pair — fast VOP2 ops, hidden under the MFMAs.
#include <hip/hip_runtime.h>
#include <stdlib.h>

#include "iris_device.hpp"

namespace iris {

typedef int v8i __attribute__((ext_vector_type(8)));
typedef float v16f __attribute__((ext_vector_type(16)));

constexpr int kTileRecs = 32;
constexpr int kTileUint4 = kPlaneGroups * 64;  // 6400 uint4 = 102400 B per tile
constexpr int kMfmaTiles = 4;    // tiles per wave (128 templates)
constexpr int kMfmaWgs = 2;      // workgroups per CU the register budget allows
constexpr int kSplitStages = 6;  // load ring depth of the K-split (small-range) form
// tiles per workgroup of the K-split form: every query-fragment load (2 per chunk pair and
// wave, from L2) feeds this many tiles -- at 1 the query stream is twice the template stream
constexpr int kSplitT = 2;

__device__ __forceinline__ v16f mfma_fp4(const v8i &a, const v8i &b, const v16f &c) {
    // cbsz = blgp = 4: both operands e2m1; scales 127 = 2^0 (e8m0)
    return __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(a, b, c, 4, 4, 0, 127, 0, 127);
}

// Query-side den operand from the enc operand: |enc| as fp4 1.0, doubled to
// 2.0 in the dwords whose template-side value is 0.5 (fragment dwords 1, 3).
struct QFrag {
    v8i am, ae;
};
__device__ __forceinline__ QFrag qfrag_of(const uint4 &qe) {
    QFrag f;
    f.ae = v8i{(int)qe.x, (int)qe.y, (int)qe.z, (int)qe.w, 0, 0, 0, 0};
    f.am = v8i{(int)(qe.x & 0x22222222u), (int)((qe.y & 0x22222222u) << 1), (int)(qe.z & 0x22222222u),
               (int)((qe.w & 0x22222222u) << 1), 0, 0, 0, 0};
    return f;
}

// One 64-bit chunk of K for one tile.  x0/x1: the lane's interleaved dwords.
__device__ __forceinline__ void chunk_step(uint32_t x0, uint32_t x1, const QFrag &q, v16f &den, v16f &s) {
    const v8i bm = {(int)(x0 & 0x22222222u), (int)(x0 & 0x11111111u), (int)(x1 & 0x22222222u),
                    (int)(x1 & 0x11111111u), 0, 0, 0, 0};
    const v8i be = {(int)(x0 & 0xAAAAAAAAu), (int)((x0 << 1) & 0xAAAAAAAAu), (int)(x1 & 0xAAAAAAAAu),
                    (int)((x1 << 1) & 0xAAAAAAAAu), 0, 0, 0, 0};
    den = mfma_fp4(q.am, bm, den);
    s = mfma_fp4(q.ae, be, s);
}

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ uint4 stream_load(const uint4 *p) {
    const u32x4 v = __builtin_nontemporal_load((const u32x4 *)p);
    return make_uint4(v.x, v.y, v.z, v.w);
}

enum { MF_COUNTS = 0, MF_SEARCH = 1 };

// KS > 1 (small ranges, T = kSplitT): the KS waves of a tile group split K -- wave w computes
// chunk groups [w' * 100 / KS, +100 / KS) of tiles T * (blockIdx.x * (4 / KS) + w / KS) + t (w' = w % KS)
// -- and the partial sums (exact integers in f32) meet in LDS before the epilogue, so a range of
// a few hundred tiles still puts several waves on every SIMD.
// FUSED (search, small grids): the last workgroup to finish folds every workgroup's
// partial and writes the winner to fin.dst itself (iris_device.hpp, fold_partials_last).
template <int MODE, int T = kMfmaTiles, int KS = 1, bool FUSED = false>
__global__ void __launch_bounds__(64 * kWaveSlots, kMfmaWgs)
    template_mfma_kernel(const uint4 *__restrict__ db, const uint4 *__restrict__ qfrag, uint64_t tile0,
                         uint64_t ntiles, uint64_t first, uint64_t end, uint16_t *__restrict__ num_out,
                         uint16_t *__restrict__ den_out, double *__restrict__ dist_out,
                         Partial *__restrict__ partials, FusedFinish fin) {
    constexpr int W = kWaveSlots;
    static_assert(KS == 1 || (W % KS == 0 && kPlaneGroups % KS == 0), "K-split geometry");
    const int lane = threadIdx.x & 63;
    const int wslot = threadIdx.x >> 6;
    const int slice = wslot % KS;
    const uint64_t wave = (uint64_t)blockIdx.x * (W / KS) + wslot / KS;
    const uint64_t tw = wave * T;  // first tile (relative to tile0) of this wave
    const bool active = tw < ntiles;  // wave-uniform
    constexpr int kG = kPlaneGroups / KS;  // chunk groups of this wave's K-slice
    const int g0 = slice * kG;

    v16f den[T], s[T];
#pragma unroll
    for (int t = 0; t < T; ++t) {
#pragma unroll
        for (int i = 0; i < 16; ++i) {
            den[t][i] = 0.f;
            s[t][i] = 0.f;
        }
    }

    if (active) {
        // 3-stage register pipeline: the loads of step g+2 are in flight
        // while step g computes (one step = 2 chunks = 16 MFMAs per wave).
        const uint4 *dp[T];
#pragma unroll
        for (int t = 0; t < T; ++t) {
            const uint64_t rel = (tw + t < ntiles) ? tw + t : ntiles - 1;  // clamp: extra tiles re-read a valid one
            dp[t] = db + (tile0 + rel) * (uint64_t)kTileUint4 + lane;
        }
        const uint4 *qp = qfrag + lane;  // chunk c: qfrag[c * 64 + lane]
        struct Stage {
            uint4 d[T];
            uint4 q0, q1;
        };
        auto load = [&](Stage &st, int g) {
            g = (g < kG ? g : kG - 1) + g0;
#pragma unroll
            for (int t = 0; t < T; ++t) st.d[t] = stream_load(dp[t] + g * 64);
            st.q0 = qp[(2 * g) * 64];
            st.q1 = qp[(2 * g + 1) * 64];
            // keep this stage's loads together and ahead of the compute that
            // follows: vmcnt retires in order, so a query load sunk next to
            // its use would also drain the HBM prefetches issued before it
            __builtin_amdgcn_sched_barrier(0);
        };
        auto compute = [&](const Stage &st) {
            const QFrag f0 = qfrag_of(st.q0);
#pragma unroll
            for (int t = 0; t < T; ++t) chunk_step(st.d[t].x, st.d[t].y, f0, den[t], s[t]);
            const QFrag f1 = qfrag_of(st.q1);
#pragma unroll
            for (int t = 0; t < T; ++t) chunk_step(st.d[t].z, st.d[t].w, f1, den[t], s[t]);
        };
        if constexpr (KS > 1) {
            // K-slice of kG = 25 steps, fully unrolled over a kSplitStages-deep ring: the wave
            // keeps (kSplitStages - 1) steps of loads in flight instead of 2, so a range of a
            // few hundred tiles -- one short slice per wave, nothing to overlap between
            // slices -- is not bound by one HBM round trip per two steps
            Stage st[kSplitStages];
#pragma unroll
            for (int i = 0; i < kSplitStages - 1; ++i) load(st[i], i);
#pragma unroll
            for (int g = 0; g < kG; ++g) {
                if (g + kSplitStages - 1 < kG) load(st[(g + kSplitStages - 1) % kSplitStages], g + kSplitStages - 1);
                compute(st[g % kSplitStages]);
            }
        } else {
            Stage sa, sb, sc;
            load(sa, 0);
            load(sb, 1);
            int g = 0;
#pragma unroll 1
            for (; g + 3 <= kG; g += 3) {
                load(sc, g + 2);
                compute(sa);
                load(sa, g + 3);
                compute(sb);
                load(sb, g + 4);
                compute(sc);
            }
            // kG = 3q + {1, 2} (100; 50): the remaining steps' data is in sa (, sb)
            if constexpr (kG % 3 >= 1) compute(sa);
            if constexpr (kG % 3 == 2) compute(sb);
        }
    }
    if constexpr (KS > 1) {  // the K-slices' partial sums -> slice 0's accumulators (exact)
        __shared__ float red[W][T][32][64];
        if (slice != 0) {
#pragma unroll
            for (int t = 0; t < T; ++t)
#pragma unroll
                for (int i = 0; i < 16; ++i) {
                    red[wslot][t][i][lane] = den[t][i];
                    red[wslot][t][16 + i][lane] = s[t][i];
                }
        }
        __syncthreads();
        if (slice == 0) {
#pragma unroll
            for (int k = 1; k < KS; ++k)
#pragma unroll
                for (int t = 0; t < T; ++t)
#pragma unroll
                    for (int i = 0; i < 16; ++i) {
                        den[t][i] += red[wslot + k][t][i][lane];
                        s[t][i] += red[wslot + k][t][16 + i][lane];
                    }
        }
    }

    // C layout: lane l holds template (l & 31) of the tile and rotation rows
    // k = (r & 3) + 8 (r >> 2) + 4 (l >> 5), r = 0..15.
    const int h = lane >> 5;
    Partial best = partial_none();
#pragma unroll
    for (int t = 0; t < T; ++t) {
        const uint64_t t0 = (tile0 + tw + t) * kTileRecs;  // global index of the tile's first template
        const bool tv = active && (tw + t < ntiles) && slice == 0;
        if constexpr (MODE == MF_COUNTS) {
            __shared__ __attribute__((aligned(16))) uint16_t sh_out[W][1024];
            uint16_t *lds = sh_out[wslot];
            if (num_out)
                store_tile_rows(num_out, lds, t0, first, end, tv, lane,
                                [&](int r) { return (uint16_t)(((int)den[t][r] - (int)s[t][r]) >> 1); });
            if (den_out)
                store_tile_rows(den_out, lds, t0, first, end, tv, lane,
                                [&](int r) { return (uint16_t)(uint32_t)den[t][r]; });
        } else {
            const uint64_t tg = t0 + (lane & 31);
            const bool valid = tv && tg >= first && tg < end;
            const uint64_t o = tg - first;
            uint32_t bn, bd;
            int br;
            best_rotation(lane, [&](int r, uint32_t &nn, uint32_t &dd) {
                dd = (uint32_t)den[t][r];
                nn = (uint32_t)(((int)dd - (int)s[t][r]) >> 1);  // num = (den - S) / 2
            }, bn, bd, br);
            if (valid && dist_out && h == 0) dist_out[o] = bd ? (double)bn / (double)bd : __builtin_inf();
            Partial c;
            c.num = bn;
            c.den = valid ? bd : 0;
            c.rot = br;
            c.pad = 0;
            c.idx = o;
            if (partial_better_dev(c, best)) best = c;
        }
    }
    if constexpr (MODE == MF_SEARCH) {
#pragma unroll
        for (int off = 32; off >= 1; off >>= 1) {
            const Partial ot = partial_shfl_xor(best, off);
            if (partial_better_dev(ot, best)) best = ot;
        }
        __shared__ Partial sh[W];
        if (lane == 0) sh[wslot] = best;
        __syncthreads();
        Partial b = sh[0];
        if (threadIdx.x == 0) {
#pragma unroll
            for (int w = 1; w < W; ++w)
                if (partial_better_dev(sh[w], b)) b = sh[w];
            if constexpr (!FUSED) partials[blockIdx.x] = b;
        }
        if constexpr (FUSED) fold_partials_last(partials, b, fin);
    }
}

// ------------------------------------------------------------------ a few queries per pass

// NQ queries against one streamed pass of the database: per 64-bit chunk and
// tile 2 NQ MFMAs share one expansion of the template bits, so up to NQ = 2 the
// pass stays near the HBM bound while one single-query pass per query would
// stream the database NQ times.  T = 4 / NQ tiles per wave keeps the NQ x T x 2
// accumulators at 128 VGPRs.  Partials: [NQ][gridDim.x].
struct QueryFrags {
    const uint4 *q[4];
};

template <int NQ>
__global__ void __launch_bounds__(256, 2)
    template_multi_kernel(const uint4 *__restrict__ db, QueryFrags qf, uint64_t tile0, uint64_t ntiles,
                          uint64_t first, uint64_t end, Partial *__restrict__ partials) {
    constexpr int T = 4 / NQ;
    const int lane = threadIdx.x & 63;
    const int wslot = threadIdx.x >> 6;
    const uint64_t wave = (uint64_t)blockIdx.x * kWaveSlots + wslot;
    const uint64_t tw = wave * T;
    const bool active = tw < ntiles;  // wave-uniform

    v16f den[NQ][T], s[NQ][T];
#pragma unroll
    for (int qi = 0; qi < NQ; ++qi)
#pragma unroll
        for (int t = 0; t < T; ++t)
#pragma unroll
            for (int i = 0; i < 16; ++i) {
                den[qi][t][i] = 0.f;
                s[qi][t][i] = 0.f;
            }

    if (active) {
        const uint4 *dp[T];
#pragma unroll
        for (int t = 0; t < T; ++t) {
            const uint64_t rel = (tw + t < ntiles) ? tw + t : ntiles - 1;
            dp[t] = db + (tile0 + rel) * (uint64_t)kTileUint4 + lane;
        }
        struct Stage {
            uint4 d[T];
            uint4 q[NQ][2];
        };
        auto load = [&](Stage &st, int g) {
            g = g < kPlaneGroups ? g : kPlaneGroups - 1;
#pragma unroll
            for (int t = 0; t < T; ++t) st.d[t] = stream_load(dp[t] + g * 64);
#pragma unroll
            for (int qi = 0; qi < NQ; ++qi) {
                st.q[qi][0] = qf.q[qi][(2 * g) * 64 + lane];
                st.q[qi][1] = qf.q[qi][(2 * g + 1) * 64 + lane];
            }
            __builtin_amdgcn_sched_barrier(0);
        };
        auto compute = [&](const Stage &st) {
#pragma unroll
            for (int qi = 0; qi < NQ; ++qi) {
                const QFrag f0 = qfrag_of(st.q[qi][0]);
#pragma unroll
                for (int t = 0; t < T; ++t) chunk_step(st.d[t].x, st.d[t].y, f0, den[qi][t], s[qi][t]);
                const QFrag f1 = qfrag_of(st.q[qi][1]);
#pragma unroll
                for (int t = 0; t < T; ++t) chunk_step(st.d[t].z, st.d[t].w, f1, den[qi][t], s[qi][t]);
            }
        };
        Stage sa, sb, sc;
        load(sa, 0);
        load(sb, 1);
        int g = 0;
#pragma unroll 1
        for (; g + 3 <= kPlaneGroups; g += 3) {
            load(sc, g + 2);
            compute(sa);
            load(sa, g + 3);
            compute(sb);
            load(sb, g + 4);
            compute(sc);
        }
        if (g < kPlaneGroups) compute(sa);
    }

    Partial best[NQ];
#pragma unroll
    for (int qi = 0; qi < NQ; ++qi) best[qi] = partial_none();
#pragma unroll
    for (int t = 0; t < T; ++t) {
        const uint64_t tg = (tile0 + tw + t) * kTileRecs + (lane & 31);
        const bool valid = active && (tw + t < ntiles) && tg >= first && tg < end;
#pragma unroll
        for (int qi = 0; qi < NQ; ++qi) {
            uint32_t bn, bd;
            int br;
            best_rotation(lane, [&](int r, uint32_t &nn, uint32_t &dd) {
                dd = (uint32_t)den[qi][t][r];
                nn = (uint32_t)(((int)dd - (int)s[qi][t][r]) >> 1);
            }, bn, bd, br);
            Partial c;
            c.num = bn;
            c.den = valid ? bd : 0;
            c.rot = br;
            c.pad = 0;
            c.idx = tg - first;
            if (partial_better_dev(c, best[qi])) best[qi] = c;
        }
    }
    __shared__ Partial sh[NQ][kWaveSlots];
#pragma unroll
    for (int qi = 0; qi < NQ; ++qi) {
#pragma unroll
        for (int off = 32; off >= 1; off >>= 1) {
            const Partial ot = partial_shfl_xor(best[qi], off);
            if (partial_better_dev(ot, best[qi])) best[qi] = ot;
        }
        if (lane == 0) sh[qi][wslot] = best[qi];
    }
    __syncthreads();
    if (threadIdx.x < NQ) {
        const int qi = threadIdx.x;
        Partial b = sh[qi][0];
#pragma unroll
        for (int w = 1; w < kWaveSlots; ++w)
            if (partial_better_dev(sh[qi][w], b)) b = sh[qi][w];
        partials[(uint64_t)qi * gridDim.x + blockIdx.x] = b;
    }
}

// ------------------------------------------------------------------ TILES layout plumbing

// reference Template record (pattern dwords 0..399, mask dwords 400..799) ->
// TILES uint4 of (record t, chunk pair g, half h)
__global__ void __launch_bounds__(256) pack_tiles_kernel(const uint32_t *__restrict__ staging,
                                                         uint4 *__restrict__ db, uint64_t t_first, uint64_t n) {
    const uint64_t total = n * (uint64_t)(2 * kPlaneGroups);
    for (uint64_t tid = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; tid < total;
         tid += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t i = tid % n, gh = tid / n;
        const int g = (int)(gh >> 1), h = (int)(gh & 1);
        const uint32_t *rec = staging + i * (2 * kPlaneDwords);
        const int w0 = 4 * g + h, w1 = 4 * g + 2 + h;
        const uint32_t em0 = rec[kPlaneDwords + w0], ep0 = rec[w0], em1 = rec[kPlaneDwords + w1], ep1 = rec[w1];
        const uint64_t t = t_first + i;
        uint4 v;
        v.x = xpack(em0 & 0xFFFFu, ep0 & 0xFFFFu);
        v.y = xpack(em0 >> 16, ep0 >> 16);
        v.z = xpack(em1 & 0xFFFFu, ep1 & 0xFFFFu);
        v.w = xpack(em1 >> 16, ep1 >> 16);
        db[(t / kTileRecs) * (uint64_t)kTileUint4 + (uint64_t)g * 64 + (t % kTileRecs) + 32 * h] = v;
    }
}

__global__ void __launch_bounds__(256) unpack_tiles_kernel(const uint4 *__restrict__ db, uint32_t *__restrict__ staging,
                                                           uint64_t t_first, uint64_t n) {
    const uint64_t total = n * (uint64_t)(2 * kPlaneGroups);
    for (uint64_t tid = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; tid < total;
         tid += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t i = tid % n, gh = tid / n;
        const int g = (int)(gh >> 1), h = (int)(gh & 1);
        const uint64_t t = t_first + i;
        const uint4 v = db[(t / kTileRecs) * (uint64_t)kTileUint4 + (uint64_t)g * 64 + (t % kTileRecs) + 32 * h];
        uint32_t a, b, c, d;
        xunpack(v.x, a, b);
        xunpack(v.y, c, d);
        uint32_t *rec = staging + i * (2 * kPlaneDwords);
        const int w0 = 4 * g + h, w1 = 4 * g + 2 + h;
        rec[kPlaneDwords + w0] = a | (c << 16);
        rec[w0] = b | (d << 16);
        xunpack(v.z, a, b);
        xunpack(v.w, c, d);
        rec[kPlaneDwords + w1] = a | (c << 16);
        rec[w1] = b | (d << 16);
    }
}

__global__ void __launch_bounds__(256) generate_tiles_kernel(uint4 *__restrict__ db, uint64_t t_first, uint64_t n,
                                                             uint64_t key, uint64_t global_index0) {
    const uint64_t total = n * (uint64_t)(2 * kPlaneGroups);
    for (uint64_t tid = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; tid < total;
         tid += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t i = tid % n, gh = tid / n;
        const int g = (int)(gh >> 1), h = (int)(gh & 1);
        const uint64_t gt = global_index0 + i;
        // dword 4g+h is half h of limb 2g, dword 4g+2+h half h of limb 2g+1
        const uint64_t m0 = gen_limb(key, gt * 400 + 200 + 2 * g), m1 = gen_limb(key, gt * 400 + 200 + 2 * g + 1);
        const uint64_t p0 = gen_limb(key, gt * 400 + 2 * g), p1 = gen_limb(key, gt * 400 + 2 * g + 1);
        const uint32_t em0 = (uint32_t)(m0 >> (32 * h)), ep0 = (uint32_t)(p0 >> (32 * h));
        const uint32_t em1 = (uint32_t)(m1 >> (32 * h)), ep1 = (uint32_t)(p1 >> (32 * h));
        const uint64_t t = t_first + i;
        uint4 v;
        v.x = xpack(em0 & 0xFFFFu, ep0 & 0xFFFFu);
        v.y = xpack(em0 >> 16, ep0 >> 16);
        v.z = xpack(em1 & 0xFFFFu, ep1 & 0xFFFFu);
        v.w = xpack(em1 >> 16, ep1 >> 16);
        db[(t / kTileRecs) * (uint64_t)kTileUint4 + (uint64_t)g * 64 + (t % kTileRecs) + 32 * h] = v;
    }
}

static int tiles_grid(uint64_t total) {
    uint64_t b = (total + 255) / 256;
    if (b > 256ull * 64) b = 256ull * 64;
    return (int)(b ? b : 1);
}

int launch_pack_tiles(void *stream, const void *staging, void *db, uint64_t t_first, uint64_t n) {
    if (n == 0) return 0;
    hipLaunchKernelGGL(pack_tiles_kernel, dim3(tiles_grid(n * 2 * kPlaneGroups)), dim3(256), 0, (hipStream_t)stream,
                       (const uint32_t *)staging, (uint4 *)db, t_first, n);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

int launch_unpack_tiles(void *stream, const void *db, void *staging, uint64_t t_first, uint64_t n) {
    if (n == 0) return 0;
    hipLaunchKernelGGL(unpack_tiles_kernel, dim3(tiles_grid(n * 2 * kPlaneGroups)), dim3(256), 0, (hipStream_t)stream,
                       (const uint4 *)db, (uint32_t *)staging, t_first, n);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

int launch_generate_tiles(void *stream, void *db, uint64_t t_first, uint64_t n, uint64_t seed, uint64_t global_index0) {
    if (n == 0) return 0;
    hipLaunchKernelGGL(generate_tiles_kernel, dim3(tiles_grid(n * 2 * kPlaneGroups)), dim3(256), 0,
                       (hipStream_t)stream, (uint4 *)db, t_first, n, gen_key(seed, 0), global_index0);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

struct TileRange {
    uint64_t tile0, ntiles, grid;
    bool fusable = false;  // small enough for the in-kernel reduce
    int tiles_per_wave;
    int ksplit;  // 4: a tile's 4 waves split K (ranges of at most kSplitTiles tiles)
};

// Below this many tiles, 4 tiles per wave would leave CUs idle (fewer than 2
// workgroups per CU): small ranges run one tile per wave, 4x the workgroups.
constexpr uint64_t kSmallTiles = 4 * kWaveSlots * 256 * 2;
// Up to this many tiles (32k templates: configs[0]'s 10k, the reference's 20k-record chunks)
// even one tile per wave leaves most SIMDs without a wave: the 4 waves of a workgroup split
// one tile's K instead.
constexpr uint64_t kSplitTiles = 1024;

static TileRange tile_range(const Hooks &h, LaunchRange r) {
    TileRange t;
    t.tile0 = r.first / kTileRecs;
    const uint64_t tile1 = (r.first + r.n + kTileRecs - 1) / kTileRecs;
    t.ntiles = tile1 - t.tile0;
    t.tiles_per_wave = t.ntiles < kSmallTiles ? 1 : kMfmaTiles;
    t.ksplit = t.ntiles <= kSplitTiles ? 4 : 1;
    // test hook: IRIS_TILES_PER_WAVE=1|4 pins the variant (tests run all three on small ranges:
    // unset = the K-split form there)
    if (h.tiles_per_wave) {
        t.tiles_per_wave = h.tiles_per_wave == 1 ? 1 : kMfmaTiles;
        t.ksplit = 1;
    }
    if (t.ksplit > 1) {
        t.tiles_per_wave = kSplitT;
        t.grid = (t.ntiles + kSplitT - 1) / kSplitT;  // kSplitT tiles per workgroup
        return t;
    }
    const uint64_t waves = (t.ntiles + t.tiles_per_wave - 1) / t.tiles_per_wave;
    t.grid = (waves + kWaveSlots - 1) / kWaveSlots;
    return t;
}

// the search's form of tile_range: one workgroup per 16 tiles (a persistent grid measured
// slower)
static TileRange search_range(const Hooks &h, LaunchRange r) {
    TileRange t = tile_range(h, r);
    t.fusable = t.grid <= (uint64_t)kFusedReduceMax;
    return t;
}

// partial records a search writes
uint32_t mfma_search_partials(const Hooks &h, LaunchRange r) { return (uint32_t)search_range(h, r).grid; }

uint32_t multi_search_partials(LaunchRange r, int nq) {
    const uint64_t tile0 = r.first / kTileRecs, tile1 = (r.first + r.n + kTileRecs - 1) / kTileRecs;
    const uint64_t waves = (tile1 - tile0 + (4 / nq) - 1) / (4 / nq);
    return (uint32_t)((waves + kWaveSlots - 1) / kWaveSlots);
}

int launch_template_multi_search(void *stream, const void *db, const void *const *qfrags, int nq, LaunchRange r,
                                 Partial *partials, uint32_t *n_partials) {
    *n_partials = multi_search_partials(r, nq);
    if (r.n == 0) return 0;
    if (nq != 2) return -1;
    const uint64_t tile0 = r.first / kTileRecs, tile1 = (r.first + r.n + kTileRecs - 1) / kTileRecs;
    QueryFrags qf{};
    for (int i = 0; i < nq; ++i) qf.q[i] = (const uint4 *)qfrags[i];
    hipLaunchKernelGGL(template_multi_kernel<2>, dim3(*n_partials), dim3(256), 0, (hipStream_t)stream,
                       (const uint4 *)db, qf, tile0, tile1 - tile0, r.first, r.first + r.n, partials);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

int launch_template_mfma_counts(const Hooks &h, void *stream, const void *db, const void *qfrag, LaunchRange r, uint16_t *num_out,
                                uint16_t *den_out) {
    if (r.n == 0) return 0;
    const TileRange t = tile_range(h, r);
    auto kern = t.ksplit > 1 ? template_mfma_kernel<MF_COUNTS, kSplitT, 4>
                : t.tiles_per_wave == 1 ? template_mfma_kernel<MF_COUNTS, 1> : template_mfma_kernel<MF_COUNTS>;
    hipLaunchKernelGGL(kern, dim3((uint32_t)t.grid), dim3(256), 0, (hipStream_t)stream,
                       (const uint4 *)db, (const uint4 *)qfrag, t.tile0, t.ntiles, r.first, r.first + r.n, num_out,
                       den_out, (double *)nullptr, (Partial *)nullptr, FusedFinish{});
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

int launch_template_mfma_search(const Hooks &h, void *stream, const void *db, const void *qfrag, LaunchRange r, double *dist_out,
                                Partial *partials, uint32_t *n_partials, const FusedFinish *fin) {
    const TileRange t = search_range(h, r);
    *n_partials = (uint32_t)t.grid;
    if (r.n == 0) return 0;
    const bool fused = fin && t.fusable;
    if (fin && !fused) return -1;  // the caller asks fused_search_ok() first
    auto kern = fused ? (t.ksplit > 1 ? template_mfma_kernel<MF_SEARCH, kSplitT, 4, true>
                         : t.tiles_per_wave == 1 ? template_mfma_kernel<MF_SEARCH, 1, 1, true>
                                                 : template_mfma_kernel<MF_SEARCH, kMfmaTiles, 1, true>)
                      : (t.ksplit > 1 ? template_mfma_kernel<MF_SEARCH, kSplitT, 4>
                         : t.tiles_per_wave == 1 ? template_mfma_kernel<MF_SEARCH, 1> : template_mfma_kernel<MF_SEARCH>);
    hipLaunchKernelGGL(kern, dim3((uint32_t)t.grid), dim3(64 * kWaveSlots), 0, (hipStream_t)stream,
                       (const uint4 *)db, (const uint4 *)qfrag, t.tile0, t.ntiles, r.first, r.first + r.n,
                       (uint16_t *)nullptr, (uint16_t *)nullptr, dist_out, partials, fin ? *fin : FusedFinish{});
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

// test hook: IRIS_FUSED_REDUCE=0 runs small searches with the separate reduce kernel
bool fused_search_ok(const Hooks &h, LaunchRange r) {
    if (!h.fused_reduce) return false;
    if (r.n == 0) return false;
    return search_range(h, r).fusable;
}

}  // namespace iris
