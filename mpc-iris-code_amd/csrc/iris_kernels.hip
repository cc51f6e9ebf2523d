// iris_kernels.hip — gfx950 (CDNA4) kernels of the masked-Hamming engine.
//
// Hot kernels:
//   template_kernel  Template masked Hamming, 1 query x 31 rotations x N
//                    (src/template.rs:49-64 per pair, min over rotations
//                    src/template.rs:43-47, argmin src/main.rs:616-621)
//   masks_kernel     MasksEngine::batch_process (src/lib.rs:69-79)
//   shares_kernel    DistanceEngine::batch_process (src/lib.rs:42-52)
// Plumbing kernels: pack / unpack (reference layout <-> device layout),
// generate (synthetic DB on the device), reduce (argmin of partials).
//
// Execution model: one wavefront owns one block of 64 records, one record per
// lane.  The 31 rotated query words of the current word position are
// wave-uniform and are held in SGPRs (s_load from a 100-800 KB table that
// stays L2/scalar-cache resident), so the inner step per (word, rotation) is
//   template: v_and + v_bitop3 + 2 x v_bcnt   (4 VALU, SGPR operands)
//   masks:    v_and + v_bcnt                  (2 VALU)
//   shares:   v_pk_mad_u16                    (1 VALU for 2 elements)
// with no LDS traffic and no cross-lane reduction.  The 31-rotation step is
// written as ONE inline-asm statement so hipcc can neither re-associate the
// popcount sums nor hoist the 62 temporaries (it spills otherwise).
#include <hip/hip_runtime.h>

#include "iris_internal.hpp"

namespace iris {

#define IRIS_REP31(X)                                                                                    \
    X(0) X(1) X(2) X(3) X(4) X(5) X(6) X(7) X(8) X(9) X(10) X(11) X(12) X(13) X(14) X(15) X(16) X(17) \
        X(18) X(19) X(20) X(21) X(22) X(23) X(24) X(25) X(26) X(27) X(28) X(29) X(30)

// ------------------------------------------------------------------ steps

// One word position, 31 rotations, Template path:
//   m = qm_r & em ; x = (qp_r ^ ep) & m ; den_r += popc(m) ; num_r += popc(x)
// bitop3 truth table 0x28 = (src0 ^ src1) & src2 with src0 = qp, src1 = ep, src2 = m.
#define T_TXT(r)                                               \
    "v_and_b32 %[m], %[qm" #r "], %[em]\n\t"                   \
    "v_bitop3_b32 %[x], %[qp" #r "], %[ep], %[m] bitop3:0x28\n\t" \
    "v_bcnt_u32_b32 %[d" #r "], %[m], %[d" #r "]\n\t"          \
    "v_bcnt_u32_b32 %[n" #r "], %[x], %[n" #r "]\n\t"
#define T_OD(r) [d##r] "+v"(den[r]),
#define T_ON(r) [n##r] "+v"(num[r]),
#define T_IM(r) [qm##r] "s"(qg[2 * r]),
#define T_IP(r) [qp##r] "s"(qg[2 * r + 1]),

__device__ __forceinline__ void template_step(uint32_t em, uint32_t ep, const uint32_t *__restrict__ qg,
                                              uint32_t (&den)[kRot], uint32_t (&num)[kRot]) {
    uint32_t m, x;
    asm volatile(IRIS_REP31(T_TXT)
                 : IRIS_REP31(T_OD) IRIS_REP31(T_ON)[m] "=&v"(m), [x] "=&v"(x)
                 : IRIS_REP31(T_IM) IRIS_REP31(T_IP)[em] "v"(em), [ep] "v"(ep));
}

__device__ __forceinline__ void template_group(const uint4 &em, const uint4 &ep, const uint32_t *__restrict__ qg,
                                               uint32_t (&den)[kRot], uint32_t (&num)[kRot]) {
    template_step(em.x, ep.x, qg, den, num);
    template_step(em.y, ep.y, qg + 1 * kTemplateTabStride, den, num);
    template_step(em.z, ep.z, qg + 2 * kTemplateTabStride, den, num);
    template_step(em.w, ep.w, qg + 3 * kTemplateTabStride, den, num);
}

// Masks path: m = q_r & e ; den_r += popc(m)
#define M_TXT(r)                                   \
    "v_and_b32 %[m], %[q" #r "], %[e]\n\t"         \
    "v_bcnt_u32_b32 %[d" #r "], %[m], %[d" #r "]\n\t"
#define M_OD(r) [d##r] "+v"(den[r]),
#define M_IQ(r) [q##r] "s"(qg[r]),

__device__ __forceinline__ void masks_step(uint32_t e, const uint32_t *__restrict__ qg, uint32_t (&den)[kRot]) {
    uint32_t m;
    asm volatile(IRIS_REP31(M_TXT) : IRIS_REP31(M_OD)[m] "=&v"(m) : IRIS_REP31(M_IQ)[e] "v"(e));
}

// Shares path: acc_r.{lo,hi} += e.{lo,hi} * q_r.{lo,hi}  (wrapping u16 lanes)
#define S_TXT(r) "v_pk_mad_u16 %[a" #r "], %[e], %[q" #r "], %[a" #r "]\n\t"
#define S_OA(r) [a##r] "+v"(acc[r]),
#define S_IQ(r) [q##r] "s"(qg[r]),
__device__ __forceinline__ void shares_step(uint32_t e, const uint32_t *__restrict__ qg, uint32_t (&acc)[kRot]) {
    uint32_t unused;
    asm volatile(IRIS_REP31(S_TXT) : IRIS_REP31(S_OA)[unused] "=v"(unused) : IRIS_REP31(S_IQ)[e] "v"(e));
}

// ------------------------------------------------------------------ search helpers

__device__ __forceinline__ bool better(const Partial &a, const Partial &b) {
    if (a.den == 0) return false;
    if (b.den == 0) return true;
    const uint32_t l = a.num * b.den, r = b.num * a.den;  // <= 12800^2 < 2^32
    if (l != r) return l < r;
    return a.idx < b.idx;
}

__device__ __forceinline__ Partial shfl_xor_partial(const Partial &c, int off) {
    Partial o;
    o.num = __shfl_xor(c.num, off);
    o.den = __shfl_xor(c.den, off);
    o.rot = __shfl_xor(c.rot, off);
    o.pad = 0;
    const uint32_t lo = __shfl_xor((uint32_t)c.idx, off);
    const uint32_t hi = __shfl_xor((uint32_t)(c.idx >> 32), off);
    o.idx = ((uint64_t)hi << 32) | lo;
    return o;
}

__device__ __forceinline__ Partial wave_best(Partial c) {
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) {
        const Partial o = shfl_xor_partial(c, off);
        if (better(o, c)) c = o;
    }
    return c;
}

// ------------------------------------------------------------------ template kernel

enum { MODE_COUNTS = 0, MODE_SEARCH = 1 };

// Each wave: one 64-record block.  Workgroup: 4 waves.
template <int MODE>
__global__ void __launch_bounds__(256, 5)
    template_kernel(const uint4 *__restrict__ db, const uint32_t *__restrict__ qtab, uint64_t blk0, uint64_t nblk,
                    uint64_t first, uint64_t end, uint16_t *__restrict__ num_out, uint16_t *__restrict__ den_out,
                    double *__restrict__ dist_out, Partial *__restrict__ partials) {
    const int lane = threadIdx.x & 63;
    const int wslot = threadIdx.x >> 6;
    const uint64_t wave = (uint64_t)blockIdx.x * kWaveSlots + wslot;
    const bool active = wave < nblk;  // wave-uniform
    const uint64_t blk = blk0 + (active ? wave : 0);

    uint32_t den[kRot], num[kRot];
#pragma unroll
    for (int r = 0; r < kRot; ++r) {
        den[r] = 0;
        num[r] = 0;
    }

    if (active) {
        const uint4 *base = db + blk * (uint64_t)(2 * kPlaneGroups * kLanes) + lane;
        uint4 emA = base[0], epA = base[kLanes];
#pragma unroll 1
        for (int g = 0; g < kPlaneGroups; g += 2) {
            const uint4 emB = base[(2 * g + 2) * kLanes], epB = base[(2 * g + 3) * kLanes];
            template_group(emA, epA, qtab + g * 4 * kTemplateTabStride, den, num);
            const int gn = (g + 2 < kPlaneGroups) ? g + 2 : g;
            emA = base[(2 * gn) * kLanes];
            epA = base[(2 * gn + 1) * kLanes];
            template_group(emB, epB, qtab + (g + 1) * 4 * kTemplateTabStride, den, num);
        }
    }

    const uint64_t t = blk * kLanes + lane;
    const bool valid = active && t >= first && t < end;
    const uint64_t o = t - first;

    if (MODE == MODE_COUNTS) {
        if (valid) {
            if (num_out) {
#pragma unroll
                for (int r = 0; r < kRot; ++r) num_out[o * kRot + r] = (uint16_t)num[r];
            }
            if (den_out) {
#pragma unroll
                for (int r = 0; r < kRot; ++r) den_out[o * kRot + r] = (uint16_t)den[r];
            }
        }
        return;
    } else {
        // min over rotations with exact integer cross-multiplication; the
        // first (lowest r) rotation wins ties — f64 quotients of distinct
        // fractions n/d with n,d <= 12800 are distinct, so this equals the
        // reference's fold(INF, f64::min) over (n as f64)/(d as f64).
        Partial c;
        c.num = 0;
        c.den = 0;
        c.rot = 0;
        c.pad = 0;
        c.idx = o;
#pragma unroll
        for (int r = 0; r < kRot; ++r) {
            const uint32_t d = den[r], n = num[r];
            if (d != 0 && (c.den == 0 || n * c.den < c.num * d)) {
                c.num = n;
                c.den = d;
                c.rot = r;
            }
        }
        if (!valid) c.den = 0;
        if (valid && dist_out) dist_out[o] = c.den ? (double)c.num / (double)c.den : __builtin_inf();

        c = wave_best(c);
        __shared__ Partial sh[kWaveSlots];
        if (lane == 0) sh[wslot] = c;
        __syncthreads();
        if (threadIdx.x == 0) {
            Partial b = sh[0];
#pragma unroll
            for (int w = 1; w < kWaveSlots; ++w)
                if (better(sh[w], b)) b = sh[w];
            partials[blockIdx.x] = b;
        }
    }
}

// ------------------------------------------------------------------ masks kernel

__global__ void __launch_bounds__(256, 8)
    masks_kernel(const uint4 *__restrict__ db, const uint32_t *__restrict__ qtab, uint64_t blk0, uint64_t nblk,
                 uint64_t first, uint64_t end, uint16_t *__restrict__ out) {
    const int lane = threadIdx.x & 63;
    const uint64_t wave = (uint64_t)blockIdx.x * kWaveSlots + (threadIdx.x >> 6);
    if (wave >= nblk) return;
    const uint64_t blk = blk0 + wave;
    uint32_t den[kRot];
#pragma unroll
    for (int r = 0; r < kRot; ++r) den[r] = 0;

    const uint4 *base = db + blk * (uint64_t)(kPlaneGroups * kLanes) + lane;
    uint4 eA = base[0];
#pragma unroll 1
    for (int g = 0; g < kPlaneGroups; g += 2) {
        const uint4 eB = base[(g + 1) * kLanes];
        const uint32_t *qg = qtab + g * 4 * kSlotTabStride;
        masks_step(eA.x, qg, den);
        masks_step(eA.y, qg + 1 * kSlotTabStride, den);
        masks_step(eA.z, qg + 2 * kSlotTabStride, den);
        masks_step(eA.w, qg + 3 * kSlotTabStride, den);
        const int gn = (g + 2 < kPlaneGroups) ? g + 2 : g;
        eA = base[gn * kLanes];
        qg += 4 * kSlotTabStride;
        masks_step(eB.x, qg, den);
        masks_step(eB.y, qg + 1 * kSlotTabStride, den);
        masks_step(eB.z, qg + 2 * kSlotTabStride, den);
        masks_step(eB.w, qg + 3 * kSlotTabStride, den);
    }
    const uint64_t t = blk * kLanes + lane;
    if (t >= first && t < end) {
        const uint64_t o = t - first;
#pragma unroll
        for (int r = 0; r < kRot; ++r) out[o * kRot + r] = (uint16_t)den[r];
    }
}

// ------------------------------------------------------------------ shares kernel

__global__ void __launch_bounds__(256, 8)
    shares_kernel(const uint4 *__restrict__ db, const uint32_t *__restrict__ qtab, uint64_t blk0, uint64_t nblk,
                  uint64_t first, uint64_t end, uint16_t *__restrict__ out) {
    const int lane = threadIdx.x & 63;
    const uint64_t wave = (uint64_t)blockIdx.x * kWaveSlots + (threadIdx.x >> 6);
    if (wave >= nblk) return;
    const uint64_t blk = blk0 + wave;
    uint32_t acc[kRot];
#pragma unroll
    for (int r = 0; r < kRot; ++r) acc[r] = 0;

    const uint4 *base = db + blk * (uint64_t)(kShareGroups * kLanes) + lane;
    uint4 eA = base[0];
#pragma unroll 1
    for (int g = 0; g < kShareGroups; g += 2) {
        const uint4 eB = base[(g + 1) * kLanes];
        const uint32_t *qg = qtab + g * 4 * kSlotTabStride;
        shares_step(eA.x, qg, acc);
        shares_step(eA.y, qg + 1 * kSlotTabStride, acc);
        shares_step(eA.z, qg + 2 * kSlotTabStride, acc);
        shares_step(eA.w, qg + 3 * kSlotTabStride, acc);
        const int gn = (g + 2 < kShareGroups) ? g + 2 : g;
        eA = base[gn * kLanes];
        qg += 4 * kSlotTabStride;
        shares_step(eB.x, qg, acc);
        shares_step(eB.y, qg + 1 * kSlotTabStride, acc);
        shares_step(eB.z, qg + 2 * kSlotTabStride, acc);
        shares_step(eB.w, qg + 3 * kSlotTabStride, acc);
    }
    const uint64_t t = blk * kLanes + lane;
    if (t >= first && t < end) {
        const uint64_t o = t - first;
#pragma unroll
        for (int r = 0; r < kRot; ++r) out[o * kRot + r] = (uint16_t)((acc[r] & 0xFFFFu) + (acc[r] >> 16));
    }
}

// ------------------------------------------------------------------ reduce

// One workgroup folds partials[i * stride] for i < n into *out.  A single
// workgroup reads ~10 B/clk, so tens of thousands of partials (one per search
// workgroup) first go through reduce_stage_kernel below.
__global__ void __launch_bounds__(1024) reduce_kernel(const Partial *__restrict__ partials, uint32_t n,
                                                      Partial *__restrict__ out, uint32_t stride, uint64_t idx_base) {
    Partial c;
    c.num = 0;
    c.den = 0;
    c.rot = 0;
    c.pad = 0;
    c.idx = ~0ull;
    for (uint32_t i = threadIdx.x; i < n; i += blockDim.x) {
        const Partial p = partials[(uint64_t)i * stride];
        if (better(p, c)) c = p;
    }
    c = wave_best(c);
    __shared__ Partial sh[16];
    const int wslot = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 0) sh[wslot] = c;
    __syncthreads();
    if (threadIdx.x == 0) {
        Partial b = sh[0];
        const int nw = (blockDim.x + 63) / 64;
        for (int w = 1; w < nw; ++w)
            if (better(sh[w], b)) b = sh[w];
        if (b.den != 0) b.idx += idx_base;  // range-relative -> caller's index space
        *out = b;
    }
}

// Cross-shard merge of a group search (iris_group.hip): recv holds, for each of the S
// shards (all ranks, all-gathered), nq winners with global indices at recv[s * stride + q];
// thread q folds query q's S candidates (exact fraction, then lowest global index, the
// resolver's strict-< scan, src/main.rs:616-621) into out[q].
__global__ void __launch_bounds__(256) group_merge_kernel(const Partial *__restrict__ recv, uint32_t S, uint32_t nq,
                                                          uint32_t stride, Partial *__restrict__ out) {
    const uint32_t q = blockIdx.x * blockDim.x + threadIdx.x;
    if (q >= nq) return;
    Partial c;
    c.num = 0;
    c.den = 0;
    c.rot = 0;
    c.pad = 0;
    c.idx = ~0ull;
    for (uint32_t s = 0; s < S; ++s) {
        const Partial p = recv[(uint64_t)s * stride + q];
        if (better(p, c)) c = p;
    }
    out[q] = c;
}

constexpr uint32_t kReduceChunk = 1024;  // partials per first-stage workgroup

// First stage: workgroup b folds partials[b * kReduceChunk, +kReduceChunk) and
// writes its winner in place at partials[b * kReduceChunk] (a slot only it reads).
__global__ void __launch_bounds__(256) reduce_stage_kernel(Partial *__restrict__ partials, uint32_t n) {
    const uint64_t base = (uint64_t)blockIdx.x * kReduceChunk;
    const uint32_t m = (uint32_t)min<uint64_t>(kReduceChunk, n - base);
    Partial c;
    c.num = 0;
    c.den = 0;
    c.rot = 0;
    c.pad = 0;
    c.idx = ~0ull;
    for (uint32_t i = threadIdx.x; i < m; i += blockDim.x) {
        const Partial p = partials[base + i];
        if (better(p, c)) c = p;
    }
    c = wave_best(c);
    __shared__ Partial sh[4];
    if ((threadIdx.x & 63) == 0) sh[threadIdx.x >> 6] = c;
    __syncthreads();  // every read of the chunk is done before its first slot is overwritten
    if (threadIdx.x == 0) {
        Partial b = sh[0];
        for (int w = 1; w < 4; ++w)
            if (better(sh[w], b)) b = sh[w];
        partials[base] = b;
    }
}

// ------------------------------------------------------------------ pack / unpack / generate

struct PackParams {
    int groups, planes, rec_dwords;
    int plane_src0, plane_src1;
};

// staging: n reference-layout records; db: device layout.  Thread per (record, group).
__global__ void __launch_bounds__(256) pack_kernel(const uint4 *__restrict__ staging, uint4 *__restrict__ db,
                                                   uint64_t t_first, uint64_t n, PackParams p) {
    const uint64_t total = n * (uint64_t)p.groups;
    for (uint64_t tid = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; tid < total;
         tid += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t i = tid % n, G = tid / n;
        const int pl = (int)(G % p.planes);
        const uint64_t g = G / p.planes;
        const uint64_t src = (i * p.rec_dwords + (pl ? p.plane_src1 : p.plane_src0) + g * 4) / 4;
        const uint64_t t = t_first + i;
        const uint64_t dst = (t / kLanes) * (uint64_t)p.groups * kLanes + G * kLanes + (t % kLanes);
        db[dst] = staging[src];
    }
}

__global__ void __launch_bounds__(256) unpack_kernel(const uint4 *__restrict__ db, uint4 *__restrict__ staging,
                                                     uint64_t t_first, uint64_t n, PackParams p) {
    const uint64_t total = n * (uint64_t)p.groups;
    for (uint64_t tid = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; tid < total;
         tid += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t i = tid % n, G = tid / n;
        const int pl = (int)(G % p.planes);
        const uint64_t g = G / p.planes;
        const uint64_t dst = (i * p.rec_dwords + (pl ? p.plane_src1 : p.plane_src0) + g * 4) / 4;
        const uint64_t t = t_first + i;
        const uint64_t src = (t / kLanes) * (uint64_t)p.groups * kLanes + G * kLanes + (t % kLanes);
        staging[dst] = db[src];
    }
}

// Synthetic records written straight into the device layout.
__global__ void __launch_bounds__(256) generate_kernel(uint4 *__restrict__ db, uint64_t t_first, uint64_t n, int kind,
                                                       int groups, uint64_t key, uint64_t global_index0) {
    const uint64_t total = n * (uint64_t)groups;
    for (uint64_t tid = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; tid < total;
         tid += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t i = tid % n, G = tid / n;
        const uint64_t t = t_first + i;            // position in the DB
        const uint64_t gt = global_index0 + i;     // generator index
        uint64_t c0;
        if (kind == IRIS_KIND_TEMPLATES) {
            const uint64_t g = G >> 1, pl = G & 1;  // pl 0 = mask (ctr +200), 1 = pattern
            c0 = gt * 400 + (pl ? 0 : 200) + 2 * g;
        } else if (kind == IRIS_KIND_MASKS) {
            c0 = gt * 400 + 200 + 2 * G;
        } else {
            c0 = gt * 3200 + 2 * G;
        }
        const uint64_t lo = gen_limb(key, c0), hi = gen_limb(key, c0 + 1);
        uint4 v;
        v.x = (uint32_t)lo;
        v.y = (uint32_t)(lo >> 32);
        v.z = (uint32_t)hi;
        v.w = (uint32_t)(hi >> 32);
        const uint64_t dst = (t / kLanes) * (uint64_t)groups * kLanes + G * kLanes + (t % kLanes);
        db[dst] = v;
    }
}

// ------------------------------------------------------------------ launchers

static int grid_stride_blocks(uint64_t total) {
    uint64_t b = (total + 255) / 256;
    const uint64_t cap = 256ull * 64;  // 64 workgroups per CU
    if (b > cap) b = cap;
    if (b == 0) b = 1;
    return (int)b;
}

static PackParams pack_params(const KindInfo &k) {
    return PackParams{k.groups, k.planes, k.rec_dwords, k.plane_src[0], k.plane_src[1]};
}

static int check_launch() { return hipGetLastError() == hipSuccess ? 0 : -1; }

int launch_pack(void *stream, const KindInfo &k, const void *staging, void *db, uint64_t t_first, uint64_t n) {
    if (n == 0) return 0;
    if (k.layout == IRIS_LAYOUT_TILES) return launch_pack_tiles_kind(stream, k.kind, staging, db, t_first, n);
    hipLaunchKernelGGL(pack_kernel, dim3(grid_stride_blocks(n * k.groups)), dim3(256), 0, (hipStream_t)stream,
                       (const uint4 *)staging, (uint4 *)db, t_first, n, pack_params(k));
    return check_launch();
}

int launch_unpack(void *stream, const KindInfo &k, const void *db, void *staging, uint64_t t_first, uint64_t n) {
    if (n == 0) return 0;
    if (k.layout == IRIS_LAYOUT_TILES) return launch_unpack_tiles_kind(stream, k.kind, db, staging, t_first, n);
    hipLaunchKernelGGL(unpack_kernel, dim3(grid_stride_blocks(n * k.groups)), dim3(256), 0, (hipStream_t)stream,
                       (const uint4 *)db, (uint4 *)staging, t_first, n, pack_params(k));
    return check_launch();
}

int launch_generate(void *stream, const KindInfo &k, void *db, uint64_t t_first, uint64_t n, uint64_t seed,
                    uint64_t global_index0) {
    if (n == 0) return 0;
    if (k.layout == IRIS_LAYOUT_TILES)
        return launch_generate_tiles_kind(stream, k.kind, db, t_first, n, seed, global_index0);
    const uint64_t key = gen_key(seed, k.kind == IRIS_KIND_SHARES ? 1 : 0);
    hipLaunchKernelGGL(generate_kernel, dim3(grid_stride_blocks(n * k.groups)), dim3(256), 0, (hipStream_t)stream,
                       (uint4 *)db, t_first, n, k.kind, k.groups, key, global_index0);
    return check_launch();
}

struct BlockRange {
    uint64_t blk0, nblk, grid;
};

static BlockRange block_range(LaunchRange r) {
    BlockRange b;
    b.blk0 = r.first / kLanes;
    const uint64_t blk1 = (r.first + r.n + kLanes - 1) / kLanes;
    b.nblk = blk1 - b.blk0;
    b.grid = (b.nblk + kWaveSlots - 1) / kWaveSlots;
    return b;
}

uint32_t search_partials(LaunchRange r) { return (uint32_t)block_range(r).grid; }

int launch_template_counts(void *stream, const void *db, const void *qtab, LaunchRange r, uint16_t *num_out,
                           uint16_t *den_out) {
    if (r.n == 0) return 0;
    const BlockRange b = block_range(r);
    hipLaunchKernelGGL(template_kernel<MODE_COUNTS>, dim3((uint32_t)b.grid), dim3(256), 0, (hipStream_t)stream,
                       (const uint4 *)db, (const uint32_t *)qtab, b.blk0, b.nblk, r.first, r.first + r.n, num_out,
                       den_out, (double *)nullptr, (Partial *)nullptr);
    return check_launch();
}

int launch_template_search(void *stream, const void *db, const void *qtab, LaunchRange r, double *dist_out,
                           Partial *partials, uint32_t *n_partials) {
    const BlockRange b = block_range(r);
    *n_partials = (uint32_t)b.grid;
    if (r.n == 0) return 0;
    hipLaunchKernelGGL(template_kernel<MODE_SEARCH>, dim3((uint32_t)b.grid), dim3(256), 0, (hipStream_t)stream,
                       (const uint4 *)db, (const uint32_t *)qtab, b.blk0, b.nblk, r.first, r.first + r.n,
                       (uint16_t *)nullptr, (uint16_t *)nullptr, dist_out, partials);
    return check_launch();
}

// Consumes the partials (a large set is folded in place by a first stage).
int launch_reduce(void *stream, Partial *partials, uint32_t n_partials, Partial *out, uint64_t idx_base) {
    if (n_partials <= 4 * kReduceChunk) {
        hipLaunchKernelGGL(reduce_kernel, dim3(1), dim3(1024), 0, (hipStream_t)stream, partials, n_partials, out, 1u,
                           idx_base);
        return check_launch();
    }
    const uint32_t g = (n_partials + kReduceChunk - 1) / kReduceChunk;
    hipLaunchKernelGGL(reduce_stage_kernel, dim3(g), dim3(256), 0, (hipStream_t)stream, partials, n_partials);
    if (check_launch() != 0) return -1;
    hipLaunchKernelGGL(reduce_kernel, dim3(1), dim3(1024), 0, (hipStream_t)stream, (const Partial *)partials, g, out,
                       kReduceChunk, idx_base);
    return check_launch();
}

int launch_group_merge(void *stream, const Partial *recv, uint32_t shards, uint32_t nq, uint32_t stride, Partial *out) {
    if (nq == 0) return 0;
    hipLaunchKernelGGL(group_merge_kernel, dim3((nq + 255) / 256), dim3(256), 0, (hipStream_t)stream, recv, shards, nq,
                       stride, out);
    return check_launch();
}

int launch_masks(void *stream, const void *db, const void *qtab, LaunchRange r, uint16_t *out) {
    if (r.n == 0) return 0;
    const BlockRange b = block_range(r);
    hipLaunchKernelGGL(masks_kernel, dim3((uint32_t)b.grid), dim3(256), 0, (hipStream_t)stream, (const uint4 *)db,
                       (const uint32_t *)qtab, b.blk0, b.nblk, r.first, r.first + r.n, out);
    return check_launch();
}

int launch_shares(void *stream, const void *db, const void *qtab, LaunchRange r, uint16_t *out) {
    if (r.n == 0) return 0;
    const BlockRange b = block_range(r);
    hipLaunchKernelGGL(shares_kernel, dim3((uint32_t)b.grid), dim3(256), 0, (hipStream_t)stream, (const uint4 *)db,
                       (const uint32_t *)qtab, b.blk0, b.nblk, r.first, r.first + r.n, out);
    return check_launch();
}

}  // namespace iris
