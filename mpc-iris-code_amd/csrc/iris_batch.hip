// iris_batch.hip — many queries x 31 rotations x N templates (BASELINE configs[2]).
//
// The fp4 formulation of iris_mfma.hip turns a query batch into a GEMM with
// M = 32 rows per query (31 rotations + a zero row), N = templates, K = 12800
// bits, two products (den, encode) per K.  Neither operand fits on chip for
// 1024 queries x 10M templates, so it is tiled like a GEMM (batch_lds_kernel
// below).  A (queries) is stored like a template tile: the 31 rotated copies of
// a query packed with xpack (iris_internal.hpp) as records 0..30 of a TILES
// tile, so one expansion routine turns either side into fp4 operands.
// Workgroups sharing a query group walk the template N-groups with a stride,
// and all query groups walk the same N-groups at once, so a template tile is
// fetched from HBM about once per XCD and re-read from L2 by the other query
// groups.  Per query the kernel keeps a running best (exact fraction, lowest
// index), one partial per (query, workgroup), reduced by batch_reduce_kernel.
#include <hip/hip_runtime.h>
#include <stdlib.h>

#include "iris_device.hpp"

namespace iris {

typedef int v8i __attribute__((ext_vector_type(8)));
typedef float v16f __attribute__((ext_vector_type(16)));

constexpr int kBatchBQ = 4;                       // query padding unit of a batched engine
constexpr int kTileU4 = kPlaneGroups * 64;        // 6400 uint4 per tile

__device__ __forceinline__ v16f mfma4(const v8i &a, const v8i &b, const v16f &c) {
    return __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(a, b, c, 4, 4, 0, 127, 0, 127);
}

// one workgroup per query: reduce its G partials
__global__ void __launch_bounds__(256) batch_reduce_kernel(const Partial *__restrict__ partials, uint32_t G,
                                                           Partial *__restrict__ out, uint64_t idx_base) {
    const uint32_t q = blockIdx.x;
    Partial c;
    c.num = 0;
    c.den = 0;
    c.rot = 0;
    c.pad = 0;
    c.idx = ~0ull;
    for (uint32_t i = threadIdx.x; i < G; i += blockDim.x) {
        const Partial p = partials[(uint64_t)q * G + i];
        if (partial_better_dev(p, c)) c = p;
    }
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) {
        const Partial o = partial_shfl_xor(c, off);
        if (partial_better_dev(o, c)) c = o;
    }
    __shared__ Partial sh[4];
    if ((threadIdx.x & 63) == 0) sh[threadIdx.x >> 6] = c;
    __syncthreads();
    if (threadIdx.x == 0) {
        Partial b = sh[0];
        for (int i = 1; i < 4; ++i)
            if (partial_better_dev(sh[i], b)) b = sh[i];
        if (b.den != 0) b.idx += idx_base;
        out[q] = b;
    }
}

// ---------------------------------------------------------------------------- batch_lds_kernel
//
//   workgroup (8 waves) = BQL queries (shared by all 8 waves) x N-groups of template tiles
//   K-step              = GPL chunk pairs
//
// - A (the query group's rotation tiles) is loaded once per workgroup and K-step (plain
//   global loads a step ahead), expanded ONCE into the MFMA-ready fp4 den / encode fragments
//   and written to a 2-stage LDS ring; every wave reads its queries' fragments from it
//   (ds_read_b128, lane-linear 1-KB rows: conflict-free).
// - B (templates): each wave owns WT tiles per N-group and loads them straight into
//   registers (global_load_dwordx4, 1 KB per wave and chunk pair, one K-step ahead) and
//   expands them itself (10 VALU per 64-bit chunk).  (An LDS-DMA staged form of round 1 paid
//   ~60 issue cycles per 1-KB piece beside the MFMAs; removed in round 5, DESIGN.md appendix.)
// - One s_barrier per K-step.
// The grid holds one workgroup per CU; all query groups walk the same N-groups, so a
// template tile comes from HBM about once per XCD and from L2 after that.
//
// Waves: QW = BQL / WQL query sets x NW / QW tile sets; a wave holds WQL queries x WT tiles.
// Shipped: NW = 8, BQL = 2, WQL = 2, WT = 2 (16 tiles per N-group: each query tile read from
// beyond L2 is applied to 16 tiles; 128 accumulators).  Cross-checked alternative (the
// IRIS_BATCH_KERNEL=2 test hook): BQL = 4, WQL = 4, WT = 1 (8 tiles per N-group, the round-2
// shape), whose SIMD partners run their N-groups half a group apart (kStagger).
template <int NW, int WT, int WQL, int BQL, int GPL = 4>
__global__ void __launch_bounds__(64 * NW, 1)
    batch_lds_kernel(const uint4 *__restrict__ db, const uint4 *__restrict__ qtiles, uint64_t tile0, uint64_t ntiles,
                     uint64_t first, uint64_t end, uint32_t nqg, uint32_t G, Partial *__restrict__ partials) {
    constexpr int kGP = GPL;                        // chunk pairs per K-step
    constexpr int kSteps = kPlaneGroups / kGP;
    static_assert(kPlaneGroups % kGP == 0, "K-step must tile the 100 chunk pairs");
    constexpr int kBQ = BQL;
    constexpr int kArows = kBQ * kGP;               // compact A rows (1 KB) per K-step
    constexpr int QW = kBQ / WQL;                   // query sets
    constexpr int kTilesPerGroup = (NW / QW) * WT;  // template tiles per N-group
    static_assert(kBQ % WQL == 0 && NW % QW == 0 && kBatchBQ % kBQ == 0, "geometry");
    constexpr int kAper = (kArows + NW - 1) / NW;  // compact A rows per wave and K-step (the last may be idle)
    // [stage][chunk pair][query][den h0, enc h0, den h1, enc h1][lane]: 2 x kGP x 16 KB
    __shared__ uint4 afrag[2][kGP][kBQ][4][64];

    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int qset = w % QW, tset = w / QW;  // this wave's queries qset * WQL + qi, tiles tset * WT + t
    const uint32_t qg = blockIdx.x % nqg, gi = blockIdx.x / nqg;
    const uint64_t ngroups = (ntiles + kTilesPerGroup - 1) / kTilesPerGroup;
    const uint32_t my_groups = gi < ngroups ? (uint32_t)((ngroups - gi + G - 1) / G) : 0;
    const uint32_t total = my_groups * kSteps;
    // Stagger: the two waves sharing a SIMD (w and w + 4) run their N-groups
    // half a group apart, so one wave's epilogue (no MFMAs) overlaps its partner's MFMAs.  The
    // K-step at time s is s mod kSteps for every wave (the A fragments in LDS are shared); waves
    // 4..7 start their first group at s = off and the workgroup walks off extra steps, in which
    // the idle waves' MFMAs run on re-read rows and are discarded.
    // (the 2 x 2 per-wave shape runs 2 % faster without it: profiles/r03_batch_variants.txt)
    constexpr bool kStagger = NW == 8 && WQL == 4;
    const uint32_t off = (kStagger && w >= NW / 2) ? (uint32_t)(kSteps / 2) : 0u;
    const uint32_t walk = total ? total + (kStagger ? (uint32_t)(kSteps / 2) : 0u) : 0u;
    auto group_of = [&](uint32_t s) {  // this wave's N-group at time s (clamped while idle)
        const uint32_t r = s >= off ? (s - off) / kSteps : 0u;
        return r < my_groups ? r : my_groups - 1;
    };

    // this wave's compact A rows of a K-step: r = w + NW i -> query r % kBQ, chunk pair r / kBQ
    const uint4 *abase = qtiles + (uint64_t)(qg * kBQ) * kTileU4 + lane;
    auto load_a = [&](uint32_t s, uint4 (&aq)[kAper]) {
        const uint32_t k = s % kSteps;
#pragma unroll
        for (int i = 0; i < kAper; ++i) {
            const int r = w + NW * i;
            // plain loads: nontemporal ones (to keep the shared template tiles in L2) measured 5 %
            // slower with more bytes from beyond L2 (4.64 vs 2.94 TB, profiles/r03_batch_a_nt.txt)
            if (kArows % NW == 0 || r < kArows) aq[i] = abase[(uint64_t)(r % kBQ) * kTileU4 + (k * kGP + r / kBQ) * 64];
        }
    };
    auto b_row = [&](uint32_t s, int t) {  // tile t of this wave, chunk pair 0 of K-step s
        const uint32_t j = group_of(s), k = s % kSteps;
        const uint64_t trel = (gi + (uint64_t)j * G) * kTilesPerGroup + tset * WT + t;
        return db + (tile0 + (trel < ntiles ? trel : ntiles - 1)) * (uint64_t)kTileU4 + (k * kGP) * 64 + lane;
    };
    // compact A row -> fp4 den / encode fragments of both chunks
    auto store_a = [&](uint32_t s, const uint4 (&aq)[kAper]) {
#pragma unroll
        for (int i = 0; i < kAper; ++i) {
            const int r = w + NW * i, qi = r % kBQ, gp = r / kBQ;
            if (kArows % NW != 0 && r >= kArows) continue;
            uint4(*dst)[64] = afrag[s & 1][gp][qi];
#pragma unroll
            for (int h2 = 0; h2 < 2; ++h2) {
                const uint32_t ax = h2 ? aq[i].z : aq[i].x, ay = h2 ? aq[i].w : aq[i].y;
                dst[2 * h2][lane] = make_uint4(ax & 0x22222222u, (ax & 0x11111111u) << 2, ay & 0x22222222u,
                                               (ay & 0x11111111u) << 2);
                dst[2 * h2 + 1][lane] = make_uint4(ax & 0xAAAAAAAAu, (ax << 1) & 0xAAAAAAAAu, ay & 0xAAAAAAAAu,
                                                   (ay << 1) & 0xAAAAAAAAu);
            }
        }
    };
    auto barrier = [] {
        asm volatile("" ::: "memory");
        __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0): this wave's fragment writes landed; loads stay in flight
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
    };

    // running best per lane and query across the walk: (num | den << 16, N-group x tile << 5 | rotation);
    // den 0 = none yet
    uint32_t run_nd[WQL], run_jr[WQL];
#pragma unroll
    for (int qi = 0; qi < WQL; ++qi) {
        run_nd[qi] = 1;  // (num 1, den 0): none
        run_jr[qi] = 0;
    }
    Partial wave_best;
    v16f den[WQL][WT], sacc[WQL][WT];
    auto zero = [&] {
#pragma unroll
        for (int qi = 0; qi < WQL; ++qi)
#pragma unroll
            for (int t = 0; t < WT; ++t)
#pragma unroll
                for (int i = 0; i < 16; ++i) {
                    den[qi][t][i] = 0.f;
                    sacc[qi][t][i] = 0.f;
                }
    };
    zero();

    // B rolls through bq: chunk pair g of step s + 1 is loaded into bq[t][g] as soon as step s
    // has expanded both of its chunks — one K-step of latency cover
    uint4 bq[WT][kGP];
    if (total) {
        uint4 aq[kAper];
        load_a(0, aq);
#pragma unroll
        for (int t = 0; t < WT; ++t) {
            const uint4 *src = b_row(0, t);
#pragma unroll
            for (int g = 0; g < kGP; ++g) bq[t][g] = src[g * 64];
        }
        store_a(0, aq);
        barrier();
    }
#pragma unroll 1
    for (uint32_t s = 0; s < walk; ++s) {
        // A(s + 1) is loaded first, so waiting for it leaves step s + 1's B loads in flight;
        // branch-free: the last step re-loads its own rows (harmless) instead of skipping
        const uint32_t s1 = s + 1 < walk ? s + 1 : s;
        uint4 aq[kAper];
        load_a(s1, aq);
        const uint4(*st)[kBQ][4][64] = afrag[s & 1];
        // blocks b = 2 gp + h2 (one 64-bit chunk): block b + 1's fragment reads are issued
        // between block b's MFMAs (rolling: their latency hides behind the MFMAs)
        auto frag = [&](int b, int form, int qi) { return st[b >> 1][qset * WQL + qi][2 * (b & 1) + form][lane]; };
        uint4 fa[WQL], fe[WQL];
#pragma unroll
        for (int qi = 0; qi < WQL; ++qi) {
            fa[qi] = frag(0, 0, qi);
            fe[qi] = frag(0, 1, qi);
        }
#pragma unroll
        for (int b = 0; b < 2 * kGP; ++b) {
            const bool nb = b + 1 < 2 * kGP;
            v8i bd[WT], be[WT];
#pragma unroll
            for (int t = 0; t < WT; ++t) {
                const uint4 q = bq[t][b >> 1];
                const uint32_t bx = (b & 1) ? q.z : q.x, by = (b & 1) ? q.w : q.y;
                bd[t] = v8i{(int)(bx & 0x22222222u), (int)(bx & 0x11111111u), (int)(by & 0x22222222u),
                            (int)(by & 0x11111111u), 0, 0, 0, 0};
                be[t] = v8i{(int)(bx & 0xAAAAAAAAu), (int)((bx << 1) & 0xAAAAAAAAu), (int)(by & 0xAAAAAAAAu),
                            (int)((by << 1) & 0xAAAAAAAAu), 0, 0, 0, 0};
            }
            if (b & 1) {  // both chunks of chunk pair b >> 1 expanded: its registers take step s + 1's
#pragma unroll
                for (int t = 0; t < WT; ++t) bq[t][b >> 1] = b_row(s1, t)[(b >> 1) * 64];
            }
            uint4 na[WQL], ne[WQL];
#pragma unroll
            for (int qi = 0; qi < WQL; ++qi) {
                const v8i a_d = {(int)fa[qi].x, (int)fa[qi].y, (int)fa[qi].z, (int)fa[qi].w, 0, 0, 0, 0};
                const v8i a_e = {(int)fe[qi].x, (int)fe[qi].y, (int)fe[qi].z, (int)fe[qi].w, 0, 0, 0, 0};
#pragma unroll
                for (int t = 0; t < WT; ++t) den[qi][t] = mfma4(a_d, bd[t], den[qi][t]);
                if (nb) na[qi] = frag(b + 1, 0, qi);
#pragma unroll
                for (int t = 0; t < WT; ++t) sacc[qi][t] = mfma4(a_e, be[t], sacc[qi][t]);
                if (nb) ne[qi] = frag(b + 1, 1, qi);
            }
            __builtin_amdgcn_sched_barrier(0);
            if (nb) {
#pragma unroll
                for (int qi = 0; qi < WQL; ++qi) {
                    fa[qi] = na[qi];
                    fe[qi] = ne[qi];
                }
            }
        }
        store_a(s + 1, aq);  // the last step fills the idle stage (read by nobody)
        // a group ends at s when s + 1 - off is a multiple of kSteps; the end at s = off - 1 closes
        // a staggered wave's idle steps (nothing to record, only the zeroing)
        if (s + 1 >= off && (s + 1 - off) % kSteps == 0) {  // N-group done: this wave's tiles, every query
            const bool live = s >= off;
            const uint32_t j = live ? (s + 1 - off) / kSteps - 1 : 0u;
            // per lane and query: the best of the lane's 16 rotation rows, folded into the
            // lane's running best (no cross-lane work until the end of the walk)
            const int h = lane >> 5;
#pragma unroll
            for (int t = 0; t < WT; ++t) {
                const uint64_t trel = (gi + (uint64_t)j * G) * kTilesPerGroup + tset * WT + t;
                const uint64_t tg = (tile0 + trel) * 32 + (lane & 31);
                const bool valid = live && trel < ntiles && tg >= first && tg < end;
#pragma unroll
                for (int qi = 0; qi < WQL; ++qi) {
                    // (bn, bd) = (1, 0) is "none": a row with den 0 (no jointly valid bit; also the
                    // zero row k = 31) is (0, 0) and never wins, n * 0 < 1 * d holds for any real
                    // candidate, so the scan needs no validity tests
                    // (the selects stay compare + v_cndmask: bit-field inserts under a sign mask,
                    // forced with inline asm, measured 1.5 % slower, profiles/r03_batch_epilogue_bfi.txt)
                    uint32_t bn = 1, bd = 0, br = 0;
#pragma unroll
                    for (int r = 0; r < 16; ++r) {
                        const int k = (r & 3) + 8 * (r >> 2) + 4 * h;  // ascending in r: ties keep the lower k
                        const uint32_t dd = (uint32_t)den[qi][t][r];
                        const uint32_t nn = (uint32_t)(((int)dd - (int)sacc[qi][t][r]) >> 1);
                        if (__umul24(nn, bd) < __umul24(bn, dd)) {
                            bn = nn;
                            bd = dd;
                            br = (uint32_t)k;
                        }
                    }
                    const uint32_t rn = run_nd[qi] & 0xFFFFu, rd = run_nd[qi] >> 16;
                    // strict <: an equal fraction keeps the earlier (lower-index) template; the
                    // running best starts as (1, 0) too
                    if (valid && __umul24(bn, rd) < __umul24(rn, bd)) {
                        run_nd[qi] = bn | (bd << 16);
                        run_jr[qi] = ((j * (uint32_t)WT + (uint32_t)t) << 5) | br;
                    }
                }
            }
            zero();
        }
        barrier();
    }

    // the lanes' running bests -> one Partial per query (lane qi holds query qi's): exact
    // fraction, then the lowest index, then the lowest rotation (the two halves of a
    // template's rotations live in lanes l and l ^ 32)
    {
        Partial best = partial_none();
#pragma unroll
        for (int qi = 0; qi < WQL; ++qi) {
            Partial c = partial_none();
            if (run_nd[qi] >> 16) {
                const uint32_t jt = run_jr[qi] >> 5, jj = jt / WT, t = jt - jj * WT;
                const uint64_t trel = (gi + (uint64_t)jj * G) * kTilesPerGroup + tset * WT + t;
                c.num = run_nd[qi] & 0xFFFFu;
                c.den = run_nd[qi] >> 16;
                c.rot = (int)(run_jr[qi] & 31u);
                c.idx = (tile0 + trel) * 32 + (lane & 31) - first;
            }
#pragma unroll
            for (int off = 32; off >= 1; off >>= 1) {
                const Partial o = partial_shfl_xor(c, off);
                if (partial_better_rot(o, c)) c = o;
            }
            if (lane == qi) best = c;
        }
        wave_best = best;
    }

    __syncthreads();
    Partial *sP = (Partial *)&afrag[0][0][0][0][0];  // [wave][query of the wave]
    if (lane < WQL) sP[w * WQL + lane] = wave_best;
    __syncthreads();
    if (tid < kBQ) {  // query tid: the waves of its query set, one per tile set
        const int qs = tid / WQL, qi = tid % WQL;
        Partial b = sP[qs * WQL + qi];
        for (int ww = qs + QW; ww < NW; ww += QW)
            if (partial_better_dev(sP[ww * WQL + qi], b)) b = sP[ww * WQL + qi];
        partials[(uint64_t)(qg * kBQ + tid) * G + gi] = b;
    }
}

// IRIS_BATCH_KERNEL (a test hook, Hooks::batch_kernel, so tests cross-check both forms): 4 (default)
// = 2-query groups x 16-tile N-groups, 2 x 2 per wave (half the LDS fragment reads and half the
// query-tile bytes per template of 2; 3.5 % faster, profiles/r03_batch_variants.txt); 2 = 4-query
// groups x 8 tiles, 4 x 1 per wave (round 2)
static int batch_kernel_choice(const Hooks &h) { return h.batch_kernel == 2 ? 2 : 4; }

uint32_t batch_query_group() { return kBatchBQ; }

BatchGeometry batch_geometry(const Hooks &h, LaunchRange r, uint32_t nq) {
    BatchGeometry g;
    g.tile0 = r.first / 32;
    const uint64_t tile1 = (r.first + r.n + 31) / 32;
    g.ntiles = tile1 - g.tile0;
    const int kc = batch_kernel_choice(h);
    g.qper = kc == 4 ? 2 : 4;  // queries per query group
    g.nqg = (nq + g.qper - 1) / g.qper;
    const uint32_t tiles_per_group = kc == 4 ? 16 : 8;
    const uint64_t ngroups = (g.ntiles + tiles_per_group - 1) / tiles_per_group;
    // one 128-KB-LDS workgroup per CU: one round of workgroups
    uint64_t G = (resident_blocks(1) + g.nqg - 1) / g.nqg;
    if (G > ngroups) G = ngroups ? ngroups : 1;
    g.G = (uint32_t)G;
    return g;
}

int launch_batch(const Hooks &h, void *stream, const void *db, const void *qtiles, LaunchRange r, const BatchGeometry &g,
                 Partial *partials, Partial *out, uint64_t idx_base) {
    if (r.n == 0) return 0;
    auto kern = batch_kernel_choice(h) == 2 ? batch_lds_kernel<8, 1, 4, 4> : batch_lds_kernel<8, 2, 2, 2>;
    hipLaunchKernelGGL(kern, dim3(g.nqg * g.G), dim3(64 * 8), 0, (hipStream_t)stream, (const uint4 *)db,
                       (const uint4 *)qtiles, g.tile0, g.ntiles, r.first, r.first + r.n, g.nqg, g.G, partials);
    if (hipGetLastError() != hipSuccess) return -1;
    hipLaunchKernelGGL(batch_reduce_kernel, dim3(g.nqg * g.qper), dim3(256), 0, (hipStream_t)stream, partials, g.G, out,
                       idx_base);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

}  // namespace iris
