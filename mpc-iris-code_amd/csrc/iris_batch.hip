// iris_batch.hip — many queries x 31 rotations x N templates (BASELINE configs[2]).
//
// The fp4 formulation of iris_mfma.hip turns a query batch into a GEMM with
// M = 32 rows per query (31 rotations + a zero row), N = templates, K = 12800
// bits, two products (den, encode) per K.  Neither operand fits on chip for
// 1024 queries x 10M templates, so it is tiled like a GEMM:
//
//   workgroup (8 waves) = 4 queries x 8 template tiles (256 templates)
//   wave w              = 2 queries x 2 tiles (128 f32 accumulators)
//   K-step              = 10 chunks of 64 bits, double-buffered in LDS:
//                         A 4 queries x 10 chunks x 64 lanes x 8 B  (20 KB)
//                         B 8 tiles   x 10 chunks x 64 lanes x 8 B  (40 KB)
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
#include <stdlib.h>

#include "iris_device.hpp"

namespace iris {

typedef int v8i __attribute__((ext_vector_type(8)));
typedef float v16f __attribute__((ext_vector_type(16)));

#ifndef IRIS_BATCH_BQ
#define IRIS_BATCH_BQ 4
#endif
constexpr int BQ = IRIS_BATCH_BQ;         // queries per workgroup (query group)
#ifndef IRIS_BATCH_NW
#define IRIS_BATCH_NW 8
#endif
constexpr int NW = IRIS_BATCH_NW;         // waves per workgroup (8: one workgroup per CU, 4: two)
#ifndef IRIS_BATCH_WQ
#define IRIS_BATCH_WQ 2
#endif
constexpr int WQ = IRIS_BATCH_WQ;         // queries per wave
#ifndef IRIS_BATCH_WT
#define IRIS_BATCH_WT (4 / IRIS_BATCH_WQ)
#endif
constexpr int WT = IRIS_BATCH_WT;         // tiles per wave (WQ x WT accumulator pairs)
constexpr int kQW = BQ / WQ;              // waves per tile set
constexpr int BT = (NW / kQW) * WT;       // template tiles per N-group
#ifndef IRIS_BATCH_KSTEP
#define IRIS_BATCH_KSTEP 10
#endif
constexpr int KSTEP = IRIS_BATCH_KSTEP;   // chunks per K-step
constexpr int GP = KSTEP / 2;             // 1-KB chunk-pair rows per operand per K-step
constexpr int NSTEPS = kPlaneDwords / 2 / KSTEP;  // 20
static_assert(NSTEPS * KSTEP * 2 == kPlaneDwords && KSTEP % 2 == 0, "K-steps must tile the 200 chunks");
constexpr int kTileU4 = kPlaneGroups * 64;        // 6400 uint4 per tile

// Diagnostic builds (tools/, never the shipped library): IRIS_BATCH_DIAG = 1 drops the
// MFMAs (a VALU fold keeps the operands live), 2 drops the LDS-DMA staging (the
// ring's stale contents are computed on), 3 feeds the raw staged words to the
// MFMAs without the fp4 expansion, 4 stages every row from the first query group
// and N-group (L2-hot), 5 drops the per-K-step s_barrier.  Results are wrong by design.
#ifndef IRIS_BATCH_DIAG
#define IRIS_BATCH_DIAG 0
#endif
__device__ __forceinline__ v16f mfma4(const v8i &a, const v8i &b, const v16f &c) {
#if IRIS_BATCH_DIAG == 1
    v16f r = c;
    r[0] += __builtin_bit_cast(float, (a[0] ^ b[1]) & 1);
    return r;
#else
    return __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(a, b, c, 4, 4, 0, 127, 0, 127);
#endif
}

// s_waitcnt with only the vector-memory count bounded (expcnt, lgkmcnt at max)
#define VMCNT(n) __builtin_amdgcn_s_waitcnt(0x0F70 | ((n) & 15) | (((n) >> 4) << 14))

constexpr int kRows = GP * (BQ + BT);  // 1-KB rows per stage: 4 queries + 8 tiles, GP chunk pairs each
#ifndef IRIS_BATCH_RING
#define IRIS_BATCH_RING 2
#endif
constexpr int kRing = IRIS_BATCH_RING;  // LDS stages: kRing - 1 in flight + the one being read
constexpr int kAhead = kRing - 1;
static_assert(kAhead >= 1 && kAhead <= 3, "ring of 2..4 stages");
#ifndef IRIS_BATCH_SPREAD
#define IRIS_BATCH_SPREAD 0
#endif
constexpr int kRowsPerWave = (kRows + NW - 1) / NW;  // waves w < kRows - NW (kRowsPerWave - 1) issue one more
constexpr bool kEvenRows = kRows % NW == 0;

// Staging is LDS-DMA (global_load_lds_dwordx4, lane-linear 1-KB rows) into a
// ring of kRing stages: each K-step waits for its own rows with a counted
// vmcnt (later steps stay in flight across the raw s_barrier), then issues the
// step kRing - 1 ahead into the slot everyone finished reading a step ago.
// Default: two stages of 10-chunk steps (120 KB) — fewer barriers per chunk
// than 4-stage rings of 4-chunk steps (measured 2 % faster at 4..1024 queries).
// Each workgroup walks its N-groups as one flat stream of K-steps, so the
// pipeline never drains between N-groups.
__global__ void __launch_bounds__(64 * NW, NW <= 8 ? 8 / NW : 1)
    batch_kernel(const uint4 *__restrict__ db, const uint4 *__restrict__ qtiles, uint64_t tile0, uint64_t ntiles,
                 uint64_t first, uint64_t end, uint32_t nqg, uint32_t G, uint32_t xqg,
                 Partial *__restrict__ partials) {
    __shared__ uint4 ring[kRing][kRows][64];  // all LDS in one object (no vmcnt(0) before ds_reads)

    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    uint32_t qg, gi;
    if (xqg) {  // XCD-aware: workgroup b runs on XCD b % 8; each XCD holds xqg query groups x G slices at a time
        const uint32_t xcd = blockIdx.x & 7, local = blockIdx.x >> 3, per = xqg * G;
        const uint32_t round = local / per, wl = local - round * per;
        qg = (round * 8 + xcd) * xqg + wl / G;
        gi = wl % G;
    } else {
        qg = blockIdx.x % nqg;
        gi = blockIdx.x / nqg;
    }
    const int wq0 = (w % kQW) * WQ, wsub = (w / kQW) * WT;
    const uint64_t ngroups = (ntiles + BT - 1) / BT;
    const uint32_t my_groups = gi < ngroups ? (uint32_t)((ngroups - gi + G - 1) / G) : 0;
    const uint32_t total = my_groups * NSTEPS;

    // this wave's DMA rows: r = w, w + 8, w + 16 (rows 0..7 queries, 8..23 template tiles)
    const uint4 *src_q[kRowsPerWave];
    int row_t[kRowsPerWave];
#pragma unroll
    for (int i = 0; i < kRowsPerWave; ++i) {
        const int r = w + NW * i;
        row_t[i] = r < GP * BQ ? -1 : (r - GP * BQ) / GP;
        const int gp = r % GP;
        src_q[i] = r < GP * BQ ? qtiles + (uint64_t)(qg * BQ + r / GP) * kTileU4 + gp * 64 + lane
                               : db + gp * 64 + lane;
    }
    auto issue = [&](uint32_t s, int ilo = 0, int ihi = kRowsPerWave) {
        const uint32_t j = s / NSTEPS, k = s - j * NSTEPS;
        const uint64_t ng = gi + (uint64_t)j * G;
#pragma unroll
        for (int i = 0; i < kRowsPerWave; ++i) {
            if (i < ilo || i >= ihi) continue;  // compile-time after unrolling
            const int r = w + NW * i;
            if (!kEvenRows && r >= kRows) break;  // wave-uniform
            const uint4 *src;
            if (IRIS_BATCH_DIAG == 4) {  // every row from the first query group / N-group: L2-hot
                src = row_t[i] < 0 ? src_q[i] - (uint64_t)(qg * BQ) * kTileU4 : src_q[i] + (tile0 + row_t[i]) * (uint64_t)kTileU4;
            } else if (row_t[i] < 0) {
                src = src_q[i] + (GP * k) * 64;
            } else {
                const uint64_t trel = ng * BT + row_t[i];
                src = src_q[i] + (tile0 + (trel < ntiles ? trel : ntiles - 1)) * (uint64_t)kTileU4 + (GP * k) * 64;
            }
            // LDS-DMA in inline asm: hipcc's waitcnt pass would otherwise wait vmcnt(0)
            // before every ds_read of the ring; the counted VMCNT waits below own these
            const uint32_t dst = __builtin_amdgcn_readfirstlane(
                (uint32_t)(uintptr_t)(__attribute__((address_space(3))) void *)&ring[s % kRing][r][0]);
            if (IRIS_BATCH_DIAG == 2) continue;
            uint32_t keep;
            asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
                         : "=&s"(keep)
                         : "v"(src), "s"(dst)
                         : "memory");
        }
    };

    Partial best[WQ];
#pragma unroll
    for (int qi = 0; qi < WQ; ++qi) {
        best[qi].num = 0;
        best[qi].den = 0;
        best[qi].rot = 0;
        best[qi].pad = 0;
        best[qi].idx = ~0ull;
    }
    v16f den[WQ][WT], sacc[WQ][WT];
    auto zero = [&] {
#pragma unroll
        for (int qi = 0; qi < WQ; ++qi)
#pragma unroll
            for (int t = 0; t < WT; ++t)
#pragma unroll
                for (int i = 0; i < 16; ++i) {
                    den[qi][t][i] = 0.f;
                    sacc[qi][t][i] = 0.f;
                }
    };
    zero();
    for (uint32_t s = 0; s < (uint32_t)kAhead && s < total; ++s) issue(s);
    // static priority for the second-dispatched half of the workgroup, the loser of VALU
    // arbitration against its SIMD partner (the ROCm MI355X microarchitecture guide, "two waves
    // per SIMD", item 4; not in this repo): 3.37 -> 3.24 s on 1024 x 10M, same box
    if (w >= NW / 2) __builtin_amdgcn_s_setprio(1);

#pragma unroll 1
    for (uint32_t s = 0; s < total; ++s) {
        // wait for this step's rows (this wave's), then for everyone's
        const bool more = kEvenRows || w + NW * (kRowsPerWave - 1) < kRows;  // this wave's rows per step
        const uint32_t younger = min((uint32_t)(kAhead - 1), total - 1 - s);  // later steps still in flight
        if (kAhead >= 3 && younger >= 2) {
            if (more) VMCNT(2 * kRowsPerWave); else VMCNT(2 * (kRowsPerWave - 1));
        } else if (kAhead >= 2 && younger >= 1) {
            if (more) VMCNT(kRowsPerWave); else VMCNT(kRowsPerWave - 1);
        } else {
            VMCNT(0);
        }
        if (IRIS_BATCH_DIAG != 5) __builtin_amdgcn_s_barrier();
        if (!IRIS_BATCH_SPREAD && s + kAhead < total) issue(s + kAhead);
        const uint4(*st)[64] = ring[s % kRing];
#pragma unroll
        for (int gp = 0; gp < GP; ++gp) {
            // IRIS_BATCH_SPREAD: the next step's DMA rows issued a few per chunk pair
            if (IRIS_BATCH_SPREAD && s + kAhead < total)
                issue(s + kAhead, gp * kRowsPerWave / GP, (gp + 1) * kRowsPerWave / GP);
            uint4 a4[WQ], b4[WT];
#pragma unroll
            for (int qi = 0; qi < WQ; ++qi) a4[qi] = st[GP * (wq0 + qi) + gp][lane];
#pragma unroll
            for (int t = 0; t < WT; ++t) b4[t] = st[GP * BQ + GP * (wsub + t) + gp][lane];
#pragma unroll
            for (int h2 = 0; h2 < 2; ++h2) {
                v8i aden[WQ], aenc[WQ];
#pragma unroll
                for (int qi = 0; qi < WQ; ++qi) {
                    const uint32_t ax = h2 ? a4[qi].z : a4[qi].x, ay = h2 ? a4[qi].w : a4[qi].y;
#if IRIS_BATCH_DIAG == 3
                    aden[qi] = v8i{(int)ax, (int)ay, (int)ax, (int)ay, 0, 0, 0, 0};
                    aenc[qi] = v8i{(int)ay, (int)ax, (int)ay, (int)ax, 0, 0, 0, 0};
#else
                    aden[qi] = v8i{(int)(ax & 0x22222222u), (int)((ax & 0x11111111u) << 2), (int)(ay & 0x22222222u),
                                   (int)((ay & 0x11111111u) << 2), 0, 0, 0, 0};
                    aenc[qi] = v8i{(int)(ax & 0xAAAAAAAAu), (int)((ax << 1) & 0xAAAAAAAAu), (int)(ay & 0xAAAAAAAAu),
                                   (int)((ay << 1) & 0xAAAAAAAAu), 0, 0, 0, 0};
#endif
                }
#pragma unroll
                for (int t = 0; t < WT; ++t) {
                    const uint32_t bx = h2 ? b4[t].z : b4[t].x, by = h2 ? b4[t].w : b4[t].y;
#if IRIS_BATCH_DIAG == 3
                    const v8i bden = {(int)bx, (int)by, (int)bx, (int)by, 0, 0, 0, 0};
                    const v8i benc = {(int)by, (int)bx, (int)by, (int)bx, 0, 0, 0, 0};
#else
                    const v8i bden = {(int)(bx & 0x22222222u), (int)(bx & 0x11111111u), (int)(by & 0x22222222u),
                                      (int)(by & 0x11111111u), 0, 0, 0, 0};
                    const v8i benc = {(int)(bx & 0xAAAAAAAAu), (int)((bx << 1) & 0xAAAAAAAAu),
                                      (int)(by & 0xAAAAAAAAu), (int)((by << 1) & 0xAAAAAAAAu), 0, 0, 0, 0};
#endif
#pragma unroll
                    for (int qi = 0; qi < WQ; ++qi) {
                        den[qi][t] = mfma4(aden[qi], bden, den[qi][t]);
                        sacc[qi][t] = mfma4(aenc[qi], benc, sacc[qi][t]);
                    }
                }
            }
        }
        const uint32_t j = s / NSTEPS;
        if (s - j * NSTEPS != NSTEPS - 1) continue;
        // N-group done: per template, min over the 16 rows of this lane, then the partner half
        const uint64_t ng = gi + (uint64_t)j * G;
#pragma unroll
        for (int qi = 0; qi < WQ; ++qi)
#pragma unroll
            for (int t = 0; t < WT; ++t) {
                uint32_t bn, bd;
                int br;
                best_rotation(lane, [&](int r, uint32_t &nn, uint32_t &dd) {
                    dd = (uint32_t)den[qi][t][r];
                    nn = (uint32_t)(((int)dd - (int)sacc[qi][t][r]) >> 1);
                }, bn, bd, br);
                const uint64_t trel2 = ng * BT + wsub + t;
                const uint64_t tg = (tile0 + trel2) * 32 + (lane & 31);
                const bool valid = trel2 < ntiles && tg >= first && tg < end;
                Partial c;
                c.num = bn;
                c.den = valid ? bd : 0;
                c.rot = br;
                c.pad = 0;
                c.idx = tg - first;
                if (partial_better_dev(c, best[qi])) best[qi] = c;
            }
        zero();
    }
#pragma unroll
    for (int qi = 0; qi < WQ; ++qi)
#pragma unroll
        for (int off = 32; off >= 1; off >>= 1) {
            const Partial o = partial_shfl_xor(best[qi], off);
            if (partial_better_dev(o, best[qi])) best[qi] = o;
        }
    // the ring is idle (every DMA was waited for): reuse it for the cross-wave reduction
    VMCNT(0);
    __syncthreads();
    Partial *sP = (Partial *)&ring[0][0][0];  // [wave][WQ]
    if (lane == 0)
#pragma unroll
        for (int qi = 0; qi < WQ; ++qi) sP[w * WQ + qi] = best[qi];
    __syncthreads();
    if (tid < BQ) {  // query tid: waves with wq0 <= tid < wq0 + WQ, one per tile set
        const int qi = tid % WQ, wl = tid / WQ;
        Partial b = sP[wl * WQ + qi];
        for (int ts = 1; ts < NW / kQW; ++ts)
            if (partial_better_dev(sP[(ts * kQW + wl) * WQ + qi], b)) b = sP[(ts * kQW + wl) * WQ + qi];
        partials[(uint64_t)(qg * BQ + tid) * G + gi] = b;
    }
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
// The same GEMM (M = 32 rows per query, N = templates, K = 12800 bits, den + encode
// products) with the operand traffic re-balanced for the VALU:
//
//   workgroup (8 waves) = 4 queries (shared by all 8 waves) x 8 template tiles (one per wave)
//   K-step              = GP chunk pairs
//
// - A (the 4 queries' rotation tiles) is loaded once per workgroup and K-step (2 rows of
//   1 KB per wave, plain global loads a step ahead), expanded ONCE into the MFMA-ready fp4
//   den / encode fragments and written to a 2-stage LDS ring; every wave reads all four
//   queries' fragments from it (ds_read_b128, lane-linear 1-KB rows: conflict-free).
//   batch_kernel instead re-expands every A fragment in each of the 4 waves that use it.
// - B (templates): each wave owns one tile per N-group and loads it straight into
//   registers (global_load_dwordx4, 1 KB per wave and chunk pair, one K-step ahead) —
//   no LDS-DMA (whose issue cost, ~60 cycles per 1-KB piece beside MFMAs, was ~17 % of
//   batch_kernel) — and expands it itself (10 VALU per 64-bit chunk).
// - VALU per MFMA: 20 (B) + 12 (this wave's share of the A expansion) per 16 MFMAs,
//   against 88 in batch_kernel; one s_barrier per K-step.
// The grid holds one workgroup per CU; all query groups walk the same N-groups, so a
// template tile comes from HBM about once per XCD and from L2 after that.
#ifndef IRIS_BATCH2_GP
#define IRIS_BATCH2_GP 4
#endif
// Diagnostic builds (tools/, never the shipped library; results wrong by design):
// IRIS_BATCH2_DIAG = 1 no s_barrier, 2 no LDS fragment reads (the B operands stand in),
// 3 no B loads after the first step, 4 no A loads / expansion after the first step,
// 5 no MFMAs (a VALU fold keeps the operands live), 6 the template (B) operands expanded for chunk pair 0
// only and reused for the K-step's other pairs (their loads still consumed), 7 every workgroup loads query
// group 0's rows (the A stream L2-hot: no query-tile traffic beyond L2), 8 every wave loads N-group 0's
// tiles (the B stream L2-hot)
#ifndef IRIS_BATCH2_DIAG
#define IRIS_BATCH2_DIAG 0
#endif
// 1: block b + 1's fragment reads issued between block b's MFMAs; 0: each block reads its own
#ifndef IRIS_BATCH2_STAGGER
#define IRIS_BATCH2_STAGGER 1
#endif
#ifndef IRIS_BATCH2_ROLL
#define IRIS_BATCH2_ROLL 1
#endif
namespace lds2 {
constexpr int kGP = IRIS_BATCH2_GP;      // chunk pairs per K-step
}  // namespace lds2

// Waves: QW = kBQ / WQL query sets x NW / QW tile sets; a wave holds WQL queries x WT tiles
// and the tile sets x WT = 8 tiles per N-group.  NW = 8, WQL = 4, WT = 1: every wave reads
// all four queries' fragments from LDS (one fragment read per MFMA pair); NW = 8, WQL = 2,
// WT = 2: each fragment read feeds two tiles (half the LDS reads per MFMA), each template
// tile is loaded and expanded by the two waves of its tile set; both 128 accumulators.
// NW = 4, WQL = 4, WT = 2: one wave per SIMD, 256 accumulators.
// BQL = queries per workgroup (a query group): 4 (tiles per N-group = 8 with the shapes
// above) or 2 with WQL = 2, WT = 2 (16 tiles per N-group: each query tile read from beyond L2
// is applied to twice the templates, half the A traffic per query).
#ifndef IRIS_BATCH2_GP_Q2
#define IRIS_BATCH2_GP_Q2 4  // chunk pairs per K-step of the 2-query-group shape (5: 197 VGPRs spilled)
#endif
template <int NW, int WT, int WQL = 4, int BQL = 4, int GPL = lds2::kGP>
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
    static_assert(kBQ % WQL == 0 && NW % QW == 0 && IRIS_BATCH_BQ % kBQ == 0, "geometry");
    constexpr int kAper = (kArows + NW - 1) / NW;  // compact A rows per wave and K-step (the last may be idle)
    // [stage][chunk pair][query][den h0, enc h0, den h1, enc h1][lane]: 2 x kGP x 16 KB
    __shared__ uint4 afrag[2][kGP][kBQ][4][64];

    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int qset = w % QW, tset = w / QW;  // this wave's queries qset * WQL + qi, tiles tset * WT + t
    const uint32_t qg = blockIdx.x % nqg, gi = blockIdx.x / nqg;
    const uint64_t ngroups = (ntiles + kTilesPerGroup - 1) / kTilesPerGroup;
    const uint32_t my_groups = gi < ngroups ? (uint32_t)((ngroups - gi + G - 1) / G) : 0;
    const uint32_t total = my_groups * kSteps;
    // Stagger (IRIS_BATCH2_STAGGER): the two waves sharing a SIMD (w and w + 4) run their N-groups
    // half a group apart, so one wave's epilogue (no MFMAs) overlaps its partner's MFMAs.  The
    // K-step at time s is s mod kSteps for every wave (the A fragments in LDS are shared); waves
    // 4..7 start their first group at s = off and the workgroup walks off extra steps, in which
    // the idle waves' MFMAs run on re-read rows and are discarded.
    // (the 2 x 2 per-wave shape runs 2 % faster without it: profiles/r03_batch_variants.txt)
    constexpr bool kStagger = IRIS_BATCH2_STAGGER && NW == 8 && WQL == 4;
    const uint32_t off = (kStagger && w >= NW / 2) ? (uint32_t)(kSteps / 2) : 0u;
    const uint32_t walk = total ? total + (kStagger ? (uint32_t)(kSteps / 2) : 0u) : 0u;
    auto group_of = [&](uint32_t s) {  // this wave's N-group at time s (clamped while idle)
        const uint32_t r = s >= off ? (s - off) / kSteps : 0u;
        return r < my_groups ? r : my_groups - 1;
    };

    // this wave's compact A rows of a K-step: r = w + NW i -> query r % kBQ, chunk pair r / kBQ
    const uint4 *abase = qtiles + (uint64_t)(IRIS_BATCH2_DIAG == 7 ? 0u : qg * kBQ) * kTileU4 + lane;
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
        const uint64_t trel = IRIS_BATCH2_DIAG == 8 ? (uint64_t)(tset * WT + t)
                                                    : (gi + (uint64_t)j * G) * kTilesPerGroup + tset * WT + t;
        return db + (tile0 + (trel < ntiles ? trel : ntiles - 1)) * (uint64_t)kTileU4 + (k * kGP) * 64 + lane;
    };
    // compact A row -> fp4 den / encode fragments of both chunks (the expansion of batch_kernel)
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
        if (IRIS_BATCH2_DIAG != 1) __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
    };
    auto mma = [](const v8i &a, const v8i &b, const v16f &c) {
#if IRIS_BATCH2_DIAG == 5
        v16f r = c;
        r[0] += __builtin_bit_cast(float, (a[0] ^ b[1]) & 1);
        return r;
#else
        return mfma4(a, b, c);
#endif
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
#ifndef IRIS_BATCH2_PRIO
#define IRIS_BATCH2_PRIO 0  // 1: s_setprio 1 for waves 4..7 (helped before the stagger, costs 2.6 % with it)
#endif
    if (IRIS_BATCH2_PRIO && NW == 8 && w >= NW / 2) __builtin_amdgcn_s_setprio(1);  // the younger half (see batch_kernel)

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
        if (IRIS_BATCH2_DIAG != 4 || s == 0) load_a(s1, aq);
        const uint4(*st)[kBQ][4][64] = afrag[s & 1];
        // blocks b = 2 gp + h2 (one 64-bit chunk): block b + 1's fragment reads are issued
        // between block b's MFMAs (rolling: their latency hides behind the MFMAs)
        auto frag = [&](int b, int form, int qi) {
#if IRIS_BATCH2_DIAG == 2
            const uint4 q = bq[0][b >> 1];
            return form ? make_uint4(q.x & 0xAAAAAAAAu, q.y & 0xAAAAAAAAu, q.z & 0xAAAAAAAAu, q.w ^ qi)
                        : make_uint4(q.x & 0x22222222u, q.y & 0x11111111u, q.z & 0x22222222u, q.w & qi);
#else
            return st[b >> 1][qset * WQL + qi][2 * (b & 1) + form][lane];
#endif
        };
        uint4 fa[WQL], fe[WQL];
#pragma unroll
        for (int qi = 0; qi < WQL; ++qi) {
            fa[qi] = frag(0, 0, qi);
            fe[qi] = frag(0, 1, qi);
        }
        v8i sd[2][WT], se[2][WT];  // IRIS_BATCH2_DIAG 6: chunk pair 0's expansions, reused
#pragma unroll
        for (int b = 0; b < 2 * kGP; ++b) {
            const bool nb = b + 1 < 2 * kGP;
            v8i bd[WT], be[WT];
#pragma unroll
            for (int t = 0; t < WT; ++t) {
                const uint4 q = bq[t][b >> 1];
                if (IRIS_BATCH2_DIAG == 6 && b >= 2) {  // the load is consumed where the shipped kernel expands it
                    asm volatile("" ::"v"(q.x), "v"(q.y), "v"(q.z), "v"(q.w));
                    bd[t] = sd[b & 1][t];
                    be[t] = se[b & 1][t];
                    continue;
                }
                const uint32_t bx = (b & 1) ? q.z : q.x, by = (b & 1) ? q.w : q.y;
                bd[t] = v8i{(int)(bx & 0x22222222u), (int)(bx & 0x11111111u), (int)(by & 0x22222222u),
                            (int)(by & 0x11111111u), 0, 0, 0, 0};
                be[t] = v8i{(int)(bx & 0xAAAAAAAAu), (int)((bx << 1) & 0xAAAAAAAAu), (int)(by & 0xAAAAAAAAu),
                            (int)((by << 1) & 0xAAAAAAAAu), 0, 0, 0, 0};
                if (IRIS_BATCH2_DIAG == 6) {
                    sd[b & 1][t] = bd[t];
                    se[b & 1][t] = be[t];
                }
            }
            if ((b & 1) && (IRIS_BATCH2_DIAG != 3 || s == 0)) {  // both chunks of chunk pair b >> 1 expanded: its registers take step s + 1's
#pragma unroll
                for (int t = 0; t < WT; ++t) bq[t][b >> 1] = b_row(s1, t)[(b >> 1) * 64];
            }
            uint4 na[WQL], ne[WQL];
#pragma unroll
            for (int qi = 0; qi < WQL; ++qi) {
                if (!IRIS_BATCH2_ROLL) {
                    fa[qi] = frag(b, 0, qi);
                    fe[qi] = frag(b, 1, qi);
                }
                const v8i a_d = {(int)fa[qi].x, (int)fa[qi].y, (int)fa[qi].z, (int)fa[qi].w, 0, 0, 0, 0};
                const v8i a_e = {(int)fe[qi].x, (int)fe[qi].y, (int)fe[qi].z, (int)fe[qi].w, 0, 0, 0, 0};
#pragma unroll
                for (int t = 0; t < WT; ++t) den[qi][t] = mma(a_d, bd[t], den[qi][t]);
                if (nb && IRIS_BATCH2_ROLL) na[qi] = frag(b + 1, 0, qi);
#pragma unroll
                for (int t = 0; t < WT; ++t) sacc[qi][t] = mma(a_e, be[t], sacc[qi][t]);
                if (nb && IRIS_BATCH2_ROLL) ne[qi] = frag(b + 1, 1, qi);
            }
            __builtin_amdgcn_sched_barrier(0);
            if (nb && IRIS_BATCH2_ROLL) {
#pragma unroll
                for (int qi = 0; qi < WQL; ++qi) {
                    fa[qi] = na[qi];
                    fe[qi] = ne[qi];
                }
            }
        }
        if (IRIS_BATCH2_DIAG != 4 || s == 0) store_a(s + 1, aq);  // the last step fills the idle stage (read by nobody)
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

// IRIS_BATCH_KERNEL (a test hook, Hooks::batch_kernel, so tests run every form): 4 = batch_lds_kernel with
// 2-query groups x 16-tile N-groups, 2 x 2 per wave (default: half the LDS fragment reads and
// half the query-tile bytes per template of 2; 3.5 % faster, profiles/r03_batch_variants.txt);
// 2 = batch_lds_kernel 4-query groups x 8 tiles, 4 x 1 per wave (round 2); 3 = 4-query groups,
// 2 x 2 per wave; 1 = batch_kernel (LDS-DMA staged, round 1)
static int batch_kernel_choice(const Hooks &h) { return h.batch_kernel >= 1 && h.batch_kernel <= 4 ? h.batch_kernel : 4; }

uint32_t batch_query_group() { return BQ; }

BatchGeometry batch_geometry(const Hooks &h, LaunchRange r, uint32_t nq) {
    BatchGeometry g;
    g.tile0 = r.first / 32;
    const uint64_t tile1 = (r.first + r.n + 31) / 32;
    g.ntiles = tile1 - g.tile0;
    const int kc = batch_kernel_choice(h);
    g.qper = kc == 4 ? 2 : BQ;  // queries per query group
    g.nqg = (nq + g.qper - 1) / g.qper;
    const uint32_t tiles_per_group = kc == 1 ? BT : kc == 4 ? 16 : 8;
    const uint64_t ngroups = (g.ntiles + tiles_per_group - 1) / tiles_per_group;
    // batch_kernel: ~2 workgroups per CU in total; batch_lds_kernel (one 128-KB-LDS workgroup
    // per CU): one round of workgroups
    const uint64_t want = kc >= 2 ? resident_blocks(1) : 512;
    uint64_t G = (want + g.nqg - 1) / g.nqg;
    if (G > ngroups) G = ngroups ? ngroups : 1;
    g.G = (uint32_t)G;
    g.xqg = 0;
    // XCD-aware grid (IRIS_BATCH_XQG = query groups per XCD per round): the 32 CUs of an XCD
    // run xqg query groups x 32/xqg N-slices, so their query tiles stay in that XCD's L2
    if (kc == 1 && h.batch_xqg) {
        const uint32_t x = h.batch_xqg;
        if (x && 32 % x == 0 && g.nqg % (8 * x) == 0 && ngroups >= 32 / x) {
            g.xqg = x;
            g.G = 32 / x;
        }
    }
    return g;
}

int launch_batch(const Hooks &h, void *stream, const void *db, const void *qtiles, LaunchRange r, const BatchGeometry &g,
                 Partial *partials, Partial *out, uint64_t idx_base) {
    if (r.n == 0) return 0;
    const int kc = batch_kernel_choice(h);
    if (kc == 2)
        hipLaunchKernelGGL((batch_lds_kernel<8, 1>), dim3(g.nqg * g.G), dim3(64 * 8), 0, (hipStream_t)stream,
                           (const uint4 *)db, (const uint4 *)qtiles, g.tile0, g.ntiles, r.first, r.first + r.n, g.nqg,
                           g.G, partials);
    else if (kc == 3)  // 2 queries x 2 tiles per wave: half the LDS fragment reads per MFMA
        hipLaunchKernelGGL((batch_lds_kernel<8, 2, 2>), dim3(g.nqg * g.G), dim3(64 * 8), 0, (hipStream_t)stream,
                           (const uint4 *)db, (const uint4 *)qtiles, g.tile0, g.ntiles, r.first, r.first + r.n, g.nqg,
                           g.G, partials);
    else if (kc == 4)  // 2-query groups x 16-tile N-groups: half the query-tile traffic beyond L2
        hipLaunchKernelGGL((batch_lds_kernel<8, 2, 2, 2, IRIS_BATCH2_GP_Q2>), dim3(g.nqg * g.G), dim3(64 * 8), 0,
                           (hipStream_t)stream,
                           (const uint4 *)db, (const uint4 *)qtiles, g.tile0, g.ntiles, r.first, r.first + r.n, g.nqg,
                           g.G, partials);
    else
        hipLaunchKernelGGL(batch_kernel, dim3(g.nqg * g.G), dim3(64 * NW), 0, (hipStream_t)stream, (const uint4 *)db,
                           (const uint4 *)qtiles, g.tile0, g.ntiles, r.first, r.first + r.n, g.nqg, g.G, g.xqg,
                           partials);
    if (hipGetLastError() != hipSuccess) return -1;
    hipLaunchKernelGGL(batch_reduce_kernel, dim3(g.nqg * g.qper), dim3(256), 0, (hipStream_t)stream, partials, g.G, out,
                       idx_base);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

}  // namespace iris
