// iris_engines_mfma.hip — MasksEngine and DistanceEngine on the matrix cores.
//
// MasksEngine::batch_process (src/lib.rs:69-79): out[k][t] = popcount(rot_k(qm) & m_t)
//   = sum_b qm_k[b] * m_t[b]: fp4 e2m1 MFMA, M = 32 rotation rows, N = 32 masks,
//   K = 12800 bits, one v_mfma_scale_f32_32x32x64_f8f6f4 per 64-bit chunk.
//
// DistanceEngine::batch_process (src/lib.rs:42-52): out[k][t] = sum_i q_k[i] e_t[i]
//   mod 2^16 over 12800 u16.  With bytes a = a_hi*256 + a_lo and a' = a - 128
//   (an i8): q*e = q_lo e_lo + 256 (q_lo e_hi + q_hi e_lo)  (mod 2^16), and
//   sum x_lo y_lo = sum x'y' + 128 sum x' + 128 sum y' + 16384 K, so two i32
//   accumulators of v_mfma_i32_32x32x32_i8 over pre-biased byte planes
//     S1 = sum q'_lo e'_lo,  S2 = sum q'_lo e'_hi + q'_hi e'_lo
//   plus per-row query sums (host) and per-share byte sums (the otherwise
//   unused 32nd A row is all ones) recombine exactly mod 2^16.
//   |S| <= 2 * 12800 * 128^2 < 2^31.
#include <hip/hip_runtime.h>
#include <stdlib.h>

#include "iris_device.hpp"

namespace iris {

typedef int v4i __attribute__((ext_vector_type(4)));
typedef int v8i __attribute__((ext_vector_type(8)));
typedef int v16i __attribute__((ext_vector_type(16)));
typedef float v16f __attribute__((ext_vector_type(16)));
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

constexpr int kTile = 32;
// tiles per wave: 7 for the [u16;31] output (longer groups, fewer store bursts than 4:
// round 2 measured 8 at 2.88-2.98 vs 2.98-3.03 ms per 10M for 4; but 8 tiles need 29 VGPRs
// of scratch spills at two waves per SIMD, and 7 -- 252 VGPRs, none spilled -- runs 2.894-2.896
// vs 2.916-2.919 ms for 8, 2.894-2.900 for 6, 2.910-2.912 for 5, interleaved on one box,
// profiles/r04_masks_variants.txt); the fused resolver keeps 4 (its epilogue state at 8 tiles
// costs registers: 5.1 vs 2.7 ms)
constexpr int kMasksTiles = 7;
constexpr int kResolveTiles = 4;
template <int MODE>
constexpr int masks_tiles() { return MODE != 1 ? kMasksTiles : kResolveTiles; }
constexpr int kMasksBlocksPerCu = 2;  // persistent grid: workgroups per CU
// MasksEngine stages the compact query (51 KB) in LDS per workgroup (two workgroups per CU); the
// fused resolver (4 tiles per wave, 168 VGPRs) runs three workgroups per CU with the query read
// from L2 by every wave: 2.78 vs 2.87 ms per 10M masks + 3 x 10M share rows, interleaved on one
// box (profiles/r04_masks_variants.txt); for the [u16;31] output the same shape measured even
// (2.90-3.01 vs 2.93-3.00 ms).
constexpr int kResolveBlocksPerCu = 3;
template <int MODE>
constexpr int masks_blocks_per_cu() { return MODE != 1 ? kMasksBlocksPerCu : kResolveBlocksPerCu; }
constexpr int kSharesTiles = 2;

__device__ __forceinline__ uint4 nt_load(const uint4 *p) {
    const u32x4 v = __builtin_nontemporal_load((const u32x4 *)p);
    return make_uint4(v.x, v.y, v.z, v.w);
}

struct Tiles {
    uint64_t tile0, ntiles, grid;
};

static Tiles tiles_of(LaunchRange r, int per_wave) {
    Tiles t;
    t.tile0 = r.first / kTile;
    const uint64_t tile1 = (r.first + r.n + kTile - 1) / kTile;
    t.ntiles = tile1 - t.tile0;
    const uint64_t waves = (t.ntiles + per_wave - 1) / per_wave;
    t.grid = (waves + kWaveSlots - 1) / kWaveSlots;
    return t;
}

// ------------------------------------------------------------------ masks (fp4)

__device__ __forceinline__ v16f mfma_fp4(const v8i &a, const v8i &b, const v16f &c) {
    return __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(a, b, c, 4, 4, 0, 127, 0, 127);
}

// x: one dword of a mask tile (8 masks' nibbles); w: the compact query word of
// the same chunk (see kMaskFragUint4)
__device__ __forceinline__ v8i mask_a(uint32_t w) {
    return v8i{(int)(w & 0x44444444u), (int)(w & 0x22222222u), (int)(w & 0x11111111u), (int)((w >> 3) & 0x11111111u),
               0, 0, 0, 0};
}

__device__ __forceinline__ void mask_chunk(uint32_t x, const v8i &a, v16f &acc) {
    const v8i b = {(int)(x & 0x11111111u), (int)(x & 0x22222222u), (int)(x & 0x44444444u),
                   (int)((x >> 1) & 0x44444444u), 0, 0, 0, 0};
    acc = mfma_fp4(a, b, acc);
}

// Fused resolver operands (MASKS_RESOLVE): the participants' [n][31] u16
// outputs, row i = record first + i (src/main.rs:597-607).
struct MaskResolve {
    const uint16_t *shares[8];
    uint32_t parts;
    bool aligned;  // every share array 16-B aligned
    double *dist_out;
    Partial *partials;
};

// MASKS_PACKED: the [u16;31] rows in the read-ahead's packed form (store_tile_packed, iris_device.hpp)
enum { MASKS_OUT = 0, MASKS_RESOLVE = 1, MASKS_PACKED = 2 };

// Persistent: each wave walks the tile groups wave, wave + nwaves, ... as one
// flat stream of (group, step) K-steps, so the loads of the next group are in
// flight while the current group's rows are written out (a wave that exits
// after its stores leaves its slot idle until they are acknowledged).  The
// compact query (51 KB) is staged in LDS once per workgroup.
//
// MASKS_RESOLVE replaces the [u16;31] output with the resolver step
// (src/main.rs:510-519 + 597-621): the tile's summed shares are staged in LDS,
// each lane decodes its 16 (template, rotation) cells against the
// denominators still in its accumulators (decode_distance, src/lib.rs:97-107),
// and a running (fraction, lowest index) best per lane becomes one partial per
// workgroup — the denominators never reach memory.
template <int MODE, int T = masks_tiles<MODE>()>
__global__ void __launch_bounds__(256, masks_blocks_per_cu<MODE>())
    masks_mfma_kernel(const uint4 *__restrict__ db, const uint4 *__restrict__ qfrag, uint64_t tile0, uint64_t ntiles,
                      uint64_t first, uint64_t end, uint16_t *__restrict__ out, MaskResolve rs) {
    constexpr uint32_t kSteps = kMaskChunks / 4;  // 50 steps of 4 chunks
    const uint4 *sq = qfrag;  // the query's compact fragments: in LDS, or read from L2
    if constexpr (MODE != MASKS_RESOLVE) {
        __shared__ uint4 sq_lds[kMaskFragUint4];
        for (int i = threadIdx.x; i < (int)kMaskFragUint4; i += blockDim.x) sq_lds[i] = qfrag[i];
        __syncthreads();
        sq = sq_lds;
    }
    __shared__ __attribute__((aligned(16))) uint16_t sh_out[kWaveSlots][1024];

    const int lane = threadIdx.x & 63;
    const uint64_t wave = __builtin_amdgcn_readfirstlane(blockIdx.x * kWaveSlots + (threadIdx.x >> 6));
    const uint64_t nwaves = (uint64_t)gridDim.x * kWaveSlots;
    const uint64_t ngroups = (ntiles + T - 1) / T;
    if (MODE != MASKS_RESOLVE && wave >= ngroups) return;
    const uint32_t total = wave < ngroups ? (uint32_t)((ngroups - wave + nwaves - 1) / nwaves) * kSteps : 0;
    uint16_t *lds = sh_out[threadIdx.x >> 6];
    Partial best = partial_none();

    v16f acc[T];
    auto zero = [&] {
#pragma unroll
        for (int t = 0; t < T; ++t)
#pragma unroll
            for (int i = 0; i < 16; ++i) acc[t][i] = 0.f;
    };
    // resolver epilogue of one tile (records t0 .. t0+31 of the database)
    auto resolve_tile = [&](uint64_t t0, bool tv, const v16f &den) {
        const bool full = tv && t0 >= first && t0 + 32 <= end && ((t0 - first) & 7) == 0 && rs.aligned;
        const uint64_t e0 = (t0 - first) * kRot;  // first share element of the tile (when full)
        if (full) {  // wave-uniform: 124 16-B words per share array
            typedef unsigned short u16x8 __attribute__((ext_vector_type(8)));
            for (int i = lane; i < 32 * kRot / 8; i += 64) {
                // plain loads (nontemporal measured the same, 2.75-2.79 ms per 10M either way)
                u16x8 v = *(const u16x8 *)(rs.shares[0] + e0 + 8 * i);
                for (uint32_t p = 1; p < rs.parts; ++p) v += *(const u16x8 *)(rs.shares[p] + e0 + 8 * i);
                *(u16x8 *)&lds[8 * i] = v;
            }
        } else {
            for (int i = lane; i < 32 * kRot; i += 64) {
                const uint64_t tg = t0 + (uint64_t)(i / kRot);
                uint16_t v = 0;
                if (tv && tg >= first && tg < end) {
                    const uint64_t e = (tg - first) * kRot + (uint64_t)(i % kRot);
                    for (uint32_t p = 0; p < rs.parts; ++p) v = (uint16_t)(v + rs.shares[p][e]);
                }
                lds[i] = v;
            }
        }
        __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0): this wave's LDS writes landed
        __builtin_amdgcn_wave_barrier();
        const int h = lane >> 5;
        uint32_t bn, bd;
        int br;
        best_rotation(lane, [&](int r, uint32_t &u, uint32_t &d) {
            const int k = (r & 3) + 8 * (r >> 2) + 4 * h;
            d = (uint32_t)den[r] & 0xFFFFu;  // the MasksEngine output value (u16)
            u = k < kRot ? (uint32_t)((uint16_t)(d - lds[(lane & 31) * kRot + k]) >> 1) : 0;  // src/lib.rs:104
        }, bn, bd, br);
        const uint64_t tg = t0 + (lane & 31);
        const bool valid = tv && tg >= first && tg < end;
        if (valid && rs.dist_out && h == 0) rs.dist_out[tg - first] = bd ? (double)bn / (double)bd : __builtin_inf();
        Partial c;
        c.num = bn;
        c.den = valid ? bd : 0;
        c.rot = br;
        c.pad = 0;
        c.idx = tg - first;
        if (partial_better_dev(c, best)) best = c;
        __builtin_amdgcn_wave_barrier();  // LDS reads done before the next tile overwrites
    };
    if (total) {
        zero();
        struct Stage {
            uint4 d[T];
            uint4 w;
        };
        auto load = [&](Stage &st, uint32_t s) {
            s = s < total ? s : total - 1;
            const uint32_t j = s / kSteps, g = s - j * kSteps;
            const uint64_t tw = (wave + (uint64_t)j * nwaves) * T;
#pragma unroll
            for (int t = 0; t < T; ++t) {
                const uint64_t rel = (tw + t < ntiles) ? tw + t : ntiles - 1;
                st.d[t] = nt_load(db + (tile0 + rel) * (uint64_t)kMaskTileUint4 + g * 64 + lane);
            }
            st.w = sq[g * 64 + lane];
            __builtin_amdgcn_sched_barrier(0);
        };
        auto compute = [&](const Stage &st, uint32_t s) {
            if (s >= total) return;
            const v8i a0 = mask_a(st.w.x), a1 = mask_a(st.w.y), a2 = mask_a(st.w.z), a3 = mask_a(st.w.w);
#pragma unroll
            for (int t = 0; t < T; ++t) {
                mask_chunk(st.d[t].x, a0, acc[t]);
                mask_chunk(st.d[t].y, a1, acc[t]);
                mask_chunk(st.d[t].z, a2, acc[t]);
                mask_chunk(st.d[t].w, a3, acc[t]);
            }
            const uint32_t j = s / kSteps;
            if (s - j * kSteps == kSteps - 1) {  // group j done: write its rows / resolve it
                const uint64_t tw = (wave + (uint64_t)j * nwaves) * T;
#pragma unroll
                for (int t = 0; t < T; ++t) {
                    if constexpr (MODE == MASKS_OUT)
                        store_tile_rows(out, lds, (tile0 + tw + t) * kTile, first, end, tw + t < ntiles, lane,
                                        [&](int r) { return (uint16_t)(uint32_t)acc[t][r]; });
                    else if constexpr (MODE == MASKS_PACKED)
                        store_tile_packed((uint8_t *)out, out + (end - first) * 16, (tile0 + tw + t) * kTile, first, end,
                                          tw + t < ntiles, lane, [&](int r) { return (uint32_t)acc[t][r]; });
                    else
                        resolve_tile((tile0 + tw + t) * kTile, tw + t < ntiles, acc[t]);
                }
                zero();
            }
        };
        Stage sa, sb, sc;
        load(sa, 0);
        load(sb, 1);
#pragma unroll 1
        for (uint32_t s = 0; s < total; s += 3) {
            load(sc, s + 2);
            compute(sa, s);
            load(sa, s + 3);
            compute(sb, s + 1);
            load(sb, s + 4);
            compute(sc, s + 2);
        }
    }
    if constexpr (MODE == MASKS_RESOLVE) {
#pragma unroll
        for (int off = 32; off >= 1; off >>= 1) {
            const Partial o = partial_shfl_xor(best, off);
            if (partial_better_dev(o, best)) best = o;
        }
        __shared__ Partial sh_best[kWaveSlots];
        if (lane == 0) sh_best[threadIdx.x >> 6] = best;
        __syncthreads();
        if (threadIdx.x == 0) {
            Partial b = sh_best[0];
            for (int w = 1; w < kWaveSlots; ++w)
                if (partial_better_dev(sh_best[w], b)) b = sh_best[w];
            rs.partials[blockIdx.x] = b;
        }
    }
}

// Small ranges (up to kMasksSplitTiles tiles: the resolver's 20k-record chunks,
// src/main.rs:511-516): one tile per workgroup of KS waves, wave w summing K-slice w
// (kSteps / KS steps of 4 chunks).  Every load of the slice -- mask dwords from HBM,
// query words from L2 (no LDS staging of the whole query per workgroup) -- is issued
// up front, so the launch costs about one HBM round trip per wave instead of the
// persistent kernel's ~25 dependent ones; the slices' counts (exact integers in f32)
// meet in LDS and wave 0 writes the tile's rows.
constexpr int kMasksSplitKS = 10;
constexpr uint64_t kMasksSplitTiles = 1024;

template <int KS, bool PACKED = false>
__global__ void __launch_bounds__(64 * KS)
    masks_split_kernel(const uint4 *__restrict__ db, const uint4 *__restrict__ qfrag, uint64_t tile0,
                       uint64_t first, uint64_t end, uint16_t *__restrict__ out, DoneSignal sig) {
    constexpr int kSteps = kMaskChunks / 4;  // 50
    static_assert(kSteps % KS == 0, "K-split geometry");
    constexpr int kG = kSteps / KS;
    const int lane = threadIdx.x & 63;
    const int slice = threadIdx.x >> 6;
    const uint64_t tile = tile0 + blockIdx.x;
    const uint4 *dp = db + tile * (uint64_t)kMaskTileUint4 + (uint64_t)slice * kG * 64 + lane;
    const uint4 *qp = qfrag + (uint64_t)slice * kG * 64 + lane;
    uint4 d[kG], w[kG];
#pragma unroll
    for (int g = 0; g < kG; ++g) d[g] = nt_load(dp + g * 64);
#pragma unroll
    for (int g = 0; g < kG; ++g) w[g] = qp[g * 64];
    v16f acc;
#pragma unroll
    for (int i = 0; i < 16; ++i) acc[i] = 0.f;
#pragma unroll
    for (int g = 0; g < kG; ++g) {
        mask_chunk(d[g].x, mask_a(w[g].x), acc);
        mask_chunk(d[g].y, mask_a(w[g].y), acc);
        mask_chunk(d[g].z, mask_a(w[g].z), acc);
        mask_chunk(d[g].w, mask_a(w[g].w), acc);
    }
    __shared__ float red[KS - 1][16][64];
    __shared__ __attribute__((aligned(16))) uint16_t sh_out[1024];
    if (slice != 0) {
#pragma unroll
        for (int i = 0; i < 16; ++i) red[slice - 1][i][lane] = acc[i];
    }
    __syncthreads();
    if (slice != 0) return;
#pragma unroll
    for (int k = 0; k < KS - 1; ++k)
#pragma unroll
        for (int i = 0; i < 16; ++i) acc[i] += red[k][i][lane];
    if constexpr (PACKED) {
        store_tile_packed((uint8_t *)out, out + (end - first) * 16, tile * kTile, first, end, true, lane,
                          [&](int r) { return (uint32_t)acc[r]; });
        return;
    }
    store_tile_rows(out, sh_out, tile * kTile, first, end, true, lane,
                    [&](int r) { return (uint16_t)(uint32_t)acc[r]; }, sig.done != nullptr);
    if (sig.done) {  // wave 0 stored the workgroup's rows: once they are performed, take the ticket
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        if (lane == 0) signal_done_last(sig);
    }
}

// Tiles per wave for a range of `ntiles` tiles: `big`, unless that leaves fewer waves
// than the chip holds at two workgroups per CU — then one, for 8x / 4x / 2x the waves
// (a participant-sized chunk of 20k records is only 625 tiles).  IRIS_TILES_PER_WAVE=1|4
// pins the small or the big variant (tests run both).
static int tiles_per_wave(const Hooks &h, uint64_t ntiles, int big) {
    if (h.tiles_per_wave) return h.tiles_per_wave == 1 ? 1 : big;
    return ntiles / big < (uint64_t)resident_blocks(2) * kWaveSlots ? 1 : big;
}

int launch_masks_mfma(const Hooks &h, void *stream, const void *db, const void *qfrag, LaunchRange r, uint16_t *out,
                      DoneSignal *sig, bool packed) {
    if (sig) sig->armed = false;
    if (r.n == 0) return 0;
    const uint64_t ntiles = tiles_of(r, 1).ntiles;
    // the K-split form for small ranges (IRIS_TILES_PER_WAVE pins the persistent kernel for tests)
    if (ntiles <= kMasksSplitTiles && !h.tiles_per_wave) {
        DoneSignal s{};
        if (sig && !packed) {
            s = *sig;
            sig->armed = true;
        }
        auto kern = packed ? masks_split_kernel<kMasksSplitKS, true> : masks_split_kernel<kMasksSplitKS>;
        hipLaunchKernelGGL(kern, dim3((uint32_t)ntiles), dim3(64 * kMasksSplitKS), 0, (hipStream_t)stream,
                           (const uint4 *)db, (const uint4 *)qfrag, tiles_of(r, 1).tile0, r.first, r.first + r.n, out, s);
        return hipGetLastError() == hipSuccess ? 0 : -1;
    }
    const int tpw = tiles_per_wave(h, ntiles, kMasksTiles);
    const Tiles t = tiles_of(r, tpw);
    const uint64_t grid = std::min<uint64_t>(t.grid, resident_blocks(kMasksBlocksPerCu));
    auto kern = packed ? (tpw == 1 ? masks_mfma_kernel<MASKS_PACKED, 1> : masks_mfma_kernel<MASKS_PACKED>)
                       : (tpw == 1 ? masks_mfma_kernel<MASKS_OUT, 1> : masks_mfma_kernel<MASKS_OUT>);
    hipLaunchKernelGGL(kern, dim3((uint32_t)grid), dim3(256), 0, (hipStream_t)stream,
                       (const uint4 *)db, (const uint4 *)qfrag, t.tile0, t.ntiles, r.first, r.first + r.n, out,
                       MaskResolve{});
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

uint32_t masks_resolve_partials(const Hooks &h, LaunchRange r) {
    const Tiles t = tiles_of(r, tiles_per_wave(h, tiles_of(r, 1).ntiles, kResolveTiles));
    return (uint32_t)std::min<uint64_t>(t.grid, resident_blocks(masks_blocks_per_cu<MASKS_RESOLVE>()));
}

int launch_masks_resolve(const Hooks &h, void *stream, const void *db, const void *qfrag, LaunchRange r,
                         const uint16_t *const *shares, uint32_t parts, double *dist_out, Partial *partials) {
    if (r.n == 0) return 0;
    if (parts == 0 || parts > 8) return -1;
    const int tpw = tiles_per_wave(h, tiles_of(r, 1).ntiles, kResolveTiles);
    const Tiles t = tiles_of(r, tpw);
    const uint64_t grid = masks_resolve_partials(h, r);
    MaskResolve rs{};
    rs.aligned = true;
    for (uint32_t p = 0; p < parts; ++p) {
        rs.shares[p] = shares[p];
        rs.aligned &= ((uintptr_t)shares[p] & 15) == 0;
    }
    rs.parts = parts;
    rs.dist_out = dist_out;
    rs.partials = partials;
    auto kern = tpw == 1 ? masks_mfma_kernel<MASKS_RESOLVE, 1> : masks_mfma_kernel<MASKS_RESOLVE>;
    hipLaunchKernelGGL(kern, dim3((uint32_t)grid), dim3(256), 0, (hipStream_t)stream,
                       (const uint4 *)db, (const uint4 *)qfrag, t.tile0, t.ntiles, r.first, r.first + r.n,
                       (uint16_t *)nullptr, rs);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

// ------------------------------------------------------------------ shares (i8)

__device__ __forceinline__ v16i mfma_i8(const uint4 &a, const uint4 &b, const v16i &c) {
    const v4i av = {(int)a.x, (int)a.y, (int)a.z, (int)a.w};
    const v4i bv = {(int)b.x, (int)b.y, (int)b.z, (int)b.w};
    return __builtin_amdgcn_mfma_i32_32x32x32_i8(av, bv, c, 0, 0, 0);
}

template <int T = kSharesTiles>
__global__ void __launch_bounds__(256, 2)
    shares_mfma_kernel(const uint4 *__restrict__ db, const uint4 *__restrict__ qfrag, const int2 *__restrict__ qsum,
                       uint64_t tile0, uint64_t ntiles, uint64_t first, uint64_t end, uint16_t *__restrict__ out) {
    const int lane = threadIdx.x & 63;
    const uint64_t wave = (uint64_t)blockIdx.x * kWaveSlots + (threadIdx.x >> 6);
    constexpr int kSteps = kShareChunks / 2;  // steps of 2 chunks
    constexpr int g0 = 0;
    const uint64_t tw = wave * T;
    if (tw >= ntiles) return;
    v16i s1[T], s2[T];
#pragma unroll
    for (int t = 0; t < T; ++t)
#pragma unroll
        for (int i = 0; i < 16; ++i) {
            s1[t][i] = 0;
            s2[t][i] = 0;
        }
    const uint4 *dp[T];
#pragma unroll
    for (int t = 0; t < T; ++t) {
        const uint64_t rel = (tw + t < ntiles) ? tw + t : ntiles - 1;
        dp[t] = db + (tile0 + rel) * (uint64_t)kShareTileUint4 + lane;
    }
    const uint4 *qp = qfrag + lane;  // chunk c: lo [(2c) * 64 + lane], hi [(2c+1) * 64 + lane]
    struct Stage {
        uint4 lo[T][2], hi[T][2];
        uint4 qlo[2], qhi[2];
    };
    auto load = [&](Stage &st, int g) {
        g = g0 + (g < kSteps ? g : kSteps - 1);
#pragma unroll
        for (int i = 0; i < 2; ++i) {
            const int c = 2 * g + i;
#pragma unroll
            for (int t = 0; t < T; ++t) {
                st.lo[t][i] = nt_load(dp[t] + (2 * c) * 64);
                st.hi[t][i] = nt_load(dp[t] + (2 * c + 1) * 64);
            }
            st.qlo[i] = qp[(2 * c) * 64];
            st.qhi[i] = qp[(2 * c + 1) * 64];
        }
        __builtin_amdgcn_sched_barrier(0);
    };
    auto compute = [&](const Stage &st) {
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
            for (int t = 0; t < T; ++t) {
                s1[t] = mfma_i8(st.qlo[i], st.lo[t][i], s1[t]);
                s2[t] = mfma_i8(st.qlo[i], st.hi[t][i], s2[t]);
                s2[t] = mfma_i8(st.qhi[i], st.lo[t][i], s2[t]);
            }
    };
    Stage sa, sb, sc;
    load(sa, 0);
    load(sb, 1);
    int g = 0;
#pragma unroll 1
    for (; g + 3 <= kSteps; g += 3) {
        load(sc, g + 2);
        compute(sa);
        load(sa, g + 3);
        compute(sb);
        load(sb, g + 4);
        compute(sc);
    }
    // kSteps = 3q + {0, 1, 2} (200 = 66 * 3 + 2)
    if (g < kSteps) compute(sa);
    if (g + 1 < kSteps) compute(sb);

    // row 31 (lane t + 32, register 15) holds sum e'_lo in S1 and sum e'_hi + sum e'_lo in S2
    const int h = lane >> 5;
    const int src = (lane & 31) + 32;
    __shared__ __attribute__((aligned(16))) uint16_t sh_out[kWaveSlots][1024];
    uint16_t *lds = sh_out[threadIdx.x >> 6];
#pragma unroll
    for (int t = 0; t < T; ++t) {
        const int elo = __shfl(s1[t][15], src);
        const int ehi = __shfl(s2[t][15], src) - elo;
        store_tile_rows(out, lds, (tile0 + tw + t) * kTile, first, end, tw + t < ntiles, lane, [&](int r) {
            const int k = (r & 3) + 8 * (r >> 2) + 4 * h;
            const int2 qs = qsum[k < kRot ? k : 0];  // (sum q'_lo, sum q'_hi) of row k
            // the 16384 * K terms vanish mod 2^16 (K = 12800)
            const uint32_t lo = (uint32_t)s1[t][r] + 128u * (uint32_t)elo + 128u * (uint32_t)qs.x;
            const uint32_t cross = (uint32_t)s2[t][r] + 128u * (uint32_t)ehi + 128u * (uint32_t)qs.x +
                                   128u * (uint32_t)elo + 128u * (uint32_t)qs.y;
            return (uint16_t)(lo + 256u * cross);
        });
    }
}

// Small ranges (the participant's 20 000-record chunks, src/main.rs:427-431): a workgroup of
// KS waves owns T tiles and wave w sums K-slice w (kShareChunks / 2 / KS steps of 2 chunks);
// the slices' i32 sums meet in LDS (exact mod 2^16 like every partial here) and wave 0 writes
// the tiles' rows -- no workspace round trip through HBM and no second (combine) launch, and
// each query-fragment load (L2) feeds T tiles.
// shapes measured at 20k shares (one box, interleaved, profiles/r03_shares_split.txt): KS = 2 waves x
// 1 tile 99 us per kernel, KS = 4: 102 us, KS = 8: 103 us, KS = 4 x 2 tiles: 108 us; the round-2
// form (up to 10 slices through an HBM workspace + a combine launch) 109 + 4 us
constexpr int kSharesSplitT = 1;
constexpr int kSharesSplitKS = 2;
constexpr uint64_t kSharesSplitTiles = 4096;

template <int T, int KS>
__global__ void __launch_bounds__(64 * KS, 2)
    shares_split_kernel(const uint4 *__restrict__ db, const uint4 *__restrict__ qfrag, const int2 *__restrict__ qsum,
                        uint64_t tile0, uint64_t ntiles, uint64_t first, uint64_t end, uint16_t *__restrict__ out,
                        DoneSignal sig) {
    constexpr int kSteps = kShareChunks / 2 / KS;
    static_assert(kShareChunks % (2 * KS) == 0, "K-split geometry");
    const int lane = threadIdx.x & 63;
    const int slice = threadIdx.x >> 6;
    const uint64_t tw = (uint64_t)blockIdx.x * T;
    const int g0 = slice * kSteps;
    v16i s1[T], s2[T];
#pragma unroll
    for (int t = 0; t < T; ++t)
#pragma unroll
        for (int i = 0; i < 16; ++i) {
            s1[t][i] = 0;
            s2[t][i] = 0;
        }
    const uint4 *dp[T];
#pragma unroll
    for (int t = 0; t < T; ++t) {
        const uint64_t rel = (tw + t < ntiles) ? tw + t : ntiles - 1;
        dp[t] = db + (tile0 + rel) * (uint64_t)kShareTileUint4 + lane;
    }
    const uint4 *qp = qfrag + lane;
    struct Stage {
        uint4 lo[T][2], hi[T][2];
        uint4 qlo[2], qhi[2];
    };
    auto load = [&](Stage &st, int g) {
        g = g0 + (g < kSteps ? g : kSteps - 1);
#pragma unroll
        for (int i = 0; i < 2; ++i) {
            const int c = 2 * g + i;
#pragma unroll
            for (int t = 0; t < T; ++t) {
                st.lo[t][i] = nt_load(dp[t] + (2 * c) * 64);
                st.hi[t][i] = nt_load(dp[t] + (2 * c + 1) * 64);
            }
            st.qlo[i] = qp[(2 * c) * 64];
            st.qhi[i] = qp[(2 * c + 1) * 64];
        }
        __builtin_amdgcn_sched_barrier(0);
    };
    auto compute = [&](const Stage &st) {
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
            for (int t = 0; t < T; ++t) {
                s1[t] = mfma_i8(st.qlo[i], st.lo[t][i], s1[t]);
                s2[t] = mfma_i8(st.qlo[i], st.hi[t][i], s2[t]);
                s2[t] = mfma_i8(st.qhi[i], st.lo[t][i], s2[t]);
            }
    };
    Stage sa, sb, sc;
    load(sa, 0);
    load(sb, 1);
    int g = 0;
#pragma unroll 1
    for (; g + 3 <= kSteps; g += 3) {
        load(sc, g + 2);
        compute(sa);
        load(sa, g + 3);
        compute(sb);
        load(sb, g + 4);
        compute(sc);
    }
    if (g < kSteps) compute(sa);
    if (g + 1 < kSteps) compute(sb);

    __shared__ int red[KS - 1][T][2][16][64];
    __shared__ __attribute__((aligned(16))) uint16_t sh_out[1024];
    if (slice != 0) {
#pragma unroll
        for (int t = 0; t < T; ++t)
#pragma unroll
            for (int i = 0; i < 16; ++i) {
                red[slice - 1][t][0][i][lane] = s1[t][i];
                red[slice - 1][t][1][i][lane] = s2[t][i];
            }
    }
    __syncthreads();
    if (slice != 0) return;
#pragma unroll
    for (int k = 0; k < KS - 1; ++k)
#pragma unroll
        for (int t = 0; t < T; ++t)
#pragma unroll
            for (int i = 0; i < 16; ++i) {
                s1[t][i] += red[k][t][0][i][lane];
                s2[t][i] += red[k][t][1][i][lane];
            }
    // row 31 (lane t + 32, register 15) holds sum e'_lo in S1 and sum e'_hi + sum e'_lo in S2
    const int h = lane >> 5;
    const int src = (lane & 31) + 32;
#pragma unroll
    for (int t = 0; t < T; ++t) {
        const int elo = __shfl(s1[t][15], src);
        const int ehi = __shfl(s2[t][15], src) - elo;
        store_tile_rows(out, sh_out, (tile0 + tw + t) * kTile, first, end, tw + t < ntiles, lane, [&](int r) {
            const int k = (r & 3) + 8 * (r >> 2) + 4 * h;
            const int2 qs = qsum[k < kRot ? k : 0];  // (sum q'_lo, sum q'_hi) of row k
            const uint32_t lo = (uint32_t)s1[t][r] + 128u * (uint32_t)elo + 128u * (uint32_t)qs.x;
            const uint32_t cross = (uint32_t)s2[t][r] + 128u * (uint32_t)ehi + 128u * (uint32_t)qs.x +
                                   128u * (uint32_t)elo + 128u * (uint32_t)qs.y;
            return (uint16_t)(lo + 256u * cross);
        }, sig.done != nullptr);
    }
    if (sig.done) {  // wave 0 stored the workgroup's rows: once they are performed, take the ticket
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        if (lane == 0) signal_done_last(sig);
    }
}

// K-slices for a range (1 = no split): enough one-tile waves to fill the chip, a
// divisor of the 200 steps, at most 10.
static bool shares_lds_split(const Hooks &h, uint64_t ntiles) {
    return ntiles <= kSharesSplitTiles && !h.tiles_per_wave;
}

int launch_shares_mfma(const Hooks &h, void *stream, const void *db, const void *qfrag, LaunchRange r, uint16_t *out,
                       DoneSignal *sig) {
    if (sig) sig->armed = false;
    if (r.n == 0) return 0;
    const int2 *qsum = (const int2 *)((const uint4 *)qfrag + kShareFragUint4);
    if (shares_lds_split(h, tiles_of(r, 1).ntiles)) {
        const Tiles t = tiles_of(r, 1);
        DoneSignal s{};
        if (sig) {
            s = *sig;
            sig->armed = true;
        }
        hipLaunchKernelGGL((shares_split_kernel<kSharesSplitT, kSharesSplitKS>),
                           dim3((uint32_t)((t.ntiles + kSharesSplitT - 1) / kSharesSplitT)), dim3(64 * kSharesSplitKS), 0,
                           (hipStream_t)stream, (const uint4 *)db, (const uint4 *)qfrag, qsum, t.tile0, t.ntiles, r.first,
                           r.first + r.n, out, s);
        return hipGetLastError() == hipSuccess ? 0 : -1;
    }
    const int tpw = tiles_per_wave(h, tiles_of(r, 1).ntiles, kSharesTiles);
    const Tiles t = tiles_of(r, tpw);
    auto kern = tpw == 1 ? shares_mfma_kernel<1> : shares_mfma_kernel<>;
    hipLaunchKernelGGL(kern, dim3((uint32_t)t.grid), dim3(256), 0, (hipStream_t)stream, (const uint4 *)db,
                       (const uint4 *)qfrag, qsum, t.tile0, t.ntiles, r.first, r.first + r.n, out);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

// ------------------------------------------------------------------ TILES plumbing (masks, shares)

// masks: thread per (record, step g, half h): mask dwords {8g+h, 8g+2+h, 8g+4+h, 8g+6+h}
__global__ void __launch_bounds__(256) pack_masks_tiles(const uint32_t *__restrict__ staging, uint4 *__restrict__ db,
                                                        uint64_t t_first, uint64_t n, int inverse) {
    const uint64_t total = n * (uint64_t)(2 * (kMaskChunks / 4));
    for (uint64_t tid = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; tid < total;
         tid += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t i = tid % n, gh = tid / n;
        const int g = (int)(gh >> 1), h = (int)(gh & 1);
        const uint64_t t = t_first + i;
        uint4 *dst = db + (t / kTile) * (uint64_t)kMaskTileUint4 + (uint64_t)g * 64 + (t % kTile) + 32 * h;
        uint32_t *rec = (uint32_t *)staging + i * kPlaneDwords;
        const int w = 8 * g + h;
        if (!inverse) {
            *dst = make_uint4(rec[w], rec[w + 2], rec[w + 4], rec[w + 6]);
        } else {
            const uint4 v = *dst;
            rec[w] = v.x;
            rec[w + 2] = v.y;
            rec[w + 4] = v.z;
            rec[w + 6] = v.w;
        }
    }
}

__global__ void __launch_bounds__(256) generate_masks_tiles(uint4 *__restrict__ db, uint64_t t_first, uint64_t n,
                                                            uint64_t key, uint64_t global_index0) {
    const uint64_t total = n * (uint64_t)(2 * (kMaskChunks / 4));
    for (uint64_t tid = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; tid < total;
         tid += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t i = tid % n, gh = tid / n;
        const int g = (int)(gh >> 1), h = (int)(gh & 1);
        const uint64_t gt = global_index0 + i, t = t_first + i;
        uint32_t v[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) v[q] = (uint32_t)(gen_limb(key, gt * 400 + 200 + 4 * g + q) >> (32 * h));
        db[(t / kTile) * (uint64_t)kMaskTileUint4 + (uint64_t)g * 64 + (t % kTile) + 32 * h] =
            make_uint4(v[0], v[1], v[2], v[3]);
    }
}

// shares: thread per (record, chunk c, half h): elements 32c + 16h .. +15 -> lo / hi byte planes ^ 0x80
__device__ __forceinline__ void join_bytes(const uint4 &lo_, const uint4 &hi_, uint32_t *dst8) {
    const uint32_t lo[4] = {lo_.x ^ 0x80808080u, lo_.y ^ 0x80808080u, lo_.z ^ 0x80808080u, lo_.w ^ 0x80808080u};
    const uint32_t hi[4] = {hi_.x ^ 0x80808080u, hi_.y ^ 0x80808080u, hi_.z ^ 0x80808080u, hi_.w ^ 0x80808080u};
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        dst8[2 * q] = (lo[q] & 0xFFu) | ((hi[q] & 0xFFu) << 8) | ((lo[q] & 0xFF00u) << 8) | ((hi[q] & 0xFF00u) << 16);
        dst8[2 * q + 1] = ((lo[q] >> 16) & 0xFFu) | ((hi[q] >> 8) & 0xFF00u) | ((lo[q] >> 8) & 0xFF0000u) |
                          (hi[q] & 0xFF000000u);
    }
}

__global__ void __launch_bounds__(256) pack_shares_tiles(const uint32_t *__restrict__ staging, uint4 *__restrict__ db,
                                                         uint64_t t_first, uint64_t n, int inverse) {
    const uint64_t total = n * (uint64_t)(2 * kShareChunks);
    for (uint64_t tid = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; tid < total;
         tid += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t i = tid % n, ch = tid / n;
        const int c = (int)(ch >> 1), h = (int)(ch & 1);
        const uint64_t t = t_first + i;
        uint4 *base = db + (t / kTile) * (uint64_t)kShareTileUint4 + (t % kTile) + 32 * h;
        uint32_t *rec = (uint32_t *)staging + i * kShareDwords + (32 * c + 16 * h) / 2;
        if (!inverse) {
            uint4 lo, hi;
            split_bytes(rec, lo, hi);
            base[(2 * c) * 64] = lo;
            base[(2 * c + 1) * 64] = hi;
        } else {
            join_bytes(base[(2 * c) * 64], base[(2 * c + 1) * 64], rec);
        }
    }
}

__global__ void __launch_bounds__(256) generate_shares_tiles(uint4 *__restrict__ db, uint64_t t_first, uint64_t n,
                                                             uint64_t key, uint64_t global_index0) {
    const uint64_t total = n * (uint64_t)(2 * kShareChunks);
    for (uint64_t tid = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; tid < total;
         tid += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t i = tid % n, ch = tid / n;
        const int c = (int)(ch >> 1), h = (int)(ch & 1);
        const uint64_t gt = global_index0 + i, t = t_first + i;
        uint32_t src[8];
#pragma unroll
        for (int q = 0; q < 4; ++q) {  // limbs (32c + 16h)/4 + q, 4 u16 each
            const uint64_t v = gen_limb(key, gt * 3200 + 8 * c + 4 * h + q);
            src[2 * q] = (uint32_t)v;
            src[2 * q + 1] = (uint32_t)(v >> 32);
        }
        uint4 lo, hi;
        split_bytes(src, lo, hi);
        uint4 *base = db + (t / kTile) * (uint64_t)kShareTileUint4 + (t % kTile) + 32 * h;
        base[(2 * c) * 64] = lo;
        base[(2 * c + 1) * 64] = hi;
    }
}

static int plumb_grid(uint64_t total) {
    uint64_t b = (total + 255) / 256;
    if (b > 256ull * 64) b = 256ull * 64;
    return (int)(b ? b : 1);
}

int launch_pack_tiles_kind(void *stream, int kind, const void *staging, void *db, uint64_t t_first, uint64_t n) {
    if (n == 0) return 0;
    hipStream_t s = (hipStream_t)stream;
    if (kind == IRIS_KIND_TEMPLATES) return launch_pack_tiles(stream, staging, db, t_first, n);
    if (kind == IRIS_KIND_MASKS)
        hipLaunchKernelGGL(pack_masks_tiles, dim3(plumb_grid(n * kMaskChunks / 2)), dim3(256), 0, s,
                           (const uint32_t *)staging, (uint4 *)db, t_first, n, 0);
    else
        hipLaunchKernelGGL(pack_shares_tiles, dim3(plumb_grid(n * 2 * kShareChunks)), dim3(256), 0, s,
                           (const uint32_t *)staging, (uint4 *)db, t_first, n, 0);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

int launch_unpack_tiles_kind(void *stream, int kind, const void *db, void *staging, uint64_t t_first, uint64_t n) {
    if (n == 0) return 0;
    hipStream_t s = (hipStream_t)stream;
    if (kind == IRIS_KIND_TEMPLATES) return launch_unpack_tiles(stream, db, staging, t_first, n);
    if (kind == IRIS_KIND_MASKS)
        hipLaunchKernelGGL(pack_masks_tiles, dim3(plumb_grid(n * kMaskChunks / 2)), dim3(256), 0, s,
                           (const uint32_t *)staging, (uint4 *)db, t_first, n, 1);
    else
        hipLaunchKernelGGL(pack_shares_tiles, dim3(plumb_grid(n * 2 * kShareChunks)), dim3(256), 0, s,
                           (const uint32_t *)staging, (uint4 *)db, t_first, n, 1);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

int launch_generate_tiles_kind(void *stream, int kind, void *db, uint64_t t_first, uint64_t n, uint64_t seed,
                               uint64_t global_index0) {
    if (n == 0) return 0;
    hipStream_t s = (hipStream_t)stream;
    if (kind == IRIS_KIND_TEMPLATES) return launch_generate_tiles(stream, db, t_first, n, seed, global_index0);
    if (kind == IRIS_KIND_MASKS)
        hipLaunchKernelGGL(generate_masks_tiles, dim3(plumb_grid(n * kMaskChunks / 2)), dim3(256), 0, s, (uint4 *)db,
                           t_first, n, gen_key(seed, 0), global_index0);
    else
        hipLaunchKernelGGL(generate_shares_tiles, dim3(plumb_grid(n * 2 * kShareChunks)), dim3(256), 0, s,
                           (uint4 *)db, t_first, n, gen_key(seed, 1), global_index0);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

}  // namespace iris
