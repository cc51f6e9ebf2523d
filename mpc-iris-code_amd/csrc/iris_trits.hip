// iris_trits.hip — the TRITS template layout (2560 B per template) and its
// fp4 MFMA search / counts kernel.
//
// Why: the TILES search kernel (iris_mfma.hip) reads its 3200 B per template at
// the read bandwidth its occupancy allows, so the next gain has to come from
// reading fewer bytes.  A template position only ever contributes through
// em and ep & em: num = popcount((qp ^ ep) & qm & em), den = popcount(qm & em)
// (src/template.rs:49-64), and encode() maps a position to 0 / +1 / -1
// (src/lib.rs:16-26).  The pattern bit under a zero mask is never read, so a
// position is one of three states and five of them fit one byte (3^5 = 243):
// 12800 positions in 2560 B, 20 % fewer HBM bytes than TILES.
//
// Decode: a 243-entry table maps a byte to the fp4 e2m1 encode() values of its
// five positions (T_w: nibble i = digit i; T_s = T_w << 4, nibbles 1..5).  The
// tables live in LDS in 32 copies each, one 256-B bank row per entry: T_w at
// dwords 0..31 and T_s at dwords 32..63 of row e, lane l reading copy l & 31.
// ds_read_b32 banks are (address / 4) mod 32 per 32-lane half, so the 32 lanes of
// a half always hit 32 distinct banks (no conflict whatever the data), and both
// tables share the address: one v_perm_b32 (byte 1 = the data byte, byte 0 =
// 4 * (lane & 31)), T_s through the instruction's offset field.
//
// Byte roles: every 8 bytes (40 positions) decode to five stream dwords.  Bytes
// 0..3 (W_j, read from T_w) fill nibbles 0..4 of dword j; bytes 4..7 (S_j, read
// from T_s) put digits 0..2 in nibbles 5..7 of dword j and digits 3, 4 in
// nibbles 2j, 2j+1 of dword 4:  dword j = (s_j << 16) | w_j (one v_lshl_or_b32:
// the shift drops digits 3, 4) and dword 4 = byte 2 of s_0..s_3 (two v_perm_b32
// and an or) -- 7 VALU per 8 bytes.  The den operand is the same nibbles
// & 0x22222222 (|enc| = 1.0).
//
// K order: the MFMA sums over K, so any bijection between a lane's fp4 slots
// and template positions works as long as the query fragments use the same
// one.  Lane L = t + 32h of a tile owns positions [320G + 160h, +160) of its
// template in 5-chunk group G, as one 160-nibble stream; chunk c of the group
// is nibbles [32c, 32c + 32) = plane dword 10G + 5h + c of both operands
// (iris_internal.hpp: kTritTileUint4, trit_pos, TRITS fragments).
#include <hip/hip_runtime.h>
#include <stdlib.h>

#include <type_traits>

#include "iris_device.hpp"

namespace iris {

namespace {

typedef int v8i __attribute__((ext_vector_type(8)));
typedef float v16f __attribute__((ext_vector_type(16)));
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

constexpr int kTileRecs = 32;
constexpr int kLutStride = 64;  // dwords per table entry: T_w copies 0..31, T_s copies 32..63 (one 256-B bank row)
constexpr int kLutStage = 252 * kLutStride;  // dword offset of the staged 256-entry constant
constexpr int kHalfStages = 2 * kTritGroups;  // 80 uint4 per lane and template
#ifndef IRIS_TRITS_TILES
#define IRIS_TRITS_TILES 2
#endif
constexpr int kTritTiles = IRIS_TRITS_TILES;  // tiles per wave
// VALU per step (T = 2: 80 decode + 8 / 12 query-operand ands), spread over the step's MFMAs
#ifndef IRIS_TRITS_NV_ODD
#define IRIS_TRITS_NV_ODD 88
#endif
#ifndef IRIS_TRITS_NV_EVEN
#define IRIS_TRITS_NV_EVEN 92
#endif

// the decode table, computed at compile time (filling LDS from it costs one load + one
// store per entry instead of ~35 VALU of base-3 arithmetic)
struct TritLut {
    uint32_t v[256];
    constexpr TritLut() : v() {
        for (int b = 0; b < 256; ++b) {
            uint32_t x = 0, r = (uint32_t)b;
            for (int i = 0; i < 5; ++i) {
                const uint32_t d = r % 3;
                r /= 3;
                x |= (d == 0 ? 0u : d == 1 ? 0x2u : 0xAu) << (4 * i);
            }
            v[b] = b < 243 ? x : 0u;
        }
    }
};
__constant__ constexpr TritLut kTritLut{};

__device__ __forceinline__ v16f mfma_fp4(const v8i &a, const v8i &b, const v16f &c) {
    // cbsz = blgp = 4: both operands e2m1; scales 127 = 2^0 (e8m0)
    return __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(a, b, c, 4, 4, 0, 127, 0, 127);
}

__device__ __forceinline__ uint4 stream_load(const uint4 *p) {
    const u32x4 v = __builtin_nontemporal_load((const u32x4 *)p);
    return make_uint4(v.x, v.y, v.z, v.w);
}

// one 64-position chunk of one tile: B = the decoded nibbles, A = the query fragment
__device__ __forceinline__ void tchunk(uint32_t b0, uint32_t b1, uint32_t b2, uint32_t b3, const v8i &am,
                                       const v8i &ae, v16f &den, v16f &s) {
    const v8i be = {(int)b0, (int)b1, (int)b2, (int)b3, 0, 0, 0, 0};
    const v8i bm = {(int)(b0 & 0x22222222u), (int)(b1 & 0x22222222u), (int)(b2 & 0x22222222u),
                    (int)(b3 & 0x22222222u), 0, 0, 0, 0};
#ifndef IRIS_TRITS_DIAG
#define IRIS_TRITS_DIAG 0
#endif
    // diagnostic builds only (tools/, results wrong by design): 1 = no den MFMA, 2 = no MFMAs
    // (operands kept live by an empty asm)
    if constexpr (IRIS_TRITS_DIAG == 0) {
        den = mfma_fp4(am, bm, den);
        s = mfma_fp4(ae, be, s);
    } else if constexpr (IRIS_TRITS_DIAG == 1) {
        asm volatile("" ::"v"(bm), "v"(am));
        s = mfma_fp4(ae, be, s);
    } else {
        asm volatile("" ::"v"(bm), "v"(be), "v"(am), "v"(ae));
    }
}

// (a << s) | b as one instruction (hipcc would otherwise emit a shift and a v_or / v_bitop3)
template <int S>
__device__ __forceinline__ uint32_t lshl_or_i(uint32_t a, uint32_t b) {
    uint32_t r;
    asm("v_lshl_or_b32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "I"(S), "v"(b));
    return r;
}
#define lshl_or(a, s, b) lshl_or_i<s>((a), (b))

struct QF {
    v8i am, ae;
};
__device__ __forceinline__ QF qf_of(uint32_t x, uint32_t y, uint32_t z, uint32_t w) {
    QF f;
    f.ae = v8i{(int)x, (int)y, (int)z, (int)w, 0, 0, 0, 0};
    f.am = v8i{(int)(x & 0x22222222u), (int)(y & 0x22222222u), (int)(z & 0x22222222u), (int)(w & 0x22222222u),
               0, 0, 0, 0};
    return f;
}

}  // namespace

enum { TR_COUNTS = 0, TR_SEARCH = 1 };

// Grid: one wave per T tiles, 4 waves per workgroup, 2 workgroups per CU (the
// 64-KB table each).  Per lane and tile the template streams as 80 uint4
// half-stages; half-stage 2G decodes to chunks 5G, 5G+1 and the first half of
// chunk 5G+2, half-stage 2G+1 to the rest of 5G+2, 5G+3, 5G+4 (the query
// fragment of chunk 5G+2 is loaded as two uint2 halves the same way).  Three
// stage buffers: the loads of half-stage i+2 are in flight while i computes.
template <int MODE, int T>
__global__ void __launch_bounds__(256, 2)
    trits_mfma_kernel(const uint4 *__restrict__ db, const uint4 *__restrict__ qfrag, uint64_t tile0, uint64_t ntiles,
                      uint64_t first, uint64_t end, uint16_t *__restrict__ num_out, uint16_t *__restrict__ den_out,
                      double *__restrict__ dist_out, Partial *__restrict__ partials) {
    // the table: the 1-KB constant staged through rows 252..255 (never read: bytes are < 243),
    // one global load per thread, then rows 0..242 written from LDS (a wave reads one row:
    // broadcast; writes consecutive dwords: conflict-free)
    __shared__ __attribute__((aligned(16))) uint32_t lut[256 * kLutStride];  // also the 16-B store staging of the epilogue
    lut[kLutStage + threadIdx.x] = kTritLut.v[threadIdx.x];
    __syncthreads();
    for (int i = threadIdx.x; i < 243 * kLutStride; i += 256) lut[i] = lut[kLutStage + (i >> 6)] << ((i & 32) >> 3);
    __syncthreads();

    const int lane = threadIdx.x & 63;
    const int wslot = threadIdx.x >> 6;
    const uint64_t wave = (uint64_t)blockIdx.x * kWaveSlots + wslot;
    const uint64_t tw = wave * T;
    const bool active = tw < ntiles;  // wave-uniform

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
        const uint32_t laneoff = (uint32_t)(lane & 31) * 4u;
        const char *lutb = (const char *)lut;
        // table entries of the 16 bytes of v for this lane's copy (16 ds_read_b32): dwords 0, 2
        // hold W bytes (T_w), dwords 1, 3 S bytes (T_s, 128 B further in the row)
        auto lookups = [&](const uint4 &v, uint32_t *e) {
            const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
            for (int i = 0; i < 16; ++i)
                e[i] = *(const uint32_t *)(lutb + ((i >> 2) & 1) * 128 +
                                           __builtin_amdgcn_perm(w[i >> 2], laneoff, 0x0C0C0400u + ((i & 3) << 8)));
        };
        // 16 entries (80 nibbles) -> 10 stream dwords: 8 entries -> 5 dwords, twice, in 7 VALU each
        auto combine = [&](const uint32_t *e, uint32_t *d) {
#pragma unroll
            for (int q = 0; q < 2; ++q) {
                const uint32_t *w = e + 8 * q, *t = e + 8 * q + 4;
                uint32_t *o = d + 5 * q;
#pragma unroll
                for (int j = 0; j < 4; ++j) o[j] = lshl_or(t[j], 16, w[j]);
                o[4] = __builtin_amdgcn_perm(t[1], t[0], 0x0C0C0602u) | __builtin_amdgcn_perm(t[3], t[2], 0x06020C0Cu);
            }
        };

        const uint4 *dp[T];
#pragma unroll
        for (int t = 0; t < T; ++t) {
            const uint64_t rel = (tw + t < ntiles) ? tw + t : ntiles - 1;  // clamp: extra tiles re-read a valid one
            dp[t] = db + (tile0 + rel) * (uint64_t)kTritTileUint4 + lane;
        }
        const uint4 *qp = qfrag + lane;  // chunk C: qfrag[C * 64 + lane]
        struct Stage {
            uint4 d[T];
            uint4 qa, qb;  // even: chunks 5G, 5G+1; odd: 5G+3, 5G+4
            uint2 qc;      // even: first half of chunk 5G+2; odd: second half
        };
        struct QS {
            uint4 qa, qb;
            uint2 qc;
        };
        auto load = [&](Stage &st, int hs, auto odd) {  // hs: half-stage 0..79, odd = its parity (static)
            hs = hs < kHalfStages ? hs : kHalfStages - 1;
            const int G = hs >> 1;
#pragma unroll
            for (int t = 0; t < T; ++t) st.d[t] = stream_load(dp[t] + hs * 64);
            const uint2 *c2 = (const uint2 *)(qp + (5 * G + 2) * 64);
            if constexpr (!decltype(odd)::value) {
                st.qa = qp[(5 * G) * 64];
                st.qb = qp[(5 * G + 1) * 64];
                st.qc = c2[0];
            } else {
                st.qc = c2[1];
                st.qa = qp[(5 * G + 3) * 64];
                st.qb = qp[(5 * G + 4) * 64];
            }
            // loads of one stage stay together, ahead of the compute that follows (vmcnt
            // retires in order: a query load sunk to its use would drain the prefetches)
            __builtin_amdgcn_sched_barrier(0);
        };

        // Software pipeline over half-stages: step(i) decodes half-stage i (table reads +
        // combine, VALU/LDS) while the MFMAs of half-stage i-1 run, so one wave keeps the
        // matrix pipe and the VALU busy together; the MFMAs go chunk-major over the tiles
        // (a dependent accumulation is 2T instructions apart).
        uint32_t dv[2][T][10];  // decoded stream dwords of the last even [0] / odd [1] half-stage
        QS qs[2];
        uint2 carry_b[T];       // even half-stage's dwords 8, 9: first half of chunk 5G+2
        uint2 carry_q;
        auto decode = [&](const Stage &st, uint32_t (&d)[T][10]) {
            uint32_t e[2][16];
            lookups(st.d[0], e[0]);
#pragma unroll
            for (int t = 0; t < T; ++t) {
                if (t + 1 < T) lookups(st.d[t + 1], e[(t + 1) & 1]);  // in flight during this combine
                combine(e[t & 1], d[t]);
            }
        };
        auto mfmas = [&](auto odd) {  // the MFMAs of the last decoded half-stage of this parity
            constexpr bool O = decltype(odd)::value;
            const uint32_t(&d)[T][10] = dv[O];
            const QS &q = qs[O];
            if constexpr (!O) {
                const QF f0 = qf_of(q.qa.x, q.qa.y, q.qa.z, q.qa.w);
#pragma unroll
                for (int t = 0; t < T; ++t) tchunk(d[t][0], d[t][1], d[t][2], d[t][3], f0.am, f0.ae, den[t], s[t]);
                const QF f1 = qf_of(q.qb.x, q.qb.y, q.qb.z, q.qb.w);
#pragma unroll
                for (int t = 0; t < T; ++t) tchunk(d[t][4], d[t][5], d[t][6], d[t][7], f1.am, f1.ae, den[t], s[t]);
#pragma unroll
                for (int t = 0; t < T; ++t) carry_b[t] = make_uint2(d[t][8], d[t][9]);
                carry_q = q.qc;
            } else {
                const QF f2 = qf_of(carry_q.x, carry_q.y, q.qc.x, q.qc.y);
#pragma unroll
                for (int t = 0; t < T; ++t) tchunk(carry_b[t].x, carry_b[t].y, d[t][0], d[t][1], f2.am, f2.ae, den[t], s[t]);
                const QF f3 = qf_of(q.qa.x, q.qa.y, q.qa.z, q.qa.w);
#pragma unroll
                for (int t = 0; t < T; ++t) tchunk(d[t][2], d[t][3], d[t][4], d[t][5], f3.am, f3.ae, den[t], s[t]);
                const QF f4 = qf_of(q.qb.x, q.qb.y, q.qb.z, q.qb.w);
#pragma unroll
                for (int t = 0; t < T; ++t) tchunk(d[t][6], d[t][7], d[t][8], d[t][9], f4.am, f4.ae, den[t], s[t]);
            }
        };
        // one step: decode half-stage i (parity P) from st and run half-stage i-1's MFMAs,
        // interleaved: per MFMA ~9 VALU and ~3 table reads of the decode
        auto step = [&](const Stage &st, auto odd) {
            constexpr bool P = decltype(odd)::value;
            qs[P] = QS{st.qa, st.qb, st.qc};
            decode(st, dv[P]);
            mfmas(std::integral_constant<bool, !P>{});
            constexpr int nm = (P ? 4 : 6) * T;  // MFMAs of the previous (opposite-parity) half-stage
            constexpr int nv = (P ? IRIS_TRITS_NV_ODD : IRIS_TRITS_NV_EVEN) / nm;  // the step's VALU spread evenly
#pragma unroll
            for (int k = 0; k < nm; ++k) {
                __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);   // 1 MFMA
                __builtin_amdgcn_sched_group_barrier(0x002, nv, 0);  // VALU
                __builtin_amdgcn_sched_group_barrier(0x100, 16 * T / nm + 1, 0);  // table reads
            }
            __builtin_amdgcn_sched_barrier(0);
        };
        const std::false_type even{};
        const std::true_type odd{};
        // three stage buffers: half-stage i lives in buffer i % 3; its loads are issued two
        // steps ahead (a fourth buffer, three steps ahead, measured 4 % slower: 5.32 vs
        // 5.13 ms per 10M)
        Stage sa, sb, sc;
        load(sa, 0, even);
        load(sb, 1, odd);
        load(sc, 2, even);
        qs[0] = QS{sa.qa, sa.qb, sa.qc};
        decode(sa, dv[0]);  // half-stage 0: nothing to overlap yet
        __builtin_amdgcn_sched_barrier(0);
        int hs = 1;
#pragma unroll 1
        for (; hs + 6 <= kHalfStages; hs += 6) {  // 13 rounds: half-stages 1..78
            load(sa, hs + 2, odd);
            step(sb, odd);
            load(sb, hs + 3, even);
            step(sc, even);
            load(sc, hs + 4, odd);
            step(sa, odd);
            load(sa, hs + 5, even);
            step(sb, even);
            load(sb, hs + 6, odd);
            step(sc, odd);
            load(sc, hs + 7, even);
            step(sa, even);
        }
        // kHalfStages = 80 = 1 + 13 * 6 + 1: half-stage 79 (odd, in sb) remains, then its MFMAs
        step(sb, odd);
        mfmas(odd);
    }

    // epilogue: as template_mfma_kernel's (C layout: lane l holds template l & 31,
    // rotation rows k = (r & 3) + 8 (r >> 2) + 4 (l >> 5), r = 0..15)
    const int h = lane >> 5;
    Partial best = partial_none();
#pragma unroll
    for (int t = 0; t < T; ++t) {
        const uint64_t t0 = (tile0 + tw + t) * kTileRecs;
        const bool tv = active && (tw + t < ntiles);
        if constexpr (MODE == TR_COUNTS) {
            // the table is dead by now: its first 8 KB stage the output rows
            __syncthreads();
            uint16_t *lds = (uint16_t *)lut + wslot * 1024;
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
    if constexpr (MODE == TR_SEARCH) {
#pragma unroll
        for (int off = 32; off >= 1; off >>= 1) {
            const Partial ot = partial_shfl_xor(best, off);
            if (partial_better_dev(ot, best)) best = ot;
        }
        __shared__ Partial sh[kWaveSlots];
        if (lane == 0) sh[wslot] = best;
        __syncthreads();
        if (threadIdx.x == 0) {
            Partial b = sh[0];
#pragma unroll
            for (int w = 1; w < kWaveSlots; ++w)
                if (partial_better_dev(sh[w], b)) b = sh[w];
            partials[blockIdx.x] = b;
        }
    }
}

// ------------------------------------------------------------------ layout plumbing

namespace {

// half-stage s (bytes 16s .. 16s+15) of a lane's 160-position window (m, p: its 5 plane
// dwords); byte jj holds the positions trit_pos(s, jj, 0..4)
__device__ __forceinline__ uint4 trit_half(const uint32_t *m, const uint32_t *p, int s) {
    uint32_t v[4] = {0, 0, 0, 0};
#pragma unroll
    for (int jj = 0; jj < 16; ++jj) {
        uint32_t m5 = 0, p5 = 0;
#pragma unroll
        for (int k = 0; k < 5; ++k) {
            const int x = trit_pos(s, jj, k);
            m5 |= ((m[x >> 5] >> (x & 31)) & 1u) << k;
            p5 |= ((p[x >> 5] >> (x & 31)) & 1u) << k;
        }
        v[jj >> 2] |= trit_byte(m5, p5) << (8 * (jj & 3));
    }
    return make_uint4(v[0], v[1], v[2], v[3]);
}

__device__ __forceinline__ uint64_t trit_index(uint64_t t, int G, int h, int s) {
    return (t / kTileRecs) * (uint64_t)kTritTileUint4 + (uint64_t)(2 * G + s) * 64 + (t % kTileRecs) + 32 * h;
}

}  // namespace

// thread per (record, G, h, s): reference record (pattern dwords 0..399, mask
// 400..799) -> one uint4 of the TRITS tile
__global__ void __launch_bounds__(256) pack_trits_kernel(const uint32_t *__restrict__ staging,
                                                         uint4 *__restrict__ db, uint64_t t_first, uint64_t n) {
    const uint64_t total = n * (uint64_t)(4 * kTritGroups);
    for (uint64_t tid = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; tid < total;
         tid += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t i = tid % n, q = tid / n;
        const int s = (int)(q & 1), h = (int)((q >> 1) & 1), G = (int)(q >> 2);
        const uint32_t *rec = staging + i * (2 * kPlaneDwords);
        const int w0 = 10 * G + 5 * h;
        uint32_t m[5], p[5];
#pragma unroll
        for (int k = 0; k < 5; ++k) {
            m[k] = rec[kPlaneDwords + w0 + k];
            p[k] = rec[w0 + k];
        }
        db[trit_index(t_first + i, G, h, s)] = trit_half(m, p, s);
    }
}

// thread per (record, plane dword w): mask dword and pattern & mask dword
__global__ void __launch_bounds__(256) unpack_trits_kernel(const uint4 *__restrict__ db,
                                                           uint32_t *__restrict__ staging, uint64_t t_first,
                                                           uint64_t n) {
    const uint64_t total = n * (uint64_t)kPlaneDwords;
    for (uint64_t tid = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; tid < total;
         tid += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t i = tid % n;
        const int w = (int)(tid / n);
        const int G = w / 10, r = w - 10 * G, h = r / 5, c = r % 5;
        const uint64_t t = t_first + i;
        uint32_t em = 0, ep = 0;
        for (int b = 0; b < 32; ++b) {
            int s, jj, k;
            trit_slot(32 * c + b, s, jj, k);
            const uint4 *src = db + trit_index(t, G, h, s);
            uint32_t v = ((const uint8_t *)src)[jj];
            for (; k > 0; --k) v /= 3;
            const uint32_t dgt = v % 3;
            em |= (dgt != 0 ? 1u : 0u) << b;
            ep |= (dgt == 2 ? 1u : 0u) << b;
        }
        uint32_t *rec = staging + i * (2 * kPlaneDwords);
        rec[kPlaneDwords + w] = em;
        rec[w] = ep;
    }
}

// synthetic records (DESIGN.md §5 generator) straight into the TRITS layout
__global__ void __launch_bounds__(256) generate_trits_kernel(uint4 *__restrict__ db, uint64_t t_first, uint64_t n,
                                                             uint64_t key, uint64_t global_index0) {
    const uint64_t total = n * (uint64_t)(4 * kTritGroups);
    for (uint64_t tid = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; tid < total;
         tid += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t i = tid % n, q = tid / n;
        const int s = (int)(q & 1), h = (int)((q >> 1) & 1), G = (int)(q >> 2);
        const uint64_t gt = global_index0 + i;
        const int w0 = 10 * G + 5 * h;
        uint32_t m[5], p[5];
        // plane dword W is half W & 1 of limb W >> 1 (pattern limb j = ctr t*400 + j, mask 200 + j)
#pragma unroll
        for (int k = 0; k < 5; ++k) {
            const int wd = w0 + k, half = wd & 1;
            m[k] = (uint32_t)(gen_limb(key, gt * 400 + 200 + (wd >> 1)) >> (32 * half));
            p[k] = (uint32_t)(gen_limb(key, gt * 400 + (wd >> 1)) >> (32 * half));
        }
        db[trit_index(t_first + i, G, h, s)] = trit_half(m, p, s);
    }
}

namespace {

int grid_of(uint64_t total) {
    uint64_t b = (total + 255) / 256;
    if (b > 256ull * 64) b = 256ull * 64;
    return (int)(b ? b : 1);
}

struct TritRange {
    uint64_t tile0, ntiles, grid;
    int tiles_per_wave;
};

// below this many tiles, kTritTiles per wave would leave CUs idle: one tile per wave
constexpr uint64_t kSmallTritTiles = (uint64_t)kTritTiles * kWaveSlots * 256 * 2;

TritRange trit_range(LaunchRange r) {
    TritRange t;
    t.tile0 = r.first / kTileRecs;
    const uint64_t tile1 = (r.first + r.n + kTileRecs - 1) / kTileRecs;
    t.ntiles = tile1 - t.tile0;
    t.tiles_per_wave = t.ntiles < kSmallTritTiles ? 1 : kTritTiles;
    // test hook, as for TILES: IRIS_TILES_PER_WAVE=1|4 pins the variant
    if (const char *f = getenv("IRIS_TILES_PER_WAVE")) t.tiles_per_wave = atoi(f) == 1 ? 1 : kTritTiles;
    const uint64_t waves = (t.ntiles + t.tiles_per_wave - 1) / t.tiles_per_wave;
    t.grid = (waves + kWaveSlots - 1) / kWaveSlots;
    return t;
}

}  // namespace

int launch_pack_trits(void *stream, const void *staging, void *db, uint64_t t_first, uint64_t n) {
    if (n == 0) return 0;
    hipLaunchKernelGGL(pack_trits_kernel, dim3(grid_of(n * 4 * kTritGroups)), dim3(256), 0, (hipStream_t)stream,
                       (const uint32_t *)staging, (uint4 *)db, t_first, n);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

int launch_unpack_trits(void *stream, const void *db, void *staging, uint64_t t_first, uint64_t n) {
    if (n == 0) return 0;
    hipLaunchKernelGGL(unpack_trits_kernel, dim3(grid_of(n * kPlaneDwords)), dim3(256), 0, (hipStream_t)stream,
                       (const uint4 *)db, (uint32_t *)staging, t_first, n);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

int launch_generate_trits(void *stream, void *db, uint64_t t_first, uint64_t n, uint64_t seed, uint64_t global_index0) {
    if (n == 0) return 0;
    hipLaunchKernelGGL(generate_trits_kernel, dim3(grid_of(n * 4 * kTritGroups)), dim3(256), 0, (hipStream_t)stream,
                       (uint4 *)db, t_first, n, gen_key(seed, 0), global_index0);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

uint32_t trits_search_partials(LaunchRange r) { return (uint32_t)trit_range(r).grid; }

int launch_trits_search(void *stream, const void *db, const void *qfrag, LaunchRange r, double *dist_out,
                        Partial *partials, uint32_t *n_partials) {
    const TritRange t = trit_range(r);
    *n_partials = (uint32_t)t.grid;
    if (r.n == 0) return 0;
    auto kern = t.tiles_per_wave == 1 ? trits_mfma_kernel<TR_SEARCH, 1> : trits_mfma_kernel<TR_SEARCH, kTritTiles>;
    hipLaunchKernelGGL(kern, dim3((uint32_t)t.grid), dim3(256), 0, (hipStream_t)stream, (const uint4 *)db,
                       (const uint4 *)qfrag, t.tile0, t.ntiles, r.first, r.first + r.n, (uint16_t *)nullptr,
                       (uint16_t *)nullptr, dist_out, partials);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

int launch_trits_counts(void *stream, const void *db, const void *qfrag, LaunchRange r, uint16_t *num_out,
                        uint16_t *den_out) {
    if (r.n == 0) return 0;
    const TritRange t = trit_range(r);
    auto kern = t.tiles_per_wave == 1 ? trits_mfma_kernel<TR_COUNTS, 1> : trits_mfma_kernel<TR_COUNTS, kTritTiles>;
    hipLaunchKernelGGL(kern, dim3((uint32_t)t.grid), dim3(256), 0, (hipStream_t)stream, (const uint4 *)db,
                       (const uint4 *)qfrag, t.tile0, t.ntiles, r.first, r.first + r.n, num_out, den_out,
                       (double *)nullptr, (Partial *)nullptr);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

}  // namespace iris
