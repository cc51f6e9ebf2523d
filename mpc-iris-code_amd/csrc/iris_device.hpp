// iris_device.hpp — device helpers shared by the MFMA kernels.
#pragma once
#include <hip/hip_runtime.h>

#include <atomic>

#include "iris_internal.hpp"

namespace iris {

// Workgroups of one launch that fit on the current device at `per_cu` per CU
// (persistent grids); cached per device ordinal.
static inline uint64_t resident_blocks(int per_cu) {
    static std::atomic<int> cus[64];  // zero-initialised (static storage)
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) dev = 0;
    int n = cus[dev].load(std::memory_order_relaxed);
    if (n == 0) {
        if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0) n = 256;
        cus[dev].store(n, std::memory_order_relaxed);
    }
    return (uint64_t)n * per_cu;
}


typedef unsigned int u32x4_nt __attribute__((ext_vector_type(4)));

// 16-B store written through the XCD's L2 (sc1: the line leaves L2 and is dropped there; the same
// cost as a plain 16-B store, MI355X_MICROARCH.md "stores of each flavour").
__device__ __forceinline__ void store16_wt(uint4 *dst, const uint4 &v) {
    const u32x4_nt w = {v.x, v.y, v.z, v.w};
    asm volatile("global_store_dwordx4 %0, %1, off sc1" ::"v"(dst), "v"(w) : "memory");
}

// Writes one 32-record tile's [32][31] u16 output rows.  In the 32x32 MFMA C
// layout lane l holds rows k = (r & 3) + 8 (r >> 2) + 4 (l >> 5), r = 0..15, of
// record (l & 31); `val(r)` returns that value.  A tile fully inside
// [first, end) whose output offset is 16-B aligned is staged through the
// wave's 2 KB LDS buffer and written with 124 16-byte stores (1984 B); other
// tiles fall back to per-element stores of their valid records.
// wt (a kernel that signals completion before it ends, DoneSignal): every row byte is written
// through L2 (sc1), so once the storing wave's vmcnt(0) wait returns the rows are in memory, where a
// reader on any XCD -- a kernel on another stream, a copy engine -- finds them without this launch's
// end-of-kernel write-back (nontemporal and plain stores stay dirty in the XCD's L2 until then).
template <class F>
__device__ __forceinline__ void store_tile_rows(uint16_t *__restrict__ out, uint16_t *lds, uint64_t tile_t0,
                                                uint64_t first, uint64_t end, bool tile_valid, int lane, F val,
                                                bool wt = false) {
    const int h = lane >> 5;
    const bool full = tile_valid && tile_t0 >= first && tile_t0 + 32 <= end && ((tile_t0 - first) & 7) == 0 &&
                      (((uintptr_t)out & 15) == 0);
    if (full) {  // wave-uniform
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const int k = (r & 3) + 8 * (r >> 2) + 4 * h;
            if (k < kRot) lds[(lane & 31) * kRot + k] = val(r);
        }
        uint4 *dst = (uint4 *)(out + (tile_t0 - first) * kRot);
        const uint4 *src = (const uint4 *)lds;
        // streamed out with nontemporal stores: the rows are not re-read by this launch
        constexpr int kStores = 32 * kRot * 2 / 16;
        if (wt) {  // wave-uniform
            for (int i = lane; i < kStores; i += 64) store16_wt(&dst[i], src[i]);
            return;
        }
        for (int i = lane; i < kStores; i += 64) {
            const uint4 v = src[i];
            const u32x4_nt w = {v.x, v.y, v.z, v.w};
            __builtin_nontemporal_store(w, (u32x4_nt *)&dst[i]);
        }
    } else {
        const uint64_t tg = tile_t0 + (lane & 31);
        if (!tile_valid || tg < first || tg >= end) return;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const int k = (r & 3) + 8 * (r >> 2) + 4 * h;
            if (k >= kRot) continue;
            if (wt)  // agent-scope relaxed store: global_store_short ... sc1
                __hip_atomic_store(&out[(tg - first) * kRot + k], val(r), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            else
                out[(tg - first) * kRot + k] = val(r);
        }
    }
}

// Writes one 32-record tile's MasksEngine rows in the packed form the read-ahead windows carry over
// the host link (32 B per record instead of 62, iris_api.hip kPackedRecBytes): record i of the
// range [first, end) at pk + 32 i holds bytes 0..30 = row[k] - 64 B and byte 31 = B, where
// B = min_k row[k] >> 6 (den <= 12800, so B <= 200), whenever every row[k] - 64 B fits a byte;
// otherwise byte 31 is 0xFF and the row is stored in full at esc + 31 i.  Random masks never
// escape (the 31 rotations' counts span ~115-220); structured ones (a block of masked columns) do.
// In the 32x32 MFMA C layout lane l holds rows k = (r & 3) + 8 (r >> 2) + 4 h, h = l >> 5, of record
// l & 31, so its registers 4j..4j+3 are the record's bytes 8j + 4h .. +3 (record dword 2j + h); after
// swapping two dwords with its partner lane l ^ 32, half 0 holds the record's bytes 0..15 and half 1
// bytes 16..31, and a wave's 64 16-B stores cover a tile's 1024 B contiguously.
template <class F>
__device__ __forceinline__ void store_tile_packed(uint8_t *__restrict__ pk, uint16_t *__restrict__ esc, uint64_t tile_t0,
                                                  uint64_t first, uint64_t end, bool tile_valid, int lane, F val) {
    const int h = lane >> 5;
    uint32_t v[16];
    uint32_t lo = 0xFFFFu, hi = 0;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
        const int k = (r & 3) + 8 * (r >> 2) + 4 * h;
        v[r] = val(r);
        if (k < kRot) {
            lo = v[r] < lo ? v[r] : lo;
            hi = v[r] > hi ? v[r] : hi;
        }
    }
    const uint32_t plo = __shfl_xor(lo, 32), phi = __shfl_xor(hi, 32);
    lo = plo < lo ? plo : lo;
    hi = phi > hi ? phi : hi;
    const uint32_t b = lo >> 6, base = b << 6;
    const bool escape = hi - base > 255u;
    uint32_t dw[4];
#pragma unroll
    for (int j = 0; j < 4; ++j)
        dw[j] = ((v[4 * j] - base) & 0xFFu) | ((v[4 * j + 1] - base) & 0xFFu) << 8 | ((v[4 * j + 2] - base) & 0xFFu) << 16 |
                ((v[4 * j + 3] - base) & 0xFFu) << 24;
    if (h) dw[3] = (dw[3] & 0x00FFFFFFu) | (escape ? 0xFFu : b) << 24;  // byte 31: row k = 31 is the zero row
    const uint32_t sa = __shfl_xor(h ? dw[0] : dw[2], 32), sb = __shfl_xor(h ? dw[1] : dw[3], 32);
    const u32x4_nt w = h ? u32x4_nt{sa, dw[2], sb, dw[3]} : u32x4_nt{dw[0], sa, dw[1], sb};
    const uint64_t tg = tile_t0 + (lane & 31);
    if (!tile_valid || tg < first || tg >= end) return;
    __builtin_nontemporal_store(w, (u32x4_nt *)(pk + (tg - first) * 32 + 16 * h));
    if (escape) {
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const int k = (r & 3) + 8 * (r >> 2) + 4 * h;
            if (k < kRot) esc[(tg - first) * kRot + k] = (uint16_t)v[r];
        }
    }
}

// Shares TILES planes: 16 u16 elements (8 dwords) -> the low-byte and
// high-byte planes, each byte XOR 0x80 (the byte - 128 as i8), 16 B each.
__device__ __forceinline__ void split_bytes(const uint32_t *src8, uint4 &lo, uint4 &hi) {
    uint32_t l[4], hh[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const uint32_t a = src8[2 * q], b = src8[2 * q + 1];  // elements 4q..4q+3
        // v_perm_b32: bytes 0-3 of the selector space are a's, 4-7 are b's
        l[q] = __builtin_amdgcn_perm(b, a, 0x06040200u) ^ 0x80808080u;   // a0 a2 b0 b2
        hh[q] = __builtin_amdgcn_perm(b, a, 0x07050301u) ^ 0x80808080u;  // a1 a3 b1 b3
    }
    lo = make_uint4(l[0], l[1], l[2], l[3]);
    hi = make_uint4(hh[0], hh[1], hh[2], hh[3]);
}

// Candidate order of the resolver / search argmin: exact fraction (u32 cross-
// multiplication, num and den < 2^16), then the lowest index; den = 0 is "no
// candidate" (NaN / +inf in the reference, never selected by a strict <).
// (__umul24: num, den < 2^16, so the 24-bit multiply's low 32 bits are the exact product, at
// full rate where a 32-bit v_mul_lo_u32 issues at a quarter)
__device__ __forceinline__ bool partial_better_dev(const Partial &a, const Partial &b) {
    if (a.den == 0) return false;
    if (b.den == 0) return true;
    const uint32_t l = __umul24(a.num, b.den), r = __umul24(b.num, a.den);
    if (l != r) return l < r;
    return a.idx < b.idx;
}
// as partial_better_dev, then the lower rotation (two candidates of one template)
__device__ __forceinline__ bool partial_better_rot(const Partial &a, const Partial &b) {
    if (a.den == 0) return false;
    if (b.den == 0) return true;
    const uint32_t l = __umul24(a.num, b.den), r = __umul24(b.num, a.den);
    if (l != r) return l < r;
    if (a.idx != b.idx) return a.idx < b.idx;
    return a.rot < b.rot;
}

__device__ __forceinline__ Partial partial_shfl_xor(const Partial &c, int off) {
    Partial o;
    o.num = __shfl_xor(c.num, off);
    o.den = __shfl_xor(c.den, off);
    o.rot = __shfl_xor(c.rot, off);
    o.pad = 0;
    const uint32_t lo = __shfl_xor((uint32_t)c.idx, off), hi = __shfl_xor((uint32_t)(c.idx >> 32), off);
    o.idx = ((uint64_t)hi << 32) | lo;
    return o;
}

// One template's best rotation from a 32x32 MFMA C tile: lane l holds rows
// k = (r & 3) + 8 (r >> 2) + 4 (l >> 5), r = 0..15, of template l & 31, and
// frac(r, num, den) yields row r's fraction.  Exact order (u32 cross-
// multiplication; den = 0 is no candidate), lowest rotation on ties; after the
// exchange with lane l ^ 32 both halves hold the template's best (k in 0..30).
template <class F>
__device__ __forceinline__ void best_rotation(int lane, F frac, uint32_t &bn, uint32_t &bd, int &br) {
    const int h = lane >> 5;
    bn = 0;
    bd = 0;
    br = 0;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
        const int k = (r & 3) + 8 * (r >> 2) + 4 * h;  // ascending in r within a half
        uint32_t nn, dd;
        frac(r, nn, dd);
        if (k < kRot && dd != 0 && (bd == 0 || __umul24(nn, bd) < __umul24(bn, dd))) {
            bn = nn;
            bd = dd;
            br = k;
        }
    }
    const uint32_t pn = __shfl_xor(bn, 32), pd = __shfl_xor(bd, 32);
    const int pr = __shfl_xor(br, 32);
    const uint32_t pl = __umul24(pn, bd), pr_ = __umul24(bn, pd);
    if (pd != 0 && (bd == 0 || pl < pr_ || (pl == pr_ && pr < br))) {
        bn = pn;
        bd = pd;
        br = pr;
    }
}

__device__ __forceinline__ Partial partial_none() {
    Partial p;
    p.num = 0;
    p.den = 0;
    p.rot = 0;
    p.pad = 0;
    p.idx = ~0ull;
    return p;
}

// Last-workgroup reduction (a search's partials reduce without a second launch).  Thread 0
// publishes this workgroup's partial with agent-scope atomic stores (sc1: written through
// past the XCD's L2, coherent across the XCDs without an L2 writeback / invalidate -- a full
// __threadfence here drops every XCD's L2, the L2-resident query fragments with it, once per
// workgroup, and doubled a 20k-template search), waits for them to complete, and takes a
// ticket with an agent-scope atomic add; the workgroup that draws gridDim.x - 1 reads every
// partial with agent-scope (sc1) atomic loads (MI355X_MICROARCH.md, inter-workgroup
// visibility: the first hand-off row), folds them in the
// search order (exact fraction, then lowest index), writes the winner with idx + idx_base to
// fin.dst (pinned host or device memory) and resets the ticket for the next launch.
// at agent scope (sc1 stores / loads, the form of MI355X_MICROARCH.md's first hand-off row)
#define IRIS_FUSED_SCOPE __HIP_MEMORY_SCOPE_AGENT
__device__ __forceinline__ void publish_partial(Partial *p, const Partial &b) {
    uint64_t *w = (uint64_t *)p;
    __hip_atomic_store(w, (uint64_t)b.num | ((uint64_t)b.den << 32), __ATOMIC_RELAXED, IRIS_FUSED_SCOPE);
    __hip_atomic_store(w + 1, (uint64_t)(uint32_t)b.rot, __ATOMIC_RELAXED, IRIS_FUSED_SCOPE);
    __hip_atomic_store(w + 2, b.idx, __ATOMIC_RELAXED, IRIS_FUSED_SCOPE);
}
__device__ __forceinline__ Partial read_partial(const Partial *p) {
    uint64_t *w = (uint64_t *)p;
    const uint64_t a = __hip_atomic_load(w, __ATOMIC_RELAXED, IRIS_FUSED_SCOPE);
    const uint64_t r = __hip_atomic_load(w + 1, __ATOMIC_RELAXED, IRIS_FUSED_SCOPE);
    Partial q;
    q.num = (uint32_t)a;
    q.den = (uint32_t)(a >> 32);
    q.rot = (int32_t)(uint32_t)r;
    q.pad = 0;
    q.idx = __hip_atomic_load(w + 2, __ATOMIC_RELAXED, IRIS_FUSED_SCOPE);
    return q;
}
constexpr uint32_t kTicketGroups = 8;    // sub-tickets of fold_partials_last
constexpr uint32_t kTicketStride = 64;   // words between tickets (256 B: separate lines)
// thread 0 holds this workgroup's winner b (the caller has not stored it)
__device__ __forceinline__ void fold_partials_last(Partial *partials, const Partial &b0, const FusedFinish &fin) {
    __shared__ int last;
    if (threadIdx.x == 0) {
        publish_partial(&partials[blockIdx.x], b0);
        // the stores are performed (vmcnt also counts stores on gfx9) before the ticket is taken;
        // a release fence at agent / system scope would add the L2 writeback this avoids
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        // two-level ticket: workgroup b counts at sub-ticket b % 8 (its own 256-B line), the last
        // of each of those groups at the top word -- the same-address atomics of a launch are
        // serialised where they are performed, ~6 ns each, so 625 on one word cost ~4 us of tail
        const uint32_t c = blockIdx.x % kTicketGroups, groups = gridDim.x < kTicketGroups ? gridDim.x : kTicketGroups;
        const uint32_t members = (gridDim.x - c + kTicketGroups - 1) / kTicketGroups;
        uint32_t *sub = fin.ticket + kTicketStride * (1 + c);
        last = 0;
        if (__hip_atomic_fetch_add(sub, 1u, __ATOMIC_RELAXED, IRIS_FUSED_SCOPE) == members - 1) {
            __hip_atomic_store(sub, 0u, __ATOMIC_RELAXED, IRIS_FUSED_SCOPE);  // for the next launch
            last = __hip_atomic_fetch_add(fin.ticket, 1u, __ATOMIC_RELAXED, IRIS_FUSED_SCOPE) == groups - 1;
        }
    }
    __syncthreads();
    if (!last) return;  // workgroup-uniform
    Partial c = partial_none();
    for (uint32_t i = threadIdx.x; i < gridDim.x; i += blockDim.x) {
        const Partial p = read_partial(&partials[i]);
        if (partial_better_dev(p, c)) c = p;
    }
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) {
        const Partial o = partial_shfl_xor(c, off);
        if (partial_better_dev(o, c)) c = o;
    }
    __shared__ Partial sw[16];
    if ((threadIdx.x & 63) == 0) sw[threadIdx.x >> 6] = c;
    __syncthreads();
    if (threadIdx.x == 0) {
        Partial b = sw[0];
        for (uint32_t w = 1; w < (blockDim.x + 63) / 64; ++w)
            if (partial_better_dev(sw[w], b)) b = sw[w];
        if (b.den != 0) b.idx += fin.idx_base;
        __hip_atomic_store(fin.ticket, 0u, __ATOMIC_RELAXED, IRIS_FUSED_SCOPE);  // for the next launch
        if (fin.done) {
            // write-through to the host, completed, then the sequence word the host polls
            uint64_t *w = (uint64_t *)fin.dst;
            __hip_atomic_store(w, (uint64_t)b.num | ((uint64_t)b.den << 32), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            __hip_atomic_store(w + 1, (uint64_t)(uint32_t)b.rot, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            __hip_atomic_store(w + 2, b.idx, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            __hip_atomic_store(fin.done, fin.seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        } else {
            *fin.dst = b;
        }
    }
}

// Completion word of a blocking device-output call (DoneSignal): called by ONE thread of each
// workgroup once that workgroup's stores have completed (its waves waited for vmcnt(0)); the
// last workgroup to arrive (the two-level ticket of fold_partials_last) resets the ticket and
// stores the sequence number into the coherent host word the caller spins on.
__device__ __forceinline__ void signal_done_last(const DoneSignal &s) {
    const uint32_t c = blockIdx.x % kTicketGroups, groups = gridDim.x < kTicketGroups ? gridDim.x : kTicketGroups;
    const uint32_t members = (gridDim.x - c + kTicketGroups - 1) / kTicketGroups;
    uint32_t *sub = s.ticket + kTicketStride * (1 + c);
    if (__hip_atomic_fetch_add(sub, 1u, __ATOMIC_RELAXED, IRIS_FUSED_SCOPE) != members - 1) return;
    __hip_atomic_store(sub, 0u, __ATOMIC_RELAXED, IRIS_FUSED_SCOPE);  // for the next launch
    if (__hip_atomic_fetch_add(s.ticket, 1u, __ATOMIC_RELAXED, IRIS_FUSED_SCOPE) != groups - 1) return;
    __hip_atomic_store(s.ticket, 0u, __ATOMIC_RELAXED, IRIS_FUSED_SCOPE);
    __hip_atomic_store(s.done, s.seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

}  // namespace iris
