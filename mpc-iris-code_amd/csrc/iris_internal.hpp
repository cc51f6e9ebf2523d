// iris_internal.hpp — device layouts, generator and launch declarations shared
// by the HIP kernels (iris_kernels.hip) and the C ABI (iris_api.hip).
//
// Device layout: records are grouped in blocks of 64 — one
// record per lane of a wavefront — and each block stores, for every 16-byte
// group g of a record plane, the 64 lanes' 16 bytes contiguously (1 KiB).
// One `global_load_dwordx4` of a wave therefore reads 1 KiB fully coalesced,
// and every lane holds word 4g..4g+3 of its own record: the rotated query
// words are then wave-uniform and live in SGPRs (no LDS, no cross-lane
// reduction).
#pragma once
#include <stdint.h>
#include <stddef.h>
#include <sys/types.h>

#include "../../include/iris_hip.h"

#if defined(__HIPCC__)
#define IRIS_HD __host__ __device__
#else
#define IRIS_HD
#endif

namespace iris {

constexpr int kLanes = 64;            // records per block (= wavefront width)
constexpr int kRot = IRIS_ROTATIONS;  // 31
constexpr int kWaveSlots = 4;         // waves per workgroup (256 threads)

// dwords of one record plane (12800 bits) and its 16-byte groups
constexpr int kPlaneDwords = IRIS_BITS / 32;     // 400
constexpr int kPlaneGroups = kPlaneDwords / 4;   // 100
constexpr int kShareDwords = IRIS_BITS / 2;      // 6400 (two u16 per dword)
constexpr int kShareGroups = kShareDwords / 4;   // 1600

// Device layouts.
//  LANES (VALU kernels): blocks of 64 records, one per lane; for each 16-byte
//    group G of a record the 64 lanes' 16 B are contiguous (1 KiB):
//      TEMPLATES: G = 2*g + p, p = 0 mask plane, p = 1 pattern plane  (200 groups)
//      MASKS:     G = g                                               (100 groups)
//      SHARES:    G = g                                               (1600 groups)
//  TILES (MFMA kernels, TEMPLATES only): tiles of 32 records.  For chunk pair
//    g (template bits [128g, 128g+128) of both planes) lane L = t + 32h holds
//    one uint4 {X0(2g,h), X1(2g,h), X0(2g+1,h), X1(2g+1,h)}: the interleaved
//    mask/pattern bits of plane dword w = 2c + h (see xpack below), which is
//    exactly the fp4 B-operand fragment source of lane L for chunk c.
struct KindInfo {
    int kind;
    int layout;         // IRIS_LAYOUT_LANES or IRIS_LAYOUT_TILES
    int block;          // records per block (64 lanes or 32-record tiles)
    int groups;         // 16-byte groups per record (LANES) / per lane (TILES)
    int planes;         // planes interleaved per g (LANES)
    int rec_dwords;     // dwords per record in the reference layout
    int plane_src[2];   // dword offset of plane p inside the reference record
    size_t rec_bytes;   // bytes per reference record
};

inline KindInfo kind_info(int kind, int layout = IRIS_LAYOUT_LANES) {
    switch (kind) {
    case IRIS_KIND_TEMPLATES:
        if (layout == IRIS_LAYOUT_TILES) return {kind, layout, 32, kPlaneGroups, 2, 2 * kPlaneDwords, {kPlaneDwords, 0}, 3200};
        return {kind, IRIS_LAYOUT_LANES, 64, 2 * kPlaneGroups, 2, 2 * kPlaneDwords, {kPlaneDwords, 0}, 3200};
    case IRIS_KIND_MASKS:
        if (layout == IRIS_LAYOUT_TILES) return {kind, layout, 32, kPlaneGroups / 2, 1, kPlaneDwords, {0, 0}, 1600};
        return {kind, IRIS_LAYOUT_LANES, 64, kPlaneGroups, 1, kPlaneDwords, {0, 0}, 1600};
    case IRIS_KIND_SHARES:
        if (layout == IRIS_LAYOUT_TILES) return {kind, layout, 32, kShareDwords / 16, 2, kShareDwords, {0, 0}, 25600};
        return {kind, IRIS_LAYOUT_LANES, 64, kShareGroups, 1, kShareDwords, {0, 0}, 25600};
    default: return {0, 0, 0, 0, 0, 0, {0, 0}, 0};
    }
}

inline size_t block_bytes(const KindInfo &k) { return (size_t)k.block * k.rec_bytes; }

// TILES interleave of 16 mask bits and 16 pattern bits into one dword:
//   nibble p: bit0 = em[2p+1], bit1 = em[2p], bit2 = ep[2p+1], bit3 = ep[2p]
// so that (x & 0xAAAAAAAA) and ((x+x) & 0xAAAAAAAA) are fp4 e2m1 values
// {0, +1, -1} = encode() of K positions 2p and 2p+1, and (x & 0x22222222),
// (x & 0x11111111) are the mask bits as fp4 1.0 and 0.5.
IRIS_HD inline uint32_t xpack(uint32_t em16, uint32_t ep16) {
    uint32_t x = 0;
    for (int p = 0; p < 8; ++p) {
        x |= ((em16 >> (2 * p + 1)) & 1u) << (4 * p);
        x |= ((em16 >> (2 * p)) & 1u) << (4 * p + 1);
        x |= ((ep16 >> (2 * p + 1)) & 1u) << (4 * p + 2);
        x |= ((ep16 >> (2 * p)) & 1u) << (4 * p + 3);
    }
    return x;
}
IRIS_HD inline void xunpack(uint32_t x, uint32_t &em16, uint32_t &ep16) {
    em16 = 0;
    ep16 = 0;
    for (int p = 0; p < 8; ++p) {
        em16 |= ((x >> (4 * p)) & 1u) << (2 * p + 1);
        em16 |= ((x >> (4 * p + 1)) & 1u) << (2 * p);
        ep16 |= ((x >> (4 * p + 2)) & 1u) << (2 * p + 1);
        ep16 |= ((x >> (4 * p + 3)) & 1u) << (2 * p);
    }
}
// fp4 K index j (0..31) of a lane's fragment <-> bit of the lane's plane dword
IRIS_HD inline int frag_bit(int j) { return (j & 16) + 2 * (j & 7) + ((j >> 3) & 1); }

// MFMA query fragments: for chunk c (template bits [64c, 64c+64)) and lane
// L = k + 32h (k = rotation index 0..30, 31 = zero row), one uint4 at
// [c * 64 + L]: fp4 e2m1 of encode(q rotated by k - 15) at bit frag_bit(j) of
// plane dword 2c + h (+1.0 = 0x2, -1.0 = 0xA, 0).  The den operand is derived
// from it in-kernel (|enc|, doubled where the template side carries 0.5).
constexpr int kFragDwords = 4;

// TILES layouts of the other kinds (iris_mfma.hip):
//  MASKS  (fp4, den only): tile of 32 masks = 3200 uint4.  uint4 [g*64 + L]
//    (g = 0..49, L = t + 32h) = mask dwords {8g+h, 8g+2+h, 8g+4+h, 8g+6+h}, i.e.
//    the lane's dword of chunks 4g..4g+3.  Fragment dword d of a chunk is
//    x & (0x11111111 << d) for d < 3 and (x >> 1) & 0x44444444 for d = 3, so
//    K index j <-> mask bit 4 (j % 8) + j / 8 with template-side value
//    0.5 / 1 / 2 / 2 and query-side value 2 / 1 / 0.5 / 0.5.
//  SHARES (i8): tile of 32 shares = 51200 uint4.  For chunk c (elements
//    [32c, 32c+32)) and lane L = t + 32h: uint4 [(2c) * 64 + L] = low bytes,
//    [(2c+1) * 64 + L] = high bytes of elements 32c + 16h + j (j = 0..15), each
//    XOR 0x80 (the byte minus 128 as an i8), the B fragment of
//    v_mfma_i32_32x32x32_i8 (lane l holds K = 16 (l >> 5) + j).
constexpr int kMaskTileUint4 = (kPlaneGroups / 2) * 64;   // 3200
constexpr int kShareTileUint4 = (kShareDwords / 16) * 2 * 64;  // 51200
constexpr int kMaskChunks = kPlaneDwords / 2;   // 200 chunks of 64 bits
constexpr int kShareChunks = IRIS_BITS / 32;    // 400 chunks of 32 elements
// masks A-fragments, one bit per fp4 element: uint4 [step g = 50][lane 64], one
// dword per chunk 4g + i; element j of a lane's 32 is bit 4 (j & 7) + {2, 1, 0, 3}[j >> 3]
constexpr size_t kMaskFragUint4 = (size_t)(kMaskChunks / 4) * 64;
constexpr size_t kShareFragUint4 = (size_t)kShareChunks * 64 * 2;  // + 32 int2 row constants after it
IRIS_HD inline int mask_frag_bit(int j) { return 4 * (j & 7) + (j >> 3); }
constexpr size_t kTemplateFragDwords = (size_t)(kPlaneDwords / 2) * 64 * kFragDwords;  // 200 chunks

// Rotated-query tables (built once per engine, on the device by iris_query.hip;
// the host builders below are their reference):
//   TEMPLATES: dword [w*64 + 2k] = mask_k word w, [w*64 + 2k+1] = pattern_k word w   (400 x 64)
//   MASKS:     dword [w*32 + k]  = mask_k word w                                      (400 x 32)
//   SHARES:    dword [d*32 + k]  = rot_k[2d] | rot_k[2d+1] << 16                       (6400 x 32)
// k = 0..30 is rotation r = k - 15; slot 31 (and 62, 63) is zero.
constexpr int kTemplateTabStride = 64;
constexpr int kSlotTabStride = 32;

// Per-workgroup partial result of a search (24 B).
struct Partial {
    uint32_t num;
    uint32_t den;   // 0 = no candidate
    int32_t rot;    // k index 0..30
    uint32_t pad;
    uint64_t idx;   // template index relative to the searched range start
};

// ---------------------------------------------------------------- generator
// Counter-based synthetic data: limb = splitmix64 output number
// ctr+1 of the stream keyed by (seed, stream).  Templates: stream 0, pattern
// limb j of template t = ctr t*400 + j, mask limb j = ctr t*400 + 200 + j.
// Shares: stream 1, limb j of record t = ctr t*3200 + j (4 LE u16 per limb).
IRIS_HD inline uint64_t mix64(uint64_t z) {
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
    return z ^ (z >> 31);
}
IRIS_HD inline uint64_t gen_key(uint64_t seed, uint64_t stream) {
    return mix64(seed ^ (0xD1B54A32D192ED03ULL * (stream + 1)));
}
IRIS_HD inline uint64_t gen_limb(uint64_t key, uint64_t ctr) {
    return mix64(key + (ctr + 1) * 0x9E3779B97F4A7C15ULL);
}

// ---------------------------------------------------------------- runtime configuration
// Environment knobs are read once, when a device opens (read_hooks, iris_host.cpp), into that
// device's Hooks; launchers take them from there, never from the environment.  The test-only
// hooks pin kernel variants or inject delays and faults: they are honoured only when
// IRIS_TEST_HOOKS=1 is also set, and otherwise ignored (iris_config reports both).
struct Hooks {
    // production knobs
    bool readahead = true;           // IRIS_READAHEAD=0: no read-ahead of host-output engine calls
    bool auto_resident = true;       // IRIS_AUTO_RESIDENT=0: host slices of read-only file mappings upload per call
    uint32_t group_timeout_ms = 0;   // IRIS_GROUP_TIMEOUT_MS: bound of a group exchange wait (0: auto)
    uint32_t resident_max_mb = 0;    // IRIS_RESIDENT_MAX_MB: resident file copies hold at most this (0: half the device)
    // test-only hooks (IRIS_TEST_HOOKS=1)
    bool test = false;
    int tiles_per_wave = 0;          // IRIS_TILES_PER_WAVE=1|4: pins the TILES kernels' variant (0: by range)
    bool fused_reduce = true;        // IRIS_FUSED_REDUCE=0: small searches launch the separate reduce
    int batch_kernel = 4;            // IRIS_BATCH_KERNEL=2|4: batched-query kernel shape (iris_batch.hip)
    int schedule = 0;                // IRIS_SCHEDULE=spin|yield|blocking (1|2|3): host wait mode
    bool load_pread = false;         // IRIS_LOAD_PREAD=1: file loads through the pinned-buffer path
    bool load_windows = false;       // IRIS_LOAD_WINDOWS=1: file loads DMA from registered page-cache windows
    uint32_t group_delay_us = 0;     // IRIS_GROUP_DELAY_US: side-stream spin before each group all-gather
    bool group_stall = false;        // IRIS_GROUP_STALL=1: a group all-gather waits on a peer that never comes
    bool group_unordered = false;    // IRIS_GROUP_UNORDERED=1: drop the exchange-buffer ordering (shows the race)
    int upload = 0;                  // IRIS_UPLOAD=pinned|runtime (1|2): the path of writes >= 8 MB (0: the faster lately)
    uint32_t ra_window = 0;          // IRIS_READAHEAD_WINDOW=1..64: chunks per read-ahead window (0: growing)
    uint32_t resident_budget_mb = 0; // IRIS_RESIDENT_BUDGET_MB: resident copies hold at most this (0: free memory)
    bool ra_packed = true;           // IRIS_READAHEAD_PACKED=0: masks read-ahead rows cross the host link unpacked
    uint32_t ra_window_max = 0;      // IRIS_READAHEAD_WINDOW_MAX=1..1024: cap of a read-ahead window, chunks (0: by records)
    uint32_t ignored = 0;            // bit i: test hook kHookNames[i] was set without IRIS_TEST_HOOKS=1
};
// The bound of forming a device group when IRIS_GROUP_TIMEOUT_MS is not set (iris_group.hip)
constexpr uint32_t kGroupInitTimeoutMs = 120000;
// Reads the environment (the Hooks a device opened now gets).
void read_hooks(Hooks *h);
// "key=value ..." of h plus the process-wide knobs (IRIS_COPY_HELPERS); returns the length.
size_t format_hooks(const Hooks &h, char *buf, size_t len);

// ---------------------------------------------------------------- launchers
// (defined in iris_kernels.hip; all asynchronous on `stream`)
struct LaunchRange {
    uint64_t first;  // first record index of the range
    uint64_t n;      // records in the range
};

int launch_pack(void *stream, const KindInfo &k, const void *staging, void *db, uint64_t t_first, uint64_t n);
// per-engine query tables built on the device from the query (iris_query.hip)
// q, qmask: host
int launch_query_template(void *stream, const void *q, uint32_t *tab, uint32_t *frag);
int launch_query_masks(void *stream, const void *qmask, uint32_t *tab, uint32_t *frag);
int launch_query_shares(void *stream, const void *q, uint32_t *tab, uint32_t *frag);
int launch_query_tiles(void *stream, const void *queries, uint32_t nq, uint32_t nqp, uint32_t *tiles);
// rounds: ChaCha8 / 12 / 20 (anything else: -1)
int launch_prepare_shares(void *stream, const void *templates, uint64_t m, uint64_t g0, const uint8_t key[32],
                          uint64_t nonce, uint32_t rounds, uint32_t parties, void *shares);
constexpr int kMaxPrepParties = 64;
int launch_prepare_shares_tiles(void *stream, const void *templates, uint64_t m, uint64_t g0, const uint8_t key[32],
                                uint64_t nonce, uint32_t rounds, uint32_t parties, void *const *dbs,
                                const uint64_t *t_first);
int launch_prepare_direct(void *stream, const void *tdb, uint64_t t_first, uint64_t m, uint64_t g0,
                          const uint8_t key[32], uint64_t nonce, uint32_t rounds, uint32_t parties,
                          void *const *dbs, const uint64_t *s_first, void *masks, uint64_t m_first);
int launch_unpack(void *stream, const KindInfo &k, const void *db, void *staging, uint64_t t_first, uint64_t n);
int launch_generate(void *stream, const KindInfo &k, void *db, uint64_t t_first, uint64_t n, uint64_t seed,
                    uint64_t global_index0);
int launch_template_counts(void *stream, const void *db, const void *qtab, LaunchRange r, uint16_t *num_out,
                           uint16_t *den_out);
int launch_template_mfma_counts(const Hooks &h, void *stream, const void *db, const void *qfrag, LaunchRange r, uint16_t *num_out,
                                uint16_t *den_out);
// Fused finish of a small search (grids of at most kFusedReduceMax workgroups): the last
// workgroup to finish reduces the partials and writes the winner (idx + idx_base) to dst;
// ticket is a zeroed 4-KB device block (a two-level ticket) that the kernel leaves zeroed.  done != null (dst in
// coherent host memory): dst is written through to host memory and, once those stores have
// completed, seq is stored to *done (coherent host memory) -- a blocking caller spins on
// that word instead of waiting for the end of the kernel and the runtime's completion signal.
struct FusedFinish {
    uint32_t *ticket;
    Partial *dst;
    uint64_t idx_base;
    uint32_t *done;
    uint32_t seq;
};
constexpr uint32_t kFusedReduceMax = 4096;
bool fused_search_ok(const Hooks &h, LaunchRange r);
int launch_template_mfma_search(const Hooks &h, void *stream, const void *db, const void *qfrag, LaunchRange r, double *dist_out,
                                Partial *partials, uint32_t *n_partials, const FusedFinish *fin = nullptr);
uint32_t mfma_search_partials(const Hooks &h, LaunchRange r);
// nq = 2 queries per streamed pass; partials [nq][*n_partials]
uint32_t multi_search_partials(LaunchRange r, int nq);
int launch_template_multi_search(void *stream, const void *db, const void *const *qfrags, int nq, LaunchRange r,
                                 Partial *partials, uint32_t *n_partials);
int launch_pack_tiles(void *stream, const void *staging, void *db, uint64_t t_first, uint64_t n);
int launch_unpack_tiles(void *stream, const void *db, void *staging, uint64_t t_first, uint64_t n);
int launch_generate_tiles(void *stream, void *db, uint64_t t_first, uint64_t n, uint64_t seed, uint64_t global_index0);
int launch_pack_tiles_kind(void *stream, int kind, const void *staging, void *db, uint64_t t_first, uint64_t n);
int launch_unpack_tiles_kind(void *stream, int kind, const void *db, void *staging, uint64_t t_first, uint64_t n);
int launch_generate_tiles_kind(void *stream, int kind, void *db, uint64_t t_first, uint64_t n, uint64_t seed,
                               uint64_t global_index0);
// Completion word of a blocking device-output engine call: the kernel's last workgroup, once
// every workgroup's rows are stored, stores seq into the coherent host word done (ticket: the
// device's zeroed 4-KB ticket block, left zeroed).  The launcher sets armed when the kernel it
// chose signals (the small-range K-split kernels); otherwise the caller waits for the stream.
struct DoneSignal {
    uint32_t *ticket;
    uint32_t *done;
    uint32_t seq;
    bool armed;
};
// packed: the rows in the read-ahead's packed form (store_tile_packed): out holds r.n records of
// 32 B, then r.n escape rows of 31 u16 (no completion word)
int launch_masks_mfma(const Hooks &h, void *stream, const void *db, const void *qfrag, LaunchRange r, uint16_t *out,
                      DoneSignal *sig = nullptr, bool packed = false);
uint32_t masks_resolve_partials(const Hooks &h, LaunchRange r);
int launch_masks_resolve(const Hooks &h, void *stream, const void *db, const void *qfrag, LaunchRange r,
                         const uint16_t *const *shares, uint32_t parts, double *dist_out, Partial *partials);
uint32_t resolver_partials(uint64_t n);
struct BatchGeometry {
    uint64_t tile0, ntiles;
    uint32_t nqg, G;  // query groups, workgroups per query group
    uint32_t qper;    // queries per query group (nqg * qper results; at most the engine's padding)
};
BatchGeometry batch_geometry(const Hooks &h, LaunchRange r, uint32_t nq);
uint32_t batch_query_group();  // padding unit of a batched engine's queries
int launch_batch(const Hooks &h, void *stream, const void *db, const void *qtiles, LaunchRange r, const BatchGeometry &g,
                 Partial *partials, Partial *out, uint64_t idx_base = 0);
int launch_resolver(void *stream, const uint16_t *const *shares, uint32_t parts, const uint16_t *denoms, uint64_t n,
                    double *dist_out, Partial *partials);
int launch_shares_mfma(const Hooks &h, void *stream, const void *db, const void *qfrag, LaunchRange r, uint16_t *out,
                       DoneSignal *sig = nullptr);
int launch_template_search(void *stream, const void *db, const void *qtab, LaunchRange r, double *dist_out,
                           Partial *partials, uint32_t *n_partials);
// consumes partials; the winner's idx (range-relative) is offset by idx_base
int launch_reduce(void *stream, Partial *partials, uint32_t n_partials, Partial *out, uint64_t idx_base = 0);
// group search merge: out[q] = best of recv[s * stride + q], s < shards (indices already global)
int launch_group_merge(void *stream, const Partial *recv, uint32_t shards, uint32_t nq, uint32_t stride, Partial *out);
int launch_masks(void *stream, const void *db, const void *qtab, LaunchRange r, uint16_t *out);
int launch_shares(void *stream, const void *db, const void *qtab, LaunchRange r, uint16_t *out);

// number of partial records launch_template_search writes for a range
uint32_t search_partials(LaunchRange r);

// ---------------------------------------------------------------- host helpers (iris_host.cpp)
void bits_rotated(const uint64_t *in, int amount, uint64_t *out);
void encoded_rotated(const uint16_t *in, int amount, uint16_t *out);
void encode_template(const iris_template_t *t, uint16_t *out);
void build_template_table(const iris_template_t *q, uint32_t *tab);                  // 400*64 dwords
void build_template_frags(const iris_template_t *q, uint32_t *frag);                 // kTemplateFragDwords
void build_masks_frags(const uint64_t *const *vectors, int count, uint32_t *frag);    // kMaskFragUint4 uint4 (compact)
void build_query_tile(const iris_template_t *q, uint32_t *tile);                      // 6400 uint4 (TILES tile)
void build_shares_frags(const uint16_t *const *vectors, int count, uint32_t *frag);   // kShareFragUint4 uint4 + 64 int
void build_masks_table(const uint64_t *const *vectors, int count, uint32_t *tab);     // 400*32
void build_shares_table(const uint16_t *const *vectors, int count, uint32_t *tab);    // 6400*32
void build_masks_rotations(const uint64_t *query, uint32_t *tab);
void build_shares_rotations(const uint16_t *query, uint32_t *tab);
bool partial_better(const Partial &a, const Partial &b);
// memcpy split over a few persistent helper threads (copies of at least 256 KB)
void parallel_copy(void *dst, const void *src, size_t bytes, int lane = 0);  // lane: the device ordinal
// pread of [off, off + bytes) of fd into dst, split over the same helper threads; false if a read
// failed or the file ended early
bool parallel_pread(int fd, void *dst, size_t bytes, off_t off, int lane = 0);
// MasksEngine rows of n records in the read-ahead's packed form (store_tile_packed, iris_device.hpp:
// 32 B per record at pk, escaped rows in full at esc) expanded into [n][31] u16 at out, split over
// the same helper threads
void parallel_expand(uint16_t *out, const uint8_t *pk, const uint16_t *esc, size_t n, int lane = 0);
void expand_packed_rows(uint16_t *out, const uint8_t *pk, const uint16_t *esc, size_t n);  // one thread
// memcpy whose destination lines are written with non-temporal stores (AVX-512, >= 4 KB); one thread
void copy_nt(char *dst, const char *src, size_t n);
// dst[i] = src[0][i] + ... + src[k-1][i] mod 2^16 (k <= 8): one thread / the device's helper pool
void sum_u16(uint16_t *dst, const uint16_t *const *src, int k, size_t n);
void parallel_sum_u16(uint16_t *dst, const uint16_t *const *src, int k, size_t n, int lane = 0);

}  // namespace iris
