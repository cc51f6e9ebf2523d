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

// Groups of 16 B per record on the device ("G" index) and planes per group row.
//   TEMPLATES: G = 2*g + p, p = 0 mask plane, p = 1 pattern plane  (200 groups)
//   MASKS:     G = g                                               (100 groups)
//   SHARES:    G = g                                               (1600 groups)
struct KindInfo {
    int kind;
    int groups;         // 16-byte groups per record
    int planes;         // planes interleaved per g
    int rec_dwords;     // dwords per record in the reference layout
    int plane_src[2];   // dword offset of plane p inside the reference record
    size_t rec_bytes;   // bytes per reference record
};

inline KindInfo kind_info(int kind) {
    switch (kind) {
    case IRIS_KIND_TEMPLATES: return {kind, 2 * kPlaneGroups, 2, 2 * kPlaneDwords, {kPlaneDwords, 0}, 3200};
    case IRIS_KIND_MASKS: return {kind, kPlaneGroups, 1, kPlaneDwords, {0, 0}, 1600};
    case IRIS_KIND_SHARES: return {kind, kShareGroups, 1, kShareDwords, {0, 0}, 25600};
    default: return {0, 0, 0, 0, {0, 0}, 0};
    }
}

inline size_t block_bytes(const KindInfo &k) { return (size_t)k.groups * kLanes * 16; }

// Rotated-query tables (built on the host, uploaded once per engine):
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

// ---------------------------------------------------------------- launchers
// (defined in iris_kernels.hip; all asynchronous on `stream`)
struct LaunchRange {
    uint64_t first;  // first record index of the range
    uint64_t n;      // records in the range
};

int launch_pack(void *stream, const KindInfo &k, const void *staging, void *db, uint64_t t_first, uint64_t n);
int launch_unpack(void *stream, const KindInfo &k, const void *db, void *staging, uint64_t t_first, uint64_t n);
int launch_generate(void *stream, const KindInfo &k, void *db, uint64_t t_first, uint64_t n, uint64_t seed,
                    uint64_t global_index0);
int launch_template_counts(void *stream, const void *db, const void *qtab, LaunchRange r, uint16_t *num_out,
                           uint16_t *den_out);
int launch_template_search(void *stream, const void *db, const void *qtab, LaunchRange r, double *dist_out,
                           Partial *partials, uint32_t *n_partials);
int launch_reduce(void *stream, const Partial *partials, uint32_t n_partials, Partial *out);
int launch_masks(void *stream, const void *db, const void *qtab, LaunchRange r, uint16_t *out);
int launch_shares(void *stream, const void *db, const void *qtab, LaunchRange r, uint16_t *out);

// number of partial records launch_template_search writes for a range
uint32_t search_partials(LaunchRange r);

// ---------------------------------------------------------------- host helpers (iris_host.cpp)
void bits_rotated(const uint64_t *in, int amount, uint64_t *out);
void encoded_rotated(const uint16_t *in, int amount, uint16_t *out);
void encode_template(const iris_template_t *t, uint16_t *out);
void build_template_table(const iris_template_t *q, uint32_t *tab);                  // 400*64 dwords
void build_masks_table(const uint64_t *const *vectors, int count, uint32_t *tab);     // 400*32
void build_shares_table(const uint16_t *const *vectors, int count, uint32_t *tab);    // 6400*32
void build_masks_rotations(const uint64_t *query, uint32_t *tab);
void build_shares_rotations(const uint16_t *query, uint32_t *tab);
bool partial_better(const Partial &a, const Partial &b);

}  // namespace iris
