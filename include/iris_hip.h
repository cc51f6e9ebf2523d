/*
 * iris_hip.h — C ABI of the MI355X-native masked-Hamming iris-matching engine.
 *
 * This is the drop-in boundary for the hot path of recmo/mpc-iris-code
 * (reference v0.8.0).  Every entry point names the reference interface it
 * replaces (path:line inside the reference repository).  The Rust-side
 * binding a maintainer would add (`src/arch/hip.rs`) is in INTEGRATION.md.
 *
 * Conventions
 *  - Plain pointers and sizes only.  Host buffers are owned by the caller;
 *    device buffers are owned by the library behind opaque handles.
 *  - Every function returns an int status: 0 = ok, < 0 = error.  The message
 *    of the last error on the calling thread is returned by iris_last_error().
 *    (The reference panics on `assert_eq!(out.len(), db.len())`,
 *    src/lib.rs:43,70; the Rust shim maps IRIS_E_ARG back to that panic.)
 *  - All calls are blocking: when they return, host outputs are filled, as the
 *    reference's synchronous `batch_process` (src/lib.rs:42,69).
 *  - Handles are thread-safe: calls on one device are serialised internally
 *    (the reference engines are `Sync` and shared by rayon workers).
 *  - Calls switch to their handle's device internally and leave the calling
 *    thread's current HIP device as they found it.
 *  - Record layouts are the reference's in-memory / on-disk layouts
 *    (bytemuck views, little-endian):
 *      Bits        = uint64_t[200]            (src/bits.rs:13-15)      1600 B
 *      EncodedBits = uint16_t[12800]          (src/encoded_bits.rs:13-15) 25600 B
 *      Template    = { Bits pattern; Bits mask; } (src/template.rs:11-29) 3200 B
 *    On the device the library keeps its own lane-interleaved layout
 *    (DESIGN.md §3); conversion happens on upload / read-back.
 */
#ifndef IRIS_HIP_H
#define IRIS_HIP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Geometry: src/lib.rs:10-12, src/bits.rs:10-11 */
#define IRIS_COLS 200
#define IRIS_ROWS 64
#define IRIS_BITS 12800
#define IRIS_LIMBS 200
#define IRIS_ROTATIONS 31   /* r = k - 15, k = 0..30 (src/lib.rs:34,61) */
#define IRIS_MAX_ROTATION 15

/* Status codes */
#define IRIS_OK 0
#define IRIS_E_ARG (-1)       /* bad argument / length mismatch            */
#define IRIS_E_HIP (-2)       /* HIP runtime error                          */
#define IRIS_E_NOMEM (-3)     /* device or host allocation failed          */
#define IRIS_E_NODEV (-4)     /* no usable gfx950 device                    */
#define IRIS_E_RANGE (-5)     /* index range outside the database          */
#define IRIS_E_IO (-6)        /* file open / read / write failed            */
#define IRIS_E_FORMAT (-7)    /* malformed JSON template file               */

/* Database record kinds */
#define IRIS_KIND_MASKS 1     /* records are Bits (the resolver's masks file, src/main.rs:455-469) */
#define IRIS_KIND_SHARES 2    /* records are EncodedBits (a participant's share file, src/main.rs:386-400) */
#define IRIS_KIND_TEMPLATES 3 /* records are Template (plaintext masked Hamming, src/template.rs) */

/* Device layouts of a database (iris_db_create_ex) */
#define IRIS_LAYOUT_DEFAULT 0 /* TILES                                          */
#define IRIS_LAYOUT_LANES 1   /* record-per-lane blocks of 64 (VALU kernels)   */
#define IRIS_LAYOUT_TILES 2   /* 32-record MFMA tiles (fp4 / i8 kernels)        */
/* (3 was the search-only TRITS template layout of rounds 2-3; removed, refused as unknown) */

typedef struct iris_template {
    uint64_t pattern[IRIS_LIMBS];
    uint64_t mask[IRIS_LIMBS];
} iris_template_t;

/* Result of a search: the reference resolver's (min_distance, min_index)
 * pair (src/main.rs:581-582, 616-621) plus the exact fraction behind it.   */
typedef struct iris_match {
    double distance;   /* f64 value, +inf when no template has a valid rotation */
    uint64_t index;    /* global template index; UINT64_MAX when distance is +inf */
    uint32_t num;      /* uneq count of the winning rotation                   */
    uint32_t den;      /* jointly-valid bit count of the winning rotation      */
    int32_t rotation;  /* winning r in -15..15 (lowest r on ties); 0 if none   */
    uint32_t reserved;
} iris_match_t;

typedef struct iris_device iris_device_t;
typedef struct iris_db iris_db_t;
typedef struct iris_engine iris_engine_t;
typedef struct iris_pending iris_pending_t;

/* ---------------------------------------------------------------- errors */
const char *iris_last_error(void);
const char *iris_version(void);
/* Runtime configuration, read from the environment once when a device opens:
 * "key=value ..." into buf (NUL-terminated, truncated to len); *needed (may be
 * NULL) receives the full length without the NUL.  dev == NULL: what a device
 * opened now would use.  Production knobs: IRIS_READAHEAD, IRIS_AUTO_RESIDENT,
 * IRIS_GROUP_TIMEOUT_MS, IRIS_COPY_HELPERS (process-wide).  Test-only hooks
 * (IRIS_TILES_PER_WAVE, IRIS_FUSED_REDUCE, IRIS_BATCH_KERNEL, IRIS_SCHEDULE,
 * IRIS_LOAD_PREAD, IRIS_LOAD_WINDOWS, IRIS_GROUP_DELAY_US, IRIS_GROUP_STALL,
 * IRIS_GROUP_UNORDERED, IRIS_UPLOAD, IRIS_READAHEAD_WINDOW, IRIS_RESIDENT_BUDGET_MB,
 * IRIS_READAHEAD_PACKED, IRIS_READAHEAD_WINDOW_MAX) take effect only with IRIS_TEST_HOOKS=1;
 * otherwise they are ignored and listed as "ignored=...".  With dev != NULL the
 * device's own facts follow: numa_node= (host NUMA node of its PCI function, -1
 * unknown), upload_gbps=P/R (recent rates of large writes through the pinned
 * slots / the runtime's copy, GB/s; 0 = not measured yet), resident= (the
 * record files it keeps resident for host-slice calls: count and bytes) and
 * readahead_windows=L/R/M (read-ahead launches of host-output engine calls since
 * the last iris_device_reset_stats, the records they computed, the largest
 * window in records) and abandoned_inits=P/T (RCCL communicator inits of this
 * device that a group formation gave up on at its bound: still pending inside
 * RCCL / all in this process; while one is pending the device forms no further
 * multi-rank group in this process).  group_init_timeout_ms= is the bound of
 * forming a group (IRIS_GROUP_TIMEOUT_MS, else 120000). */
int iris_config(const iris_device_t *dev, char *buf, size_t len, size_t *needed);

/* --------------------------------------------------------------- devices */
int iris_device_count(int *count);
/* Opens a HIP device (must be gfx950).  Owns one non-blocking HIP stream. */
int iris_device_open(int ordinal, iris_device_t **out);
int iris_device_close(iris_device_t *dev);
int iris_device_synchronize(iris_device_t *dev);
/* The device's stream as a hipStream_t, for callers that order their own work. */
int iris_device_stream(iris_device_t *dev, void **stream);
/* Free and total device memory in bytes (sizing a resident database: a template
 * takes 3200 B, a mask 1600 B, a share 25600 B; the reference mmaps its files
 * instead, src/main.rs:389,458). */
int iris_device_memory(iris_device_t *dev, size_t *free_bytes, size_t *total_bytes);
/* Kernel timing with HIP events recorded on the device stream around every
 * launch of the named kernel family ("template_search", "template_counts",
 * "masks", "shares", ...).  Disabled by default. */
int iris_device_set_profiling(iris_device_t *dev, int enabled);
int iris_device_kernel_stats(iris_device_t *dev, const char *kernel, uint64_t *launches,
                             double *total_ms, uint64_t *items);
/* The largest launch of the named kernel family since the last reset: its items
 * (records) and its duration (ms; the latest of equal-sized ones); 0 / 0 if none.
 * A walk's biggest read-ahead window, for its HBM fraction. */
int iris_device_kernel_stats_largest(iris_device_t *dev, const char *kernel, uint64_t *items, double *ms);
int iris_device_reset_stats(iris_device_t *dev);
/* Raw device memory for outputs that stay on the GPU (e.g. per-template distances). */
int iris_device_alloc(iris_device_t *dev, size_t bytes, void **ptr);
int iris_device_free(iris_device_t *dev, void *ptr);
int iris_memcpy_d2h(iris_device_t *dev, void *host, const void *device, size_t bytes);
int iris_memcpy_h2d(iris_device_t *dev, void *device, const void *host, size_t bytes);

/* -------------------------------------------------------------- databases
 * Device-resident database of `kind` records.  Replaces the mmap'd share /
 * masks files the reference keeps in host memory (src/main.rs:389,458).     */
int iris_db_create(iris_device_t *dev, int kind, uint64_t capacity, iris_db_t **out);
/* As iris_db_create with an explicit device layout (IRIS_LAYOUT_*).  The
 * layout only selects the kernel family; results are identical. */
int iris_db_create_ex(iris_device_t *dev, int kind, uint64_t capacity, int layout, iris_db_t **out);
int iris_db_layout(const iris_db_t *db, int *layout);
int iris_db_destroy(iris_db_t *db);
int iris_db_len(const iris_db_t *db, uint64_t *len);
int iris_db_capacity(const iris_db_t *db, uint64_t *cap);
int iris_db_kind(const iris_db_t *db, int *kind);
/* Appends n host records (reference layout) at the end. */
int iris_db_append(iris_db_t *db, const void *records, uint64_t n);
/* Overwrites records [index, index+n) (must lie inside [0, len]) — grows len if needed. */
int iris_db_write(iris_db_t *db, uint64_t index, const void *records, uint64_t n);
/* Reads records [first, first+n) back to the reference layout. */
int iris_db_read(const iris_db_t *db, uint64_t first, uint64_t n, void *records);
/* Appends n synthetic records generated on the device by the counter-based
 * generator of DESIGN.md §5 (template index t = global_index0 + i): uniform
 * random bits / u16 as the reference's `rng.gen()` (src/bits.rs:95-101,
 * src/encoded_bits.rs:81-87, src/template.rs:67-74). */
int iris_db_generate(iris_db_t *db, uint64_t n, uint64_t seed, uint64_t global_index0);
int iris_db_clear(iris_db_t *db);
/* Drops the records [len, current length) (no device work; later appends overwrite them). */
int iris_db_truncate(iris_db_t *db, uint64_t len);

/* ---------------------------------------------------------------- host residency
 * The reference's participant and resolver mmap their record file once and
 * call batch_process(out, chunk) on 20 000-record slices of the mapping
 * (src/main.rs:389-391, 426-431; 458-460, 511-516).  iris_db_attach_host
 * declares that db's records [0, n) are the n records of the host array at
 * `host` (e.g. that mapping): with upload != 0 the (empty) database receives
 * them now; with upload == 0 it must already hold exactly them (e.g. loaded
 * from the same file with iris_db_load_file; the first, middle and last
 * record are compared).  From then on iris_engine_batch_process_host on any
 * record range inside the array (same kind, whole records) runs the engine on
 * the resident copy and uploads nothing; other slices still upload.  The host
 * array must stay unchanged while attached; any write to the database
 * (append, write, generate, clear, truncate, load, prepare) or its
 * destruction detaches it. */
int iris_db_attach_host(iris_db_t *db, const void *host, uint64_t n, int upload);
int iris_db_detach_host(iris_db_t *db);

/* ---------------------------------------------------------------- on-disk formats
 * Record files hold the raw little-endian bytes of a record slice
 * (bytemuck::bytes_of): `prepare` writes them and `participant` / `resolver`
 * mmap them (src/main.rs:299-309,341,353-357,386-400,455-469):
 *   IRIS_KIND_MASKS      *.masks    Bits        1600 B
 *   IRIS_KIND_SHARES     *.share-i  EncodedBits 25600 B
 *   IRIS_KIND_TEMPLATES  raw Template (pattern then mask) 3200 B
 * iris_db_load_file appends records [first, first+count) of the file
 * (count = UINT64_MAX: to the end): the mapped file's page-cache pages are
 * registered with the device and copied by DMA in ~64-MB chunks, overlapping
 * the layout transpose (if registration fails, the range is read through two
 * pinned buffers by reader threads instead; IRIS_LOAD_PREAD=1 forces it); *loaded
 * (may be NULL) receives the number appended.  A file whose size is not a
 * multiple of the record size is rejected (IRIS_E_ARG), as the reference's
 * try_cast_slice does ("Share file … invalid.", src/main.rs:390-393,459-462). */
int iris_db_load_file(iris_db_t *db, const char *path, uint64_t first, uint64_t count, uint64_t *loaded);
/* Writes records [first, first+n) of db to `path` (created / truncated) in
 * the same raw format. */
int iris_db_save_file(const iris_db_t *db, const char *path, uint64_t first, uint64_t n);
/* JSON template files: a top-level array of {"pattern": hex, "mask": hex}
 * objects, each Bits the hex of its 1600 LE bytes (serde form of Template,
 * src/template.rs:11-29, src/bits.rs:74-93; read like the streaming
 * iter_json_array, src/json_stream.rs:53-60).  Read: up to cap templates go
 * to out (out may be NULL to count); *n is the number in the file;
 * IRIS_E_RANGE if it exceeds cap, IRIS_E_FORMAT with the byte offset on
 * malformed input.  Write: compact JSON, lowercase hex (hex::serialize). */
int iris_templates_read_json(const char *path, iris_template_t *out, uint64_t cap, uint64_t *n);
int iris_templates_write_json(const char *path, const iris_template_t *templates, uint64_t n);

/* ---------------------------------------------------------------- share preparation
 * The reference's `prepare` (src/main.rs:333-361) on the device: for the
 * templates [first, first+n) of a template database, appends n records to
 * each of the `parties` share databases — EncodedBits::share(parties) of
 * encode(template) (src/encoded_bits.rs:23-38, src/lib.rs:16-26): parties-1
 * uniformly random shares and a last one = encode - sum(rest) mod 2^16 —
 * and, if masks is not NULL, the template's mask to the masks database.
 * Randomness: ChaCha with `rounds` = 8, 12 or 20 (Bernstein's 64-bit-nonce
 * form) in counter mode under the caller's 256-bit key and 64-bit nonce (key
 * from a CSPRNG such as getrandom).  The reference uses rand 0.8.5's
 * thread_rng, a reseeded ChaCha12 (rand_chacha 0.3.1): 12 is its round count
 * and the recommended value.  Share j < parties-1 of global template index
 * g = index_base + first + i, elements 32b..32b+31 = the 32 LE u16 of
 * keystream block (g*(parties-1) + j)*400 + b.  Deterministic given
 * (key, nonce, g), so shards prepared on different GPUs never reuse a block. */
int iris_prepare_shares(const iris_db_t *templates, uint64_t first, uint64_t n, uint64_t index_base,
                        const uint8_t key[32], uint64_t nonce, uint32_t rounds, uint32_t parties,
                        iris_db_t *const *shares, iris_db_t *masks);

/* ---------------------------------------------------------------- engines
 * MasksEngine::new(&Bits)            src/lib.rs:60-67
 * DistanceEngine::new(&EncodedBits)  src/lib.rs:33-40
 * Template engine (query Template vs Template DB; src/template.rs:43-64)
 * Each builds the 31 rotated query copies once, as the reference does.     */
int iris_masks_engine_new(iris_device_t *dev, const uint64_t query_mask[IRIS_LIMBS], iris_engine_t **out);
int iris_distance_engine_new(iris_device_t *dev, const uint16_t query[IRIS_BITS], iris_engine_t **out);
int iris_template_engine_new(iris_device_t *dev, const iris_template_t *query, iris_engine_t **out);
int iris_engine_destroy(iris_engine_t *engine);

/* batch_process(&self, out: &mut [[u16; 31]], db: &[T])   src/lib.rs:42-52, 69-79
 * Masks engine: out[i][k] = dot_bool(rot(query_mask, k-15), db[i])
 * Distance engine: out[i][k] = dot_u16(rot(query, k-15), db[i])  (mod 2^16)
 * Device-resident form: processes db records [first, first+n); out is a host
 * array of n*31 uint16_t.  The engine kind must match the DB kind. */
int iris_engine_batch_process(iris_engine_t *engine, const iris_db_t *db, uint64_t first, uint64_t n,
                              uint16_t *out);
/* As iris_engine_batch_process, with out_device a DEVICE array of n*31
 * uint16_t (for pipelines that keep the results on the GPU).  Blocking: when
 * it returns the rows are in device memory, visible to any reader (another
 * stream, a copy engine, another process's mapping) -- a participant-sized
 * range returns on a completion word its kernel writes after storing the rows
 * through L2, before the launch itself has retired. */
int iris_engine_batch_process_device(iris_engine_t *engine, const iris_db_t *db, uint64_t first, uint64_t n,
                                     uint16_t *out_device);
/* Host-slice form with exactly the reference signature: `db` is a host array
 * of n reference-layout records, `out` a host array of n*31 uint16_t.  A slice
 * of an attached host array (iris_db_attach_host) runs on the resident copy.
 * A slice inside a read-only shared mapping of a regular file -- what the
 * participant and resolver walk (src/main.rs:386-391, 426-431; 455-460,
 * 511-516) -- runs on the device's copy of that file's records, made on first
 * use (read from the file in 256-MB granules, a call's missing ones and up to
 * 1 GB after them at once; a read that comes up short -- the file shrank --
 * drops the copy and the call uploads its slice) and kept.  Like the reference,
 * which maps the file once and treats it as immutable (src/main.rs:389; "Sync
 * from database" is a TODO at :402,415), the copy stands for the file as it was
 * read.  What every call re-checks: the file behind the mapping (device, inode,
 * size, mtime, ctime), so write(2), truncate, replace or rename-over, and a
 * mapping unmapped or replaced at the same address, drop the copy; the mapping's
 * file offset, at least every 200 ms; and three 64-byte snapshots of records in
 * the slice, which catch a change inside them whose timestamps did not move.
 * What it cannot see: stores through a writable MAP_SHARED mapping (this process's
 * or another's) into pages already dirty, which move no timestamp, outside the
 * three probed snapshots -- such records are served as they were read, for as
 * long as the copy lives.  A caller that changes its file that way calls
 * iris_device_drop_resident_range.  Copies are a cache: together at most
 * IRIS_RESIDENT_MAX_MB (default half the device), evicted least recently used
 * when a device allocation would fail, freed when their mapping is gone.  Files
 * that do not fit and IRIS_AUTO_RESIDENT=0 keep the upload path.  Any other
 * slice is uploaded (PCIe) and packed first. */
int iris_engine_batch_process_host(iris_engine_t *engine, const void *db, uint64_t n, uint16_t *out);
/* Frees the device's resident file copies (a failing iris_db_create does so too
 * before it retries); iris_config reports them as resident=count/bytes. */
int iris_device_drop_resident(iris_device_t *dev);
/* Frees the resident copy of the file mapping that holds host address ptr (of any
 * record kind), and forgets a refusal of that mapping: the next call on its slices
 * copies the file afresh.  For a caller that changed the file in a way the per-call
 * check does not see (stores through a writable shared mapping into pages already
 * dirty, see iris_engine_batch_process_host).  No copy there: nothing to do (0). */
int iris_device_drop_resident_range(iris_device_t *dev, const void *ptr);

/* Template engine, per template and rotation k: num = popcount((qp^ep)&qm&em),
 * den = popcount(qm&em) with q rotated by k-15 (src/template.rs:49-64).
 * num_out / den_out: host arrays of n*31 uint16_t (either may be NULL). */
int iris_template_counts(iris_engine_t *engine, const iris_db_t *db, uint64_t first, uint64_t n,
                         uint16_t *num_out, uint16_t *den_out);
/* Template::distance(query, db[i]) for each i (src/template.rs:43-47):
 * out is a host array of n doubles (bit-exact to the reference). */
int iris_template_distances(iris_engine_t *engine, const iris_db_t *db, uint64_t first, uint64_t n,
                            double *out);
/* Fused search: per-template distance + global min / argmin with the
 * resolver's strict-< lowest-index rule (src/main.rs:581-621).  Indices in
 * *out are global: db index + index_base.  dist_out_device (optional, may be
 * NULL) receives the n per-template distances in DEVICE memory. */
int iris_template_search(iris_engine_t *engine, const iris_db_t *db, uint64_t first, uint64_t n,
                         uint64_t index_base, double *dist_out_device, iris_match_t *out);

/* Pipelined form of iris_template_search (no reference counterpart: the
 * reference's calls block, src/lib.rs:42-53): enqueues the search and returns
 * at once; iris_pending_wait blocks for THAT search only and frees the handle,
 * so the next query's search can be enqueued (and its engine built) while the
 * caller exchanges or consumes this result.  The engine may be destroyed
 * before the wait; the database must stay alive and unmodified until it. */
int iris_template_search_async(iris_engine_t *engine, const iris_db_t *db, uint64_t first, uint64_t n,
                               uint64_t index_base, iris_pending_t **out);
int iris_pending_wait(iris_pending_t *pending, iris_match_t *out);

/* Batched queries (BASELINE configs[2]): nq query Templates searched against
 * one TILES template database in one pass; out[q] is query q's best match
 * (same rules as iris_template_search).  DB layout must be TILES, except for
 * nq <= 3, which runs as streaming passes over any layout. */
int iris_template_batch_engine_new(iris_device_t *dev, const iris_template_t *queries, uint32_t nq,
                                   iris_engine_t **out);
int iris_template_batch_search(iris_engine_t *engine, const iris_db_t *db, uint64_t first, uint64_t n,
                               uint64_t index_base, iris_match_t *out);

/* ---------------------------------------------------------------- resolver
 * The resolver's aggregation (src/main.rs:597-621) fused on the GPU: for each
 * entry i, num = wrapping sum over the `parts` participants' [u16;31] shares,
 * decode_distance(num, denoms[i]) (src/lib.rs:97-107), then the first entry
 * with a strictly smaller distance.  out->index = index_base + i, out->num =
 * the decoded uneq count, out->den = the denominator.  At most 8 parts.
 * Device form: all arrays are DEVICE arrays of n*31 uint16_t.            */
int iris_resolver_search(iris_device_t *dev, const uint16_t *const *shares_device, uint32_t parts,
                         const uint16_t *denoms_device, uint64_t n, uint64_t index_base, double *dist_out_device,
                         iris_match_t *out);
/* The resolver step with the denominators computed on the fly: `engine` is
 * the MasksEngine of the query mask, records [first, first+n) of the masks
 * database give the denominators (MasksEngine::batch_process, never written
 * to memory on the TILES layout), shares_device[p] are DEVICE arrays of n*31
 * uint16_t with row i belonging to record first+i (src/main.rs:510-519 +
 * 597-621 in one pass).  Same result as iris_resolver_search over the
 * engine's output; indices are i + index_base. */
int iris_resolver_search_masks(iris_engine_t *engine, const iris_db_t *masks_db, uint64_t first, uint64_t n,
                               const uint16_t *const *shares_device, uint32_t parts, uint64_t index_base,
                               double *dist_out_device, iris_match_t *out);
/* iris_resolver_search_masks with the participants' outputs in host memory (src/main.rs:510-519 +
 * 597-621: the rows as they arrive over the network; the reference's resolver computes the masks
 * denominators itself, here fused): shares[p] are host arrays of n x 31 u16, row i = record
 * first + i.  The parts are summed (wrapping u16) on the host while the previous chunk's sum is
 * copied and searched; blocking, one result; indices are i + index_base. */
int iris_resolver_search_masks_host(iris_engine_t *engine, const iris_db_t *masks_db, uint64_t first, uint64_t n,
                                    const uint16_t *const *shares, uint32_t parts, uint64_t index_base,
                                    iris_match_t *out);
/* Host form: shares[p] and denoms are host arrays, uploaded in chunks -- through the device's pinned
 * upload slots, overlapped with the kernels, or by the runtime's copy, whichever moved this
 * device's large host uploads faster lately (as for iris_db_write); blocking, one result. */
int iris_resolver_search_host(iris_device_t *dev, const uint16_t *const *shares, uint32_t parts,
                              const uint16_t *denoms, uint64_t n, uint64_t index_base, iris_match_t *out);

/* ------------------------------------------------------------ arch plugin
 * The reference's backend plugin point (src/arch/mod.rs:5):
 *   dot_bool(&[u64;200], &[u64;200]) -> u16   src/arch/generic.rs:4-9
 *   dot_u16(&[u16;12800], &[u16;12800]) -> u16 src/arch/generic.rs:11-16
 * Batched all-pairs form (the criterion shapes of src/arch/mod.rs:29,53):
 * out[j*na + i] = dot(a[i], b[j]) for i < na, j < nb. */
int iris_dot_bool_batch(iris_device_t *dev, const uint64_t *a, uint64_t na, const uint64_t *b, uint64_t nb,
                        uint16_t *out);
int iris_dot_u16_batch(iris_device_t *dev, const uint16_t *a, uint64_t na, const uint16_t *b, uint64_t nb,
                       uint16_t *out);

/* ------------------------------------------------- host-side value helpers
 * CPU implementations of the value-type operations the engines are built
 * from; they need no GPU. */
/* Bits::rotated (src/bits.rs:18-29,178-205): out[row,col] = in[row,(col-amount) mod 200] */
int iris_bits_rotated(const uint64_t in[IRIS_LIMBS], int32_t amount, uint64_t out[IRIS_LIMBS]);
/* EncodedBits::rotated (src/encoded_bits.rs:40-58) */
int iris_encoded_rotated(const uint16_t in[IRIS_BITS], int32_t amount, uint16_t out[IRIS_BITS]);
/* encode(&Template) (src/lib.rs:16-26): mask - 2*(pattern&mask) per bit as u16 */
int iris_encode(const iris_template_t *t, uint16_t out[IRIS_BITS]);
/* decode_distance(&[u16;31], &[u16;31]) -> f64 (src/lib.rs:97-107) */
int iris_decode_distance(const uint16_t distances[IRIS_ROTATIONS], const uint16_t denominators[IRIS_ROTATIONS],
                         double *out);
/* Diagnostics for the query tables an engine builds on the device
 * (iris_query.hip): iris_engine_query_tables copies an engine's rotated-query
 * table and MFMA fragments to the host; iris_host_query_tables builds the same
 * bytes with the host reference builders.  kind = IRIS_KIND_*; for
 * IRIS_KIND_TEMPLATES nq = 0 is a single-query engine and nq >= 4 the tiles of
 * a batched engine of nq queries (`query` = nq templates; `tab` unused).  The
 * sizes must be the layout's exactly (IRIS_E_ARG otherwise; see
 * iris_query_table_sizes). */
int iris_query_table_sizes(int kind, uint32_t nq, size_t *tab_bytes, size_t *frag_bytes);
int iris_engine_query_tables(const iris_engine_t *engine, void *tab, size_t tab_bytes, void *frag,
                             size_t frag_bytes);
int iris_host_query_tables(int kind, const void *query, uint32_t nq, void *tab, size_t tab_bytes, void *frag,
                           size_t frag_bytes);
/* Merges per-shard search results into the global one (min fraction, then
 * lowest index) — the cross-shard step of the resolver's argmin (src/main.rs:616-621). */
int iris_match_merge(const iris_match_t *records, uint64_t count, iris_match_t *out);

/* ------------------------------------------------------- device groups (multi-GPU)
 * The reference fans a query out to its participants and folds their answers
 * with a sequential strict-< minimum (src/main.rs:486-504, 616-621).  Here a
 * template database is split into contiguous shards across the gfx950 devices
 * of a group — shard s of S holds global records [s*N/S, (s+1)*N/S) — every
 * device searches its own shards with no data-path communication, and the
 * per-shard winners (24 B each, global indices) are exchanged with one RCCL
 * ncclAllGather over xGMI (librccl from /opt/rocm) and merged on every device
 * (exact fraction, then the lowest global index).
 *
 * Two ways to form a group:
 *  - iris_group_create: ONE process drives `n` devices (ncclCommInitAll's form:
 *    one id, every device a rank, created inside one RCCL group).
 *  - iris_group_create_rank: one device per process (e.g. a torchrun rank):
 *    rank 0 calls iris_group_unique_id and hands the 128 id bytes to every
 *    rank (any side channel); each rank then calls iris_group_create_rank with
 *    the same id.  Every rank makes the same group calls (SPMD); each holds
 *    and fills only its own shards.
 * Forming a group is bounded: RCCL's init (which blocks until every rank has
 * arrived) runs on a helper thread waited for at most IRIS_GROUP_TIMEOUT_MS
 * (default 120 s); if a peer never arrives the call fails (IRIS_E_HIP) instead
 * of hanging, the pending init is abandoned (it aborts its communicators should
 * it ever complete) and the device stays usable.  While such an init is still
 * pending, a multi-rank group on that device is refused at once (IRIS_E_HIP:
 * start a fresh process; iris_config's abandoned_inits counts them), so failed
 * formations cannot pile up in a long-lived process; 1-rank groups still form.
 * A formed group all-gathers
 * every rank's PCI bus id over its communicators (iris_group_rccl_info).
 * Group calls are blocking and serialised per group, like the device calls.
 *
 * Failure: waiting for an exchange is bounded.  The clock starts when every
 * local device has reached the all-gather (only the peers can hold it up) and
 * RCCL's asynchronous error is polled meanwhile; on expiry or error the
 * group's communicators are aborted (ncclCommAbort), the call returns
 * IRIS_E_HIP, and every later call on the group or its databases fails the
 * same way (the destroys excepted).  A rank whose own enqueue fails aborts too,
 * so its peers see an error rather than a hang.  Bound: IRIS_GROUP_TIMEOUT_MS,
 * iris_group_set_timeout, else max(30 s, 10 x the call's local work). */
#define IRIS_GROUP_ID_BYTES 128
typedef struct iris_group iris_group_t;
typedef struct iris_group_db iris_group_db_t;
typedef struct iris_group_pending iris_group_pending_t;

int iris_group_create(const int *ordinals, uint32_t n, iris_group_t **out);
int iris_group_unique_id(uint8_t id[IRIS_GROUP_ID_BYTES]);
int iris_group_create_rank(int ordinal, uint32_t nranks, uint32_t rank, const uint8_t id[IRIS_GROUP_ID_BYTES],
                           iris_group_t **out);
int iris_group_destroy(iris_group_t *group);
/* ms > 0: the exchange wait bound of this group's later calls; 0: automatic. */
int iris_group_set_timeout(iris_group_t *group, uint32_t ms);
/* local_devices: devices this process drives; ranks: RCCL ranks in the group
 * (all processes); first_rank: the rank of local device 0. */
int iris_group_info(const iris_group_t *group, uint32_t *local_devices, uint32_t *ranks, uint32_t *first_rank);
/* What RCCL itself reports for the group: *comm_ranks = ncclCommCount of its
 * communicators, and (bus_ids may be NULL; len >= ranks * IRIS_GROUP_BUS_ID_BYTES)
 * every rank's device PCI bus id ("0000:05:00.0", NUL-terminated) at
 * bus_ids + rank * IRIS_GROUP_BUS_ID_BYTES, gathered over the group's own RCCL
 * all-gather when it formed. */
#define IRIS_GROUP_BUS_ID_BYTES 32
int iris_group_rccl_info(const iris_group_t *group, uint32_t *comm_ranks, char *bus_ids, size_t len);
/* Local device i of the group (borrowed: valid until iris_group_destroy), e.g.
 * for iris_device_set_profiling / iris_device_kernel_stats. */
int iris_group_device(const iris_group_t *group, uint32_t i, iris_device_t **dev);

/* A sharded database of `total` records of `kind` over the whole group:
 * S = ranks * shards_per_device contiguous shards (shards_per_device >= 1;
 * more than one splits a device's range into several shards, each searched
 * and exchanged separately).  Every record starts empty (a zero mask: never a
 * candidate, as the reference's NaN rows, src/lib.rs:105-106).  layout as
 * iris_db_create_ex.  A process holds the shards of its local devices. */
int iris_group_db_create(iris_group_t *group, int kind, uint64_t total, int layout, uint32_t shards_per_device,
                         iris_group_db_t **out);
int iris_group_db_destroy(iris_group_db_t *gdb);
/* total records; S = shards in the group; the local shards are [first_shard, first_shard + local_shards). */
int iris_group_db_info(const iris_group_db_t *gdb, uint64_t *total, uint32_t *shards, uint32_t *first_shard,
                       uint32_t *local_shards);
/* Local shard i (0 <= i < local_shards): its database (borrowed; searchable with
 * the single-device calls) and the global index of its record 0. */
int iris_group_db_shard(const iris_group_db_t *gdb, uint32_t i, iris_db_t **db, uint64_t *first, uint64_t *count);
/* Fills every local shard with the synthetic records of iris_db_generate
 * (generator index = global index), all local devices in parallel. */
int iris_group_db_generate(iris_group_db_t *gdb, uint64_t seed);
/* records = host records of the global range [index, index+n) (reference
 * layout); the part held by this process's shards is written. */
int iris_group_db_write(iris_group_db_t *gdb, uint64_t index, const void *records, uint64_t n);
/* Reads the global range [index, index+n) back; it must lie in local shards. */
int iris_group_db_read(const iris_group_db_t *gdb, uint64_t index, uint64_t n, void *records);
/* Global record i <- record first+i of a raw record file (iris_db_load_file's
 * formats and DMA path), local shards only, all local devices in parallel; the
 * file must hold first + total records (IRIS_E_RANGE otherwise). */
int iris_group_db_load_file(iris_group_db_t *gdb, const char *path, uint64_t first);

/* 1 query against the whole sharded template database: on every device the
 * query's engine is built, each local shard searched, the winners all-gathered
 * over RCCL and merged; *out = the global (min distance, lowest index) as
 * iris_template_search over the concatenated database (index = global). */
int iris_group_template_search(iris_group_db_t *gdb, const iris_template_t *query, iris_match_t *out);
/* Pipelined form: enqueues the search, the exchange and the merge, returns at
 * once; wait blocks for THAT search and frees the handle (every local device
 * must agree on the merged winner, IRIS_E_HIP otherwise). */
int iris_group_template_search_async(iris_group_db_t *gdb, const iris_template_t *query, iris_group_pending_t **out);
int iris_group_pending_wait(iris_group_pending_t *pending, iris_match_t *out);
/* nq queries in one pass per shard (iris_template_batch_search rules: TILES
 * layout for nq > 3); out[q] = query q's global winner. */
int iris_group_template_batch_search(iris_group_db_t *gdb, const iris_template_t *queries, uint32_t nq,
                                     iris_match_t *out);

#ifdef __cplusplus
}
#endif
#endif /* IRIS_HIP_H */
