// iris_handles.hpp — opaque handle structs of the C ABI and the helpers the
// API translation units share (errors, workspaces, timed launches).
#pragma once
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <functional>
#include <map>
#include <mutex>
#include <string>
#include <vector>

#include "iris_internal.hpp"

using iris::KindInfo;

// ------------------------------------------------------------------ errors

inline thread_local std::string g_err;

inline int fail(int code, const std::string &msg) {
    g_err = msg;
    return code;
}

#define HIPCHK(x)                                                                                   \
    do {                                                                                            \
        hipError_t e_ = (x);                                                                        \
        if (e_ != hipSuccess) return fail(IRIS_E_HIP, std::string(#x) + ": " + hipGetErrorString(e_)); \
    } while (0)

#define CHK(x)                   \
    do {                         \
        int rc_ = (x);           \
        if (rc_ != 0) return rc_; \
    } while (0)

#define ARG(cond, msg)                                    \
    do {                                                  \
        if (!(cond)) return fail(IRIS_E_ARG, (msg));      \
    } while (0)

// ------------------------------------------------------------------ handles

struct KStat {
    uint64_t launches = 0, items = 0;
    double ms = 0;
    uint64_t max_items = 0;  // the largest launch (the latest of equal ones) and its duration
    double max_ms = 0;
};

struct Pending {
    std::string name;
    hipEvent_t a, b;
    uint64_t items;
};

struct DevBuf {
    void *p = nullptr;
    size_t cap = 0;
};

constexpr int kUploadRing = 2;  // pinned upload slots per device (db_write_pinned)

// The path of a device's large writes (db_write_locked): the helper threads' pinned slots (0) or the
// runtime's copy of the pageable source (1).  Which is faster depends on the caller's array -- the
// runtime's copy ran some arrays at 29-30 GB/s and others at 53, the slots both at 48-52
// (profiles/r04_host_upload.txt, r04_upload_participant.txt) -- so each path's recent rate is kept
// (EWMA) and the faster one taken, the other re-measured every 16th write.
struct UploadTune {
    double gbps[2] = {0, 0};  // bytes per second, EWMA
    uint32_t n[2] = {0, 0};
    uint64_t writes = 0;
    bool no_pinned = false;  // the slots' pinned buffers could not be allocated
    // each path is taken twice before the two are compared: its first use pays one-time setup (the
    // pinned slots' allocation, ~ms) and is not counted
    int pick() {
        const uint64_t w = writes++;
        if (no_pinned) return 1;
        if (n[0] < 2) return 0;
        if (n[1] < 2) return 1;
        const int best = gbps[0] >= gbps[1] ? 0 : 1;
        return w % 16 == 15 ? best ^ 1 : best;
    }
    void record(int p, double rate) {
        if (n[p]++ == 0) return;
        gbps[p] = n[p] == 2 ? rate : 0.75 * gbps[p] + 0.25 * rate;
    }
};

struct iris_device {
    int ordinal = 0;
    int numa_node = -1;  // host NUMA node of the device's PCI function (-1: unknown)
    iris::Hooks hooks;  // environment knobs, read once when the device opened
    hipStream_t stream = nullptr;
    std::recursive_mutex mu;
    bool profiling = false;
    std::map<std::string, KStat> stats;
    std::vector<Pending> pending;
    std::vector<hipEvent_t> event_pool;
    DevBuf partials, result, staging, out_a, out_b;
    DevBuf tempdb;  // the host-slice calls' transient database (TempDb, iris_api.hip)
    // zeroed device word of the fused (last-workgroup) search reduce; searches on the stream
    // are serialised, and each launch leaves it zeroed
    DevBuf ticket;
    // pinned host words the reduce kernels write their final Partials into (no
    // device-to-host copy between the last kernel and the stream sync)
    void *host_result = nullptr;
    size_t host_result_cap = 0;
    // coherent pinned word a blocking small search's last workgroup stores its sequence
    // number into after its result (iris::FusedFinish::done); the host spins on it
    uint32_t *host_done = nullptr;
    uint32_t done_seq = 0;
    // pinned result slots of asynchronous searches (iris_template_search_async)
    std::vector<iris::Partial *> free_slots;
    std::vector<void *> slot_blocks;
    // asynchronous searches reduce on a side stream, so the next search starts as soon as
    // this one's kernel ends: partials alternate between two buffers, each guarded by the
    // event recorded after the last reduce that read it (created on first use)
    hipStream_t aux = nullptr;
    // read-ahead windows alternate between aux (buffer 0) and aux2 (buffer 1), so that a window's
    // kernel starts on the CUs the one before it leaves while it drains (created with aux)
    hipStream_t aux2 = nullptr;
    DevBuf apart[2];
    hipEvent_t apart_read[2] = {nullptr, nullptr}, apart_written[2] = {nullptr, nullptr};
    int apart_next = 0;
    // handles alive on this device (1 for the device handle itself + 1 per database
    // and engine handle): the device is torn down when the last one is released,
    // so handles may be destroyed in any order
    std::atomic<int> refs{1};
    // freed engines' query buffers, reused by later engines (stream-ordered)
    std::vector<std::pair<size_t, void *>> qpool;
    // freed engines' pinned read-ahead row buffers (the participant builds an engine per request)
    std::vector<std::pair<size_t, void *>> rows_pool;
    // pinned slots of large database writes (db_write_pinned): the host fills one while the copy
    // engine drains the others; upin_ev[b] is recorded after the copy that read upin[b]
    void *upin[kUploadRing] = {};
    size_t upin_cap = 0;
    hipEvent_t upin_ev[kUploadRing] = {};
    UploadTune upload_tune;
    UploadTune resolver_tune;  // the same choice for iris_resolver_search_host (its pinned path sums the parts)
    // recorded on the device stream before every read-ahead launch and waited for by the side
    // stream: the launch follows whatever the device stream holds (the engine's query build,
    // writes to the database)
    hipEvent_t ra_order = nullptr;
    // databases attached to a host array (iris_db_attach_host): host-slice engine calls
    // on a range inside one of them run on the resident copy
    std::vector<struct iris_db *> attached;
    // read-only file mappings kept resident for host-slice calls (iris_resident.hip), the address
    // ranges found ineligible, and the use counter of their LRU eviction
    std::vector<struct Resident *> resident;
    struct NotResident {
        uintptr_t lo, hi;
        std::chrono::steady_clock::time_point until;  // re-examined after this (memory frees, addresses get reused)
    };
    std::vector<NotResident> not_resident;
    uint64_t resident_clock = 0;
    std::string resident_skip;  // why the last mapping refused was not made resident (iris_config)
    // the copy a host-slice call is running on (or filling): never evicted under it (PinResident)
    const struct iris_db *resident_pin = nullptr;
    std::chrono::steady_clock::time_point resident_swept{};  // last sweep for copies of vanished mappings
    // read-ahead launches, the records they computed and the largest window, since the last
    // iris_device_reset_stats (iris_config "readahead_windows")
    uint64_t ra_launches = 0, ra_records = 0, ra_window_max = 0;
};

struct iris_db {
    iris_device *dev = nullptr;
    KindInfo k{};
    uint64_t len = 0, cap = 0;
    void *data = nullptr;
    // iris_db_attach_host: records [0, host_n) equal the host array at host_base
    uintptr_t host_base = 0;
    uint64_t host_n = 0;
    // process-unique, renewed by every change of the records (db_detach) and every attachment:
    // an engine's read-ahead rows are valid for one version of one database
    uint64_t version = 0;
};

inline uint64_t next_db_version() {
    static std::atomic<uint64_t> v{0};
    return ++v;
}

// Read-ahead of a masks / distance engine's host-output calls (host slices of an attached or
// resident file array, iris_engine_batch_process_host, or ranges of a resident database,
// iris_engine_batch_process): the reference's participant and resolver walk their file in
// consecutive 20 000-record chunks (src/main.rs:427-431, 511-516), so while the rows of one window
// of chunks are copied to the caller, the engine already computes the next window on the device's
// side stream, its kernel storing the rows straight into the other of two pinned host buffers; a
// call whose range lies in a window of the same version of the same database only copies its rows
// out.  Speculation starts with the second consecutive call.
struct Readahead {
    struct Window {
        const struct iris_db *db = nullptr;
        uint64_t version = 0, first = 0, n = 0;  // the records whose rows rows[b] holds (once computed[b])
        bool live = false;
    };
    Window win[2];
    void *rows[2] = {nullptr, nullptr};      // pinned host [n][31] u16 rows
    size_t cap = 0;                          // bytes of each
    hipEvent_t computed[2] = {nullptr, nullptr};  // after the kernel into rows[b], on stream on[b]
    hipStream_t on[2] = {nullptr, nullptr};      // the stream of the last kernel into rows[b]
    // the previous call's range end: a call that starts there (or was read ahead) is part of a
    // walk, and only then is the next window computed speculatively (a random-access caller
    // never pays for rows it does not ask for)
    const struct iris_db *last_db = nullptr;
    uint64_t last_version = 0, last_end = 0;
    uint64_t grow = 0;  // records of the walk's latest window (the next one is twice its chunks)
};

struct iris_engine {
    iris_device *dev = nullptr;
    int kind = 0;             // IRIS_KIND_* of the DB it runs against
    void *qbuf = nullptr;     // one device allocation holding qtab, qfrag and the query
    size_t qbuf_bytes = 0;
    void *qtab = nullptr;     // SGPR rotated-query table (LANES kernels)
    void *qfrag = nullptr;    // MFMA query fragments (TILES kernels)
    uint32_t nq = 0;          // > 0: batched template engine (qfrag = nq padded query tiles)
    std::vector<iris_engine *> sub;  // streaming batched engine: one single-query engine per query
    Readahead ra;             // masks / distance engines: host-slice calls on attached databases
};

// Up to this many queries a batch runs as streaming passes over the database —
// two queries per pass (template_multi_kernel<2>), an odd last one alone —
// instead of the LDS-tiled GEMM (batch_kernel), which pads to groups of 4
// queries.  Measured per 10M templates: 2 queries 7.5 ms (GEMM 13.4 ms), 3
// queries 12.3 ms (GEMM ~14 ms); from 4 queries on the GEMM is ahead.
constexpr uint32_t kBatchStreamMax = 3;

namespace iris_api {

inline int set_device(iris_device *d) {
    HIPCHK(hipSetDevice(d->ordinal));
    return 0;
}

// The library switches to a handle's device for its own HIP calls; every entry point that may do so
// declares IRIS_KEEP_DEVICE() first, which puts the calling thread back on its own current device
// when the call returns (a C caller's or a framework's device choice is left as it was).
struct KeepDevice {
    int prev = -1;
    KeepDevice() {
        if (hipGetDevice(&prev) != hipSuccess) prev = -1;
    }
    ~KeepDevice() {
        if (prev >= 0) (void)hipSetDevice(prev);
    }
    KeepDevice(const KeepDevice &) = delete;
    KeepDevice &operator=(const KeepDevice &) = delete;
};
#define IRIS_KEEP_DEVICE() iris_api::KeepDevice keep_device_

// hipMalloc on the device; when it fails, resident file copies (iris_resident.hip, a cache) are
// evicted least recently used first -- never the one a call is running on -- and it is tried
// again.  IRIS_E_NOMEM once nothing is left to evict.  Caller holds the device lock.
int dev_malloc(struct iris_device *d, void **p, size_t bytes, const char *what);

inline int ensure(struct iris_device *d, DevBuf &b, size_t bytes) {
    if (bytes <= b.cap) return 0;
    if (b.p) HIPCHK(hipFree(b.p));
    b.p = nullptr;
    b.cap = 0;
    size_t want = std::max(bytes, (size_t)4096);
    CHK(dev_malloc(d, &b.p, want, "workspace"));
    b.cap = want;
    return 0;
}

// `bytes` of pinned, device-visible host memory for final results (grown on demand).
inline int ensure_host_result(iris_device *d, size_t bytes) {
    if (bytes <= d->host_result_cap) return 0;
    if (d->host_result) HIPCHK(hipHostFree(d->host_result));
    d->host_result = nullptr;
    d->host_result_cap = 0;
    const size_t want = std::max(bytes, (size_t)4096);
    // coherent: a fused search writes its winner through to it and the host reads it
    // while the kernel may still be retiring (search_locked)
    hipError_t e = hipHostMalloc(&d->host_result, want, hipHostMallocCoherent | hipHostMallocMapped);
    if (e != hipSuccess) return fail(IRIS_E_NOMEM, std::string("hipHostMalloc result: ") + hipGetErrorString(e));
    d->host_result_cap = want;
    return 0;
}

inline int ensure_host_done(iris_device *d) {
    if (d->host_done) return 0;
    void *p = nullptr;
    hipError_t e = hipHostMalloc(&p, 256, hipHostMallocCoherent | hipHostMallocMapped);
    if (e != hipSuccess) return fail(IRIS_E_NOMEM, std::string("hipHostMalloc done word: ") + hipGetErrorString(e));
    d->host_done = (uint32_t *)p;
    __atomic_store_n(d->host_done, 0u, __ATOMIC_RELEASE);
    return 0;
}

// Spins until the kernel enqueued last stores `seq` into d->host_done.  The stream is
// queried every few thousand polls, so a failed launch is reported rather than waited on.
inline int wait_done(iris_device *d, uint32_t seq) {
    for (uint32_t spins = 1;; ++spins) {
        if (__atomic_load_n(d->host_done, __ATOMIC_ACQUIRE) == seq) return 0;
        if ((spins & 4095) == 0) {
            const hipError_t q = hipStreamQuery(d->stream);
            if (q == hipSuccess) {
                if (__atomic_load_n(d->host_done, __ATOMIC_ACQUIRE) == seq) return 0;
                return fail(IRIS_E_HIP, "kernel completed without publishing its completion word");
            }
            if (q != hipErrorNotReady) return fail(IRIS_E_HIP, std::string("hipStreamQuery: ") + hipGetErrorString(q));
        }
        __builtin_ia32_pause();
    }
}

// A pinned host slot for one asynchronous search result (blocks of 256 slots).
inline int take_result_slot(iris_device *d, iris::Partial **slot) {
    if (d->free_slots.empty()) {
        constexpr int kSlots = 256;
        void *blk = nullptr;
        hipError_t e = hipHostMalloc(&blk, kSlots * sizeof(iris::Partial), hipHostMallocDefault);
        if (e != hipSuccess) return fail(IRIS_E_NOMEM, std::string("hipHostMalloc result slots: ") + hipGetErrorString(e));
        d->slot_blocks.push_back(blk);
        for (int i = kSlots - 1; i >= 0; --i) d->free_slots.push_back((iris::Partial *)blk + i);
    }
    *slot = d->free_slots.back();
    d->free_slots.pop_back();
    return 0;
}

inline hipEvent_t take_event(iris_device *d) {
    if (!d->event_pool.empty()) {
        hipEvent_t e = d->event_pool.back();
        d->event_pool.pop_back();
        return e;
    }
    hipEvent_t e = nullptr;
    if (hipEventCreate(&e) != hipSuccess) return nullptr;
    return e;
}

// Runs `launch` on the device stream, bracketed by HIP events when profiling.
template <class F>
int timed(iris_device *d, const char *name, uint64_t items, F &&launch, hipStream_t stream = nullptr) {
    if (!stream) stream = d->stream;
    hipEvent_t a = nullptr, b = nullptr;
    if (d->profiling) {
        a = take_event(d);
        b = take_event(d);
        if (a && b) HIPCHK(hipEventRecord(a, stream));
    }
    int rc = launch();
    if (rc != 0) return fail(IRIS_E_HIP, std::string("kernel launch failed: ") + name + ": " +
                                             hipGetErrorString(hipGetLastError()));
    if (d->profiling && a && b) {
        HIPCHK(hipEventRecord(b, stream));
        d->pending.push_back(Pending{name, a, b, items});
    }
    return 0;
}

// Folds the recorded kernel times whose end event has completed into the stats.
inline void fold_done(iris_device *d) {
    size_t keep = 0;
    for (size_t i = 0; i < d->pending.size(); ++i) {
        Pending &p = d->pending[i];
        float ms = 0;
        if (hipEventQuery(p.b) == hipSuccess && hipEventElapsedTime(&ms, p.a, p.b) == hipSuccess) {
            KStat &s = d->stats[p.name];
            s.launches += 1;
            s.ms += ms;
            s.items += p.items;
            if (p.items >= s.max_items) {
                s.max_items = p.items;
                s.max_ms = ms;
            }
            d->event_pool.push_back(p.a);
            d->event_pool.push_back(p.b);
        } else {
            d->pending[keep++] = p;
        }
    }
    d->pending.resize(keep);
}

// Waits for the stream, then folds recorded kernel times into the stats.
inline int sync(iris_device *d) {
    HIPCHK(hipStreamSynchronize(d->stream));
    if (d->aux) HIPCHK(hipStreamSynchronize(d->aux));
    if (d->aux2) HIPCHK(hipStreamSynchronize(d->aux2));
    fold_done(d);
    return 0;
}

inline constexpr size_t kStagingBytes = 256ull << 20;  // H2D/D2H staging per chunk

inline uint64_t chunk_records(const KindInfo &k) { return std::max<uint64_t>(64, kStagingBytes / k.rec_bytes / 64 * 64); }

inline int check_kind(int kind) {
    if (kind != IRIS_KIND_MASKS && kind != IRIS_KIND_SHARES && kind != IRIS_KIND_TEMPLATES)
        return fail(IRIS_E_ARG, "unknown record kind");
    return 0;
}

// Any change to a database's records ends its host attachment (caller holds the device lock).
inline void db_detach(iris_db *db) {
    db->version = next_db_version();  // read-ahead rows of the old records no longer match
    if (!db->host_base) return;
    auto &v = db->dev->attached;
    v.erase(std::remove(v.begin(), v.end(), db), v.end());
    db->host_base = 0;
    db->host_n = 0;
}

inline int ensure_ticket(iris_device *d) {
    if (d->ticket.p) return 0;
    CHK(ensure(d, d->ticket, 4096));  // the top word + 8 sub-tickets 256 B apart (iris_device.hpp)
    HIPCHK(hipMemsetAsync(d->ticket.p, 0, 4096, d->stream));
    return 0;
}

inline int ensure_aux(iris_device *d) {
    if (!d->aux) HIPCHK(hipStreamCreateWithFlags(&d->aux, hipStreamNonBlocking));
    if (!d->aux2) HIPCHK(hipStreamCreateWithFlags(&d->aux2, hipStreamNonBlocking));
    return 0;
}

// Waits for the side streams (errors ignored: teardown paths)
inline void side_sync(iris_device *d) {
    if (d->aux) (void)hipStreamSynchronize(d->aux);
    if (d->aux2) (void)hipStreamSynchronize(d->aux2);
}

// Shared by the API translation units (defined in iris_api.hip).
void device_retain(iris_device *d);
void device_release(iris_device *d);  // tears the device down with its last handle
void engine_free(iris_engine *e);     // query buffer back to the device's pool (stream-ordered)
// single-query template engine (query passed by value to the build kernel); caller holds d->mu
int template_engine_locked(iris_device *d, const iris_template_t *query, iris_engine **out);
// Enqueues the search of [first, first+n) of db and its partials reduce; the winner (idx =
// range-relative index + idx_base) lands in `dst` (pinned host or device memory); nothing
// waits.  side = true: the reduce runs on the device's side stream over one of two
// alternating partials buffers, and `done` (if given) is recorded there after it.
// host_done / seq: the fused small-range form also stores seq into the coherent host word
// host_done after writing dst; *flagged reports whether that form ran (else nothing is stored).
int search_enqueue(iris_engine *e, const iris_db *db, uint64_t first, uint64_t n, double *dist_dev, iris::Partial *dst,
                   bool side = false, hipEvent_t done = nullptr, uint64_t idx_base = 0, uint32_t *host_done = nullptr,
                   uint32_t seq = 0, bool *flagged = nullptr);
// Fills dst with the source bytes [off, off + bytes) of a write; false on a read error (errno set).
using SlotFill = std::function<bool(void *dst, size_t off, size_t bytes)>;
// Stores host records [0, n) at database index `index` through two pinned 64-MB slots the helper
// threads fill (caller holds the device lock; the database is detached already); waits for the device.
// fill (optional) fills the slots instead of a copy from `records` (e.g. pread from a file).
// IRIS_E_NOMEM only before anything was written (the pinned slots or the staging buffer).
int db_write_pinned(iris_db *db, uint64_t index, const void *records, uint64_t n, const SlotFill *fill = nullptr);
// db_write's store without the detach: host records [0, n) at index (index <= len; grows len).
int db_store_locked(iris_db *db, uint64_t index, const void *records, uint64_t n);
// A host slice [ptr, ptr + n records of `kind`) inside a read-only shared mapping of a regular
// file: *db = the device's resident copy of that mapping's records (uploaded granule by granule
// on first use), *first = the slice's record index in it, *end = the end of the resident run
// from there (a read-ahead bound).  *db = nullptr: not such a slice, IRIS_AUTO_RESIDENT=0, or
// the file does not fit the device -- the caller uploads.  Caller holds the device lock.
int resident_slice(iris_device *d, int kind, const void *ptr, uint64_t n, iris_db **db, uint64_t *first,
                   uint64_t *end);
void resident_drop_all(iris_device *d);  // frees every resident copy (waits for the device's streams)
// frees the least recently used copy that no call is running on; false if there is none
bool resident_evict_one(iris_device *d);
// frees the copies whose mapping or file is gone (at most once a second unless forced)
void resident_sweep(iris_device *d, bool force = false);
// marks a resident copy as in use by the current call (no eviction frees it meanwhile)
struct PinResident {
    iris_device *d;
    const iris_db *prev;
    PinResident(iris_device *dev, const iris_db *db) : d(dev), prev(dev->resident_pin) { d->resident_pin = db; }
    ~PinResident() { d->resident_pin = prev; }
    PinResident(const PinResident &) = delete;
    PinResident &operator=(const PinResident &) = delete;
};
// frees the copy of the mapping holding p and forgets refusals of addresses there; true if one was freed
bool resident_drop_at(iris_device *d, uintptr_t p);
// count and device bytes of the resident copies, and how many check their file through a held
// descriptor (map_files unreadable)
void resident_stats(const iris_device *d, uint64_t *count, uint64_t *bytes, int *via_fd);
// Abandoned RCCL communicator inits of device `ordinal` in this process (iris_group.hip): still
// pending inside RCCL, and all since the process started
void abandoned_inits(int ordinal, uint64_t *pending, uint64_t *total);
// Partial (indices offset by base) -> iris_match_t; +inf / UINT64_MAX when none
void match_from(const iris::Partial &r, bool any, uint64_t base, iris_match_t *out);

}  // namespace iris_api
