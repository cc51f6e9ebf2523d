// iris_api.hip — the C ABI (include/iris_hip.h): devices, device-resident
// databases, engines, arch plugin entry points and host helpers.
//
// Every call is blocking and serialised per device (one HIP stream per
// device).  Errors never throw across the ABI: they return a negative status
// and set a thread-local message (iris_last_error).
#include <hip/hip_runtime.h>

#include <math.h>
#include <stdio.h>
#include <ctype.h>
#include <string.h>
#include <unistd.h>

#include <algorithm>
#include <chrono>
#include <map>
#include <mutex>
#include <new>
#include <string>
#include <vector>

#include "iris_internal.hpp"

using namespace iris;

#include "iris_handles.hpp"

using namespace iris_api;

namespace {

constexpr size_t kUploadSlot = 64ull << 20;  // bytes per pinned upload slot
constexpr int kUploadSlots = kUploadRing;                       // slots per device (iris_handles.hpp)
constexpr size_t kUploadPieceMin = 4ull << 20;  // a write is cut into at least 4 slots of at least this
constexpr size_t kUploadTuneMin = 8ull << 20;   // writes from this size choose their path by measurement (UploadTune)

// The device's pinned upload slots (kUploadSlot bytes each) and their events, allocated once.
int ensure_upin(iris_device *d) {
    if (d->upin_cap >= kUploadSlot) return 0;
    CHK(sync(d));  // no copy uses the old buffers any more
    for (int b = 0; b < kUploadSlots; ++b)
        if (d->upin[b]) HIPCHK(hipHostFree(d->upin[b]));
    for (int b = 0; b < kUploadSlots; ++b) d->upin[b] = nullptr;
    for (int b = 0; b < kUploadSlots; ++b) {
        const hipError_t e = hipHostMalloc(&d->upin[b], kUploadSlot, hipHostMallocDefault);
        if (e != hipSuccess) {
            d->upin[b] = nullptr;
            return fail(IRIS_E_NOMEM, std::string("hipHostMalloc upload buffer: ") + hipGetErrorString(e));
        }
    }
    for (int b = 0; b < kUploadSlots; ++b)
        if (!d->upin_ev[b]) HIPCHK(hipEventCreateWithFlags(&d->upin_ev[b], hipEventDisableTiming));
    d->upin_cap = kUploadSlot;
    return 0;
}

}  // namespace

// A large write through pinned slots: the helper threads copy each slot's records from the
// caller's pageable array into one of two pinned buffers, the copy engine moves it to one of two
// device staging slots and the pack kernel stores it, while the host already fills the other
// pinned buffer.  The runtime's copy of a pageable source ran at 29-30 GB/s for some caller arrays
// and 53 GB/s for others; this path moved 48-52 GB/s for both (profiles/r04_host_upload.txt).
// Writes of 8 MB and more take whichever of the two was faster lately (UploadTune);
// IRIS_UPLOAD=pinned|runtime (test hook) pins one.
int iris_api::db_write_pinned(iris_db *db, uint64_t index, const void *records, uint64_t n, const SlotFill *fill) {
    iris_device *d = db->dev;
    const KindInfo &k = db->k;
    // at least four slots per write (so the host's copy of one overlaps the copy engine's of another)
    const size_t piece = std::min(kUploadSlot, std::max(kUploadPieceMin, (size_t)n * k.rec_bytes / 4));
    const uint64_t ch = std::max<uint64_t>(64, piece / k.rec_bytes / 64 * 64);
    const size_t slot = (size_t)ch * k.rec_bytes;
    CHK(ensure_upin(d));  // host first: an IRIS_E_NOMEM with the slots in place is the device's
    CHK(ensure(d, d->staging, kUploadSlots * slot));
    int rc = 0;
    uint64_t c = 0;
    for (uint64_t done = 0; done < n && rc == 0; done += ch, ++c) {
        const uint64_t m = std::min<uint64_t>(ch, n - done);
        const int b = (int)(c % kUploadSlots);
        // pinned buffer b was last read by the copy of slot c - kUploadSlots (this call) or by the previous
        // call's copies (which ended with a sync)
        if (c >= (uint64_t)kUploadSlots && hipEventSynchronize(d->upin_ev[b]) != hipSuccess) {
            rc = fail(IRIS_E_HIP, "hipEventSynchronize");
            break;
        }
        if (fill) {
            if (!(*fill)(d->upin[b], (size_t)done * k.rec_bytes, (size_t)m * k.rec_bytes)) {
                rc = fail(IRIS_E_IO, "read failed (I/O error, or the file shrank under the load)");
                break;
            }
        } else {
            parallel_copy(d->upin[b], (const char *)records + done * k.rec_bytes, (size_t)m * k.rec_bytes, d->ordinal);
        }
        void *stage = (char *)d->staging.p + (size_t)b * slot;
        if (hipMemcpyAsync(stage, d->upin[b], (size_t)m * k.rec_bytes, hipMemcpyHostToDevice, d->stream) != hipSuccess) {
            rc = fail(IRIS_E_HIP, "hipMemcpyAsync upload");
            break;
        }
        if (hipEventRecord(d->upin_ev[b], d->stream) != hipSuccess) {
            rc = fail(IRIS_E_HIP, "hipEventRecord");
            break;
        }
        rc = timed(d, "pack", m, [&] { return launch_pack(d->stream, k, stage, db->data, index + done, m); });
    }
    const int rs = sync(d);  // the pinned buffers are free again when the call returns
    CHK(rc);
    CHK(rs);
    db->len = std::max(db->len, index + n);
    return 0;
}

namespace {

int db_write_runtime(iris_db *db, uint64_t index, const void *records, uint64_t n);

}  // namespace

int iris_api::db_store_locked(iris_db *db, uint64_t index, const void *records, uint64_t n) {
    iris_device *d = db->dev;
    if (index > db->len) return fail(IRIS_E_RANGE, "iris_db_write: index beyond the end of the database");
    if (n > db->cap - index) return fail(IRIS_E_RANGE, "iris_db_write: database capacity exceeded");
    if (n == 0) return 0;
    ARG(records != nullptr, "iris_db_write: records is NULL");
    const KindInfo &k = db->k;
    const size_t bytes = (size_t)n * k.rec_bytes;
    if (d->hooks.upload == 1 && bytes >= kUploadTuneMin) return db_write_pinned(db, index, records, n);
    if (d->hooks.upload == 0 && bytes >= kUploadTuneMin) {
        // the faster path for this caller's arrays, as measured on its recent writes
        UploadTune &u = d->upload_tune;
        const int path = u.pick();
        const auto t0 = std::chrono::steady_clock::now();
        int rc = path == 0 ? db_write_pinned(db, index, records, n) : db_write_runtime(db, index, records, n);
        if (rc == IRIS_E_NOMEM && path == 0 && d->upin_cap < kUploadSlot) {
            // no pinned host memory for the slots: the runtime's copy from now on (a device
            // allocation failure is the caller's error and leaves the tuner as it was)
            u.no_pinned = true;
            return db_write_runtime(db, index, records, n);
        }
        CHK(rc);
        u.record(path, (double)bytes / std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count());
        return 0;
    }
    return db_write_runtime(db, index, records, n);
}

namespace {

int db_write_locked(iris_db *db, uint64_t index, const void *records, uint64_t n) {
    db_detach(db);
    return db_store_locked(db, index, records, n);
}

// The runtime's copy of the pageable source, through one 256-MB staging chunk at a time.
int db_write_runtime(iris_db *db, uint64_t index, const void *records, uint64_t n) {
    iris_device *d = db->dev;
    const KindInfo &k = db->k;
    const uint64_t ch = chunk_records(k);
    CHK(ensure(d, d->staging, std::min<uint64_t>(n, ch) * k.rec_bytes));
    for (uint64_t done = 0; done < n; done += ch) {
        const uint64_t m = std::min<uint64_t>(ch, n - done);
        HIPCHK(hipMemcpyAsync(d->staging.p, (const char *)records + done * k.rec_bytes, m * k.rec_bytes,
                              hipMemcpyHostToDevice, d->stream));
        CHK(timed(d, "pack", m, [&] { return launch_pack(d->stream, k, d->staging.p, db->data, index + done, m); }));
        CHK(sync(d));  // staging is reused by the next chunk
    }
    db->len = std::max(db->len, index + n);
    return 0;
}

// A transient device DB holding host records (the host-slice engine forms).  Its memory is the
// device's cached workspace (grown on demand, kept until the device closes): a hipMalloc + hipFree
// per call cost a participant-sized upload call ~0.1 ms.  Callers hold the device lock.
struct TempDb {
    iris_db db;
};

int temp_db(iris_device *d, int kind, uint64_t cap, TempDb &t) {
    t.db.dev = d;
    t.db.k = kind_info(kind, IRIS_LAYOUT_TILES);
    t.db.cap = (cap + t.db.k.block - 1) / t.db.k.block * t.db.k.block;
    t.db.len = 0;
    const size_t bytes = std::max<uint64_t>(1, t.db.cap / t.db.k.block) * block_bytes(t.db.k);
    CHK(ensure(d, d->tempdb, bytes));
    t.db.data = d->tempdb.p;
    // the last block's records past the range stay zero (as a fresh database's)
    HIPCHK(hipMemsetAsync(t.db.data, 0, bytes, d->stream));
    return 0;
}

int range_ok(const iris_db *db, uint64_t first, uint64_t n) {
    if (first > db->len || n > db->len - first) return fail(IRIS_E_RANGE, "record range outside the database");
    return 0;
}

constexpr uint64_t kU16Chunk = 4ull << 20;  // records per engine launch of the host-output forms

// Enqueues the engine kernel over [first, first+n) of db, [n][31] u16 rows to the device buffer
// o, on `stream` (default: the device stream); nothing waits.  sig (TILES only): the kernel's
// completion word, if the kernel chosen signals one (sig->armed).
int enqueue_u16_engine(iris_engine *e, const iris_db *db, uint64_t first, uint64_t n, uint16_t *o,
                       hipStream_t stream = nullptr, DoneSignal *sig = nullptr, bool packed = false) {
    iris_device *d = e->dev;
    if (!stream) stream = d->stream;
    LaunchRange r{first, n};
    const bool tiles = db->k.layout == IRIS_LAYOUT_TILES;
    if (sig) sig->armed = false;
    if (e->kind == IRIS_KIND_MASKS)
        return timed(d, "masks", n, [&] {
            return tiles ? launch_masks_mfma(d->hooks, stream, db->data, e->qfrag, r, o, sig, packed)
                         : launch_masks(stream, db->data, e->qtab, r, o);
        }, stream);
    return timed(d, "shares", n, [&] {
        return tiles ? launch_shares_mfma(d->hooks, stream, db->data, e->qfrag, r, o, sig)
                     : launch_shares(stream, db->data, e->qtab, r, o);
    }, stream);
}

int run_u16_engine_pinned(iris_engine *e, const iris_db *db, uint64_t first, uint64_t n, uint16_t *out);

// Engine kernel over [first, first+n) of db, u16 [n][31] outputs to host.
int run_u16_engine(iris_engine *e, const iris_db *db, uint64_t first, uint64_t n, uint16_t *out) {
    iris_device *d = e->dev;
    if (db->k.layout == IRIS_LAYOUT_TILES) {
        // out of pinned host memory for the row buffers (nothing launched yet): the device-buffer form
        const int rc = run_u16_engine_pinned(e, db, first, n, out);
        if (rc != IRIS_E_NOMEM) return rc;
    }
    CHK(ensure(d, d->out_a, std::min<uint64_t>(n, kU16Chunk) * kRot * 2));
    for (uint64_t done = 0; done < n; done += kU16Chunk) {
        const uint64_t m = std::min<uint64_t>(kU16Chunk, n - done);
        CHK(enqueue_u16_engine(e, db, first + done, m, (uint16_t *)d->out_a.p));
        HIPCHK(hipMemcpyAsync(out + done * kRot, d->out_a.p, m * kRot * 2, hipMemcpyDeviceToHost, d->stream));
        CHK(sync(d));
    }
    return 0;
}

// ---- read-ahead of host-output engine calls (iris_handles.hpp, Readahead)

// calls of at most this many records (62 MB of rows per buffer) go through the read-ahead
constexpr uint64_t kReadaheadMax = 1ull << 20;
// A MasksEngine window's rows cross the host link packed (store_tile_packed, iris_device.hpp): 32 B
// per record, then an escape row of 31 u16 per record that only rows spanning more than a byte
// use; the copy-out expands them into the caller's [u16; 31] (parallel_expand).  The resolver's
// 20 000-mask walk is bound by its rows crossing the host link (~44 GB/s: 23 us of a 28-us call
// with the rows unpacked).
constexpr size_t kPackedRecBytes = 32;
bool ra_packed(const iris_engine *e) { return e->kind == IRIS_KIND_MASKS && e->dev->hooks.ra_packed; }
// bytes of a read-ahead buffer per record
size_t ra_rec_bytes(const iris_engine *e) { return ra_packed(e) ? kPackedRecBytes + kRot * 2 : kRot * 2; }

// A walk's read-ahead windows grow geometrically: the walk's first window is one chunk, each later
// one twice the chunks of the window before it, up to kWindowRecords records (and kWindowRowsMax of
// rows per buffer).  Consecutive windows run on two side streams, so a window's kernel starts on
// the CUs the one before it leaves while it drains: the ramp and drain of a launch (~74 us of a
// 100k-share window's 446 us on one stream, profiles/r05u_shares_window_kernels.txt) no longer
// call for big windows, and a call waits for its whole window, so windows beyond ~160k records
// only delay the host (a 3M-mask walk: 1.03e9 records/s from C++ with windows up to 880k,
// profiles/r06c_walk_host_masks.txt; measured per cap in profiles/r06d_window_caps.txt).
constexpr uint64_t kWindowRecords = 160000;
constexpr size_t kWindowRowsMax = 64ull << 20;

uint64_t window_chunks_max(const iris_db *db, uint64_t n) {
    uint64_t w = std::max<uint64_t>(1, kWindowRecords / n);
    if (db->dev->hooks.ra_window_max) w = db->dev->hooks.ra_window_max;  // test hook: another cap
    return std::max<uint64_t>(1, std::min<uint64_t>(w, kWindowRowsMax / ((size_t)n * kRot * 2)));
}

// Records of a walk's window of chunks of n records that follows a window of `prev` records (0: the
// walk's first window), with `avail` records left in the run.
uint64_t window_records(const iris_db *db, uint64_t n, uint64_t prev, uint64_t avail) {
    uint64_t w = prev ? 2 * ((prev + n - 1) / n) : 1;
    if (db->dev->hooks.ra_window) w = db->dev->hooks.ra_window;  // test hook: a fixed window
    w = std::min(w, window_chunks_max(db, n));
    return std::min<uint64_t>(w * n, avail);
}

// TILES databases only: their kernels store the rows as 16-B runs (store_tile_rows), which the
// host link takes well; the LANES kernels' 2-byte stores would each be a host-link write.
// IRIS_READAHEAD=0 turns it off (Hooks::readahead; tests run both forms).
bool readahead_ok(const iris_db *db, uint64_t n) {
    return db->dev->hooks.readahead && n <= kReadaheadMax && db->k.layout == IRIS_LAYOUT_TILES;
}

// Waits for the engine's read-ahead kernels (side streams): the row buffers may be reused or freed
// when this returns.  The windows' rows stay valid (a change of the database changes its version).
int ra_wait(iris_engine *e) {
    Readahead &ra = e->ra;
    if (!ra.computed[0]) return 0;
    iris_device *d = e->dev;
    if (d->aux) HIPCHK(hipStreamSynchronize(d->aux));
    if (d->aux2) HIPCHK(hipStreamSynchronize(d->aux2));
    if (ra.on[0] == d->stream || ra.on[1] == d->stream) HIPCHK(hipStreamSynchronize(d->stream));
    if (d->profiling) fold_done(d);
    return 0;
}

constexpr size_t kRowsPoolMax = 8;

// A pinned row buffer of at least `bytes` from the device's pool (at most twice the size), else new.
int rows_take(iris_device *d, size_t bytes, void **p, size_t *got) {
    for (size_t i = 0; i < d->rows_pool.size(); ++i) {
        const size_t b = d->rows_pool[i].first;
        if (b >= bytes && b <= 2 * bytes) {
            *p = d->rows_pool[i].second;
            *got = b;
            d->rows_pool.erase(d->rows_pool.begin() + i);
            return 0;
        }
    }
    const hipError_t err = hipHostMalloc(p, bytes, hipHostMallocDefault);
    if (err != hipSuccess) return fail(IRIS_E_NOMEM, std::string("read-ahead rows: ") + hipGetErrorString(err));
    *got = bytes;
    return 0;
}

// Back to the pool; a full pool frees its oldest buffer, so the sizes callers use now stay
// pooled (a pool full of another walk's sizes cost every later walk two hipHostMalloc and two
// hipHostFree of ~0.8 ms each, profiles/r05_rows_pool_trace.txt).
void rows_give(iris_device *d, void *p, size_t bytes) {
    if (!p) return;
    if (d->rows_pool.size() >= kRowsPoolMax) {
        (void)hipHostFree(d->rows_pool.front().second);
        d->rows_pool.erase(d->rows_pool.begin());
    }
    d->rows_pool.emplace_back(bytes, p);
}

// records per kernel of the pinned-rows form (62 MB of rows per buffer)
constexpr uint64_t kPinnedRowsChunk = 1ull << 20;

// The host-output form for TILES databases: each chunk's kernel stores its rows straight into one
// of two pinned host buffers (16-B runs over the host link, as the read-ahead does), and the helper
// threads copy them to `out` while the next chunk's kernel runs.  The copy engines' D2H into a
// caller's pageable array ran at 3-8 GB/s on some boxes (profiles/r03_host_rows.txt).  MasksEngine
// rows cross the link packed, as the read-ahead's do (ra_packed), and are expanded on the way out.
int run_u16_engine_pinned(iris_engine *e, const iris_db *db, uint64_t first, uint64_t n, uint16_t *out) {
    iris_device *d = e->dev;
    const uint64_t ch = std::min<uint64_t>(n, kPinnedRowsChunk);
    const bool pk = ra_packed(e);
    const size_t want = std::max<size_t>((size_t)ch * ra_rec_bytes(e), 4096);
    void *rows[2] = {nullptr, nullptr};
    size_t got[2] = {0, 0};
    hipEvent_t ev[2] = {nullptr, nullptr};
    const int nb = n > ch ? 2 : 1;
    int rc = 0;
    for (int b = 0; b < nb && rc == 0; ++b) {
        rc = rows_take(d, want, &rows[b], &got[b]);
        if (rc == 0 && !(ev[b] = take_event(d))) rc = fail(IRIS_E_HIP, "hipEventCreate failed");
    }
    // chunk c's rows go to rows[c & 1]; its kernel is enqueued before chunk c - 1's rows are
    // copied out, and rows[c & 1] was last read by the (synchronous) copy of chunk c - 2
    auto launch = [&](uint64_t c) -> int {
        const uint64_t a = c * ch, m = std::min<uint64_t>(ch, n - a);
        CHK(enqueue_u16_engine(e, db, first + a, m, (uint16_t *)rows[c & 1], nullptr, nullptr, pk));
        HIPCHK(hipEventRecord(ev[c & 1], d->stream));
        return 0;
    };
    const uint64_t chunks = (n + ch - 1) / ch;
    if (rc == 0) rc = launch(0);
    for (uint64_t c = 0; c < chunks && rc == 0; ++c) {
        if (c + 1 < chunks) rc = launch(c + 1);
        if (rc == 0 && hipEventSynchronize(ev[c & 1]) != hipSuccess) rc = fail(IRIS_E_HIP, "hipEventSynchronize");
        if (rc == 0) {
            const uint64_t a = c * ch, m = std::min<uint64_t>(ch, n - a);
            if (pk) {
                const uint8_t *p = (const uint8_t *)rows[c & 1];
                parallel_expand(out + a * kRot, p, (const uint16_t *)(p + m * kPackedRecBytes), m, d->ordinal);
            } else {
                parallel_copy(out + a * kRot, rows[c & 1], (size_t)m * kRot * 2, d->ordinal);
            }
        }
    }
    // on failure a kernel may still be storing into the buffers: drain before they go back
    if (rc != 0) (void)hipStreamSynchronize(d->stream);
    for (int b = 0; b < nb; ++b) {
        rows_give(d, rows[b], got[b]);
        if (ev[b]) d->event_pool.push_back(ev[b]);
    }
    if (rc == 0 && d->profiling) fold_done(d);
    return rc;
}

void ra_release(iris_engine *e) {
    Readahead &ra = e->ra;
    if (!ra.computed[0]) return;
    (void)hipSetDevice(e->dev->ordinal);
    (void)ra_wait(e);  // no kernel writes the buffers any more: they go back to the pool
    for (int b = 0; b < 2; ++b) {
        rows_give(e->dev, ra.rows[b], ra.cap);
        (void)hipEventDestroy(ra.computed[b]);
    }
    ra = Readahead{};
}

// Enqueues the engine kernel over [first, first+n) of db on the buffer's side stream (or the busy
// device stream, below); it stores
// the rows straight into the pinned buffer rows[b] (over the host link, no copy-engine DMA) and
// records computed[b]; win[b] describes them from now on.  rows[b] is not being read: the host
// copies out synchronously.  grow = false: if the buffers are too small, launch nothing
// (*launched = false) rather than reallocate them under the other window's rows.  New buffers
// hold at least `reserve` records' rows: a new engine's first call (one chunk) sizes them for the
// windows a walk from there goes on to, so they are not reallocated at its second call.
int ra_launch(iris_engine *e, const iris_db *a, uint64_t first, uint64_t n, int b, bool grow = true,
              bool *launched = nullptr, uint64_t reserve = 0) {
    Readahead &ra = e->ra;
    iris_device *d = e->dev;
    if (launched) *launched = false;
    CHK(ensure_aux(d));
    if (!ra.computed[0])
        for (int i = 0; i < 2; ++i) HIPCHK(hipEventCreateWithFlags(&ra.computed[i], hipEventDisableTiming));
    const size_t rec = ra_rec_bytes(e);
    const size_t bytes = (size_t)n * rec;
    if (bytes > ra.cap) {
        if (!grow) return 0;
        CHK(ra_wait(e));  // no kernel in flight writes either buffer
        for (int i = 0; i < 2; ++i) rows_give(d, ra.rows[i], ra.cap);
        ra.rows[0] = ra.rows[1] = nullptr;
        ra.win[0].live = ra.win[1].live = false;
        ra.cap = 0;
        const size_t want = std::max({bytes, (size_t)reserve * rec, (size_t)4096});
        size_t got[2] = {0, 0};
        for (int i = 0; i < 2; ++i) CHK(rows_take(d, want, &ra.rows[i], &got[i]));
        ra.cap = std::min(got[0], got[1]);
    }
    // ordered after everything enqueued on the device stream so far: the engine's query tables
    // (built there when the engine was created) and any write to the database.  An idle device
    // stream (the steady state of a chunk walk: its work is all on the side stream) needs no
    // event -- the cross-stream wait costs ~10 us per launch (profiles/r03_readahead.txt)
    // buffer b's windows run on their own side stream: the next window's kernel is not queued
    // behind this one's drain (the two write different buffers and only read the database)
    // An engine's first window goes on the device stream itself, behind its query tables (built
    // there just before): no query of the stream and no cross-stream event, which had cost 6-35 us
    // of a walk's first call (profiles/r06ae_first_call_phases.txt).  Nothing of the engine is in
    // flight then; by its next launch the call has waited for this window, and a busy device
    // stream orders the side stream after everything on it, this window included.
    hipStream_t side = b ? d->aux2 : d->aux;
    if (!ra.on[0] && !ra.on[1]) {
        side = d->stream;
    } else {
        const hipError_t idle = hipStreamQuery(d->stream);
        if (idle != hipSuccess) {
            if (idle != hipErrorNotReady) return fail(IRIS_E_HIP, std::string("hipStreamQuery: ") + hipGetErrorString(idle));
            if (!d->ra_order) HIPCHK(hipEventCreateWithFlags(&d->ra_order, hipEventDisableTiming));
            HIPCHK(hipEventRecord(d->ra_order, d->stream));
            HIPCHK(hipStreamWaitEvent(side, d->ra_order, 0));
        }
    }
    ra.win[b].live = false;
    ra.on[b] = side;
    CHK(enqueue_u16_engine(e, a, first, n, (uint16_t *)ra.rows[b], side, nullptr, ra_packed(e)));
    HIPCHK(hipEventRecord(ra.computed[b], side));
    ra.win[b] = Readahead::Window{a, a->version, first, n, true};
    d->ra_launches += 1;
    d->ra_records += n;
    d->ra_window_max = std::max(d->ra_window_max, n);
    if (launched) *launched = true;
    return 0;
}

// A host-output call on records [first, first+n) of db (records [0, end) exist).  Its rows come
// from a read-ahead window that holds them (same version of the same database), else they are
// computed now -- a whole window of consecutive chunks when the call continues a walk.  While a
// window's rows are copied out, the window after it is already computed into the other buffer
// (one launch of a growing number of chunks, window_records, on the other side stream), and a
// random-access caller never pays for rows it does not ask for.  The copy is the CPU's, split
// over helper threads: the copy engines' D2H of these 1.24 MB took 31 us on one box and
// 150-275 us (8 GB/s) on others, and queued behind the side stream's event it fell into the slow
// form on boxes that had the fast one (profiles/r03_host_rows.txt, r03_readahead.txt).
int readahead_u16_call(iris_engine *e, const iris_db *a, uint64_t first, uint64_t n, uint64_t end, uint16_t *out) {
    Readahead &ra = e->ra;
    iris_device *d = e->dev;
    auto holds = [&](int b) {
        const Readahead::Window &w = ra.win[b];
        return w.live && w.db == a && w.version == a->version && w.first <= first && first + n <= w.first + w.n;
    };
    int b = holds(0) ? 0 : holds(1) ? 1 : -1;
    // a walk: this call continues where the last one ended (or was read ahead for)
    const bool walk = b >= 0 || (ra.last_db == a && ra.last_version == a->version && ra.last_end == first);
    if (b < 0) {  // a miss: into the buffer whose window starts earlier (the one a walk has left)
        b = !ra.win[0].live ? 0 : !ra.win[1].live ? 1 : ra.win[0].first <= ra.win[1].first ? 0 : 1;
        // a walk's window follows the one the walk was in; a random-access call computes its range
        const uint64_t wn = walk ? window_records(a, n, ra.grow ? ra.grow : n, end - first) : n;
        // new buffers take the walk's largest window (not reallocated under it as the windows grow)
        const uint64_t reserve = std::min<uint64_t>(window_chunks_max(a, n) * n, end - first);
        CHK(ra_launch(e, a, first, std::max(wn, n), b, true, nullptr, reserve));
        ra.grow = std::max(wn, n);
    }
    const Readahead::Window w = ra.win[b];
    ra.last_db = a;
    ra.last_version = a->version;
    ra.last_end = first + n;
    // the walk's next window, into the other buffer (whose window the walk has left behind)
    const uint64_t next = w.first + w.n;
    if (walk && next < end) {
        const Readahead::Window &o = ra.win[b ^ 1];
        if (!(o.live && o.db == a && o.version == a->version && o.first == next)) {
            const uint64_t nn = window_records(a, n, w.n, end - next);
            bool launched = false;
            CHK(ra_launch(e, a, next, nn, b ^ 1, false, &launched));
            if (launched) ra.grow = nn;
        }
    }
    HIPCHK(hipEventSynchronize(ra.computed[b]));
    const uint64_t at = first - w.first;
    if (ra_packed(e)) {
        const uint8_t *pk = (const uint8_t *)ra.rows[b];
        parallel_expand(out, pk + at * kPackedRecBytes, (const uint16_t *)(pk + w.n * kPackedRecBytes) + at * kRot, n,
                        d->ordinal);
    } else {
        parallel_copy(out, (const char *)ra.rows[b] + (size_t)at * kRot * 2, (size_t)n * kRot * 2, d->ordinal);
    }
    if (d->profiling) fold_done(d);
    return 0;
}

constexpr size_t kQbufAlign = 256;
constexpr size_t kQpoolMax = 16;

inline size_t qalign(size_t b) { return (b + kQbufAlign - 1) / kQbufAlign * kQbufAlign; }

// A query buffer of at least `bytes`: a pooled one of up to twice the size, else hipMalloc.
int qbuf_take(iris_device *d, size_t bytes, void **p, size_t *got) {
    size_t best = SIZE_MAX, bi = 0;
    for (size_t i = 0; i < d->qpool.size(); ++i) {
        const size_t b = d->qpool[i].first;
        if (b >= bytes && b <= 2 * bytes && b < best) {
            best = b;
            bi = i;
        }
    }
    if (best != SIZE_MAX) {
        *p = d->qpool[bi].second;
        *got = best;
        d->qpool.erase(d->qpool.begin() + bi);
        return 0;
    }
    CHK(dev_malloc(d, p, bytes, "query buffer"));
    *got = bytes;
    return 0;
}

}  // namespace

void iris_api::engine_free(iris_engine *e) {
    if (!e) return;
    for (iris_engine *c : e->sub) engine_free(c);
    ra_release(e);
    if (e->qbuf) {
        iris_device *d = e->dev;
        // later users of the buffer are ordered after this engine's kernels on the device stream
        if (d->qpool.size() < kQpoolMax) d->qpool.emplace_back(e->qbuf_bytes, e->qbuf);
        else (void)hipFree(e->qbuf);
    }
    delete e;
}

namespace {

// A new engine whose query buffer holds [table | fragments | extra] (each 256-B aligned).
int engine_alloc(iris_device *dev, int kind, size_t tab_bytes, size_t frag_bytes, size_t extra_bytes,
                 iris_engine **out, void **extra = nullptr) {
    iris_engine *e = new (std::nothrow) iris_engine();
    if (!e) return fail(IRIS_E_NOMEM, "out of host memory");
    e->dev = dev;
    e->kind = kind;
    const size_t total = qalign(tab_bytes) + qalign(frag_bytes) + qalign(extra_bytes);
    int rc = qbuf_take(dev, total, &e->qbuf, &e->qbuf_bytes);
    if (rc != 0) {
        delete e;
        return rc;
    }
    char *base = (char *)e->qbuf;
    e->qtab = tab_bytes ? base : nullptr;
    e->qfrag = frag_bytes ? base + qalign(tab_bytes) : nullptr;
    if (extra) *extra = base + qalign(tab_bytes) + qalign(frag_bytes);
    *out = e;
    return 0;
}

// Uploads host-built tables (LANES table and, optionally, TILES fragments) of a new engine.
int engine_new(iris_device *dev, int kind, const void *table, size_t bytes, iris_engine **out,
               const void *frag = nullptr, size_t frag_bytes = 0) {
    iris_engine *e = nullptr;
    CHK(engine_alloc(dev, kind, bytes, frag ? frag_bytes : 0, 0, &e));
    hipError_t err = hipMemcpyAsync(e->qtab, table, bytes, hipMemcpyHostToDevice, dev->stream);
    if (err == hipSuccess && frag) err = hipMemcpyAsync(e->qfrag, frag, frag_bytes, hipMemcpyHostToDevice, dev->stream);
    if (err != hipSuccess) {
        engine_free(e);
        return fail(IRIS_E_HIP, std::string("upload query table: ") + hipGetErrorString(err));
    }
    *out = e;
    return 0;
}

// A new engine whose tables `build(stream, host_query, tab, frag)` fills from the host
// query passed in the kernel arguments (template and mask queries, iris_query.hip).
template <class B>
int engine_from_host_query(iris_device *dev, int kind, const void *query, size_t tab_bytes, size_t frag_bytes,
                           iris_engine **out, B &&build) {
    iris_engine *e = nullptr;
    CHK(engine_alloc(dev, kind, tab_bytes, frag_bytes, 0, &e));
    if (build(dev->stream, query, (uint32_t *)e->qtab, (uint32_t *)e->qfrag) != 0) {
        const hipError_t err = hipGetLastError();
        engine_free(e);
        return fail(IRIS_E_HIP, std::string("build query tables: ") + hipGetErrorString(err));
    }
    *out = e;
    return 0;
}

// Uploads a query (`qbytes` from the host) and builds the engine's tables from it
// on the device with `build(stream, query_dev, tab, frag)` (iris_query.hip).
template <class B>
int engine_from_query(iris_device *dev, int kind, const void *query, size_t qbytes, size_t tab_bytes,
                      size_t frag_bytes, iris_engine **out, B &&build) {
    iris_engine *e = nullptr;
    void *qdev = nullptr;
    CHK(engine_alloc(dev, kind, tab_bytes, frag_bytes, qbytes, &e, &qdev));
    hipError_t err = hipMemcpyAsync(qdev, query, qbytes, hipMemcpyHostToDevice, dev->stream);
    if (err != hipSuccess || build(dev->stream, qdev, (uint32_t *)e->qtab, (uint32_t *)e->qfrag) != 0) {
        if (err == hipSuccess) err = hipGetLastError();
        engine_free(e);
        return fail(IRIS_E_HIP, std::string("build query tables: ") + hipGetErrorString(err));
    }
    *out = e;
    return 0;
}

// The host NUMA node the device hangs off (sysfs of its PCI function); a one-node host is node 0;
// -1 when unknown.
int device_numa_node(int ordinal) {
    char bus[64] = {0};
    if (hipDeviceGetPCIBusId(bus, sizeof(bus) - 1, ordinal) != hipSuccess) return -1;
    for (char *c = bus; *c; ++c) *c = (char)tolower((unsigned char)*c);
    const std::string path = std::string("/sys/bus/pci/devices/") + bus + "/numa_node";
    int node = -1;
    if (FILE *f = fopen(path.c_str(), "r")) {
        if (fscanf(f, "%d", &node) != 1) node = -1;
        fclose(f);
    }
    if (node < 0 && access("/sys/devices/system/node/node1", F_OK) != 0 && access("/sys/devices/system/node/node0", F_OK) == 0)
        node = 0;
    return node;
}

void device_teardown(iris_device *d) {
    {
        std::lock_guard<std::recursive_mutex> g(d->mu);
        (void)hipSetDevice(d->ordinal);
        resident_drop_all(d);
        (void)hipStreamSynchronize(d->stream);
        for (DevBuf *b : {&d->partials, &d->result, &d->staging, &d->out_a, &d->out_b, &d->ticket, &d->tempdb})
            if (b->p) (void)hipFree(b->p);
        side_sync(d);
        for (int b = 0; b < 2; ++b) {
            if (d->apart[b].p) (void)hipFree(d->apart[b].p);
            if (d->apart_read[b]) (void)hipEventDestroy(d->apart_read[b]);
            if (d->apart_written[b]) (void)hipEventDestroy(d->apart_written[b]);
        }
        for (int b = 0; b < kUploadRing; ++b) {
            if (d->upin[b]) (void)hipHostFree(d->upin[b]);
            if (d->upin_ev[b]) (void)hipEventDestroy(d->upin_ev[b]);
        }
        if (d->aux) (void)hipStreamDestroy(d->aux);
        if (d->aux2) (void)hipStreamDestroy(d->aux2);
        if (d->host_result) (void)hipHostFree(d->host_result);
        if (d->host_done) (void)hipHostFree(d->host_done);
        for (void *b : d->slot_blocks) (void)hipHostFree(b);
        for (auto &q : d->qpool) (void)hipFree(q.second);
        d->qpool.clear();
        for (auto &q : d->rows_pool) (void)hipHostFree(q.second);
        d->rows_pool.clear();
        if (d->ra_order) (void)hipEventDestroy(d->ra_order);
        for (auto &p : d->pending) {
            (void)hipEventDestroy(p.a);
            (void)hipEventDestroy(p.b);
        }
        for (auto e : d->event_pool) (void)hipEventDestroy(e);
        (void)hipStreamDestroy(d->stream);
    }
    delete d;
}

}  // namespace

void iris_api::device_retain(iris_device *d) { d->refs.fetch_add(1, std::memory_order_relaxed); }
void iris_api::device_release(iris_device *d) {
    if (d->refs.fetch_sub(1, std::memory_order_acq_rel) == 1) device_teardown(d);
}

namespace {

constexpr size_t kMaskFragBytes = kMaskFragUint4 * 16;
constexpr size_t kShareFragBytes = kShareFragUint4 * 16 + 32 * 8;

double rust_f64_min(double a, double b) {
    if (isnan(a)) return b;
    if (isnan(b)) return a;
    return a < b ? a : b;
}

}  // namespace

// ================================================================== C ABI

extern "C" {

const char *iris_last_error(void) { return g_err.c_str(); }
#ifndef IRIS_BUILD_KNOBS
#define IRIS_BUILD_KNOBS ""
#endif
// "iris-hip X (gfx950)", plus " knobs: -DIRIS_..." when the build set compile-time knobs
const char *iris_version(void) {
    static const std::string v = std::string("iris-hip 0.3.0 (gfx950)") +
                                 (sizeof(IRIS_BUILD_KNOBS) > 1 ? std::string(" knobs: ") + IRIS_BUILD_KNOBS : std::string());
    return v.c_str();
}

int iris_config(const iris_device_t *d, char *buf, size_t len, size_t *needed) {
    ARG(buf || len == 0, "NULL buffer");
    Hooks now;
    if (!d) read_hooks(&now);
    std::string s(format_hooks(d ? d->hooks : now, nullptr, 0), '\0');
    format_hooks(d ? d->hooks : now, &s[0], s.size() + 1);
    if (d) {
        s += " numa_node=" + std::to_string(d->numa_node);
        char r[96];  // large writes' measured rates (GB/s) through the pinned slots / the runtime's copy
        snprintf(r, sizeof(r), " upload_gbps=%.1f/%.1f", d->upload_tune.gbps[0] / 1e9, d->upload_tune.gbps[1] / 1e9);
        s += r;
        uint64_t rc = 0, rbytes = 0;
        int via_fd = 0;
        std::string skip;
        {
            std::lock_guard<std::recursive_mutex> g(const_cast<iris_device *>(d)->mu);
            resident_stats(d, &rc, &rbytes, &via_fd);
            skip = d->resident_skip;
            // read-ahead windows since the last iris_device_reset_stats: launches, records computed,
            // the largest window (records)
            s += " readahead_windows=" + std::to_string(d->ra_launches) + "/" + std::to_string(d->ra_records) + "/" +
                 std::to_string(d->ra_window_max);
        }
        s += " resident=" + std::to_string(rc) + "/" + std::to_string(rbytes) + " resident_via_fd=" + std::to_string(via_fd);
        uint64_t ab_pending = 0, ab_total = 0;  // RCCL inits abandoned on a formation timeout: pending/total
        abandoned_inits(d->ordinal, &ab_pending, &ab_total);
        s += " abandoned_inits=" + std::to_string(ab_pending) + "/" + std::to_string(ab_total);
        if (!skip.empty()) {  // one token: spaces and '=' replaced
            for (char &c : skip)
                if (c == ' ' || c == '=') c = '_';
            s += " resident_skip=" + skip;
        }
    }
    if (buf && len) {
        const size_t n = std::min(len - 1, s.size());
        memcpy(buf, s.data(), n);
        buf[n] = 0;
    }
    if (needed) *needed = s.size();
    return 0;
}

int iris_device_count(int *count) {
    ARG(count, "count is NULL");
    int n = 0;
    hipError_t e = hipGetDeviceCount(&n);
    if (e != hipSuccess) n = 0;
    *count = n;
    return 0;
}

int iris_device_open(int ordinal, iris_device_t **out) {
    IRIS_KEEP_DEVICE();
    ARG(out, "out is NULL");
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n == 0) return fail(IRIS_E_NODEV, "no HIP device visible");
    if (ordinal < 0 || ordinal >= n) return fail(IRIS_E_NODEV, "device ordinal out of range");
    hipDeviceProp_t prop;
    HIPCHK(hipGetDeviceProperties(&prop, ordinal));
    if (strncmp(prop.gcnArchName, "gfx950", 6) != 0)
        return fail(IRIS_E_NODEV, std::string("device is ") + prop.gcnArchName + ", this build targets gfx950");
    iris_device *d = new (std::nothrow) iris_device();
    if (!d) return fail(IRIS_E_NOMEM, "out of host memory");
    d->ordinal = ordinal;
    read_hooks(&d->hooks);  // the environment's knobs, once (iris_config reports them)
    if (d->hooks.ignored) {  // said once per process: a test hook in a production environment does nothing
        static std::once_flag warned;
        std::call_once(warned, [&] {
            char buf[512];
            format_hooks(d->hooks, buf, sizeof(buf));
            fprintf(stderr, "iris-hip: test-only hooks ignored (IRIS_TEST_HOOKS is not 1): %s\n", strstr(buf, "ignored="));
        });
    }
    hipError_t e = hipSetDevice(ordinal);
    // test hook IRIS_SCHEDULE = spin | yield | blocking: how host waits on this device behave
    // (takes effect only before the process's first context on the device)
    if (d->hooks.schedule) {
        const unsigned f = d->hooks.schedule == 1   ? hipDeviceScheduleSpin
                           : d->hooks.schedule == 2 ? hipDeviceScheduleYield
                                                    : hipDeviceScheduleBlockingSync;
        (void)hipSetDeviceFlags(f);
        (void)hipGetLastError();
    }
    if (e == hipSuccess) e = hipStreamCreateWithFlags(&d->stream, hipStreamNonBlocking);
    if (e == hipSuccess) d->numa_node = device_numa_node(ordinal);
    if (e != hipSuccess) {
        delete d;
        return fail(IRIS_E_HIP, std::string("stream create: ") + hipGetErrorString(e));
    }
    *out = d;
    return 0;
}

int iris_device_close(iris_device_t *d) {
    IRIS_KEEP_DEVICE();
    if (!d) return 0;
    device_release(d);  // torn down now, or when its last database / engine is destroyed
    return 0;
}

int iris_device_synchronize(iris_device_t *d) {
    IRIS_KEEP_DEVICE();
    ARG(d, "device is NULL");
    std::lock_guard<std::recursive_mutex> g(d->mu);
    CHK(set_device(d));
    resident_sweep(d);  // copies of mappings that are gone free their memory (at most once a second)
    return sync(d);
}

int iris_device_stream(iris_device_t *d, void **stream) {
    ARG(d && stream, "NULL argument");
    *stream = (void *)d->stream;
    return 0;
}

int iris_device_memory(iris_device_t *d, size_t *free_bytes, size_t *total_bytes) {
    IRIS_KEEP_DEVICE();
    ARG(d && free_bytes && total_bytes, "NULL argument");
    std::lock_guard<std::recursive_mutex> g(d->mu);
    CHK(set_device(d));
    HIPCHK(hipMemGetInfo(free_bytes, total_bytes));
    return 0;
}

int iris_device_set_profiling(iris_device_t *d, int enabled) {
    IRIS_KEEP_DEVICE();
    ARG(d, "device is NULL");
    std::lock_guard<std::recursive_mutex> g(d->mu);
    d->profiling = enabled != 0;
    return 0;
}

int iris_device_kernel_stats(iris_device_t *d, const char *kernel, uint64_t *launches, double *total_ms,
                             uint64_t *items) {
    IRIS_KEEP_DEVICE();
    ARG(d && kernel, "NULL argument");
    std::lock_guard<std::recursive_mutex> g(d->mu);
    auto it = d->stats.find(kernel);
    KStat s = it == d->stats.end() ? KStat{} : it->second;
    if (launches) *launches = s.launches;
    if (total_ms) *total_ms = s.ms;
    if (items) *items = s.items;
    return 0;
}

int iris_device_kernel_stats_largest(iris_device_t *d, const char *kernel, uint64_t *items, double *ms) {
    IRIS_KEEP_DEVICE();
    ARG(d && kernel, "NULL argument");
    std::lock_guard<std::recursive_mutex> g(d->mu);
    fold_done(d);
    auto it = d->stats.find(kernel);
    KStat s = it == d->stats.end() ? KStat{} : it->second;
    if (items) *items = s.max_items;
    if (ms) *ms = s.max_ms;
    return 0;
}

int iris_device_reset_stats(iris_device_t *d) {
    IRIS_KEEP_DEVICE();
    ARG(d, "device is NULL");
    std::lock_guard<std::recursive_mutex> g(d->mu);
    d->stats.clear();
    d->ra_launches = d->ra_records = d->ra_window_max = 0;
    return 0;
}

int iris_device_alloc(iris_device_t *d, size_t bytes, void **ptr) {
    IRIS_KEEP_DEVICE();
    ARG(d && ptr, "NULL argument");
    std::lock_guard<std::recursive_mutex> g(d->mu);
    CHK(set_device(d));
    return dev_malloc(d, ptr, std::max<size_t>(bytes, 1), "iris_device_alloc");
}

int iris_device_free(iris_device_t *d, void *ptr) {
    IRIS_KEEP_DEVICE();
    ARG(d, "device is NULL");
    std::lock_guard<std::recursive_mutex> g(d->mu);
    CHK(set_device(d));
    if (ptr) HIPCHK(hipFree(ptr));
    return 0;
}

int iris_memcpy_d2h(iris_device_t *d, void *host, const void *device, size_t bytes) {
    IRIS_KEEP_DEVICE();
    ARG(d && (bytes == 0 || (host && device)), "NULL argument");
    std::lock_guard<std::recursive_mutex> g(d->mu);
    CHK(set_device(d));
    HIPCHK(hipMemcpyAsync(host, device, bytes, hipMemcpyDeviceToHost, d->stream));
    return sync(d);
}

int iris_memcpy_h2d(iris_device_t *d, void *device, const void *host, size_t bytes) {
    IRIS_KEEP_DEVICE();
    ARG(d && (bytes == 0 || (host && device)), "NULL argument");
    std::lock_guard<std::recursive_mutex> g(d->mu);
    CHK(set_device(d));
    HIPCHK(hipMemcpyAsync(device, host, bytes, hipMemcpyHostToDevice, d->stream));
    return sync(d);
}

// ------------------------------------------------------------------ databases

int iris_db_create(iris_device_t *d, int kind, uint64_t capacity, iris_db_t **out) {
    return iris_db_create_ex(d, kind, capacity, IRIS_LAYOUT_DEFAULT, out);
}

int iris_db_create_ex(iris_device_t *d, int kind, uint64_t capacity, int layout, iris_db_t **out) {
    IRIS_KEEP_DEVICE();
    ARG(d && out, "NULL argument");
    CHK(check_kind(kind));
    if (layout == IRIS_LAYOUT_DEFAULT) layout = IRIS_LAYOUT_TILES;
    ARG(layout == IRIS_LAYOUT_LANES || layout == IRIS_LAYOUT_TILES, "unknown layout");
    std::lock_guard<std::recursive_mutex> g(d->mu);
    CHK(set_device(d));
    iris_db *db = new (std::nothrow) iris_db();
    if (db) db->version = next_db_version();
    if (!db) return fail(IRIS_E_NOMEM, "out of host memory");
    db->dev = d;
    db->k = kind_info(kind, layout);
    const uint64_t blocks = std::max<uint64_t>(1, capacity / db->k.block + (capacity % db->k.block != 0));
    size_t bytes = 0;
    if (__builtin_mul_overflow(blocks, (uint64_t)block_bytes(db->k), &bytes)) {
        delete db;
        return fail(IRIS_E_NOMEM, "database capacity overflows the address space");
    }
    db->cap = capacity == 0 ? 0 : blocks * db->k.block;
    // the caller's database before cached file copies (evicted least recently used first)
    if (dev_malloc(d, &db->data, bytes, "database") != 0) {
        delete db;
        return IRIS_E_NOMEM;
    }
    // zeroed padding records: a zero mask gives den = 0, i.e. "no candidate"
    hipError_t e = hipMemsetAsync(db->data, 0, bytes, d->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(d->stream);
    if (e != hipSuccess) {
        (void)hipFree(db->data);
        delete db;
        return fail(IRIS_E_HIP, std::string("memset database: ") + hipGetErrorString(e));
    }
    device_retain(d);
    *out = db;
    return 0;
}

int iris_db_layout(const iris_db_t *db, int *layout) {
    ARG(db && layout, "NULL argument");
    *layout = db->k.layout;
    return 0;
}

int iris_db_destroy(iris_db_t *db) {
    IRIS_KEEP_DEVICE();
    if (!db) return 0;
    iris_device *d = db->dev;
    {
        std::lock_guard<std::recursive_mutex> g(d->mu);
        (void)hipSetDevice(d->ordinal);
        (void)hipStreamSynchronize(d->stream);
        side_sync(d);  // a read-ahead kernel may still read it
        db_detach(db);
        if (db->data) (void)hipFree(db->data);
    }
    delete db;
    device_release(d);
    return 0;
}

int iris_db_len(const iris_db_t *db, uint64_t *len) {
    ARG(db && len, "NULL argument");
    *len = db->len;
    return 0;
}

int iris_db_capacity(const iris_db_t *db, uint64_t *cap) {
    ARG(db && cap, "NULL argument");
    *cap = db->cap;
    return 0;
}

int iris_db_kind(const iris_db_t *db, int *kind) {
    ARG(db && kind, "NULL argument");
    *kind = db->k.kind;
    return 0;
}

int iris_db_append(iris_db_t *db, const void *records, uint64_t n) {
    IRIS_KEEP_DEVICE();
    ARG(db, "database is NULL");
    std::lock_guard<std::recursive_mutex> g(db->dev->mu);
    CHK(set_device(db->dev));
    return db_write_locked(db, db->len, records, n);
}

int iris_db_write(iris_db_t *db, uint64_t index, const void *records, uint64_t n) {
    IRIS_KEEP_DEVICE();
    ARG(db, "database is NULL");
    std::lock_guard<std::recursive_mutex> g(db->dev->mu);
    CHK(set_device(db->dev));
    return db_write_locked(db, index, records, n);
}

int iris_db_read(const iris_db_t *db, uint64_t first, uint64_t n, void *records) {
    IRIS_KEEP_DEVICE();
    ARG(db, "database is NULL");
    iris_device *d = db->dev;
    std::lock_guard<std::recursive_mutex> g(d->mu);
    CHK(set_device(d));
    CHK(range_ok(db, first, n));
    if (n == 0) return 0;
    ARG(records, "records is NULL");
    const KindInfo &k = db->k;
    if ((size_t)n * k.rec_bytes >= kUploadTuneMin && ensure_upin(d) == 0) {
        // the upload slots run backwards: slot c is unpacked and copied into pinned buffer c % 2 by the
        // device while the helper threads copy slot c - 1 into the caller's array
        const uint64_t ch = std::max<uint64_t>(64, kUploadSlot / k.rec_bytes / 64 * 64);
        const size_t slot = (size_t)ch * k.rec_bytes;
        CHK(ensure(d, d->staging, kUploadSlots * slot));
        const uint64_t chunks = (n + ch - 1) / ch;
        int rc = 0;
        auto enqueue = [&](uint64_t c) -> int {
            const int b = (int)(c % kUploadSlots);
            const uint64_t a = c * ch, m = std::min<uint64_t>(ch, n - a);
            void *stage = (char *)d->staging.p + (size_t)b * slot;
            CHK(timed(d, "unpack", m, [&] { return launch_unpack(d->stream, k, db->data, stage, first + a, m); }));
            HIPCHK(hipMemcpyAsync(d->upin[b], stage, (size_t)m * k.rec_bytes, hipMemcpyDeviceToHost, d->stream));
            HIPCHK(hipEventRecord(d->upin_ev[b], d->stream));
            return 0;
        };
        rc = enqueue(0);
        for (uint64_t c = 0; c < chunks && rc == 0; ++c) {
            // pinned buffer (c + 1) % slots was last read by the (synchronous) copy-out of slot c + 1 - slots
            if (c + 1 < chunks) rc = enqueue(c + 1);
            if (rc == 0 && hipEventSynchronize(d->upin_ev[c % kUploadSlots]) != hipSuccess) rc = fail(IRIS_E_HIP, "hipEventSynchronize");
            if (rc == 0) {
                const uint64_t a = c * ch, m = std::min<uint64_t>(ch, n - a);
                parallel_copy((char *)records + a * k.rec_bytes, d->upin[c % kUploadSlots], (size_t)m * k.rec_bytes, d->ordinal);
            }
        }
        const int rs = sync(d);
        CHK(rc);
        return rs;
    }
    const uint64_t ch = chunk_records(k);
    CHK(ensure(d, d->staging, std::min<uint64_t>(n, ch) * k.rec_bytes));
    for (uint64_t done = 0; done < n; done += ch) {
        const uint64_t m = std::min<uint64_t>(ch, n - done);
        CHK(timed(d, "unpack", m, [&] { return launch_unpack(d->stream, k, db->data, d->staging.p, first + done, m); }));
        HIPCHK(hipMemcpyAsync((char *)records + done * k.rec_bytes, d->staging.p, m * k.rec_bytes,
                              hipMemcpyDeviceToHost, d->stream));
        CHK(sync(d));
    }
    return 0;
}

int iris_db_generate(iris_db_t *db, uint64_t n, uint64_t seed, uint64_t global_index0) {
    IRIS_KEEP_DEVICE();
    ARG(db, "database is NULL");
    iris_device *d = db->dev;
    std::lock_guard<std::recursive_mutex> g(d->mu);
    CHK(set_device(d));
    if (n > db->cap - db->len) return fail(IRIS_E_RANGE, "iris_db_generate: database capacity exceeded");
    if (n == 0) return 0;
    db_detach(db);
    CHK(timed(d, "generate", n, [&] { return launch_generate(d->stream, db->k, db->data, db->len, n, seed, global_index0); }));
    CHK(sync(d));
    db->len += n;
    return 0;
}

int iris_db_truncate(iris_db_t *db, uint64_t len) {
    IRIS_KEEP_DEVICE();
    ARG(db, "database is NULL");
    std::lock_guard<std::recursive_mutex> g(db->dev->mu);
    if (len > db->len) return fail(IRIS_E_RANGE, "iris_db_truncate: len beyond the current length");
    if (len != db->len) db_detach(db);
    db->len = len;
    return 0;
}

int iris_db_attach_host(iris_db_t *db, const void *host, uint64_t n, int upload) {
    IRIS_KEEP_DEVICE();
    ARG(db && (host || n == 0), "NULL argument");
    iris_device *d = db->dev;
    std::lock_guard<std::recursive_mutex> g(d->mu);
    CHK(set_device(d));
    db_detach(db);
    const size_t rb = db->k.rec_bytes;
    if (upload) {
        ARG(db->len == 0, "iris_db_attach_host(upload): the database must be empty");
        CHK(db_write_locked(db, 0, host, n));
    } else {
        ARG(db->len == n, "iris_db_attach_host: the database must hold exactly the n records of the host array");
        // the caller's promise (e.g. the same file loaded with iris_db_load_file) is spot-checked
        const uint64_t probe[3] = {0, n / 2, n ? n - 1 : 0};
        std::vector<char> rec(rb);
        for (int i = 0; i < 3 && n; ++i) {
            CHK(iris_db_read(db, probe[i], 1, rec.data()));
            if (memcmp(rec.data(), (const char *)host + probe[i] * rb, rb) != 0)
                return fail(IRIS_E_ARG, "iris_db_attach_host: record " + std::to_string(probe[i]) +
                                            " of the database differs from the host array");
        }
    }
    if (n == 0) return 0;
    db->host_base = (uintptr_t)host;
    db->host_n = n;
    db->version = next_db_version();
    d->attached.push_back(db);
    return 0;
}

int iris_db_detach_host(iris_db_t *db) {
    IRIS_KEEP_DEVICE();
    ARG(db, "database is NULL");
    std::lock_guard<std::recursive_mutex> g(db->dev->mu);
    db_detach(db);
    return 0;
}

int iris_db_clear(iris_db_t *db) {
    IRIS_KEEP_DEVICE();
    ARG(db, "database is NULL");
    std::lock_guard<std::recursive_mutex> g(db->dev->mu);
    CHK(set_device(db->dev));
    db_detach(db);
    const size_t bytes = std::max<uint64_t>(1, db->cap / db->k.block) * block_bytes(db->k);
    HIPCHK(hipMemsetAsync(db->data, 0, bytes, db->dev->stream));
    CHK(sync(db->dev));
    db->len = 0;
    return 0;
}

// ------------------------------------------------------------------ engines

int iris_masks_engine_new(iris_device_t *d, const uint64_t query_mask[IRIS_LIMBS], iris_engine_t **out) {
    IRIS_KEEP_DEVICE();
    ARG(d && query_mask && out, "NULL argument");
    std::lock_guard<std::recursive_mutex> g(d->mu);
    CHK(set_device(d));
    CHK(engine_from_host_query(d, IRIS_KIND_MASKS, query_mask, (size_t)kPlaneDwords * kSlotTabStride * 4,
                               kMaskFragBytes, out, launch_query_masks));
    device_retain(d);
    return 0;
}

int iris_distance_engine_new(iris_device_t *d, const uint16_t query[IRIS_BITS], iris_engine_t **out) {
    IRIS_KEEP_DEVICE();
    ARG(d && query && out, "NULL argument");
    std::lock_guard<std::recursive_mutex> g(d->mu);
    CHK(set_device(d));
    CHK(engine_from_query(d, IRIS_KIND_SHARES, query, IRIS_BITS * 2, (size_t)kShareDwords * kSlotTabStride * 4,
                          kShareFragBytes, out, launch_query_shares));
    device_retain(d);
    return 0;
}

}  // extern "C"

int iris_api::template_engine_locked(iris_device *d, const iris_template_t *query, iris_engine **out) {
    // [LANES table | TILES fragments], both built by one launch
    return engine_from_host_query(d, IRIS_KIND_TEMPLATES, query, (size_t)kPlaneDwords * kTemplateTabStride * 4,
                                  kTemplateFragDwords * 4, out, launch_query_template);
}

extern "C" {

int iris_template_engine_new(iris_device_t *d, const iris_template_t *query, iris_engine_t **out) {
    IRIS_KEEP_DEVICE();
    ARG(d && query && out, "NULL argument");
    std::lock_guard<std::recursive_mutex> g(d->mu);
    CHK(set_device(d));
    CHK(template_engine_locked(d, query, out));
    device_retain(d);
    return 0;
}

int iris_engine_destroy(iris_engine_t *e) {
    IRIS_KEEP_DEVICE();
    if (!e) return 0;
    iris_device *d = e->dev;
    {
        std::lock_guard<std::recursive_mutex> g(d->mu);
        // no wait on the device stream: the query buffer goes back to the device's pool and its
        // reuse is stream-ordered; an engine that read ahead waits for its side-stream kernels
        // before its pinned row buffers go back (ra_release)
        engine_free(e);
    }
    device_release(d);
    return 0;
}

int iris_engine_batch_process(iris_engine_t *e, const iris_db_t *db, uint64_t first, uint64_t n, uint16_t *out) {
    IRIS_KEEP_DEVICE();
    ARG(e && db, "NULL argument");
    ARG(e->kind == IRIS_KIND_MASKS || e->kind == IRIS_KIND_SHARES, "batch_process needs a masks or distance engine");
    ARG(db->k.kind == e->kind, "engine kind does not match the database kind");
    ARG(e->dev == db->dev, "engine and database live on different devices");
    std::lock_guard<std::recursive_mutex> g(e->dev->mu);
    CHK(set_device(e->dev));
    CHK(range_ok(db, first, n));
    if (n == 0) return 0;
    ARG(out, "out is NULL");
    if (readahead_ok(db, n)) return readahead_u16_call(e, db, first, n, db->len, out);
    CHK(ra_wait(e));
    return run_u16_engine(e, db, first, n, out);
}

int iris_engine_batch_process_device(iris_engine_t *e, const iris_db_t *db, uint64_t first, uint64_t n,
                                     uint16_t *out_device) {
    IRIS_KEEP_DEVICE();
    ARG(e && db, "NULL argument");
    ARG(e->kind == IRIS_KIND_MASKS || e->kind == IRIS_KIND_SHARES, "batch_process needs a masks or distance engine");
    ARG(db->k.kind == e->kind, "engine kind does not match the database kind");
    ARG(e->dev == db->dev, "engine and database live on different devices");
    iris_device *d = e->dev;
    std::lock_guard<std::recursive_mutex> g(d->mu);
    CHK(set_device(d));
    CHK(range_ok(db, first, n));
    if (n == 0) return 0;
    ARG(out_device, "out is NULL");
    // a participant-sized range: the kernel's last workgroup publishes a sequence word in coherent
    // host memory once every row is stored, and the call returns when it lands (as the small
    // search does) -- later work on the device stream, the rows' consumers, follows the kernel
    DoneSignal sig{};
    if (db->k.layout == IRIS_LAYOUT_TILES) {
        CHK(ensure_ticket(d));
        CHK(ensure_host_done(d));
        sig.ticket = (uint32_t *)d->ticket.p;
        sig.done = d->host_done;
        sig.seq = ++d->done_seq;
        if (sig.seq == 0) sig.seq = ++d->done_seq;  // 0 is the word's initial value
    }
    CHK(enqueue_u16_engine(e, db, first, n, out_device, nullptr, sig.done ? &sig : nullptr));
    if (!sig.armed) return sync(d);
    CHK(wait_done(d, sig.seq));
    if (d->profiling) fold_done(d);
    return 0;
}

int iris_engine_batch_process_host(iris_engine_t *e, const void *records, uint64_t n, uint16_t *out) {
    IRIS_KEEP_DEVICE();
    ARG(e, "engine is NULL");
    ARG(e->kind == IRIS_KIND_MASKS || e->kind == IRIS_KIND_SHARES, "batch_process needs a masks or distance engine");
    iris_device *d = e->dev;
    std::lock_guard<std::recursive_mutex> g(d->mu);
    CHK(set_device(d));
    if (n == 0) return 0;
    ARG(records && out, "NULL argument");
    const KindInfo k = kind_info(e->kind);
    // a slice of an attached host array: run on its resident copy, nothing is uploaded
    const uintptr_t p = (uintptr_t)records;
    for (iris_db *a : d->attached) {
        if (a->k.kind != e->kind || p < a->host_base) continue;
        const uintptr_t off = p - a->host_base;
        if (off % k.rec_bytes != 0 || off / k.rec_bytes > a->host_n || n > a->host_n - off / k.rec_bytes) continue;
        if (readahead_ok(a, n)) return readahead_u16_call(e, a, off / k.rec_bytes, n, a->host_n, out);
        CHK(ra_wait(e));
        return run_u16_engine(e, a, off / k.rec_bytes, n, out);
    }
    // a slice of a read-only record file mapping (the reference's participant / resolver walk):
    // run on the device's resident copy of the file (iris_resident.hip)
    iris_db *rdb = nullptr;
    uint64_t rfirst = 0, rend = 0;
    CHK(resident_slice(d, e->kind, records, n, &rdb, &rfirst, &rend));
    if (rdb) {
        PinResident pin(d, rdb);  // a workspace allocation below may evict copies: not this one
        if (readahead_ok(rdb, n)) return readahead_u16_call(e, rdb, rfirst, n, rend, out);
        CHK(ra_wait(e));
        return run_u16_engine(e, rdb, rfirst, n, out);
    }
    const uint64_t ch = std::min<uint64_t>(n, 1ull << 20 >> (e->kind == IRIS_KIND_SHARES ? 4 : 0));
    TempDb t;
    CHK(temp_db(d, e->kind, ch, t));
    for (uint64_t done = 0; done < n; done += ch) {
        const uint64_t m = std::min<uint64_t>(ch, n - done);
        t.db.len = 0;
        CHK(db_write_locked(&t.db, 0, (const char *)records + done * k.rec_bytes, m));
        CHK(run_u16_engine(e, &t.db, 0, m, out + done * kRot));
    }
    return 0;
}

static int template_args(iris_engine_t *e, const iris_db_t *db) {
    ARG(e && db, "NULL argument");
    ARG(e->kind == IRIS_KIND_TEMPLATES && e->nq == 0, "not a single-query template engine");
    ARG(db->k.kind == IRIS_KIND_TEMPLATES, "database does not hold templates");
    ARG(e->dev == db->dev, "engine and database live on different devices");
    return 0;
}

int iris_template_counts(iris_engine_t *e, const iris_db_t *db, uint64_t first, uint64_t n, uint16_t *num_out,
                         uint16_t *den_out) {
    IRIS_KEEP_DEVICE();
    CHK(template_args(e, db));
    iris_device *d = e->dev;
    std::lock_guard<std::recursive_mutex> g(d->mu);
    CHK(set_device(d));
    CHK(range_ok(db, first, n));
    if (n == 0 || (!num_out && !den_out)) return 0;
    const uint64_t ch = 4ull << 20;
    const size_t bytes = std::min<uint64_t>(n, ch) * kRot * 2;
    CHK(ensure(d, d->out_a, bytes));
    CHK(ensure(d, d->out_b, bytes));
    for (uint64_t done = 0; done < n; done += ch) {
        const uint64_t m = std::min<uint64_t>(ch, n - done);
        LaunchRange r{first + done, m};
        uint16_t *na = num_out ? (uint16_t *)d->out_a.p : nullptr;
        uint16_t *da = den_out ? (uint16_t *)d->out_b.p : nullptr;
        CHK(timed(d, "template_counts", m, [&] {
            return db->k.layout == IRIS_LAYOUT_TILES
                       ? launch_template_mfma_counts(d->hooks, d->stream, db->data, e->qfrag, r, na, da)
                       : launch_template_counts(d->stream, db->data, e->qtab, r, na, da);
        }));
        if (num_out)
            HIPCHK(hipMemcpyAsync(num_out + done * kRot, d->out_a.p, m * kRot * 2, hipMemcpyDeviceToHost, d->stream));
        if (den_out)
            HIPCHK(hipMemcpyAsync(den_out + done * kRot, d->out_b.p, m * kRot * 2, hipMemcpyDeviceToHost, d->stream));
        CHK(sync(d));
    }
    return 0;
}

// Enqueues the search of [first, first+n) and its reduce, whose winner lands in
// `dst` (pinned host memory); nothing waits.  side = true (asynchronous
// searches): the reduce runs on the side stream over one of two alternating
// partials buffers, and `done` (if given) is recorded there after it.
}  // extern "C"

int iris_api::search_enqueue(iris_engine_t *e, const iris_db_t *db, uint64_t first, uint64_t n, double *dist_dev,
                             Partial *dst, bool side, hipEvent_t done, uint64_t idx_base, uint32_t *host_done,
                             uint32_t seq, bool *flagged) {
    iris_device *d = e->dev;
    if (flagged) *flagged = false;
    if (n == 0) return 0;
    LaunchRange r{first, n};
    const int layout = db->k.layout;
    if (layout == IRIS_LAYOUT_TILES && fused_search_ok(d->hooks, r)) {
        // small range: the kernel's last workgroup reduces and writes dst itself (no reduce launch)
        CHK(ensure_ticket(d));
        CHK(ensure(d, d->partials, (size_t)mfma_search_partials(d->hooks, r) * sizeof(Partial)));
        const FusedFinish fin{(uint32_t *)d->ticket.p, dst, idx_base, host_done, seq};
        uint32_t written = 0;
        CHK(timed(d, "template_search", n, [&] {
            return launch_template_mfma_search(d->hooks, d->stream, db->data, e->qfrag, r, dist_dev, (Partial *)d->partials.p,
                                               &written, &fin);
        }));
        if (flagged) *flagged = host_done != nullptr;
        if (!side) return 0;
        // later side-stream work (a group's all-gather) and `done` follow the kernel
        CHK(ensure_aux(d));
        const int b = d->apart_next;
        d->apart_next ^= 1;
        if (!d->apart_written[b]) HIPCHK(hipEventCreateWithFlags(&d->apart_written[b], hipEventDisableTiming));
        HIPCHK(hipEventRecord(d->apart_written[b], d->stream));
        HIPCHK(hipStreamWaitEvent(d->aux, d->apart_written[b], 0));
        if (done) HIPCHK(hipEventRecord(done, d->aux));
        return 0;
    }
    const uint32_t np = layout == IRIS_LAYOUT_TILES ? mfma_search_partials(d->hooks, r) : search_partials(r);
    const size_t pbytes = (size_t)std::max<uint32_t>(np, 1) * sizeof(Partial);
    DevBuf *buf = &d->partials;
    int b = 0;
    if (side) {
        CHK(ensure_aux(d));
        b = d->apart_next;
        d->apart_next ^= 1;
        buf = &d->apart[b];
        for (hipEvent_t *ev : {&d->apart_read[b], &d->apart_written[b]})
            if (!*ev) HIPCHK(hipEventCreateWithFlags(ev, hipEventDisableTiming));
        // the reduce that last read this buffer (two searches ago) precedes the overwrite
        HIPCHK(hipStreamWaitEvent(d->stream, d->apart_read[b], 0));
    }
    CHK(ensure(d, *buf, pbytes));
    Partial *part = (Partial *)buf->p;
    uint32_t written = 0;
    CHK(timed(d, "template_search", n, [&] {
        if (layout == IRIS_LAYOUT_TILES)
            return launch_template_mfma_search(d->hooks, d->stream, db->data, e->qfrag, r, dist_dev, part, &written);
        return launch_template_search(d->stream, db->data, e->qtab, r, dist_dev, part, &written);
    }));
    if (!side)  // the reduce writes the winner straight into pinned host memory: no copy before the wait
        return timed(d, "reduce", written, [&] { return launch_reduce(d->stream, part, written, dst, idx_base); });
    HIPCHK(hipEventRecord(d->apart_written[b], d->stream));
    HIPCHK(hipStreamWaitEvent(d->aux, d->apart_written[b], 0));
    CHK(timed(d, "reduce", written, [&] { return launch_reduce(d->aux, part, written, dst, idx_base); }, d->aux));
    HIPCHK(hipEventRecord(d->apart_read[b], d->aux));
    if (done) HIPCHK(hipEventRecord(done, d->aux));
    return 0;
}

extern "C" {

static int search_locked(iris_engine_t *e, const iris_db_t *db, uint64_t first, uint64_t n, uint64_t index_base,
                         double *dist_dev, iris_match_t *out) {
    iris_device *d = e->dev;
    CHK(ensure_host_result(d, sizeof(Partial)));
    // Without a device distances output the caller needs only the winner: a small (fused)
    // search publishes it with a sequence word in coherent host memory, and the call returns
    // as soon as that word lands -- no wait for the kernel's retirement and completion signal
    // (the kernel's tail is ordered before anything later enqueued on the stream).
    uint32_t *done_word = nullptr, seq = 0;
    if (!dist_dev) {
        CHK(ensure_host_done(d));
        done_word = d->host_done;
        seq = ++d->done_seq;
        if (seq == 0) seq = ++d->done_seq;  // 0 is the word's initial value
    }
    bool flagged = false;
    CHK(search_enqueue(e, db, first, n, dist_dev, (Partial *)d->host_result, false, nullptr, 0, done_word, seq,
                       &flagged));
    Partial res{};
    if (flagged) {
        CHK(wait_done(d, seq));
        if (d->profiling) fold_done(d);  // the timing events of earlier searches
    } else
        CHK(sync(d));
    if (n > 0) memcpy(&res, d->host_result, sizeof(Partial));
    if (out) {
        if (n == 0 || res.den == 0) {
            out->distance = INFINITY;
            out->index = UINT64_MAX;
            out->num = 0;
            out->den = 0;
            out->rotation = 0;
        } else {
            out->distance = (double)res.num / (double)res.den;
            out->index = index_base + first + res.idx;
            out->num = res.num;
            out->den = res.den;
            out->rotation = res.rot - IRIS_MAX_ROTATION;
        }
        out->reserved = 0;
    }
    return 0;
}

// two queries in one streamed pass (TILES databases; LANES runs them one at a time)
static int pair_search_locked(iris_engine_t *a, iris_engine_t *b, const iris_db_t *db, uint64_t first, uint64_t n,
                              uint64_t index_base, iris_match_t *out) {
    if (db->k.layout != IRIS_LAYOUT_TILES) {
        CHK(search_locked(a, db, first, n, index_base, nullptr, out));
        return search_locked(b, db, first, n, index_base, nullptr, out + 1);
    }
    iris_device *d = a->dev;
    LaunchRange r{first, n};
    const uint32_t np = multi_search_partials(r, 2);
    CHK(ensure(d, d->partials, (size_t)std::max<uint32_t>(2 * np, 1) * sizeof(Partial)));
    CHK(ensure_host_result(d, 2 * sizeof(Partial)));
    const void *qf[2] = {a->qfrag, b->qfrag};
    uint32_t written = 0;
    CHK(timed(d, "template_batch", 2 * n, [&] {
        return launch_template_multi_search(d->stream, db->data, qf, 2, r, (Partial *)d->partials.p, &written);
    }));
    Partial res[2] = {};
    if (n > 0) {
        for (int q = 0; q < 2; ++q)
            CHK(timed(d, "reduce", written, [&] {
                return launch_reduce(d->stream, (Partial *)d->partials.p + (size_t)q * written, written,
                                     (Partial *)d->host_result + q);
            }));
    }
    CHK(sync(d));
    if (n > 0) memcpy(res, d->host_result, 2 * sizeof(Partial));
    for (int q = 0; q < 2; ++q) {
        iris_match_t &m = out[q];
        if (n == 0 || res[q].den == 0) {
            m.distance = INFINITY;
            m.index = UINT64_MAX;
            m.num = 0;
            m.den = 0;
            m.rotation = 0;
        } else {
            m.distance = (double)res[q].num / (double)res[q].den;
            m.index = index_base + first + res[q].idx;
            m.num = res[q].num;
            m.den = res[q].den;
            m.rotation = res[q].rot - IRIS_MAX_ROTATION;
        }
        m.reserved = 0;
    }
    return 0;
}

int iris_template_search(iris_engine_t *e, const iris_db_t *db, uint64_t first, uint64_t n, uint64_t index_base,
                         double *dist_out_device, iris_match_t *out) {
    IRIS_KEEP_DEVICE();
    CHK(template_args(e, db));
    std::lock_guard<std::recursive_mutex> g(e->dev->mu);
    CHK(set_device(e->dev));
    CHK(range_ok(db, first, n));
    ARG(out, "out is NULL");
    return search_locked(e, db, first, n, index_base, dist_out_device, out);
}

}  // extern "C"

void iris_api::match_from(const Partial &r, bool any, uint64_t base, iris_match_t *out) {
    if (!any || r.den == 0) {
        out->distance = INFINITY;
        out->index = UINT64_MAX;
        out->num = 0;
        out->den = 0;
        out->rotation = 0;
    } else {
        out->distance = (double)r.num / (double)r.den;
        out->index = base + r.idx;
        out->num = r.num;
        out->den = r.den;
        out->rotation = r.rot - IRIS_MAX_ROTATION;
    }
    out->reserved = 0;
}

extern "C" {

struct iris_pending {
    iris_device *dev = nullptr;
    hipEvent_t ev = nullptr;    // recorded after the reduce (null for an empty range)
    Partial *slot = nullptr;    // pinned host slot the reduce writes
    uint64_t n = 0, base = 0;   // range size; index_base + first
};

int iris_template_search_async(iris_engine_t *e, const iris_db_t *db, uint64_t first, uint64_t n,
                               uint64_t index_base, iris_pending_t **out) {
    IRIS_KEEP_DEVICE();
    CHK(template_args(e, db));
    ARG(out, "out is NULL");
    iris_device *d = e->dev;
    std::lock_guard<std::recursive_mutex> g(d->mu);
    CHK(set_device(d));
    CHK(range_ok(db, first, n));
    iris_pending *p = new (std::nothrow) iris_pending();
    if (!p) return fail(IRIS_E_NOMEM, "out of host memory");
    p->dev = d;
    p->n = n;
    p->base = index_base + first;
    int rc = take_result_slot(d, &p->slot);
    if (rc == 0 && n > 0) {
        p->ev = take_event(d);
        if (!p->ev) rc = fail(IRIS_E_HIP, "hipEventCreate failed");
    }
    if (rc == 0) rc = search_enqueue(e, db, first, n, nullptr, p->slot, true, p->ev);
    if (rc != 0) {
        if (p->slot) d->free_slots.push_back(p->slot);
        if (p->ev) d->event_pool.push_back(p->ev);
        delete p;
        return rc;
    }
    device_retain(d);
    *out = p;
    return 0;
}

int iris_pending_wait(iris_pending_t *p, iris_match_t *out) {
    IRIS_KEEP_DEVICE();
    ARG(p, "pending is NULL");
    iris_device *d = p->dev;
    hipError_t err = hipSuccess;
    if (p->ev) err = hipEventSynchronize(p->ev);  // this search only: later enqueued work keeps running
    Partial res{};
    if (p->n > 0 && err == hipSuccess) memcpy(&res, p->slot, sizeof(Partial));
    {
        std::lock_guard<std::recursive_mutex> g(d->mu);
        d->free_slots.push_back(p->slot);
        if (p->ev) d->event_pool.push_back(p->ev);
        fold_done(d);
    }
    const uint64_t n = p->n, base = p->base;
    delete p;
    device_release(d);
    if (err != hipSuccess) return fail(IRIS_E_HIP, std::string("hipEventSynchronize: ") + hipGetErrorString(err));
    if (out) match_from(res, n > 0, base, out);
    return 0;
}

int iris_template_distances(iris_engine_t *e, const iris_db_t *db, uint64_t first, uint64_t n, double *out) {
    IRIS_KEEP_DEVICE();
    CHK(template_args(e, db));
    iris_device *d = e->dev;
    std::lock_guard<std::recursive_mutex> g(d->mu);
    CHK(set_device(d));
    CHK(range_ok(db, first, n));
    if (n == 0) return 0;
    ARG(out, "out is NULL");
    const uint64_t ch = 16ull << 20;
    CHK(ensure(d, d->out_a, std::min<uint64_t>(n, ch) * sizeof(double)));
    for (uint64_t done = 0; done < n; done += ch) {
        const uint64_t m = std::min<uint64_t>(ch, n - done);
        iris_match_t ignored;
        CHK(search_locked(e, db, first + done, m, 0, (double *)d->out_a.p, &ignored));
        HIPCHK(hipMemcpyAsync(out + done, d->out_a.p, m * sizeof(double), hipMemcpyDeviceToHost, d->stream));
        CHK(sync(d));
    }
    return 0;
}

// ------------------------------------------------------------------ batched queries

int iris_template_batch_engine_new(iris_device_t *d, const iris_template_t *queries, uint32_t nq, iris_engine_t **out) {
    IRIS_KEEP_DEVICE();
    ARG(d && out && (nq == 0 || queries), "NULL argument");
    ARG(nq > 0, "a batch needs at least one query");
    std::lock_guard<std::recursive_mutex> g(d->mu);
    CHK(set_device(d));
    if (nq <= kBatchStreamMax) {
        iris_engine *e = new (std::nothrow) iris_engine();
        if (!e) return fail(IRIS_E_NOMEM, "out of host memory");
        e->dev = d;
        e->kind = IRIS_KIND_TEMPLATES;
        e->nq = nq;
        for (uint32_t i = 0; i < nq; ++i) {
            iris_engine *c = nullptr;
            const int rc = template_engine_locked(d, queries + i, &c);
            if (rc != 0) {
                engine_free(e);
                return rc;
            }
            e->sub.push_back(c);
        }
        device_retain(d);
        *out = e;
        return 0;
    }
    const uint32_t qgs = batch_query_group();
    const uint32_t nqp = (nq + qgs - 1) / qgs * qgs;  // padded to the kernel's query groups (zero tiles: no candidate)
    const size_t tile_bytes = (size_t)16 * kPlaneGroups * 64;
    CHK(engine_from_query(d, IRIS_KIND_TEMPLATES, queries, (size_t)nq * sizeof(iris_template_t), 0,
                          (size_t)nqp * tile_bytes, out, [&](void *stream, const void *q, uint32_t *, uint32_t *frag) {
                              return launch_query_tiles(stream, q, nq, nqp, frag);
                          }));
    (*out)->nq = nq;
    device_retain(d);
    return 0;
}

int iris_template_batch_search(iris_engine_t *e, const iris_db_t *db, uint64_t first, uint64_t n, uint64_t index_base,
                               iris_match_t *out) {
    IRIS_KEEP_DEVICE();
    ARG(e && db && out, "NULL argument");
    ARG(e->kind == IRIS_KIND_TEMPLATES && e->nq > 0, "not a batched template engine");
    ARG(db->k.kind == IRIS_KIND_TEMPLATES, "database does not hold templates");
    // batches of up to kBatchStreamMax queries stream (any layout); the GEMM reads TILES
    ARG(db->k.layout == IRIS_LAYOUT_TILES || !e->sub.empty(),
        "batched search of more than 3 queries needs a template database in the TILES layout");
    ARG(e->dev == db->dev, "engine and database live on different devices");
    iris_device *d = e->dev;
    std::lock_guard<std::recursive_mutex> g(d->mu);
    CHK(set_device(d));
    CHK(range_ok(db, first, n));
    if (!e->sub.empty()) {
        uint32_t q = 0;
        for (; q + 2 <= e->nq; q += 2) CHK(pair_search_locked(e->sub[q], e->sub[q + 1], db, first, n, index_base, out + q));
        if (q < e->nq) CHK(search_locked(e->sub[q], db, first, n, index_base, nullptr, out + q));
        return 0;
    }
    LaunchRange r{first, n};
    const BatchGeometry geo = batch_geometry(d->hooks, r, e->nq);
    const uint32_t nqp = geo.nqg * geo.qper;
    std::vector<Partial> res(nqp);
    if (n > 0) {
        CHK(ensure(d, d->partials, (size_t)nqp * geo.G * sizeof(Partial)));
        CHK(ensure_host_result(d, (size_t)nqp * sizeof(Partial)));
        CHK(timed(d, "template_batch", n * e->nq, [&] {
            return launch_batch(d->hooks, d->stream, db->data, e->qfrag, r, geo, (Partial *)d->partials.p,
                                (Partial *)d->host_result);
        }));
    }
    CHK(sync(d));
    if (n > 0) memcpy(res.data(), d->host_result, nqp * sizeof(Partial));
    for (uint32_t q = 0; q < e->nq; ++q) {
        const Partial &p = res[q];
        iris_match_t &m = out[q];
        if (n == 0 || p.den == 0) {
            m.distance = INFINITY;
            m.index = UINT64_MAX;
            m.num = 0;
            m.den = 0;
            m.rotation = 0;
        } else {
            m.distance = (double)p.num / (double)p.den;
            m.index = index_base + first + p.idx;
            m.num = p.num;
            m.den = p.den;
            m.rotation = p.rot - IRIS_MAX_ROTATION;
        }
        m.reserved = 0;
    }
    return 0;
}

// ------------------------------------------------------------------ resolver

static int resolver_finish(iris_device *d, uint32_t np, Partial *res) {
    if (np) {
        CHK(ensure_host_result(d, sizeof(Partial)));
        CHK(timed(d, "reduce", np, [&] { return launch_reduce(d->stream, (Partial *)d->partials.p, np, (Partial *)d->host_result); }));
    }
    CHK(sync(d));
    if (np) memcpy(res, d->host_result, sizeof(Partial));
    return 0;
}


// Partial.idx values of one launch are row indices of that launch; chunked
// host calls merge the per-chunk winners on the host in chunk order.
int iris_resolver_search(iris_device_t *d, const uint16_t *const *shares, uint32_t parts, const uint16_t *denoms,
                         uint64_t n, uint64_t index_base, double *dist_out_device, iris_match_t *out) {
    IRIS_KEEP_DEVICE();
    ARG(d && out, "NULL argument");
    ARG(parts >= 1 && parts <= 8, "parts must be 1..8");
    ARG(n == 0 || (shares && denoms), "NULL argument");
    for (uint32_t p = 0; n && p < parts; ++p) ARG(shares[p], "NULL share array");
    std::lock_guard<std::recursive_mutex> g(d->mu);
    CHK(set_device(d));
    const uint32_t np = resolver_partials(n);
    CHK(ensure(d, d->partials, (size_t)std::max<uint32_t>(np, 1) * sizeof(Partial)));
    CHK(timed(d, "resolver", n, [&] {
        return launch_resolver(d->stream, shares, parts, denoms, n, dist_out_device, (Partial *)d->partials.p);
    }));
    Partial res{};
    CHK(resolver_finish(d, n ? np : 0, &res));
    match_from(res, n > 0, index_base, out);
    return 0;
}

// The resolver step with the denominators computed on the fly from the masks
// database (src/main.rs:510-519 + 597-621): TILES runs the fused
// masks_mfma_kernel<MASKS_RESOLVE>; LANES the masks kernel into a workspace
// and then the resolver kernel.
int iris_resolver_search_masks(iris_engine_t *e, const iris_db_t *db, uint64_t first, uint64_t n,
                               const uint16_t *const *shares_device, uint32_t parts, uint64_t index_base,
                               double *dist_out_device, iris_match_t *out) {
    IRIS_KEEP_DEVICE();
    ARG(e && db && out, "NULL argument");
    ARG(parts >= 1 && parts <= 8, "parts must be 1..8");
    ARG(e->kind == IRIS_KIND_MASKS && db->k.kind == IRIS_KIND_MASKS, "needs a masks engine and a masks database");
    ARG(e->dev == db->dev, "engine and database live on different devices");
    ARG(n == 0 || shares_device, "NULL argument");
    for (uint32_t p = 0; n && p < parts; ++p) ARG(shares_device[p], "NULL share array");
    iris_device *d = e->dev;
    std::lock_guard<std::recursive_mutex> g(d->mu);
    CHK(set_device(d));
    CHK(range_ok(db, first, n));
    LaunchRange r{first, n};
    Partial res{};
    if (db->k.layout == IRIS_LAYOUT_TILES) {
        const uint32_t np = n ? masks_resolve_partials(d->hooks, r) : 0;
        CHK(ensure(d, d->partials, (size_t)std::max<uint32_t>(np, 1) * sizeof(Partial)));
        CHK(timed(d, "masks_resolve", n, [&] {
            return launch_masks_resolve(d->hooks, d->stream, db->data, e->qfrag, r, shares_device, parts, dist_out_device,
                                        (Partial *)d->partials.p);
        }));
        CHK(resolver_finish(d, np, &res));
    } else {
        CHK(ensure(d, d->out_a, std::max<uint64_t>(n, 1) * kRot * 2));
        CHK(timed(d, "masks", n, [&] { return launch_masks(d->stream, db->data, e->qtab, r, (uint16_t *)d->out_a.p); }));
        const uint32_t np = resolver_partials(n);
        CHK(ensure(d, d->partials, (size_t)std::max<uint32_t>(np, 1) * sizeof(Partial)));
        CHK(timed(d, "resolver", n, [&] {
            return launch_resolver(d->stream, shares_device, parts, (const uint16_t *)d->out_a.p, n, dist_out_device,
                                   (Partial *)d->partials.p);
        }));
        CHK(resolver_finish(d, n ? np : 0, &res));
    }
    match_from(res, n > 0, index_base, out);
    return 0;
}

// The resolver step from host share arrays and the resident masks database (src/main.rs:510-519 +
// 597-621, the shares as they arrive from the participants): the helper threads sum each chunk's
// parts into a pinned upload slot (62 B per record over the host link), the copy engine moves it to a
// device staging slot, and the fused masks + resolve kernel computes the denominators on the fly
// against the summed rows; each chunk's winner is reduced into its own pinned result slot, the host
// fills the next slot meanwhile, and the call waits once.  LANES databases run chunk by chunk through
// iris_resolver_search_masks.
int iris_resolver_search_masks_host(iris_engine_t *e, const iris_db_t *db, uint64_t first, uint64_t n,
                                    const uint16_t *const *shares, uint32_t parts, uint64_t index_base,
                                    iris_match_t *out) {
    IRIS_KEEP_DEVICE();
    ARG(e && db && out, "NULL argument");
    ARG(parts >= 1 && parts <= 8, "parts must be 1..8");
    ARG(e->kind == IRIS_KIND_MASKS && db->k.kind == IRIS_KIND_MASKS, "needs a masks engine and a masks database");
    ARG(e->dev == db->dev, "engine and database live on different devices");
    ARG(n == 0 || shares, "NULL argument");
    for (uint32_t p = 0; n && p < parts; ++p) ARG(shares[p], "NULL share array");
    iris_device *d = e->dev;
    std::lock_guard<std::recursive_mutex> g(d->mu);
    CHK(set_device(d));
    CHK(range_ok(db, first, n));
    iris_match_t best;
    match_from(Partial{}, false, 0, &best);
    if (n == 0) {
        *out = best;
        return 0;
    }
    const size_t row = (size_t)kRot * 2;
    const uint64_t ch = std::min<uint64_t>(n, kUploadSlot / row / 64 * 64);
    const uint64_t chunks = (n + ch - 1) / ch;
    CHK(ensure_upin(d));
    CHK(ensure(d, d->staging, kUploadSlots * (size_t)ch * row));
    const bool tiles = db->k.layout == IRIS_LAYOUT_TILES;
    uint32_t np_max = 1;
    for (uint64_t c = 0; tiles && c < chunks; ++c)
        np_max = std::max(np_max, masks_resolve_partials(d->hooks, LaunchRange{first + c * ch, std::min(ch, n - c * ch)}));
    if (tiles) {
        CHK(ensure(d, d->partials, (size_t)np_max * sizeof(Partial)));
        CHK(ensure_host_result(d, (size_t)chunks * sizeof(Partial)));
    }
    Partial *res = (Partial *)d->host_result;
    int rc = 0;
    for (uint64_t c = 0; c < chunks && rc == 0; ++c) {
        const uint64_t a = c * ch, m = std::min<uint64_t>(ch, n - a);
        const int b = (int)(c % kUploadSlots);
        // pinned slot b was last read by the copy of chunk c - kUploadSlots
        if (c >= (uint64_t)kUploadSlots && hipEventSynchronize(d->upin_ev[b]) != hipSuccess) {
            rc = fail(IRIS_E_HIP, "hipEventSynchronize");
            break;
        }
        const uint16_t *src[8];
        for (uint32_t p = 0; p < parts; ++p) src[p] = shares[p] + a * kRot;
        parallel_sum_u16((uint16_t *)d->upin[b], src, (int)parts, m * kRot, d->ordinal);
        char *stage = (char *)d->staging.p + (size_t)b * ch * row;
        if (hipMemcpyAsync(stage, d->upin[b], m * row, hipMemcpyHostToDevice, d->stream) != hipSuccess ||
            hipEventRecord(d->upin_ev[b], d->stream) != hipSuccess) {
            rc = fail(IRIS_E_HIP, "hipMemcpyAsync upload");
            break;
        }
        const uint16_t *dsum = (const uint16_t *)stage;
        if (!tiles) {  // the summed rows through the LANES form, one chunk at a time
            iris_match_t cm;
            rc = iris_resolver_search_masks(e, db, first + a, m, &dsum, 1, index_base + a, nullptr, &cm);
            if (rc == 0) {
                iris_match_t pair[2] = {best, cm};
                rc = iris_match_merge(pair, 2, &best);
            }
            continue;
        }
        const LaunchRange r{first + a, m};
        const uint32_t np = masks_resolve_partials(d->hooks, r);
        rc = timed(d, "masks_resolve", m, [&] {
            return launch_masks_resolve(d->hooks, d->stream, db->data, e->qfrag, r, &dsum, 1, nullptr,
                                        (Partial *)d->partials.p);
        });
        // the chunk's winner, its index offset to the call's records, into result slot c
        if (rc == 0)
            rc = timed(d, "reduce", np, [&] { return launch_reduce(d->stream, (Partial *)d->partials.p, np, res + c, a); });
    }
    const int rs = sync(d);  // the pinned slots are free again and every chunk's winner is in place
    CHK(rc);
    CHK(rs);
    for (uint64_t c = 0; tiles && c < chunks; ++c) {
        iris_match_t pair[2] = {best, {}};
        match_from(res[c], true, index_base, &pair[1]);
        CHK(iris_match_merge(pair, 2, &best));
    }
    *out = best;
    return 0;
}

// The resolver step over host arrays (the participants' rows as they arrive, src/main.rs:597-621):
// the helper threads sum a chunk's parts (the wrapping u16 sum the kernel would take first,
// src/main.rs:601-605) into one pinned upload slot beside a copy of its denominators -- 124 B per
// record cross the host link instead of 62 (P + 1) -- the copy engine moves the slot into a device
// staging slot, and the records are decoded + reduced there (the reduce writes the chunk's winner, its index already
// offset, into a pinned result slot), while the host fills the other slot with the next chunk; the
// call waits once, at the end, and merges the chunks' winners in chunk order.  The runtime's own
// copy of a pageable source ran at 29-30 GB/s for some caller arrays and 53-55 GB/s for others
// (profiles/r04_host_upload.txt, r06am_host_resolver.txt), so, as large database writes do, the
// call takes whichever of the two forms was faster lately (a tuner of its own, resolver_tune).
static int resolver_host_pinned(iris_device *d, const uint16_t *const *shares, uint32_t parts, const uint16_t *denoms,
                                uint64_t n, uint64_t index_base, iris_match_t *out) {
    iris_match_t best;
    match_from(Partial{}, false, 0, &best);
    const size_t row = (size_t)kRot * 2;
    const uint32_t arrays = 2;
    // records per slot (the parts' summed rows, then the denominators), a multiple of 64
    const uint64_t ch = std::min<uint64_t>(n, std::max<uint64_t>(64, kUploadSlot / (arrays * row) / 64 * 64));
    const uint64_t chunks = (n + ch - 1) / ch;
    const size_t slot = (size_t)ch * arrays * row;
    CHK(ensure_upin(d));
    CHK(ensure(d, d->staging, kUploadSlots * slot));
    CHK(ensure(d, d->partials, (size_t)std::max<uint32_t>(resolver_partials(ch), 1) * sizeof(Partial)));
    CHK(ensure_host_result(d, (size_t)chunks * sizeof(Partial)));
    Partial *res = (Partial *)d->host_result;
    int rc = 0;
    for (uint64_t c = 0; c < chunks && rc == 0; ++c) {
        const uint64_t a = c * ch, m = std::min<uint64_t>(ch, n - a);
        const int b = (int)(c % kUploadSlots);
        // pinned slot b was last read by the copy of chunk c - kUploadSlots (the previous call's
        // copies ended with its sync)
        if (c >= (uint64_t)kUploadSlots && hipEventSynchronize(d->upin_ev[b]) != hipSuccess) {
            rc = fail(IRIS_E_HIP, "hipEventSynchronize");
            break;
        }
        char *pin = (char *)d->upin[b];
        const uint16_t *src[8];
        for (uint32_t p = 0; p < parts; ++p) src[p] = shares[p] + a * kRot;
        parallel_sum_u16((uint16_t *)pin, src, (int)parts, m * kRot, d->ordinal);
        parallel_copy(pin + m * row, (const char *)(denoms + a * kRot), m * row, d->ordinal);
        char *stage = (char *)d->staging.p + (size_t)b * slot;
        if (hipMemcpyAsync(stage, pin, (size_t)arrays * m * row, hipMemcpyHostToDevice, d->stream) != hipSuccess ||
            hipEventRecord(d->upin_ev[b], d->stream) != hipSuccess) {
            rc = fail(IRIS_E_HIP, "hipMemcpyAsync upload");
            break;
        }
        const uint16_t *dsum = (const uint16_t *)stage;
        const uint16_t *dden = (const uint16_t *)(stage + m * row);
        const uint32_t np = resolver_partials(m);
        rc = timed(d, "resolver", m, [&] {
            return launch_resolver(d->stream, &dsum, 1, dden, m, nullptr, (Partial *)d->partials.p);
        });
        // the chunk's winner, its index offset to the call's records, into result slot c
        if (rc == 0)
            rc = timed(d, "reduce", np, [&] { return launch_reduce(d->stream, (Partial *)d->partials.p, np, res + c, a); });
    }
    const int rs = sync(d);  // the pinned slots are free again and every chunk's winner is in place
    CHK(rc);
    CHK(rs);
    for (uint64_t c = 0; c < chunks; ++c) {
        iris_match_t pair[2] = {best, {}};
        match_from(res[c], true, index_base, &pair[1]);
        CHK(iris_match_merge(pair, 2, &best));
    }
    *out = best;
    return 0;
}

// The runtime's copy of each pageable array into device staging, one chunk of up to 1M records at a
// time, and the device-input resolver on it.
static int resolver_host_runtime(iris_device *d, const uint16_t *const *shares, uint32_t parts, const uint16_t *denoms,
                                 uint64_t n, uint64_t index_base, iris_match_t *out) {
    const uint64_t ch = std::min<uint64_t>(n, 1ull << 20);
    const size_t row = (size_t)kRot * 2;
    CHK(ensure(d, d->staging, std::max<uint64_t>(ch, 1) * row * (parts + 1)));
    iris_match_t best;
    match_from(Partial{}, false, 0, &best);
    for (uint64_t done = 0; done < n; done += ch) {
        const uint64_t m = std::min<uint64_t>(ch, n - done);
        const uint16_t *dev_sh[8];
        for (uint32_t p = 0; p <= parts; ++p) {
            uint16_t *dst = (uint16_t *)((char *)d->staging.p + (size_t)p * ch * row);
            HIPCHK(hipMemcpyAsync(dst, (p < parts ? shares[p] : denoms) + done * kRot, m * row, hipMemcpyHostToDevice,
                                  d->stream));
            if (p < parts) dev_sh[p] = dst;
        }
        const uint16_t *dden = (const uint16_t *)((char *)d->staging.p + (size_t)parts * ch * row);
        iris_match_t cm;
        CHK(iris_resolver_search(d, dev_sh, parts, dden, m, index_base + done, nullptr, &cm));
        iris_match_t pair[2] = {best, cm};
        CHK(iris_match_merge(pair, 2, &best));
    }
    *out = best;
    return 0;
}

int iris_resolver_search_host(iris_device_t *d, const uint16_t *const *shares, uint32_t parts, const uint16_t *denoms,
                              uint64_t n, uint64_t index_base, iris_match_t *out) {
    IRIS_KEEP_DEVICE();
    ARG(d && out, "NULL argument");
    ARG(parts >= 1 && parts <= 8, "parts must be 1..8");
    ARG(n == 0 || (shares && denoms), "NULL argument");
    for (uint32_t p = 0; n && p < parts; ++p) ARG(shares[p], "NULL share array");
    std::lock_guard<std::recursive_mutex> g(d->mu);
    CHK(set_device(d));
    if (n == 0) {
        match_from(Partial{}, false, 0, out);
        return 0;
    }
    const size_t bytes = (size_t)n * kRot * 2 * (parts + 1);
    if (d->hooks.upload == 1 || d->hooks.upload == 2 || bytes < kUploadTuneMin)  // test hook, or small: one path
        return (d->hooks.upload == 1 ? resolver_host_pinned : resolver_host_runtime)(d, shares, parts, denoms, n,
                                                                                      index_base, out);
    UploadTune &u = d->resolver_tune;
    const int path = u.pick();
    const auto t0 = std::chrono::steady_clock::now();
    int rc = path == 0 ? resolver_host_pinned(d, shares, parts, denoms, n, index_base, out)
                       : resolver_host_runtime(d, shares, parts, denoms, n, index_base, out);
    if (rc == IRIS_E_NOMEM && path == 0 && d->upin_cap < kUploadSlot) {  // no pinned slots: the runtime's copy
        u.no_pinned = true;
        return resolver_host_runtime(d, shares, parts, denoms, n, index_base, out);
    }
    CHK(rc);
    u.record(path, (double)bytes / std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count());
    return 0;
}

// ------------------------------------------------------------------ arch plugin

int iris_dot_bool_batch(iris_device_t *d, const uint64_t *a, uint64_t na, const uint64_t *b, uint64_t nb,
                        uint16_t *out) {
    IRIS_KEEP_DEVICE();
    ARG(d, "device is NULL");
    std::lock_guard<std::recursive_mutex> g(d->mu);
    CHK(set_device(d));
    if (na == 0 || nb == 0) return 0;
    ARG(a && b && out, "NULL argument");
    TempDb t;
    CHK(temp_db(d, IRIS_KIND_MASKS, nb, t));
    CHK(db_write_locked(&t.db, 0, b, nb));
    std::vector<uint16_t> tmp(nb * kRot);
    std::vector<uint32_t> tab((size_t)kPlaneDwords * kSlotTabStride);
    std::vector<uint32_t> frag(kMaskFragBytes / 4);
    for (uint64_t i0 = 0; i0 < na; i0 += kRot) {
        const int cnt = (int)std::min<uint64_t>(kRot, na - i0);
        const uint64_t *ptrs[kRot];
        for (int k = 0; k < cnt; ++k) ptrs[k] = a + (i0 + k) * IRIS_LIMBS;
        build_masks_table(ptrs, cnt, tab.data());
        build_masks_frags(ptrs, cnt, frag.data());
        iris_engine *e = nullptr;
        CHK(engine_new(d, IRIS_KIND_MASKS, tab.data(), tab.size() * 4, &e, frag.data(), kMaskFragBytes));
        int rc = run_u16_engine(e, &t.db, 0, nb, tmp.data());
        engine_free(e);
        CHK(rc);
        for (uint64_t j = 0; j < nb; ++j)
            for (int k = 0; k < cnt; ++k) out[j * na + i0 + k] = tmp[j * kRot + k];
    }
    return 0;
}

int iris_dot_u16_batch(iris_device_t *d, const uint16_t *a, uint64_t na, const uint16_t *b, uint64_t nb,
                       uint16_t *out) {
    IRIS_KEEP_DEVICE();
    ARG(d, "device is NULL");
    std::lock_guard<std::recursive_mutex> g(d->mu);
    CHK(set_device(d));
    if (na == 0 || nb == 0) return 0;
    ARG(a && b && out, "NULL argument");
    TempDb t;
    CHK(temp_db(d, IRIS_KIND_SHARES, nb, t));
    CHK(db_write_locked(&t.db, 0, b, nb));
    std::vector<uint16_t> tmp(nb * kRot);
    std::vector<uint32_t> tab((size_t)kShareDwords * kSlotTabStride);
    std::vector<uint32_t> frag(kShareFragBytes / 4);
    for (uint64_t i0 = 0; i0 < na; i0 += kRot) {
        const int cnt = (int)std::min<uint64_t>(kRot, na - i0);
        const uint16_t *ptrs[kRot];
        for (int k = 0; k < cnt; ++k) ptrs[k] = a + (i0 + k) * IRIS_BITS;
        build_shares_table(ptrs, cnt, tab.data());
        build_shares_frags(ptrs, cnt, frag.data());
        iris_engine *e = nullptr;
        CHK(engine_new(d, IRIS_KIND_SHARES, tab.data(), tab.size() * 4, &e, frag.data(), kShareFragBytes));
        int rc = run_u16_engine(e, &t.db, 0, nb, tmp.data());
        engine_free(e);
        CHK(rc);
        for (uint64_t j = 0; j < nb; ++j)
            for (int k = 0; k < cnt; ++k) out[j * na + i0 + k] = tmp[j * kRot + k];
    }
    return 0;
}

// ------------------------------------------------------------------ host helpers

int iris_bits_rotated(const uint64_t in[IRIS_LIMBS], int32_t amount, uint64_t out[IRIS_LIMBS]) {
    ARG(in && out, "NULL argument");
    bits_rotated(in, amount, out);
    return 0;
}

int iris_encoded_rotated(const uint16_t in[IRIS_BITS], int32_t amount, uint16_t out[IRIS_BITS]) {
    ARG(in && out, "NULL argument");
    if (in == out) {
        std::vector<uint16_t> tmp(in, in + IRIS_BITS);
        encoded_rotated(tmp.data(), amount, out);
    } else {
        encoded_rotated(in, amount, out);
    }
    return 0;
}

int iris_encode(const iris_template_t *t, uint16_t out[IRIS_BITS]) {
    ARG(t && out, "NULL argument");
    encode_template(t, out);
    return 0;
}

int iris_decode_distance(const uint16_t distances[IRIS_ROTATIONS], const uint16_t denominators[IRIS_ROTATIONS],
                         double *out) {
    ARG(distances && denominators && out, "NULL argument");
    double acc = INFINITY;
    for (int k = 0; k < kRot; ++k) {
        const uint16_t n = distances[k], dd = denominators[k];
        const uint16_t uneq = (uint16_t)((uint16_t)(dd - n) / 2);  // src/lib.rs:104
        acc = rust_f64_min(acc, (double)uneq / (double)dd);        // src/lib.rs:105-106
    }
    *out = acc;
    return 0;
}

int iris_query_table_sizes(int kind, uint32_t nq, size_t *tab_bytes, size_t *frag_bytes) {
    ARG(tab_bytes && frag_bytes, "NULL argument");
    switch (kind) {
    case IRIS_KIND_TEMPLATES:
        ARG(nq == 0 || nq > kBatchStreamMax, "nq must be 0 (single query) or a tiled batch (> 3 queries)");
        *tab_bytes = nq ? 0 : (size_t)kPlaneDwords * kTemplateTabStride * 4;
        *frag_bytes = nq ? (size_t)(nq + batch_query_group() - 1) / batch_query_group() * batch_query_group() * 16 * kPlaneGroups * 64 : kTemplateFragDwords * 4;
        return 0;
    case IRIS_KIND_MASKS:
        *tab_bytes = (size_t)kPlaneDwords * kSlotTabStride * 4;
        *frag_bytes = kMaskFragBytes;
        return 0;
    case IRIS_KIND_SHARES:
        *tab_bytes = (size_t)kShareDwords * kSlotTabStride * 4;
        *frag_bytes = kShareFragBytes;
        return 0;
    default: return fail(IRIS_E_ARG, "unknown record kind");
    }
}

int iris_engine_query_tables(const iris_engine_t *e, void *tab, size_t tab_bytes, void *frag, size_t frag_bytes) {
    IRIS_KEEP_DEVICE();
    ARG(e, "engine is NULL");
    ARG(e->sub.empty(), "a streamed batch engine (<= 3 queries) holds one engine per query");
    size_t tb = 0, fb = 0;
    CHK(iris_query_table_sizes(e->kind, e->nq, &tb, &fb));
    ARG(tab_bytes == tb && frag_bytes == fb, "table sizes do not match the engine's layout");
    ARG((tb == 0 || tab) && frag, "NULL argument");
    iris_device *d = e->dev;
    std::lock_guard<std::recursive_mutex> g(d->mu);
    CHK(set_device(d));
    if (tb) HIPCHK(hipMemcpyAsync(tab, e->qtab, tb, hipMemcpyDeviceToHost, d->stream));
    HIPCHK(hipMemcpyAsync(frag, e->qfrag, fb, hipMemcpyDeviceToHost, d->stream));
    return sync(d);
}

int iris_host_query_tables(int kind, const void *query, uint32_t nq, void *tab, size_t tab_bytes, void *frag,
                           size_t frag_bytes) {
    ARG(query, "query is NULL");
    size_t tb = 0, fb = 0;
    CHK(iris_query_table_sizes(kind, nq, &tb, &fb));
    ARG(tab_bytes == tb && frag_bytes == fb, "table sizes do not match the layout");
    ARG((tb == 0 || tab) && frag, "NULL argument");
    if (kind == IRIS_KIND_TEMPLATES && nq) {
        const size_t tile_dw = (size_t)4 * kPlaneGroups * 64;
        memset(frag, 0, fb);
        for (uint32_t i = 0; i < nq; ++i)
            build_query_tile((const iris_template_t *)query + i, (uint32_t *)frag + i * tile_dw);
    } else if (kind == IRIS_KIND_TEMPLATES) {
        build_template_table((const iris_template_t *)query, (uint32_t *)tab);
        build_template_frags((const iris_template_t *)query, (uint32_t *)frag);
    } else if (kind == IRIS_KIND_MASKS) {
        build_masks_rotations((const uint64_t *)query, (uint32_t *)tab);
        std::vector<uint64_t> rot((size_t)kRot * IRIS_LIMBS);
        const uint64_t *ptrs[kRot];
        for (int k = 0; k < kRot; ++k) {
            bits_rotated((const uint64_t *)query, k - 15, &rot[(size_t)k * IRIS_LIMBS]);
            ptrs[k] = &rot[(size_t)k * IRIS_LIMBS];
        }
        build_masks_frags(ptrs, kRot, (uint32_t *)frag);
    } else {
        build_shares_rotations((const uint16_t *)query, (uint32_t *)tab);
        std::vector<uint16_t> rot((size_t)kRot * IRIS_BITS);
        const uint16_t *ptrs[kRot];
        for (int k = 0; k < kRot; ++k) {
            encoded_rotated((const uint16_t *)query, k - 15, &rot[(size_t)k * IRIS_BITS]);
            ptrs[k] = &rot[(size_t)k * IRIS_BITS];
        }
        build_shares_frags(ptrs, kRot, (uint32_t *)frag);
    }
    return 0;
}

int iris_match_merge(const iris_match_t *recs, uint64_t count, iris_match_t *out) {
    ARG(out && (count == 0 || recs), "NULL argument");
    iris_match_t best;
    best.distance = INFINITY;
    best.index = UINT64_MAX;
    best.num = 0;
    best.den = 0;
    best.rotation = 0;
    best.reserved = 0;
    for (uint64_t i = 0; i < count; ++i) {
        const iris_match_t &c = recs[i];
        if (c.den == 0 || c.index == UINT64_MAX) continue;
        bool take = best.den == 0;
        if (!take) {
            const uint64_t l = (uint64_t)c.num * best.den, r = (uint64_t)best.num * c.den;
            take = l < r || (l == r && c.index < best.index);
        }
        if (take) best = c;
    }
    *out = best;
    return 0;
}

}  // extern "C"
