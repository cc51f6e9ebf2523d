// iris_group.hip — device groups (include/iris_hip.h, "device groups"): a
// template database split into contiguous shards over the gfx950 devices of a
// group, searched on every device with no data-path communication; the
// per-shard winners are exchanged with one RCCL ncclAllGather over xGMI and
// merged on every device.
//
// Reference counterpart: the resolver's fan-out of a query to its participants
// and the sequential strict-< minimum over their answers (src/main.rs:486-504,
// 616-621) — here the "participants" are shards of one database, and the
// minimum is exact (u32 cross-multiplied fractions, then the lowest global
// index), so the group's answer equals a single search over the concatenated
// database.
//
// Exchange record: one Partial (24 B: num, den, rotation, global index) per
// shard and query.  Pipelined searches run the partials reduce, the all-gather
// and the merge on each device's side stream, in order, so one send / recv
// buffer per device serves every search in flight while the next search's
// kernel already runs on the main stream.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>
#include <string.h>

#include <new>
#include <thread>

#include "iris_handles.hpp"

using namespace iris;
using namespace iris_api;

#define NCCLCHK(x)                                                                                         \
    do {                                                                                                   \
        ncclResult_t r_ = (x);                                                                             \
        if (r_ != ncclSuccess) return fail(IRIS_E_HIP, std::string(#x) + ": " + ncclGetErrorString(r_)); \
    } while (0)

struct iris_group {
    std::vector<iris_device *> devs;  // local devices (owned)
    std::vector<ncclComm_t> comms;    // comms[i]: local device i, RCCL rank rank0 + i
    uint32_t ranks = 0, rank0 = 0;
    std::mutex mu;                    // serialises group calls
    std::atomic<int> refs{1};         // the group handle + each database and pending search
};

struct iris_group_db {
    iris_group *g = nullptr;
    int kind = 0, layout = 0;
    uint64_t total = 0;
    uint32_t spd = 1, S = 0, first_shard = 0;
    std::vector<iris_db *> shards;          // local shard i lives on local device i / spd
    std::vector<uint64_t> first, count;     // global index of record 0, records
    std::vector<DevBuf> send, recv;         // per local device: [spd] / [S] Partials (single query)
};

struct iris_group_pending {
    iris_group *g = nullptr;
    std::vector<Partial *> slots;  // pinned merge result of each local device
    std::vector<hipEvent_t> evs;   // recorded after each device's merge
};

namespace {

void group_teardown(iris_group *g) {
    for (size_t i = 0; i < g->comms.size(); ++i) {
        if (!g->comms[i]) continue;
        (void)hipSetDevice(g->devs[i]->ordinal);
        (void)hipStreamSynchronize(g->devs[i]->stream);
        if (g->devs[i]->aux) (void)hipStreamSynchronize(g->devs[i]->aux);
        (void)ncclCommDestroy(g->comms[i]);
    }
    for (iris_device *d : g->devs) iris_device_close(d);
    delete g;
}

void group_retain(iris_group *g) { g->refs.fetch_add(1, std::memory_order_relaxed); }
void group_release(iris_group *g) {
    if (g->refs.fetch_sub(1, std::memory_order_acq_rel) == 1) group_teardown(g);
}

// Opens the local devices; on failure closes what was opened.
int open_devices(iris_group *g, const int *ordinals, uint32_t n) {
    for (uint32_t i = 0; i < n; ++i) {
        for (uint32_t j = 0; j < i; ++j)
            if (ordinals[j] == ordinals[i]) return fail(IRIS_E_ARG, "a device appears twice in the group (RCCL needs one rank per device)");
        iris_device *d = nullptr;
        CHK(iris_device_open(ordinals[i], &d));
        g->devs.push_back(d);
        CHK(set_device(d));
        CHK(ensure_aux(d));
    }
    return 0;
}

// Runs fn(i) for every local device i, one host thread per device when there are
// several; returns the first failure (its message re-raised on this thread).
template <class F>
int per_device(iris_group *g, F &&fn) {
    const size_t n = g->devs.size();
    if (n == 1) return fn(0);
    std::vector<int> rc(n, 0);
    std::vector<std::string> msg(n);
    std::vector<std::thread> th;
    for (size_t i = 0; i < n; ++i)
        th.emplace_back([&, i] {
            rc[i] = fn(i);
            if (rc[i] != 0) msg[i] = g_err;
        });
    for (auto &t : th) t.join();
    for (size_t i = 0; i < n; ++i)
        if (rc[i] != 0) return fail(rc[i], msg[i]);
    return 0;
}

// Locks every local device (in order) for the duration of a group enqueue.
struct DeviceLocks {
    std::vector<std::unique_lock<std::recursive_mutex>> l;
    explicit DeviceLocks(iris_group *g) {
        for (iris_device *d : g->devs) l.emplace_back(d->mu);
    }
};

inline uint64_t shard_first(uint64_t total, uint32_t S, uint32_t s) {
    return (uint64_t)((unsigned __int128)total * s / S);
}

int search_args(iris_group_db *gdb) {
    ARG(gdb, "NULL argument");
    ARG(gdb->kind == IRIS_KIND_TEMPLATES, "group search needs a template database");
    return 0;
}

bool same_partial(const Partial &a, const Partial &b) {
    if (a.den == 0 || b.den == 0) return a.den == b.den;
    return a.num == b.num && a.den == b.den && a.rot == b.rot && a.idx == b.idx;
}

// All local devices' merged winners must agree (every device merges the same gathered records).
int agree(const std::vector<Partial> &res, uint32_t nq, uint32_t stride, Partial *out) {
    for (size_t i = 1; i < res.size() / stride; ++i)
        for (uint32_t q = 0; q < nq; ++q)
            if (!same_partial(res[q], res[i * stride + q]))
                return fail(IRIS_E_HIP, "group merge: local devices disagree on the winner of query " + std::to_string(q));
    for (uint32_t q = 0; q < nq; ++q) out[q] = res[q];
    return 0;
}

void fill_match(const Partial &p, iris_match_t *m) { match_from(p, true, 0, m); }

// Frees a group database's shards and exchange buffers (caller holds the group lock).
void gdb_free_locked(iris_group_db *gdb) {
    iris_group *g = gdb->g;
    for (iris_db *db : gdb->shards) iris_db_destroy(db);  // waits for its device
    for (size_t i = 0; i < gdb->send.size(); ++i) {
        iris_device *d = g->devs[i];
        std::lock_guard<std::recursive_mutex> l(d->mu);
        (void)hipSetDevice(d->ordinal);
        if (d->aux) (void)hipStreamSynchronize(d->aux);
        if (gdb->send[i].p) (void)hipFree(gdb->send[i].p);
        if (gdb->recv[i].p) (void)hipFree(gdb->recv[i].p);
    }
    delete gdb;
}

}  // namespace

extern "C" {

int iris_group_unique_id(uint8_t id[IRIS_GROUP_ID_BYTES]) {
    ARG(id, "NULL argument");
    static_assert(sizeof(ncclUniqueId) == IRIS_GROUP_ID_BYTES, "RCCL unique id size");
    ncclUniqueId u;
    NCCLCHK(ncclGetUniqueId(&u));
    memcpy(id, &u, sizeof(u));
    return 0;
}

int iris_group_create(const int *ordinals, uint32_t n, iris_group_t **out) {
    IRIS_KEEP_DEVICE();
    ARG(ordinals && out && n > 0, "a group needs at least one device");
    iris_group *g = new (std::nothrow) iris_group();
    if (!g) return fail(IRIS_E_NOMEM, "out of host memory");
    g->ranks = n;
    g->rank0 = 0;
    int rc = open_devices(g, ordinals, n);
    if (rc == 0) {
        g->comms.assign(n, nullptr);
        const ncclResult_t r = ncclCommInitAll(g->comms.data(), (int)n, ordinals);
        if (r != ncclSuccess) {
            g->comms.assign(n, nullptr);
            rc = fail(IRIS_E_HIP, std::string("ncclCommInitAll: ") + ncclGetErrorString(r));
        }
    }
    if (rc != 0) {
        const std::string m = g_err;
        group_teardown(g);
        return fail(rc, m);
    }
    *out = g;
    return 0;
}

int iris_group_create_rank(int ordinal, uint32_t nranks, uint32_t rank, const uint8_t id[IRIS_GROUP_ID_BYTES],
                           iris_group_t **out) {
    IRIS_KEEP_DEVICE();
    ARG(id && out, "NULL argument");
    ARG(nranks > 0 && rank < nranks, "rank must be below nranks");
    iris_group *g = new (std::nothrow) iris_group();
    if (!g) return fail(IRIS_E_NOMEM, "out of host memory");
    g->ranks = nranks;
    g->rank0 = rank;
    int rc = open_devices(g, &ordinal, 1);
    if (rc == 0) {
        ncclUniqueId u;
        memcpy(&u, id, sizeof(u));
        g->comms.assign(1, nullptr);
        const ncclResult_t r = ncclCommInitRank(&g->comms[0], (int)nranks, u, (int)rank);
        if (r != ncclSuccess) {
            g->comms[0] = nullptr;
            rc = fail(IRIS_E_HIP, std::string("ncclCommInitRank: ") + ncclGetErrorString(r));
        }
    }
    if (rc != 0) {
        const std::string m = g_err;
        group_teardown(g);
        return fail(rc, m);
    }
    *out = g;
    return 0;
}

int iris_group_destroy(iris_group_t *g) {
    IRIS_KEEP_DEVICE();
    if (!g) return 0;
    group_release(g);  // torn down now, or with its last database / pending search
    return 0;
}

int iris_group_info(const iris_group_t *g, uint32_t *local_devices, uint32_t *ranks, uint32_t *first_rank) {
    ARG(g, "NULL argument");
    if (local_devices) *local_devices = (uint32_t)g->devs.size();
    if (ranks) *ranks = g->ranks;
    if (first_rank) *first_rank = g->rank0;
    return 0;
}

int iris_group_device(const iris_group_t *g, uint32_t i, iris_device_t **dev) {
    ARG(g && dev, "NULL argument");
    ARG(i < g->devs.size(), "device index out of range");
    *dev = g->devs[i];
    return 0;
}

int iris_group_db_destroy(iris_group_db_t *gdb) {
    IRIS_KEEP_DEVICE();
    if (!gdb) return 0;
    iris_group *g = gdb->g;
    {
        std::lock_guard<std::mutex> gl(g->mu);
        gdb_free_locked(gdb);
    }
    group_release(g);
    return 0;
}

int iris_group_db_create(iris_group_t *g, int kind, uint64_t total, int layout, uint32_t spd, iris_group_db_t **out) {
    IRIS_KEEP_DEVICE();
    ARG(g && out, "NULL argument");
    ARG(spd >= 1, "shards_per_device must be at least 1");
    CHK(check_kind(kind));
    std::lock_guard<std::mutex> gl(g->mu);
    iris_group_db *gdb = new (std::nothrow) iris_group_db();
    if (!gdb) return fail(IRIS_E_NOMEM, "out of host memory");
    gdb->g = g;
    group_retain(g);
    gdb->kind = kind;
    gdb->layout = layout;
    gdb->total = total;
    gdb->spd = spd;
    gdb->S = g->ranks * spd;
    gdb->first_shard = g->rank0 * spd;
    const uint32_t L = (uint32_t)g->devs.size();
    int rc = 0;
    for (uint32_t i = 0; i < L * spd && rc == 0; ++i) {
        const uint32_t s = gdb->first_shard + i;
        const uint64_t f = shard_first(total, gdb->S, s), c = shard_first(total, gdb->S, s + 1) - f;
        iris_db *db = nullptr;
        rc = iris_db_create_ex(g->devs[i / spd], kind, c, layout, &db);
        if (rc != 0) break;
        db->len = c;  // zero records: empty masks, never a candidate
        gdb->shards.push_back(db);
        gdb->first.push_back(f);
        gdb->count.push_back(c);
    }
    gdb->send.resize(L);
    gdb->recv.resize(L);
    for (uint32_t i = 0; i < L && rc == 0; ++i) {
        iris_device *d = g->devs[i];
        std::lock_guard<std::recursive_mutex> l(d->mu);
        rc = set_device(d);
        if (rc == 0) rc = ensure(gdb->send[i], (size_t)spd * sizeof(Partial));
        if (rc == 0) rc = ensure(gdb->recv[i], (size_t)gdb->S * sizeof(Partial));
    }
    if (rc != 0) {
        const std::string m = g_err;
        gdb_free_locked(gdb);
        group_release(g);  // never the last reference: the caller's group handle holds one
        return fail(rc, m);
    }
    *out = gdb;
    return 0;
}

int iris_group_db_info(const iris_group_db_t *gdb, uint64_t *total, uint32_t *shards, uint32_t *first_shard,
                       uint32_t *local_shards) {
    ARG(gdb, "NULL argument");
    if (total) *total = gdb->total;
    if (shards) *shards = gdb->S;
    if (first_shard) *first_shard = gdb->first_shard;
    if (local_shards) *local_shards = (uint32_t)gdb->shards.size();
    return 0;
}

int iris_group_db_shard(const iris_group_db_t *gdb, uint32_t i, iris_db_t **db, uint64_t *first, uint64_t *count) {
    ARG(gdb, "NULL argument");
    ARG(i < gdb->shards.size(), "shard index out of range");
    if (db) *db = gdb->shards[i];
    if (first) *first = gdb->first[i];
    if (count) *count = gdb->count[i];
    return 0;
}

int iris_group_db_generate(iris_group_db_t *gdb, uint64_t seed) {
    IRIS_KEEP_DEVICE();
    ARG(gdb, "NULL argument");
    iris_group *g = gdb->g;
    std::lock_guard<std::mutex> gl(g->mu);
    return per_device(g, [&](size_t i) {
        for (uint32_t j = 0; j < gdb->spd; ++j) {
            const size_t s = i * gdb->spd + j;
            iris_db *db = gdb->shards[s];
            db->len = 0;
            const int rc = iris_db_generate(db, gdb->count[s], seed, gdb->first[s]);
            db->len = gdb->count[s];
            CHK(rc);
        }
        return 0;
    });
}

int iris_group_db_write(iris_group_db_t *gdb, uint64_t index, const void *records, uint64_t n) {
    IRIS_KEEP_DEVICE();
    ARG(gdb, "NULL argument");
    if (index > gdb->total || n > gdb->total - index) return fail(IRIS_E_RANGE, "record range outside the group database");
    if (n == 0) return 0;
    ARG(records, "records is NULL");
    const size_t rb = kind_info(gdb->kind).rec_bytes;
    std::lock_guard<std::mutex> gl(gdb->g->mu);
    for (size_t s = 0; s < gdb->shards.size(); ++s) {
        const uint64_t lo = std::max(index, gdb->first[s]), hi = std::min(index + n, gdb->first[s] + gdb->count[s]);
        if (lo >= hi) continue;
        CHK(iris_db_write(gdb->shards[s], lo - gdb->first[s], (const char *)records + (lo - index) * rb, hi - lo));
    }
    return 0;
}

int iris_group_db_read(const iris_group_db_t *gdb, uint64_t index, uint64_t n, void *records) {
    IRIS_KEEP_DEVICE();
    ARG(gdb, "NULL argument");
    if (index > gdb->total || n > gdb->total - index) return fail(IRIS_E_RANGE, "record range outside the group database");
    if (n == 0) return 0;
    ARG(records, "records is NULL");
    const uint64_t lo_local = gdb->shards.empty() ? 0 : gdb->first.front();
    const uint64_t hi_local = gdb->shards.empty() ? 0 : gdb->first.back() + gdb->count.back();
    if (index < lo_local || index + n > hi_local)
        return fail(IRIS_E_RANGE, "iris_group_db_read: the range is not held by this process's shards");
    const size_t rb = kind_info(gdb->kind).rec_bytes;
    std::lock_guard<std::mutex> gl(gdb->g->mu);
    for (size_t s = 0; s < gdb->shards.size(); ++s) {
        const uint64_t lo = std::max(index, gdb->first[s]), hi = std::min(index + n, gdb->first[s] + gdb->count[s]);
        if (lo >= hi) continue;
        CHK(iris_db_read(gdb->shards[s], lo - gdb->first[s], hi - lo, (char *)records + (lo - index) * rb));
    }
    return 0;
}

int iris_group_db_load_file(iris_group_db_t *gdb, const char *path, uint64_t first) {
    IRIS_KEEP_DEVICE();
    ARG(gdb && path, "NULL argument");
    iris_group *g = gdb->g;
    std::lock_guard<std::mutex> gl(g->mu);
    return per_device(g, [&](size_t i) {
        for (uint32_t j = 0; j < gdb->spd; ++j) {
            const size_t s = i * gdb->spd + j;
            iris_db *db = gdb->shards[s];
            const uint64_t c = gdb->count[s];
            if (c == 0) continue;
            db->len = 0;
            uint64_t got = 0;
            const int rc = iris_db_load_file(db, path, first + gdb->first[s], c, &got);
            db->len = c;
            CHK(rc);
            if (got != c)
                return fail(IRIS_E_RANGE, std::string("iris_group_db_load_file: ") + path + " holds fewer than first + total records");
        }
        return 0;
    });
}

int iris_group_template_search_async(iris_group_db_t *gdb, const iris_template_t *query, iris_group_pending_t **out) {
    IRIS_KEEP_DEVICE();
    CHK(search_args(gdb));
    ARG(query && out, "NULL argument");
    iris_group *g = gdb->g;
    std::lock_guard<std::mutex> gl(g->mu);
    DeviceLocks locks(g);
    const size_t L = g->devs.size();
    iris_group_pending *p = new (std::nothrow) iris_group_pending();
    if (!p) return fail(IRIS_E_NOMEM, "out of host memory");
    p->g = g;
    p->slots.assign(L, nullptr);
    p->evs.assign(L, nullptr);
    auto abandon = [&](int rc) {
        const std::string m = g_err;
        for (size_t i = 0; i < L; ++i) {
            iris_device *d = g->devs[i];
            (void)hipSetDevice(d->ordinal);
            (void)hipStreamSynchronize(d->stream);
            if (d->aux) (void)hipStreamSynchronize(d->aux);
            if (p->slots[i]) d->free_slots.push_back(p->slots[i]);
            if (p->evs[i]) d->event_pool.push_back(p->evs[i]);
        }
        delete p;
        return fail(rc, m);
    };
    // per device: the query's engine, then every local shard's search + reduce (side stream)
    for (size_t i = 0; i < L; ++i) {
        iris_device *d = g->devs[i];
        int rc = set_device(d);
        iris_engine *e = nullptr;
        if (rc == 0) rc = take_result_slot(d, &p->slots[i]);
        if (rc == 0 && !(p->evs[i] = take_event(d))) rc = fail(IRIS_E_HIP, "hipEventCreate failed");
        if (rc == 0) rc = template_engine_locked(d, query, &e);
        Partial *send = (Partial *)gdb->send[i].p;
        for (uint32_t j = 0; rc == 0 && j < gdb->spd; ++j) {
            const size_t s = i * gdb->spd + j;
            if (gdb->count[s] == 0) {  // an empty shard sends "no candidate"
                if (hipMemsetAsync(send + j, 0, sizeof(Partial), d->aux) != hipSuccess)
                    rc = fail(IRIS_E_HIP, "hipMemsetAsync");
            } else {
                rc = search_enqueue(e, gdb->shards[s], 0, gdb->count[s], nullptr, send + j, true, nullptr, gdb->first[s]);
            }
        }
        if (e) engine_free(e);
        if (rc != 0) return abandon(rc);
    }
    // the exchange: every device's shard winners to every device (side streams, in order after the reduces)
    {
        ncclResult_t r = ncclGroupStart();
        for (size_t i = 0; r == ncclSuccess && i < L; ++i)
            r = ncclAllGather(gdb->send[i].p, gdb->recv[i].p, (size_t)gdb->spd * sizeof(Partial), ncclUint8, g->comms[i],
                              g->devs[i]->aux);
        const ncclResult_t r2 = ncclGroupEnd();
        if (r == ncclSuccess) r = r2;
        if (r != ncclSuccess) return abandon(fail(IRIS_E_HIP, std::string("ncclAllGather: ") + ncclGetErrorString(r)));
    }
    for (size_t i = 0; i < L; ++i) {
        iris_device *d = g->devs[i];
        int rc = set_device(d);
        if (rc == 0)
            rc = timed(d, "group_merge", gdb->S, [&] {
                return launch_group_merge(d->aux, (const Partial *)gdb->recv[i].p, gdb->S, 1, 1, p->slots[i]);
            }, d->aux);
        if (rc == 0 && hipEventRecord(p->evs[i], d->aux) != hipSuccess) rc = fail(IRIS_E_HIP, "hipEventRecord");
        if (rc != 0) return abandon(rc);
    }
    group_retain(g);
    *out = p;
    return 0;
}

int iris_group_pending_wait(iris_group_pending_t *p, iris_match_t *out) {
    IRIS_KEEP_DEVICE();
    ARG(p, "pending is NULL");
    iris_group *g = p->g;
    const size_t L = g->devs.size();
    std::vector<Partial> res(L);
    hipError_t err = hipSuccess;
    for (size_t i = 0; i < L; ++i) {
        const hipError_t e = hipEventSynchronize(p->evs[i]);
        if (e != hipSuccess && err == hipSuccess) err = e;
        if (e == hipSuccess) memcpy(&res[i], p->slots[i], sizeof(Partial));
    }
    for (size_t i = 0; i < L; ++i) {
        iris_device *d = g->devs[i];
        std::lock_guard<std::recursive_mutex> l(d->mu);
        d->free_slots.push_back(p->slots[i]);
        d->event_pool.push_back(p->evs[i]);
        fold_done(d);
    }
    delete p;
    group_release(g);
    if (err != hipSuccess) return fail(IRIS_E_HIP, std::string("hipEventSynchronize: ") + hipGetErrorString(err));
    Partial best;
    CHK(agree(res, 1, 1, &best));
    if (out) fill_match(best, out);
    return 0;
}

int iris_group_template_search(iris_group_db_t *gdb, const iris_template_t *query, iris_match_t *out) {
    IRIS_KEEP_DEVICE();
    ARG(out, "out is NULL");
    iris_group_pending *p = nullptr;
    CHK(iris_group_template_search_async(gdb, query, &p));
    return iris_group_pending_wait(p, out);
}

int iris_group_template_batch_search(iris_group_db_t *gdb, const iris_template_t *queries, uint32_t nq,
                                     iris_match_t *out) {
    IRIS_KEEP_DEVICE();
    CHK(search_args(gdb));
    ARG(queries && out, "NULL argument");
    ARG(nq > 0, "a batch needs at least one query");
    ARG(nq <= kBatchStreamMax || gdb->layout == IRIS_LAYOUT_DEFAULT || gdb->layout == IRIS_LAYOUT_TILES,
        "batched search of more than 3 queries needs a template database in the TILES layout");
    iris_group *g = gdb->g;
    std::lock_guard<std::mutex> gl(g->mu);
    DeviceLocks locks(g);
    const size_t L = g->devs.size();
    const uint32_t spd = gdb->spd, S = gdb->S;
    const uint32_t stride = nq <= kBatchStreamMax ? nq : (nq + batch_query_group() - 1) / batch_query_group() * batch_query_group();
    std::vector<DevBuf> send(L), recv(L);
    std::vector<iris_engine *> eng(L, nullptr);
    auto cleanup = [&] {
        for (size_t i = 0; i < L; ++i) {
            iris_device *d = g->devs[i];
            (void)hipSetDevice(d->ordinal);
            (void)hipStreamSynchronize(d->stream);
            if (eng[i]) iris_engine_destroy(eng[i]);
            if (send[i].p) (void)hipFree(send[i].p);
            if (recv[i].p) (void)hipFree(recv[i].p);
        }
    };
    int rc = 0;
    for (size_t i = 0; i < L && rc == 0; ++i) {
        iris_device *d = g->devs[i];
        rc = set_device(d);
        if (rc == 0) rc = ensure(send[i], (size_t)spd * stride * sizeof(Partial));
        if (rc == 0) rc = ensure(recv[i], (size_t)S * stride * sizeof(Partial));
        if (rc == 0) rc = ensure_host_result(d, (size_t)stride * sizeof(Partial));
        if (rc == 0) rc = iris_template_batch_engine_new(d, queries, nq, &eng[i]);
        if (rc != 0) break;
        iris_engine *e = eng[i];
        Partial *sbuf = (Partial *)send[i].p;
        if (hipMemsetAsync(sbuf, 0, (size_t)spd * stride * sizeof(Partial), d->stream) != hipSuccess) {
            rc = fail(IRIS_E_HIP, "hipMemsetAsync");
            break;
        }
        if (!e->sub.empty()) {  // up to 3 queries: one streamed search per query and shard
            for (uint32_t j = 0; rc == 0 && j < spd; ++j) {
                const size_t s = i * spd + j;
                for (uint32_t q = 0; rc == 0 && q < nq; ++q)
                    rc = search_enqueue(e->sub[q], gdb->shards[s], 0, gdb->count[s], nullptr, sbuf + (size_t)j * stride + q,
                                        false, nullptr, gdb->first[s]);
            }
        } else {  // the LDS-tiled GEMM per shard (iris_batch.hip)
            size_t pmax = 0;
            for (uint32_t j = 0; j < spd; ++j) {
                const size_t s = i * spd + j;
                const BatchGeometry geo = batch_geometry(LaunchRange{0, gdb->count[s]}, nq);
                pmax = std::max(pmax, (size_t)geo.nqg * geo.qper * geo.G * sizeof(Partial));
            }
            rc = ensure(d->partials, pmax);
            for (uint32_t j = 0; rc == 0 && j < spd; ++j) {
                const size_t s = i * spd + j;
                if (gdb->count[s] == 0) continue;
                const LaunchRange r{0, gdb->count[s]};
                const BatchGeometry geo = batch_geometry(r, nq);
                rc = timed(d, "template_batch", r.n * nq, [&] {
                    return launch_batch(d->stream, gdb->shards[s]->data, e->qfrag, r, geo, (Partial *)d->partials.p,
                                        sbuf + (size_t)j * stride, gdb->first[s]);
                });
            }
        }
    }
    if (rc == 0) {
        ncclResult_t r = ncclGroupStart();
        for (size_t i = 0; r == ncclSuccess && i < L; ++i)
            r = ncclAllGather(send[i].p, recv[i].p, (size_t)spd * stride * sizeof(Partial), ncclUint8, g->comms[i],
                              g->devs[i]->stream);
        const ncclResult_t r2 = ncclGroupEnd();
        if (r == ncclSuccess) r = r2;
        if (r != ncclSuccess) rc = fail(IRIS_E_HIP, std::string("ncclAllGather: ") + ncclGetErrorString(r));
    }
    for (size_t i = 0; i < L && rc == 0; ++i) {
        iris_device *d = g->devs[i];
        rc = set_device(d);
        if (rc == 0)
            rc = timed(d, "group_merge", (uint64_t)S * nq, [&] {
                return launch_group_merge(d->stream, (const Partial *)recv[i].p, S, nq, stride, (Partial *)d->host_result);
            });
    }
    std::vector<Partial> res((size_t)L * stride);
    for (size_t i = 0; i < L && rc == 0; ++i) {
        iris_device *d = g->devs[i];
        rc = set_device(d);
        if (rc == 0) rc = sync(d);
        if (rc == 0) memcpy(&res[i * stride], d->host_result, (size_t)nq * sizeof(Partial));
    }
    const std::string m = rc != 0 ? g_err : std::string();
    cleanup();
    if (rc != 0) return fail(rc, m);
    std::vector<Partial> best(nq);
    CHK(agree(res, nq, stride, best.data()));
    for (uint32_t q = 0; q < nq; ++q) fill_match(best[q], out + q);
    return 0;
}

}  // extern "C"
