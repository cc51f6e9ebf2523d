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
// and the merge on each device's side stream, in order, while the next search's
// kernel already runs on the main stream.  The shard winners are written into a
// ring of kSendRing send slots per device: a small (fused) shard search writes
// its winner from the kernel itself, on the MAIN stream, so search k's kernels
// wait for the all-gather that last read their slot (search k - kSendRing) --
// without that order a search's kernel could overwrite the winners an earlier
// search's all-gather, delayed by a slow peer, has not sent yet.  The recv buffer
// is written and read on the side stream only, in order.
//
// Failure: the wait for a search (or batch) is bounded.  Its clock starts when
// every local device has reached the exchange, i.e. when only the all-gather
// (which waits for the peers) and the merge are left; RCCL's asynchronous error
// is polled meanwhile.  On expiry or error the group's communicators are
// aborted (ncclCommAbort) and the call returns IRIS_E_HIP; the group then
// refuses every further call except the destroys.  Forming the group is bounded
// too: RCCL's init blocks until every rank has arrived (even non-blocking
// communicators do, in RCCL 2.27.7), so it runs on a helper thread the caller
// waits for with the group's bound; a rank whose peers never arrive fails
// instead of hanging and abandons that thread's init.  An ncclGroupEnd that
// returns ncclInProgress (non-blocking communicators, should a caller's RCCL
// make them) is waited for, bounded, before anything is ordered after the
// all-gather.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>
#include <string.h>

#include <array>
#include <map>
#include <condition_variable>
#include <memory>
#include <mutex>
#include <chrono>
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

constexpr uint32_t kSendRing = 4;  // send slots per device (pipelined searches in flight per slot reuse)

struct iris_group {
    std::vector<iris_device *> devs;  // local devices (owned)
    std::vector<ncclComm_t> comms;    // comms[i]: local device i, RCCL rank rank0 + i
    uint32_t ranks = 0, rank0 = 0;
    // what RCCL itself reports: ncclCommCount of the communicators, and every rank's PCI bus id
    // (gathered over the group's own all-gather when it formed)
    uint32_t comm_count = 0;
    std::vector<std::string> bus_ids;
    std::mutex mu;                    // serialises group calls
    std::atomic<int> refs{1};         // the group handle + each database and pending search
    uint32_t timeout_ms = 0;          // exchange wait bound (0: auto, group_timeout)
    // set when the communicators were aborted: every later call fails with broken_msg
    std::atomic<bool> broken{false};
    std::string broken_msg;
    // test hook IRIS_GROUP_STALL: coherent host word the stalled all-gathers wait on
    uint32_t *release = nullptr;
};

struct iris_group_db {
    iris_group *g = nullptr;
    int kind = 0, layout = 0;
    uint64_t total = 0;
    uint32_t spd = 1, S = 0, first_shard = 0;
    std::vector<iris_db *> shards;          // local shard i lives on local device i / spd
    std::vector<uint64_t> first, count;     // global index of record 0, records
    std::vector<DevBuf> send, recv;         // per local device: [kSendRing][spd] / [S] Partials (single query)
    // per local device and send slot: recorded on the side stream after the all-gather that read it
    std::vector<std::array<hipEvent_t, kSendRing>> sent;
    uint64_t searches = 0;                  // ring cursor: search k uses send slot k % kSendRing
    uint64_t max_count = 0;                 // largest local shard (the wait bound's estimate)
};

struct iris_group_pending {
    iris_group *g = nullptr;
    std::vector<Partial *> slots;  // pinned merge result of each local device
    std::vector<hipEvent_t> evs;   // recorded after each device's merge
    std::vector<hipEvent_t> reached;  // recorded on each side stream just before the exchange
    uint32_t timeout_ms = 0;
};

namespace {

void group_teardown(iris_group *g) {
    bool live = false;
    for (size_t i = 0; i < g->comms.size(); ++i) {
        if (!g->comms[i]) continue;
        live = true;
        (void)hipSetDevice(g->devs[i]->ordinal);
        (void)hipStreamSynchronize(g->devs[i]->stream);
        side_sync(g->devs[i]);
    }
    // One thread owns all local communicators: finalize them inside one RCCL group (each flushes
    // its outstanding work without waiting for the others), then destroy them.  Aborted
    // communicators (a broken group) are already gone.
    if (live) {
        ncclResult_t r = ncclGroupStart();
        for (size_t i = 0; r == ncclSuccess && i < g->comms.size(); ++i)
            if (g->comms[i]) r = ncclCommFinalize(g->comms[i]);
        const ncclResult_t r2 = ncclGroupEnd();
        for (size_t i = 0; i < g->comms.size(); ++i) {
            if (!g->comms[i]) continue;
            if (r == ncclSuccess && r2 == ncclSuccess)
                (void)ncclCommDestroy(g->comms[i]);
            else
                (void)ncclCommAbort(g->comms[i]);  // finalize failed: release without flushing
        }
    }
    for (iris_device *d : g->devs) iris_device_close(d);
    if (g->release) (void)hipHostFree(g->release);
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

int usable(const iris_group *g) {
    if (g->broken.load(std::memory_order_acquire))
        return fail(IRIS_E_HIP, "the device group was aborted (" + g->broken_msg + "); destroy it and form a new one");
    return 0;
}

int search_args(iris_group_db *gdb) {
    ARG(gdb, "NULL argument");
    ARG(gdb->kind == IRIS_KIND_TEMPLATES, "group search needs a template database");
    return usable(gdb->g);
}

// ---- test hooks (IRIS_TEST_HOOKS=1, iris_internal.hpp Hooks): a one-thread kernel on the side stream
// before the all-gather that spins on the wall clock for `ticks` (IRIS_GROUP_DELAY_US: a slow peer), or
// until the host sets *release, at most `ticks` (IRIS_GROUP_STALL: a peer that never arrives; the
// grid always drains within the cap)

constexpr uint64_t kStallCapUs = 60ull * 1000 * 1000;

__global__ void hook_spin_kernel(uint64_t ticks, const uint32_t *release) {
    const uint64_t t0 = wall_clock64();
    while (wall_clock64() - t0 < ticks) {
        if (release && __hip_atomic_load(release, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != 0) return;
        __builtin_amdgcn_s_sleep(8);
    }
}

int enqueue_hooks(iris_group *g, iris_device *d, hipStream_t stream) {
    const Hooks &h = d->hooks;
    if (!h.group_delay_us && !h.group_stall) return 0;
    int khz = 0;
    HIPCHK(hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, d->ordinal));
    if (h.group_delay_us)
        hipLaunchKernelGGL(hook_spin_kernel, dim3(1), dim3(1), 0, stream, (uint64_t)h.group_delay_us * khz / 1000,
                           (const uint32_t *)nullptr);
    if (h.group_stall) {
        if (!g->release) {
            void *p = nullptr;
            HIPCHK(hipHostMalloc(&p, 64, hipHostMallocCoherent | hipHostMallocMapped));
            g->release = (uint32_t *)p;
            __atomic_store_n(g->release, 0u, __ATOMIC_RELEASE);
        }
        hipLaunchKernelGGL(hook_spin_kernel, dim3(1), dim3(1), 0, stream, kStallCapUs * khz / 1000,
                           (const uint32_t *)g->release);
    }
    HIPCHK(hipGetLastError());
    return 0;
}

bool stall_hooked(const iris_group *g) {
    for (const iris_device *d : g->devs)
        if (d->hooks.group_stall) return true;
    return false;
}

// ---- bounded waits and abort

// The exchange wait bound: IRIS_GROUP_TIMEOUT_MS / iris_group_set_timeout, else 10 x the local
// work the call enqueued (at 5e10 comparisons/s, a fifth of one GPU's single-query rate), at least
// 30 s -- generous: it only has to turn a lost peer from a hang into an error.
uint32_t group_timeout(const iris_group *g, uint64_t records, uint32_t nq) {
    if (g->timeout_ms) return g->timeout_ms;
    if (g->devs[0]->hooks.group_timeout_ms) return g->devs[0]->hooks.group_timeout_ms;
    const double est_ms = (double)records * nq * kRot / 5e10 * 1e3;
    return (uint32_t)std::min(24.0 * 3600 * 1000, std::max(30000.0, 10 * est_ms));
}

// True when every device stream and side stream of the group has drained within `ms`.
bool drain(iris_group *g, uint32_t ms) {
    const auto t0 = std::chrono::steady_clock::now();
    for (;;) {
        bool idle = true;
        for (iris_device *d : g->devs) {
            (void)hipSetDevice(d->ordinal);
            if (hipStreamQuery(d->stream) == hipErrorNotReady) idle = false;
            if (d->aux && hipStreamQuery(d->aux) == hipErrorNotReady) idle = false;
        }
        if (idle) return true;
        if (std::chrono::steady_clock::now() - t0 > std::chrono::milliseconds(ms)) return false;
        std::this_thread::sleep_for(std::chrono::microseconds(200));
    }
}

// Aborts the group's communicators (an all-gather stuck on a lost peer polls RCCL's abort flag and
// ends) and marks the group broken.  Returns whether the streams drained (only then may the
// caller recycle what the aborted work wrote into).  Caller holds g->mu.
bool group_abort(iris_group *g, const std::string &why) {
    if (!g->broken.load(std::memory_order_acquire)) {
        g->broken_msg = why;
        g->broken.store(true, std::memory_order_release);
    }
    const bool stalled = stall_hooked(g);
    if (g->release) __atomic_store_n(g->release, 1u, __ATOMIC_RELEASE);
    // The stall hook stands in for a lost peer but holds its (1-rank) all-gather back rather than
    // inside RCCL: let it run out first, so no RCCL work is still queued when the communicator goes.
    bool drained = stalled ? drain(g, 10000) : true;
    for (size_t i = 0; i < g->comms.size(); ++i) {
        if (!g->comms[i]) continue;
        (void)hipSetDevice(g->devs[i]->ordinal);
        (void)ncclCommAbort(g->comms[i]);
        g->comms[i] = nullptr;
    }
    if (!stalled) drained = drain(g, 10000);
    return drained;
}

// Waits for every done[i] (one per local device), bounded as described at the top of the file.
// Returns 0, or fails after aborting the group; *drained tells whether the devices are idle.
// locked: the caller holds g->mu (else the abort takes it).
int group_wait(iris_group *g, const std::vector<hipEvent_t> &reached, const std::vector<hipEvent_t> &done,
               uint32_t timeout_ms, bool locked, bool *drained) {
    *drained = true;
    using clk = std::chrono::steady_clock;
    const auto t_start = clk::now();
    bool at_exchange = false;
    clk::time_point t_reached;
    std::string why;
    for (uint64_t it = 0;; ++it) {
        bool all = true;
        for (size_t i = 0; i < done.size() && why.empty(); ++i) {
            (void)hipSetDevice(g->devs[i]->ordinal);
            const hipError_t q = hipEventQuery(done[i]);
            if (q == hipErrorNotReady)
                all = false;
            else if (q != hipSuccess)
                why = std::string("hipEventQuery: ") + hipGetErrorString(q);
        }
        if (all && why.empty()) return 0;
        if (why.empty() && !at_exchange) {
            bool r = true;
            for (size_t i = 0; i < reached.size() && r; ++i) {
                (void)hipSetDevice(g->devs[i]->ordinal);
                r = hipEventQuery(reached[i]) == hipSuccess;
            }
            if (r) {
                at_exchange = true;
                t_reached = clk::now();
            }
        }
        if (why.empty() && (it & 255) == 255) {
            // the communicators are polled under g->mu: another thread's abort (holding it) frees
            // them; a caller without the lock skips the poll while someone else holds it
            std::unique_lock<std::mutex> gl(g->mu, std::defer_lock);
            if (locked || gl.try_lock()) {
                if (g->broken.load(std::memory_order_acquire)) why = "the device group was aborted (" + g->broken_msg + ")";
                for (size_t i = 0; i < g->comms.size() && why.empty(); ++i) {
                    ncclResult_t ae = ncclSuccess;
                    if (g->comms[i] && ncclCommGetAsyncError(g->comms[i], &ae) == ncclSuccess && ae != ncclSuccess &&
                        ae != ncclInProgress)
                        why = std::string("RCCL asynchronous error: ") + ncclGetErrorString(ae);
                }
            }
            if (why.empty() && at_exchange && clk::now() - t_reached > std::chrono::milliseconds(timeout_ms))
                why = "the exchange did not complete within " + std::to_string(timeout_ms) +
                      " ms (a peer rank failed or is unreachable)";
        }
        if (!why.empty()) {
            std::unique_lock<std::mutex> gl(g->mu, std::defer_lock);
            if (!locked) gl.lock();
            *drained = group_abort(g, why);
            return fail(IRIS_E_HIP, "device group aborted: " + why +
                                        (*drained ? std::string() : std::string(" (device work still outstanding)")));
        }
        if (clk::now() - t_start < std::chrono::milliseconds(2))
            __builtin_ia32_pause();
        else
            std::this_thread::sleep_for(std::chrono::microseconds(20));
    }
}

// Waits until every communicator of g is ready -- a non-blocking init, or the launch of a group
// whose ncclGroupEnd returned ncclInProgress -- at most `ms`; fails with the first asynchronous
// error or on expiry (the caller aborts).
int comms_ready(iris_group *g, uint32_t ms, const std::string &what) {
    using clk = std::chrono::steady_clock;
    const auto t0 = clk::now();
    for (;;) {
        bool all = true;
        for (size_t i = 0; i < g->comms.size(); ++i) {
            if (!g->comms[i]) continue;
            ncclResult_t st = ncclSuccess;
            const ncclResult_t r = ncclCommGetAsyncError(g->comms[i], &st);
            if (r != ncclSuccess) return fail(IRIS_E_HIP, what + ": ncclCommGetAsyncError: " + ncclGetErrorString(r));
            if (st == ncclInProgress)
                all = false;
            else if (st != ncclSuccess)
                return fail(IRIS_E_HIP, what + ": " + ncclGetErrorString(st) + " (" + ncclGetLastError(g->comms[i]) + ")");
        }
        if (all) return 0;
        const auto dt = clk::now() - t0;
        if (dt > std::chrono::milliseconds(ms))
            return fail(IRIS_E_HIP, what + " did not complete within " + std::to_string(ms) +
                                        " ms (a peer rank failed, never started, or is unreachable)");
        if (dt < std::chrono::milliseconds(2))
            __builtin_ia32_pause();
        else
            std::this_thread::sleep_for(std::chrono::microseconds(100));
    }
}

// The bound of forming a group: IRIS_GROUP_TIMEOUT_MS / iris_group_set_timeout's knob, else 120 s
// (eight ranks' bootstrap and topology discovery take seconds).
uint32_t init_timeout(const iris_group *g) {
    const uint32_t h = g->devs.empty() ? 0 : g->devs[0]->hooks.group_timeout_ms;
    return h ? h : kGroupInitTimeoutMs;
}

// Abandoned inits per device ordinal, process-wide: `pending` are still blocked inside RCCL (each
// holds a helper thread, its bootstrap sockets and a partial communicator until its peers come, if
// ever), `total` counts every one since the process started (iris_config "abandoned_inits").
struct Abandoned {
    std::mutex mu;
    std::map<int, std::pair<uint64_t, uint64_t>> by_ordinal;  // ordinal -> (pending, total)
};
Abandoned &abandoned() {
    static Abandoned *a = new Abandoned();  // never destroyed: abandoned helper threads may outlive main
    return *a;
}

// A communicator init that may never finish (a peer that never starts): RCCL 2.27.7 blocks inside
// ncclCommInitRankConfig / ncclGroupEnd even with config.blocking = 0
// (profiles/r05_rccl_nonblocking_init.txt), so the init runs on a helper thread of its own and the
// caller waits for it with a bound.  On expiry the caller leaves; the job is abandoned and owns
// everything it uses -- should its init ever complete, it aborts the communicators itself.
struct InitJob {
    std::mutex mu;
    std::condition_variable cv;
    bool done = false, abandoned = false;
    ncclResult_t r = ncclSuccess;
    std::string err;
    std::vector<int> ordinals;
    std::vector<ncclComm_t> comms;
    ncclUniqueId u;
    int nranks = 0, rank0 = 0;
};

void init_job_run(std::shared_ptr<InitJob> job) {
    ncclResult_t r = ncclGroupStart();
    for (size_t i = 0; r == ncclSuccess && i < job->ordinals.size(); ++i) {
        if (hipSetDevice(job->ordinals[i]) != hipSuccess) {
            r = ncclInvalidArgument;
            break;
        }
        r = ncclCommInitRank(&job->comms[i], job->nranks, job->u, job->rank0 + (int)i);
    }
    const ncclResult_t r2 = ncclGroupEnd();
    if (r == ncclSuccess) r = r2;
    std::lock_guard<std::mutex> l(job->mu);
    job->r = r;
    if (r != ncclSuccess) job->err = ncclGetErrorString(r);
    job->done = true;
    if (job->abandoned) {  // nobody waits any more: release what was created
        for (size_t i = 0; i < job->comms.size(); ++i)
            if (job->comms[i]) {
                (void)hipSetDevice(job->ordinals[i]);
                (void)ncclCommAbort(job->comms[i]);
            }
        std::lock_guard<std::mutex> a(abandoned().mu);
        for (int o : job->ordinals) abandoned().by_ordinal[o].first -= 1;
        return;
    }
    job->cv.notify_all();
}

// Creates the communicators of the local devices as RCCL ranks rank0 + i of nranks (one RCCL
// group, ncclCommInitAll's form for several local devices) and waits at most the group's bound.
int comm_init(iris_group *g, const ncclUniqueId &u) {
    const size_t L = g->devs.size();
    g->comms.assign(L, nullptr);
    if (g->ranks > 1) {  // a multi-rank init beside a pending abandoned one would pile another on top
        std::lock_guard<std::mutex> a(abandoned().mu);
        for (iris_device *d : g->devs) {
            auto it = abandoned().by_ordinal.find(d->ordinal);
            if (it != abandoned().by_ordinal.end() && it->second.first > 0)
                return fail(IRIS_E_HIP, "an abandoned RCCL communicator init on device " + std::to_string(d->ordinal) +
                                            " is still pending (a peer rank never arrived): this process forms no "
                                            "further multi-rank group on it -- start a fresh process (1-rank groups "
                                            "still form)");
        }
    }
    auto job = std::make_shared<InitJob>();
    for (iris_device *d : g->devs) job->ordinals.push_back(d->ordinal);
    job->comms.assign(L, nullptr);
    job->u = u;
    job->nranks = (int)g->ranks;
    job->rank0 = (int)g->rank0;
    try {
        std::thread(init_job_run, job).detach();
    } catch (...) {
        return fail(IRIS_E_NOMEM, "cannot start the RCCL init thread");
    }
    const uint32_t ms = init_timeout(g);
    std::unique_lock<std::mutex> l(job->mu);
    if (!job->cv.wait_for(l, std::chrono::milliseconds(ms), [&] { return job->done; })) {
        job->abandoned = true;
        {
            std::lock_guard<std::mutex> a(abandoned().mu);
            for (int o : job->ordinals) {
                abandoned().by_ordinal[o].first += 1;
                abandoned().by_ordinal[o].second += 1;
            }
        }
        return fail(IRIS_E_HIP, "RCCL communicator init (" + std::to_string(g->ranks) + " ranks) did not complete within " +
                                    std::to_string(ms) + " ms (a peer rank failed, never started, or is unreachable); "
                                    "the pending init is abandoned");
    }
    if (job->r != ncclSuccess) {
        for (size_t i = 0; i < L; ++i)
            if (job->comms[i]) {
                (void)hipSetDevice(job->ordinals[i]);
                (void)ncclCommAbort(job->comms[i]);
            }
        return fail(IRIS_E_HIP, "ncclCommInitRank: " + job->err);
    }
    g->comms = job->comms;
    return 0;
}

// ncclGroupEnd of an exchange: ncclInProgress (non-blocking communicators) waits, bounded, for the
// group's launch, so that work enqueued after it on the streams follows the all-gather.
ncclResult_t group_end_launched(iris_group *g, uint32_t ms, int *rc) {
    const ncclResult_t r = ncclGroupEnd();
    if (r == ncclInProgress) {
        *rc = comms_ready(g, ms, "RCCL all-gather launch");
        return *rc == 0 ? ncclSuccess : ncclInternalError;
    }
    return r;
}

// What RCCL's ranks are: ncclCommCount of the new communicators, and every rank's device PCI bus
// id over the group's own all-gather (bounded like a search's exchange).
int gather_bus_ids(iris_group *g) {
    const size_t L = g->devs.size();
    constexpr size_t B = IRIS_GROUP_BUS_ID_BYTES;
    for (size_t i = 0; i < L; ++i) {
        int count = 0;
        NCCLCHK(ncclCommCount(g->comms[i], &count));
        if (i == 0) g->comm_count = (uint32_t)count;
        if ((uint32_t)count != g->comm_count || g->comm_count != g->ranks)
            return fail(IRIS_E_HIP, "RCCL communicator holds " + std::to_string(count) + " ranks, the group " +
                                        std::to_string(g->ranks));
    }
    struct Bufs {
        std::vector<void *> p;
        ~Bufs() {
            for (void *q : p)
                if (q) (void)hipFree(q);
        }
    } bufs;
    std::vector<void *> send(L, nullptr), recv(L, nullptr);
    std::vector<hipEvent_t> reached(L, nullptr), done(L, nullptr);
    auto give_events = [&] {
        for (size_t i = 0; i < L; ++i) {
            if (reached[i]) g->devs[i]->event_pool.push_back(reached[i]);
            if (done[i]) g->devs[i]->event_pool.push_back(done[i]);
        }
    };
    int rc = 0;
    for (size_t i = 0; i < L && rc == 0; ++i) {
        iris_device *d = g->devs[i];
        rc = set_device(d);
        char bus[B] = {0};
        if (rc == 0 && hipDeviceGetPCIBusId(bus, (int)B - 1, d->ordinal) != hipSuccess) rc = fail(IRIS_E_HIP, "hipDeviceGetPCIBusId");
        if (rc == 0 && (hipMalloc(&send[i], B) != hipSuccess || hipMalloc(&recv[i], B * g->ranks) != hipSuccess))
            rc = fail(IRIS_E_NOMEM, "hipMalloc bus id buffers");
        bufs.p.push_back(send[i]);
        bufs.p.push_back(recv[i]);
        if (rc == 0 && hipMemcpyAsync(send[i], bus, B, hipMemcpyHostToDevice, d->aux) != hipSuccess) rc = fail(IRIS_E_HIP, "hipMemcpyAsync");
        if (rc == 0 && hipStreamSynchronize(d->aux) != hipSuccess) rc = fail(IRIS_E_HIP, "hipStreamSynchronize");
        if (rc == 0 && !((reached[i] = take_event(d)) && (done[i] = take_event(d)))) rc = fail(IRIS_E_HIP, "hipEventCreate failed");
        if (rc == 0 && hipEventRecord(reached[i], d->aux) != hipSuccess) rc = fail(IRIS_E_HIP, "hipEventRecord");
    }
    if (rc != 0) {
        give_events();
        return rc;
    }
    ncclResult_t r = ncclGroupStart();
    for (size_t i = 0; r == ncclSuccess && i < L; ++i) {
        r = ncclAllGather(send[i], recv[i], B, ncclUint8, g->comms[i], g->devs[i]->aux);
        if (r == ncclInProgress) r = ncclSuccess;
    }
    const ncclResult_t r2 = group_end_launched(g, init_timeout(g), &rc);
    if (rc == 0 && r == ncclSuccess) r = r2;
    if (rc == 0 && r != ncclSuccess) rc = fail(IRIS_E_HIP, std::string("ncclAllGather (bus ids): ") + ncclGetErrorString(r));
    for (size_t i = 0; i < L && rc == 0; ++i) {
        (void)hipSetDevice(g->devs[i]->ordinal);
        if (hipEventRecord(done[i], g->devs[i]->aux) != hipSuccess) rc = fail(IRIS_E_HIP, "hipEventRecord");
    }
    bool drained = true;
    if (rc != 0) {
        const std::string m = g_err;
        drained = group_abort(g, "bus id exchange: " + m);
        rc = fail(rc, m);
    } else {
        rc = group_wait(g, reached, done, init_timeout(g), false, &drained);
    }
    if (rc == 0) {
        std::vector<char> all(B * g->ranks);
        (void)hipSetDevice(g->devs[0]->ordinal);
        if (hipMemcpy(all.data(), recv[0], all.size(), hipMemcpyDeviceToHost) != hipSuccess) rc = fail(IRIS_E_HIP, "hipMemcpy bus ids");
        for (uint32_t k = 0; rc == 0 && k < g->ranks; ++k) g->bus_ids.emplace_back(all.data() + k * B, strnlen(all.data() + k * B, B));
    }
    if (!drained) bufs.p.clear();  // aborted work may still write them: leaked rather than freed
    else give_events();
    return rc;
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
        side_sync(d);
        if (gdb->send[i].p) (void)hipFree(gdb->send[i].p);
        if (gdb->recv[i].p) (void)hipFree(gdb->recv[i].p);
        if (i < gdb->sent.size())
            for (hipEvent_t &e : gdb->sent[i])
                if (e) (void)hipEventDestroy(e);
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
    if (rc == 0) {  // ncclCommInitAll's form: one id, every local device a rank, in one RCCL group
        ncclUniqueId u;
        const ncclResult_t r = ncclGetUniqueId(&u);
        rc = r == ncclSuccess ? comm_init(g, u) : fail(IRIS_E_HIP, std::string("ncclGetUniqueId: ") + ncclGetErrorString(r));
    }
    if (rc == 0) rc = gather_bus_ids(g);
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
        rc = comm_init(g, u);
    }
    if (rc == 0) rc = gather_bus_ids(g);
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

int iris_group_rccl_info(const iris_group_t *g, uint32_t *comm_ranks, char *bus_ids, size_t len) {
    ARG(g, "NULL argument");
    if (comm_ranks) *comm_ranks = g->comm_count;
    if (bus_ids) {
        ARG(len >= (size_t)g->ranks * IRIS_GROUP_BUS_ID_BYTES, "bus_ids needs ranks * IRIS_GROUP_BUS_ID_BYTES bytes");
        memset(bus_ids, 0, (size_t)g->ranks * IRIS_GROUP_BUS_ID_BYTES);
        for (size_t r = 0; r < g->bus_ids.size() && r < g->ranks; ++r)
            memcpy(bus_ids + r * IRIS_GROUP_BUS_ID_BYTES, g->bus_ids[r].c_str(),
                   std::min(g->bus_ids[r].size(), (size_t)IRIS_GROUP_BUS_ID_BYTES - 1));
    }
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

int iris_group_set_timeout(iris_group_t *g, uint32_t ms) {
    ARG(g, "NULL argument");
    std::lock_guard<std::mutex> gl(g->mu);
    g->timeout_ms = ms;
    return 0;
}

int iris_group_db_create(iris_group_t *g, int kind, uint64_t total, int layout, uint32_t spd, iris_group_db_t **out) {
    IRIS_KEEP_DEVICE();
    ARG(g && out, "NULL argument");
    ARG(spd >= 1, "shards_per_device must be at least 1");
    CHK(check_kind(kind));
    CHK(usable(g));
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
        gdb->max_count = std::max(gdb->max_count, c);
    }
    gdb->send.resize(L);
    gdb->recv.resize(L);
    gdb->sent.resize(L);
    for (auto &ev : gdb->sent) ev.fill(nullptr);
    for (uint32_t i = 0; i < L && rc == 0; ++i) {
        iris_device *d = g->devs[i];
        std::lock_guard<std::recursive_mutex> l(d->mu);
        rc = set_device(d);
        if (rc == 0) rc = ensure(d, gdb->send[i], (size_t)kSendRing * spd * sizeof(Partial));
        if (rc == 0) rc = ensure(d, gdb->recv[i], (size_t)gdb->S * sizeof(Partial));
        for (uint32_t b = 0; rc == 0 && b < kSendRing; ++b)
            if (hipEventCreateWithFlags(&gdb->sent[i][b], hipEventDisableTiming) != hipSuccess) {
                gdb->sent[i][b] = nullptr;
                rc = fail(IRIS_E_HIP, "hipEventCreate failed");
            }
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
    CHK(usable(gdb->g));
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
    CHK(usable(gdb->g));
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
    CHK(usable(gdb->g));
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
    CHK(usable(gdb->g));
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
    CHK(usable(g));
    DeviceLocks locks(g);
    const size_t L = g->devs.size();
    const bool remote = g->ranks > L;  // peers in other processes take part in the exchange
    iris_group_pending *p = new (std::nothrow) iris_group_pending();
    if (!p) return fail(IRIS_E_NOMEM, "out of host memory");
    p->g = g;
    p->slots.assign(L, nullptr);
    p->evs.assign(L, nullptr);
    p->reached.assign(L, nullptr);
    p->timeout_ms = group_timeout(g, gdb->max_count, 1);
    auto abandon = [&](int rc, bool gather_started) {
        const std::string m = g_err;
        // The peers are (or will be) inside this search's all-gather, and this process's
        // communicators are out of step with theirs: abort rather than let every rank hang.  The
        // abort comes first: an earlier search's all-gather still queued on a side stream may be
        // waiting for a lost peer, and only the abort ends it (group_abort drains with a bound).
        bool drained = true;
        if (remote || gather_started) {
            drained = group_abort(g, "a rank failed to enqueue its search: " + m);
        } else {
            for (iris_device *d : g->devs) {
                (void)hipSetDevice(d->ordinal);
                (void)hipStreamSynchronize(d->stream);
                side_sync(d);
            }
        }
        if (drained)  // otherwise aborted work may still write them: leaked rather than reused
            for (size_t i = 0; i < L; ++i) {
                iris_device *d = g->devs[i];
                if (p->slots[i]) d->free_slots.push_back(p->slots[i]);
                if (p->evs[i]) d->event_pool.push_back(p->evs[i]);
                if (p->reached[i]) d->event_pool.push_back(p->reached[i]);
            }
        delete p;
        return fail(rc, m);
    };
    const uint32_t b = (uint32_t)(gdb->searches++ % kSendRing);
    // per device: the query's engine, then every local shard's search + reduce into send slot b
    for (size_t i = 0; i < L; ++i) {
        iris_device *d = g->devs[i];
        int rc = set_device(d);
        iris_engine *e = nullptr;
        if (rc == 0) rc = take_result_slot(d, &p->slots[i]);
        if (rc == 0 && !(p->evs[i] = take_event(d))) rc = fail(IRIS_E_HIP, "hipEventCreate failed");
        if (rc == 0 && !(p->reached[i] = take_event(d))) rc = fail(IRIS_E_HIP, "hipEventCreate failed");
        if (rc == 0) rc = template_engine_locked(d, query, &e);
        Partial *send = (Partial *)gdb->send[i].p + (size_t)b * gdb->spd;
        // a fused shard search writes its winner from the kernel, on the device stream: the
        // all-gather that last read slot b (search k - kSendRing, side stream) precedes it
        if (rc == 0 && !d->hooks.group_unordered && hipStreamWaitEvent(d->stream, gdb->sent[i][b], 0) != hipSuccess)
            rc = fail(IRIS_E_HIP, "hipStreamWaitEvent");
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
        if (rc == 0 && hipEventRecord(p->reached[i], d->aux) != hipSuccess) rc = fail(IRIS_E_HIP, "hipEventRecord");
        if (rc == 0) rc = enqueue_hooks(g, d, d->aux);
        if (rc != 0) return abandon(rc, false);
    }
    // the exchange: every device's shard winners to every device (side streams, in order after the reduces)
    {
        ncclResult_t r = ncclGroupStart();
        for (size_t i = 0; r == ncclSuccess && i < L; ++i) {
            r = ncclAllGather((Partial *)gdb->send[i].p + (size_t)b * gdb->spd, gdb->recv[i].p,
                              (size_t)gdb->spd * sizeof(Partial), ncclUint8, g->comms[i], g->devs[i]->aux);
            if (r == ncclInProgress) r = ncclSuccess;
        }
        int lrc = 0;
        const ncclResult_t r2 = group_end_launched(g, p->timeout_ms, &lrc);
        if (lrc != 0) return abandon(lrc, true);
        if (r == ncclSuccess) r = r2;
        if (r != ncclSuccess) return abandon(fail(IRIS_E_HIP, std::string("ncclAllGather: ") + ncclGetErrorString(r)), true);
    }
    for (size_t i = 0; i < L; ++i) {
        iris_device *d = g->devs[i];
        int rc = set_device(d);
        if (rc == 0 && hipEventRecord(gdb->sent[i][b], d->aux) != hipSuccess) rc = fail(IRIS_E_HIP, "hipEventRecord");
        if (rc == 0)
            rc = timed(d, "group_merge", gdb->S, [&] {
                return launch_group_merge(d->aux, (const Partial *)gdb->recv[i].p, gdb->S, 1, 1, p->slots[i]);
            }, d->aux);
        if (rc == 0 && hipEventRecord(p->evs[i], d->aux) != hipSuccess) rc = fail(IRIS_E_HIP, "hipEventRecord");
        if (rc != 0) return abandon(rc, true);
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
    bool drained = true;
    const int rc = group_wait(g, p->reached, p->evs, p->timeout_ms, false, &drained);
    const std::string m = rc ? g_err : std::string();
    if (rc == 0)
        for (size_t i = 0; i < L; ++i) memcpy(&res[i], p->slots[i], sizeof(Partial));
    if (drained)  // otherwise aborted work may still write them: leaked rather than reused
        for (size_t i = 0; i < L; ++i) {
            iris_device *d = g->devs[i];
            std::lock_guard<std::recursive_mutex> l(d->mu);
            d->free_slots.push_back(p->slots[i]);
            d->event_pool.push_back(p->evs[i]);
            d->event_pool.push_back(p->reached[i]);
            fold_done(d);
        }
    delete p;
    group_release(g);
    if (rc != 0) return fail(rc, m);
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
    CHK(usable(g));
    DeviceLocks locks(g);
    const size_t L = g->devs.size();
    const bool remote = g->ranks > L;
    std::vector<hipEvent_t> reached(L, nullptr), done(L, nullptr);
    bool gather_started = false;
    const uint32_t spd = gdb->spd, S = gdb->S;
    const uint32_t stride = nq <= kBatchStreamMax ? nq : (nq + batch_query_group() - 1) / batch_query_group() * batch_query_group();
    std::vector<DevBuf> send(L), recv(L);
    std::vector<iris_engine *> eng(L, nullptr);
    bool drained = true;
    auto cleanup = [&] {
        if (!drained) return;  // aborted work may still use them: leaked rather than freed
        for (size_t i = 0; i < L; ++i) {
            iris_device *d = g->devs[i];
            (void)hipSetDevice(d->ordinal);
            (void)hipStreamSynchronize(d->stream);
            if (eng[i]) iris_engine_destroy(eng[i]);
            if (send[i].p) (void)hipFree(send[i].p);
            if (recv[i].p) (void)hipFree(recv[i].p);
            if (reached[i]) d->event_pool.push_back(reached[i]);
            if (done[i]) d->event_pool.push_back(done[i]);
        }
    };
    int rc = 0;
    for (size_t i = 0; i < L && rc == 0; ++i) {
        iris_device *d = g->devs[i];
        rc = set_device(d);
        if (rc == 0) rc = ensure(d, send[i], (size_t)spd * stride * sizeof(Partial));
        if (rc == 0) rc = ensure(d, recv[i], (size_t)S * stride * sizeof(Partial));
        if (rc == 0) rc = ensure_host_result(d, (size_t)stride * sizeof(Partial));
        if (rc == 0 && !(reached[i] = take_event(d))) rc = fail(IRIS_E_HIP, "hipEventCreate failed");
        if (rc == 0 && !(done[i] = take_event(d))) rc = fail(IRIS_E_HIP, "hipEventCreate failed");
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
                const BatchGeometry geo = batch_geometry(d->hooks, LaunchRange{0, gdb->count[s]}, nq);
                pmax = std::max(pmax, (size_t)geo.nqg * geo.qper * geo.G * sizeof(Partial));
            }
            rc = ensure(d, d->partials, pmax);
            for (uint32_t j = 0; rc == 0 && j < spd; ++j) {
                const size_t s = i * spd + j;
                if (gdb->count[s] == 0) continue;
                const LaunchRange r{0, gdb->count[s]};
                const BatchGeometry geo = batch_geometry(d->hooks, r, nq);
                rc = timed(d, "template_batch", r.n * nq, [&] {
                    return launch_batch(d->hooks, d->stream, gdb->shards[s]->data, e->qfrag, r, geo, (Partial *)d->partials.p,
                                        sbuf + (size_t)j * stride, gdb->first[s]);
                });
            }
        }
        if (rc == 0 && hipEventRecord(reached[i], d->stream) != hipSuccess) rc = fail(IRIS_E_HIP, "hipEventRecord");
        if (rc == 0) rc = enqueue_hooks(g, d, d->stream);
    }
    if (rc == 0) {
        gather_started = true;
        ncclResult_t r = ncclGroupStart();
        for (size_t i = 0; r == ncclSuccess && i < L; ++i) {
            r = ncclAllGather(send[i].p, recv[i].p, (size_t)spd * stride * sizeof(Partial), ncclUint8, g->comms[i],
                              g->devs[i]->stream);
            if (r == ncclInProgress) r = ncclSuccess;
        }
        const ncclResult_t r2 = group_end_launched(g, group_timeout(g, gdb->max_count, nq), &rc);
        if (r == ncclSuccess) r = r2;
        if (rc == 0 && r != ncclSuccess) rc = fail(IRIS_E_HIP, std::string("ncclAllGather: ") + ncclGetErrorString(r));
    }
    for (size_t i = 0; i < L && rc == 0; ++i) {
        iris_device *d = g->devs[i];
        rc = set_device(d);
        if (rc == 0)
            rc = timed(d, "group_merge", (uint64_t)S * nq, [&] {
                return launch_group_merge(d->stream, (const Partial *)recv[i].p, S, nq, stride, (Partial *)d->host_result);
            });
        if (rc == 0 && hipEventRecord(done[i], d->stream) != hipSuccess) rc = fail(IRIS_E_HIP, "hipEventRecord");
    }
    if (rc != 0 && (remote || gather_started)) {  // the peers are inside (or headed for) this exchange
        const std::string m = g_err;
        drained = group_abort(g, "a rank failed to enqueue its batch search: " + m);
        rc = fail(rc, m);
    }
    if (rc == 0) rc = group_wait(g, reached, done, group_timeout(g, gdb->max_count, nq), true, &drained);
    std::vector<Partial> res((size_t)L * stride);
    for (size_t i = 0; i < L && rc == 0; ++i) {
        iris_device *d = g->devs[i];
        rc = set_device(d);
        if (rc == 0) fold_done(d);
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

void iris_api::abandoned_inits(int ordinal, uint64_t *pending, uint64_t *total) {
    std::lock_guard<std::mutex> a(abandoned().mu);
    auto it = abandoned().by_ordinal.find(ordinal);
    *pending = it == abandoned().by_ordinal.end() ? 0 : it->second.first;
    *total = it == abandoned().by_ordinal.end() ? 0 : it->second.second;
}
