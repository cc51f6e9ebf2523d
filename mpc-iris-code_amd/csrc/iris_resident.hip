// iris_resident.hip — record files kept resident for the reference's unchanged call sites.
//
// The participant and the resolver mmap their record file once (src/main.rs:386-391, 455-460)
// and call batch_process(out, chunk) on 20 000-record slices of that mapping for every request
// (src/main.rs:426-431, 511-516).  Through iris_engine_batch_process_host each such call would
// move its slice over PCIe, which cannot beat a CPU scan of the same bytes from DRAM
// (profiles/r04ae_bench_host-masks_chunk20k.jsonl: 0.72x the 16-thread CPU port).  Not moving
// the bytes is what helps: a slice that lies inside a read-only, shared, file-backed mapping of a
// regular file is served from a device copy of the whole mapping, made granule by granule (256 MB)
// the first time a call touches it, so the first walk costs what the upload path costs and every
// later walk reads HBM only.  Granules are read from the file (pread by the helper threads into the
// pinned upload slots), not through the caller's mapping: a file that shrinks or fails to read
// under the fill is a short read -- the copy is dropped and the call uploads its own slice, as it
// would without this path -- rather than a SIGBUS on a page past the new end of the file.
//
// Staleness: the copy stands for (st_dev, st_ino, st_size, st_mtim, st_ctim) of the mapped file,
// re-checked on every call with one stat of /proc/self/map_files/<lo>-<hi> (the kernel's link to
// the file behind exactly that mapping: a mapping that went away or was replaced fails or shows
// another inode; ~2.5 us), plus a probe of three records of the slice against 64-byte snapshots
// taken when their granule was uploaded (a write the timestamps miss: their granularity is the
// kernel's tick).  A changed file drops its copy; the call then starts over.  Where map_files
// cannot be read (it needs ptrace-read access to the process, which some sandboxes withhold) the
// copy holds the mapped file open (opened by the mapping's path and checked to be its inode) and
// fstats that instead,
// and re-reads the mapping's line of /proc/self/maps at least every 200 ms to notice a remap (a
// read of /proc/self/maps costs ~0.4 ms in a process with ~500 mappings; the slice probe covers a
// remap in between).
//
// Not made resident: anonymous or writable memory, private mappings, files larger than the
// device's free memory (less a reserve; older copies are evicted first, least recently used),
// IRIS_AUTO_RESIDENT=0.  Those slices keep the upload path.  A device allocation that fails
// (iris_db_create) drops every resident copy and retries.
#include <errno.h>
#include <fcntl.h>
#include <stdio.h>
#include <string.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <chrono>
#include <string>
#include <vector>

#include "iris_handles.hpp"

using namespace iris;
using namespace iris_api;

namespace {

constexpr size_t kGranuleBytes = 256ull << 20;  // residency unit of a copy
// a fill reads ahead up to this much in one pipelined write, under the device lock: 1 GB keeps a
// first walk's fill near the load path's rate while another thread's calls on the device wait at
// most ~25 ms for it (4 GB runs held them ~0.1 s)
constexpr size_t kFillRunBytes = 1ull << 30;
constexpr size_t kSnapBytes = 64;              // probe snapshot of every 64th record
constexpr uint64_t kSnapStride = 64;
constexpr size_t kNotResidentMax = 4096;       // remembered ineligible address ranges
constexpr int kNotResidentSeconds = 5;         // how long a refusal stands before the range is re-examined

}  // namespace

struct Resident {
    int kind = 0;
    uintptr_t lo = 0, hi = 0;  // the mapping (one VMA)
    uintptr_t base = 0;        // address of record 0 (the first whole record of the slices seen)
    uint64_t file_off = 0;     // its offset in the file
    uint64_t nrec = 0;
    std::string link;          // /proc/self/map_files/<lo>-<hi>
    int fd = -1;               // >= 0: map_files unreadable; the mapped file, held open
    uint64_t inode = 0;        // of the mapping (/proc/self/maps)
    uint64_t vma_off = 0;      // the mapping's file offset (/proc/self/maps)
    std::string path;
    std::chrono::steady_clock::time_point vma_checked;
    struct stat st {};
    iris_db *db = nullptr;
    size_t dev_bytes = 0;
    uint64_t gran = 0;              // records per granule
    std::vector<uint8_t> have;      // granule uploaded
    std::vector<uint8_t> snap;      // kSnapBytes of record i * kSnapStride
    uint64_t last_use = 0;
};

namespace {

bool same_time(const struct timespec &a, const struct timespec &b) {
    return a.tv_sec == b.tv_sec && a.tv_nsec == b.tv_nsec;
}

void free_copy(iris_device *d, Resident *r) {
    // a read-ahead kernel on the side stream may still read the copy
    (void)hipStreamSynchronize(d->stream);
    side_sync(d);
    if (r->db) {
        if (r->db->data) (void)hipFree(r->db->data);
        delete r->db;
    }
    if (r->fd >= 0) ::close(r->fd);
    delete r;
}

void drop(iris_device *d, Resident *r) {
    auto &v = d->resident;
    v.erase(std::remove(v.begin(), v.end(), r), v.end());
    free_copy(d, r);
}

void remember_not_resident(iris_device *d, uintptr_t lo, uintptr_t hi, const std::string &why) {
    if (d->not_resident.size() >= kNotResidentMax) d->not_resident.clear();
    d->not_resident.push_back({lo, hi, std::chrono::steady_clock::now() + std::chrono::seconds(kNotResidentSeconds)});
    d->resident_skip = why;
}

// The mapping of /proc/self/maps that holds address p.
struct Vma {
    uintptr_t lo = 0, hi = 0;
    char perms[8] = {0};
    uint64_t off = 0;
    uint64_t inode = 0;
    unsigned int maj = 0, mnr = 0;
    std::string path;
};

bool find_vma(uintptr_t p, Vma *out) {
    FILE *f = fopen("/proc/self/maps", "re");
    if (!f) return false;
    char line[4352];
    bool found = false;
    while (fgets(line, sizeof(line), f)) {
        unsigned long lo, hi, off, ino;
        unsigned int maj, mnr;
        char perms[8];
        int pos = 0;
        if (sscanf(line, "%lx-%lx %7s %lx %x:%x %lu %n", &lo, &hi, perms, &off, &maj, &mnr, &ino, &pos) < 7) continue;
        if (p < lo || p >= hi) continue;
        out->lo = lo;
        out->hi = hi;
        memcpy(out->perms, perms, sizeof(perms));
        out->off = off;
        out->inode = ino;
        out->maj = maj;
        out->mnr = mnr;
        std::string path = line + pos;
        while (!path.empty() && (path.back() == '\n' || path.back() == ' ')) path.pop_back();
        out->path = path;
        found = true;
        break;
    }
    fclose(f);
    return found;
}

// The mapped file's stat: through map_files, or (where that is unreadable) the held descriptor.
bool file_stat(const Resident *r, struct stat *st) {
    return r->fd >= 0 ? fstat(r->fd, st) == 0 : stat(r->link.c_str(), st) == 0;
}

// Whether the mapping is still the one the copy was made of: the same range, file, path, file
// offset and read-only.  map_files answers the file with every stat but not the offset (the same
// file mapped again at the same address from another offset), so both forms re-read
// /proc/self/maps when asked (now) and at least every 200 ms; the slice probe covers a remap in
// between.
bool vma_same(Resident *r, bool now) {
    const auto t = std::chrono::steady_clock::now();
    if (!now && t - r->vma_checked < std::chrono::milliseconds(200)) return true;
    Vma v;
    if (!find_vma(r->lo, &v) || v.lo != r->lo || v.hi != r->hi || v.inode != r->inode || v.path != r->path ||
        v.off != r->vma_off || v.perms[1] != '-')
        return false;
    r->vma_checked = t;
    return true;
}

// A new resident copy of the file mapping that holds the slice [p, p + n records), or nullptr
// (not eligible: remembered as such).  Errors are not reported: the caller uploads instead.
Resident *make_resident(iris_device *d, int kind, uintptr_t p, uint64_t n) {
    const KindInfo k = kind_info(kind, IRIS_LAYOUT_TILES);
    const size_t rb = k.rec_bytes;
    Vma v;
    if (!find_vma(p, &v)) {
        d->resident_skip = "no mapping holds the slice";
        return nullptr;
    }
    auto ineligible = [&](const std::string &why) -> Resident * {
        remember_not_resident(d, v.lo, v.hi, why);
        return nullptr;
    };
    // read-only (not writable), shared, backed by a named file
    if (v.perms[0] != 'r' || v.perms[1] != '-' || v.perms[3] != 's')
        return ineligible(std::string("mapping is not read-only shared (") + v.perms + ")");
    if (v.inode == 0 || v.path.empty() || v.path[0] != '/' || v.path.find(" (deleted)") != std::string::npos)
        return ineligible("mapping is not backed by a named file");
    char link[96];
    snprintf(link, sizeof(link), "/proc/self/map_files/%lx-%lx", (unsigned long)v.lo, (unsigned long)v.hi);
    struct stat st;
    int fd = -1;
    if (stat(link, &st) != 0) {
        // map_files unreadable here: the mapped file by its path, if it is the mapping's inode (the
        // device number is not compared: on overlay file systems /proc/self/maps shows the lower
        // layer's, which st_dev does not)
        const int err = errno;
        fd = ::open(v.path.c_str(), O_RDONLY | O_CLOEXEC);
        if (fd < 0 || fstat(fd, &st) != 0 || (uint64_t)st.st_ino != v.inode) {
            if (fd >= 0) ::close(fd);
            return ineligible(std::string("map_files: ") + strerror(err) + "; the path is not the mapped file");
        }
    }
    if (!S_ISREG(st.st_mode) || (uint64_t)st.st_ino != v.inode) {
        if (fd >= 0) ::close(fd);
        return ineligible("mapping is not a regular file");
    }
    if ((uint64_t)st.st_size <= v.off) {
        if (fd >= 0) ::close(fd);
        return ineligible("mapping lies past the end of its file");
    }
    const uintptr_t data_end = v.lo + std::min<uint64_t>(v.hi - v.lo, (uint64_t)st.st_size - v.off);
    const uintptr_t base = v.lo + (p - v.lo) % rb;
    auto refuse = [&](const std::string &why) -> Resident * {
        if (fd >= 0) ::close(fd);
        return ineligible(why);
    };
    if (data_end < base + rb) return refuse("mapping holds no whole record");
    const uint64_t nrec = (data_end - base) / rb;
    if ((p - base) / rb + n > nrec) {  // the slice runs past the file's records
        if (fd >= 0) ::close(fd);
        return nullptr;
    }
    const uint64_t blocks = (nrec + k.block - 1) / k.block;
    const size_t dev_bytes = (size_t)blocks * block_bytes(k);
    // copies of mappings that are gone (unmapped, or their file replaced) free their memory first
    for (size_t i = d->resident.size(); i-- > 0;) {
        Resident *o = d->resident[i];
        struct stat ost;
        if (!file_stat(o, &ost) || ost.st_ino != o->st.st_ino || ost.st_dev != o->st.st_dev || !vma_same(o, true))
            drop(d, o);
    }
    // room: the device's free memory less a reserve, after evicting older copies if need be, and at
    // most the cap of all copies together: IRIS_RESIDENT_MAX_MB, else half the device (a participant
    // and a resolver process sharing a GPU cannot take all of it from each other); the test hook
    // IRIS_RESIDENT_BUDGET_MB stands in for a full device
    size_t free_b = 0, total_b = 0;
    if (hipMemGetInfo(&free_b, &total_b) != hipSuccess) return refuse("hipMemGetInfo failed");
    const size_t reserve = std::max<size_t>(2ull << 30, total_b / 32);
    size_t evictable = 0;
    for (Resident *r : d->resident)
        if (r->db != d->resident_pin) evictable += r->dev_bytes;
    const size_t cap = d->hooks.resident_budget_mb ? (size_t)d->hooks.resident_budget_mb << 20
                       : d->hooks.resident_max_mb   ? (size_t)d->hooks.resident_max_mb << 20
                                                    : total_b / 2;
    size_t held = 0;
    for (Resident *r : d->resident) held += r->dev_bytes;
    if (dev_bytes + reserve > free_b + evictable || dev_bytes > cap || held - evictable + dev_bytes > cap)
        return refuse("the file (" + std::to_string(dev_bytes >> 20) + " MB on the device) does not fit the free memory "
                      "or the copies' cap (" + std::to_string(cap >> 20) + " MB)");
    while (dev_bytes + reserve > free_b && resident_evict_one(d)) {
        if (hipMemGetInfo(&free_b, &total_b) != hipSuccess) return refuse("hipMemGetInfo failed");
    }
    for (;;) {
        held = 0;
        for (Resident *r : d->resident) held += r->dev_bytes;
        if (held + dev_bytes <= cap || !resident_evict_one(d)) break;
    }
    Resident *r = new (std::nothrow) Resident();
    if (!r) return refuse("out of host memory");
    r->fd = fd;  // owned by r from here
    r->db = new (std::nothrow) iris_db();
    if (!r->db || dev_malloc(d, &r->db->data, dev_bytes, "resident copy") != 0) {
        (void)hipGetLastError();
        if (r->db) r->db->data = nullptr;
        free_copy(d, r);
        return ineligible("hipMalloc of the copy failed");
    }
    // zeroed: the last block's padding records are never candidates
    if (hipMemsetAsync(r->db->data, 0, dev_bytes, d->stream) != hipSuccess) {
        free_copy(d, r);
        return nullptr;
    }
    r->db->dev = d;
    r->db->k = k;
    r->db->cap = blocks * k.block;
    r->db->len = nrec;  // every record is addressable; only uploaded granules are ever computed on
    r->db->version = next_db_version();
    r->kind = kind;
    r->lo = v.lo;
    r->hi = v.hi;
    r->base = base;
    r->file_off = v.off + (base - v.lo);
    r->nrec = nrec;
    r->link = link;
    r->inode = v.inode;
    r->vma_off = v.off;
    r->path = v.path;
    r->vma_checked = std::chrono::steady_clock::now();
    r->st = st;
    r->dev_bytes = dev_bytes;
    r->gran = std::max<uint64_t>(64, kGranuleBytes / rb / 64 * 64);
    r->have.assign((nrec + r->gran - 1) / r->gran, 0);
    r->snap.assign((nrec + kSnapStride - 1) / kSnapStride * kSnapBytes, 0);
    d->resident.push_back(r);
    return r;
}

// The mapped file opened for reading (the held descriptor, else by the mapping's path if that is
// still the mapping's inode), or -1.
int open_mapped(const Resident *r, bool *owned) {
    *owned = false;
    if (r->fd >= 0) return r->fd;
    const int fd = ::open(r->path.c_str(), O_RDONLY | O_CLOEXEC);
    struct stat st;
    if (fd >= 0 && fstat(fd, &st) == 0 && S_ISREG(st.st_mode) && (uint64_t)st.st_ino == r->inode) {
        *owned = true;
        return fd;
    }
    if (fd >= 0) ::close(fd);
    return -1;
}

// Snapshots of the records [a, a + m) held at `recs` (record a first).
void take_snapshots(Resident *r, uint64_t a, uint64_t m, const char *recs) {
    const size_t rb = r->db->k.rec_bytes;
    for (uint64_t i = (a + kSnapStride - 1) / kSnapStride * kSnapStride; i < a + m; i += kSnapStride)
        memcpy(&r->snap[i / kSnapStride * kSnapBytes], recs + (i - a) * rb, std::min(kSnapBytes, rb));
}

// Uploads the granules of [first, first + n) that are not resident yet, read from the file by the
// helper threads into the pinned upload slots (snapshots taken from the slots).  Where the file
// cannot be opened or no pinned slots can be had, from the caller's mapping through the tuned upload.
// A run of missing granules goes as one write, extended ahead of the slice up to kFillRunBytes: the
// slot pipeline's fill and drain then come once per run, not once per granule (a first walk over
// 3.2 GB took 0.135 s granule by granule, against ~75 ms for the pipelined load of the same file).
int fill(iris_device *d, Resident *r, uint64_t first, uint64_t n) {
    const size_t rb = r->db->k.rec_bytes;
    int fd = -1;
    bool owned = false, tried = false;
    int rc = 0;
    for (uint64_t g = first / r->gran; g * r->gran < first + n && rc == 0;) {
        if (r->have[g]) {
            ++g;
            continue;
        }
        if (!tried) {
            fd = open_mapped(r, &owned);
            tried = true;
        }
        uint64_t ge = g + 1;  // the run [g, ge): the slice's missing granules, then read-ahead
        while (ge < r->have.size() && !r->have[ge] &&
               (ge * r->gran < first + n || (ge + 1 - g) * r->gran * rb <= kFillRunBytes))
            ++ge;
        const uint64_t a = g * r->gran, m = std::min<uint64_t>(ge * r->gran, r->nrec) - a;
        rc = IRIS_E_NOMEM;
        if (fd >= 0) {
            const SlotFill read = [&](void *dst, size_t off, size_t bytes) {
                if (!parallel_pread(fd, dst, bytes, (long)(r->file_off + a * rb + off), d->ordinal)) return false;
                take_snapshots(r, a + off / rb, bytes / rb, (const char *)dst);
                return true;
            };
            rc = db_write_pinned(r->db, a, nullptr, m, &read);
        }
        if (rc == IRIS_E_NOMEM) {  // no descriptor, or no pinned slots: the mapping itself
            const char *src = (const char *)r->base + a * rb;
            rc = db_store_locked(r->db, a, src, m);
            if (rc == 0) take_snapshots(r, a, m, src);
        }
        if (rc == 0) std::fill(r->have.begin() + g, r->have.begin() + ge, (uint8_t)1);
        g = ge;
    }
    if (owned) ::close(fd);
    return rc;
}

// The slice's probe: up to three snapshotted records inside [first, first + n) still equal the mapping.
bool probe_ok(const Resident *r, uint64_t first, uint64_t n) {
    const size_t rb = r->db->k.rec_bytes, cmp = std::min(kSnapBytes, rb);
    const uint64_t p0 = (first + kSnapStride - 1) / kSnapStride, p2 = (first + n - 1) / kSnapStride;
    if (p0 > p2) return true;  // no snapshotted record in a slice this short
    const uint64_t ps[3] = {p0, (p0 + p2) / 2, p2};
    for (uint64_t q : ps)
        if (memcmp(&r->snap[q * kSnapBytes], (const char *)r->base + q * kSnapStride * rb, cmp) != 0) return false;
    return true;
}

}  // namespace

int iris_api::resident_slice(iris_device *d, int kind, const void *ptr, uint64_t n, iris_db **db, uint64_t *first,
                             uint64_t *end) {
    *db = nullptr;
    if (!d->hooks.auto_resident || n == 0) return 0;
    resident_sweep(d);
    const uintptr_t p = (uintptr_t)ptr;
    const size_t rb = kind_info(kind, IRIS_LAYOUT_TILES).rec_bytes;
    for (int attempt = 0; attempt < 2; ++attempt) {
        Resident *r = nullptr;
        for (Resident *c : d->resident)
            if (c->kind == kind && p >= c->lo && p < c->hi) {
                r = c;
                break;
            }
        if (!r) {
            const auto t = std::chrono::steady_clock::now();
            bool refused = false;
            for (size_t i = 0; i < d->not_resident.size();) {
                const auto &x = d->not_resident[i];
                if (t >= x.until) {  // expired: dropped, the range is examined afresh
                    d->not_resident[i] = d->not_resident.back();
                    d->not_resident.pop_back();
                    continue;
                }
                refused |= p >= x.lo && p < x.hi;
                ++i;
            }
            if (refused) return 0;
            r = make_resident(d, kind, p, n);
            if (!r) return 0;
        }
        // whole records of this copy's record grid, inside the file's records
        if (p < r->base || (p - r->base) % rb != 0 || (p - r->base) / rb + n > r->nrec) return 0;
        struct stat st;
        if (!file_stat(r, &st) || st.st_dev != r->st.st_dev || st.st_ino != r->st.st_ino ||
            st.st_size != r->st.st_size || !same_time(st.st_mtim, r->st.st_mtim) ||
            !same_time(st.st_ctim, r->st.st_ctim) || !vma_same(r, false)) {
            drop(d, r);  // the mapping went away or its file changed: start over
            continue;
        }
        const uint64_t f = (p - r->base) / rb;
        PinResident pin(d, r->db);  // the fill's workspaces may evict copies: not this one
        if (fill(d, r, f, n) != 0) {  // a short read (the file shrank) or an I/O error: this call uploads
            const uintptr_t lo = r->lo, hi = r->hi;
            drop(d, r);
            remember_not_resident(d, lo, hi, "filling the copy failed: " + g_err);
            return 0;
        }
        if (!probe_ok(r, f, n)) {  // written without a timestamp change: start over
            drop(d, r);
            continue;
        }
        r->last_use = ++d->resident_clock;
        uint64_t g = f / r->gran;
        while (g < r->have.size() && r->have[g]) ++g;
        *db = r->db;
        *first = f;
        *end = std::min<uint64_t>(r->nrec, g * r->gran);
        return 0;
    }
    return 0;  // changed twice in one call: this call uploads
}

void iris_api::resident_drop_all(iris_device *d) {
    while (!d->resident.empty()) drop(d, d->resident.back());
    d->not_resident.clear();
}

bool iris_api::resident_evict_one(iris_device *d) {
    Resident *lru = nullptr;
    for (Resident *r : d->resident)
        if (r->db != d->resident_pin && (!lru || r->last_use < lru->last_use)) lru = r;
    if (!lru) return false;
    drop(d, lru);
    return true;
}

void iris_api::resident_sweep(iris_device *d, bool force) {
    const auto t = std::chrono::steady_clock::now();
    if (d->resident.empty() || (!force && t - d->resident_swept < std::chrono::seconds(1))) return;
    d->resident_swept = t;
    for (size_t i = d->resident.size(); i-- > 0;) {
        Resident *r = d->resident[i];
        if (r->db == d->resident_pin) continue;
        struct stat st;
        if (!file_stat(r, &st) || st.st_ino != r->st.st_ino || st.st_dev != r->st.st_dev || !vma_same(r, true))
            drop(d, r);  // its mapping was unmapped or replaced, or its file is gone
    }
}

int iris_api::dev_malloc(iris_device *d, void **p, size_t bytes, const char *what) {
    hipError_t e = hipMalloc(p, bytes);
    if (e == hipSuccess) return 0;
    (void)hipGetLastError();
    resident_sweep(d, true);
    for (;;) {
        e = hipMalloc(p, bytes);
        if (e == hipSuccess) return 0;
        (void)hipGetLastError();
        if (!resident_evict_one(d)) break;
    }
    *p = nullptr;
    return fail(IRIS_E_NOMEM, std::string("hipMalloc ") + what + " (" + std::to_string(bytes) + " B): " + hipGetErrorString(e));
}

bool iris_api::resident_drop_at(iris_device *d, uintptr_t p) {
    auto &nr = d->not_resident;
    nr.erase(std::remove_if(nr.begin(), nr.end(), [&](const iris_device::NotResident &x) { return p >= x.lo && p < x.hi; }),
             nr.end());
    for (Resident *r : d->resident)
        if (p >= r->lo && p < r->hi) {
            drop(d, r);
            return true;
        }
    return false;
}

void iris_api::resident_stats(const iris_device *d, uint64_t *count, uint64_t *bytes, int *via_fd) {
    *count = d->resident.size();
    *bytes = 0;
    *via_fd = 0;
    for (const Resident *r : d->resident) {
        *bytes += r->dev_bytes;
        *via_fd += r->fd >= 0;
    }
}

extern "C" int iris_device_drop_resident_range(iris_device_t *d, const void *ptr) {
    IRIS_KEEP_DEVICE();
    ARG(d && ptr, "NULL argument");
    std::lock_guard<std::recursive_mutex> g(d->mu);
    CHK(set_device(d));
    (void)resident_drop_at(d, (uintptr_t)ptr);
    return 0;
}

extern "C" int iris_device_drop_resident(iris_device_t *d) {
    IRIS_KEEP_DEVICE();
    ARG(d, "device is NULL");
    std::lock_guard<std::recursive_mutex> g(d->mu);
    CHK(set_device(d));
    resident_drop_all(d);
    return 0;
}
