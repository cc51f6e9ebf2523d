// iris_io.hip — the reference's on-disk record formats <-> device databases,
// its JSON template format, and the C ABI of share
// preparation (row 4; kernel in iris_prepare.hip).
//
// Record files are the raw little-endian bytes of bytemuck::bytes_of over a
// slice of records, exactly what `prepare` writes and `participant` /
// `resolver` mmap (src/main.rs:299-309,341,353-357,386-400,455-469):
//   *.masks      concatenated Bits        (1600 B, u64 limbs)
//   *.share-i    concatenated EncodedBits (25600 B, u16 elements)
//   templates    concatenated Template    (3200 B, pattern then mask)
// Loading maps the file and sends it through the pinned upload slots of large
// writes (the device's helper threads copy 64-MB slots out of the mapping while
// the copy engine drains the other into a staging slot that the pack kernel
// transposes into the TILES layout).  A load that starts while another is in
// flight DMAs straight out of the page cache instead (its mapped pages are
// registered with the device chunk by chunk: no host copy); if the pages cannot
// be registered, reader threads fill two pinned buffers (pread) while the device
// copies the other, so the load runs at the slower of file read and PCIe.
//
// JSON: a top-level array of {"pattern": hex, "mask": hex} objects — serde's
// form of Template with Bits as the lowercase hex of its 1600 LE bytes
// (src/template.rs:11-29, src/bits.rs:74-93), read one object at a time like
// src/json_stream.rs:53-60.
#include <errno.h>
#include <fcntl.h>
#include <stdlib.h>
#include <string.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <atomic>
#include <cstdio>
#include <thread>

#include "iris_handles.hpp"

using namespace iris;
using namespace iris_api;

namespace {

constexpr size_t kIoChunkBytes = 64ull << 20;  // per pinned buffer
constexpr int kReadThreads = 8;

struct Fd {
    int fd = -1;
    ~Fd() {
        if (fd >= 0) ::close(fd);
    }
};

struct Pinned {
    void *p = nullptr;
    ~Pinned() {
        if (p) (void)hipHostFree(p);
    }
};

struct Event {
    hipEvent_t e = nullptr;
    ~Event() {
        if (e) (void)hipEventDestroy(e);
    }
};

// pread/pwrite of [off, off+bytes) split over kReadThreads threads; false on error.
bool parallel_io(int fd, char *buf, size_t bytes, off_t off, bool write) {
    const size_t per = (bytes + kReadThreads - 1) / kReadThreads;
    bool ok[kReadThreads];
    std::vector<std::thread> th;
    for (int i = 0; i < kReadThreads; ++i) {
        ok[i] = true;
        const size_t lo = std::min(bytes, i * per), hi = std::min(bytes, lo + per);
        if (lo == hi) continue;
        th.emplace_back([=, &ok] {
            size_t done = lo;
            while (done < hi) {
                const ssize_t r = write ? ::pwrite(fd, buf + done, hi - done, off + (off_t)done)
                                        : ::pread(fd, buf + done, hi - done, off + (off_t)done);
                if (r < 0 && errno == EINTR) continue;
                if (r <= 0) {
                    ok[i] = false;
                    return;
                }
                done += (size_t)r;
            }
        });
    }
    for (auto &t : th) t.join();
    for (int i = 0; i < kReadThreads; ++i)
        if (!ok[i]) return false;
    return true;
}

const char *kind_name(int kind) {
    return kind == IRIS_KIND_MASKS ? "masks" : kind == IRIS_KIND_SHARES ? "share" : "template";
}

}  // namespace

extern "C" {

int iris_db_load_file(iris_db_t *db, const char *path, uint64_t first, uint64_t count, uint64_t *loaded) {
    IRIS_KEEP_DEVICE();
    ARG(db && path, "NULL argument");
    if (loaded) *loaded = 0;
    iris_device *d = db->dev;
    std::lock_guard<std::recursive_mutex> g(d->mu);
    CHK(set_device(d));
    const KindInfo &k = db->k;
    Fd f;
    f.fd = ::open(path, O_RDONLY | O_CLOEXEC);
    if (f.fd < 0) return fail(IRIS_E_IO, std::string("failed to open ") + path + ": " + strerror(errno));
    struct stat st;
    if (::fstat(f.fd, &st) != 0) return fail(IRIS_E_IO, std::string("stat ") + path + ": " + strerror(errno));
    const uint64_t size = (uint64_t)st.st_size;
    // bytemuck::try_cast_slice fails on a partial record (src/main.rs:392-393, 461-462)
    if (size % k.rec_bytes != 0)
        return fail(IRIS_E_ARG, std::string(kind_name(k.kind)) + " file " + path + " invalid: " +
                                    std::to_string(size) + " bytes is not a multiple of " +
                                    std::to_string(k.rec_bytes));
    const uint64_t total = size / k.rec_bytes;
    if (first > total) return fail(IRIS_E_RANGE, "iris_db_load_file: first record beyond the end of the file");
    const uint64_t n = std::min<uint64_t>(count, total - first);
    if (n > db->cap - db->len) return fail(IRIS_E_RANGE, "iris_db_load_file: database capacity exceeded");
    if (n == 0) return 0;
    db_detach(db);

    const uint64_t ch = std::max<uint64_t>(1, kIoChunkBytes / k.rec_bytes);
    const size_t chb = ch * k.rec_bytes;
    CHK(ensure(d, d->staging, 2 * chb));
    const uint64_t base = db->len;
    Event done[2];
    for (int b = 0; b < 2; ++b) HIPCHK(hipEventCreateWithFlags(&done[b].e, hipEventDisableTiming));
    // Fast path: DMA straight out of the page cache.  The file is mapped and each
    // chunk's pages are registered with the device (hipHostRegister, read-only) while
    // the previous chunk copies; no host-side copy (measured 56 GB/s against 41 GB/s
    // for pread into pinned buffers, tools/ubench_file_dma.cpp).  Falls back to the
    // pread path if the mapping cannot be registered.
    {
        // Chunks end on page boundaries so that no page is registered twice: chunk sizes are
        // multiples of `unit` records (unit * rec_bytes is a multiple of the page), after a
        // first chunk that runs up to the first page-aligned record boundary.
        const size_t page = (size_t)sysconf(_SC_PAGESIZE);
        size_t gcd = page, rem = k.rec_bytes;
        while (rem) {
            const size_t t = gcd % rem;
            gcd = rem;
            rem = t;
        }
        const uint64_t unit = page / gcd;
        const uint64_t pch = std::max<uint64_t>(unit, ch / unit * unit);
        const uint64_t lead = (first + unit - 1) / unit * unit - first;  // records before an aligned boundary
        const bool force_pread = db->dev->hooks.load_pread;  // test hook: the fallback path
        void *map = pch <= ch && !force_pread ? ::mmap(nullptr, (size_t)size, PROT_READ, MAP_SHARED, f.fd, 0)
                                              : MAP_FAILED;
        // loads running at once in this process (a device group's per-device loads): those after the
        // first keep the registered windows, which take no host copy -- eight GPUs' slot copies
        // would all read host memory at once (unmeasured here: one GPU per box)
        static std::atomic<int> loads{0};
        struct InFlight {
            int before;
            InFlight() : before(loads.fetch_add(1)) {}
            ~InFlight() { loads.fetch_sub(1); }
        } in_flight;
        if (map != MAP_FAILED && in_flight.before == 0 && !d->hooks.load_windows) {
            // reader threads pread the file into two pinned slots while the copy engine drains the
            // other (the path of large writes, db_write_pinned); the registered windows below
            // moved 35-37 GB/s including their registration (profiles/r04_load_slots.txt).  pread,
            // not a copy out of the mapping: a file truncated under the load or a failing page is
            // an IRIS_E_IO return, not a SIGBUS
            const off_t off0 = (off_t)first * (off_t)k.rec_bytes;
            const SlotFill fill = [&](void *dst, size_t off, size_t bytes) {
                return parallel_pread(f.fd, dst, bytes, off0 + (off_t)off, d->ordinal);
            };
            const int rc = db_write_pinned(db, base, nullptr, n, &fill);
            if (rc != IRIS_E_NOMEM) {  // no pinned memory for the slots: the registered windows below
                ::munmap(map, (size_t)size);
                CHK(rc);
                if (loaded) *loaded = n;
                return 0;
            }
        }
        if (map != MAP_FAILED) {
            // hipHostUnregister waits for the device, so windows stay registered (their
            // registration overlapping the previous window's copy) and are released in
            // batches of up to 4 GB
            constexpr size_t kPinBatch = 4ull << 30;
            std::vector<char *> reg;
            size_t pinned = 0;
            bool ok = true;
            int rc = 0;
            auto release = [&] {
                if (reg.empty()) return hipSuccess;
                const hipError_t e = hipStreamSynchronize(d->stream);
                for (char *w : reg) (void)hipHostUnregister(w);
                reg.clear();
                pinned = 0;
                return e;
            };
            uint64_t off = 0;
            for (int i = 0; off < n; ++i) {
                const int b = i & 1;
                const uint64_t m = std::min<uint64_t>(i == 0 && lead ? lead : pch, n - off);
                const size_t s0 = (size_t)(first + off) * k.rec_bytes, s1 = s0 + (size_t)m * k.rec_bytes;
                char *a0 = (char *)map + s0 / page * page;
                const size_t alen = std::min((s1 + page - 1) / page * page, (size_t)size) - s0 / page * page;
                if (pinned + alen > kPinBatch && release() != hipSuccess) {
                    rc = fail(IRIS_E_HIP, "load: stream synchronize");
                    break;
                }
                if (hipHostRegister(a0, alen, hipHostRegisterReadOnly) != hipSuccess) {
                    (void)hipGetLastError();
                    ok = false;  // e.g. a file system whose pages cannot be pinned
                    break;
                }
                reg.push_back(a0);
                pinned += alen;
                char *dst = (char *)d->staging.p + (size_t)b * chb;
                const hipError_t e = hipMemcpyAsync(dst, (char *)map + s0, s1 - s0, hipMemcpyHostToDevice, d->stream);
                if (e != hipSuccess) { rc = fail(IRIS_E_HIP, std::string("load: copy: ") + hipGetErrorString(e)); break; }
                rc = timed(d, "pack", m, [&] { return launch_pack(d->stream, k, dst, db->data, base + off, m); });
                if (rc != 0) break;
                off += m;
            }
            const int src = sync(d);
            (void)release();
            ::munmap(map, (size_t)size);
            if (rc != 0) return rc;
            if (src != 0) return src;
            if (ok) {
                db->len = base + n;
                if (loaded) *loaded = n;
                return 0;
            }
            // not registrable: redo the whole range through pinned buffers below
        }
    }
    Pinned host[2];
    for (int b = 0; b < 2; ++b) HIPCHK(hipHostMalloc(&host[b].p, chb, hipHostMallocDefault));
    uint64_t off = 0;
    for (int i = 0; off < n; ++i, off += ch) {
        const int b = i & 1;
        const uint64_t m = std::min<uint64_t>(ch, n - off);
        HIPCHK(hipEventSynchronize(done[b].e));  // the H2D copy that last read host[b] has finished
        if (!parallel_io(f.fd, (char *)host[b].p, m * k.rec_bytes, (off_t)((first + off) * k.rec_bytes), false))
            return fail(IRIS_E_IO, std::string("read ") + path + ": " + strerror(errno));
        char *dst = (char *)d->staging.p + (size_t)b * chb;
        HIPCHK(hipMemcpyAsync(dst, host[b].p, m * k.rec_bytes, hipMemcpyHostToDevice, d->stream));
        HIPCHK(hipEventRecord(done[b].e, d->stream));
        CHK(timed(d, "pack", m, [&] { return launch_pack(d->stream, k, dst, db->data, base + off, m); }));
    }
    CHK(sync(d));
    db->len = base + n;
    if (loaded) *loaded = n;
    return 0;
}

int iris_db_save_file(const iris_db_t *db, const char *path, uint64_t first, uint64_t n) {
    IRIS_KEEP_DEVICE();
    ARG(db && path, "NULL argument");
    iris_device *d = db->dev;
    std::lock_guard<std::recursive_mutex> g(d->mu);
    CHK(set_device(d));
    if (first > db->len || n > db->len - first) return fail(IRIS_E_RANGE, "record range outside the database");
    const KindInfo &k = db->k;
    Fd f;
    f.fd = ::open(path, O_WRONLY | O_CREAT | O_TRUNC | O_CLOEXEC, 0644);
    if (f.fd < 0) return fail(IRIS_E_IO, std::string("failed to create ") + path + ": " + strerror(errno));
    if (n == 0) return 0;
    const uint64_t ch = std::max<uint64_t>(1, kIoChunkBytes / k.rec_bytes);
    const size_t chb = ch * k.rec_bytes;
    Pinned host[2];
    Event ready[2];
    for (int b = 0; b < 2; ++b) {
        HIPCHK(hipHostMalloc(&host[b].p, chb, hipHostMallocDefault));
        HIPCHK(hipEventCreateWithFlags(&ready[b].e, hipEventDisableTiming));
    }
    CHK(ensure(d, d->staging, 2 * chb));
    // issue chunk i's unpack + D2H, then write chunk i-1 while it runs
    uint64_t prev_off = 0, prev_m = 0;
    for (uint64_t off = 0, i = 0; off < n || prev_m; ++i) {
        const int b = (int)(i & 1);
        uint64_t m = 0;
        if (off < n) {
            m = std::min<uint64_t>(ch, n - off);
            char *src = (char *)d->staging.p + (size_t)b * chb;
            CHK(timed(d, "unpack", m, [&] { return launch_unpack(d->stream, k, db->data, src, first + off, m); }));
            HIPCHK(hipMemcpyAsync(host[b].p, src, m * k.rec_bytes, hipMemcpyDeviceToHost, d->stream));
            HIPCHK(hipEventRecord(ready[b].e, d->stream));
        }
        if (prev_m) {
            const int pb = b ^ 1;
            HIPCHK(hipEventSynchronize(ready[pb].e));
            if (!parallel_io(f.fd, (char *)host[pb].p, prev_m * k.rec_bytes, (off_t)(prev_off * k.rec_bytes), true))
                return fail(IRIS_E_IO, std::string("write ") + path + ": " + strerror(errno));
        }
        prev_off = off;
        prev_m = m;
        off += m;
    }
    CHK(sync(d));
    return 0;
}

}  // extern "C"

// ------------------------------------------------------------------ JSON templates

namespace {

struct JsonIn {
    FILE *f = nullptr;
    uint64_t pos = 0;
    ~JsonIn() {
        if (f) fclose(f);
    }
    int get() {
        const int c = getc_unlocked(f);
        if (c != EOF) ++pos;
        return c;
    }
    int skip_ws() {
        int c;
        do c = get();
        while (c == ' ' || c == '\t' || c == '\n' || c == '\r');
        return c;
    }
};

int hexval(int c) {
    if (c >= '0' && c <= '9') return c - '0';
    if (c >= 'a' && c <= 'f') return c - 'a' + 10;
    if (c >= 'A' && c <= 'F') return c - 'A' + 10;  // hex::deserialize accepts both cases
    return -1;
}

int json_err(const JsonIn &in, const std::string &what) {
    return fail(IRIS_E_FORMAT, "JSON templates: " + what + " at byte " + std::to_string(in.pos));
}

// reads a JSON string (after its opening quote) of plain characters into s
int read_key(JsonIn &in, std::string &s) {
    s.clear();
    for (;;) {
        const int c = in.get();
        if (c == EOF) return json_err(in, "unterminated string");
        if (c == '"') return 0;
        if (c == '\\') return json_err(in, "escape in key");
        s.push_back((char)c);
        if (s.size() > 64) return json_err(in, "key too long");
    }
}

// reads a hex string (after its opening quote) of exactly IRIS_LIMBS * 8 bytes into limbs (LE)
int read_bits_hex(JsonIn &in, uint64_t *limbs) {
    uint8_t *bytes = (uint8_t *)limbs;
    const size_t nb = IRIS_LIMBS * 8;
    size_t i = 0;
    for (;;) {
        const int c = in.get();
        if (c == EOF) return json_err(in, "unterminated string");
        if (c == '"') break;
        const int lo_c = in.get();
        const int hi = hexval(c), lo = hexval(lo_c);
        if (hi < 0 || lo < 0) return json_err(in, "invalid hex digit");
        if (i >= nb) return json_err(in, "Bits hex longer than 1600 bytes");
        bytes[i++] = (uint8_t)(hi * 16 + lo);
    }
    // try_cast_slice + try_into to [u64; 200] (src/bits.rs:84-92)
    if (i != nb) return json_err(in, "Bits hex is " + std::to_string(i) + " bytes, expected 1600");
    return 0;
}

int read_template(JsonIn &in, iris_template_t *t) {
    bool have_p = false, have_m = false;
    int c = in.skip_ws();
    if (c != '{') return json_err(in, "expected '{'");
    c = in.skip_ws();
    if (c == '}') return json_err(in, "missing field `pattern`");
    for (;;) {
        if (c != '"') return json_err(in, "expected a key");
        std::string key;
        CHK(read_key(in, key));
        if (in.skip_ws() != ':') return json_err(in, "expected ':'");
        if (in.skip_ws() != '"') return json_err(in, "expected a hex string");
        uint64_t tmp[IRIS_LIMBS];
        if (key == "pattern") {
            if (have_p) return json_err(in, "duplicate field `pattern`");
            CHK(read_bits_hex(in, t->pattern));
            have_p = true;
        } else if (key == "mask") {
            if (have_m) return json_err(in, "duplicate field `mask`");
            CHK(read_bits_hex(in, t->mask));
            have_m = true;
        } else {
            CHK(read_bits_hex(in, tmp));  // serde ignores unknown fields of this shape
        }
        c = in.skip_ws();
        if (c == '}') break;
        if (c != ',') return json_err(in, "expected ',' or '}'");
        c = in.skip_ws();
    }
    if (!have_p) return json_err(in, "missing field `pattern`");
    if (!have_m) return json_err(in, "missing field `mask`");
    return 0;
}

}  // namespace

extern "C" {

int iris_templates_read_json(const char *path, iris_template_t *out, uint64_t cap, uint64_t *n) {
    ARG(path && n, "NULL argument");
    *n = 0;
    JsonIn in;
    in.f = fopen(path, "rb");
    if (!in.f) return fail(IRIS_E_IO, std::string("failed to open ") + path + ": " + strerror(errno));
    int c = in.skip_ws();
    if (c != '[') return json_err(in, "`[` not found");
    c = in.skip_ws();
    if (c == ']') return 0;
    ungetc(c, in.f);
    --in.pos;
    iris_template_t scratch;
    for (uint64_t i = 0;; ++i) {
        iris_template_t *t = (out && i < cap) ? out + i : &scratch;
        CHK(read_template(in, t));
        *n = i + 1;
        c = in.skip_ws();
        if (c == ']') break;
        if (c != ',') return json_err(in, "`,` or `]` not found");
    }
    if (out && *n > cap) return fail(IRIS_E_RANGE, "iris_templates_read_json: more templates than cap (n holds the count)");
    return 0;
}

int iris_templates_write_json(const char *path, const iris_template_t *t, uint64_t n) {
    ARG(path && (t || n == 0), "NULL argument");
    FILE *f = fopen(path, "wb");
    if (!f) return fail(IRIS_E_IO, std::string("failed to create ") + path + ": " + strerror(errno));
    static const char *hex = "0123456789abcdef";
    std::string line;
    bool ok = fputc('[', f) != EOF;
    for (uint64_t i = 0; ok && i < n; ++i) {
        line.clear();
        line += i ? "," : "";
        for (int part = 0; part < 2; ++part) {
            line += part ? "\"mask\":\"" : "{\"pattern\":\"";
            const uint8_t *b = (const uint8_t *)(part ? t[i].mask : t[i].pattern);
            for (int j = 0; j < IRIS_LIMBS * 8; ++j) {
                line.push_back(hex[b[j] >> 4]);
                line.push_back(hex[b[j] & 15]);
            }
            line += part ? "\"}" : "\",";
        }
        ok = fwrite(line.data(), 1, line.size(), f) == line.size();
    }
    ok = ok && fputc(']', f) != EOF;
    ok = (fclose(f) == 0) && ok;
    if (!ok) return fail(IRIS_E_IO, std::string("write ") + path + ": " + strerror(errno));
    return 0;
}

}  // extern "C"

// ------------------------------------------------------------------ share preparation

extern "C" int iris_prepare_shares(const iris_db_t *templates, uint64_t first, uint64_t n, uint64_t index_base,
                                   const uint8_t key[32], uint64_t nonce, uint32_t rounds, uint32_t parties,
                                   iris_db_t *const *shares, iris_db_t *masks) {
    ARG(templates && key && shares, "NULL argument");
    ARG(rounds == 8 || rounds == 12 || rounds == 20, "rounds must be 8, 12 or 20 (ChaCha8/12/20)");
    ARG(parties >= 1 && parties <= 64, "parties must be 1..64 (EncodedBits::share asserts n > 0)");
    ARG(templates->k.kind == IRIS_KIND_TEMPLATES, "iris_prepare_shares needs a template database");
    iris_device *d = templates->dev;
    for (uint32_t j = 0; j < parties; ++j) {
        ARG(shares[j] && shares[j]->k.kind == IRIS_KIND_SHARES, "shares[j] must be a share database");
        ARG(shares[j]->dev == d, "all databases must live on one device");
        for (uint32_t i = 0; i < j; ++i) ARG(shares[i] != shares[j], "share databases must be distinct");
        if (n > shares[j]->cap - shares[j]->len) return fail(IRIS_E_RANGE, "share database capacity exceeded");
    }
    if (masks) {
        ARG(masks->k.kind == IRIS_KIND_MASKS && masks->dev == d, "masks must be a masks database on the same device");
        if (n > masks->cap - masks->len) return fail(IRIS_E_RANGE, "masks database capacity exceeded");
    }
    std::lock_guard<std::recursive_mutex> g(d->mu);
    CHK(set_device(d));
    if (first > templates->len || n > templates->len - first)
        return fail(IRIS_E_RANGE, "record range outside the database");
    if (n == 0) return 0;
    for (uint32_t j = 0; j < parties; ++j) db_detach(shares[j]);
    if (masks) db_detach(masks);
    bool all_tiles = templates->k.layout == IRIS_LAYOUT_TILES && (!masks || masks->k.layout == IRIS_LAYOUT_TILES);
    for (uint32_t j = 0; j < parties; ++j) all_tiles &= shares[j]->k.layout == IRIS_LAYOUT_TILES;
    if (all_tiles) {  // one in-place launch: TILES templates -> TILES shares + masks
        std::vector<void *> dbp(parties);
        std::vector<uint64_t> sf(parties);
        for (uint32_t j = 0; j < parties; ++j) {
            dbp[j] = shares[j]->data;
            sf[j] = shares[j]->len;
        }
        CHK(timed(d, "prepare", n, [&] {
            return launch_prepare_direct(d->stream, templates->data, first, n, index_base + first, key, nonce, rounds, parties,
                                         dbp.data(), sf.data(), masks ? masks->data : nullptr, masks ? masks->len : 0);
        }));
        CHK(sync(d));
        for (uint32_t j = 0; j < parties; ++j) shares[j]->len += n;
        if (masks) masks->len += n;
        return 0;
    }
    // staging per record: template (3200 B) | mask (1600 B) | the shares (25600 B each) unless
    // every share database is TILES, which the keystream kernel writes in place
    bool direct = true;
    for (uint32_t j = 0; j < parties; ++j) direct &= shares[j]->k.layout == IRIS_LAYOUT_TILES;
    const size_t tb = kind_info(IRIS_KIND_TEMPLATES, IRIS_LAYOUT_TILES).rec_bytes;
    const size_t mb = kind_info(IRIS_KIND_MASKS, IRIS_LAYOUT_TILES).rec_bytes;
    const size_t sb = kind_info(IRIS_KIND_SHARES, IRIS_LAYOUT_TILES).rec_bytes;
    const size_t per = tb + mb + (direct ? 0 : (size_t)parties * sb);
    const uint64_t ch = std::max<uint64_t>(64, (kStagingBytes / per) / 64 * 64);
    const uint64_t m0 = std::min<uint64_t>(ch, n);
    CHK(ensure(d, d->staging, m0 * per));
    char *st_t = (char *)d->staging.p, *st_m = st_t + m0 * tb, *st_s = st_m + m0 * mb;
    std::vector<uint64_t> base(parties), tf(parties);
    std::vector<void *> dbp(parties);
    for (uint32_t j = 0; j < parties; ++j) {
        base[j] = shares[j]->len;
        dbp[j] = shares[j]->data;
    }
    const uint64_t mbase = masks ? masks->len : 0;
    for (uint64_t off = 0; off < n; off += ch) {
        const uint64_t m = std::min<uint64_t>(ch, n - off);
        CHK(timed(d, "unpack", m,
                  [&] { return launch_unpack(d->stream, templates->k, templates->data, st_t, first + off, m); }));
        if (direct) {
            for (uint32_t j = 0; j < parties; ++j) tf[j] = base[j] + off;
            CHK(timed(d, "prepare", m, [&] {
                return launch_prepare_shares_tiles(d->stream, st_t, m, index_base + first + off, key, nonce, rounds, parties,
                                                   dbp.data(), tf.data());
            }));
        } else {
            CHK(timed(d, "prepare", m, [&] {
                return launch_prepare_shares(d->stream, st_t, m, index_base + first + off, key, nonce, rounds, parties, st_s);
            }));
            for (uint32_t j = 0; j < parties; ++j)
                CHK(timed(d, "pack", m, [&] {
                    return launch_pack(d->stream, shares[j]->k, st_s + (size_t)j * m * sb, shares[j]->data,
                                       base[j] + off, m);
                }));
        }
        if (masks) {
            HIPCHK(hipMemcpy2DAsync(st_m, mb, st_t + mb, tb, mb, m, hipMemcpyDeviceToDevice, d->stream));
            CHK(timed(d, "pack", m, [&] { return launch_pack(d->stream, masks->k, st_m, masks->data, mbase + off, m); }));
        }
        CHK(sync(d));
    }
    for (uint32_t j = 0; j < parties; ++j) shares[j]->len = base[j] + n;
    if (masks) masks->len = mbase + n;
    return 0;
}
