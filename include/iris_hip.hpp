/*
 * iris_hip.hpp — the reference's Rust API, restated in C++17 over the C ABI.
 *
 * recmo/mpc-iris-code is compiled Rust and this image has no Rust toolchain,
 * so the host side above include/iris_hip.h is this header: the same names,
 * argument meaning and error behaviour as the crate's public items
 *   src/lib.rs          COLS ROWS BITS, encode, DistanceEngine, MasksEngine,
 *                       distances, denominators, decode_distance
 *   src/bits.rs         Bits (rotate, rotated, count_ones, dot, index, & | ^ !)
 *   src/encoded_bits.rs EncodedBits (share, rotate, rotated, sum, dot,
 *                       From<&Bits>, - + * and their assign forms)
 *   src/template.rs     Template (rotate, rotated, distance, fraction_hamming)
 *   src/arch/mod.rs     arch::dot_bool, arch::dot_u16
 * plus the device-resident forms the GPU adds (Device, Database,
 * TemplateEngine, resolver_search, prepare_shares).  A Rust panic
 * (`assert_eq!(out.len(), db.len())`, src/lib.rs:43,70) is an
 * iris_hip::Error exception carrying the ABI status (IRIS_E_ARG).
 *
 * Everything that compares bits runs on the GPU: Bits::dot / EncodedBits::dot
 * are one-pair calls of the arch kernels, Template::distance a one-record
 * TemplateEngine — correct but launch-bound, as the reference's per-pair
 * functions are; batch through the engines.  Value-type plumbing (rotation,
 * encode, wrapping arithmetic, bit access) is host code, as in the reference.
 *
 * Header-only; link with -liris_hip (mpc-iris-code_amd/libiris_hip.so).
 */
#ifndef IRIS_HIP_HPP
#define IRIS_HIP_HPP

#include <array>
#include <cstdint>
#include <cstring>
#include <memory>
#include <mutex>
#include <stdexcept>
#include <string>
#include <vector>

#include <sys/random.h>

#include "iris_hip.h"

namespace mpc_iris_code {

constexpr std::size_t COLS = IRIS_COLS;              // src/lib.rs:10
constexpr std::size_t ROWS = IRIS_ROWS;              // src/lib.rs:11
constexpr std::size_t BITS = IRIS_BITS;              // src/lib.rs:12
constexpr std::size_t LIMBS = IRIS_LIMBS;            // src/bits.rs:10
constexpr std::size_t ROTATIONS = IRIS_ROTATIONS;    // 31 = -15..=15
using Rotations = std::array<uint16_t, ROTATIONS>;   // [u16; 31]
using Match = iris_match_t;

class Error : public std::runtime_error {
public:
    Error(int code, const std::string &msg) : std::runtime_error("iris_hip error " + std::to_string(code) + ": " + msg), code(code) {}
    int code;
};

inline void check(int rc) {
    if (rc != 0) throw Error(rc, iris_last_error());
}

// ------------------------------------------------------------------ device

class Device {
public:
    explicit Device(int ordinal = 0) { check(iris_device_open(ordinal, &h_)); }
    ~Device() {
        if (h_) iris_device_close(h_);
    }
    Device(const Device &) = delete;
    Device &operator=(const Device &) = delete;
    iris_device_t *handle() const { return h_; }
    void synchronize() const { check(iris_device_synchronize(h_)); }
    // Frees the resident copy of the file mapping holding `p` (after rewriting the file through a
    // writable mapping, which the per-call check does not see); drop_resident() frees them all.
    void drop_resident_range(const void *p) const { check(iris_device_drop_resident_range(h_, p)); }
    void drop_resident() const { check(iris_device_drop_resident(h_)); }
    // The process-wide device the value types' per-pair GPU calls use (ordinal 0).
    static Device &default_device() {
        static Device d(0);
        return d;
    }

private:
    iris_device_t *h_ = nullptr;
};

// ------------------------------------------------------------------ Bits (src/bits.rs)

struct Bits {
    std::array<uint64_t, LIMBS> limbs{};  // pub [u64; LIMBS], little-endian bit order

    void rotate(int32_t amount) { *this = rotated(amount); }
    Bits rotated(int32_t amount) const {
        Bits out;
        check(iris_bits_rotated(limbs.data(), amount, out.limbs.data()));
        return out;
    }
    uint16_t count_ones() const {
        unsigned n = 0;
        for (uint64_t l : limbs) n += (unsigned)__builtin_popcountll(l);
        return (uint16_t)n;
    }
    uint16_t dot(const Bits &other) const;  // arch::dot_bool (GPU)
    bool operator[](std::size_t i) const { return (limbs[i / 64] >> (i % 64)) & 1u; }
    void set(std::size_t i, bool v) {
        const uint64_t b = uint64_t(1) << (i % 64);
        limbs[i / 64] = v ? (limbs[i / 64] | b) : (limbs[i / 64] & ~b);
    }
    bool operator==(const Bits &o) const { return limbs == o.limbs; }
    bool operator!=(const Bits &o) const { return limbs != o.limbs; }
    Bits operator~() const {
        Bits r;
        for (std::size_t i = 0; i < LIMBS; ++i) r.limbs[i] = ~limbs[i];
        return r;
    }
#define IRIS_BITS_OP(op)                                                                  \
    Bits &operator op##=(const Bits &o) {                                                 \
        for (std::size_t i = 0; i < LIMBS; ++i) limbs[i] op## = o.limbs[i];               \
        return *this;                                                                     \
    }                                                                                     \
    Bits operator op(const Bits &o) const {                                               \
        Bits r = *this;                                                                   \
        r op## = o;                                                                       \
        return r;                                                                         \
    }
    IRIS_BITS_OP(&)
    IRIS_BITS_OP(|)
    IRIS_BITS_OP(^)
#undef IRIS_BITS_OP
    // rng.gen::<Bits>() (src/bits.rs:95-101): uniform bits from the OS CSPRNG
    static Bits random() {
        Bits b;
        fill_random(b.limbs.data(), sizeof(b.limbs));
        return b;
    }
    static void fill_random(void *p, std::size_t n) {
        for (std::size_t done = 0; done < n;) {
            const ssize_t r = getrandom((char *)p + done, n - done, 0);
            if (r <= 0) throw Error(IRIS_E_ARG, "getrandom failed");
            done += (std::size_t)r;
        }
    }
};
static_assert(sizeof(Bits) == 1600, "Bits is the 1600-byte record of the .masks files");

// ------------------------------------------------------------------ EncodedBits (src/encoded_bits.rs)

struct EncodedBits {
    std::array<uint16_t, BITS> v{};  // pub [u16; BITS]

    EncodedBits() = default;
    // From<&Bits> (src/encoded_bits.rs:75-79): bit i -> 0 / 1
    explicit EncodedBits(const Bits &bits) {
        for (std::size_t i = 0; i < BITS; ++i) v[i] = bits[i] ? 1 : 0;
    }
    void rotate(int32_t amount) { *this = rotated(amount); }
    EncodedBits rotated(int32_t amount) const {
        EncodedBits out;
        check(iris_encoded_rotated(v.data(), amount, out.v.data()));
        return out;
    }
    uint16_t sum() const {  // wrapping sum (src/encoded_bits.rs:60-62)
        uint16_t s = 0;
        for (uint16_t x : v) s = (uint16_t)(s + x);
        return s;
    }
    uint16_t dot(const EncodedBits &other) const;  // arch::dot_u16 (GPU)
    // EncodedBits::share (src/encoded_bits.rs:23-38): n-1 uniform shares from the
    // OS CSPRNG, the last = self - sum(rest).  (Database-scale preparation runs on
    // the GPU: prepare_shares below.)
    std::vector<EncodedBits> share(std::size_t n) const {
        if (n == 0) throw Error(IRIS_E_ARG, "share: n must be > 0");  // assert!(n > 0)
        std::vector<EncodedBits> out(n);
        EncodedBits last = *this;
        for (std::size_t j = 0; j + 1 < n; ++j) {
            Bits::fill_random(out[j].v.data(), sizeof(out[j].v));
            last -= out[j];
        }
        out[n - 1] = last;
        return out;
    }
    bool operator==(const EncodedBits &o) const { return v == o.v; }
    bool operator!=(const EncodedBits &o) const { return v != o.v; }
    EncodedBits operator-() const {
        EncodedBits r;
        for (std::size_t i = 0; i < BITS; ++i) r.v[i] = (uint16_t)(0u - v[i]);
        return r;
    }
#define IRIS_ENC_OP(op)                                                                   \
    EncodedBits &operator op##=(const EncodedBits &o) {                                   \
        for (std::size_t i = 0; i < BITS; ++i) v[i] = (uint16_t)(v[i] op o.v[i]);         \
        return *this;                                                                     \
    }                                                                                     \
    EncodedBits operator op(const EncodedBits &o) const {                                 \
        EncodedBits r = *this;                                                            \
        r op## = o;                                                                       \
        return r;                                                                         \
    }
    IRIS_ENC_OP(+)
    IRIS_ENC_OP(-)
    IRIS_ENC_OP(*)
#undef IRIS_ENC_OP
    static EncodedBits random() {
        EncodedBits e;
        Bits::fill_random(e.v.data(), sizeof(e.v));
        return e;
    }
};
static_assert(sizeof(EncodedBits) == 25600, "EncodedBits is the 25600-byte record of the .share-i files");

// ------------------------------------------------------------------ Template (src/template.rs)

struct Template {
    Bits pattern;
    Bits mask;

    void rotate(int32_t amount) {
        pattern.rotate(amount);
        mask.rotate(amount);
    }
    Template rotated(int32_t amount) const {
        Template t = *this;
        t.rotate(amount);
        return t;
    }
    double distance(const Template &other) const;          // min over -15..=15 (GPU)
    double fraction_hamming(const Template &other) const;  // rotation 0 (GPU)
    bool operator==(const Template &o) const { return pattern == o.pattern && mask == o.mask; }
    static Template random() { return Template{Bits::random(), Bits::random()}; }
    const iris_template_t *c() const { return reinterpret_cast<const iris_template_t *>(this); }
};
static_assert(sizeof(Template) == sizeof(iris_template_t), "Template is pattern then mask, 3200 B");

// encode (src/lib.rs:16-26): mask - 2 (pattern & mask) as u16
inline EncodedBits encode(const Template &t) {
    EncodedBits out;
    check(iris_encode(t.c(), out.v.data()));
    return out;
}

// decode_distance (src/lib.rs:97-107)
inline double decode_distance(const Rotations &distances, const Rotations &denominators) {
    double d = 0;
    check(iris_decode_distance(distances.data(), denominators.data(), &d));
    return d;
}

// ------------------------------------------------------------------ arch (src/arch/mod.rs)

namespace arch {
// dot_bool / dot_u16 (src/arch/generic.rs:4-16), one pair on the GPU
inline uint16_t dot_bool(const std::array<uint64_t, LIMBS> &a, const std::array<uint64_t, LIMBS> &b,
                         Device &dev = Device::default_device()) {
    uint16_t out = 0;
    check(iris_dot_bool_batch(dev.handle(), a.data(), 1, b.data(), 1, &out));
    return out;
}
inline uint16_t dot_u16(const std::array<uint16_t, BITS> &a, const std::array<uint16_t, BITS> &b,
                        Device &dev = Device::default_device()) {
    uint16_t out = 0;
    check(iris_dot_u16_batch(dev.handle(), a.data(), 1, b.data(), 1, &out));
    return out;
}
// all pairs: out[j * na + i] = dot(a[i], b[j]) (the criterion shapes of src/arch/mod.rs:29,53)
inline std::vector<uint16_t> dot_bool_batch(const std::vector<Bits> &a, const std::vector<Bits> &b,
                                            Device &dev = Device::default_device()) {
    std::vector<uint16_t> out(a.size() * b.size());
    check(iris_dot_bool_batch(dev.handle(), a.empty() ? nullptr : a[0].limbs.data(), a.size(),
                              b.empty() ? nullptr : b[0].limbs.data(), b.size(), out.data()));
    return out;
}
inline std::vector<uint16_t> dot_u16_batch(const std::vector<EncodedBits> &a, const std::vector<EncodedBits> &b,
                                           Device &dev = Device::default_device()) {
    std::vector<uint16_t> out(a.size() * b.size());
    check(iris_dot_u16_batch(dev.handle(), a.empty() ? nullptr : a[0].v.data(), a.size(),
                             b.empty() ? nullptr : b[0].v.data(), b.size(), out.data()));
    return out;
}
}  // namespace arch

inline uint16_t Bits::dot(const Bits &other) const { return arch::dot_bool(limbs, other.limbs); }
inline uint16_t EncodedBits::dot(const EncodedBits &other) const { return arch::dot_u16(v, other.v); }

// ------------------------------------------------------------------ device-resident databases

class Database {
public:
    // kind: IRIS_KIND_MASKS (Bits), IRIS_KIND_SHARES (EncodedBits), IRIS_KIND_TEMPLATES (Template)
    Database(Device &dev, int kind, uint64_t capacity, int layout = IRIS_LAYOUT_DEFAULT) : dev_(&dev) {
        check(iris_db_create_ex(dev.handle(), kind, capacity, layout, &h_));
    }
    ~Database() {
        if (h_) iris_db_destroy(h_);
    }
    Database(const Database &) = delete;
    Database &operator=(const Database &) = delete;
    iris_db_t *handle() const { return h_; }
    Device &device() const { return *dev_; }
    uint64_t len() const {
        uint64_t n = 0;
        check(iris_db_len(h_, &n));
        return n;
    }
    template <class Rec>
    void append(const std::vector<Rec> &records) {
        check(iris_db_append(h_, records.data(), records.size()));
    }
    template <class Rec>
    void append(const Rec *records, uint64_t n) {
        check(iris_db_append(h_, records, n));
    }
    template <class Rec>
    std::vector<Rec> read(uint64_t first, uint64_t n) const {
        std::vector<Rec> out(n);
        check(iris_db_read(h_, first, n, out.data()));
        return out;
    }
    // the reference's on-disk files (src/main.rs:386-400, 455-469)
    uint64_t load_file(const std::string &path, uint64_t first = 0, uint64_t count = UINT64_MAX) {
        uint64_t got = 0;
        check(iris_db_load_file(h_, path.c_str(), first, count, &got));
        return got;
    }
    void save_file(const std::string &path, uint64_t first, uint64_t n) const {
        check(iris_db_save_file(h_, path.c_str(), first, n));
    }
    void generate(uint64_t n, uint64_t seed, uint64_t global_index0) { check(iris_db_generate(h_, n, seed, global_index0)); }
    // This database is the device copy of the host array `records` (e.g. the mmap'd record
    // file, src/main.rs:389-391, 458-460): batch_process(out, slice) on slices of it then runs
    // on the resident copy (iris_db_attach_host).  upload: fill the empty database from it;
    // otherwise it must already hold exactly these records.  `records` must outlive the
    // attachment and stay unchanged; any write or detach() ends it.
    template <class Rec>
    void attach_host(const Rec *records, uint64_t n, bool upload = true) {
        check(iris_db_attach_host(h_, records, n, upload ? 1 : 0));
    }
    void detach_host() { check(iris_db_detach_host(h_)); }

private:
    Device *dev_;
    iris_db_t *h_ = nullptr;
};

// ------------------------------------------------------------------ device groups (multi-GPU)

// Devices searched together: the resolver's fan-out and sequential minimum
// (src/main.rs:486-504, 616-621) over contiguous shards of one template database, the
// per-shard winners all-gathered by the library's RCCL communicator.
class Group {
public:
    explicit Group(const std::vector<int> &ordinals) {
        check(iris_group_create(ordinals.data(), (uint32_t)ordinals.size(), &h_));
    }
    // one device of a multi-process group; `id` from unique_id() on rank 0
    Group(int ordinal, uint32_t nranks, uint32_t rank, const std::array<uint8_t, IRIS_GROUP_ID_BYTES> &id) {
        check(iris_group_create_rank(ordinal, nranks, rank, id.data(), &h_));
    }
    static std::array<uint8_t, IRIS_GROUP_ID_BYTES> unique_id() {
        std::array<uint8_t, IRIS_GROUP_ID_BYTES> id{};
        check(iris_group_unique_id(id.data()));
        return id;
    }
    ~Group() {
        if (h_) iris_group_destroy(h_);
    }
    Group(const Group &) = delete;
    Group &operator=(const Group &) = delete;
    iris_group_t *handle() const { return h_; }
    // bound of the exchange waits of later calls (0: automatic); see include/iris_hip.h
    void set_timeout(uint32_t ms) { check(iris_group_set_timeout(h_, ms)); }

private:
    iris_group_t *h_ = nullptr;
};

class GroupPendingSearch {
public:
    explicit GroupPendingSearch(iris_group_pending_t *p) : p_(p) {}
    GroupPendingSearch(GroupPendingSearch &&o) noexcept : p_(o.p_) { o.p_ = nullptr; }
    GroupPendingSearch(const GroupPendingSearch &) = delete;
    GroupPendingSearch &operator=(const GroupPendingSearch &) = delete;
    ~GroupPendingSearch() {
        if (p_) (void)iris_group_pending_wait(p_, nullptr);
    }
    Match wait() {
        if (!p_) throw Error(IRIS_E_ARG, "GroupPendingSearch::wait called twice");
        Match m{};
        iris_group_pending_t *p = p_;
        p_ = nullptr;
        check(iris_group_pending_wait(p, &m));
        return m;
    }

private:
    iris_group_pending_t *p_;
};

// `total` templates split into ranks x shards_per_device contiguous shards over a Group
class ShardedDatabase {
public:
    ShardedDatabase(Group &g, uint64_t total, int layout = IRIS_LAYOUT_DEFAULT, uint32_t shards_per_device = 1) {
        check(iris_group_db_create(g.handle(), IRIS_KIND_TEMPLATES, total, layout, shards_per_device, &h_));
    }
    ~ShardedDatabase() {
        if (h_) iris_group_db_destroy(h_);
    }
    ShardedDatabase(const ShardedDatabase &) = delete;
    ShardedDatabase &operator=(const ShardedDatabase &) = delete;
    void generate(uint64_t seed) { check(iris_group_db_generate(h_, seed)); }
    void write(uint64_t index, const Template *records, uint64_t n) { check(iris_group_db_write(h_, index, records, n)); }
    void load_file(const std::string &path, uint64_t first = 0) { check(iris_group_db_load_file(h_, path.c_str(), first)); }
    Match search(const Template &query) {
        Match m{};
        check(iris_group_template_search(h_, query.c(), &m));
        return m;
    }
    GroupPendingSearch search_async(const Template &query) {
        iris_group_pending_t *p = nullptr;
        check(iris_group_template_search_async(h_, query.c(), &p));
        return GroupPendingSearch(p);
    }
    std::vector<Match> batch_search(const std::vector<Template> &queries) {
        std::vector<Match> out(queries.size());
        static_assert(sizeof(Template) == sizeof(iris_template_t), "Template is the reference's 3200-B record");
        check(iris_group_template_batch_search(h_, queries.empty() ? nullptr : queries[0].c(), (uint32_t)queries.size(),
                                               out.data()));
        return out;
    }

private:
    iris_group_db_t *h_ = nullptr;
};

// ------------------------------------------------------------------ engines (src/lib.rs:28-80)

namespace detail {
class Engine {
public:
    Engine(const Engine &) = delete;
    Engine &operator=(const Engine &) = delete;
    ~Engine() {
        if (h_) iris_engine_destroy(h_);
    }
    iris_engine_t *handle() const { return h_; }

protected:
    Engine() = default;
    iris_engine_t *h_ = nullptr;
};
}  // namespace detail

// batch_process(&self, out: &mut [[u16; 31]], db: &[T]): assert_eq!(out.len(), db.len())
class DistanceEngine : public detail::Engine {
public:
    explicit DistanceEngine(const EncodedBits &query, Device &dev = Device::default_device()) {
        check(iris_distance_engine_new(dev.handle(), query.v.data(), &h_));
    }
    void batch_process(std::vector<Rotations> &out, const std::vector<EncodedBits> &db) const {
        if (out.size() != db.size()) throw Error(IRIS_E_ARG, "assert_eq!(out.len(), db.len())");
        check(iris_engine_batch_process_host(h_, db.data(), db.size(), out.empty() ? nullptr : out[0].data()));
    }
    // device-resident share database, records [first, first + out.size())
    void batch_process(std::vector<Rotations> &out, const Database &db, uint64_t first = 0) const {
        check(iris_engine_batch_process(h_, db.handle(), first, out.size(), out.empty() ? nullptr : out[0].data()));
    }
};

class MasksEngine : public detail::Engine {
public:
    explicit MasksEngine(const Bits &query, Device &dev = Device::default_device()) {
        check(iris_masks_engine_new(dev.handle(), query.limbs.data(), &h_));
    }
    void batch_process(std::vector<Rotations> &out, const std::vector<Bits> &db) const {
        if (out.size() != db.size()) throw Error(IRIS_E_ARG, "assert_eq!(out.len(), db.len())");
        check(iris_engine_batch_process_host(h_, db.data(), db.size(), out.empty() ? nullptr : out[0].data()));
    }
    void batch_process(std::vector<Rotations> &out, const Database &db, uint64_t first = 0) const {
        check(iris_engine_batch_process(h_, db.handle(), first, out.size(), out.empty() ? nullptr : out[0].data()));
    }
    // The resolver step with these denominators computed on the fly (src/main.rs:510-519 +
    // 597-621): shares_device[p] are device arrays of n * 31 u16 for records [first, first+n).
    Match resolve(const Database &db, const std::vector<const uint16_t *> &shares_device, uint64_t first, uint64_t n,
                  uint64_t index_base = 0) const {
        Match m{};
        check(iris_resolver_search_masks(h_, db.handle(), first, n, shares_device.data(), (uint32_t)shares_device.size(),
                                         index_base, nullptr, &m));
        return m;
    }
    // The same with the participants' outputs in host memory (the rows as they arrive): summed on
    // the host, the sum uploaded (iris_resolver_search_masks_host).
    Match resolve_host(const Database &db, const std::vector<const std::vector<Rotations> *> &shares, uint64_t first,
                       uint64_t index_base = 0) const {
        std::vector<const uint16_t *> p;
        const uint64_t n = shares.empty() ? 0 : shares[0]->size();
        for (const auto *s : shares) {
            if (s->size() != n) throw Error(IRIS_E_ARG, "share arrays of different lengths");
            p.push_back(s->empty() ? nullptr : (*s)[0].data());
        }
        Match m{};
        check(iris_resolver_search_masks_host(h_, db.handle(), first, n, p.data(), (uint32_t)p.size(), index_base, &m));
        return m;
    }
};

// An enqueued search (TemplateEngine::search_async): wait() once for its Match;
// destroying it unwaited waits and discards the result.
class PendingSearch {
public:
    explicit PendingSearch(iris_pending_t *p) : p_(p) {}
    PendingSearch(PendingSearch &&o) noexcept : p_(o.p_) { o.p_ = nullptr; }
    PendingSearch &operator=(PendingSearch &&o) noexcept {
        if (this != &o) {
            if (p_) (void)iris_pending_wait(p_, nullptr);
            p_ = o.p_;
            o.p_ = nullptr;
        }
        return *this;
    }
    PendingSearch(const PendingSearch &) = delete;
    PendingSearch &operator=(const PendingSearch &) = delete;
    ~PendingSearch() {
        if (p_) (void)iris_pending_wait(p_, nullptr);
    }
    Match wait() {
        if (!p_) throw Error(IRIS_E_ARG, "PendingSearch::wait called twice");
        Match m{};
        iris_pending_t *p = p_;
        p_ = nullptr;
        check(iris_pending_wait(p, &m));
        return m;
    }

private:
    iris_pending_t *p_;
};

// Template vs Template database (src/template.rs:43-64) with the resolver's argmin.
class TemplateEngine : public detail::Engine {
public:
    explicit TemplateEngine(const Template &query, Device &dev = Device::default_device()) {
        check(iris_template_engine_new(dev.handle(), query.c(), &h_));
    }
    Match search(const Database &db, uint64_t first, uint64_t n, uint64_t index_base = 0) const {
        Match m{};
        check(iris_template_search(h_, db.handle(), first, n, index_base, nullptr, &m));
        return m;
    }
    // pipelined form: returns once the search is enqueued (the engine may be destroyed before the wait)
    PendingSearch search_async(const Database &db, uint64_t first, uint64_t n, uint64_t index_base = 0) const {
        iris_pending_t *p = nullptr;
        check(iris_template_search_async(h_, db.handle(), first, n, index_base, &p));
        return PendingSearch(p);
    }
    std::vector<double> distances(const Database &db, uint64_t first, uint64_t n) const {
        std::vector<double> out(n);
        check(iris_template_distances(h_, db.handle(), first, n, out.data()));
        return out;
    }
    void counts(const Database &db, uint64_t first, uint64_t n, std::vector<Rotations> &num,
                std::vector<Rotations> &den) const {
        num.resize(n);
        den.resize(n);
        check(iris_template_counts(h_, db.handle(), first, n, n ? num[0].data() : nullptr, n ? den[0].data() : nullptr));
    }
};

// distances / denominators (src/lib.rs:82-94): single-entry wrappers
inline Rotations distances(const EncodedBits &query, const EncodedBits &entry) {
    std::vector<Rotations> out(1);
    DistanceEngine(query).batch_process(out, std::vector<EncodedBits>{entry});
    return out[0];
}
inline Rotations denominators(const Bits &query, const Bits &entry) {
    std::vector<Rotations> out(1);
    MasksEngine(query).batch_process(out, std::vector<Bits>{entry});
    return out[0];
}

inline double Template::distance(const Template &other) const {
    Device &dev = Device::default_device();
    Database db(dev, IRIS_KIND_TEMPLATES, 1);
    db.append(&other, 1);
    return TemplateEngine(*this, dev).distances(db, 0, 1)[0];
}

inline double Template::fraction_hamming(const Template &other) const {
    Device &dev = Device::default_device();
    Database db(dev, IRIS_KIND_TEMPLATES, 1);
    db.append(&other, 1);
    std::vector<Rotations> num, den;
    TemplateEngine(*this, dev).counts(db, 0, 1, num, den);
    const uint16_t n = num[0][IRIS_MAX_ROTATION], d = den[0][IRIS_MAX_ROTATION];  // rotation 0
    return (double)n / (double)d;  // 0/0 = NaN as in the reference
}

// ------------------------------------------------------------------ resolver / prepare

// src/main.rs:597-621 over host arrays: shares[p][i], denominators[i]
inline Match resolver_search(const std::vector<std::vector<Rotations>> &shares, const std::vector<Rotations> &denominators,
                             uint64_t index_base = 0, Device &dev = Device::default_device()) {
    std::vector<const uint16_t *> p;
    for (const auto &s : shares) {
        if (s.size() != denominators.size()) throw Error(IRIS_E_ARG, "shares and denominators differ in length");
        p.push_back(s.empty() ? nullptr : s[0].data());
    }
    Match m{};
    check(iris_resolver_search_host(dev.handle(), p.data(), (uint32_t)p.size(),
                                    denominators.empty() ? nullptr : denominators[0].data(), denominators.size(),
                                    index_base, &m));
    return m;
}

// `prepare` (src/main.rs:333-361) on the device: shares of encode(templates[first..first+n))
inline void prepare_shares(const Database &templates, uint64_t first, uint64_t n, const std::array<uint8_t, 32> &key,
                           const std::vector<Database *> &shares, Database *masks = nullptr, uint64_t nonce = 0,
                           uint64_t index_base = 0, uint32_t rounds = 12) {
    std::vector<iris_db_t *> h;
    for (Database *d : shares) h.push_back(d->handle());
    check(iris_prepare_shares(templates.handle(), first, n, index_base, key.data(), nonce, rounds, (uint32_t)h.size(),
                              h.data(), masks ? masks->handle() : nullptr));
}

}  // namespace mpc_iris_code

#endif  // IRIS_HIP_HPP
