// iris_host.cpp — host-side value-type operations and rotated-query tables.
//
// These run once per engine (31 rotations of one query), never per template.
// Rotation is implemented by its defining formula
//     rot(b, r)[row, col] = b[row, (col - r) mod 200]
// (the reference reaches the same permutation with whole-byte rotates plus a
// carry chain, src/bits.rs:178-205; tests pin the two against each other).
#include <math.h>
#include <stdlib.h>
#include <string.h>

#include "iris_internal.hpp"

namespace iris {

static inline int wrap_col(int c) {
    c %= IRIS_COLS;
    return c < 0 ? c + IRIS_COLS : c;
}

static inline int get_bit(const uint64_t *b, int i) { return (int)((b[i >> 6] >> (i & 63)) & 1u); }

// Bits::rotated (src/bits.rs:18-29)
void bits_rotated(const uint64_t *in, int amount, uint64_t *out) {
    uint64_t tmp[IRIS_LIMBS];
    memset(tmp, 0, sizeof(tmp));
    for (int row = 0; row < IRIS_ROWS; ++row)
        for (int col = 0; col < IRIS_COLS; ++col) {
            const int src = row * IRIS_COLS + wrap_col(col - amount);
            const int dst = row * IRIS_COLS + col;
            tmp[dst >> 6] |= (uint64_t)get_bit(in, src) << (dst & 63);
        }
    memcpy(out, tmp, sizeof(tmp));
}

// EncodedBits::rotated (src/encoded_bits.rs:40-58)
void encoded_rotated(const uint16_t *in, int amount, uint16_t *out) {
    for (int row = 0; row < IRIS_ROWS; ++row)
        for (int col = 0; col < IRIS_COLS; ++col)
            out[row * IRIS_COLS + col] = in[row * IRIS_COLS + wrap_col(col - amount)];
}

// encode (src/lib.rs:16-26): mask - 2 * (pattern & mask), wrapping u16
void encode_template(const iris_template_t *t, uint16_t *out) {
    for (int i = 0; i < IRIS_BITS; ++i) {
        const int m = get_bit(t->mask, i);
        const int p = get_bit(t->pattern, i) & m;
        out[i] = (uint16_t)(m - 2 * p);
    }
}

static inline uint32_t dword_of(const uint64_t *limbs, int w) { return (uint32_t)(limbs[w >> 1] >> (32 * (w & 1))); }

// Rotations of DistanceEngine::new / MasksEngine::new (src/lib.rs:33-40, 60-67),
// k = 0..30 <-> r = k - 15, laid out for the SGPR-operand kernels.
void build_template_table(const iris_template_t *q, uint32_t *tab) {
    memset(tab, 0, sizeof(uint32_t) * kPlaneDwords * kTemplateTabStride);
    for (int k = 0; k < kRot; ++k) {
        uint64_t m[IRIS_LIMBS], p[IRIS_LIMBS];
        bits_rotated(q->mask, k - 15, m);
        bits_rotated(q->pattern, k - 15, p);
        for (int w = 0; w < kPlaneDwords; ++w) {
            tab[w * kTemplateTabStride + 2 * k] = dword_of(m, w);
            tab[w * kTemplateTabStride + 2 * k + 1] = dword_of(p, w);
        }
    }
}

void build_masks_table(const uint64_t *const *vectors, int count, uint32_t *tab) {
    memset(tab, 0, sizeof(uint32_t) * kPlaneDwords * kSlotTabStride);
    for (int k = 0; k < count && k < kRot; ++k)
        for (int w = 0; w < kPlaneDwords; ++w) tab[w * kSlotTabStride + k] = dword_of(vectors[k], w);
}

void build_shares_table(const uint16_t *const *vectors, int count, uint32_t *tab) {
    memset(tab, 0, sizeof(uint32_t) * kShareDwords * kSlotTabStride);
    for (int k = 0; k < count && k < kRot; ++k)
        for (int d = 0; d < kShareDwords; ++d)
            tab[d * kSlotTabStride + k] = (uint32_t)vectors[k][2 * d] | ((uint32_t)vectors[k][2 * d + 1] << 16);
}

void build_masks_rotations(const uint64_t *query, uint32_t *tab) {
    static thread_local uint64_t rot[kRot][IRIS_LIMBS];
    const uint64_t *ptrs[kRot];
    for (int k = 0; k < kRot; ++k) {
        bits_rotated(query, k - 15, rot[k]);
        ptrs[k] = rot[k];
    }
    build_masks_table(ptrs, kRot, tab);
}

void build_shares_rotations(const uint16_t *query, uint32_t *tab) {
    static thread_local uint16_t rot[kRot][IRIS_BITS];
    const uint16_t *ptrs[kRot];
    for (int k = 0; k < kRot; ++k) {
        encoded_rotated(query, k - 15, rot[k]);
        ptrs[k] = rot[k];
    }
    build_shares_table(ptrs, kRot, tab);
}

bool partial_better(const Partial &a, const Partial &b) {
    if (a.den == 0) return false;
    if (b.den == 0) return true;
    const uint64_t l = (uint64_t)a.num * b.den, r = (uint64_t)b.num * a.den;
    if (l != r) return l < r;
    return a.idx < b.idx;
}

}  // namespace iris

namespace iris {

// Query A-fragments of the fp4 MFMA template kernel (iris_mfma.hip).
void build_template_frags(const iris_template_t *q, uint32_t *frag) {
    memset(frag, 0, sizeof(uint32_t) * kTemplateFragDwords);
    for (int k = 0; k < kRot; ++k) {
        uint64_t m[IRIS_LIMBS], p[IRIS_LIMBS];
        bits_rotated(q->mask, k - 15, m);
        bits_rotated(q->pattern, k - 15, p);
        for (int c = 0; c < kPlaneDwords / 2; ++c)
            for (int h = 0; h < 2; ++h) {
                const int w = 2 * c + h;
                const uint32_t mw = dword_of(m, w), pw = dword_of(p, w);
                uint32_t *f = frag + ((size_t)c * 64 + k + 32 * h) * kFragDwords;
                for (int j = 0; j < 32; ++j) {
                    const int b = frag_bit(j);
                    if (!((mw >> b) & 1u)) continue;
                    const uint32_t code = ((pw >> b) & 1u) ? 0xAu : 0x2u;  // -1.0 / +1.0
                    f[j / 8] |= code << (4 * (j % 8));
                }
            }
    }
}

}  // namespace iris

namespace iris {

// fp4 A-fragments of masks_mfma_kernel: row k = vectors[k] (rotations for
// MasksEngine, arbitrary vectors for dot_bool); value 2 / 1 / 0.5 / 0.5 by
// fragment dword, matching the template-side 0.5 / 1 / 2 / 2 (iris_internal.hpp).
void build_masks_frags(const uint64_t *const *vectors, int count, uint32_t *frag) {
    // element j of dword j / 8 has fp4 code {4, 2, 1, 1}[j / 8] (2.0, 1.0, 0.5, 0.5 against the
    // B codes 0.5, 1.0, 2.0, 2.0 of mask_chunk); the kernel selects code bits 2, 1, 0 in place
    // and shifts bit 3 down to bit 0
    static const int bitpos[4] = {2, 1, 0, 3};
    memset(frag, 0, sizeof(uint32_t) * 4 * kMaskFragUint4);
    for (int k = 0; k < count && k < kRot; ++k)
        for (int c = 0; c < kMaskChunks; ++c)
            for (int h = 0; h < 2; ++h) {
                const uint32_t x = dword_of(vectors[k], 2 * c + h);
                uint32_t *f = frag + ((size_t)(c / 4) * 64 + k + 32 * h) * 4 + (c % 4);
                for (int j = 0; j < 32; ++j)
                    if ((x >> mask_frag_bit(j)) & 1u) *f |= 1u << (4 * (j % 8) + bitpos[j / 8]);
            }
}

// i8 A-fragments of shares_mfma_kernel: low / high bytes of row k's elements
// minus 128; row 31 is all ones (per-share byte sums).  After the fragments:
// 32 int2 row constants (sum of biased low bytes, sum of biased high bytes).
void build_shares_frags(const uint16_t *const *vectors, int count, uint32_t *frag) {
    memset(frag, 0, sizeof(uint32_t) * 4 * kShareFragUint4 + 32 * 8);
    int32_t *qsum = (int32_t *)(frag + 4 * kShareFragUint4);
    uint8_t *bytes = (uint8_t *)frag;
    for (int c = 0; c < kShareChunks; ++c)
        for (int h = 0; h < 2; ++h)
            for (int k = 0; k < 32; ++k) {
                uint8_t *lo = bytes + (((size_t)(2 * c) * 64) + k + 32 * h) * 16;
                uint8_t *hi = bytes + (((size_t)(2 * c + 1) * 64) + k + 32 * h) * 16;
                for (int j = 0; j < 16; ++j) {
                    if (k == 31) {
                        lo[j] = 1;
                        hi[j] = 1;
                    } else if (k < count) {
                        const uint16_t e = vectors[k][32 * c + 16 * h + j];
                        lo[j] = (uint8_t)((e & 0xFFu) ^ 0x80u);
                        hi[j] = (uint8_t)((e >> 8) ^ 0x80u);
                        qsum[2 * k] += (int8_t)lo[j];
                        qsum[2 * k + 1] += (int8_t)hi[j];
                    }
                }
            }
}

}  // namespace iris

namespace iris {

// The 31 rotated copies of a query packed as records 0..30 of a TILES tile
// (record 31 zero): the A operand of the batched kernel (iris_batch.hip).
void build_query_tile(const iris_template_t *q, uint32_t *tile) {
    memset(tile, 0, sizeof(uint32_t) * 4 * kPlaneGroups * 64);
    for (int k = 0; k < kRot; ++k) {
        uint64_t m[IRIS_LIMBS], p[IRIS_LIMBS];
        bits_rotated(q->mask, k - 15, m);
        bits_rotated(q->pattern, k - 15, p);
        for (int g = 0; g < kPlaneGroups; ++g)
            for (int h = 0; h < 2; ++h) {
                const uint32_t em0 = dword_of(m, 4 * g + h), ep0 = dword_of(p, 4 * g + h);
                const uint32_t em1 = dword_of(m, 4 * g + 2 + h), ep1 = dword_of(p, 4 * g + 2 + h);
                uint32_t *v = tile + ((size_t)g * 64 + k + 32 * h) * 4;
                v[0] = xpack(em0 & 0xFFFFu, ep0 & 0xFFFFu);
                v[1] = xpack(em0 >> 16, ep0 >> 16);
                v[2] = xpack(em1 & 0xFFFFu, ep1 & 0xFFFFu);
                v[3] = xpack(em1 >> 16, ep1 >> 16);
            }
    }
}

}  // namespace iris

// ------------------------------------------------------------------ parallel host copies

#include <algorithm>
#include <atomic>
#include <condition_variable>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include <errno.h>
#include <immintrin.h>
#include <unistd.h>

namespace iris {

namespace {

// Packed MasksEngine rows (store_tile_packed): bytes 0..30 of a record are row[k] - 64 B, byte 31
// is B, or 0xFF for a row stored in full in the escape rows.  Records go in increasing order, and
// each is written as one 64-B store whose last 2 bytes the next record's store overwrites; the
// last record of a range is written exactly (its successor may belong to another thread).
__attribute__((target("avx512bw,avx512vl"))) inline void expand_one(uint16_t *o, const uint8_t *p, const uint16_t *e,
                                                                     bool exact) {
    const uint32_t b = p[31];
    if (b == 0xFFu) {
        memcpy(o, e, kRot * 2);
        return;
    }
    const __m512i w = _mm512_add_epi16(_mm512_cvtepu8_epi16(_mm256_loadu_si256((const __m256i *)p)),
                                       _mm512_set1_epi16((short)(b << 6)));
    if (exact)
        _mm512_mask_storeu_epi16(o, 0x7FFFFFFFu, w);
    else
        _mm512_storeu_si512((void *)o, w);
}

__attribute__((target("avx512bw,avx512vl"))) void expand_plain(uint16_t *out, const uint8_t *pk, const uint16_t *esc,
                                                                 size_t n) {
    for (size_t i = 0; i < n; ++i) expand_one(out + kRot * i, pk + 32 * i, esc + kRot * i, i + 1 == n);
}

// 32 records are 1984 B = 31 cache lines, so from the first record that starts on a 64-B boundary
// the rows go out in blocks of 32: expanded into an L1 staging block, then written with 31
// non-temporal 64-B stores -- the caller's array is not read for ownership first (a store
// that misses the cache reads its line before writing it): 1.55x the plain stores' rate into an
// array beyond the caches on this container's host (profiles/r06_expand_nt.txt).
__attribute__((target("avx512bw,avx512vl"))) void expand_avx512(uint16_t *out, const uint8_t *pk, const uint16_t *esc,
                                                                  size_t n) {
    size_t i = 0;
    while (i < n && ((uintptr_t)(out + kRot * i) & 63)) ++i;
    if (i + 32 > n) {
        expand_plain(out, pk, esc, n);
        return;
    }
    expand_plain(out, pk, esc, i);
    alignas(64) uint16_t st[32 * kRot + 32];
    for (; i + 32 <= n; i += 32) {
        for (int r = 0; r < 32; ++r) expand_one(st + kRot * r, pk + 32 * (i + r), esc + kRot * (i + r), false);
        __m512i *d = (__m512i *)(out + kRot * i);
        for (int l = 0; l < kRot; ++l) _mm512_stream_si512(d + l, _mm512_load_si512((const __m512i *)st + l));
    }
    expand_plain(out + kRot * i, pk + 32 * i, esc + kRot * i, n - i);
    _mm_sfence();  // the streamed lines are globally visible before this thread reports its part done
}

// A copy whose destination lines are written with non-temporal 64-B stores (from the first 64-B
// boundary of dst on; the source may have any alignment): the caller's array is not read for
// ownership first, as plain stores into lines that miss the caches do (the packed rows' expansion
// measured 1.0 against 1.9 ns per 62-B row, profiles/r06b_expand_nt_epyc.txt).
__attribute__((target("avx512f"))) void copy_nt_avx512(char *dst, const char *src, size_t n) {
    const size_t head = std::min<size_t>(n, (64 - ((uintptr_t)dst & 63)) & 63);
    memcpy(dst, src, head);
    dst += head;
    src += head;
    n -= head;
    size_t i = 0;
    for (; i + 256 <= n; i += 256) {
        const __m512i a = _mm512_loadu_si512(src + i), b = _mm512_loadu_si512(src + i + 64),
                      c = _mm512_loadu_si512(src + i + 128), d = _mm512_loadu_si512(src + i + 192);
        _mm512_stream_si512((__m512i *)(dst + i), a);
        _mm512_stream_si512((__m512i *)(dst + i + 64), b);
        _mm512_stream_si512((__m512i *)(dst + i + 128), c);
        _mm512_stream_si512((__m512i *)(dst + i + 192), d);
    }
    for (; i + 64 <= n; i += 64) _mm512_stream_si512((__m512i *)(dst + i), _mm512_loadu_si512(src + i));
    memcpy(dst + i, src + i, n - i);
    _mm_sfence();  // the streamed lines are globally visible before this thread reports its part done
}

// dst[i] = src[0][i] + ... + src[k-1][i] (mod 2^16), dst written with non-temporal 64-B stores from its
// first 64-B boundary on (the sources may have any alignment)
__attribute__((target("avx512bw"))) void sum_u16_avx512(uint16_t *dst, const uint16_t *const *src, int k, size_t n) {
    auto scalar = [&](size_t a, size_t b) {
        for (size_t i = a; i < b; ++i) {
            uint16_t v = src[0][i];
            for (int j = 1; j < k; ++j) v = (uint16_t)(v + src[j][i]);
            dst[i] = v;
        }
    };
    size_t i = std::min<size_t>(n, ((64 - ((uintptr_t)dst & 63)) & 63) / 2);
    if ((uintptr_t)dst & 1) i = n;  // not even u16-aligned: no vector stores
    scalar(0, i);
    for (; i + 32 <= n; i += 32) {
        __m512i v = _mm512_loadu_si512(src[0] + i);
        for (int j = 1; j < k; ++j) v = _mm512_add_epi16(v, _mm512_loadu_si512(src[j] + i));
        _mm512_stream_si512((__m512i *)(dst + i), v);
    }
    scalar(i, n);
    _mm_sfence();
}

void expand_scalar(uint16_t *out, const uint8_t *pk, const uint16_t *esc, size_t n) {
    for (size_t i = 0; i < n; ++i) {
        const uint8_t *p = pk + 32 * i;
        uint16_t *o = out + kRot * i;
        if (p[31] == 0xFFu) {
            memcpy(o, esc + kRot * i, kRot * 2);
            continue;
        }
        const uint16_t base = (uint16_t)(p[31] << 6);
        for (int k = 0; k < kRot; ++k) o[k] = (uint16_t)(base + p[k]);
    }
}

const bool kHaveAvx512 = __builtin_cpu_supports("avx512bw") && __builtin_cpu_supports("avx512vl");

// Helper threads (one pool per device) for copying an engine call's rows out of pinned memory
// into the caller's buffer (read-ahead, iris_api.hip) and a large write's records into the pinned
// upload slots: one core reads ~25 GB/s from DRAM, so a 1.24-MB participant-sized chunk costs
// ~45 us on one thread.  A job is split into twice as many parts as there are threads, and parts
// are claimed from one atomic word (the job's number in the high half, the next part in the low
// half): the caller works through them too, so a helper that is still asleep when a job starts (the
// first call of a walk after a pause) costs a share of the work, not its wake-up latency.  The
// helpers spin for a while after each job (calls of a chunk walk arrive every few tens of us) and
// then block.
}  // namespace

void copy_nt(char *dst, const char *src, size_t n) {
    if (kHaveAvx512 && n >= 4096)
        copy_nt_avx512(dst, src, n);
    else
        memcpy(dst, src, n);
}

void sum_u16(uint16_t *dst, const uint16_t *const *src, int k, size_t n) {
    if (kHaveAvx512) {
        sum_u16_avx512(dst, src, k, n);
        return;
    }
    for (size_t i = 0; i < n; ++i) {
        uint16_t v = src[0][i];
        for (int j = 1; j < k; ++j) v = (uint16_t)(v + src[j][i]);
        dst[i] = v;
    }
}

namespace {

class CopyPool {
   public:
    explicit CopyPool(int helpers) : pid_(getpid()), nthreads_(helpers + 1), nparts_(2 * nthreads_) {
        for (int i = 0; i < helpers; ++i) threads_.emplace_back([this] { worker(); });
        for (auto &t : threads_) t.detach();  // never joined: the pool lives as long as the process
    }
    pid_t pid() const { return pid_; }

    // src != nullptr: memcpy; else pread from fd at file offset off.  Returns false if a read failed
    // (an I/O error, or the file ended before `bytes`).  esc != nullptr: expand `bytes` packed
    // MasksEngine records at src (escape rows at esc) into dst instead.
    // sums != nullptr: dst = the wrapping u16 sum of nsum arrays of `bytes` elements (sum_u16)
    bool run(char *dst, const char *src, size_t bytes, int fd = -1, off_t off = 0, const uint16_t *esc = nullptr,
             const uint16_t *const *sums = nullptr, int nsum = 0) {
        std::lock_guard<std::mutex> one(run_mu_);  // one job at a time (devices may call concurrently)
        dst_ = dst;
        src_ = src;
        esc_ = esc;
        nsum_ = sums ? nsum : 0;
        for (int j = 0; j < nsum_; ++j) sums_[j] = sums[j];
        bytes_ = bytes;
        fd_ = fd;
        off_ = off;
        ok_.store(true, std::memory_order_relaxed);
        done_.store(0, std::memory_order_relaxed);
        const uint64_t job = ++job_;
        claim_.store(job << 32, std::memory_order_release);  // publishes the fields above
        {
            std::lock_guard<std::mutex> l(mu_);
            gen_.store(job, std::memory_order_release);
        }
        cv_.notify_all();
        work(job);
        while (done_.load(std::memory_order_acquire) != nparts_) __builtin_ia32_pause();
        return ok_.load(std::memory_order_acquire);
    }

   private:
    // claims and runs parts of job `job` until none is left (or a newer job has replaced it)
    void work(uint64_t job) {
        for (;;) {
            uint64_t v = claim_.load(std::memory_order_acquire);
            int k;
            do {
                if ((v >> 32) != (job & 0xFFFFFFFFu) || (int)(v & 0xFFFFFFFFu) >= nparts_) return;
                k = (int)(v & 0xFFFFFFFFu);
            } while (!claim_.compare_exchange_weak(v, v + 1, std::memory_order_acq_rel, std::memory_order_acquire));
            part(k);
            done_.fetch_add(1, std::memory_order_release);
        }
    }
    void part(int id) {
        const int np = nparts_;
        if (nsum_) {  // bytes_ u16 elements, parts of whole 64-B runs
            const size_t per = ((bytes_ + np - 1) / np + 31) & ~(size_t)31;
            const size_t a = std::min(bytes_, (size_t)id * per), b = std::min(bytes_, a + per);
            if (a < b) {
                const uint16_t *srcs[kMaxSum];
                for (int j = 0; j < nsum_; ++j) srcs[j] = sums_[j] + a;
                sum_u16((uint16_t *)dst_ + a, srcs, nsum_, b - a);
            }
            return;
        }
        if (esc_) {  // bytes_ records, split on record boundaries
            const size_t per = (bytes_ + np - 1) / np;
            const size_t a = std::min(bytes_, (size_t)id * per), b = std::min(bytes_, a + per);
            if (a < b) expand_packed_rows((uint16_t *)dst_ + kRot * a, (const uint8_t *)src_ + 32 * a, esc_ + kRot * a, b - a);
            return;
        }
        const size_t per = ((bytes_ + np - 1) / np + 63) & ~(size_t)63;
        const size_t a = std::min(bytes_, (size_t)id * per), b = std::min(bytes_, a + per);
        if (a >= b) return;
        if (src_) {
            copy_nt(dst_ + a, src_ + a, b - a);
            return;
        }
        for (size_t done = a; done < b;) {
            const ssize_t r = ::pread(fd_, dst_ + done, b - done, off_ + (off_t)done);
            if (r < 0 && errno == EINTR) continue;
            if (r <= 0) {
                ok_.store(false, std::memory_order_relaxed);
                return;
            }
            done += (size_t)r;
        }
    }
    void worker() {
        uint64_t seen = 0;
        for (;;) {
            uint64_t g;
            for (int spins = 0; (g = gen_.load(std::memory_order_acquire)) == seen;) {
                if (++spins < (1 << 16)) {
                    __builtin_ia32_pause();
                } else {
                    std::unique_lock<std::mutex> l(mu_);
                    cv_.wait(l, [&] { return gen_.load(std::memory_order_acquire) != seen; });
                    spins = 0;
                }
            }
            seen = g;
            work(g);
        }
    }
    pid_t pid_;
    const int nthreads_;  // helpers + the caller
    std::vector<std::thread> threads_;
    std::mutex run_mu_, mu_;
    std::condition_variable cv_;
    std::atomic<uint64_t> gen_{0};    // the newest job's number (wakes the helpers)
    std::atomic<uint64_t> claim_{0};  // (job number << 32) | next unclaimed part
    std::atomic<int> done_{0};        // parts of the current job finished
    uint64_t job_ = 0;
    const int nparts_;    // parts per job (fixed: a late helper reads it unsynchronised)
    char *dst_ = nullptr;
    const char *src_ = nullptr;
    const uint16_t *esc_ = nullptr;
    static constexpr int kMaxSum = 8;
    const uint16_t *sums_[kMaxSum] = {};
    int nsum_ = 0;
    size_t bytes_ = 0;
    int fd_ = -1;
    off_t off_ = 0;
    std::atomic<bool> ok_{true};
};

constexpr size_t kParallelCopyMin = 256 << 10;

// Helper threads per device pool (3: with the caller, 4 parts).  7 were measured on the boxes'
// 16-CPU quota for a 3M-mask walk's copy-out and gave no reliable gain: 1.24 / 1.09 / 0.95e9
// records/s against 1.12 / 1.17 / 1.11e9 with 3, alternating on one box and across boxes
// (profiles/r06k_helpers_ab.txt).  IRIS_COPY_HELPERS (0..15) overrides; read when the pool is created.
constexpr int kCopyHelpers = 3;

int copy_helpers() {
    const char *e = getenv("IRIS_COPY_HELPERS");
    if (!e || !*e) return kCopyHelpers;
    const int v = atoi(e);
    return v < 0 ? 0 : v > 15 ? 15 : v;
}

}  // namespace

// ---------------------------------------------------------------- runtime configuration

namespace {

// Test-only hooks in the order of Hooks::ignored's bits.
constexpr const char *kHookNames[] = {"IRIS_TILES_PER_WAVE",  "IRIS_FUSED_REDUCE", "IRIS_BATCH_KERNEL",
                                      "IRIS_SCHEDULE",        "IRIS_LOAD_PREAD",   "IRIS_GROUP_DELAY_US",
                                      "IRIS_GROUP_STALL",     "IRIS_GROUP_UNORDERED", "IRIS_UPLOAD",
                                      "IRIS_LOAD_WINDOWS",    "IRIS_READAHEAD_WINDOW", "IRIS_RESIDENT_BUDGET_MB",
                                      "IRIS_READAHEAD_PACKED", "IRIS_READAHEAD_WINDOW_MAX"};
constexpr int kNumHooks = (int)(sizeof(kHookNames) / sizeof(kHookNames[0]));

const char *env(const char *name) {
    const char *v = getenv(name);
    return v && *v ? v : nullptr;
}

uint32_t env_u32(const char *v, uint32_t max) {
    const long long x = atoll(v);
    return x < 0 ? 0u : x > (long long)max ? max : (uint32_t)x;
}

}  // namespace

void read_hooks(Hooks *h) {
    *h = Hooks{};
    if (const char *v = env("IRIS_READAHEAD")) h->readahead = v[0] != '0';
    if (const char *v = env("IRIS_AUTO_RESIDENT")) h->auto_resident = v[0] != '0';
    if (const char *v = env("IRIS_GROUP_TIMEOUT_MS")) h->group_timeout_ms = env_u32(v, 24u * 3600 * 1000);
    if (const char *v = env("IRIS_RESIDENT_MAX_MB")) h->resident_max_mb = env_u32(v, 1u << 30);
    const char *t = env("IRIS_TEST_HOOKS");
    h->test = t && t[0] == '1';
    for (int i = 0; i < kNumHooks; ++i) {
        const char *v = env(kHookNames[i]);
        if (!v) continue;
        if (!h->test) {
            h->ignored |= 1u << i;
            continue;
        }
        switch (i) {
        case 0: h->tiles_per_wave = atoi(v) == 1 ? 1 : 4; break;
        case 1: h->fused_reduce = v[0] != '0'; break;
        case 2: h->batch_kernel = atoi(v) == 2 ? 2 : 4; break;
        case 3: h->schedule = !strcmp(v, "spin") ? 1 : !strcmp(v, "yield") ? 2 : !strcmp(v, "blocking") ? 3 : 0; break;
        case 4: h->load_pread = v[0] != '0'; break;
        case 5: h->group_delay_us = env_u32(v, 1000000); break;
        case 6: h->group_stall = v[0] != '0'; break;
        case 7: h->group_unordered = v[0] != '0'; break;
        case 8: h->upload = !strcmp(v, "pinned") ? 1 : !strcmp(v, "runtime") ? 2 : 0; break;
        case 9: h->load_windows = v[0] != '0'; break;
        case 10: h->ra_window = env_u32(v, 64); break;
        case 11: h->resident_budget_mb = env_u32(v, 1u << 30); break;
        case 12: h->ra_packed = v[0] != '0'; break;
        case 13: h->ra_window_max = env_u32(v, 1024); break;
        }
    }
}

size_t format_hooks(const Hooks &h, char *buf, size_t len) {
    static const char *sched[] = {"auto", "spin", "yield", "blocking"};
    static const char *upload_names[] = {"auto", "pinned", "runtime", "auto"};
    std::string s = "readahead=" + std::to_string(h.readahead) + " auto_resident=" + std::to_string(h.auto_resident) +
                    " group_timeout_ms=" +
                    (h.group_timeout_ms ? std::to_string(h.group_timeout_ms) : std::string("auto")) +
                    " group_init_timeout_ms=" +
                    std::to_string(h.group_timeout_ms ? h.group_timeout_ms : kGroupInitTimeoutMs) +
                    " resident_max_mb=" + (h.resident_max_mb ? std::to_string(h.resident_max_mb) : std::string("auto")) +
                    " copy_helpers=" + std::to_string(copy_helpers()) + " test_hooks=" + std::to_string(h.test);
    if (h.test)
        s += " tiles_per_wave=" + (h.tiles_per_wave ? std::to_string(h.tiles_per_wave) : std::string("auto")) +
             " fused_reduce=" + std::to_string(h.fused_reduce) + " batch_kernel=" + std::to_string(h.batch_kernel) +
             " schedule=" + sched[h.schedule & 3] +
             " load_pread=" + std::to_string(h.load_pread) +
             " load_windows=" + std::to_string(h.load_windows) + " readahead_window=" + std::to_string(h.ra_window) +
             " resident_budget_mb=" + std::to_string(h.resident_budget_mb) +
             " readahead_packed=" + std::to_string(h.ra_packed) +
             " readahead_window_max=" + std::to_string(h.ra_window_max) +
             " group_delay_us=" + std::to_string(h.group_delay_us) +
             " group_stall=" + std::to_string(h.group_stall) + " group_unordered=" + std::to_string(h.group_unordered) +
             " upload=" + upload_names[h.upload & 3];
    std::string ign;
    for (int i = 0; i < kNumHooks; ++i)
        if (h.ignored >> i & 1u) ign += (ign.empty() ? "" : ",") + std::string(kHookNames[i]);
    if (!ign.empty()) s += " ignored=" + ign;
    if (buf && len) {
        const size_t n = std::min(len - 1, s.size());
        memcpy(buf, s.data(), n);
        buf[n] = 0;
    }
    return s.size();
}

namespace {

// one pool per device (lane = ordinal): devices driven from their own threads (a device group's
// loads, concurrent host-slice calls) copy in parallel instead of queueing on one pool
CopyPool *pool_of(int lane) {
    constexpr int kLanes = 16;
    static std::mutex create_mu;
    static CopyPool *pools[kLanes] = {};  // leaked on purpose (detached helpers)
    const int l = ((lane % kLanes) + kLanes) % kLanes;
    std::lock_guard<std::mutex> g(create_mu);
    if (!pools[l] || pools[l]->pid() != getpid()) pools[l] = new CopyPool(copy_helpers());  // a forked child gets its own
    return pools[l];
}

}  // namespace

void parallel_copy(void *dst, const void *src, size_t bytes, int lane) {
    if (bytes < kParallelCopyMin) {
        memcpy(dst, src, bytes);
        return;
    }
    (void)pool_of(lane)->run((char *)dst, (const char *)src, bytes);
}

bool parallel_pread(int fd, void *dst, size_t bytes, off_t off, int lane) {
    return pool_of(lane)->run((char *)dst, nullptr, bytes, fd, off);
}

void expand_packed_rows(uint16_t *out, const uint8_t *pk, const uint16_t *esc, size_t n) {
    if (kHaveAvx512)
        expand_avx512(out, pk, esc, n);
    else
        expand_scalar(out, pk, esc, n);
}

void parallel_sum_u16(uint16_t *dst, const uint16_t *const *src, int k, size_t n, int lane) {
    if (k < 1 || k > 8) return;
    if (n * 2 * (size_t)k < kParallelCopyMin) {
        sum_u16(dst, src, k, n);
        return;
    }
    (void)pool_of(lane)->run((char *)dst, nullptr, n, -1, 0, nullptr, src, k);
}

void parallel_expand(uint16_t *out, const uint8_t *pk, const uint16_t *esc, size_t n, int lane) {
    if (n * kRot * 2 < kParallelCopyMin) {
        expand_packed_rows(out, pk, esc, n);
        return;
    }
    (void)pool_of(lane)->run((char *)out, (const char *)pk, n, -1, 0, esc);
}

}  // namespace iris
