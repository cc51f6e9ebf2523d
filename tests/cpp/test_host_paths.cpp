// The library's host-side copy-out paths, on the CPU (no GPU needed): the expansion of packed
// MasksEngine rows (store_tile_packed's format, csrc/iris_device.hpp; csrc/iris_host.cpp
// expand_packed_rows / parallel_expand: the AVX-512 form with its non-temporal 32-record blocks,
// escaped rows, every alignment of the caller's array) against a scalar restatement, and the
// helper pool's parallel_copy under concurrent callers (parts claimed by whoever is free), and
// copy_nt (non-temporal stores from dst's first 64-B boundary) at every source / destination offset,
// and sum_u16 / parallel_sum_u16 (the resolver's wrapping share sums) against a scalar sum.
// These are library internals, declared here as the library defines them (iris_internal.hpp).
#include <atomic>
#include <cstdio>
#include <cstring>
#include <random>
#include <thread>
#include <vector>

namespace iris {
void parallel_copy(void *dst, const void *src, size_t bytes, int lane);
void parallel_expand(uint16_t *out, const uint8_t *pk, const uint16_t *esc, size_t n, int lane);
void expand_packed_rows(uint16_t *out, const uint8_t *pk, const uint16_t *esc, size_t n);
void copy_nt(char *dst, const char *src, size_t n);
void sum_u16(uint16_t *dst, const uint16_t *const *src, int k, size_t n);
void parallel_sum_u16(uint16_t *dst, const uint16_t *const *src, int k, size_t n, int lane);
}  // namespace iris

static int failures = 0;
#define CHECK(c)                                                              \
    do {                                                                      \
        if (!(c)) {                                                           \
            std::fprintf(stderr, "CHECK failed %s:%d: %s\n", __FILE__, __LINE__, #c); \
            ++failures;                                                       \
        }                                                                     \
    } while (0)

// n packed records (32 B) and their escape rows; `want` the [n][31] rows they stand for
static void make_packed(std::mt19937_64 &r, size_t n, std::vector<uint8_t> &pk, std::vector<uint16_t> &esc,
                        std::vector<uint16_t> &want) {
    pk.assign(n * 32, 0);
    esc.assign(n * 31, 0);
    want.assign(n * 31, 0);
    for (size_t i = 0; i < n; ++i) {
        uint16_t *w = &want[i * 31];
        if (r() % 5 == 0) {  // an escaped row: counts spanning more than a byte
            for (int k = 0; k < 31; ++k) w[k] = esc[i * 31 + k] = (uint16_t)(r() % 12801);
            pk[i * 32 + 31] = 0xFF;
            continue;
        }
        const uint32_t b = (uint32_t)(r() % 201);  // B = min >> 6
        for (int k = 0; k < 31; ++k) {
            const uint32_t d = (uint32_t)(r() % 256);
            pk[i * 32 + k] = (uint8_t)d;
            w[k] = (uint16_t)((b << 6) + d);
        }
        pk[i * 32 + 31] = (uint8_t)b;
    }
}

int main() {
    std::mt19937_64 r(7);
    // every alignment of the destination (u16 steps across a 64-B line), many lengths
    for (size_t n : {0, 1, 2, 31, 32, 33, 63, 64, 65, 100, 257, 1000}) {
        std::vector<uint8_t> pk;
        std::vector<uint16_t> esc, want;
        make_packed(r, n, pk, esc, want);
        for (int shift = 0; shift < 32; ++shift) {
            std::vector<uint16_t> buf(n * 31 + 64 + 32, 0xABCD);
            uint16_t *out = buf.data() + shift;
            iris::expand_packed_rows(out, pk.data(), esc.data(), n);
            CHECK(std::memcmp(out, want.data(), n * 31 * 2) == 0);
            // nothing written past the last row
            for (size_t j = shift + n * 31; j < buf.size(); ++j) CHECK(buf[j] == 0xABCD);
            for (int j = 0; j < shift; ++j) CHECK(buf[j] == 0xABCD);
        }
    }
    // copy_nt: every destination and source offset within a line, lengths around its 4-KB threshold,
    // the 256-B unrolled body and the 64-B tail; nothing outside [dst, dst + n) is written
    {
        std::vector<char> src(70000 + 128);
        for (auto &c : src) c = (char)r();
        for (size_t n : {0, 1, 63, 64, 65, 4095, 4096, 4097, 4096 + 255, 4096 + 256 + 63, 65536 + 17}) {
            for (int so = 0; so < 64; so += 7) {
                for (int dof = 0; dof < 64; ++dof) {
                    std::vector<char> buf(n + 192, (char)0x5A);
                    char *dst = buf.data() + 64 + dof - ((uintptr_t)(buf.data() + 64) & 63);
                    iris::copy_nt(dst, src.data() + so, n);
                    CHECK(std::memcmp(dst, src.data() + so, n) == 0);
                    for (char *q = buf.data(); q < dst; ++q) CHECK(*q == (char)0x5A);
                    for (char *q = dst + n; q < buf.data() + buf.size(); ++q) CHECK(*q == (char)0x5A);
                }
            }
        }
    }
    // sum_u16: 1..8 sources at assorted offsets, every u16 offset of the destination within a line
    {
        const size_t maxn = 5000;
        std::vector<std::vector<uint16_t>> srcv(8, std::vector<uint16_t>(maxn + 64));
        for (auto &v : srcv)
            for (auto &x : v) x = (uint16_t)r();
        for (int k = 1; k <= 8; ++k)
            for (size_t n : {0, 1, 31, 32, 33, 95, 1000, 4999}) {
                const uint16_t *src[8];
                for (int j = 0; j < k; ++j) src[j] = srcv[j].data() + (j * 7) % 40;
                std::vector<uint16_t> want(n);
                for (size_t i = 0; i < n; ++i) {
                    uint32_t v = 0;
                    for (int j = 0; j < k; ++j) v += src[j][i];
                    want[i] = (uint16_t)v;
                }
                for (int dof = 0; dof < 32; dof += 3) {
                    std::vector<uint16_t> buf(n + 96, 0x7777);
                    uint16_t *dst = buf.data() + 32 + dof - (((uintptr_t)(buf.data() + 32) & 63) / 2);
                    iris::sum_u16(dst, src, k, n);
                    CHECK(std::memcmp(dst, want.data(), n * 2) == 0);
                    for (uint16_t *q = buf.data(); q < dst; ++q) CHECK(*q == 0x7777);
                    for (uint16_t *q = dst + n; q < buf.data() + buf.size(); ++q) CHECK(*q == 0x7777);
                }
            }
    }
    // the helper pool: a participant-sized chunk (20 000 records) and a window, from 4 threads at once
    {
        std::vector<std::thread> ts;
        std::atomic<int> bad{0};
        for (int t = 0; t < 4; ++t)
            ts.emplace_back([t, &bad] {
                std::mt19937_64 rr(100 + t);
                for (int it = 0; it < 20; ++it) {
                    const size_t n = it % 2 ? 20000 : 1 + rr() % 60000;
                    std::vector<uint8_t> pk;
                    std::vector<uint16_t> esc, want;
                    make_packed(rr, n, pk, esc, want);
                    std::vector<uint16_t> out(n * 31 + 3, 0x5555);
                    iris::parallel_expand(out.data() + (it % 3), pk.data(), esc.data(), n, t % 2);
                    if (std::memcmp(out.data() + (it % 3), want.data(), n * 31 * 2) != 0) ++bad;
                    std::vector<char> a(1 + rr() % (3 << 20)), b(a.size(), 0);
                    for (auto &c : a) c = (char)rr();
                    iris::parallel_copy(b.data(), a.data(), a.size(), t % 2);
                    if (a != b) ++bad;
                    // three share arrays of a chunk summed by the pool (the resolver's host form)
                    const size_t ne = 1 + rr() % (2 << 20);
                    std::vector<uint16_t> s0(ne), s1(ne), s2(ne), sum(ne + 1, 0);
                    for (size_t i = 0; i < ne; ++i) s0[i] = (uint16_t)rr(), s1[i] = (uint16_t)rr(), s2[i] = (uint16_t)rr();
                    const uint16_t *ss[3] = {s0.data(), s1.data(), s2.data()};
                    iris::parallel_sum_u16(sum.data() + (it % 2), ss, 3, ne, t % 2);
                    for (size_t i = 0; i < ne; ++i)
                        if (sum[i + (it % 2)] != (uint16_t)(s0[i] + s1[i] + s2[i])) {
                            ++bad;
                            break;
                        }
                }
            });
        for (auto &t : ts) t.join();
        CHECK(bad.load() == 0);
    }
    std::printf("host paths: %d failures\n", failures);
    return failures ? 1 : 0;
}
