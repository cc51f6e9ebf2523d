// iris_prepare.hip — secret-share preparation on the device (SURVEY.md §8(f)
// row 4): the reference's `prepare` (src/main.rs:333-361) turns every
// Template into a `.masks` record (its mask) and `count` additive shares of
// encode(template) (EncodedBits::share, src/encoded_bits.rs:23-38): count-1
// uniformly random EncodedBits and a last share = encode - sum(rest), mod 2^16.
//
// Randomness: ChaCha (D. J. Bernstein's original: 64-bit nonce, 64-bit block
// counter) with 8, 12 or 20 rounds, keyed by the caller's 256-bit key, in
// counter mode, so every (template, share, 64-byte block) is an independent
// thread of work:
//   block counter = (g * (parties-1) + j) * 400 + b   (g = global template index)
//   share j, elements 32b .. 32b+31 = the block's 32 little-endian u16.
// The reference draws from rand 0.8.5's thread_rng (src/encoded_bits.rs:27),
// whose core is rand_chacha 0.3.1's ChaCha12 (same block function, 12 rounds;
// Cargo.lock) reseeded from the OS; the default here is therefore 12 rounds.
// Its stream is unseeded and not reproducible, so parity here is against the
// oracle's restatement of this derivation (oracle/iris_oracle.c, pinned by the
// RFC 8439 ChaCha20 vectors and the published ChaCha8/12 zero-key vectors)
// plus the share-sum identity.
//
// One thread per (template, block b): element block b of encode(t) needs
// pattern and mask dword b only (element i = bit i, LE limbs), so the thread
// computes parties-1 keystream blocks, writes them as 64-byte rows of shares
// 0..parties-2, and the last share's row as encode minus their sum.
#include <hip/hip_runtime.h>

#include "iris_device.hpp"

namespace iris {

struct ChachaKey {
    uint32_t k[8];
};

__device__ __forceinline__ uint32_t rotl(uint32_t x, int r) { return __builtin_rotateleft32(x, r); }

#define CC_QR(a, b, c, d)   \
    a += b;                 \
    d = rotl(d ^ a, 16);    \
    c += d;                 \
    b = rotl(b ^ c, 12);    \
    a += b;                 \
    d = rotl(d ^ a, 8);     \
    c += d;                 \
    b = rotl(b ^ c, 7);

// DR double rounds: 4 = ChaCha8, 6 = ChaCha12, 10 = ChaCha20
template <int DR>
__device__ __forceinline__ void chacha_block(const ChachaKey &key, uint64_t nonce, uint64_t counter,
                                             uint32_t out[16]) {
    const uint32_t in[16] = {0x61707865u, 0x3320646eu, 0x79622d32u, 0x6b206574u, key.k[0], key.k[1],
                             key.k[2],    key.k[3],    key.k[4],    key.k[5],    key.k[6], key.k[7],
                             (uint32_t)counter, (uint32_t)(counter >> 32), (uint32_t)nonce,
                             (uint32_t)(nonce >> 32)};
    uint32_t x[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) x[i] = in[i];
#pragma unroll 2
    for (int r = 0; r < DR; ++r) {
        CC_QR(x[0], x[4], x[8], x[12]);
        CC_QR(x[1], x[5], x[9], x[13]);
        CC_QR(x[2], x[6], x[10], x[14]);
        CC_QR(x[3], x[7], x[11], x[15]);
        CC_QR(x[0], x[5], x[10], x[15]);
        CC_QR(x[1], x[6], x[11], x[12]);
        CC_QR(x[2], x[7], x[8], x[13]);
        CC_QR(x[3], x[4], x[9], x[14]);
    }
#pragma unroll
    for (int i = 0; i < 16; ++i) out[i] = x[i] + in[i];
}

constexpr int kBlocks = IRIS_BITS / 32;  // 400 keystream blocks per share

// two independent u16 lanes: (a - b) mod 2^16 per half (v_pk_sub_u16)
__device__ __forceinline__ uint32_t pk_sub_u16(uint32_t a, uint32_t b) {
    typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));
    const u16x2 r = __builtin_bit_cast(u16x2, a) - __builtin_bit_cast(u16x2, b);
    return __builtin_bit_cast(uint32_t, r);
}

// templates: m reference-layout records (pattern dwords 0..399, mask 400..799)
// shares: [parties][m][12800] u16
template <int DR>
__global__ void __launch_bounds__(256) prepare_shares_kernel(const uint32_t *__restrict__ templates, uint64_t m,
                                                             uint64_t g0, ChachaKey key, uint64_t nonce,
                                                             uint32_t parties, uint16_t *__restrict__ shares) {
    const uint64_t total = m * kBlocks;
    for (uint64_t tid = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; tid < total;
         tid += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t i = tid / kBlocks;
        const int b = (int)(tid - i * kBlocks);
        const uint32_t pw = templates[i * (2 * kPlaneDwords) + b];
        const uint32_t mw = templates[i * (2 * kPlaneDwords) + kPlaneDwords + b];
        // last[e] accumulates encode - sum, two u16 lanes per dword (independent mod 2^16 halves)
        uint32_t last[16];
#pragma unroll
        for (int w = 0; w < 16; ++w) {
            const uint32_t m0 = (mw >> (2 * w)) & 1u, m1 = (mw >> (2 * w + 1)) & 1u;
            const uint32_t p0 = (pw >> (2 * w)) & 1u, p1 = (pw >> (2 * w + 1)) & 1u;
            const uint32_t e0 = (m0 - 2u * (p0 & m0)) & 0xFFFFu, e1 = (m1 - 2u * (p1 & m1)) & 0xFFFFu;
            last[w] = e0 | (e1 << 16);
        }
        const uint64_t g = g0 + i;
        for (uint32_t j = 0; j + 1 < parties; ++j) {
            uint32_t r[16];
            chacha_block<DR>(key, nonce, (g * (parties - 1) + j) * kBlocks + (uint64_t)b, r);
            uint4 *dst = (uint4 *)(shares + ((uint64_t)j * m + i) * IRIS_BITS + 32 * b);
#pragma unroll
            for (int q = 0; q < 4; ++q) dst[q] = make_uint4(r[4 * q], r[4 * q + 1], r[4 * q + 2], r[4 * q + 3]);
#pragma unroll
            for (int w = 0; w < 16; ++w) last[w] = pk_sub_u16(last[w], r[w]);
        }
        uint4 *dst = (uint4 *)(shares + ((uint64_t)(parties - 1) * m + i) * IRIS_BITS + 32 * b);
#pragma unroll
        for (int q = 0; q < 4; ++q)
            dst[q] = make_uint4(last[4 * q], last[4 * q + 1], last[4 * q + 2], last[4 * q + 3]);
    }
}

// Direct form for TILES share databases: a workgroup takes 64 consecutive
// templates (lane = template) and its 4 waves split the 400 blocks, so each
// (share, block) store of a wave is two 512-B runs of the TILES byte planes
// (split_bytes) and the template dwords come through L1 (a 64 x 128-B window).
// No staging copy of the shares: they are written once, in place.
struct ShareDsts {
    uint4 *db[kMaxPrepParties];
    uint64_t t_first[kMaxPrepParties];  // database index of template 0 of the launch
};

// Share rows leave with nontemporal stores: 19.4 vs 20.2 ms per 1M templates (ChaCha12, 3
// parties, interleaved runs on one box).  Loading the next block's template pair ahead of
// the stores (vmcnt counts stores too on gfx9) measured no change; write-through policies
// (sc1, sc0 sc1, nt sc1) were 0.5-2 % slower than nt.
__device__ __forceinline__ void st_share(uint4 *p, const uint4 v) {
    const u32x4_nt w = {v.x, v.y, v.z, v.w};
    __builtin_nontemporal_store(w, (u32x4_nt *)p);
}

__device__ __forceinline__ void store_share_block(uint4 *db, uint64_t t, int b, const uint32_t w[16]) {
    uint4 *base = db + (t / 32) * (uint64_t)kShareTileUint4 + (t % 32);
    uint4 lo, hi;
    split_bytes(w, lo, hi);  // elements 32b .. 32b+15: half 0
    st_share(base + (2 * b) * 64, lo);
    st_share(base + (2 * b + 1) * 64, hi);
    split_bytes(w + 8, lo, hi);  // elements 32b+16 .. 32b+31: half 1
    st_share(base + (2 * b) * 64 + 32, lo);
    st_share(base + (2 * b + 1) * 64 + 32, hi);
}

template <int DR>
__global__ void __launch_bounds__(256) prepare_shares_tiles_kernel(const uint32_t *__restrict__ templates, uint64_t m,
                                                                   uint64_t g0, ChachaKey key, uint64_t nonce,
                                                                   uint32_t parties, ShareDsts dst) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const uint64_t i = (uint64_t)blockIdx.x * 64 + lane;
    if (i >= m) return;
    const uint32_t *rec = templates + i * (2 * kPlaneDwords);
    const uint64_t g = g0 + i;
    for (int b = w; b < kBlocks; b += 4) {
        const uint32_t pw = rec[b], mw = rec[kPlaneDwords + b];
        uint32_t last[16];
#pragma unroll
        for (int q = 0; q < 16; ++q) {
            const uint32_t m0 = (mw >> (2 * q)) & 1u, m1 = (mw >> (2 * q + 1)) & 1u;
            const uint32_t p0 = (pw >> (2 * q)) & 1u, p1 = (pw >> (2 * q + 1)) & 1u;
            last[q] = ((m0 - 2u * (p0 & m0)) & 0xFFFFu) | (((m1 - 2u * (p1 & m1)) & 0xFFFFu) << 16);
        }
        for (uint32_t j = 0; j + 1 < parties; ++j) {
            uint32_t r[16];
            chacha_block<DR>(key, nonce, (g * (parties - 1) + j) * kBlocks + (uint64_t)b, r);
            store_share_block(dst.db[j], dst.t_first[j] + i, b, r);
#pragma unroll
            for (int q = 0; q < 16; ++q) last[q] = pk_sub_u16(last[q], r[q]);
        }
        store_share_block(dst.db[parties - 1], dst.t_first[parties - 1] + i, b, last);
    }
}

// The 16 mask bits of an xpacked dword (nibble p: bit 1 = em[2p], bit 0 = em[2p+1]) as a
// plain 16-bit mask word: swap the pair, then compact two bits per nibble (SWAR).
__device__ __forceinline__ uint32_t xmask(uint32_t x) {
    uint32_t m = ((x & 0x11111111u) << 1) | ((x >> 1) & 0x11111111u);  // em[2p] bit 0, em[2p+1] bit 1
    m = (m | (m >> 2)) & 0x0F0F0F0Fu;
    m = (m | (m >> 4)) & 0x00FF00FFu;
    return (m | (m >> 8)) & 0xFFFFu;
}

// Fully in place: templates read from a TILES template database (one 8-byte
// xpacked pair per (template, dword b), unpacked with xunpack), shares and the
// optional masks written straight into TILES databases — one launch, no
// staging.  The masks dword b of record t is component (b & 6) / 2 of the
// 16-byte word (b / 8, half b & 1) of its tile (pack_masks_tiles' layout).
template <int DR>
__global__ void __launch_bounds__(256) prepare_direct_kernel(const uint4 *__restrict__ tdb, uint64_t t_first,
                                                             uint64_t m, uint64_t g0, ChachaKey key, uint64_t nonce,
                                                             uint32_t parties, ShareDsts dst, uint4 *masks,
                                                             uint64_t m_first) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const uint64_t i = (uint64_t)blockIdx.x * 64 + lane;
    const uint64_t tt = t_first + i;
    const uint4 *tbase = tdb + (tt / 32) * (uint64_t)(kPlaneGroups * 64) + (tt % 32);
    uint32_t *mbase = nullptr;
    if (masks) {
        const uint64_t mt = m_first + i;
        mbase = (uint32_t *)(masks + (mt / 32) * (uint64_t)kMaskTileUint4 + (mt % 32));
    }
    // encode() of an element pair from its xpacked nibble (ep[2q], ep[2q+1], em[2q], em[2q+1] in
    // bits 3..0): a 16-entry table in LDS; a wave's lanes read at most 16 distinct dwords in 16
    // distinct banks (broadcasts otherwise), so the lookups never conflict
    __shared__ uint32_t enc_lut[16];
    if (threadIdx.x < 16) {
        const uint32_t n = threadIdx.x, m0 = (n >> 1) & 1u, m1 = n & 1u, p0 = (n >> 3) & 1u, p1 = (n >> 2) & 1u;
        enc_lut[n] = ((m0 - 2u * (p0 & m0)) & 0xFFFFu) | (((m1 - 2u * (p1 & m1)) & 0xFFFFu) << 16);
    }
    __syncthreads();
    if (i >= m) return;
    const uint64_t g = g0 + i;
    for (int b = w; b < kBlocks; b += 4) {
        // dword b of the pattern / mask planes: word (b / 4, half b & 1), pair (b >> 1) & 1
        const uint2 x = ((const uint2 *)(tbase + (b >> 2) * 64 + 32 * (b & 1)))[(b >> 1) & 1];
        if (mbase) mbase[4 * ((b >> 3) * 64 + 32 * (b & 1)) + ((b & 6) >> 1)] = xmask(x.x) | (xmask(x.y) << 16);
        uint32_t last[16];
#pragma unroll
        for (int q = 0; q < 16; ++q) {
            const uint32_t xx = q < 8 ? x.x : x.y, sh = 4 * (q & 7);
            const uint32_t off = sh >= 2 ? (xx >> (sh - 2)) & 0x3Cu : (xx << 2) & 0x3Cu;
            last[q] = *(const uint32_t *)((const char *)enc_lut + off);
        }
        for (uint32_t j = 0; j + 1 < parties; ++j) {
            uint32_t r[16];
            chacha_block<DR>(key, nonce, (g * (parties - 1) + j) * kBlocks + (uint64_t)b, r);
            store_share_block(dst.db[j], dst.t_first[j] + i, b, r);
#pragma unroll
            for (int q = 0; q < 16; ++q) last[q] = pk_sub_u16(last[q], r[q]);
        }
        store_share_block(dst.db[parties - 1], dst.t_first[parties - 1] + i, b, last);
    }
}

static ChachaKey load_key(const uint8_t key[32]) {
    ChachaKey k;
    for (int i = 0; i < 8; ++i)
        k.k[i] = (uint32_t)key[4 * i] | ((uint32_t)key[4 * i + 1] << 8) | ((uint32_t)key[4 * i + 2] << 16) |
                 ((uint32_t)key[4 * i + 3] << 24);
    return k;
}

// the kernel instance for a round count (8, 12, 20); nullptr for any other
template <typename K>
static K by_rounds(uint32_t rounds, K k8, K k12, K k20) {
    return rounds == 8 ? k8 : rounds == 12 ? k12 : rounds == 20 ? k20 : nullptr;
}

int launch_prepare_direct(void *stream, const void *tdb, uint64_t t_first, uint64_t m, uint64_t g0,
                          const uint8_t key[32], uint64_t nonce, uint32_t rounds, uint32_t parties,
                          void *const *dbs, const uint64_t *s_first, void *masks, uint64_t m_first) {
    if (m == 0) return 0;
    if (parties == 0 || parties > (uint32_t)kMaxPrepParties) return -1;
    const ChachaKey k = load_key(key);
    ShareDsts d{};
    for (uint32_t j = 0; j < parties; ++j) {
        d.db[j] = (uint4 *)dbs[j];
        d.t_first[j] = s_first[j];
    }
    const auto kern = by_rounds(rounds, prepare_direct_kernel<4>, prepare_direct_kernel<6>, prepare_direct_kernel<10>);
    if (!kern) return -1;
    hipLaunchKernelGGL(kern, dim3((uint32_t)((m + 63) / 64)), dim3(256), 0, (hipStream_t)stream,
                       (const uint4 *)tdb, t_first, m, g0, k, nonce, parties, d, (uint4 *)masks, m_first);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

int launch_prepare_shares_tiles(void *stream, const void *templates, uint64_t m, uint64_t g0, const uint8_t key[32],
                                uint64_t nonce, uint32_t rounds, uint32_t parties, void *const *dbs, const uint64_t *t_first) {
    if (m == 0) return 0;
    if (parties == 0 || parties > (uint32_t)kMaxPrepParties) return -1;
    const ChachaKey k = load_key(key);
    ShareDsts d{};
    for (uint32_t j = 0; j < parties; ++j) {
        d.db[j] = (uint4 *)dbs[j];
        d.t_first[j] = t_first[j];
    }
    const auto kern = by_rounds(rounds, prepare_shares_tiles_kernel<4>, prepare_shares_tiles_kernel<6>,
                                 prepare_shares_tiles_kernel<10>);
    if (!kern) return -1;
    hipLaunchKernelGGL(kern, dim3((uint32_t)((m + 63) / 64)), dim3(256), 0, (hipStream_t)stream,
                       (const uint32_t *)templates, m, g0, k, nonce, parties, d);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

int launch_prepare_shares(void *stream, const void *templates, uint64_t m, uint64_t g0, const uint8_t key[32],
                          uint64_t nonce, uint32_t rounds, uint32_t parties, void *shares) {
    if (m == 0) return 0;
    const ChachaKey k = load_key(key);
    const uint64_t total = m * kBlocks;
    uint64_t grid = (total + 255) / 256;
    if (grid > 256ull * 64) grid = 256ull * 64;
    const auto kern = by_rounds(rounds, prepare_shares_kernel<4>, prepare_shares_kernel<6>, prepare_shares_kernel<10>);
    if (!kern) return -1;
    hipLaunchKernelGGL(kern, dim3((uint32_t)grid), dim3(256), 0, (hipStream_t)stream,
                       (const uint32_t *)templates, m, g0, k, nonce, parties, (uint16_t *)shares);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

}  // namespace iris
