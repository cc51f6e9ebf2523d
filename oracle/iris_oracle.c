/*
 * iris_oracle.c — TEST INFRASTRUCTURE ONLY (see iris_oracle.h).
 *
 * Plain-C restatement of the reference's CPU path.  Each function cites the
 * reference lines it follows.  The rotation is restated the way the
 * reference implements it (whole-byte rotate + carry chain inside a 25-byte
 * row), NOT by the col-(r) formula the product uses, so that the two are
 * independent.  Multi-threaded batch forms mirror rayon's `par_iter` over
 * database entries (src/lib.rs:44,71); they are the CPU baseline.
 */
#include "iris_oracle.h"

#include <math.h>
#include <pthread.h>
#include <stdlib.h>
#include <string.h>

/* ------------------------------------------------------------ rotations */

/* slice::rotate_left / rotate_right on 25 bytes (core::slice semantics) */
static void bytes_rotate_left(uint8_t *a, int n, int k) {
    uint8_t tmp[ORC_BYTES_PER_ROW];
    k %= n;
    for (int i = 0; i < n; ++i) tmp[i] = a[(i + k) % n];
    memcpy(a, tmp, (size_t)n);
}
static void bytes_rotate_right(uint8_t *a, int n, int k) { bytes_rotate_left(a, n, (n - (k % n)) % n); }

/* fn rotate_row (src/bits.rs:178-205), operating on one 25-byte row. */
static void rotate_row(uint8_t a[ORC_BYTES_PER_ROW], int amount) {
    if (amount <= -8) {
        bytes_rotate_left(a, ORC_BYTES_PER_ROW, (-amount) / 8); /* :180 */
        amount %= 8;                                           /* :181 (Rust % truncates) */
    } else if (amount >= 8) {
        bytes_rotate_right(a, ORC_BYTES_PER_ROW, amount / 8); /* :183 */
        amount %= 8;
    }
    if (amount < 0) { /* :186-194 */
        int r = -amount, l = 8 - r;
        uint8_t carry = (uint8_t)(a[0] << l);
        for (int i = ORC_BYTES_PER_ROW - 1; i >= 0; --i) {
            uint8_t old = a[i];
            a[i] = (uint8_t)((old >> r) | carry);
            carry = (uint8_t)(old << l);
        }
    } else if (amount > 0) { /* :195-203 */
        int l = amount, r = 8 - l;
        uint8_t carry = (uint8_t)(a[ORC_BYTES_PER_ROW - 1] >> r);
        for (int i = 0; i < ORC_BYTES_PER_ROW; ++i) {
            uint8_t old = a[i];
            a[i] = (uint8_t)((old << l) | carry);
            carry = (uint8_t)(old >> r);
        }
    }
}

/* Bits::rotate / rotated (src/bits.rs:18-29): per 25-byte chunk of the LE byte view */
void orc_bits_rotated(const uint64_t in[ORC_LIMBS], int amount, uint64_t out[ORC_LIMBS]) {
    uint8_t bytes[ORC_LIMBS * 8];
    for (int i = 0; i < ORC_LIMBS; ++i)
        for (int b = 0; b < 8; ++b) bytes[i * 8 + b] = (uint8_t)(in[i] >> (8 * b));
    for (int row = 0; row < ORC_ROWS; ++row) rotate_row(bytes + row * ORC_BYTES_PER_ROW, amount);
    for (int i = 0; i < ORC_LIMBS; ++i) {
        uint64_t v = 0;
        for (int b = 0; b < 8; ++b) v |= (uint64_t)bytes[i * 8 + b] << (8 * b);
        out[i] = v;
    }
}

/* EncodedBits::rotate (src/encoded_bits.rs:40-52): rows of COLS u16 */
void orc_encoded_rotated(const uint16_t in[ORC_BITS], int amount, uint16_t out[ORC_BITS]) {
    for (int row = 0; row < ORC_ROWS; ++row) {
        const uint16_t *src = in + row * ORC_COLS;
        uint16_t *dst = out + row * ORC_COLS;
        if (amount < 0) { /* rotate_left(|amount|) */
            int k = (-amount) % ORC_COLS;
            for (int i = 0; i < ORC_COLS; ++i) dst[i] = src[(i + k) % ORC_COLS];
        } else if (amount > 0) { /* rotate_right(amount) */
            int k = amount % ORC_COLS;
            for (int i = 0; i < ORC_COLS; ++i) dst[(i + k) % ORC_COLS] = src[i];
        } else {
            memcpy(dst, src, sizeof(uint16_t) * ORC_COLS);
        }
    }
}

/* impl From<&Bits> for EncodedBits (src/encoded_bits.rs:75-79), Bits Index (src/bits.rs:44-57) */
void orc_encoded_from_bits(const uint64_t in[ORC_LIMBS], uint16_t out[ORC_BITS]) {
    for (int i = 0; i < ORC_BITS; ++i) out[i] = (uint16_t)((in[i / 64] >> (i % 64)) & 1u);
}

/* encode (src/lib.rs:16-26): pattern &= mask; mask - pattern - pattern (wrapping u16) */
void orc_encode(const orc_template *t, uint16_t out[ORC_BITS]) {
    uint64_t p[ORC_LIMBS];
    uint16_t pe[ORC_BITS], me[ORC_BITS];
    for (int i = 0; i < ORC_LIMBS; ++i) p[i] = t->pattern[i] & t->mask[i];
    orc_encoded_from_bits(p, pe);
    orc_encoded_from_bits(t->mask, me);
    for (int i = 0; i < ORC_BITS; ++i) out[i] = (uint16_t)(me[i] - pe[i] - pe[i]);
}

/* ------------------------------------------------------------ arch */

/* generic::dot_bool (src/arch/generic.rs:4-9) */
uint16_t orc_dot_bool(const uint64_t a[ORC_LIMBS], const uint64_t b[ORC_LIMBS]) {
    uint16_t s = 0;
    for (int i = 0; i < ORC_LIMBS; ++i) s = (uint16_t)(s + (uint16_t)__builtin_popcountll(a[i] & b[i]));
    return s;
}

/* generic::dot_u16 (src/arch/generic.rs:11-16): wrapping_mul, wrapping_add */
uint16_t orc_dot_u16(const uint16_t a[ORC_BITS], const uint16_t b[ORC_BITS]) {
    uint32_t s = 0; /* mod 2^16 at the end is identical to wrapping u16 adds */
    for (int i = 0; i < ORC_BITS; ++i) s += (uint32_t)(uint16_t)((uint32_t)a[i] * (uint32_t)b[i]);
    return (uint16_t)s;
}

/* The criterion harness (src/arch/mod.rs:22-72): for b in db { for a in queries { f(a, b) } },
 * one thread, as criterion runs it. */
void orc_dot_bool_pairs(const uint64_t *a, uint64_t na, const uint64_t *b, uint64_t nb, uint16_t *out) {
    for (uint64_t j = 0; j < nb; ++j)
        for (uint64_t i = 0; i < na; ++i) out[j * na + i] = orc_dot_bool(a + i * ORC_LIMBS, b + j * ORC_LIMBS);
}

void orc_dot_u16_pairs(const uint16_t *a, uint64_t na, const uint16_t *b, uint64_t nb, uint16_t *out) {
    for (uint64_t j = 0; j < nb; ++j)
        for (uint64_t i = 0; i < na; ++i) out[j * na + i] = orc_dot_u16(a + i * ORC_BITS, b + j * ORC_BITS);
}

/* ------------------------------------------------------------ threading */

typedef void (*range_fn)(void *ctx, uint64_t lo, uint64_t hi);
typedef struct {
    range_fn fn;
    void *ctx;
    uint64_t lo, hi;
} range_job;

static void *range_thread(void *p) {
    range_job *j = (range_job *)p;
    j->fn(j->ctx, j->lo, j->hi);
    return NULL;
}

static void parallel_for(uint64_t n, int threads, range_fn fn, void *ctx) {
    if (threads <= 1 || n < 64) {
        fn(ctx, 0, n);
        return;
    }
    if (threads > 256) threads = 256;
    pthread_t tid[256];
    range_job jobs[256];
    uint64_t chunk = (n + (uint64_t)threads - 1) / (uint64_t)threads;
    int started = 0;
    for (int t = 0; t < threads; ++t) {
        uint64_t lo = (uint64_t)t * chunk, hi = lo + chunk;
        if (lo >= n) break;
        if (hi > n) hi = n;
        jobs[t] = (range_job){fn, ctx, lo, hi};
        if (pthread_create(&tid[t], NULL, range_thread, &jobs[t]) != 0) {
            fn(ctx, lo, hi);
            jobs[t].fn = NULL;
        }
        started = t + 1;
    }
    for (int t = 0; t < started; ++t)
        if (jobs[t].fn) pthread_join(tid[t], NULL);
}

/* ------------------------------------------------------------ engines */

/* MasksEngine (src/lib.rs:55-80): rotations built once, then per entry 31 dot_bool */
typedef struct {
    uint64_t rot[ORC_ROT][ORC_LIMBS];
    const uint64_t *db;
    uint16_t *out;
} masks_ctx;

static void masks_range(void *p, uint64_t lo, uint64_t hi) {
    masks_ctx *c = (masks_ctx *)p;
    for (uint64_t i = lo; i < hi; ++i)
        for (int k = 0; k < ORC_ROT; ++k) c->out[i * ORC_ROT + k] = orc_dot_bool(c->rot[k], c->db + i * ORC_LIMBS);
}

void orc_masks_batch(const uint64_t query[ORC_LIMBS], const uint64_t *db, uint64_t n, uint16_t *out, int threads) {
    masks_ctx *c = (masks_ctx *)malloc(sizeof(masks_ctx));
    for (int k = 0; k < ORC_ROT; ++k) orc_bits_rotated(query, k - 15, c->rot[k]);
    c->db = db;
    c->out = out;
    parallel_for(n, threads, masks_range, c);
    free(c);
}

/* DistanceEngine (src/lib.rs:28-53) */
typedef struct {
    uint16_t rot[ORC_ROT][ORC_BITS];
    const uint16_t *db;
    uint16_t *out;
} dist_ctx;

static void dist_range(void *p, uint64_t lo, uint64_t hi) {
    dist_ctx *c = (dist_ctx *)p;
    for (uint64_t i = lo; i < hi; ++i)
        for (int k = 0; k < ORC_ROT; ++k) c->out[i * ORC_ROT + k] = orc_dot_u16(c->rot[k], c->db + i * ORC_BITS);
}

void orc_distance_batch(const uint16_t query[ORC_BITS], const uint16_t *db, uint64_t n, uint16_t *out, int threads) {
    dist_ctx *c = (dist_ctx *)malloc(sizeof(dist_ctx));
    for (int k = 0; k < ORC_ROT; ++k) orc_encoded_rotated(query, k - 15, c->rot[k]);
    c->db = db;
    c->out = out;
    parallel_for(n, threads, dist_range, c);
    free(c);
}

/* ------------------------------------------------------------ Template */

/* Template::fraction_hamming (src/template.rs:49-64) — the counting part */
void orc_fraction_hamming_counts(const orc_template *a, const orc_template *b, uint32_t *num, uint32_t *den) {
    uint32_t n = 0, d = 0;
    for (int i = 0; i < ORC_LIMBS; ++i) {
        uint64_t m = a->mask[i] & b->mask[i];
        uint64_t p = (a->pattern[i] ^ b->pattern[i]) & m;
        n += (uint32_t)__builtin_popcountll(p);
        d += (uint32_t)__builtin_popcountll(m);
    }
    *num = n;
    *den = d;
}

/* (num as f64) / (den as f64): 0/0 = NaN */
double orc_fraction_hamming(const orc_template *a, const orc_template *b) {
    uint32_t n, d;
    orc_fraction_hamming_counts(a, b, &n, &d);
    return (double)n / (double)d;
}

/* Rust f64::min: if one operand is NaN, the other is returned */
static double rust_f64_min(double a, double b) {
    if (isnan(a)) return b;
    if (isnan(b)) return a;
    return a < b ? a : b;
}

/* Template::rotate (src/template.rs:32-36) */
static void template_rotated(const orc_template *t, int amount, orc_template *out) {
    orc_bits_rotated(t->mask, amount, out->mask);
    orc_bits_rotated(t->pattern, amount, out->pattern);
}

/* Template::distance (src/template.rs:43-47): self rotated per pair */
double orc_template_distance(const orc_template *a, const orc_template *b) {
    double acc = INFINITY;
    for (int r = -15; r <= 15; ++r) {
        orc_template ar;
        template_rotated(a, r, &ar);
        acc = rust_f64_min(acc, orc_fraction_hamming(&ar, b));
    }
    return acc;
}

typedef struct {
    orc_template rot[ORC_ROT];
    const orc_template *db;
    uint16_t *num_out, *den_out;
    double *dist_out;
} tmpl_ctx;

/* Engine-style batch: the 31 rotated queries are built once (as src/lib.rs:33-40
 * does for the other engines); per pair the loop body is fraction_hamming. */
static void tmpl_range(void *p, uint64_t lo, uint64_t hi) {
    tmpl_ctx *c = (tmpl_ctx *)p;
    for (uint64_t i = lo; i < hi; ++i) {
        double acc = INFINITY;
        for (int k = 0; k < ORC_ROT; ++k) {
            uint32_t n, d;
            orc_fraction_hamming_counts(&c->rot[k], c->db + i, &n, &d);
            if (c->num_out) c->num_out[i * ORC_ROT + k] = (uint16_t)n;
            if (c->den_out) c->den_out[i * ORC_ROT + k] = (uint16_t)d;
            acc = rust_f64_min(acc, (double)n / (double)d);
        }
        if (c->dist_out) c->dist_out[i] = acc;
    }
}

static void tmpl_batch(const orc_template *query, const orc_template *db, uint64_t n, uint16_t *num_out,
                       uint16_t *den_out, double *dist_out, int threads) {
    tmpl_ctx *c = (tmpl_ctx *)malloc(sizeof(tmpl_ctx));
    for (int k = 0; k < ORC_ROT; ++k) template_rotated(query, k - 15, &c->rot[k]);
    c->db = db;
    c->num_out = num_out;
    c->den_out = den_out;
    c->dist_out = dist_out;
    parallel_for(n, threads, tmpl_range, c);
    free(c);
}

void orc_template_counts_batch(const orc_template *query, const orc_template *db, uint64_t n, uint16_t *num_out,
                               uint16_t *den_out, int threads) {
    tmpl_batch(query, db, n, num_out, den_out, NULL, threads);
}

void orc_template_distances_batch(const orc_template *query, const orc_template *db, uint64_t n, double *out,
                                  int threads) {
    tmpl_batch(query, db, n, NULL, NULL, out, threads);
}

/* ------------------------------------------------------------ decode / resolver */

/* decode_distance (src/lib.rs:97-107) */
double orc_decode_distance(const uint16_t distances[ORC_ROT], const uint16_t denominators[ORC_ROT]) {
    double acc = INFINITY;
    for (int k = 0; k < ORC_ROT; ++k) {
        uint16_t n = distances[k], d = denominators[k];
        uint16_t uneq = (uint16_t)((uint16_t)(d - n) / 2);
        acc = rust_f64_min(acc, (double)uneq / (double)d);
    }
    return acc;
}

/* resolver aggregation (src/main.rs:581-582, 616-621): strict <, first index wins */
void orc_argmin(const double *dist, uint64_t n, double *min_distance, uint64_t *min_index) {
    double best = INFINITY;
    uint64_t idx = UINT64_MAX;
    for (uint64_t j = 0; j < n; ++j)
        if (dist[j] < best) {
            best = dist[j];
            idx = j;
        }
    *min_distance = best;
    *min_index = idx;
}

/* resolver combine (src/main.rs:597-612): wrapping sum of the parts' [u16;31], then decode.
 * shares is [parts][n][31], denoms is [n][31].  The reference runs this loop as a rayon
 * into_par_iter over the entries (src/main.rs:597-612); threads splits the entries the same way
 * (the argmin after it stays sequential, src/main.rs:616-621). */
typedef struct {
    const uint16_t *shares;
    uint32_t parts;
    const uint16_t *denoms;
    uint64_t n;
    double *out;
} combine_ctx;

static void combine_range(void *p, uint64_t lo, uint64_t hi) {
    const combine_ctx *c = (const combine_ctx *)p;
    for (uint64_t i = lo; i < hi; ++i) {
        uint16_t num[ORC_ROT] = {0};
        for (uint32_t q = 0; q < c->parts; ++q)
            for (int k = 0; k < ORC_ROT; ++k)
                num[k] = (uint16_t)(num[k] + c->shares[((uint64_t)q * c->n + i) * ORC_ROT + k]);
        c->out[i] = orc_decode_distance(num, c->denoms + i * ORC_ROT);
    }
}

void orc_resolver_combine(const uint16_t *shares, uint32_t parts, const uint16_t *denoms, uint64_t n,
                          double *dist_out, int threads) {
    combine_ctx c = {shares, parts, denoms, n, dist_out};
    parallel_for(n, threads, combine_range, &c);
}

/* ------------------------------------------------------------ generator */

static uint64_t mix64(uint64_t z) {
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
    return z ^ (z >> 31);
}

/* limb = splitmix64 output number ctr+1 of the stream keyed by (seed, stream) */
uint64_t orc_gen_limb(uint64_t seed, uint64_t stream, uint64_t ctr) {
    uint64_t key = mix64(seed ^ (0xD1B54A32D192ED03ULL * (stream + 1)));
    return mix64(key + (ctr + 1) * 0x9E3779B97F4A7C15ULL);
}

/* Template t: pattern limbs are counters t*400 + j, mask limbs t*400 + 200 + j (stream 0) */
void orc_gen_template(uint64_t seed, uint64_t t, orc_template *out) {
    for (int j = 0; j < ORC_LIMBS; ++j) {
        out->pattern[j] = orc_gen_limb(seed, 0, t * 400 + (uint64_t)j);
        out->mask[j] = orc_gen_limb(seed, 0, t * 400 + 200 + (uint64_t)j);
    }
}

/* EncodedBits t: 3200 limbs, counters t*3200 + j (stream 1), LE u16 lanes */
void orc_gen_share(uint64_t seed, uint64_t t, uint16_t out[ORC_BITS]) {
    for (int j = 0; j < ORC_BITS / 4; ++j) {
        uint64_t v = orc_gen_limb(seed, 1, t * 3200 + (uint64_t)j);
        for (int e = 0; e < 4; ++e) out[j * 4 + e] = (uint16_t)(v >> (16 * e));
    }
}

void orc_gen_templates(uint64_t seed, uint64_t t0, uint64_t n, orc_template *out) {
    for (uint64_t i = 0; i < n; ++i) orc_gen_template(seed, t0 + i, out + i);
}

/* Masks DB generated with the same seed = the mask planes of the template DB */
void orc_gen_masks(uint64_t seed, uint64_t t0, uint64_t n, uint64_t *out) {
    for (uint64_t i = 0; i < n; ++i)
        for (int j = 0; j < ORC_LIMBS; ++j) out[i * ORC_LIMBS + j] = orc_gen_limb(seed, 0, (t0 + i) * 400 + 200 + (uint64_t)j);
}

void orc_gen_shares(uint64_t seed, uint64_t t0, uint64_t n, uint16_t *out) {
    for (uint64_t i = 0; i < n; ++i) orc_gen_share(seed, t0 + i, out + i * ORC_BITS);
}

/* ------------------------------------------------------------ share preparation */

static uint32_t orc_rotl32(uint32_t x, int r) { return (x << r) | (x >> (32 - r)); }

#define ORC_QR(a, b, c, d)                  \
    do {                                    \
        a += b; d ^= a; d = orc_rotl32(d, 16); \
        c += d; b ^= c; b = orc_rotl32(b, 12); \
        a += b; d ^= a; d = orc_rotl32(d, 8);  \
        c += d; b ^= c; b = orc_rotl32(b, 7);  \
    } while (0)

void orc_chacha_block(const uint8_t key[32], uint64_t nonce, uint64_t counter, uint32_t rounds, uint8_t out[64]) {
    uint32_t in[16], x[16];
    in[0] = 0x61707865u; /* "expand 32-byte k" */
    in[1] = 0x3320646eu;
    in[2] = 0x79622d32u;
    in[3] = 0x6b206574u;
    for (int i = 0; i < 8; ++i)
        in[4 + i] = (uint32_t)key[4 * i] | ((uint32_t)key[4 * i + 1] << 8) | ((uint32_t)key[4 * i + 2] << 16) |
                    ((uint32_t)key[4 * i + 3] << 24);
    in[12] = (uint32_t)counter;
    in[13] = (uint32_t)(counter >> 32);
    in[14] = (uint32_t)nonce;
    in[15] = (uint32_t)(nonce >> 32);
    memcpy(x, in, sizeof x);
    for (uint32_t r = 0; r < rounds / 2; ++r) { /* double rounds: column then diagonal */
        ORC_QR(x[0], x[4], x[8], x[12]);
        ORC_QR(x[1], x[5], x[9], x[13]);
        ORC_QR(x[2], x[6], x[10], x[14]);
        ORC_QR(x[3], x[7], x[11], x[15]);
        ORC_QR(x[0], x[5], x[10], x[15]);
        ORC_QR(x[1], x[6], x[11], x[12]);
        ORC_QR(x[2], x[7], x[8], x[13]);
        ORC_QR(x[3], x[4], x[9], x[14]);
    }
    for (int i = 0; i < 16; ++i) {
        const uint32_t v = x[i] + in[i];
        out[4 * i] = (uint8_t)v;
        out[4 * i + 1] = (uint8_t)(v >> 8);
        out[4 * i + 2] = (uint8_t)(v >> 16);
        out[4 * i + 3] = (uint8_t)(v >> 24);
    }
}

/* prepare (src/main.rs:333-361): per template encode + EncodedBits::share(parties), a rayon
 * par_iter over the templates in the reference (src/main.rs:337-344); threads splits them the
 * same way (every template's keystream blocks depend only on its global index) */
typedef struct {
    const orc_template *t;
    uint64_t n, index_base, nonce;
    const uint8_t *key;
    uint32_t rounds, parties;
    uint16_t *shares;
    uint64_t *masks;
} prepare_ctx;

static void prepare_range(void *p, uint64_t lo, uint64_t hi) {
    const prepare_ctx *c = (const prepare_ctx *)p;
    uint16_t enc[ORC_BITS];
    uint8_t blk[64];
    const uint32_t parties = c->parties;
    for (uint64_t i = lo; i < hi; ++i) {
        const uint64_t g = c->index_base + i;
        orc_encode(&c->t[i], enc);
        uint16_t *last = c->shares + ((uint64_t)(parties - 1) * c->n + i) * ORC_BITS;
        memcpy(last, enc, sizeof enc);
        for (uint32_t j = 0; j + 1 < parties; ++j) {
            uint16_t *sh = c->shares + ((uint64_t)j * c->n + i) * ORC_BITS;
            for (int b = 0; b < ORC_BITS / 32; ++b) {
                orc_chacha_block(c->key, c->nonce, (g * (parties - 1) + j) * (ORC_BITS / 32) + (uint64_t)b, c->rounds, blk);
                for (int e = 0; e < 32; ++e) {
                    const uint16_t v = (uint16_t)(blk[2 * e] | (blk[2 * e + 1] << 8));
                    sh[32 * b + e] = v;
                    last[32 * b + e] = (uint16_t)(last[32 * b + e] - v);
                }
            }
        }
        if (c->masks) memcpy(c->masks + i * ORC_LIMBS, c->t[i].mask, sizeof c->t[i].mask);
    }
}

void orc_prepare_shares(const orc_template *t, uint64_t n, uint64_t index_base, const uint8_t key[32],
                        uint64_t nonce, uint32_t rounds, uint32_t parties, uint16_t *shares, uint64_t *masks,
                        int threads) {
    prepare_ctx c = {t, n, index_base, nonce, key, rounds, parties, shares, masks};
    parallel_for(n, threads, prepare_range, &c);
}
