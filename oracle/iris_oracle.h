/*
 * iris_oracle.h — TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement of the reference (recmo/mpc-iris-code v0.8.0) hot path,
 * used as the parity checker in tests/, in __graft_entry__.smoke() and as the
 * `cpu_baseline` leg of bench.py.  Nothing in the product (mpc-iris-code_amd/)
 * links, imports or calls this code.
 *
 * Parity status: the reference is Rust and cannot be compiled in this image
 * (no cargo/rustc), and its real-data fixtures (data/templates.json,
 * data/distances.json) are git-ignored and absent.  This restatement is
 * pinned by (a) the reference's own known-answer / property tests, ported in
 * tests/test_oracle.py (src/bits.rs:213-247, src/encoded_bits.rs:190-236,
 * src/lib.rs:117-163, src/arch/sve.rs:79-108), and (b) agreement with an
 * independent numpy restatement (oracle/oracle_np.py) on every committed
 * golden vector (tests/golden/).
 */
#ifndef IRIS_ORACLE_H
#define IRIS_ORACLE_H
#include <stdint.h>

#define ORC_COLS 200
#define ORC_ROWS 64
#define ORC_BITS 12800
#define ORC_LIMBS 200
#define ORC_BYTES_PER_ROW 25
#define ORC_ROT 31

typedef struct {
    uint64_t pattern[ORC_LIMBS];
    uint64_t mask[ORC_LIMBS];
} orc_template;

/* value types */
void orc_bits_rotated(const uint64_t in[ORC_LIMBS], int amount, uint64_t out[ORC_LIMBS]);
void orc_encoded_rotated(const uint16_t in[ORC_BITS], int amount, uint16_t out[ORC_BITS]);
void orc_encoded_from_bits(const uint64_t in[ORC_LIMBS], uint16_t out[ORC_BITS]);
void orc_encode(const orc_template *t, uint16_t out[ORC_BITS]);

/* arch kernels */
uint16_t orc_dot_bool(const uint64_t a[ORC_LIMBS], const uint64_t b[ORC_LIMBS]);
uint16_t orc_dot_u16(const uint16_t a[ORC_BITS], const uint16_t b[ORC_BITS]);
/* the criterion harness loop (src/arch/mod.rs:34-41, 62-69): for b in db { for a in queries },
 * single-threaded; out[j*na + i] = dot(a[i], b[j]) */
void orc_dot_bool_pairs(const uint64_t *a, uint64_t na, const uint64_t *b, uint64_t nb, uint16_t *out);
void orc_dot_u16_pairs(const uint16_t *a, uint64_t na, const uint16_t *b, uint64_t nb, uint16_t *out);

/* engines (batch_process); out is [n][31] */
void orc_masks_batch(const uint64_t query[ORC_LIMBS], const uint64_t *db, uint64_t n, uint16_t *out, int threads);
void orc_distance_batch(const uint16_t query[ORC_BITS], const uint16_t *db, uint64_t n, uint16_t *out, int threads);

/* Template */
void orc_fraction_hamming_counts(const orc_template *a, const orc_template *b, uint32_t *num, uint32_t *den);
double orc_fraction_hamming(const orc_template *a, const orc_template *b);
double orc_template_distance(const orc_template *a, const orc_template *b);
void orc_template_counts_batch(const orc_template *query, const orc_template *db, uint64_t n, uint16_t *num_out,
                               uint16_t *den_out, int threads);
void orc_template_distances_batch(const orc_template *query, const orc_template *db, uint64_t n, double *out,
                                  int threads);

/* decode + resolver */
double orc_decode_distance(const uint16_t distances[ORC_ROT], const uint16_t denominators[ORC_ROT]);
void orc_argmin(const double *dist, uint64_t n, double *min_distance, uint64_t *min_index);
void orc_resolver_combine(const uint16_t *shares, uint32_t parts, const uint16_t *denoms, uint64_t n,
                          double *dist_out, int threads);

/* synthetic data generator */
uint64_t orc_gen_limb(uint64_t seed, uint64_t stream, uint64_t ctr);
void orc_gen_template(uint64_t seed, uint64_t t, orc_template *out);
void orc_gen_share(uint64_t seed, uint64_t t, uint16_t out[ORC_BITS]);
void orc_gen_templates(uint64_t seed, uint64_t t0, uint64_t n, orc_template *out);
void orc_gen_masks(uint64_t seed, uint64_t t0, uint64_t n, uint64_t *out);
void orc_gen_shares(uint64_t seed, uint64_t t0, uint64_t n, uint16_t *out);

/* share preparation.  ChaCha block function with
 * `rounds` (8, 12, 20) rounds, D. J. Bernstein's original parameterisation
 * (64-bit block counter in state words 12-13, 64-bit nonce in words 14-15),
 * which is also rand_chacha 0.3.1's (the reference's thread_rng core is its
 * ChaCha12, rand 0.8.5); RFC 8439 §2.3 is the 20-round function with the 128
 * bits split 32/96, so its test vectors apply. */
void orc_chacha_block(const uint8_t key[32], uint64_t nonce, uint64_t counter, uint32_t rounds, uint8_t out[64]);
/* EncodedBits::share (src/encoded_bits.rs:23-38) of encode(t[i]) for
 * template index g = index_base + i: shares j < parties-1 are the ChaCha
 * (`rounds`) keystream blocks counter = (g * (parties-1) + j) * 400 + b, b = 0..399
 * (element 32b + e = little-endian u16 e of block b); the last share is
 * encode(t) minus their sum (mod 2^16).  shares: [parties][n][12800];
 * masks (may be NULL): [n][200], the `.masks` records (src/main.rs:333-342). */
void orc_prepare_shares(const orc_template *t, uint64_t n, uint64_t index_base, const uint8_t key[32],
                        uint64_t nonce, uint32_t rounds, uint32_t parties, uint16_t *shares, uint64_t *masks,
                        int threads);

#endif
