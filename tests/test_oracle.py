"""CPU: pin the oracle.  The reference's own unit tests (ported, seeded instead
of thread_rng) run against the C oracle and the numpy restatement, and the
committed golden vectors are re-derived by both."""
import numpy as np
import pytest

from oracle import oracle_c as oc
from oracle import oracle_np as on

ROT = 31


@pytest.fixture(scope="module")
def rng():
    return np.random.default_rng(2024)


# ---- src/bits.rs tests ---------------------------------------------------------------


def test_limbs_exact():  # src/bits.rs:213-216
    assert 200 * 64 == 12800 and 25 * 8 == 200


def test_index(rng):  # src/bits.rs:219-232: bit i = byte i/8, bit i%8 of the LE byte view
    for _ in range(5):
        bits = rng.integers(0, 2**64, 200, dtype=np.uint64)
        by = bits.view(np.uint8)
        mat = on.bits_to_matrix(bits).reshape(-1)
        for loc in map(int, rng.choice(12800, 500, replace=False)):
            expected = bool(by[loc // 8] & (1 << (loc % 8)))
            assert bool((int(bits[loc // 64]) >> (loc % 64)) & 1) == expected
            assert bool(mat[loc]) == expected


def test_bits_rotated_inverse(rng):  # src/bits.rs:235-247
    for _ in range(20):
        bits = rng.integers(0, 2**64, 200, dtype=np.uint64)
        for amount in range(-15, 16):
            assert (oc.bits_rotated(oc.bits_rotated(bits, amount), -amount) == bits).all(), amount


def test_bits_rotation_c_vs_numpy(rng):
    for _ in range(10):
        bits = rng.integers(0, 2**64, 200, dtype=np.uint64)
        for amount in range(-15, 16):
            assert (oc.bits_rotated(bits, amount) == on.bits_rotated(bits, amount)).all(), amount


# ---- src/encoded_bits.rs tests -------------------------------------------------------


def test_encoded_rotated_inverse(rng):  # src/encoded_bits.rs:190-203
    for _ in range(10):
        s = rng.integers(0, 2**16, 12800, dtype=np.uint16)
        for amount in range(-15, 16):
            assert (oc.encoded_rotated(oc.encoded_rotated(s, amount), -amount) == s).all()


def test_encoded_rotated_number():  # src/encoded_bits.rs:206-219 (known answer)
    i = np.arange(12800)
    row, col = i // 200, i % 200
    secret = ((row << 8) | col).astype(np.uint16)
    for amount in range(-15, 16):
        rotated = oc.encoded_rotated(secret, amount)
        expect_col = (200 + col - amount) % 200
        assert (rotated == ((row << 8) | expect_col).astype(np.uint16)).all(), amount
        assert (on.encoded_rotated(secret, amount) == rotated).all()


def test_encoded_rotated_bits(rng):  # src/encoded_bits.rs:222-236
    for _ in range(10):
        bits = rng.integers(0, 2**64, 200, dtype=np.uint64)
        secret = on.encoded_from_bits(bits)
        for amount in range(-15, 16):
            assert (on.encoded_from_bits(oc.bits_rotated(bits, amount)) == oc.encoded_rotated(secret, amount)).all()


# ---- src/lib.rs tests ----------------------------------------------------------------


def test_preprocess(rng):  # src/lib.rs:117-132
    for _ in range(10):
        t = rng.integers(0, 2**64, 400, dtype=np.uint64)
        enc = oc.encode(t)
        m = on.bits_to_matrix(t[200:]).reshape(-1)
        p = on.bits_to_matrix(t[:200]).reshape(-1)
        assert set(np.unique(enc).tolist()) <= {0, 1, 0xFFFF}
        assert ((enc == 0xFFFF) == ((m == 1) & (p == 1))).all()
        assert ((enc == 0) == (m == 0)).all()
        assert ((enc == 1) == ((m == 1) & (p == 0))).all()
        assert (on.encode(t[:200], t[200:]) == enc).all()


def test_dotproduct(rng):  # src/lib.rs:134-163
    for _ in range(10):
        a = rng.integers(0, 2**64, 400, dtype=np.uint64)
        b = rng.integers(0, 2**64, 400, dtype=np.uint64)
        am, ap = on.bits_to_matrix(a[200:]).reshape(-1), on.bits_to_matrix(a[:200]).reshape(-1)
        bm, bp = on.bits_to_matrix(b[200:]).reshape(-1), on.bits_to_matrix(b[:200]).reshape(-1)
        both = (am == 1) & (bm == 1)
        equal = int((both & (ap == bp)).sum())
        uneq = int((both & (ap != bp)).sum())
        s = np.int16(np.uint16(oc.dot_u16(oc.encode(a), oc.encode(b))).view(np.int16))
        assert equal - uneq == s
        assert equal + uneq == int(both.sum())
        assert (int(both.sum()) - s) % 2 == 0
        assert uneq == (int(both.sum()) - s) // 2


# ---- src/arch tests ------------------------------------------------------------------


def test_dot_u16_wrapping(rng):  # src/arch/sve.rs:79-108 (u64 accumulate, truncate)
    for _ in range(10):
        a = rng.integers(0, 2**16, 12800, dtype=np.uint16)
        b = rng.integers(0, 2**16, 12800, dtype=np.uint16)
        expected = int((a.astype(np.uint64) * b.astype(np.uint64)).sum()) & 0xFFFF
        assert oc.dot_u16(a, b) == expected
        assert int(on.dot_u16(a, b)) == expected


def test_dot_bool(rng):
    for _ in range(10):
        a = rng.integers(0, 2**64, 200, dtype=np.uint64)
        b = rng.integers(0, 2**64, 200, dtype=np.uint64)
        expected = sum(bin(int(x) & int(y)).count("1") for x, y in zip(a, b))
        assert oc.dot_bool(a, b) == expected == int(on.dot_bool(a, b))


# ---- engines, Template, decode ---------------------------------------------------------


def test_template_paths_agree(rng):
    db = oc.gen_templates(5, 0, 64)
    q = db[0]
    num, den = oc.template_counts(q, db)
    n2, d2 = on.template_counts(q[:200], q[200:], db[:, :200], db[:, 200:])
    assert (num == n2).all() and (den == d2).all()
    dist = oc.template_distances(q, db)
    assert (dist.view(np.uint64) == on.template_distances(q[:200], q[200:], db[:, :200], db[:, 200:]).view(np.uint64)).all()
    for i in range(0, 64, 7):  # per-pair Template::distance (rotates per pair)
        assert oc.template_distance(q, db[i]) == dist[i]
    assert (oc.masks_batch(q[200:], db[:, 200:]) == den).all()


def test_encrypted_distances_identity(rng):  # src/lib.rs:165-193 semantics on synthetic data
    db = oc.gen_templates(9, 100, 12)
    q = db[0]
    enc_q = oc.encode(q)
    enc = np.stack([oc.encode(t) for t in db])
    d = oc.distance_batch(enc_q, enc)
    den = oc.masks_batch(q[200:], db[:, 200:])
    dist = oc.template_distances(q, db)
    for i in range(db.shape[0]):
        assert oc.decode_distance(d[i], den[i]) == dist[i]


def test_decode_nan_inf():
    # den = 0 everywhere -> every quotient NaN or inf -> fold gives +inf
    assert oc.decode_distance(np.zeros(31, np.uint16), np.zeros(31, np.uint16)) == np.inf
    assert np.isinf(on.decode_distance(np.zeros(31, np.uint16), np.zeros(31, np.uint16)))


def test_argmin_tiebreak():
    d = np.array([np.inf, 0.5, 0.25, 0.25, np.nan, 0.3])
    assert oc.argmin(d) == (0.25, 2)
    assert oc.argmin(np.array([np.inf, np.inf])) == (np.inf, 2**64 - 1)


def test_generator_c_vs_numpy():
    assert (oc.gen_templates(42, 1000, 5) == oc.templates_array(*on.gen_templates(42, 1000, 5))).all()
    assert (oc.gen_shares(42, 7, 2) == on.gen_shares(42, 7, 2)).all()
    assert (oc.gen_masks(42, 7, 3) == on.gen_templates(42, 7, 3)[1]).all()


# ---- golden vectors ------------------------------------------------------------------------


def test_golden_vectors(golden):
    q, db = golden["query"], golden["db"]
    num, den = oc.template_counts(q, db)
    assert (num == golden["num"]).all() and (den == golden["den"]).all()
    dist = oc.template_distances(q, db)
    assert (dist.view(np.uint64) == golden["dist_bits"]).all()
    n2, d2 = on.template_counts(q[:200], q[200:], db[:, :200], db[:, 200:])
    assert (n2 == golden["num"]).all() and (d2 == golden["den"]).all()
    best, idx = oc.argmin(dist)
    assert np.float64(best).view(np.uint64) == golden["argmin_dist_bits"] and idx == int(golden["argmin_index"])
    assert (oc.masks_batch(q[200:], db[:, 200:]) == golden["masks_out"]).all()
    assert (oc.encode(q) == golden["enc_query"]).all()
    for k in range(3):
        assert (oc.distance_batch(golden["enc_query"], golden["shares"][k]) == golden["share_out"][k]).all()
    rs = oc.resolver_combine(golden["share_out"], golden["masks_out"][: golden["enc_db"].shape[0]])
    assert (rs.view(np.uint64) == golden["dist_bits"][: rs.shape[0]]).all()
    for r in range(-15, 16):
        assert (oc.bits_rotated(q[200:], r) == golden["rot_mask"][r + 15]).all()
    assert oc.dot_u16(golden["wrap_a"], golden["wrap_b"]) == int(golden["wrap_dot"])
