"""CPU: the oracle against the reference's own specification (/root/reference/specification.ipynb,
restated here from its text; the notebook holds no code or outputs): the ring representation of
masked bitvectors (F, U, T -> -1, 0, 1), the fractional Hamming distance as
fhd(a, b) = 1/2 - sum(a * b) / (2 * sum((a * b)^2)), the distance as the minimum over rotations
r in [-15, 15] of the 64 x 200 bit matrix's columns, and "Iriscode SMPC v1": per-party share dot
products d_ijr mod 2^16, summed by the coordinator, with m_ir = popcount(rot(a_m, r) & b_im).

These are written from the formulas, independently of oracle/ (numpy on {-1, 0, 1} matrices,
fractions compared exactly), so they pin the oracle's arithmetic to the reference's definitions;
they cannot pin the reference's code paths (no Rust toolchain; its data/ fixtures are absent).
The specification writes the rotation as rot(b, n)[i, j] = b[i, (j + n) mod 200]; the code's
Bits::rotate (src/bits.rs:18-29, 178-205) moves the other way, so rotation indices differ in sign
and the distance (a minimum over a symmetric range) does not."""
from fractions import Fraction

import numpy as np
import pytest

from oracle import oracle_c as oc

ROWS, COLS = 64, 200


def bits_matrix(limbs):
    """[u64; 200] -> 64 x 200 {0, 1} (bit i = row i / 200, column i % 200; LE, src/bits.rs:44-57)."""
    return np.unpackbits(np.ascontiguousarray(limbs, np.uint64).view(np.uint8), bitorder="little").reshape(ROWS, COLS)


def ring(template):
    """Masked bitvector of a template in the ring: m - 2 b m (spec: 'the reverse mapping')."""
    p, m = bits_matrix(template[:200]).astype(np.int64), bits_matrix(template[200:]).astype(np.int64)
    return m - 2 * p * m


def rot_spec(a, n):
    """rot(b, n)[i, j] = b[i, (j + n) mod 200] (spec, 'Rotations')."""
    return np.roll(a, -n, axis=1)


def fhd(a, b):
    """(numerator, denominator) of fhd(a, b) = 1/2 - sum(a b) / (2 sum((a b)^2)) = (m - s) / (2 m)."""
    ab = a * b
    s, m = int(ab.sum()), int((ab * ab).sum())
    return (m - s, 2 * m)


def dist_spec(a, b):
    fr = [fhd(rot_spec(a, r), b) for r in range(-15, 16)]
    fr = [Fraction(x, y) for x, y in fr if y]
    return min(fr) if fr else None


@pytest.fixture(scope="module")
def templates():
    return oc.gen_templates(777, 0, 40)


def test_ring_operations(templates):
    """count(a) = sum(a^2), popcount(a) = 1/2 sum(a^2 + a), a xor b = -a b for available entries,
    and popcount(a xor b) / count(a xor b) equals the fhd formula (spec, 'Masked binary operations
    in rings', 'Fractional hamming distance')."""
    for i in range(0, 40, 2):
        a, b = ring(templates[i]), ring(templates[i + 1])
        pa, ma = bits_matrix(templates[i][:200]), bits_matrix(templates[i][200:])
        assert int((a * a).sum()) == int(ma.sum())
        # 1/2 (a^2 + a) is 1 where a = +1 (T): under the reverse mapping m - 2 b m that is b = 0, so
        # it extracts NOT b -- the specification's "data bits" and the code's pattern bits
        # (encode, src/lib.rs:16-26) are complements; fhd, being symmetric, does not care
        assert int(((a * a + a) // 2).sum()) == int((ma & (1 - pa)).sum())
        x = -a * b
        both = (a != 0) & (b != 0)
        assert ((x == 1) == (both & (a != b))).all() and ((x == -1) == (both & (a == b))).all()
        popc, cnt = int(((x * x + x) // 2).sum()), int((x * x).sum())
        assert Fraction(popc, cnt) == Fraction(*fhd(a, b))


def test_distance_is_the_spec_minimum(templates):
    """The oracle's Template::distance (src/template.rs:43-64) equals the specification's
    dist(a, b) = min over r in [-15, 15] of fhd(rot(a, r), b), as the correctly rounded f64 of the
    exact minimum fraction, for 190 pairs including rotated copies."""
    q = templates[0]
    db = templates.copy()
    db[5] = np.concatenate([oc.bits_rotated(q[:200], 7), oc.bits_rotated(q[200:], 7)])  # a rotated copy
    got = oc.template_distances(q, db)
    a = ring(q)
    for i in range(len(db)):
        want = dist_spec(a, ring(db[i]))
        assert np.float64(got[i]).view(np.uint64) == np.float64(float(want)).view(np.uint64), i
    assert got[5] == 0.0
    for i in range(1, 12):  # pairs among the other records too
        for j in range(i + 1, 12):
            want = dist_spec(ring(templates[i]), ring(templates[j]))
            assert oc.template_distance(templates[i], templates[j]) == float(want), (i, j)


def test_smpc_v1_recovers_the_distance(templates):
    """'Iriscode SMPC v1': the database's ring vectors split into 3 additive shares mod 2^16 (the
    oracle's EncodedBits::share of encode(t)); each party computes d_ijr = sum(rot(a, r) b_ij)
    mod 2^16 against the clear query; the coordinator sums them mod 2^16 (signed: |d| <= 12800),
    computes m_ir = popcount(rot(a_m, r) & b_im) from the masks alone and
    dist = min_r (1/2 - d_ir / (2 m_ir)), which equals the plaintext distance -- and the oracle's
    resolver combine (src/main.rs:597-612) returns the same value."""
    q, db = templates[0], templates[1:13]
    shares, masks = oc.prepare_shares(db, bytes(range(32)), parties=3)
    a = ring(q)
    am = bits_matrix(q[200:]).astype(np.int64)
    want = oc.template_distances(q, db)
    rows_s = np.zeros((3, len(db), 31), np.uint16)
    rows_m = np.zeros((len(db), 31), np.uint16)
    for i in range(len(db)):
        bm = bits_matrix(masks[i]).astype(np.int64)
        best = None
        for k, r in enumerate(range(-15, 16)):
            ra = rot_spec(a, r).reshape(-1)
            d = sum(int((ra * shares[j, i].astype(np.int64)).sum()) % 65536 for j in range(3)) % 65536
            d = d - 65536 if d >= 32768 else d
            m = int((rot_spec(am, r) * bm).sum())
            f = Fraction(m - d, 2 * m)
            best = f if best is None else min(best, f)
            for j in range(3):  # the same rows in the code's layout: rotation k = 15 - r
                rows_s[j, i, 15 - r] = int((ra * shares[j, i].astype(np.int64)).sum()) % 65536
            rows_m[i, 15 - r] = m
        assert float(best) == want[i], i
    assert (oc.resolver_combine(rows_s, rows_m) == want).all()
