"""TEST INFRASTRUCTURE ONLY — independent numpy restatement of the reference path.

Used to cross-check the C oracle (oracle/iris_oracle.c) and to produce the
golden fixtures in tests/golden/.  It restates the reference's semantics by
the *formulas* (bit matrix 64 x 200, rotation = np.roll along columns), while
the C oracle restates the reference's byte/carry *algorithm*; agreement of the
two pins the rotation direction and bit order.

Reference citations (recmo/mpc-iris-code v0.8.0):
  bit order        src/bits.rs:44-57 (bit i = limb i/64, bit i%64; LE bytes)
  rotation         src/bits.rs:18-29,178-205; src/encoded_bits.rs:40-52
  dot_bool/dot_u16 src/arch/generic.rs:4-16
  encode           src/lib.rs:16-26
  engines          src/lib.rs:28-94
  decode_distance  src/lib.rs:97-107
  fraction_hamming src/template.rs:49-64, distance src/template.rs:43-47
  argmin           src/main.rs:581-582,616-621
"""
import numpy as np

COLS, ROWS, BITS, LIMBS, ROT = 200, 64, 12800, 200, 31

# ----------------------------------------------------------------- layouts


def bits_to_matrix(limbs):
    """[..., 200] u64 -> [..., 64, 200] u8 of 0/1 (bit i at row i//200, col i%200)."""
    limbs = np.asarray(limbs, dtype="<u8")
    b = np.unpackbits(limbs.view(np.uint8).reshape(limbs.shape[:-1] + (1600,)), axis=-1, bitorder="little")
    return b.reshape(limbs.shape[:-1] + (ROWS, COLS))


def matrix_to_bits(m):
    m = np.asarray(m, dtype=np.uint8).reshape(m.shape[:-2] + (BITS,))
    packed = np.packbits(m, axis=-1, bitorder="little")
    return np.ascontiguousarray(packed).view("<u8").reshape(m.shape[:-1] + (LIMBS,))


# ----------------------------------------------------------------- value types


def bits_rotated(limbs, amount):
    """rot(b, r)[row, col] = b[row, (col - r) mod 200]."""
    return matrix_to_bits(np.roll(bits_to_matrix(limbs), amount, axis=-1))


def encoded_rotated(enc, amount):
    e = np.asarray(enc, dtype=np.uint16).reshape(np.shape(enc)[:-1] + (ROWS, COLS))
    return np.roll(e, amount, axis=-1).reshape(np.shape(enc))


def encoded_from_bits(limbs):
    return bits_to_matrix(limbs).reshape(np.shape(limbs)[:-1] + (BITS,)).astype(np.uint16)


def encode(pattern, mask):
    p = encoded_from_bits(np.asarray(pattern, dtype=np.uint64) & np.asarray(mask, dtype=np.uint64))
    m = encoded_from_bits(mask)
    return (m.astype(np.int64) - 2 * p.astype(np.int64)).astype(np.uint16)


# ----------------------------------------------------------------- arch


def _pc(x):
    # SWAR popcount on uint64 arrays
    x = x - ((x >> np.uint64(1)) & np.uint64(0x5555555555555555))
    x = (x & np.uint64(0x3333333333333333)) + ((x >> np.uint64(2)) & np.uint64(0x3333333333333333))
    x = (x + (x >> np.uint64(4))) & np.uint64(0x0F0F0F0F0F0F0F0F)
    return ((x * np.uint64(0x0101010101010101)) >> np.uint64(56)).astype(np.int64)


def dot_bool(a, b):
    return (_pc(np.asarray(a, np.uint64) & np.asarray(b, np.uint64)).sum(-1) & 0xFFFF).astype(np.uint16)


def dot_u16(a, b):
    prod = (np.asarray(a, np.uint64) * np.asarray(b, np.uint64)) & np.uint64(0xFFFF)
    return (prod.sum(-1) & np.uint64(0xFFFF)).astype(np.uint16)


# ----------------------------------------------------------------- engines


def masks_batch(query_mask, db):
    """MasksEngine::batch_process -> [n, 31] u16."""
    rot = np.stack([bits_rotated(query_mask, k - 15) for k in range(ROT)])  # [31, 200]
    db = np.asarray(db, np.uint64)
    return dot_bool(db[:, None, :], rot[None, :, :])


def distance_batch(query, db):
    """DistanceEngine::batch_process -> [n, 31] u16 (wrapping)."""
    rot = np.stack([encoded_rotated(query, k - 15) for k in range(ROT)]).astype(np.uint64)  # [31, 12800]
    db = np.asarray(db, np.uint64)
    out = np.empty((db.shape[0], ROT), np.uint16)
    for i in range(db.shape[0]):
        out[i] = ((rot * db[i][None, :]) & np.uint64(0xFFFF)).sum(-1) & np.uint64(0xFFFF)
    return out


def template_counts(q_pattern, q_mask, db_pattern, db_mask):
    """num/den per (entry, rotation): [n, 31] int64 each (src/template.rs:49-64)."""
    rp = np.stack([bits_rotated(q_pattern, k - 15) for k in range(ROT)])
    rm = np.stack([bits_rotated(q_mask, k - 15) for k in range(ROT)])
    dp = np.asarray(db_pattern, np.uint64)[:, None, :]
    dm = np.asarray(db_mask, np.uint64)[:, None, :]
    m = rm[None] & dm
    num = _pc((rp[None] ^ dp) & m).sum(-1)
    den = _pc(m).sum(-1)
    return num, den


def rust_min_fold(values, axis=-1):
    """fold(f64::INFINITY, f64::min): NaN ignored."""
    v = np.where(np.isnan(values), np.inf, values)
    return v.min(axis=axis)


def template_distances(q_pattern, q_mask, db_pattern, db_mask):
    num, den = template_counts(q_pattern, q_mask, db_pattern, db_mask)
    with np.errstate(divide="ignore", invalid="ignore"):
        frac = num.astype(np.float64) / den.astype(np.float64)
    return rust_min_fold(frac)


def decode_distance(distances, denominators):
    d = np.asarray(denominators, np.uint16)
    n = np.asarray(distances, np.uint16)
    uneq = ((d.astype(np.int64) - n.astype(np.int64)) & 0xFFFF) // 2
    with np.errstate(divide="ignore", invalid="ignore"):
        frac = uneq.astype(np.float64) / d.astype(np.float64)
    return rust_min_fold(frac)


def argmin(dist):
    """Strict <, lowest index wins; +inf never selected (index = 2**64-1)."""
    dist = np.asarray(dist, np.float64)
    best, idx = np.inf, 2**64 - 1
    finite = np.where(dist < np.inf)[0]
    if finite.size:
        j = int(finite[np.argmin(dist[finite])])
        best, idx = float(dist[j]), j
    return best, idx


# ----------------------------------------------------------------- generator

_M1, _M2, _G, _K = 0xBF58476D1CE4E5B9, 0x94D049BB133111EB, 0x9E3779B97F4A7C15, 0xD1B54A32D192ED03
_MASK = (1 << 64) - 1


def _mix64_int(z):
    z = ((z ^ (z >> 30)) * _M1) & _MASK
    z = ((z ^ (z >> 27)) * _M2) & _MASK
    return z ^ (z >> 31)


def _mix64_np(z):
    z = np.asarray(z, np.uint64)
    with np.errstate(over="ignore"):
        z = (z ^ (z >> np.uint64(30))) * np.uint64(_M1)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(_M2)
    return z ^ (z >> np.uint64(31))


def gen_limbs(seed, stream, ctr):
    key = _mix64_int((seed ^ ((_K * (stream + 1)) & _MASK)) & _MASK)
    ctr = np.asarray(ctr, np.uint64)
    with np.errstate(over="ignore"):
        z = np.uint64(key) + (ctr + np.uint64(1)) * np.uint64(_G)
    return _mix64_np(z)


def gen_templates(seed, t0, n):
    """-> (pattern [n,200], mask [n,200]) u64."""
    t = np.arange(t0, t0 + n, dtype=np.uint64)[:, None]
    j = np.arange(LIMBS, dtype=np.uint64)[None, :]
    pattern = gen_limbs(seed, 0, t * np.uint64(400) + j)
    mask = gen_limbs(seed, 0, t * np.uint64(400) + np.uint64(200) + j)
    return pattern, mask


def gen_shares(seed, t0, n):
    t = np.arange(t0, t0 + n, dtype=np.uint64)[:, None]
    j = np.arange(BITS // 4, dtype=np.uint64)[None, :]
    limbs = np.ascontiguousarray(gen_limbs(seed, 1, t * np.uint64(3200) + j))
    return limbs.view("<u2").reshape(n, BITS)


# ---------------------------------------------------------------- share preparation (§8(f) row 4)

def _rotl32(x, r):
    return ((x << np.uint32(r)) | (x >> np.uint32(32 - r))).astype(np.uint32)


def chacha_blocks(key, nonce, counters, rounds=20):
    """Vectorised ChaCha blocks (DJB: 64-bit nonce, 64-bit counter; 8/12/20 rounds; rand_chacha
    0.3.1's layout) -> uint8 [len(counters), 64]."""
    k = np.frombuffer(bytes(key), "<u4")
    c = np.asarray(counters, np.uint64)
    n = c.size
    st = np.empty((16, n), np.uint32)
    st[0:4] = np.array([0x61707865, 0x3320646E, 0x79622D32, 0x6B206574], np.uint32)[:, None]
    st[4:12] = k[:, None]
    st[12] = (c & np.uint64(0xFFFFFFFF)).astype(np.uint32)
    st[13] = (c >> np.uint64(32)).astype(np.uint32)
    st[14] = np.uint32(nonce & 0xFFFFFFFF)
    st[15] = np.uint32(nonce >> 32)
    x = st.copy()

    def qr(a, b, cc, d):
        x[a] += x[b]; x[d] = _rotl32(x[d] ^ x[a], 16)
        x[cc] += x[d]; x[b] = _rotl32(x[b] ^ x[cc], 12)
        x[a] += x[b]; x[d] = _rotl32(x[d] ^ x[a], 8)
        x[cc] += x[d]; x[b] = _rotl32(x[b] ^ x[cc], 7)

    for _ in range(rounds // 2):
        qr(0, 4, 8, 12); qr(1, 5, 9, 13); qr(2, 6, 10, 14); qr(3, 7, 11, 15)
        qr(0, 5, 10, 15); qr(1, 6, 11, 12); qr(2, 7, 8, 13); qr(3, 4, 9, 14)
    out = (x + st).astype("<u4").T.copy()
    return out.view(np.uint8).reshape(n, 64)


def prepare_shares(templates, key, nonce=0, parties=3, index_base=0, rounds=12):
    """EncodedBits::share (src/encoded_bits.rs:23-38) with the counter-mode ChaCha
    derivation of oracle/iris_oracle.h (12 rounds: rand 0.8.5's thread_rng core):
    shares [parties][n][12800], masks [n][200]."""
    t = np.asarray(templates, np.uint64).reshape(-1, 400)
    n = t.shape[0]
    shares = np.zeros((parties, n, 12800), np.uint16)
    for i in range(n):
        g = index_base + i
        last = encode(t[i, :200], t[i, 200:]).astype(np.uint16)
        for j in range(parties - 1):
            ctr = (g * (parties - 1) + j) * 400 + np.arange(400, dtype=np.uint64)
            sh = chacha_blocks(key, nonce, ctr, rounds).view("<u2").reshape(12800)
            shares[j, i] = sh
            last = (last - sh).astype(np.uint16)
        shares[parties - 1, i] = last
    return shares, t[:, 200:].copy()
