"""TEST INFRASTRUCTURE ONLY — ctypes binding of the C oracle (oracle/liboracle.so).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg use this.
"""
import ctypes
import os
import pathlib

import numpy as np

HERE = pathlib.Path(__file__).resolve().parent
ROT, LIMBS, BITS = 31, 200, 12800

_lib = None


def build(path=None, march="x86-64-v3"):
    """Compile the oracle (gcc) into `path` (default oracle/liboracle.so)."""
    import subprocess

    out = pathlib.Path(path) if path else HERE / "liboracle.so"
    cmd = ["gcc", "-O3", f"-march={march}", "-fPIC", "-std=c11", "-pthread", "-shared", "-o", str(out),
           str(HERE / "iris_oracle.c"), "-lm"]
    subprocess.run(cmd, check=True)
    return out


def load(path=None):
    global _lib
    if path is None and _lib is not None:
        return _lib
    p = pathlib.Path(path) if path else HERE / "liboracle.so"
    if not p.exists():
        build(p)
    lib = ctypes.CDLL(str(p))
    P = ctypes.c_void_p
    u64, i32 = ctypes.c_uint64, ctypes.c_int
    lib.orc_bits_rotated.argtypes = [P, i32, P]
    lib.orc_encoded_rotated.argtypes = [P, i32, P]
    lib.orc_encode.argtypes = [P, P]
    lib.orc_dot_bool.argtypes = [P, P]
    lib.orc_dot_bool.restype = ctypes.c_uint16
    lib.orc_dot_u16.argtypes = [P, P]
    lib.orc_dot_u16.restype = ctypes.c_uint16
    lib.orc_dot_bool_pairs.argtypes = [P, u64, P, u64, P]
    lib.orc_dot_u16_pairs.argtypes = [P, u64, P, u64, P]
    lib.orc_masks_batch.argtypes = [P, P, u64, P, i32]
    lib.orc_distance_batch.argtypes = [P, P, u64, P, i32]
    lib.orc_template_distance.argtypes = [P, P]
    lib.orc_template_distance.restype = ctypes.c_double
    lib.orc_template_counts_batch.argtypes = [P, P, u64, P, P, i32]
    lib.orc_template_distances_batch.argtypes = [P, P, u64, P, i32]
    lib.orc_decode_distance.argtypes = [P, P]
    lib.orc_decode_distance.restype = ctypes.c_double
    lib.orc_argmin.argtypes = [P, u64, P, P]
    lib.orc_resolver_combine.argtypes = [P, ctypes.c_uint32, P, u64, P, ctypes.c_int]
    lib.orc_gen_templates.argtypes = [u64, u64, u64, P]
    lib.orc_gen_masks.argtypes = [u64, u64, u64, P]
    lib.orc_gen_shares.argtypes = [u64, u64, u64, P]
    lib.orc_chacha_block.argtypes = [P, u64, u64, ctypes.c_uint32, P]
    lib.orc_prepare_shares.argtypes = [P, u64, u64, P, u64, ctypes.c_uint32, ctypes.c_uint32, P, P, ctypes.c_int]
    if path is None:
        _lib = lib
    return lib


def _p(a):
    return a.ctypes.data_as(ctypes.c_void_p)


def _threads(threads):
    return threads if threads else min(16, os.cpu_count() or 1)


def templates_array(pattern, mask):
    """[n,200] pattern + [n,200] mask -> [n,400] u64 in Template layout (pattern first)."""
    return np.ascontiguousarray(np.concatenate([np.asarray(pattern, np.uint64), np.asarray(mask, np.uint64)], axis=-1))


def bits_rotated(limbs, amount):
    a = np.ascontiguousarray(limbs, np.uint64)
    out = np.empty(LIMBS, np.uint64)
    load().orc_bits_rotated(_p(a), int(amount), _p(out))
    return out


def encoded_rotated(enc, amount):
    a = np.ascontiguousarray(enc, np.uint16)
    out = np.empty(BITS, np.uint16)
    load().orc_encoded_rotated(_p(a), int(amount), _p(out))
    return out


def encode(template):
    t = np.ascontiguousarray(template, np.uint64)
    out = np.empty(BITS, np.uint16)
    load().orc_encode(_p(t), _p(out))
    return out


def dot_bool(a, b):
    return int(load().orc_dot_bool(_p(np.ascontiguousarray(a, np.uint64)), _p(np.ascontiguousarray(b, np.uint64))))


def dot_u16(a, b):
    return int(load().orc_dot_u16(_p(np.ascontiguousarray(a, np.uint16)), _p(np.ascontiguousarray(b, np.uint16))))


def dot_bool_pairs(a, b):
    """out[j, i] = dot_bool(a[i], b[j]), the criterion loop order (src/arch/mod.rs:34-41)."""
    a = np.ascontiguousarray(a, np.uint64).reshape(-1, LIMBS)
    b = np.ascontiguousarray(b, np.uint64).reshape(-1, LIMBS)
    out = np.empty((b.shape[0], a.shape[0]), np.uint16)
    load().orc_dot_bool_pairs(_p(a), a.shape[0], _p(b), b.shape[0], _p(out))
    return out


def dot_u16_pairs(a, b):
    """out[j, i] = dot_u16(a[i], b[j]) (src/arch/mod.rs:62-69)."""
    a = np.ascontiguousarray(a, np.uint16).reshape(-1, BITS)
    b = np.ascontiguousarray(b, np.uint16).reshape(-1, BITS)
    out = np.empty((b.shape[0], a.shape[0]), np.uint16)
    load().orc_dot_u16_pairs(_p(a), a.shape[0], _p(b), b.shape[0], _p(out))
    return out


def masks_batch(query_mask, db, threads=None):
    db = np.ascontiguousarray(db, np.uint64)
    n = db.shape[0]
    out = np.empty((n, ROT), np.uint16)
    load().orc_masks_batch(_p(np.ascontiguousarray(query_mask, np.uint64)), _p(db), n, _p(out), _threads(threads))
    return out


def distance_batch(query, db, threads=None):
    db = np.ascontiguousarray(db, np.uint16)
    n = db.shape[0]
    out = np.empty((n, ROT), np.uint16)
    load().orc_distance_batch(_p(np.ascontiguousarray(query, np.uint16)), _p(db), n, _p(out), _threads(threads))
    return out


def template_counts(query, db, threads=None):
    """query [400] u64 (Template), db [n,400] -> (num [n,31], den [n,31]) u16."""
    db = np.ascontiguousarray(db, np.uint64)
    n = db.shape[0]
    num = np.empty((n, ROT), np.uint16)
    den = np.empty((n, ROT), np.uint16)
    load().orc_template_counts_batch(_p(np.ascontiguousarray(query, np.uint64)), _p(db), n, _p(num), _p(den),
                                     _threads(threads))
    return num, den


def template_distances(query, db, threads=None):
    db = np.ascontiguousarray(db, np.uint64)
    n = db.shape[0]
    out = np.empty(n, np.float64)
    load().orc_template_distances_batch(_p(np.ascontiguousarray(query, np.uint64)), _p(db), n, _p(out),
                                        _threads(threads))
    return out


def template_distance(a, b):
    return float(load().orc_template_distance(_p(np.ascontiguousarray(a, np.uint64)),
                                              _p(np.ascontiguousarray(b, np.uint64))))


def decode_distance(distances, denominators):
    return float(load().orc_decode_distance(_p(np.ascontiguousarray(distances, np.uint16)),
                                            _p(np.ascontiguousarray(denominators, np.uint16))))


def argmin(dist):
    dist = np.ascontiguousarray(dist, np.float64)
    d = np.zeros(1, np.float64)
    i = np.zeros(1, np.uint64)
    load().orc_argmin(_p(dist), dist.shape[0], _p(d), _p(i))
    return float(d[0]), int(i[0])


def resolver_combine(shares, denoms, threads=None):
    shares = np.ascontiguousarray(shares, np.uint16)  # [parts, n, 31]
    denoms = np.ascontiguousarray(denoms, np.uint16)  # [n, 31]
    parts, n = shares.shape[0], shares.shape[1]
    out = np.empty(n, np.float64)
    load().orc_resolver_combine(_p(shares), parts, _p(denoms), n, _p(out), _threads(threads))
    return out


def gen_templates(seed, t0, n):
    out = np.empty((n, 400), np.uint64)
    load().orc_gen_templates(seed, t0, n, _p(out))
    return out


def gen_masks(seed, t0, n):
    out = np.empty((n, LIMBS), np.uint64)
    load().orc_gen_masks(seed, t0, n, _p(out))
    return out


def gen_shares(seed, t0, n):
    out = np.empty((n, BITS), np.uint16)
    load().orc_gen_shares(seed, t0, n, _p(out))
    return out


def chacha_block(key, nonce, counter, rounds=20):
    """64 keystream bytes (DJB ChaCha, 8/12/20 rounds: 64-bit nonce, 64-bit block counter)."""
    k = np.frombuffer(bytes(key), np.uint8).copy()
    assert k.size == 32
    out = np.zeros(64, np.uint8)
    load().orc_chacha_block(_p(k), int(nonce), int(counter), int(rounds), _p(out))
    return out.tobytes()


def prepare_shares(templates, key, nonce=0, parties=3, index_base=0, rounds=12, threads=None):
    """EncodedBits::share of encode(t) with the ChaCha stream of orc_prepare_shares:
    returns (shares [parties][n][12800] u16, masks [n][200] u64)."""
    t = np.ascontiguousarray(np.asarray(templates, np.uint64).reshape(-1, 400))
    n = t.shape[0]
    k = np.frombuffer(bytes(key), np.uint8).copy()
    assert k.size == 32
    shares = np.zeros((parties, n, 12800), np.uint16)
    masks = np.zeros((n, 200), np.uint64)
    load().orc_prepare_shares(_p(t), n, int(index_base), _p(k), int(nonce), int(rounds), int(parties), _p(shares),
                              _p(masks), _threads(threads))
    return shares, masks
