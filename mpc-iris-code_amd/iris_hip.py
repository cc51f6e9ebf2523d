"""iris_hip — Python mirror of the reference's engine API over the C ABI.

Mirrors recmo/mpc-iris-code (v0.8.0) names and argument meaning:

    reference (Rust)                              here
    Bits / EncodedBits / Template (value types)   Bits / EncodedBits / Template
    encode(&Template) -> EncodedBits              encode(template)          src/lib.rs:16-26
    DistanceEngine::new / batch_process           DistanceEngine            src/lib.rs:28-53
    MasksEngine::new / batch_process              MasksEngine               src/lib.rs:55-80
    distances / denominators                      distances / denominators  src/lib.rs:82-94
    decode_distance                               decode_distance           src/lib.rs:97-107
    Template::distance / fraction_hamming         TemplateEngine            src/template.rs:43-64
    arch::dot_bool / arch::dot_u16                dot_bool / dot_u16        src/arch/generic.rs:4-16

Every compute call goes to libiris_hip.so (hand-written gfx950 kernels).  If
the library or a gfx950 device is missing the calls raise — there is no CPU
fallback in this module.
"""
from __future__ import annotations

import ctypes
import math
import os
import pathlib
import threading

import numpy as np

HERE = pathlib.Path(__file__).resolve().parent
# IRIS_HIP_LIB points at an alternative in-tree build (kernel experiments under tools/)
LIB_PATH = pathlib.Path(os.environ.get("IRIS_HIP_LIB", HERE / "libiris_hip.so"))


def _load_pycall():
    """The per-call fast path (csrc/iris_pycall.c, built beside the library and linked to it): the
    host-slice engine call without ctypes' per-call marshalling; None where it is not built or a
    non-default library is in use (IRIS_HIP_LIB).  Loaded on the first such call, after
    load_library(), so that importing this module loads no HIP runtime: a process that imports
    torch later (bench.py's ranks) keeps the load order it had without the fast path (torch bundles
    its own libamdhip64.so.7; whichever is mapped first serves both)."""
    global _pycall
    with _lock:
        if _pycall is not _UNLOADED:
            return _pycall
        _pycall = None
        p = HERE / "_iris_pycall.so"
        if "IRIS_HIP_LIB" in os.environ or not p.exists():
            return None
        import importlib.util
        try:
            spec = importlib.util.spec_from_file_location("_iris_pycall", p)
            mod = importlib.util.module_from_spec(spec)
            spec.loader.exec_module(mod)
        except (ImportError, OSError):
            return None
        _pycall = mod
        return mod


_UNLOADED = object()
_pycall = _UNLOADED
_NULL = ctypes.c_void_p()

COLS, ROWS, BITS, LIMBS, ROTATIONS = 200, 64, 12800, 200, 31
KIND_MASKS, KIND_SHARES, KIND_TEMPLATES = 1, 2, 3
LAYOUT_DEFAULT, LAYOUT_LANES, LAYOUT_TILES = 0, 1, 2
_REC_DTYPE = {KIND_MASKS: (np.uint64, LIMBS), KIND_SHARES: (np.uint16, BITS), KIND_TEMPLATES: (np.uint64, 2 * LIMBS)}


class IrisError(RuntimeError):
    def __init__(self, code, msg):
        super().__init__(f"iris_hip error {code}: {msg}")
        self.code = code


class Match(ctypes.Structure):
    """iris_match_t: the resolver's (min_distance, min_index) (src/main.rs:581-621)."""

    _fields_ = [("distance", ctypes.c_double), ("index", ctypes.c_uint64), ("num", ctypes.c_uint32),
                ("den", ctypes.c_uint32), ("rotation", ctypes.c_int32), ("reserved", ctypes.c_uint32)]

    def __repr__(self):
        return (f"Match(distance={self.distance!r}, index={self.index}, num={self.num}, den={self.den}, "
                f"rotation={self.rotation})")


_lib = None
_lock = threading.Lock()


def load_library(path=None):
    """Load libiris_hip.so (fails loudly when it is absent)."""
    global _lib
    if _lib is not None and path is None:  # per-call fast path: no lock once loaded
        return _lib
    with _lock:
        if _lib is not None and path is None:
            return _lib
        p = pathlib.Path(path) if path else LIB_PATH
        if not p.exists():
            raise IrisError(-4, f"{p} not built: run `make -C {HERE}` (or __graft_entry__.build())")
        lib = ctypes.CDLL(str(p))
        P, u64, i32 = ctypes.c_void_p, ctypes.c_uint64, ctypes.c_int32
        PP = ctypes.POINTER(ctypes.c_void_p)
        sig = {
            "iris_last_error": ([], ctypes.c_char_p),
            "iris_version": ([], ctypes.c_char_p),
            "iris_config": ([P, ctypes.c_char_p, ctypes.c_size_t, ctypes.POINTER(ctypes.c_size_t)], ctypes.c_int),
            "iris_device_count": ([ctypes.POINTER(ctypes.c_int)], ctypes.c_int),
            "iris_device_open": ([ctypes.c_int, PP], ctypes.c_int),
            "iris_device_close": ([P], ctypes.c_int),
            "iris_device_synchronize": ([P], ctypes.c_int),
            "iris_device_stream": ([P, PP], ctypes.c_int),
            "iris_device_memory": ([P, ctypes.POINTER(ctypes.c_size_t), ctypes.POINTER(ctypes.c_size_t)],
                                   ctypes.c_int),
            "iris_template_search_async": ([P, P, u64, u64, u64, PP], ctypes.c_int),
            "iris_pending_wait": ([P, ctypes.POINTER(Match)], ctypes.c_int),
            "iris_device_set_profiling": ([P, ctypes.c_int], ctypes.c_int),
            "iris_device_kernel_stats": ([P, ctypes.c_char_p, ctypes.POINTER(u64), ctypes.POINTER(ctypes.c_double),
                                          ctypes.POINTER(u64)], ctypes.c_int),
            "iris_device_reset_stats": ([P], ctypes.c_int),
            "iris_device_alloc": ([P, ctypes.c_size_t, PP], ctypes.c_int),
            "iris_device_free": ([P, P], ctypes.c_int),
            "iris_device_drop_resident": ([P], ctypes.c_int),
            "iris_device_drop_resident_range": ([P, P], ctypes.c_int),
            "iris_device_kernel_stats_largest": ([P, ctypes.c_char_p, ctypes.POINTER(u64), ctypes.POINTER(ctypes.c_double)],
                                                 ctypes.c_int),
            "iris_memcpy_d2h": ([P, P, P, ctypes.c_size_t], ctypes.c_int),
            "iris_db_create": ([P, ctypes.c_int, u64, PP], ctypes.c_int),
            "iris_db_create_ex": ([P, ctypes.c_int, u64, ctypes.c_int, PP], ctypes.c_int),
            "iris_db_layout": ([P, ctypes.POINTER(ctypes.c_int)], ctypes.c_int),
            "iris_db_destroy": ([P], ctypes.c_int),
            "iris_db_len": ([P, ctypes.POINTER(u64)], ctypes.c_int),
            "iris_db_capacity": ([P, ctypes.POINTER(u64)], ctypes.c_int),
            "iris_db_kind": ([P, ctypes.POINTER(ctypes.c_int)], ctypes.c_int),
            "iris_db_append": ([P, P, u64], ctypes.c_int),
            "iris_db_write": ([P, u64, P, u64], ctypes.c_int),
            "iris_db_read": ([P, u64, u64, P], ctypes.c_int),
            "iris_db_generate": ([P, u64, u64, u64], ctypes.c_int),
            "iris_db_clear": ([P], ctypes.c_int),
            "iris_db_truncate": ([P, u64], ctypes.c_int),
            "iris_memcpy_h2d": ([P, P, P, ctypes.c_size_t], ctypes.c_int),
            "iris_db_load_file": ([P, ctypes.c_char_p, u64, u64, ctypes.POINTER(u64)], ctypes.c_int),
            "iris_db_save_file": ([P, ctypes.c_char_p, u64, u64], ctypes.c_int),
            "iris_templates_read_json": ([ctypes.c_char_p, P, u64, ctypes.POINTER(u64)], ctypes.c_int),
            "iris_templates_write_json": ([ctypes.c_char_p, P, u64], ctypes.c_int),
            "iris_resolver_search_masks": ([P, P, u64, u64, P, ctypes.c_uint32, u64, P, ctypes.POINTER(Match)],
                                           ctypes.c_int),
            "iris_resolver_search_masks_host": ([P, P, u64, u64, P, ctypes.c_uint32, u64, ctypes.POINTER(Match)],
                                                ctypes.c_int),
            "iris_prepare_shares": ([P, u64, u64, u64, P, u64, ctypes.c_uint32, ctypes.c_uint32, P, P], ctypes.c_int),
            "iris_masks_engine_new": ([P, P, PP], ctypes.c_int),
            "iris_distance_engine_new": ([P, P, PP], ctypes.c_int),
            "iris_template_engine_new": ([P, P, PP], ctypes.c_int),
            "iris_engine_destroy": ([P], ctypes.c_int),
            "iris_engine_batch_process": ([P, P, u64, u64, P], ctypes.c_int),
            "iris_engine_batch_process_host": ([P, P, u64, P], ctypes.c_int),
            "iris_engine_batch_process_device": ([P, P, u64, u64, P], ctypes.c_int),
            "iris_template_counts": ([P, P, u64, u64, P, P], ctypes.c_int),
            "iris_template_distances": ([P, P, u64, u64, P], ctypes.c_int),
            "iris_template_search": ([P, P, u64, u64, u64, P, ctypes.POINTER(Match)], ctypes.c_int),
            "iris_template_batch_engine_new": ([P, P, ctypes.c_uint32, PP], ctypes.c_int),
            "iris_template_batch_search": ([P, P, u64, u64, u64, ctypes.POINTER(Match)], ctypes.c_int),
            "iris_resolver_search": ([P, ctypes.POINTER(ctypes.c_void_p), ctypes.c_uint32, P, u64, u64, P,
                                      ctypes.POINTER(Match)], ctypes.c_int),
            "iris_resolver_search_host": ([P, ctypes.POINTER(ctypes.c_void_p), ctypes.c_uint32, P, u64, u64,
                                           ctypes.POINTER(Match)], ctypes.c_int),
            "iris_dot_bool_batch": ([P, P, u64, P, u64, P], ctypes.c_int),
            "iris_dot_u16_batch": ([P, P, u64, P, u64, P], ctypes.c_int),
            "iris_bits_rotated": ([P, i32, P], ctypes.c_int),
            "iris_encoded_rotated": ([P, i32, P], ctypes.c_int),
            "iris_encode": ([P, P], ctypes.c_int),
            "iris_decode_distance": ([P, P, ctypes.POINTER(ctypes.c_double)], ctypes.c_int),
            "iris_match_merge": ([ctypes.POINTER(Match), u64, ctypes.POINTER(Match)], ctypes.c_int),
            "iris_query_table_sizes": ([ctypes.c_int, ctypes.c_uint32, ctypes.POINTER(ctypes.c_size_t),
                                        ctypes.POINTER(ctypes.c_size_t)], ctypes.c_int),
            "iris_engine_query_tables": ([P, P, ctypes.c_size_t, P, ctypes.c_size_t], ctypes.c_int),
            "iris_host_query_tables": ([ctypes.c_int, P, ctypes.c_uint32, P, ctypes.c_size_t, P, ctypes.c_size_t],
                                       ctypes.c_int),
            "iris_db_attach_host": ([P, P, u64, ctypes.c_int], ctypes.c_int),
            "iris_db_detach_host": ([P], ctypes.c_int),
            "iris_group_create": ([ctypes.POINTER(ctypes.c_int), ctypes.c_uint32, PP], ctypes.c_int),
            "iris_group_unique_id": ([P], ctypes.c_int),
            "iris_group_create_rank": ([ctypes.c_int, ctypes.c_uint32, ctypes.c_uint32, P, PP], ctypes.c_int),
            "iris_group_destroy": ([P], ctypes.c_int),
            "iris_group_set_timeout": ([P, ctypes.c_uint32], ctypes.c_int),
            "iris_group_info": ([P, ctypes.POINTER(ctypes.c_uint32), ctypes.POINTER(ctypes.c_uint32),
                                 ctypes.POINTER(ctypes.c_uint32)], ctypes.c_int),
            "iris_group_device": ([P, ctypes.c_uint32, PP], ctypes.c_int),
            "iris_group_rccl_info": ([P, ctypes.POINTER(ctypes.c_uint32), ctypes.c_char_p, ctypes.c_size_t], ctypes.c_int),
            "iris_group_db_create": ([P, ctypes.c_int, u64, ctypes.c_int, ctypes.c_uint32, PP], ctypes.c_int),
            "iris_group_db_destroy": ([P], ctypes.c_int),
            "iris_group_db_info": ([P, ctypes.POINTER(u64), ctypes.POINTER(ctypes.c_uint32),
                                    ctypes.POINTER(ctypes.c_uint32), ctypes.POINTER(ctypes.c_uint32)], ctypes.c_int),
            "iris_group_db_shard": ([P, ctypes.c_uint32, PP, ctypes.POINTER(u64), ctypes.POINTER(u64)], ctypes.c_int),
            "iris_group_db_generate": ([P, u64], ctypes.c_int),
            "iris_group_db_write": ([P, u64, P, u64], ctypes.c_int),
            "iris_group_db_read": ([P, u64, u64, P], ctypes.c_int),
            "iris_group_db_load_file": ([P, ctypes.c_char_p, u64], ctypes.c_int),
            "iris_group_template_search": ([P, P, ctypes.POINTER(Match)], ctypes.c_int),
            "iris_group_template_search_async": ([P, P, PP], ctypes.c_int),
            "iris_group_pending_wait": ([P, ctypes.POINTER(Match)], ctypes.c_int),
            "iris_group_template_batch_search": ([P, P, ctypes.c_uint32, ctypes.POINTER(Match)], ctypes.c_int),
        }
        for name, (args, res) in sig.items():
            f = getattr(lib, name)
            f.argtypes = args
            f.restype = res
        if path is None:
            _lib = lib
        return lib


def exported_symbols():
    return [
        "iris_last_error", "iris_version", "iris_config", "iris_device_count", "iris_device_open", "iris_device_close",
        "iris_device_synchronize", "iris_device_stream", "iris_device_set_profiling", "iris_device_kernel_stats",
        "iris_device_reset_stats", "iris_device_alloc", "iris_device_free", "iris_device_drop_resident",
        "iris_device_drop_resident_range", "iris_device_kernel_stats_largest",
        "iris_memcpy_d2h", "iris_db_create",
        "iris_db_create_ex", "iris_db_layout",
        "iris_db_destroy", "iris_db_len", "iris_db_capacity", "iris_db_kind", "iris_db_append", "iris_db_write",
        "iris_db_read", "iris_db_generate", "iris_db_clear", "iris_masks_engine_new", "iris_distance_engine_new",
        "iris_template_engine_new", "iris_engine_destroy", "iris_engine_batch_process",
        "iris_engine_batch_process_host", "iris_engine_batch_process_device", "iris_template_counts", "iris_template_distances", "iris_template_search",
        "iris_template_batch_engine_new", "iris_template_batch_search", "iris_resolver_search",
        "iris_resolver_search_host", "iris_dot_bool_batch", "iris_dot_u16_batch", "iris_bits_rotated", "iris_encoded_rotated", "iris_encode",
        "iris_decode_distance", "iris_match_merge", "iris_db_load_file", "iris_db_save_file",
        "iris_templates_read_json", "iris_templates_write_json", "iris_prepare_shares",
        "iris_db_truncate", "iris_memcpy_h2d", "iris_resolver_search_masks", "iris_resolver_search_masks_host",
        "iris_query_table_sizes", "iris_engine_query_tables", "iris_host_query_tables", "iris_device_memory",
        "iris_template_search_async", "iris_pending_wait",
        "iris_db_attach_host", "iris_db_detach_host",
        "iris_group_create", "iris_group_unique_id", "iris_group_create_rank", "iris_group_destroy", "iris_group_set_timeout", "iris_group_info",
        "iris_group_device", "iris_group_rccl_info", "iris_group_db_create", "iris_group_db_destroy", "iris_group_db_info",
        "iris_group_db_shard", "iris_group_db_generate", "iris_group_db_write", "iris_group_db_read",
        "iris_group_db_load_file", "iris_group_template_search", "iris_group_template_search_async",
        "iris_group_pending_wait", "iris_group_template_batch_search",
    ]


def query_table_sizes(kind, nq=0):
    """(table bytes, fragment bytes) of an engine's rotated-query tables."""
    tb, fb = ctypes.c_size_t(), ctypes.c_size_t()
    _check(load_library().iris_query_table_sizes(int(kind), int(nq), ctypes.byref(tb), ctypes.byref(fb)))
    return tb.value, fb.value


def host_query_tables(kind, query, nq=0):
    """The rotated-query table and MFMA fragments of `query` built by the host reference
    builders (CPU only) -> (table uint8 array, fragments uint8 array)."""
    tb, fb = query_table_sizes(kind, nq)
    q = np.ascontiguousarray(query)
    tab, frag = np.zeros(tb, np.uint8), np.zeros(fb, np.uint8)
    _check(load_library().iris_host_query_tables(int(kind), _ptr(q), int(nq), _ptr(tab) if tb else None, tb,
                                                 _ptr(frag), fb))
    return tab, frag


def read_templates_json(path):
    """JSON array of {"pattern": hex, "mask": hex} (src/bits.rs:74-93) -> uint64 [n, 400]
    (pattern limbs then mask limbs, the Template byte layout)."""
    lib = load_library()
    n = ctypes.c_uint64(0)
    _check(lib.iris_templates_read_json(os.fsencode(path), None, 0, ctypes.byref(n)))
    out = np.zeros((n.value, 2 * LIMBS), np.uint64)
    if n.value:
        _check(lib.iris_templates_read_json(os.fsencode(path), _ptr(out), n.value, ctypes.byref(n)))
    return out


def write_templates_json(path, templates):
    """Inverse of read_templates_json (compact JSON, lowercase hex)."""
    a = np.ascontiguousarray(np.asarray(templates, np.uint64).reshape(-1, 2 * LIMBS))
    _check(load_library().iris_templates_write_json(os.fsencode(path), _ptr(a), a.shape[0]))


def prepare_shares(templates, shares, masks=None, key=None, nonce=0, first=0, n=None, index_base=0, rounds=12):
    """`prepare` on the device (src/main.rs:333-361): appends EncodedBits::share(len(shares))
    of encode(templates[first:first+n]) to the share Databases and, optionally, the masks to
    a masks Database.  key: 32 bytes (default: os.urandom, a CSPRNG).  rounds: ChaCha8/12/20;
    12 is the reference's generator (rand 0.8.5 thread_rng = ChaCha12).  Returns the key."""
    if key is None:
        key = os.urandom(32)
    key = bytes(key)
    if len(key) != 32:
        raise ValueError("key must be 32 bytes")
    if n is None:
        n = len(templates) - int(first)
    kbuf = (ctypes.c_uint8 * 32).from_buffer_copy(key)
    arr = (ctypes.c_void_p * len(shares))(*[s.handle for s in shares])
    _check(load_library().iris_prepare_shares(templates.handle, int(first), int(n), int(index_base), kbuf,
                                              int(nonce), int(rounds), len(shares), arr,
                                              masks.handle if masks is not None else None))
    return key


def _check(rc):
    if rc != 0:
        raise IrisError(rc, load_library().iris_last_error().decode(errors="replace"))


def _ptr(a):
    return a.ctypes.data_as(ctypes.c_void_p)


def _c(a, dtype):
    return np.ascontiguousarray(a, dtype=dtype)


# ====================================================================== value types


class Bits:
    """12 800-bit vector, `[u64; 200]` (src/bits.rs:13-15)."""

    __slots__ = ("limbs",)

    def __init__(self, limbs=None):
        self.limbs = np.zeros(LIMBS, np.uint64) if limbs is None else _c(limbs, np.uint64).reshape(LIMBS).copy()

    @classmethod
    def random(cls, rng):
        return cls(rng.integers(0, 2**64, LIMBS, dtype=np.uint64))

    def __getitem__(self, i):  # Index<usize> (src/bits.rs:44-57)
        if not 0 <= i < BITS:
            raise IndexError(i)
        return bool((int(self.limbs[i // 64]) >> (i % 64)) & 1)

    def __eq__(self, other):
        return isinstance(other, Bits) and bool((self.limbs == other.limbs).all())

    def rotated(self, amount):
        out = np.empty(LIMBS, np.uint64)
        _check(load_library().iris_bits_rotated(_ptr(self.limbs), int(amount), _ptr(out)))
        return Bits(out)

    def count_ones(self):
        return int(np.unpackbits(self.limbs.view(np.uint8)).sum())

    def __and__(self, other):
        return Bits(self.limbs & other.limbs)

    def __or__(self, other):
        return Bits(self.limbs | other.limbs)

    def __xor__(self, other):
        return Bits(self.limbs ^ other.limbs)

    def __invert__(self):
        return Bits(~self.limbs)

    def dot(self, other):  # Bits::dot -> arch::dot_bool (src/bits.rs:35-37)
        return dot_bool(self, other)

    def to_hex(self):  # serde: hex of the LE bytes (src/bits.rs:74-81)
        return self.limbs.astype("<u8").tobytes().hex()

    @classmethod
    def from_hex(cls, s):
        b = bytes.fromhex(s)
        if len(b) != 1600:
            raise ValueError("expected 1600 bytes")
        return cls(np.frombuffer(b, "<u8"))


class EncodedBits:
    """`[u16; 12800]` ring vector (src/encoded_bits.rs:13-15)."""

    __slots__ = ("values",)

    def __init__(self, values=None):
        self.values = np.zeros(BITS, np.uint16) if values is None else _c(values, np.uint16).reshape(BITS).copy()

    @classmethod
    def random(cls, rng):
        return cls(rng.integers(0, 2**16, BITS, dtype=np.uint16))

    @classmethod
    def from_bits(cls, bits):  # From<&Bits> (src/encoded_bits.rs:75-79)
        return cls(np.unpackbits(bits.limbs.view(np.uint8), bitorder="little").astype(np.uint16))

    def __eq__(self, other):
        return isinstance(other, EncodedBits) and bool((self.values == other.values).all())

    def rotated(self, amount):
        out = np.empty(BITS, np.uint16)
        _check(load_library().iris_encoded_rotated(_ptr(self.values), int(amount), _ptr(out)))
        return EncodedBits(out)

    def sum(self):
        return int(self.values.astype(np.uint64).sum() & 0xFFFF)

    def __add__(self, other):
        return EncodedBits(self.values + other.values)

    def __sub__(self, other):
        return EncodedBits(self.values - other.values)

    def __mul__(self, other):
        return EncodedBits(self.values * other.values)

    def __neg__(self):
        return EncodedBits(np.uint16(0) - self.values)

    def dot(self, other):  # EncodedBits::dot -> arch::dot_u16 (src/encoded_bits.rs:64-66)
        return dot_u16(self, other)

    def share(self, n, rng):
        """n additive shares mod 2^16 (src/encoded_bits.rs:23-38); host-side offline prep."""
        assert n > 0
        shares = [EncodedBits.random(rng) for _ in range(n - 1)]
        acc = np.zeros(BITS, np.uint16)
        for s in shares:
            acc = acc + s.values
        shares.append(EncodedBits(self.values - acc))
        return shares


class Template:
    """`#[repr(C)] { pattern: Bits, mask: Bits }` (src/template.rs:11-29)."""

    __slots__ = ("pattern", "mask")

    def __init__(self, pattern=None, mask=None):
        self.pattern = pattern if isinstance(pattern, Bits) else Bits(pattern)
        self.mask = mask if isinstance(mask, Bits) else Bits(mask)

    @classmethod
    def random(cls, rng):
        return cls(Bits.random(rng), Bits.random(rng))

    @classmethod
    def from_array(cls, a):
        a = _c(a, np.uint64).reshape(2 * LIMBS)
        return cls(a[:LIMBS], a[LIMBS:])

    def to_array(self):
        return np.concatenate([self.pattern.limbs, self.mask.limbs])

    def rotated(self, amount):
        return Template(self.pattern.rotated(amount), self.mask.rotated(amount))

    def __eq__(self, other):
        return isinstance(other, Template) and self.pattern == other.pattern and self.mask == other.mask

    def distance(self, other, device=None):
        """Template::distance (src/template.rs:43-47), on the GPU."""
        dev = device or default_device()
        with TemplateEngine(dev, self) as eng:
            return float(eng.distances_host(other.to_array()[None, :])[0])


def encode(template):
    """encode(&Template) -> EncodedBits (src/lib.rs:16-26)."""
    t = template.to_array() if isinstance(template, Template) else _c(template, np.uint64)
    out = np.empty(BITS, np.uint16)
    _check(load_library().iris_encode(_ptr(_c(t, np.uint64)), _ptr(out)))
    return EncodedBits(out)


def decode_distance(distances, denominators):
    """decode_distance(&[u16;31], &[u16;31]) -> f64 (src/lib.rs:97-107)."""
    out = ctypes.c_double()
    _check(load_library().iris_decode_distance(_ptr(_c(distances, np.uint16)), _ptr(_c(denominators, np.uint16)),
                                               ctypes.byref(out)))
    return out.value


def merge_matches(matches):
    """Cross-shard argmin merge (src/main.rs:616-621 semantics)."""
    arr = (Match * max(1, len(matches)))(*matches) if matches else (Match * 1)()
    out = Match()
    _check(load_library().iris_match_merge(arr, len(matches), ctypes.byref(out)))
    return out


# ====================================================================== devices / databases


class Device:
    """One HIP device (gfx950) and its stream."""

    def __init__(self, ordinal=0):
        lib = load_library()
        h = ctypes.c_void_p()
        _check(lib.iris_device_open(int(ordinal), ctypes.byref(h)))
        self.handle = h
        self.ordinal = ordinal

    @staticmethod
    def count():
        n = ctypes.c_int()
        _check(load_library().iris_device_count(ctypes.byref(n)))
        return n.value

    def close(self):
        if self.handle:
            load_library().iris_device_close(self.handle)
            self.handle = None

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def synchronize(self):
        _check(load_library().iris_device_synchronize(self.handle))

    def config(self):
        """The environment knobs this device read when it opened (iris_config), as a dict."""
        return config(self)

    def memory(self):
        """(free, total) device memory in bytes."""
        f, t = ctypes.c_size_t(), ctypes.c_size_t()
        _check(load_library().iris_device_memory(self.handle, ctypes.byref(f), ctypes.byref(t)))
        return f.value, t.value

    def resident(self):
        """(count, bytes) of the record-file copies this device keeps resident for host-slice calls."""
        c, b = self.config()["resident"].split("/")
        return int(c), int(b)

    def drop_resident(self):
        """Frees the device's resident record-file copies (iris_device_drop_resident)."""
        _check(load_library().iris_device_drop_resident(self.handle))

    def drop_resident_range(self, array):
        """Frees the resident copy of the file mapping that holds `array`'s first byte
        (iris_device_drop_resident_range): after changing the file through a writable mapping."""
        a = np.asarray(array)
        _check(load_library().iris_device_drop_resident_range(self.handle, ctypes.c_void_p(a.ctypes.data)))

    def stream(self):
        s = ctypes.c_void_p()
        _check(load_library().iris_device_stream(self.handle, ctypes.byref(s)))
        return s.value

    def set_profiling(self, enabled=True):
        _check(load_library().iris_device_set_profiling(self.handle, 1 if enabled else 0))

    def reset_stats(self):
        _check(load_library().iris_device_reset_stats(self.handle))

    def kernel_stats(self, name):
        """-> (launches, total_ms, items) recorded with HIP events on the device stream."""
        l, ms, it = ctypes.c_uint64(), ctypes.c_double(), ctypes.c_uint64()
        _check(load_library().iris_device_kernel_stats(self.handle, name.encode(), ctypes.byref(l), ctypes.byref(ms),
                                                        ctypes.byref(it)))
        return l.value, ms.value, it.value

    def kernel_stats_largest(self, name):
        """-> (items, ms) of the largest launch of the kernel family since the last reset."""
        it, ms = ctypes.c_uint64(), ctypes.c_double()
        _check(load_library().iris_device_kernel_stats_largest(self.handle, name.encode(), ctypes.byref(it),
                                                                ctypes.byref(ms)))
        return it.value, ms.value

    def alloc(self, nbytes):
        p = ctypes.c_void_p()
        _check(load_library().iris_device_alloc(self.handle, int(nbytes), ctypes.byref(p)))
        return p.value

    def free(self, ptr):
        _check(load_library().iris_device_free(self.handle, ctypes.c_void_p(ptr)))

    def d2h(self, host_array, device_ptr):
        _check(load_library().iris_memcpy_d2h(self.handle, _ptr(host_array), ctypes.c_void_p(device_ptr),
                                               host_array.nbytes))

    def h2d(self, device_ptr, host_array):
        a = np.ascontiguousarray(host_array)
        _check(load_library().iris_memcpy_h2d(self.handle, ctypes.c_void_p(device_ptr), _ptr(a), a.nbytes))


def config(device=None):
    """iris_config as a dict: the knobs of `device`, or (None) those a device opened now would get.
    Test-only hooks set without IRIS_TEST_HOOKS=1 appear under "ignored" (a list)."""
    lib = load_library()
    h = device.handle if device is not None else None
    need = ctypes.c_size_t()
    _check(lib.iris_config(h, None, 0, ctypes.byref(need)))
    buf = ctypes.create_string_buffer(need.value + 1)
    _check(lib.iris_config(h, buf, len(buf), None))
    out = {}
    for kv in buf.value.decode().split():
        k, v = kv.split("=", 1)
        out[k] = v.split(",") if k == "ignored" else v
    return out


_default = None


def default_device():
    global _default
    if _default is None:
        _default = Device(0)
    return _default


def _records(kind, records):
    dt, width = _REC_DTYPE[kind]
    if isinstance(records, (Bits, EncodedBits, Template)):
        records = [records]
    if isinstance(records, (list, tuple)):
        rows = []
        for r in records:
            if isinstance(r, Bits):
                rows.append(r.limbs)
            elif isinstance(r, EncodedBits):
                rows.append(r.values)
            elif isinstance(r, Template):
                rows.append(r.to_array())
            else:
                rows.append(np.asarray(r))
        records = np.stack(rows) if rows else np.zeros((0, width), dt)
    a = _c(records, dt)
    if a.ndim == 1:
        a = a.reshape(1, -1)
    if a.shape[-1] != width:
        raise IrisError(-1, f"records must have {width} {np.dtype(dt).name} per row, got shape {a.shape}")
    return a


class Database:
    """Device-resident database (replaces the reference's mmap'd share/masks files)."""

    def __init__(self, device, kind, capacity, layout=LAYOUT_DEFAULT):
        self.device = device
        self.kind = kind
        h = ctypes.c_void_p()
        _check(load_library().iris_db_create_ex(device.handle, int(kind), int(capacity), int(layout),
                                                ctypes.byref(h)))
        self.handle = h

    @property
    def layout(self):
        v = ctypes.c_int()
        _check(load_library().iris_db_layout(self.handle, ctypes.byref(v)))
        return v.value

    def close(self):
        if self.handle:
            self._release_attached()
            load_library().iris_db_destroy(self.handle)
            self.handle = None

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _release_attached(self):
        # every change of the records ends the attachment in the library: the host array is
        # writable again (if it was before attach_host)
        a = getattr(self, "_attached", None)
        if a is not None and getattr(self, "_attached_writable", False):
            a.setflags(write=True)
        self._attached = None

    def __len__(self):
        n = ctypes.c_uint64()
        _check(load_library().iris_db_len(self.handle, ctypes.byref(n)))
        return n.value

    @property
    def capacity(self):
        n = ctypes.c_uint64()
        _check(load_library().iris_db_capacity(self.handle, ctypes.byref(n)))
        return n.value

    def append(self, records):
        a = _records(self.kind, records)
        self._release_attached()
        _check(load_library().iris_db_append(self.handle, _ptr(a), a.shape[0]))

    def write(self, index, records):
        a = _records(self.kind, records)
        self._release_attached()
        _check(load_library().iris_db_write(self.handle, int(index), _ptr(a), a.shape[0]))

    def read(self, first, n):
        dt, width = _REC_DTYPE[self.kind]
        out = np.empty((n, width), dt)
        _check(load_library().iris_db_read(self.handle, int(first), int(n), _ptr(out)))
        return out

    def generate(self, n, seed, global_index0=None):
        """Append n synthetic records; generator index defaults to the DB position."""
        g0 = len(self) if global_index0 is None else global_index0
        self._release_attached()
        _check(load_library().iris_db_generate(self.handle, int(n), int(seed), int(g0)))

    def clear(self):
        self._release_attached()
        _check(load_library().iris_db_clear(self.handle))

    def truncate(self, n):
        if int(n) != len(self):
            self._release_attached()
        _check(load_library().iris_db_truncate(self.handle, int(n)))

    def load_file(self, path, first=0, count=None):
        """Appends records [first, first+count) of a raw record file (.masks / .share-i /
        raw templates; src/main.rs:386-400,455-469).  Returns the number appended."""
        got = ctypes.c_uint64(0)
        cnt = (1 << 64) - 1 if count is None else int(count)
        self._release_attached()
        _check(load_library().iris_db_load_file(self.handle, os.fsencode(path), int(first), cnt,
                                                ctypes.byref(got)))
        return got.value

    def save_file(self, path, first=0, n=None):
        """Writes records [first, first+n) to a raw record file."""
        if n is None:
            n = len(self) - int(first)
        _check(load_library().iris_db_save_file(self.handle, os.fsencode(path), int(first), int(n)))

    def attach_host(self, host, upload=True):
        """Declares this database the resident copy of the host record array `host` (e.g. a
        memory-mapped record file, src/main.rs:389-391,458-460): upload=True fills the (empty)
        database from it; upload=False checks it already holds them.  Engine batch_process
        calls on slices (numpy views) of `host` then run on the device copy without an
        upload.  Keeps a reference to `host` while attached and makes that array read-only
        until the attachment ends (detach_host, or any write to the database): the device copy
        would not see a change (other views of the same memory are not locked -- the rows must
        stay unchanged while attached, as include/iris_hip.h says)."""
        a = host if isinstance(host, np.ndarray) else np.asarray(host)
        dt, width = _REC_DTYPE[self.kind]
        if a.dtype != dt or a.ndim != 2 or a.shape[1] != width or not a.flags["C_CONTIGUOUS"]:
            raise IrisError(-1, f"host must be a C-contiguous [n, {width}] {np.dtype(dt).name} array")
        self._release_attached()
        _check(load_library().iris_db_attach_host(self.handle, _ptr(a), a.shape[0], 1 if upload else 0))
        self._attached = a
        self._attached_writable = bool(a.flags.writeable)
        if self._attached_writable:
            a.setflags(write=False)

    def detach_host(self):
        _check(load_library().iris_db_detach_host(self.handle))
        self._release_attached()


# ====================================================================== engines


class _Engine:
    kind = 0

    def close(self):
        if getattr(self, "handle", None):
            load_library().iris_engine_destroy(self.handle)
            self.handle = None

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def query_tables(self):
        """The engine's device-built rotated-query table and MFMA fragments, copied to
        the host -> (table uint8 array, fragments uint8 array)."""
        tb, fb = query_table_sizes(self.kind, getattr(self, "nq", 0))
        tab, frag = np.zeros(tb, np.uint8), np.zeros(fb, np.uint8)
        _check(load_library().iris_engine_query_tables(self.handle, _ptr(tab) if tb else None, tb, _ptr(frag), fb))
        return tab, frag

    def batch_process(self, out, db, first=0, n=None):
        """batch_process(&self, out: &mut [[u16;31]], db: &[T]) (src/lib.rs:42-52, 69-79).

        `db` is a Database (records [first, first+n)) or a host array / list of records.
        `out` is a [n, 31] uint16 array (filled in place)."""
        lib = load_library()
        if out.dtype != np.uint16 or not out.flags.c_contiguous or out.ndim != 2 or out.shape[1] != ROTATIONS:
            raise IrisError(-1, "out must be a C-contiguous [n, 31] uint16 array")
        dt, width = _REC_DTYPE[self.kind]
        if (isinstance(db, np.ndarray) and db.dtype == dt and db.ndim == 2 and db.shape[1] == width
                and db.flags.c_contiguous and out.shape[0] == db.shape[0]):
            # the chunk walk's call (a contiguous slice of the caller's record array): passed as is,
            # with none of the conversions below, through the buffer protocol where the fast path
            # is built (csrc/iris_pycall.c), else ctypes
            pc = _pycall if _pycall is not _UNLOADED else _load_pycall()
            if pc is not None:
                rc = pc.batch_process_host((self.handle or _NULL).value or 0, db, out, db.itemsize * width)
            else:
                rc = lib.iris_engine_batch_process_host(self.handle, db.ctypes.data, db.shape[0], out.ctypes.data)
            if rc:
                _check(rc)
            return out
        if isinstance(db, Database):
            n = (len(db) - first) if n is None else n
            if out.shape[0] != n:  # assert_eq!(out.len(), db.len()) (src/lib.rs:43,70)
                raise IrisError(-1, f"assertion `out.len() == db.len()` failed: {out.shape[0]} != {n}")
            _check(lib.iris_engine_batch_process(self.handle, db.handle, int(first), int(n), _ptr(out)))
        else:
            a = _records(self.kind, db)  # a contiguous view of the caller's array is passed as is
            if out.shape[0] != a.shape[0]:
                raise IrisError(-1, f"assertion `out.len() == db.len()` failed: {out.shape[0]} != {a.shape[0]}")
            _check(lib.iris_engine_batch_process_host(self.handle, _ptr(a), a.shape[0], _ptr(out)))
        return out


def _batch_process_device(self, db, out_device_ptr, first=0, n=None):
    """Results stay on the GPU: out_device_ptr is a device array of n*31 u16."""
    n = (len(db) - first) if n is None else n
    rc = load_library().iris_engine_batch_process_device(self.handle, db.handle, int(first), int(n), int(out_device_ptr))
    if rc:
        _check(rc)


_Engine.batch_process_device = _batch_process_device


class MasksEngine(_Engine):
    """MasksEngine (src/lib.rs:55-80): out[k] = dot_bool(rot(query, k-15), entry)."""

    kind = KIND_MASKS

    def __init__(self, device, query):
        self.device = device
        q = query.limbs if isinstance(query, Bits) else _c(query, np.uint64)
        h = ctypes.c_void_p()
        _check(load_library().iris_masks_engine_new(device.handle, _ptr(_c(q, np.uint64)), ctypes.byref(h)))
        self.handle = h

    def resolve(self, db, shares, first=0, n=None, index_base=0, dist_out_device=None):
        """The resolver step with this engine's denominators computed on the fly
        (src/main.rs:510-519 + 597-621): shares = the participants' [n,31] u16 outputs,
        host arrays or device pointers.  Host arrays (and no dist_out_device) go through
        iris_resolver_search_masks_host: summed on the host, the sum uploaded.  -> Match."""
        if n is None:
            n = len(db) - int(first)
        dev = self.device
        if dist_out_device is None and shares and not any(isinstance(a, int) for a in shares):
            arrs = [_c(a, np.uint16) for a in shares]
            for a in arrs:
                if a.shape != (n, ROTATIONS):
                    raise IrisError(-1, "shares must be [n, 31] uint16")
            ptrs = (ctypes.c_void_p * len(arrs))(*[a.ctypes.data for a in arrs])
            m = Match()
            _check(load_library().iris_resolver_search_masks_host(self.handle, db.handle, int(first), int(n), ptrs,
                                                                  len(arrs), int(index_base), ctypes.byref(m)))
            return m
        tmp = []
        try:
            ptrs = []
            for a in shares:
                if isinstance(a, int):
                    ptrs.append(a)
                    continue
                a = _c(a, np.uint16)
                if a.shape != (n, ROTATIONS):
                    raise IrisError(-1, "shares must be [n, 31] uint16")
                p = dev.alloc(max(a.nbytes, 16))
                tmp.append(p)
                dev.h2d(p, a)
                ptrs.append(p)
            arr = (ctypes.c_void_p * len(ptrs))(*ptrs)
            m = Match()
            _check(load_library().iris_resolver_search_masks(self.handle, db.handle, int(first), int(n), arr,
                                                             len(ptrs), int(index_base),
                                                             ctypes.c_void_p(dist_out_device or 0), ctypes.byref(m)))
            return m
        finally:
            for p in tmp:
                dev.free(p)


class DistanceEngine(_Engine):
    """DistanceEngine (src/lib.rs:28-53): out[k] = dot_u16(rot(query, k-15), entry)."""

    kind = KIND_SHARES

    def __init__(self, device, query):
        self.device = device
        q = query.values if isinstance(query, EncodedBits) else _c(query, np.uint16)
        h = ctypes.c_void_p()
        _check(load_library().iris_distance_engine_new(device.handle, _ptr(_c(q, np.uint16)), ctypes.byref(h)))
        self.handle = h


class TemplateEngine(_Engine):
    """Masked fractional Hamming of one query Template against a Template DB
    (src/template.rs:43-64): counts per rotation, distances, fused argmin."""

    kind = KIND_TEMPLATES

    def __init__(self, device, query):
        self.device = device
        q = query.to_array() if isinstance(query, Template) else _c(query, np.uint64)
        h = ctypes.c_void_p()
        _check(load_library().iris_template_engine_new(device.handle, _ptr(_c(q, np.uint64)), ctypes.byref(h)))
        self.handle = h

    def counts(self, db, first=0, n=None):
        """-> (num [n,31] u16, den [n,31] u16)."""
        n = (len(db) - first) if n is None else n
        num = np.empty((n, ROTATIONS), np.uint16)
        den = np.empty((n, ROTATIONS), np.uint16)
        _check(load_library().iris_template_counts(self.handle, db.handle, int(first), int(n), _ptr(num), _ptr(den)))
        return num, den

    def distances(self, db, first=0, n=None):
        """Template::distance(query, db[i]) for every i -> [n] f64."""
        n = (len(db) - first) if n is None else n
        out = np.empty(n, np.float64)
        _check(load_library().iris_template_distances(self.handle, db.handle, int(first), int(n), _ptr(out)))
        return out

    def distances_host(self, records, layout=LAYOUT_DEFAULT):
        a = _records(KIND_TEMPLATES, records)
        with Database(self.device, KIND_TEMPLATES, max(1, a.shape[0]), layout) as db:
            db.append(a)
            return self.distances(db)

    def search_async(self, db, first=0, n=None, index_base=0):
        """Enqueue the fused min/argmin and return at once -> PendingSearch (wait() -> Match)."""
        n = (len(db) - first) if n is None else n
        h = ctypes.c_void_p()
        _check(load_library().iris_template_search_async(self.handle, db.handle, int(first), int(n),
                                                         int(index_base), ctypes.byref(h)))
        return PendingSearch(h)

    def search(self, db, first=0, n=None, index_base=0, dist_out_device=None):
        """Fused min/argmin (src/main.rs:581-621) -> Match."""
        n = (len(db) - first) if n is None else n
        m = Match()
        rc = load_library().iris_template_search(self.handle, db.handle, int(first), int(n), int(index_base),
                                                 dist_out_device or None, ctypes.byref(m))
        if rc:
            _check(rc)
        return m


class PendingSearch:
    """An enqueued search (TemplateEngine.search_async); wait() -> Match, once."""

    def __init__(self, handle):
        self.handle = handle

    def wait(self):
        if self.handle is None:
            raise IrisError(-1, "PendingSearch.wait called twice")
        m = Match()
        h, self.handle = self.handle, None
        _check(load_library().iris_pending_wait(h, ctypes.byref(m)))
        return m

    def __del__(self):
        if getattr(self, "handle", None) is not None:
            try:
                load_library().iris_pending_wait(self.handle, None)
            except Exception:
                pass


class TemplateBatchEngine(_Engine):
    """Many query Templates against one template DB in one pass (configs[2])."""

    kind = KIND_TEMPLATES

    def __init__(self, device, queries):
        self.device = device
        q = _records(KIND_TEMPLATES, queries)
        self.nq = q.shape[0]
        h = ctypes.c_void_p()
        _check(load_library().iris_template_batch_engine_new(device.handle, _ptr(q), self.nq, ctypes.byref(h)))
        self.handle = h

    def search(self, db, first=0, n=None, index_base=0):
        n = (len(db) - first) if n is None else n
        out = (Match * self.nq)()
        _check(load_library().iris_template_batch_search(self.handle, db.handle, int(first), int(n), int(index_base),
                                                         out))
        return list(out)


# ====================================================================== device groups


class Group:
    """Devices searched together (include/iris_hip.h "device groups"): a sharded template
    database, per-shard winners all-gathered over RCCL and merged on every device.
    Group(ordinals) drives several devices from this process (ncclCommInitAll);
    Group.rank(ordinal, nranks, rank, uid) is one device of a multi-process group whose
    128-byte id comes from Group.unique_id() on rank 0."""

    def __init__(self, ordinals=(0,), _handle=None):
        if _handle is not None:
            self.handle = _handle
        else:
            ords = (ctypes.c_int * len(ordinals))(*[int(o) for o in ordinals])
            h = ctypes.c_void_p()
            _check(load_library().iris_group_create(ords, len(ordinals), ctypes.byref(h)))
            self.handle = h
        l, r, f = ctypes.c_uint32(), ctypes.c_uint32(), ctypes.c_uint32()
        _check(load_library().iris_group_info(self.handle, ctypes.byref(l), ctypes.byref(r), ctypes.byref(f)))
        self.local_devices, self.ranks, self.first_rank = l.value, r.value, f.value
        # what RCCL reports: its communicators' rank count and every rank's device PCI bus id
        cr = ctypes.c_uint32()
        ids = ctypes.create_string_buffer(32 * self.ranks)
        _check(load_library().iris_group_rccl_info(self.handle, ctypes.byref(cr), ids, len(ids)))
        self.rccl_nranks = cr.value
        self.rccl_devices = [ids.raw[32 * k:32 * (k + 1)].split(b"\0", 1)[0].decode() for k in range(self.ranks)]
        self.devices = []
        for i in range(self.local_devices):
            d = ctypes.c_void_p()
            _check(load_library().iris_group_device(self.handle, i, ctypes.byref(d)))
            self.devices.append(_BorrowedDevice(d))

    @staticmethod
    def unique_id():
        buf = (ctypes.c_uint8 * 128)()
        _check(load_library().iris_group_unique_id(buf))
        return bytes(buf)

    @classmethod
    def rank(cls, ordinal, nranks, rank, uid):
        if len(uid) != 128:
            raise ValueError("the group id is 128 bytes")
        buf = (ctypes.c_uint8 * 128).from_buffer_copy(bytes(uid))
        h = ctypes.c_void_p()
        _check(load_library().iris_group_create_rank(int(ordinal), int(nranks), int(rank), buf, ctypes.byref(h)))
        return cls(_handle=h)

    def set_timeout(self, ms):
        """Bound (ms) of the exchange waits of later calls; 0 = automatic (iris_group_set_timeout)."""
        _check(load_library().iris_group_set_timeout(self.handle, int(ms)))

    def close(self):
        if getattr(self, "handle", None):
            load_library().iris_group_destroy(self.handle)
            self.handle = None

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class _BorrowedDevice(Device):
    """A group's device handle (owned by the group: close() does nothing)."""

    def __init__(self, handle):
        self.handle = handle
        self.ordinal = None

    def close(self):
        self.handle = None


class _BorrowedDatabase(Database):
    """A group shard's database (owned by the group database: close() does nothing)."""

    def __init__(self, handle, device, kind):
        self.handle = handle
        self.device = device
        self.kind = kind

    def close(self):
        self.handle = None


class GroupDatabase:
    """`total` records of `kind` in S = ranks x shards_per_device contiguous shards over a
    Group; every record starts empty (never a candidate)."""

    def __init__(self, group, kind, total, layout=LAYOUT_DEFAULT, shards_per_device=1):
        self.group = group
        self.kind = kind
        h = ctypes.c_void_p()
        _check(load_library().iris_group_db_create(group.handle, int(kind), int(total), int(layout),
                                                   int(shards_per_device), ctypes.byref(h)))
        self.handle = h
        t, S, f, l = ctypes.c_uint64(), ctypes.c_uint32(), ctypes.c_uint32(), ctypes.c_uint32()
        _check(load_library().iris_group_db_info(h, ctypes.byref(t), ctypes.byref(S), ctypes.byref(f),
                                                 ctypes.byref(l)))
        self.total, self.shards, self.first_shard, self.local_shards = t.value, S.value, f.value, l.value

    def shard(self, i):
        """-> (first global index, count) of local shard i."""
        f, c = ctypes.c_uint64(), ctypes.c_uint64()
        _check(load_library().iris_group_db_shard(self.handle, int(i), None, ctypes.byref(f), ctypes.byref(c)))
        return f.value, c.value

    def shard_db(self, i):
        """Local shard i as a Database (borrowed: owned by this group database), e.g. for a
        local search with no exchange; its record j is global record shard(i)[0] + j."""
        h = ctypes.c_void_p()
        _check(load_library().iris_group_db_shard(self.handle, int(i), ctypes.byref(h), None, None))
        spd = self.local_shards // self.group.local_devices
        return _BorrowedDatabase(h, self.group.devices[int(i) // spd], self.kind)

    def close(self):
        if getattr(self, "handle", None):
            load_library().iris_group_db_destroy(self.handle)
            self.handle = None

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __len__(self):
        return self.total

    def generate(self, seed):
        _check(load_library().iris_group_db_generate(self.handle, int(seed)))

    def write(self, index, records):
        a = _records(self.kind, records)
        _check(load_library().iris_group_db_write(self.handle, int(index), _ptr(a), a.shape[0]))

    def read(self, index, n):
        dt, width = _REC_DTYPE[self.kind]
        out = np.empty((n, width), dt)
        _check(load_library().iris_group_db_read(self.handle, int(index), int(n), _ptr(out)))
        return out

    def load_file(self, path, first=0):
        _check(load_library().iris_group_db_load_file(self.handle, os.fsencode(path), int(first)))

    def search(self, query):
        """Global (min distance, lowest index) of one query Template -> Match."""
        q = query.to_array() if isinstance(query, Template) else _c(query, np.uint64)
        m = Match()
        _check(load_library().iris_group_template_search(self.handle, _ptr(_c(q, np.uint64)), ctypes.byref(m)))
        return m

    def search_async(self, query):
        q = query.to_array() if isinstance(query, Template) else _c(query, np.uint64)
        h = ctypes.c_void_p()
        _check(load_library().iris_group_template_search_async(self.handle, _ptr(_c(q, np.uint64)), ctypes.byref(h)))
        return GroupPendingSearch(h)

    def batch_search(self, queries):
        q = _records(KIND_TEMPLATES, queries)
        out = (Match * q.shape[0])()
        _check(load_library().iris_group_template_batch_search(self.handle, _ptr(q), q.shape[0], out))
        return list(out)


class GroupPendingSearch:
    """An enqueued group search; wait() -> Match, once."""

    def __init__(self, handle):
        self.handle = handle

    def wait(self):
        if self.handle is None:
            raise IrisError(-1, "GroupPendingSearch.wait called twice")
        m = Match()
        h, self.handle = self.handle, None
        _check(load_library().iris_group_pending_wait(h, ctypes.byref(m)))
        return m

    def __del__(self):
        if getattr(self, "handle", None) is not None:
            try:
                load_library().iris_group_pending_wait(self.handle, None)
            except Exception:
                pass


def distances(query, entry, device=None):
    """distances(&EncodedBits, &EncodedBits) -> [u16; 31] (src/lib.rs:82-87)."""
    dev = device or default_device()
    out = np.empty((1, ROTATIONS), np.uint16)
    with DistanceEngine(dev, query) as eng:
        eng.batch_process(out, [entry])
    return out[0]


def denominators(query, entry, device=None):
    """denominators(&Bits, &Bits) -> [u16; 31] (src/lib.rs:89-94)."""
    dev = device or default_device()
    out = np.empty((1, ROTATIONS), np.uint16)
    with MasksEngine(dev, query) as eng:
        eng.batch_process(out, [entry])
    return out[0]


# ====================================================================== resolver


def resolver_search(shares, denominators, index_base=0, device=None):
    """The resolver's aggregation (src/main.rs:597-621) on the GPU: wrapping sum
    of the participants' [n,31] u16 shares, decode_distance with the [n,31]
    denominators, min over rotations, strict-< lowest-index argmin -> Match."""
    dev = device or default_device()
    arrs = [_c(s, np.uint16) for s in shares]
    den = _c(denominators, np.uint16)
    n = den.shape[0]
    for a in arrs:
        if a.shape != (n, ROTATIONS):
            raise IrisError(-1, "shares and denominators must all be [n, 31] uint16")
    ptrs = (ctypes.c_void_p * len(arrs))(*[a.ctypes.data for a in arrs])
    m = Match()
    _check(load_library().iris_resolver_search_host(dev.handle, ptrs, len(arrs), _ptr(den), n, int(index_base),
                                                    ctypes.byref(m)))
    return m


def resolver_search_device(device, share_ptrs, denoms_ptr, n, index_base=0, dist_out_device=None):
    """Device-resident form: share_ptrs / denoms_ptr are device arrays of n*31 u16."""
    ptrs = (ctypes.c_void_p * len(share_ptrs))(*share_ptrs)
    m = Match()
    _check(load_library().iris_resolver_search(device.handle, ptrs, len(share_ptrs), ctypes.c_void_p(denoms_ptr), int(n),
                                               int(index_base), ctypes.c_void_p(dist_out_device or 0),
                                               ctypes.byref(m)))
    return m


# ====================================================================== arch plugin


def dot_bool_batch(a, b, device=None):
    """out[j, i] = dot_bool(a[i], b[j]) (src/arch/generic.rs:4-9)."""
    dev = device or default_device()
    a = _records(KIND_MASKS, a)
    b = _records(KIND_MASKS, b)
    out = np.empty((b.shape[0], a.shape[0]), np.uint16)
    _check(load_library().iris_dot_bool_batch(dev.handle, _ptr(a), a.shape[0], _ptr(b), b.shape[0], _ptr(out)))
    return out


def dot_u16_batch(a, b, device=None):
    """out[j, i] = dot_u16(a[i], b[j]) (src/arch/generic.rs:11-16)."""
    dev = device or default_device()
    a = _records(KIND_SHARES, a)
    b = _records(KIND_SHARES, b)
    out = np.empty((b.shape[0], a.shape[0]), np.uint16)
    _check(load_library().iris_dot_u16_batch(dev.handle, _ptr(a), a.shape[0], _ptr(b), b.shape[0], _ptr(out)))
    return out


def dot_bool(a, b, device=None):
    return int(dot_bool_batch([a], [b], device)[0, 0])


def dot_u16(a, b, device=None):
    return int(dot_u16_batch([a], [b], device)[0, 0])


def f64_bits(x):
    return int(np.float64(x).view(np.uint64))


__all__ = [
    "Bits", "EncodedBits", "Template", "encode", "decode_distance", "resolver_search", "resolver_search_device", "distances", "denominators", "MasksEngine",
    "DistanceEngine", "TemplateEngine", "TemplateBatchEngine", "Device", "Database", "Match", "merge_matches", "dot_bool", "dot_u16",
    "Group", "GroupDatabase", "GroupPendingSearch",
    "dot_bool_batch", "dot_u16_batch", "IrisError", "load_library", "KIND_MASKS", "KIND_SHARES", "KIND_TEMPLATES",
    "LAYOUT_DEFAULT", "LAYOUT_LANES", "LAYOUT_TILES", "config",
    "ROTATIONS", "BITS", "LIMBS", "COLS", "ROWS",
]
