"""CPU: the C-ABI library loads, exports every symbol include/iris_hip.h
declares, and its host-side helpers (no GPU needed) match the oracle."""
import ctypes
import pathlib
import re

import numpy as np
import os

import pytest

import iris_hip as ih
from oracle import oracle_c as oc

ROOT = pathlib.Path(__file__).resolve().parents[1]


def header_symbols():
    text = (ROOT / "include" / "iris_hip.h").read_text()
    return sorted(set(re.findall(r"^\s*(?:const char \*|int )\s*(iris_\w+)\s*\(", text, flags=re.M)))


def test_header_symbols_exported():
    lib = ctypes.CDLL(str(ih.LIB_PATH))
    syms = header_symbols()
    assert len(syms) >= 35
    missing = [s for s in syms if not hasattr(lib, s)]
    assert not missing, missing
    assert sorted(ih.exported_symbols()) == syms


def test_version():
    assert b"gfx950" in ih.load_library().iris_version()


def test_no_device_fails_loudly():
    if ih.Device.count() > 0:
        pytest.skip("a GPU is visible")
    with pytest.raises(ih.IrisError):
        ih.Device(0)


def test_bits_rotated_matches_oracle():
    rng = np.random.default_rng(1)
    for _ in range(5):
        b = ih.Bits.random(rng)
        for r in range(-15, 16):
            assert (b.rotated(r).limbs == oc.bits_rotated(b.limbs, r)).all()
            assert b.rotated(r).rotated(-r) == b


def test_encoded_rotated_matches_oracle():
    rng = np.random.default_rng(2)
    e = ih.EncodedBits.random(rng)
    for r in range(-15, 16):
        assert (e.rotated(r).values == oc.encoded_rotated(e.values, r)).all()
    b = ih.Bits.random(rng)
    for r in (-15, -1, 3, 15):  # src/encoded_bits.rs:222-236
        assert ih.EncodedBits.from_bits(b.rotated(r)) == ih.EncodedBits.from_bits(b).rotated(r)


def test_encode_matches_oracle(golden):
    t = ih.Template.from_array(golden["query"])
    assert (ih.encode(t).values == golden["enc_query"]).all()
    rng = np.random.default_rng(3)
    for _ in range(5):
        t = ih.Template.random(rng)
        assert (ih.encode(t).values == oc.encode(t.to_array())).all()


def test_decode_distance_matches_oracle(golden):
    rng = np.random.default_rng(4)
    for _ in range(200):
        n = rng.integers(0, 2**16, 31, dtype=np.uint16)
        d = rng.integers(0, 2**16, 31, dtype=np.uint16)
        if rng.random() < 0.2:
            d[:] = 0
        got, want = ih.decode_distance(n, d), oc.decode_distance(n, d)
        assert np.float64(got).view(np.uint64) == np.float64(want).view(np.uint64)
    share_sum = golden["share_out"].astype(np.uint64).sum(0).astype(np.uint16)
    for i in range(share_sum.shape[0]):
        got = ih.decode_distance(share_sum[i], golden["masks_out"][i])
        assert np.float64(got).view(np.uint64) == golden["dist_bits"][i]


def test_match_merge_rules():
    M = ih.Match
    inf = float("inf")
    recs = [M(inf, 2**64 - 1, 0, 0, 0, 0), M(0.5, 40, 2, 4, 0, 0), M(0.5, 12, 3, 6, 2, 0), M(0.75, 1, 3, 4, 0, 0)]
    best = ih.merge_matches(recs)
    assert (best.index, best.num, best.den) == (12, 3, 6)  # equal fraction, lowest index
    none = ih.merge_matches([M(inf, 2**64 - 1, 0, 0, 0, 0)])
    assert none.index == 2**64 - 1 and none.distance == inf
    assert ih.merge_matches([]).index == 2**64 - 1


def test_value_types():
    rng = np.random.default_rng(5)
    b = ih.Bits.random(rng)
    assert ih.Bits.from_hex(b.to_hex()) == b
    for i in (0, 1, 63, 64, 12799):
        assert b[i] == bool((int(b.limbs[i // 64]) >> (i % 64)) & 1)
    e = ih.EncodedBits.random(rng)
    shares = e.share(3, rng)
    assert (sum((s.values.astype(np.uint64) for s in shares)) & 0xFFFF == e.values).all()


def test_python_fast_path_links_the_shipped_library():
    """The fast path is linked to the shipped libiris_hip.so (a variant build such as
    tools/asan_host.sh's must not relink it to its own library)."""
    p = pathlib.Path(ih.__file__).parent / "_iris_pycall.so"
    if not p.exists():
        pytest.skip("no Python headers here: the fast path is not built")
    data = p.read_bytes()
    assert b"libiris_hip.so\0" in data and b"libiris_asan.so" not in data


def test_python_fast_path_extension():
    """The Python mirror's per-call fast path (csrc/iris_pycall.c) is built beside the library and
    used: it passes the caller's buffers to iris_engine_batch_process_host unchanged, so its
    errors are the library's (a NULL engine: IRIS_E_ARG), and a length mismatch between the
    records and the rows is refused before the call."""
    if "IRIS_HIP_LIB" in os.environ:  # another library build (tools/asan_host.sh): the ctypes path is used
        pytest.skip("IRIS_HIP_LIB names a non-default library; the fast path is linked to the default one")
    ih.load_library()
    pc = ih._load_pycall()
    assert pc is not None and ih._pycall is pc, "mpc-iris-code_amd/_iris_pycall.so not built"
    recs, out = np.zeros((2, 200), np.uint64), np.zeros((2, 31), np.uint16)
    assert pc.batch_process_host(0, recs, out, 1600) == ih.load_library().iris_engine_batch_process_host(
        None, recs.ctypes.data, 2, out.ctypes.data) == -1
    assert "engine is NULL" in ih.load_library().iris_last_error().decode()
    assert pc.batch_process_host(0, recs, np.zeros((3, 31), np.uint16), 1600) == -1  # 2 records, 3 rows
    with pytest.raises(ValueError):  # rows must be writable
        ro = np.zeros((2, 31), np.uint16)
        ro.setflags(write=False)
        pc.batch_process_host(0, recs, ro, 1600)
