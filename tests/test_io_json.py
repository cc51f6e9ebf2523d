"""JSON template files (src/template.rs:11-29 serde form, Bits as the hex of its
1600 LE bytes, src/bits.rs:74-93), parsed by libiris_hip's host-side reader.
Checked against Python's json + bytes.fromhex as an independent decoder.
Host code only: runs without a GPU."""
import json

import numpy as np
import pytest

import iris_hip as ih
from oracle import oracle_c as oc


def _hex(limbs):
    return np.asarray(limbs, "<u8").tobytes().hex()


def _py_decode(path):
    out = []
    for obj in json.load(open(path)):
        p = np.frombuffer(bytes.fromhex(obj["pattern"]), "<u8")
        m = np.frombuffer(bytes.fromhex(obj["mask"]), "<u8")
        out.append(np.concatenate([p, m]))
    return np.array(out, np.uint64).reshape(-1, 400)


def test_write_read_roundtrip(tmp_path):
    t = oc.gen_templates(3, 0, 17)
    path = tmp_path / "t.json"
    ih.write_templates_json(path, t)
    assert (_py_decode(path) == t).all()  # independent decoder agrees on the format
    assert (ih.read_templates_json(path) == t).all()
    text = path.read_text()
    assert text.startswith('[{"pattern":"') and text == text.lower()


def test_python_written_variants(tmp_path):
    """Whitespace, field order, uppercase hex (hex::deserialize accepts it)."""
    t = oc.gen_templates(4, 0, 5)
    objs = []
    for i, r in enumerate(t):
        p, m = _hex(r[:200]), _hex(r[200:])
        objs.append({"mask": m.upper(), "pattern": p} if i % 2 else {"pattern": p, "mask": m})
    path = tmp_path / "v.json"
    path.write_text("  \n" + json.dumps(objs, indent=3) + "\n")
    assert (ih.read_templates_json(path) == t).all()


def test_empty_array(tmp_path):
    path = tmp_path / "e.json"
    path.write_text(" [ ] ")
    assert ih.read_templates_json(path).shape == (0, 400)


@pytest.mark.parametrize("text,what", [
    ('{"pattern": "00"}', "`[` not found"),
    ('[{"pattern": "%s"}]', "missing field `mask`"),
    ('[{"pattern": "%s", "mask": "%s"} {', "`,` or `]` not found"),
    ('[{"pattern": "%s", "mask": "00"}]', "expected 1600"),
    ('[{"pattern": "%s", "mask": "zz%s"}]', "invalid hex digit"),
    ('[{"pattern": "%s", "mask": "%s", "mask": "%s"}]', "duplicate field"),
    ('[{"pattern": "%s", "mask": "%s"}', "`,` or `]` not found"),
])
def test_malformed(tmp_path, text, what):
    h = "00" * 1600
    path = tmp_path / "bad.json"
    path.write_text(text.replace("%s", h))
    with pytest.raises(ih.IrisError) as ei:
        ih.read_templates_json(path)
    assert ei.value.code == -7 and what in str(ei.value)


def test_missing_file(tmp_path):
    with pytest.raises(ih.IrisError) as ei:
        ih.read_templates_json(tmp_path / "absent.json")
    assert ei.value.code == -6


def test_mutated_files_never_crash(tmp_path):
    """Truncations and byte mutations of a valid file: the reader either returns records
    that Python's decoder also accepts or raises IrisError — never crashes or reads past
    the buffer (this test also runs against the host-ASan build of the library)."""
    t = oc.gen_templates(5, 0, 3)
    good = tmp_path / "g.json"
    ih.write_templates_json(good, t)
    base = good.read_bytes()
    rng = np.random.default_rng(12)
    path = tmp_path / "m.json"
    cuts = [0, 1, 2, 15, len(base) // 2, len(base) - 2, len(base) - 1]
    variants = [base[:c] for c in cuts]
    alphabet = b'[]{}",: \n0123456789abcdefABCDEFxyz\\'
    for _ in range(120):
        b = bytearray(base)
        for _ in range(int(rng.integers(1, 4))):
            b[int(rng.integers(0, len(b)))] = alphabet[int(rng.integers(0, len(alphabet)))]
        variants.append(bytes(b))
    for v in variants:
        path.write_bytes(v)
        try:
            got = ih.read_templates_json(path)
        except ih.IrisError as e:
            assert e.code in (-7, -6), e
            continue
        try:
            want = _py_decode(path)
        except (ValueError, KeyError, TypeError):
            continue  # the reader is more lenient than json.load on e.g. trailing bytes
        assert got.shape[0] == want.shape[0] and (got == want).all()
