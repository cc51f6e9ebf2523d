"""On-disk record files -> device databases: the raw
.masks / .share-i / template files the reference's `prepare` writes and its
`participant` / `resolver` mmap (src/main.rs:299-309,386-400,455-469)."""
import numpy as np
import pytest

import iris_hip as ih
from oracle import oracle_c as oc

pytestmark = pytest.mark.gpu
ROT = 31
KINDS = [(ih.KIND_MASKS, np.uint64, 200), (ih.KIND_SHARES, np.uint16, 12800), (ih.KIND_TEMPLATES, np.uint64, 400)]


def _records(kind, dtype, width, n, seed):
    rng = np.random.default_rng(seed)
    info = np.iinfo(dtype)
    return rng.integers(0, info.max, (n, width), dtype=dtype, endpoint=True)


@pytest.mark.parametrize("layout", [ih.LAYOUT_TILES, ih.LAYOUT_LANES], ids=["tiles", "lanes"])
@pytest.mark.parametrize("kind,dtype,width", KINDS, ids=["masks", "shares", "templates"])
def test_load_save_roundtrip(device, tmp_path, kind, dtype, width, layout):
    recs = _records(kind, dtype, width, 101, kind)
    path = tmp_path / "db.bin"
    recs.astype(np.dtype(dtype).newbyteorder("<")).tofile(path)
    with ih.Database(device, kind, 200, layout) as db:
        db.append(recs[:3])                                 # loads append after existing records
        assert db.load_file(path, first=10, count=50) == 50
        assert db.load_file(path, first=90) == 11          # to the end of the file
        assert len(db) == 64
        got = db.read(0, 64)
        assert (got[:3] == recs[:3]).all()
        assert (got[3:53] == recs[10:60]).all()
        assert (got[53:] == recs[90:]).all()
        out = tmp_path / "out.bin"
        db.save_file(out, first=3, n=50)
        assert out.read_bytes() == recs[10:60].tobytes()


def test_invalid_file_size(device, tmp_path):
    """A partial record is rejected like bytemuck::try_cast_slice (src/main.rs:390-393)."""
    path = tmp_path / "x.share-0"
    path.write_bytes(b"\0" * (25600 * 2 + 7))
    with ih.Database(device, ih.KIND_SHARES, 10) as db:
        with pytest.raises(ih.IrisError) as ei:
            db.load_file(path)
        assert ei.value.code == -1 and "invalid" in str(ei.value)
        assert len(db) == 0
        with pytest.raises(ih.IrisError) as ei:
            db.load_file(tmp_path / "missing.masks")
        assert ei.value.code == -6


def test_capacity_checked(device, tmp_path):
    path = tmp_path / "m.masks"
    _records(1, np.uint64, 200, 200, 1).tofile(path)
    with ih.Database(device, ih.KIND_MASKS, 10) as db:
        cap = db.capacity  # rounded up to whole tiles
        assert 10 <= cap < 200
        with pytest.raises(ih.IrisError) as ei:
            db.load_file(path)
        assert ei.value.code == -5 and len(db) == 0
        assert db.load_file(path, count=cap) == cap


@pytest.fixture(params=["slots", "windows", "pread"])
def load_device(request, device, hooked_device):
    """The loader's three paths: reader threads pread into the two pinned upload slots (the
    default for a load with no other in flight), DMA from registered page-cache windows of the
    mapping (a concurrent per-device load in a group; forced by the IRIS_LOAD_WINDOWS test
    hook), and pread into the loader's own pinned buffers (the fallback when the pages cannot
    be registered; forced by IRIS_LOAD_PREAD)."""
    if request.param == "pread":
        return hooked_device(IRIS_LOAD_PREAD="1")
    if request.param == "windows":
        return hooked_device(IRIS_LOAD_WINDOWS="1")
    return device


def test_multi_chunk_unaligned_templates(load_device, tmp_path):
    """A 96-MB template file loaded from an unaligned first record: a short leading chunk up
    to a page-aligned record boundary, then full chunks, then a ragged last one."""
    device = load_device
    n, first = 30_000, 13
    recs = oc.gen_templates(91, 0, n)
    path = tmp_path / "t.bin"
    recs.tofile(path)
    with ih.Database(device, ih.KIND_TEMPLATES, n) as db:
        assert db.load_file(path, first=first) == n - first
        assert (db.read(0, n - first) == recs[first:]).all()


def test_multi_chunk_masks_file(load_device, tmp_path):
    """50 000 masks = 80 MB: more than one 64 MB pinned buffer, so the double
    buffering and chunk offsets are exercised; then the engine runs on it."""
    device = load_device
    n = 50_000
    recs = oc.gen_templates(77, 0, n)[:, 200:].copy()
    path = tmp_path / "big.masks"
    recs.tofile(path)
    q = oc.gen_templates(78, 0, 1)[0]
    with ih.Database(device, ih.KIND_MASKS, n) as db, ih.MasksEngine(device, q[200:]) as eng:
        assert db.load_file(path) == n
        idx = np.array([0, 1, 41919, 41920, 41942, 41943, 41944, n - 1])  # around the chunk boundaries
        assert (db.read(0, n) == recs).all()
        out = np.empty((n, ROT), np.uint16)
        eng.batch_process(out, db)
        assert (out[idx] == oc.masks_batch(q[200:], recs[idx])).all()


def test_mpc_from_files(device, tmp_path):
    """`prepare` output files (masks + 2 shares, written like src/main.rs:333-372)
    loaded by the participants / resolver; fused resolver == plaintext search."""
    n = 2000
    templates = oc.gen_templates(93, 0, n)
    q = templates[777].copy()
    q[200:203] = 0
    enc = np.stack([oc.encode(t) for t in templates])
    s0 = np.random.default_rng(9).integers(0, 2**16, enc.shape, dtype=np.uint16)
    s1 = (enc - s0).astype(np.uint16)
    templates[:, 200:].tofile(tmp_path / "db.masks")
    s0.tofile(tmp_path / "db.share-0")
    s1.tofile(tmp_path / "db.share-1")
    ih.write_templates_json(tmp_path / "db.json", templates)
    enc_q = ih.encode(ih.Template.from_array(q))
    outs = []
    for i in range(2):
        with ih.Database(device, ih.KIND_SHARES, n) as db, ih.DistanceEngine(device, enc_q) as eng:
            db.load_file(tmp_path / f"db.share-{i}")
            out = np.empty((n, ROT), np.uint16)
            eng.batch_process(out, db)
            outs.append(out)
    with ih.Database(device, ih.KIND_MASKS, n) as mdb, ih.MasksEngine(device, q[200:]) as me:
        mdb.load_file(tmp_path / "db.masks")
        den = np.empty((n, ROT), np.uint16)
        me.batch_process(den, mdb)
    m = ih.resolver_search(outs, den, device=device)
    with ih.Database(device, ih.KIND_TEMPLATES, n) as tdb, ih.TemplateEngine(device, q) as te:
        tdb.append(ih.read_templates_json(tmp_path / "db.json"))
        ref = te.search(tdb)
    best, idx = oc.argmin(oc.template_distances(q, templates))
    assert m.index == ref.index == idx == 777
    assert np.float64(m.distance).view(np.uint64) == np.float64(best).view(np.uint64)
