"""GPU: the reference's call sites, unchanged, on a record file it maps.  The participant and
the resolver mmap their file read-only (memmap2's `map`: PROT_READ, MAP_SHARED) and call
batch_process(out, chunk) on 20 000-record slices of the mapping for every request
(src/main.rs:386-391, 426-431; 455-460, 511-516).  With no attach call, such a slice runs on
the device's copy of the file (iris_resident.hip): the first walk uploads it granule by
granule, later walks upload nothing ("pack" launches count uploads), and every row equals the
oracle's.  A rewritten file serves its new rows; a mapping replaced at the same address
serves the new file's; anonymous and writable arrays, and IRIS_AUTO_RESIDENT=0, keep the
per-call upload."""
import gc
import os

import numpy as np
import pytest

import iris_hip as ih
from oracle import oracle_c as oc

pytestmark = pytest.mark.gpu
SEED = 53
CHUNK = 20_000  # BATCH_SIZE, src/main.rs:428, 473


@pytest.fixture(autouse=True)
def no_resident_left(device):
    yield
    device.drop_resident()  # the session device keeps nothing from one test into the next


def gen(kind, seed, n):
    return oc.gen_masks(seed, 0, n) if kind == ih.KIND_MASKS else oc.gen_shares(seed, 0, n)


def engine_and_oracle(device, kind, seed):
    qt = oc.gen_templates(seed, 0, 1)[0]
    if kind == ih.KIND_MASKS:
        q = qt[200:]
        return ih.MasksEngine(device, q), lambda recs: oc.masks_batch(q, recs)
    q = oc.encode(qt)
    return ih.DistanceEngine(device, q), lambda recs: oc.distance_batch(q, recs)


def mapped(path, kind, n, mode="r"):
    dt, width = (np.uint64, 200) if kind == ih.KIND_MASKS else (np.uint16, 12800)
    return np.memmap(path, dtype=dt, mode=mode, shape=(n, width))


def walk(eng, recs, chunk=CHUNK):
    out = np.empty((recs.shape[0], 31), np.uint16)
    for a in range(0, recs.shape[0], chunk):
        eng.batch_process(out[a:a + chunk], recs[a:a + chunk])
    return out


def uploads(device):
    return device.kernel_stats("pack")[0]


def check_sample(out, recs, want_fn, rng, k=6):
    """Rows of k random 20k chunks' first/last 50 records plus the file's first and last rows."""
    n = recs.shape[0]
    idx = {0, n - 1}
    for a in rng.choice(max(1, n // CHUNK), min(k, max(1, n // CHUNK)), replace=False):
        a = int(a) * CHUNK
        idx.update(range(a, min(n, a + 50)))
        idx.update(range(max(0, min(n, a + CHUNK) - 50), min(n, a + CHUNK)))
    idx = np.array(sorted(idx))
    want = want_fn(np.ascontiguousarray(recs[idx]))
    assert (out[idx] == want).all()


@pytest.mark.parametrize("kind", [ih.KIND_MASKS, ih.KIND_SHARES], ids=["resolver-masks", "participant-shares"])
def test_mapped_file_walk_is_resident(device, tmp_path, kind):
    """Three granules (masks 400 000 x 1600 B, shares 25 000 x 25 600 B: ~640 MB either way) and
    a ragged last chunk: the first walk uploads each granule once, the second uploads nothing."""
    n = 400_003 if kind == ih.KIND_MASKS else 25_003
    path = tmp_path / "db.records"
    gen(kind, SEED, n).tofile(path)
    recs = mapped(path, kind, n)
    eng, want_fn = engine_and_oracle(device, kind, SEED + 1)
    rng = np.random.default_rng(5)
    with eng:
        device.reset_stats()
        device.set_profiling(True)
        try:
            first = walk(eng, recs)
            device.synchronize()
            up1 = uploads(device)
            assert up1 >= 3  # at least one upload per granule
            count, nbytes = device.resident()
            assert count == 1 and nbytes >= recs.nbytes, device.config()
            second = walk(eng, recs)
            third = walk(eng, recs, chunk=7_777)  # other slice sizes hit the same copy
            device.synchronize()
            assert uploads(device) == up1  # nothing uploaded after the first walk
        finally:
            device.set_profiling(False)
    assert (first == second).all() and (first == third).all()
    check_sample(first, recs, want_fn, rng)
    del recs


@pytest.mark.parametrize("restore_mtime", [False, True], ids=["new-mtime", "mtime-restored"])
def test_rewritten_file_serves_fresh_rows(device, tmp_path, restore_mtime):
    """The file is rewritten in place (same inode, same size) under the live mapping: the next
    walk's rows are the new records' (the stat check, or with the old mtime put back, the
    ctime / the slice probe, notices)."""
    kind, n = ih.KIND_MASKS, 45_001
    path = tmp_path / "m.masks"
    old, new = gen(kind, SEED, n), gen(kind, SEED + 7, n)
    old.tofile(path)
    recs = mapped(path, kind, n)
    eng, want_fn = engine_and_oracle(device, kind, SEED + 2)
    with eng:
        a = walk(eng, recs)
        assert (a == want_fn(old)).all()
        st = os.stat(path)
        with open(path, "r+b") as f:
            f.write(new.tobytes())
        if restore_mtime:
            os.utime(path, ns=(st.st_atime_ns, st.st_mtime_ns))
        else:
            os.utime(path, ns=(st.st_atime_ns, st.st_mtime_ns + 1_000_000_000))
        assert (np.asarray(recs[:3]) == new[:3]).all()  # the mapping shows the new bytes
        b = walk(eng, recs)
        assert (b == want_fn(new)).all()
    del recs


def test_mapping_replaced_at_same_address(device, tmp_path):
    """Unmap file A, map file B (same size): whatever address B lands at, its rows are B's."""
    kind, n = ih.KIND_MASKS, 30_000
    pa, pb = tmp_path / "a.masks", tmp_path / "b.masks"
    ra, rb = gen(kind, SEED + 3, n), gen(kind, SEED + 4, n)
    ra.tofile(pa)
    rb.tofile(pb)
    eng, want_fn = engine_and_oracle(device, kind, SEED + 5)
    with eng:
        ma = mapped(pa, kind, n)
        addr_a = ma.ctypes.data
        assert (walk(eng, ma) == want_fn(ra)).all()
        ma._mmap.close()
        del ma
        gc.collect()
        mb = mapped(pb, kind, n)
        same = mb.ctypes.data == addr_a
        assert (walk(eng, mb) == want_fn(rb)).all(), f"same address: {same}"
        del mb


@pytest.mark.parametrize("form", ["anonymous", "writable", "opted-out"])
def test_other_arrays_upload_per_call(device, hooked_device, tmp_path, monkeypatch, form):
    """An anonymous array, a writable (r+) mapping, and a device opened with IRIS_AUTO_RESIDENT=0
    upload on every walk and keep no copy; their rows equal the oracle's."""
    kind, n = ih.KIND_MASKS, 41_000
    host = gen(kind, SEED + 6, n)
    dev = device
    if form == "anonymous":
        recs = host
    else:
        path = tmp_path / "w.masks"
        host.tofile(path)
        recs = mapped(path, kind, n, mode="r+" if form == "writable" else "r")
        if form == "opted-out":
            with monkeypatch.context() as m:
                m.setenv("IRIS_AUTO_RESIDENT", "0")
                dev = ih.Device(0)
            assert dev.config()["auto_resident"] == "0"
    eng, want_fn = engine_and_oracle(dev, kind, SEED + 8)
    try:
        with eng:
            dev.reset_stats()
            dev.set_profiling(True)
            try:
                calls = -(-n // CHUNK)
                a = walk(eng, recs)
                dev.synchronize()
                u1 = uploads(dev)
                b = walk(eng, recs)
                dev.synchronize()
                # every call of both walks uploads (at least one pack launch each; the tuned upload
                # path may split a call's records into several)
                assert u1 >= calls and uploads(dev) - u1 >= calls, (u1, uploads(dev))
            finally:
                dev.set_profiling(False)
            assert dev.resident() == (0, 0)
        assert (a == b).all() and (a == want_fn(host)).all()
    finally:
        if dev is not device:
            dev.close()
    del recs


def test_drop_resident_and_unaligned_slices(device, tmp_path):
    """drop_resident frees the copy (the next walk uploads again); a view of the file on another
    record grid (8 bytes in) is still served correctly."""
    kind, n = ih.KIND_MASKS, 25_000
    path = tmp_path / "d.masks"
    host = gen(kind, SEED + 9, n)
    host.tofile(path)
    recs = mapped(path, kind, n)
    eng, want_fn = engine_and_oracle(device, kind, SEED + 10)
    want = want_fn(host)
    with eng:
        assert (walk(eng, recs) == want).all()
        assert device.resident()[0] == 1
        device.drop_resident()
        assert device.resident() == (0, 0)
        device.reset_stats()
        device.set_profiling(True)
        try:
            assert (walk(eng, recs) == want).all()
            device.synchronize()
            assert uploads(device) > 0
        finally:
            device.set_profiling(False)
        # bytes 8.. of a second mapping viewed as records: another record grid
        raw = np.memmap(path, dtype=np.uint64, mode="r")
        shifted = raw[1:1 + 200 * 100].reshape(100, 200)
        out = np.empty((100, 31), np.uint16)
        eng.batch_process(out, shifted)
        assert (out == want_fn(np.ascontiguousarray(shifted))).all()
        del raw, shifted
    del recs


def test_file_with_header_and_truncated_file(device, tmp_path):
    """Records after a 5000-byte header (the mapping starts at a page-aligned file offset, the
    records 904 bytes into it: the granules are read from the file at that offset); then the file
    is cut to fewer records under the live mapping: calls on the records still in the file serve
    them (the size change drops the copy, a new one of the shorter file is made)."""
    kind, n, hdr = ih.KIND_MASKS, 30_000, 5000
    path = tmp_path / "h.masks"
    host = gen(kind, SEED + 11, n)
    with open(path, "wb") as f:
        f.write(np.random.default_rng(1).integers(0, 256, hdr, dtype=np.uint8).tobytes())
        f.write(host.tobytes())
    recs = np.memmap(path, dtype=np.uint64, mode="r", offset=hdr, shape=(n, 200))
    eng, want_fn = engine_and_oracle(device, kind, SEED + 12)
    want = want_fn(host)
    with eng:
        assert (walk(eng, recs) == want).all()
        assert device.resident()[0] == 1, device.config()
        keep = 12_345
        os.truncate(path, hdr + keep * 1600)
        out = walk(eng, recs[:keep], chunk=5_000)
        assert (out == want[:keep]).all()
        assert device.resident()[0] == 1, device.config()
    del recs


def test_concurrent_walks_share_one_copy(device, tmp_path):
    """Two request threads (each its own engine and query, as concurrent participant requests)
    walk the same mapped file at once, three walks each: one resident copy serves both, and every
    walk's rows are its own query's (the engines' read-ahead windows never serve each other)."""
    import threading
    kind, n = ih.KIND_MASKS, 90_001
    path = tmp_path / "c.masks"
    host = gen(kind, SEED + 13, n)
    host.tofile(path)
    recs = mapped(path, kind, n)
    results, errors = {}, []

    def request(i):
        try:
            want = None
            for w in range(3):  # a new engine per walk, as per request
                eng, want_fn = engine_and_oracle(device, kind, SEED + 20 + i)
                with eng:
                    out = walk(eng, recs, chunk=CHUNK if i == 0 else 13_000)
                if want is None:
                    want = want_fn(host)
                results[(i, w)] = (out == want).all()
        except Exception as exc:  # reported by the main thread
            errors.append(repr(exc))

    threads = [threading.Thread(target=request, args=(i,)) for i in range(2)]
    for t in threads:
        t.start()
    for t in threads:
        t.join(timeout=100)
    assert not errors, errors
    assert len(results) == 6 and all(results.values()), results
    assert device.resident()[0] == 1
    del recs


def test_budget_evicts_least_recently_used_and_refuses_too_large(hooked_device, tmp_path):
    """IRIS_RESIDENT_BUDGET_MB (test hook) caps what the copies may hold, standing in for a full
    device: with room for one of two 160-MB files, walking the second evicts the first (least
    recently used) and walking the first again evicts the second; a 288-MB file is refused (it
    uploads every walk and iris_config says why) and the copy in place stays.  Rows equal the
    oracle's throughout."""
    kind, n, nbig = ih.KIND_MASKS, 100_000, 180_000
    dev = hooked_device(IRIS_RESIDENT_BUDGET_MB=250)
    files = []
    for i, cnt in enumerate((n, n, nbig)):
        p = tmp_path / f"f{i}.masks"
        h = gen(kind, SEED + 30 + i, cnt)
        h.tofile(p)
        files.append((h, mapped(p, kind, cnt)))
    eng, want_fn = engine_and_oracle(dev, kind, SEED + 33)
    wants = [want_fn(h) for h, _ in files]
    dev.set_profiling(True)
    try:
        with eng:
            def walk_uploads(i):
                dev.reset_stats()
                assert (walk(eng, files[i][1]) == wants[i]).all()
                dev.synchronize()
                return uploads(dev)

            assert walk_uploads(0) > 0 and dev.resident()[0] == 1
            assert walk_uploads(0) == 0
            assert walk_uploads(1) > 0 and dev.resident()[0] == 1  # file 0's copy evicted
            assert walk_uploads(1) == 0
            assert walk_uploads(0) > 0 and dev.resident()[0] == 1  # and back
            calls = -(-nbig // CHUNK)
            assert walk_uploads(2) >= calls and walk_uploads(2) >= calls  # refused: uploads per call
            assert "does_not_fit" in dev.config()["resident_skip"], dev.config()  # spaces show as _
            assert dev.resident()[0] == 1 and walk_uploads(0) == 0  # file 0's copy stayed
    finally:
        dev.set_profiling(False)
    del files
