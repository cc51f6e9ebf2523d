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
import readahead_policy as ra_policy
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


def test_concurrent_walk_and_resolver_host_forms(device, tmp_path):
    """A masks walk of a mapped file on one thread while another runs the resolver's host forms
    (iris_resolver_search_host and iris_resolver_search_masks_host, several upload chunks each) on
    the same device: they share the device's pinned upload slots, staging and helper pool (the
    device lock orders them); every result equals the oracle's."""
    import threading
    kind, n = ih.KIND_MASKS, 90_001
    path = tmp_path / "r.masks"
    host = gen(kind, SEED + 17, n)
    host.tofile(path)
    recs = mapped(path, kind, n)
    rng = np.random.default_rng(9)
    nr = 600_000  # > one 541k-record slot of summed shares + denominators
    parts = [rng.integers(0, 2**16, (nr, 31), dtype=np.uint16) for _ in range(3)]
    den = rng.integers(0, 12801, (nr, 31), dtype=np.uint16)
    want_r = oc.argmin(oc.resolver_combine(np.stack(parts), den))
    mq = host[n // 3].copy()
    sh = [p[:n] for p in parts]
    want_m = oc.argmin(oc.resolver_combine(np.stack(sh), oc.masks_batch(mq, host)))
    errors, ok = [], {}

    def walker():
        try:
            for w in range(3):
                eng, want_fn = engine_and_oracle(device, kind, SEED + 30 + w)
                with eng:
                    out = walk(eng, recs, chunk=CHUNK)
                ok[("walk", w)] = bool((out == want_fn(host)).all())
        except Exception as exc:
            errors.append(repr(exc))

    def resolver():
        try:
            with ih.Database(device, kind, n) as mdb, ih.MasksEngine(device, mq) as me:
                mdb.append(host)
                for r in range(3):
                    m = ih.resolver_search(parts, den, device=device)
                    ok[("host", r)] = m.index == want_r[1] and np.float64(m.distance) == np.float64(want_r[0])
                    mm = me.resolve(mdb, sh)
                    ok[("masks_host", r)] = mm.index == want_m[1] and np.float64(mm.distance) == np.float64(want_m[0])
        except Exception as exc:
            errors.append(repr(exc))

    threads = [threading.Thread(target=walker), threading.Thread(target=resolver)]
    for t in threads:
        t.start()
    for t in threads:
        t.join(timeout=100)
    assert not errors, errors
    assert len(ok) == 9 and all(ok.values()), ok
    del recs


def test_mpc_request_through_files(device, tmp_path):
    """The reference's MPC request end to end through its unchanged call sites (tools/mpc_request.py
    at test size): `prepare` writes three share files and a masks file (src/main.rs:333-361), each
    participant walks its mapped share file in 20k batch_process calls with a fresh engine
    (:386-431), the resolver loads the masks file and aggregates the participants' host rows with the
    fused step (iris_resolver_search_masks_host, :455-621); the answer equals the plaintext search
    and the oracle's."""
    n, k, rot = 45_001, 30_000, -5
    with ih.Database(device, ih.KIND_TEMPLATES, n) as tdb:
        tdb.generate(n, 77)
        templ = tdb.read(0, n)
        q = templ[k].copy()
        qp = ih.Bits(q[:200]).rotated(rot).limbs.copy()
        qp[9] ^= np.uint64(0x0F0F0F0F)
        query = np.concatenate([qp, ih.Bits(q[200:]).rotated(rot).limbs])
        with ih.TemplateEngine(device, query) as te:
            plain = te.search(tdb)
        sdbs = [ih.Database(device, ih.KIND_SHARES, n) for _ in range(3)]
        mdb = ih.Database(device, ih.KIND_MASKS, n)
        ih.prepare_shares(tdb, sdbs, mdb, key=bytes(range(32)))
        for i, sdb in enumerate(sdbs):
            sdb.save_file(tmp_path / f"db.share-{i}")
            sdb.close()
        mdb.save_file(tmp_path / "db.masks")
        mdb.close()
    best, idx = oc.argmin(oc.template_distances(query, templ))
    assert plain.index == idx == k
    shares = [mapped(tmp_path / f"db.share-{i}", ih.KIND_SHARES, n) for i in range(3)]
    enc_q = ih.encode(ih.Template.from_array(query))
    rows = []
    for i in range(3):
        with ih.DistanceEngine(device, enc_q) as e:
            rows.append(walk(e, shares[i]))
    with ih.Database(device, ih.KIND_MASKS, n) as rdb, ih.MasksEngine(device, query[200:]) as me:
        assert rdb.load_file(tmp_path / "db.masks") == n
        m = me.resolve(rdb, rows)
    assert m.index == plain.index == k and m.rotation == plain.rotation
    assert np.float64(m.distance).view(np.uint64) == np.float64(best).view(np.uint64)
    del shares


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


def walk_counted(device, eng, recs, chunk):
    device.reset_stats()
    out = walk(eng, recs, chunk)
    device.synchronize()
    return out, ra_policy.counters(device)


@pytest.mark.parametrize("kind,n,chunk", [(ih.KIND_MASKS, 1_200_000, CHUNK), (ih.KIND_SHARES, 100_000, 2_000)],
                         ids=["masks-1.2M", "shares-100k"])
def test_long_walk_windows_grow(device, hooked_device, tmp_path, kind, n, chunk):
    """A long walk of a mapped file (masks: 1.2M records in the resolver's 20k chunks, 1.9 GB;
    shares: 100k in 2 000-record chunks, 2.6 GB): after the untimed first walk, a walk with a
    fresh engine reads ahead in windows of 1, 2, 4, ... chunks up to the rows cap, then shrinking
    to the walk's end -- counted by the library (readahead_windows: launches, records, largest
    window), each record computed exactly once.  Rows equal the oracle on samples and, all of them,
    the rows of the same walk on a device that computes every call alone (IRIS_READAHEAD=0)."""
    path = tmp_path / "long.records"
    gen(kind, SEED + 40, n).tofile(path)
    recs = mapped(path, kind, n)
    rng = np.random.default_rng(8)
    want_windows = ra_policy.windows(n, chunk)
    qt = oc.gen_templates(SEED + 41, 0, 1)[0]
    q = qt[200:] if kind == ih.KIND_MASKS else oc.encode(qt)
    Eng = ih.MasksEngine if kind == ih.KIND_MASKS else ih.DistanceEngine
    with Eng(device, q) as eng:
        walk(eng, recs, chunk)  # makes the file resident
    with Eng(device, q) as eng:
        out, (launches, records, largest) = walk_counted(device, eng, recs, chunk)
    assert records == n, (records, n)  # every record once
    assert (launches, largest) == (len(want_windows), max(want_windows)), (launches, largest, want_windows)
    assert max(want_windows) >= 4 * chunk
    idx = np.unique(np.concatenate([rng.choice(n, 300, replace=False), [0, n - 1, chunk - 1, chunk]]))
    sample = np.ascontiguousarray(recs[idx])
    want = oc.masks_batch(q, sample) if kind == ih.KIND_MASKS else oc.distance_batch(q, sample)
    assert (out[idx] == want).all()
    plain = hooked_device(IRIS_READAHEAD="0")
    with Eng(plain, q) as eng:
        ref = walk(eng, recs, chunk)
    assert (out == ref).all()
    del recs


def structured_masks(n, rng, block_every=3):
    """Masks where every `block_every`-th record is a block of columns (an occlusion-like mask:
    columns [c0, c0 + w) of every row), the rest uniform random: against a block query the block
    records' counts change by 64 per column of rotation, so most of their rows span far more than
    a byte and take the packed form's escape path (store_tile_packed)."""
    out = oc.gen_masks(int(rng.integers(1 << 30)), 0, n)
    for i in range(0, n, block_every):
        c0, w = int(rng.integers(0, 200)), int(rng.integers(20, 120))
        bits = np.zeros((64, 200), np.uint8)
        bits[:, (np.arange(w) + c0) % 200] = 1
        out[i] = np.packbits(bits.reshape(12800), bitorder="little").view(np.uint64)
    return out


def test_packed_rows_escape_path(device, hooked_device, tmp_path):
    """The masks read-ahead's rows cross the host link packed (32 B per record, a base + 31 byte
    offsets); a row whose 31 counts span more than a byte escapes to a full row.  A block query
    mask (columns 40..109) against a file of random and block masks: every row of a 20k-chunk walk
    equals the oracle's, escaped and packed alike, and equals the same walk with the packing off
    (IRIS_READAHEAD_PACKED=0)."""
    n = 90_001
    rng = np.random.default_rng(9)
    host = structured_masks(n, rng)
    qbits = np.zeros((64, 200), np.uint8)
    qbits[:, 40:110] = 1
    q = np.packbits(qbits.reshape(12800), bitorder="little").view(np.uint64)
    want = oc.masks_batch(q, host)
    spans = want.max(axis=1).astype(int) - (want.min(axis=1).astype(int) // 64) * 64
    assert (spans > 255).sum() > n // 6 and (spans <= 255).sum() > n // 2  # both forms occur
    path = tmp_path / "s.masks"
    host.tofile(path)
    recs = mapped(path, ih.KIND_MASKS, n)
    with ih.MasksEngine(device, q) as eng:
        for _ in range(2):  # the first walk fills the copy, the second is all read-ahead windows
            assert (walk(eng, recs) == want).all()
    unpacked = hooked_device(IRIS_READAHEAD_PACKED="0")
    with ih.MasksEngine(unpacked, q) as eng:
        assert (walk(eng, recs) == want).all()
        assert (walk(eng, recs, chunk=7_777) == want).all()
    del recs


def test_drop_resident_range_after_writes_through_a_mapping(device, tmp_path):
    """Records rewritten in place through a second, writable mapping of the file (np.memmap r+, the
    store path whose timestamps the per-call check may not see once the pages are dirty): after
    iris_device_drop_resident_range on the read-only mapping, the next walk copies the file afresh
    and serves the new rows.  The call leaves other files' copies alone and is a no-op on an
    address without a copy."""
    kind, n = ih.KIND_MASKS, 45_000
    pa, pb = tmp_path / "a.masks", tmp_path / "b.masks"
    old, new, other = gen(kind, SEED + 50, n), gen(kind, SEED + 51, n), gen(kind, SEED + 52, n)
    old.tofile(pa)
    other.tofile(pb)
    recs, recs_b = mapped(pa, kind, n), mapped(pb, kind, n)
    eng, want_fn = engine_and_oracle(device, kind, SEED + 53)
    with eng:
        assert (walk(eng, recs) == want_fn(old)).all()
        assert (walk(eng, recs_b) == want_fn(other)).all()
        assert device.resident()[0] == 2
        rw = np.memmap(pa, dtype=np.uint64, mode="r+", shape=(n, 200))
        sl = slice(1_000, 31_000)
        rw[sl] = new[sl]
        rw.flush()
        del rw
        old[sl] = new[sl]
        device.drop_resident_range(recs[5])  # any address inside the mapping
        assert device.resident()[0] == 1  # b's copy stays
        device.drop_resident_range(np.zeros(4))  # no copy there
        assert device.resident()[0] == 1
        assert (walk(eng, recs) == want_fn(old)).all()
        assert device.resident()[0] == 2
    del recs, recs_b


def test_copies_of_unmapped_files_are_swept(device, tmp_path):
    """A copy whose mapping was unmapped frees its device memory at the next device sync (or
    host-slice call) a second later, without a make_resident pass to notice it."""
    import time
    kind, n = ih.KIND_MASKS, 25_000
    path = tmp_path / "u.masks"
    gen(kind, SEED + 60, n).tofile(path)
    recs = mapped(path, kind, n)
    eng, _ = engine_and_oracle(device, kind, SEED + 61)
    with eng:
        walk(eng, recs)
    assert device.resident()[0] == 1
    recs._mmap.close()
    del recs
    gc.collect()
    time.sleep(1.2)
    device.synchronize()
    assert device.resident() == (0, 0), device.config()


def test_device_alloc_evicts_resident_copies(device, tmp_path):
    """Device memory held by resident copies is a cache: an iris_device_alloc that does not fit
    beside them evicts them (least recently used first) instead of failing."""
    kind, n = ih.KIND_MASKS, 1_300_000  # a ~2 GB copy
    path = tmp_path / "e.masks"
    gen(kind, SEED + 62, n).tofile(path)
    recs = mapped(path, kind, n)
    eng, _ = engine_and_oracle(device, kind, SEED + 63)
    with eng:
        walk(eng, recs[:40_000])
    count, held = device.resident()
    assert count == 1 and held >= n * 1600
    free, _ = device.memory()
    ptrs = []
    try:
        ptrs.append(device.alloc(free - (1 << 30)))  # leaves 1 GB beside the 2-GB copy
        ptrs.append(device.alloc(2 << 30))  # fits only once the copy is gone
        assert device.resident() == (0, 0)
    finally:
        for p in ptrs:
            device.free(p)
    del recs


def test_same_file_remapped_at_another_offset(device, tmp_path):
    """The same file unmapped and mapped again from another file offset (64 records = 100 KiB in,
    page aligned), wherever the new mapping lands -- at the old address the file's inode, size and
    times all still match: the rows are those of the records at the new offset."""
    kind, n, skip = ih.KIND_MASKS, 40_000, 64
    path = tmp_path / "o.masks"
    host = gen(kind, SEED + 70, n)
    host.tofile(path)
    eng, want_fn = engine_and_oracle(device, kind, SEED + 71)
    want = want_fn(host)
    with eng:
        a = mapped(path, kind, n)
        assert (walk(eng, a) == want).all()
        a._mmap.close()
        del a
        gc.collect()
        b = np.memmap(path, dtype=np.uint64, mode="r", offset=skip * 1600, shape=(n - skip, 200))
        assert (walk(eng, b) == want[skip:]).all()
        del b


def test_resident_cap_production_knob(monkeypatch, tmp_path):
    """IRIS_RESIDENT_MAX_MB (production knob, no test opt-in): the copies together hold at most
    that much; a file above it is refused (it uploads per call, iris_config says why), one below
    it is kept.  Rows equal the oracle either way."""
    kind, small, big = ih.KIND_MASKS, 60_000, 150_000  # 96 MB and 240 MB
    files = []
    for i, cnt in enumerate((small, big)):
        p = tmp_path / f"cap{i}.masks"
        h = gen(kind, SEED + 80 + i, cnt)
        h.tofile(p)
        files.append((h, mapped(p, kind, cnt)))
    with monkeypatch.context() as m:
        m.setenv("IRIS_RESIDENT_MAX_MB", "200")
        dev = ih.Device(0)
    try:
        assert dev.config()["resident_max_mb"] == "200" and "ignored" not in dev.config()
        eng, want_fn = engine_and_oracle(dev, kind, SEED + 82)
        with eng:
            assert (walk(eng, files[0][1]) == want_fn(files[0][0])).all()
            assert dev.resident()[0] == 1
            assert (walk(eng, files[1][1]) == want_fn(files[1][0])).all()
            assert "cap" in dev.config()["resident_skip"], dev.config()
            assert dev.resident()[0] == 1 and dev.resident()[1] < 200 << 20
    finally:
        dev.drop_resident()
        dev.close()
    del files


def test_kernel_stats_largest(device):
    """iris_device_kernel_stats_largest: the largest launch of a kernel family since the last reset
    (a walk's biggest read-ahead window) and its duration."""
    n = 50_000
    q = oc.gen_masks(SEED + 90, 0, 1)[0]
    with ih.Database(device, ih.KIND_MASKS, n) as db, ih.MasksEngine(device, q) as eng:
        db.generate(n, SEED + 91)
        out = device.alloc(n * 31 * 2)
        try:
            device.reset_stats()
            device.set_profiling(True)
            for m in (1_000, n, 7_000):
                eng.batch_process_device(db, out, 0, m)
            device.synchronize()
            items, ms = device.kernel_stats_largest("masks")
            assert items == n and ms > 0
            device.reset_stats()
            assert device.kernel_stats_largest("masks") == (0, 0.0)
        finally:
            device.set_profiling(False)
            device.free(out)
