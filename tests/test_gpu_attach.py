"""GPU: host residency (iris_db_attach_host).  The reference's participant and resolver
mmap their record file and call batch_process(out, chunk) on 20 000-record slices of the
mapping (src/main.rs:389-391, 426-431; 458-460, 511-516).  Once the array is attached, a
host-slice call on any range inside it runs on the resident copy: its rows equal the
oracle's and no record is uploaded (no "pack" launch); slices of other arrays, and of an
array whose database was modified, still take the upload path."""
import numpy as np
import pytest

import iris_hip as ih
import readahead_policy as ra_policy
from oracle import oracle_c as oc

pytestmark = pytest.mark.gpu
SEED = 31


def pack_launches(dev):
    return dev.kernel_stats("pack")[0]


@pytest.mark.parametrize("kind", [ih.KIND_MASKS, ih.KIND_SHARES])
@pytest.mark.parametrize("layout", [ih.LAYOUT_TILES, ih.LAYOUT_LANES])
def test_attached_slices_run_resident(device, kind, layout):
    n = 3001 if kind == ih.KIND_MASKS else 700
    host = oc.gen_masks(SEED, 0, n) if kind == ih.KIND_MASKS else oc.gen_shares(SEED, 0, n)
    qt = oc.gen_templates(SEED + 1, 0, 1)[0]
    if kind == ih.KIND_MASKS:
        eng, want = ih.MasksEngine(device, qt[200:]), oc.masks_batch(qt[200:], host)
    else:
        q = oc.encode(qt)
        eng, want = ih.DistanceEngine(device, q), oc.distance_batch(q, host)
    with eng, ih.Database(device, kind, n, layout) as db:
        db.attach_host(host)
        device.reset_stats()
        device.set_profiling(True)
        try:
            for a, b in ((0, n), (0, 1), (n - 1, n), (17, 17 + 333), (64, 65), (n // 2, n)):
                out = np.empty((b - a, 31), np.uint16)
                eng.batch_process(out, host[a:b])
                assert (out == want[a:b]).all(), (a, b)
            device.synchronize()
            assert pack_launches(device) == 0  # nothing uploaded
            # a copy of the same records is another host array: uploaded
            out = np.empty((10, 31), np.uint16)
            eng.batch_process(out, host[5:15].copy())
            assert (out == want[5:15]).all()
            device.synchronize()
            assert pack_launches(device) > 0
        finally:
            device.set_profiling(False)


def test_attach_without_upload_and_detach_on_write(device, tmp_path):
    n = 2000
    host = oc.gen_masks(SEED, 0, n)
    path = tmp_path / "m.masks"
    host.tofile(path)
    q = oc.gen_masks(SEED + 2, 0, 1)[0]
    want = oc.masks_batch(q, host)
    with ih.MasksEngine(device, q) as eng, ih.Database(device, ih.KIND_MASKS, n) as db:
        db.load_file(path)
        bad = host.copy()
        bad[n - 1, 3] ^= np.uint64(1)
        with pytest.raises(ih.IrisError):
            db.attach_host(bad, upload=False)  # the last record differs
        db.attach_host(host, upload=False)
        device.reset_stats()
        device.set_profiling(True)
        try:
            out = np.empty((500, 31), np.uint16)
            eng.batch_process(out, host[1000:1500])
            assert (out == want[1000:1500]).all()
            device.synchronize()
            assert pack_launches(device) == 0
            db.write(0, host[:1])  # any write detaches: the next slice call uploads again
            eng.batch_process(out, host[1000:1500])
            assert (out == want[1000:1500]).all()
            device.synchronize()
            assert pack_launches(device) > 1
        finally:
            device.set_profiling(False)
        with pytest.raises(ih.IrisError):
            db.attach_host(host, upload=True)  # upload needs an empty database


def test_attach_kind_and_alignment_rules(device):
    n = 300
    host = oc.gen_masks(SEED, 0, n)
    q = oc.gen_masks(SEED + 3, 0, 1)[0]
    with ih.Database(device, ih.KIND_MASKS, n) as db, ih.MasksEngine(device, q) as eng:
        db.attach_host(host)
        device.reset_stats()
        device.set_profiling(True)
        try:
            # a range that is not whole records of the array (shifted by one u64) is uploaded
            flat = host.reshape(-1)
            shifted = flat[1:1 + 200 * 10].reshape(10, 200)
            out = np.empty((10, 31), np.uint16)
            eng.batch_process(out, shifted)
            assert (out == oc.masks_batch(q, shifted.copy())).all()
            device.synchronize()
            assert pack_launches(device) > 0
        finally:
            device.set_profiling(False)
    with pytest.raises(ih.IrisError):  # layout 3 (the removed TRITS layout) is unknown
        ih.Database(device, ih.KIND_TEMPLATES, 10, 3)


def launches(dev, name):
    return dev.kernel_stats(name)[0]


@pytest.mark.parametrize("kind", [ih.KIND_MASKS, ih.KIND_SHARES])
@pytest.mark.parametrize("readahead", ["1", "0"])
def test_attached_chunk_walk_readahead(device, hooked_device, kind, readahead):
    """The reference's loop (src/main.rs:427-431, 511-516): consecutive equal chunks of the
    attached file, the last one short.  With readahead every chunk after the first comes from
    the engine's read-ahead windows (growing: 2, 4, ... chunks per launch, tests/readahead_policy.py),
    every record computed once."""
    if readahead == "0":  # a production knob, read when the device opens
        device = hooked_device(IRIS_READAHEAD="0")
        assert device.config()["readahead"] == "0"
    n, chunk = (5003, 1000) if kind == ih.KIND_MASKS else (1301, 300)
    host = oc.gen_masks(SEED + 5, 0, n) if kind == ih.KIND_MASKS else oc.gen_shares(SEED + 5, 0, n)
    qt = oc.gen_templates(SEED + 6, 0, 1)[0]
    if kind == ih.KIND_MASKS:
        eng, want, kname = ih.MasksEngine(device, qt[200:]), oc.masks_batch(qt[200:], host), "masks"
    else:
        q = oc.encode(qt)
        eng, want, kname = ih.DistanceEngine(device, q), oc.distance_batch(q, host), "shares"
    with eng, ih.Database(device, kind, n) as db:
        db.attach_host(host)
        device.reset_stats()
        device.set_profiling(True)
        try:
            per_walk = (n + chunk - 1) // chunk
            for walk in range(2):
                for a in range(0, n, chunk):
                    out = np.empty((min(chunk, n - a), 31), np.uint16)
                    eng.batch_process(out, host[a:a + chunk])
                    assert (out == want[a:a + chunk]).all(), (walk, a)
                device.synchronize()
                nl, _, items = device.kernel_stats(kname)
                if readahead == "0":
                    assert nl == per_walk * (walk + 1) and items == n * (walk + 1)
                elif walk == 0:  # chunk 0, then the growing windows: every record computed once
                    assert nl == len(ra_policy.windows(n, chunk)) and items == n, (nl, items)
                    assert ra_policy.counters(device) == (nl, n, max(ra_policy.windows(n, chunk)))
                else:  # the second walk recomputes at most its first chunk (the window its
                    # rows were in was regrown)
                    assert nl <= 2 * len(ra_policy.windows(n, chunk)) + 1 and items <= 2 * n + chunk, (nl, items)
            assert launches(device, "pack") == 0
            # out of order: every call still returns its own rows (misses recompute)
            for a, b in ((2000 % n, 2000 % n + 7), (0, chunk), (0, chunk), (n - 5, n), (chunk, 2 * chunk), (1, 2)):
                out = np.empty((b - a, 31), np.uint16)
                eng.batch_process(out, host[a:b])
                assert (out == want[a:b]).all(), (a, b)
        finally:
            device.set_profiling(False)


def test_readahead_dropped_when_attachment_changes(device):
    """A read-ahead chunk belongs to one attachment: rewriting the database and re-attaching
    the same host buffer with new contents (same address) must not serve the old rows."""
    n, chunk = 4000, 1000
    host = oc.gen_masks(SEED + 7, 0, n)
    new = oc.gen_masks(SEED + 8, 0, n)
    q = oc.gen_masks(SEED + 9, 0, 1)[0]
    with ih.MasksEngine(device, q) as eng, ih.Database(device, ih.KIND_MASKS, n) as db:
        db.attach_host(host)
        out = np.empty((chunk, 31), np.uint16)
        eng.batch_process(out, host[:chunk])  # chunk 1 is now read ahead from the old contents
        assert (out == oc.masks_batch(q, host[:chunk])).all()
        with pytest.raises(ValueError):  # read-only while attached (the device copy would not see it)
            host[0, 0] = 1
        db.detach_host()
        host[:] = new
        db.write(0, host)
        db.attach_host(host, upload=False)  # same address, new attachment
        eng.batch_process(out, host[chunk:2 * chunk])
        assert (out == oc.masks_batch(q, new[chunk:2 * chunk])).all()
        # and an engine destroyed with a read-ahead in flight releases it
        eng.batch_process(out, host[2 * chunk:3 * chunk])
    device.synchronize()


def test_resident_range_walk_readahead(device):
    """iris_engine_batch_process over consecutive ranges of a resident database (host output)
    reads ahead too; a write into the database between two calls drops the read-ahead rows."""
    n, chunk = 3500, 800
    recs = oc.gen_masks(SEED + 10, 0, n)
    q = oc.gen_masks(SEED + 11, 0, 1)[0]
    with ih.MasksEngine(device, q) as eng, ih.Database(device, ih.KIND_MASKS, n) as db:
        db.append(recs)
        want = oc.masks_batch(q, recs)
        device.reset_stats()
        device.set_profiling(True)
        try:
            for a in range(0, n, chunk):
                m = min(chunk, n - a)
                out = np.empty((m, 31), np.uint16)
                eng.batch_process(out, db, first=a, n=m)
                assert (out == want[a:a + m]).all(), a
            device.synchronize()
            nl, _, items = device.kernel_stats("masks")
            assert items == n and 1 < nl < (n + chunk - 1) // chunk  # windows of chunks, each record once
        finally:
            device.set_profiling(False)
        out = np.empty((chunk, 31), np.uint16)
        eng.batch_process(out, db, first=0, n=chunk)  # [chunk, 2 chunk) is read ahead now
        recs[chunk:2 * chunk] = oc.gen_masks(SEED + 12, 0, chunk)
        db.write(chunk, recs[chunk:2 * chunk])
        eng.batch_process(out, db, first=chunk, n=chunk)
        assert (out == oc.masks_batch(q, recs[chunk:2 * chunk])).all()


@pytest.mark.parametrize("kind", [ih.KIND_MASKS, ih.KIND_SHARES])
def test_participant_sized_chunks(device, kind):
    """20 000-record chunks (1.24 MB of rows each: the read-ahead's helper-thread copy path),
    consecutive and then repeated, against the oracle."""
    n, chunk = (45_000, 20_000) if kind == ih.KIND_MASKS else (25_000, 20_000)
    host = oc.gen_masks(SEED + 13, 0, n) if kind == ih.KIND_MASKS else oc.gen_shares(SEED + 13, 0, n)
    qt = oc.gen_templates(SEED + 14, 0, 1)[0]
    if kind == ih.KIND_MASKS:
        eng, want = ih.MasksEngine(device, qt[200:]), oc.masks_batch(qt[200:], host)
    else:
        q = oc.encode(qt)
        eng, want = ih.DistanceEngine(device, q), oc.distance_batch(q, host)
    with eng, ih.Database(device, kind, n) as db:
        db.attach_host(host)
        for a in list(range(0, n, chunk)) + [0, 0, chunk]:
            out = np.empty((min(chunk, n - a), 31), np.uint16)
            eng.batch_process(out, host[a:a + chunk])
            assert (out == want[a:a + chunk]).all(), a


def test_concurrent_chunk_walks(device):
    """The participant and the resolver run their loops in worker threads (src/main.rs:425, 510):
    two threads, each with its own engine, walk one attached array in 20 000-record chunks at the
    same time (read-ahead kernels interleave on the side stream, copies share the helper pool)."""
    import threading

    n, chunk = 60_000, 20_000
    host = oc.gen_masks(SEED + 15, 0, n)
    qs = oc.gen_masks(SEED + 16, 0, 2)
    wants = [oc.masks_batch(q, host) for q in qs]
    errors = []
    with ih.Database(device, ih.KIND_MASKS, n) as db:
        db.attach_host(host)

        def walk(i):
            try:
                with ih.MasksEngine(device, qs[i]) as eng:
                    for rep in range(3):
                        for a in range(0, n, chunk):
                            out = np.empty((chunk, 31), np.uint16)
                            eng.batch_process(out, host[a:a + chunk])
                            if not (out == wants[i][a:a + chunk]).all():
                                errors.append((i, rep, a))
            except Exception as ex:  # reported below
                errors.append((i, repr(ex)))

        threads = [threading.Thread(target=walk, args=(i,)) for i in range(2)]
        for th in threads:
            th.start()
        for th in threads:
            th.join()
    assert not errors, errors


@pytest.mark.parametrize("kind", [ih.KIND_MASKS, ih.KIND_SHARES])
def test_fresh_engine_first_call(device, kind):
    """An engine's query tables are built on the device stream when it is created, and a database
    is written there too; the read-ahead kernels run on the side stream, so the first call of a
    fresh engine must be ordered after both (engines reuse pooled query buffers: a call that ran
    early would see the previous engine's query)."""
    n = 3000 if kind == ih.KIND_MASKS else 600
    rng = np.random.default_rng(77)
    for it in range(6):
        host = (oc.gen_masks(SEED + 20 + it, 0, n) if kind == ih.KIND_MASKS
                else oc.gen_shares(SEED + 20 + it, 0, n))
        qt = oc.gen_templates(SEED + 40 + it, 0, 1)[0]
        with ih.Database(device, kind, n) as db:
            db.append(host)
            if kind == ih.KIND_MASKS:
                eng, want = ih.MasksEngine(device, qt[200:]), oc.masks_batch(qt[200:], host)
            else:
                q = oc.encode(qt)
                eng, want = ih.DistanceEngine(device, q), oc.distance_batch(q, host)
            with eng:
                out = np.empty((n, 31), np.uint16)
                eng.batch_process(out, db)
                assert (out == want).all(), it
                a = int(rng.integers(0, n - 10))
                out2 = np.empty((10, 31), np.uint16)
                eng.batch_process(out2, db, first=a, n=10)
                assert (out2 == want[a:a + 10]).all(), it


@pytest.mark.parametrize("kind", [ih.KIND_MASKS, ih.KIND_SHARES])
def test_device_output_chunks_return_on_completion_word(device, kind):
    """Participant-sized device-output calls (iris_engine_batch_process_device) return when the
    kernel's last workgroup publishes the completion word, not at the stream's end: chunk after
    chunk into the SAME device buffer (each call's rows overwrite the last one's), each read back
    at once and compared with the oracle, with a ragged last chunk, a one-record call and the
    other engine kind interleaved on the same device stream."""
    if kind == ih.KIND_MASKS:
        n, chunk = 45_001, 20_000
        recs = oc.gen_masks(SEED + 20, 0, n)
        q = oc.gen_masks(SEED + 21, 0, 1)[0]
        eng, oracle = ih.MasksEngine(device, q), (lambda r: oc.masks_batch(q, r))
        other_kind, other_recs = ih.KIND_SHARES, oc.gen_shares(SEED + 22, 0, 64)
        other_q = oc.gen_shares(SEED + 23, 0, 1)[0]
        other = ih.DistanceEngine(device, other_q)
        other_want = oc.distance_batch(other_q, other_recs)
    else:
        n, chunk = 4_501, 2_000
        recs = oc.gen_shares(SEED + 24, 0, n)
        q = oc.gen_shares(SEED + 25, 0, 1)[0]
        eng, oracle = ih.DistanceEngine(device, q), (lambda r: oc.distance_batch(q, r))
        other_kind, other_recs = ih.KIND_MASKS, oc.gen_masks(SEED + 26, 0, 64)
        other_q = oc.gen_masks(SEED + 27, 0, 1)[0]
        other = ih.MasksEngine(device, other_q)
        other_want = oc.masks_batch(other_q, other_recs)
    want = oracle(recs)
    with eng, other, ih.Database(device, kind, n) as db, ih.Database(device, other_kind, 64) as odb:
        db.append(recs)
        odb.append(other_recs)
        out = device.alloc(chunk * 31 * 2)
        oout = device.alloc(64 * 31 * 2)
        try:
            for walk in range(2):
                for a in list(range(0, n, chunk)) + [n - 1]:
                    m = min(chunk, n - a)
                    eng.batch_process_device(db, out, first=a, n=m)
                    other.batch_process_device(odb, oout)
                    rows = np.empty((m, 31), np.uint16)
                    device.d2h(rows, out)
                    assert (rows == want[a:a + m]).all(), (walk, a)
                    orows = np.empty((64, 31), np.uint16)
                    device.d2h(orows, oout)
                    assert (orows == other_want).all(), (walk, a)
        finally:
            device.free(out)
            device.free(oout)


@pytest.mark.parametrize("kind", [ih.KIND_MASKS, ih.KIND_SHARES])
def test_device_output_rows_visible_to_unordered_reader(device, kind):
    """A device-output call returns on the kernel's completion word, before the launch has ended
    (and before its end-of-kernel cache write-back): the rows must already be in memory for a
    reader that is not ordered after the library's stream -- here the runtime's own blocking
    hipMemcpy on the null stream, issued the moment the call returns (the library's stream is
    non-blocking, so nothing orders the two).  The signalling kernels write their rows through
    the XCD's L2 for this (store_tile_rows, wt).  A build without the write-through
    (-DIRIS_ROWS_WT=0) also passed on the box it ran on (gpurun_out r04l): the copy starts
    microseconds after the launch's own end-of-kernel write-back, so this pins the contract
    rather than catching the unfixed timing window."""
    import ctypes

    # the runtime the library runs on: the loaded object of its NEEDED soname (a process that also
    # imports torch maps torch's bundled libamdhip64.so too; "libamdhip64.so" may name that one)
    hip = ctypes.CDLL("libamdhip64.so.7")
    hip.hipMemcpy.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int]
    if kind == ih.KIND_MASKS:
        n, chunk = 60_000, 20_000
        recs = oc.gen_masks(SEED + 30, 0, n)
        q = oc.gen_masks(SEED + 31, 0, 1)[0]
        eng, want = ih.MasksEngine(device, q), oc.masks_batch(q, recs)
    else:
        n, chunk = 6_000, 2_000
        recs = oc.gen_shares(SEED + 32, 0, n)
        q = oc.gen_shares(SEED + 33, 0, 1)[0]
        eng, want = ih.DistanceEngine(device, q), oc.distance_batch(q, recs)
    with eng, ih.Database(device, kind, n) as db:
        db.append(recs)
        out = device.alloc(chunk * 31 * 2)
        rows = np.empty((chunk, 31), np.uint16)
        try:
            for it in range(12):
                a = (it % 3) * chunk  # each call overwrites the previous call's rows in the same buffer
                eng.batch_process_device(db, out, first=a, n=chunk)
                assert hip.hipMemcpy(rows.ctypes.data, out, rows.nbytes, 2) == 0  # hipMemcpyDeviceToHost
                assert (rows == want[a:a + chunk]).all(), it
        finally:
            device.free(out)
