"""GPU: host residency (iris_db_attach_host).  The reference's participant and resolver
mmap their record file and call batch_process(out, chunk) on 20 000-record slices of the
mapping (src/main.rs:389-391, 426-431; 458-460, 511-516).  Once the array is attached, a
host-slice call on any range inside it runs on the resident copy: its rows equal the
oracle's and no record is uploaded (no "pack" launch); slices of other arrays, and of an
array whose database was modified, still take the upload path."""
import numpy as np
import pytest

import iris_hip as ih
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
    with ih.Database(device, ih.KIND_TEMPLATES, 10, ih.LAYOUT_TRITS) as tdb:
        with pytest.raises(ih.IrisError):
            tdb.attach_host(oc.gen_templates(1, 0, 10))  # search-only layout: not exact records
        tdb.generate(10, 1)
        with pytest.raises(ih.IrisError):
            tdb.save_file("/tmp/never_written.templates")
