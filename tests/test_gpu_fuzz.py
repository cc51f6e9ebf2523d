"""Randomised ranges against the oracle: 24 draws of (records, first, n, layout) per
entry point exercise every tile / block boundary case of the kernels' epilogues
(ragged first and last tiles, offsets that are not multiples of 8 — the element-wise
store path — and one-record ranges).  Fixed seed, so failures reproduce."""
import numpy as np
import pytest

import iris_hip as ih
from oracle import oracle_c as oc

pytestmark = pytest.mark.gpu
ROT = 31
DRAWS = 24


def _draws(seed, max_records):
    rng = np.random.default_rng(seed)
    for _ in range(DRAWS):
        total = int(rng.integers(1, max_records))
        first = int(rng.integers(0, total))
        n = int(rng.integers(0, total - first + 1))
        layout = [ih.LAYOUT_TILES, ih.LAYOUT_LANES][int(rng.integers(0, 2))]
        yield total, first, n, layout


def bits_eq(a, b):
    return (np.asarray(a, np.float64).view(np.uint64) == np.asarray(b, np.float64).view(np.uint64)).all()


@pytest.mark.parametrize("tiles_per_wave", ["auto", "1", "4"])
def test_fuzz_templates(device, hooked_device, tiles_per_wave):
    # small ranges run one tile per wave by default; "4" pins the large-range variant
    if tiles_per_wave != "auto":
        device = hooked_device(IRIS_TILES_PER_WAVE=tiles_per_wave)
    recs = oc.gen_templates(101, 0, 700)
    for i, (total, first, n, layout) in enumerate(_draws(1, 700)):
        q = recs[(i * 37) % total].copy()
        q[:200] ^= np.uint64(1 << (i % 64))
        with ih.Database(device, ih.KIND_TEMPLATES, total, layout) as db, ih.TemplateEngine(device, q) as eng:
            db.append(recs[:total])
            num, den = eng.counts(db, first, n)
            wn, wd = oc.template_counts(q, recs[first:first + n])
            assert (num == wn).all() and (den == wd).all(), (total, first, n, layout)
            d = eng.distances(db, first, n)
            wdist = oc.template_distances(q, recs[first:first + n])
            assert bits_eq(d, wdist), (total, first, n, layout)
            m = eng.search(db, first, n, index_base=5)
            best, idx = oc.argmin(wdist) if n else (np.inf, 2**64 - 1)
            assert bits_eq(m.distance, best)
            assert m.index == (idx + 5 + first if idx != 2**64 - 1 else idx), (total, first, n, layout)


@pytest.mark.parametrize("tiles_per_wave", ["auto", "1", "4"])
def test_fuzz_masks_and_shares(device, hooked_device, tiles_per_wave):
    # small ranges run one tile per wave (shares: split over K-slices) by default; "1" pins
    # one tile per wave without the K-split, "4" the large-range variants
    if tiles_per_wave != "auto":
        device = hooked_device(IRIS_TILES_PER_WAVE=tiles_per_wave)
    masks = oc.gen_templates(102, 0, 600)[:, 200:].copy()
    shares = np.random.default_rng(103).integers(0, 2**16, (300, 12800), dtype=np.uint16)
    for i, (total, first, n, layout) in enumerate(_draws(2, 300)):
        qm = masks[(i * 11) % total]
        qs = shares[(i * 7) % total]
        with ih.Database(device, ih.KIND_MASKS, total, layout) as mdb, ih.MasksEngine(device, qm) as me, \
                ih.Database(device, ih.KIND_SHARES, total, layout) as sdb, ih.DistanceEngine(device, qs) as de:
            mdb.append(masks[:total])
            sdb.append(shares[:total])
            out = np.empty((n, ROT), np.uint16)
            me.batch_process(out, mdb, first=first, n=n)
            assert (out == oc.masks_batch(qm, masks[first:first + n])).all(), (total, first, n, layout)
            out2 = np.empty((n, ROT), np.uint16)
            de.batch_process(out2, sdb, first=first, n=n)
            assert (out2 == oc.distance_batch(qs, shares[first:first + n])).all(), (total, first, n, layout)
            parts = [np.random.default_rng(i + p).integers(0, 2**16, (n, ROT), dtype=np.uint16) for p in range(2)]
            m = me.resolve(mdb, parts, first=first, n=n)
            if n:
                best, idx = oc.argmin(oc.resolver_combine(np.stack(parts), out))
                assert m.index == idx and bits_eq(m.distance, best), (total, first, n, layout)
            else:
                assert m.index == 2**64 - 1


def test_fused_reduce_equals_reduce_kernel(device, hooked_device):
    """Small searches finish in the kernel (its last workgroup folds the partials, published
    with system-scope atomics across the XCDs): 300 random queries over ranges up to the
    fused limit (4096 workgroups) must equal the separate reduce kernel (a device opened with
    IRIS_FUSED_REDUCE=0, holding the same records) and the oracle."""
    import iris_hip as ih
    from oracle import oracle_c as oc

    n = 140_000
    rng = np.random.default_rng(12)
    ref = oc.gen_templates(5, 0, n)
    unfused = hooked_device(IRIS_FUSED_REDUCE="0")
    with ih.Database(device, ih.KIND_TEMPLATES, n) as db, ih.Database(unfused, ih.KIND_TEMPLATES, n) as udb:
        db.generate(n, 5)
        udb.generate(n, 5)
        for it in range(300):
            q = oc.gen_templates(1000 + it, 0, 1)[0]
            first = int(rng.integers(0, n - 1))
            cnt = int(rng.integers(1, min(n - first, 130_000) + 1))
            if it % 4 == 0:  # a planted answer somewhere in the range
                site = first + int(rng.integers(0, cnt))
                p = ih.Bits(q[:200]).rotated(int(rng.integers(-15, 16))).limbs
                m = ih.Bits(q[200:]).rotated(0).limbs
                db.write(site, np.concatenate([p, m])[None, :])
                udb.write(site, np.concatenate([p, m])[None, :])
                ref[site] = np.concatenate([p, m])
            with ih.TemplateEngine(device, q) as eng, ih.TemplateEngine(unfused, q) as ueng:
                a = eng.search(db, first, cnt, index_base=7)
                b = ueng.search(udb, first, cnt, index_base=7)
            assert (a.index, a.num, a.den, a.rotation) == (b.index, b.num, b.den, b.rotation), (it, a, b)
            if it % 25 == 0:
                best, idx = oc.argmin(oc.template_distances(q, ref[first:first + cnt]))
                assert a.index == idx + first + 7 and a.distance == best


@pytest.mark.parametrize("tiles_per_wave", ["auto", "1", "4"])
def test_fuzz_readahead_walks(device, hooked_device, tiles_per_wave):
    """The read-ahead (growing windows on two side streams; masks rows packed to 32 B with a
    full-row escape) under random walks over a resident database: 40 walks of random chunk sizes
    (1..4 000 records) from random starting records, some abandoned after a few calls, some
    broken by a random-access call, against the oracle's rows.  Masks are a mix of random and
    block (occlusion-like) records, so packed and escaped rows interleave within tiles; the query
    alternates between a random and a block mask."""
    if tiles_per_wave != "auto":
        device = hooked_device(IRIS_TILES_PER_WAVE=tiles_per_wave)
    rng = np.random.default_rng(77)
    n = 30_000
    masks = oc.gen_masks(78, 0, n)
    for i in range(0, n, 4):
        c0, w = int(rng.integers(0, 200)), int(rng.integers(10, 150))
        bits = np.zeros((64, 200), np.uint8)
        bits[:, (np.arange(w) + c0) % 200] = 1
        masks[i] = np.packbits(bits.reshape(12800), bitorder="little").view(np.uint64)
    qblock = np.zeros((64, 200), np.uint8)
    qblock[:, 30:130] = 1
    queries = [oc.gen_masks(79, 0, 1)[0], np.packbits(qblock.reshape(12800), bitorder="little").view(np.uint64)]
    wants = [oc.masks_batch(q, masks) for q in queries]
    shares = np.random.default_rng(80).integers(0, 2**16, (3_000, 12800), dtype=np.uint16)
    qs = shares[17].copy()
    want_s = oc.distance_batch(qs, shares)
    with ih.Database(device, ih.KIND_MASKS, n) as mdb, ih.Database(device, ih.KIND_SHARES, len(shares)) as sdb:
        mdb.append(masks)
        sdb.append(shares)
        for walk in range(40):
            kind = "shares" if walk % 5 == 4 else "masks"
            db, total = (sdb, len(shares)) if kind == "shares" else (mdb, n)
            want = want_s if kind == "shares" else wants[walk % 2]
            eng = ih.DistanceEngine(device, qs) if kind == "shares" else ih.MasksEngine(device, queries[walk % 2])
            with eng:
                chunk = int(rng.integers(1, 4_001 if kind == "masks" else 400))
                a = int(rng.integers(0, total))
                calls = int(rng.integers(1, 40))
                for c in range(calls):
                    if a >= total:
                        break
                    if c and rng.random() < 0.1:  # a random-access call inside the walk
                        r0 = int(rng.integers(0, total))
                        r1 = min(total, r0 + int(rng.integers(1, 3_000)))
                        out = np.empty((r1 - r0, ROT), np.uint16)
                        eng.batch_process(out, db, first=r0, n=r1 - r0)
                        assert (out == want[r0:r1]).all(), (walk, "random", r0, r1)
                    m = min(chunk, total - a)
                    out = np.empty((m, ROT), np.uint16)
                    eng.batch_process(out, db, first=a, n=m)
                    assert (out == want[a:a + m]).all(), (walk, kind, chunk, a, m)
                    a += m
