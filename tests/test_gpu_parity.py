"""GPU parity: every hot-path entry point of libiris_hip.so (called through the
C ABI) is compared bit-exactly with the CPU oracle on the same seeded inputs,
on the committed golden vectors, and — at sizes the oracle cannot cover — via
size-independent properties (planted known answers, sampled oracle checks)."""
import numpy as np
import pytest

import iris_hip as ih
from oracle import oracle_c as oc

pytestmark = pytest.mark.gpu
ROT = 31
SEED = 42


def bits_eq(a, b):
    return (np.asarray(a, np.float64).view(np.uint64) == np.asarray(b, np.float64).view(np.uint64)).all()


LAYOUTS = [ih.LAYOUT_TILES, ih.LAYOUT_LANES]


@pytest.fixture(scope="module", params=LAYOUTS, ids=["tiles-mfma", "lanes-valu"])
def layout(request):
    return request.param


@pytest.fixture(scope="module")
def tdb(device, layout):
    """1000 generated templates (not a multiple of 32 or 64)."""
    db = ih.Database(device, ih.KIND_TEMPLATES, 1000, layout)
    db.generate(1000, SEED)
    assert db.layout == layout
    yield db
    db.close()


# ---------------------------------------------------------------- storage


def test_layouts_agree(device):
    """The TILES (fp4 MFMA) and LANES (VALU popcount) kernels give identical
    counts, distances and argmin on the same 3000 templates."""
    q = oc.gen_templates(77, 0, 1)[0]
    outs = []
    for lay in LAYOUTS:
        with ih.Database(device, ih.KIND_TEMPLATES, 3000, lay) as db, ih.TemplateEngine(device, q) as eng:
            db.generate(3000, 31)
            outs.append((eng.counts(db), eng.distances(db), eng.search(db)))
    (n0, d0), dist0, m0 = outs[0]
    (n1, d1), dist1, m1 = outs[1]
    assert (n0 == n1).all() and (d0 == d1).all() and bits_eq(dist0, dist1)
    assert (m0.index, m0.num, m0.den, m0.rotation) == (m1.index, m1.num, m1.den, m1.rotation)


def test_generate_matches_oracle(device, tdb, layout):
    got = tdb.read(0, 1000)
    assert (got == oc.gen_templates(SEED, 0, 1000)).all()
    with ih.Database(device, ih.KIND_MASKS, 200, layout) as m:
        m.generate(130, SEED, global_index0=500)
        assert (m.read(0, 130) == oc.gen_masks(SEED, 500, 130)).all()
    with ih.Database(device, ih.KIND_SHARES, 100, layout) as s:
        s.generate(70, SEED)
        assert (s.read(0, 70) == oc.gen_shares(SEED, 0, 70)).all()


def test_masks_shares_roundtrip(device, layout):
    rng = np.random.default_rng(4)
    masks = rng.integers(0, 2**64, (77, 200), dtype=np.uint64)
    shares = rng.integers(0, 2**16, (45, 12800), dtype=np.uint16)
    with ih.Database(device, ih.KIND_MASKS, 100, layout) as m:
        m.append(masks)
        assert (m.read(0, 77) == masks).all()
        m.write(33, masks[:2])
        assert (m.read(33, 2) == masks[:2]).all()
    with ih.Database(device, ih.KIND_SHARES, 64, layout) as s:
        s.append(shares)
        assert (s.read(0, 45) == shares).all()


def test_append_write_read_roundtrip(device, layout):
    rng = np.random.default_rng(1)
    recs = rng.integers(0, 2**64, (150, 400), dtype=np.uint64)
    with ih.Database(device, ih.KIND_TEMPLATES, 300, layout) as db:
        db.append(recs[:77])
        db.append(recs[77:])
        assert len(db) == 150
        assert (db.read(0, 150) == recs).all()
        db.write(10, recs[:5])
        expect = recs.copy()
        expect[10:15] = recs[:5]
        assert (db.read(0, 150) == expect).all()
        assert (db.read(63, 3) == expect[63:66]).all()
        with pytest.raises(ih.IrisError):
            db.read(100, 51)
        with pytest.raises(ih.IrisError):
            db.write(151, recs[:1])


@pytest.mark.parametrize("kind", [ih.KIND_MASKS, ih.KIND_SHARES, ih.KIND_TEMPLATES])
def test_db_capacity_overflow_rejected(device, kind):
    """A capacity whose byte size overflows 64 bits fails cleanly instead of allocating a
    wrapped-around size."""
    for cap in (2**64 - 1, 2**62):
        with pytest.raises(ih.IrisError):
            ih.Database(device, kind, cap)


# ---------------------------------------------------------------- Template path


def test_template_counts_match_oracle(device, tdb):
    ref = tdb.read(0, 1000)
    q = ref[3].copy()
    q[:200] ^= np.uint64(0x0F0F)  # not an exact DB member
    with ih.TemplateEngine(device, q) as eng:
        num, den = eng.counts(tdb)
        onum, oden = oc.template_counts(q, ref)
        assert (num == onum).all() and (den == oden).all()
        # ragged sub-range not aligned to the 64-record blocks
        num2, den2 = eng.counts(tdb, first=37, n=500)
        assert (num2 == onum[37:537]).all() and (den2 == oden[37:537]).all()


def test_template_distances_and_search(device, tdb):
    ref = tdb.read(0, 1000)
    q = oc.gen_templates(SEED + 1, 0, 1)[0]
    with ih.TemplateEngine(device, q) as eng:
        d = eng.distances(tdb)
        od = oc.template_distances(q, ref)
        assert bits_eq(d, od)
        m = eng.search(tdb)
        best, idx = oc.argmin(od)
        assert m.index == idx and bits_eq(m.distance, best)
        assert m.den > 0 and bits_eq(m.num / m.den, best)
        num, den = oc.template_counts(q, ref[idx:idx + 1])
        assert num[0, m.rotation + 15] == m.num and den[0, m.rotation + 15] == m.den
        # sub-range + index base
        m2 = eng.search(tdb, first=100, n=333, index_base=10_000)
        b2, i2 = oc.argmin(od[100:433])
        assert m2.index == 10_000 + 100 + i2 and bits_eq(m2.distance, b2)


def test_planted_rotated_copies(device, layout):
    """A rotated, lightly flipped copy of the query is the unique best match."""
    rng = np.random.default_rng(3)
    n = 5000
    with ih.Database(device, ih.KIND_TEMPLATES, n, layout) as db:
        db.generate(n, 9)
        q = oc.gen_templates(1234, 0, 1)[0]
        for pos, r in ((4321, 15), (17, -15), (2500, 0)):
            p = oc.bits_rotated(q[:200], r)  # entry = rot(q, r): engine rotation r matches
            mk = oc.bits_rotated(q[200:], r)
            flips = np.zeros(200, np.uint64)
            for b in map(int, rng.choice(12800, 25, replace=False)):
                flips[b // 64] |= np.uint64(1 << (b % 64))
            db.write(pos, np.concatenate([p ^ flips, mk])[None, :])
        ref = db.read(0, n)
        with ih.TemplateEngine(device, q) as eng:
            m = eng.search(db)
            best, idx = oc.argmin(oc.template_distances(q, ref))
            assert m.index == idx and bits_eq(m.distance, best)
            d = eng.distances(db)
            for pos, r in ((4321, 15), (17, -15), (2500, 0)):
                num, den = eng.counts(db, first=pos, n=1)
                k = int(np.argmin(num[0] / den[0]))
                assert k - 15 == r and d[pos] < 0.01


def test_template_edge_cases(device, golden, layout):
    q, db_ref = golden["query"], golden["db"]
    with ih.Database(device, ih.KIND_TEMPLATES, db_ref.shape[0], layout) as db:
        db.append(db_ref)
        with ih.TemplateEngine(device, q) as eng:
            num, den = eng.counts(db)
            assert (num == golden["num"]).all() and (den == golden["den"]).all()
            d = eng.distances(db)
            assert (d.view(np.uint64) == golden["dist_bits"]).all()
            m = eng.search(db)
            assert m.index == int(golden["argmin_index"])
            assert np.float64(m.distance).view(np.uint64) == golden["argmin_dist_bits"]
            # empty range
            e = eng.search(db, first=5, n=0)
            assert e.index == 2**64 - 1 and e.distance == np.inf
            assert eng.distances(db, first=0, n=0).shape == (0,)
            # empty-mask entry only -> +inf, no index (src/main.rs:581-582)
            empty_pos = int(np.where(np.isinf(d))[0][0])
            z = eng.search(db, first=empty_pos, n=1)
            assert z.index == 2**64 - 1 and z.distance == np.inf


def test_template_all_invalid_db(device, layout):
    with ih.Database(device, ih.KIND_TEMPLATES, 130, layout) as db:
        db.append(np.zeros((130, 400), np.uint64))
        with ih.TemplateEngine(device, oc.gen_templates(1, 0, 1)[0]) as eng:
            m = eng.search(db)
            assert m.index == 2**64 - 1 and m.distance == np.inf
            assert np.isinf(eng.distances(db)).all()


def test_template_distance_value_type(device, golden):
    a = ih.Template.from_array(golden["query"])
    b = ih.Template.from_array(golden["db"][0])
    assert np.float64(a.distance(b, device)).view(np.uint64) == golden["dist_bits"][0]
    assert a.distance(b, device) == oc.template_distance(golden["query"], golden["db"][0])


# ---------------------------------------------------------------- MasksEngine / DistanceEngine


def test_masks_engine(device, golden, layout):
    q, db_ref = golden["query"], golden["db"]
    with ih.MasksEngine(device, q[200:]) as eng:
        out = np.empty((db_ref.shape[0], ROT), np.uint16)
        eng.batch_process(out, db_ref[:, 200:])  # host slice, reference signature
        assert (out == golden["masks_out"]).all()
        with ih.Database(device, ih.KIND_MASKS, 2000, layout) as db:
            db.generate(1999, 5)
            ref = db.read(0, 1999)
            out = np.empty((1999, ROT), np.uint16)
            eng.batch_process(out, db)
            assert (out == oc.masks_batch(q[200:], ref)).all()
            out2 = np.empty((100, ROT), np.uint16)
            eng.batch_process(out2, db, first=1899, n=100)
            assert (out2 == oc.masks_batch(q[200:], ref[1899:])).all()
        with pytest.raises(ih.IrisError):  # assert_eq!(out.len(), db.len())
            eng.batch_process(np.empty((3, ROT), np.uint16), db_ref[:2, 200:])


def test_distance_engine(device, golden, layout):
    enc_q = golden["enc_query"]
    with ih.DistanceEngine(device, enc_q) as eng:
        for k in range(3):
            out = np.empty((golden["shares"].shape[1], ROT), np.uint16)
            eng.batch_process(out, golden["shares"][k])
            assert (out == golden["share_out"][k]).all()
        with ih.Database(device, ih.KIND_SHARES, 300, layout) as db:
            db.generate(257, 8)
            ref = db.read(0, 257)
            assert (ref == oc.gen_shares(8, 0, 257)).all()
            out = np.empty((257, ROT), np.uint16)
            eng.batch_process(out, db)
            assert (out == oc.distance_batch(enc_q, ref)).all()
            out2 = np.empty((100, ROT), np.uint16)
            eng.batch_process(out2, db, first=157, n=100)
            assert (out2 == oc.distance_batch(enc_q, ref[157:])).all()


def test_distance_engine_arbitrary_query(device, layout):
    """DistanceEngine::new accepts any EncodedBits, not only encode() output:
    uniform u16 query and shares, plus the all-0xFFFF wraparound case."""
    rng = np.random.default_rng(12)
    q = rng.integers(0, 2**16, 12800, dtype=np.uint16)
    shares = rng.integers(0, 2**16, (70, 12800), dtype=np.uint16)
    shares[5] = 0xFFFF
    with ih.DistanceEngine(device, q) as eng, ih.Database(device, ih.KIND_SHARES, 70, layout) as db:
        db.append(shares)
        out = np.empty((70, ROT), np.uint16)
        eng.batch_process(out, db)
        assert (out == oc.distance_batch(q, shares)).all()
        ptr = device.alloc(70 * ROT * 2)
        try:
            eng.batch_process_device(db, ptr)
            dev_out = np.empty((70, ROT), np.uint16)
            device.d2h(dev_out, ptr)
        finally:
            device.free(ptr)
        assert (dev_out == out).all()


def test_resolver_decode_matches_template_distance(device, golden):
    """src/lib.rs:165-193 on synthetic data: shares -> DistanceEngine, masks ->
    MasksEngine, wrapping sum + decode_distance == Template::distance."""
    q, db_ref = golden["query"], golden["db"]
    ns = golden["enc_db"].shape[0]
    parts = []
    with ih.DistanceEngine(device, ih.encode(ih.Template.from_array(q))) as eng:
        for k in range(3):
            out = np.empty((ns, ROT), np.uint16)
            eng.batch_process(out, golden["shares"][k])
            parts.append(out)
    den = ih.denominators(ih.Bits(q[200:]), ih.Bits(db_ref[0, 200:]), device)
    assert (den == golden["masks_out"][0]).all()
    total = (parts[0].astype(np.uint64) + parts[1] + parts[2]).astype(np.uint16)
    for i in range(ns):
        got = ih.decode_distance(total[i], golden["masks_out"][i])
        assert np.float64(got).view(np.uint64) == golden["dist_bits"][i]


def test_u16_wraparound(device, golden):
    assert ih.dot_u16(ih.EncodedBits(golden["wrap_a"]), ih.EncodedBits(golden["wrap_b"]), device) == int(golden["wrap_dot"])
    ones = np.full(12800, 0xFFFF, np.uint16)
    assert ih.dot_u16(ones, ones, device) == (12800 % 65536)


# ---------------------------------------------------------------- arch plugin (criterion shapes)


# the criterion shapes of src/arch/mod.rs:29 (dot_bool) and :53 (dot_u16), sampled checks
@pytest.mark.parametrize("na,nb", [(1, 1), (1, 1000), (31, 1000), (1, 100_000), (40, 70)])
def test_dot_bool_batch(device, na, nb):
    rng = np.random.default_rng(na * 7 + nb)
    a = rng.integers(0, 2**64, (na, 200), dtype=np.uint64)
    b = rng.integers(0, 2**64, (nb, 200), dtype=np.uint64)
    out = ih.dot_bool_batch(a, b, device)
    for j in list(range(0, nb, max(1, nb // 50))) + [nb - 1]:
        for i in range(na):
            assert out[j, i] == oc.dot_bool(a[i], b[j])


@pytest.mark.parametrize("na,nb", [(1, 1), (1, 1000), (31, 1000), (1, 100_000), (31, 100_000), (33, 5)])
def test_dot_u16_batch(device, na, nb):
    rng = np.random.default_rng(na * 11 + nb)
    a = rng.integers(0, 2**16, (na, 12800), dtype=np.uint16)
    b = rng.integers(0, 2**16, (nb, 12800), dtype=np.uint16)
    out = ih.dot_u16_batch(a, b, device)
    for j in list(range(0, nb, max(1, nb // 20))) + [nb - 1]:
        for i in range(0, na, max(1, na // 4)):
            assert out[j, i] == oc.dot_u16(a[i], b[j])


def test_config0_one_query_10k(device):
    """BASELINE configs[0] (1 query x 10k templates x 31 rotations, the reference's
    CPU-runnable case): Template distances, argmin, masks and share outputs against the
    oracle on every record."""
    n = 10_000
    t = oc.gen_templates(111, 0, n)
    q = oc.gen_templates(112, 0, 1)[0]
    with ih.Database(device, ih.KIND_TEMPLATES, n) as tdb, ih.TemplateEngine(device, q) as te, \
            ih.Database(device, ih.KIND_MASKS, n) as mdb, ih.MasksEngine(device, q[200:]) as me:
        tdb.append(t)
        mdb.append(t[:, 200:])
        want = oc.template_distances(q, t)
        assert bits_eq(te.distances(tdb), want)
        best, idx = oc.argmin(want)
        m = te.search(tdb)
        assert m.index == idx and bits_eq(m.distance, best)
        out = np.empty((n, ROT), np.uint16)
        me.batch_process(out, mdb)
        assert (out == oc.masks_batch(q[200:], t[:, 200:])).all()


# ---------------------------------------------------------------- large-size properties


def test_large_search_properties(device, layout):
    """2M templates (6.4 GB): planted known answer + sampled oracle checks of
    the per-template distances left on the device."""
    n = 2_000_000
    rng = np.random.default_rng(99)
    with ih.Database(device, ih.KIND_TEMPLATES, n, layout) as db:
        db.generate(n, 2024)
        q = oc.gen_templates(555, 0, 1)[0]
        plant = 1_765_432
        rec = np.concatenate([oc.bits_rotated(q[:200], 4), oc.bits_rotated(q[200:], 4)])
        rec[5] ^= np.uint64(0xFF)
        db.write(plant, rec[None, :])
        with ih.TemplateEngine(device, q) as eng:
            ptr = device.alloc(n * 8)
            try:
                m = eng.search(db, dist_out_device=ptr)
                dist = np.empty(n, np.float64)
                device.d2h(dist, ptr)
            finally:
                device.free(ptr)
            assert m.index == plant and m.rotation == 4
            assert bits_eq(m.distance, dist[plant])
            assert dist.min() == m.distance and int(np.argmin(dist)) == plant
            idx = np.sort(rng.choice(n, 3000, replace=False))
            sample = db.read(0, 1)  # warm
            for lo in range(0, 3000, 500):
                ii = idx[lo:lo + 500]
                recs = np.stack([db.read(int(i), 1)[0] for i in ii])
                assert bits_eq(dist[ii], oc.template_distances(q, recs))
            assert sample.shape == (1, 400)


def test_search_async_pipeline(device, layout):
    """iris_template_search_async: several searches in flight (engines destroyed right
    after enqueueing), waited out of order, with a blocking call in between; each
    result equals the blocking search and the oracle."""
    n = 20_000
    recs = oc.gen_templates(4242, 0, n)
    rng = np.random.default_rng(8)
    with ih.Database(device, ih.KIND_TEMPLATES, n, layout) as db:
        db.append(recs)
        qs = []
        for i in range(6):
            q = recs[int(rng.integers(0, n))].copy()
            q[int(rng.integers(0, 400))] ^= np.uint64(1 << int(rng.integers(0, 64)))
            qs.append(q)
        pend = []
        for i, q in enumerate(qs):
            with ih.TemplateEngine(device, q) as e:
                first, cnt = (0, n) if i % 3 else (123, n - 5000)
                pend.append((e.search_async(db, first, cnt, index_base=7), first, cnt))
        with ih.TemplateEngine(device, qs[0]) as e:  # a blocking call while searches are queued
            assert len(e.distances(db, 0, 10)) == 10
        with ih.TemplateEngine(device, qs[1]) as e:
            empty = e.search_async(db, 5, 0).wait()
        assert empty.distance == np.inf and empty.index == 2**64 - 1
        order = [5, 0, 3, 1, 4, 2]
        for i in order:
            p, first, cnt = pend[i]
            m = p.wait()
            want_d, want_i = oc.argmin(oc.template_distances(qs[i], recs[first:first + cnt]))
            assert bits_eq(m.distance, want_d) and m.index == want_i + first + 7
            with ih.TemplateEngine(device, qs[i]) as e:
                ms = e.search(db, first, cnt, index_base=7)
            assert (ms.distance, ms.index, ms.num, ms.den, ms.rotation) == (m.distance, m.index, m.num, m.den,
                                                                             m.rotation)
        with pytest.raises(ih.IrisError):
            pend[0][0].wait()


def test_max_capacity_search(device):
    """A template database filling the HBM (≈85M templates, 272 GB on an MI355X): 64-bit
    tile and record offsets past 2^32 bytes and ~170k search partials.  Planted known
    answers at both ends, an equal-distance copy (lowest index wins), a tail range with
    an unaligned offset, and sampled distances against the oracle."""
    free, _ = device.memory()
    n = min(85_000_000, (free - (8 << 30)) // 3200)
    assert n > 40_000_000, f"only {free / 1e9:.0f} GB free"
    rng = np.random.default_rng(5)
    with ih.Database(device, ih.KIND_TEMPLATES, n) as db:
        db.generate(n, 31337)
        q = oc.gen_templates(777, 0, 1)[0]
        rec = np.concatenate([oc.bits_rotated(q[:200], -7), oc.bits_rotated(q[200:], -7)])
        rec[3] ^= np.uint64(0xF0F0)
        last = n - 3
        db.write(last, rec[None, :])
        db.write(n - 40_000_001, rec[None, :])  # same distance, lower index: wins the full search
        with ih.TemplateEngine(device, q) as eng:
            m = eng.search(db)
            assert m.index == n - 40_000_001 and m.rotation == -7
            first = n - 1_000_003  # unaligned tail range: only the copy at `last` is inside
            mt = eng.search(db, first, n - first, index_base=0)
            assert mt.index == last and mt.rotation == -7 and bits_eq(mt.distance, m.distance)
            ii = np.sort(rng.choice(n, 400, replace=False))
            recs = np.stack([db.read(int(i), 1)[0] for i in ii])
            d = np.array([eng.distances(db, int(i), 1)[0] for i in ii])
            assert bits_eq(d, oc.template_distances(q, recs))
            want = oc.template_distances(q, rec[None, :])[0]
            assert bits_eq(m.distance, want)


def test_max_capacity_masks(device):
    """A masks database filling the HBM beside its full [n][31] output (~150M masks, 240 GB
    + 9 GB): the whole range into device memory, then sampled rows at both ends and across
    the 2^32-record-byte boundaries against the oracle, and a host-output sub-range at the
    end of the database."""
    free, _ = device.memory()
    n = min(150_000_000, (free - (12 << 30)) // (1600 + 62))
    assert n > 60_000_000, f"only {free / 1e9:.0f} GB free"
    seed = 4711
    q = oc.gen_templates(99, 0, 1)[0][200:]
    with ih.Database(device, ih.KIND_MASKS, n) as db, ih.MasksEngine(device, q) as eng:
        db.generate(n, seed)
        out = device.alloc(n * ROT * 2)
        try:
            eng.batch_process_device(db, out)
            for lo in (0, (1 << 32) // 1600 - 500, n // 2, n - 1000):
                rows = np.empty((1000, ROT), np.uint16)
                device.d2h(rows, out + lo * ROT * 2)
                want = oc.masks_batch(q, oc.gen_templates(seed, lo, 1000)[:, 200:])
                assert (rows == want).all(), lo
        finally:
            device.free(out)
        tail = np.empty((777, ROT), np.uint16)
        eng.batch_process(tail, db, first=n - 777, n=777)
        assert (tail == oc.masks_batch(q, oc.gen_templates(seed, n - 777, 777)[:, 200:])).all()


def test_host_output_chunks(device):
    """Host-output engine calls larger than one pinned-rows chunk (1M records): a resident range of
    2.3M masks (three kernels into two alternating pinned buffers), an uploaded host slice of 1.1M
    masks (two temporary-database chunks) and of 70k shares (two), each equal to the device-output
    form over the same records and to the oracle on sampled rows."""
    seed, n = 808, 2_300_000
    q = oc.gen_templates(98, 0, 1)[0]
    qblock = np.zeros((64, 200), np.uint8)
    qblock[:, 20:120] = 1
    qm = np.packbits(qblock.reshape(12800), bitorder="little").view(np.uint64)
    with ih.Database(device, ih.KIND_MASKS, n) as db, ih.MasksEngine(device, qm) as eng:
        db.generate(n, seed)
        # block (occlusion-like) masks around the pinned-rows chunk boundaries: against the block
        # query their rows span more than a byte, so the packed rows' escape path runs there
        rng = np.random.default_rng(12)
        for lo in (0, (1 << 20) - 300, 2 * (1 << 20) - 7):
            blk = np.zeros((600, 64, 200), np.uint8)
            for i in range(0, 600, 2):
                c0, w = int(rng.integers(0, 200)), int(rng.integers(10, 150))
                blk[i][:, (np.arange(w) + c0) % 200] = 1
            recs = db.read(lo, 600)
            recs[::2] = np.packbits(blk.reshape(600, 12800), axis=1, bitorder="little").view(np.uint64)[::2]
            db.write(lo, recs)
        dev_out = device.alloc(n * ROT * 2)
        try:
            eng.batch_process_device(db, dev_out)
            want = np.empty((n, ROT), np.uint16)
            device.d2h(want, dev_out)
        finally:
            device.free(dev_out)
        out = np.empty((n, ROT), np.uint16)
        eng.batch_process(out, db, first=0, n=n)
        assert (out == want).all()
        for lo in (0, (1 << 20) - 300, 2 * (1 << 20) - 5, n - 1000):
            assert (out[lo:lo + 1000] == oc.masks_batch(qm, db.read(lo, 1000))).all(), lo
        m = 1_100_000
        host = db.read(7, m)
        out2 = np.empty((m, ROT), np.uint16)
        eng.batch_process(out2, host)  # not attached: uploaded per call
        assert (out2 == want[7:7 + m]).all()
    ns = 70_000
    with ih.Database(device, ih.KIND_SHARES, ns) as sdb, ih.DistanceEngine(device, ih.encode(ih.Template.from_array(q))) as de:
        shares = np.random.default_rng(5).integers(0, 65536, (ns, 12800), dtype=np.uint16)
        sdb.append(shares)
        want = np.empty((ns, ROT), np.uint16)
        de.batch_process(want, sdb)
        out = np.empty((ns, ROT), np.uint16)
        de.batch_process(out, shares)  # not attached: uploaded per call
        assert (out == want).all()
        ii = np.array([0, 65535, 65536, ns - 1])
        assert (out[ii] == oc.distance_batch(oc.encode(q), shares[ii])).all()


# ---------------------------------------------------------------- resolver (src/main.rs:597-621)


def test_resolver_fused_matches_oracle(device, golden):
    share_out, masks_out = golden["share_out"], golden["masks_out"][: golden["share_out"].shape[1]]
    want = oc.resolver_combine(share_out, masks_out)
    best, idx = oc.argmin(want)
    m = ih.resolver_search(list(share_out), masks_out, device=device)
    assert m.index == idx and bits_eq(m.distance, best)
    # random garbage shares (den = 0 rows, uneq > den, ties): decode semantics
    rng = np.random.default_rng(21)
    n = 5000
    parts = [rng.integers(0, 2**16, (n, ROT), dtype=np.uint16) for _ in range(3)]
    den = rng.integers(0, 40, (n, ROT), dtype=np.uint16)
    den[rng.random((n, ROT)) < 0.3] = 0
    den[17] = 0
    want = oc.resolver_combine(np.stack(parts), den)
    best, idx = oc.argmin(want)
    m = ih.resolver_search(parts, den, index_base=100, device=device)
    assert m.index == 100 + idx and bits_eq(m.distance, best)
    z = ih.resolver_search([np.zeros((3, ROT), np.uint16)], np.zeros((3, ROT), np.uint16), device=device)
    assert z.index == 2**64 - 1 and z.distance == np.inf


@pytest.mark.parametrize("path", ["pinned", "runtime", "tuned"])
def test_resolver_host_chunks(device, hooked_device, path):
    """The host-array form across several chunks (pinned slots: 3 parts + denominators, 270 592
    records per 64-MB slot; the runtime's copy: 1M-record chunks), each path pinned by IRIS_UPLOAD
    and the default that picks by measured rate: 700 001 records, the best distance planted in
    the last chunk, then (equal) also in the first, so the chunks' winners merge to the lower
    index; and a 2-part call on garbage shares (ties at distance 0)."""
    dev = device if path == "tuned" else hooked_device(IRIS_UPLOAD=path)
    rng = np.random.default_rng(77)
    n = 700_001
    den = rng.integers(1000, 12801, (n, ROT)).astype(np.int64)
    # shares of realistic dot products: uneq within [3/8, 1/2] of den (distances >= 0.375), the
    # encoded dot den - 2 uneq split into 3 uniform additive shares (src/encoded_bits.rs:23-38)
    uneq = den // 2 - ((den // 8) * rng.random((n, ROT))).astype(np.int64)
    total = (den - 2 * uneq) % 2**16
    parts = [rng.integers(0, 2**16, (n, ROT), dtype=np.uint16) for _ in range(2)]
    parts.append(((total - parts[0] - parts[1]) % 2**16).astype(np.uint16))
    den = den.astype(np.uint16)

    def plant(i, u):  # distance u / 6000 at rotation 4 of record i
        den[i, 4] = 6000
        parts[2][i, 4] = ((6000 - 2 * u) - int(parts[0][i, 4]) - int(parts[1][i, 4])) % 2**16
    plant(n - 3, 60)
    want = oc.resolver_combine(np.stack(parts), den)
    best, idx = oc.argmin(want)
    assert idx == n - 3
    m = ih.resolver_search(parts, den, index_base=7, device=dev)
    assert m.index == 7 + idx and bits_eq(m.distance, best)
    plant(12, 60)  # the same distance in the first chunk: the lower index wins
    want = oc.resolver_combine(np.stack(parts), den)
    best, idx = oc.argmin(want)
    assert idx == 12
    m = ih.resolver_search(parts, den, device=dev)
    assert m.index == 12 and bits_eq(m.distance, best)
    want2 = oc.resolver_combine(np.stack(parts[:2]), den)
    best2, idx2 = oc.argmin(want2)
    m2 = ih.resolver_search(parts[:2], den, device=dev)
    assert m2.index == idx2 and bits_eq(m2.distance, best2)


@pytest.mark.parametrize("offset", [0, 2, 6])
def test_resolver_device_alignment(device, offset):
    """Device form with arrays at 16-B aligned and misaligned addresses (the kernel's
    16-B word path and its element-wise fallback) and a ragged tail (n % 64 != 0)."""
    rng = np.random.default_rng(offset)
    n = 1000 + 37
    parts = [rng.integers(0, 2**16, (n, ROT), dtype=np.uint16) for _ in range(2)]
    den = rng.integers(0, 12801, (n, ROT), dtype=np.uint16)
    want = oc.resolver_combine(np.stack(parts), den)
    best, idx = oc.argmin(want)
    ptrs = []
    for a in parts + [den]:
        p = device.alloc(a.nbytes + 16)
        device.h2d(p + offset, a)
        ptrs.append(p)
    dist = device.alloc(n * 8)
    try:
        m = ih.resolver_search_device(device, [p + offset for p in ptrs[:2]], ptrs[2] + offset, n,
                                      dist_out_device=dist)
        got = np.empty(n, np.float64)
        device.d2h(got, dist)
    finally:
        for p in ptrs + [dist]:
            device.free(p)
    assert m.index == idx and bits_eq(m.distance, best)
    assert bits_eq(got, want)


def test_mpc_end_to_end(device, layout):
    """The reference's MPC flow on synthetic data: the resolver holds the masks,
    3 participants hold additive shares of encode(template); DistanceEngine on
    each share DB + MasksEngine + fused resolver == plaintext Template search."""
    n = 3000
    rng = np.random.default_rng(5)
    templates = oc.gen_templates(91, 0, n)
    q = templates[1234].copy()
    q[:200] ^= np.uint64(0x3)
    enc = np.stack([oc.encode(t) for t in templates])
    s0 = rng.integers(0, 2**16, enc.shape, dtype=np.uint16)
    s1 = rng.integers(0, 2**16, enc.shape, dtype=np.uint16)
    s2 = (enc - s0 - s1).astype(np.uint16)  # EncodedBits::share (src/encoded_bits.rs:23-38)
    enc_q = ih.encode(ih.Template.from_array(q))
    outs = []
    for share in (s0, s1, s2):
        with ih.Database(device, ih.KIND_SHARES, n, layout) as db, ih.DistanceEngine(device, enc_q) as eng:
            db.append(share)
            out = np.empty((n, ROT), np.uint16)
            eng.batch_process(out, db)
            outs.append(out)
    with ih.Database(device, ih.KIND_MASKS, n, layout) as mdb, ih.MasksEngine(device, q[200:]) as me:
        mdb.append(templates[:, 200:])
        den = np.empty((n, ROT), np.uint16)
        me.batch_process(den, mdb)
    m = ih.resolver_search(outs, den, device=device)
    with ih.Database(device, ih.KIND_TEMPLATES, n, layout) as tdb, ih.TemplateEngine(device, q) as te:
        tdb.append(templates)
        ref = te.search(tdb)
    best, idx = oc.argmin(oc.template_distances(q, templates))
    assert m.index == ref.index == idx == 1234
    assert bits_eq(m.distance, best) and bits_eq(ref.distance, best)


# ---------------------------------------------------------------- batched queries (configs[2])


@pytest.mark.parametrize("nq", [1, 2, 3, 9])
def test_batch_search_matches_single(device, nq):
    """nq queries (1-2: the single-query dispatch; 3, 9: padded query groups of the
    batched kernel) against 5000 templates (a partial N-group): every query's best
    equals the single-query search and the oracle."""
    n = 5000
    db_ref = oc.gen_templates(61, 0, n)
    queries = oc.gen_templates(62, 0, max(nq, 9))
    queries[3] = db_ref[4321]          # exact member -> distance 0
    queries[7, :200] = db_ref[17, :200] ^ np.uint64(0x5)
    queries[7, 200:] = db_ref[17, 200:]
    queries[5, 200:] = 0               # empty query mask -> no candidate
    queries[0] = queries[3] if nq < 3 else queries[0]
    queries[1] = queries[5] if nq < 3 else queries[1]
    queries = queries[:nq].copy()
    with ih.Database(device, ih.KIND_TEMPLATES, n) as db:
        db.append(db_ref)
        with ih.TemplateBatchEngine(device, queries) as be:
            got = be.search(db)
            sub = be.search(db, first=1000, n=3333, index_base=7)
        for q in range(nq):
            want_d, want_i = oc.argmin(oc.template_distances(queries[q], db_ref))
            assert got[q].index == want_i and bits_eq(got[q].distance, want_d), q
            with ih.TemplateEngine(device, queries[q]) as eng:
                one = eng.search(db)
            assert (one.index, one.num, one.den, one.rotation) == (got[q].index, got[q].num, got[q].den, got[q].rotation)
            sd, si = oc.argmin(oc.template_distances(queries[q], db_ref[1000:4333]))
            assert sub[q].index == (7 + 1000 + si if si != 2**64 - 1 else si) and bits_eq(sub[q].distance, sd), q
    if nq > 5:
        assert got[3].index == 4321 and got[3].distance == 0.0
        assert got[5].index == 2**64 - 1
    if nq < 3:
        assert got[0].index == 4321 and got[0].distance == 0.0
    if nq == 2:
        assert got[1].index == 2**64 - 1


# ---------------------------------------------------------------- fused masks + resolver


@pytest.mark.parametrize("tiles_per_wave", ["auto", "4"])
@pytest.mark.parametrize("first,n", [(0, 3000), (37, 1000), (64, 64), (5, 1)])
def test_resolver_masks_fused(device, hooked_device, layout, first, n, tiles_per_wave):
    """MasksEngine.resolve == MasksEngine.batch_process + resolver_search == oracle, on
    random participant outputs (ties, den = 0 rows) and a planted near-copy."""
    if tiles_per_wave != "auto":  # pin the large-range variant on these small ranges
        device = hooked_device(IRIS_TILES_PER_WAVE=tiles_per_wave)
    total = 3100
    masks = oc.gen_templates(61, 0, total)[:, 200:].copy()
    q = masks[first + n // 2].copy()
    rng = np.random.default_rng(first + n)
    parts = [rng.integers(0, 2**16, (n, ROT), dtype=np.uint16) for _ in range(3)]
    with ih.Database(device, ih.KIND_MASKS, total, layout) as db, ih.MasksEngine(device, q) as eng:
        db.append(masks)
        den = np.empty((n, ROT), np.uint16)
        eng.batch_process(den, db, first=first, n=n)
        assert (den == oc.masks_batch(q, masks[first:first + n])).all()
        # make the planted record's shares decode to a small distance
        parts[2][n // 2] = (den[n // 2] - 20 - parts[0][n // 2] - parts[1][n // 2]).astype(np.uint16)
        want = oc.resolver_combine(np.stack(parts), den)
        best, idx = oc.argmin(want)
        dist = device.alloc(n * 8)
        try:
            m = eng.resolve(db, parts, first=first, n=n, index_base=1000, dist_out_device=dist)
            got = np.empty(n, np.float64)
            device.d2h(got, dist)
        finally:
            device.free(dist)
    assert m.index == 1000 + idx and bits_eq(m.distance, best)
    assert bits_eq(got, want)
    ref = ih.resolver_search(parts, den, index_base=1000, device=device)
    assert ref.index == m.index and ref.rotation == m.rotation


@pytest.mark.parametrize("layout_", ["tiles", "lanes"])
def test_resolver_masks_host_chunks(device, layout_):
    """MasksEngine.resolve with the participants' outputs as host arrays
    (iris_resolver_search_masks_host: the parts summed on the host, the sum uploaded, the masks
    denominators computed on the fly) over 1 100 037 records from record 5 -- two upload chunks of
    1 082 368 records, the planted winner in the second -- and over a short range, against the oracle
    and the device-pointer form."""
    lay = {"tiles": ih.LAYOUT_TILES, "lanes": ih.LAYOUT_LANES}[layout_]
    n, first = 1_100_037, 5
    total = first + n + 3
    masks = np.empty((total, 200), np.uint64)
    for a in range(0, total, 200_000):  # the generator's templates, masks half
        masks[a:a + 200_000] = oc.gen_templates(83, a, min(200_000, total - a))[:, 200:]
    q = masks[first + 1_090_000].copy()
    rng = np.random.default_rng(3)
    with ih.Database(device, ih.KIND_MASKS, total, lay) as db, ih.MasksEngine(device, q) as eng:
        db.append(masks)
        den = oc.masks_batch(q, masks[first:first + n])
        parts = [rng.integers(0, 2**16, (n, ROT), dtype=np.uint16) for _ in range(3)]
        # realistic shares: encoded dots den - 2 uneq, uneq in [3/8, 1/2] of den; one planted near-copy
        uneq = (den // 2 - ((den // 8) * rng.random((n, ROT))).astype(np.int64)).astype(np.int64)
        total_dot = (den.astype(np.int64) - 2 * uneq) % 2**16
        parts[2] = ((total_dot - parts[0] - parts[1]) % 2**16).astype(np.uint16)
        i = 1_090_000
        parts[2][i] = ((den[i].astype(np.int64) - 20 - parts[0][i] - parts[1][i]) % 2**16).astype(np.uint16)
        want = oc.resolver_combine(np.stack(parts), den)
        best, idx = oc.argmin(want)
        assert idx == i
        m = eng.resolve(db, parts, first=first, n=n, index_base=11)
        assert m.index == 11 + idx and bits_eq(m.distance, best)
        # a short range through both forms
        sl = slice(1000, 1000 + 4321)
        sp = [p[sl] for p in parts]
        want_s = oc.resolver_combine(np.stack(sp), den[sl])
        bs, js = oc.argmin(want_s)
        mh = eng.resolve(db, sp, first=first + 1000, n=4321)
        ptrs = []
        try:
            for p in sp:
                ptrs.append(device.alloc(p.nbytes))
                device.h2d(ptrs[-1], np.ascontiguousarray(p))
            md = eng.resolve(db, ptrs, first=first + 1000, n=4321)
        finally:
            for p in ptrs:
                device.free(p)
        assert mh.index == md.index == js and bits_eq(mh.distance, bs) and bits_eq(md.distance, bs)


def test_empty_ranges(device, layout):
    """Every entry point accepts an empty range (the reference's loops over empty slices)."""
    masks = oc.gen_templates(71, 0, 40)
    with ih.Database(device, ih.KIND_MASKS, 40, layout) as mdb, ih.MasksEngine(device, masks[0, 200:]) as me, \
            ih.Database(device, ih.KIND_SHARES, 8, layout) as sdb, \
            ih.DistanceEngine(device, np.zeros(12800, np.uint16)) as de, \
            ih.Database(device, ih.KIND_TEMPLATES, 40, layout) as tdb:
        out = np.empty((0, ROT), np.uint16)
        me.batch_process(out, mdb)                      # empty database
        de.batch_process(out, sdb)
        mdb.append(masks[:, 200:])
        tdb.append(masks)
        me.batch_process(out, mdb, first=40, n=0)       # empty range at the end
        m = me.resolve(mdb, [np.empty((0, ROT), np.uint16)], first=3, n=0)
        assert m.index == 2**64 - 1 and m.distance == np.inf
        r = ih.resolver_search([np.empty((0, ROT), np.uint16)], np.empty((0, ROT), np.uint16), device=device)
        assert r.index == 2**64 - 1
        sh = ih.Database(device, ih.KIND_SHARES, 8, layout)
        ih.prepare_shares(tdb, [sh], first=40, n=0)
        assert len(sh) == 0
        sh.close()
        if layout == ih.LAYOUT_TILES:  # the batched engine runs on TILES databases
            with ih.TemplateBatchEngine(device, masks[:3]) as be:
                ms = be.search(tdb, first=0, n=0)
                assert all(x.index == 2**64 - 1 for x in ms)


def test_concurrent_callers(device):
    """Engines are Sync in the reference (shared across rayon workers, called from
    spawn_blocking threads, src/main.rs:425,510,597): concurrent calls on one device
    from several host threads give the sequential results."""
    import threading

    n = 2000
    t = oc.gen_templates(81, 0, n)
    queries = [t[i].copy() for i in (3, 700, 1500, 1999)]
    with ih.Database(device, ih.KIND_TEMPLATES, n) as tdb, ih.Database(device, ih.KIND_MASKS, n) as mdb:
        tdb.append(t)
        mdb.append(t[:, 200:])
        want = []
        for q in queries:
            with ih.TemplateEngine(device, q) as te, ih.MasksEngine(device, q[200:]) as me:
                out = np.empty((n, ROT), np.uint16)
                me.batch_process(out, mdb)
                want.append((te.search(tdb), out))
        got = [None] * len(queries)
        errors = []

        def work(i):
            try:
                for _ in range(5):
                    with ih.TemplateEngine(device, queries[i]) as te, ih.MasksEngine(device, queries[i][200:]) as me:
                        out = np.empty((n, ROT), np.uint16)
                        me.batch_process(out, mdb)
                        got[i] = (te.search(tdb), out)
            except Exception as ex:  # reported below
                errors.append(ex)

        threads = [threading.Thread(target=work, args=(i,)) for i in range(len(queries))]
        for th in threads:
            th.start()
        for th in threads:
            th.join()
    assert not errors
    for (wm, wo), (gm, go) in zip(want, got):
        assert gm.index == wm.index and bits_eq(gm.distance, wm.distance)
        assert (go == wo).all()


def test_calls_keep_the_callers_current_device(device):
    """Every entry point that switches to its handle's device puts the calling thread back on
    its own current device (include/iris_hip.h); with one GPU only the path is exercised (the
    before / after devices are equal by construction), from a fresh thread and from this one."""
    import ctypes
    import threading

    # by soname: the HIP runtime instance libiris_hip.so is bound to (torch's copy, if torch came first)
    hip = ctypes.CDLL("libamdhip64.so.7")
    cur = ctypes.c_int(-1)

    def current():
        assert hip.hipGetDevice(ctypes.byref(cur)) == 0
        return cur.value

    t = oc.gen_templates(5, 0, 700)

    def calls():
        before = current()
        db = ih.Database(device, ih.KIND_TEMPLATES, len(t))
        db.append(t)
        with ih.TemplateEngine(device, t[3]) as te:
            m = te.search(db)
        db.close()
        assert m.index == 3 and m.distance == 0.0
        assert current() == before

    calls()
    errors = []

    def in_thread():
        try:
            calls()
        except Exception as ex:  # reported below
            errors.append(ex)

    th = threading.Thread(target=in_thread)
    th.start()
    th.join()
    assert not errors


def test_persistent_search_ranges_vs_oracle(device):
    """Ranges of more than 8192 tiles run the persistent search kernel (template_search_dyn_kernel:
    one grid of resident workgroups, each wave walking 4-tile units until the range runs out).
    Against the oracle on every template: the full database, a range ragged at both ends (neither
    end on a tile), and a mid-database range whose unit count leaves the last round of waves
    partly idle; distances bit for bit, and the winner with a planted tie far apart in the range
    (equal fractions: the lower index must win, whichever wave holds which)."""
    n = 300_007
    seed = 20260417
    recs = oc.gen_templates(seed, 0, n)
    q = oc.gen_templates(seed + 1, 0, 1)[0]
    near = oc.bits_rotated(q[:200], 7)
    twin = np.concatenate([near ^ np.uint64(0x0101), oc.bits_rotated(q[200:], 7)])
    for pos in (12_345, 287_001, 150_000):
        recs[pos] = twin
    with ih.Database(device, ih.KIND_TEMPLATES, n) as db:
        db.append(recs)
        want = oc.template_distances(q, recs)
        with ih.TemplateEngine(device, q) as eng:
            for first, m in ((0, n), (13, n - 13 - 5), (1_000, 270_001)):
                d = eng.distances(db, first=first, n=m)
                assert bits_eq(d, want[first:first + m]), (first, m)
                got = eng.search(db, first=first, n=m, index_base=7)
                best, idx = oc.argmin(want[first:first + m])
                assert got.index == 7 + first + idx and bits_eq(got.distance, best), (first, m, got)
            assert eng.search(db).index == 12_345
            assert eng.search(db, first=13_000, n=n - 13_000).index == 150_000


@pytest.mark.parametrize("path", ["pinned", "runtime"])
def test_large_write_paths(hooked_device, path):
    """Database writes of at least 8 MB go through two pinned slots filled by the helper threads or the
    runtime's copy of the pageable source (by measured rate; IRIS_UPLOAD pins one): both store the
    same records, including an unaligned start index and a last slot shorter than the others."""
    dev = hooked_device(IRIS_UPLOAD=path)
    assert dev.config()["upload"] == path
    rng = np.random.default_rng(11)
    n = 130_000  # 208 MB of masks: four 64-MB slots, the last one partial
    masks = rng.integers(0, 2**64, (n, 200), dtype=np.uint64)
    with ih.Database(dev, ih.KIND_MASKS, n + 100) as db:
        db.append(masks[:3])
        db.append(masks[3:])
        for lo in (0, 40_000, n - 50):
            assert (db.read(lo, 50) == masks[lo:lo + 50]).all(), lo
        shares = rng.integers(0, 2**16, (5_300, 12800), dtype=np.uint16)  # 136 MB, three slots
        with ih.Database(dev, ih.KIND_SHARES, 5_300) as sdb:
            sdb.append(shares)
            for lo in (0, 2_559, 2_560, 5_250):
                assert (sdb.read(lo, 50) == shares[lo:lo + 50]).all(), lo


def test_upload_path_tuning(hooked_device):
    """Without a pinned path, writes of 8 MB and more take each path twice (the first use of each,
    which pays its one-time setup, is not counted), then the faster one, re-measuring the other every
    16th write; iris_config reports the rates.  Every write stores the same records whichever path it
    took."""
    dev = hooked_device()
    rng = np.random.default_rng(12)
    masks = rng.integers(0, 2**64, (10_000, 200), dtype=np.uint64)  # 16 MB per write
    with ih.Database(dev, ih.KIND_MASKS, 10_000) as db:
        for i in range(20):
            db.truncate(0)
            db.append(masks if i % 2 == 0 else masks[::-1].copy())
            want = masks if i % 2 == 0 else masks[::-1]
            for lo in (0, 4_321, 9_950):
                assert (db.read(lo, 50) == want[lo:lo + 50]).all(), (i, lo)
    pinned, runtime = (float(x) for x in dev.config()["upload_gbps"].split("/"))
    assert pinned > 0 and runtime > 0
