"""GPU parity at the BASELINE configurations' own sizes.

configs[2] (1024 batched queries x 31 rotations x 10M templates): the batched kernel at
its production shape — 256 query groups, many N-groups per workgroup through the LDS-DMA
ring — against the oracle on every query (4k and 200k templates, ragged tails, sub-ranges),
and at full size through planted known answers in several query groups plus the
single-query search (itself oracle-checked) for unplanted queries.

configs[3] (u16-share DistanceEngine x 10M, 256 GB): the whole database in HBM, sampled rows
at both ends and across the 2^32-byte offsets against the oracle.

Reference semantics: src/template.rs:43-64 (Template::distance), src/main.rs:616-621 (first
strict minimum), src/lib.rs:42-52 (DistanceEngine::batch_process)."""
import numpy as np
import pytest

import iris_hip as ih
from oracle import oracle_c as oc

pytestmark = pytest.mark.gpu
ROT = 31
NONE = 2**64 - 1


def bits_eq(a, b):
    return (np.asarray(a, np.float64).view(np.uint64) == np.asarray(b, np.float64).view(np.uint64)).all()


def expected_winner(q, recs, base=0):
    """Oracle (distance, index, num, den, rotation) of the search over recs: the lowest index
    among the minimal distances (src/main.rs:616-621), and within the winner the minimal
    fraction at the lowest rotation (the library's documented rule for iris_match_t)."""
    d = oc.template_distances(q, recs)
    best, idx = oc.argmin(d)
    if idx == NONE:
        return best, NONE, None, None, None
    num, den = oc.template_counts(q, recs[idx:idx + 1])
    k_best = None
    for k in range(ROT):
        if den[0, k] == 0:
            continue
        if k_best is None or int(num[0, k]) * int(den[0, k_best]) < int(num[0, k_best]) * int(den[0, k]):
            k_best = k
    return best, idx + base, int(num[0, k_best]), int(den[0, k_best]), k_best - 15


def planted(q, rotation, flip_limb=9):
    rec = np.concatenate([oc.bits_rotated(q[:200], rotation), oc.bits_rotated(q[200:], rotation)])
    rec[flip_limb] ^= np.uint64(0x0F0F00000F0F)
    return rec


def check_all(got, queries, recs, base=0):
    for qi, q in enumerate(queries):
        d, idx, num, den, rot = expected_winner(q, recs, base)
        g = got[qi]
        assert bits_eq(g.distance, d) and g.index == idx, (qi, g, d, idx)
        if idx != NONE:
            assert (g.num, g.den, g.rotation) == (num, den, rot), (qi, g)


@pytest.mark.parametrize("kernel", ["4", "2"], ids=["batch_lds_q2", "batch_lds_q4"])
def test_batch_1024_queries_vs_oracle(device, hooked_device, kernel):
    """Q = 1024 (256 query groups) over 4099 templates and a ragged sub-range: every query's
    distance bits, index, winning fraction and rotation equal the oracle's (both batched
    kernel shapes: the IRIS_BATCH_KERNEL test hook; 4 is the default, 2 the cross-check)."""
    if kernel != "4":
        device = hooked_device(IRIS_BATCH_KERNEL=kernel)
    n, nq = 4099, 1024
    recs = oc.gen_templates(811, 0, n)
    queries = oc.gen_templates(812, 0, nq)
    # exact members, rotated near-copies at the rotation extremes, empty query masks and an
    # equal-distance pair (the lower index must win), spread over many query groups
    for qi, (src, rot) in {3: (100, 0), 255: (4000, 15), 511: (2048, -15), 1020: (7, 4), 1023: (4098, -1)}.items():
        recs[src] = planted(queries[qi], rot)
    recs[3000] = recs[100]
    queries[600, 200:] = 0
    queries[1001, 200:] = 0
    with ih.Database(device, ih.KIND_TEMPLATES, n) as db:
        db.append(recs)
        with ih.TemplateBatchEngine(device, queries) as be:
            got = be.search(db)
            sub = be.search(db, first=517, n=3001, index_base=11)
    check_all(got, queries, recs)
    check_all(sub, queries, recs[517:3518], base=11 + 517)
    assert got[3].index == 100 and got[255].index == 4000 and got[255].rotation == 15
    assert got[511].index == 2048 and got[511].rotation == -15
    assert got[600].index == NONE and got[600].distance == np.inf


@pytest.mark.parametrize("kernel", ["4", "2"], ids=["batch_lds_q2", "batch_lds_q4"])
@pytest.mark.parametrize("nq", [64, 1024])
def test_batch_many_groups_200k(device, hooked_device, nq, kernel):
    """Q = 64 and 1024 over 200 003 templates (6252 tiles: many N-groups per workgroup and a
    ragged last tile): every query against the oracle (Q = 64) or, for Q = 1024, every query
    against the single-query search and 48 of them against the oracle."""
    if kernel != "4":
        device = hooked_device(IRIS_BATCH_KERNEL=kernel)
    n = 200_003
    recs = oc.gen_templates(913, 0, n)
    queries = oc.gen_templates(914, 0, nq)
    sites = {0: (199_999, 9), nq // 2: (1_234, -15), nq - 1: (200_002, 15), nq // 4 + 1: (77_777, 0)}
    for qi, (site, rot) in sites.items():
        recs[site] = planted(queries[qi], rot)
    with ih.Database(device, ih.KIND_TEMPLATES, n) as db:
        db.append(recs)
        with ih.TemplateBatchEngine(device, queries) as be:
            got = be.search(db)
            tail = be.search(db, first=150_001, n=n - 150_001, index_base=0)
        for qi, (site, rot) in sites.items():
            assert got[qi].index == site and got[qi].rotation == rot, qi
        if nq <= 64:
            check_all(got, queries, recs)
        else:
            pick = np.random.default_rng(3).choice(nq, 48, replace=False)
            check_all([got[i] for i in pick], queries[pick], recs)
            for qi in range(nq):
                with ih.TemplateEngine(device, queries[qi]) as eng:
                    one = eng.search(db)
                    ot = eng.search(db, first=150_001, n=n - 150_001)
                g = got[qi]
                assert (one.index, one.num, one.den, one.rotation) == (g.index, g.num, g.den, g.rotation), qi
                assert bits_eq(one.distance, g.distance)
                t = tail[qi]
                assert (ot.index, ot.num, ot.den, ot.rotation) == (t.index, t.num, t.den, t.rotation), qi


def test_batch_sizes_vs_oracle(device):
    """Batch sizes around the GEMM's query-group padding (4 .. 97 queries: full, ragged and single-query
    last groups): every query of every batch against the oracle, full range and a ragged sub-range,
    with planted winners at the rotation extremes.  (These sizes also pinned the row-packed variant
    measured in round 4, profiles/r04_batch_rows_power.txt.)"""
    n = 4099
    recs = oc.gen_templates(821, 0, n)
    with ih.Database(device, ih.KIND_TEMPLATES, n) as db:
        for nq in (4, 5, 17, 32, 33, 63, 64, 65, 97):
            queries = oc.gen_templates(822 + nq, 0, nq)
            sites = {1: (4098 - nq, 15), nq - 1: (nq, -15), nq // 2: (2 * nq + 1, 0)}
            recs_q = recs.copy()
            for qi, (site, rot) in sites.items():
                recs_q[site] = planted(queries[qi], rot)
            db.clear()
            db.append(recs_q)
            with ih.TemplateBatchEngine(device, queries) as be:
                got = be.search(db)
                sub = be.search(db, first=3, n=4001, index_base=5)
            check_all(got, queries, recs_q)
            check_all(sub, queries, recs_q[3:4004], base=5 + 3)
            for qi, (site, rot) in sites.items():
                assert got[qi].index == site and got[qi].rotation == rot, (nq, qi, got[qi])


def test_batch_1024_full_size(device):
    """configs[2] at full size: 1024 queries x 10M resident templates in one pass.  Planted
    answers for 8 queries in 8 query groups (rotations 0, +-15, ...) must be found with the
    oracle's distance bits; 24 unplanted queries must equal the single-query search, whose
    winner's distance is re-checked against the oracle on the record read back."""
    n, nq = 10_000_000, 1024
    seed = 20251016
    queries = oc.gen_templates(915, 0, nq)
    plant_q = [0, 5, 130, 257, 512, 700, 901, 1023]
    rots = [0, 15, -15, 3, -8, 11, -1, 7]
    sites = [9_999_999, 0, 31, 4_999_968, 7_654_321, 2**32 // 3200 + 5, 123_457, 9_999_968]
    with ih.Database(device, ih.KIND_TEMPLATES, n) as db:
        db.generate(n, seed)
        for qi, rot, site in zip(plant_q, rots, sites):
            db.write(site, planted(queries[qi], rot)[None, :])
        with ih.TemplateBatchEngine(device, queries) as be:
            got = be.search(db)
        assert len({q // 4 for q in plant_q}) == 8
        for qi, rot, site in zip(plant_q, rots, sites):
            want = oc.template_distances(queries[qi], planted(queries[qi], rot)[None, :])[0]
            assert got[qi].index == site and got[qi].rotation == rot, (qi, got[qi])
            assert bits_eq(got[qi].distance, want)
        others = [q for q in np.random.default_rng(4).choice(nq, 30, replace=False) if q not in plant_q][:24]
        for qi in others:
            with ih.TemplateEngine(device, queries[qi]) as eng:
                one = eng.search(db)
            g = got[qi]
            assert (one.index, one.num, one.den, one.rotation) == (g.index, g.num, g.den, g.rotation), qi
            rec = db.read(int(g.index), 1)
            assert bits_eq(g.distance, oc.template_distances(queries[qi], rec)[0])


def test_shares_hbm_scale(device):
    """configs[3] at full size: 10M EncodedBits shares (256 GB) resident, the whole range
    through DistanceEngine into device memory, then rows sampled at both ends and across the
    2^32-, 2^33- and 2^37-byte record offsets against the oracle, plus a host-output range at
    the end and a uniform-u16 query (shares are not encode() output)."""
    free, _ = device.memory()
    n = min(10_000_000, (free - (10 << 30)) // (25600 + 62))
    assert n > 5_000_000, f"only {free / 1e9:.0f} GB free"
    seed = 6007
    q = oc.gen_shares(6008, 0, 1)[0]
    with ih.Database(device, ih.KIND_SHARES, n) as db, ih.DistanceEngine(device, q) as eng:
        db.generate(n, seed)
        out = device.alloc(n * ROT * 2)
        try:
            eng.batch_process_device(db, out)
            for lo in (0, (1 << 32) // 25600 - 40, (1 << 33) // 25600 - 40, (1 << 37) // 25600 - 40, n // 2,
                       n - 100):
                lo = min(lo, n - 100)
                rows = np.empty((100, ROT), np.uint16)
                device.d2h(rows, out + lo * ROT * 2)
                want = oc.distance_batch(q, oc.gen_shares(seed, lo, 100))
                assert (rows == want).all(), lo
        finally:
            device.free(out)
        tail = np.empty((333, ROT), np.uint16)
        eng.batch_process(tail, db, first=n - 333, n=333)
        assert (tail == oc.distance_batch(q, oc.gen_shares(seed, n - 333, 333))).all()
