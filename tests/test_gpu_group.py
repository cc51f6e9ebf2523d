"""GPU: device groups (iris_group_*, csrc/iris_group.hip) — a template database split
into contiguous shards, each searched on its device, the per-shard winners all-gathered
over RCCL (librccl from /opt/rocm) and merged with the resolver's rule: exact fraction,
then the lowest global index (src/main.rs:616-621).  On the one-GPU box a group has one
device (a 1-rank RCCL communicator); shards_per_device > 1 splits its range into several
logical shards that are searched and exchanged separately, so cross-shard ties and empty
shards are exercised.  Every answer must equal a single-device search of the same records
and the CPU oracle (Template::distance, src/template.rs:43-64)."""
import numpy as np
import pytest

import iris_hip as ih
from oracle import oracle_c as oc

pytestmark = pytest.mark.gpu
SEED = 77


def planted(query, r, flips=0):
    p = ih.Bits(query[:200]).rotated(r).limbs.copy()
    m = ih.Bits(query[200:]).rotated(r).limbs
    p[3] ^= np.uint64(flips)
    return np.concatenate([p, m])


def oracle_best(query, recs):
    d = oc.template_distances(query, recs)
    return oc.argmin(d)


def same(m, best, idx):
    return m.index == idx and np.float64(m.distance).view(np.uint64) == np.float64(best).view(np.uint64)


@pytest.fixture(scope="module")
def group():
    with ih.Group([0]) as g:
        assert (g.local_devices, g.ranks, g.first_rank) == (1, 1, 0)
        yield g


@pytest.fixture
def hooked_group(monkeypatch):
    """hooked_group(IRIS_X="v", ...): a one-device group whose device read the test hooks
    when it opened (IRIS_TEST_HOOKS=1 just for the open, like conftest.hooked_device)."""
    groups = []

    def open_(**env):
        with monkeypatch.context() as m:
            m.setenv("IRIS_TEST_HOOKS", "1")
            for k, v in env.items():
                m.setenv(k, str(v))
            g = ih.Group([0])
        groups.append(g)
        assert g.devices[0].config()["test_hooks"] == "1"
        return g

    yield open_
    for g in groups:
        g.close()


# IRIS_GROUP_DELAY_US: the side stream spins this long before every all-gather (a slow peer), so a
# later search's kernels run while an earlier search's winners still wait to be sent
DELAY_US = 3000


@pytest.mark.parametrize("spd", [1, 3, 8])
def test_group_search_equals_single_device_and_oracle(group, device, spd):
    n = 5003
    ref = oc.gen_templates(SEED, 0, n)
    query = oc.gen_templates(SEED + 1, 0, 1)[0]
    with ih.GroupDatabase(group, ih.KIND_TEMPLATES, n, shards_per_device=spd) as gdb:
        assert gdb.shards == spd and gdb.local_shards == spd and gdb.total == n
        bounds = [gdb.shard(i) for i in range(spd)]
        assert bounds[0][0] == 0 and sum(c for _, c in bounds) == n
        assert all(bounds[i][0] + bounds[i][1] == bounds[i + 1][0] for i in range(spd - 1))
        gdb.generate(SEED)
        assert (gdb.read(0, n) == ref).all()
        site = 4321
        rec = planted(query, -6, 0x0F0F)
        gdb.write(site, rec[None, :])
        ref[site] = rec
        m = gdb.search(query)
        best, idx = oracle_best(query, ref)
        assert same(m, best, idx) and idx == site and m.rotation == -6
        with ih.Database(device, ih.KIND_TEMPLATES, n) as db, ih.TemplateEngine(device, query) as eng:
            db.append(ref)
            s = eng.search(db)
        assert (s.index, s.num, s.den, s.rotation) == (m.index, m.num, m.den, m.rotation)


def test_group_cross_shard_tie_lowest_global_index(group):
    """Two exact copies of the query (distance 0) in different logical shards: the lower
    global index wins whichever shard reports first; a strictly better one in a later shard
    beats both."""
    n, spd = 4099, 4
    query = oc.gen_templates(SEED + 2, 0, 1)[0]
    with ih.GroupDatabase(group, ih.KIND_TEMPLATES, n, shards_per_device=spd) as gdb:
        gdb.generate(SEED)
        lo, hi = gdb.shard(1)[0] + 5, gdb.shard(3)[0] + 7
        exact = planted(query, 0)
        gdb.write(hi, exact[None, :])
        gdb.write(lo, exact[None, :])
        m = gdb.search(query)
        assert m.index == lo and m.distance == 0.0 and m.rotation == 0
        # the tie at the shard boundary: last record of shard 2 and first of shard 3
        f3 = gdb.shard(3)[0]
        gdb.write(f3 - 1, exact[None, :])
        gdb.write(f3, exact[None, :])
        assert gdb.search(query).index == lo
        # a copy whose valid bits are all equal but fewer: still distance 0, lowest index rules
        ref = gdb.read(0, n)
        best, idx = oracle_best(query, ref)
        assert same(gdb.search(query), best, idx)


def test_group_empty_shards_and_tiny_db(group):
    query = oc.gen_templates(SEED + 3, 0, 1)[0]
    with ih.GroupDatabase(group, ih.KIND_TEMPLATES, 3, shards_per_device=8) as gdb:
        assert sum(gdb.shard(i)[1] for i in range(8)) == 3
        m = gdb.search(query)  # nothing written: every record is empty
        assert m.index == 2**64 - 1 and m.distance == float("inf")
        gdb.generate(SEED)
        ref = gdb.read(0, 3)
        best, idx = oracle_best(query, ref)
        assert same(gdb.search(query), best, idx)
    with ih.GroupDatabase(group, ih.KIND_TEMPLATES, 0) as gdb:
        assert gdb.search(query).index == 2**64 - 1


def async_out_of_order(g, nq=9):
    """nq pipelined searches over 2 small shards (the fused kernel writes each shard's winner
    into the exchange buffer itself), waited out of order: -> (got, want index)."""
    n, spd = 40000, 2
    qs = oc.gen_templates(SEED + 10, 0, nq)
    with ih.GroupDatabase(g, ih.KIND_TEMPLATES, n, shards_per_device=spd) as gdb:
        gdb.generate(SEED)
        for k, q in enumerate(qs):
            gdb.write(1000 + 4100 * k, planted(q, (k % 5) - 2, 0x3)[None, :])
        ref = gdb.read(0, n)
        pend = [gdb.search_async(q) for q in qs]
        got = [None] * nq
        for k in list(range(3, nq)) + [0, 2, 1]:
            got[k] = pend[k].wait()
    want = [oracle_best(q, ref) for q in qs]
    return got, want


@pytest.mark.parametrize("side", ["plain", "delayed"])
def test_group_async_out_of_order(group, hooked_group, side):
    """Pipelined searches, waited out of order; "delayed": every all-gather is held back by the
    IRIS_GROUP_DELAY_US hook, so searches k + 4, k + 8 (the send-slot ring) run their kernels
    before search k's winners are sent -- each must still get its own answer."""
    g = group if side == "plain" else hooked_group(IRIS_GROUP_DELAY_US=DELAY_US)
    got, want = async_out_of_order(g)
    for k, (best, idx) in enumerate(want):
        assert same(got[k], best, idx) and idx == 1000 + 4100 * k, (k, got[k], idx)


def test_group_delay_hook_reaches_the_race_window(hooked_group):
    """The same run with the exchange-buffer ordering dropped (IRIS_GROUP_UNORDERED, test-only):
    later searches overwrite the winners of earlier ones before they are sent, so some answers
    are wrong -- the delayed test above exercises the write-after-read hazard it guards."""
    g = hooked_group(IRIS_GROUP_DELAY_US=DELAY_US, IRIS_GROUP_UNORDERED=1)
    got, want = async_out_of_order(g)
    wrong = [k for k, (best, idx) in enumerate(want) if not same(got[k], best, idx)]
    assert wrong, "the delayed all-gathers never met a reused send slot"


@pytest.mark.parametrize("layout", [ih.LAYOUT_LANES])
def test_group_other_layouts(group, layout):
    n = 3001
    ref = oc.gen_templates(SEED, 0, n)
    query = oc.gen_templates(SEED + 4, 0, 1)[0]
    with ih.GroupDatabase(group, ih.KIND_TEMPLATES, n, layout, shards_per_device=3) as gdb:
        gdb.generate(SEED)
        gdb.write(2999, planted(query, 15, 0x11)[None, :])
        ref[2999] = planted(query, 15, 0x11)
        best, idx = oracle_best(query, ref)
        m = gdb.search(query)
        assert same(m, best, idx) and idx == 2999 and m.rotation == 15


@pytest.mark.parametrize("nq", [2, 3, 9])
def test_group_batch_search(group, device, nq):
    n, spd = 6000, 3
    ref = oc.gen_templates(SEED, 0, n)
    qs = oc.gen_templates(SEED + 20, 0, nq)
    with ih.GroupDatabase(group, ih.KIND_TEMPLATES, n, shards_per_device=spd) as gdb:
        gdb.generate(SEED)
        sites = [gdb.shard(k % spd)[0] + 17 * k + 3 for k in range(nq)]
        for k, s in enumerate(sites):
            if k % 2 == 0:  # every other query gets a planted answer
                rec = planted(qs[k], (k % 31) - 15, 0x5)
                gdb.write(s, rec[None, :])
                ref[s] = rec
        got = gdb.batch_search(qs)
        for k, q in enumerate(qs):
            best, idx = oracle_best(q, ref)
            assert same(got[k], best, idx), (k, got[k], best, idx)


def test_group_write_read_across_shards_and_load_file(group, tmp_path):
    n, spd = 2500, 4
    rng = np.random.default_rng(5)
    recs = rng.integers(0, 2**64, (n, 400), dtype=np.uint64)
    path = tmp_path / "t.templates"
    recs.tofile(path)
    with ih.GroupDatabase(group, ih.KIND_TEMPLATES, n - 100, shards_per_device=spd) as gdb:
        gdb.load_file(path, first=100)
        assert (gdb.read(0, n - 100) == recs[100:]).all()
        a, b = gdb.shard(2)[0] - 3, gdb.shard(2)[0] + 4  # a range across a shard boundary
        gdb.write(a, recs[:b - a])
        assert (gdb.read(a, b - a) == recs[:b - a]).all()
        query = recs[7]
        best, idx = oracle_best(query, gdb.read(0, n - 100))
        assert same(gdb.search(query), best, idx)
    with ih.GroupDatabase(group, ih.KIND_TEMPLATES, n, shards_per_device=spd) as gdb:
        with pytest.raises(ih.IrisError):
            gdb.load_file(path, first=1)  # the file holds fewer than first + total records


def test_group_rejects_duplicate_device_and_bad_args():
    with pytest.raises(ih.IrisError):
        ih.Group([0, 0])
    with ih.Group([0]) as g:
        with pytest.raises(ih.IrisError):
            ih.GroupDatabase(g, ih.KIND_TEMPLATES, 10, shards_per_device=0)
        with ih.GroupDatabase(g, ih.KIND_MASKS, 10) as gdb:
            with pytest.raises(ih.IrisError):
                gdb.search(oc.gen_templates(1, 0, 1)[0])


def test_group_single_rank_communicator():
    """The multi-process form (helper-thread ncclCommInitRank (bounded)) with one rank: what each
    torchrun rank of bench.py builds; RCCL itself reports one rank on this GPU."""
    uid = ih.Group.unique_id()
    assert len(uid) == 128
    n = 3000
    ref = oc.gen_templates(SEED, 0, n)
    query = ref[1234].copy()
    query[5] ^= np.uint64(0xFF)
    with ih.Group.rank(0, 1, 0, uid) as g:
        assert (g.local_devices, g.ranks, g.first_rank) == (1, 1, 0)
        assert g.rccl_nranks == 1 and len(g.rccl_devices) == 1 and ":" in g.rccl_devices[0]
        with ih.GroupDatabase(g, ih.KIND_TEMPLATES, n, shards_per_device=2) as gdb:
            gdb.generate(SEED)
            best, idx = oracle_best(query, ref)
            assert same(gdb.search(query), best, idx) and idx == 1234


MISSING_PEER_CHILD = r"""
import json, os, sys, time
import numpy as np
import iris_hip as ih
from oracle import oracle_c as oc

t0 = time.monotonic()
err = None
try:
    ih.Group.rank(0, 2, 0, ih.Group.unique_id())  # rank 1 never comes
except ih.IrisError as e:
    err = str(e)
dt = time.monotonic() - t0
# a second 2-rank formation while the first init is still pending inside RCCL: refused at once
t1 = time.monotonic()
err2 = None
try:
    ih.Group.rank(0, 2, 0, ih.Group.unique_id())
except ih.IrisError as e:
    err2 = str(e)
dt2 = time.monotonic() - t1
probe = ih.Device(0)
abandoned = probe.config()["abandoned_inits"]
probe.close()
n = 2000
ref = oc.gen_templates(80, 0, n)
query = ref[777].copy()
best, idx = oc.argmin(oc.template_distances(query, ref))
dev = ih.Device(0)
with ih.Database(dev, ih.KIND_TEMPLATES, n) as db:
    db.append(ref)
    with ih.TemplateEngine(dev, query) as eng:
        m1 = eng.search(db)
with ih.Group.rank(0, 1, 0, ih.Group.unique_id()) as g:
    with ih.GroupDatabase(g, ih.KIND_TEMPLATES, n) as gdb:
        gdb.write(0, ref)
        m2 = gdb.search(query)
dev.close()
print(json.dumps({"err": err, "dt": dt, "err2": err2, "dt2": dt2, "abandoned": abandoned, "want": [int(idx), float(best)],
                  "single": [int(m1.index), m1.distance], "group": [int(m2.index), m2.distance]}))
sys.stdout.flush()
"""


def test_group_missing_peer_fails_within_bound(tmp_path):
    """A 2-rank group whose second rank never comes: forming it must fail within the bound
    (IRIS_GROUP_TIMEOUT_MS, read when the group's device opens) instead of hanging in RCCL's
    init; a second 2-rank formation while that init is still pending is refused at once (one
    abandoned init per device at most, iris_config abandoned_inits=1/1); the same process's GPU
    then searches and forms a 1-rank group normally, and the process exits although the abandoned
    init never finished.  Run in a child process so that
    its exit is part of what is tested."""
    import json
    import os
    import subprocess
    import sys
    import time

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, IRIS_GROUP_TIMEOUT_MS="6000",
               PYTHONPATH=os.pathsep.join([os.path.join(root, "mpc-iris-code_amd"), root]))
    script = tmp_path / "child.py"
    script.write_text(MISSING_PEER_CHILD)
    t0 = time.monotonic()
    r = subprocess.run([sys.executable, str(script)], cwd=root, env=env, capture_output=True, text=True,
                       timeout=150)
    wall = time.monotonic() - t0
    assert r.returncode == 0, (r.returncode, r.stderr[-3000:])
    d = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1])
    assert d["err"] and "did not complete within 6000 ms" in d["err"], d
    assert d["dt"] < 6 + 10, d  # the bound, plus opening the device
    # bounded leftovers: the second multi-rank attempt is refused without waiting, and says why
    assert d["err2"] and "still pending" in d["err2"] and "fresh process" in d["err2"], d
    assert d["dt2"] < 2, d
    assert d["abandoned"] == "1/1", d
    want_idx, want_d = d["want"]
    assert d["single"][0] == want_idx and d["group"][0] == want_idx == 777
    assert np.float64(d["single"][1]).view(np.uint64) == np.float64(want_d).view(np.uint64)
    assert np.float64(d["group"][1]).view(np.uint64) == np.float64(want_d).view(np.uint64)
    assert wall < 120, wall  # the child exited with the abandoned init still pending


TWO_RANK_CHILD = r"""
import json, os, sys, time
import iris_hip as ih

rank, idfile = int(sys.argv[1]), sys.argv[2]
if rank == 0:
    uid = ih.Group.unique_id()
    with open(idfile + ".tmp", "wb") as f:
        f.write(uid)
    os.rename(idfile + ".tmp", idfile)
else:
    t = time.monotonic()
    while not os.path.exists(idfile) and time.monotonic() - t < 60:
        time.sleep(0.01)
    with open(idfile, "rb") as f:
        uid = f.read()
t0 = time.monotonic()
err = None
try:
    ih.Group.rank(0, 2, rank, uid)  # both ranks on device 0
except ih.IrisError as e:
    err = str(e)
dt = time.monotonic() - t0
with ih.Group.rank(0, 1, 0, ih.Group.unique_id()) as g:  # the device still forms a group and searches
    with ih.GroupDatabase(g, ih.KIND_TEMPLATES, 3000) as gdb:
        gdb.generate(7)
        m = gdb.search(gdb.read(1234, 1)[0])
print(json.dumps({"err": err, "dt": dt, "found": [int(m.index), m.distance]}))
sys.stdout.flush()
"""


def test_group_two_ranks_bootstrap_then_refuse_one_device(tmp_path):
    """Two processes form one 2-rank group on the box's single GPU: RCCL's bootstrap must connect
    the ranks (each then finds the other's device in the exchanged peer table -- "Duplicate GPU
    detected: rank 0 and rank 1", which only a completed bootstrap can report) and refuses two
    ranks on one device; each create_rank fails with RCCL's error well inside the bound, not a
    hang, and each process's GPU then forms a 1-rank group and searches normally.  The one
    multi-process RCCL exchange a one-GPU box can run."""
    import json
    import os
    import subprocess
    import sys
    import time

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, IRIS_GROUP_TIMEOUT_MS="30000", NCCL_DEBUG="WARN",
               PYTHONPATH=os.pathsep.join([os.path.join(root, "mpc-iris-code_amd"), root]))
    script = tmp_path / "rank.py"
    script.write_text(TWO_RANK_CHILD)
    idfile = str(tmp_path / "uid")
    t0 = time.monotonic()
    procs = [subprocess.Popen([sys.executable, str(script), str(r), idfile], cwd=root, env=env,
                              stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True) for r in range(2)]
    outs = []
    try:
        for p in procs:
            outs.append(p.communicate(timeout=150))
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
                p.wait()
    assert time.monotonic() - t0 < 150
    logs = "".join(o + e for o, e in outs)  # RCCL's NCCL_DEBUG lines go to stdout
    for p, (out, err) in zip(procs, outs):
        assert p.returncode == 0, (p.returncode, err[-3000:])
        d = json.loads([ln for ln in out.splitlines() if ln.startswith("{")][-1])
        assert d["err"] and "ncclCommInitRank" in d["err"] and "did not complete" not in d["err"], d
        assert d["dt"] < 30, d
        assert d["found"] == [1234, 0.0], d
    assert "Duplicate GPU detected" in logs, logs[-3000:]


@pytest.mark.parametrize("side", ["plain", "delayed"])
def test_group_configs4_shape_on_one_gpu(group, hooked_group, device, side):
    """configs[4]'s shape rehearsed on the one GPU: 8 logical shards as 8 GPUs would hold them
    (10M templates, so that the single-device copy for the comparison fits beside it), an exact
    tie between the last record of shard 0 and a record of the last shard (the lower global
    index must win), then queries whose planted answers sit on both sides of every shard
    boundary, searched pipelined through the group and compared with the single-device search
    of the same records."""
    n, spd = 10_000_000, 8
    if side == "delayed":  # every all-gather held back: the next searches' kernels run before it
        group = hooked_group(IRIS_GROUP_DELAY_US=DELAY_US)
    query = oc.gen_templates(SEED + 40, 0, 1)[0]
    with ih.GroupDatabase(group, ih.KIND_TEMPLATES, n, shards_per_device=spd) as gdb, \
            ih.Database(device, ih.KIND_TEMPLATES, n) as db:
        gdb.generate(SEED)
        db.generate(n, SEED)
        firsts = [gdb.shard(i)[0] for i in range(spd)]
        exact = planted(query, 3)
        for site in (n - 2, firsts[1] - 1):
            gdb.write(site, exact[None, :])
            db.write(site, exact[None, :])
        m = gdb.search(query)
        assert m.index == firsts[1] - 1 and m.distance == 0.0 and m.rotation == 3
        sites = [s for f in firsts[1:] for s in (f, f - 2)]
        qs = [oc.gen_templates(SEED + 50 + k, 0, 1)[0] for k in range(len(sites))]
        for k, (site, q) in enumerate(zip(sites, qs)):
            rec = planted(q, (k % 31) - 15, 0x3 << (k % 60))
            gdb.write(site, rec[None, :])
            db.write(site, rec[None, :])
        pend = [gdb.search_async(q) for q in qs]
        for k, (q, p) in enumerate(zip(qs, pend)):
            g = p.wait()
            with ih.TemplateEngine(device, q) as eng:
                s1 = eng.search(db)
            assert (g.index, g.num, g.den, g.rotation) == (s1.index, s1.num, s1.den, s1.rotation), (k, g, s1)
            assert g.index == sites[k]


@pytest.mark.parametrize("form", ["search", "async", "batch"])
def test_group_lost_peer_is_an_error_not_a_hang(hooked_group, form):
    """IRIS_GROUP_STALL holds every all-gather back as a peer that never arrives would: the
    wait must give up after the group's bound, abort the communicator and fail; the group
    then refuses further calls, and destroying the database and the group returns."""
    import time

    g = hooked_group(IRIS_GROUP_STALL=1)
    g.set_timeout(700)
    n = 5000
    query = oc.gen_templates(SEED + 60, 0, 1)[0]
    gdb = ih.GroupDatabase(g, ih.KIND_TEMPLATES, n, shards_per_device=2)
    gdb.generate(SEED)
    t0 = time.monotonic()
    with pytest.raises(ih.IrisError) as ei:
        if form == "search":
            gdb.search(query)
        elif form == "async":
            gdb.search_async(query).wait()
        else:
            gdb.batch_search(oc.gen_templates(SEED + 61, 0, 9))
    assert time.monotonic() - t0 < 20, "the bound did not end the wait"
    assert "aborted" in str(ei.value) and "700 ms" in str(ei.value)
    with pytest.raises(ih.IrisError) as ei2:  # the group is broken from now on
        gdb.search(query)
    assert "aborted" in str(ei2.value)
    with pytest.raises(ih.IrisError):
        ih.GroupDatabase(g, ih.KIND_TEMPLATES, 10)
    gdb.close()
    g.close()


def test_group_finalizes_and_reforms(group):
    """A healthy group tears down through ncclCommFinalize + ncclCommDestroy; a new group on
    the same device then works (the communicator was released)."""
    query = oc.gen_templates(SEED + 70, 0, 1)[0]
    for _ in range(3):
        with ih.Group([0]) as g, ih.GroupDatabase(g, ih.KIND_TEMPLATES, 3000, shards_per_device=2) as gdb:
            gdb.generate(SEED)
            best, idx = oracle_best(query, gdb.read(0, 3000))
            assert same(gdb.search(query), best, idx)
