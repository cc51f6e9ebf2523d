"""Share preparation on the device (the reference's
`prepare`, src/main.rs:333-361, EncodedBits::share src/encoded_bits.rs:23-38):
bit-exact against the oracle's restatement of the ChaCha (8/12/20-round) counter-mode
derivation, and the prepared shares drive the MPC flow to the plaintext answer."""
import numpy as np
import pytest

import iris_hip as ih
from oracle import oracle_c as oc

pytestmark = pytest.mark.gpu
ROT = 31
KEY = bytes(range(7, 39))


@pytest.mark.parametrize("layout", [ih.LAYOUT_TILES, ih.LAYOUT_LANES], ids=["tiles", "lanes"])
@pytest.mark.parametrize("parties,rounds", [(1, 12), (2, 12), (3, 12), (3, 20), (2, 8)])
def test_prepare_matches_oracle(device, layout, parties, rounds):
    n = 70
    t = oc.gen_templates(31, 0, n)
    want_s, want_m = oc.prepare_shares(t[5:5 + 60], KEY, nonce=11, parties=parties, index_base=1000 + 5,
                                       rounds=rounds)
    with ih.Database(device, ih.KIND_TEMPLATES, n, layout) as tdb:
        tdb.append(t)
        sdbs = [ih.Database(device, ih.KIND_SHARES, 64, layout) for _ in range(parties)]
        with ih.Database(device, ih.KIND_MASKS, 64, layout) as mdb:
            mdb.append(t[:1, 200:])  # appends after existing records
            ih.prepare_shares(tdb, sdbs, mdb, key=KEY, nonce=11, first=5, n=60, index_base=1000, rounds=rounds)
            assert len(mdb) == 61 and (mdb.read(1, 60) == want_m).all()
        for j, db in enumerate(sdbs):
            assert len(db) == 60
            assert (db.read(0, 60) == want_s[j]).all()
            db.close()


def test_prepare_multi_chunk_sampled(device):
    """60 000 templates x 3 parties span two staging chunks (55 872 templates each with
    in-place TILES shares); sampled records are checked against the oracle at their own
    global index, all of them via the share-sum identity."""
    n = 60_000
    with ih.Database(device, ih.KIND_TEMPLATES, n) as tdb:
        tdb.generate(n, 99)
        sdbs = [ih.Database(device, ih.KIND_SHARES, n) for _ in range(3)]
        key = ih.prepare_shares(tdb, sdbs)  # random key from os.urandom
        assert len(key) == 32
        for i in (0, 1, 55871, 55872, 55873, n - 1):
            rec = tdb.read(i, 1)
            want, _ = oc.prepare_shares(rec, key, parties=3, index_base=i)
            for j in range(3):
                assert (sdbs[j].read(i, 1)[0] == want[j, 0]).all()
        # sum identity on everything, via the dot engine: sum_j <q, s_j> == <q, encode(t)> per rotation
        q = ih.encode(ih.Template.from_array(tdb.read(17, 1)[0]))
        acc = np.zeros((n, ROT), np.uint32)
        with ih.DistanceEngine(device, q) as eng:
            for db in sdbs:
                out = np.empty((n, ROT), np.uint16)
                eng.batch_process(out, db)
                acc += out
            enc = np.stack([oc.encode(x) for x in tdb.read(0, 64)])
            with ih.Database(device, ih.KIND_SHARES, 64) as edb:
                edb.append(enc)
                direct = np.empty((64, ROT), np.uint16)
                eng.batch_process(direct, edb)
        assert ((acc[:64] % 65536) == direct).all()
        for db in sdbs:
            db.close()


def test_mpc_with_device_prepared_shares(device):
    n = 1500
    templates = oc.gen_templates(55, 0, n)
    q = templates[999].copy()
    q[:200] ^= np.uint64(0x10)
    with ih.Database(device, ih.KIND_TEMPLATES, n) as tdb, ih.TemplateEngine(device, q) as te:
        tdb.append(templates)
        sdbs = [ih.Database(device, ih.KIND_SHARES, n) for _ in range(3)]
        mdb = ih.Database(device, ih.KIND_MASKS, n)
        ih.prepare_shares(tdb, sdbs, mdb)
        enc_q = ih.encode(ih.Template.from_array(q))
        outs = []
        for db in sdbs:
            with ih.DistanceEngine(device, enc_q) as eng:
                out = np.empty((n, ROT), np.uint16)
                eng.batch_process(out, db)
                outs.append(out)
        with ih.MasksEngine(device, q[200:]) as me:
            den = np.empty((n, ROT), np.uint16)
            me.batch_process(den, mdb)
        m = ih.resolver_search(outs, den, device=device)
        ref = te.search(tdb)
        for db in sdbs + [mdb]:
            db.close()
    best, idx = oc.argmin(oc.template_distances(q, templates))
    assert m.index == ref.index == idx == 999
    assert np.float64(m.distance).view(np.uint64) == np.float64(best).view(np.uint64)


def test_prepare_argument_errors(device):
    with ih.Database(device, ih.KIND_TEMPLATES, 10) as tdb, ih.Database(device, ih.KIND_SHARES, 10) as s, \
            ih.Database(device, ih.KIND_MASKS, 10) as m:
        tdb.generate(10, 1)
        with pytest.raises(ih.IrisError):
            ih.prepare_shares(tdb, [s, s])         # the same database twice
        with pytest.raises(ih.IrisError):
            ih.prepare_shares(tdb, [m])            # wrong kind
        with pytest.raises(ih.IrisError):
            ih.prepare_shares(tdb, [s], first=5, n=10)  # outside the template range
        with pytest.raises(ih.IrisError):
            ih.prepare_shares(tdb, [s], rounds=10)      # not ChaCha8/12/20
        assert len(s) == 0
