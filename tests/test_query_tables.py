"""Rotated-query tables of the engines (the query side of every kernel).

CPU: the host reference builders (iris_host.cpp, via iris_host_query_tables) against
a numpy restatement of each layout (iris_internal.hpp) over the oracle's rotation
(Bits::rotated / EncodedBits::rotated, src/bits.rs:18-29, src/encoded_bits.rs:40-58).
GPU: the tables an engine builds on the device (iris_query.hip) equal the host
builders' bytes exactly, for every kind, for edge-case queries and batched tiles."""
import numpy as np
import pytest

import iris_hip as ih
from oracle import oracle_np as on

ROT = 31
J = np.arange(32)
FRAG_BIT = (J & 16) + 2 * (J & 7) + ((J >> 3) & 1)      # template fp4 element j <-> dword bit
MASK_FRAG_BIT = 4 * (J & 7) + (J >> 3)                  # masks fp4 element j <-> dword bit
MASK_CODE_SHIFT = 4 * (J & 7) + np.array([2, 1, 0, 3])[J >> 3]


def dwords(limbs):
    return np.ascontiguousarray(limbs, np.uint64).view(np.uint32)


def rotations(limbs):
    """[31, 400] dwords of rot(limbs, k - 15)."""
    return np.stack([dwords(on.bits_rotated(limbs, k - 15)) for k in range(ROT)])


def expect_template(q):
    pattern, mask = q[:200], q[200:]
    m, p = rotations(mask), rotations(pattern)
    tab = np.zeros((400, 64), np.uint32)
    tab[:, 0:62:2] = m.T
    tab[:, 1:62:2] = p.T
    frag = np.zeros((200, 64, 4), np.uint32)
    for k in range(ROT):
        for h in range(2):
            mw = m[k, h::2][:, None]  # dword 2c + h, [200, 1]
            pw = p[k, h::2][:, None]
            mb = (mw >> FRAG_BIT) & 1
            pb = (pw >> FRAG_BIT) & 1
            code = mb * np.where(pb == 1, 0xA, 0x2).astype(np.uint32)  # [200, 32]
            for d in range(4):
                frag[:, k + 32 * h, d] = np.bitwise_or.reduce(
                    code[:, 8 * d:8 * d + 8] << (4 * np.arange(8, dtype=np.uint32)), axis=1)
    return tab, frag


def expect_masks(qmask):
    m = rotations(qmask)
    tab = np.zeros((400, 32), np.uint32)
    tab[:, :ROT] = m.T
    frag = np.zeros((50, 64, 4), np.uint32)
    for k in range(ROT):
        for h in range(2):
            x = m[k, h::2][:, None]  # [200 chunks, 1]
            f = np.bitwise_or.reduce(((x >> MASK_FRAG_BIT) & 1) << MASK_CODE_SHIFT.astype(np.uint32), axis=1)
            frag[:, k + 32 * h, :] = f.reshape(50, 4)
    return tab, frag


def expect_shares(q):
    rot = np.stack([on.encoded_rotated(q, k - 15) for k in range(ROT)]).astype(np.uint32)  # [31, 12800]
    tab = np.zeros((6400, 32), np.uint32)
    tab[:, :ROT] = (rot[:, 0::2] | (rot[:, 1::2] << 16)).T
    frag = np.ones((400, 2, 64, 16), np.uint8)  # [chunk, lo/hi, lane, j]; row 31 all ones
    e = rot.reshape(ROT, 400, 2, 16)  # [k, c, h, j]
    lo = ((e & 0xFF) ^ 0x80).astype(np.uint8)
    hi = ((e >> 8) ^ 0x80).astype(np.uint8)
    for h in range(2):
        frag[:, 0, h * 32:h * 32 + ROT, :] = lo[:, :, h, :].transpose(1, 0, 2)
        frag[:, 1, h * 32:h * 32 + ROT, :] = hi[:, :, h, :].transpose(1, 0, 2)
    qsum = np.zeros((32, 2), np.int32)
    qsum[:ROT, 0] = lo.astype(np.int8).astype(np.int32).reshape(ROT, -1).sum(1)
    qsum[:ROT, 1] = hi.astype(np.int8).astype(np.int32).reshape(ROT, -1).sum(1)
    return tab, np.concatenate([frag.reshape(-1), qsum.reshape(-1).view(np.uint8)])


def xpack(em16, ep16):
    x = np.zeros_like(em16)
    for p in range(8):
        x |= ((em16 >> (2 * p + 1)) & 1) << (4 * p)
        x |= ((em16 >> (2 * p)) & 1) << (4 * p + 1)
        x |= ((ep16 >> (2 * p + 1)) & 1) << (4 * p + 2)
        x |= ((ep16 >> (2 * p)) & 1) << (4 * p + 3)
    return x


def expect_tiles(queries):
    nq = len(queries)
    nqp = (nq + 3) // 4 * 4
    tiles = np.zeros((nqp, 100, 64, 4), np.uint32)
    for i, q in enumerate(queries):
        m, p = rotations(q[200:]), rotations(q[:200])
        for h in range(2):
            em0, ep0 = m[:, h::4], p[:, h::4]          # dword 4g + h, [31, 100]
            em1, ep1 = m[:, 2 + h::4], p[:, 2 + h::4]  # dword 4g + 2 + h
            v = [xpack(em0 & 0xFFFF, ep0 & 0xFFFF), xpack(em0 >> 16, ep0 >> 16),
                 xpack(em1 & 0xFFFF, ep1 & 0xFFFF), xpack(em1 >> 16, ep1 >> 16)]
            for d in range(4):
                tiles[i, :, 32 * h:32 * h + ROT, d] = v[d].T
    return tiles


def queries(rng):
    """Random queries plus the edges: empty mask, full mask, single bits at row ends."""
    out = [np.concatenate([rng.integers(0, 2**63, 200, dtype=np.uint64) * 2 + rng.integers(0, 2, 200, dtype=np.uint64),
                           rng.integers(0, 2**63, 200, dtype=np.uint64) * 2 + rng.integers(0, 2, 200, dtype=np.uint64)])
           for _ in range(2)]
    out.append(np.zeros(400, np.uint64))
    out.append(np.full(400, np.uint64(2**64 - 1)))
    edge = np.zeros(400, np.uint64)
    for bit in (0, 199, 200, 12799):  # first / last column of rows 0, 63
        edge[200 + bit // 64] |= np.uint64(1) << np.uint64(bit % 64)
        edge[bit // 64] |= np.uint64(1) << np.uint64((bit + 1) % 64)
    out.append(edge)
    return out


def test_host_template_tables():
    for q in queries(np.random.default_rng(5))[:3]:
        tab, frag = ih.host_query_tables(ih.KIND_TEMPLATES, q)
        et, ef = expect_template(q)
        assert (tab.view(np.uint32).reshape(400, 64) == et).all()
        assert (frag.view(np.uint32).reshape(200, 64, 4) == ef).all()


def test_host_masks_tables():
    for q in queries(np.random.default_rng(6))[:3]:
        tab, frag = ih.host_query_tables(ih.KIND_MASKS, q[200:])
        et, ef = expect_masks(q[200:])
        assert (tab.view(np.uint32).reshape(400, 32) == et).all()
        assert (frag.view(np.uint32).reshape(50, 64, 4) == ef).all()


def test_host_shares_tables():
    rng = np.random.default_rng(7)
    for q in (rng.integers(0, 65536, 12800, dtype=np.uint16), np.full(12800, 65535, np.uint16)):
        tab, frag = ih.host_query_tables(ih.KIND_SHARES, q)
        et, ef = expect_shares(q)
        assert (tab.view(np.uint32).reshape(6400, 32) == et).all()
        assert (frag == ef).all()


def test_host_batch_tiles():
    qs = queries(np.random.default_rng(8))
    tab, frag = ih.host_query_tables(ih.KIND_TEMPLATES, np.stack(qs), nq=len(qs))
    assert tab.size == 0
    assert (frag.view(np.uint32).reshape(-1, 100, 64, 4) == expect_tiles(qs)).all()


def test_table_sizes_reject_bad_arguments():
    with pytest.raises(ih.IrisError):
        ih.query_table_sizes(ih.KIND_TEMPLATES, 2)  # streamed batches have no tiles
    with pytest.raises(ih.IrisError):
        ih.query_table_sizes(99)


@pytest.mark.gpu
def test_device_tables_equal_host(device):
    rng = np.random.default_rng(9)
    for q in queries(rng):
        with ih.TemplateEngine(device, ih.Template.from_array(q)) as e:
            dt, df = e.query_tables()
        ht, hf = ih.host_query_tables(ih.KIND_TEMPLATES, q)
        assert (dt == ht).all() and (df == hf).all()
        with ih.MasksEngine(device, ih.Bits(q[200:])) as e:
            dt, df = e.query_tables()
        ht, hf = ih.host_query_tables(ih.KIND_MASKS, q[200:])
        assert (dt == ht).all() and (df == hf).all()
    for q in (rng.integers(0, 65536, 12800, dtype=np.uint16), np.zeros(12800, np.uint16),
              np.full(12800, 65535, np.uint16)):
        with ih.DistanceEngine(device, ih.EncodedBits(q)) as e:
            dt, df = e.query_tables()
        ht, hf = ih.host_query_tables(ih.KIND_SHARES, q)
        assert (dt == ht).all() and (df == hf).all()


@pytest.mark.gpu
@pytest.mark.parametrize("nq", [4, 5, 9])
def test_device_batch_tiles_equal_host(device, nq):
    rng = np.random.default_rng(10 + nq)
    qs = (queries(rng) * 3)[:nq]
    with ih.TemplateBatchEngine(device, np.stack(qs)) as e:
        _, df = e.query_tables()
    _, hf = ih.host_query_tables(ih.KIND_TEMPLATES, np.stack(qs), nq=nq)
    assert (df == hf).all()


@pytest.mark.gpu
def test_engine_pool_reuse_and_handle_order(device):
    """Engines recycle query buffers through the device pool (no stale tables), and a
    device closed before its databases / engines stays alive until they are freed."""
    rng = np.random.default_rng(11)
    qs = queries(rng)
    for i in range(40):
        q = qs[i % len(qs)]
        with ih.TemplateEngine(device, ih.Template.from_array(q)) as e:
            dt, df = e.query_tables()
        ht, hf = ih.host_query_tables(ih.KIND_TEMPLATES, q)
        assert (dt == ht).all() and (df == hf).all()
    dev = ih.Device(0)
    db = ih.Database(dev, ih.KIND_TEMPLATES, 1000)
    db.generate(1000, 3)
    eng = ih.TemplateEngine(dev, ih.Template.from_array(qs[0]))
    dev.close()  # handles outlive it
    m = eng.search(db)
    db2 = ih.Database(device, ih.KIND_TEMPLATES, 1000)
    db2.generate(1000, 3)
    with ih.TemplateEngine(device, ih.Template.from_array(qs[0])) as e2:
        m2 = e2.search(db2)
    assert (m.index, m.num, m.den, m.rotation) == (m2.index, m2.num, m2.den, m2.rotation)
    assert m.den > 0
    eng.close()
    db.close()
