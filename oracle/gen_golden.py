"""TEST INFRASTRUCTURE ONLY — writes tests/golden/golden_v1.npz.

Inputs come from the DESIGN.md §5 counter-based generator (seed 42) plus
hand-built edge cases; expected outputs come from the C oracle and are only
written after the independent numpy restatement reproduces every one of them.
The reference's own real-data fixtures (data/templates.json, distances.json)
are absent from the reference checkout, so these vectors are the pinned set.

    python oracle/gen_golden.py
"""
import pathlib
import sys

import numpy as np

ROOT = pathlib.Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))

from oracle import oracle_c as oc  # noqa: E402
from oracle import oracle_np as on  # noqa: E402

SEED = 42
N_TEMPLATES = 24
N_SHARES = 6


def edge_templates(q):
    """Edge cases: identical, rotated copies at +-15 (+ light flips), empty mask,
    full mask, all-ones pattern, single valid bit."""
    rng = np.random.default_rng(7)
    out = []
    out.append(q.copy())  # identical -> distance 0 at r = 0
    for r in (15, -15, 7):
        p = oc.bits_rotated(q[:200], -r)
        m = oc.bits_rotated(q[200:], -r)
        flips = np.zeros(200, np.uint64)
        for b in rng.choice(12800, 40, replace=False):
            flips[b // 64] |= np.uint64(1) << np.uint64(b % 64)
        out.append(np.concatenate([p ^ flips, m]))
    out.append(np.concatenate([q[:200], np.zeros(200, np.uint64)]))  # empty mask -> +inf
    out.append(np.concatenate([q[:200], np.full(200, np.uint64(2**64 - 1))]))  # full mask
    out.append(np.full(400, np.uint64(2**64 - 1)))  # all ones
    single = np.zeros(400, np.uint64)
    single[200 + 3] = np.uint64(1) << np.uint64(5)
    out.append(single)  # one valid bit
    return np.stack(out)


def main():
    db = oc.gen_templates(SEED, 0, N_TEMPLATES)
    query = db[0].copy()
    db = np.concatenate([db[1:], edge_templates(query)])
    n = db.shape[0]

    num, den = oc.template_counts(query, db)
    dist = oc.template_distances(query, db)
    best, best_idx = oc.argmin(dist)
    masks_out = oc.masks_batch(query[200:], db[:, 200:])

    # numpy restatement must agree exactly
    n2, d2 = on.template_counts(query[:200], query[200:], db[:, :200], db[:, 200:])
    assert (n2 == num).all() and (d2 == den).all()
    dd = on.template_distances(query[:200], query[200:], db[:, :200], db[:, 200:])
    assert (dd.view(np.uint64) == dist.view(np.uint64)).all()
    assert on.argmin(dist) == (best, best_idx)
    assert (on.masks_batch(query[200:], db[:, 200:]) == masks_out).all()
    for i in range(n):
        assert oc.template_distance(query, db[i]) == dist[i] or (np.isinf(dist[i]) and np.isinf(oc.template_distance(query, db[i])))

    # encoded path (DistanceEngine + decode), resolver with 3 additive shares
    enc_q = oc.encode(query)
    enc_db = np.stack([oc.encode(t) for t in db[:N_SHARES]])
    assert (on.encode(db[:N_SHARES, :200], db[:N_SHARES, 200:]) == enc_db).all()
    rng = np.random.default_rng(11)
    s0 = rng.integers(0, 2**16, enc_db.shape, dtype=np.uint16)
    s1 = rng.integers(0, 2**16, enc_db.shape, dtype=np.uint16)
    s2 = (enc_db - s0 - s1).astype(np.uint16)
    share_out = np.stack([oc.distance_batch(enc_q, s) for s in (s0, s1, s2)])
    for k, s in enumerate((s0, s1, s2)):
        assert (on.distance_batch(enc_q, s) == share_out[k]).all()
    resolved = oc.resolver_combine(share_out, masks_out[:N_SHARES])
    assert (resolved.view(np.uint64) == dist[:N_SHARES].view(np.uint64)).all()

    # rotations of the query mask (Bits::rotated reference algorithm vs formula)
    rot_mask = np.stack([oc.bits_rotated(query[200:], r) for r in range(-15, 16)])
    assert all((on.bits_rotated(query[200:], r) == rot_mask[r + 15]).all() for r in range(-15, 16))

    # dot_u16 wraparound case
    wrap_a = np.full(12800, 0xFFFF, np.uint16)
    wrap_b = np.arange(12800, dtype=np.uint16) * np.uint16(7919)
    wrap_dot = np.uint16(oc.dot_u16(wrap_a, wrap_b))
    assert int(on.dot_u16(wrap_a, wrap_b)) == int(wrap_dot)

    out = ROOT / "tests" / "golden" / "golden_v1.npz"
    out.parent.mkdir(parents=True, exist_ok=True)
    np.savez_compressed(
        out,
        seed=np.uint64(SEED), query=query, db=db, num=num, den=den, dist_bits=dist.view(np.uint64),
        argmin_dist_bits=np.float64(best).view(np.uint64), argmin_index=np.uint64(best_idx),
        masks_out=masks_out, enc_query=enc_q, enc_db=enc_db, shares=np.stack([s0, s1, s2]),
        share_out=share_out, rot_mask=rot_mask, wrap_a=wrap_a, wrap_b=wrap_b, wrap_dot=wrap_dot,
    )
    print(f"wrote {out} ({out.stat().st_size} bytes); argmin {best} @ {best_idx}")


if __name__ == "__main__":
    main()
