"""Diagnostic: per-call wall time of MasksEngine / DistanceEngine.batch_process on consecutive
20 000-record host slices of an attached array (the reference's resolver / participant loop),
with and without read-ahead.  usage: python tools/ra_diag.py masks|shares [n] [reps]"""
import pathlib
import sys
import time

ROOT = pathlib.Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "mpc-iris-code_amd"))
import numpy as np  # noqa: E402

import iris_hip as ih  # noqa: E402

kind = sys.argv[1]
n = int(sys.argv[2]) if len(sys.argv) > 2 else 400_000
reps = int(sys.argv[3]) if len(sys.argv) > 3 else 5
chunk = 20_000
rng = np.random.default_rng(1)
dev = ih.Device(0)
q = ih.Template.random(rng).to_array()
if kind == "masks":
    host = rng.integers(0, 2**63, (n, 200), dtype=np.uint64)
    eng, k = ih.MasksEngine(dev, q[200:]), ih.KIND_MASKS
else:
    host = rng.integers(0, 65536, (n, 12800), dtype=np.uint16)
    eng, k = ih.DistanceEngine(dev, ih.encode(ih.Template.from_array(q))), ih.KIND_SHARES
db = ih.Database(dev, k, n)
db.attach_host(host)
import mmap  # noqa: E402


def fresh_4k(m):
    """A new anonymous mapping per chunk, as the reference's vec![0; len] of 1.24 MB gets from
    malloc: 4-KB pages (no 2-MB-aligned span), zero-filled on first touch."""
    mm = mmap.mmap(-1, m * 31 * 2)
    return np.frombuffer(mm, np.uint16).reshape(m, 31)


for label, fresh in (("reused out", 0), ("fresh out per chunk", 1), ("fresh 4-KB mapping per chunk", 2)):
    hout = np.empty((n, 31), np.uint16)
    times = []
    for r in range(reps):
        for a in range(0, n, chunk):
            m = min(chunk, n - a)
            o = (np.empty((m, 31), np.uint16) if fresh == 1 else fresh_4k(m) if fresh == 2 else hout[a:a + chunk])
            t0 = time.perf_counter()
            eng.batch_process(o, host[a:a + chunk])
            times.append(time.perf_counter() - t0)
    t = np.array(times[len(times) // reps:]) * 1e6
    print(f"{kind} {label}: per call median {np.median(t):.1f} us  p10 {np.percentile(t, 10):.1f}  p90 {np.percentile(t, 90):.1f}")
