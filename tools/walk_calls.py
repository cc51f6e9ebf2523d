"""Per-call times of the reference's chunk walk (20 000-record batch_process calls, one engine
per walk as the participant builds one per request) over a mapped record file (the library's
resident copy, no attach) and over an attached anonymous array, side by side:
    python tools/walk_calls.py [masks|shares] [walks] [records]"""
import os
import sys
import tempfile
import time

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "mpc-iris-code_amd"))
import iris_hip as ih  # noqa: E402

kind_name = sys.argv[1] if len(sys.argv) > 1 else "shares"
walks = int(sys.argv[2]) if len(sys.argv) > 2 else 4
shares = kind_name == "shares"
n, chunk = (200_000, 20_000) if shares else (2_000_000, 20_000)
if len(sys.argv) > 3:
    n = int(sys.argv[3])
kind = ih.KIND_SHARES if shares else ih.KIND_MASKS
rng = np.random.default_rng(3)
host = (rng.integers(0, 65536, (n, 12800), dtype=np.uint16) if shares
        else rng.integers(0, 2**63, (n, 200), dtype=np.uint64))  # noqa: E501
path = os.path.join(tempfile.gettempdir(), f"walk_calls_{os.getpid()}.rec")
host.tofile(path)
mm = np.memmap(path, dtype=host.dtype, mode="r", shape=host.shape)
dev = ih.Device(0)
print("config:", {k: v for k, v in dev.config().items() if "readahead" in k or k == "test_hooks"})
q = (ih.encode(ih.Template.from_array(rng.integers(0, 2**63, 400, dtype=np.uint64))) if shares
     else rng.integers(0, 2**63, 200, dtype=np.uint64))


def engine():
    return ih.DistanceEngine(dev, q) if shares else ih.MasksEngine(dev, q)


out = np.empty((n, 31), np.uint16)


def walk(arr):
    times = []
    t_new = time.perf_counter()
    with engine() as e:
        t_eng = time.perf_counter() - t_new
        for a in range(0, n, chunk):
            t = time.perf_counter()
            e.batch_process(out[a:a + chunk], arr[a:a + chunk])
            times.append(time.perf_counter() - t)
    t_all = time.perf_counter() - t_new
    return t_eng, times, t_all


db = ih.Database(dev, kind, n)
db.attach_host(host)
for label, arr in (("mmap", mm), ("attached", host)):
    for w in range(walks):
        t_eng, times, t_all = walk(arr)
        st = sorted(times)
        print(f"{label} walk {w}: engine {t_eng * 1e6:.0f} us, walk {t_all * 1e3:.3f} ms ({n / t_all:.3g} records/s), "
              f"calls us median {st[len(st) // 2] * 1e6:.1f} p90 {st[len(st) * 9 // 10] * 1e6:.1f}, first ones:",
              " ".join(f"{x * 1e6:.0f}" for x in times[:12]), flush=True)
print("config:", {k: v for k, v in dev.config().items() if k.startswith("resident")})
db.close()
dev.close()
del mm
os.unlink(path)
