"""Round 4: Database.read of a large range (iris_db_read) into a fresh numpy array and into a reused one, best of
3, for the library IRIS_HIP_LIB points at.   python tools/read_paths.py NAME"""
import pathlib
import sys
import time

import numpy as np

ROOT = pathlib.Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "mpc-iris-code_amd"))
import iris_hip as ih  # noqa: E402

name = sys.argv[1]
dev = ih.Device(0)
for kind, n, label in ((ih.KIND_MASKS, 2_000_000, "2M masks"), (ih.KIND_SHARES, 200_000, "200k shares")):
    with ih.Database(dev, kind, n) as db:
        db.generate(n, 42)
        a = db.read(0, n)
        fresh, reused = [], []
        for _ in range(3):
            t = time.perf_counter()
            b = db.read(0, n)
            fresh.append(time.perf_counter() - t)
            assert (b == a).all()
            del b
        lib = ih.load_library()
        for _ in range(3):
            t = time.perf_counter()
            ih._check(lib.iris_db_read(db.handle, 0, n, ih._ptr(a)))
            reused.append(time.perf_counter() - t)
        print(f"{name:8s} {label:12s} fresh array {min(fresh) * 1e3:7.1f} ms ({a.nbytes / min(fresh) / 1e9:5.1f} GB/s)  "
              f"reused array {min(reused) * 1e3:7.1f} ms ({a.nbytes / min(reused) / 1e9:5.1f} GB/s)", flush=True)
dev.close()
