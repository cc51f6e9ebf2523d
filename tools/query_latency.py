"""Diagnostic: per-query latency of the serving loop (new query -> TemplateEngine ->
search -> result) against the search alone, on a resident 10M-template TILES database."""
import pathlib
import sys
import time

ROOT = pathlib.Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "mpc-iris-code_amd"))
import numpy as np  # noqa: E402

import iris_hip as ih  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 10_000_000
dev = ih.Device(0)
db = ih.Database(dev, ih.KIND_TEMPLATES, n)
db.generate(n, 7)
rng = np.random.default_rng(1)
queries = [ih.Template.random(rng) for _ in range(30)]


def timeit(label, fn, reps=20):
    fn()
    t = []
    for i in range(reps):
        t0 = time.perf_counter()
        fn(i)
        t.append(time.perf_counter() - t0)
    t = np.array(t) * 1e3
    print(f"{label:40s} median {np.median(t):8.3f} ms  min {t.min():8.3f} ms")


eng = ih.TemplateEngine(dev, queries[0])
timeit("search only (engine reused)", lambda i=0: eng.search(db))
timeit("engine create + destroy", lambda i=0: ih.TemplateEngine(dev, queries[i % 30]).close())
timeit("create + search + destroy", lambda i=0: (lambda e: (e.search(db), e.close()))(ih.TemplateEngine(dev, queries[i % 30])))
small = ih.Database(dev, ih.KIND_TEMPLATES, 32 * 1024)
small.generate(32 * 1024, 3)
timeit("create + search(32k) + destroy", lambda i=0: (lambda e: (e.search(small), e.close()))(ih.TemplateEngine(dev, queries[i % 30])))
timeit("search(32k) only", lambda i=0: eng.search(small))
