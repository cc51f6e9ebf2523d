"""Diagnostic: does overlapping consecutive searches on two streams (two device handles on
one GPU, each with its own 10M-template database) beat back-to-back searches on one?"""
import sys
import time

sys.path.insert(0, "mpc-iris-code_amd")
import numpy as np  # noqa: E402

import iris_hip as ih  # noqa: E402

n = 10_000_000
devs = [ih.Device(0), ih.Device(0)]
dbs = [ih.Database(d, ih.KIND_TEMPLATES, n) for d in devs]
for i, db in enumerate(dbs):
    db.generate(n, 11 + i)
rng = np.random.default_rng(3)
qs = [ih.Template.random(rng).to_array() for _ in range(8)]
K = 40


def one_stream():
    pend = None
    for i in range(K):
        e = ih.TemplateEngine(devs[0], qs[i % 8])
        p = e.search_async(dbs[0])
        e.close()
        if pend is not None:
            pend.wait()
        pend = p
    pend.wait()


def two_streams():
    pend = []
    for i in range(K):
        d = i % 2
        e = ih.TemplateEngine(devs[d], qs[i % 8])
        pend.append(e.search_async(dbs[d]))
        e.close()
        if len(pend) > 2:
            pend.pop(0).wait()
    for p in pend:
        p.wait()


for f in (one_stream, two_streams, one_stream, two_streams):
    f()
    devs[0].synchronize(); devs[1].synchronize()
    t0 = time.perf_counter()
    f()
    devs[0].synchronize(); devs[1].synchronize()
    dt = time.perf_counter() - t0
    print(f"{f.__name__:12s} {dt / K * 1e3:.3f} ms per search", flush=True)
