"""Diagnostic: wall time per participant-sized call (20 000 records, src/main.rs:428,473)
against the kernel time recorded with HIP events, for the call forms a participant /
resolver makes with one engine per request (the engine built once, reused per chunk):

  search      TemplateEngine.search (kernel + partials reduce + result to the host)
  masks-dev   MasksEngine.batch_process_device (rows stay in HBM)
  masks-host  MasksEngine.batch_process into a host array (rows D2H)
  shares-dev  DistanceEngine.batch_process_device

usage: python tools/chunk_latency.py [n=20000] [calls=3000]"""
import json
import pathlib
import sys
import time

ROOT = pathlib.Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "mpc-iris-code_amd"))
import numpy as np  # noqa: E402

import iris_hip as ih  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 20_000
calls = int(sys.argv[2]) if len(sys.argv) > 2 else 3000
dev = ih.Device(0)
q = ih.Template.random(np.random.default_rng(1)).to_array()
tdb = ih.Database(dev, ih.KIND_TEMPLATES, n)
tdb.generate(n, 7)
mdb = ih.Database(dev, ih.KIND_MASKS, n)
mdb.generate(n, 7)
sdb = ih.Database(dev, ih.KIND_SHARES, n)
sdb.generate(n, 7)
out_dev = dev.alloc(n * 31 * 2)
hout = np.empty((n, 31), np.uint16)
te = ih.TemplateEngine(dev, q)
me = ih.MasksEngine(dev, q[200:])
de = ih.DistanceEngine(dev, ih.encode(ih.Template.from_array(q)))
forms = {
    "search": ("template_search", lambda: te.search(tdb)),
    "masks-dev": ("masks", lambda: me.batch_process_device(mdb, out_dev)),
    "masks-host": ("masks", lambda: me.batch_process(hout, mdb)),
    "shares-dev": ("shares", lambda: de.batch_process_device(sdb, out_dev)),
}
res = {}
for name, (kname, fn) in forms.items():
    t_end = time.perf_counter() + 1.0
    while time.perf_counter() < t_end:  # warm
        fn()
    t = np.empty(calls)  # wall time per call, no event recording
    for i in range(calls):
        t0 = time.perf_counter()
        fn()
        t[i] = time.perf_counter() - t0
    dev.reset_stats()  # kernel time from HIP events in a separate pass
    dev.set_profiling(True)
    for i in range(min(calls, 500)):
        fn()
    dev.set_profiling(False)
    launches, kms, _ = dev.kernel_stats(kname)
    _, rms, _ = dev.kernel_stats("reduce")
    res[name] = {"call_us_median": float(np.median(t) * 1e6), "call_us_mean": float(t.mean() * 1e6),
                 "kernel_us": kms / max(1, launches) * 1e3, "reduce_us": rms / max(1, launches) * 1e3,
                 "ratio_median": float(np.median(t) * 1e6) / (kms / max(1, launches) * 1e3)}
    print(name, json.dumps(res[name]))
print(json.dumps({"n": n, "calls": calls, "forms": res}))
