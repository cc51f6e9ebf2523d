"""Diagnostic (round 4): the timeline of one 10M-template search launch, from a build with
-DIRIS_MFMA_DIAG=4 (IRIS_HIP_LIB=.../libiris_tl.so): every workgroup's start / end on the
constant-rate clock (100 MHz) and its XCD.  Prints the launch span, how long the grid takes to fill
the chip and to drain, the workgroup durations, and the in-flight workgroup count over time."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "mpc-iris-code_amd"))
import iris_hip as ih  # noqa: E402

N = int(os.environ.get("N", 10_000_000))
TICK_US = 0.01  # s_memrealtime: 100 MHz

with ih.Device(0) as dev, ih.Database(dev, ih.KIND_TEMPLATES, N) as db:
    db.generate(N, 42)
    q = np.random.default_rng(1).integers(0, 2**63, 400, dtype=np.uint64)
    buf = dev.alloc(N * 8)
    with ih.TemplateEngine(dev, q) as eng:
        for _ in range(30):  # warm-up
            eng.search(db)
        runs = []
        for rep in range(5):
            eng.search(db, dist_out_device=buf)
            raw = np.empty(N, np.uint64)
            dev.d2h(raw, buf)
            runs.append(raw)
    dev.free(buf)

grid = (N + 32 * 16 - 1) // (32 * 16)
for rep, raw in enumerate(runs):
    tl = raw[: 3 * grid].reshape(grid, 3).astype(np.int64)
    t0, t1, xcc = tl[:, 0], tl[:, 1], tl[:, 2]
    base = t0.min()
    s, e = (t0 - base) * TICK_US, (t1 - base) * TICK_US
    span = e.max()
    dur = e - s
    # in-flight workgroups over time (1-us bins)
    bins = np.arange(0, span + 1, 1.0)
    cnt = np.zeros(len(bins))
    for a, b in zip(s, e):
        cnt[int(a):int(b) + 1] += 1
    full = cnt.max()
    fill_us = np.argmax(cnt >= 0.95 * full)
    drain_from = len(cnt) - np.argmax(cnt[::-1] >= 0.95 * full)
    lost = np.sum(full - cnt[: len(cnt)]) / full  # us of full-chip time not used
    print(f"run {rep}: span {span:.1f} us, wg duration median {np.median(dur):.1f} us (p5 {np.percentile(dur, 5):.1f}, "
          f"p95 {np.percentile(dur, 95):.1f}), max in flight {full:.0f}, 95%-full reached at {fill_us} us, "
          f"below 95% from {drain_from} us ({span - drain_from:.1f} us drain), under-full time {lost:.1f} us-equivalent; "
          f"last start {s.max():.1f} us; per-XCD end spread {np.ptp([e[xcc == x].max() for x in range(8)]):.1f} us")
    if rep == 0:
        print("  in flight every 100 us:", " ".join(str(int(c)) for c in cnt[::100]))
        print("  last 200 us in 10-us steps:", " ".join(str(int(c)) for c in cnt[-200::10]))
