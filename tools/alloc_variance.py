"""Diagnostic: is the search time's bimodality tied to the database allocation?  Allocates
a fresh 10M-template database six times in one process and times 20 searches on each."""
import sys
import time

sys.path.insert(0, "mpc-iris-code_amd")
import numpy as np  # noqa: E402

import iris_hip as ih  # noqa: E402

n = 10_000_000
dev = ih.Device(0)
q = ih.Template.random(np.random.default_rng(1)).to_array()
keep = []
for trial in range(6):
    db = ih.Database(dev, ih.KIND_TEMPLATES, n)
    db.generate(n, 7)
    with ih.TemplateEngine(dev, q) as e:
        e.search(db)
        dev.reset_stats()
        dev.set_profiling(True)
        for _ in range(20):
            e.search(db)
        dev.set_profiling(False)
    launches, ms, _ = dev.kernel_stats("template_search")
    print(f"allocation {trial}: kernel {ms / launches:.3f} ms", flush=True)
    if trial % 2:
        keep.append(db)  # keep every other one alive so the next lands elsewhere
    else:
        db.close()
