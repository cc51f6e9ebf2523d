"""Diagnostic: does the search time depend on where the engine's query fragments land?
Keeps 12 engines alive at once (distinct buffers) and times 20 searches with each."""
import sys

sys.path.insert(0, "mpc-iris-code_amd")
import numpy as np  # noqa: E402

import iris_hip as ih  # noqa: E402

n = 10_000_000
dev = ih.Device(0)
db = ih.Database(dev, ih.KIND_TEMPLATES, n)
db.generate(n, 7)
q = ih.Template.random(np.random.default_rng(1)).to_array()
engines = [ih.TemplateEngine(dev, q) for _ in range(12)]
res = []
for i, e in enumerate(engines):
    e.search(db)
    dev.reset_stats()
    dev.set_profiling(True)
    for _ in range(20):
        e.search(db)
    dev.set_profiling(False)
    launches, ms, _ = dev.kernel_stats("template_search")
    res.append(ms / launches)
    print(f"engine {i:2d}: kernel {ms / launches:.3f} ms", flush=True)
print("spread %.2f %%" % ((max(res) - min(res)) / min(res) * 100))
