"""What the library sees of a read-only record-file mapping on this box: the mapping's
/proc/self/maps line, whether /proc/self/map_files answers for it, and (with a GPU) whether a
MasksEngine walk over it is served from a resident copy (iris_config's resident fields)."""
import os
import sys
import tempfile

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "mpc-iris-code_amd"))
import iris_hip as ih  # noqa: E402

n = 40_000
path = os.path.join(tempfile.gettempdir(), f"resident_diag_{os.getpid()}.masks")
np.random.default_rng(1).integers(0, 2**63, (n, 200), dtype=np.uint64).tofile(path)
m = np.memmap(path, dtype=np.uint64, mode="r", shape=(n, 200))
addr = m.ctypes.data
line = None
with open("/proc/self/maps") as f:
    for ln in f:
        lo, hi = (int(x, 16) for x in ln.split()[0].split("-"))
        if lo <= addr < hi:
            line = ln.strip()
            link = f"/proc/self/map_files/{lo:x}-{hi:x}"
print("maps:", line)
try:
    st = os.stat(link)
    print("map_files stat ok: ino", st.st_ino, "size", st.st_size)
except OSError as e:
    print("map_files stat failed:", e)
print("file stat: ino", os.stat(path).st_ino, "dev", os.stat(path).st_dev)
if ih.Device.count() > 0:
    dev = ih.Device(0)
    with ih.MasksEngine(dev, np.ones(200, np.uint64)) as eng:
        out = np.empty((n, 31), np.uint16)
        for a in range(0, n, 20_000):
            eng.batch_process(out[a:a + 20_000], m[a:a + 20_000])
    c = dev.config()
    print("resident:", c.get("resident"), "via_fd:", c.get("resident_via_fd"), "skip:", c.get("resident_skip"))
    dev.close()
del m
os.unlink(path)
