"""Round 4: the upload path of a non-attached host-slice masks call against where the caller's records
come from -- the bench's array (records read back from the device, Database.read), a fresh numpy copy of it,
and a read-only np.memmap of a file holding them (the reference's participant maps its record file,
src/main.rs:389-391) -- for each upload path pinned by the IRIS_UPLOAD test hook.
    python tools/upload_sources.py OUTDIR"""
import os
import pathlib
import sys
import time

import numpy as np

ROOT = pathlib.Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "mpc-iris-code_amd"))
sys.path.insert(0, str(ROOT))
import bench  # noqa: E402  (pages_nodes)
import iris_hip as ih  # noqa: E402

N = 2_000_000


def backing(a):
    """Rss / AnonHugePages (kB) of the mappings that hold the array (/proc/self/smaps): whether its
    pages are 2-MB transparent huge pages, 4-KB pages or a file's page cache."""
    lo, hi = a.ctypes.data, a.ctypes.data + a.nbytes
    rss = huge = 0
    name = ""
    cur = None
    for line in open("/proc/self/smaps"):
        f = line.split()
        if "-" in f[0] and len(f) >= 5 and all(c in "0123456789abcdef-" for c in f[0]):
            s0, e0 = (int(x, 16) for x in f[0].split("-"))
            cur = s0 < hi and e0 > lo
            if cur and len(f) >= 6:
                name = f[5]
        elif cur and f[0] == "Rss:":
            rss += int(f[1])
        elif cur and f[0] == "AnonHugePages:":
            huge += int(f[1])
    return {"rss_kB": rss, "anon_huge_kB": huge, "file": name}


out_dir = pathlib.Path(sys.argv[1])
out_dir.mkdir(parents=True, exist_ok=True)
os.environ["IRIS_TEST_HOOKS"] = "1"
devs = {}
for path in ("pinned", "runtime"):
    os.environ["IRIS_UPLOAD"] = path
    devs[path] = ih.Device(0)
del os.environ["IRIS_UPLOAD"], os.environ["IRIS_TEST_HOOKS"]
d0 = devs["pinned"]
with ih.Database(d0, ih.KIND_MASKS, N) as g:
    g.generate(N, 42)
    read_back = g.read(0, N)
fresh = np.empty_like(read_back)
np.copyto(fresh, read_back)
fpath = out_dir / "masks.bin"
read_back.tofile(fpath)
mapped = np.memmap(fpath, dtype=np.uint64, mode="r", shape=(N, 200))
_ = int(np.asarray(mapped[::4096]).sum())  # page cache warm (the file was just written)
q = read_back[7]
want = None
for src_name, src in (("read_back", read_back), ("fresh_copy", fresh), ("memmap", mapped)):
    for path, dev in devs.items():
        eng = ih.MasksEngine(dev, q)
        out = np.empty((N, 31), np.uint16)
        eng.batch_process(out, src)  # warm-up
        if want is None:
            want = out.copy()
        assert (out == want).all()
        ts = []
        for _ in range(3):
            t = time.perf_counter()
            eng.batch_process(out, src)
            ts.append(time.perf_counter() - t)
        eng.close()
        best = min(ts)
        print(f"{src_name:10s} {path:8s} ms {best * 1e3:7.2f} GB/s {src.nbytes / best / 1e9:5.1f} "
              f"pages {bench.pages_nodes(np.asarray(src))} gpu_node {dev.config()['numa_node']} {backing(src)}", flush=True)
del mapped
fpath.unlink()
for d in devs.values():
    d.close()
