import os, sys, time, pathlib
sys.path.insert(0, "mpc-iris-code_amd")
import iris_hip as ih
dev = ih.Device(0)
n = 1_000_000
src = ih.Database(dev, ih.KIND_TEMPLATES, n); src.generate(n, 5)
p = pathlib.Path("/tmp/ld_diag.templates"); src.save_file(p)
tdb = ih.Database(dev, ih.KIND_TEMPLATES, n)
def run(label):
    ts = []
    for _ in range(3):
        tdb.truncate(0); t0 = time.perf_counter(); tdb.load_file(p); ts.append(time.perf_counter() - t0)
    print(label, ["%.1f ms" % (t * 1e3) for t in ts], "%.1f GB/s" % (3.2 / min(ts)), flush=True)
run("right after save  mmap ")
os.environ["IRIS_LOAD_PREAD"] = "1"; run("right after save  pread")
del os.environ["IRIS_LOAD_PREAD"]
os.system("sync"); time.sleep(5)
run("after sync        mmap ")
os.environ["IRIS_LOAD_PREAD"] = "1"; run("after sync        pread")
os.system("df -h /tmp | tail -1")
p.unlink()
