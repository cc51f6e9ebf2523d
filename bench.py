"""Headline benchmark: 1 query x 31 rotations x N templates, masked Hamming
(Template path) with fused min/argmin, on N GPUs (one process per GPU).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--n-per-gpu T]
    torchrun --nproc-per-node N bench.py --gpus N ...

`python bench.py --gpus N` with N > 1 and no launcher starts the N ranks itself
(torch.distributed.run as a child process, before this process touches a GPU)
and exits with their status; every rank checks that the process group really
has N ranks (and, on RCCL, that it owns a GPU of its own) and exits non-zero
otherwise, so a scaling run can never print a one-GPU line for N GPUs.

A step = one search of the query against every resident template on every
rank (the query engine build, the kernel, the partials reduce) plus, for N > 1,
the RCCL all-gather of the per-shard minima and their merge.  Steps are
pipelined by default (iris_template_search_async): step i+1's search is
enqueued before step i's result is waited for and exchanged, so the host work
and the exchange overlap the next kernel; --no-pipeline waits step by step.  The database is synthetic (the
DESIGN.md §5 generator, uniform random pattern and mask bits as the
reference's rng.gen::<Template>()), generated on each GPU so that shard k
holds global templates [k*T, (k+1)*T) — inputs are resident in HBM before
the timed region.  Rotated, lightly perturbed copies of the query (of four
queries in four query groups for --workload batch) are planted at known global
indices; every run checks they are found (exit 3 otherwise).
"""
import argparse
import json
import os
import pathlib
import socket
import subprocess
import sys
import tempfile
import time

import numpy as np

ROOT = pathlib.Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "mpc-iris-code_amd"))

import iris_hip as ih  # noqa: E402  (loads libiris_hip.so; no HIP call until a Device is opened)

METRIC = "template comparisons/sec (query×rotations×DB) + % HBM roofline, 1/2/4/8 GPU"
HBM_PEAK_GBS = 8000.0        # MI355X_MICROARCH.md: 8.0 TB/s spec
HBM_GUIDE_COPY_GBS = 6290.0  # MI355X_MICROARCH.md: float4 copy (read + write), not a read ceiling
# best pure 16-B read stream over 32 GB on this part after a 1.5-s warm-up
# (tools/ubench_stream.hip, profiles/r01_ubench_read_stream_warm.txt: 7.02 TB/s at 12 waves
# per CU, 6.78 TB/s at the search kernel's 8)
HBM_READ_CEILING_GBS = 7016.0
# integer VALU issue ceiling for v_bcnt/v_bitop3 (16 lanes/clk/SIMD measured, tools/ubench_ops.hip)
VALU_INT_PEAK_OPS = 256 * 4 * 16 * 2.4e9
FP4_DENSE_PEAK_MACS = 10e15 / 2            # MI355X_MICROARCH.md: ~10 PF dense fp4
MFMA_MACS_PER_TEMPLATE = 2 * 12800 * 31    # algorithmic: den + enc products of the 31 rotations
MFMA_MACS_ISSUED_PER_TEMPLATE = 2 * 12800 * 32  # issued: the 32x32 tile carries a zero 32nd row
BYTES_PER_TEMPLATE = 3200    # pattern + mask planes, read once per query
VALU_OPS_PER_TEMPLATE = 400 * 31 * 4   # words x rotations x (and, bitop3, 2x bcnt)
ROT = 31
SEED = 20251015
GPU_WORKLOADS = ("search", "masks", "shares", "batch")
AUX_WORKLOADS = ("resolver", "host-resolver", "resolve-masks", "host-resolve-masks", "prepare", "load", "host-shares", "host-masks", "criterion")


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--n-per-gpu", type=int, default=None,
                    help="records per GPU (default 10M; search with 2+ ranks: 12.5M, so 8 ranks are configs[4]'s 100M)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--reuse-engine", action="store_true",
                    help="build the query engine once instead of once per step (default: per step, in the timed region)")
    ap.add_argument("--no-pipeline", action="store_true",
                    help="search: wait for each step's result before enqueueing the next query "
                         "(default: the next query's search is enqueued before this one's result is "
                         "waited for and exchanged)")
    ap.add_argument("--prewarm-s", type=float, default=3.0,
                    help="seconds of untimed steps before the warmup steps (the GPU reaches its steady "
                         "streaming rate after ~0.5-1 s of load)")
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--layout", choices=["tiles", "lanes"], default="tiles",
                    help="tiles = MFMA kernels (default), lanes = VALU kernels")
    ap.add_argument("--queries", type=int, default=1024, help="queries per batch (workload batch)")
    ap.add_argument("--workload", choices=list(GPU_WORKLOADS + AUX_WORKLOADS), default="search",
                    help="search = Template masked Hamming + argmin (configs[1], default); "
                         "masks = MasksEngine denominators; shares = DistanceEngine u16 share dot (configs[3]); "
                         "batch = --queries queries x 31 rotations x N templates in one pass (configs[2]); "
                         "resolver = fused share sum + decode + argmin over --parties [n][31] outputs; "
                         "resolve-masks = the same with the denominators computed on the fly from a masks DB; "
                         "prepare = GPU share preparation of n templates into --parties share DBs + masks; "
                         "load = raw template file (page-cached) -> resident TILES database; "
                         "host-shares / host-masks = batch_process over host slices (the reference signature); "
                         "criterion = configs[0]: 1 query x 31 x 10k search plus the arch dot shapes of "
                         "src/arch/mod.rs:22-72, beside the CPU criterion loop")
    ap.add_argument("--parties", type=int, default=3, help="parties (workloads resolver, prepare)")
    ap.add_argument("--rounds", type=int, default=12, choices=[8, 12, 20],
                    help="ChaCha rounds for --workload prepare (12 = the reference's thread_rng, rand 0.8.5)")
    ap.add_argument("--single-process", action="store_true",
                    help="search / batch: ONE process drives --gpus devices as a library device group "
                         "(iris_group_*: one RCCL communicator per device, all-gather of the shard winners) instead of "
                         "one torchrun rank per GPU")
    ap.add_argument("--attached", action="store_true",
                    help="host-shares / host-masks: the host array is attached to a resident database "
                         "(iris_db_attach_host), so the reference-signature calls on its slices upload nothing")
    ap.add_argument("--chunk", type=int, default=None,
                    help="host-shares / host-masks: records per batch_process call (the reference's "
                         "participant / resolver use 20 000, src/main.rs:428,473; default: 20 000 with "
                         "--attached or --mmap, else the whole array in one call)")
    ap.add_argument("--mmap", action="store_true",
                    help="host-shares / host-masks: the records are a file mapped read-only (np.memmap, as "
                         "the participant / resolver map theirs, src/main.rs:386-391, 455-460) and the calls "
                         "walk its slices with no attach call (the library keeps the file resident)")
    ap.add_argument("--no-auto-resident", action="store_true",
                    help="open the device with IRIS_AUTO_RESIDENT=0 (slices of file mappings upload per call)")
    ap.add_argument("--dry-run", action="store_true",
                    help="launcher rehearsal without a GPU: start / join the ranks, check the world size, "
                         "exchange and merge a synthetic per-rank result over gloo, print the line (value null)")
    return ap.parse_args()


def planted_record(query, rotation, flips=0x00FF00FF00FF00FF):
    p = ih.Bits(query[:200]).rotated(rotation).limbs.copy()
    m = ih.Bits(query[200:]).rotated(rotation).limbs
    p[7] ^= np.uint64(flips)  # 32 flipped bits
    return np.concatenate([p, m])


def plant_sites(total, count):
    """`count` distinct global indices inside [0, total) for planted answers (the first is
    3/4 of the way in, so with 2+ ranks it lies in a later rank's shard)."""
    if total <= 0:
        return []
    base = total * 3 // 4 + min(12345, total // 8)
    step = max(1, total // 7)
    sites = []
    for k in range(count):
        s = (base + k * step) % total
        while s in sites:
            s = (s + 1) % total
        sites.append(s)
        if len(sites) == total:
            break
    return sites


def batch_plant_queries(nq):
    """Queries that get a planted answer in the batch run: four query groups apart
    (group = 4 consecutive queries, iris_batch.hip BQ), including the first and last."""
    return sorted({nq // 2, 0, nq - 1, nq // 4 + 1} & set(range(nq)))


def pages_nodes(a, samples=32):
    """{NUMA node: sampled pages} of a host array (move_pages query form; {} if unavailable):
    where the caller's records live decides how fast an upload can go."""
    import ctypes

    try:
        libc = ctypes.CDLL(None, use_errno=True)
        base, nbytes = a.ctypes.data, a.nbytes
        pages = (ctypes.c_void_p * samples)(*[(base + nbytes * i // samples) & ~4095 for i in range(samples)])
        status = (ctypes.c_int * samples)()
        if libc.syscall(279, 0, ctypes.c_ulong(samples), pages, None, status, 0) != 0:  # SYS_move_pages (x86-64)
            return {}
        out = {}
        for v in status:
            out[int(v)] = out.get(int(v), 0) + 1
        return out
    except (OSError, AttributeError):
        return {}


def gen_records(dev, kind, n, seed):
    """Host copies of records from the library's on-device generator."""
    with ih.Database(dev, kind, max(n, 1)) as g:
        g.generate(n, seed)
        return g.read(0, n)


# Result checks of the bench (numpy restatements, independent of the kernels; the
# oracle/ package is used only by the cpu_baseline leg).
def check_masks_rows(qmask, recs):
    """[s, 31] popcount(rot(qmask, k-15) & rec) (src/lib.rs:69-79)."""
    rot = np.stack([ih.Bits(qmask).rotated(k - 15).limbs for k in range(ROT)])
    x = (np.asarray(recs, np.uint64)[:, None, :] & rot[None, :, :]).view(np.uint8)
    return np.unpackbits(x, axis=-1).sum(axis=-1).astype(np.uint16)


def check_shares_rows(q, recs):
    """[s, 31] sum(rot(q, k-15) * rec) mod 2^16 (src/lib.rs:42-52)."""
    rot = np.stack([ih.EncodedBits(q).rotated(k - 15).values for k in range(ROT)]).astype(np.uint64)
    return ((np.asarray(recs, np.uint64) @ rot.T) % 65536).astype(np.uint16)


def check_resolver(shares, denoms):
    """The resolver loop (src/main.rs:597-621): wrapping share sum, decode_distance
    (src/lib.rs:97-107), first strict minimum -> (distance, index)."""
    num = np.add.reduce(np.asarray(shares, np.uint16), axis=0, dtype=np.uint16)
    den = np.asarray(denoms, np.uint16)
    uneq = ((den - num).astype(np.uint16) >> 1).astype(np.float64)
    with np.errstate(divide="ignore", invalid="ignore"):
        d = np.where(den != 0, uneq / den.astype(np.float64), np.inf).min(axis=1)
    idx = int(np.argmin(d))
    return (float(d[idx]), idx) if np.isfinite(d[idx]) else (float("inf"), 2**64 - 1)


# ---------------------------------------------------------------------------- CPU baseline


def cpu_info():
    """Where the CPU leg runs: the CPUs this process may use (its affinity mask, which is
    what the leg's thread count is), the machine's count and the cgroup's CPU quota."""
    try:
        model = next(l.split(":", 1)[1].strip() for l in open("/proc/cpuinfo") if l.startswith("model name"))
    except Exception:
        model = "unknown"
    quota = None
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        quota = None if q == "max" else int(q) / int(per)
    except Exception:
        pass
    return {"model": model, "nproc": os.cpu_count(), "affinity_cpus": len(os.sched_getaffinity(0)),
            "cgroup_cpu_quota": quota}


def _time_passes(fn, seconds, max_passes=1000):
    passes, t = 0, 0.0
    while (t < seconds or passes == 0) and passes < max_passes:
        t0 = time.perf_counter()
        fn()
        t += time.perf_counter() - t0
        passes += 1
    return passes, t


def cpu_baseline(args, reserve=0):
    """The oracle's CPU restatement of the reference path for this workload (test
    infrastructure: oracle/), compiled -O3 -march=native for this host and run on every
    CPU the process may use, timed on a bounded sample (~--cpu-seconds) of the same
    workload.  Rates are per the workload's unit, so they compare with `value`."""
    from oracle import oracle_c as oc

    info = cpu_info()
    # every CPU the process may run on: its affinity mask, unless the cgroup's CPU quota grants
    # less CPU time than that (on the GPU box: 256 CPUs in the mask, a 16-CPU quota; 256
    # threads under that quota measured 2.9e8 comparisons/s against 4.0e8 with 16,
    # profiles/r02_bench_search_cpu256.jsonl), in which case one thread per quota CPU
    threads = info["affinity_cpus"]
    if info["cgroup_cpu_quota"]:
        threads = max(1, min(threads, int(-(-info["cgroup_cpu_quota"] // 1))))
    # reserve: CPUs left to a concurrent GPU-driving thread (the leg runs beside the untimed
    # pre-warm, so the GPU is busy while the CPU is measured; the thread count says so)
    threads = max(1, threads - reserve)
    path = pathlib.Path(tempfile.gettempdir()) / f"liboracle_native_{os.getpid()}.so"
    try:
        oc.build(path, march="native")
        oc_lib = oc.load(str(path))
        flags = "gcc -O3 -march=native"
    except Exception:
        oc_lib = oc.load()  # the prebuilt x86-64-v3 oracle
        flags = "gcc -O3 -march=x86-64-v3"
    finally:
        path.unlink(missing_ok=True)
    oc._lib = oc_lib  # the oracle_c helpers below use this build
    wl = args.workload
    secs = args.cpu_seconds
    extra = {}
    if wl in ("search", "batch"):
        n = 1_000_000  # 3.2 GB of templates: far beyond the CPU caches, streamed from DRAM each pass
        nq = 1 if wl == "search" else 4
        db = oc.gen_templates(SEED, 0, n)
        qs = oc.gen_templates(SEED + 1, 0, nq)
        out = np.empty(n, np.float64)
        d, i = np.zeros(1, np.float64), np.zeros(1, np.uint64)

        def run():
            for q in qs:  # per query: Template::distance per pair + the resolver's argmin
                oc_lib.orc_template_distances_batch(oc._p(q), oc._p(db), n, oc._p(out), threads)
                oc_lib.orc_argmin(oc._p(out), n, oc._p(d), oc._p(i))

        passes, t = _time_passes(run, secs)
        value, unit = ROT * n * nq * passes / t, "template comparisons/s"
        sample = (f"{passes} passes of {nq} quer{'y' if nq == 1 else 'ies'} x 31 rotations x {n} templates "
                  "(the fractional Hamming of src/template.rs:49-64 per pair and rotation + argmin, src/main.rs:616-621; "
                  "the 31 rotated queries are built once per query, engine-style, rather than per pair as "
                  "Template::distance does, src/template.rs:43-47 -- a stronger-than-reference CPU baseline)")
    elif wl in ("masks", "host-masks"):
        n = 2_000_000  # 3.2 GB of masks
        db = oc.gen_masks(SEED, 0, n)
        q = oc.gen_masks(SEED + 1, 0, 1)[0]
        out = np.empty((n, ROT), np.uint16)
        passes, t = _time_passes(lambda: oc_lib.orc_masks_batch(oc._p(q), oc._p(db), n, oc._p(out), threads), secs)
        value, unit = n * passes / t, "records/s"
        if wl == "masks":  # the GPU line's unit
            value, unit = ROT * value, "template comparisons/s"
        sample = f"{passes} passes of MasksEngine::batch_process over {n} masks (src/lib.rs:69-79)"
    elif wl in ("shares", "host-shares"):
        n = 100_000  # 2.56 GB of shares (the 10M-share DB does not fit host RAM): extrapolated per record
        db = oc.gen_shares(SEED, 0, n)
        q = oc.encode(oc.gen_templates(SEED + 1, 0, 1)[0])
        out = np.empty((n, ROT), np.uint16)
        passes, t = _time_passes(lambda: oc_lib.orc_distance_batch(oc._p(q), oc._p(db), n, oc._p(out), threads),
                                 secs)
        value = n * passes / t
        unit = "records/s" if wl == "host-shares" else "template comparisons/s"
        if wl == "shares":
            value *= ROT
        sample = (f"{passes} passes of DistanceEngine::batch_process (dot_u16, src/lib.rs:42-52, "
                  f"src/arch/generic.rs:11-16) over {n} shares, per-record rate extrapolated")
    elif wl in ("resolver", "host-resolver", "resolve-masks", "host-resolve-masks"):
        n = 2_000_000
        rng = np.random.default_rng(SEED)
        shares = rng.integers(0, 65536, (args.parties, n, ROT), dtype=np.uint16)
        denoms = rng.integers(0, 12801, (n, ROT), dtype=np.uint16)
        out = np.empty(n, np.float64)
        d, i = np.zeros(1, np.float64), np.zeros(1, np.uint64)

        def run():
            # the share sum + decode split over the threads (rayon into_par_iter, src/main.rs:597-612);
            # the argmin stays sequential (src/main.rs:616-621)
            oc_lib.orc_resolver_combine(oc._p(shares), args.parties, oc._p(denoms), n, oc._p(out), threads)
            oc_lib.orc_argmin(oc._p(out), n, oc._p(d), oc._p(i))

        passes, t = _time_passes(run, secs)
        value, unit = n * passes / t, "records/s"
        sample = (f"{passes} passes of the share sum + decode (parallel over entries, as the reference's rayon "
                  f"into_par_iter, src/main.rs:597-612) + sequential argmin (src/main.rs:616-621) over {n} entries")
        if wl in ("resolve-masks", "host-resolve-masks"):
            sample += " (the masks engine's denominators are not included)"
    elif wl == "prepare":
        n = 2000 * threads
        tmpl = oc.gen_templates(SEED, 0, n)
        passes, t = _time_passes(lambda: oc.prepare_shares(tmpl, bytes(range(32)), parties=args.parties,
                                                           rounds=args.rounds, threads=threads), secs)
        value, unit = n * passes / t, "templates/s"
        sample = (f"{passes} passes of encode + EncodedBits::share({args.parties}) (ChaCha{args.rounds}) over {n} "
                  "templates, parallel over templates as the reference's rayon par_iter (src/main.rs:337-344)")
    elif wl == "criterion":
        threads = 1  # criterion runs the loop on one thread (src/arch/mod.rs:34-41)
        shapes = {}
        rng = np.random.default_rng(SEED)
        for name, shp in (("dot_bool", [(1, 1), (1, 1000), (31, 1000), (1, 100_000)]),
                          ("dot_u16", [(1, 1), (1, 1000), (31, 1000), (1, 100_000), (31, 100_000)])):
            for a, b in shp:
                if name == "dot_bool":
                    av = rng.integers(0, 2**63, (a, 200), dtype=np.uint64)
                    bv = rng.integers(0, 2**63, (b, 200), dtype=np.uint64)
                    fn = lambda: oc.dot_bool_pairs(av, bv)  # noqa: E731
                else:
                    av = rng.integers(0, 65536, (a, 12800), dtype=np.uint16)
                    bv = rng.integers(0, 65536, (b, 12800), dtype=np.uint16)
                    fn = lambda: oc.dot_u16_pairs(av, bv)  # noqa: E731
                p, tt = _time_passes(fn, min(2.0, secs / 9))
                shapes[f"{name}/{a * b}"] = a * b * p / tt
        n = 10_000
        db = oc.gen_templates(SEED, 0, n)
        q = oc.gen_templates(SEED + 1, 0, 1)[0]
        out = np.empty(n, np.float64)
        passes, t = _time_passes(lambda: oc_lib.orc_template_distances_batch(oc._p(q), oc._p(db), n, oc._p(out), 1),
                                 min(2.0, secs / 5))
        value, unit = ROT * n * passes / t, "template comparisons/s"
        extra["criterion_elements_per_s"] = shapes
        sample = (f"configs[0]: {passes} passes of 1 query x 31 x {n} templates (Template::distance), one thread; "
                  "criterion shapes of src/arch/mod.rs:29,53 timed with the same loop order")
    else:  # load: a PCIe/page-cache path with no CPU compute counterpart (the reference mmaps)
        return None
    return {"value": value, "unit": unit, "cores": threads, "threads": threads, "kind": "port",
            "sample": f"{sample}, {t:.2f} s, {threads} thread(s) on {info['model']}, {flags} oracle/iris_oracle.c",
            "host": info, **extra}


def cxx_walk(shares, n, path, walks=6):
    """tools/walk_host (C++ against the C ABI, as the reference's Rust participant / resolver would
    call it) walking the bench's own mapped file in 20 000-record calls, one engine per walk, in a
    child process with its own device context (its first walk makes the file resident there):
    the records/s of the walks after the first, without the Python binding's ~3.5 us per call."""
    exe = pathlib.Path(tempfile.gettempdir()) / f"walk_host_{os.getpid()}"  # built from this tree's source
    try:
        subprocess.run(["g++", "-O2", "-std=c++17", "-I", str(ROOT / "include"), str(ROOT / "tools" / "walk_host.cpp"),
                        "-L", str(ROOT / "mpc-iris-code_amd"), "-liris_hip",
                        f"-Wl,-rpath,{ROOT / 'mpc-iris-code_amd'}", "-Wl,-rpath-link,/opt/rocm/lib", "-o", str(exe)],
                       check=True, capture_output=True, timeout=120)
        r = subprocess.run([str(exe), "shares" if shares else "masks", str(n), str(walks), str(path)],
                           capture_output=True, text=True, timeout=300)
        exe.unlink(missing_ok=True)
        rates = [float(l.split(",")[1].split()[0]) for l in r.stdout.splitlines() if l.startswith("walk ")][1:]
        calls = [l for l in r.stdout.splitlines() if l.startswith("calls after walk 0")]
        if r.returncode != 0 or not rates:
            return {"error": f"rc={r.returncode} " + (r.stderr + r.stdout)[-300:]}
        rates.sort()
        return {"records_per_s_median": rates[len(rates) // 2], "records_per_s_walks": rates,
                "calls": calls[0] if calls else None, "source": "tools/walk_host.cpp"}
    except Exception as ex:  # reported, never fatal
        return {"error": str(ex)[-300:]}


def load_traffic(workload, n_per_launch, layout):
    """HBM bytes per launch of the workload's kernel from the committed PMC run
    (profiles/*_pmc_<workload>[_lanes].json, FETCH_SIZE/WRITE_SIZE in separate passes,
    corrected per MI355X_MICROARCH.md §HBM by tools/pmc_summarize.py), scaled to this
    launch size; (None, None) if absent."""
    suffix = "" if layout == "tiles" else "_" + layout
    for p in sorted((ROOT / "profiles").glob(f"*_pmc_{workload}{suffix}.json"), reverse=True):
        try:
            j = json.loads(p.read_text())
            if j.get("layout") != layout:
                continue
            return j["hbm_bytes_per_record"] * n_per_launch, p.name
        except Exception:
            continue
    return None, None


def batch_pmc():
    """SQ-counter figures of the 1024-query batched launch from the committed profile
    (tools/pmc_batch.sh, profiles/r02_pmc_batch_sq.json): VALU and LDS instructions per MFMA
    and the bytes fetched beyond L2, reported beside the MFMA roofline fraction."""
    try:
        p = sorted((ROOT / "profiles").glob("r*_pmc_batch_sq.json"))[-1]  # the newest round's
        j = json.loads(p.read_text())
    except Exception:
        return None
    out = {"valu_per_mfma": j["valu_per_mfma_incl_mfma"], "valu_per_mfma_excl_mfma": j["valu_per_mfma_excl_mfma"],
           "lds_insts_per_mfma": j["lds_insts_per_mfma"], "beyond_l2_bytes_per_launch": j["beyond_l2_bytes_per_launch"],
           "source": "profiles/" + p.name + " (committed rocprofv3 --pmc run of this command)"}
    if "energy" in j:  # round 4 on: nJ per MFMA against the fp4 MFMA alone, same box
        e = j["energy"]
        out["energy"] = {k: e[k] for k in ("nj_per_mfma_batch", "nj_per_mfma_mfma_alone", "gap",
                                           "batch_rate_vs_mfma_alone", "source")}
    return out


# ---------------------------------------------------------------------------- launching


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def launch_ranks(args):
    """`python bench.py --gpus N` (N > 1) without a launcher: run the N ranks under
    torch.distributed.run as a CHILD process and return their exit status (this process may
    have initialised HIP by counting devices, so it must only ever spawn children, never
    re-exec).  Refuses (rc 2) when the RCCL path is asked for more GPUs than are visible."""
    backend = "gloo" if args.dry_run else os.environ.get("IRIS_DIST_BACKEND", "nccl")
    if backend == "nccl":
        have = ih.Device.count()
        if have < args.gpus:
            print(f"error: --gpus {args.gpus} needs {args.gpus} visible GPUs for one RCCL rank each; "
                  f"{have} visible", file=sys.stderr)
            return 2
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), str(pathlib.Path(__file__).resolve()),
           *sys.argv[1:]]
    env = dict(os.environ, IRIS_BENCH_LAUNCHER="bench.py")
    return subprocess.call(cmd, env=env)


class Ranks:
    """Who this process is in a multi-rank run.

    backend "nccl" (the default, one rank per GPU): torch.distributed runs on gloo (CPU) for
    the rendezvous, barriers and the max-over-ranks timing only; the data-path exchange is
    the library's own RCCL communicator (iris_group_create_rank, librccl from /opt/rocm):
    rank 0's 128-byte id is broadcast over gloo, every rank joins with its GPU, and the
    shard winners are all-gathered by the library.  IRIS_DIST_BACKEND=gloo rehearses the
    flow without RCCL (several ranks may then share one GPU): the winners go through torch
    CPU tensors and iris_match_merge.  --single-process: one process, a library group over
    --gpus devices, no torch at all."""

    def __init__(self, args):
        self.world = int(os.environ.get("WORLD_SIZE", "1"))
        self.rank = int(os.environ.get("RANK", "0"))
        self.local = int(os.environ.get("LOCAL_RANK", "0"))
        self.dist = None
        self.group = None
        self.backend = None
        self.ordinal = 0
        self.group_form_s = None
        self.rccl_error = None  # why the RCCL group did not form (the run fell back to gloo)
        self.stray_group = None
        if args.single_process:
            if "WORLD_SIZE" in os.environ and self.world > 1:
                raise SystemExit("error: --single-process drives every GPU from one process; do not launch ranks")
            self.world, self.rank = 1, 0
            self.backend = "rccl (library group, one process: helper-thread ncclCommInitRank (bounded) per device)"
            return
        if self.world != args.gpus:
            raise SystemExit(f"error: --gpus {args.gpus} but the launcher started WORLD_SIZE={self.world} ranks")
        backend = "gloo" if args.dry_run else os.environ.get("IRIS_DIST_BACKEND", "nccl")
        # IRIS_FORCE_DIST=1 runs the process-group path even for one rank (a one-GPU rehearsal
        # of the RCCL exchange, barriers and max-over-ranks timing)
        if self.world == 1 and os.environ.get("IRIS_FORCE_DIST") != "1":
            return
        import torch.distributed as dist

        if not args.dry_run:
            have = ih.Device.count()
            # a launcher that gives each rank only its own GPU (a *_VISIBLE_DEVICES list per rank)
            # leaves one device visible: that one is the rank's (RCCL refuses two ranks on one GPU)
            own = have == 1 and any(os.environ.get(v) for v in
                                    ("HIP_VISIBLE_DEVICES", "ROCR_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES"))
            if backend == "nccl" and self.local >= have and not own:
                raise SystemExit(f"error: rank {self.rank} (local {self.local}) has no GPU of its own: {have} visible")
            self.ordinal = 0 if own else self.local % max(1, have)
        # bounded: a rank that never starts fails the others here instead of holding them for
        # torch's default 30 minutes (IRIS_DIST_TIMEOUT_S overrides)
        import datetime

        dist.init_process_group("gloo", rank=self.rank, world_size=self.world,
                                timeout=datetime.timedelta(seconds=float(os.environ.get("IRIS_DIST_TIMEOUT_S", "300"))))
        if dist.get_world_size() != args.gpus:
            raise SystemExit(f"error: process group has {dist.get_world_size()} ranks, --gpus {args.gpus}")
        self.dist = dist
        self.backend = ("gloo" if backend == "gloo" else
                        "rccl (library group, helper-thread ncclCommInitRank (bounded); gloo control)")
        self.rccl = backend == "nccl"

    def join_group(self, args):
        """The library device group of this run (None: single device, or the gloo rehearsal)."""
        # one node (the bench contract): RCCL's bootstrap sockets over loopback; the data path is
        # xGMI peer-to-peer either way (a caller's own setting wins)
        os.environ.setdefault("NCCL_SOCKET_IFNAME", "lo")
        t0 = time.perf_counter()
        if args.single_process:
            self.group = ih.Group(list(range(args.gpus)))
        elif self.dist is not None and self.rccl:
            box = [ih.Group.unique_id() if self.rank == 0 else None]
            self.dist.broadcast_object_list(box, src=0)
            err = None
            try:
                self.group = ih.Group.rank(self.ordinal, self.world, self.rank, box[0])
            except Exception as ex:  # bounded: a formation that cannot finish fails, never hangs
                err = f"rank {self.rank}: {ex}"
            # every rank learns whether every rank formed the group, so all take the same path
            errs = [None] * self.world
            self.dist.all_gather_object(errs, err)
            failed = [e for e in errs if e]
            if failed:
                if os.environ.get("IRIS_RCCL_FALLBACK", "1") == "0":
                    raise SystemExit(f"error: the RCCL group did not form: {'; '.join(failed)}")
                # the search still runs, its winners exchanged over gloo (the rehearsal path), and
                # the line says so; a communicator that formed on this rank only is left open
                # (tearing it down would wait for the ranks that failed)
                self.rccl_error = "; ".join(failed)
                self.stray_group, self.group, self.rccl = self.group, None, False
                self.backend = "gloo exchange (fallback: the RCCL group did not form on every rank)"
        # wall time of forming the group (RCCL init + the bus-id all-gather), max over ranks below
        self.group_form_s = time.perf_counter() - t0 if self.group is not None else None
        return self.group

    def barrier(self):
        if self.dist is not None:
            self.dist.barrier()

    def max_over_ranks(self, x):
        if self.dist is None:
            return x
        import torch

        t = torch.tensor([x], dtype=torch.float64)
        self.dist.all_reduce(t, op=self.dist.ReduceOp.MAX)
        return float(t.item())

    def gather_lists(self, xs):
        """Every rank's list of floats, concatenated in rank order (the same on every rank)."""
        if self.dist is None:
            return list(xs)
        out = [None] * self.dist.get_world_size()
        self.dist.all_gather_object(out, [float(x) for x in xs])
        return [x for part in out for x in part]

    def close(self):
        if self.group is not None:
            self.group.close()
        if self.dist is not None:
            self.dist.destroy_process_group()


def launcher_name():
    if os.environ.get("IRIS_BENCH_LAUNCHER"):
        return "bench.py (torch.distributed.run child)"
    return "torch.distributed.run" if "WORLD_SIZE" in os.environ else "none"


def dry_run(args, ranks):
    """No GPU: each rank contributes a synthetic shard result (equal distances, so the
    lowest global index — rank 0's — must win the merge, src/main.rs:616-621)."""
    import iris_dist

    n = args.n_per_gpu or 10_000_000
    t0 = time.perf_counter()
    local = ih.Match(0.25, ranks.rank * n + 7, 10, 40, -3, 0)
    merged = iris_dist.allgather_merge(local) if ranks.dist is not None else local
    elapsed = ranks.max_over_ranks(time.perf_counter() - t0)
    # the per-rank gather the real line uses for every GPU's kernel time (kernel.per_rank_kernel_ms)
    gathered = [int(x) for x in ranks.gather_lists([ranks.rank])]
    ok = merged.index == 7 and merged.distance == 0.25 and gathered == list(range(ranks.world))
    if ranks.rank == 0:
        print(json.dumps({"metric": METRIC, "value": None, "unit": "template comparisons/s", "n_gpus": ranks.world,
                          "ranks_seen": ranks.world, "backend": ranks.backend, "launcher": launcher_name(),
                          "dry_run": True, "steps": 0, "warmup": 0, "ms_per_step": elapsed * 1e3,
                          "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": None,
                          "data": "none (dry run)",
                          "config": {"workload": "launcher rehearsal", "templates_per_gpu": n},
                          "check": {"merged_index": int(merged.index), "gathered_ranks": gathered,
                                    "ok": bool(ok)}}))
    ranks.close()
    if not ok:
        sys.exit(3)


# ---------------------------------------------------------------------------- single-GPU lines


def run_aux(args, dev):
    """Single-GPU lines for the §8(f) workloads beside the hot path: the fused
    resolver (share sum + decode + argmin), GPU share preparation, file loading,
    the host-slice engine calls and configs[0]'s criterion shapes."""
    P = args.parties
    rng = np.random.default_rng(SEED)
    ptrs = []
    extra = {}
    if args.workload in ("resolver", "host-resolver"):
        n = args.n_per_gpu
        shares = rng.integers(0, 65536, (P, n, ROT), dtype=np.uint16)
        denoms = rng.integers(0, 12801, (n, ROT), dtype=np.uint16)
        if args.workload == "resolver":
            for j in range(P + 1):
                ptrs.append(dev.alloc(n * ROT * 2))
                dev.h2d(ptrs[j], shares[j] if j < P else denoms)

            def step():
                return ih.resolver_search_device(dev, ptrs[:P], ptrs[P], n)
        else:
            host_parts = list(shares)

            def step():  # the rows in host memory, as they arrive from the participants
                return ih.resolver_search(host_parts, denoms, device=dev)

        kname, unit = "resolver", "records/s"
        rec_bytes = (P + 1) * ROT * 2  # P share rows + the denominator row, read once
        workload = (f"resolver: {P} participants' [u16;31] outputs + denominators -> min/argmin (src/main.rs:597-621)"
                    + (", host arrays: pinned-slot uploads overlapped with the kernels (PCIe-inclusive)"
                       if args.workload == "host-resolver" else ""))
    elif args.workload in ("resolve-masks", "host-resolve-masks"):
        n = args.n_per_gpu
        shares = rng.integers(0, 65536, (P, n, ROT), dtype=np.uint16)
        host_form = args.workload == "host-resolve-masks"
        if not host_form:
            for j in range(P):
                ptrs.append(dev.alloc(n * ROT * 2))
                dev.h2d(ptrs[j], shares[j])
        mdb = ih.Database(dev, ih.KIND_MASKS, n)
        mdb.generate(n, SEED)
        qmask = gen_records(dev, ih.KIND_MASKS, 1, SEED + 1)[0]
        eng = ih.MasksEngine(dev, qmask)
        host_parts = list(shares)

        def step():  # host form: the rows in host memory as they arrive, summed there, the sum uploaded
            return eng.resolve(mdb, host_parts if host_form else ptrs[:P])

        kname, unit = "masks_resolve", "records/s"
        rec_bytes = 1600 + P * ROT * 2  # the mask + P share rows; no denominators in memory
        workload = (f"resolver step with on-the-fly denominators: masks DB + {P} participants' [u16;31] "
                    "outputs -> min/argmin (src/main.rs:510-519 + 597-621)"
                    + (", the outputs in host memory: summed on the host, the sum uploaded (PCIe-inclusive)"
                       if host_form else ""))
    elif args.workload == "load":
        n = min(args.n_per_gpu, 1_000_000)  # a 3.2 GB file
        fpath = pathlib.Path(tempfile.gettempdir()) / f"iris_bench_{os.getpid()}.templates"
        src = ih.Database(dev, ih.KIND_TEMPLATES, n)
        src.generate(n, SEED)
        src.save_file(fpath)  # also leaves the file in the page cache
        tdb = ih.Database(dev, ih.KIND_TEMPLATES, n)

        def step():
            tdb.truncate(0)
            return tdb.load_file(fpath)

        kname, unit = "pack", "templates/s"
        rec_bytes = 2 * 3200  # the transpose kernel: reference layout in, TILES out
        workload = "raw template file (page cache) -> DMA from registered page-cache windows -> TILES transpose (src/main.rs:386-400)"
    elif args.workload in ("host-shares", "host-masks"):
        shares_wl = args.workload == "host-shares"
        kind = ih.KIND_SHARES if shares_wl else ih.KIND_MASKS
        rec_size = 25600 if shares_wl else 1600
        file_walk = args.mmap and not args.attached
        if file_walk:
            # the participant / resolver walk their whole file per request (src/main.rs:426-431,
            # 511-516; "3 million entries", specification.ipynb:173): 1M shares (25.6 GB) / 3M masks
            # (4.8 GB) by default, fewer only if the temp directory's file system has no room for them
            n = args.n_per_gpu if args.n_explicit else (1_000_000 if shares_wl else 3_000_000)
            import shutil
            room = shutil.disk_usage(tempfile.gettempdir()).free - (4 << 30)
            if n * rec_size > room:
                n = max(20_000, room // rec_size // 20_000 * 20_000)
                extra["file_records_reduced_to_fit"] = {"free_bytes": room + (4 << 30), "records": n}
        else:
            n = min(args.n_per_gpu, 200_000 if shares_wl else 2_000_000)  # 5.1 GB / 3.2 GB of host records
        qt = gen_records(dev, ih.KIND_TEMPLATES, 1, SEED + 1)[0]
        # one engine per walk, as the participant and the resolver build one per request
        # (src/main.rs:427, 512): no walk is served from rows an earlier walk computed
        dt, width = (np.uint16, 12800) if shares_wl else (np.uint64, 200)
        if shares_wl:
            qenc = ih.encode(ih.Template.from_array(qt))

            def new_engine():
                return ih.DistanceEngine(dev, qenc)
        else:
            def new_engine():
                return ih.MasksEngine(dev, qt[200:])
        mpath = None
        if args.mmap:  # the record file the participant / resolver maps (page-cached after the write)
            # written from the on-device generator 1 GB at a time (uniform u16 shares / mask bits)
            mpath = pathlib.Path(tempfile.gettempdir()) / f"iris_bench_{os.getpid()}.records"
            t_gen = time.perf_counter()
            per = max(1, (1 << 30) // rec_size)
            with ih.Database(dev, kind, min(n, per)) as g, open(mpath, "wb") as f:
                for a in range(0, n, per):
                    m = min(per, n - a)
                    g.truncate(0)
                    g.generate(m, SEED, global_index0=a)
                    g.read(0, m).tofile(f)
            extra["file"] = {"records": n, "bytes": n * rec_size, "write_s": time.perf_counter() - t_gen}
            host = np.memmap(mpath, dtype=dt, mode="r", shape=(n, width))
        elif shares_wl:
            host = rng.integers(0, 65536, (n, 12800), dtype=np.uint16)
        else:
            host = gen_records(dev, ih.KIND_MASKS, n, SEED)
        hout = np.empty((n, ROT), np.uint16)
        chunk = args.chunk or (20_000 if (args.attached or args.mmap) else n)
        adb = None
        if args.mmap:
            # the first walk makes the file resident (granule uploads): timed apart from the steps
            t_first = time.perf_counter()
            with new_engine() as eng:
                for a in range(0, n, chunk):
                    eng.batch_process(hout[a:a + chunk], host[a:a + chunk])
            extra["first_walk_s"] = time.perf_counter() - t_first
            extra["resident"] = dict(zip(("count", "bytes"), dev.resident()))
        extra["host_pages_numa"] = {"pages_by_node": pages_nodes(host), "gpu_node": dev.config().get("numa_node")}
        extra["copy_helpers"] = int(dev.config().get("copy_helpers", 0))  # copy-out threads besides the caller
        if args.attached:  # the mmap'd file's device copy (iris_db_attach_host), made once
            adb = ih.Database(dev, kind, n)
            t_att = time.perf_counter()
            adb.attach_host(host)
            extra["attach_s"] = time.perf_counter() - t_att

        first_calls = []  # engine creation + the walk's first call (a request's first rows)

        def step():
            t1 = time.perf_counter()
            with new_engine() as eng:
                eng.batch_process(hout[0:chunk], host[0:chunk])
                first_calls.append(time.perf_counter() - t1)
                for a in range(chunk, n, chunk):
                    eng.batch_process(hout[a:a + chunk], host[a:a + chunk])

        kname, unit = ("shares" if shares_wl else "masks"), "records/s"
        rec_bytes = host.shape[1] * host.itemsize
        workload = (f"{'DistanceEngine' if shares_wl else 'MasksEngine'}::batch_process(out, db: &[T]) over host "
                    f"slices of {chunk} records (src/lib.rs:42-52, 69-79; the participant / resolver loop of "
                    "src/main.rs:426-431, 511-516): "
                    + "one engine per walk (per request, src/main.rs:427, 512); "
                    + ("the host array is attached to its resident copy (iris_db_attach_host): no upload"
                       if args.attached else
                       ("slices of a read-only file mapping, no attach call: "
                        + ("IRIS_AUTO_RESIDENT=0, every slice uploaded (PCIe-inclusive)" if args.no_auto_resident
                           else "served from the library's resident copy of the file (made by an untimed first "
                                "walk, first_walk_s), re-validated on every call"))
                       if args.mmap else
                       "H2D of the pageable slice (runtime-staged) + TILES pack per 256-MB chunk, then the "
                       "engine kernel; PCIe-inclusive"))
    elif args.workload == "criterion":
        # configs[0]: 1 query x 31 x 10k templates (resident), plus the arch shapes below
        n = min(args.n_per_gpu, 10_000)
        tdb = ih.Database(dev, ih.KIND_TEMPLATES, n)
        tdb.generate(n, SEED)
        query = gen_records(dev, ih.KIND_TEMPLATES, 1, SEED + 1)[0]
        plant = plant_sites(n, 1)[0]
        tdb.write(plant, planted_record(query, 9)[None, :])
        eng = ih.TemplateEngine(dev, query)

        def step():
            return eng.search(tdb)

        kname, unit = "template_search", "template comparisons/s"
        rec_bytes = 3200
        workload = ("configs[0]: 1 query x 31 rotations x 10k templates (cache-resident: plumbing, no roofline "
                    "claim) + the criterion shapes of src/arch/mod.rs:22-72 through iris_dot_*_batch (host arrays)")
        shapes = {}
        for name, fn, shp, words, dt in (
                ("dot_bool", ih.dot_bool_batch, [(1, 1), (1, 1000), (31, 1000), (1, 100_000)], 200, np.uint64),
                ("dot_u16", ih.dot_u16_batch, [(1, 1), (1, 1000), (31, 1000), (1, 100_000), (31, 100_000)], 12800,
                 np.uint16)):
            for a, b in shp:
                av = rng.integers(0, np.iinfo(dt).max, (a, words), dtype=dt)
                bv = rng.integers(0, np.iinfo(dt).max, (b, words), dtype=dt)
                fn(av, bv, dev)
                p, tt = _time_passes(lambda: fn(av, bv, dev), 0.3, 200)
                shapes[f"{name}/{a * b}"] = a * b * p / tt
        extra["criterion_elements_per_s"] = shapes
        extra["criterion_note"] = "all-pairs calls with host arrays in and out (PCIe and launch included)"
    else:
        n = min(args.n_per_gpu, 1_000_000)  # 3 share DBs of 1M = 77 GB
        tdb = ih.Database(dev, ih.KIND_TEMPLATES, n)
        tdb.generate(n, SEED)
        sdbs = [ih.Database(dev, ih.KIND_SHARES, n) for _ in range(P)]
        mdb = ih.Database(dev, ih.KIND_MASKS, n)
        key = bytes(range(32))

        def step():
            for db in sdbs + [mdb]:
                db.truncate(0)
            ih.prepare_shares(tdb, sdbs, mdb, key=key, rounds=args.rounds)

        kname, unit = "prepare", "templates/s"
        rec_bytes = 3200 + P * 25600  # template in, P shares out (the prepare kernel)
        workload = (f"prepare: EncodedBits::share({P}) of encode(t) + masks, ChaCha{args.rounds} counter mode "
                    "(src/main.rs:333-361)")
    t_pre = time.perf_counter()  # untimed pre-warm, as in main()
    while time.perf_counter() - t_pre < args.prewarm_s:
        step()
    for _ in range(args.warmup):
        m = step()
    # host-slice lines: their steps are timed without the HIP timing events (which slow the
    # read-ahead's cross-stream hand-off several-fold, profiles/r03_readahead.txt) and the kernel
    # times come from a separate profiled pass of the same steps; every other line times its
    # steps with the events on
    separate = args.workload in ("host-shares", "host-masks")
    dev.reset_stats()
    dev.set_profiling(not separate)
    dev.synchronize()
    if separate:
        first_calls.clear()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        m = step()
    dev.synchronize()
    elapsed = time.perf_counter() - t0
    if separate:
        fc = sorted(first_calls)
        extra["first_call_ms"] = {"median": fc[len(fc) // 2] * 1e3, "max": fc[-1] * 1e3,
                                  "is": "engine creation + the walk's first batch_process call, timed steps"}
        dev.reset_stats()
        dev.set_profiling(True)
        for _ in range(args.steps):
            step()
        dev.synchronize()
        extra["kernel_times_from"] = "a separate profiled pass of the same steps (the timed steps run unprofiled)"
        ra = [int(x) for x in dev.config().get("readahead_windows", "0/0/0").split("/")]
        walk_stats = dev.kernel_stats(kname)
        # the walk's largest window as one launch on its own (in the walk, consecutive windows run on
        # two side streams and overlap, so their event times are not per-kernel durations): the same
        # engine kernel over that many resident records, [u16;31] rows to HBM
        big = ra[2]
        alone = None
        if big:
            with ih.Database(dev, kind, big) as bdb:
                bdb.generate(big, SEED + 3)
                bout = dev.alloc(big * ROT * 2)
                try:
                    with new_engine() as beng:
                        beng.batch_process_device(bdb, bout, 0, big)
                        dev.synchronize()
                        dev.reset_stats()
                        dev.set_profiling(True)
                        for _ in range(5):
                            beng.batch_process_device(bdb, bout, 0, big)
                        dev.synchronize()
                        dev.set_profiling(False)
                finally:
                    dev.free(bout)
            bl, bms, _ = dev.kernel_stats("shares" if shares_wl else "masks")
            bms /= max(1, bl)
            alone = {"records": big, "kernel_ms": bms,
                     "hbm_frac": big * rec_bytes / (bms * 1e-3) / 1e9 / HBM_PEAK_GBS if bms else None,
                     "is": "the largest window's size as one device-output launch on its own, 5 launches"}
        extra["readahead"] = {
            "launches_per_walk": ra[0] / args.steps, "records_computed_per_walk": ra[1] / args.steps,
            "largest_window_records": ra[2],
            "largest_window_kernel_alone": alone,
            "windows": "1, 2, 4, ... chunks up to 160 000 records, alternating between two side streams",
            "rows_over_host_link": ("packed: 32 B per record (base + 31 byte offsets, full-row escape)"
                                    if not shares_wl else "[u16;31]: 62 B per record")}
    dev.set_profiling(False)
    launches, kms, items = walk_stats if separate else dev.kernel_stats(kname)
    achieved = rec_bytes * items / (kms * 1e-3) / 1e9
    if separate:
        # host-slice walks: end to end, the records' bytes over the walk's wall time (their windows'
        # kernels overlap on two side streams, so summed kernel times are not a duration)
        achieved = rec_bytes * n * args.steps / elapsed / 1e9
        extra["roofline_is"] = "end to end: the walked records' bytes / the timed walks' wall time"
        if args.mmap or args.attached:
            # the rows crossing the host link (kernel stores into pinned memory): packed masks rows
            # 32 B per record, shares rows 62 B; against the measured device -> pinned-host rate of
            # kernel stores at window sizes (53.1 GB/s for 5 MB, profiles/r06h_ubench_d2h.txt)
            row_bytes = 62 if shares_wl else 32
            link = row_bytes * n * args.steps / elapsed / 1e9
            extra["host_link"] = {"row_bytes_per_record": row_bytes, "achieved_GBps": link,
                                  "measured_GBps": 53.1, "frac": link / 53.1,
                                  "source": "tools/ubench_d2h.hip (profiles/r06h_ubench_d2h.txt)"}
    if args.workload in ("resolve-masks", "host-resolve-masks"):  # denominators from the (separately checked) masks engine
        denoms = np.empty((n, ROT), np.uint16)
        eng.batch_process(denoms, mdb)
        sample = np.random.default_rng(1).choice(n, 64, replace=False)
        recs = np.stack([mdb.read(int(i), 1)[0] for i in sample])
        assert (denoms[sample] == check_masks_rows(qmask, recs)).all()
    if args.workload in ("resolver", "host-resolver", "resolve-masks", "host-resolve-masks"):
        best, idx = check_resolver(shares, denoms)
        ok = m.index == idx and np.float64(m.distance).view(np.uint64) == np.float64(best).view(np.uint64)
        check = {"expected_index": int(idx), "found_index": int(m.index), "ok": bool(ok)}
    elif args.workload in ("host-shares", "host-masks"):
        if args.attached:  # the same chunks through the resident calls, for comparison
            hdev = dev.alloc(chunk * ROT * 2)
            res = {}
            def walk_db(form):
                with new_engine() as eng:
                    for a in range(0, n, chunk):
                        if form == "host_out":
                            eng.batch_process(hout[a:a + chunk], adb, first=a, n=min(chunk, n - a))
                        else:
                            eng.batch_process_device(adb, hdev, first=a, n=min(chunk, n - a))

            for form in ("host_out", "device_out"):
                for _ in range(2):
                    walk_db(form)
                dev.synchronize()
                tr = time.perf_counter()
                for _ in range(args.steps):
                    walk_db(form)
                dev.synchronize()
                res[form + "_records_per_s"] = n * args.steps / (time.perf_counter() - tr)
            dev.free(hdev)
            res["attached_vs_device_out"] = (n * args.steps / elapsed) / res["device_out_records_per_s"]
            res["attached_vs_host_out"] = (n * args.steps / elapsed) / res["host_out_records_per_s"]
            extra["resident_same_chunks"] = res
        sample = np.random.default_rng(2).choice(n, 16, replace=False)
        want = (check_shares_rows(ih.encode(ih.Template.from_array(qt)).values, host[sample])
                if args.workload == "host-shares" else check_masks_rows(qt[200:], host[sample]))
        ok = bool((hout[sample] == want).all())
        check = {"sampled_outputs_checked": len(sample), "ok": ok}
        if file_walk:  # the same walk of the same file from C++, no Python between the calls
            extra["cxx_walk"] = cxx_walk(shares_wl, n, mpath)
        if mpath is not None:
            del host
            mpath.unlink()
    elif args.workload == "load":
        sample = [0, n // 3, n - 1]
        ok = m == n and all((tdb.read(i, 1) == src.read(i, 1)).all() for i in sample)
        fpath.unlink()
        check = {"sampled_templates_vs_source": len(sample), "ok": bool(ok)}
    elif args.workload == "criterion":
        ok = m.index == plant and m.rotation == 9
        check = {"planted_index": plant, "found_index": int(m.index), "rotation": int(m.rotation), "ok": bool(ok)}
    else:  # EncodedBits::share identity: the shares sum to encode(template); masks copied
        sample = [0, n // 3, n - 1]
        ok = True
        for i in sample:
            t = tdb.read(i, 1)[0]
            total = np.add.reduce(np.stack([sdbs[j].read(i, 1)[0] for j in range(P)]), axis=0, dtype=np.uint16)
            ok &= bool((total == ih.encode(ih.Template.from_array(t)).values).all())
            ok &= bool((mdb.read(i, 1)[0] == t[200:]).all())
        check = {"sampled_templates_share_identity": len(sample), "ok": bool(ok)}
    cpu = None
    if not args.no_cpu_baseline:
        try:
            cpu = cpu_baseline(args)
        except Exception as ex:  # reported, never fatal
            cpu = {"value": None, "error": str(ex)}
    per_unit = ROT if args.workload == "criterion" else 1
    line = {
        "metric": {"resolver": "resolver records/s (share sum + decode + argmin)",
                   "host-resolver": "resolver records/s over host arrays (share sum + decode + argmin, PCIe-inclusive)",
                   "resolve-masks": "resolver records/s (masks engine + share sum + decode + argmin, fused)",
                   "host-resolve-masks": "resolver records/s (masks engine + decode + argmin fused; shares from host memory, PCIe-inclusive)",
                   "prepare": "templates prepared/s (shares + masks)",
                   "load": "templates loaded/s (file -> resident database, PCIe-inclusive)",
                   "host-shares": "share records/s through batch_process over host slices (PCIe-inclusive)",
                   "host-masks": "mask records/s through batch_process over host slices (PCIe-inclusive)",
                   "criterion": METRIC}[args.workload],
        "value": per_unit * n * args.steps / elapsed, "unit": unit, "n_gpus": 1, "ranks_seen": 1, "backend": None,
        "launcher": launcher_name(), "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": elapsed / args.steps * 1e3, "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None,
        "dtype": {"resolver": "u16 (wrapping share sums) -> u32 cross-multiplied fractions",
                  "host-resolver": "u16 (wrapping share sums) -> u32 cross-multiplied fractions",
                  "resolve-masks": "fp4 e2m1 MFMA -> f32 denominators, u16 share sums",
                  "host-resolve-masks": "fp4 e2m1 MFMA -> f32 denominators, u16 share sums",
                  "prepare": "u32 (ChaCha keystream) -> u16 shares",
                  "load": "u8 (record bytes)",
                  "host-shares": "i8 MFMA -> i32 (u16 shares as biased byte planes)",
                  "host-masks": "fp4 e2m1 MFMA -> f32 (0/1 products)",
                  "criterion": "fp4 e2m1 MFMA -> f32 (0/+-1 products)"}[args.workload],
        "data": "synthetic (uniform random u16 / on-device generated templates)",
        "config": {"workload": workload, "records_per_gpu": n, "parties": P,
                   **({"chunk": chunk, "attached": bool(args.attached), "mmap": bool(args.mmap),
                       "auto_resident": not args.no_auto_resident}
                      if args.workload in ("host-shares", "host-masks") else {})},
        "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": achieved / HBM_PEAK_GBS,
                     "traffic": load_traffic(args.workload, n, "tiles")[0]
                     if args.workload in ("resolver", "resolve-masks") else None,
                     "traffic_source": "committed PMC bytes per record (profiles/), scaled to this launch"
                     if args.workload in ("resolver", "resolve-masks") else None},
        "kernel": {"name": kname, "avg_ms": kms / max(1, launches), "launches": launches,
                   "bytes_per_record": rec_bytes},
        "file_GBps": (n * 3200 * args.steps / elapsed / 1e9) if args.workload == "load" else None,
        "host_input_GBps": (n * rec_bytes * args.steps / elapsed / 1e9)
        if (args.workload in ("host-shares", "host-masks") and not args.attached
            and not (args.mmap and not args.no_auto_resident)) or args.workload == "host-resolver"
        else (n * P * ROT * 2 * args.steps / elapsed / 1e9) if args.workload == "host-resolve-masks" else None,
        "cpu_baseline": cpu,
        "check": check,
        **extra,
    }
    print(json.dumps(line))
    for p in ptrs:
        dev.free(p)
    if not ok:
        print("result check failed", file=sys.stderr)
        sys.exit(3)


def main():
    args = parse()
    if args.gpus < 1:
        raise SystemExit("error: --gpus must be >= 1")
    if "WORLD_SIZE" not in os.environ and args.gpus > 1 and not args.single_process:
        sys.exit(launch_ranks(args))
    ranks = Ranks(args)
    if args.dry_run:
        return dry_run(args, ranks)
    world_gpus = args.gpus  # GPUs in the run (ranks x 1, or one process x --gpus)
    rank = ranks.rank
    args.n_explicit = args.n_per_gpu is not None
    if args.n_per_gpu is None:  # configs[1] at N=1; configs[4] (100M over 8 GPUs) at N=8
        args.n_per_gpu = 12_500_000 if (args.workload == "search" and world_gpus > 1) else 10_000_000
    n = args.n_per_gpu
    total = n * world_gpus
    if args.workload in AUX_WORKLOADS:
        if world_gpus > 1:
            raise SystemExit(f"workload {args.workload} is a single-GPU line (run without --gpus / torchrun)")
        if args.no_auto_resident:
            os.environ["IRIS_AUTO_RESIDENT"] = "0"  # read when the device opens
        return run_aux(args, ih.Device(0))
    if args.single_process and args.workload not in ("search", "batch"):
        raise SystemExit("--single-process runs the group search (--workload search / batch)")
    layout = {"tiles": ih.LAYOUT_TILES, "lanes": ih.LAYOUT_LANES}[args.layout]
    kind = {"search": ih.KIND_TEMPLATES, "batch": ih.KIND_TEMPLATES, "masks": ih.KIND_MASKS,
            "shares": ih.KIND_SHARES}[args.workload]
    nq = args.queries if args.workload == "batch" else 1

    # the library device group: the search / batch exchange of every multi-GPU run (RCCL)
    group = ranks.join_group(args) if args.workload in ("search", "batch") else None
    group_form_s = ranks.max_over_ranks(ranks.group_form_s) if ranks.group_form_s is not None else None
    if group is not None:
        devs = group.devices
    else:
        devs = [ih.Device(ranks.ordinal)]
    dev = devs[0]
    lo = rank * n  # this process's first global record (torchrun ranks; 0 for a single process)

    t0 = time.time()
    if group is not None:
        gdb = ih.GroupDatabase(group, kind, total, layout)
        gdb.generate(SEED)
        shards = [gdb.shard_db(i) for i in range(gdb.local_shards)]
        shard_lo = [gdb.shard(i)[0] for i in range(gdb.local_shards)]
    else:
        gdb = None
        db = ih.Database(dev, kind, n, layout)
        db.generate(n, SEED, global_index0=lo)
        shards, shard_lo = [db], [lo]
    gen_s = time.time() - t0

    query = gen_records(dev, ih.KIND_TEMPLATES, 1, SEED + 1)[0]
    out_dev = None
    # planted known answers: (query index, global index, rotation)
    plants = []
    if args.workload == "search":
        plants = [(0, plant_sites(total, 1)[0], 9)]
    elif args.workload == "batch":
        batch_q = gen_records(dev, ih.KIND_TEMPLATES, nq, SEED + 2)
        batch_q[nq // 2] = query
        pq = batch_plant_queries(nq)
        rots = [9, -15, 15, 0, -7]
        plants = [(q, site, rots[k % len(rots)]) for k, (q, site) in enumerate(zip(pq, plant_sites(total, len(pq))))]
    for q, site, r in plants:
        rec = planted_record(query if args.workload == "search" else batch_q[q], r)[None, :]
        if gdb is not None:
            gdb.write(site, rec)  # every rank writes the part it holds (SPMD)
        elif lo <= site < lo + n:
            db.write(site - lo, rec)
    if args.workload in ("masks", "shares"):
        out_dev = dev.alloc(n * ROT * 2)
    share_query = ih.encode(ih.Template.from_array(query)) if args.workload == "shares" else None

    def new_engine(d=dev):
        """The query's engine: its 31 rotations in the kernels' layouts, built on the device
        (DistanceEngine::new / MasksEngine::new, src/lib.rs:33-40, 60-67)."""
        if args.workload == "search":
            return ih.TemplateEngine(d, query)
        if args.workload == "batch":
            return ih.TemplateBatchEngine(d, batch_q)
        if args.workload == "masks":
            return ih.MasksEngine(d, query[200:])
        return ih.DistanceEngine(d, share_query)

    # by default every step prepares its query's engine and frees it again, as the reference's
    # participant does per request (src/main.rs:427-431); --reuse-engine keeps one engine (the
    # group search always builds its engines inside the step)
    eng = new_engine() if args.reuse_engine and group is None else None
    # IRIS_DIST_BACKEND=gloo: the search winners go through torch CPU tensors
    rehearsal = ranks.dist is not None and group is None and args.workload in ("search", "batch")
    if rehearsal:
        import iris_dist

    def sync_all():
        for d in devs:
            d.synchronize()
        ranks.barrier()
        for d in devs:
            d.synchronize()

    def local_step():
        """This process's shards searched with no exchange (the pre-warm: ranks run
        different numbers of these, so no collective may be inside)."""
        if args.workload in ("search", "batch") and group is not None:
            engs = [new_engine(s.device) for s in shards]
            try:
                if args.workload == "search":
                    pend = [e.search_async(s, index_base=b) for e, s, b in zip(engs, shards, shard_lo)]
                    for p in pend:
                        p.wait()
                else:
                    for e, s, b in zip(engs, shards, shard_lo):
                        e.search(s, index_base=b)
            finally:
                for e in engs:
                    e.close()
            return
        step(exchange=False)

    def step(exchange=True):
        if group is not None:
            return gdb.search(query) if args.workload == "search" else gdb.batch_search(batch_q)
        e = eng if eng is not None else new_engine()
        try:
            if args.workload == "batch":
                ms = e.search(db, index_base=lo)
                return iris_dist.allgather_merge_many(ms) if rehearsal and exchange else ms
            if args.workload != "search":
                e.batch_process_device(db, out_dev, 0, n)  # [n][31] u16 left in HBM (n known, as out.len())
                return None
            m = e.search(db, 0, n, index_base=lo)
            return iris_dist.allgather_merge(m) if rehearsal and exchange else m
        finally:
            if eng is None:
                e.close()

    pipelined = args.workload == "search" and not args.no_pipeline

    def run_steps(k):
        """k steps; pipelined: step i+1's search (engines, kernels and — in a group — the
        RCCL all-gather and merge) is enqueued before step i's result is waited for, so the
        host work and the exchange overlap the next kernel.  Every step's search runs to
        completion and every result is exchanged and merged inside the call."""
        if not pipelined:
            m = None
            for _ in range(k):
                m = step()
            return m

        def finish(p):
            m = p.wait()
            return iris_dist.allgather_merge(m) if rehearsal else m

        pend, m = None, None
        for _ in range(k):
            if group is not None:
                p = gdb.search_async(query)
            else:
                e = eng if eng is not None else new_engine()
                p = e.search_async(db, index_base=lo)
                if eng is None:
                    e.close()
            if pend is not None:
                m = finish(pend)
            pend = p
        return finish(pend) if pend is not None else m

    # the CPU baseline (rank 0 of a one-GPU run): measured on its own, before any GPU step,
    # on every CPU the process may use (not beside the GPU-driving loop)
    cpu = None
    if rank == 0 and world_gpus == 1 and not args.no_cpu_baseline:
        try:
            cpu = cpu_baseline(args)
        except Exception as ex:  # reported, never fatal
            cpu = {"value": None, "error": str(ex)}
    # pre-warm: the GPU needs ~0.5-1 s of sustained streaming before the search reaches its
    # steady rate (tools/engine_variance.py: the first ~100 searches of a process run up to 4 %
    # slower, then settle); untimed, like the warmup steps, and reported under "setup"
    t_pre = time.perf_counter()
    prewarm_steps = 0
    while time.perf_counter() - t_pre < args.prewarm_s:
        local_step()
        prewarm_steps += 1
    prewarm_s = time.perf_counter() - t_pre
    if args.warmup:
        m = run_steps(args.warmup)
    for d in devs:
        d.reset_stats()
        d.set_profiling(True)
    sync_all()
    t0 = time.perf_counter()
    m = run_steps(args.steps)
    sync_all()
    elapsed = time.perf_counter() - t0
    for d in devs:
        d.set_profiling(False)
    elapsed = ranks.max_over_ranks(elapsed)
    # participant-sized steps (tens of us): the HIP timing events around every launch are part of
    # the timed region above, as the roofline needs; the same number of steps is timed once more
    # without them, which is the wall time a caller sees per call
    unprofiled_ms = None
    if elapsed / args.steps < 1e-3:
        sync_all()
        t1 = time.perf_counter()
        run_steps(args.steps)
        sync_all()
        unprofiled_ms = ranks.max_over_ranks(time.perf_counter() - t1) / args.steps * 1e3

    kname = {"search": "template_search", "batch": "template_batch", "masks": "masks", "shares": "shares"}[args.workload]
    rec_bytes = {"search": BYTES_PER_TEMPLATE,
                 "batch": BYTES_PER_TEMPLATE, "masks": 1600, "shares": 25600}[args.workload]
    if args.workload in ("search", "batch"):
        results = [m] if args.workload == "search" else m
        found = [{"query": q, "planted_index": site, "found_index": int(results[q].index),
                  "rotation": int(results[q].rotation), "planted_rotation": r,
                  "distance": results[q].distance} for q, site, r in plants]
        ok = all(f["found_index"] == f["planted_index"] and f["rotation"] == f["planted_rotation"] for f in found)
        check = ({**found[0], "ok": bool(ok)} if args.workload == "search"
                 else {"planted_queries": found, "query_groups": sorted({f["query"] // 4 for f in found}),
                       "ok": bool(ok)})
        if args.workload == "batch":
            m = results[plants[0][0]]
    else:  # spot-check 64 outputs
        sample = np.random.default_rng(0).choice(n, 64, replace=False)
        full = np.empty((n, ROT), np.uint16)
        dev.d2h(full, out_dev)
        recs = np.stack([db.read(int(i), 1)[0] for i in sample])
        want = (check_masks_rows(query[200:], recs) if args.workload == "masks"
                else check_shares_rows(ih.encode(ih.Template.from_array(query)).values, recs))
        ok = bool((full[sample] == want).all())
        check = {"sampled_outputs_checked": 64, "ok": bool(ok)}
        del full
    # kernel time per launch: averaged over this process's devices (each searches its own shards)
    stats = [d.kernel_stats(kname) for d in devs]
    if sum(s[0] for s in stats) == 0 and args.workload == "batch":  # a 1-3 query batch streams
        stats = [d.kernel_stats("template_search") for d in devs]
    launches = sum(s[0] for s in stats)
    kms = sum(s[1] for s in stats)
    rms = sum(d.kernel_stats("reduce")[1] for d in devs)
    per_dev_ms = [s[1] / max(1, s[0]) for s in stats]
    # every GPU's average kernel time, in rank order (torchrun ranks gather theirs; a single
    # process holds all of its devices'): the roofline is the SLOWEST GPU's, which sets the step
    per_gpu_ms = ranks.gather_lists(per_dev_ms)
    per_gpu_step_ms = ranks.gather_lists([s[1] / max(1, args.steps) for s in stats])
    avg_ms = max(per_gpu_ms) if per_gpu_ms else kms / max(1, launches)
    n_launch = total // world_gpus  # records per launch (one shard per device)
    # kernel time of one step on the slowest device (a batch of 1-3 queries streams: several launches per step)
    step_kernel_ms = max(per_gpu_step_ms) if per_gpu_step_ms else kms / max(1, len(devs)) / max(1, args.steps)
    achieved = rec_bytes * n_launch / (avg_ms * 1e-3) / 1e9
    # batch: bytes fetched beyond L2 per 1024-query launch, from the SAME committed PMC run as
    # kernel.pmc (the template DB about once per XCD + the query tiles re-streamed from the MALL)
    bpmc = batch_pmc() if args.workload == "batch" and nq == 1024 else None
    if args.workload != "batch":
        traffic, traffic_src = load_traffic(args.workload, n_launch, args.layout)
    else:
        traffic, traffic_src = ((bpmc["beyond_l2_bytes_per_launch"], bpmc["source"].split(" ")[0][len("profiles/"):])
                                if bpmc else (None, None))
    ms_per_step = elapsed / args.steps * 1e3
    value = ROT * total * nq / (elapsed / args.steps)
    mfma_frac = MFMA_MACS_PER_TEMPLATE * n_launch * nq / (step_kernel_ms * 1e-3) / FP4_DENSE_PEAK_MACS

    if rank == 0:
        line = {
            "metric": METRIC,
            "value": value,
            "unit": "template comparisons/s",
            "value_per_gpu": value / world_gpus,
            "n_gpus": world_gpus,
            "ranks_seen": ranks.dist.get_world_size() if ranks.dist is not None else 1,
            # what the library's RCCL communicator itself reports (ncclCommCount, and every rank's
            # device PCI bus id gathered over that communicator), not torch's view
            "rccl_nranks": group.rccl_nranks if group is not None else None,
            "rccl_devices": group.rccl_devices if group is not None else None,
            "group_form_s": group_form_s,
            **({"rccl_error": ranks.rccl_error} if ranks.rccl_error else {}),
            "rccl_init_timeout_ms": (int(dev.config()["group_init_timeout_ms"]) if group is not None else None),
            "processes": ranks.world,
            "backend": ranks.backend,
            "launcher": launcher_name() if not args.single_process else "none (one process, library device group)",
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": ms_per_step,
            **({"ms_per_step_unprofiled": unprofiled_ms} if unprofiled_ms is not None else {}),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            # the arithmetic the kernel computes in; every sum is an exact integer either way
            "dtype": {("shares", "tiles"): "i8 MFMA -> i32 (u16 shares as biased byte planes)",
                      ("shares", "lanes"): "u16 (v_pk_mad_u16)"}.get(
                          (args.workload, args.layout),
                          "fp4 e2m1 MFMA -> f32 (0/+-1 products)" if args.layout != "lanes" else "u32 (VALU popcount)"),
            "data": "synthetic (on-device counter-based generator, uniform random pattern+mask bits; planted known answer)",
            "config": {
                "workload": {
                    "search": "1 query x 31 rotations x N templates, Template masked Hamming + fused min/argmin (BASELINE configs[1] at N=1: 10M; 12.5M per GPU from 2 GPUs, configs[4] = 100M over 8 GPUs)",
                    "masks": "MasksEngine: 1 query mask x 31 rotations x N masks, [u16;31] denominators left in HBM",
                    "shares": "DistanceEngine: 1 encoded query x 31 rotations x N u16 shares, [u16;31] left in HBM (BASELINE configs[3])",
                    "batch": f"{nq} queries x 31 rotations x N templates in one pass, per-query min/argmin (BASELINE configs[2])",
                }[args.workload],
                "templates_per_gpu": n, "total_templates": total, "queries": nq, "rotations": ROT,
                "bytes_per_template": rec_bytes, "parallelism": f"db-shard x{world_gpus}", "layout": args.layout,
                "engine_per_step": not args.reuse_engine or group is not None,
                "pipelined": pipelined,
                "exchange": ("library RCCL all-gather of 24-B shard winners + on-device merge (iris_group_*)"
                             if group is not None else
                             "torch gloo all-gather of 32-B matches + iris_match_merge "
                             + ("(fallback)" if ranks.rccl_error else "(rehearsal)")
                             if rehearsal else None),
            },
            "roofline": ({
                "bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
                "traffic_source": ("committed PMC bytes per record (profiles/" + traffic_src + "), scaled to this launch")
                if traffic_src else None,
            } if args.workload != "batch" else {
                # compute-bound: fp4 MFMA FLOPs (2 per MAC) of the den + encode products, 31 rotation rows
                "bound": "mfma", "achieved": 2 * MFMA_MACS_PER_TEMPLATE * n_launch * nq / (step_kernel_ms * 1e-3) / 1e12,
                "peak": 2 * FP4_DENSE_PEAK_MACS / 1e12, "unit": "TFLOP/s",
                "frac": mfma_frac,
                "issued_frac": mfma_frac * MFMA_MACS_ISSUED_PER_TEMPLATE / MFMA_MACS_PER_TEMPLATE,
                "traffic": traffic,
                "traffic_source": ("committed PMC bytes per launch (profiles/" + traffic_src + ")")
                if traffic_src else None,
            }),
            "kernel": {
                "name": {("search", "tiles"): "template_mfma_kernel<MF_SEARCH> (fp4 MFMA)",
                         ("search", "lanes"): "template_kernel<MODE_SEARCH> (VALU popcount)",
                         ("masks", "tiles"): "masks_mfma_kernel (fp4 MFMA)",
                         ("masks", "lanes"): "masks_kernel (VALU popcount)",
                         ("shares", "tiles"): "shares_mfma_kernel (i8 MFMA)",
                         ("shares", "lanes"): "shares_kernel (VALU v_pk_mad_u16)",
                         ("batch", "tiles"): "batch_lds_kernel<8,2,2,2> (fp4 MFMA GEMM: 2-query groups x 16-tile N-groups, 2 x 2 per wave, LDS query-fragment ring)"}[(args.workload, args.layout)],
                "avg_ms": avg_ms, "avg_ms_is": "the slowest GPU's average (it sets the step)",
                "launches": launches, "per_device_avg_ms": per_dev_ms,
                "per_rank_kernel_ms": per_gpu_ms,
                "kernel_ms_min": min(per_gpu_ms) if per_gpu_ms else None,
                "kernel_ms_max": max(per_gpu_ms) if per_gpu_ms else None,
                "reduce_avg_ms": rms / max(1, launches),
                "frac_of_guide_copy_bw": achieved / HBM_GUIDE_COPY_GBS,
                "frac_of_read_ceiling": achieved / HBM_READ_CEILING_GBS,
                "valu_int_frac": (VALU_OPS_PER_TEMPLATE * n_launch / (avg_ms * 1e-3) / VALU_INT_PEAK_OPS
                                  if args.layout == "lanes" and args.workload == "search" else None),
                "mfma_fp4_frac": mfma_frac if args.layout != "lanes" and args.workload in ("search", "batch") else None,
                "traffic_note": ("FETCH_SIZE counts every L2 miss, Infinity-Cache hits included: the query tiles "
                                 "are re-streamed from the 256-MB MALL for each N-group, "
                                 "the template DB comes from HBM about once per XCD" if args.workload == "batch"
                                 else None),
                "pmc": bpmc,
            },
            "cpu_baseline": cpu,
            "check": check,
            "setup": {"generate_s": gen_s, "prewarm_s": prewarm_s, "prewarm_steps": prewarm_steps},
        }
        print(json.dumps(line))
    if out_dev is not None:
        dev.free(out_dev)
    if eng is not None:
        eng.close()
    if gdb is not None:
        gdb.close()
    else:
        db.close()
        dev.close()
    # the run is the claimed one only if RCCL saw --gpus ranks on as many distinct devices
    rccl_bad = None
    if group is not None:
        if group.rccl_nranks != world_gpus:
            rccl_bad = f"RCCL communicator holds {group.rccl_nranks} ranks, --gpus {world_gpus}"
        elif len(set(group.rccl_devices)) != len(group.rccl_devices):
            rccl_bad = f"two RCCL ranks on one device: {group.rccl_devices}"
    ranks.close()
    if not ok:
        print(f"result check failed: {check}", file=sys.stderr)
        sys.exit(3)
    if rccl_bad:
        print(f"RCCL check failed: {rccl_bad}", file=sys.stderr)
        sys.exit(4)


if __name__ == "__main__":
    main()
