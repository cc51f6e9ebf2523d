"""Round-4 configs[2] evidence from ONE box (tools/gpu_r04e.sh, gpurun_out/r04e): the FETCH_SIZE /
WRITE_SIZE passes, the three SQ passes (tools/pmc_batch.sh), rocprofv3 kernel stats and the package
power beside the batched kernel and beside the fp4 MFMA alone -> profiles/r04_pmc_batch.json and
profiles/r04_pmc_batch_sq.json (the same launch shape; bench.py reads roofline.traffic and kernel.pmc
from the latter, so both come from one run), profiles/r04_batch_energy.txt."""
import csv
import json
import pathlib
import re
import sys

ROOT = pathlib.Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "tools"))
import power_summary  # noqa: E402

R = ROOT / "gpurun_out" / "r04e"
K = "batch_lds_kernel"


def per_launch(d, name):
    by = {}
    for f in d.rglob("*counter_collection.csv"):
        for row in csv.DictReader(open(f)):
            if row["Counter_Name"] == name and K in row["Kernel_Name"]:
                by[row["Dispatch_Id"]] = by.get(row["Dispatch_Id"], 0.0) + float(row["Counter_Value"])
    big = [v for v in by.values() if v >= 0.5 * max(by.values())]
    return sum(big) / len(big), len(big)


def main():
    fetch, nf = per_launch(R / "pmc_FETCH_SIZE", "FETCH_SIZE")
    write, _ = per_launch(R / "pmc_WRITE_SIZE", "WRITE_SIZE")
    rd, wr = fetch * 1024 * 2, write * 1024
    n = 10_000_000
    stats = next((R / "prof").rglob("*kernel_stats.csv"))
    kms = next(float(r["AverageNs"]) / 1e6 for r in csv.DictReader(open(stats)) if K in r["Name"])
    sq = {}
    for line in open(R / "sq" / "summary.txt"):
        k, v = line.split()
        sq[k] = float(v)
    launches = nf  # one batched launch per SQ pass (bench --steps 1 --warmup 0)
    mfma, valu, lds = sq["SQ_INSTS_MFMA"], sq["SQ_INSTS_VALU"], sq["SQ_INSTS_LDS"]
    clock = sq["GRBM_GUI_ACTIVE"] / 8 / (kms * 1e-3) / 1e9
    cmd = "tools/gpu_r04e.sh (one box): rocprofv3 --pmc FETCH_SIZE | WRITE_SIZE | 3 SQ passes -- python3 bench.py --workload batch --queries 1024 --steps 1 --warmup 0 --prewarm-s 0"
    (ROOT / "profiles" / "r04_pmc_batch.json").write_text(json.dumps({
        "round": 4, "workload": "batch", "layout": "tiles", "kernel": K, "command": cmd,
        "n_records_per_launch": n, "FETCH_SIZE_kB_raw": fetch, "WRITE_SIZE_kB_raw": write,
        "correction": "read bytes = FETCH_SIZE*1024*2, write bytes = WRITE_SIZE*1024 (MI355X_MICROARCH.md §HBM)",
        "hbm_read_bytes_per_launch": rd, "hbm_write_bytes_per_launch": wr, "hbm_bytes_per_launch": rd + wr,
        "hbm_bytes_per_record": (rd + wr) / n, "algorithmic_bytes_per_record": 3200}, indent=1) + "\n")
    # energy per MFMA: package power x time / MFMAs, the batched kernel vs the MFMA alone
    pb, cb, nb = power_summary.steady(power_summary.samples(R / "batch.pwr"))
    pa, ca, na = power_summary.steady(power_summary.samples(R / "mfma_alone.pwr"))
    alone = open(R / "mfma_alone.txt").read()
    m = re.search(r"seconds ([\d.]+)\s+mfma ([\d.e+]+)", alone)
    ta, ma = float(m.group(1)), float(m.group(2))
    idle = float(re.search(r"SOCKET_POWER: (\d+) W", open(R / "idle.txt").read()).group(1))
    eb, ea = pb * kms * 1e-3 / mfma, pa * ta / ma
    db, da = (pb - idle) * kms * 1e-3 / mfma, (pa - idle) * ta / ma
    rate_alone = ma / ta
    (ROOT / "profiles" / "r04_pmc_batch_sq.json").write_text(json.dumps({
        "round": 4, "kernel": "batch_lds_kernel<8,2,2,2> (2-query groups x 16-tile N-groups, 2 queries x 2 tiles per wave)",
        "queries": 1024, "templates": n, "command": cmd, "launches_in_profile": launches,
        "per_launch": sq,
        "valu_per_mfma_incl_mfma": valu / mfma, "valu_per_mfma_excl_mfma": valu / mfma - 1,
        "lds_insts_per_mfma": lds / mfma, "lds_bank_conflict_cycles": sq["SQ_LDS_BANK_CONFLICT"],
        "beyond_l2_bytes_per_launch": rd + wr, "fetch_size_kb": fetch, "write_size_kb": write,
        "beyond_l2_source": "FETCH_SIZE x 1024 x 2 + WRITE_SIZE x 1024 (MI355X_MICROARCH.md HBM section), separate passes, same box and launch shape (profiles/r04_pmc_batch.json)",
        "kernel_avg_ms_rocprof_stats": kms, "kernel_stats": "profiles/r04_kernel_stats_batch.csv",
        "clock_ghz_from_grbm": clock,
        "mfma_cycles_per_mfma_per_simd": sq["SQ_VALU_MFMA_BUSY_CYCLES"] / 4 / mfma * 1.0,
        "energy": {"package_power_w_batch": pb, "package_power_w_mfma_alone": pa, "idle_w": idle,
                   "nj_per_mfma_batch": eb * 1e9, "nj_per_mfma_mfma_alone": ea * 1e9, "gap": eb / ea - 1,
                   "dynamic_nj_per_mfma_batch": db * 1e9, "dynamic_nj_per_mfma_mfma_alone": da * 1e9,
                   "dynamic_gap": db / da - 1,
                   "mfma_alone_rate_per_s": rate_alone, "batch_rate_vs_mfma_alone": mfma / (kms * 1e-3) / rate_alone,
                   "source": "profiles/r04_batch_energy.txt"}}, indent=1) + "\n")
    lines = [
        "# configs[2] energy per MFMA, one box (tools/gpu_r04e.sh, gpurun_out/r04e): package power (amd-smi metric, polled",
        "# ~0.35 s) while bench.py --workload batch --queries 1024 runs (4 steps) and while tools/ubench_mfma_power runs the",
        "# same fp4 MFMA alone (2 waves per SIMD, random operands of the kernel's nibble density) for 12 s.",
        f"idle package power: {idle:.0f} W",
        f"batch:      steady {nb} samples, median {pb:.0f} W; kernel {kms:.1f} ms (rocprof stats); {mfma:.4e} MFMA per launch (SQ_INSTS_MFMA)",
        f"mfma alone: steady {na} samples, median {pa:.0f} W; {ta:.3f} s, {ma:.4e} MFMA ({rate_alone:.4e} MFMA/s)",
        f"energy per MFMA (package):       batch {eb * 1e9:.2f} nJ, MFMA alone {ea * 1e9:.2f} nJ -> gap {100 * (eb / ea - 1):.1f} %",
        f"energy per MFMA (above idle):    batch {db * 1e9:.2f} nJ, MFMA alone {da * 1e9:.2f} nJ -> gap {100 * (db / da - 1):.1f} %",
        f"batch MFMA rate / MFMA-alone rate: {mfma / (kms * 1e-3) / rate_alone:.3f}; clock from GRBM_GUI_ACTIVE {clock:.2f} GHz",
        f"per MFMA: {valu / mfma - 1:.2f} VALU (excl. MFMA), {lds / mfma:.3f} LDS, {sq['SQ_INSTS_SALU'] / mfma:.2f} SALU, {sq['SQ_INSTS_VMEM'] / mfma:.3f} VMEM instructions",
        f"beyond L2 per launch: {(rd + wr) / 1e12:.2f} TB (FETCH_SIZE x 2 + WRITE_SIZE, same box)",
        "samples (time: package W / amd-smi mean GFX_0..7 CLK MHz -- the amd-smi clock field reads ~1.0 GHz here against",
        f"{clock:.2f} GHz from GRBM_GUI_ACTIVE per XCD, so the PMC clock is the one quoted):",
    ]
    for f in ("batch.pwr", "mfma_alone.pwr"):
        s = power_summary.samples(R / f)
        t0 = s[0][0]
        lines.append(f + ": " + " ".join(f"{t - t0:.1f}s:{p:.0f}W" for t, p, c in s))
    (ROOT / "profiles" / "r04_batch_energy.txt").write_text("\n".join(lines) + "\n")
    import shutil
    shutil.copy(stats, ROOT / "profiles" / "r04_kernel_stats_batch.csv")
    print("\n".join(lines[:12]))


if __name__ == "__main__":
    main()
