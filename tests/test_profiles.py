"""CPU: the committed evidence.  Every bench.py line kept under profiles/ must carry a
passing result check (a failed known-answer check is never cited as a measurement), and
the headline lines must carry the contract's roofline and cpu_baseline objects."""
import json
import pathlib

ROOT = pathlib.Path(__file__).resolve().parents[1]


def _lines():
    for p in sorted((ROOT / "profiles").glob("*.jsonl")):
        for i, line in enumerate(p.read_text().splitlines()):
            if line.strip():
                yield p.name, i, json.loads(line)


def test_every_committed_bench_line_passed_its_check():
    n = 0
    for name, i, d in _lines():
        assert (d.get("check") or {}).get("ok") is True, f"{name}:{i + 1} {d.get('check')}"
        n += 1
    assert n > 10


def test_round2_headline_lines_carry_roofline_and_cpu_baseline():
    for tag in ("search", "shares", "batch", "masks"):
        p = ROOT / "profiles" / f"r02_bench_{tag}.jsonl"
        d = json.loads(p.read_text().splitlines()[-1])
        r = d["roofline"]
        assert r["bound"] in ("hbm", "mfma") and r["peak"] > 0 and abs(r["frac"] - r["achieved"] / r["peak"]) < 1e-9
        c = d["cpu_baseline"]
        assert c["value"] > 0 and c["cores"] >= 1 and c["kind"] in ("port", "reference")
