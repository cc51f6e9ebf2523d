"""Copy bench.py JSON lines from logs into a profiles/ file — only lines whose result
check passed.  Exits 1 (and writes nothing for that line) when a line's check failed or
is missing, so a failed known-answer check can never become committed evidence.

    python tools/keep_bench.py profiles/r02_bench_x.jsonl gpurun_out/a.log [more.log ...]
"""
import json
import pathlib
import sys


def main(argv):
    if len(argv) < 3:
        raise SystemExit(__doc__)
    dst = pathlib.Path(argv[1])
    kept, bad = [], 0
    for src in argv[2:]:
        for line in pathlib.Path(src).read_text().splitlines():
            if not line.startswith("{"):
                continue
            d = json.loads(line)
            if not (d.get("check") or {}).get("ok"):
                print(f"{src}: result check failed or missing, not kept: {d.get('check')}", file=sys.stderr)
                bad += 1
                continue
            kept.append(line)
    with dst.open("a") as f:
        for line in kept:
            f.write(line + "\n")
    print(f"kept {len(kept)} line(s) in {dst}, refused {bad}")
    return 1 if bad else 0


if __name__ == "__main__":
    sys.exit(main(sys.argv))
