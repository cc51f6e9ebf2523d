"""Summarise `amd-smi metric -g 0 -p -c` samples polled beside a run (tools/gpu_r04e.sh): per file,
the samples (time, SOCKET_POWER, mean GFX clock) and the steady-state medians over the samples
within 15 % of the run's peak power.  usage: python tools/power_summary.py FILE.pwr ..."""
import re
import statistics
import sys


def samples(path):
    out, t, p, clks = [], None, None, []
    for line in open(path):
        if line.startswith("T "):
            if t is not None and p is not None:
                out.append((t, p, statistics.mean(clks) if clks else None))
            t, p, clks = float(line.split()[1]), None, []
        elif "SOCKET_POWER" in line:
            m = re.search(r"(\d+) W", line)
            p = float(m.group(1)) if m else None
        elif re.match(r"\s+CLK: \d+ MHz", line):
            clks.append(float(re.search(r"(\d+) MHz", line).group(1)))
    if t is not None and p is not None:
        out.append((t, p, statistics.mean(clks) if clks else None))
    return out


def steady(s):
    peak = max(p for _, p, _ in s)
    keep = [(p, c) for _, p, c in s if p >= 0.85 * peak]
    return statistics.median(p for p, _ in keep), statistics.median(c for _, c in keep if c), len(keep)


if __name__ == "__main__":
    for f in sys.argv[1:]:
        s = samples(f)
        t0 = s[0][0]
        print(f, " ".join(f"{t - t0:.1f}s:{p:.0f}W/{c:.0f}" for t, p, c in s))
        p, c, n = steady(s)
        print(f"  steady samples {n}: power median {p:.0f} W, GFX clock median {c:.0f} MHz")
