"""CPU: the TRITS layout's position map (csrc/iris_internal.hpp trit_pos / trit_slot)
against a restatement of the search kernel's decode (csrc/iris_trits.hip: the T_w / T_s
tables, `lookups` and `combine`).  The host map is what the pack / unpack / generate
kernels use; the decode is what the search kernel reads, so the two must agree
position for position for the GPU results to equal the oracle's."""
import pathlib
import subprocess

import numpy as np

ROOT = pathlib.Path(__file__).resolve().parents[1]
CSRC = ROOT / "mpc-iris-code_amd" / "csrc"

PROG = r"""
#include "iris_internal.hpp"
#include <cstdio>
int main() {
    int seen[160] = {0}, bad = 0;
    for (int s = 0; s < 2; ++s)
        for (int jj = 0; jj < 16; ++jj)
            for (int k = 0; k < 5; ++k) {
                const int x = iris::trit_pos(s, jj, k);
                int s2, j2, k2;
                iris::trit_slot(x, s2, j2, k2);
                if (x < 0 || x >= 160 || s2 != s || j2 != jj || k2 != k) ++bad;
                else ++seen[x];
                std::printf("%d %d %d %d\n", s, jj, k, x);
            }
    for (int x = 0; x < 160; ++x) bad += seen[x] != 1;
    std::printf("bad %d\n", bad);
    // trit_byte / trit_decode round trip on every byte value
    for (uint32_t m = 0; m < 32; ++m)
        for (uint32_t p = 0; p < 32; ++p) {
            const uint32_t v = iris::trit_byte(m, p), d = iris::trit_decode(v);
            for (int i = 0; i < 5; ++i) {
                const uint32_t want = ((m >> i) & 1u) ? (((p >> i) & 1u) ? 0xAu : 0x2u) : 0u;
                if (v >= 243 || ((d >> (4 * i)) & 15u) != want) ++bad;
            }
        }
    std::printf("bad %d\n", bad);
    return bad != 0;
}
"""


def _code(d):
    return (0x0, 0x2, 0xA)[d]


def _t_w(v):
    x = 0
    for i in range(5):
        x |= _code(v % 3) << (4 * i)
        v //= 3
    return x


def _combine(half):
    """The kernel's decode of one lane's 16-byte half-stage into 10 stream dwords."""
    e = [(_t_w(b) << (4 if (i >> 2) & 1 else 0)) & 0xFFFFFFFF for i, b in enumerate(half)]
    out = []
    for q in range(2):
        w, t = e[8 * q:8 * q + 4], e[8 * q + 4:8 * q + 8]
        out += [((t[j] << 16) | w[j]) & 0xFFFFFFFF for j in range(4)]
        out.append(sum(((t[j] >> 16) & 0xFF) << (8 * j) for j in range(4)))
    return out


def test_trit_layout_matches_decode(tmp_path):
    exe = tmp_path / "trit_map"
    src = tmp_path / "trit_map.cpp"
    src.write_text(PROG)
    subprocess.run(["g++", "-std=c++17", "-O1", f"-I{CSRC}", str(src), "-o", str(exe)], check=True)
    res = subprocess.run([str(exe)], capture_output=True, text=True)
    lines = res.stdout.split("\n")
    assert res.returncode == 0 and "bad 0" in lines, res.stdout[-200:]
    pos = {}
    for ln in lines:
        f = ln.split()
        if len(f) == 4:
            s, jj, k, x = map(int, f)
            pos[(s, jj, k)] = x
    assert len(pos) == 160
    rng = np.random.default_rng(5)
    for trial in range(200):
        for s in range(2):
            half = [int(b) for b in rng.integers(0, 243, 16)]
            if trial == 0:
                half = [242] * 16 if s else [0] * 16
            dw = _combine(half)
            for jj, b in enumerate(half):
                v = b
                for k in range(5):
                    x = pos[(s, jj, k)] - 80 * s  # the half-stage's own nibble
                    assert 0 <= x < 80
                    got = (dw[x // 8] >> (4 * (x % 8))) & 0xF
                    assert got == _code(v % 3), (s, jj, k)
                    v //= 3
