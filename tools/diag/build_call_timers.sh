#!/bin/bash
# Builds tools/diag/libiris_hip_timers.so: the library with per-phase timers in the host-slice call
# (iris_engine_batch_process_host -> readahead_u16_call: set_device, resident_slice, window launch,
# event wait, copy-out; IRIS_DIAG_PLAIN=1 expands with plain stores), from a patched COPY of the sources (the tree's sources stay untimed).
# Run here (CPU); tools/diag/call_timers.sh runs the C++ walk against it on the GPU box.
set -e
ROOT=$(cd "$(dirname "$0")/../.." && pwd)
W=$(mktemp -d)
mkdir -p $W/mpc-iris-code_amd
cp -r $ROOT/mpc-iris-code_amd/Makefile $ROOT/mpc-iris-code_amd/csrc $W/mpc-iris-code_amd/
cp -r $ROOT/include $W/
python3 - $W/mpc-iris-code_amd/csrc/iris_api.hip <<'PY'
import sys
p = sys.argv[1]; s = open(p).read()
hdr = '''
#include <algorithm>
#include <array>
#include <chrono>
#include <cstdio>
#include <vector>
namespace {
struct CallTimers {
    std::vector<std::array<double, 8>> calls;
    ~CallTimers() {
        if (calls.size() < 12) return;
        const size_t skip = calls.size() / 6;  // the first of 6 walks (resident fill, first touch of out)
        std::fprintf(stderr, "call timers (%zu calls after walk 0, median / p90 us):", calls.size() - skip);
        const char *nm[] = {"", "set_device", "resident_slice", "launch", "event_sync", "expand"};
        for (int i = 1; i <= 5; ++i) {
            std::vector<double> v;
            for (size_t c = skip; c < calls.size(); ++c) v.push_back(calls[c][i]);
            std::sort(v.begin(), v.end());
            std::fprintf(stderr, " %s %.2f/%.2f", nm[i], v[v.size() / 2], v[v.size() * 9 / 10]);
        }
        std::fprintf(stderr, "\\n");
        const size_t per = calls.size() / 6;  // each walk's first call (a new engine's first window)
        for (size_t c = per; c < calls.size(); c += per)
            std::fprintf(stderr, "first call of walk %zu: set_device %.2f resident_slice %.2f launch %.2f event_sync %.2f expand %.2f (launch: aux+events %.2f, order event %.2f)\\n",
                         c / per, calls[c][1], calls[c][2], calls[c][3], calls[c][4], calls[c][5], calls[c][6], calls[c][7]);
    }
} g_ct;
thread_local std::array<double, 8> g_cur;
thread_local double g_t0;
inline double nowus() { return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count(); }
inline void mark(int i) { const double t = nowus(); g_cur[i] = t - g_t0; g_t0 = t; }
}
'''
def sub(old, new):
    global s
    assert s.count(old) == 1, old
    s = s.replace(old, new)
i = s.index('// ---- read-ahead of host-output engine calls')
s = s[:i] + hdr + s[i:]
sub('    HIPCHK(hipEventSynchronize(ra.computed[b]));\n    const uint64_t at = first - w.first;',
    '    mark(3);\n    HIPCHK(hipEventSynchronize(ra.computed[b]));\n    mark(4);\n    const uint64_t at = first - w.first;')
sub('(size_t)n * kRot * 2, d->ordinal);\n    }\n    if (d->profiling) fold_done(d);\n    return 0;',
    '(size_t)n * kRot * 2, d->ordinal);\n    }\n    mark(5);\n    g_ct.calls.push_back(g_cur);\n    if (d->profiling) fold_done(d);\n    return 0;')
sub('uint16_t *out) {\n    IRIS_KEEP_DEVICE();\n    ARG(e, "engine is NULL");\n    ARG(e->kind == IRIS_KIND_MASKS || e->kind == IRIS_KIND_SHARES, "batch_process',
    'uint16_t *out) {\n    g_t0 = nowus();\n    IRIS_KEEP_DEVICE();\n    ARG(e, "engine is NULL");\n    ARG(e->kind == IRIS_KIND_MASKS || e->kind == IRIS_KIND_SHARES, "batch_process')
sub('    CHK(set_device(d));\n    if (n == 0) return 0;\n    ARG(records && out, "NULL argument");\n    const KindInfo k = kind_info(e->kind);\n    // a slice of an attached',
    '    CHK(set_device(d));\n    mark(1);\n    if (n == 0) return 0;\n    ARG(records && out, "NULL argument");\n    const KindInfo k = kind_info(e->kind);\n    // a slice of an attached')
sub('    CHK(resident_slice(d, e->kind, records, n, &rdb, &rfirst, &rend));\n    if (rdb) {',
    '    CHK(resident_slice(d, e->kind, records, n, &rdb, &rfirst, &rend));\n    mark(2);\n    if (rdb) {')
# sub-phases of a window launch: [6] ensure_aux + event creation, [7] the order event on the device stream
sub('    if (launched) *launched = false;\n    CHK(ensure_aux(d));',
    '    if (launched) *launched = false;\n    const double s0 = nowus();\n    CHK(ensure_aux(d));')
sub('    const size_t rec = ra_rec_bytes(e);\n    const size_t bytes = (size_t)n * rec;',
    '    g_cur[6] += nowus() - s0;\n    const size_t rec = ra_rec_bytes(e);\n    const size_t bytes = (size_t)n * rec;')
sub('    hipStream_t side = b ? d->aux2 : d->aux;\n',
    '    hipStream_t side = b ? d->aux2 : d->aux;\n    const double s2 = nowus();\n')
sub('    ra.win[b].live = false;\n    ra.on[b] = side;\n    CHK(enqueue_u16_engine',
    '    g_cur[7] += nowus() - s2;\n    ra.win[b].live = false;\n    ra.on[b] = side;\n    CHK(enqueue_u16_engine')
sub('    g_t0 = nowus();\n    IRIS_KEEP_DEVICE();', '    g_t0 = nowus();\n    g_cur[6] = g_cur[7] = 0;\n    IRIS_KEEP_DEVICE();')
open(p, 'w').write(s)
# IRIS_DIAG_PLAIN=1: the copy-out's expansion with plain stores instead of non-temporal blocks
h = p.replace('iris_api.hip', 'iris_host.cpp'); t = open(h).read()
old = '    if (kHaveAvx512)\n        expand_avx512(out, pk, esc, n);'
assert t.count(old) == 1
t = t.replace(old, '    static const bool plain = getenv("IRIS_DIAG_PLAIN") != nullptr;\n    if (kHaveAvx512)\n        (plain ? expand_plain : expand_avx512)(out, pk, esc, n);')
# IRIS_DIAG_HELPER_CPUS=a-b,c-d: the helpers run on those CPUs; IRIS_DIAG_SPREAD=1: helper i runs on the CPUs of the (i+1)-th L3 domain after the pool creator's
# (of the CPUs this process may use); IRIS_DIAG_TOPO=1 prints the domains and where threads run
spread = r"""
#include <sched.h>
#include <stdio.h>
static std::vector<std::vector<int>> diag_l3_domains() {
    cpu_set_t allowed; CPU_ZERO(&allowed); sched_getaffinity(0, sizeof(allowed), &allowed);
    std::vector<std::vector<int>> doms; std::vector<std::string> keys;
    for (int c = 0; c < CPU_SETSIZE; ++c) {
        if (!CPU_ISSET(c, &allowed)) continue;
        char path[128]; snprintf(path, sizeof(path), "/sys/devices/system/cpu/cpu%d/cache/index3/shared_cpu_list", c);
        FILE *f = fopen(path, "r"); if (!f) continue;
        char buf[256] = {}; if (!fgets(buf, sizeof(buf), f)) buf[0] = 0; fclose(f);
        std::string k(buf); size_t i = 0;
        for (; i < keys.size() && keys[i] != k; ++i) {}
        if (i == keys.size()) { keys.push_back(k); doms.emplace_back(); }
        doms[i].push_back(c);
    }
    return doms;
}
static void diag_place(int helper, int creator) {
    static const bool on = getenv("IRIS_DIAG_SPREAD") != nullptr, topo = getenv("IRIS_DIAG_TOPO") != nullptr;
    static std::vector<std::vector<int>> doms = diag_l3_domains();
    const int home = creator;
    if (topo && helper == 0) {
        fprintf(stderr, "diag: %zu L3 domains allowed, creator on cpu %d; sizes:", doms.size(), home);
        for (auto &d : doms) fprintf(stderr, " %zu(first %d)", d.size(), d.empty() ? -1 : d[0]);
        fprintf(stderr, "\n");
    }
    if (const char *cl = getenv("IRIS_DIAG_HELPER_CPUS")) {  // "a-b,c-d": the helpers' CPUs
        cpu_set_t set; CPU_ZERO(&set);
        for (const char *q = cl; *q;) {
            char *e; const long a = strtol(q, &e, 10); long b = a;
            if (*e == '-') b = strtol(e + 1, &e, 10);
            for (long c = a; c <= b; ++c) CPU_SET((int)c, &set);
            q = *e == ',' ? e + 1 : e;
            if (e == q && *q) break;
        }
        sched_setaffinity(0, sizeof(set), &set);
        return;
    }
    if (getenv("IRIS_DIAG_NODE")) {  // the CPUs of the pool creator's NUMA node (of those allowed)
        int node = -1;
        for (int n = 0; n < 64 && node < 0; ++n) {
            char path[128]; snprintf(path, sizeof(path), "/sys/devices/system/cpu/cpu%d/node%d", home, n);
            if (access(path, F_OK) == 0) node = n;
        }
        char path[128]; snprintf(path, sizeof(path), "/sys/devices/system/node/node%d/cpulist", node);
        FILE *f = fopen(path, "r"); char buf[512] = {};
        if (!f || !fgets(buf, sizeof(buf), f)) { if (f) fclose(f); return; }
        fclose(f);
        cpu_set_t allowed; CPU_ZERO(&allowed); sched_getaffinity(0, sizeof(allowed), &allowed);
        cpu_set_t set; CPU_ZERO(&set);
        for (const char *q = buf; *q && *q != '\n';) {
            char *e; const long a = strtol(q, &e, 10); long b = a;
            if (*e == '-') b = strtol(e + 1, &e, 10);
            for (long c = a; c <= b; ++c) if (CPU_ISSET((int)c, &allowed)) CPU_SET((int)c, &set);
            q = *e == ',' ? e + 1 : e;
            if (e == q) break;
        }
        if (CPU_COUNT(&set)) sched_setaffinity(0, sizeof(set), &set);
        if (topo) fprintf(stderr, "diag: helper %d -> node %d (creator cpu %d)\n", helper, node, home);
        return;
    }
    if (!on || doms.size() < 2) return;
    size_t h = 0;
    for (size_t i = 0; i < doms.size(); ++i) for (int c : doms[i]) if (c == home) h = i;
    const auto &d = doms[(h + 1 + helper) % doms.size()];
    cpu_set_t set; CPU_ZERO(&set); for (int c : d) CPU_SET(c, &set);
    sched_setaffinity(0, sizeof(set), &set);
}
"""
old = 'class CopyPool {'
assert t.count(old) == 1
t = t.replace(old, spread + old)
old = '        for (int i = 0; i < helpers; ++i) threads_.emplace_back([this] { worker(); });'
assert t.count(old) == 1
t = t.replace(old, '        for (int i = 0; i < helpers; ++i) threads_.emplace_back([this, i, c = sched_getcpu()] { diag_place(i, c); if (getenv("IRIS_DIAG_TOPO")) fprintf(stderr, "diag: helper %d on cpu %d\\n", i, sched_getcpu()); worker(); });')
open(h, 'w').write(t)
PY
make -C $W/mpc-iris-code_amd -j8 LIB=libiris_hip_timers.so libiris_hip_timers.so >/dev/null
cp $W/mpc-iris-code_amd/libiris_hip_timers.so $ROOT/tools/diag/
rm -rf $W
echo "built tools/diag/libiris_hip_timers.so"
