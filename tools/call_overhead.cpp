// Diagnostic: wall time of participant-sized blocking calls from C++ (no Python), to split
// a call's fixed cost between the HIP runtime (launch + blocking wait) and the binding.
//   masks-dev: iris_engine_batch_process_device over 20 000 masks (rows stay in HBM)
//   shares-dev: the same over 20 000 u16 shares (DistanceEngine)
//   search:    iris_template_search over 20 000 templates (in-kernel reduce)
//   empty:     iris_device_synchronize on an idle stream
// build: g++ -O2 -std=c++17 -I include tools/call_overhead.cpp -L mpc-iris-code_amd -liris_hip
//        -Wl,-rpath,$PWD/mpc-iris-code_amd -Wl,-rpath-link,/opt/rocm/lib -o tools/call_overhead
#include <algorithm>
#include <chrono>
#include <cstdio>
#include <vector>

#include "iris_hip.h"

static double now_us() {
    return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

template <class F>
static void timeit(const char *name, F &&f, int calls = 3000) {
    for (int i = 0; i < 300; ++i) f();
    std::vector<double> t(calls);
    for (int i = 0; i < calls; ++i) {
        const double a = now_us();
        f();
        t[i] = now_us() - a;
    }
    std::sort(t.begin(), t.end());
    std::printf("%-10s median %.2f us  p10 %.2f us  p90 %.2f us\n", name, t[calls / 2], t[calls / 10], t[calls * 9 / 10]);
}

int main() {
    const uint64_t n = 20000;
    iris_device_t *d = nullptr;
    if (iris_device_open(0, &d)) return std::printf("open: %s\n", iris_last_error()), 1;
    iris_db_t *mdb = nullptr, *tdb = nullptr, *sdb = nullptr;
    iris_db_create(d, IRIS_KIND_MASKS, n, &mdb);
    iris_db_generate(mdb, n, 7, 0);
    iris_db_create(d, IRIS_KIND_TEMPLATES, n, &tdb);
    iris_db_generate(tdb, n, 7, 0);
    iris_db_create(d, IRIS_KIND_SHARES, n, &sdb);
    iris_db_generate(sdb, n, 7, 0);
    std::vector<uint64_t> q(400, 0x5555aaaa3333ccccull);
    std::vector<uint16_t> sq(IRIS_BITS);
    for (size_t i = 0; i < sq.size(); ++i) sq[i] = (uint16_t)(i * 40503u + 7u);
    iris_engine_t *me = nullptr, *te = nullptr, *se = nullptr;
    iris_distance_engine_new(d, sq.data(), &se);
    iris_masks_engine_new(d, q.data() + 200, &me);
    iris_template_engine_new(d, (const iris_template_t *)q.data(), &te);
    void *out = nullptr;
    iris_device_alloc(d, n * 31 * 2, &out);
    std::vector<uint16_t> hout(n * 31);
    timeit("empty", [&] { iris_device_synchronize(d); });
    timeit("masks-dev", [&] { iris_engine_batch_process_device(me, mdb, 0, n, (uint16_t *)out); });
    timeit("shares-dev", [&] { iris_engine_batch_process_device(se, sdb, 0, n, (uint16_t *)out); }, 1000);
    timeit("masks-host", [&] { iris_engine_batch_process(me, mdb, 0, n, hout.data()); });
    iris_match_t m;
    timeit("search", [&] { iris_template_search(te, tdb, 0, n, 0, nullptr, &m); });
    iris_device_set_profiling(d, 1);
    for (int i = 0; i < 500; ++i) {
        iris_engine_batch_process_device(me, mdb, 0, n, (uint16_t *)out);
        iris_template_search(te, tdb, 0, n, 0, nullptr, &m);
        iris_engine_batch_process_device(se, sdb, 0, n, (uint16_t *)out);
    }
    iris_device_synchronize(d);
    for (const char *k : {"masks", "template_search", "shares"}) {
        uint64_t l = 0, it = 0;
        double ms = 0;
        iris_device_kernel_stats(d, k, &l, &ms, &it);
        std::printf("kernel %-16s %.2f us\n", k, ms / l * 1e3);
    }
    iris_device_free(d, out);
    iris_engine_destroy(me);
    iris_engine_destroy(te);
    iris_engine_destroy(se);
    iris_db_destroy(sdb);
    iris_db_destroy(mdb);
    iris_db_destroy(tdb);
    iris_device_close(d);
    return 0;
}
