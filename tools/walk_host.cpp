// Diagnostic: the reference's chunk walk from C++ (no Python): a record file written from the
// on-device generator, mapped PROT_READ / MAP_SHARED (memmap2's Mmap::map, src/main.rs:389,458),
// walked in 20 000-record iris_engine_batch_process_host calls with a fresh engine per walk
// (src/main.rs:426-431, 511-516).  Prints per-walk records/s and per-call percentiles.
//   walk_host masks|shares RECORDS WALKS [FILE|-] [fresh]   (FILE: walk that record file instead,
//   written first if it does not exist; fresh: every call's rows go to a new calloc'd chunk-sized buffer, freed after the call,
//   as the reference's loops allocate `vec![..; chunk.len()]` per chunk, src/main.rs:429,514)
// build: g++ -O2 -std=c++17 -I include tools/walk_host.cpp -L mpc-iris-code_amd -liris_hip
//        -Wl,-rpath,$PWD/mpc-iris-code_amd -Wl,-rpath-link,/opt/rocm/lib -o tools/walk_host
#include <fcntl.h>
#include <stdlib.h>
#include <string.h>
#include <sys/mman.h>
#include <unistd.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <string>
#include <vector>

#include "iris_hip.h"

#define CK(x)                                                                    \
    do {                                                                         \
        if ((x) != 0) {                                                          \
            std::fprintf(stderr, "%s failed: %s\n", #x, iris_last_error());      \
            return 1;                                                            \
        }                                                                        \
    } while (0)

static double now_us() {
    return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

int main(int argc, char **argv) {
    setvbuf(stdout, nullptr, _IOLBF, 0);  // line-buffered: a run that dies still shows its walks
    const bool shares = argc > 1 && std::string(argv[1]) == "shares";
    const uint64_t n = argc > 2 ? strtoull(argv[2], nullptr, 10) : (shares ? 1000000 : 3000000);
    const int walks = argc > 3 ? atoi(argv[3]) : 8;
    const uint64_t chunk = 20000;
    const int kind = shares ? IRIS_KIND_SHARES : IRIS_KIND_MASKS;
    const size_t rb = shares ? 25600 : 1600;
    iris_device_t *dev = nullptr;
    CK(iris_device_open(0, &dev));
    const char *tmp = getenv("TMPDIR") ? getenv("TMPDIR") : "/tmp";
    const bool given = argc > 4 && std::string(argv[4]) != "-";
    const bool fresh = argc > 5 && std::string(argv[5]) == "fresh";
    const std::string path = given ? std::string(argv[4]) : std::string(tmp) + "/walk_host_" + std::to_string(getpid()) + ".rec";
    if (!given || access(path.c_str(), F_OK) != 0) {  // a FILE that does not exist yet is written and kept
        const uint64_t per = (1ull << 30) / rb;
        iris_db_t *g = nullptr;
        CK(iris_db_create(dev, kind, std::min(n, per), &g));
        int fd = ::open(path.c_str(), O_WRONLY | O_CREAT | O_TRUNC, 0600);
        std::vector<char> buf(std::min(n, per) * rb);
        for (uint64_t a = 0; a < n; a += per) {
            const uint64_t m = std::min(per, n - a);
            CK(iris_db_truncate(g, 0));
            CK(iris_db_generate(g, m, 7, a));
            CK(iris_db_read(g, 0, m, buf.data()));
            if (::write(fd, buf.data(), m * rb) != (ssize_t)(m * rb)) return 2;
        }
        ::close(fd);
        iris_db_destroy(g);
    }
    const int fd = ::open(path.c_str(), O_RDONLY);
    const char *map = (const char *)mmap(nullptr, n * rb, PROT_READ, MAP_SHARED, fd, 0);
    std::vector<uint16_t> out(n * 31);
    uint64_t qm[IRIS_LIMBS];
    for (int i = 0; i < IRIS_LIMBS; ++i) qm[i] = 0x9E3779B97F4A7C15ull * (i + 1);
    std::vector<uint16_t> qs(IRIS_BITS);
    for (int i = 0; i < IRIS_BITS; ++i) qs[i] = (uint16_t)(i * 40503u);
    std::vector<double> calls;
    for (int w = 0; w < walks; ++w) {
        const double t0 = now_us();
        iris_engine_t *e = nullptr;
        CK(shares ? iris_distance_engine_new(dev, qs.data(), &e) : iris_masks_engine_new(dev, qm, &e));
        std::vector<double> t;
        for (uint64_t a = 0; a < n; a += chunk) {
            const uint64_t m = std::min(chunk, n - a);
            uint16_t *dst = out.data() + a * 31;
            if (fresh) dst = (uint16_t *)calloc(m * 31, 2);
            const double c = now_us();
            CK(iris_engine_batch_process_host(e, map + a * rb, m, dst));
            t.push_back(now_us() - c);
            if (fresh) {
                out[a * 31] = dst[0];  // the rows are used
                free(dst);
            }
        }
        iris_engine_destroy(e);
        const double dt = now_us() - t0;
        if (w > 0) calls.insert(calls.end(), t.begin(), t.end());
        std::printf("walk %d: %.3f ms, %.3g records/s, first call %.1f us\n", w, dt / 1e3, n / dt * 1e6, t[0]);
    }
    std::sort(calls.begin(), calls.end());
    std::printf("calls after walk 0: median %.1f us  p10 %.1f  p90 %.1f  p99 %.1f  max %.1f\n", calls[calls.size() / 2],
                calls[calls.size() / 10], calls[calls.size() * 9 / 10], calls[calls.size() * 99 / 100], calls.back());
    char cfg[4096];
    iris_config(dev, cfg, sizeof(cfg), nullptr);
    std::printf("config: %s\n", cfg);
    munmap((void *)map, n * rb);
    ::close(fd);
    if (!given) ::unlink(path.c_str());
    iris_device_close(dev);
    return 0;
}
