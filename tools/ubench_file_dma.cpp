// Diagnostic: file (page cache) -> device bandwidth, three ways:
//   A) 8 threads pread into a pinned buffer, then hipMemcpyAsync (the library's loader)
//   B) mmap the file, hipHostRegister each 64-MB window, DMA straight from the page cache
//   C) hipMemcpyAsync straight from the (unregistered) mmap (the runtime stages it)
// usage: ubench_file_dma <file> <bytes>   (the file is created if shorter than <bytes>)
#include <fcntl.h>
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <chrono>
#include <thread>
#include <vector>

static double now() {
    return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

#define CK(x)                                                                          \
    do {                                                                               \
        hipError_t e_ = (x);                                                           \
        if (e_ != hipSuccess) {                                                        \
            fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));                    \
            exit(1);                                                                   \
        }                                                                              \
    } while (0)

int main(int argc, char **argv) {
    const char *path = argc > 1 ? argv[1] : "/tmp/ubench_file_dma.bin";
    const size_t bytes = argc > 2 ? strtoull(argv[2], nullptr, 10) : (3200ull << 20);
    const size_t chunk = 64ull << 20;
    int fd = open(path, O_RDWR | O_CREAT, 0644);
    struct stat st;
    fstat(fd, &st);
    if ((size_t)st.st_size < bytes) {
        std::vector<char> buf(chunk);
        for (size_t i = 0; i < chunk; ++i) buf[i] = (char)(i * 2654435761u >> 13);
        for (size_t off = 0; off < bytes; off += chunk) {
            if (pwrite(fd, buf.data(), std::min(chunk, bytes - off), off) < 0) return 1;
        }
    }
    void *dev;
    CK(hipMalloc(&dev, bytes));
    hipStream_t s;
    CK(hipStreamCreate(&s));
    // warm the page cache
    {
        std::vector<char> buf(chunk);
        for (size_t off = 0; off < bytes; off += chunk)
            if (pread(fd, buf.data(), std::min(chunk, bytes - off), off) < 0) return 1;
    }
    // A) pinned double buffer + 8 reader threads
    {
        void *pin[2];
        CK(hipHostMalloc(&pin[0], chunk, hipHostMallocDefault));
        CK(hipHostMalloc(&pin[1], chunk, hipHostMallocDefault));
        hipEvent_t ev[2];
        CK(hipEventCreate(&ev[0]));
        CK(hipEventCreate(&ev[1]));
        const double t0 = now();
        int k = 0;
        for (size_t off = 0; off < bytes; off += chunk, k ^= 1) {
            const size_t m = std::min(chunk, bytes - off);
            CK(hipEventSynchronize(ev[k]));
            std::vector<std::thread> th;
            const size_t per = (m + 7) / 8;
            for (int i = 0; i < 8; ++i)
                th.emplace_back([&, i] {
                    const size_t lo = std::min(m, i * per), hi = std::min(m, lo + per);
                    if (hi > lo && pread(fd, (char *)pin[k] + lo, hi - lo, off + lo) < 0) abort();
                });
            for (auto &t : th) t.join();
            CK(hipMemcpyAsync((char *)dev + off, pin[k], m, hipMemcpyHostToDevice, s));
            CK(hipEventRecord(ev[k], s));
        }
        CK(hipStreamSynchronize(s));
        const double dt = now() - t0;
        printf("A pread x8 -> pinned -> device     %7.1f ms  %6.1f GB/s\n", dt * 1e3, bytes / dt / 1e9);
    }
    // B) register each window of the mapping, DMA from the page cache (mmap inside the timing)
    char *map = nullptr;
    {
        const double t0 = now();
        map = (char *)mmap(nullptr, bytes, PROT_READ, MAP_SHARED, fd, 0);
        if (map == MAP_FAILED) return 1;
        double treg = 0;
        std::vector<void *> regs;
        for (size_t off = 0; off < bytes; off += chunk) {
            const size_t m = std::min(chunk, bytes - off);
            const double r0 = now();
            hipError_t e = hipHostRegister(map + off, m, hipHostRegisterReadOnly);
            treg += now() - r0;
            if (e != hipSuccess) {
                printf("B hipHostRegister on the file mapping failed: %s\n", hipGetErrorString(e));
                break;
            }
            regs.push_back(map + off);
            CK(hipMemcpyAsync((char *)dev + off, map + off, m, hipMemcpyHostToDevice, s));
        }
        CK(hipStreamSynchronize(s));
        const double dt = now() - t0;
        for (void *p : regs) (void)hipHostUnregister(p);
        if (regs.size() * chunk >= bytes)
            printf("B register mmap windows -> device  %7.1f ms  %6.1f GB/s  (register %.1f ms)\n", dt * 1e3,
                   bytes / dt / 1e9, treg * 1e3);
    }
    // B2) as B, but a 2-window ring: window i-2 is unregistered (after its copy) before
    //     window i is registered — the library loader's structure
    for (int ring : {2, 8}) {
        std::vector<hipEvent_t> ev(ring);
        std::vector<char *> reg(ring, nullptr);
        for (auto &e : ev) CK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
        const double t0 = now();
        double tun = 0;
        int i = 0;
        for (size_t off = 0; off < bytes; off += chunk, ++i) {
            const int b = i % ring;
            const size_t m = std::min(chunk, bytes - off);
            if (reg[b]) {
                CK(hipEventSynchronize(ev[b]));
                const double u0 = now();
                CK(hipHostUnregister(reg[b]));
                tun += now() - u0;
            }
            CK(hipHostRegister(map + off, m, hipHostRegisterReadOnly));
            reg[b] = map + off;
            CK(hipMemcpyAsync((char *)dev + off, map + off, m, hipMemcpyHostToDevice, s));
            CK(hipEventRecord(ev[b], s));
        }
        CK(hipStreamSynchronize(s));
        const double dt = now() - t0;
        for (char *r : reg)
            if (r) CK(hipHostUnregister(r));
        printf("B2 ring %d register/unregister      %7.1f ms  %6.1f GB/s  (unregister %.1f ms)\n", ring, dt * 1e3,
               bytes / dt / 1e9, tun * 1e3);
    }
    // C) plain hipMemcpyAsync from the mapping
    {
        const double t0 = now();
        for (size_t off = 0; off < bytes; off += chunk)
            CK(hipMemcpyAsync((char *)dev + off, map + off, std::min(chunk, bytes - off), hipMemcpyHostToDevice, s));
        CK(hipStreamSynchronize(s));
        const double dt = now() - t0;
        printf("C memcpy from mmap (runtime stage) %7.1f ms  %6.1f GB/s\n", dt * 1e3, bytes / dt / 1e9);
    }
    munmap(map, bytes);
    close(fd);
    unlink(path);
    return 0;
}
