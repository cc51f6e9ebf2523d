// Diagnostic: round-trip latency of one small kernel launch on gfx950, by how the host waits.
//   sync-1 / sync-625   launch (1 or 625 workgroups of 256 threads) + hipStreamSynchronize
//   event-625           launch + hipEventRecord + hipEventSynchronize
//   flag-1 / flag-625   launch of a kernel whose last workgroup stores a sequence number into
//                       coherent pinned host memory (system-scope release store), host spins on it
//   launch-only         the CPU time of hipLaunchKernelGGL itself (stream drained every 64)
// build: hipcc -O2 --offload-arch=gfx950 -x hip tools/ubench_launch.cpp -o tools/ubench_launch
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstring>
#include <sys/mman.h>

#include <thread>
#include <vector>

#define CK(x)                                                                    \
    do {                                                                         \
        hipError_t e_ = (x);                                                     \
        if (e_ != hipSuccess) {                                                  \
            std::printf("%s: %s\n", #x, hipGetErrorString(e_));                  \
            return 1;                                                            \
        }                                                                        \
    } while (0)

__global__ void k_empty() {}

// the workgroup that draws the last ticket publishes `seq` to the host word
__global__ void k_flag(unsigned *ticket, unsigned *host_flag, unsigned seq) {
    __shared__ int last;
    if (threadIdx.x == 0) {
        last = gridDim.x == 1 ||
               __hip_atomic_fetch_add(ticket, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == gridDim.x - 1;
        if (last && gridDim.x > 1) __hip_atomic_store(ticket, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (last) __hip_atomic_store(host_flag, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    }
}

// copies n16 16-byte words into coherent host memory with write-through stores, then
// publishes `seq` like k_flag once every workgroup's stores have completed
__global__ void k_rows(const uint4 *src, uint4 *dst, size_t n16, unsigned *ticket, unsigned *host_flag, unsigned seq) {
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n16; i += (size_t)gridDim.x * blockDim.x) {
        const uint4 v = src[i];
        __hip_atomic_store((unsigned long long *)&dst[i], (unsigned long long)v.x | ((unsigned long long)v.y << 32),
                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        __hip_atomic_store((unsigned long long *)&dst[i] + 1, (unsigned long long)v.z | ((unsigned long long)v.w << 32),
                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    __shared__ int last;
    if (threadIdx.x == 0) {
        last = __hip_atomic_fetch_add(ticket, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == gridDim.x - 1;
        if (last) {
            __hip_atomic_store(ticket, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_store(host_flag, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
        }
    }
}

// plain 16-B stores (nt = 1: nontemporal) into host memory; visible to the host at kernel end
template <int NT>
__global__ void k_rows_plain(const uint4 *src, uint4 *dst, size_t n16) {
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n16; i += (size_t)gridDim.x * blockDim.x) {
        const uint4 v = src[i];
        typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
        if (NT)
            __builtin_nontemporal_store(u32x4{v.x, v.y, v.z, v.w}, (u32x4 *)&dst[i]);
        else
            dst[i] = v;
    }
}

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
    std::printf("%-12s median %7.2f us  p10 %7.2f us  p90 %7.2f us\n", name, t[calls / 2], t[calls / 10],
                t[calls * 9 / 10]);
}

int main() {
    hipStream_t s;
    CK(hipSetDevice(0));
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    unsigned *ticket = nullptr, *flag = nullptr;
    CK(hipMalloc(&ticket, 256));
    CK(hipMemset(ticket, 0, 256));
    CK(hipHostMalloc(&flag, 4096, hipHostMallocCoherent | hipHostMallocMapped));
    *flag = 0;
    hipEvent_t ev;
    CK(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
    unsigned seq = 0;
    bool bad = false;
    auto spin = [&](unsigned want) {
        volatile unsigned *f = flag;
        const double t0 = now_us();
        while (*f != want) {
            if (now_us() - t0 > 2e6) {  // 2 s: the kernel never published
                bad = true;
                return;
            }
        }
    };
    timeit("sync-1", [&] {
        hipLaunchKernelGGL(k_empty, dim3(1), dim3(256), 0, s);
        (void)hipStreamSynchronize(s);
    });
    timeit("sync-625", [&] {
        hipLaunchKernelGGL(k_empty, dim3(625), dim3(256), 0, s);
        (void)hipStreamSynchronize(s);
    });
    timeit("event-625", [&] {
        hipLaunchKernelGGL(k_empty, dim3(625), dim3(256), 0, s);
        (void)hipEventRecord(ev, s);
        (void)hipEventSynchronize(ev);
    });
    timeit("flag-1", [&] {
        hipLaunchKernelGGL(k_flag, dim3(1), dim3(256), 0, s, ticket, flag, ++seq);
        spin(seq);
    });
    CK(hipStreamSynchronize(s));
    timeit("flag-625", [&] {
        hipLaunchKernelGGL(k_flag, dim3(625), dim3(256), 0, s, ticket, flag, ++seq);
        spin(seq);
    });
    CK(hipStreamSynchronize(s));
    int i = 0;
    timeit("launch-only", [&] {
        hipLaunchKernelGGL(k_empty, dim3(625), dim3(256), 0, s);
        if (++i % 64 == 0) (void)hipStreamSynchronize(s);
    });
    CK(hipStreamSynchronize(s));

    // the [20000][31] u16 rows of a participant-sized MasksEngine call (1.24 MB) to the host
    const size_t rows = 20000ull * 31 * 2;
    void *dev = nullptr, *pinned = nullptr, *pinned_c = nullptr;
    CK(hipMalloc(&dev, rows));
    CK(hipMemset(dev, 1, rows));
    CK(hipHostMalloc(&pinned, rows, hipHostMallocDefault));
    CK(hipHostMalloc(&pinned_c, rows, hipHostMallocCoherent | hipHostMallocMapped));
    std::vector<char> pageable(rows, 0);
    timeit("d2h-pageable", [&] {
        (void)hipMemcpyAsync(pageable.data(), dev, rows, hipMemcpyDeviceToHost, s);
        (void)hipStreamSynchronize(s);
    }, 1000);
    timeit("d2h-pinned", [&] {
        (void)hipMemcpyAsync(pinned, dev, rows, hipMemcpyDeviceToHost, s);
        (void)hipStreamSynchronize(s);
    }, 1000);
    timeit("memcpy-pin", [&] { std::memcpy(pageable.data(), pinned, rows); }, 1000);
    timeit("memcpy-coh", [&] { std::memcpy(pageable.data(), pinned_c, rows); }, 1000);
    timeit("kplain-pin", [&] {
        hipLaunchKernelGGL(k_rows_plain<0>, dim3(304), dim3(256), 0, s, (const uint4 *)dev, (uint4 *)pinned, rows / 16);
        (void)hipStreamSynchronize(s);
    }, 1000);
    timeit("knt-pin", [&] {
        hipLaunchKernelGGL(k_rows_plain<1>, dim3(304), dim3(256), 0, s, (const uint4 *)dev, (uint4 *)pinned, rows / 16);
        (void)hipStreamSynchronize(s);
    }, 1000);
    timeit("kplain-coh", [&] {
        hipLaunchKernelGGL(k_rows_plain<0>, dim3(304), dim3(256), 0, s, (const uint4 *)dev, (uint4 *)pinned_c, rows / 16);
        (void)hipStreamSynchronize(s);
    }, 1000);
    timeit("kplain+memcpy", [&] {
        hipLaunchKernelGGL(k_rows_plain<0>, dim3(304), dim3(256), 0, s, (const uint4 *)dev, (uint4 *)pinned, rows / 16);
        (void)hipStreamSynchronize(s);
        std::memcpy(pageable.data(), pinned, rows);
    }, 1000);
    timeit("d2h-pin+memcpy", [&] {
        (void)hipMemcpyAsync(pinned, dev, rows, hipMemcpyDeviceToHost, s);
        (void)hipStreamSynchronize(s);
        std::memcpy(pageable.data(), pinned, rows);
    }, 1000);
    // destination page size: a 2-MB-aligned buffer advised to huge pages vs one forced to 4-KB pages
    char *thp = (char *)mmap(nullptr, 8 << 20, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS, -1, 0);
    char *small = (char *)mmap(nullptr, 8 << 20, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS, -1, 0);
    char *thp_al = (char *)(((uintptr_t)thp + (2 << 20) - 1) & ~(uintptr_t)((2 << 20) - 1));
    madvise(thp_al, 4 << 20, MADV_HUGEPAGE);
    madvise(small, 8 << 20, MADV_NOHUGEPAGE);
    std::memset(thp_al, 0, 4 << 20);
    std::memset(small, 0, 8 << 20);
    timeit("d2h-thp", [&] {
        (void)hipMemcpyAsync(thp_al, dev, rows, hipMemcpyDeviceToHost, s);
        (void)hipStreamSynchronize(s);
    }, 1000);
    timeit("d2h-4k", [&] {
        (void)hipMemcpyAsync(small, dev, rows, hipMemcpyDeviceToHost, s);
        (void)hipStreamSynchronize(s);
    }, 1000);
    timeit("reg+d2h-4k", [&] {  // page-lock the destination for this call only
        (void)hipHostRegister(small, rows, hipHostRegisterDefault);
        (void)hipMemcpyAsync(small, dev, rows, hipMemcpyDeviceToHost, s);
        (void)hipStreamSynchronize(s);
        (void)hipHostUnregister(small);
    }, 300);
    auto mt_copy = [&](char *dst, const char *src, size_t bytes, int nt) {
        std::vector<std::thread> th;
        const size_t per = (bytes / nt + 63) & ~(size_t)63;
        for (int i = 0; i < nt; ++i) {
            const size_t a = i * per, b = std::min(bytes, a + per);
            if (a < b) th.emplace_back([=] { std::memcpy(dst + a, src + a, b - a); });
        }
        for (auto &t : th) t.join();
    };
    for (int nt : {1, 4}) {
        char name[32];
        std::snprintf(name, sizeof name, "kpin+cp%d-4k", nt);
        timeit(name, [&] {
            hipLaunchKernelGGL(k_rows_plain<0>, dim3(304), dim3(256), 0, s, (const uint4 *)dev, (uint4 *)pinned, rows / 16);
            (void)hipStreamSynchronize(s);
            mt_copy(small, (const char *)pinned, rows, nt);
        }, 1000);
    }
    munmap(thp, 8 << 20);
    munmap(small, 8 << 20);
    // the same D2H after a kernel on the same stream, and behind a cross-stream event while the
    // other stream runs a kernel (the read-ahead's shape)
    void *dev2 = nullptr;
    CK(hipMalloc(&dev2, rows));
    hipStream_t s2;
    CK(hipStreamCreateWithFlags(&s2, hipStreamNonBlocking));
    hipEvent_t e1, e2;
    CK(hipEventCreateWithFlags(&e1, hipEventDisableTiming));
    CK(hipEventCreateWithFlags(&e2, hipEventDisableTiming));
    timeit("kern+d2h", [&] {
        hipLaunchKernelGGL(k_rows_plain<0>, dim3(304), dim3(256), 0, s, (const uint4 *)dev, (uint4 *)dev2, rows / 16);
        (void)hipMemcpyAsync(pageable.data(), dev2, rows, hipMemcpyDeviceToHost, s);
        (void)hipStreamSynchronize(s);
    }, 1000);
    timeit("xwait+d2h", [&] {
        hipLaunchKernelGGL(k_rows_plain<0>, dim3(304), dim3(256), 0, s2, (const uint4 *)dev, (uint4 *)dev2, rows / 16);
        (void)hipEventRecord(e1, s2);
        (void)hipStreamWaitEvent(s, e1, 0);
        (void)hipMemcpyAsync(pageable.data(), dev2, rows, hipMemcpyDeviceToHost, s);
        (void)hipEventRecord(e2, s);
        (void)hipEventSynchronize(e2);
    }, 1000);
    timeit("xwait+d2h+k", [&] {  // + the next kernel on s2 while the copy runs
        hipLaunchKernelGGL(k_rows_plain<0>, dim3(304), dim3(256), 0, s2, (const uint4 *)dev, (uint4 *)dev2, rows / 16);
        (void)hipEventRecord(e1, s2);
        (void)hipStreamWaitEvent(s, e1, 0);
        hipLaunchKernelGGL(k_rows_plain<0>, dim3(304), dim3(256), 0, s2, (const uint4 *)dev, (uint4 *)pinned, rows / 16);
        (void)hipMemcpyAsync(pageable.data(), dev2, rows, hipMemcpyDeviceToHost, s);
        (void)hipEventRecord(e2, s);
        (void)hipEventSynchronize(e2);
    }, 1000);
    CK(hipStreamSynchronize(s2));
    timeit("kern-to-coh", [&] {
        hipLaunchKernelGGL(k_rows, dim3(625), dim3(256), 0, s, (const uint4 *)dev, (uint4 *)pinned_c,
                           rows / 16, ticket, flag, ++seq);
        spin(seq);
    }, 50);
    CK(hipStreamSynchronize(s));
    CK(hipFree(dev));
    CK(hipHostFree(pinned));
    CK(hipHostFree(pinned_c));
    std::printf("flag timeouts: %s\n", bad ? "YES" : "none");
    CK(hipHostFree(flag));
    CK(hipFree(ticket));
    return bad ? 2 : 0;
}
