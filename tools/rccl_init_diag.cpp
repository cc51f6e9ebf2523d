// What a non-blocking RCCL communicator init does when its peer never comes, step by step with
// timestamps (stderr): tools/rccl_init_diag [grouped 0|1] [wait_ms].  Built by hand:
//   hipcc -O2 -o tools/rccl_init_diag tools/rccl_init_diag.cpp -lrccl
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>
#include <stdio.h>
#include <stdlib.h>
#include <unistd.h>

#include <chrono>
#include <thread>

static double now_s() {
    static const auto t0 = std::chrono::steady_clock::now();
    return std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
}
#define LOG(...) do { fprintf(stderr, "[%7.3f] ", now_s()); fprintf(stderr, __VA_ARGS__); fputc('\n', stderr); } while (0)

int main(int argc, char **argv) {
    const int grouped = argc > 1 ? atoi(argv[1]) : 1;
    const int wait_ms = argc > 2 ? atoi(argv[2]) : 3000;
    (void)hipSetDevice(0);
    // watchdog: a call that never returns ends the process (exit 3) instead of hanging it
    std::thread([wait_ms] {
        std::this_thread::sleep_for(std::chrono::milliseconds(wait_ms + 8000));
        LOG("watchdog: still blocked %d ms after the start; exiting", wait_ms + 8000);
        fflush(stderr);
        _exit(3);
    }).detach();
    ncclUniqueId u;
    LOG("ncclGetUniqueId -> %d", (int)ncclGetUniqueId(&u));
    ncclConfig_t cfg = NCCL_CONFIG_INITIALIZER;
    cfg.blocking = 0;
    ncclComm_t comm = nullptr;
    if (grouped) LOG("ncclGroupStart -> %d", (int)ncclGroupStart());
    LOG("ncclCommInitRankConfig(nranks 2, rank 0) ...");
    ncclResult_t r = ncclCommInitRankConfig(&comm, 2, u, 0, &cfg);
    LOG("  -> %d (%s), comm %p", (int)r, ncclGetErrorString(r), (void *)comm);
    if (grouped) {
        LOG("ncclGroupEnd ...");
        r = ncclGroupEnd();
        LOG("  -> %d (%s), comm %p", (int)r, ncclGetErrorString(r), (void *)comm);
    }
    const auto t0 = std::chrono::steady_clock::now();
    int polls = 0;
    for (;;) {
        ncclResult_t st = ncclSuccess;
        r = comm ? ncclCommGetAsyncError(comm, &st) : ncclInvalidArgument;
        ++polls;
        if (polls == 1 || polls % 2000 == 0) LOG("poll %d: GetAsyncError -> %d, state %d", polls, (int)r, (int)st);
        if (r != ncclSuccess || st != ncclInProgress) break;
        if (std::chrono::steady_clock::now() - t0 > std::chrono::milliseconds(wait_ms)) {
            LOG("bound reached after %d polls", polls);
            break;
        }
        std::this_thread::sleep_for(std::chrono::microseconds(500));
    }
    LOG("ncclCommAbort ...");
    r = comm ? ncclCommAbort(comm) : ncclInvalidArgument;
    LOG("  -> %d (%s)", (int)r, ncclGetErrorString(r));
    LOG("hipMalloc after abort -> %d", (int)hipMalloc((void **)&comm, 4096));
    LOG("done");
    return 0;
}
