// Developer micro-benchmark: what a dependency between two tiny kernels costs on this stack
// (the epoch chain of the device-resident runner is a sequence of latency-bound kernels on
// two streams joined by events).  Prints the mean wall time per chain link, measured over
// many repetitions, for:
//   plain      k;k              on one stream
//   timing     k;event;k        a timing event recorded between them
//   sync-ev    k;event;k        an ordering-only event (hipEventDisableTiming)
//   fork-join  k | side k | k   main -> side -> main through two ordering-only events
//   graph      the fork-join chain captured once into a hipGraph and replayed
//   flag-fj    the fork-join without events: the producer stream's kernel publishes an epoch
//              number (agent-scope release store), the consumer stream runs a one-wave
//              kernel that polls it (bounded: gives up after 2 ms and counts a timeout)
//   flag-fj2   the same with the publishing done by a one-wave kernel after the producer
// Build: hipcc --offload-arch=gfx950 -O2 tools/gap_bench.hip -o /tmp/gap_bench
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>

__global__ void k_tiny(int* p) {
    if (threadIdx.x == 0 && blockIdx.x == 0) p[0] += 1;
}

__global__ void k_tiny_pub(int* p, unsigned* flag, unsigned v) {
    if (threadIdx.x == 0 && blockIdx.x == 0) {
        p[0] += 1;
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
        __hip_atomic_store(flag, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
}

__global__ void k_pub(unsigned* flag, unsigned v) {
    if (threadIdx.x == 0) {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
        __hip_atomic_store(flag, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
}

__global__ void k_wait(const unsigned* flag, unsigned v, unsigned* timeouts) {
    if (threadIdx.x == 0) {
        const uint64_t t0 = wall_clock64();
        while ((int)(__hip_atomic_load(flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) - v) < 0) {
            __builtin_amdgcn_s_sleep(1);
            if (wall_clock64() - t0 > 200000ull) {        // 2 ms at 100 MHz
                atomicAdd(timeouts, 1u);
                break;
            }
        }
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    }
}

#define CK(x)                                                                  \
    do {                                                                       \
        hipError_t e_ = (x);                                                   \
        if (e_ != hipSuccess) {                                                \
            printf("%s failed: %s\n", #x, hipGetErrorString(e_));              \
            return 1;                                                          \
        }                                                                      \
    } while (0)

int main() {
    int* d;
    CK(hipMalloc(&d, 64));
    CK(hipMemset(d, 0, 64));
    hipStream_t s, side;
    CK(hipStreamCreateWithPriority(&s, hipStreamNonBlocking, -1));
    CK(hipStreamCreateWithPriority(&side, hipStreamNonBlocking, -1));
    hipEvent_t et, es1, es2;
    CK(hipEventCreate(&et));
    CK(hipEventCreateWithFlags(&es1, hipEventDisableTiming));
    CK(hipEventCreateWithFlags(&es2, hipEventDisableTiming));
    const int N = 4000;
    auto run = [&](const char* name, auto body, int links) {
        for (int i = 0; i < 200; ++i) body();
        (void)hipDeviceSynchronize();
        auto t0 = std::chrono::steady_clock::now();
        for (int i = 0; i < N; ++i) body();
        (void)hipDeviceSynchronize();
        double us = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count();
        printf("%-10s %7.2f us per link (%d links per rep)\n", name, us / N / links, links);
    };
    run("plain", [&] { hipLaunchKernelGGL(k_tiny, dim3(1), dim3(64), 0, s, d); }, 1);
    run("timing", [&] {
        hipLaunchKernelGGL(k_tiny, dim3(1), dim3(64), 0, s, d);
        (void)hipEventRecord(et, s);
    }, 1);
    run("sync-ev", [&] {
        hipLaunchKernelGGL(k_tiny, dim3(1), dim3(64), 0, s, d);
        (void)hipEventRecord(es1, s);
    }, 1);
    auto forkjoin = [&] {
        hipLaunchKernelGGL(k_tiny, dim3(1), dim3(64), 0, s, d);
        (void)hipEventRecord(es1, s);
        (void)hipStreamWaitEvent(side, es1, 0);
        hipLaunchKernelGGL(k_tiny, dim3(1), dim3(64), 0, side, d + 1);
        (void)hipEventRecord(es2, side);
        (void)hipStreamWaitEvent(s, es2, 0);
    };
    run("fork-join", forkjoin, 2);
    hipGraph_t g;
    hipGraphExec_t ge;
    CK(hipStreamBeginCapture(s, hipStreamCaptureModeGlobal));
    for (int i = 0; i < 16; ++i) forkjoin();
    CK(hipStreamEndCapture(s, &g));
    CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
    run("graph", [&] { (void)hipGraphLaunch(ge, s); }, 32);
    hipGraph_t g2;
    hipGraphExec_t ge2;
    CK(hipStreamBeginCapture(s, hipStreamCaptureModeGlobal));
    for (int i = 0; i < 32; ++i) hipLaunchKernelGGL(k_tiny, dim3(1), dim3(64), 0, s, d);
    CK(hipStreamEndCapture(s, &g2));
    CK(hipGraphInstantiate(&ge2, g2, nullptr, nullptr, 0));
    run("graph-1s", [&] { (void)hipGraphLaunch(ge2, s); }, 32);
    unsigned* fl;
    CK(hipMalloc(&fl, 64));
    CK(hipMemset(fl, 0, 64));
    unsigned seq = 0;
    auto flagfj = [&] {
        ++seq;
        hipLaunchKernelGGL(k_tiny_pub, dim3(1), dim3(64), 0, s, d, fl, seq);
        hipLaunchKernelGGL(k_wait, dim3(1), dim3(64), 0, side, fl, seq, fl + 8);
        hipLaunchKernelGGL(k_tiny_pub, dim3(1), dim3(64), 0, side, d + 1, fl + 4, seq);
        hipLaunchKernelGGL(k_wait, dim3(1), dim3(64), 0, s, fl + 4, seq, fl + 8);
    };
    run("flag-fj", flagfj, 2);
    auto flagfj2 = [&] {
        ++seq;
        hipLaunchKernelGGL(k_tiny, dim3(1), dim3(64), 0, s, d);
        hipLaunchKernelGGL(k_pub, dim3(1), dim3(64), 0, s, fl, seq);
        hipLaunchKernelGGL(k_wait, dim3(1), dim3(64), 0, side, fl, seq, fl + 8);
        hipLaunchKernelGGL(k_tiny, dim3(1), dim3(64), 0, side, d + 1);
        hipLaunchKernelGGL(k_pub, dim3(1), dim3(64), 0, side, fl + 4, seq);
        hipLaunchKernelGGL(k_wait, dim3(1), dim3(64), 0, s, fl + 4, seq, fl + 8);
    };
    run("flag-fj2", flagfj2, 2);
    unsigned to = 0;
    CK(hipMemcpy(&to, fl + 8, 4, hipMemcpyDeviceToHost));
    printf("flag timeouts %u\n", to);
    int h = 0;
    CK(hipMemcpy(&h, d, 4, hipMemcpyDeviceToHost));
    printf("counter %d\n", h);
    return 0;
}
