// Developer micro-benchmark: what a dependency between two tiny kernels costs on this stack
// (the epoch chain of the device-resident runner is a sequence of latency-bound kernels on
// two streams joined by events).  Prints the mean wall time per chain link, measured over
// many repetitions, for:
//   plain      k;k              on one stream
//   timing     k;event;k        a timing event recorded between them
//   sync-ev    k;event;k        an ordering-only event (hipEventDisableTiming)
//   fork-join  k | side k | k   main -> side -> main through two ordering-only events
//   graph      the fork-join chain captured once into a hipGraph and replayed
// Build: hipcc --offload-arch=gfx950 -O2 tools/gap_bench.hip -o /tmp/gap_bench
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>

__global__ void k_tiny(int* p) {
    if (threadIdx.x == 0 && blockIdx.x == 0) p[0] += 1;
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
    int h = 0;
    CK(hipMemcpy(&h, d, 4, hipMemcpyDeviceToHost));
    printf("counter %d\n", h);
    return 0;
}
