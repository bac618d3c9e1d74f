// Dependent-latency probe (round 6): how many cycles does one wave need per dependent fp64
// operation on gfx950, and per row of the DDM p chain (p += RN((x - p) / n): sub, mul, fma,
// fma, add), alone on the GPU?  One wave per launch, s_memtime (core clock) around the loop.
//   hipcc --offload-arch=gfx950 -O3 -ffp-contract=off tools/lat_bench.hip -o tools/lat_bench
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

__device__ __forceinline__ double div_rn(double a, double n, double r) {
    const double q0 = a * r;
    const double e = __builtin_fma(-q0, n, a);
    return __builtin_fma(e, r, q0);
}

template <int kMode>
__global__ void k_lat(double* out, uint64_t* cyc, int iters, double seed) {
    double p = seed + threadIdx.x * 1e-9;
    double n = 17.0;
    const double r = 1.0 / n;
    const uint64_t t0 = __builtin_readcyclecounter();
    if (kMode == 0) {            // fma chain
        for (int i = 0; i < iters; ++i) p = __builtin_fma(p, 0.999999, 1e-7);
    } else if (kMode == 1) {     // add chain
        for (int i = 0; i < iters; ++i) p = p + 1e-9;
    } else if (kMode == 2) {     // the DDM p row (x from a bit pattern)
        const uint32_t bits = 0x10204081u;
        for (int i = 0; i < iters; ++i) {
            const double x = (double)((bits >> (i & 31)) & 1u);
            p = p + div_rn(x - p, n, r);
        }
    } else if (kMode == 3) {     // the DDM p row, 4-op form for x == 0 rows: q0 = -p * r
        for (int i = 0; i < iters; ++i) {
            const double q0 = -p * r;
            const double e = __builtin_fma(-q0, n, -p);
            p = p + __builtin_fma(e, r, q0);
        }
    } else if (kMode == 4) {     // i32 add chain
        int v = (int)seed;
        for (int i = 0; i < iters; ++i) v = v * 3 + 1;
        p = v;
    } else if (kMode == 5) {     // f32 fma chain
        float f = (float)p;
        for (int i = 0; i < iters; ++i) f = __builtin_fmaf(f, 0.999f, 1e-7f);
        p = f;
    }
    const uint64_t t1 = __builtin_readcyclecounter();
    out[threadIdx.x] = p;
    if (threadIdx.x == 0) cyc[0] = t1 - t0;
}

int main() {
    double* out;
    uint64_t* cyc;
    hipMalloc(&out, 64 * sizeof(double));
    hipMalloc(&cyc, sizeof(uint64_t));
    const int iters = 100000;
    const char* names[] = {"f64 fma chain", "f64 add chain", "DDM p row (5 ops)", "DDM p row x=0 (4 ops)",
                           "i32 mad chain", "f32 fma chain"};
    for (int mode = 0; mode < 6; ++mode) {
        for (int rep = 0; rep < 2; ++rep) {
            auto k = mode == 0 ? k_lat<0> : mode == 1 ? k_lat<1> : mode == 2 ? k_lat<2> : mode == 3 ? k_lat<3>
                   : mode == 4 ? k_lat<4> : k_lat<5>;
            hipEvent_t a, b;
            hipEventCreate(&a);
            hipEventCreate(&b);
            hipEventRecord(a);
            hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, out, cyc, iters, 0.5);
            hipEventRecord(b);
            hipEventSynchronize(b);
            float ms = 0;
            hipEventElapsedTime(&ms, a, b);
            uint64_t c = 0;
            hipMemcpy(&c, cyc, 8, hipMemcpyDeviceToHost);
            if (rep == 1)
                printf("%-24s %8.2f cycles/iter  %8.2f ns/iter (event)\n", names[mode], (double)c / iters,
                       ms * 1e6 / iters);
        }
    }
    return 0;
}
