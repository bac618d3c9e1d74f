// Measurement aid (not product code): how many HBM bytes and how much time a read of only
// the HEAD of every 100-row batch of configs[3]'s error streams costs against streaming all
// of them.  The DDM consumes a batch only up to its change (DDM_Process.py:150-152), on
// C4 13.6 % of the rows; whether reading less pays depends on the granularity at which
// the L2 fetches from HBM (32 / 64 / 128 B), which this measures.
//   hipcc --offload-arch=gfx950 -O3 tools/skipread_bench.hip -o tools/skipread_bench
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <cstdlib>

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

__global__ void k_fill(uint8_t* p, int64_t n) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n / 4; i += (int64_t)gridDim.x * blockDim.x) {
        uint64_t z = (uint64_t)i * 0x9E3779B97F4A7C15ull;
        z ^= z >> 29; z *= 0xBF58476D1CE4E5B9ull; z ^= z >> 32;
        uint32_t w = 0;
        for (int k = 0; k < 4; ++k) w |= (uint32_t)(((z >> (8 * k)) & 0xff) < 26) << (8 * k);
        reinterpret_cast<uint32_t*>(p)[i] = w;
    }
}

// every byte, coalesced 16-B loads, grid-stride
__global__ __launch_bounds__(256) void k_stream(const u32x4* __restrict__ p, int64_t n16, uint32_t* out) {
    uint32_t acc = 0;
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n16; i += (int64_t)gridDim.x * 256) {
        const u32x4 v = __builtin_nontemporal_load(p + i);
        acc ^= v.x ^ v.y ^ v.z ^ v.w;
    }
    if (acc == 0x12345678u) out[0] = acc;
}

// the first NCH 16-B chunks of every batch, one lane per batch (batches 100 B apart)
template <int NCH>
__global__ __launch_bounds__(256) void k_heads(const uint8_t* __restrict__ p, int64_t n_streams, int L, int pb, int nb,
                                               uint32_t* out) {
    uint32_t acc = 0;
    const int64_t nbt = n_streams * nb;
    for (int64_t b = (int64_t)blockIdx.x * 256 + threadIdx.x; b < nbt; b += (int64_t)gridDim.x * 256) {
        const int64_t s = b / nb;
        const int j = (int)(b - s * nb);
        const int64_t st = s * L + (int64_t)j * pb;
        const u32x4* c = reinterpret_cast<const u32x4*>(p + (st & ~(int64_t)15));
#pragma unroll
        for (int k = 0; k < NCH; ++k) {
            const u32x4 v = __builtin_nontemporal_load(c + k);
            acc ^= v.x ^ v.y ^ v.z ^ v.w;
        }
    }
    if (acc == 0x12345678u) out[0] = acc;
}

int main(int argc, char** argv) {
    const int64_t S = argc > 1 ? atoll(argv[1]) : 1000000;
    const int L = 4096, pb = 100, nb = (L + pb - 1) / pb;
    const int64_t n = S * L;
    uint8_t* p;
    uint32_t* out;
    CK(hipMalloc(&p, n + 64));
    CK(hipMalloc(&out, 64));
    hipLaunchKernelGGL(k_fill, dim3(8192), dim3(256), 0, 0, p, n);
    CK(hipDeviceSynchronize());
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    int dev = 0, cus = 256;
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
    const char* names[] = {"stream_all", "heads_16B", "heads_32B", "heads_48B", "heads_64B", "heads_112B"};
    for (int kind = 0; kind < 6; ++kind) {
        for (int grid_mul : {8, 32}) {
            float best = 1e30f, tot = 0;
            const int reps = 6;
            for (int r = 0; r < reps; ++r) {
                CK(hipEventRecord(a, 0));
                const dim3 g(cus * grid_mul), t(256);
                switch (kind) {
                    case 0: hipLaunchKernelGGL(k_stream, g, t, 0, 0, reinterpret_cast<const u32x4*>(p), n / 16, out); break;
                    case 1: hipLaunchKernelGGL(k_heads<1>, g, t, 0, 0, p, S, L, pb, nb, out); break;
                    case 2: hipLaunchKernelGGL(k_heads<2>, g, t, 0, 0, p, S, L, pb, nb, out); break;
                    case 3: hipLaunchKernelGGL(k_heads<3>, g, t, 0, 0, p, S, L, pb, nb, out); break;
                    case 4: hipLaunchKernelGGL(k_heads<4>, g, t, 0, 0, p, S, L, pb, nb, out); break;
                    case 5: hipLaunchKernelGGL(k_heads<7>, g, t, 0, 0, p, S, L, pb, nb, out); break;
                }
                CK(hipEventRecord(b, 0));
                CK(hipEventSynchronize(b));
                float ms = 0;
                CK(hipEventElapsedTime(&ms, a, b));
                if (r > 0) { tot += ms; if (ms < best) best = ms; }
            }
            printf("%-11s grid=%4dxCU  best %.4f ms  avg %.4f ms  nominal %.2f TB/s\n", names[kind], grid_mul, best,
                   tot / (reps - 1), (double)n / (best * 1e-3) / 1e12);
        }
    }
    CK(hipFree(p));
    return 0;
}
