// Measurement aid (not product code): the predict's read pattern -- a workgroup's tile of
// 2,048 rows x 27 f32 feature columns, 4 rows per thread by 16-byte loads -- from the
// feature-major layout the partitions use (column f at X + f * ld, ld = 125M rows: the
// columns of one tile are 500 MB apart) against a tile-major one (a tile's 27 columns
// contiguous, 221 KB), same bytes, same loads.
//   hipcc --offload-arch=gfx950 -O3 tools/layout_bench.hip -o tools/layout_bench
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>
#include <cstdlib>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

constexpr int F = 27, TILE = 2048, THREADS = 512;
typedef float f32x4 __attribute__((ext_vector_type(4)));

// kTiled 0: X[f * ld + row]; 1: X[(tile * F + f) * TILE + row % TILE]
template <int kTiled>
__global__ __launch_bounds__(THREADS) void k_read(const float* __restrict__ X, int64_t ld, int64_t n_tiles,
                                                  int64_t tile0, float* out) {
    float acc = 0.f;
    for (int64_t t = tile0 + blockIdx.x; t < tile0 + n_tiles; t += gridDim.x) {
        const int r = 4 * threadIdx.x;
#pragma unroll 9
        for (int f = 0; f < F; ++f) {
            const float* p = kTiled ? X + ((t * F + f) * TILE + r) : X + (f * ld + t * TILE + r);
            const f32x4 v = __builtin_nontemporal_load(reinterpret_cast<const f32x4*>(p));
            acc += v.x + v.y + v.z + v.w;
        }
    }
    if (acc == 1.2345f) out[0] = acc;
}

__global__ void k_init(float* X, int64_t n) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
        X[i] = (float)(i & 1023);
}

int main() {
    const int64_t ld = 125000000;                       // rows per partition (C3)
    const int64_t n = (int64_t)F * ld;                 // 13.5 GB
    float* X;
    float* out;
    CK(hipMalloc(&X, n * 4));
    CK(hipMalloc(&out, 64));
    hipLaunchKernelGGL(k_init, dim3(8192), dim3(256), 0, 0, X, n);
    CK(hipDeviceSynchronize());
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    // a window of 1.15M rows (one C3 epoch's window of one partition) = 562 tiles, and a
    // launch-sized 9.2M rows = 4,492 tiles, each at several positions of the partition
    for (int64_t tiles : {(int64_t)562, (int64_t)4492}) {
        for (int kTiled = 0; kTiled < 2; ++kTiled) {
            for (int grid : {1024, 2048}) {
                float tot = 0;
                int cnt = 0;
                for (int rep = 0; rep < 8; ++rep) {
                    const int64_t t0 = (rep * 7919) % (ld / TILE - tiles);
                    CK(hipEventRecord(a, 0));
                    if (kTiled) hipLaunchKernelGGL(k_read<1>, dim3(grid), dim3(THREADS), 0, 0, X, ld, tiles, t0, out);
                    else hipLaunchKernelGGL(k_read<0>, dim3(grid), dim3(THREADS), 0, 0, X, ld, tiles, t0, out);
                    CK(hipEventRecord(b, 0));
                    CK(hipEventSynchronize(b));
                    float ms = 0;
                    CK(hipEventElapsedTime(&ms, a, b));
                    if (rep > 0) { tot += ms; ++cnt; }
                }
                const double bytes = (double)tiles * TILE * F * 4;
                printf("tiles=%5ld %-13s grid=%4d  %.4f ms  %.2f TB/s\n", (long)tiles, kTiled ? "tile-major" : "feature-major",
                       grid, tot / cnt, bytes / (tot / cnt * 1e-3) / 1e12);
            }
        }
    }
    return 0;
}
