// Synthetic benchmark inputs generated in HBM.
//
// rialto.csv is not shipped (.MISSING_LARGE_BLOBS:1), so the rialto-shaped streams
// are synthetic: class blocks (sorted by class as DDM_Process.py:51 leaves the
// stream), partitioned row % n_parts (DDM_Process.py:225), with noise-free separable
// features so every class change is one abrupt drift.  All values come from a
// counter hash, so any row can be regenerated independently (and on any GPU count).
#include "common.h"

namespace {

__device__ __forceinline__ uint64_t mix64(uint64_t z) {
    z += 0x9e3779b97f4a7c15ull;
    z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
    z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
    return z ^ (z >> 31);
}

__device__ __forceinline__ double unit(uint64_t seed, uint64_t a, uint64_t b) {
    const uint64_t h = mix64(seed ^ mix64(a * 0x2545f4914f6cdd1dull + b));
    return (double)(h >> 11) * 0x1.0p-53;
}

__global__ __launch_bounds__(256) void k_block_labels(int32_t* __restrict__ y, int64_t n, int64_t part,
                                                      int64_t n_parts, int64_t block_rows, int n_classes) {
    for (int64_t r = (int64_t)blockIdx.x * 256 + threadIdx.x; r < n; r += (int64_t)gridDim.x * 256) {
        const int64_t g = r * n_parts + part;
        y[r] = (int32_t)((g / block_rows) % n_classes);
    }
}

// configs[4] (C5): class blocks whose global boundaries sit at k*period + jitter_k,
// jitter_k ~ U[-jitter, jitter] (jitter_0 = 0, jitter < period/2), block k of class
// k % n_classes, and each label flipped to another class with probability flip.  A row's
// block is found from its own boundary neighbourhood, so any row regenerates alone.
__device__ __forceinline__ int64_t jit_boundary(uint64_t seed, int64_t k, int64_t period, int64_t jitter) {
    if (k <= 0 || jitter == 0) return k * period;
    const int64_t j = (int64_t)(unit(seed, (uint64_t)k, 0xb10c0001ull) * (double)(2 * jitter + 1)) - jitter;
    return k * period + j;
}

__global__ __launch_bounds__(256) void k_jitter_labels(int32_t* __restrict__ y, int64_t n, int64_t part,
                                                       int64_t n_parts, int64_t period, int64_t jitter,
                                                       int n_classes, double flip, uint64_t seed) {
    for (int64_t r = (int64_t)blockIdx.x * 256 + threadIdx.x; r < n; r += (int64_t)gridDim.x * 256) {
        const int64_t g = r * n_parts + part;
        int64_t k = g / period;
        if (g < jit_boundary(seed, k, period, jitter)) --k;
        else if (g >= jit_boundary(seed, k + 1, period, jitter)) ++k;
        int c = (int)(k % n_classes);
        if (flip > 0.0 && n_classes > 1 && unit(seed ^ 0x7f4a7c15ull, (uint64_t)g, 0xf119ull) < flip)
            c = (c + 1 + (int)(unit(seed ^ 0x7f4a7c15ull, (uint64_t)g, 0xf11aull) * (n_classes - 1))) % n_classes;
        y[r] = c;
    }
}

// base(c, f) in {0.05, 0.15, ..., 0.95}: for classes c != c' (mod 10) every feature
// differs by >= 0.1 while the noise stays below 0.05, so classes are separable on
// every feature.
__global__ __launch_bounds__(256) void k_features(float* __restrict__ X, int64_t ld, int F,
                                                  const int32_t* __restrict__ y, int64_t n, int64_t row0,
                                                  int64_t row_stride, uint64_t seed, float noise) {
    for (int64_t r = (int64_t)blockIdx.x * 256 + threadIdx.x; r < n; r += (int64_t)gridDim.x * 256) {
        const int c = y[r];
        const uint64_t g = (uint64_t)(row0 + r * row_stride);
        for (int f = 0; f < F; ++f) {
            const float base = 0.05f + 0.1f * (float)((c * 7 + f * 3) % 10);
            X[(int64_t)f * ld + r] = base + noise * (float)unit(seed, g, (uint64_t)f);
        }
    }
}

__global__ __launch_bounds__(256) void k_bernoulli(uint8_t* __restrict__ err, int64_t n_streams, int64_t len,
                                                   uint64_t seed) {
    const int64_t s = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (s >= n_streams) return;
    const double r0 = 0.01 + 0.19 * unit(seed, (uint64_t)s, 0xffff0001ull);
    const double r1 = r0 + 0.05 + 0.25 * unit(seed, (uint64_t)s, 0xffff0002ull);
    const int64_t tau = (int64_t)(unit(seed, (uint64_t)s, 0xffff0003ull) * (double)len);
    uint8_t* out = err + s * len;
    for (int64_t i = 0; i < len; i += 4) {
        uint32_t w = 0;
        for (int k = 0; k < 4 && i + k < len; ++k) {
            const double u = unit(seed ^ 0x5bd1e995ull, (uint64_t)s, (uint64_t)(i + k));
            w |= (uint32_t)(u < (i + k < tau ? r0 : r1)) << (8 * k);
        }
        if (i + 4 <= len && ((len & 3) == 0))
            *reinterpret_cast<uint32_t*>(out + i) = w;
        else
            for (int k = 0; k < 4 && i + k < len; ++k) out[i + k] = (uint8_t)((w >> (8 * k)) & 1);
    }
}

}  // namespace

extern "C" int ddm_synth_block_labels(int32_t* y, int64_t n_rows, int64_t part, int64_t n_parts, int64_t block_rows,
                                      int32_t n_classes, ddm_stream_t stream) {
    if (!y || n_rows < 0 || n_parts <= 0 || part < 0 || part >= n_parts || block_rows <= 0 || n_classes <= 0) {
        ddm::set_error("ddm_synth_block_labels: invalid argument");
        return DDM_E_ARG;
    }
    if (n_rows == 0) return 0;
    const int64_t blocks = std::min<int64_t>(ddm::ceil_div(n_rows, 256), 4096);
    hipLaunchKernelGGL(k_block_labels, dim3((unsigned)blocks), dim3(256), 0, ddm::as_hip(stream), y, n_rows, part,
                       n_parts, block_rows, (int)n_classes);
    return ddm::launch_status("ddm_synth_block_labels");
}

extern "C" int ddm_synth_jitter_labels(int32_t* y, int64_t n_rows, int64_t part, int64_t n_parts, int64_t period,
                                       int64_t jitter, int32_t n_classes, double flip, uint64_t seed,
                                       ddm_stream_t stream) {
    if (!y || n_rows < 0 || n_parts <= 0 || part < 0 || part >= n_parts || period <= 0 || jitter < 0 ||
        2 * jitter >= period || n_classes <= 0 || !(flip >= 0.0 && flip <= 1.0)) {
        ddm::set_error("ddm_synth_jitter_labels: invalid argument");
        return DDM_E_ARG;
    }
    if (n_rows == 0) return 0;
    const int64_t blocks = std::min<int64_t>(ddm::ceil_div(n_rows, 256), 4096);
    hipLaunchKernelGGL(k_jitter_labels, dim3((unsigned)blocks), dim3(256), 0, ddm::as_hip(stream), y, n_rows, part,
                       n_parts, period, jitter, (int)n_classes, flip, seed);
    return ddm::launch_status("ddm_synth_jitter_labels");
}

extern "C" int ddm_synth_features(float* X, int64_t ld, int32_t n_features, const int32_t* y, int64_t n_rows,
                                  int64_t row0, int64_t row_stride, uint64_t seed, float noise, ddm_stream_t stream) {
    if (!X || !y || n_rows < 0 || ld < n_rows || n_features <= 0) {
        ddm::set_error("ddm_synth_features: invalid argument");
        return DDM_E_ARG;
    }
    if (n_rows == 0) return 0;
    const int64_t blocks = std::min<int64_t>(ddm::ceil_div(n_rows, 256), 8192);
    hipLaunchKernelGGL(k_features, dim3((unsigned)blocks), dim3(256), 0, ddm::as_hip(stream), X, ld, (int)n_features,
                       y, n_rows, row0, row_stride, seed, noise);
    return ddm::launch_status("ddm_synth_features");
}

extern "C" int ddm_synth_bernoulli_streams(uint8_t* err, int64_t n_streams, int64_t len, uint64_t seed,
                                           ddm_stream_t stream) {
    if (!err || n_streams < 0 || len < 0) {
        ddm::set_error("ddm_synth_bernoulli_streams: invalid argument");
        return DDM_E_ARG;
    }
    if (n_streams == 0 || len == 0) return 0;
    hipLaunchKernelGGL(k_bernoulli, dim3((unsigned)ddm::ceil_div(n_streams, 256)), dim3(256), 0,
                       ddm::as_hip(stream), err, n_streams, len, seed);
    return ddm::launch_status("ddm_synth_bernoulli_streams");
}
