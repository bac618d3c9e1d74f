// Measurement aid (not product code): the streaming front of a configs[3] scan -- 16-byte
// coalesced loads of 64-batch fills (100-row batches, 4096-row streams), folded to bits in
// an LDS image, every lane cutting its batch's 128 bits out and storing 8 bytes -- in the
// forms a redesigned ddm_scan_batches could take:
//   order:  fills grid-strided over the waves (a sweeping window) or each wave a contiguous
//           range of fills;
//   depth:  one fill in flight (loads issued after the image of the current fill) or two
//           (the next fill's loads issued before it);
//   waves:  per CU.
//   hipcc --offload-arch=gfx950 -O3 tools/fill_bench.hip -o tools/fill_bench
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>
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

__device__ __forceinline__ uint32_t fold16(u32x4 v) {
    const uint32_t lo = __builtin_amdgcn_udot4(v.y, 0x80402010u, __builtin_amdgcn_udot4(v.x, 0x08040201u, 0u, false), false);
    const uint32_t hi = __builtin_amdgcn_udot4(v.w, 0x80402010u, __builtin_amdgcn_udot4(v.z, 0x08040201u, 0u, false), false);
    return lo | (hi << 8);
}

struct Geo {       // batches [b0, b0 + 64): 64 consecutive batches of equal-length streams
    uint32_t a0;   // first 16-B chunk's byte (relative to the chunk base, 32-bit: < 4 GiB here)
    int64_t base;  // byte of chunk 0
    int o, blen, nch;
};

// b / nb by a 32-bit magic multiply (b < 2^31, nb < 2^16)
__device__ __forceinline__ uint32_t divnb(uint32_t b, uint32_t magic, int sh) { return __umulhi(b, magic) >> sh; }

__device__ __forceinline__ Geo geo(int64_t f, int64_t n_items, int L, int pb, int nb, uint32_t magic, int sh, int lane) {
    Geo g;
    const uint32_t b0 = (uint32_t)(f << 6);
    const uint32_t bl = min(b0 + (uint32_t)lane, (uint32_t)(n_items - 1));
    const uint32_t s = divnb(bl, magic, sh);
    const uint32_t j = bl - s * (uint32_t)nb;
    const int64_t start = (int64_t)s * L + (int64_t)j * pb;
    const int64_t st0 = (int64_t)(uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)(start)) |
                        ((int64_t)__builtin_amdgcn_readfirstlane((uint32_t)(start >> 32)) << 32);
    g.base = st0 & ~(int64_t)15;
    g.o = (int)(start - g.base);
    g.blen = min(pb, L - (int)j * pb);
    const int endl = __builtin_amdgcn_readlane(g.o + g.blen, 63);
    g.nch = (endl + 15) >> 4;
    return g;
}

template <int K>
__device__ __forceinline__ void loads(const uint8_t* __restrict__ p, const Geo& g, int lane, u32x4 (&v)[K]) {
#pragma unroll
    for (int k = 0; k < K; ++k)
        v[k] = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(p + g.base + 16 * min(k * 64 + lane, g.nch - 1)));
}

template <int K>
__device__ __forceinline__ void image_and_cut(const u32x4 (&v)[K], const Geo& g, int lane, uint64_t* img,
                                              uint64_t& m0, uint64_t& m1) {
    uint16_t* img16 = reinterpret_cast<uint16_t*>(img);
#pragma unroll
    for (int k = 0; k < K; ++k) img16[k * 64 + lane] = (uint16_t)fold16(v[k]);
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    const int wo = g.o >> 6, sh = g.o & 63;
    const uint64_t x0 = img[wo], x1 = img[wo + 1], x2 = img[wo + 2];
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    m0 = sh ? (x0 >> sh) | (x1 << (64 - sh)) : x0;
    m1 = sh ? (x1 >> sh) | (x2 << (64 - sh)) : x1;
}

// kOrder 0: grid-stride fills; 1: contiguous fill range per wave.  kDepth 1 or 2.
// kStore 0: no per-batch store (a data-dependent never-taken one); kImage 0: no LDS image
// (the loaded words xor-folded in registers)
template <int kOrder, int kDepth, int kStore = 1, int kImage = 1>
__global__ __launch_bounds__(256) void k_fills(const uint8_t* __restrict__ p, int64_t n_items, int L, int pb, int nb,
                                               uint32_t magic, int sh, int2* __restrict__ out) {
    constexpr int K = 7;
    __shared__ uint64_t img_all[4][K * 64 * 2 / 8 + 4];
    __shared__ int2 stage[4][4 * 64];
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    uint64_t* img = img_all[wv];
    const int64_t wave = (int64_t)blockIdx.x * 4 + wv, n_waves = (int64_t)gridDim.x * 4;
    const int64_t nfill = (n_items + 63) >> 6;
    int64_t f0, f1, step;
    if (kOrder == 0) {
        f0 = wave; f1 = nfill; step = n_waves;
    } else {
        const int64_t per = (nfill + n_waves - 1) / n_waves;
        f0 = wave * per; f1 = min(nfill, f0 + per); step = 1;
    }
    if (f0 >= f1) return;
    Geo g = geo(f0, n_items, L, pb, nb, magic, sh, lane);
    u32x4 v[K];
    loads<K>(p, g, lane, v);
    for (int64_t f = f0; f < f1; f += step) {
        const int64_t fn = min(f + step, f1 - 1);
        const Geo gn = geo(fn, n_items, L, pb, nb, magic, sh, lane);
        uint64_t m0, m1;
        if (!kImage) {
            uint32_t x = 0;
#pragma unroll
            for (int k = 0; k < K; ++k) x ^= v[k].x ^ v[k].y ^ v[k].z ^ v[k].w;
            m0 = x;
            m1 = g.o;
            loads<K>(p, gn, lane, v);
        } else if (kDepth == 2) {
            u32x4 w[K];
            loads<K>(p, gn, lane, w);
            image_and_cut<K>(v, g, lane, img, m0, m1);
#pragma unroll
            for (int k = 0; k < K; ++k) v[k] = w[k];
        } else {
            image_and_cut<K>(v, g, lane, img, m0, m1);
            loads<K>(p, gn, lane, v);
        }
        const int64_t b = (f << 6) + lane;
        if (kStore == 3) {
            // the wave's results of 4 consecutive fills staged in LDS, written as 2 KB by
            // 16-byte stores (range order: consecutive fills are consecutive batches)
            const int slot = (int)((f - f0) & 3);
            stage[wv][slot * 64 + lane] = make_int2((int)(m0 ^ m1), (int)((m0 ^ m1) >> 32));
            if (slot == 3 || f + 1 >= f1) {
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
                __builtin_amdgcn_wave_barrier();
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
                const int64_t fb = f - slot;
                const int4* st4 = reinterpret_cast<const int4*>(stage[wv]);
#pragma unroll
                for (int q = 0; q < 2; ++q) {
                    const int e = q * 64 + lane;           // int4 e = batches 2e, 2e + 1
                    const int64_t bb = (fb << 6) + 2 * e;
                    if (2 * e < (slot + 1) * 64 && bb + 1 < n_items)
                        reinterpret_cast<int4*>(out)[bb >> 1] = st4[e];
                }
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
                __builtin_amdgcn_wave_barrier();
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            }
        } else if (kStore == 5) {           // u8 per batch
            if (b < n_items) reinterpret_cast<uint8_t*>(out)[b] = (uint8_t)(m0 ^ m1);
        } else if (kStore == 6) {           // int2 per batch into a 64 KB L2-resident window
            if (b < n_items) out[b & 8191] = make_int2((int)(m0 ^ m1), (int)((m0 ^ m1) >> 32));
        } else if (kStore == 7) {           // int2 per batch, every other fill only
            if (b < n_items && (f & 1)) out[b] = make_int2((int)(m0 ^ m1), (int)((m0 ^ m1) >> 32));
        } else if (kStore == 4) {
            if (b < n_items) reinterpret_cast<uint16_t*>(out)[b] = (uint16_t)(m0 ^ m1);
        } else if (kStore == 2) {
            if (b < n_items) {
                __builtin_nontemporal_store((int)(m0 ^ m1), reinterpret_cast<int*>(out) + 2 * b);
                __builtin_nontemporal_store((int)((m0 ^ m1) >> 32), reinterpret_cast<int*>(out) + 2 * b + 1);
            }
        } else if (b < n_items && (kStore || (m0 ^ m1) == 0x1234567890abcdefull))
            out[b] = make_int2((int)(m0 ^ m1), (int)((m0 ^ m1) >> 32));
        g = gn;
    }
}

int main(int argc, char** argv) {
    const int64_t S = argc > 1 ? atoll(argv[1]) : 1000000;
    const int L = 4096, pb = 100, nb = (L + pb - 1) / pb;
    const int64_t n = S * L, n_items = S * nb;
    // magic for b / nb over every b < n_items: the largest shift whose multiplier fits 32 bits
    int shv = -1;
    uint32_t magic = 0;
    for (int s = 31; s >= 0 && shv < 0; --s) {
        const uint64_t m = (((uint64_t)1 << (32 + s)) + nb - 1) / nb;
        if (m >> 32) continue;
        bool ok = true;
        for (uint64_t b2 = 0; b2 < (uint64_t)n_items && ok; ++b2)
            ok = ((b2 * m) >> (32 + s)) == b2 / nb;
        if (ok) { shv = s; magic = (uint32_t)m; }
    }
    if (shv < 0) { printf("no magic\n"); return 1; }
    uint8_t* p;
    int2* out;
    CK(hipMalloc(&p, n + 256));
    CK(hipMalloc(&out, n_items * 8));
    hipLaunchKernelGGL(k_fill, dim3(8192), dim3(256), 0, 0, p, n);
    CK(hipDeviceSynchronize());
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    int cus = 256;
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    struct V { const char* name; void (*k)(const uint8_t*, int64_t, int, int, int, uint32_t, int, int2*); };
    V vs[] = {{"stride_d1", k_fills<0, 1>}, {"stride_u8store", k_fills<0, 1, 5>},
              {"stride_l2store", k_fills<0, 1, 6>}, {"stride_halfstore", k_fills<0, 1, 7>},
              {"stride_nostore", k_fills<0, 1, 0>}};
    for (const V& v : vs) {
        for (int wpc : {8, 16, 32}) {     // waves per CU
            const int blocks = cus * wpc / 4;
            float best = 1e30f, tot = 0;
            const int reps = 6;
            for (int r = 0; r < reps; ++r) {
                CK(hipEventRecord(a, 0));
                hipLaunchKernelGGL(v.k, dim3(blocks), dim3(256), 0, 0, p, n_items, L, pb, nb, magic, shv, out);
                CK(hipEventRecord(b, 0));
                CK(hipEventSynchronize(b));
                float ms = 0;
                CK(hipEventElapsedTime(&ms, a, b));
                if (r > 0) { tot += ms; if (ms < best) best = ms; }
            }
            printf("%-18s waves/CU=%2d  best %.4f ms  avg %.4f ms  %.2f TB/s (read+8B/batch)\n", v.name, wpc, best,
                   tot / (reps - 1), (double)(n + n_items * 8) / (best * 1e-3) / 1e12);
        }
    }
    return 0;
}
