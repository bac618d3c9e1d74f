// Which CUs a CU-masked stream's workgroups run on (developer tool, round 6): every
// workgroup's first lane stores its HW_ID and XCC_ID registers; the host counts the
// distinct (XCC, SE, SH, CU) slots for a plain stream and for ddm_stream_create_cu_stride
// streams of stride 2, 4, 8.
//   hipcc --offload-arch=gfx950 -O2 -I include tools/cu_probe.hip \
//     -L distributed-drift-detection_amd/ddm_amd -lddm_amd -Wl,-rpath,... -o tools/cu_probe
#include <hip/hip_runtime.h>

#include <cstdio>
#include <set>
#include <tuple>
#include <vector>

#include "ddm_amd.h"

__global__ void k_probe(uint32_t* out, int spin) {
    if (threadIdx.x == 0) {
        const uint32_t hw = __builtin_amdgcn_s_getreg((31 << 11) | (0 << 6) | 4);    // HW_REG_HW_ID
        const uint32_t xcc = __builtin_amdgcn_s_getreg((31 << 11) | (0 << 6) | 20);  // HW_REG_XCC_ID
        out[2 * blockIdx.x] = hw;
        out[2 * blockIdx.x + 1] = xcc;
    }
    const long long t0 = clock64();
    while (clock64() - t0 < spin) {
    }
}

int main() {
    const int n = 8192;
    uint32_t* d = nullptr;
    if (hipMalloc(&d, 2 * n * sizeof(uint32_t)) != hipSuccess) return 1;
    std::vector<uint32_t> h(2 * n);
    for (int stride : {1, 2, 4, 8}) {
        hipStream_t s = nullptr;
        int ncu = 0;
        if (stride == 1) {
            if (hipStreamCreate(&s) != hipSuccess) return 1;
        } else {
            ddm_stream_t raw = nullptr;
            if (ddm_stream_create_cu_stride(stride, 0, &raw, &ncu) != 0) {
                printf("stride %d: %s\n", stride, ddm_last_error());
                return 1;
            }
            s = reinterpret_cast<hipStream_t>(raw);
        }
        hipLaunchKernelGGL(k_probe, dim3(n), dim3(64), 0, s, d, 20000);
        if (hipStreamSynchronize(s) != hipSuccess) return 1;
        if (hipMemcpy(h.data(), d, 2 * n * sizeof(uint32_t), hipMemcpyDeviceToHost) != hipSuccess) return 1;
        std::set<std::tuple<int, int, int, int>> cus;
        std::set<int> xccs;
        for (int b = 0; b < n; ++b) {
            const uint32_t hw = h[2 * b], xcc = h[2 * b + 1] & 0xf;
            cus.insert({(int)xcc, (int)((hw >> 13) & 7), (int)((hw >> 12) & 1), (int)((hw >> 8) & 15)});
            xccs.insert((int)xcc);
        }
        printf("{\"stride\": %d, \"mask_cus\": %d, \"distinct_cus\": %zu, \"xccs\": %zu}\n", stride, ncu, cus.size(),
               xccs.size());
        hipStreamDestroy(s);
    }
    hipFree(d);
    return 0;
}
