// tools/timepyr.hip — times 2x2x2 mean pyramid levels 1-3 of an N^3 u16 volume (the bench's
// config P level 0): the product's per-level launches (launch_downsample), the product's fused
// launch (launch_pyramid_fused) and the experimental variants of tools/pyr_variants.hpp, and
// checks that every variant's levels equal the per-level ones bit for bit (not a product path).
//   tools/timepyr N [variant ...]   variants: perlevel fused v<INT><GZ>  e.g. v0_64 v1_512
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "../zarrs_tools_amd/csrc/zt_device.hpp"
#include "../zarrs_tools_amd/csrc/zt_kernels.hpp"
#include "pyr_variants.hpp"

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { \
    printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

__global__ void count_diff(const uint16_t* x, const uint16_t* y, size_t n,
                           unsigned long long* bad) {
    unsigned long long c = 0;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n;
         i += (size_t)gridDim.x * blockDim.x)
        c += x[i] != y[i];
    if (c) atomicAdd(bad, c);
}

int main(int argc, char** argv) {
    const int64_t n = argc > 1 ? atoll(argv[1]) : 4096;
    int64_t sh[4][3];
    for (int l = 0; l < 4; ++l)
        for (int d = 0; d < 3; ++d) sh[l][d] = n >> l;
    size_t numel[4];
    uint16_t* buf[4];
    for (int l = 0; l < 4; ++l) {
        numel[l] = (size_t)sh[l][0] * sh[l][1] * sh[l][2];
        CK(hipMalloc(&buf[l], numel[l] * 2));
    }
    hipStream_t s;
    CK(hipStreamCreate(&s));
    CK(zt::launch_synth_u16(buf[0], (int64_t)numel[0], n * n, 0, 0x5EED2025ull, s));
    CK(hipStreamSynchronize(s));
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));

    auto perlevel = [&]() {
        for (int l = 0; l < 3; ++l) {
            zt::DSParams p{};
            p.ndim = 3;
            p.out_numel = (int64_t)numel[l + 1];
            p.win_numel = 8;
            for (int d = 0; d < 3; ++d) {
                p.in_shape[d] = sh[l][d];
                p.out_shape[d] = sh[l + 1][d];
                p.win[d] = 2;
            }
            CK(zt::launch_downsample(buf[l], zt::kU16, buf[l + 1], zt::kU16, p, false, s));
        }
    };
    perlevel();
    CK(hipStreamSynchronize(s));
    uint16_t* ref[4] = {nullptr, nullptr, nullptr, nullptr};
    for (int l = 1; l < 4; ++l) {
        CK(hipMalloc(&ref[l], numel[l] * 2));
        CK(hipMemcpy(ref[l], buf[l], numel[l] * 2, hipMemcpyDeviceToDevice));
    }
    unsigned long long* bad;
    CK(hipMalloc(&bad, 8));
    const double bytes = 2.0 * (numel[0] + numel[1] + numel[2] + numel[3]);

    for (int vi = 2; vi < argc; ++vi) {
        const std::string v = argv[vi];
        for (int l = 1; l < 4; ++l) CK(hipMemsetAsync(buf[l], 0xA5, numel[l] * 2, s));
        auto run = [&]() {
            if (v == "perlevel") {
                perlevel();
            } else if (v == "fused") {
                void* outs[3] = {buf[1], buf[2], buf[3]};
                CK(zt::launch_pyramid_fused(buf[0], zt::kU16, sh, 3, outs, s));
            } else {
                int im = 0, gz = 65535;
                sscanf(v.c_str(), "v%d_%d", &im, &gz);
                CK(pyrv::launch(buf[0], buf[1], buf[2], buf[3], sh, im, gz, s));
            }
        };
        run();
        CK(hipStreamSynchronize(s));
        CK(hipMemset(bad, 0, 8));
        for (int l = 1; l < 4; ++l)
            hipLaunchKernelGGL(count_diff, dim3(8192), dim3(256), 0, s, buf[l], ref[l], numel[l], bad);
        unsigned long long nbad = 0;
        CK(hipMemcpy(&nbad, bad, 8, hipMemcpyDeviceToHost));
        const bool ok = nbad == 0;
        std::vector<float> t;
        for (int r = 0; r < 5; ++r) {
            CK(hipEventRecord(a, s));
            run();
            CK(hipEventRecord(b, s));
            CK(hipEventSynchronize(b));
            float ms;
            CK(hipEventElapsedTime(&ms, a, b));
            t.push_back(ms);
        }
        std::sort(t.begin(), t.end());
        printf("%-12s median %8.3f ms  min %8.3f ms  %7.1f GB/s  levels %s\n", v.c_str(), t[2], t[0],
               bytes / (t[2] * 1e6), ok ? "identical" : "DIFFER");
        fflush(stdout);
    }
    return 0;
}
