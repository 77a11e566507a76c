// tools/timecfg.hip — times two tile configurations of gf3d_fused_kernel (64x32 tiles of 1024
// threads, one workgroup per CU, against 64x16 tiles of 512 threads, two per CU) on the same r=4
// f32 N^3 volume and compares their outputs. Not a product path.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "gf_fused_variants.hpp"

using namespace zt;

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { \
    printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

template <typename F>
static float time_it(F&& launch, hipStream_t s, int reps) {
    hipEvent_t a, b;
    CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
    CK(launch());
    CK(hipStreamSynchronize(s));
    std::vector<float> t;
    for (int r = 0; r < reps; ++r) {
        CK(hipEventRecord(a, s));
        CK(launch());
        CK(hipEventRecord(b, s));
        CK(hipEventSynchronize(b));
        float ms; CK(hipEventElapsedTime(&ms, a, b));
        t.push_back(ms);
    }
    std::sort(t.begin(), t.end());
    return t[t.size() / 2];
}

int main(int argc, char** argv) {
    const int n = argc > 1 ? atoi(argv[1]) : 2048;
    const int reps = argc > 2 ? atoi(argv[2]) : 5;
    const size_t vox = (size_t)n * n * n;
    float *in, *o8, *o9;
    CK(hipMalloc(&in, vox * 4)); CK(hipMalloc(&o8, vox * 4)); CK(hipMalloc(&o9, vox * 4));
    std::vector<float> h((size_t)n * n);
    for (int z = 0; z < n; ++z) {
        for (size_t i = 0; i < h.size(); ++i)
            h[i] = (float)(((i + (size_t)z * 7919u) * 2654435761u) % 1000) * 0.1f +
                   ((i % n) < (size_t)n / 2 ? 0.0f : 200.0f);
        CK(hipMemcpy(in + (size_t)z * n * n, h.data(), h.size() * 4, hipMemcpyHostToDevice));
    }
    GFParams p{};
    p.in = in; p.in_sz = (int64_t)n * n; p.in_sy = n; p.out_sz = (int64_t)n * n;
    p.out_sy = n; p.in_z0 = 0; p.zlo = 0; p.zhi = n; p.nz = p.ny = p.nx = n;
    p.oz0 = p.oy0 = p.ox0 = 0; p.onz = p.ony = p.onx = n; p.zseg = std::min(256, n);
    p.eps = 2500.0f;
    hipStream_t s; CK(hipStreamCreate(&s));
    GFParams p8 = p, p9 = p;
    p8.out = o8; p9.out = o9;
    const float t8 = time_it([&] { return launch_fused_cfg<4, 32, 1024, float, float>(p8, s); },
                             s, reps);
    const float t9 = time_it([&] { return launch_fused_cfg<4, 16, 512, float, float>(p9, s); },
                             s, reps);
    std::vector<float> a(vox), b(vox);
    CK(hipMemcpy(a.data(), o8, vox * 4, hipMemcpyDeviceToHost));
    CK(hipMemcpy(b.data(), o9, vox * 4, hipMemcpyDeviceToHost));
    double maxrel = 0.0;
    size_t same = 0, worst = 0;
    for (size_t i = 0; i < vox; ++i) {
        if (a[i] == b[i]) { ++same; continue; }
        const double d = std::fabs((double)a[i] - (double)b[i]) /
                         std::max(1.0, std::fabs((double)a[i]));
        if (!(d <= maxrel)) { maxrel = d; worst = i; }
    }
    const double gb = (double)vox * 8.0 / 1e9;
    printf("n=%d  64x32/1024 %8.3f ms (%6.1f GB/s)  64x16/512 %8.3f ms (%6.1f GB/s)  max rel diff %.3e at %zu "
           "(%g vs %g)  identical %.4f\n", n, t8, gb / (t8 / 1e3), t9, gb / (t9 / 1e3), maxrel,
           worst, a[worst], b[worst], (double)same / (double)vox);
    return maxrel <= 1e-5 ? 0 : 3;
}
