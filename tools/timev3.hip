// tools/timev3.hip — A/B harness for the third fused guided-filter design (gf_v3.hpp) against the
// round-2 kernel (gf_fused.hpp): times both on an N^3 f32 volume (r = 4 or 2, the bench's
// step + noise shape) and compares their outputs on sampled slices (not a product path).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "gf_v3.hpp"

using namespace zt;
#ifndef TV_R
#define TV_R 4
#endif

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { \
    printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

template <typename F>
static float time_it(F f, hipStream_t s, int reps, std::vector<float>& all) {
    hipEvent_t a, b;
    CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
    CK(f());
    CK(hipStreamSynchronize(s));
    for (int r = 0; r < reps; ++r) {
        CK(hipEventRecord(a, s));
        CK(f());
        CK(hipEventRecord(b, s));
        CK(hipEventSynchronize(b));
        float ms; CK(hipEventElapsedTime(&ms, a, b));
        all.push_back(ms);
    }
    std::sort(all.begin(), all.end());
    return all[all.size() / 2];
}

int main(int argc, char** argv) {
    const int n = argc > 1 ? atoi(argv[1]) : 2048;
    const int zseg = argc > 2 ? atoi(argv[2]) : 512;
    const int which = argc > 3 ? atoi(argv[3]) : 3;  // 1: old only, 2: new only, 3: both
    const size_t vox = (size_t)n * n * n;
    float *in, *o1, *o2;
    CK(hipMalloc(&in, vox * 4)); CK(hipMalloc(&o1, vox * 4)); CK(hipMalloc(&o2, vox * 4));
    std::vector<float> h((size_t)n * n);
    for (int z = 0; z < n; ++z) {
        for (size_t i = 0; i < h.size(); ++i)
            h[i] = (float)(((i + (size_t)z * 7919u) * 2654435761u) % 1000) * 0.1f +
                   ((i % n) < (size_t)n / 2 ? 0.0f : 500.0f);
        CK(hipMemcpy(in + (size_t)z * n * n, h.data(), h.size() * 4, hipMemcpyHostToDevice));
    }
    GFParams p{};
    p.in = in; p.in_sz = (int64_t)n * n; p.in_sy = n; p.out_sz = (int64_t)n * n;
    p.out_sy = n; p.in_z0 = 0; p.zlo = 0; p.zhi = n; p.nz = p.ny = p.nx = n;
    p.oz0 = p.oy0 = p.ox0 = 0; p.onz = p.ony = p.onx = n; p.zseg = zseg; p.eps = 2500.0f;
    hipStream_t s; CK(hipStreamCreate(&s));
    std::vector<float> t1, t2;
    float m1 = 0, m2 = 0;
    if (which & 1) {
        GFParams q = p; q.out = o1;
        m1 = time_it([&] { return launch_fused_cfg<TV_R, 32, 1024, float, float>(q, s); }, s, 5, t1);
    }
    if (which & 2) {
        GFParams q = p; q.out = o2;
        m2 = time_it([&] { return launch_v3_cfg<TV_R, float, float>(q, s); }, s, 5, t2);
    }
    printf("n=%d r=%d zseg=%d  old median %8.3f ms (min %8.3f)  v3 median %8.3f ms (min %8.3f)\n",
           n, TV_R, zseg, m1, which & 1 ? t1[0] : 0.f, m2, which & 2 ? t2[0] : 0.f);
    if (which == 3) {
        std::vector<float> a((size_t)n * n), b((size_t)n * n);
        double maxrel = 0.0; size_t ndiff = 0, ntot = 0;
        for (int z : {0, 1, 4, 5, n / 2, n - 5, n - 1}) {
            CK(hipMemcpy(a.data(), o1 + (size_t)z * n * n, a.size() * 4, hipMemcpyDeviceToHost));
            CK(hipMemcpy(b.data(), o2 + (size_t)z * n * n, b.size() * 4, hipMemcpyDeviceToHost));
            for (size_t i = 0; i < a.size(); ++i) {
                const double d = std::fabs((double)a[i] - (double)b[i]) / std::max(1.0, std::fabs((double)a[i]));
                if (!(d <= maxrel)) maxrel = std::isnan(d) ? 1e30 : std::max(maxrel, d);
                ndiff += a[i] != b[i];
                ++ntot;
            }
        }
        printf("compare: max rel diff %.3e, %.2f %% of sampled voxels differ\n", maxrel,
               100.0 * ndiff / ntot);
    }
    return 0;
}
