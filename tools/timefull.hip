// tools/timefull.hip — times the fused guided-filter kernel (r=4, f32, N^3) only; used to compare
// builds of the same kernel with different compiler flags (not a product path).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "gf_fused_variants.hpp"

using namespace zt;

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { \
    printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

int main(int argc, char** argv) {
    int n = argc > 1 ? atoi(argv[1]) : 2048;
    const char* tag = argc > 2 ? argv[2] : "";
    size_t vox = (size_t)n * n * n;
    float *in, *out;
    CK(hipMalloc(&in, vox * 4)); CK(hipMalloc(&out, vox * 4));
    std::vector<float> h((size_t)n * n);
    for (size_t i = 0; i < h.size(); ++i) h[i] = (float)((i * 2654435761u) % 1000) * 0.1f;
    for (int z = 0; z < n; ++z) CK(hipMemcpy(in + (size_t)z * n * n, h.data(), h.size() * 4,
                                             hipMemcpyHostToDevice));
    GFParams p{};
    p.in = in; p.out = out; p.in_sz = (int64_t)n * n; p.in_sy = n; p.out_sz = (int64_t)n * n;
    p.out_sy = n; p.in_z0 = 0; p.zlo = 0; p.zhi = n; p.nz = p.ny = p.nx = n;
    p.oz0 = p.oy0 = p.ox0 = 0; p.onz = p.ony = p.onx = n; p.zseg = 256; p.eps = 2500.0f;
    hipStream_t s; CK(hipStreamCreate(&s));
    hipEvent_t a, b;
    CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
    std::vector<float> t;
    CK((launch_fused_cfg<4, 32, 1024, float, float>(p, s)));
    for (int r = 0; r < 5; ++r) {
        CK(hipEventRecord(a, s));
        CK((launch_fused_cfg<4, 32, 1024, float, float>(p, s)));
        CK(hipEventRecord(b, s));
        CK(hipEventSynchronize(b));
        float ms; CK(hipEventElapsedTime(&ms, a, b));
        t.push_back(ms);
    }
    std::sort(t.begin(), t.end());
    printf("%-24s median %8.3f ms  min %8.3f ms\n", tag, t[2], t[0]);
    return 0;
}
