// tools/timeg4.hip — times the fused 4-D guided-filter kernel (g4_fused.hip, r=2, f32,
// (4, N, N, N)) and prints a checksum, so builds with compile-time geometry flags (-DG4_KX2=...)
// can be compared (not a product path; the round-2 load ablations, profiles/r02_ab_harness.txt,
// are no longer in the product source). Build: tools/timeg4.sh build NAME "-DFLAGS"...
#include "../zarrs_tools_amd/csrc/g4_fused.hip"

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { \
    printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

int main(int argc, char** argv) {
    const int n = argc > 1 ? atoi(argv[1]) : 1024;
    const char* tag = argc > 2 ? argv[2] : "";
    const int T = 4;
    const size_t vox = (size_t)T * n * n * n;
    float *in, *out;
    CK(hipMalloc(&in, vox * 4));
    CK(hipMalloc(&out, vox * 4));
    std::vector<float> h((size_t)n * n);
    for (int s = 0; s < T * n; ++s) {
        for (size_t i = 0; i < h.size(); ++i)
            h[i] = (float)(((i + (size_t)s * 7919u) * 2654435761u) % 1000) * 0.1f +
                   ((i % n) < (size_t)n / 2 ? 0.0f : 500.0f);
        CK(hipMemcpy(in + (size_t)s * n * n, h.data(), h.size() * 4, hipMemcpyHostToDevice));
    }
    zt::NdGeom g{};
    g.ndim = 4;
    const int64_t sh[4] = {T, n, n, n};
    int64_t st = 1;
    for (int d = 3; d >= 0; --d) {
        g.shape[d] = sh[d];
        g.in_strides[d] = st;
        g.out_strides[d] = st;
        g.out_start[d] = 0;
        g.out_shape[d] = sh[d];
        st *= sh[d];
    }
    g.numel = g.out_numel = (int64_t)vox;
    hipStream_t s;
    CK(hipStreamCreate(&s));
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    CK(zt::launch_guided4d_fused(in, out, zt::kF32, g, 2, 2500.0f, s));
    std::vector<float> t;
    for (int r = 0; r < 5; ++r) {
        CK(hipEventRecord(a, s));
        CK(zt::launch_guided4d_fused(in, out, zt::kF32, g, 2, 2500.0f, s));
        CK(hipEventRecord(b, s));
        CK(hipEventSynchronize(b));
        float ms;
        CK(hipEventElapsedTime(&ms, a, b));
        t.push_back(ms);
    }
    std::sort(t.begin(), t.end());
    double sum = 0.0;
    for (int z : {0, 3, n / 2, n - 1}) {
        CK(hipMemcpy(h.data(), out + (size_t)z * n * n, h.size() * 4, hipMemcpyDeviceToHost));
        for (float v : h) sum += v;
    }
    printf("%-24s median %8.3f ms  min %8.3f ms  checksum %.9e\n", tag, t[2], t[0], sum);
    return 0;
}
