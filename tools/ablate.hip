// tools/ablate.hip — timing-only ablations of the fused guided-filter kernel (not a product path).
// Builds variants of gf3d_fused_kernel<4, 32, 1024, float, float, ABL> and times each on an
// N^3 f32 volume with interleaved rounds in one process (cdna_hip_programming.md §5.4 rule 24).
// Variants with ABL != 0 compute wrong results on purpose.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "gf_fused_variants.hpp"

using namespace zt;

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { \
    printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

template <int ABL>
float run(const GFParams& p, hipStream_t s, int reps) {
    hipEvent_t a, b;
    CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
    CK((launch_fused_cfg<4, 32, 1024, float, float, ABL>(p, s)));
    CK(hipEventRecord(a, s));
    for (int i = 0; i < reps; ++i) CK((launch_fused_cfg<4, 32, 1024, float, float, ABL>(p, s)));
    CK(hipEventRecord(b, s));
    CK(hipEventSynchronize(b));
    float ms; CK(hipEventElapsedTime(&ms, a, b));
    return ms / reps;
}

int main(int argc, char** argv) {
    int n = argc > 1 ? atoi(argv[1]) : 1024;
    size_t vox = (size_t)n * n * n;
    float *in, *out;
    CK(hipMalloc(&in, vox * 4)); CK(hipMalloc(&out, vox * 4));
    std::vector<float> h((size_t)n * n);
    for (size_t i = 0; i < h.size(); ++i) h[i] = (float)((i * 2654435761u) % 1000) * 0.1f;
    for (int z = 0; z < n; ++z) CK(hipMemcpy(in + (size_t)z * n * n, h.data(), h.size() * 4,
                                             hipMemcpyHostToDevice));
    GFParams p{};
    p.in = in; p.out = out; p.in_sz = (int64_t)n * n; p.in_sy = n; p.out_sz = (int64_t)n * n;
    p.out_sy = n; p.in_z0 = 0; p.zlo = 0; p.zhi = n; p.nz = p.ny = p.nx = n; p.oz0 = p.oy0 = p.ox0 = 0;
    p.onz = p.ony = p.onx = n; p.zseg = 256; p.eps = 2500.0f;
    hipStream_t s; CK(hipStreamCreate(&s));
    const char* names[] = {"full", "no leave load (1)", "no Lc load (2)", "no v5 load (4)",
                           "no enter load (8)", "no loads (15)", "no barrier (16)",
                           "no pointwise (32)", "P5 1 LDS read (64)", "P4 1 LDS read (128)",
                           "P3 1 LDS read (256)", "no stage1 DPP (512)", "1-read P3+P4+P5 (448)", "no P12 (1024)",
                           "no P3 (2048)", "no P4 (4096)", "no P5 (8192)", "no P3,P4,P5", "nothing but loads/stores"};
    constexpr int NV = 19;
    std::vector<std::vector<float>> t(NV);
    for (int round = 0; round < 3; ++round) {
        t[0].push_back(run<0>(p, s, 3));
        t[1].push_back(run<1>(p, s, 3));
        t[2].push_back(run<2>(p, s, 3));
        t[3].push_back(run<4>(p, s, 3));
        t[4].push_back(run<8>(p, s, 3));
        t[5].push_back(run<15>(p, s, 3));
        t[6].push_back(run<16>(p, s, 3));
        t[7].push_back(run<32>(p, s, 3));
        t[8].push_back(run<64>(p, s, 3));
        t[9].push_back(run<128>(p, s, 3));
        t[10].push_back(run<256>(p, s, 3));
        t[11].push_back(run<512>(p, s, 3));
        t[12].push_back(run<448>(p, s, 3));
        t[13].push_back(run<1024>(p, s, 3));
        t[14].push_back(run<2048>(p, s, 3));
        t[15].push_back(run<4096>(p, s, 3));
        t[16].push_back(run<8192>(p, s, 3));
        t[17].push_back(run<2048 + 4096 + 8192>(p, s, 3));
        t[18].push_back(run<1024 + 2048 + 4096 + 8192>(p, s, 3));
    }
    for (int i = 0; i < NV; ++i) {
        std::sort(t[i].begin(), t[i].end());
        printf("%-30s median %8.3f ms  min %8.3f ms  (%.1f GB/s algorithmic)\n", names[i],
               t[i][1], t[i][0], vox * 8.0 / (t[i][1] * 1e-3) / 1e9);
    }
    return 0;
}
