// tools/trace_steps.hip — s_memtime stamps of one workgroup's march (ABL 16384): for 18 steps and
// 16 waves, the cycle at which each wave enters C0, finishes issuing C0, enters C1 and finishes
// issuing C1. Prints per-interval spans and the per-wave arrival skew (not a product path).
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
    int blk = argc > 2 ? atoi(argv[2]) : 3000;
    size_t vox = (size_t)n * n * n;
    float *in, *out;
    unsigned long long* tr;
    CK(hipMalloc(&in, vox * 4)); CK(hipMalloc(&out, vox * 4));
    CK(hipMalloc(&tr, 18 * 16 * 8 * 8));
    CK(hipMemset(tr, 0, 18 * 16 * 8 * 8));
    std::vector<float> h((size_t)n * n);
    for (size_t i = 0; i < h.size(); ++i) h[i] = (float)((i * 2654435761u) % 1000) * 0.1f;
    for (int z = 0; z < n; ++z) CK(hipMemcpy(in + (size_t)z * n * n, h.data(), h.size() * 4,
                                             hipMemcpyHostToDevice));
    GFParams p{};
    p.in = in; p.out = out; p.in_sz = (int64_t)n * n; p.in_sy = n; p.out_sz = (int64_t)n * n;
    p.out_sy = n; p.in_z0 = 0; p.zlo = 0; p.zhi = n; p.nz = p.ny = p.nx = n;
    p.oz0 = p.oy0 = p.ox0 = 0; p.onz = p.ony = p.onx = n; p.zseg = 256; p.eps = 2500.0f;
    p.trace = tr; p.trace_block = blk;
    hipStream_t s; CK(hipStreamCreate(&s));
    CK((launch_fused_cfg<4, 32, 1024, float, float, 16384>(p, s)));
    CK(hipStreamSynchronize(s));
    std::vector<unsigned long long> t(18 * 16 * 8);
    CK(hipMemcpy(t.data(), tr, t.size() * 8, hipMemcpyDeviceToHost));
    double c0 = 0, c1 = 0, w0 = 0, w1 = 0;
    std::vector<double> fin0(16), fin1(16), p3(16), p12s(16), p12e(16);
    for (int st = 0; st + 1 < 18; ++st) {
        auto T = [&](int w, int k) { return (double)t[(st * 16 + w) * 8 + k]; };
        auto Tn = [&](int w, int k) { return (double)t[((st + 1) * 16 + w) * 8 + k]; };
        double s0 = 1e30, e0 = 0, s1 = 1e30, e1 = 0, s0n = 1e30;
        for (int w = 0; w < 16; ++w) {
            s0 = std::min(s0, T(w, 0)); e0 = std::max(e0, T(w, 1));
            s1 = std::min(s1, T(w, 2)); e1 = std::max(e1, T(w, 3));
            s0n = std::min(s0n, Tn(w, 0));
        }
        c0 += s1 - s0; c1 += s0n - s1;
        for (int w = 0; w < 16; ++w) {
            fin0[w] += T(w, 1) - s0;  // when wave w finished issuing C0, from C0 start
            fin1[w] += T(w, 3) - s1;
            p3[w] += T(w, 4) - s0;
            p12s[w] += T(w, 6) - s1;
            p12e[w] += T(w, 5) - s1;
        }
        w0 += e0 - s0; w1 += e1 - s1;
    }
    const int ns = 17;
    printf("block %d: per step  C0 span %.0f (last issue at %.0f)  C1 span %.0f (last issue at %.0f)  step %.0f cycles\n",
           blk, c0 / ns, w0 / ns, c1 / ns, w1 / ns, (c0 + c1) / ns);
    printf("wave: C0 [P3 done, P5 done]  C1 [staging done, P12 done, P4 done] (cycles from interval start)\n");
    for (int w = 0; w < 16; ++w)
        printf("  w%2d  %6.0f %6.0f   %6.0f %6.0f %6.0f\n", w, p3[w] / ns, fin0[w] / ns, p12s[w] / ns,
               p12e[w] / ns, fin1[w] / ns);
    return 0;
}
