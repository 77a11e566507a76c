// tools/timek.hip — times the fused guided-filter kernel (r=4, f32, N^3, the bench's synthetic
// step+noise-like input) and prints a checksum of the output, so builds with different
// compile-time work splits (-DGF_K3=, -DGF_K4=, ...) and launch modes (-DTK_LAUNCH=) can be
// compared (not a product path).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <type_traits>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "../zarrs_tools_amd/csrc/gf_fused.hpp"

using namespace zt;
#ifndef TK_TY
#define TK_TY 32
#endif
#ifndef TK_R
#define TK_R 4
#endif
#ifndef TK_NT
#define TK_NT 1024
#endif

#ifdef TK_U16
using TIN = uint16_t;  // integer input (-DTK_U16): the stage-1 integer path
#else
using TIN = float;
#endif

#ifndef TK_LAUNCH
#define TK_LAUNCH 0  // 0: launch_fused_cfg; 1: mode 1 over every tile; 2: mode 0 over every tile
                     // (timing only: the border tiles' output is wrong)
#endif

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { \
    printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

int main(int argc, char** argv) {
    int n = argc > 1 ? atoi(argv[1]) : 2048;
    const char* tag = argc > 2 ? argv[2] : "";
    // argv[4]: extra elements per row (pitch n + pad): separates the cache-set behaviour of
    // power-of-two row pitches from the kernel's own cost
    const int pad = argc > 4 ? atoi(argv[4]) : 0;
    const int pitch = n + pad;
    size_t vox = (size_t)n * n * pitch;
    TIN* in;
    float* out;
    CK(hipMalloc(&in, vox * sizeof(TIN))); CK(hipMalloc(&out, vox * 4));
    std::vector<float> h((size_t)n * pitch);
    std::vector<TIN> hi((size_t)n * pitch);
    for (int z = 0; z < n; ++z) {
        for (size_t i = 0; i < h.size(); ++i) {
            h[i] = (float)(((i + (size_t)z * 7919u) * 2654435761u) % 1000) * 0.1f +
                   ((i % pitch) < (size_t)n / 2 ? 0.0f : 500.0f);
            hi[i] = std::is_same<TIN, float>::value ? (TIN)h[i] : (TIN)(h[i] * 10.0f);
        }
        CK(hipMemcpy(in + (size_t)z * n * pitch, hi.data(), hi.size() * sizeof(TIN),
                     hipMemcpyHostToDevice));
    }
    GFParams p{};
    p.in = in; p.out = out; p.in_sz = (int64_t)n * pitch; p.in_sy = pitch; p.out_sz = (int64_t)n * pitch;
    p.out_sy = pitch; p.in_z0 = 0; p.zlo = 0; p.zhi = n; p.nz = p.ny = p.nx = n;
    p.oz0 = p.oy0 = p.ox0 = 0; p.onz = p.ony = p.onx = n; p.zseg = (argc > 3 && atoi(argv[3]) > 0) ? atoi(argv[3]) : 256; p.eps = 2500.0f;
    hipStream_t s; CK(hipStreamCreate(&s));
    auto launch = [&](const GFParams& p0, hipStream_t st) -> hipError_t {
        if (TK_LAUNCH == 0) return launch_fused_cfg<TK_R, TK_TY, TK_NT, TIN, float>(p0, st);
        using C = GFConfig<TK_R, TK_TY, TK_NT>;
        GFParams q = p0;
        volatile float one = 1.0f;
        q.rcp_w3 = one / (float)C::W3;
        q.tiles_x = (q.onx + C::TX - 1) / C::TX;
        q.tiles_y = (q.ony + TK_TY - 1) / TK_TY;
        q.nseg = (q.onz + q.zseg - 1) / q.zseg;
        const long long nwg = (long long)q.tiles_x * q.tiles_y * q.nseg;
        if (TK_LAUNCH == 1) {
            q.itx0 = q.itx1 = q.ity0 = q.ity1 = 0;
            return launch_fused_variant<TK_R, TK_TY, TK_NT, TIN, float, 1>(q, nwg, st);
        }
        if (TK_LAUNCH == 3) {
            // interior tiles in mode 0 on `st`, the border tiles in mode 1 concurrently on a
            // second stream (launched first), joined back into `st`
            static hipStream_t s2 = nullptr;
            static hipEvent_t e0, e1;
            if (!s2) {
                CK(hipStreamCreateWithFlags(&s2, hipStreamNonBlocking));
                CK(hipEventCreateWithFlags(&e0, hipEventDisableTiming));
                CK(hipEventCreateWithFlags(&e1, hipEventDisableTiming));
            }
            interior_tiles(q.ox0, q.ox0 + q.onx, q.nx, C::TX, TK_R, 0, q.tiles_x, q.itx0, q.itx1);
            interior_tiles(q.oy0, q.oy0 + q.ony, q.ny, TK_TY, TK_R, 0, q.tiles_y, q.ity0, q.ity1);
            const long long n_int = (long long)(q.itx1 - q.itx0) * (q.ity1 - q.ity0) * q.nseg;
            CK(hipEventRecord(e0, st));
            CK(hipStreamWaitEvent(s2, e0, 0));
            CK((launch_fused_variant<TK_R, TK_TY, TK_NT, TIN, float, 1>(q, nwg, s2)));
            CK(hipEventRecord(e1, s2));
            CK((launch_fused_variant<TK_R, TK_TY, TK_NT, TIN, float, 0>(q, n_int, st)));
            return hipStreamWaitEvent(st, e1, 0);
        }
        q.itx0 = 0; q.itx1 = q.tiles_x; q.ity0 = 0; q.ity1 = q.tiles_y;
        return launch_fused_variant<TK_R, TK_TY, TK_NT, TIN, float, 0>(q, nwg, st);
    };
    hipEvent_t a, b;
    CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
    std::vector<float> t;
    CK(launch(p, s));
    for (int r = 0; r < 5; ++r) {
        CK(hipEventRecord(a, s));
        CK(launch(p, s));
        CK(hipEventRecord(b, s));
        CK(hipEventSynchronize(b));
        float ms; CK(hipEventElapsedTime(&ms, a, b));
        t.push_back(ms);
    }
    std::sort(t.begin(), t.end());
    // checksum over a few slices
    double sum = 0.0, mx = 0.0;
    for (int z : {0, 3, n / 2, n - 1}) {
        CK(hipMemcpy(h.data(), out + (size_t)z * n * pitch, h.size() * 4, hipMemcpyDeviceToHost));
        for (size_t i = 0; i < h.size(); ++i)
            if ((int)(i % pitch) < n) { sum += h[i]; mx = std::max(mx, (double)h[i]); }
    }
    printf("%-24s median %8.3f ms  min %8.3f ms  checksum %.9e max %.6f\n", tag, t[2], t[0], sum,
           mx);
    return 0;
}
