// tools/timetshare.hip — times the 4-D guided filter (launch_guided4d: the t-march stage 1 and
// box3_final_kernel) on config T's per-GPU share geometry (a (20, 264, N, N) f32 block, output
// timepoints [4, 20) x planes [4, 260), r = 2) and prints a checksum, so compile-time geometry
// flags (-DG4_TM_MZ=...) can be compared (not a product path).
#include "../zarrs_tools_amd/csrc/guided4d.hip"

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { \
    printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

int main(int argc, char** argv) {
    const int n = argc > 1 ? atoi(argv[1]) : 1024;
    const char* tag = argc > 2 ? argv[2] : "";
    const int T = 20, nz = 264, R = 2;
    const size_t vox = (size_t)T * nz * n * n;
    float *in, *out;
    void* scratch;
    CK(hipMalloc(&in, vox * 4));
    const int64_t osh[4] = {16, 256, n, n};
    const size_t ovox = (size_t)osh[0] * osh[1] * n * n;
    CK(hipMalloc(&out, ovox * 4));
    CK(hipMalloc(&scratch, zt::guided4d_scratch_bytes((int64_t)vox, false)));
    std::vector<float> h((size_t)n * n);
    for (int s = 0; s < T * nz; ++s) {
        for (size_t i = 0; i < h.size(); ++i)
            h[i] = (float)(((i + (size_t)s * 7919u) * 2654435761u) % 1000) * 0.1f +
                   ((i % n) < (size_t)n / 2 ? 0.0f : 500.0f);
        CK(hipMemcpy(in + (size_t)s * n * n, h.data(), h.size() * 4, hipMemcpyHostToDevice));
    }
    zt::NdGeom g{};
    g.ndim = 4;
    const int64_t sh[4] = {T, nz, n, n}, o0[4] = {4, 4, 0, 0};
    int64_t st = 1, ost = 1;
    for (int d = 3; d >= 0; --d) {
        g.shape[d] = sh[d];
        g.in_strides[d] = st;
        g.out_strides[d] = ost;
        g.out_start[d] = o0[d];
        g.out_shape[d] = osh[d];
        st *= sh[d];
        ost *= osh[d];
    }
    g.numel = (int64_t)vox;
    g.out_numel = (int64_t)ovox;
    hipStream_t s;
    CK(hipStreamCreate(&s));
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    auto run = [&] {
        return zt::launch_guided4d(in, zt::kF32, out, zt::kF32, g, R, 2500.0f, scratch, s);
    };
    CK(run());
    std::vector<float> t;
    for (int r = 0; r < 5; ++r) {
        CK(hipEventRecord(a, s));
        CK(run());
        CK(hipEventRecord(b, s));
        CK(hipEventSynchronize(b));
        float ms;
        CK(hipEventElapsedTime(&ms, a, b));
        t.push_back(ms);
    }
    std::sort(t.begin(), t.end());
    double sum = 0.0;
    for (size_t p : {(size_t)0, (size_t)1000, ovox / ((size_t)n * n) - 1}) {
        CK(hipMemcpy(h.data(), out + p * n * n, h.size() * 4, hipMemcpyDeviceToHost));
        for (float v : h) sum += v;
    }
    printf("%-24s median %8.3f ms  min %8.3f ms  checksum %.9e\n", tag, t[2], t[0], sum);
    return 0;
}
