// tools/timeg4rows.hip — times the four-kernel 4-D path (guided4d.hip) on one (t, z) row of config
// T's real share: input (12, 264, 1024, 1024) f32, output timepoints [4, 8) x planes [4, 260) x
// the whole plane, r = 2, eps = 2500 — what zt_guided_filter_apply_array runs per row since the
// chunk-row grouping. Build variants with -DG4_BOX_TY=... (box3 march tile height); prints the
// median of 5 calls and a checksum of the output (not a product path).
#include "../zarrs_tools_amd/csrc/guided4d.hip"
#include "../zarrs_tools_amd/csrc/cast.hip"

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
    printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

int main(int argc, char** argv) {
    const char* tag = argc > 1 ? argv[1] : "";
    const int T = 12, NZ = 264, NY = argc > 2 ? atoi(argv[2]) : 1024, NX = NY;
    const int64_t plane = (int64_t)NY * NX, vol = (int64_t)NZ * plane, n = T * vol;
    float *in, *out;
    void* scratch;
    const int OT = 4, OZ = 256;
    CK(hipMalloc(&in, n * 4));
    CK(hipMalloc(&out, (int64_t)OT * OZ * plane * 4));
    CK(hipMalloc(&scratch, (size_t)zt::guided4d_scratch_bytes(n, true)));
    std::vector<float> h(plane);
    for (int t = 0; t < T; ++t)
        for (int z = 0; z < NZ; ++z) {
            for (int64_t i = 0; i < plane; ++i)
                h[i] = (float)(((i + (int64_t)z * 7919 + t * 104729) * 2654435761u) % 1000) * 0.1f +
                       ((i % NX) < NX / 2 ? 0.0f : 500.0f);
            CK(hipMemcpy(in + t * vol + z * plane, h.data(), plane * 4, hipMemcpyHostToDevice));
        }
    zt::NdGeom g{};
    g.ndim = 4;
    const int64_t sh[4] = {T, NZ, NY, NX}, os[4] = {OT, OZ, NY, NX};
    const int64_t ost[4] = {4, 4, 0, 0};
    for (int d = 0; d < 4; ++d) {
        g.shape[d] = sh[d];
        g.out_start[d] = ost[d];
        g.out_shape[d] = os[d];
    }
    g.in_strides[3] = 1; g.in_strides[2] = NX; g.in_strides[1] = plane; g.in_strides[0] = vol;
    g.out_strides[3] = 1; g.out_strides[2] = NX; g.out_strides[1] = plane; g.out_strides[0] = (int64_t)OZ * plane;
    g.numel = n;
    g.out_numel = (int64_t)OT * OZ * plane;
    hipStream_t s;
    CK(hipStreamCreate(&s));
    auto run = [&] { CK(zt::launch_guided4d(in, zt::kF32, out, zt::kF32, g, 2, 2500.0f, scratch, s)); };
    run();
    CK(hipStreamSynchronize(s));
    hipEvent_t a, b;
    CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
    std::vector<float> t;
    for (int r = 0; r < 5; ++r) {
        CK(hipEventRecord(a, s)); run(); CK(hipEventRecord(b, s)); CK(hipEventSynchronize(b));
        float ms; CK(hipEventElapsedTime(&ms, a, b)); t.push_back(ms);
    }
    std::sort(t.begin(), t.end());
    double sum = 0.0;
    for (int z : {0, 100, 255}) {
        CK(hipMemcpy(h.data(), out + (int64_t)(1 * OZ + z) * plane, plane * 4, hipMemcpyDeviceToHost));
        for (float v : h) sum += v;
    }
    printf("%-16s median %8.3f ms  min %8.3f ms  checksum %.9e\n", tag, t[2], t[0], sum);
    return 0;
}
