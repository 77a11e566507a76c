// tools/ubench.hip — issue-rate microbenchmarks of the VALU / LDS instructions the fused
// guided-filter kernel is made of (not a product path). One 1024-thread workgroup per CU
// (4 waves per SIMD, the fused kernel's occupancy), 8 independent chains per lane; prints
// SIMD cycles per wave-instruction from s_memtime deltas (median over waves).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { \
    printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

constexpr int kIters = 512;
typedef unsigned int u4 __attribute__((ext_vector_type(4)));

#define REP8(X) X(0) X(1) X(2) X(3) X(4) X(5) X(6) X(7)

template <int OP>
__global__ __launch_bounds__(1024) void ubench(float* out, long long* cyc) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    double d[8];
    float f[8];
    float g[8];
    for (int i = 0; i < 8; ++i) {
        d[i] = threadIdx.x * 0.5 + i;
        f[i] = threadIdx.x * 0.25f + i;
        g[i] = 1.0f + i;
    }
    const double dd = 1.0000001;
    const float ff = 1.0001f;
    __syncthreads();
    const long long t0 = __builtin_amdgcn_s_memtime();
    for (int it = 0; it < kIters; ++it) {
        if constexpr (OP == 0) {  // v_add_f64
#define X(i) asm volatile("v_add_f64 %0, %0, %1" : "+v"(d[i]) : "v"(dd));
            REP8(X)
#undef X
        } else if constexpr (OP == 1) {  // v_cvt_f64_f32
#define X(i) asm volatile("v_cvt_f64_f32 %0, %1" : "=v"(d[i]) : "v"(f[i]));
            REP8(X)
#undef X
        } else if constexpr (OP == 2) {  // v_cvt_f32_f64
#define X(i) asm volatile("v_cvt_f32_f64 %0, %1" : "=v"(f[i]) : "v"(d[i]));
            REP8(X)
#undef X
        } else if constexpr (OP == 3) {  // v_add_f32
#define X(i) asm volatile("v_add_f32 %0, %0, %1" : "+v"(f[i]) : "v"(ff));
            REP8(X)
#undef X
        } else if constexpr (OP == 4) {  // v_pk_add_f32 (operands as 64-bit register pairs)
#define X(i) asm volatile("v_pk_add_f32 %0, %0, %1" : "+v"(d[i]) : "v"(dd));
            REP8(X)
#undef X
        } else if constexpr (OP == 5) {  // v_add_f32 with a DPP source (row_shr:1)
#define X(i) asm volatile("v_add_f32_dpp %0, %1, %0 row_shr:1 row_mask:0xf bank_mask:0xf bound_ctrl:1" : "+v"(f[i]) : "v"(g[i]));
            REP8(X)
#undef X
        } else if constexpr (OP == 6) {  // v_mov_b32 DPP wave_shr:1
#define X(i) asm volatile("v_mov_b32_dpp %0, %1 wave_shr:1 row_mask:0xf bank_mask:0xf bound_ctrl:1" : "=v"(f[i]) : "v"(g[i]));
            REP8(X)
#undef X
        } else if constexpr (OP == 7) {  // v_rcp_f32
#define X(i) asm volatile("v_rcp_f32 %0, %1" : "=v"(f[i]) : "v"(g[i]));
            REP8(X)
#undef X
        } else if constexpr (OP == 8) {  // v_fma_f64
#define X(i) asm volatile("v_fma_f64 %0, %0, %1, %1" : "+v"(d[i]) : "v"(dd));
            REP8(X)
#undef X
        } else if constexpr (OP == 9) {  // v_fma_f32
#define X(i) asm volatile("v_fma_f32 %0, %0, %1, %1" : "+v"(f[i]) : "v"(ff));
            REP8(X)
#undef X
        } else if constexpr (OP == 10) {  // v_add_u32
#define X(i) asm volatile("v_add_u32 %0, %0, %1" : "+v"(f[i]) : "v"(ff));
            REP8(X)
#undef X
        } else if constexpr (OP == 11) {  // ds_read_b64, conflict-free (lane-consecutive)
            const unsigned a = threadIdx.x * 8;
#define X(i) asm volatile("ds_read_b64 %0, %1 offset:%2" : "=v"(d[i]) : "v"(a), "i"(i * 8192));
            REP8(X)
#undef X
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        } else if constexpr (OP == 12) {  // ds_write_b64
            const unsigned a = threadIdx.x * 8;
#define X(i) asm volatile("ds_write_b64 %0, %1 offset:%2" :: "v"(a), "v"(d[i]), "i"(i * 8192));
            REP8(X)
#undef X
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        } else if constexpr (OP == 13) {  // ds_read_b128
            const unsigned a = threadIdx.x * 16;
            u4 q0, q1, q2, q3;
            asm volatile("ds_read_b128 %0, %1 offset:0" : "=v"(q0) : "v"(a));
            asm volatile("ds_read_b128 %0, %1 offset:16384" : "=v"(q1) : "v"(a));
            asm volatile("ds_read_b128 %0, %1 offset:32768" : "=v"(q2) : "v"(a));
            asm volatile("ds_read_b128 %0, %1 offset:49152" : "=v"(q3) : "v"(a));
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            f[0] += __uint_as_float(q0.x ^ q1.y ^ q2.z ^ q3.w);
        } else if constexpr (OP == 14) {  // ds_write_b128
            const unsigned a = threadIdx.x * 16;
            u4 q = {__float_as_uint(f[0]), __float_as_uint(f[1]), __float_as_uint(f[2]), __float_as_uint(f[3])};
            asm volatile("ds_write_b128 %0, %1 offset:0" :: "v"(a), "v"(q));
            asm volatile("ds_write_b128 %0, %1 offset:16384" :: "v"(a), "v"(q));
            asm volatile("ds_write_b128 %0, %1 offset:32768" :: "v"(a), "v"(q));
            asm volatile("ds_write_b128 %0, %1 offset:49152" :: "v"(a), "v"(q));
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        } else if constexpr (OP == 15) {  // f64 DPP moves (two v_mov_b32_dpp row_shr:1)
#define X(i) asm volatile("v_mov_b32_dpp %0, %1 row_shr:1 row_mask:0xf bank_mask:0xf bound_ctrl:1" : "=v"(f[i]) : "v"(g[i]));
            REP8(X)
#undef X
        } else if constexpr (OP == 16) {  // v_mul_f32 (for the pointwise mix)
#define X(i) asm volatile("v_mul_f32 %0, %0, %1" : "+v"(f[i]) : "v"(ff));
            REP8(X)
#undef X
        } else if constexpr (OP == 17) {  // v_add_f32 with DPP wave_shr:1
#define X(i) asm volatile("v_add_f32_dpp %0, %1, %0 wave_shr:1 row_mask:0xf bank_mask:0xf bound_ctrl:1" : "+v"(f[i]) : "v"(g[i]));
            REP8(X)
#undef X
        }
    }
    const long long t1 = __builtin_amdgcn_s_memtime();
    float acc = 0.0f;
    for (int i = 0; i < 8; ++i) acc += (float)d[i] + f[i];
    out[blockIdx.x * 1024 + threadIdx.x] = acc;
    if ((threadIdx.x & 63) == 0) cyc[blockIdx.x * 16 + threadIdx.x / 64] = t1 - t0;
}

template <int OP>
int run(const char* name, int ninstr_per_iter, float* out, long long* cyc, int nblk) {
    const int lds = 128 * 1024;  // one workgroup per CU
    CK(hipFuncSetAttribute((const void*)ubench<OP>, hipFuncAttributeMaxDynamicSharedMemorySize, lds));
    hipLaunchKernelGGL(ubench<OP>, dim3(nblk), dim3(1024), lds, 0, out, cyc);
    CK(hipDeviceSynchronize());
    hipLaunchKernelGGL(ubench<OP>, dim3(nblk), dim3(1024), lds, 0, out, cyc);
    CK(hipDeviceSynchronize());
    std::vector<long long> h(nblk * 16);
    CK(hipMemcpy(h.data(), cyc, h.size() * 8, hipMemcpyDeviceToHost));
    std::sort(h.begin(), h.end());
    const double med = (double)h[h.size() / 2];
    // 4 waves share a SIMD: SIMD cycles per wave-instruction = elapsed / (4 * instructions)
    printf("%-28s %7.2f SIMD cycles per wave-instruction (s_memtime ticks, median wave)\n", name,
           med / (4.0 * kIters * ninstr_per_iter));
    return 0;
}

int main() {
    float* out;
    long long* cyc;
    const int nblk = 256;
    CK(hipMalloc(&out, nblk * 1024 * 4));
    CK(hipMalloc(&cyc, nblk * 16 * 8));
    run<3>("v_add_f32", 8, out, cyc, nblk);
    run<9>("v_fma_f32", 8, out, cyc, nblk);
    run<16>("v_mul_f32", 8, out, cyc, nblk);
    run<10>("v_add_u32", 8, out, cyc, nblk);
    run<4>("v_pk_add_f32", 8, out, cyc, nblk);
    run<0>("v_add_f64", 8, out, cyc, nblk);
    run<8>("v_fma_f64", 8, out, cyc, nblk);
    run<1>("v_cvt_f64_f32", 8, out, cyc, nblk);
    run<2>("v_cvt_f32_f64", 8, out, cyc, nblk);
    run<7>("v_rcp_f32", 8, out, cyc, nblk);
    run<5>("v_add_f32_dpp row_shr:1", 8, out, cyc, nblk);
    run<17>("v_add_f32_dpp wave_shr:1", 8, out, cyc, nblk);
    run<6>("v_mov_b32_dpp wave_shr:1", 8, out, cyc, nblk);
    run<15>("v_mov_b32_dpp row_shr:1", 8, out, cyc, nblk);
    run<11>("ds_read_b64 (per CU: /4)", 8, out, cyc, nblk);
    run<12>("ds_write_b64 (per CU: /4)", 8, out, cyc, nblk);
    run<13>("ds_read_b128 (per CU: /4)", 4, out, cyc, nblk);
    run<14>("ds_write_b128 (per CU: /4)", 4, out, cyc, nblk);
    return 0;
}
