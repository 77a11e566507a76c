// tools/ubench_valu.hip — issue cost of the VALU instructions the fused guided kernel is made of,
// measured with 16 waves per CU (one 1024-thread workgroup per CU, 4 waves per SIMD), 8
// independent chains per wave. Prints SIMD-cycles per wave-instruction (clock from s_memtime
// vs s_memrealtime inside the kernel). Not a product path.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                              \
    do {                                                                                   \
        hipError_t e_ = (x);                                                               \
        if (e_ != hipSuccess) {                                                            \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));      \
            exit(1);                                                                       \
        }                                                                                  \
    } while (0)

constexpr int ITERS = 4096;

#define BODY8(OP) OP(0) OP(1) OP(2) OP(3) OP(4) OP(5) OP(6) OP(7)

template <int KIND>
__global__ __launch_bounds__(1024) void ub(float* out, long long* clk) {
    double d[8];
    float f[8], g[8];
    for (int i = 0; i < 8; ++i) {
        d[i] = threadIdx.x * 0.5 + i;
        f[i] = threadIdx.x * 0.25f + i;
        g[i] = threadIdx.x * 0.125f + i;
    }
    const long long t0 = __builtin_amdgcn_s_memtime();
    const long long r0 = __builtin_amdgcn_s_memrealtime();
    for (int it = 0; it < ITERS; ++it) {
#define F64(i) asm volatile("v_add_f64 %0, %0, %1" : "+v"(d[i]) : "v"(d[(i + 1) & 7]));
#define F32(i) asm volatile("v_add_f32 %0, %0, %1" : "+v"(f[i]) : "v"(g[i]));
#define PK(i) asm volatile("v_pk_add_f32 %0, %0, %1" : "+v"(d[i]) : "v"(d[(i + 3) & 7]));
#define CVT(i) asm volatile("v_cvt_f64_f32 %0, %1" : "=v"(d[i]) : "v"(f[i]));
#define DPP(i) asm volatile("v_mov_b32_dpp %0, %1 wave_shr:1 bound_ctrl:0" : "=v"(f[i]) : "v"(g[i]));
#define MUL24(i) asm volatile("v_mul_u32_u24 %0, %0, %1" : "+v"(f[i]) : "v"(g[i]));
#define MULLO(i) asm volatile("v_mul_lo_u32 %0, %0, %1" : "+v"(f[i]) : "v"(g[i]));
#define FMA64(i) asm volatile("v_fma_f64 %0, %0, %1, %1" : "+v"(d[i]) : "v"(d[(i + 1) & 7]));
        if constexpr (KIND == 0) { BODY8(F64) BODY8(F64) }
        if constexpr (KIND == 1) { BODY8(F32) BODY8(F32) }
        if constexpr (KIND == 2) { BODY8(PK) BODY8(PK) }
        if constexpr (KIND == 3) { BODY8(CVT) BODY8(CVT) }
        if constexpr (KIND == 4) { BODY8(DPP) BODY8(DPP) }
        if constexpr (KIND == 5) { BODY8(MUL24) BODY8(MUL24) }
        if constexpr (KIND == 6) { BODY8(MULLO) BODY8(MULLO) }
        if constexpr (KIND == 7) { BODY8(FMA64) BODY8(FMA64) }
        if constexpr (KIND == 8) { BODY8(F64) BODY8(F32) }
    }
    const long long t1 = __builtin_amdgcn_s_memtime();
    const long long r1 = __builtin_amdgcn_s_memrealtime();
    float s = 0.f;
    for (int i = 0; i < 8; ++i) s += (float)d[i] + f[i];
    out[blockIdx.x * 1024 + threadIdx.x] = s;
    if (threadIdx.x == 0) {
        clk[blockIdx.x * 2] = t1 - t0;
        clk[blockIdx.x * 2 + 1] = r1 - r0;
    }
}

template <int K>
void run(const char* name, int nblk, float* out, long long* clk, long long* h) {
    ub<K><<<nblk, 1024>>>(out, clk);
    CK(hipDeviceSynchronize());
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    CK(hipEventRecord(a));
    ub<K><<<nblk, 1024>>>(out, clk);
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    float ms;
    CK(hipEventElapsedTime(&ms, a, b));
    CK(hipMemcpy(h, clk, nblk * 16, hipMemcpyDeviceToHost));
    double cyc = 0, rt = 0;
    for (int i = 0; i < nblk; ++i) { cyc += h[2 * i]; rt += h[2 * i + 1]; }
    cyc /= nblk;
    rt /= nblk;
    const double ghz = cyc / rt * 0.1;  // memrealtime: 100 MHz
    // per SIMD: 4 waves x ITERS x 16 instructions
    const double per = cyc / (4.0 * ITERS * 16);
    printf("%-10s %.2f SIMD-cycles per wave-instruction (clock %.2f GHz, %.3f ms)\n", name, per, ghz, ms);
}

int main() {
    const int nblk = 256;
    float* out;
    long long *clk, *h;
    CK(hipMalloc(&out, nblk * 1024 * 4));
    CK(hipMalloc(&clk, nblk * 16));
    h = (long long*)malloc(nblk * 16);
    run<0>("add_f64", nblk, out, clk, h);
    run<1>("add_f32", nblk, out, clk, h);
    run<2>("pk_add", nblk, out, clk, h);
    run<3>("cvt_f64", nblk, out, clk, h);
    run<4>("dpp_mov", nblk, out, clk, h);
    run<5>("mul_u24", nblk, out, clk, h);
    run<6>("mul_lo", nblk, out, clk, h);
    run<7>("fma_f64", nblk, out, clk, h);
    run<8>("f64+f32", nblk, out, clk, h);
    return 0;
}
