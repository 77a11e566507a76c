// guided4d.hip — the 4-D guided filter (config T: a (T, Z, Y, X) time series, every axis windowed
// alike, guided_filter.rs:117-199 with get_block clamping on all four axes).
//
// The box mean over (t, z, y, x) is separable and linear, so the 4-D sums are t-window sums of
// per-timepoint 3-D box sums:  box4(f)(t) = sum_{t' in W(t)} box3(f(t')), and stage 2 may take
// the t-window first: box4(a, b) = box3(tbox(a, b)). Windows clamp at the block bounds (= the
// array bounds with the 2r halo). Two stages:
//   stage 1 -> TAB(t) = t-window sums of (a, b) for the output timepoints (f64, rounded once),
//       with U3 = exact f64 3-D window sums of v, U4 = t-window of U3 (exact),
//       u = RN(RN_f32(U4) / c4), s = (v-u)^2, a = s/(s+eps), b = (1-a)u (guided_filter.rs:126-142):
//       r <= 2: one t-march (g4_tmarch_tab_kernel), U3 never in HBM;
//       r 3-6: K1 box3_march<float -> double> writes U3, g4_tab_kernel writes TAB over it;
//   K3f box3_final_kernel: the box3 z-march of TAB over the output box with the final stage,
//       mean = RN_f32(S4) / c4, out = RN(RN(v * mean_a) + mean_b) cast to TOut
//       (guided_filter.rs:144-163, :101-102).
// Divisions: u = RN(U) / c correctly rounded (IEEE, or Markstein with RN(1/c) in the t-march), a
// within 1 ulp in the t-march (IEEE elsewhere); stage 1 exact, stage 2 with f64 t-sums.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdlib>
#include <type_traits>

#include "g4_limits.hpp"
#include "zt_device.hpp"
#include "zt_kernels.hpp"

namespace zt {

namespace {

struct dd2 {  // two f64 accumulators (the (a, b) pair)
    double x, y;
};

__device__ __forceinline__ void acc_zero(double& a) { a = 0.0; }
__device__ __forceinline__ void acc_zero(dd2& a) { a.x = a.y = 0.0; }
__device__ __forceinline__ void acc_add(double& a, float v) { a += (double)v; }
__device__ __forceinline__ void acc_sub(double& a, float v) { a -= (double)v; }
__device__ __forceinline__ void acc_add(dd2& a, float2 v) { a.x += (double)v.x; a.y += (double)v.y; }
__device__ __forceinline__ void acc_sub(dd2& a, float2 v) { a.x -= (double)v.x; a.y -= (double)v.y; }
__device__ __forceinline__ void acc_add(double& a, double v) { a += v; }
__device__ __forceinline__ void acc_sub(double& a, double v) { a -= v; }
__device__ __forceinline__ void acc_add(dd2& a, const dd2& v) { a.x += v.x; a.y += v.y; }
__device__ __forceinline__ void acc_sub(dd2& a, const dd2& v) { a.x -= v.x; a.y -= v.y; }
__device__ __forceinline__ void acc_add(float2& a, float2 v) { a.x += v.x; a.y += v.y; }
__device__ __forceinline__ void acc_sub(float2& a, float2 v) { a.x -= v.x; a.y -= v.y; }
__device__ __forceinline__ void put(double& o, double a) { o = a; }
__device__ __forceinline__ void put(float2& o, const dd2& a) { o = make_float2((float)a.x, (float)a.y); }
template <typename TV> __device__ __forceinline__ TV zero_v();
template <> __device__ __forceinline__ float zero_v<float>() { return 0.0f; }
template <> __device__ __forceinline__ float2 zero_v<float2>() { return make_float2(0.0f, 0.0f); }

// compile-time loop: f(integral_constant<I>) for I in [B, E)
template <int B, int E, typename F>
__device__ __forceinline__ void g4_static_for(F&& f) {
    if constexpr (B < E) {
        f(std::integral_constant<int, B>{});
        g4_static_for<B + 1, E>(f);
    }
}

__device__ __forceinline__ int ccount(int i, int n, int r) {
    const int lo = i - r < 0 ? 0 : i - r;
    const int hi = i + r > n - 1 ? n - 1 : i + r;
    return hi - lo + 1;
}

#ifndef G4_BOX_TY
#define G4_BOX_TY 16  // box3 march tile height (tools/timeg4rows.hip A/B)
#endif
#ifndef G4_BOX_KY
#define G4_BOX_KY 4  // y-window outputs per thread; kTX * kTY / kKY must equal kNT
#endif
constexpr int kTX = 64, kTY = G4_BOX_TY, kNT = 256, kKX = 4, kKY = G4_BOX_KY;
static_assert(kTX * (kTY / kKY) == kNT, "the y-window items cover the tile once");
constexpr int kPX = 64, kPY = 4;  // K2 / K4 thread blocks: 4 rows of 64 x
// element strides of a (T, nz, ny, nx) input with unit-stride x (the chunk's halo'd box read in
// place from the resident array, or a C-order scratch copy)
struct Str3 {
    int64_t t, z, y;
};

#ifndef G4_LDS_BARRIER
#define G4_LDS_BARRIER 0
#endif
// The box3 marches' step barrier. __syncthreads() also waits for every global load in flight,
// i.e. for the next step's prefetched entering slice; G4_LDS_BARRIER=1 waits for LDS only, so the
// prefetch stays in flight across the barrier (the compiler still waits for it at its first use).
// Measured slower on the T share (57.1-57.2 against 55.2-55.4 ms, profiles/r04_ldsbar_ab.jsonl).
__device__ __forceinline__ void box3_barrier() {
#if G4_LDS_BARRIER
    __asm__ volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
#else
    __syncthreads();
#endif
}

// XCD-aware block order. Consecutive linear block ids are dispatched round-robin over the 8 XCDs
// (each with its own L2); give each XCD a contiguous run of (tile, timepoint) ids instead, so the
// workgroups resident on one XCD march neighbouring tiles whose aprons share that XCD's L2 lines.
__device__ __forceinline__ void xcd_block(int& bx, int& by) {
    const int64_t gx = gridDim.x, total = gx * gridDim.y;
    const int64_t lin = blockIdx.x + (int64_t)blockIdx.y * gx;
    const int64_t lid = total % 8 == 0 ? (lin % 8) * (total / 8) + lin / 8 : lin;
    bx = (int)(lid % gx);
    by = (int)(lid / gx);
}

// The z-window ring: with the last 2R + 1 entering slices of a thread's apron points held in
// registers, the leaving slice of the running z-window is never re-read from memory (with ~8
// resident workgroups per CU its lines are long gone from L2 by then; the T share's box3 marches
// read 2-2.5x their compulsory bytes without the ring). Used when the ring fits in 64 VGPRs.
template <int R, typename TV, int NPT>
constexpr bool box3_ring() {
    return NPT * (2 * R + 1) * (int)(sizeof(TV) / 4) <= 64;
}

// 3-D window sums (radius R, clamped to the volume) of every timepoint volume of a (T, nz, ny, nx)
// C-order array: a workgroup marches one 64 x 16 xy tile through zseg slices of one timepoint.
// Each thread keeps the running z-window of its points of the (tile + R) apron in registers
// (the entering slice prefetched a step ahead; the leaving one from the ring, box3_ring, or
// prefetched too); x- then y-window sums go through LDS.
template <int R, typename TV, typename TA, typename TO>
__global__ __launch_bounds__(kNT) void box3_march_kernel(const TV* __restrict__ in,
                                                         TO* __restrict__ out, int nz, int ny,
                                                         int nx, int zseg, int tiles_x,
                                                         int tiles_y, Str3 is) {
    constexpr int EX = kTX + 2 * R, EY = kTY + 2 * R, NE = EX * EY;
    constexpr int NPT = (NE + kNT - 1) / kNT;
    constexpr int W = 2 * R + 1;
    __shared__ TA Z[EY][EX];
    __shared__ TA X[EY][kTX];
    int bx, t;
    xcd_block(bx, t);
    const int ntile = tiles_x * tiles_y;
    const int seg = bx / ntile, tile = bx % ntile;
    const int x0 = (tile % tiles_x) * kTX, y0 = (tile / tiles_x) * kTY;
    const int z0 = seg * zseg, z1 = min(z0 + zseg, nz);
    const int64_t plane = (int64_t)ny * nx;
    const TV* vol = in + (int64_t)t * is.t;  // input: strided (x unit-stride); output: C order
    TO* ovol = out + (int64_t)t * nz * plane;

    // owned apron points: index into the plane (or -1 outside the volume / past the apron)
    int64_t pidx[NPT];
    int ey_[NPT], ex_[NPT];
#pragma unroll
    for (int k = 0; k < NPT; ++k) {
        const int e = threadIdx.x + k * kNT;
        const int ey = e / EX, ex = e % EX;
        const int gy = y0 - R + ey, gx = x0 - R + ex;
        ey_[k] = e < NE ? ey : -1;
        ex_[k] = ex;
        pidx[k] = (e < NE && gy >= 0 && gy < ny && gx >= 0 && gx < nx) ? (int64_t)gy * is.y + gx : -1;
    }
    auto load = [&](int z, int k) -> TV {
        return (pidx[k] >= 0 && z >= 0 && z < nz) ? vol[(int64_t)z * is.z + pidx[k]] : zero_v<TV>();
    };
    // x- and y-window sums of the Z slice of output slice z (the caller filled Z)
    auto xy_windows = [&](int z) {
        box3_barrier();
        // x-window: EY rows x (kTX / kKX) segments of kKX outputs
        for (int it = threadIdx.x; it < EY * (kTX / kKX); it += kNT) {
            const int ey = it / (kTX / kKX), sx = (it % (kTX / kKX)) * kKX;
            TA s;
            acc_zero(s);
#pragma unroll
            for (int j = 0; j <= 2 * R; ++j) acc_add(s, Z[ey][sx + j]);
            X[ey][sx] = s;
#pragma unroll
            for (int j = 1; j < kKX; ++j) {
                acc_add(s, Z[ey][sx + j + 2 * R]);
                acc_sub(s, Z[ey][sx + j - 1]);
                X[ey][sx + j] = s;
            }
        }
        box3_barrier();
        // y-window: kTX columns x (kTY / kKY) segments; lanes on consecutive x (coalesced)
        const int tx = threadIdx.x % kTX, sy = (threadIdx.x / kTX) * kKY;
        const int gx = x0 + tx;
        TA s;
        acc_zero(s);
#pragma unroll
        for (int j = 0; j <= 2 * R; ++j) acc_add(s, X[sy + j][tx]);
#pragma unroll
        for (int j = 0; j < kKY; ++j) {
            if (j > 0) {
                acc_add(s, X[sy + j + 2 * R][tx]);
                acc_sub(s, X[sy + j - 1][tx]);
            }
            const int gy = y0 + sy + j;
            if (gx < nx && gy < ny) put(ovol[(int64_t)z * plane + (int64_t)gy * nx + gx], s);
        }
        // (the next step's Z writes come after every thread passed the barrier above, i.e.
        //  after all x-window reads of Z; the next X writes follow its first barrier)
    };
    TA zs[NPT];
    TV pa[NPT];
    if constexpr (box3_ring<R, TV, NPT>()) {
        // ring[j] holds slice z0 - R - 1 + j (mod W): the leaving slice of step z sits in slot
        // (z - z0) % W, the slot the entering slice z + R then takes over
        TV ring[W][NPT];
#pragma unroll
        for (int k = 0; k < NPT; ++k) {
            acc_zero(zs[k]);
#pragma unroll
            for (int j = 0; j < W; ++j) {  // the window of slice z0 - 1
                ring[j][k] = load(z0 - R - 1 + j, k);
                acc_add(zs[k], ring[j][k]);
            }
            pa[k] = load(z0 + R, k);
        }
        for (int zb = z0; zb < z1; zb += W) {
#pragma unroll
            for (int j = 0; j < W; ++j) {
                const int z = zb + j;
                if (z < z1) {  // uniform per workgroup
#pragma unroll
                    for (int k = 0; k < NPT; ++k) {
                        acc_add(zs[k], pa[k]);
                        acc_sub(zs[k], ring[j][k]);
                        ring[j][k] = pa[k];
                        if (ey_[k] >= 0) Z[ey_[k]][ex_[k]] = zs[k];
                    }
#pragma unroll
                    for (int k = 0; k < NPT; ++k) pa[k] = load(z + 1 + R, k);
                    xy_windows(z);
                }
            }
        }
    } else {
#pragma unroll
        for (int k = 0; k < NPT; ++k) {  // window of slice z0 - 1
            acc_zero(zs[k]);
            for (int z = z0 - 1 - R; z <= z0 - 1 + R; ++z) acc_add(zs[k], load(z, k));
        }
        TV ps[NPT];
#pragma unroll
        for (int k = 0; k < NPT; ++k) {
            pa[k] = load(z0 + R, k);
            ps[k] = load(z0 - R - 1, k);
        }
        for (int z = z0; z < z1; ++z) {
#pragma unroll
            for (int k = 0; k < NPT; ++k) {
                acc_add(zs[k], pa[k]);
                acc_sub(zs[k], ps[k]);
                if (ey_[k] >= 0) Z[ey_[k]][ex_[k]] = zs[k];
            }
#pragma unroll
            for (int k = 0; k < NPT; ++k) {  // next step's entering / leaving slices
                pa[k] = load(z + 1 + R, k);
                ps[k] = load(z - R, k);
            }
            xy_windows(z);
        }
    }
}

// ---- three-kernel form (round 4): stage 2 as box3 of the t-window sums ------------------------
// box4(a, b) = box3(tbox(a, b)) (the sums are separable; stage 2 is rounded to f32 anyway), so
//   K2t: per voxel, all T timepoints in registers: U4 = t-window of U3 (exact), u, a, b, and
//        TAB(t) = t-window sums of (a, b) (f64, rounded to f32 once) for the OUTPUT timepoints
//        only, written over U3's storage (a thread reads every U3 of its voxel first);
//   K3f: box3 z-march of TAB over the output box with the final stage fused into its output:
//        mean = (f32)S4 / c4, out = RN(RN(v * ma) + mb) (guided_filter.rs:144-163), stored as TOut.
// Against K2 / K3 / K4 this drops the AB and S3 round trips and K3's halo timepoints: about
// 12 + 12 + 16 B per voxel instead of ~64.
template <int TMAX, int R>
__global__ __launch_bounds__(256) void g4_tab_kernel(double* __restrict__ U3T,
                                                     const float* __restrict__ v, int T, int t0,
                                                     int ont, int nz, int ny, int nx, float eps,
                                                     Str3 vs) {
    const int64_t vol = (int64_t)nz * ny * nx;
    const int x = blockIdx.x * kPX + threadIdx.x, y = blockIdx.y * kPY + threadIdx.y;
    if (x >= nx || y >= ny) return;
    const int cyx = ccount(y, ny, R) * ccount(x, nx, R);
    float2* TAB = reinterpret_cast<float2*>(U3T);
    const int tlo = t0 - R, thi = t0 + ont + R;  // (a, b) needed on [tlo, thi)
    for (int z = blockIdx.z; z < nz; z += gridDim.z) {
        const int64_t i = ((int64_t)z * ny + y) * nx + x;
        const int c3 = ccount(z, nz, R) * cyx;
        double U[TMAX];
#pragma unroll
        for (int t = 0; t < TMAX; ++t) U[t] = t < T ? U3T[t * vol + i] : 0.0;
        float2 ab[TMAX];
        double W = 0.0;  // t-window of U3 for timepoint t (values past T are 0)
#pragma unroll
        for (int j = 0; j < R && j < TMAX; ++j) W += U[j];
#pragma unroll
        for (int t = 0; t < TMAX + R; ++t) {
            if (t < TMAX) {
                if (t + R < TMAX) W += U[t + R];
                if (t - R - 1 >= 0) W -= U[t - R - 1];
                ab[t] = make_float2(0.f, 0.f);
                if (t < T && t >= tlo && t < thi) {
                    const int ta = max(t - R, 0), tb = min(t + R, T - 1);
                    const float cnt = (float)(c3 * (tb - ta + 1));
                    const float u = (float)W / cnt;  // summed_area_table_mean
                    const float d = v[t * vs.t + (int64_t)z * vs.z + (int64_t)y * vs.y + x] - u;
                    const float sq = d * d;  // (v - u).powf(2.0)
                    const float a = sq / (sq + eps);
                    ab[t] = make_float2(a, (1.0f - a) * u);
                }
            }
            const int tt = t - R;  // every (a, b) of its window is known now
            if (tt >= 0 && tt < TMAX && tt < T && tt >= t0 && tt < t0 + ont) {
                double sa = 0.0, sb = 0.0;
#pragma unroll
                for (int j = -R; j <= R; ++j)
                    if (tt + j >= 0 && tt + j < TMAX) {
                        sa += (double)ab[tt + j].x;
                        sb += (double)ab[tt + j].y;
                    }
                TAB[(int64_t)(tt - t0) * vol + i] = make_float2((float)sa, (float)sb);
            }
        }
    }
}

// ---- t-march stage 1 (round 5): K1 and K2t in one kernel, no U3 in HBM --------------------------
// One workgroup owns a 16 x 16 x kMZ (x, y, z) tile of the TAB region (the output box + R, clamped to
// the block) and marches along t. Per step t it stages v(t) on the tile + 2R apron in LDS and forms
// U3(t) = the exact f64 3-D window sums of its voxels (x, y passes through LDS, the z pass from LDS
// into registers); each thread keeps, for its VP voxels, a register ring of the last 2R + 1 U3 and
// (a, b) values, so U4 = the t-window of U3 (exact), u, a, b (guided_filter.rs:126-142 with 4-D
// counts) and TAB = the t-window sums of (a, b) (f64, rounded to f32 once) follow R and 2R steps
// later, exactly as g4_tab_kernel forms them from U3. The t-march is unrolled by 2R + 1 so every
// ring slot is a compile-time register. HBM: v once (+ the apron's L2 / MALL re-reads) and TAB
// written; the f64 U3 (8 B per input voxel written and read back) never leaves the CU.
#ifndef G4_TM_PFD
#define G4_TM_PFD 1  // stage loads issued this many steps ahead (1-4 within 2 %)
#endif
#ifndef G4_TM_KX
#define G4_TM_KX 4  // t-march x-pass outputs per item
#endif
#ifndef G4_TM_KY
#define G4_TM_KY 4  // t-march y-pass outputs per item
#endif
#ifndef G4_TM_VP
#define G4_TM_VP 3  // t-march voxels per thread (along z): 1024 threads, 128 VGPRs, 4 waves per SIMD
                    // (4 voxels: 768 threads, 3 waves, 1.6 % slower; profiles/r06_tmarch_vp3.txt)
#endif
constexpr int kMX = 16, kMY = 16, kMZ = kG4TmarchTileZ;  // tile (x, y, z) (g4_limits.hpp)
constexpr int kMVP = G4_TM_VP, kMNT = kMX * kMY * kMZ / kMVP;  // voxels per thread; threads

// Buffer (SRD) accesses of the t-march: 32-bit byte offsets from a per-step base, out-of-range
// offsets read 0 / drop the store, so the march has no branch around a memory instruction (the
// compiler's vmcnt accounting then keeps the next step's loads in flight across the barriers).
using g4rsrc = __amdgpu_buffer_rsrc_t;
typedef unsigned int u32x2g4 __attribute__((ext_vector_type(2)));
constexpr int kG4Bad = (int)0x80000000;
__device__ __forceinline__ g4rsrc g4_rsrc(const void* base, uint32_t bytes) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, (int)bytes,
                                             0x00020000);
}
__device__ __forceinline__ float g4_ld(g4rsrc r, int off) {
    return __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(r, off, 0, 0));
}
// LDS-only workgroup barrier (__syncthreads would also wait for the loads in flight)
__device__ __forceinline__ void g4_lds_barrier() {
    __asm__ volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
}
__device__ __forceinline__ int g4_opaque(int v) {
    __asm__ volatile("" : "+v"(v));
    return v;
}

// g4_tmarch_offsets_fit (g4_limits.hpp): the host check of the t-march's 32-bit offsets.

// x / d for an integer count d given rcp = RN(1/d): Markstein's correction makes the quotient
// correctly rounded (= IEEE division) in 3 VALU ops (as gf_fused.hpp's div_by_count).
__device__ __forceinline__ float g4_div_by_count(float x, float d, float rcp) {
    const float q = x * rcp;
    const float r = __builtin_fmaf(-q, d, x);
    return __builtin_fmaf(r, rcp, q);
}
// s / (s + eps): rcp, one Newton step and Markstein's correction (within 1 ulp, almost always
// correctly rounded; 0/0 gives NaN as in the reference), as gf_fused.hpp's fast_div.
__device__ __forceinline__ float g4_fast_div(float x, float d) {
    float y = __builtin_amdgcn_rcpf(d);
    const float e = __builtin_fmaf(-d, y, 1.0f);
    y = __builtin_fmaf(e, y, y);
    const float q = x * y;
    const float r = __builtin_fmaf(-d, q, x);
    return __builtin_fmaf(r, y, q);
}

template <int R>
__global__ __launch_bounds__(kMNT) void g4_tmarch_tab_kernel(const float* __restrict__ v, Str3 vs,
                                                             float2* __restrict__ TAB, int T,
                                                             int t0, int ont, int nz, int ny,
                                                             int nx, int zlo, int ylo, int xlo,
                                                             int tnx, int tny, int tnz, int ntx,
                                                             int nty, float eps) {
    constexpr int W = 2 * R + 1, VP = kMVP;
    constexpr int SX = kMX + 2 * R, SY = kMY + 2 * R, SZ = kMZ + 2 * R, NS = SX * SY * SZ;
    constexpr int NPS = (NS + kMNT - 1) / kMNT;  // staged elements per thread
    constexpr int KX = G4_TM_KX, KY = G4_TM_KY;  // x / y sliding outputs per item
    constexpr int NXI = SZ * SY * (kMX / KX);    // x-pass items
    constexpr int NYI = SZ * kMX * (kMY / KY);   // y-pass items
    static_assert(kMZ % VP == 0 && kMX * kMY * (kMZ / VP) == kMNT, "voxels cover the tile");
    // (padded LDS pitches that remove the x pass's 4-way bank conflicts measured within 1 %:
    //  profiles/r05_tmarch_ab.txt, call J; the index arithmetic costs the registers instead)
    __shared__ float Vs[SZ][SY][SX];
    __shared__ double Xs[SZ][SY][kMX];
    __shared__ double Ys[SZ][kMY][kMX];
    // RN(1/c) for the 4-D window counts c <= (2R+1)^4 (u by Markstein's correction: = IEEE)
    constexpr int W4 = (2 * R + 1) * (2 * R + 1) * (2 * R + 1) * (2 * R + 1);
    __shared__ float rtab[W4 + 1];
    for (int c = threadIdx.x; c <= W4; c += kMNT) rtab[c] = c > 0 ? 1.0f / (float)c : 0.0f;
    g4_lds_barrier();

    // XCD-aware block order (xcd_block): each XCD marches a contiguous run of neighbouring tiles
    const int64_t nb = gridDim.x;
    const int64_t b = blockIdx.x;
    const int64_t lid = nb % 8 == 0 ? (b % 8) * (nb / 8) + b / 8 : b;
    const int tx = (int)(lid % ntx), ty = (int)((lid / ntx) % nty), tz = (int)(lid / ((int64_t)ntx * nty));
    const int x0 = xlo + tx * kMX, y0 = ylo + ty * kMY, z0 = zlo + tz * kMZ;
    const int xend = xlo + tnx, yend = ylo + tny, zend = zlo + tnz;

    // staged elements: v(t) on the tile + 2R apron, staged through LDS (one coalesced load per
    // element; reading each x-pass item's row segment straight from global memory instead, 1.6x
    // the load instructions, measured 1.35x slower: profiles/r05_tmarch_ab.txt). Byte offsets
    // from plane z0 - R of a timepoint, shifted up to plane 0 when that plane lies below the
    // block (buffer bases must not precede the allocation); kG4Bad outside the block (reads 0:
    // the zero padding of the clamped windows).
    const int zsh = min(z0 - R, 0);
    const int64_t vbase = (int64_t)(z0 - R - zsh) * vs.z;
    int soff[NPS];
#pragma unroll
    for (int k = 0; k < NPS; ++k) {
        const int e = threadIdx.x + k * kMNT;
        const int ez = e / (SY * SX), ey = (e / SX) % SY, ex = e % SX;
        const int gz = z0 - R + ez, gy = y0 - R + ey, gx = x0 - R + ex;
        const bool in = e < NS && gz >= 0 && gz < nz && gy >= 0 && gy < ny && gx >= 0 && gx < nx;
        soff[k] = in ? (int)(((ez + zsh) * vs.z + gy * vs.y + gx) * 4) : kG4Bad;
    }
    // (soff, voff and toff are step-invariant registers with kG4Bad already selected, so the
    //  accesses take them as they are: passing them through g4_opaque added a register copy per
    //  access, 1 % of the T share, profiles/r06_plain_offsets.txt)
    // staged values of steps t + 1 .. t + PFD (pre[0 .. PFD - 1]): the loads of a step stay in
    // flight for PFD steps
    constexpr int PFD = G4_TM_PFD;
    float pre[PFD][NPS];
    auto load_stage = [&](float (&dst)[NPS], int t) {
        const bool ok = (unsigned)t < (unsigned)T;
        const g4rsrc r = g4_rsrc(v + (ok ? (int64_t)t * vs.t + vbase : 0), ok ? 0x7FFFFFF0u : 0u);
#pragma unroll
        for (int k = 0; k < NPS; ++k) dst[k] = g4_ld(r, soff[k]);
    };

    // this thread's voxels: (x, y) and VP consecutive z
    const int lx = threadIdx.x % kMX, ly = (threadIdx.x / kMX) % kMY,
              lz = VP * (threadIdx.x / (kMX * kMY));
    const int gx = x0 + lx, gy = y0 + ly;
    bool own[VP];
    int c3[VP], toff[VP], voff[VP];  // count; TAB and v byte offsets from the tile's plane z0
#pragma unroll
    for (int q = 0; q < VP; ++q) {
        const int gz = z0 + lz + q;
        own[q] = gx < xend && gy < yend && gz < zend;
        c3[q] = ccount(gz, nz, R) * ccount(gy, ny, R) * ccount(gx, nx, R);
        toff[q] = own[q] ? (((lz + q) * ny + gy) * nx + gx) * 8 : kG4Bad;
        voff[q] = own[q] ? (int)(((lz + q) * vs.z + gy * vs.y + gx) * 4) : kG4Bad;
    }
    const int64_t vol = (int64_t)nz * ny * nx;
    const int tlo = t0 - R, thi = t0 + ont + R;  // (a, b) needed on [tlo, thi)
    const int tb = max(0, t0 - 2 * R), te = min(T, t0 + ont + 2 * R);  // U3 needed on [tb, te)
    const int nsteps = (te - tb + 2 * R + W - 1) / W * W;

    double ru[W][VP];   // U3 ring: slot (t - tb) % W holds U3(t)
    float2 rab[W][VP];  // (a, b) ring: slot (tau - tb) % W holds ab(tau)
    double SA[VP], SB[VP];  // running t-window sums of (a, b) (exact: f64 sums of f32 values)

#pragma unroll
    for (int q = 0; q < VP; ++q) {
        SA[q] = SB[q] = 0.0;
#pragma unroll
        for (int j = 0; j < W; ++j) {
            ru[j][q] = 0.0;
            rab[j][q] = make_float2(0.f, 0.f);
        }
    }
#pragma unroll
    for (int d = 0; d < PFD; ++d) load_stage(pre[d], tb + d);
    for (int tb0 = tb; tb0 < tb + nsteps; tb0 += W) {
        g4_static_for<0, W>([&](auto kc) {
            constexpr int k = decltype(kc)::value;
            const int t = tb0 + k;
            const int tau = t - R;  // (a, b) of this step
            const int tp = tau - R;  // TAB of this step: the t-window [tp - R, tp + R] of (a, b)
            // v(tau) at this thread's voxels, for s = (v - u)^2 (read early, used last)
            float vt[VP];
            {
                const bool ok = (unsigned)tau < (unsigned)T;
                const g4rsrc r = g4_rsrc(v + (ok ? (int64_t)tau * vs.t + (int64_t)z0 * vs.z : 0),
                                         ok ? 0x7FFFFFF0u : 0u);
#pragma unroll
                for (int q = 0; q < VP; ++q) vt[q] = g4_ld(r, voff[q]);
            }
            double u3[VP];
#pragma unroll
            for (int q = 0; q < VP; ++q) u3[q] = 0.0;
            // stage 1 of step t; past te its U3 feeds no emitted window, so the LDS passes are
            // skipped there (a uniform branch with no global access inside)
            float* const Vf = &Vs[0][0][0];
#pragma unroll
            for (int j = 0; j < NPS; ++j)
                if (threadIdx.x + j * kMNT < NS) Vf[threadIdx.x + j * kMNT] = pre[0][j];
#pragma unroll
            for (int d = 0; d + 1 < PFD; ++d)
#pragma unroll
                for (int j = 0; j < NPS; ++j) pre[d][j] = pre[d + 1][j];
            load_stage(pre[PFD - 1], t + PFD);
            if (t < te) {
            g4_lds_barrier();
            for (int it = threadIdx.x; it < NXI; it += kMNT) {  // x-window sums (exact f64)
                const int row = it / (kMX / KX), sx = (it % (kMX / KX)) * KX;
                const float* src = &Vs[0][0][0] + row * SX + sx;
                double* dst = &Xs[0][0][0] + row * kMX + sx;
                double s = 0.0;
#pragma unroll
                for (int j = 0; j <= 2 * R; ++j) s += (double)src[j];
                dst[0] = s;
#pragma unroll
                for (int j = 1; j < KX; ++j) {
                    s += (double)src[j + 2 * R];
                    s -= (double)src[j - 1];
                    dst[j] = s;
                }
            }
            g4_lds_barrier();
            for (int it = threadIdx.x; it < NYI; it += kMNT) {  // y-window sums, lanes on x
                const int xx = it % kMX, sy = ((it / kMX) % (kMY / KY)) * KY,
                          ez = it / (kMX * (kMY / KY));
                double s = 0.0;
#pragma unroll
                for (int j = 0; j <= 2 * R; ++j) s += Xs[ez][sy + j][xx];
                Ys[ez][sy][xx] = s;
#pragma unroll
                for (int j = 1; j < KY; ++j) {
                    s += Xs[ez][sy + j + 2 * R][xx];
                    s -= Xs[ez][sy + j - 1][xx];
                    Ys[ez][sy + j][xx] = s;
                }
            }
            g4_lds_barrier();
            {  // z-window sums of this thread's VP voxels (exact f64)
                double zs[VP + 2 * R];
#pragma unroll
                for (int j = 0; j < VP + 2 * R; ++j) zs[j] = Ys[lz + j][ly][lx];
                double s = 0.0;
#pragma unroll
                for (int j = 0; j <= 2 * R; ++j) s += zs[j];
                u3[0] = s;
#pragma unroll
                for (int q = 1; q < VP; ++q) {
                    s += zs[q + 2 * R];
                    s -= zs[q - 1];
                    u3[q] = s;
                }
            }
            }
            // U4(tau): the t-window [t - 2R, t] of U3, the ring after U3(t) entered
            constexpr int su = k, sab = (k - R + W) % W;
            const bool need_ab = tau >= tlo && tau < thi && tau >= 0 && tau < T;
            const int ct = min(tau + R, T - 1) - max(tau - R, 0) + 1;
            const bool emit = tp >= t0 && tp < t0 + ont;
            const g4rsrc rt = g4_rsrc(TAB + (emit ? (int64_t)(tp - t0) * vol + (int64_t)z0 * ny * nx : 0),
                                      emit ? 0x7FFFFFF0u : 0u);
#pragma unroll
            for (int q = 0; q < VP; ++q) {
                ru[su][q] = u3[q];
                double U4 = 0.0;  // the ring's sum (exact: any order; a running sum spills)
#pragma unroll
                for (int j = 0; j < W; ++j) U4 += ru[j][q];
                // u = RN(U4) / c (summed_area_table_mean: Markstein = IEEE division); a within
                // 1 ulp (IEEE divisions here: 1.2 % slower, profiles/r06_tmarch_fastdiv.txt)
                const int ci = c3[q] * ct;
                const float u = g4_div_by_count((float)U4, (float)ci, rtab[ci]);
                const float d = vt[q] - u;
                const float sq = d * d;  // (v - u).powf(2.0)
                const float a = g4_fast_div(sq, sq + eps);
                const float2 ab = need_ab ? make_float2(a, (1.0f - a) * u) : make_float2(0.f, 0.f);
                SA[q] += (double)ab.x;
                SB[q] += (double)ab.y;
                SA[q] -= (double)rab[sab][q].x;
                SB[q] -= (double)rab[sab][q].y;
                rab[sab][q] = ab;
                const float2 o = make_float2((float)SA[q], (float)SB[q]);
                __builtin_amdgcn_raw_buffer_store_b64(
                    (u32x2g4){__float_as_uint(o.x), __float_as_uint(o.y)}, rt, toff[q], 0, 0);
            }
        });
    }
}

__device__ __forceinline__ void store_dtype(void* out, int dtype, int64_t i, float o) {
    switch (dtype) {
    case kBool: case kU8: static_cast<uint8_t*>(out)[i] = from_f32<uint8_t>(o); break;
    case kI8: static_cast<int8_t*>(out)[i] = from_f32<int8_t>(o); break;
    case kI16: static_cast<int16_t*>(out)[i] = from_f32<int16_t>(o); break;
    case kI32: static_cast<int32_t*>(out)[i] = from_f32<int32_t>(o); break;
    case kI64: static_cast<int64_t*>(out)[i] = from_f32<int64_t>(o); break;
    case kU16: static_cast<uint16_t*>(out)[i] = from_f32<uint16_t>(o); break;
    case kU32: static_cast<uint32_t*>(out)[i] = from_f32<uint32_t>(o); break;
    case kU64: static_cast<uint64_t*>(out)[i] = from_f32<uint64_t>(o); break;
    case kBF16: static_cast<bf16_t*>(out)[i] = from_f32<bf16_t>(o); break;
    case kF16: static_cast<f16_t*>(out)[i] = from_f32<f16_t>(o); break;
    case kF64: static_cast<double*>(out)[i] = from_f32<double>(o); break;
    default: static_cast<float*>(out)[i] = o; break;
    }
}

// K3f: one workgroup marches one 64 x kTY xy tile of the OUTPUT box through a z segment of it, for
// one output timepoint; the running z-window (f64 pair) covers the tile's R apron, whose loads
// reach into the block's halo (zero outside the block: the clamped windows). The leaving slice
// comes from a register ring when it fits (box3_ring), as in box3_march_kernel.
// TYF: output tile height (kTY; 64 x 32 tiles measured 55.9 against 54.0 ms on the T share in
// round 4, and in the F32 form 14.64 against 13.76 ms per launch in round 6:
// profiles/r06_box3final_ty32.txt)
// F32 (f32 output, unit x strides, 32-bit offsets checked on the host: box3_final_f32_fits):
// every global access is a buffer access with an out-of-range offset instead of a branch, the
// step barriers wait for LDS only and the march runs whole blocks of 2R + 1 steps (the padded
// steps store nothing), so the next step's TAB loads stay in flight across the barriers.
template <int R, bool RING, int TYF, bool F32 = false>
__global__ __launch_bounds__(RING ? kTX * TYF / 2 : kNT) void box3_final_kernel(
    const float2* __restrict__ TAB,
                                                         const float* __restrict__ v,
                                                         void* __restrict__ out, int dtype_out,
                                                         NdGeom g, int zseg, int tiles_x,
                                                         int tiles_y, Str3 vs) {
    static_assert(!F32 || RING, "the buffer-access form is the ring march");
    // RING: two outputs per thread in the y-window (512 threads for 64 x 16 tiles), so a thread
    // owns half the apron points and its ring fits without cutting occupancy
    constexpr int NT = RING ? kTX * TYF / 2 : kNT, KY = kTX * TYF / NT;
    constexpr int EX = kTX + 2 * R, EY = TYF + 2 * R, NE = EX * EY;
    constexpr int NPT = (NE + NT - 1) / NT;
    constexpr int W = 2 * R + 1;
    // the running z-window is an f64 pair in registers (exact add / subtract); the x and y
    // windows of it go through LDS as f32 pairs (stage 2 is rounded to f32 anyway: half the LDS
    // bytes and f32 instead of f64 adds; the x / y sliding sums span kKX / kKY outputs only)
    __shared__ float2 Z[EY][EX];
    __shared__ float2 X[EY][kTX];
    const int T = (int)g.shape[0], nz = (int)g.shape[1], ny = (int)g.shape[2],
              nx = (int)g.shape[3];
    int bx, ot;
    xcd_block(bx, ot);
    const int t = ot + (int)g.out_start[0];
    const int ntile = tiles_x * tiles_y;
    const int seg = bx / ntile, tile = bx % ntile;
    const int ox0 = (int)g.out_start[3], oy0 = (int)g.out_start[2], oz0 = (int)g.out_start[1];
    const int ox1 = ox0 + (int)g.out_shape[3], oy1 = oy0 + (int)g.out_shape[2];
    const int x0 = ox0 + (tile % tiles_x) * kTX, y0 = oy0 + (tile / tiles_x) * TYF;
    const int z0 = oz0 + seg * zseg, z1 = min(z0 + zseg, oz0 + (int)g.out_shape[1]);
    const int64_t plane = (int64_t)ny * nx;
    const float2* vol = TAB + (int64_t)ot * nz * plane;
    const int ct = min(t + R, T - 1) - max(t - R, 0) + 1;

    // owned apron points: plane index (or -1) and Z offset (or -1). The ring variant needs every
    // register it can get: 32-bit plane indices (the host checks ny * nx < 2^31)
    using PI = std::conditional_t<RING, int, int64_t>;
    PI pidx[NPT];
    int zoff[NPT];
#pragma unroll
    for (int k = 0; k < NPT; ++k) {
        const int e = threadIdx.x + k * NT;
        const int ey = e / EX, ex = e % EX;
        const int gy = y0 - R + ey, gx = x0 - R + ex;
        zoff[k] = e < NE ? e : -1;  // Z[ey][ex] == (&Z[0][0])[e]
        pidx[k] = (e < NE && gy >= 0 && gy < ny && gx >= 0 && gx < nx) ? (PI)gy * nx + gx : (PI)-1;
    }
    float2* const Zf = &Z[0][0];
    // F32: the byte offsets of the owned apron points, this thread's v loads and output stores,
    // selected once (kG4Bad outside) and used as they are at every access
    int boff[NPT], vof[KY], oof[KY];
    if constexpr (F32) {
#pragma unroll
        for (int k = 0; k < NPT; ++k) boff[k] = pidx[k] >= 0 ? (int)pidx[k] * 8 : kG4Bad;
        const int tx = threadIdx.x % kTX, sy = (threadIdx.x / kTX) * KY;
        const int gx = x0 + tx;
#pragma unroll
        for (int j = 0; j < KY; ++j) {
            const int gy = y0 + sy + j;
            const bool in = gx < ox1 && gy < oy1;
            vof[j] = in ? (int)((gy * vs.y + gx) * 4) : kG4Bad;
            oof[j] = in ? (int)(((gy - oy0) * g.out_strides[2] + (gx - ox0)) * 4) : kG4Bad;
        }
    }
    // (selected at the access instead, through g4_opaque: box3_final 14.20 against 14.08 ms,
    //  profiles/r06_plain_offsets.txt)
    auto load = [&](int z, int k) -> float2 {
        if constexpr (F32) {
            const bool ok = (unsigned)z < (unsigned)nz;
            const g4rsrc r = g4_rsrc(vol + (ok ? (int64_t)z * plane : 0), ok ? 0x7FFFFFF0u : 0u);
            const u32x2g4 q = __builtin_amdgcn_raw_buffer_load_b64(r, boff[k], 0, 0);
            return make_float2(__uint_as_float(q.x), __uint_as_float(q.y));
        } else {
            return (pidx[k] >= 0 && z >= 0 && z < nz) ? vol[(int64_t)z * plane + pidx[k]]
                                                       : make_float2(0.f, 0.f);
        }
    };
    auto step_barrier = [] {
        if constexpr (F32) g4_lds_barrier();
        else box3_barrier();
    };
    // F32: v of this thread's outputs of step z, loaded before the step's TAB prefetch so that
    // waiting for it does not wait for the prefetch (vmcnt counts in issue order)
    auto v_load = [&](int z, float (&vv)[KY]) {
        if constexpr (F32) {
            const bool zok = z < z1;
            const g4rsrc rv = g4_rsrc(v + (zok ? t * vs.t + (int64_t)z * vs.z : 0),
                                      zok ? 0x7FFFFFF0u : 0u);
#pragma unroll
            for (int j = 0; j < KY; ++j) vv[j] = g4_ld(rv, vof[j]);
        }
    };
    // x / y windows of the Z slice of output slice z and the final stage
    auto xy_final = [&](int z, const float (&vvp)[KY]) {
        step_barrier();
        for (int it = threadIdx.x; it < EY * (kTX / kKX); it += NT) {
            const int ey = it / (kTX / kKX), sx = (it % (kTX / kKX)) * kKX;
            float2 sacc = make_float2(0.f, 0.f);
#pragma unroll
            for (int j = 0; j <= 2 * R; ++j) acc_add(sacc, Z[ey][sx + j]);
            X[ey][sx] = sacc;
#pragma unroll
            for (int j = 1; j < kKX; ++j) {
                acc_add(sacc, Z[ey][sx + j + 2 * R]);
                acc_sub(sacc, Z[ey][sx + j - 1]);
                X[ey][sx + j] = sacc;
            }
        }
        step_barrier();
        const int tx = threadIdx.x % kTX, sy = (threadIdx.x / kTX) * KY;
        const int gx = x0 + tx;
        const int czx = ccount(min(z, nz - 1), nz, R) * ccount(gx, nx, R) * ct;
        float2 sacc = make_float2(0.f, 0.f);
#pragma unroll
        for (int j = 0; j <= 2 * R; ++j) acc_add(sacc, X[sy + j][tx]);
#pragma unroll
        for (int j = 0; j < KY; ++j) {
            if (j > 0) {
                acc_add(sacc, X[sy + j + 2 * R][tx]);
                acc_sub(sacc, X[sy + j - 1][tx]);
            }
            const int gy = y0 + sy + j;
            if constexpr (F32) {
                // z past the segment (padded steps): zero-record descriptors, nothing stored
                const bool zok = z < z1;
                const bool in = gx < ox1 && gy < oy1;
                const float cnt = (float)(czx * ccount(min(gy, ny - 1), ny, R));
                const float ma = (float)sacc.x / cnt, mb = (float)sacc.y / cnt;
                const float o = __fadd_rn(__fmul_rn(vvp[j], ma), mb);  // v *= ma; v += mb
                const g4rsrc ro = g4_rsrc(
                    static_cast<float*>(out) +
                        (zok ? ot * g.out_strides[0] + (int64_t)(z - oz0) * g.out_strides[1] : 0),
                    zok ? 0x7FFFFFF0u : 0u);
                (void)in;
                __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(o), ro, oof[j], 0, 2);
            } else if (gx < ox1 && gy < oy1) {
                const float cnt = (float)(czx * ccount(gy, ny, R));
                const float ma = (float)sacc.x / cnt, mb = (float)sacc.y / cnt;
                const float vv = v[t * vs.t + (int64_t)z * vs.z + (int64_t)gy * vs.y + gx];
                const float o = __fadd_rn(__fmul_rn(vv, ma), mb);  // v *= ma; v += mb
                store_dtype(out, dtype_out,
                            ot * g.out_strides[0] + (z - oz0) * g.out_strides[1] +
                                (gy - oy0) * g.out_strides[2] + (gx - ox0) * g.out_strides[3],
                            o);
            }
        }
    };
    dd2 zs[NPT];
    float2 pa[NPT];
    if constexpr (RING && box3_ring<R, float2, NPT>()) {
        float2 ring[W][NPT];  // slot (z - z0) % W: the leaving slice of step z (box3_march_kernel)
#pragma unroll
        for (int k = 0; k < NPT; ++k) {
            acc_zero(zs[k]);
#pragma unroll
            for (int j = 0; j < W; ++j) {
                ring[j][k] = load(z0 - R - 1 + j, k);
                acc_add(zs[k], ring[j][k]);
            }
            pa[k] = load(z0 + R, k);
        }
        for (int zb = z0; zb < z1; zb += W) {
#pragma unroll
            for (int j = 0; j < W; ++j) {
                const int z = zb + j;
                if (F32 || z < z1) {  // uniform per workgroup (F32: padded steps store nothing)
#pragma unroll
                    for (int k = 0; k < NPT; ++k) {
                        acc_add(zs[k], pa[k]);
                        acc_sub(zs[k], ring[j][k]);
                        ring[j][k] = pa[k];
                        if (zoff[k] >= 0) Zf[zoff[k]] = make_float2((float)zs[k].x, (float)zs[k].y);
                    }
                    float vv[KY];
                    v_load(z, vv);
#pragma unroll
                    for (int k = 0; k < NPT; ++k) pa[k] = load(z + 1 + R, k);
                    xy_final(z, vv);
                }
            }
        }
    } else {
#pragma unroll
        for (int k = 0; k < NPT; ++k) {  // window of slice z0 - 1
            acc_zero(zs[k]);
            for (int z = z0 - 1 - R; z <= z0 - 1 + R; ++z) acc_add(zs[k], load(z, k));
        }
        float2 ps[NPT];
#pragma unroll
        for (int k = 0; k < NPT; ++k) {
            pa[k] = load(z0 + R, k);
            ps[k] = load(z0 - R - 1, k);
        }
        for (int z = z0; z < z1; ++z) {
#pragma unroll
            for (int k = 0; k < NPT; ++k) {
                acc_add(zs[k], pa[k]);
                acc_sub(zs[k], ps[k]);
                if (zoff[k] >= 0) Zf[zoff[k]] = make_float2((float)zs[k].x, (float)zs[k].y);
            }
            float vv[KY] = {};
            v_load(z, vv);  // F32 only (the generic form reads v in xy_final)
#pragma unroll
            for (int k = 0; k < NPT; ++k) {
                pa[k] = load(z + 1 + R, k);
                ps[k] = load(z - R, k);
            }
            xy_final(z, vv);
        }
    }
}

template <int R, typename TV, typename TA, typename TO>
hipError_t launch_box3(const TV* in, TO* out, int T, int nz, int ny, int nx, Str3 is,
                       hipStream_t s) {
    const int tiles_x = (nx + kTX - 1) / kTX, tiles_y = (ny + kTY - 1) / kTY;
    const int64_t tiles = (int64_t)tiles_x * tiles_y;
    // z segments: enough workgroups for the chip (>= ~4 per CU), at least 16 slices each
    int nseg = (int)std::max<int64_t>(1, std::min<int64_t>((nz + 15) / 16, (4096 + tiles * T - 1) / (tiles * T)));
    const int zseg = (nz + nseg - 1) / nseg;
    nseg = (nz + zseg - 1) / zseg;
    const int64_t gx = tiles * nseg;
    if (gx > 0x7FFFFFFF || T > 65535) return hipErrorInvalidValue;
    hipLaunchKernelGGL((box3_march_kernel<R, TV, TA, TO>), dim3((unsigned)gx, (unsigned)T),
                       dim3(kNT), 0, s, in, out, nz, ny, nx, zseg, tiles_x, tiles_y, is);
    return hipGetLastError();
}

template <typename TV, typename TA, typename TO>
hipError_t launch_box3_r(int r, const TV* in, TO* out, int T, int nz, int ny, int nx, Str3 is,
                         hipStream_t s) {
    switch (r) {
    case 1: return launch_box3<1, TV, TA, TO>(in, out, T, nz, ny, nx, is, s);
    case 2: return launch_box3<2, TV, TA, TO>(in, out, T, nz, ny, nx, is, s);
    case 3: return launch_box3<3, TV, TA, TO>(in, out, T, nz, ny, nx, is, s);
    case 4: return launch_box3<4, TV, TA, TO>(in, out, T, nz, ny, nx, is, s);
    case 5: return launch_box3<5, TV, TA, TO>(in, out, T, nz, ny, nx, is, s);
    case 6: return launch_box3<6, TV, TA, TO>(in, out, T, nz, ny, nx, is, s);
    default: return hipErrorInvalidValue;
    }
}

}  // namespace

// radius <= 6: the f64-pair LDS tiles of K3 stay within 64 KB; T <= 32 and ny <= 65535 are
// checked by the caller (K2 / K4 hold a voxel's timepoints in registers, y is grid.y)
bool guided4d_supports(int radius) { return radius >= 1 && radius <= 6; }

int64_t guided4d_scratch_bytes(int64_t numel, bool gather) {
    // U3 / TAB (8 B) | v (4 B, when the input is not a contiguous f32 block)
    return numel * (8 + (gather ? 4 : 0)) + 64;
}

hipError_t launch_guided4d(const void* in, int dtype_in, void* out, int dtype_out,
                           const NdGeom& g, int radius, float eps, void* scratch, hipStream_t s) {
    const int T = (int)g.shape[0], nz = (int)g.shape[1], ny = (int)g.shape[2],
              nx = (int)g.shape[3];
    const int64_t n = g.numel;
    if (n <= 0 || g.out_numel <= 0) return hipSuccess;
    if (T > 32) return hipErrorInvalidValue;
    char* base = static_cast<char*>(scratch);
    double* U3 = reinterpret_cast<double*>(base);  // U3, then TAB (float2) over it
    float2* TAB = reinterpret_cast<float2*>(base);
    // f32 with unit-stride x is read in place (strided t / z / y); other element types or
    // strides are first copied to C-order f32 in scratch
    const bool in_place = dtype_in == kF32 && g.in_strides[3] == 1;
    const float* v = static_cast<const float*>(in);
    Str3 vs{g.in_strides[0], g.in_strides[1], g.in_strides[2]};
    hipError_t e;
    if (!in_place) {
        float* vv = reinterpret_cast<float*>(base + n * 8);
        for (int t = 0; t < T; ++t) {
            const size_t esz = dtype_size(dtype_in);
            e = launch_cast_to_f32_3d(static_cast<const char*>(in) + esz * t * g.in_strides[0],
                                      dtype_in, g.in_strides[1], g.in_strides[2],
                                      vv + (int64_t)t * nz * ny * nx, nz, ny, nx, s);
            if (e != hipSuccess) return e;
        }
        v = vv;
        vs = Str3{(int64_t)nz * ny * nx, (int64_t)ny * nx, (int64_t)nx};
    }
    const int t0 = (int)g.out_start[0], ont = (int)g.out_shape[0];
    const int64_t onx = g.out_shape[3], ony = g.out_shape[2], onz = g.out_shape[1];
    // the t-march's buffer accesses use 32-bit byte offsets from per-step tile bases
    const int64_t vs3[3] = {vs.t, vs.z, vs.y};
    const bool tmarch_fits = g4_tmarch_offsets_fit(vs3, ny, nx, radius);
    if (radius <= 2 && tmarch_fits) {
        // stage 1 and the (a, b) t-window sums in one t-march (g4_tmarch_tab_kernel): TAB on the
        // voxels box3_final_kernel reads (the output box + R, and the plane its z-window seed
        // adds and removes again), clamped to the block
        const int oz0 = (int)g.out_start[1], oy0 = (int)g.out_start[2], ox0 = (int)g.out_start[3];
        const int zlo = std::max(0, oz0 - radius - 1), zhi = (int)std::min<int64_t>(nz, oz0 + onz + radius);
        const int ylo = std::max(0, oy0 - radius), yhi = (int)std::min<int64_t>(ny, oy0 + ony + radius);
        const int xlo = std::max(0, ox0 - radius), xhi = (int)std::min<int64_t>(nx, ox0 + onx + radius);
        const int ntx = (xhi - xlo + kMX - 1) / kMX, nty = (yhi - ylo + kMY - 1) / kMY,
                  ntz = (zhi - zlo + kMZ - 1) / kMZ;
        const int64_t nb = (int64_t)ntx * nty * ntz;
        if (nb <= 0) return hipSuccess;
        if (nb > 0x7FFFFFFF) return hipErrorInvalidValue;
#define ZT_G4_TM(RR)                                                                              \
        hipLaunchKernelGGL((g4_tmarch_tab_kernel<RR>), dim3((unsigned)nb), dim3(kMNT), 0, s, v, vs, \
                           TAB, T, t0, ont, nz, ny, nx, zlo, ylo, xlo, xhi - xlo, yhi - ylo,      \
                           zhi - zlo, ntx, nty, eps)
        if (radius == 1) ZT_G4_TM(1);
        else ZT_G4_TM(2);
#undef ZT_G4_TM
    } else {
        // K1: U3 = exact 3-D window sums of every timepoint; K2t: u, a, b and their t-window
        // sums for the output timepoints, written over U3 (a thread reads every U3 of its voxel
        // first)
        if (ny > 65535 || g.out_shape[2] > 65535) return hipErrorInvalidValue;  // K1 / K2t grids
        e = launch_box3_r<float, double, double>(radius, v, U3, T, nz, ny, nx, vs, s);
        if (e != hipSuccess) return e;
        const int64_t pgx = (nx + kPX - 1) / kPX, pgy = (ny + kPY - 1) / kPY;
        const dim3 pgrid((unsigned)pgx, (unsigned)pgy,
                         (unsigned)std::min<int64_t>(nz, std::max<int64_t>(1, 65536 / (pgy * pgx) + 1)));
        const dim3 pblock(kPX, kPY);
        auto k2t = [&](auto tm, auto rr) {
            constexpr int TM = decltype(tm)::value, RR = decltype(rr)::value;
            hipLaunchKernelGGL((g4_tab_kernel<TM, RR>), pgrid, pblock, 0, s, U3, v, T, t0, ont, nz,
                               ny, nx, eps, vs);
        };
        auto k2r = [&](auto tm) {
            switch (radius) {
            case 1: k2t(tm, std::integral_constant<int, 1>{}); break;
            case 2: k2t(tm, std::integral_constant<int, 2>{}); break;
            case 3: k2t(tm, std::integral_constant<int, 3>{}); break;
            case 4: k2t(tm, std::integral_constant<int, 4>{}); break;
            case 5: k2t(tm, std::integral_constant<int, 5>{}); break;
            case 6: k2t(tm, std::integral_constant<int, 6>{}); break;
            default: break;
            }
        };
        if (T <= 4) k2r(std::integral_constant<int, 4>{});
        else if (T <= 16) k2r(std::integral_constant<int, 16>{});
        else k2r(std::integral_constant<int, 32>{});
    }
    if ((e = hipGetLastError()) != hipSuccess) return e;
    // K3f: box3 z-march of TAB with the final stage (the z-window ring in registers; 32-bit plane
    // indices, so planes past 2^31 elements take the re-reading form)
    const bool ring = (int64_t)ny * nx < ((int64_t)1 << 31);
    // f32 output with unit x strides and 32-bit byte offsets within a TAB plane, a v plane and
    // an output plane: the buffer-access march
    const bool f32_fast = dtype_out == kF32 && g.out_strides[3] == 1 &&
                          (int64_t)ny * nx * 8 < ((int64_t)1 << 31) &&
                          ((ny - 1) * vs.y + nx) * 4 < ((int64_t)1 << 31) &&
                          ((ony - 1) * g.out_strides[2] + onx) * 4 < ((int64_t)1 << 31);
    const int tiles_x = (int)((onx + kTX - 1) / kTX), tiles_y = (int)((ony + kTY - 1) / kTY);
    const int64_t tiles = (int64_t)tiles_x * tiles_y;
    int nseg = (int)std::max<int64_t>(
        1, std::min<int64_t>((onz + 15) / 16, (4096 + tiles * ont - 1) / (tiles * ont)));
    const int zseg = (int)((onz + nseg - 1) / nseg);
    nseg = (int)((onz + zseg - 1) / zseg);
    const int64_t gx = tiles * nseg;
    if (gx > 0x7FFFFFFF || ont > 65535) return hipErrorInvalidValue;
    const dim3 fg((unsigned)gx, (unsigned)ont);
    switch (radius) {
#define ZT_G4_K3F(RR)                                                                             \
    case RR:                                                                                      \
        if (ring && f32_fast)                                                                     \
            hipLaunchKernelGGL((box3_final_kernel<RR, true, kTY, true>), fg, dim3(kTX * kTY / 2), 0,\
                               s, TAB, v, out, dtype_out, g, zseg, tiles_x, tiles_y, vs);         \
        else if (ring)                                                                            \
            hipLaunchKernelGGL((box3_final_kernel<RR, true, kTY>), fg, dim3(kTX * kTY / 2), 0, s, TAB,\
                               v, out, dtype_out, g, zseg, tiles_x, tiles_y, vs);                 \
        else                                                                                      \
            hipLaunchKernelGGL((box3_final_kernel<RR, false, kTY>), fg, dim3(kNT), 0, s, TAB, v,   \
                               out, dtype_out, g, zseg, tiles_x, tiles_y, vs);                    \
        break;
        ZT_G4_K3F(1) ZT_G4_K3F(2) ZT_G4_K3F(3) ZT_G4_K3F(4) ZT_G4_K3F(5) ZT_G4_K3F(6)
#undef ZT_G4_K3F
    default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

}  // namespace zt
