// guided4d.hip — the 4-D guided filter (config T: a (T, Z, Y, X) time series, every axis windowed
// alike, guided_filter.rs:117-199 with get_block clamping on all four axes).
//
// The box mean over (t, z, y, x) is separable and linear, so the 4-D sums are t-window sums of
// per-timepoint 3-D box sums:  box4(f)(t) = sum_{t' in W(t)} box3(f(t')). The default is three
// kernels (K1, then g4_tab_kernel and box3_final_kernel, described above them); ZT_G4_LEGACY=1
// keeps the original four over the halo'd block (windows clamp at the block bounds = the array
// bounds):
//   K1 box3_march<float -> double>:  U3(t) = 3-D window sums of v, exact f64 (f64 sums of f32
//       values), one z-march per (timepoint, xy tile);
//   K2 pointwise (all t of a voxel in one thread): U4 = t-window sums of U3 (exact),
//       u = RN(RN_f32(U4) / c4), s = (v-u)^2, a = s/(s+eps), b = (1-a)u  ->  AB (float2);
//   K3 box3_march<float2 -> float2>: S3(t) = 3-D window sums of (a, b), f64 accumulation rounded
//       to f32 once;
//   K4 final (output region only): S4 = t-window sums of S3 (f64), mean = RN_f32(S4) / c4,
//       out = RN(RN(v * mean_a) + mean_b) cast to TOut (guided_filter.rs:144-163, :101-102).
// HBM traffic about 64 B per voxel (v read twice, U3 / AB / S3 written and read once) against the
// separable path's ~160; every division is IEEE (correctly rounded), stage 1 exact, stage 2 with
// f64 accumulation, so the result is closer to the reference's f64-SAT means than the 3-D kernel's.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdlib>
#include <type_traits>

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

// K2: u, s, a, b for every timepoint of a voxel (guided_filter.rs:126-142) with 4-D counts.
// One thread per (y, x) of a 4 x 64 block (3-D grid: no 64-bit index division; 64-wide rows keep
// a chunk's 264-wide halo'd rows 83 % busy where 256-wide rows left half the lanes idle); the T
// values of U3 are read once into registers (T <= TMAX at compile time).
template <int TMAX>
__global__ __launch_bounds__(256) void g4_pointwise_kernel(const double* __restrict__ U3,
                                                           const float* __restrict__ v,
                                                           float2* __restrict__ AB, int T,
                                                           int ta_ab, int tb_ab, int nz, int ny,
                                                           int nx, int r, float eps, Str3 vs) {
    const int64_t vol = (int64_t)nz * ny * nx;
    const int x = blockIdx.x * kPX + threadIdx.x, y = blockIdx.y * kPY + threadIdx.y;
    if (x >= nx || y >= ny) return;
    const int cyx = ccount(y, ny, r) * ccount(x, nx, r);
    for (int z = blockIdx.z; z < nz; z += gridDim.z) {
        const int64_t i = ((int64_t)z * ny + y) * nx + x;
        const int c3 = ccount(z, nz, r) * cyx;
        double U[TMAX];
#pragma unroll
        for (int t = 0; t < TMAX; ++t) U[t] = t < T ? U3[t * vol + i] : 0.0;
#pragma unroll
        for (int t = 0; t < TMAX; ++t) {
            if (t >= T || t < ta_ab || t >= tb_ab) continue;  // only the (a, b) K4 reads
            double U4 = 0.0;
            const int ta = max(t - r, 0), tb = min(t + r, T - 1);
#pragma unroll
            for (int tt = 0; tt < TMAX; ++tt)
                if (tt >= ta && tt <= tb) U4 += U[tt];
            const float cnt = (float)(c3 * (tb - ta + 1));
            const float u = (float)U4 / cnt;  // summed_area_table_mean: (sum as f32) / count
            const float d = v[t * vs.t + (int64_t)z * vs.z + (int64_t)y * vs.y + x] - u;
            const float s = d * d;  // (v - u).powf(2.0)
            const float a = s / (s + eps);
            const float b = (1.0f - a) * u;
            AB[t * vol + i] = make_float2(a, b);
        }
    }
}

// K4: the output region [o0, o0 + on) of the block: t-window sums of S3, means, v*ma + mb.
template <int TMAX, typename TOut>
__global__ __launch_bounds__(256) void g4_final_kernel(const float2* __restrict__ S3,
                                                       const float* __restrict__ v,
                                                       TOut* __restrict__ out, NdGeom g, int r,
                                                       Str3 vs) {
    const int T = (int)g.shape[0], nz = (int)g.shape[1], ny = (int)g.shape[2],
              nx = (int)g.shape[3];
    const int64_t vol = (int64_t)nz * ny * nx;
    const int ox = blockIdx.x * kPX + threadIdx.x, oy = blockIdx.y * kPY + threadIdx.y;
    if (ox >= (int)g.out_shape[3] || oy >= (int)g.out_shape[2]) return;
    const int x = ox + (int)g.out_start[3], y = oy + (int)g.out_start[2];
    const int cyx = ccount(y, ny, r) * ccount(x, nx, r);
    const int t0 = (int)g.out_start[0], ont = (int)g.out_shape[0];
    const int tlo = max(t0 - r, 0), thi = min(t0 + ont + r, T);
    for (int oz = blockIdx.z; oz < (int)g.out_shape[1]; oz += gridDim.z) {
        const int z = oz + (int)g.out_start[1];
        const int64_t bi = ((int64_t)z * ny + y) * nx + x;
        const int c3 = ccount(z, nz, r) * cyx;
        const int64_t dbase = oz * g.out_strides[1] + oy * g.out_strides[2] + ox * g.out_strides[3];
        // only the timepoints the output windows read (a slab's outer halo timepoints feed
        // stage 1 alone)
        float2 S[TMAX];
#pragma unroll
        for (int t = 0; t < TMAX; ++t)
            S[t] = t >= tlo && t < thi ? S3[t * vol + bi] : make_float2(0.f, 0.f);
#pragma unroll
        for (int ot = 0; ot < TMAX; ++ot) {
            if (ot >= ont) continue;
            const int t = ot + t0;
            const int ta = max(t - r, 0), tb = min(t + r, T - 1);
            double sa = 0.0, sb = 0.0;
#pragma unroll
            for (int tt = 0; tt < TMAX; ++tt)
                if (tt >= ta && tt <= tb) {
                    sa += (double)S[tt].x;
                    sb += (double)S[tt].y;
                }
            const float cnt = (float)(c3 * (tb - ta + 1));
            const float ma = (float)sa / cnt, mb = (float)sb / cnt;
            const float vv = v[t * vs.t + (int64_t)z * vs.z + (int64_t)y * vs.y + x];
            const float o = __fadd_rn(__fmul_rn(vv, ma), mb);  // v *= ma; v += mb
            out[dbase + ot * g.out_strides[0]] = from_f32<TOut>(o);
        }
    }
}

// K2 / K4 for blocks of up to TMAX = 32 timepoints (config T's (t, z) block shares: 16 output
// timepoints plus the 2r halo): the t-window sums slide along t in registers (the radius R a
// template parameter, so the entering and leaving timepoints are compile-time register indices)
// instead of one masked sum per output timepoint (O(T) instead of O(T^2) adds per voxel). Values
// past T are zero, so the running window stays exact (f64 sums of f64 / f32 values).
template <int TMAX, int R>
__global__ __launch_bounds__(256) void g4_pointwise_slide_kernel(const double* __restrict__ U3,
                                                                 const float* __restrict__ v,
                                                                 float2* __restrict__ AB, int T,
                                                                 int ta_ab, int tb_ab, int nz,
                                                                 int ny, int nx, float eps,
                                                                 Str3 vs) {
    const int64_t vol = (int64_t)nz * ny * nx;
    const int x = blockIdx.x * kPX + threadIdx.x, y = blockIdx.y * kPY + threadIdx.y;
    if (x >= nx || y >= ny) return;
    const int cyx = ccount(y, ny, R) * ccount(x, nx, R);
    for (int z = blockIdx.z; z < nz; z += gridDim.z) {
        const int64_t i = ((int64_t)z * ny + y) * nx + x;
        const int c3 = ccount(z, nz, R) * cyx;
        double U[TMAX];
#pragma unroll
        for (int t = 0; t < TMAX; ++t) U[t] = t < T ? U3[t * vol + i] : 0.0;
        double W = 0.0;  // window of t = 0: [0, R]
#pragma unroll
        for (int j = 0; j <= R && j < TMAX; ++j) W += U[j];
#pragma unroll
        for (int t = 0; t < TMAX; ++t) {
            if (t > 0) {
                if (t + R < TMAX) W += U[t + R];
                if (t - R - 1 >= 0) W -= U[t - R - 1];
            }
            if (t >= T || t < ta_ab || t >= tb_ab) continue;  // only the (a, b) K4 reads
            const int ta = max(t - R, 0), tb = min(t + R, T - 1);
            const float cnt = (float)(c3 * (tb - ta + 1));
            const float u = (float)W / cnt;  // summed_area_table_mean: (sum as f32) / count
            const float d = v[t * vs.t + (int64_t)z * vs.z + (int64_t)y * vs.y + x] - u;
            const float sq = d * d;  // (v - u).powf(2.0)
            const float a = sq / (sq + eps);
            const float b = (1.0f - a) * u;
            AB[t * vol + i] = make_float2(a, b);
        }
    }
}

template <int TMAX, int R, typename TOut>
__global__ __launch_bounds__(256) void g4_final_slide_kernel(const float2* __restrict__ S3,
                                                             const float* __restrict__ v,
                                                             TOut* __restrict__ out, NdGeom g,
                                                             Str3 vs) {
    const int T = (int)g.shape[0], nz = (int)g.shape[1], ny = (int)g.shape[2],
              nx = (int)g.shape[3];
    const int64_t vol = (int64_t)nz * ny * nx;
    const int ox = blockIdx.x * kPX + threadIdx.x, oy = blockIdx.y * kPY + threadIdx.y;
    if (ox >= (int)g.out_shape[3] || oy >= (int)g.out_shape[2]) return;
    const int x = ox + (int)g.out_start[3], y = oy + (int)g.out_start[2];
    const int cyx = ccount(y, ny, R) * ccount(x, nx, R);
    const int t0 = (int)g.out_start[0], ont = (int)g.out_shape[0];
    const int tlo = max(t0 - R, 0), thi = min(t0 + ont + R, T);
    for (int oz = blockIdx.z; oz < (int)g.out_shape[1]; oz += gridDim.z) {
        const int z = oz + (int)g.out_start[1];
        const int64_t bi = ((int64_t)z * ny + y) * nx + x;
        const int c3 = ccount(z, nz, R) * cyx;
        const int64_t dbase = oz * g.out_strides[1] + oy * g.out_strides[2] + ox * g.out_strides[3];
        float2 S[TMAX];
#pragma unroll
        for (int t = 0; t < TMAX; ++t)
            S[t] = t >= tlo && t < thi ? S3[t * vol + bi] : make_float2(0.f, 0.f);
        double sa = 0.0, sb = 0.0;  // window of t = 0
#pragma unroll
        for (int j = 0; j <= R && j < TMAX; ++j) {
            sa += (double)S[j].x;
            sb += (double)S[j].y;
        }
#pragma unroll
        for (int t = 0; t < TMAX; ++t) {
            if (t > 0) {
                if (t + R < TMAX) { sa += (double)S[t + R].x; sb += (double)S[t + R].y; }
                if (t - R - 1 >= 0) { sa -= (double)S[t - R - 1].x; sb -= (double)S[t - R - 1].y; }
            }
            const int ot = t - t0;
            if (ot < 0 || ot >= ont || t >= T) continue;
            const int ta = max(t - R, 0), tb = min(t + R, T - 1);
            const float cnt = (float)(c3 * (tb - ta + 1));
            const float ma = (float)sa / cnt, mb = (float)sb / cnt;
            const float vv = v[t * vs.t + (int64_t)z * vs.z + (int64_t)y * vs.y + x];
            const float o = __fadd_rn(__fmul_rn(vv, ma), mb);  // v *= ma; v += mb
            out[dbase + ot * g.out_strides[0]] = from_f32<TOut>(o);
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
// TYF: output tile height (kTY; 64 x 32 tiles measured 55.9 against 54.0 ms on the T share)
template <int R, bool RING, int TYF>
__global__ __launch_bounds__(RING ? kTX * TYF / 2 : kNT) void box3_final_kernel(
    const float2* __restrict__ TAB,
                                                         const float* __restrict__ v,
                                                         void* __restrict__ out, int dtype_out,
                                                         NdGeom g, int zseg, int tiles_x,
                                                         int tiles_y, Str3 vs) {
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
    auto load = [&](int z, int k) -> float2 {
        return (pidx[k] >= 0 && z >= 0 && z < nz) ? vol[(int64_t)z * plane + pidx[k]]
                                                   : make_float2(0.f, 0.f);
    };
    // x / y windows of the Z slice of output slice z and the final stage
    auto xy_final = [&](int z) {
        box3_barrier();
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
        box3_barrier();
        const int tx = threadIdx.x % kTX, sy = (threadIdx.x / kTX) * KY;
        const int gx = x0 + tx;
        const int czx = ccount(z, nz, R) * ccount(gx, nx, R) * ct;
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
            if (gx < ox1 && gy < oy1) {
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
                if (z < z1) {  // uniform per workgroup
#pragma unroll
                    for (int k = 0; k < NPT; ++k) {
                        acc_add(zs[k], pa[k]);
                        acc_sub(zs[k], ring[j][k]);
                        ring[j][k] = pa[k];
                        if (zoff[k] >= 0) Zf[zoff[k]] = make_float2((float)zs[k].x, (float)zs[k].y);
                    }
#pragma unroll
                    for (int k = 0; k < NPT; ++k) pa[k] = load(z + 1 + R, k);
                    xy_final(z);
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
#pragma unroll
            for (int k = 0; k < NPT; ++k) {
                pa[k] = load(z + 1 + R, k);
                ps[k] = load(z - R, k);
            }
            xy_final(z);
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

// ZT_G4_LEGACY=1: the four-kernel form (K2 / K3 / K4 with the AB and S3 round trips; A/B runs)
static bool g4_legacy() {
    static const bool on = [] {
        const char* e = getenv("ZT_G4_LEGACY");
        return e && e[0] == '1';
    }();
    return on;
}

// ZT_G4_FINAL_RING=0: box3_final_kernel re-reads the leaving slice instead of holding the z-window
// ring in registers (A/B runs)
static bool g4_final_ring() {
    static const bool on = [] {
        const char* e = getenv("ZT_G4_FINAL_RING");
        return !(e && e[0] == '0');
    }();
    return on;
}

int64_t guided4d_scratch_bytes(int64_t numel, bool gather) {
    // U3 / S3 / TAB (8 B) | AB (8 B, four-kernel form only) | v (4 B, when the input is not a
    // contiguous f32 block)
    return numel * ((g4_legacy() ? 16 : 8) + (gather ? 4 : 0)) + 64;
}

hipError_t launch_guided4d(const void* in, int dtype_in, void* out, int dtype_out,
                           const NdGeom& g, int radius, float eps, void* scratch, hipStream_t s) {
    const int T = (int)g.shape[0], nz = (int)g.shape[1], ny = (int)g.shape[2],
              nx = (int)g.shape[3];
    const int64_t n = g.numel;
    if (n <= 0 || g.out_numel <= 0) return hipSuccess;
    char* base = static_cast<char*>(scratch);
    double* U3 = reinterpret_cast<double*>(base);          // later S3 (float2) in place
    float2* AB = reinterpret_cast<float2*>(base + n * 8);
    // f32 with unit-stride x is read in place (strided t / z / y); other element types or
    // strides are first copied to C-order f32 in scratch
    const bool in_place = dtype_in == kF32 && g.in_strides[3] == 1;
    const float* v = static_cast<const float*>(in);
    Str3 vs{g.in_strides[0], g.in_strides[1], g.in_strides[2]};
    hipError_t e;
    if (!in_place) {
        float* vv = reinterpret_cast<float*>(base + n * 16);
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
    e = launch_box3_r<float, double, double>(radius, v, U3, T, nz, ny, nx, vs, s);
    if (e != hipSuccess) return e;
    if (ny > 65535 || g.out_shape[2] > 65535) return hipErrorInvalidValue;  // grid.y
    if (!g4_legacy()) {
        // three-kernel form: K2t (u, a, b and their t-window sums for the output timepoints)
        // then the box3 march of those with the final stage in its output (K3f)
        const int t0 = (int)g.out_start[0], ont = (int)g.out_shape[0];
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
        else if (T <= 32) k2r(std::integral_constant<int, 32>{});
        else return hipErrorInvalidValue;
        if ((e = hipGetLastError()) != hipSuccess) return e;
        const int64_t onx = g.out_shape[3], ony = g.out_shape[2], onz = g.out_shape[1];
        const bool ring = g4_final_ring() && (int64_t)ny * nx < ((int64_t)1 << 31);
        const int tiles_x = (int)((onx + kTX - 1) / kTX), tiles_y = (int)((ony + kTY - 1) / kTY);
        const int64_t tiles = (int64_t)tiles_x * tiles_y;
        int nseg = (int)std::max<int64_t>(
            1, std::min<int64_t>((onz + 15) / 16, (4096 + tiles * ont - 1) / (tiles * ont)));
        const int zseg = (int)((onz + nseg - 1) / nseg);
        nseg = (int)((onz + zseg - 1) / zseg);
        const int64_t gx = tiles * nseg;
        if (gx > 0x7FFFFFFF || ont > 65535) return hipErrorInvalidValue;
        const float2* TAB = reinterpret_cast<const float2*>(U3);
        const dim3 fg((unsigned)gx, (unsigned)ont);
        switch (radius) {
#define ZT_G4_K3F(RR)                                                                             \
    case RR:                                                                                      \
        if (ring)                                                                                 \
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
    // (a, b) are needed only within R timepoints of the output's (a slab's halo timepoints
    // beyond that feed stage 1 alone)
    const int ta_ab = std::max<int>(0, (int)g.out_start[0] - radius);
    const int tb_ab = std::min<int>(T, (int)(g.out_start[0] + g.out_shape[0]) + radius);
    const int64_t pgx = (nx + kPX - 1) / kPX, pgy = (ny + kPY - 1) / kPY;
    const dim3 pgrid((unsigned)pgx, (unsigned)pgy,
                     (unsigned)std::min<int64_t>(nz, std::max<int64_t>(1, 65536 / (pgy * pgx) + 1)));
    const dim3 pblock(kPX, kPY);
    if (T <= 4)
        hipLaunchKernelGGL(g4_pointwise_kernel<4>, pgrid, pblock, 0, s, U3, v, AB, T, ta_ab,
                           tb_ab, nz, ny, nx, radius, eps, vs);
    else if (T <= 16)
        hipLaunchKernelGGL(g4_pointwise_kernel<16>, pgrid, pblock, 0, s, U3, v, AB, T, ta_ab,
                           tb_ab, nz, ny, nx, radius, eps, vs);
    else if (T <= 32) {  // config T's (t, z) block shares: 16 output timepoints + the 2r halo
        switch (radius) {
#define ZT_G4_K2(RR)                                                                              \
    case RR:                                                                                      \
        hipLaunchKernelGGL((g4_pointwise_slide_kernel<32, RR>), pgrid, pblock, 0, s, U3, v, AB, T, \
                           ta_ab, tb_ab, nz, ny, nx, eps, vs);                                    \
        break;
        ZT_G4_K2(1) ZT_G4_K2(2) ZT_G4_K2(3) ZT_G4_K2(4) ZT_G4_K2(5) ZT_G4_K2(6)
#undef ZT_G4_K2
        default: return hipErrorInvalidValue;
        }
    } else
        return hipErrorInvalidValue;
    if ((e = hipGetLastError()) != hipSuccess) return e;
    float2* S3 = reinterpret_cast<float2*>(U3);
    {  // K3 on the timepoints whose (a, b) sums K4 reads
        const int64_t vol = (int64_t)nz * ny * nx;
        e = launch_box3_r<float2, dd2, float2>(radius, AB + ta_ab * vol, S3 + ta_ab * vol,
                                               tb_ab - ta_ab, nz, ny, nx,
                                               Str3{vol, (int64_t)ny * nx, (int64_t)nx}, s);
    }
    if (e != hipSuccess) return e;
    const int64_t onx = g.out_shape[3], ony = g.out_shape[2], onz = g.out_shape[1];
    const int64_t fgx = (onx + kPX - 1) / kPX, fgy = (ony + kPY - 1) / kPY;
    const dim3 fgrid((unsigned)fgx, (unsigned)fgy,
                     (unsigned)std::min<int64_t>(onz, std::max<int64_t>(1, 65536 / (fgy * fgx) + 1)));
    e = hipErrorInvalidValue;
    if (T <= 4) {
        ZT_DISPATCH_DTYPE(dtype_out, TO,
            hipLaunchKernelGGL((g4_final_kernel<4, TO>), fgrid, dim3(kPX, kPY), 0, s, S3, v,
                               static_cast<TO*>(out), g, radius, vs);
            e = hipGetLastError())
    } else if (T <= 16) {
        ZT_DISPATCH_DTYPE(dtype_out, TO,
            hipLaunchKernelGGL((g4_final_kernel<16, TO>), fgrid, dim3(kPX, kPY), 0, s, S3, v,
                               static_cast<TO*>(out), g, radius, vs);
            e = hipGetLastError())
    } else {
        auto launch = [&](auto rr) {
            constexpr int RR = decltype(rr)::value;
            ZT_DISPATCH_DTYPE(dtype_out, TO,
                hipLaunchKernelGGL((g4_final_slide_kernel<32, RR, TO>), fgrid, dim3(kPX, kPY), 0,
                                   s, S3, v, static_cast<TO*>(out), g, vs);
                e = hipGetLastError())
        };
        switch (radius) {
        case 1: launch(std::integral_constant<int, 1>{}); break;
        case 2: launch(std::integral_constant<int, 2>{}); break;
        case 3: launch(std::integral_constant<int, 3>{}); break;
        case 4: launch(std::integral_constant<int, 4>{}); break;
        case 5: launch(std::integral_constant<int, 5>{}); break;
        case 6: launch(std::integral_constant<int, 6>{}); break;
        default: return hipErrorInvalidValue;
        }
    }
    return e;
}

}  // namespace zt
