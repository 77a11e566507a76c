// g4_fused.hip — the 4-D guided filter in one z-march for blocks of at most 4 timepoints (config
// T's per-GPU share): guided_filter.rs:117-164 with get_block clamping on all four axes
// (:166-184), both stages and every timepoint of an xy tile in one workgroup, so v is read from
// HBM about once and the output written once (against ~64 B per voxel for the four-kernel path
// of guided4d.hip).
//
// A workgroup owns a 64 x 8 xy output tile for all T <= 4 timepoints and marches
// z through a segment of output slices; stage 1 runs R slices ahead of stage 2. Per step, with
// zc the stage-1 slice and zo = zc - R the output slice:
//   S1  running z-window (f64, exact) of v on the (64+4R) x (8+4R) apron of every timepoint:
//       + entering slice zc+R, - leaving slice zc-R-1                         -> Z1 (LDS, f64)
//   S2  x-window sums of Z1 rows on the (64+2R) columns                          -> X1 (LDS, f64)
//   S3  y-window sums -> U3(t) on the (64+2R) x (8+2R) apron; t-window sums -> U4 (exact);
//       u = RN(RN_f32(U4) / c4), s = (v-u)^2, a = s/(s+eps), b = (1-a)u (count divisions
//       correctly rounded through an LDS table of RN(1/c); a within 1 ulp);
//       zero outside the block (the clamped sums of stage 2)                   -> Lab (LDS, f32 x2)
//   S4  x-window sums of (a, b) rows on the 64 tile columns                    -> Hab (LDS, f32 x2)
//   S5  y-window sums + t-window sums of (a, b) -> P(zc), kept in an LDS history of the last
//       2R+1 slices whose sum is the z-window;
//       out(zo) = RN(RN(v * RN(S4a / c4)) + RN(S4b / c4)).
// A workgroup has 1024 threads (4 waves per SIMD) and ~154 KB of LDS. Four LDS barriers per
// step; Z1/Lab and X1/Hab share LDS (their lifetimes alternate). Stage 1 is exact like the 3-D
// kernel's; stage 2's xy and t sums are f32 (the tolerance of DESIGN.md §4).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <type_traits>

#include "zt_device.hpp"
#include "zt_kernels.hpp"

namespace zt {

namespace {

constexpr int kFTX = 64, kFTY = 8, kFTS = 4;  // tile width, height, timepoints per block
#ifndef G4_Q4
#define G4_Q4 1  // quad loads in S1 where the geometry allows (see g4_fused_kernel)
#endif
#ifndef G4_KX2
#define G4_KX2 5  // S2 outputs per item: 4 x 16 x ceil(68 / 5) = 896 items, one pass of 1024
                  // threads (4 per item: 1088, a second pass for one wave)
#endif
#ifndef G4_STX
#define G4_STX 4  // XCD super-tile of the tile walk: tiles along x
#endif
#ifndef G4_STY
#define G4_STY 16  // ... along y (4 x 16: 35.98 ms vs 36.24 for whole rows)
#endif

template <int R>
struct G4FConfig {
    static constexpr int TX = kFTX, TY = kFTY, TS = kFTS, W = 2 * R + 1;
    static constexpr int E2X = TX + 4 * R, E2Y = TY + 4 * R;  // stage-1 apron
    static constexpr int E1X = TX + 2 * R, E1Y = TY + 2 * R;  // (a, b) apron
    static constexpr int NT = 1024;  // one workgroup per CU, 4 waves per SIMD
    static constexpr int NE2 = E2X * E2Y, NPT = (NE2 + NT - 1) / NT;  // S1 points per thread per t
    static constexpr int PZ = ((E2X + 4 + 1) / 2) * 2;  // Z1 pitch (x-sum segments read past E2X)
    static constexpr int KX2 = G4_KX2, NSX2 = (E1X + KX2 - 1) / KX2, NI2 = TS * E2Y * NSX2;
    static constexpr int KY3 = 2, NSY3 = (E1Y + KY3 - 1) / KY3, NI3 = E1X * NSY3;
    static constexpr int KX4 = 8, NI4 = TS * E1Y * (TX / KX4);
    static constexpr int NI5 = TX * TY;
    static constexpr int SZ_A = std::max<int>(TS * E2Y * PZ * 8, TS * E1Y * E1X * 8);
    static constexpr int SZ_B = std::max<int>(TS * E2Y * E1X * 8, TS * E1Y * TX * 8);
    static_assert(E1Y % KY3 == 0, "S3 segments tile the apron rows (X1 reads stay in E2Y)");
    static constexpr int SZ_RING = W * TS * TY * TX * 8;  // stage-2 slice history (float2)
    static constexpr int W4 = W * W * W * W;              // largest window count
    static constexpr int SZ_RCP = ((W4 + 1) * 4 + 15) / 16 * 16;
    static constexpr int LDS = SZ_A + SZ_B + SZ_RING + SZ_RCP;
    static_assert(NI3 <= NT && NI4 <= NT && NI5 <= NT, "one item per thread in S3-S5");
    static_assert(TX % KX4 == 0, "S4 segments");
    static_assert(LDS <= 160 * 1024, "LDS budget");
};

struct G4FParams {
    const float* v;  // (T, nz, ny, nx) f32, C order (the halo'd block)
    void* out;       // output region, strides os
    int T, nz, ny, nx;
    int o0[4], on[4];
    int64_t os[4];
    int zseg, tiles_x, tiles_y;
    float eps;
};

__device__ __forceinline__ int fcount(int i, int n, int r) {
    const int lo = i - r < 0 ? 0 : i - r;
    const int hi = i + r > n - 1 ? n - 1 : i + r;
    return hi - lo + 1;
}

// Buffer (SRD) loads: 32-bit byte offsets and the hardware range check (an offset past
// num_records reads 0), so out-of-block points need no branch and no 64-bit address math.
using rsrc_t = __amdgpu_buffer_rsrc_t;
constexpr int kBad = (int)0x80000000;  // >= num_records of any slice: reads 0
__device__ __forceinline__ rsrc_t make_rsrc(const void* base, uint32_t bytes) {
    // built from kernel arguments and loop counters only (wave-uniform): stays in SGPRs
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, (int)bytes,
                                             0x00020000);
}
__device__ __forceinline__ float ldb(rsrc_t r, int off) {
    return __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(r, off, 0, 0));
}

// Packed pair of f32 (v_pk_add_f32 / v_pk_mul_f32 / v_pk_fma_f32: both lanes in one issue).
typedef float f2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ f2 pk_fma(f2 a, f2 b, f2 c) { return __builtin_elementwise_fma(a, b, c); }

// x / d for an integer count d given rcp = RN(1/d): Markstein's correction makes the quotient
// correctly rounded (= IEEE division) in 3 VALU ops (as gf_fused.hpp's div_by_count).
__device__ __forceinline__ float div_by_count(float x, float d, float rcp) {
    const float q = x * rcp;
    const float r = __builtin_fmaf(-q, d, x);
    return __builtin_fmaf(r, rcp, q);
}
// s / (s + eps): rcp, one Newton step and Markstein's correction (within 1 ulp, almost always
// correctly rounded; 0/0 gives NaN as in the reference), as gf_fused.hpp's fast_div.
__device__ __forceinline__ float fast_div(float x, float d) {
    float y = __builtin_amdgcn_rcpf(d);
    const float e = __builtin_fmaf(-d, y, 1.0f);
    y = __builtin_fmaf(e, y, y);
    const float q = x * y;
    const float r = __builtin_fmaf(-d, q, x);
    return __builtin_fmaf(r, y, q);
}

// Workgroup barrier for the LDS hand-offs only: __syncthreads() also fences global memory, which
// would drain the loads kept in flight across it (the next slices' prefetches).
__device__ __forceinline__ void lds_barrier() {
    __asm__ volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
}

template <int B, int E, typename F>
__device__ __forceinline__ void sfor(F&& f) {
    if constexpr (B < E) {
        f(std::integral_constant<int, B>{});
        sfor<B + 1, E>(f);
    }
}

// Q4: S1 reads 16-byte quads (4 consecutive x) instead of single elements: 4x fewer
// vector-memory instructions for the stage-1 slices. Needs quads that never straddle the block
// edge (x origin of the apron and the block width multiples of 4: r = 2 with aligned geometry);
// waves [4t, 4t + 4) then hold timepoint t's quads, so each load's slice descriptor stays
// wave-uniform.
template <int R, typename TOut, bool Q4>
__global__ __launch_bounds__(G4FConfig<R>::NT) void g4_fused_kernel(G4FParams p) {
    using C = G4FConfig<R>;
    constexpr int TX = C::TX, TY = C::TY, TS = C::TS, W = C::W, NT = C::NT, NPT = C::NPT;
    constexpr int E2X = C::E2X, E2Y = C::E2Y, E1X = C::E1X, E1Y = C::E1Y, PZ = C::PZ;
    extern __shared__ __attribute__((aligned(16))) char smem[];
    double* Z1 = reinterpret_cast<double*>(smem);                  // [TS][E2Y][PZ]
    float2* Lab = reinterpret_cast<float2*>(smem);                 // [TS][E1Y][E1X]
    double* X1 = reinterpret_cast<double*>(smem + C::SZ_A);        // [TS][E2Y][E1X]
    float2* Hab = reinterpret_cast<float2*>(smem + C::SZ_A);       // [TS][E1Y][TX]
    float2* Ring = reinterpret_cast<float2*>(smem + C::SZ_A + C::SZ_B);  // [W][TS][TY * TX]
    float* rcp_tab = reinterpret_cast<float*>(smem + C::SZ_A + C::SZ_B + C::SZ_RING);
    // RN(1/c) of every window count c (Markstein's correction below needs it exactly); published
    // by the first step's barriers
    for (int c = threadIdx.x; c <= C::W4; c += NT) rcp_tab[c] = c > 0 ? 1.0f / (float)c : 0.0f;
    const int tid = threadIdx.x;
    // wave index as a scalar: phases with fewer items than threads branch around whole idle
    // waves (an exec-masked pass over the code would still cost their issue slots)
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int T = p.T, nz = p.nz, ny = p.ny, nx = p.nx;
    const int64_t plane = (int64_t)ny * nx, vol = (int64_t)nz * plane;

    // XCD-aware block -> (tile, z segment): consecutive logical ids (x-adjacent tiles of one
    // segment) share an XCD, whose L2 then holds the shared apron columns.
    const int nwg = gridDim.x, b = blockIdx.x;
    const int lid = (nwg % 8 == 0) ? (b % 8) * (nwg / 8) + b / 8 : b;
    const int ntiles = p.tiles_x * p.tiles_y;
    const int tile = lid % ntiles, seg = lid / ntiles;
    // tiles walked in G4_STX x G4_STY super-tiles (as gf3d_fused_kernel), so the co-resident
    // workgroups of an XCD cover a compact region whose aprons its L2 shares
    int tx_, ty_;
    {
        const int gtx = p.tiles_x, gty = p.tiles_y, stx = G4_STX, sty = G4_STY;
        const int full_y = gty / sty * sty, per_srow = gtx * sty;
        int t = tile;
        if (t < full_y * gtx) {
            const int sr = t / per_srow, r = t % per_srow, full_x = gtx / stx * stx;
            if (r < full_x * sty) {
                tx_ = (r / (stx * sty)) * stx + r % stx;
                ty_ = sr * sty + (r / stx) % sty;
            } else {
                const int rr = r - full_x * sty, w = gtx - full_x;
                tx_ = full_x + rr % w;
                ty_ = sr * sty + rr / w;
            }
        } else {
            t -= full_y * gtx;
            tx_ = t % gtx;
            ty_ = full_y + t / gtx;
        }
    }
    const int x0 = p.o0[3] + tx_ * TX, y0 = p.o0[2] + ty_ * TY;
    const int xe = p.o0[3] + p.on[3], ye = p.o0[2] + p.on[2];
    const int zo_begin = p.o0[1] + seg * p.zseg;
    const int zo_end = min(zo_begin + p.zseg, p.o0[1] + p.on[1]);
    const int ot0 = p.o0[0], ot1 = p.o0[0] + p.on[0];

    // ---- S1 points: (ey, ex) of the stage-1 apron, the same for every timepoint ----------
    int off[NPT];  // byte offset in the plane, or kBad outside the block / past the apron
#pragma unroll
    for (int k = 0; k < NPT; ++k) {
        const int e = tid + k * NT;
        const int ey = e / E2X, ex = e - (e / E2X) * E2X;
        const int gy = y0 - 2 * R + ey, gx = x0 - 2 * R + ex;
        off[k] = (e < C::NE2 && gy >= 0 && gy < ny && gx >= 0 && gx < nx) ? (gy * nx + gx) * 4 : kBad;
    }
    const uint32_t plane_bytes = (uint32_t)(plane * 4);
    const char* vbytes = reinterpret_cast<const char*>(p.v);
    const int64_t vol_bytes = vol * 4, plane_bytes64 = plane * 4;
    // descriptor of slice z of timepoint t (0 records outside the block: loads read 0); built
    // once per slice and step, shared by the thread's points
    auto slice = [&](int t, int z) -> rsrc_t {
        const bool in = t < T && (unsigned)z < (unsigned)nz;  // wave-uniform
        return make_rsrc(vbytes + (in ? t * vol_bytes + z * plane_bytes64 : 0), in ? plane_bytes : 0u);
    };
    auto ldv = [&](int t, int z, int o) -> float { return ldb(slice(t, z), o); };
    const int zc_begin = zo_begin - R, zc_end = zo_end + R;  // stage-1 slices of this march
    // element form: every thread NPT apron points of every timepoint
    constexpr int TSE = Q4 ? 1 : TS, NPE = Q4 ? 1 : NPT;
    double zv[TSE][NPE];
    float pa[TSE][NPE], ps[TSE][NPE];
    // quad form: timepoint tq (wave-uniform), NPQ quads of its apron per thread
    constexpr int NQR = E2X / 4, NQT = E2Y * NQR, LPT = NT / TS;
    constexpr int NPQ = Q4 ? (NQT + LPT - 1) / LPT : 1;
    static_assert(!Q4 || (E2X % 4 == 0 && NT % (64 * TS) == 0), "quad S1 geometry");
    const int tq = wave / (NT / 64 / TS), lq = tid - tq * LPT;
    int offq[NPQ], z1q[NPQ];
    double zq[NPQ][4];
    float paq[NPQ][4], psq[NPQ][4];
    auto ldq = [&](rsrc_t r, int o, float (&v)[4]) {
        typedef unsigned int u4 __attribute__((ext_vector_type(4)));
        const u4 q = __builtin_amdgcn_raw_buffer_load_b128(r, o, 0, 0);
        v[0] = __uint_as_float(q.x); v[1] = __uint_as_float(q.y);
        v[2] = __uint_as_float(q.z); v[3] = __uint_as_float(q.w);
    };
    if constexpr (Q4) {
#pragma unroll
        for (int k = 0; k < NPQ; ++k) {
            const int qi = lq + LPT * k, ey = qi / NQR, cq = qi - (qi / NQR) * NQR;
            const int gy = y0 - 2 * R + ey, gx = x0 - 2 * R + 4 * cq;
            offq[k] = (qi < NQT && gy >= 0 && gy < ny && gx >= 0 && gx < nx) ? (gy * nx + gx) * 4 : kBad;
            z1q[k] = qi < NQT ? (tq * E2Y + ey) * PZ + 4 * cq : -1;
#pragma unroll
            for (int e = 0; e < 4; ++e) zq[k][e] = 0.0;
            for (int z = zc_begin - 1 - R; z <= zc_begin - 1 + R; ++z) {
                float v[4];
                ldq(slice(tq, z), offq[k], v);
#pragma unroll
                for (int e = 0; e < 4; ++e) zq[k][e] += (double)v[e];
            }
            ldq(slice(tq, zc_begin + R), offq[k], paq[k]);
            ldq(slice(tq, zc_begin - R - 1), offq[k], psq[k]);
        }
    } else {
#pragma unroll
        for (int t = 0; t < TS; ++t)
#pragma unroll
            for (int k = 0; k < NPT; ++k) {
                double s = 0.0;
                for (int z = zc_begin - 1 - R; z <= zc_begin - 1 + R; ++z) s += (double)ldv(t, z, off[k]);
                zv[t][k] = s;
                pa[t][k] = ldv(t, zc_begin + R, off[k]);
                ps[t][k] = ldv(t, zc_begin - R - 1, off[k]);
            }
    }

    // ---- S3 item: column ex1 of the (a, b) apron, rows [KY3*sg, KY3*sg + KY3) --------------
    const int i3 = tid < C::NI3 ? tid : -1;
    const int ex3 = i3 % E1X, sg3 = i3 / E1X;
    const int gx3 = x0 - R + ex3;
    int off3[C::KY3];
#pragma unroll
    for (int j = 0; j < C::KY3; ++j) {
        const int ey = sg3 * C::KY3 + j, gy = y0 - R + ey;
        off3[j] = (i3 >= 0 && ey < E1Y && gy >= 0 && gy < ny && gx3 >= 0 && gx3 < nx) ? (gy * nx + gx3) * 4 : kBad;
    }
    float v3[TS][C::KY3];  // v at the S3 points of the current stage-1 slice (prefetched)
    // ---- S5 item: output (y, x) of the tile ----------------------------------------------
    const int x5 = tid % TX, y5 = tid / TX;  // tid < TX * TY
    const int gx5 = x0 + x5, gy5 = y0 + y5;
    const bool live5 = tid < C::NI5 && gx5 < xe && gy5 < ye;
    const int off5 = live5 ? (gy5 * nx + gx5) * 4 : kBad;
    const int cyx5 = live5 ? fcount(gy5, ny, R) * fcount(gx5, nx, R) : 0;
    float v5[TS];
    // stage-2 z-window: the sum of the last W slice sums P, kept in LDS (each thread only touches
    // its own slots, so no barrier), summed in a fixed slot order without subtraction
    if (tid < C::NI5)
        for (int sl = 0; sl < W * TS; ++sl) Ring[sl * (TY * TX) + tid] = make_float2(0.0f, 0.0f);
    auto load_v3 = [&](int zc) {
#pragma unroll
        for (int t = 0; t < TS; ++t) {
            const rsrc_t rs = slice(t, zc);
#pragma unroll
            for (int j = 0; j < C::KY3; ++j) v3[t][j] = ldb(rs, off3[j]);
        }
    };
    auto load_v5 = [&](int zo) {
#pragma unroll
        for (int t = 0; t < TS; ++t) v5[t] = ldv(t, zo, off5);
    };
    load_v5(zc_begin - R);
    load_v3(zc_begin);  // S3's v of the first stage-1 slice; later slices a step ahead

    // count factors of the t-windows (clamped to the block's T)
    int ta_[TS], tb_[TS];
#pragma unroll
    for (int t = 0; t < TS; ++t) {
        ta_[t] = max(t - R, 0);
        tb_[t] = min(t + R, T - 1);
    }

    const int nsteps = zc_end - zc_begin;
    for (int i = 0, slot = 0; i < nsteps; ++i, slot = slot + 1 == W ? 0 : slot + 1) {
        {
            const int zc = zc_begin + i, zo = zc - R;
            // S1: z-window update, Z1 writes, next step's entering / leaving slices
            if constexpr (Q4) {
#pragma unroll
                for (int k = 0; k < NPQ; ++k) {
#pragma unroll
                    for (int e = 0; e < 4; ++e) {
                        zq[k][e] = zq[k][e] + (double)paq[k][e];
                        zq[k][e] = zq[k][e] - (double)psq[k][e];
                    }
                    if (z1q[k] >= 0) {
                        double2* d = reinterpret_cast<double2*>(Z1 + z1q[k]);
                        d[0] = make_double2(zq[k][0], zq[k][1]);
                        d[1] = make_double2(zq[k][2], zq[k][3]);
                    }
                }
                const rsrc_t ra = slice(tq, zc + 1 + R), rl = slice(tq, zc - R);
#pragma unroll
                for (int k = 0; k < NPQ; ++k) {
                    ldq(ra, offq[k], paq[k]);
                    ldq(rl, offq[k], psq[k]);
                }
            } else {
#pragma unroll
            for (int t = 0; t < TS; ++t)
#pragma unroll
                for (int k = 0; k < NPT; ++k) {
                    zv[t][k] = zv[t][k] + (double)pa[t][k];
                    zv[t][k] = zv[t][k] - (double)ps[t][k];
                    const int e = tid + k * NT;
                    if (e < C::NE2) Z1[(t * E2Y + e / E2X) * PZ + e % E2X] = zv[t][k];
                }
#pragma unroll
            for (int t = 0; t < TS; ++t) {
                const rsrc_t ra = slice(t, zc + 1 + R), rl = slice(t, zc - R);
#pragma unroll
                for (int k = 0; k < NPT; ++k) {
                    pa[t][k] = ldb(ra, off[k]);
                    ps[t][k] = ldb(rl, off[k]);
                }
            }
            }
            lds_barrier();
            // S2: x-window sums of every apron row (f64)
            for (int it = tid; it < C::NI2; it += NT) {
                const int sx = (it % C::NSX2) * C::KX2, row = it / C::NSX2;  // row = t*E2Y + ey
                const double* src = Z1 + row * PZ + sx;
                double in[C::KX2 + 2 * R];
#pragma unroll
                for (int j = 0; j < C::KX2 + 2 * R; ++j) in[j] = src[j];
                double s = 0.0;
#pragma unroll
                for (int j = 0; j <= 2 * R; ++j) s += in[j];
                double* dst = X1 + row * E1X + sx;
#pragma unroll
                for (int j = 0; j < C::KX2; ++j) {
                    if (j > 0) s = s + in[j + 2 * R] - in[j - 1];
                    if (sx + j < E1X) dst[j] = s;
                }
            }
            lds_barrier();
            // S3: y-window sums, t-window sums, pointwise stage -> Lab
            if (wave < (C::NI3 + 63) / 64 && i3 >= 0) {
                // v3 = v of slice zc, loaded a step ago (outside any branch, so the wait here is
                // for that load only, not a drain of this step's prefetches)
                double U3[TS][C::KY3];
#pragma unroll
                for (int t = 0; t < TS; ++t) {
                    const double* src = X1 + (t * E2Y + sg3 * C::KY3) * E1X + ex3;
                    double in[C::KY3 + 2 * R];
#pragma unroll
                    for (int j = 0; j < C::KY3 + 2 * R; ++j) in[j] = src[j * E1X];
                    double s = 0.0;
#pragma unroll
                    for (int j = 0; j <= 2 * R; ++j) s += in[j];
                    U3[t][0] = s;
#pragma unroll
                    for (int j = 1; j < C::KY3; ++j) {
                        s = s + in[j + 2 * R] - in[j - 1];
                        U3[t][j] = s;
                    }
                }
                const bool zin = (unsigned)zc < (unsigned)nz;
                const int czx = zin && gx3 >= 0 && gx3 < nx ? fcount(zc, nz, R) * fcount(gx3, nx, R) : 0;
                static_assert(C::KY3 == 2, "the pointwise stage works on the item's row pair");
                const int ey0 = sg3 * 2, gyp = y0 - R + ey0;
                const int cz0 = gyp >= 0 && gyp < ny ? czx * fcount(gyp, ny, R) : 0;
                const int cz1 = gyp + 1 >= 0 && gyp + 1 < ny ? czx * fcount(gyp + 1, ny, R) : 0;
#pragma unroll
                for (int t = 0; t < TS; ++t) {
                    double U0 = 0.0, U1 = 0.0;
#pragma unroll
                    for (int tt = 0; tt < TS; ++tt)
                        if (tt >= ta_[t] && tt <= tb_[t]) {
                            U0 += U3[tt][0];
                            U1 += U3[tt][1];
                        }
                    // the pair of rows in packed f32 (one issue per op for both):
                    // u = RN(RN_f32(U4) / c) (Markstein with RN(1/c): correctly rounded),
                    // s = (v-u)^2, a = s/(s+eps), b = (1-a)u   (guided_filter.rs:126-137)
                    const int nt = tb_[t] - ta_[t] + 1, c0 = cz0 * nt, c1 = cz1 * nt;
                    const f2 Uf = {(float)U0, (float)U1};
                    const f2 fc = {(float)c0, (float)c1}, rc = {rcp_tab[c0], rcp_tab[c1]};
                    f2 q = Uf * rc;
                    f2 r = pk_fma(-q, fc, Uf);
                    const f2 u = pk_fma(r, rc, q);
                    const f2 d = (f2){v3[t][0], v3[t][1]} - u;
                    const f2 sq = d * d;  // (v - u).powf(2.0)
                    const f2 den = sq + (f2){p.eps, p.eps};
                    f2 y = {__builtin_amdgcn_rcpf(den.x), __builtin_amdgcn_rcpf(den.y)};
                    const f2 e = pk_fma(-den, y, (f2){1.0f, 1.0f});
                    y = pk_fma(e, y, y);
                    q = sq * y;
                    r = pk_fma(-den, q, sq);
                    const f2 a = pk_fma(r, y, q);
                    const f2 b = ((f2){1.0f, 1.0f} - a) * u;
                    const bool ok0 = c0 > 0 && t < T, ok1 = c1 > 0 && t < T;
                    float2* dst = Lab + (t * E1Y + ey0) * E1X + ex3;
                    dst[0] = ok0 ? make_float2(a.x, b.x) : make_float2(0.0f, 0.0f);
                    dst[E1X] = ok1 ? make_float2(a.y, b.y) : make_float2(0.0f, 0.0f);
                }
            }
            lds_barrier();
            // S4: x-window sums of (a, b) rows on the tile columns
            if (wave < (C::NI4 + 63) / 64 && tid < C::NI4) {
                const int sx = (tid % (TX / C::KX4)) * C::KX4, row = tid / (TX / C::KX4);
                const int t = row / E1Y, ey = row - t * E1Y;
                const f2* src = reinterpret_cast<const f2*>(Lab + (t * E1Y + ey) * E1X + sx);
                f2 in[C::KX4 + 2 * R];
#pragma unroll
                for (int j = 0; j < C::KX4 + 2 * R; ++j) in[j] = src[j];
                f2 sab = in[0];
#pragma unroll
                for (int j = 1; j <= 2 * R; ++j) sab = sab + in[j];
                f2* dst = reinterpret_cast<f2*>(Hab + row * TX + sx);
                dst[0] = sab;
#pragma unroll
                for (int j = 1; j < C::KX4; ++j) {
                    sab = sab + in[j + 2 * R] - in[j - 1];
                    dst[j] = sab;
                }
            }
            lds_barrier();
            // S5: y-window and t-window sums -> ring; emit out(zo) once the ring is full
            if (wave < (C::NI5 + 63) / 64 && tid < C::NI5) {
                f2 P3[TS];
#pragma unroll
                for (int t = 0; t < TS; ++t) {
                    const f2* src = reinterpret_cast<const f2*>(Hab + (t * E1Y + y5) * TX + x5);
                    f2 sab = src[0];
#pragma unroll
                    for (int j = 1; j <= 2 * R; ++j) sab = sab + src[j * TX];
                    P3[t] = sab;
                }
                f2* ring = reinterpret_cast<f2*>(Ring);
#pragma unroll
                for (int t = 0; t < TS; ++t) {
                    f2 sab = {0.0f, 0.0f};
#pragma unroll
                    for (int tt = 0; tt < TS; ++tt)
                        if (tt >= ta_[t] && tt <= tb_[t]) sab = sab + P3[tt];
                    ring[(slot * TS + t) * (TY * TX) + tid] = sab;
                }
                if (i >= 2 * R && live5) {
                    const int cz5 = fcount(zo, nz, R) * cyx5;
#pragma unroll
                    for (int t = 0; t < TS; ++t) {
                        if (t < ot0 || t >= ot1) continue;
                        f2 sab = ring[t * (TY * TX) + tid];
#pragma unroll
                        for (int sl = 1; sl < W; ++sl) sab = sab + ring[(sl * TS + t) * (TY * TX) + tid];
                        const int c = cz5 * (tb_[t] - ta_[t] + 1);
                        const f2 rc = {rcp_tab[c], rcp_tab[c]}, fc = {(float)c, (float)c};
                        // (mean_a, mean_b) = RN(S / c), Markstein (correctly rounded)
                        const f2 q = sab * rc;
                        const f2 m = pk_fma(pk_fma(-q, fc, sab), rc, q);
                        const float o = __fadd_rn(__fmul_rn(v5[t], m.x), m.y);  // v *= ma; v += mb
                        static_cast<TOut*>(p.out)[(t - ot0) * p.os[0] +
                                                  (int64_t)(zo - p.o0[1]) * p.os[1] +
                                                  (int64_t)(gy5 - p.o0[2]) * p.os[2] +
                                                  (int64_t)(gx5 - p.o0[3]) * p.os[3]] =
                            from_f32<TOut>(o);
                    }
                }
            }
            load_v5(zo + 1);
            load_v3(zc + 1);  // L2 hits: the slice entered stage 1 R steps ago
            // the next step's Z1 / Lab writes follow this step's S4 reads (third barrier); its X1
            // writes follow its first barrier, after every S5 read of Hab
        }
    }
}

template <int R, typename TOut>
hipError_t launch_fused4(G4FParams p, hipStream_t s) {
    using C = G4FConfig<R>;
    p.tiles_x = (p.on[3] + C::TX - 1) / C::TX;
    p.tiles_y = (p.on[2] + C::TY - 1) / C::TY;
    const int64_t tiles = (int64_t)p.tiles_x * p.tiles_y;
    // z segments: enough workgroups for about four per CU, at least 32 output slices each
    // (a segment recomputes 2R stage-1 slices)
    int64_t nseg = std::max<int64_t>(1, std::min<int64_t>((p.on[1] + 31) / 32, (1024 + tiles - 1) / tiles));
    p.zseg = (int)((p.on[1] + nseg - 1) / nseg);
    nseg = (p.on[1] + p.zseg - 1) / p.zseg;
    const int64_t gx = tiles * nseg;
    if (gx > 0x7FFFFFFF) return hipErrorInvalidValue;
    // quad S1 (Q4) when no quad of the stage-1 apron straddles the block's x edges
    const bool q4 = R == 2 && G4_Q4 && p.nx % 4 == 0 && p.o0[3] % 4 == 0 &&
                    (uintptr_t)p.v % 16 == 0;
    auto kern = q4 ? g4_fused_kernel<R, TOut, true> : g4_fused_kernel<R, TOut, false>;
    // > 64 KB of dynamic LDS needs the opt-in, once per device (a bit per device)
    // (one mask per kernel variant)
    static std::atomic<uint64_t> attr_q[2] = {{0}, {0}};
    std::atomic<uint64_t>& attr = attr_q[q4 ? 1 : 0];
    int dev = 0;
    if (hipError_t e = hipGetDevice(&dev)) return e;
    if (!(attr.load(std::memory_order_relaxed) & (1ull << (dev & 63)))) {
        hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(kern),
                                           hipFuncAttributeMaxDynamicSharedMemorySize, C::LDS);
        if (e != hipSuccess) return e;
        attr.fetch_or(1ull << (dev & 63), std::memory_order_relaxed);
    }
    hipLaunchKernelGGL(kern, dim3((unsigned)gx), dim3(C::NT), C::LDS, s, p);
    return hipGetLastError();
}

}  // namespace

bool guided4d_fused_supports(int radius, const NdGeom& g) {
    // slices addressed by 32-bit byte offsets
    return (radius == 1 || radius == 2) && g.ndim == 4 && g.shape[0] <= kFTS &&
           g.shape[1] <= 0x7FFFFFFF && g.shape[2] * g.shape[3] * 4 <= 0x7FFFFFFF;
}

hipError_t launch_guided4d_fused(const float* v, void* out, int dtype_out, const NdGeom& g,
                                 int radius, float eps, hipStream_t s) {
    if (g.numel <= 0 || g.out_numel <= 0) return hipSuccess;
    if (!guided4d_fused_supports(radius, g)) return hipErrorInvalidValue;
    G4FParams p{};
    p.v = v;
    p.out = out;
    p.T = (int)g.shape[0];
    p.nz = (int)g.shape[1];
    p.ny = (int)g.shape[2];
    p.nx = (int)g.shape[3];
    p.eps = eps;
    for (int d = 0; d < 4; ++d) {
        p.o0[d] = (int)g.out_start[d];
        p.on[d] = (int)g.out_shape[d];
        p.os[d] = g.out_strides[d];
    }
    hipError_t e = hipErrorInvalidValue;
    if (radius == 1) {
        ZT_DISPATCH_DTYPE(dtype_out, TO, e = (launch_fused4<1, TO>(p, s)))
    } else {
        ZT_DISPATCH_DTYPE(dtype_out, TO, e = (launch_fused4<2, TO>(p, s)))
    }
    return e;
}

}  // namespace zt
