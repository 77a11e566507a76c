// gf_fused.hpp — the fused 2.5-D guided-filter kernel template (see guided_filter.hip for the
// design notes). Instantiated per radius in gf_fused_r<R>.hip so the instantiations compile in
// parallel; guided_filter.hip dispatches.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include <type_traits>

#include "zt_device.hpp"
#include "zt_kernels.hpp"

namespace zt {

// ---------------------------------------------------------------------------------------------
// Window sums of 2R+1 consecutive values by a fixed binary tree.
// out[i] = sum(in[i .. i+2R]) for i < K. in has K + 2R entries (registers).
// ---------------------------------------------------------------------------------------------
template <int R, int K>
__device__ __forceinline__ void tree_window_sums(const float (&in)[K + 2 * R], float (&out)[K]) {
    constexpr int W = 2 * R + 1;
    if constexpr (W == 1) {
#pragma unroll
        for (int i = 0; i < K; ++i) out[i] = in[i];
    } else {
        // levels: L[0] = in (width 1), L[1] = pairs (width 2), L[2] = quads, ...
        constexpr int N = K + 2 * R;
        float p2[N], p4[N], p8[N], p16[N], p32[N], p64[N], p128[N];
#pragma unroll
        for (int i = 0; i + 1 < N; ++i) p2[i] = in[i] + in[i + 1];
        if constexpr (W >= 4) {
#pragma unroll
            for (int i = 0; i + 3 < N; ++i) p4[i] = p2[i] + p2[i + 2];
        }
        if constexpr (W >= 8) {
#pragma unroll
            for (int i = 0; i + 7 < N; ++i) p8[i] = p4[i] + p4[i + 4];
        }
        if constexpr (W >= 16) {
#pragma unroll
            for (int i = 0; i + 15 < N; ++i) p16[i] = p8[i] + p8[i + 8];
        }
        if constexpr (W >= 32) {
#pragma unroll
            for (int i = 0; i + 31 < N; ++i) p32[i] = p16[i] + p16[i + 16];
        }
        if constexpr (W >= 64) {
#pragma unroll
            for (int i = 0; i + 63 < N; ++i) p64[i] = p32[i] + p32[i + 32];
        }
        if constexpr (W >= 128) {
#pragma unroll
            for (int i = 0; i + 127 < N; ++i) p128[i] = p64[i] + p64[i + 64];
        }
#pragma unroll
        for (int i = 0; i < K; ++i) {
            // largest power first, then the remaining set bits of W from high to low
            float acc = 0.0f;
            int off = 0;
            bool first = true;
#pragma unroll
            for (int b = 7; b >= 0; --b) {
                if (W & (1 << b)) {
                    float piece;
                    switch (b) {
                    case 0: piece = in[i + off]; break;
                    case 1: piece = p2[i + off]; break;
                    case 2: piece = p4[i + off]; break;
                    case 3: piece = p8[i + off]; break;
                    case 4: piece = p16[i + off]; break;
                    case 5: piece = p32[i + off]; break;
                    case 6: piece = p64[i + off]; break;
                    default: piece = p128[i + off]; break;
                    }
                    acc = first ? piece : acc + piece;
                    first = false;
                    off += 1 << b;
                }
            }
            out[i] = acc;
        }
    }
}

__device__ __forceinline__ int clamped_count(int i, int n, int r) {
    int lo = i - r < 0 ? 0 : i - r;
    int hi = i + r > n - 1 ? n - 1 : i + r;
    return hi - lo + 1;
}

// ---------------------------------------------------------------------------------------------
// Compile-time ring dispatch: call f(integral_constant<SLOT>) for the runtime slot.
// ---------------------------------------------------------------------------------------------
template <int S, int W>
struct RingDispatch {
    template <typename F>
    __device__ __forceinline__ static void run(int slot, F&& f) {
        if (slot == S) f(std::integral_constant<int, S>{});
        else RingDispatch<S + 1, W>::run(slot, f);
    }
};
template <int W>
struct RingDispatch<W, W> {
    template <typename F>
    __device__ __forceinline__ static void run(int, F&&) {}
};

// ---------------------------------------------------------------------------------------------
// Sliding window sums in f64 (stage 1: the box sums of v). Sums of f32 values in f64 are exact
// for any realistic dynamic range, so the order is immaterial and u = (f32)sum / count rounds
// exactly like the reference's f64 summed-area-table sum (summed_area_table.rs:398-410).
// ---------------------------------------------------------------------------------------------
template <int R, int K>
__device__ __forceinline__ void slide_sums_f64(const double (&in)[K + 2 * R], double (&out)[K]) {
    double s = in[0];
#pragma unroll
    for (int j = 1; j <= 2 * R; ++j) s += in[j];
    out[0] = s;
#pragma unroll
    for (int i = 1; i < K; ++i) {
        s = s + in[i + 2 * R];
        s = s - in[i - 1];
        out[i] = s;
    }
}

// Workgroup barrier for LDS hand-offs only. __syncthreads() also fences global memory, which
// makes the compiler drain every outstanding global load (vmcnt(0)) — including the next step's
// prefetches this kernel keeps in flight across the barrier.
__device__ __forceinline__ void lds_barrier() {
    __asm__ volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
}

// ---------------------------------------------------------------------------------------------
// The fused kernel.
// ---------------------------------------------------------------------------------------------
template <int R, int TY, int NT>
struct GFConfig {
    static constexpr int TX = 64;
    static constexpr int W = 2 * R + 1;
    static constexpr int E2X = TX + 4 * R, E2Y = TY + 4 * R;  // v / Zv apron
    static constexpr int E1X = TX + 2 * R, E1Y = TY + 2 * R;  // u / a / b apron
    static constexpr int odd(int x) { return (x & 1) ? x : x + 1; }
    static constexpr int PV = odd(E2X);   // Lv pitch (f64)  x-pass reads rows, lane <-> row
    static constexpr int PH = odd(E1X);   // Hx pitch (f64)  x-pass writes rows, lane <-> row
    static constexpr int PA = odd(E1X);   // La/Lb pitch (f32)
    static constexpr int PB = odd(TX);    // Ha/Hb pitch (f32)
    static constexpr int K2 = 4, K3 = 4, K4 = 4;
    static constexpr int K5 = TX * TY / NT;          // outputs per thread (ring width)
    static constexpr int S2 = (E1X + K2 - 1) / K2;   // segments per row, P2
    static constexpr int S3 = (E1Y + K3 - 1) / K3;   // segments per column, P3
    static constexpr int S4 = TX / K4;               // segments per row, P4
    static constexpr int N2 = E2Y * S2, N3 = E1X * S3, N4 = E1Y * S4;  // work items
    static constexpr int NE2 = E2X * E2Y;
    static constexpr int NP1 = (NE2 + NT - 1) / NT;  // apron positions per thread, P1
    // LDS in bytes. Region A: Lv (f64; P1 write, P2 read) aliased with La/Lb (f32; P3 write,
    // P4 read). Region B: Hx (f64; P2 write, P3 read) aliased with Ha/Hb (f32; P4 write, P5
    // read). Slack covers the over-read of the last (partial) segment.
    static constexpr int SLACK = 16 * 1024;
    static constexpr int SZ_LV = E2Y * PV * 8;
    static constexpr int SZ_LAB = 2 * E1Y * PA * 4;
    static constexpr int SZ_A = ((SZ_LV > SZ_LAB ? SZ_LV : SZ_LAB) + SLACK + 15) / 16 * 16;
    static constexpr int SZ_HX = E2Y * PH * 8;
    static constexpr int SZ_HAB = 2 * E1Y * PB * 4;
    static constexpr int SZ_B = ((SZ_HX > SZ_HAB ? SZ_HX : SZ_HAB) + SLACK + 15) / 16 * 16;
    static constexpr int LDS_BYTES = SZ_A + SZ_B;
    static_assert(TX * TY % NT == 0, "tile must divide evenly over the threads");
    static_assert(TY % K5 == 0, "ring segment must divide the tile height");
    static_assert(TX % K4 == 0, "P4 segment must divide the tile width");
    static_assert(N3 <= NT && N4 <= NT, "one P3/P4 work item per thread");
    static_assert(NP1 <= 32, "validity mask");
    static_assert(LDS_BYTES <= 160 * 1024, "LDS budget");
};

template <int R, int TY, int NT, typename TIn, typename TOut>
__global__ __launch_bounds__(NT) void gf3d_fused_kernel(GFParams p) {
    using C = GFConfig<R, TY, NT>;
    constexpr int TX = C::TX, W = C::W;
    constexpr int K5 = C::K5;
    extern __shared__ __attribute__((aligned(16))) char smem[];
    double* Lv = reinterpret_cast<double*>(smem);
    float* La = reinterpret_cast<float*>(smem);
    float* Lb = La + C::E1Y * C::PA;
    double* Hx = reinterpret_cast<double*>(smem + C::SZ_A);
    float* Ha = reinterpret_cast<float*>(smem + C::SZ_A);
    float* Hb = Ha + C::E1Y * C::PB;

    const TIn* __restrict__ in = static_cast<const TIn*>(p.in);
    TOut* __restrict__ out = static_cast<TOut*>(p.out);

    // XCD-aware block -> tile: blocks b and b+8 share an XCD, so give each XCD a contiguous run
    // of tiles (neighbouring tiles share their xy apron through that XCD's L2).
    const int nwg = gridDim.x;
    const int b = blockIdx.x;
    const int lid = (nwg % 8 == 0) ? (b % 8) * (nwg / 8) + b / 8 : b;
    const int tile_x = lid % p.tiles_x;
    const int tile_y = (lid / p.tiles_x) % p.tiles_y;
    const int seg = lid / (p.tiles_x * p.tiles_y);

    const int x0 = p.ox0 + tile_x * TX;
    const int y0 = p.oy0 + tile_y * TY;
    const int ox_end = p.ox0 + p.onx, oy_end = p.oy0 + p.ony;
    const int zo_begin = p.oz0 + seg * p.zseg;
    const int zo_end = min(zo_begin + p.zseg, p.oz0 + p.onz);
    const int nz = p.nz, ny = p.ny, nx = p.nx;
    const float eps = p.eps;
    const int tid0 = threadIdx.x;

    auto slice_ptr = [&](int z) -> const TIn* {
        return in + (int64_t)(z - p.in_z0) * p.in_sz;
    };

    // ---- P1 ownership: apron positions i = tid + k*NT of the (E2X x E2Y) plane -------------
    double zv[C::NP1];
    int32_t poff[C::NP1];  // y*sy + x element offset within a slice (valid positions)
    uint32_t pvalid = 0;   // bit k: position k is inside the domain
#pragma unroll
    for (int k = 0; k < C::NP1; ++k) {
        int i = tid0 + k * NT;
        int ey = i / C::E2X, ex = i % C::E2X;
        int gy = y0 - 2 * R + ey, gx = x0 - 2 * R + ex;
        bool ok = i < C::NE2 && gy >= 0 && gy < ny && gx >= 0 && gx < nx;
        pvalid |= ok ? (1u << k) : 0u;
        poff[k] = ok ? (int32_t)((int64_t)gy * p.in_sy + gx) : 0;
        zv[k] = 0.0;
    }

    const int zc_begin = zo_begin - R, zc_end = zo_end + R;
    const int zc0 = max(zc_begin, 0);  // first in-domain step
    // The running window advances only on in-domain steps; seed it for the first of them:
    // Zv(zc0 - 1) = sum of v over z in [zc0-1-R, zc0-1+R] clamped to [0, nz).
    {
        int zlo = max(zc0 - 1 - R, 0), zhi = min(zc0 - 1 + R, nz - 1);
        for (int z = zlo; z <= zhi; ++z) {
            const TIn* sp = slice_ptr(z);
#pragma unroll
            for (int k = 0; k < C::NP1; ++k)
                if (pvalid & (1u << k)) zv[k] += (double)Elem<TIn>::to_f32(sp[poff[k]]);
        }
    }

    // ---- prefetch registers: next step's entering/leaving slices (P1), centre slice (P3),
    //      output slice (emit). Issued one step ahead so HBM latency hides under a step. -----
    float pa[C::NP1], ps[C::NP1], pc3[C::K3], pv5[K5];
    auto prefetch = [&](int zc, int tid) {
        const int za = zc + R, zs = zc - R - 1;
        const bool ina = zc >= 0 && zc < nz && za < nz, ins = zc >= 0 && zc < nz && zs >= 0;
        const TIn* sa = slice_ptr(ina ? za : 0);
        const TIn* ss = slice_ptr(ins ? zs : 0);
#pragma unroll
        for (int k = 0; k < C::NP1; ++k) {
            const bool ok = (pvalid >> k) & 1u;
            pa[k] = (ok && ina) ? Elem<TIn>::to_f32(sa[poff[k]]) : 0.0f;
            ps[k] = (ok && ins) ? Elem<TIn>::to_f32(ss[poff[k]]) : 0.0f;
        }
        // P3 item of this thread: column col3, rows sg3*K3 + j of the E1 apron
        const bool zin = zc >= 0 && zc < nz;
        const int col3 = tid % C::E1X, sg3 = tid / C::E1X;
        const int gx = x0 - R + col3;
        const TIn* sc = slice_ptr(zin ? zc : 0);
#pragma unroll
        for (int j = 0; j < C::K3; ++j) {
            const int gy = y0 - R + sg3 * C::K3 + j;
            const bool ok = zin && tid < C::N3 && gx >= 0 && gx < nx && gy >= 0 && gy < ny &&
                            sg3 * C::K3 + j < C::E1Y;
            pc3[j] = ok ? Elem<TIn>::to_f32(sc[(int64_t)gy * p.in_sy + gx]) : 0.0f;
        }
        // emit: v(zo) for zo = zc - R at this thread's K5 outputs
        const int zo = zc - R;
        const bool zok = zo >= zo_begin && zo < zo_end;
        const int ox = x0 + tid % TX;
        const TIn* sv = slice_ptr(zok ? zo : zo_begin);
#pragma unroll
        for (int j = 0; j < K5; ++j) {
            const int oy = y0 + (tid / TX) * K5 + j;
            const bool ok = zok && ox < ox_end && oy < oy_end;
            pv5[j] = ok ? Elem<TIn>::to_f32(sv[(int64_t)oy * p.in_sy + ox]) : 0.0f;
        }
    };

    float ring_a[W][K5], ring_b[W][K5];
#pragma unroll
    for (int s = 0; s < W; ++s)
#pragma unroll
        for (int j = 0; j < K5; ++j) ring_a[s][j] = ring_b[s][j] = 0.0f;

    prefetch(zc_begin, tid0);
    int slot = 0;
    for (int zc = zc_begin; zc < zc_end; ++zc) {
        // Launder the thread index every step so the per-phase LDS addresses are recomputed
        // (a few VALU ops) instead of being hoisted out of the z-loop into ~40 live VGPRs.
        int tid = threadIdx.x;
        __asm__ volatile("" : "+v"(tid));
        // Consume this step's prefetched values, then issue the next step's loads.
        float ca[C::NP1], cs[C::NP1], cc3[C::K3], cv5[K5];
#pragma unroll
        for (int k = 0; k < C::NP1; ++k) { ca[k] = pa[k]; cs[k] = ps[k]; }
#pragma unroll
        for (int j = 0; j < C::K3; ++j) cc3[j] = pc3[j];
#pragma unroll
        for (int j = 0; j < K5; ++j) cv5[j] = pv5[j];
        if (zc + 1 < zc_end) prefetch(zc + 1, tid);

        float s2a[K5], s2b[K5];
        if (zc >= 0 && zc < nz) {
            // ---- P1: running z-window of v (f64) on the E2 apron -> Lv ----------------------
#pragma unroll
            for (int k = 0; k < C::NP1; ++k) {
                zv[k] = zv[k] + (double)ca[k];  // entering slice zc+R (0 when outside)
                zv[k] = zv[k] - (double)cs[k];  // leaving slice zc-R-1 (0 when outside)
                const int i = tid + k * NT;
                if (i < C::NE2) {
                    const int ey = i / C::E2X, ex = i % C::E2X;
                    Lv[ey * C::PV + ex] = zv[k];
                }
            }
            lds_barrier();
            // ---- P2: x-window sums (f64) of Lv rows -> Hx (E2Y rows x E1X cols) -------------
#pragma unroll 1
            for (int item = tid; item < C::N2; item += NT) {
                const int row = item % C::E2Y, sg = item / C::E2Y;
                const double* src = Lv + row * C::PV + sg * C::K2;
                double vin[C::K2 + 2 * R], vout[C::K2];
#pragma unroll
                for (int j = 0; j < C::K2 + 2 * R; ++j) vin[j] = src[j];
                slide_sums_f64<R, C::K2>(vin, vout);
#pragma unroll
                for (int j = 0; j < C::K2; ++j)
                    if (sg * C::K2 + j < C::E1X) Hx[row * C::PH + sg * C::K2 + j] = vout[j];
            }
            lds_barrier();
            // ---- P3: y-window sums (f64) of Hx columns -> U on E1; pointwise a, b -----------
            if (tid < C::N3) {
                const int col = tid % C::E1X, sg = tid / C::E1X;
                const double* src = Hx + (sg * C::K3) * C::PH + col;
                double vin[C::K3 + 2 * R], U[C::K3];
#pragma unroll
                for (int j = 0; j < C::K3 + 2 * R; ++j) vin[j] = src[j * C::PH];
                slide_sums_f64<R, C::K3>(vin, U);
                const int gx = x0 - R + col;
                const bool xin = gx >= 0 && gx < nx;
                const int cxz = xin ? clamped_count(gx, nx, R) * clamped_count(zc, nz, R) : 1;
#pragma unroll
                for (int j = 0; j < C::K3; ++j) {
                    const int ey = sg * C::K3 + j;
                    const int gy = y0 - R + ey;
                    float a = 0.0f, bb = 0.0f;
                    if (ey < C::E1Y && xin && gy >= 0 && gy < ny) {
                        // summed_area_table_mean: (sum as f32) / (count as f32)
                        const float cnt = (float)(clamped_count(gy, ny, R) * cxz);
                        const float u = (float)U[j] / cnt;
                        const float d = cc3[j] - u;
                        const float s = d * d;       // (v - u).powf(2.0)
                        a = s / (s + eps);
                        bb = (1.0f - a) * u;
                    }
                    if (ey < C::E1Y) {
                        La[ey * C::PA + col] = a;
                        Lb[ey * C::PA + col] = bb;
                    }
                }
            }
            lds_barrier();
            // ---- P4: x-window sums of La/Lb rows -> Ha/Hb (E1Y rows x TX cols) --------------
            if (tid < C::N4) {
                const int row = tid % C::E1Y, sg = tid / C::E1Y;
                {
                    const float* src = La + row * C::PA + sg * C::K4;
                    float vin[C::K4 + 2 * R], vout[C::K4];
#pragma unroll
                    for (int j = 0; j < C::K4 + 2 * R; ++j) vin[j] = src[j];
                    tree_window_sums<R, C::K4>(vin, vout);
#pragma unroll
                    for (int j = 0; j < C::K4; ++j) Ha[row * C::PB + sg * C::K4 + j] = vout[j];
                }
                {
                    const float* src = Lb + row * C::PA + sg * C::K4;
                    float vin[C::K4 + 2 * R], vout[C::K4];
#pragma unroll
                    for (int j = 0; j < C::K4 + 2 * R; ++j) vin[j] = src[j];
                    tree_window_sums<R, C::K4>(vin, vout);
#pragma unroll
                    for (int j = 0; j < C::K4; ++j) Hb[row * C::PB + sg * C::K4 + j] = vout[j];
                }
            }
            lds_barrier();
            // ---- P5: y-window sums of Ha/Hb columns -> this slice's tile sums ---------------
            {
                const int col5 = tid % TX, seg5 = tid / TX;
                const float* srca = Ha + (seg5 * K5) * C::PB + col5;
                const float* srcb = Hb + (seg5 * K5) * C::PB + col5;
                float vin[K5 + 2 * R];
#pragma unroll
                for (int j = 0; j < K5 + 2 * R; ++j) vin[j] = srca[j * C::PB];
                tree_window_sums<R, K5>(vin, s2a);
#pragma unroll
                for (int j = 0; j < K5 + 2 * R; ++j) vin[j] = srcb[j * C::PB];
                tree_window_sums<R, K5>(vin, s2b);
            }
        } else {
#pragma unroll
            for (int j = 0; j < K5; ++j) s2a[j] = s2b[j] = 0.0f;
        }

        // ---- ring update; z-window sums (oldest -> newest) for zo = zc - R ------------------
        const int zo = zc - R;
        float A[K5], B[K5];
        RingDispatch<0, W>::run(slot, [&](auto slot_c) {
            constexpr int SL = decltype(slot_c)::value;
#pragma unroll
            for (int j = 0; j < K5; ++j) {
                ring_a[SL][j] = s2a[j];
                ring_b[SL][j] = s2b[j];
                float za[W], zb[W];
#pragma unroll
                for (int t = 0; t < W; ++t) {
                    za[t] = ring_a[(SL + 1 + t) % W][j];
                    zb[t] = ring_b[(SL + 1 + t) % W][j];
                }
                float sa[1], sb[1];
                tree_window_sums<R, 1>(za, sa);
                tree_window_sums<R, 1>(zb, sb);
                A[j] = sa[0];
                B[j] = sb[0];
            }
        });
        const int ox5 = x0 + tid % TX;
        if (zo >= zo_begin && ox5 < ox_end) {
            const int cxz = clamped_count(ox5, nx, R) * clamped_count(zo, nz, R);
            TOut* po = out + (int64_t)(zo - p.oz0) * p.out_sz;
#pragma unroll
            for (int j = 0; j < K5; ++j) {
                const int oy = y0 + (tid / TX) * K5 + j;
                if (oy < oy_end) {
                    const float cnt = (float)(clamped_count(oy, ny, R) * cxz);
                    const float ma = A[j] / cnt;
                    const float mb = B[j] / cnt;
                    const float o = __fadd_rn(__fmul_rn(cv5[j], ma), mb);  // v *= ma; v += mb
                    po[(int64_t)(oy - p.oy0) * p.out_sy + (ox5 - p.ox0)] = from_f32<TOut>(o);
                }
            }
        }
        slot = slot + 1 == W ? 0 : slot + 1;
    }
}

// ---------------------------------------------------------------------------------------------
// Launch: pick the tile configuration for the radius, dispatch dtypes.
// ---------------------------------------------------------------------------------------------
template <int R, int TY, int NT, typename TIn, typename TOut>
inline hipError_t launch_fused_cfg(const GFParams& p0, hipStream_t stream) {
    using C = GFConfig<R, TY, NT>;
    GFParams p = p0;
    p.tiles_x = (p.onx + C::TX - 1) / C::TX;
    p.tiles_y = (p.ony + TY - 1) / TY;
    p.nseg = (p.onz + p.zseg - 1) / p.zseg;
    const size_t lds = (size_t)C::LDS_BYTES;
    auto kern = gf3d_fused_kernel<R, TY, NT, TIn, TOut>;
    static bool attr_set = false;  // per instantiation
    if (!attr_set) {
        hipError_t e = hipFuncSetAttribute((const void*)kern,
                                           hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
        if (e != hipSuccess) return e;
        attr_set = true;
    }
    const long long nwg = (long long)p.tiles_x * p.tiles_y * p.nseg;
    if (nwg <= 0) return hipSuccess;
    if (nwg > 0x7FFFFFFFLL) return hipErrorInvalidValue;
    hipLaunchKernelGGL(kern, dim3((unsigned)nwg), dim3(NT), lds, stream, p);
    return hipGetLastError();
}


// Element-type pairs with a direct fused instantiation (the rest are staged through f32).
inline bool fused_fast_dtype(int d) { return d == kF32 || d == kU16 || d == kU8 || d == kBool; }

#define ZT_FUSED_PAIRS(R, TY, NT)                                                                 \
    hipError_t launch_fused_radius_##R(const GFParams& p, int din, int dout, hipStream_t s) {     \
        auto pick_out = [&](auto tin) -> hipError_t {                                             \
            using TI = decltype(tin);                                                             \
            switch (dout) {                                                                       \
            case kF32: return launch_fused_cfg<R, TY, NT, TI, float>(p, s);                       \
            case kU16: return launch_fused_cfg<R, TY, NT, TI, uint16_t>(p, s);                    \
            case kU8: case kBool: return launch_fused_cfg<R, TY, NT, TI, uint8_t>(p, s);          \
            default: return hipErrorInvalidValue;                                                 \
            }                                                                                     \
        };                                                                                        \
        switch (din) {                                                                            \
        case kF32: return pick_out(float{});                                                      \
        case kU16: return pick_out(uint16_t{});                                                   \
        case kU8: case kBool: return pick_out(uint8_t{});                                         \
        default: return hipErrorInvalidValue;                                                     \
        }                                                                                         \
    }

}  // namespace zt
