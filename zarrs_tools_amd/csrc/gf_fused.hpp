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

// Generic version for vector element types (float2 = the (a, b) pair of stage 2).
template <int R, int K, typename T>
__device__ __forceinline__ void tree_window_sums_t(const T (&in)[K + 2 * R], T (&out)[K]) {
    constexpr int W = 2 * R + 1;
    constexpr int N = K + 2 * R;
    if constexpr (W == 1) {
#pragma unroll
        for (int i = 0; i < K; ++i) out[i] = in[i];
    } else {
        T p2[N], p4[N], p8[N], p16[N];
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
        static_assert(W < 32, "fused radii only");
#pragma unroll
        for (int i = 0; i < K; ++i) {
            T acc{};
            int off = 0;
            bool first = true;
#pragma unroll
            for (int b = 4; b >= 0; --b) {
                if (W & (1 << b)) {
                    T piece;
                    switch (b) {
                    case 0: piece = in[i + off]; break;
                    case 1: piece = p2[i + off]; break;
                    case 2: piece = p4[i + off]; break;
                    case 3: piece = p8[i + off]; break;
                    default: piece = p16[i + off]; break;
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

// Compile-time loop: f(integral_constant<I>) for I in [B, E).
template <int B, int E, typename F>
__device__ __forceinline__ void static_for(F&& f) {
    if constexpr (B < E) {
        f(std::integral_constant<int, B>{});
        static_for<B + 1, E>(f);
    }
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
// exactly like the reference's f64 summed-area-table sum (summed_area_table.rs:398-410). That
// matters: a = s/(s+eps) with s = (v-u)^2 is ill-conditioned in u for small eps, so u must be
// the reference's u bit for bit.
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

// s / (s + eps): rcp + one Newton step + Markstein correction (6 VALU ops instead of the ~12 of
// IEEE division; within 1 ulp, almost always correctly rounded). Special values follow IEEE:
// 0/0 and inf/inf give NaN as in the reference.
__device__ __forceinline__ float fast_div(float x, float d) {
    float y = __builtin_amdgcn_rcpf(d);
    float e = __builtin_fmaf(-d, y, 1.0f);
    y = __builtin_fmaf(e, y, y);
    float q = x * y;
    float r = __builtin_fmaf(-d, q, x);
    return __builtin_fmaf(r, y, q);
}

// Workgroup barrier for LDS hand-offs only. __syncthreads() also fences global memory, which
// makes the compiler drain every outstanding global load (vmcnt(0)) — including the loads this
// kernel keeps in flight across the barrier.
__device__ __forceinline__ void lds_barrier() {
    __asm__ volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
}
template <int ABL>
__device__ __forceinline__ void lds_barrier_abl() {
    if constexpr (ABL & 16) __asm__ volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    else lds_barrier();
}

// x / d for an integer count d given rcp = RN(1/d): Markstein's correction step makes the
// quotient correctly rounded (checked exhaustively-by-sampling for d <= 70000, tools/README),
// so this equals IEEE division at 3 VALU ops instead of ~11.
__device__ __forceinline__ float div_by_count(float x, float d, float rcp) {
    float q = x * rcp;
    float r = __builtin_fmaf(-q, d, x);
    return __builtin_fmaf(r, rcp, q);
}

// ---- buffer (SRD) loads/stores: 32-bit byte offsets, hardware range check (an offset past
//      num_records reads 0 / drops the store), no 64-bit address math per access. -----------
using rsrc_t = __amdgpu_buffer_rsrc_t;
constexpr int kBadOff = (int)0x80000000;  // >= num_records of any slice: reads 0, writes drop

__device__ __forceinline__ rsrc_t make_rsrc(const void* base, uint32_t bytes) {
    // Callers build descriptors only from kernel arguments and loop counters (wave-uniform
    // scalars), so hipcc keeps them in SGPRs: no readfirstlane, no waterfall loops (T20).
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, (int)bytes,
                                             0x00020000);
}

template <typename T> struct Buf;
template <> struct Buf<float> {
    __device__ static float load(rsrc_t r, int off) {
        return __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(r, off, 0, 0));
    }
    // Output stores are streamed with the non-temporal hint (aux 2 = nt) so they do not evict
    // the input slices the march re-reads from L2 a few steps later.
    __device__ static void store(float v, rsrc_t r, int off) {
        __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(uint32_t, v), r, off, 0, 2);
    }
};
template <> struct Buf<uint16_t> {
    __device__ static float load(rsrc_t r, int off) {
        return (float)(uint16_t)__builtin_amdgcn_raw_buffer_load_b16(r, off, 0, 0);
    }
    __device__ static void store(uint16_t v, rsrc_t r, int off) {
        __builtin_amdgcn_raw_buffer_store_b16(v, r, off, 0, 2);
    }
};
template <> struct Buf<uint8_t> {
    __device__ static float load(rsrc_t r, int off) {
        return (float)(uint8_t)__builtin_amdgcn_raw_buffer_load_b8(r, off, 0, 0);
    }
    __device__ static void store(uint8_t v, rsrc_t r, int off) {
        __builtin_amdgcn_raw_buffer_store_b8(v, r, off, 0, 2);
    }
};

// ---------------------------------------------------------------------------------------------
// The fused kernel.
//
// Software-pipelined phases, two LDS barriers per z-step. Iteration `i` runs
//   C0: P3(i)  [U -> a,b on the E1 apron]  +  P1(i+1) [z-window of v]  +  P5(i-1) [y-sums,
//       z-ring, emit out(i-1-R)]
//   C1: P4(i)  [x-sums of (a,b)]           +  P2(i+1) [x-sums of the v z-window]
// with separate LDS buffers per hand-off (Lv, Hx, Lab, Hab), so each barrier interval holds
// independent work from different slices (better wave balance, half the barriers of a
// straight P1..P5 sequence).
// ---------------------------------------------------------------------------------------------
template <int R, int TY, int NT>
struct GFConfig {
    static constexpr int TX = 64;
    static constexpr int W = 2 * R + 1;
    static constexpr int E2X = TX + 4 * R, E2Y = TY + 4 * R;  // v / Zv apron
    static constexpr int E1X = TX + 2 * R, E1Y = TY + 2 * R;  // u / a / b apron
    // Pitches in 8-byte elements, = 2 mod 4: 16-B aligned rows and conflict-free ds_*_b128
    // when lanes walk rows (16-lane groups land on distinct 4-bank slots).
    static constexpr int p2m4(int x) { return x + ((2 - x % 4) + 4) % 4; }
    static constexpr int PV = p2m4(E2X);  // Lv  (f64)    P1 writes, P2 reads rows
    static constexpr int PH = p2m4(E1X);  // Hx  (f64)    P2 writes rows, P3 reads columns
    static constexpr int PA = p2m4(E1X);  // Lab (float2) P3 writes, P4 reads rows
    static constexpr int PB = p2m4(TX);   // Hab (float2) P4 writes rows, P5 reads columns
    static constexpr int K2 = 4, K3 = 4, K4 = 4;
    static constexpr int K5 = TX * TY / NT;          // outputs per thread (ring width)
    static constexpr int S2 = (E1X + K2 - 1) / K2;   // segments per row, P2
    static constexpr int S3 = (E1Y + K3 - 1) / K3;   // segments per column, P3
    static constexpr int S4 = TX / K4;               // segments per row, P4
    static constexpr int N2 = E2Y * S2, N3 = E1X * S3, N4 = E1Y * S4;  // work items
    static constexpr int R1 = NT / E2X;              // P1: apron rows per pass
    static constexpr int NP1 = (E2Y + R1 - 1) / R1;  // P1: passes (positions per thread)
    static constexpr int W3 = W * W * W;             // interior window count
    static constexpr int al(int b) { return (b + 255) / 256 * 256; }
    static constexpr int SZ_LV = al((E2Y + 1) * PV * 8);
    static constexpr int SZ_HX = al((E2Y + K3) * PH * 8);
    static constexpr int SZ_LAB = al((E1Y + 1) * PA * 8);
    static constexpr int SZ_HAB = al((E1Y + 1) * PB * 8);
    static constexpr int OFF_HX = SZ_LV, OFF_LAB = OFF_HX + SZ_HX, OFF_HAB = OFF_LAB + SZ_LAB;
    static constexpr int OFF_RCP = OFF_HAB + SZ_HAB;
    static constexpr int SZ_RCP = al((W3 + 1) * 4);  // RN(1/c) for window counts c <= W^3
    static constexpr int LDS_BYTES = OFF_RCP + SZ_RCP;
    // item -> thread placement: heavy phases on different waves (see C0 / C1)
    static constexpr int T3 = NT - N3;  // P3 items on the top threads
    static constexpr int T2 = NT - N2;  // P2 items on the top threads, P4 on the bottom
    static_assert(TX * TY % NT == 0, "tile must divide evenly over the threads");
    static_assert(TY % K5 == 0, "ring segment must divide the tile height");
    static_assert(TX % K4 == 0, "P4 segment must divide the tile width");
    static_assert(N2 <= NT && N3 <= NT && N4 <= NT, "one work item per thread per phase");
    static_assert(R1 >= 1, "P1 needs a full apron row per pass");
    static_assert(LDS_BYTES <= 160 * 1024, "LDS budget");
};

template <int R, int TY, int NT, typename TIn, typename TOut, int ABL = 0>
__global__ __launch_bounds__(NT) void gf3d_fused_kernel(GFParams p) {
    using C = GFConfig<R, TY, NT>;
    constexpr int TX = C::TX, W = C::W;
    constexpr int K5 = C::K5;
    constexpr int ESZ = (int)sizeof(TIn), OSZ = (int)sizeof(TOut);
    extern __shared__ __attribute__((aligned(16))) char smem[];
    double* Lv = reinterpret_cast<double*>(smem);
    double* Hx = reinterpret_cast<double*>(smem + C::OFF_HX);
    float2* Lab = reinterpret_cast<float2*>(smem + C::OFF_LAB);
    float2* Hab = reinterpret_cast<float2*>(smem + C::OFF_HAB);
    float* rcp_tab = reinterpret_cast<float*>(smem + C::OFF_RCP);
    // Correctly rounded reciprocals of every possible window count, for div_by_count
    // (Markstein's correction needs RN(1/c) exactly). Published by the prologue's barriers.
    for (int c = threadIdx.x; c <= C::W3; c += NT) rcp_tab[c] = c > 0 ? 1.0f / (float)c : 0.0f;

    // XCD-aware block -> tile. Blocks b and b+8 share an XCD; give each XCD a contiguous run of
    // logical ids and walk them in 8x4-tile super-tiles, so the WGs resident on one XCD cover a
    // compact 512x128 region whose xy aprons and z reloads stay in that XCD's 4 MB L2.
    const int nwg = gridDim.x;
    const int b = blockIdx.x;
    const int lid = (nwg % 8 == 0) ? (b % 8) * (nwg / 8) + b / 8 : b;
    const int ntiles = p.tiles_x * p.tiles_y;
    const int seg = lid / ntiles;
    int t = lid % ntiles;
    int tile_x, tile_y;
    {
        const int stx = 8, sty = 4;
        const int full_y = p.tiles_y / sty * sty;
        const int per_srow = p.tiles_x * sty;
        if (t < full_y * p.tiles_x) {
            const int sr = t / per_srow, r = t % per_srow;
            const int full_x = p.tiles_x / stx * stx;
            if (r < full_x * sty) {
                tile_x = (r / (stx * sty)) * stx + r % stx;
                tile_y = sr * sty + (r / stx) % sty;
            } else {
                const int rr = r - full_x * sty, w = p.tiles_x - full_x;
                tile_x = full_x + rr % w;
                tile_y = sr * sty + rr / w;
            }
        } else {
            t -= full_y * p.tiles_x;
            tile_x = t % p.tiles_x;
            tile_y = full_y + t / p.tiles_x;
        }
    }

    const int x0 = p.ox0 + tile_x * TX;
    const int y0 = p.oy0 + tile_y * TY;
    const int ox_end = p.ox0 + p.onx, oy_end = p.oy0 + p.ony;
    const int zo_begin = p.oz0 + seg * p.zseg;
    const int zo_end = min(zo_begin + p.zseg, p.oz0 + p.onz);
    const int nz = p.nz, ny = p.ny, nx = p.nx;
    const float eps = p.eps;
    const uint32_t slice_bytes = (uint32_t)((int64_t)(p.ny - 1) * p.in_sy + p.nx) * ESZ;
    const uint32_t oslice_bytes =
        (uint32_t)((int64_t)(p.ony - 1) * p.out_sy + p.onx) * OSZ;
    const int sy = (int)p.in_sy, osy = (int)p.out_sy;  // 32-bit: slices < 2 GiB (host check)

    const char* in_base = static_cast<const char*>(p.in);
    auto slice_rsrc = [&](int z) -> rsrc_t {
        const bool ok = z >= 0 && z < nz;
        const char* base = in_base + (ok ? (int64_t)(z - p.in_z0) * p.in_sz * ESZ : 0);
        return make_rsrc(base, ok ? slice_bytes : 0u);
    };

    // ---- per-thread, step-invariant byte offsets (kBadOff where outside the domain) --------
    const int tid0 = threadIdx.x;
    int p1off[C::NP1];
    {
        const int row0 = tid0 / C::E2X, col = tid0 % C::E2X;
        const int gx = x0 - 2 * R + col;
        const bool xin = tid0 < C::R1 * C::E2X && gx >= 0 && gx < nx;
#pragma unroll
        for (int k = 0; k < C::NP1; ++k) {
            const int row = row0 + k * C::R1;
            const int gy = y0 - 2 * R + row;
            const bool ok = xin && row < C::E2Y && gy >= 0 && gy < ny;
            p1off[k] = ok ? (gy * sy + gx) * ESZ : kBadOff;
        }
    }

    double zv[C::NP1];
#pragma unroll
    for (int k = 0; k < C::NP1; ++k) zv[k] = 0.0;
    const int zc_begin = zo_begin - R, zc_end = zo_end + R;  // stage-1 slices of this march
    // Running z-window: seed Zv(zc_begin - 1) = sum of v over [zc_begin-1-R, zc_begin-1+R]
    // clamped to [0, nz); every later step adds the entering and subtracts the leaving slice
    // (both 0 outside the domain), so the window stays exact through out-of-domain steps.
    {
        const int zlo = max(zc_begin - 1 - R, 0), zhi = min(zc_begin - 1 + R, nz - 1);
        for (int z = zlo; z <= zhi; ++z) {
            const rsrc_t rs = slice_rsrc(z);
#pragma unroll
            for (int k = 0; k < C::NP1; ++k) zv[k] += (double)Buf<TIn>::load(rs, p1off[k]);
        }
    }

    float ring_a[W][K5], ring_b[W][K5];
#pragma unroll
    for (int s = 0; s < W; ++s)
#pragma unroll
        for (int j = 0; j < K5; ++j) ring_a[s][j] = ring_b[s][j] = 0.0f;
    double za_run[K5], zb_run[K5];
#pragma unroll
    for (int j = 0; j < K5; ++j) za_run[j] = zb_run[j] = 0.0;

    // ---- phase bodies ----------------------------------------------------------------------
    float pa[C::NP1], ps[C::NP1];  // P1 inputs for the next stage-1 slice (prefetched)
    auto load_p1 = [&](int zc) {    // entering slice zc+R and leaving slice zc-R-1 of step zc
        const rsrc_t ra = slice_rsrc(zc + R);
        const rsrc_t rs = slice_rsrc(zc - R - 1);
#pragma unroll
        for (int k = 0; k < C::NP1; ++k) {
            pa[k] = (ABL & 8) ? 1.0f : Buf<TIn>::load(ra, p1off[k]);
            ps[k] = (ABL & 1) ? 0.5f : Buf<TIn>::load(rs, p1off[k]);
        }
    };
    auto do_p1 = [&](int tid) {  // z-window of v (f64) on the E2 apron -> Lv
        const int row0 = tid / C::E2X, col = tid % C::E2X;
        double* dst = Lv + row0 * C::PV + col;
        const bool act = tid < C::R1 * C::E2X;
#pragma unroll
        for (int k = 0; k < C::NP1; ++k) {
            zv[k] = zv[k] + (double)pa[k];  // entering slice zc+R (0 outside the domain)
            zv[k] = zv[k] - (double)ps[k];  // leaving slice zc-R-1 (0 outside the domain)
            if (act && row0 + k * C::R1 < C::E2Y) dst[k * C::R1 * C::PV] = zv[k];
        }
    };
    auto do_p2 = [&](int tid) {  // x-window sums (f64) of Lv rows -> Hx
        const int item = tid - C::T2;
        if (item < 0) return;
        const int row = item % C::E2Y, sg = item / C::E2Y;
        const double2* src =
            reinterpret_cast<const double2*>(Lv + row * C::PV + sg * C::K2);
        double vin[C::K2 + 2 * R], vout[C::K2];
#pragma unroll
        for (int j = 0; j < (C::K2 + 2 * R) / 2; ++j) {
            const double2 d2 = src[j];
            vin[2 * j] = d2.x;
            vin[2 * j + 1] = d2.y;
        }
        if constexpr ((C::K2 + 2 * R) % 2) vin[C::K2 + 2 * R - 1] = Lv[row * C::PV + sg * C::K2 + C::K2 + 2 * R - 1];
        slide_sums_f64<R, C::K2>(vin, vout);
        double2* dst = reinterpret_cast<double2*>(Hx + row * C::PH + sg * C::K2);
#pragma unroll
        for (int j = 0; j < C::K2 / 2; ++j)
            if (sg * C::K2 + 2 * j < C::E1X) dst[j] = make_double2(vout[2 * j], vout[2 * j + 1]);
    };
    float v3[C::K3];  // v at the P3 item's E1 positions, slice i (prefetched one step ahead)
    auto load_v3 = [&](int tid, int zc) {
        const int item = tid - C::T3;
        const int col = item % C::E1X, sg = item / C::E1X;
        const int gx = x0 - R + col;
        const bool xin = item >= 0 && gx >= 0 && gx < nx;
        const rsrc_t rc = slice_rsrc(zc);
#pragma unroll
        for (int j = 0; j < C::K3; ++j) {
            const int ey = sg * C::K3 + j, gy = y0 - R + ey;
            const bool ok = xin && ey < C::E1Y && gy >= 0 && gy < ny;
            v3[j] = (ABL & 2) ? 1.0f
                              : Buf<TIn>::load(rc, ok ? (gy * sy + gx) * ESZ : kBadOff);
        }
    };
    auto do_p3 = [&](int tid, int zc) {  // y-window (f64) of Hx -> U; a, b -> Lab
        const int item = tid - C::T3;
        if (item < 0) return;
        const int col = item % C::E1X, sg = item / C::E1X;
        const double* src = Hx + (sg * C::K3) * C::PH + col;
        double vin[C::K3 + 2 * R], U[C::K3];
#pragma unroll
        for (int j = 0; j < C::K3 + 2 * R; ++j) vin[j] = src[j * C::PH];
        slide_sums_f64<R, C::K3>(vin, U);
        const int gx = x0 - R + col;
        const bool xzin = gx >= 0 && gx < nx && zc >= 0 && zc < nz;
        const int cxz = clamped_count(gx, nx, R) * clamped_count(zc, nz, R);
#pragma unroll
        for (int j = 0; j < C::K3; ++j) {
            const int ey = sg * C::K3 + j;
            const int gy = y0 - R + ey;
            // summed_area_table_mean: (sum as f32) / (count as f32)
            const int cnt = clamped_count(gy, ny, R) * cxz;
            const float fc = (float)cnt;
            const float rc = rcp_tab[cnt];
            const float u = div_by_count((float)U[j], fc, rc);
            const float d = v3[j] - u;
            const float s = d * d;  // (v - u).powf(2.0)
            float a, bb;
            if constexpr (ABL & 32) {
                a = s; bb = u;
            } else {
                a = fast_div(s, s + eps);
                bb = (1.0f - a) * u;
            }
            const bool ok = xzin && gy >= 0 && gy < ny;  // zero outside: clamped window sums
            if (ey < C::E1Y) Lab[ey * C::PA + col] = ok ? make_float2(a, bb) : make_float2(0.f, 0.f);
        }
    };
    auto do_p4 = [&](int tid) {  // x-window sums of (a, b) rows -> Hab
        const int item = tid;
        if (item >= C::N4) return;
        const int row = item % C::E1Y, sg = item / C::E1Y;
        const float4* src = reinterpret_cast<const float4*>(Lab + row * C::PA + sg * C::K4);
        float2 vin[C::K4 + 2 * R], vout[C::K4];
#pragma unroll
        for (int j = 0; j < (C::K4 + 2 * R) / 2; ++j) {
            const float4 f = src[j];
            vin[2 * j] = make_float2(f.x, f.y);
            vin[2 * j + 1] = make_float2(f.z, f.w);
        }
        if constexpr ((C::K4 + 2 * R) % 2) vin[C::K4 + 2 * R - 1] = Lab[row * C::PA + sg * C::K4 + C::K4 + 2 * R - 1];
        tree_window_sums_t<R, C::K4>(vin, vout);
        float4* dst = reinterpret_cast<float4*>(Hab + row * C::PB + sg * C::K4);
#pragma unroll
        for (int j = 0; j < C::K4 / 2; ++j)
            dst[j] = make_float4(vout[2 * j].x, vout[2 * j].y, vout[2 * j + 1].x, vout[2 * j + 1].y);
    };
    float v5[K5];  // v at this thread's outputs for the slice being emitted (prefetched)
    auto load_v5 = [&](int tid, int zo) {
        const int ox = x0 + tid % TX, oyb = y0 + (tid / TX) * K5;
        const bool zok = zo >= zo_begin && zo < zo_end;
        const rsrc_t rv = slice_rsrc(zok ? zo : -1);
#pragma unroll
        for (int j = 0; j < K5; ++j) {
            const int oy = oyb + j;
            const bool ok = ox < ox_end && oy < oy_end;
            v5[j] = (ABL & 4) ? 1.0f
                              : Buf<TIn>::load(rv, ok ? (oy * sy + ox) * ESZ : kBadOff);
        }
    };
    auto do_p5 = [&](int tid, int zc, auto slot_c) {  // y-window -> slice sums; ring; emit zc-R
        const int col5 = tid % TX, seg5 = tid / TX;
        const float2* src = Hab + (seg5 * K5) * C::PB + col5;
        float2 vin[K5 + 2 * R], s2[K5];
#pragma unroll
        for (int j = 0; j < K5 + 2 * R; ++j) vin[j] = src[j * C::PB];
        tree_window_sums_t<R, K5>(vin, s2);
        // Ring of the last W slice sums, indexed by a compile-time slot (the march is unrolled
        // by W, so every index is static and the ring stays in registers with no moves): the
        // z-window is an exact f64 running sum, the ring supplies the leaving entry.
        constexpr int SL = decltype(slot_c)::value;
        float A[K5], B[K5];
#pragma unroll
        for (int j = 0; j < K5; ++j) {
            const float olda = ring_a[SL][j], oldb = ring_b[SL][j];
            ring_a[SL][j] = s2[j].x;
            ring_b[SL][j] = s2[j].y;
            za_run[j] = za_run[j] + (double)s2[j].x;
            za_run[j] = za_run[j] - (double)olda;
            zb_run[j] = zb_run[j] + (double)s2[j].y;
            zb_run[j] = zb_run[j] - (double)oldb;
            A[j] = (float)za_run[j];
            B[j] = (float)zb_run[j];
        }
        const int zo = zc - R;
        if (zo >= zo_begin) {
            const int ox = x0 + col5, oyb = y0 + seg5 * K5;
            const int cxz = clamped_count(ox, nx, R) * clamped_count(zo, nz, R);
            const char* obase = static_cast<const char*>(p.out) +
                                (int64_t)(zo - p.oz0) * p.out_sz * OSZ;
            const rsrc_t ro = make_rsrc(obase, oslice_bytes);
#pragma unroll
            for (int j = 0; j < K5; ++j) {
                const int oy = oyb + j;
                const int cnt = clamped_count(oy, ny, R) * cxz;
                const float fc = (float)cnt;
                const float rc = rcp_tab[cnt];
                const float ma = div_by_count(A[j], fc, rc);
                const float mb = div_by_count(B[j], fc, rc);
                const float o = __fadd_rn(__fmul_rn(v5[j], ma), mb);  // v *= ma; v += mb
                const bool ok = ox < ox_end && oy < oy_end;
                const int off = ok ? ((oy - p.oy0) * osy + (ox - p.ox0)) * OSZ : kBadOff;
                Buf<TOut>::store(from_f32<TOut>(o), ro, off);
            }
        }
    };

    // ---- prologue: stage 1 of the first slice up to Hx ------------------------------------
    load_p1(zc_begin);
    do_p1(tid0);
    lds_barrier_abl<ABL>();
    do_p2(tid0);
    if (zc_begin + 1 < zc_end) load_p1(zc_begin + 1);
    load_v3(tid0, zc_begin);
    lds_barrier_abl<ABL>();

    // ---- pipelined march, unrolled by W so the ring slot of every P5 is a constant ----------
    for (int i0 = zc_begin; i0 < zc_end; i0 += W) {
        static_for<0, W>([&](auto kc) {
            constexpr int k = decltype(kc)::value;
            const int i = i0 + k;
            if (i >= zc_end) return;
            const int tid = threadIdx.x;
            const bool has_next = i + 1 < zc_end;
            // C0: P3(i) + P1(i+1) + P5(i-1)
            do_p3(tid, i);
            if (has_next) do_p1(tid);
            if (i > zc_begin) do_p5(tid, i - 1, std::integral_constant<int, (k + W - 1) % W>{});
            // loads for the next iteration's C0 (latency hides under C1 and the barriers)
            if (i + 2 < zc_end) load_p1(i + 2);
            if (has_next) load_v3(tid, i + 1);
            load_v5(tid, i - R);
            lds_barrier_abl<ABL>();
            // C1: P4(i) + P2(i+1)
            do_p4(tid);
            if (has_next) do_p2(tid);
            lds_barrier_abl<ABL>();
        });
    }
    // ---- epilogue: stage 2 tail of the last slice (runtime slot -> dispatch, once) ----------
    RingDispatch<0, W>::run((zc_end - 1 - zc_begin) % W, [&](auto slot_c) {
        do_p5((int)threadIdx.x, zc_end - 1, slot_c);
    });
}

// ---------------------------------------------------------------------------------------------
// Launch: pick the tile configuration for the radius, dispatch dtypes.
// ---------------------------------------------------------------------------------------------
template <int R, int TY, int NT, typename TIn, typename TOut>
inline hipError_t launch_fused_cfg(const GFParams& p0, hipStream_t stream) {
    using C = GFConfig<R, TY, NT>;
    GFParams p = p0;
    {
        const float w3 = (float)(C::W3);
        volatile float one = 1.0f;  // IEEE division on the host: RN(1/W^3)
        p.rcp_w3 = one / w3;
    }
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
