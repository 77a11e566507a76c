// gf_fused.hpp — the fused 2.5-D guided-filter kernel template (see guided_filter.hip for the
// design notes). Instantiated per radius in gf_fused_r<R>.hip so the instantiations compile in
// parallel; guided_filter.hip dispatches.
#pragma once

#include <hip/hip_runtime.h>

#include <atomic>
#include <stdint.h>

#include <algorithm>
#include <type_traits>

#include "zt_device.hpp"
#include "zt_kernels.hpp"

// Tuning knobs (tools/timek.hip sweeps them with -D; profiles/r02_ab_harness.txt). Variants that
// were measured slower were deleted; their numbers stay in DESIGN.md §3.1.
#ifndef GF_K4_R4
#define GF_K4_R4 8  // r = 4: P4 outputs per item (8 x per item, -2 %)
#endif
#ifndef GF_ORDER_R4
#define GF_ORDER_R4 2  // r = 4: P4 issued ahead of P12 in C1 (-2 %)
#endif
#ifndef GF_ORDER
#define GF_ORDER 0  // other radii: P4 after P12 in C1
#endif
#ifndef GF_PRIO
#define GF_PRIO 1  // s_setprio phase reordering (measured -4.5% at 2048^3 r=4 with the b128 Hx writes)
#endif
#ifndef GF_HX_B128
#define GF_HX_B128 1  // 16-byte Hx writes for even R (fewer LDS bank conflicts: -2% at r=4)
#endif
#ifndef GF_P1RING_MAXR
#define GF_P1RING_MAXR 2  // stage-1 z-window ring in registers up to this radius (see GFConfig)
#endif
#ifndef GF_K3
#define GF_K3 4  // P3 outputs per thread (column segment of the f64 y-window)
#endif
#ifndef GF_K4
#define GF_K4 4  // P4 outputs per thread (row segment of the (a, b) x-window)
#endif
#ifndef GF_STX
#define GF_STX 4  // XCD super-tile: tiles along x (4 x 16 measured best: 31.2 vs 31.9 ms for 8 x 4)
#endif
#ifndef GF_STY
#define GF_STY 16  // XCD super-tile: tiles along y
#endif
#ifndef GF_P1PFD
#define GF_P1PFD 2  // stage-1 slices prefetched this many steps ahead at r = 4 (1 or 2)
#endif
#ifndef GF_P1PFD_R2
#define GF_P1PFD_R2 2  // the same at r <= 2 (stage-1 ring: entering quads only)
#endif
#ifndef GF_WAVE_SKIP
#define GF_WAVE_SKIP 1  // P4: idle waves branch around the phase
#endif

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


// Packed pair of f32 (v_pk_add_f32 / v_pk_mul_f32 / v_pk_fma_f32: both lanes for one issue).
typedef float f2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ f2 pk_fma(f2 a, f2 b, f2 c) { return __builtin_elementwise_fma(a, b, c); }

// Window sums of W = 2R+1 consecutive values for K consecutive outputs sharing one core:
// every window contains in[K-1 .. W-1], so out_i = (in[i..K-2]) + core + (in[W..W+i-1]) with
// the left parts built as suffix sums and the right parts as prefix sums: W + 3K - 6 adds
// instead of a tree per output (9 vs 16 for K=2, 15 vs 26 for K=4 at R=4). Falls back to the
// tree when K > W (tiny radii).
template <int R, int K, typename T>
__device__ __forceinline__ void core_window_sums(const T (&in)[K + 2 * R], T (&out)[K]);

__device__ __forceinline__ int clamped_count(int i, int n, int r) {
    int lo = i - r < 0 ? 0 : i - r;
    int hi = i + r > n - 1 ? n - 1 : i + r;
    return hi - lo + 1;
}
// Product of window counts (each <= 2R + 1 <= 17, products <= 17^3): the full-rate 24-bit
// multiply instead of v_mul_lo_u32.
__device__ __forceinline__ int cmul(int a, int b) { return (int)__umul24((unsigned)a, (unsigned)b); }

template <int R, int K, typename T>
__device__ __forceinline__ void core_window_sums(const T (&in)[K + 2 * R], T (&out)[K]) {
    constexpr int W = 2 * R + 1;
    if constexpr (K > W || K < 2) {
        tree_window_sums_t<R, K>(in, out);
    } else {
        // core = in[K-1 .. W-1] summed pairwise (balanced)
        constexpr int NC = W - K + 1;
        T c[NC];
#pragma unroll
        for (int j = 0; j < NC; ++j) c[j] = in[K - 1 + j];
#pragma unroll
        for (int w = 1; w < NC; w *= 2) {
#pragma unroll
            for (int j = 0; j + w < NC; j += 2 * w) c[j] = c[j] + c[j + w];
        }
        const T core = c[0];
        T left[K], right[K];  // left[i] = in[i..K-2], right[i] = in[W..W+i-1]
        if constexpr (K >= 2) {
            left[K - 2] = in[K - 2];
#pragma unroll
            for (int i = K - 3; i >= 0; --i) left[i] = in[i] + left[i + 1];
            right[1] = in[W];
#pragma unroll
            for (int i = 2; i < K; ++i) right[i] = right[i - 1] + in[W + i - 1];
        }
        out[0] = left[0] + core;
#pragma unroll
        for (int i = 1; i < K - 1; ++i) out[i] = (left[i] + core) + right[i];
        out[K - 1] = core + right[K - 1];
    }
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
template <int R, int K, typename T>
__device__ __forceinline__ void slide_sums_exact(const T (&in)[K + 2 * R], T (&out)[K]) {
    // exact sums (f64 of f32 values, or 32-bit integers): any association gives the same
    // value, so the first window is a balanced tree and each later one adds an independently
    // formed difference (chain depth log2(W) + K - 1 instead of 2R + 2(K - 1))
    T c[2 * R + 1];
#pragma unroll
    for (int j = 0; j <= 2 * R; ++j) c[j] = in[j];
#pragma unroll
    for (int w = 1; w <= 2 * R; w *= 2) {
#pragma unroll
        for (int j = 0; j + w <= 2 * R; j += 2 * w) c[j] = c[j] + c[j + w];
    }
    T d[K];
#pragma unroll
    for (int i = 1; i < K; ++i) d[i] = in[i + 2 * R] - in[i - 1];
    out[0] = c[0];
#pragma unroll
    for (int i = 1; i < K; ++i) out[i] = out[i - 1] + d[i];
}

// Stage-1 arithmetic per input type. 8- and 16-bit integer inputs are summed exactly in 32-bit
// integers (a window of W^3 <= 17^3 values of at most 65535 stays below 2^31): the same U as the
// reference's f64 SAT of their `as f32` values, at one 2-cycle add per term instead of f64
// conversions and adds, one DPP move per neighbour instead of two, and 4-byte Hx elements.
template <typename T> struct S1 {
    using acc = double;  // window sums
    using in = float;    // loaded stage-1 values
    static constexpr int HXB = 8;
};
template <> struct S1<uint8_t> { using acc = int; using in = int; static constexpr int HXB = 4; };
template <> struct S1<uint16_t> { using acc = int; using in = int; static constexpr int HXB = 4; };

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
#ifndef GF_OUT_AUX
#define GF_OUT_AUX 2  // f32 output stores: 2 = nt (see Buf<float>::store)
#endif
constexpr int kBadOff = (int)0x80000000;  // >= num_records of any slice: reads 0, writes drop

__device__ __forceinline__ rsrc_t make_rsrc(const void* base, uint32_t bytes) {
    // Callers build descriptors only from kernel arguments and loop counters (wave-uniform
    // scalars), so hipcc keeps them in SGPRs: no readfirstlane, no waterfall loops (T20).
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, (int)bytes,
                                             0x00020000);
}

template <typename T> struct Buf;
template <> struct Buf<float> {
    template <int AUX = 0>
    __device__ static float load(rsrc_t r, int off) {
        return __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(r, off, 0, AUX));
    }
    // Output stores are streamed with the non-temporal hint (aux 2 = nt) so they do not evict
    // the input slices the march re-reads from L2 a few steps later.
    __device__ static void store(float v, rsrc_t r, int off) {
        __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(uint32_t, v), r, off, 0, GF_OUT_AUX);
    }
};
template <> struct Buf<uint16_t> {
    template <int AUX = 0>
    __device__ static float load(rsrc_t r, int off) {
        return (float)(uint16_t)__builtin_amdgcn_raw_buffer_load_b16(r, off, 0, AUX);
    }
    __device__ static int load_int(rsrc_t r, int off) {
        return (int)(uint16_t)__builtin_amdgcn_raw_buffer_load_b16(r, off, 0, 0);
    }
    __device__ static void store(uint16_t v, rsrc_t r, int off) {
        __builtin_amdgcn_raw_buffer_store_b16(v, r, off, 0, 2);
    }
};
template <> struct Buf<uint8_t> {
    template <int AUX = 0>
    __device__ static float load(rsrc_t r, int off) {
        return (float)(uint8_t)__builtin_amdgcn_raw_buffer_load_b8(r, off, 0, AUX);
    }
    __device__ static int load_int(rsrc_t r, int off) {
        return (int)(uint8_t)__builtin_amdgcn_raw_buffer_load_b8(r, off, 0, 0);
    }
    __device__ static void store(uint8_t v, rsrc_t r, int off) {
        __builtin_amdgcn_raw_buffer_store_b8(v, r, off, 0, 2);
    }
};

// ---- DPP wave shifts of an f64 (lane i <- lane i-1 / i+1; GFX9 wave_shr:1 / wave_shl:1) ----
// bound_ctrl set: lanes whose source lies outside the wave read 0, so no "old" value has to be
// materialised in the destination first (update_dpp with old = 0 costs a v_mov per DPP move).
__device__ __forceinline__ double dpp_from_lower(double v) {
    const int lo = __builtin_amdgcn_mov_dpp(__double2loint(v), 0x138, 0xF, 0xF, true);
    const int hi = __builtin_amdgcn_mov_dpp(__double2hiint(v), 0x138, 0xF, 0xF, true);
    return __hiloint2double(hi, lo);
}
__device__ __forceinline__ double dpp_from_upper(double v) {
    const int lo = __builtin_amdgcn_mov_dpp(__double2loint(v), 0x130, 0xF, 0xF, true);
    const int hi = __builtin_amdgcn_mov_dpp(__double2hiint(v), 0x130, 0xF, 0xF, true);
    return __hiloint2double(hi, lo);
}
__device__ __forceinline__ int dpp_from_lower(int v) {
    return __builtin_amdgcn_mov_dpp(v, 0x138, 0xF, 0xF, true);
}
__device__ __forceinline__ int dpp_from_upper(int v) {
    return __builtin_amdgcn_mov_dpp(v, 0x130, 0xF, 0xF, true);
}

// ---- 4 consecutive elements (one 16/8/4-byte buffer access per lane) ----------------------
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));

template <typename T> struct Quad;
template <> struct Quad<float> {
    template <int AUX = 0>
    __device__ static void load(rsrc_t r, int off, float (&v)[4]) {
        const u32x4 q = __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, AUX);
        // (not __builtin_bit_cast on q.y: clang reads element 0 for a bit_cast of a vector
        //  element lvalue)
        v[0] = __uint_as_float(q.x); v[1] = __uint_as_float(q.y);
        v[2] = __uint_as_float(q.z); v[3] = __uint_as_float(q.w);
    }
    __device__ static void store(const float (&v)[4], rsrc_t r, int off) {
        const u32x4 q = {__float_as_uint(v[0]), __float_as_uint(v[1]), __float_as_uint(v[2]),
                         __float_as_uint(v[3])};
        __builtin_amdgcn_raw_buffer_store_b128(q, r, off, 0, GF_OUT_AUX);
    }
};
template <> struct Quad<uint16_t> {
    template <int AUX = 0>
    __device__ static void load(rsrc_t r, int off, float (&v)[4]) {
        const u32x2 q = __builtin_amdgcn_raw_buffer_load_b64(r, off, 0, AUX);
        v[0] = (float)(q.x & 0xffffu); v[1] = (float)(q.x >> 16);
        v[2] = (float)(q.y & 0xffffu); v[3] = (float)(q.y >> 16);
    }
    __device__ static void load(rsrc_t r, int off, int (&v)[4]) {
        const u32x2 q = __builtin_amdgcn_raw_buffer_load_b64(r, off, 0, 0);
        v[0] = (int)(q.x & 0xffffu); v[1] = (int)(q.x >> 16);
        v[2] = (int)(q.y & 0xffffu); v[3] = (int)(q.y >> 16);
    }
    __device__ static void store(const float (&v)[4], rsrc_t r, int off) {
        const uint32_t a = (uint32_t)from_f32<uint16_t>(v[0]) | ((uint32_t)from_f32<uint16_t>(v[1]) << 16);
        const uint32_t b = (uint32_t)from_f32<uint16_t>(v[2]) | ((uint32_t)from_f32<uint16_t>(v[3]) << 16);
        __builtin_amdgcn_raw_buffer_store_b64((u32x2){a, b}, r, off, 0, 2);
    }
};
template <> struct Quad<uint8_t> {
    template <int AUX = 0>
    __device__ static void load(rsrc_t r, int off, float (&v)[4]) {
        const uint32_t q = __builtin_amdgcn_raw_buffer_load_b32(r, off, 0, AUX);
        v[0] = (float)(q & 0xffu); v[1] = (float)((q >> 8) & 0xffu);
        v[2] = (float)((q >> 16) & 0xffu); v[3] = (float)(q >> 24);
    }
    __device__ static void load(rsrc_t r, int off, int (&v)[4]) {
        const uint32_t q = __builtin_amdgcn_raw_buffer_load_b32(r, off, 0, 0);
        v[0] = (int)(q & 0xffu); v[1] = (int)((q >> 8) & 0xffu);
        v[2] = (int)((q >> 16) & 0xffu); v[3] = (int)(q >> 24);
    }
    __device__ static void store(const float (&v)[4], rsrc_t r, int off) {
        const uint32_t a = (uint32_t)from_f32<uint8_t>(v[0]) | ((uint32_t)from_f32<uint8_t>(v[1]) << 8) |
                           ((uint32_t)from_f32<uint8_t>(v[2]) << 16) | ((uint32_t)from_f32<uint8_t>(v[3]) << 24);
        __builtin_amdgcn_raw_buffer_store_b32(a, r, off, 0, 2);
    }
};

// Hide a value from the optimiser: keeps `ok ? off : kBadOff` a v_cndmask feeding one
// unconditional buffer access (otherwise the select becomes an exec-masked branch around two
// accesses, and the compiler's vmcnt accounting across the branch drains the loads in flight).
__device__ __forceinline__ int opaque(int v) {
    __asm__ volatile("" : "+v"(v));
    return v;
}

// A quad whose elements may lie partly outside the domain (edge tiles): element e is read at
// off + e*size when bit e of mask is set, else reads 0 (kBadOff). Interior tiles use Quad::load.
template <typename T>
__device__ __forceinline__ void load_quad_masked(rsrc_t r, int off, int mask, float (&v)[4]) {
#pragma unroll
    for (int e = 0; e < 4; ++e)
        v[e] = Buf<T>::load(r, (mask >> e) & 1 ? off + e * (int)sizeof(T) : kBadOff);
}
template <typename T>
__device__ __forceinline__ void load_quad_masked(rsrc_t r, int off, int mask, int (&v)[4]) {
#pragma unroll
    for (int e = 0; e < 4; ++e)
        v[e] = Buf<T>::load_int(r, (mask >> e) & 1 ? off + e * (int)sizeof(T) : kBadOff);
}
template <typename T>
__device__ __forceinline__ void store_quad_masked(const float (&v)[4], rsrc_t r, int off, int mask) {
#pragma unroll
    for (int e = 0; e < 4; ++e)
        Buf<T>::store(from_f32<T>(v[e]), r, (mask >> e) & 1 ? off + e * (int)sizeof(T) : kBadOff);
}

// ---------------------------------------------------------------------------------------------
// The fused kernel.
//
// Software-pipelined phases, two LDS barriers per z-step. Iteration `i` runs
//   C0: P3(i)  [U -> a,b on the E1 apron]  +  P1(i+1) [z-window of v]  +  P5(i-1) [y-sums,
//       z-blocks, out(i-1-R) -> Lout]
//   C1: P4(i)  [x-sums of (a,b)]  +  P2(i+1) [x-sums of the v z-window]  +  staging: Lout ->
//       global (16-B stores), v of slice i+1 -> Lc (P3's input), v of slice i-R -> Lv5 (P5's)
// with separate LDS buffers per hand-off, so each barrier interval holds independent work from
// different slices. Every global access is a 16-byte-per-lane quad (4 consecutive x) in
// interior tiles: the kernel is bound by vector-memory instruction issue otherwise (one dword
// per lane cost about as much as the whole pointwise stage).
// ---------------------------------------------------------------------------------------------
template <int R, int TY, int NT, int HXB = 8>
struct GFConfig {
    static constexpr int TX = 64;
    static constexpr int W = 2 * R + 1;
    static constexpr int HXB_ = HXB;  // bytes per Hx element
    static constexpr int E2X = TX + 4 * R, E2Y = TY + 4 * R;  // v / Zv apron
    static constexpr int E1X = TX + 2 * R, E1Y = TY + 2 * R;  // u / a / b apron
    // Pitches in 8-byte elements, = 2 mod 4: 16-B aligned rows and conflict-free ds_*_b128
    // when lanes walk rows (16-lane groups land on distinct 4-bank slots).
    static constexpr int p2m4(int x) { return x + ((2 - x % 4) + 4) % 4; }
    // Hx (f64, or int32 for 8/16-bit integer inputs; HXB bytes): P12 writes rows, P3 reads
    // columns. 4-byte rows: pitch a multiple of 4 (16-byte aligned rows) and not of 8.
    static constexpr int ph4(int x) { return (x + 3) / 4 * 4 + ((x + 3) / 4 * 4 % 8 == 0 ? 4 : 0); }
    static constexpr int PH = HXB == 8 ? p2m4(E1X) : ph4(E1X);
    static constexpr int PA = p2m4(E1X);  // Lab (float2) P3 writes, P4 reads rows
    static constexpr int PB = p2m4(TX);   // Hab (float2) P4 writes rows, P5 reads columns
    // r = 4 (the headline radius, 64 x 32 tiles): 8 outputs per P4 item and P4 issued ahead of
    // P12 in C1 (each -2 % at 2048^3, tools/timek.sh); other radii keep the defaults (unmeasured)
    static constexpr bool R4 = R == 4 && TY == 32 && NT == 1024;
    static constexpr int K3 = GF_K3, K4 = R4 ? GF_K4_R4 : GF_K4;
    static constexpr int ORDER = R4 ? GF_ORDER_R4 : GF_ORDER;
    static constexpr int K5 = TX * TY / NT;          // outputs per thread (ring width)
    static constexpr int S3 = (E1Y + K3 - 1) / K3;   // segments per column, P3
    static constexpr int S4 = TX / K4;               // segments per row, P4
    static constexpr int N3 = E1X * S3, N4 = E1Y * S4;  // work items
    // P12: one lane per quad (4 consecutive x) of an E2 row, whole rows per wave, so the
    // x-neighbour quads of the window sums come from adjacent lanes (DPP), never across waves
    static constexpr int QPL = 1;  // quads per lane
    static constexpr int EPL = 4 * QPL;                    // elements per lane
    static constexpr int NQ1X = E2X / EPL;                 // lanes per E2 row
    static constexpr int RPW = 64 / NQ1X;                  // E2 rows per wave
    static constexpr int NWAVE = NT / 64;
    static constexpr int NQP1 = (E2Y + RPW * NWAVE - 1) / (RPW * NWAVE);  // passes
    // single pass: P12 rows on the top waves (P4 works on the bottom ones)
    static constexpr int W12 = NQP1 == 1 ? NWAVE - (E2Y + RPW - 1) / RPW : 0;
    static constexpr int NB = (R + EPL - 1) / EPL;         // neighbour lanes on each side
    // P1 ring: the last W entering stage-1 quads of a lane held in registers, so the leaving
    // slice of the running z-window is never re-read (W * NQP1 * 4 VGPRs: 20 at r = 2, where the
    // 64 x 32 tile leaves ~40 free; at r = 4 the kernel has 5 to spare, so it re-reads)
    static constexpr bool P1RING = R <= GF_P1RING_MAXR;
    static constexpr int NQ5 = TX / 4 * TY;                  // output tile quads
    static constexpr int W3 = W * W * W;                     // interior window count
    static constexpr int al(int b) { return (b + 255) / 256 * 256; }
    static constexpr int SZ_HX = al((E2Y + K3) * PH * HXB);
    static constexpr int SZ_LAB = al((E1Y + 1) * PA * 8);
    static constexpr int SZ_HAB = al((E1Y + 1) * PB * 8);
    static constexpr int SZ_RCP = al((W3 + 1) * 4);  // RN(1/c) for window counts c <= W^3
    static constexpr int OFF_HX = 0, OFF_LAB = OFF_HX + SZ_HX;
    static constexpr int OFF_HAB = OFF_LAB + SZ_LAB;
    static constexpr int OFF_RCP = OFF_HAB + SZ_HAB;
    static constexpr int LDS_BYTES = OFF_RCP + SZ_RCP;
    // item -> thread placement: heavy phases on different waves (see C0 / C1)
    static constexpr int T3 = NT - N3;  // first thread of the P3 items (the top N3 threads)
    static_assert(TX * TY % NT == 0, "tile must divide evenly over the threads");
    static_assert(TY % K5 == 0, "ring segment must divide the tile height");
    static_assert(TX % K4 == 0, "P4 segment must divide the tile width");
    static_assert(N3 <= NT && N4 <= NT, "one work item per thread per phase");
    static_assert(RPW >= 1, "an E2 row fits one wave");
    static_assert(E2X % 4 == 0, "E2 rows are whole quads");
    static_assert(E2X % EPL == 0, "E2 rows are whole lane items");
    static_assert(LDS_BYTES <= 160 * 1024, "LDS budget");
};

// MODE 0 (interior): the tiles [itx0, itx1) x [ity0, ity1) whose whole apron lies inside the
//   domain and whose output tile lies inside the output box: unmasked 16-byte accesses, and the
//   window counts depend on z only, so they are computed once per step (wave-uniform) and P3 / P5
//   carry no per-lane count or zeroing logic and no branch.
// MODE 1 (quad): every tile of a quad-aligned geometry (each 4-element quad of a global access
//   wholly inside or wholly outside the domain / output box): unmasked accesses, the outside
//   quads through kBadOff, per-lane clamped counts and zeroing (one grid: see launch_fused_cfg).
// MODE 2 (edge): the border tiles otherwise: element-wise masked accesses. Its grid covers all
//   tiles; the interior ones (mode 0's) return at once. Separate kernels
// rather than runtime branches keep each march free of control flow around its memory
// instructions, so the compiler's vmcnt accounting stays exact (a branch there made it drain
// every load).
template <int R, int TY, int NT, typename TIn, typename TOut, int MODE>
__global__ __launch_bounds__(NT) void gf3d_fused_kernel(GFParams p) {
    using C = GFConfig<R, TY, NT, S1<TIn>::HXB>;
    using SA = typename S1<TIn>::acc;  // stage-1 window sums (exact)
    using SI = typename S1<TIn>::in;   // loaded stage-1 values
    constexpr bool EDGE = MODE == 2, INTERIOR = MODE == 0;
    constexpr int TX = C::TX, W = C::W;
    constexpr int K5 = C::K5;
    constexpr int ESZ = (int)sizeof(TIn), OSZ = (int)sizeof(TOut);
    extern __shared__ __attribute__((aligned(16))) char smem[];
    SA* const Hx = reinterpret_cast<SA*>(smem + C::OFF_HX);
    float2* const Lab = reinterpret_cast<float2*>(smem + C::OFF_LAB);
    float2* const Hab = reinterpret_cast<float2*>(smem + C::OFF_HAB);
    float* const rcp_tab = reinterpret_cast<float*>(smem + C::OFF_RCP);
    // Correctly rounded reciprocals of every possible window count, for div_by_count
    // (Markstein's correction needs RN(1/c) exactly). Published by the prologue's barrier.
    for (int c = threadIdx.x; c <= C::W3; c += NT) rcp_tab[c] = c > 0 ? 1.0f / (float)c : 0.0f;

    // XCD-aware block -> tile. Blocks b and b+8 share an XCD; give each XCD a contiguous run of
    // logical ids and walk them in GF_STX x GF_STY-tile super-tiles, so the WGs resident on one
    // XCD cover a compact region whose xy aprons and z reloads stay in that XCD's 4 MB L2.
    const int nwg = gridDim.x;
    const int b = blockIdx.x;
    const int lid = (nwg % 8 == 0) ? (b % 8) * (nwg / 8) + b / 8 : b;
    const int gtx = INTERIOR ? p.itx1 - p.itx0 : p.tiles_x;  // this launch's tile grid
    const int gty = INTERIOR ? p.ity1 - p.ity0 : p.tiles_y;
    const int ntiles = gtx * gty;
    const int seg = lid / ntiles;
    int t = lid % ntiles;
    int tile_x, tile_y;
    {
        const int stx = GF_STX, sty = GF_STY;
        const int full_y = gty / sty * sty;
        const int per_srow = gtx * sty;
        if (t < full_y * gtx) {
            const int sr = t / per_srow, r = t % per_srow;
            const int full_x = gtx / stx * stx;
            if (r < full_x * sty) {
                tile_x = (r / (stx * sty)) * stx + r % stx;
                tile_y = sr * sty + (r / stx) % sty;
            } else {
                const int rr = r - full_x * sty, w = gtx - full_x;
                tile_x = full_x + rr % w;
                tile_y = sr * sty + rr / w;
            }
        } else {
            t -= full_y * gtx;
            tile_x = t % gtx;
            tile_y = full_y + t / gtx;
        }
    }
    if constexpr (INTERIOR) {
        tile_x += p.itx0;
        tile_y += p.ity0;
    } else {
        if (tile_x >= p.itx0 && tile_x < p.itx1 && tile_y >= p.ity0 && tile_y < p.ity1) return;
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
    // Planes outside [zlo, zhi) (outside the domain, or outside a slab's rows) read as 0: a slab
    // carries the 2r halo of its output rows, so they only feed steps that emit nothing.
    const int zlo = p.zlo, zspan = p.zhi - p.zlo;
    auto slice_rsrc = [&](int z) -> rsrc_t {
        const bool ok = (unsigned)(z - zlo) < (unsigned)zspan;
        const char* base = in_base + (ok ? (int64_t)(z - p.in_z0) * p.in_sz * ESZ : 0);
        return make_rsrc(base, ok ? slice_bytes : 0u);
    };

    const int zc_begin = zo_begin - R, zc_end = zo_end + R;  // stage-1 slices of this march

    // ---- per-thread, step-invariant quad offsets and in-domain masks -----------------------
    const int tid0 = threadIdx.x;
    constexpr int EPL = C::EPL;
    int q1off[C::NQP1], q1mask[C::NQP1];
    // P12 lane -> (E2 row, lane item = 4 consecutive x) for pass k
    auto p12_pos = [&](int tid, int k, int& row, int& cq) -> bool {
        const int w = tid / 64 - C::W12, l = tid % 64;
        row = (k * C::NWAVE + w) * C::RPW + l / C::NQ1X;
        cq = l % C::NQ1X;
        return w >= 0 && l < C::RPW * C::NQ1X && row < C::E2Y;
    };
#pragma unroll
    for (int k = 0; k < C::NQP1; ++k) {
        int row, cq;
        const bool valid = p12_pos(tid0, k, row, cq);
        const int gx = x0 - 2 * R + EPL * cq, gy = y0 - 2 * R + row;
        int m = 0;
        if (valid && gy >= 0 && gy < ny) {
#pragma unroll
            for (int e = 0; e < 4; ++e) m |= (gx + e >= 0 && gx + e < nx) ? (1 << e) : 0;
        }
        q1mask[k] = m;
        q1off[k] = (EDGE ? valid : m == 0xF) ? (gy * sy + gx) * ESZ : kBadOff;
    }
    auto load_quad = [&](rsrc_t r, int off, int mask, SI (&v)[4]) {
        if constexpr (EDGE) load_quad_masked<TIn>(r, off, mask, v);
        else Quad<TIn>::load(r, off, v);
    };

    SA zv[C::NQP1][EPL];
#pragma unroll
    for (int k = 0; k < C::NQP1; ++k)
#pragma unroll
        for (int e = 0; e < EPL; ++e) zv[k][e] = (SA)0;
    // Running z-window: seed Zv(zc_begin - 1) = sum of v over [zc_begin-1-R, zc_begin-1+R]
    // clamped to [0, nz); every later step adds the entering and subtracts the leaving slice
    // (both 0 outside the domain), so the window stays exact through out-of-domain steps.
    // With the P1 ring, P12(c) (entering slice c+R, leaving c-R-1) uses slot
    // (c - zc_begin + W - 1) % W: the prologue's P12(zc_begin) slot W-1, the march's P12(i+1) of
    // unrolled step k slot k. Seed slice zc_begin-1-R+j entered as P12(zc_begin-1-2R+j): slot
    // (j + W - 1) % W.
    SI ring1[C::P1RING ? W : 1][C::NQP1][EPL];
    if constexpr (C::P1RING) {
        static_for<0, W>([&](auto jc) {
            constexpr int j = decltype(jc)::value;
            const rsrc_t rs = slice_rsrc(zc_begin - 1 - R + j);  // 0 outside [zlo, zhi)
#pragma unroll
            for (int k = 0; k < C::NQP1; ++k) {
                SI v[4];
                load_quad(rs, q1off[k], q1mask[k], v);
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    ring1[(j + W - 1) % W][k][e] = v[e];
                    zv[k][e] += (SA)v[e];
                }
            }
        });
    } else {
        const int za = max(zc_begin - 1 - R, 0), zb_ = min(zc_begin - 1 + R, nz - 1);
        for (int z = za; z <= zb_; ++z) {
            const rsrc_t rs = slice_rsrc(z);
#pragma unroll
            for (int k = 0; k < C::NQP1; ++k) {
                SI v[4];
                load_quad(rs, q1off[k], q1mask[k], v);
#pragma unroll
                for (int e = 0; e < 4; ++e) zv[k][e] += (SA)v[e];
            }
        }
    }

    f2 ring[W][K5], pre[K5];  // stage-2 z blocks (see do_p5)
#pragma unroll
    for (int s = 0; s < W; ++s)
#pragma unroll
        for (int j = 0; j < K5; ++j) ring[s][j] = (f2){0.0f, 0.0f};
#pragma unroll
    for (int j = 0; j < K5; ++j) pre[j] = (f2){0.0f, 0.0f};

    // ---- phase bodies ----------------------------------------------------------------------
    // P1 inputs of the next PF stage-1 slices (prefetched PF steps ahead; buffer b feeds the P12
    // of the unrolled steps k with k % PF == b)
    // Two steps ahead at r = 4 and r <= 2 (profiles/r05_p1_prefetch2*.txt: r = 4 f32 -5 % on a
    // box where the march took 30 ms, neutral on a 28.7 ms box, u16 -1 to -3 %; r = 1, 2 -1 to
    // -3.6 %); one step elsewhere (r = 3 / 5 measured +0.5-0.9 %; r > 5 and the masked edge mode
    // spill the second buffer).
    constexpr int PF = EDGE ? 1 : R == 4 ? GF_P1PFD : R <= 2 ? GF_P1PFD_R2 : 1;
    SI pa[PF][C::NQP1][EPL], ps[PF][C::NQP1][EPL];
    float vc[C::K3];  // v of the next P3 slice at this thread's item (prefetched)
    float v5[K5];     // v of the next P5 output slice at this thread's outputs
#pragma unroll
    for (int j = 0; j < K5; ++j) v5[j] = 0.0f;
    auto load_p1 = [&](auto bc, rsrc_t ra, rsrc_t rs) {  // entering zc+R, leaving zc-R-1
        constexpr int b = decltype(bc)::value;
#pragma unroll
        for (int k = 0; k < C::NQP1; ++k) {
            SI a4[4], s4[4];
            load_quad(ra, q1off[k], q1mask[k], a4);
            if constexpr (!C::P1RING) load_quad(rs, q1off[k], q1mask[k], s4);
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                pa[b][k][e] = a4[e];
                if constexpr (!C::P1RING) ps[b][k][e] = s4[e];
            }
        }
    };
    // P12: z-window of v (f64, running) and its x-window sums on the E2 apron -> Hx. The x
    // neighbours come from the adjacent lanes' quads by DPP wave shifts (whole rows per wave),
    // so the z-window never goes through LDS.
    auto do_p12 = [&](int tid, auto slotc, auto bc) {
        constexpr int sl = decltype(slotc)::value;  // P1 ring slot of this step
        constexpr int b = decltype(bc)::value;      // prefetch buffer of this step
#pragma unroll
        for (int k = 0; k < C::NQP1; ++k) {
            int row, cq;
            const bool valid = p12_pos(tid, k, row, cq);
#pragma unroll
            for (int e = 0; e < EPL; ++e) {
                zv[k][e] = zv[k][e] + (SA)pa[b][k][e];  // entering slice (0 outside the domain)
                if constexpr (C::P1RING) {
                    zv[k][e] = zv[k][e] - (SA)ring1[sl][k][e];  // leaving slice, from the ring
                    ring1[sl][k][e] = pa[b][k][e];
                } else {
                    zv[k][e] = zv[k][e] - (SA)ps[b][k][e];  // leaving slice (0 outside the domain)
                }
            }
            constexpr int NB = C::NB;
            SA win[EPL * (2 * NB + 1)];  // lane items cq-NB .. cq+NB
#pragma unroll
            for (int e = 0; e < EPL; ++e) win[EPL * NB + e] = zv[k][e];
            // only the R elements next to the own item are read (the others' moves are dead)
#pragma unroll
            for (int n = 1; n <= NB; ++n)
#pragma unroll
                for (int e = 0; e < EPL; ++e) {
                    win[EPL * (NB - n) + e] = dpp_from_lower(win[EPL * (NB - n + 1) + e]);
                    win[EPL * (NB + n) + e] = dpp_from_upper(win[EPL * (NB + n - 1) + e]);
                }
            SA vin[EPL + 2 * R], hs[EPL];
#pragma unroll
            for (int j = 0; j < EPL + 2 * R; ++j) vin[j] = win[EPL * NB - R + j];
            slide_sums_exact<R, EPL>(vin, hs);
            if constexpr (C::HXB_ == 4 && R % 4 == 0) {
                // int32 rows: the item's 4 outputs are one 16-byte aligned quad of Hx
                const int col4 = EPL * cq - R;
                if (valid && col4 >= 0 && col4 + 3 < C::E1X)
                    *reinterpret_cast<int4*>(Hx + row * C::PH + col4) =
                        make_int4(hs[0], hs[1], hs[2], hs[3]);
            } else if constexpr (C::HXB_ == 4 && R % 2 == 0) {
#pragma unroll
                for (int h = 0; h < EPL / 2; ++h) {
                    const int colh = EPL * cq + 2 * h - R;
                    if (valid && colh >= 0 && colh + 1 < C::E1X)
                        *reinterpret_cast<int2*>(Hx + row * C::PH + colh) =
                            make_int2(hs[2 * h], hs[2 * h + 1]);
                }
            } else if constexpr (C::HXB_ == 8 && GF_HX_B128 && R % 2 == 0) {
                // even R: the item's outputs land on 16-byte aligned column pairs of Hx (E1X and
                // the pitch are even): b128 writes (b64 writes of lanes 32 B apart conflict)
#pragma unroll
                for (int h = 0; h < EPL / 2; ++h) {
                    const int colh = EPL * cq + 2 * h - R;
                    if (valid && colh >= 0 && colh + 1 < C::E1X)
                        *reinterpret_cast<double2*>(Hx + row * C::PH + colh) =
                            make_double2(hs[2 * h], hs[2 * h + 1]);
                }
            } else {
#pragma unroll
                for (int e = 0; e < EPL; ++e) {
                    const int col = EPL * cq + e - R;  // Hx column (x - (x0 - R))
                    if (valid && col >= 0 && col < C::E1X) Hx[row * C::PH + col] = hs[e];
                }
            }
        }
    };
    // Pointwise stage on NP pairs of E1 positions, packed (both lanes of every op in one issue):
    //   u = RN(RN(U) / c)   (summed_area_table_mean, exact: Markstein with rcp = RN(1/c))
    //   s = (v - u)^2;  a = s / (s + eps);  b = (1 - a) * u          (guided_filter.rs:126-137)
    constexpr int NP3 = C::K3 / 2;
    auto pointwise = [&](const f2 (&Uf)[NP3], const f2 (&v)[NP3], const f2 (&fc)[NP3],
                         const f2 (&rc)[NP3], f2 (&a)[NP3], f2 (&bb)[NP3]) {
        f2 q[NP3], r[NP3], u[NP3], sq[NP3], den[NP3], y[NP3], e[NP3];
#pragma unroll
        for (int k = 0; k < NP3; ++k) q[k] = Uf[k] * rc[k];
#pragma unroll
        for (int k = 0; k < NP3; ++k) r[k] = pk_fma(-q[k], fc[k], Uf[k]);
#pragma unroll
        for (int k = 0; k < NP3; ++k) u[k] = pk_fma(r[k], rc[k], q[k]);
#pragma unroll
        for (int k = 0; k < NP3; ++k) sq[k] = v[k] - u[k];
#pragma unroll
        for (int k = 0; k < NP3; ++k) sq[k] = sq[k] * sq[k];  // (v - u).powf(2.0)
#pragma unroll
        for (int k = 0; k < NP3; ++k) den[k] = sq[k] + (f2){eps, eps};
#pragma unroll
        for (int k = 0; k < NP3; ++k)
            y[k] = (f2){__builtin_amdgcn_rcpf(den[k].x), __builtin_amdgcn_rcpf(den[k].y)};
        // a = s / (s + eps): Markstein's correction on v_rcp_f32 (within 1 ulp)
#pragma unroll
        for (int k = 0; k < NP3; ++k) q[k] = sq[k] * y[k];
#pragma unroll
        for (int k = 0; k < NP3; ++k) r[k] = pk_fma(-den[k], q[k], sq[k]);
#pragma unroll
        for (int k = 0; k < NP3; ++k) a[k] = pk_fma(r[k], y[k], q[k]);
#pragma unroll
        for (int k = 0; k < NP3; ++k) e[k] = (f2){1.0f, 1.0f} - a[k];
#pragma unroll
        for (int k = 0; k < NP3; ++k) bb[k] = e[k] * u[k];
    };
    static_assert(C::K3 % 2 == 0, "P3 works on pairs");
    // every P3 segment lies inside the apron: unconditional Lab stores (a guard lets the compiler
    // sink the second pair's pointwise chain into it, serialising the pairs)
    constexpr bool kRowsWhole = C::E1Y % C::K3 == 0;
    auto p3_load = [&](int tid, SA (&vin)[C::K3 + 2 * R]) {  // P3's Hx column segment
        const int item = tid - C::T3;
        if (item < 0) return;
        const int col = item % C::E1X, sg = item / C::E1X;
        const SA* src = Hx + (sg * C::K3) * C::PH + col;
#pragma unroll
        for (int j = 0; j < C::K3 + 2 * R; ++j) vin[j] = src[j * C::PH];
    };
    auto do_p3 = [&](int tid, int zc, const SA (&vin)[C::K3 + 2 * R]) {
        // y-window (f64) of Hx -> U; a, b -> Lab
        const int item = tid - C::T3;
        if (item < 0) return;
        const int col = item % C::E1X, sg = item / C::E1X;
        SA U[C::K3];
        slide_sums_exact<R, C::K3>(vin, U);
        f2* lab = reinterpret_cast<f2*>(Lab);
        f2 Uf[NP3], vv[NP3], fc[NP3], rc[NP3], a[NP3], bb[NP3];
#pragma unroll
        for (int k = 0; k < NP3; ++k) {
            Uf[k] = (f2){(float)U[2 * k], (float)U[2 * k + 1]};
            vv[k] = (f2){vc[2 * k], vc[2 * k + 1]};  // v of slice zc, loaded a half-step ago
        }
        if constexpr (INTERIOR) {
            // every E1 point of the tile has the full x and y windows: count = W^2 * cz(zc)
            // (wave-uniform); planes outside the domain hold no (a, b)
            const bool zin = (unsigned)zc < (unsigned)nz;
            const int cnt = W * W * clamped_count(min(max(zc, 0), nz - 1), nz, R);
            const float fcs = (float)cnt, rcs = rcp_tab[cnt];
#pragma unroll
            for (int k = 0; k < NP3; ++k) {
                fc[k] = (f2){fcs, fcs};
                rc[k] = (f2){rcs, rcs};
            }
            pointwise(Uf, vv, fc, rc, a, bb);
#pragma unroll
            for (int k = 0; k < NP3; ++k) {
                const int ey = sg * C::K3 + 2 * k;
                const f2 ab0 = zin ? __builtin_shufflevector(a[k], bb[k], 0, 2) : (f2){0.f, 0.f};
                const f2 ab1 = zin ? __builtin_shufflevector(a[k], bb[k], 1, 3) : (f2){0.f, 0.f};
                if (kRowsWhole || ey < C::E1Y) lab[ey * C::PA + col] = ab0;
                if (kRowsWhole || ey + 1 < C::E1Y) lab[(ey + 1) * C::PA + col] = ab1;
            }
        } else {
            const int gx = x0 - R + col;
            const bool xzin = gx >= 0 && gx < nx && zc >= 0 && zc < nz;
            const int cxz = cmul(clamped_count(gx, nx, R), clamped_count(zc, nz, R));
#pragma unroll
            for (int k = 0; k < NP3; ++k) {
                const int gy = y0 - R + sg * C::K3 + 2 * k;
                const int c0 = cmul(clamped_count(gy, ny, R), cxz), c1 = cmul(clamped_count(gy + 1, ny, R), cxz);
                fc[k] = (f2){(float)c0, (float)c1};
                rc[k] = (f2){rcp_tab[c0], rcp_tab[c1]};
            }
            pointwise(Uf, vv, fc, rc, a, bb);
#pragma unroll
            for (int k = 0; k < NP3; ++k) {
                const int ey = sg * C::K3 + 2 * k;
                const int gy = y0 - R + ey;
                // zero outside the domain: the clamped window sums of stage 2
                const bool ok0 = xzin && gy >= 0 && gy < ny, ok1 = xzin && gy + 1 >= 0 && gy + 1 < ny;
                if (kRowsWhole || ey < C::E1Y) lab[ey * C::PA + col] = ok0 ? (f2){a[k].x, bb[k].x} : (f2){0.f, 0.f};
                if (kRowsWhole || ey + 1 < C::E1Y)
                    lab[(ey + 1) * C::PA + col] = ok1 ? (f2){a[k].y, bb[k].y} : (f2){0.f, 0.f};
            }
        }
    };
    auto do_p4 = [&](int tid) {  // x-window sums of (a, b) rows -> Hab
        const int item = tid;
#if GF_WAVE_SKIP
        // whole waves past the items branch around the phase (scalar test): exec-masked they
        // would still spend their issue slots on it
        if (__builtin_amdgcn_readfirstlane(tid >> 6) * 64 >= C::N4) return;
#endif
        if (item >= C::N4) return;
        const int row = item % C::E1Y, sg = item / C::E1Y;
        const float4* src = reinterpret_cast<const float4*>(Lab + row * C::PA + sg * C::K4);
        f2 vin[C::K4 + 2 * R], vout[C::K4];
#pragma unroll
        for (int j = 0; j < (C::K4 + 2 * R) / 2; ++j) {
            const float4 f = src[j];
            vin[2 * j] = (f2){f.x, f.y};
            vin[2 * j + 1] = (f2){f.z, f.w};
        }
        if constexpr ((C::K4 + 2 * R) % 2) {
            const float2 t = Lab[row * C::PA + sg * C::K4 + C::K4 + 2 * R - 1];
            vin[C::K4 + 2 * R - 1] = (f2){t.x, t.y};
        }
        core_window_sums<R, C::K4>(vin, vout);
        float4* dst = reinterpret_cast<float4*>(Hab + row * C::PB + sg * C::K4);
#pragma unroll
        for (int j = 0; j < C::K4 / 2; ++j)
            dst[j] = make_float4(vout[2 * j].x, vout[2 * j].y, vout[2 * j + 1].x, vout[2 * j + 1].y);
    };
    // Stage-2 z-window by prefix/suffix sums over blocks of W slices (van Herk / Gil-Werman):
    // the march is unrolled by W, so the position P of a slice in its block is a compile-time
    // constant. ring[P] holds the raw slice sum of the current block until the block's last
    // slice, when it is turned into the suffix sum over [P, W) in place; a window ending at
    // position P of block B+1 is suffix_B(P+1) + prefix_{B+1}(P). ~3 packed adds per output
    // instead of an f64 running sum (10 ops).
    rsrc_t ro5;  // the output slice P5 stores to this step
    auto p5_load = [&](int tid, f2 (&vin)[K5 + 2 * R]) {  // P5's Hab column segment
        const int col5 = tid % TX, seg5 = tid / TX;
        const f2* src = reinterpret_cast<const f2*>(Hab) + (seg5 * K5) * C::PB + col5;
#pragma unroll
        for (int j = 0; j < K5 + 2 * R; ++j) vin[j] = src[j * C::PB];
    };
    auto do_p5 = [&](int tid, int zc, auto slot_c, const f2 (&vin)[K5 + 2 * R]) {
        // y-window -> slice sums; z; out -> global
        const int col5 = tid % TX, seg5 = tid / TX;
        f2 s2[K5];
        core_window_sums<R, K5>(vin, s2);
        constexpr int P = decltype(slot_c)::value;
        f2 AB[K5];
#pragma unroll
        for (int j = 0; j < K5; ++j) {
            pre[j] = (P == 0) ? s2[j] : pre[j] + s2[j];
            if constexpr (P == W - 1) AB[j] = pre[j];
            else AB[j] = ring[(P + 1) % W][j] + pre[j];
            ring[P][j] = s2[j];
        }
        if constexpr (P == W - 1) {
#pragma unroll
            for (int q = W - 2; q >= 0; --q)
#pragma unroll
                for (int j = 0; j < K5; ++j) ring[q][j] = ring[q][j] + ring[q + 1][j];
        }
        const int zo = zc - R;
        const int ox = x0 + col5, oyb = y0 + seg5 * K5;
        // steps that emit nothing run too, their stores dropped by the descriptor; the z count
        // is clamped so its table index stays valid there
        const int zq = min(max(zo, 0), nz - 1);
        f2 rc[K5];
        if constexpr (INTERIOR) {
            const float r = rcp_tab[W * W * clamped_count(zq, nz, R)];  // wave-uniform
#pragma unroll
            for (int j = 0; j < K5; ++j) rc[j] = (f2){r, r};
        } else {
            const int cxz = cmul(clamped_count(ox, nx, R), clamped_count(zq, nz, R));
#pragma unroll
            for (int j = 0; j < K5; ++j) {
                const float r = rcp_tab[cmul(clamped_count(oyb + j, ny, R), cxz)];
                rc[j] = (f2){r, r};
            }
        }
        // (sum as f32) * RN(1/count) for a and b together: the stage-2 means (one multiply; the
        // f32 sums already differ from the reference's f64 SAT sums by a few ulp)
#pragma unroll
        for (int j = 0; j < K5; ++j) {
            const f2 q = AB[j] * rc[j];
            const int oy = oyb + j;
            const float o = __fadd_rn(__fmul_rn(v5[j], q.x), q.y);  // v*=ma; v+=mb
            const int off = (ox < ox_end && oy < oy_end)
                                ? ((oy - p.oy0) * osy + (ox - p.ox0)) * OSZ : kBadOff;
            Buf<TOut>::store(from_f32<TOut>(o), ro5, opaque(off));
        }
    };

    // ---- v loaders: one element per access, lanes on consecutive x (coalesced rows) -------------
    // Every global access of the march below is unconditional, in the same order every step:
    // out-of-range slices, inactive lanes and non-emitting steps use null descriptors or
    // kBadOff instead of branches. Branches around memory instructions make the compiler's
    // vmcnt accounting fall back to draining the loads just issued (measured: a 1.6x slower
    // kernel); straight-line, it waits for exactly the step-old load it needs.
    // Positions outside the domain either read 0 through the range check or read a neighbour
    // row's value that is never used (P3 zeroes its out-of-domain (a, b); P5's store drops).
    auto load_p3v = [&](rsrc_t r) {
        const int item = (int)threadIdx.x - C::T3;
        const int col = item % C::E1X, sg = item / C::E1X;
        const int gx = x0 - R + col, gy0 = y0 - R + sg * C::K3;
#pragma unroll
        for (int k = 0; k < C::K3; ++k) {
            const int gy = gy0 + k;
            bool ok = item >= 0;
            if constexpr (EDGE) ok = ok && (unsigned)gx < (unsigned)nx && (unsigned)gy < (unsigned)ny;
            vc[k] = Buf<TIn>::load(r, opaque(ok ? (gy * sy + gx) * ESZ : kBadOff));
        }
    };
    auto load_p5v = [&](rsrc_t r) {
        const int col5 = (int)threadIdx.x % TX, seg5 = (int)threadIdx.x / TX;
        const int ox = x0 + col5, oyb = y0 + seg5 * K5;
#pragma unroll
        for (int j = 0; j < K5; ++j) {
            const int oy = oyb + j;
            const bool ok = ox < ox_end && oy < oy_end;
            v5[j] = Buf<TIn>::load(r, opaque(ok ? (oy * sy + ox) * ESZ : kBadOff));
        }
    };

    // ---- prologue: stage 1 of the first slice up to Hx; prefetch step 1 ---------------------
    using B0 = std::integral_constant<int, 0>;
    using BL = std::integral_constant<int, PF - 1>;
    load_p1(BL{}, slice_rsrc(zc_begin + R), slice_rsrc(zc_begin - R - 1));
    load_p3v(slice_rsrc(zc_begin));
    do_p12(tid0, std::integral_constant<int, W - 1>{}, BL{});
    load_p1(B0{}, slice_rsrc(zc_begin + 1 + R), slice_rsrc(zc_begin - R));
    if constexpr (PF == 2) load_p1(BL{}, slice_rsrc(zc_begin + 2 + R), slice_rsrc(zc_begin + 1 - R));
    lds_barrier();

    // ---- slice streams: descriptors advanced by one slice per step (two 32-bit adds each)
    //      instead of rebuilt from z (a 64-bit multiply and range checks per descriptor) ------
    // step i reads slice zb = i+1-R (leaving slice of P1(i+2), and v5), zb+R+1 = i+2 (P3's v)
    // and zb+2R+1 = i+2+R (entering slice of P1(i+2)); it stores output slice zs = i-1-R.
    const int64_t sstride = p.in_sz * ESZ, osstride = p.out_sz * OSZ;
    const int64_t off_a = (int64_t)(2 * R + 1) * sstride;
    int zb = zc_begin + 1 - R;
    int64_t ob = (int64_t)(zb - p.in_z0) * sstride;
    int zs = zc_begin - 1 - R;  // output slice of this step's P5
    int64_t os = (int64_t)(zs - p.oz0) * osstride;
    const char* out_base = static_cast<const char*>(p.out);
    const unsigned nzo = (unsigned)(zo_end - zo_begin);
    auto rs_in = [&](int64_t off, int z) {
        return make_rsrc(in_base + off, (unsigned)(z - zlo) < (unsigned)zspan ? slice_bytes : 0u);
    };

    // ---- pipelined march, unrolled by W so the ring slot of every P5 is a constant ----------
    // Iteration i runs
    //   C0: P3(i) [U -> a,b on the E1 apron] + P5(i-1) [y-sums, z-blocks, out(i-1-R)]
    //   C1: the loads of the next step, P12(i+1) [z-window of v, x-sums], P4(i) [x-sums of (a,b)]
    // with separate LDS buffers per hand-off, so each barrier interval holds independent work
    // from different slices. The step count is padded to a multiple of W, at least one past the
    // last stage-1 slice so that P5 / the store of the last output slice happen inside the loop:
    // no guards inside. Padded steps emit nothing (zo >= zo_end).
    constexpr int UN = PF * W;  // unrolled steps: every ring slot and prefetch buffer a constant
    const int n_steps = (zc_end - zc_begin + 1 + UN - 1) / UN * UN;
    for (int i0 = zc_begin; i0 < zc_begin + n_steps; i0 += UN) {
        static_for<0, UN>([&](auto kc) {
            constexpr int k = decltype(kc)::value;
            const int i = i0 + k;
            const int tid = threadIdx.x;
            const rsrc_t r_b = rs_in(ob, zb);
            ro5 = make_rsrc(out_base + os, (unsigned)(zs - zo_begin) < nzo ? oslice_bytes : 0u);
            // Fair progress across the waves of a SIMD: the hardware issues oldest-first, which
            // staggers the waves so the youngest runs its last phase alone, latency exposed. A
            // wave drops its priority as it completes a phase, so laggards catch up.
            if constexpr (GF_PRIO) __builtin_amdgcn_s_setprio(3);
            // C0: P3(i) + P5(i-1) (LDS and registers only). P5 runs unconditionally, so no
            // branch separates its stores from the loads waited on later (the first call's slice
            // lies in no emitted window, and its stores go to a zero-record descriptor)
            // (each phase's LDS reads issued right before its arithmetic: hoisting P5's, or both
            //  phases', ahead of P3 measured +1-4 %, profiles/r05_c0_hoist.txt)
            SA vin3[C::K3 + 2 * R];
            p3_load(tid, vin3);
            do_p3(tid, i, vin3);
            if constexpr (GF_PRIO) __builtin_amdgcn_s_setprio(1);
            f2 vin5[K5 + 2 * R];
            p5_load(tid, vin5);
            do_p5(tid, i - 1, std::integral_constant<int, (k + W - 1) % W>{}, vin5);
            lds_barrier();
            if constexpr (GF_PRIO) __builtin_amdgcn_s_setprio(3);
            // C1: the loads of the next step, P12(i+1), P4(i). Every wait here is for a load
            // issued a step ago.
            load_p3v(rs_in(ob + (int64_t)R * sstride, zb + R));  // P3 slice i+1
            load_p5v(rs_in(ob - sstride, zb - 1));                // P5 slice i-R
            if constexpr (C::ORDER & 2) do_p4(tid);
            using BK = std::integral_constant<int, k % PF>;
            do_p12(tid, std::integral_constant<int, k % W>{}, BK{});
            if constexpr (PF == 2)  // for P12(i+3): entering slice i+3+R, leaving i+2-R
                load_p1(BK{}, rs_in(ob + off_a + sstride, zb + 2 * R + 2), rs_in(ob + sstride, zb + 1));
            else
                load_p1(BK{}, rs_in(ob + off_a, zb + 2 * R + 1), r_b);
            if constexpr (GF_PRIO) __builtin_amdgcn_s_setprio(1);
            if constexpr (!(C::ORDER & 2)) do_p4(tid);
            lds_barrier();
            ++zb;
            ob += sstride;
            ++zs;
            os += osstride;
        });
    }
}

// ---------------------------------------------------------------------------------------------
// Launch: pick the tile configuration for the radius, dispatch dtypes.
// ---------------------------------------------------------------------------------------------
inline long long floor_div(long long a, long long b) { return a >= 0 ? a / b : -((-a + b - 1) / b); }
inline long long ceil_div(long long a, long long b) { return -floor_div(-a, b); }

// Interior tile range along one axis: tiles t with origin o0 + t*T such that the whole E2 apron
// [o0 + t*T - 2R, o0 + t*T + T + 2R + slack) is inside [0, n) and the output tile inside
// [o0, o_end). Returns [lo, hi) (empty when lo >= hi).
inline void interior_tiles(long long o0, long long o_end, long long n, int T, int R, int slack,
                           int ntiles, int& lo, int& hi) {
    long long l = ceil_div(2LL * R - o0, T);
    long long h = floor_div(std::min(n - 2LL * R - slack, o_end) - T - o0, T) + 1;
    l = std::max(l, 0LL);
    h = std::min(h, (long long)ntiles);
    if (h < l) h = l;
    lo = (int)l;
    hi = (int)h;
}

// > 64 KB of dynamic LDS needs the per-function opt-in, once per (kernel, device): a bit per
// device in a per-instantiation mask (one process may drive several devices).
template <typename K>
inline std::atomic<uint64_t>& attr_devices() {
    static std::atomic<uint64_t> mask{0};
    return mask;
}
inline hipError_t allow_dynamic_lds(const void* kern, int bytes, std::atomic<uint64_t>& mask) {
    int dev = 0;
    if (hipError_t e = hipGetDevice(&dev)) return e;
    const uint64_t bit = 1ull << (dev & 63);
    if (mask.load(std::memory_order_relaxed) & bit) return hipSuccess;
    if (hipError_t e = hipFuncSetAttribute(kern, hipFuncAttributeMaxDynamicSharedMemorySize, bytes))
        return e;
    mask.fetch_or(bit, std::memory_order_relaxed);
    return hipSuccess;
}

template <int R, int TY, int NT, typename TIn, typename TOut, int MODE>
inline hipError_t launch_fused_variant(const GFParams& p, long long nwg, hipStream_t stream) {
    using C = GFConfig<R, TY, NT, S1<TIn>::HXB>;
    const size_t lds = (size_t)C::LDS_BYTES;
    auto kern = gf3d_fused_kernel<R, TY, NT, TIn, TOut, MODE>;
    if (hipError_t e = allow_dynamic_lds((const void*)kern, (int)lds, attr_devices<decltype(kern)>()))
        return e;
    if (nwg <= 0) return hipSuccess;
    if (nwg > 0x7FFFFFFFLL) return hipErrorInvalidValue;
    hipLaunchKernelGGL(kern, dim3((unsigned)nwg), dim3(NT), lds, stream, p);
    return hipGetLastError();
}

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
    // Interior tiles (mode 0): the whole E2 apron inside the domain, the tile inside the output
    // box. Quad-aligned geometry (every quad starts at a multiple of 4 elements: the E2 apron at
    // x0 - 2R, the output tile at x0; the domain / output box widths multiples of 4): no quad
    // straddles a boundary, so the other tiles take the unmasked mode 1, else the masked mode 2.
    const bool quad_ok = (p.ox0 % 4 == 0) && (R % 2 == 0) && (p.nx % 4 == 0) &&
                         (p.onx % 4 == 0) && (p.in_sy % 4 == 0) && (p.in_sz % 4 == 0) &&
                         (p.out_sy % 4 == 0) && (p.out_sz % 4 == 0) &&
                         ((uintptr_t)p.in % (4 * sizeof(TIn)) == 0) &&
                         ((uintptr_t)p.out % (4 * sizeof(TOut)) == 0);
    const long long n_all = (long long)p.tiles_x * p.tiles_y;
    if (quad_ok) {
        // one grid, every tile in mode 1. Measured at 2048^3 r=4: 30.2 ms, against 35.2 ms for
        // mode 0 + a second grid of the border tiles (that grid's tail) and 30.4 ms for one grid
        // choosing the class per workgroup (both marches in one kernel: more SGPR spills); mode 0
        // alone over every tile (border output wrong, a bound only) 29.1 ms.
        p.itx0 = p.itx1 = p.ity0 = p.ity1 = 0;
        return launch_fused_variant<R, TY, NT, TIn, TOut, 1>(p, n_all * p.nseg, stream);
    }
    interior_tiles(p.ox0, p.ox0 + p.onx, p.nx, C::TX, R, 0, p.tiles_x, p.itx0, p.itx1);
    interior_tiles(p.oy0, p.oy0 + p.ony, p.ny, TY, R, 0, p.tiles_y, p.ity0, p.ity1);
    const long long n_int = (long long)(p.itx1 - p.itx0) * (p.ity1 - p.ity0);
    hipError_t e = hipSuccess;
    if (n_int > 0)
        e = launch_fused_variant<R, TY, NT, TIn, TOut, 0>(p, n_int * p.nseg, stream);
    if (e == hipSuccess && n_all > n_int)
        e = launch_fused_variant<R, TY, NT, TIn, TOut, 2>(p, n_all * p.nseg, stream);
    return e;
}

template <int R, int TY, int NT, typename TIn, typename TOut>
inline hipError_t launch_fused_auto(const GFParams& p, hipStream_t stream) {
    return launch_fused_cfg<R, TY, NT, TIn, TOut>(p, stream);
}

// Element-type pairs with a direct fused instantiation (the rest are staged through f32).
inline bool fused_fast_dtype(int d) { return d == kF32 || d == kU16 || d == kU8 || d == kBool; }

#define ZT_FUSED_PAIRS(R, TY, NT)                                                                 \
    hipError_t launch_fused_radius_##R(const GFParams& p, int din, int dout, hipStream_t s) {     \
        auto pick_out = [&](auto tin) -> hipError_t {                                             \
            using TI = decltype(tin);                                                             \
            switch (dout) {                                                                       \
            case kF32: return launch_fused_auto<R, TY, NT, TI, float>(p, s);                      \
            case kU16: return launch_fused_auto<R, TY, NT, TI, uint16_t>(p, s);                   \
            case kU8: case kBool: return launch_fused_auto<R, TY, NT, TI, uint8_t>(p, s);         \
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
