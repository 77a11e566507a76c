// tools/gf_fused_variants.hpp — the round-2 fused guided-filter kernel WITH its measured-slower variant switches (GF_ONEBAR, GF_OCT, ...) and ablation flags (ABL), kept for the A/B harnesses in tools/ (not a product path; the product kernel is zarrs_tools_amd/csrc/gf_fused.hpp).
// design notes). Instantiated per radius in gf_fused_r<R>.hip so the instantiations compile in
// parallel; guided_filter.hip dispatches.
#pragma once

#include <hip/hip_runtime.h>

#include <atomic>
#include <stdint.h>

#include <algorithm>
#include <type_traits>

#include "../zarrs_tools_amd/csrc/zt_device.hpp"
#include "../zarrs_tools_amd/csrc/zt_kernels.hpp"

#ifndef GF_T3_TOP
#define GF_T3_TOP 1
#endif
#ifndef GF_K4_R4
#define GF_K4_R4 8
#endif
#ifndef GF_ORDER_R4
#define GF_ORDER_R4 2
#endif
#ifndef GF_PRIO
#define GF_PRIO 1  // s_setprio phase reordering (measured -4.5% at 2048^3 r=4 with the b128 Hx writes)
#endif
#ifndef GF_ORDER
#define GF_ORDER 0
#endif
#ifndef GF_HX_B128
#define GF_HX_B128 1  // 16-byte Hx writes for even R (fewer LDS bank conflicts: -2% at r=4)
#endif
#ifndef GF_K3
#define GF_K3 4  // P3 outputs per thread (column segment of the f64 y-window)
#endif
#ifndef GF_K4
#define GF_K4 4  // P4 outputs per thread (row segment of the (a, b) x-window)
#endif
#ifndef GF_DIRECT
#define GF_DIRECT 1  // P3 / P5 load their v values and P5 stores its outputs directly (no Lc /
                     // Lv5 / Lout LDS staging)
#endif
#ifndef GF_ONEBAR
#define GF_ONEBAR 0  // (measured slower: 34.4 vs 32.6 ms) one barrier per z-step: every wave runs P12(i+1), P5(i-2), P3(i), P4(i-1)
                     // on double-buffered Hx / Lab / Hab (when they fit the LDS; needs GF_DIRECT)
#endif
#ifndef GF_OCT
#define GF_OCT 0  // 8 x per P12 lane: fewer instructions, but concentrated on half the waves
                  // (measured slower: 35.0 vs 31.7 ms)
#endif
#ifndef GF_P3_SPREAD
#define GF_P3_SPREAD 0  // measured slower (34.1 vs 31.8 ms): the extra issue outweighs the balance
#endif
#ifndef GF_V5_AUX
#define GF_V5_AUX 0  // cache policy of P5's v loads (the last read of an input slice)
#endif
#ifndef GF_LEAVE_AUX
#define GF_LEAVE_AUX 0  // cache policy of P1's leaving-slice loads
#endif
#ifndef GF_STX
#define GF_STX 4  // XCD super-tile: tiles along x (4 x 16 measured best: 31.2 vs 31.9 ms for 8 x 4)
#endif
#ifndef GF_STY
#define GF_STY 16  // XCD super-tile: tiles along y
#endif
#ifndef GF_WAVE_SKIP
#define GF_WAVE_SKIP 1  // P4: idle waves branch around the phase
#endif
#ifndef GF_NEWTON_A
#define GF_NEWTON_A 0  // a = s / (s + eps): Markstein's correction on v_rcp_f32 (<= 1 ulp) without
                       // the Newton step on the reciprocal (a enters only f32 window sums)
#endif
#ifndef GF_FASTDIV5
#define GF_FASTDIV5 1  // stage-2 means as sum * RN(1/count) (one multiply; the sums already
                       // differ from the reference's f64 SAT sums by a few ulp)
#endif
#ifndef GF_PW_SYNC
#define GF_PW_SYNC 0  // pointwise pairs advanced op by op (no s_nop between dependent v_pk_*)
#endif
#ifndef GF_TREE
#define GF_TREE 1  // f64 window sums as a balanced tree + independent differences (short chains)
#endif
#ifndef GF_A_RCP
#define GF_A_RCP 0  // a = s * rcp(s + eps) without Markstein's correction (<= 2 ulp)
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
template <int R, int K>
__device__ __forceinline__ void slide_sums_f64(const double (&in)[K + 2 * R], double (&out)[K]) {
    if constexpr (GF_TREE) {
        // exact sums: any association gives the same value, so the first window is a balanced
        // tree and each later one adds an independently formed difference (chain depth
        // log2(W) + K - 1 instead of 2R + 2(K - 1))
        double c[2 * R + 1];
#pragma unroll
        for (int j = 0; j <= 2 * R; ++j) c[j] = in[j];
#pragma unroll
        for (int w = 1; w <= 2 * R; w *= 2) {
#pragma unroll
            for (int j = 0; j + w <= 2 * R; j += 2 * w) c[j] = c[j] + c[j + w];
        }
        double d[K];
#pragma unroll
        for (int i = 1; i < K; ++i) d[i] = in[i + 2 * R] - in[i - 1];
        out[0] = c[0];
#pragma unroll
        for (int i = 1; i < K; ++i) out[i] = out[i - 1] + d[i];
    } else {
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
    __device__ static void store(uint16_t v, rsrc_t r, int off) {
        __builtin_amdgcn_raw_buffer_store_b16(v, r, off, 0, 2);
    }
};
template <> struct Buf<uint8_t> {
    template <int AUX = 0>
    __device__ static float load(rsrc_t r, int off) {
        return (float)(uint8_t)__builtin_amdgcn_raw_buffer_load_b8(r, off, 0, AUX);
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
template <int R, int TY, int NT>
struct GFConfig {
    static constexpr int TX = 64;
    static constexpr int W = 2 * R + 1;
    static constexpr int E2X = TX + 4 * R, E2Y = TY + 4 * R;  // v / Zv apron
    static constexpr int E1X = TX + 2 * R, E1Y = TY + 2 * R;  // u / a / b apron
    // Pitches in 8-byte elements, = 2 mod 4: 16-B aligned rows and conflict-free ds_*_b128
    // when lanes walk rows (16-lane groups land on distinct 4-bank slots).
    static constexpr int p2m4(int x) { return x + ((2 - x % 4) + 4) % 4; }
    static constexpr int PH = p2m4(E1X);  // Hx  (f64)    P12 writes rows, P3 reads columns
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
    // GF_OCT: 8 consecutive x per lane (two quads) where E2 rows are whole octets: half the
    // DPP moves and fewer sliding-sum adds per x-sum output
    static constexpr int QPL = (GF_OCT && E2X % 8 == 0 && R <= 8) ? 2 : 1;  // quads per lane
    static constexpr int EPL = 4 * QPL;                    // elements per lane
    static constexpr int NQ1X = E2X / EPL;                 // lanes per E2 row
    static constexpr int RPW = 64 / NQ1X;                  // E2 rows per wave
    static constexpr int NWAVE = NT / 64;
    static constexpr int NQP1 = (E2Y + RPW * NWAVE - 1) / (RPW * NWAVE);  // passes
    // single pass: P12 rows on the top waves (P4 works on the bottom ones)
    static constexpr int W12 = NQP1 == 1 ? NWAVE - (E2Y + RPW - 1) / RPW : 0;
    static constexpr int NB = (R + EPL - 1) / EPL;         // neighbour lanes on each side
    static constexpr int XC = R % 4;  // Lc quad grid starts XC elements left of the E1 apron
    static constexpr int NQCX = (E1X + XC + 3) / 4, NQC = NQCX * E1Y;  // Lc: the E1 apron
    static constexpr int PC = 4 * NQCX;                      // Lc pitch (floats)
    static constexpr int NQ5 = TX / 4 * TY;                  // v5 / output tile quads
    static constexpr int W3 = W * W * W;                     // interior window count
    static constexpr int al(int b) { return (b + 255) / 256 * 256; }
    static constexpr int SZ_HX = al((E2Y + K3) * PH * 8);
    static constexpr int SZ_LAB = al((E1Y + 1) * PA * 8);
    static constexpr int SZ_HAB = al((E1Y + 1) * PB * 8);
    static constexpr int SZ_LC = GF_DIRECT ? 0 : al(E1Y * PC * 4);
    static constexpr int SZ_T = GF_DIRECT ? 0 : al(TY * TX * 4);
    static constexpr int SZ_RCP = al((W3 + 1) * 4);  // RN(1/c) for window counts c <= W^3
    // single-barrier pipeline: Hx / Lab / Hab double-buffered by step parity, if they fit
    static constexpr bool ONEBAR = GF_ONEBAR && GF_DIRECT &&
                                   2 * (SZ_HX + SZ_LAB + SZ_HAB) + SZ_RCP + 256 <= 160 * 1024;
    static constexpr int NBUF = ONEBAR ? 2 : 1;
    static constexpr int OFF_HX = 0, OFF_LAB = OFF_HX + NBUF * SZ_HX;
    static constexpr int OFF_HAB = OFF_LAB + NBUF * SZ_LAB;
    static constexpr int OFF_LC = OFF_HAB + NBUF * SZ_HAB, OFF_LV5 = OFF_LC + SZ_LC;
    static constexpr int OFF_LOUT = OFF_LV5 + SZ_T, OFF_RCP = OFF_LOUT + SZ_T;
    static constexpr int OFF_DUMMY = OFF_RCP + SZ_RCP;  // 16-B sink for inactive lanes' writes
    static constexpr int LDS_BYTES = OFF_DUMMY + 256;
    // item -> thread placement: heavy phases on different waves (see C0 / C1)
    static constexpr int T3 = GF_T3_TOP ? NT - N3 : 0;  // first thread of the P3 items
    // (the bottom placement is not maintained: its P3 loads disagree with GF_DIRECT's item map)
    static_assert(GF_T3_TOP || !GF_DIRECT, "GF_T3_TOP=0 needs GF_DIRECT=0");
    static_assert(TX * TY % NT == 0, "tile must divide evenly over the threads");
    static_assert(TY % K5 == 0, "ring segment must divide the tile height");
    static_assert(TX % K4 == 0, "P4 segment must divide the tile width");
    static_assert(N3 <= NT && N4 <= NT, "one work item per thread per phase");
    static_assert(RPW >= 1, "an E2 row fits one wave");
    static_assert(GF_DIRECT || (NQC <= NT && NQ5 <= NT), "one staging quad per thread");
    static_assert(E2X % 4 == 0, "E2 rows are whole quads");
    static_assert(E2X % EPL == 0, "E2 rows are whole lane items");
    static_assert(LDS_BYTES <= 160 * 1024, "LDS budget");
};

// EDGE = false: the tiles [itx0, itx1) x [ity0, ity1), where every 4-element quad of a global
// access is either entirely inside the domain / output box or entirely outside (all tiles when
// the geometry is quad-aligned, else the interior tiles): unmasked 16-byte accesses, the
// outside quads through kBadOff. EDGE = true: every other tile (the grid covers all tiles;
// those of the first launch return at once), element-wise masked accesses. Two kernels rather
// than a runtime branch keep each march free of control flow around its memory instructions,
// so the compiler's vmcnt accounting stays exact (a branch there made it drain every load).
template <int R, int TY, int NT, typename TIn, typename TOut, bool EDGE, int ABL = 0>
__global__ __launch_bounds__(NT) void gf3d_fused_kernel(GFParams p) {
    using C = GFConfig<R, TY, NT>;
    constexpr int TX = C::TX, W = C::W;
    constexpr int K5 = C::K5;
    constexpr int ESZ = (int)sizeof(TIn), OSZ = (int)sizeof(TOut);
    extern __shared__ __attribute__((aligned(16))) char smem[];
    // (re-pointed at the buffer of the step's parity before each phase when C::ONEBAR)
    double* Hx = reinterpret_cast<double*>(smem + C::OFF_HX);
    float2* Lab = reinterpret_cast<float2*>(smem + C::OFF_LAB);
    float2* Hab = reinterpret_cast<float2*>(smem + C::OFF_HAB);
    auto set_hx = [&](int i) {
        Hx = reinterpret_cast<double*>(smem + C::OFF_HX + (i & 1) * C::SZ_HX);
    };
    auto set_lab = [&](int i) {
        Lab = reinterpret_cast<float2*>(smem + C::OFF_LAB + (i & 1) * C::SZ_LAB);
    };
    auto set_hab = [&](int i) {
        Hab = reinterpret_cast<float2*>(smem + C::OFF_HAB + (i & 1) * C::SZ_HAB);
    };
    float* Lc = reinterpret_cast<float*>(smem + C::OFF_LC);
    float* Lv5 = reinterpret_cast<float*>(smem + C::OFF_LV5);
    float* Lout = reinterpret_cast<float*>(smem + C::OFF_LOUT);
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
    const int gtx = EDGE ? p.tiles_x : p.itx1 - p.itx0;  // this launch's tile grid
    const int gty = EDGE ? p.tiles_y : p.ity1 - p.ity0;
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
    if constexpr (EDGE) {
        if (tile_x >= p.itx0 && tile_x < p.itx1 && tile_y >= p.ity0 && tile_y < p.ity1) return;
    } else {
        tile_x += p.itx0;
        tile_y += p.ity0;
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
    // Interior tiles (see launch_fused_cfg): window counts are W^3 wherever z is interior too,
    // so P3/P5 take a branch-free path with the constant correctly rounded 1/W^3
    // (host-computed).
    const bool xy_interior = x0 - 2 * R >= 0 && x0 + TX + 2 * R <= nx && y0 - 2 * R >= 0 &&
                             y0 + TY + 2 * R <= ny;  // wave-uniform
    constexpr float kW3 = (float)C::W3;
    const float rcp_w3 = p.rcp_w3;

    // ---- per-thread, step-invariant quad offsets and in-domain masks -----------------------
    const int tid0 = threadIdx.x;
    constexpr int QPL = C::QPL, EPL = C::EPL;
    int q1off[C::NQP1][QPL], q1mask[C::NQP1][QPL];
    // P12 lane -> (E2 row, lane item = EPL consecutive x) for pass k
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
#pragma unroll
        for (int h = 0; h < QPL; ++h) {
            const int gx = x0 - 2 * R + EPL * cq + 4 * h, gy = y0 - 2 * R + row;
            int m = 0;
            if (valid && gy >= 0 && gy < ny) {
#pragma unroll
                for (int e = 0; e < 4; ++e) m |= (gx + e >= 0 && gx + e < nx) ? (1 << e) : 0;
            }
            q1mask[k][h] = m;
            q1off[k][h] = (EDGE ? valid : m == 0xF) ? (gy * sy + gx) * ESZ : kBadOff;
        }
    }
    // Lc / v5 / output quads: offsets and masks are recomputed at their one use per step
    // (a few integer ops) rather than held in registers across the march.
    // P3's center slice on the E1 apron, on the quad grid of E2 (first quad starts C::XC
    // elements left of the E1 apron), so Lc quads are aligned like P1's
    auto quad_c = [&](int tid, int& off, int& mask) {
        const int row = tid / C::NQCX, cq = tid % C::NQCX;
        const int gx = x0 - R - C::XC + 4 * cq, gy = y0 - R + row;
        int m = 0;
        if (tid < C::NQC && gy >= 0 && gy < ny) {
#pragma unroll
            for (int e = 0; e < 4; ++e) m |= (gx + e >= 0 && gx + e < nx) ? (1 << e) : 0;
        }
        mask = m;
        off = (EDGE ? tid < C::NQC : m == 0xF) ? (gy * sy + gx) * ESZ : kBadOff;
    };
    auto quad_t = [&](int q, int& ox, int& oy, int& mask) {  // tile quad q: output positions
        const int row = q / (TX / 4), cq = q % (TX / 4);
        ox = x0 + 4 * cq;
        oy = y0 + row;
        int m = 0;
        if (q >= 0 && q < C::NQ5 && oy < oy_end) {
#pragma unroll
            for (int e = 0; e < 4; ++e) m |= (ox + e < ox_end) ? (1 << e) : 0;
        }
        mask = m;
    };

    auto load_quad = [&](rsrc_t r, int off, int mask, float (&v)[4]) {
        if constexpr (EDGE) load_quad_masked<TIn>(r, off, mask, v);
        else Quad<TIn>::load(r, off, v);
    };

    double zv[C::NQP1][EPL];
#pragma unroll
    for (int k = 0; k < C::NQP1; ++k)
#pragma unroll
        for (int e = 0; e < EPL; ++e) zv[k][e] = 0.0;
    // Running z-window: seed Zv(zc_begin - 1) = sum of v over [zc_begin-1-R, zc_begin-1+R]
    // clamped to [0, nz); every later step adds the entering and subtracts the leaving slice
    // (both 0 outside the domain), so the window stays exact through out-of-domain steps.
    {
        const int za = max(zc_begin - 1 - R, 0), zb_ = min(zc_begin - 1 + R, nz - 1);
        for (int z = za; z <= zb_; ++z) {
            const rsrc_t rs = slice_rsrc(z);
#pragma unroll
            for (int k = 0; k < C::NQP1; ++k)
#pragma unroll
                for (int h = 0; h < QPL; ++h) {
                    float v[4];
                    load_quad(rs, q1off[k][h], q1mask[k][h], v);
#pragma unroll
                    for (int e = 0; e < 4; ++e) zv[k][4 * h + e] += (double)v[e];
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

    // P3 item of a thread (-1: none). GF_P3_SPREAD: the items spread evenly over all waves
    // (every wave carries the same P3 work, so no SIMD finishes its share late), else the top
    // N3 threads.
    auto p3_item = [&](int tid) -> int {
        if constexpr (GF_P3_SPREAD) {
            constexpr int per = (C::N3 + C::NWAVE - 1) / C::NWAVE;
            const int l = tid % 64, it = (tid / 64) * per + l;
            return (l < per && it < C::N3) ? it : -1;
        } else {
            return tid - C::T3;
        }
    };
    // ---- phase bodies ----------------------------------------------------------------------
    float pa[C::NQP1][EPL], ps[C::NQP1][EPL];  // P1 inputs of the next stage-1 slice (prefetched)
    float vc[C::K3];  // GF_DIRECT: v of the next P3 slice at this thread's item (prefetched)
    float v5[K5];     // GF_DIRECT: v of the next P5 output slice at this thread's outputs
#pragma unroll
    for (int j = 0; j < K5; ++j) v5[j] = 0.0f;
    auto load_p1 = [&](rsrc_t ra, rsrc_t rs) {  // entering slice zc+R, leaving slice zc-R-1
#pragma unroll
        for (int k = 0; k < C::NQP1; ++k)
#pragma unroll
            for (int h = 0; h < QPL; ++h) {
                float a4[4], s4[4];
                if constexpr (ABL & 8) { for (int e = 0; e < 4; ++e) a4[e] = 1.0f; }
                else load_quad(ra, q1off[k][h], q1mask[k][h], a4);
                if constexpr (ABL & 1) { for (int e = 0; e < 4; ++e) s4[e] = 0.5f; }
                else if constexpr (!EDGE && GF_LEAVE_AUX != 0)
                    Quad<TIn>::template load<GF_LEAVE_AUX>(rs, q1off[k][h], s4);
                else load_quad(rs, q1off[k][h], q1mask[k][h], s4);
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    pa[k][4 * h + e] = a4[e];
                    ps[k][4 * h + e] = s4[e];
                }
            }
    };
    // P12: z-window of v (f64, running) and its x-window sums on the E2 apron -> Hx. The x
    // neighbours come from the adjacent lanes' quads by DPP wave shifts (whole rows per wave),
    // so the z-window never goes through LDS.
    auto do_p12 = [&](int tid) {
        if constexpr (ABL & 1024) return;
#pragma unroll
        for (int k = 0; k < C::NQP1; ++k) {
            int row, cq;
            const bool valid = p12_pos(tid, k, row, cq);
#pragma unroll
            for (int e = 0; e < EPL; ++e) {
                zv[k][e] = zv[k][e] + (double)pa[k][e];  // entering slice (0 outside the domain)
                zv[k][e] = zv[k][e] - (double)ps[k][e];  // leaving slice (0 outside the domain)
            }
            constexpr int NB = C::NB;
            double win[EPL * (2 * NB + 1)];  // lane items cq-NB .. cq+NB
#pragma unroll
            for (int e = 0; e < EPL; ++e) win[EPL * NB + e] = zv[k][e];
            // only the R elements next to the own item are read (the others' moves are dead)
#pragma unroll
            for (int n = 1; n <= NB; ++n)
#pragma unroll
                for (int e = 0; e < EPL; ++e) {
                    if constexpr (ABL & 512) {
                        win[EPL * (NB - n) + e] = win[EPL * (NB - n + 1) + e] * 0.5;
                        win[EPL * (NB + n) + e] = win[EPL * (NB + n - 1) + e] * 0.25;
                    } else {
                        win[EPL * (NB - n) + e] = dpp_from_lower(win[EPL * (NB - n + 1) + e]);
                        win[EPL * (NB + n) + e] = dpp_from_upper(win[EPL * (NB + n - 1) + e]);
                    }
                }
            double vin[EPL + 2 * R], hs[EPL];
#pragma unroll
            for (int j = 0; j < EPL + 2 * R; ++j) vin[j] = win[EPL * NB - R + j];
            slide_sums_f64<R, EPL>(vin, hs);
            if constexpr (GF_HX_B128 && R % 2 == 0) {
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
    // Pointwise stage on NP pairs of E1 positions, packed (both lanes of every op in one issue)
    // and written op-by-op across the pairs so dependent packed ops are interleaved (gfx950
    // needs an s_nop between back-to-back dependent v_pk_* otherwise):
    //   u = RN(RN(U) / c)   (summed_area_table_mean, exact: Markstein with rcp = RN(1/c))
    //   s = (v - u)^2;  a = s / (s + eps);  b = (1 - a) * u          (guided_filter.rs:126-137)
    constexpr int NP3 = C::K3 / 2;
    // The compiler schedules the pairs as separate chains, each dependent v_pk_* then waiting on
    // an s_nop; a scheduling fence after every op keeps them in lockstep instead (a fence, not
    // an asm statement: the hazard recognizer pads after inline asm).
    auto sync = [&](f2 (&)[NP3]) {
        if constexpr (GF_PW_SYNC) __builtin_amdgcn_sched_barrier(0);
    };
    auto pointwise = [&](const f2 (&Uf)[NP3], const f2 (&v)[NP3], const f2 (&fc)[NP3],
                         const f2 (&rc)[NP3], f2 (&a)[NP3], f2 (&bb)[NP3]) {
        f2 q[NP3], r[NP3], u[NP3], sq[NP3], den[NP3], y[NP3], e[NP3];
#pragma unroll
        for (int k = 0; k < NP3; ++k) q[k] = Uf[k] * rc[k];
        sync(q);
#pragma unroll
        for (int k = 0; k < NP3; ++k) r[k] = pk_fma(-q[k], fc[k], Uf[k]);
        sync(r);
#pragma unroll
        for (int k = 0; k < NP3; ++k) u[k] = pk_fma(r[k], rc[k], q[k]);
        sync(u);
#pragma unroll
        for (int k = 0; k < NP3; ++k) sq[k] = v[k] - u[k];
        sync(sq);
#pragma unroll
        for (int k = 0; k < NP3; ++k) sq[k] = sq[k] * sq[k];  // (v - u).powf(2.0)
        sync(sq);
        if constexpr (ABL & 32) {
#pragma unroll
            for (int k = 0; k < NP3; ++k) { a[k] = sq[k]; bb[k] = u[k]; }
        } else {
#pragma unroll
            for (int k = 0; k < NP3; ++k) den[k] = sq[k] + (f2){eps, eps};
            sync(den);
#pragma unroll
            for (int k = 0; k < NP3; ++k)
                y[k] = (f2){__builtin_amdgcn_rcpf(den[k].x), __builtin_amdgcn_rcpf(den[k].y)};
            sync(y);
            if constexpr (GF_NEWTON_A) {  // refine 1/den before Markstein's correction
#pragma unroll
                for (int k = 0; k < NP3; ++k) e[k] = pk_fma(-den[k], y[k], (f2){1.0f, 1.0f});
#pragma unroll
                for (int k = 0; k < NP3; ++k) y[k] = pk_fma(e[k], y[k], y[k]);
            }
#pragma unroll
            for (int k = 0; k < NP3; ++k) q[k] = sq[k] * y[k];
            sync(q);
            if constexpr (GF_A_RCP) {
#pragma unroll
                for (int k = 0; k < NP3; ++k) a[k] = q[k];
            } else {
#pragma unroll
                for (int k = 0; k < NP3; ++k) r[k] = pk_fma(-den[k], q[k], sq[k]);
                sync(r);
#pragma unroll
                for (int k = 0; k < NP3; ++k) a[k] = pk_fma(r[k], y[k], q[k]);
                sync(a);
            }
#pragma unroll
            for (int k = 0; k < NP3; ++k) e[k] = (f2){1.0f, 1.0f} - a[k];
            sync(e);
#pragma unroll
            for (int k = 0; k < NP3; ++k) bb[k] = e[k] * u[k];
        }
    };
    static_assert(C::K3 % 2 == 0, "P3 works on pairs");
    // every P3 segment lies inside the apron: unconditional Lab stores (a guard lets the compiler
    // sink the second pair's pointwise chain into it, serialising the pairs)
    constexpr bool kRowsWhole = C::E1Y % C::K3 == 0;
    auto do_p3 = [&](int tid, int zc) {  // y-window (f64) of Hx -> U; a, b -> Lab
        const int item = p3_item(tid);
        if (item < 0) return;
        if constexpr (ABL & 2048) return;
        const int col = item % C::E1X, sg = item / C::E1X;
        const double* src = Hx + (sg * C::K3) * C::PH + col;
        double vin[C::K3 + 2 * R], U[C::K3];
#pragma unroll
        for (int j = 0; j < C::K3 + 2 * R; ++j) {
            if constexpr (ABL & 256) vin[j] = j == 0 ? src[0] : vin[j - 1] * 1.0001;
            else vin[j] = src[j * C::PH];
        }
        slide_sums_f64<R, C::K3>(vin, U);
        f2* lab = reinterpret_cast<f2*>(Lab);
        f2 Uf[NP3], vv[NP3], fc[NP3], rc[NP3], a[NP3], bb[NP3];
#if GF_DIRECT
#pragma unroll
        for (int k = 0; k < NP3; ++k) {
            Uf[k] = (f2){(float)U[2 * k], (float)U[2 * k + 1]};
            vv[k] = (f2){vc[2 * k], vc[2 * k + 1]};  // v of slice zc, loaded a half-step ago
        }
#else
        const float* vsrc = Lc + (sg * C::K3) * C::PC + C::XC + col;  // v of slice zc (C1)
#pragma unroll
        for (int k = 0; k < NP3; ++k) {
            Uf[k] = (f2){(float)U[2 * k], (float)U[2 * k + 1]};
            vv[k] = (f2){vsrc[(2 * k) * C::PC], vsrc[(2 * k + 1) * C::PC]};
        }
#endif
        if (xy_interior && zc - R >= 0 && zc + R < nz) {  // wave-uniform: count = W^3
#pragma unroll
            for (int k = 0; k < NP3; ++k) {
                fc[k] = (f2){kW3, kW3};
                rc[k] = (f2){rcp_w3, rcp_w3};
            }
            pointwise(Uf, vv, fc, rc, a, bb);
#pragma unroll
            for (int k = 0; k < NP3; ++k) {
                const int ey = sg * C::K3 + 2 * k;
                if (kRowsWhole || ey < C::E1Y) lab[ey * C::PA + col] = __builtin_shufflevector(a[k], bb[k], 0, 2);
                if (kRowsWhole || ey + 1 < C::E1Y)
                    lab[(ey + 1) * C::PA + col] = __builtin_shufflevector(a[k], bb[k], 1, 3);
            }
            return;
        }
        const int gx = x0 - R + col;
        const bool xzin = gx >= 0 && gx < nx && zc >= 0 && zc < nz;
        const int cxz = clamped_count(gx, nx, R) * clamped_count(zc, nz, R);
#pragma unroll
        for (int k = 0; k < NP3; ++k) {
            const int gy = y0 - R + sg * C::K3 + 2 * k;
            const int c0 = clamped_count(gy, ny, R) * cxz, c1 = clamped_count(gy + 1, ny, R) * cxz;
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
    };
    auto do_p4 = [&](int tid) {  // x-window sums of (a, b) rows -> Hab
        const int item = tid;
#if GF_WAVE_SKIP
        // whole waves past the items branch around the phase (scalar test): exec-masked they
        // would still spend their issue slots on it
        if (__builtin_amdgcn_readfirstlane(tid >> 6) * 64 >= C::N4) return;
#endif
        if (item >= C::N4) return;
        if constexpr (ABL & 4096) return;
        const int row = item % C::E1Y, sg = item / C::E1Y;
        const float4* src = reinterpret_cast<const float4*>(Lab + row * C::PA + sg * C::K4);
        f2 vin[C::K4 + 2 * R], vout[C::K4];
        float4 f0 = src[0];
#pragma unroll
        for (int j = 0; j < (C::K4 + 2 * R) / 2; ++j) {
            float4 f;
            if constexpr (ABL & 128) { f = f0; f0.x *= 1.0001f; f0.y *= 0.999f; f0.z *= 1.001f; f0.w *= 0.9999f; }
            else f = src[j];
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
    rsrc_t ro5;  // GF_DIRECT: the output slice P5 stores to this step
    auto do_p5 = [&](int tid, int zc, auto slot_c) {  // y-window -> slice sums; z; out -> Lout
        if constexpr (ABL & 8192) return;
        const int col5 = tid % TX, seg5 = tid / TX;
        const f2* src = reinterpret_cast<const f2*>(Hab) + (seg5 * K5) * C::PB + col5;
        f2 vin[K5 + 2 * R], s2[K5];
#pragma unroll
        for (int j = 0; j < K5 + 2 * R; ++j) {
            if constexpr (ABL & 64) vin[j] = j == 0 ? src[0] : vin[j - 1] * (f2){1.0001f, 0.999f};
            else vin[j] = src[j * C::PB];
        }
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
#if !GF_DIRECT
        if (zo < zo_begin || zo >= zo_end) return;  // wave-uniform
#endif
        const int ox = x0 + col5, oyb = y0 + seg5 * K5;
        const bool interior = xy_interior && zo - R >= 0 && zo + R < nz;  // wave-uniform
        // (GF_DIRECT: steps that emit nothing run too, their stores dropped by the descriptor;
        //  the z count is clamped so its table index stays valid there)
        const int zq = min(max(zo, 0), nz - 1);
        const int cxz = interior ? 0 : clamped_count(ox, nx, R) * clamped_count(zq, nz, R);
        f2 fc[K5], rc[K5], q[K5], r[K5];
#pragma unroll
        for (int j = 0; j < K5; ++j) {
            if (interior) {
                fc[j] = (f2){kW3, kW3};
                rc[j] = (f2){rcp_w3, rcp_w3};
            } else {
                const int cnt = clamped_count(oyb + j, ny, R) * cxz;
                const float f = (float)cnt, rr = rcp_tab[cnt];
                fc[j] = (f2){f, f};
                rc[j] = (f2){rr, rr};
            }
        }
        // (sum as f32) / (count as f32) for a and b together
#pragma unroll
        for (int j = 0; j < K5; ++j) q[j] = AB[j] * rc[j];
        if constexpr (!GF_FASTDIV5) {  // correctly rounded (Markstein)
#pragma unroll
            for (int j = 0; j < K5; ++j) r[j] = pk_fma(-q[j], fc[j], AB[j]);
#pragma unroll
            for (int j = 0; j < K5; ++j) q[j] = pk_fma(r[j], rc[j], q[j]);
        }
#if GF_DIRECT
        (void)r;
#pragma unroll
        for (int j = 0; j < K5; ++j) {
            const int oy = oyb + j;
            const float o = __fadd_rn(__fmul_rn(v5[j], q[j].x), q[j].y);  // v*=ma; v+=mb
            const int off = (ox < ox_end && oy < oy_end)
                                ? ((oy - p.oy0) * osy + (ox - p.ox0)) * OSZ : kBadOff;
            Buf<TOut>::store(from_f32<TOut>(o), ro5, opaque(off));
        }
#else
#pragma unroll
        for (int j = 0; j < K5; ++j) {
            const int ty = seg5 * K5 + j;
            const float v = Lv5[ty * TX + col5];                  // v of slice zo (staged in C1)
            Lout[ty * TX + col5] = __fadd_rn(__fmul_rn(v, q[j].x), q[j].y);  // v*=ma; v+=mb
        }
#endif
    };

    // ---- C1 staging: 16-byte quads between global memory and the LDS tiles ------------------
    // Every global access of the march below is unconditional, in the same order every step:
    // out-of-range slices, inactive lanes and non-emitting steps use null descriptors or
    // kBadOff instead of branches. Branches around memory instructions make the compiler's
    // vmcnt accounting fall back to draining the loads just issued (measured: a 1.6x slower
    // kernel); straight-line, it waits for exactly the step-old load it needs.
    float cq4[4], vq4[4];  // v of the next Lc slice / the next Lv5 slice (prefetched a step ahead)
    auto load_c = [&](rsrc_t r) {
        if constexpr (ABL & 2) { for (int e = 0; e < 4; ++e) cq4[e] = 1.0f; }
        else {
            int off, mask;
            quad_c((int)threadIdx.x, off, mask);
            load_quad(r, off, mask, cq4);
        }
    };
    auto load_v5 = [&](rsrc_t r) {
        if constexpr (ABL & 4) { for (int e = 0; e < 4; ++e) vq4[e] = 1.0f; }
        else {
            const int q = (int)threadIdx.x - (NT - C::NQ5);
            int ox, oy, mask;
            quad_t(q, ox, oy, mask);
            const int off = (EDGE ? q >= 0 : mask == 0xF) ? (oy * sy + ox) * ESZ : kBadOff;
            load_quad(r, off, mask, vq4);
        }
    };
    // GF_DIRECT loaders: one element per access, lanes on consecutive x (coalesced rows).
    // Positions outside the domain either read 0 through the range check or read a neighbour
    // row's value that is never used (P3 zeroes its out-of-domain (a, b); P5's store drops).
    auto load_p3v = [&](rsrc_t r) {
        const int item = p3_item((int)threadIdx.x);
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
            v5[j] = Buf<TIn>::template load<GF_V5_AUX>(r, opaque(ok ? (oy * sy + ox) * ESZ : kBadOff));
        }
    };
    float* const dummy = reinterpret_cast<float*>(smem + C::OFF_DUMMY);  // inactive lanes' writes
    auto write_c = [&](int tid) {
        const int row = tid / C::NQCX, cq = tid % C::NQCX;
        float* dst = tid < C::NQC ? Lc + row * C::PC + 4 * cq : dummy;
        *reinterpret_cast<float4*>(dst) = make_float4(cq4[0], cq4[1], cq4[2], cq4[3]);
    };
    auto write_v5 = [&](int tid) {
        const int q = tid - (NT - C::NQ5);
        const int row = q / (TX / 4), cq = q % (TX / 4);
        float* dst = q >= 0 ? Lv5 + row * TX + 4 * cq : dummy;
        *reinterpret_cast<float4*>(dst) = make_float4(vq4[0], vq4[1], vq4[2], vq4[3]);
    };
    auto store_out = [&](int tid, rsrc_t ro) {  // Lout -> global, one quad per thread
        const bool act = tid < C::NQ5;
        const int row = act ? tid / (TX / 4) : 0, cq = act ? tid % (TX / 4) : 0;
        const float4 o4 = *reinterpret_cast<const float4*>(Lout + row * TX + 4 * cq);
        const float o[4] = {o4.x, o4.y, o4.z, o4.w};
        int ox, oy, mask;
        quad_t(tid, ox, oy, mask);
        const int off =
            (EDGE ? act : mask == 0xF) ? ((oy - p.oy0) * osy + (ox - p.ox0)) * OSZ : kBadOff;
        if constexpr (EDGE) store_quad_masked<TOut>(o, ro, off, mask);
        else Quad<TOut>::store(o, ro, off);
    };

    // ---- prologue: stage 1 of the first slice up to Hx, first Lc; prefetch step 1 -----------
    load_p1(slice_rsrc(zc_begin + R), slice_rsrc(zc_begin - R - 1));
#if GF_DIRECT
    load_p3v(slice_rsrc(zc_begin));
    if constexpr (C::ONEBAR) set_hx(zc_begin);
    do_p12(tid0);
#else
    load_c(slice_rsrc(zc_begin));
    do_p12(tid0);
    write_c(tid0);
    load_c(slice_rsrc(zc_begin + 1));
    load_v5(slice_rsrc(zc_begin - R));
#endif
    load_p1(slice_rsrc(zc_begin + 1 + R), slice_rsrc(zc_begin - R));
    lds_barrier_abl<ABL>();

    // ---- slice streams: descriptors advanced by one slice per step (two 32-bit adds each)
    //      instead of rebuilt from z (a 64-bit multiply and range checks per descriptor) ------
    // step i reads slice zb = i+1-R (leaving slice of P1(i+2), and v5), zb+R+1 = i+2 (Lc) and
    // zb+2R+1 = i+2+R (entering slice of P1(i+2)); it stores output slice zs = i-1-R.
    const int64_t sstride = p.in_sz * ESZ, osstride = p.out_sz * OSZ;
    const int64_t off_c = (int64_t)(R + 1) * sstride, off_a = (int64_t)(2 * R + 1) * sstride;
    int zb = zc_begin + 1 - R;
    int64_t ob = (int64_t)(zb - p.in_z0) * sstride;
    int zs = zc_begin - (C::ONEBAR ? 2 : 1) - R;  // output slice of this step's P5
    int64_t os = (int64_t)(zs - p.oz0) * osstride;
    const char* out_base = static_cast<const char*>(p.out);
    const unsigned nzo = (unsigned)(zo_end - zo_begin);
    auto rs_in = [&](int64_t off, int z) {
        return make_rsrc(in_base + off, (unsigned)(z - zlo) < (unsigned)zspan ? slice_bytes : 0u);
    };

    // ---- pipelined march, unrolled by W so the ring slot of every P5 is a constant ----------
    // The step count is padded to a multiple of W, at least one past the last stage-1 slice so
    // that P5/the store of the last output slice happen inside the loop: no guards inside.
    // Padded steps emit nothing (zo >= zo_end).
    // (ONEBAR: P5 runs two steps behind P3, so one more step.)
    const int n_steps = (zc_end - zc_begin + (C::ONEBAR ? 2 : 1) + W - 1) / W * W;
    for (int i0 = zc_begin; i0 < zc_begin + n_steps; i0 += W) {
        static_for<0, W>([&](auto kc) {
            constexpr int k = decltype(kc)::value;
            const int i = i0 + k;
            const int tid = threadIdx.x;
            const rsrc_t r_b = rs_in(ob, zb);
            if constexpr (C::ONEBAR) {
                // One barrier per step. Step i: P12(i+1) -> Hx[i+1], P5(i-2) <- Hab[i],
                // P3(i) <- Hx[i] -> Lab[i], P4(i-1) <- Lab[i-1] -> Hab[i-1] (buffers by parity:
                // each is written in one step and read in the next). The first steps' P4/P5
                // work on unwritten buffers for slices that lie in no emitted window (see the
                // GF_DIRECT note on P5); their stores go to zero-record descriptors.
                ro5 = make_rsrc(out_base + os,
                                (unsigned)(zs - zo_begin) < nzo ? oslice_bytes : 0u);
                if constexpr (GF_PRIO) __builtin_amdgcn_s_setprio(3);
                set_hx(i + 1);
                do_p12(tid);
                load_p1(rs_in(ob + off_a, zb + 2 * R + 1), r_b);  // for P12(i+2)
                if constexpr (GF_PRIO) __builtin_amdgcn_s_setprio(1);
                set_hab(i);
                do_p5(tid, i - 2, std::integral_constant<int, (k + 2 * W - 2) % W>{});
                load_p5v(rs_in(ob - 2 * sstride, zb - 2));  // slice i-1-R, for P5(i-1)
                set_hx(i);
                set_lab(i);
                do_p3(tid, i);
                load_p3v(rs_in(ob + (int64_t)R * sstride, zb + R));  // slice i+1, for P3(i+1)
                set_lab(i - 1);
                set_hab(i - 1);
                do_p4(tid);
                lds_barrier_abl<ABL>();
                ++zb;
                ob += sstride;
                ++zs;
                os += osstride;
                return;
            }
            // tools/ instrumentation only (ABL & 16384): per-wave stamps of one workgroup
            auto stamp = [&](int slot) {
                if constexpr (ABL & 16384) {
                    const int st = i - zc_begin - 64;
                    if ((int)blockIdx.x == p.trace_block && st >= 0 && st < 18 &&
                        (threadIdx.x & 63) == 0)
                        p.trace[(st * 16 + threadIdx.x / 64) * 8 + slot] =
                            __builtin_amdgcn_s_memtime();
                }
            };
#if GF_DIRECT
            ro5 = make_rsrc(out_base + os, (unsigned)(zs - zo_begin) < nzo ? oslice_bytes : 0u);
#endif
            stamp(0);
            // Fair progress across the waves of a SIMD: the hardware issues oldest-first, which
            // staggers the waves so the youngest runs its last phase alone, latency exposed. A
            // wave drops its priority as it completes a phase, so laggards catch up.
            if constexpr (GF_PRIO) __builtin_amdgcn_s_setprio(3);
            // C0: P3(i) + P5(i-1) (LDS and registers only)
            if constexpr (C::ORDER & 1) {
                if (i > zc_begin) do_p5(tid, i - 1, std::integral_constant<int, (k + W - 1) % W>{});
                if constexpr (GF_PRIO) __builtin_amdgcn_s_setprio(1);
                do_p3(tid, i);
            } else {
                do_p3(tid, i);
                if constexpr (GF_PRIO) __builtin_amdgcn_s_setprio(1);
                stamp(4);
                // GF_DIRECT: unconditional, so no branch separates P5's stores from the loads
                // waited on later (the first call's slice lies in no emitted window, and its
                // stores go to a zero-record descriptor)
                if (GF_DIRECT || i > zc_begin)
                    do_p5(tid, i - 1, std::integral_constant<int, (k + W - 1) % W>{});
            }
            stamp(1);
            lds_barrier_abl<ABL>();
            stamp(2);
            if constexpr (GF_PRIO) __builtin_amdgcn_s_setprio(3);
            // C1: staging (store out(i-1-R), Lc <- slice i+1, Lv5 <- slice i-R), the loads of
            // the next step, P12(i+1), P4(i). Every wait here is for a load issued a step ago.
#if GF_DIRECT
            // next step's P3 slice i+1 (= zb + R) and P5 slice i-R (= zb - 1)
            load_p3v(rs_in(ob + (int64_t)R * sstride, zb + R));
            load_p5v(rs_in(ob - sstride, zb - 1));
#else
            store_out(tid, make_rsrc(out_base + os,
                                     (unsigned)(zs - zo_begin) < nzo ? oslice_bytes : 0u));
            write_c(tid);
            write_v5(tid);
            load_c(rs_in(ob + off_c, zb + R + 1));
            load_v5(r_b);
#endif
            stamp(6);
            if constexpr (GF_PRIO >= 2) __builtin_amdgcn_s_setprio(2);
            if constexpr (C::ORDER & 2) do_p4(tid);
            do_p12(tid);
            load_p1(rs_in(ob + off_a, zb + 2 * R + 1), r_b);
            if constexpr (GF_PRIO) __builtin_amdgcn_s_setprio(1);
            stamp(5);
            if constexpr (!(C::ORDER & 2)) do_p4(tid);
            stamp(3);
            lds_barrier_abl<ABL>();
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

template <int R, int TY, int NT, typename TIn, typename TOut, bool EDGE, int ABL = 0>
inline hipError_t launch_fused_variant(const GFParams& p, long long nwg, hipStream_t stream) {
    using C = GFConfig<R, TY, NT>;
    const size_t lds = (size_t)C::LDS_BYTES;
    auto kern = gf3d_fused_kernel<R, TY, NT, TIn, TOut, EDGE, ABL>;
    if (hipError_t e = allow_dynamic_lds((const void*)kern, (int)lds, attr_devices<decltype(kern)>()))
        return e;
    if (nwg <= 0) return hipSuccess;
    if (nwg > 0x7FFFFFFFLL) return hipErrorInvalidValue;
    hipLaunchKernelGGL(kern, dim3((unsigned)nwg), dim3(NT), lds, stream, p);
    return hipGetLastError();
}

template <int R, int TY, int NT, typename TIn, typename TOut, int ABL = 0>
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
    // Quad-aligned geometry: every quad starts at a multiple of 4 elements (the E2 apron at
    // x0 - 2R, the output tile at x0), and the domain / output box widths are multiples of 4,
    // so no quad straddles a boundary: the first kernel takes every tile.
    const bool quad_ok = (p.ox0 % 4 == 0) && (R % 2 == 0) && (p.nx % 4 == 0) &&
                         (p.onx % 4 == 0) && (p.in_sy % 4 == 0) && (p.in_sz % 4 == 0) &&
                         (p.out_sy % 4 == 0) && (p.out_sz % 4 == 0) &&
                         ((uintptr_t)p.in % (4 * sizeof(TIn)) == 0) &&
                         ((uintptr_t)p.out % (4 * sizeof(TOut)) == 0);
    if (quad_ok) {
        p.itx0 = 0; p.itx1 = p.tiles_x;
        p.ity0 = 0; p.ity1 = p.tiles_y;
    } else {
        // +4 elements of x slack: the last Lc quad of a row may overhang the E1 apron
        interior_tiles(p.ox0, p.ox0 + p.onx, p.nx, C::TX, R, 4, p.tiles_x, p.itx0, p.itx1);
        interior_tiles(p.oy0, p.oy0 + p.ony, p.ny, TY, R, 0, p.tiles_y, p.ity0, p.ity1);
    }
    const long long n_int = (long long)(p.itx1 - p.itx0) * (p.ity1 - p.ity0);
    const long long n_all = (long long)p.tiles_x * p.tiles_y;
    hipError_t e = hipSuccess;
    if (n_int > 0)
        e = launch_fused_variant<R, TY, NT, TIn, TOut, false, ABL>(p, n_int * p.nseg, stream);
    if (e == hipSuccess && n_all > n_int)
        e = launch_fused_variant<R, TY, NT, TIn, TOut, true, ABL>(p, n_all * p.nseg, stream);
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
