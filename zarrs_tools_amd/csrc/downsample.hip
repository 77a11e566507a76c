// downsample.hip — mean / mode downsample (downsample.rs:64-120) and the synthetic generators.
//
// Continuous: for every COMPLETE window (ndarray exact_chunks with window = min(stride, extent),
// downsample.rs:83-86) the f64 sum of `as f64` elements in C order, folded from -0.0 as Rust's
// f64 Sum does, divided by the window length (f64), then `as TOut` (downsample.rs:87-92). The
// same order and precision as the reference, so results are bit-identical.
// Discrete: the most frequent value of the window; ties broken by the smallest value (the
// reference breaks ties by HashMap iteration order, which is unspecified — DESIGN.md §6).
//
// HBM-bound (2.25 B per input voxel for 2x u16): one thread per output element, the window
// walked in C order so a wave's x-rows are contiguous 64*s runs of input.

#include <hip/hip_runtime.h>

#include <algorithm>
#include <stdint.h>
#include <type_traits>

#include "zt_device.hpp"
#include "zt_kernels.hpp"

namespace zt {

template <typename TIn, typename TOut>
__global__ __launch_bounds__(256) void downsample_continuous_kernel(const TIn* __restrict__ in,
                                                                    TOut* __restrict__ out,
                                                                    DSParams p) {
    for (int64_t o = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; o < p.out_numel;
         o += (int64_t)gridDim.x * blockDim.x) {
        // window origin
        int64_t rem = o, base = 0, mul = 1;
        for (int d = p.ndim - 1; d >= 0; --d) {
            int64_t c = rem % p.out_shape[d];
            rem /= p.out_shape[d];
            base += c * p.win[d] * mul;
            mul *= p.in_shape[d];
        }
        double sum = -0.0;
        for (int64_t w = 0; w < p.win_numel; ++w) {
            int64_t r2 = w, off = 0, m2 = 1;
            for (int d = p.ndim - 1; d >= 0; --d) {
                int64_t c = r2 % p.win[d];
                r2 /= p.win[d];
                off += c * m2;
                m2 *= p.in_shape[d];
            }
            sum += Elem<TIn>::to_f64(in[base + off]);
        }
        out[o] = from_f64<TOut>(sum / (double)p.win_numel);
    }
}

// 3-D fast path (window wz x wy x wx, all compile-time small): C-order f64 sum, same arithmetic.
// One output per thread; the grid enumerates (x, y, z) so there is no per-output index division
// (64-bit divisions of indices past 2^32 dominated the 4096^3 pyramid's level 1).
template <typename TIn, typename TOut, int WZ, int WY, int WX>
__global__ __launch_bounds__(256) void downsample3_kernel(const TIn* __restrict__ in,
                                                          TOut* __restrict__ out, DSParams p) {
    const int64_t onx = p.out_shape[2], ony = p.out_shape[1], onz = p.out_shape[0];
    const int64_t inx = p.in_shape[2], iny = p.in_shape[1];
    const int64_t x = (int64_t)blockIdx.x * 256 + threadIdx.x, y = blockIdx.y;
    if (x >= onx) return;
    for (int64_t z = blockIdx.z; z < onz; z += gridDim.z) {
        const TIn* src = in + ((z * WZ) * iny + y * WY) * inx + x * WX;
        double sum = -0.0;
#pragma unroll
        for (int a = 0; a < WZ; ++a)
#pragma unroll
            for (int b = 0; b < WY; ++b)
#pragma unroll
                for (int c = 0; c < WX; ++c)
                    sum += Elem<TIn>::to_f64(src[(a * iny + b) * inx + c]);
        out[(z * ony + y) * onx + x] = from_f64<TOut>(sum / (double)(WZ * WY * WX));
    }
}

// `TIn as TOut` for an integer TIn (downsample.rs:117): integer -> integer wraps; integer -> f32 /
// f64 rounds to nearest in one step (a 64-bit value past 2^53 must not be rounded to f64 first);
// f16 / bf16 through f64 (exact below 2^53; beyond it f16 is infinite either way).
template <typename TOut, typename TIn>
__device__ __forceinline__ TOut int_as(TIn v) {
    if constexpr (std::is_integral<TOut>::value) return (TOut)v;
    else if constexpr (std::is_same<TOut, float>::value || std::is_same<TOut, double>::value)
        return (TOut)v;
    else return from_f64<TOut>((double)v);
}

template <typename TIn, typename TOut>
__global__ __launch_bounds__(256) void downsample_discrete_kernel(const TIn* __restrict__ in,
                                                                  TOut* __restrict__ out,
                                                                  DSParams p) {
    for (int64_t o = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; o < p.out_numel;
         o += (int64_t)gridDim.x * blockDim.x) {
        int64_t rem = o, base = 0, mul = 1;
        for (int d = p.ndim - 1; d >= 0; --d) {
            int64_t c = rem % p.out_shape[d];
            rem /= p.out_shape[d];
            base += c * p.win[d] * mul;
            mul *= p.in_shape[d];
        }
        auto at = [&](int64_t w) -> TIn {
            int64_t r2 = w, off = 0, m2 = 1;
            for (int d = p.ndim - 1; d >= 0; --d) {
                int64_t c = r2 % p.win[d];
                r2 /= p.win[d];
                off += c * m2;
                m2 *= p.in_shape[d];
            }
            return in[base + off];
        };
        TIn best = at(0);
        int64_t best_count = -1;
        for (int64_t a = 0; a < p.win_numel; ++a) {
            TIn va = at(a);
            int64_t count = 0;
            for (int64_t b = 0; b < p.win_numel; ++b) count += at(b) == va;
            if (count > best_count || (count == best_count && va < best)) {
                best_count = count;
                best = va;
            }
        }
        out[o] = int_as<TOut>(best);
    }
}

// ---------------------------------------------------------------------------------------------
// Fused 2x2x2 mean pyramid: NL = 2 or 3 levels of zarrs_ome's loop (zarrs_ome.rs:515-738, each
// level downsample.rs:72-97 of the previous one) in one launch, so the intermediate levels are
// written once and never read back. MODE: the same with the mode of each window (zarrs_ome
// --discrete, downsample.rs:99-120; pyr_mode8), each level the mode of the previous level. Every output is computed exactly as downsample3_kernel does
// it (C-order f64 sum from -0.0 of the previous level's `as`-rounded values, / 8, `as T`; 8- to
// 32-bit integers summed exactly in integers, the same value), so the levels are bit-identical
// to per-level launches.
//
// Workgroup = 4 waves; wave w holds (dz, dy) = (w >> 1, w & 1) of a 2x2 block of level-2 rows,
// lane l the level-3 column x3 = 64 bx + l. A lane reads a 4 x 4 x 8 block of level 0 (sixteen
// 8-element rows: 16-byte loads for u16, one contiguous KiB per wave-instruction), computes the
// 2 x 2 x 4 level-1 block, its 2 level-2 values, and (NL = 3) the four waves' level-2 pairs meet
// in LDS for the level-3 value. The grid covers level 1 (ceil(S1 / (4, 4, 256)) workgroups) so
// edge elements of level 1 / 2 outside any level-3 window are produced too; an output is stored
// iff it lies inside its level's shape (its inputs then lie inside theirs).
// ---------------------------------------------------------------------------------------------
struct PyrParams {
    int64_t s[4][3];  // level shapes (z, y, x), level 0 = input
};

template <typename T>
constexpr bool kPyrIntSum = std::is_integral<T>::value && sizeof(T) <= 4;

template <typename T>
__device__ __forceinline__ T pyr_mean8(const T (&v)[8]) {  // v in C order of the window
    if constexpr (kPyrIntSum<T>) {
        // the f64 sum of 8 integers of <= 32 bits is exact and so is its / 8; `as T` truncates
        // toward zero and the mean is in range: the integer quotient, the same value
        using S = std::conditional_t<(sizeof(T) <= 2), int32_t, int64_t>;
        S s = 0;
#pragma unroll
        for (int i = 0; i < 8; ++i) s += (S)v[i];
        return (T)(s / 8);
    } else {
        double s = -0.0;
#pragma unroll
        for (int i = 0; i < 8; ++i) s += Elem<T>::to_f64(v[i]);
        return from_f64<T>(s / 8.0);
    }
}

// Mode of a 2x2x2 window (downsample.rs:99-120): the most frequent value, ties to the smallest
// (the reference's HashMap order is unspecified). Sorted by a 19-comparator network
// (min / max, no masks), then one ascending scan keeps the first longest run: ~75 VALU ops where
// pairwise counting took ~110 plus mask arithmetic on the scalar unit (2.0x faster for u8 levels,
// profiles/r05_mode_pyramid.jsonl). Comparisons in the element type's value order (64-bit for
// 64-bit types).
template <typename T>
__device__ __forceinline__ T pyr_mode8(const T (&v)[8]) {
    using C = std::conditional_t<(sizeof(T) <= 4),
                                 std::conditional_t<std::is_signed<T>::value, int32_t, uint32_t>, T>;
    C s[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) s[i] = (C)v[i];
    auto cx = [&](int i, int j) {
        const C lo = s[i] < s[j] ? s[i] : s[j], hi = s[i] < s[j] ? s[j] : s[i];
        s[i] = lo;
        s[j] = hi;
    };
    cx(0, 2); cx(1, 3); cx(4, 6); cx(5, 7);
    cx(0, 4); cx(1, 5); cx(2, 6); cx(3, 7);
    cx(0, 1); cx(2, 3); cx(4, 5); cx(6, 7);
    cx(2, 4); cx(3, 5);
    cx(1, 4); cx(3, 6);
    cx(1, 2); cx(3, 4); cx(5, 6);
    C best = s[0];
    int bc = 1, run = 1;
#pragma unroll
    for (int i = 1; i < 8; ++i) {
        run = s[i] == s[i - 1] ? run + 1 : 1;
        if (run > bc) {  // strictly longer: an equal run of a larger value does not replace it
            bc = run;
            best = s[i];
        }
    }
    return (T)best;
}

template <typename T, bool MODE>
__device__ __forceinline__ T pyr_reduce8(const T (&v)[8]) {
    if constexpr (MODE) return pyr_mode8<T>(v);
    else return pyr_mean8<T>(v);
}

// XPL level-3 columns per lane: a lane's level-0 rows are 8 XPL elements. 2 for u8 through this
// generic walk would load 16-byte rows, but hipcc then keeps every byte of the 16 rows in a VGPR
// of its own (256 VGPRs, one wave per SIMD: 5.66 ms mean / 7.86 ms mode at 2048^3 against 2.76 ms
// for the mode at XPL 1), so u8 takes pyramid3_u8_kernel (packed bytes) and XPL is 1 here.
template <typename T>
constexpr int kPyrXpl = 1;

template <typename T, int NL, bool VEC, bool MODE = false>
__global__ __launch_bounds__(256) void pyramid3_fused_kernel(const T* __restrict__ in,
                                                             T* __restrict__ l1,
                                                             T* __restrict__ l2,
                                                             T* __restrict__ l3, PyrParams p) {
    constexpr int X = kPyrXpl<T>;  // level-3 columns per lane
    __shared__ T lds2[4][64][2 * X];
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int dz = w >> 1, dy = w & 1;
    const int64_t x3 = ((int64_t)blockIdx.x * 64 + lane) * X;  // first level-3 column
    const int64_t by = blockIdx.y;
    const int64_t n0y = p.s[0][1], n0x = p.s[0][2];
    const int64_t n1z = p.s[1][0], n1y = p.s[1][1], n1x = p.s[1][2];
    const int64_t n2z = p.s[2][0], n2y = p.s[2][1], n2x = p.s[2][2];
    const int64_t nz1blocks = (n1z + 3) / 4;
    for (int64_t bz = blockIdx.z; bz < nz1blocks; bz += gridDim.z) {
        // level-0 block rows: z0 = 8 bz + 4 dz + a, y0 = 8 by + 4 dy + b, x0 = 8 x3 + c; all 16
        // rows are loaded before any is used (16 loads in flight per lane), kept packed
        typedef T V8 __attribute__((ext_vector_type(8 * X)));
        V8 v[4][4];
        const int64_t z0b = 8 * bz + 4 * dz, y0b = 8 * by + 4 * dy, x0b = 8 * x3;
        const bool xfull = x0b + 8 * X <= n0x;
#pragma unroll
        for (int a = 0; a < 4; ++a)
#pragma unroll
            for (int b = 0; b < 4; ++b) {
                const int64_t z0 = z0b + a, y0 = y0b + b;
                const bool rok = z0 < p.s[0][0] && y0 < n0y;  // wave-uniform
                const T* row = in + (z0 * n0y + y0) * n0x + x0b;
                if (VEC && rok && xfull) {
                    v[a][b] = *reinterpret_cast<const V8*>(row);
                } else {
#pragma unroll
                    for (int c = 0; c < 8 * X; ++c) v[a][b][c] = (rok && x0b + c < n0x) ? row[c] : T(0);
                }
            }
        // level 1: the 2 x 2 x 4X block z1 = 4 bz + 2 dz + i, y1 = 4 by + 2 dy + j, x1 = 4 x3 + k
        T u1[2][2][4 * X];
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
            for (int j = 0; j < 2; ++j)
#pragma unroll
                for (int k = 0; k < 4 * X; ++k) {
                    const T t[8] = {v[2 * i][2 * j][2 * k],     v[2 * i][2 * j][2 * k + 1],
                                    v[2 * i][2 * j + 1][2 * k], v[2 * i][2 * j + 1][2 * k + 1],
                                    v[2 * i + 1][2 * j][2 * k], v[2 * i + 1][2 * j][2 * k + 1],
                                    v[2 * i + 1][2 * j + 1][2 * k],
                                    v[2 * i + 1][2 * j + 1][2 * k + 1]};
                    u1[i][j][k] = pyr_reduce8<T, MODE>(t);
                }
        const int64_t z1b = 4 * bz + 2 * dz, y1b = 4 * by + 2 * dy, x1b = 4 * x3;
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
            for (int j = 0; j < 2; ++j) {
                const int64_t z1 = z1b + i, y1 = y1b + j;
                if (z1 >= n1z || y1 >= n1y) continue;  // wave-uniform
                T* o = l1 + (z1 * n1y + y1) * n1x + x1b;
                if constexpr (VEC) {
                    typedef T V4 __attribute__((ext_vector_type(4 * X)));
                    if (x1b + 4 * X <= n1x) {
                        V4 q;
#pragma unroll
                        for (int k = 0; k < 4 * X; ++k) q[k] = u1[i][j][k];
                        *reinterpret_cast<V4*>(o) = q;
                        continue;
                    }
                }
#pragma unroll
                for (int k = 0; k < 4 * X; ++k)
                    if (x1b + k < n1x) o[k] = u1[i][j][k];
            }
        // level 2: z2 = 2 bz + dz, y2 = 2 by + dy, x2 = 2 x3 + m
        T u2[2 * X];
#pragma unroll
        for (int m = 0; m < 2 * X; ++m) {
            const T t[8] = {u1[0][0][2 * m], u1[0][0][2 * m + 1], u1[0][1][2 * m],
                            u1[0][1][2 * m + 1], u1[1][0][2 * m], u1[1][0][2 * m + 1],
                            u1[1][1][2 * m], u1[1][1][2 * m + 1]};
            u2[m] = pyr_reduce8<T, MODE>(t);
        }
        const int64_t z2 = 2 * bz + dz, y2 = 2 * by + dy, x2 = 2 * x3;
        if (z2 < n2z && y2 < n2y) {
            T* o = l2 + (z2 * n2y + y2) * n2x + x2;
#pragma unroll
            for (int m = 0; m < 2 * X; ++m)
                if (x2 + m < n2x) o[m] = u2[m];
        }
        if constexpr (NL == 3) {
#pragma unroll
            for (int m = 0; m < 2 * X; ++m) lds2[w][lane][m] = u2[m];
            __syncthreads();
            if (w == 0) {
#pragma unroll
                for (int q = 0; q < X; ++q) {
                    const T t[8] = {lds2[0][lane][2 * q], lds2[0][lane][2 * q + 1],
                                    lds2[1][lane][2 * q], lds2[1][lane][2 * q + 1],
                                    lds2[2][lane][2 * q], lds2[2][lane][2 * q + 1],
                                    lds2[3][lane][2 * q], lds2[3][lane][2 * q + 1]};
                    const T u3 = pyr_reduce8<T, MODE>(t);
                    if (bz < p.s[3][0] && by < p.s[3][1] && x3 + q < p.s[3][2])
                        l3[(bz * p.s[3][1] + by) * p.s[3][2] + x3 + q] = u3;
                }
            }
            __syncthreads();
        }
    }
}

// The u8 / bool / i8 pyramids: the same walk with 16-byte level-0 rows per lane (two level-3
// columns: one KiB per wave-instruction, as the u16 rows), the bytes kept packed. Every window
// reduction takes two neighbouring windows at once from four 32-bit words: window "lo" is bytes
// 0 and 1 of each word, window "hi" bytes 2 and 3 (each word one row of the 2x2x2 window, two x),
// and returns the two results in bytes 0 and 2 of one word.
//  * mean (downsample.rs:72-97): sum / 8 truncated, the exact f64 sum / 8 `as u8` / `as i8`
//    (pyr_mean8); each pair of bytes summed by v_dot4_u32_u8 (i8: v_dot4_i32_i8) against a
//    0x0101 byte mask (no byte extraction).
//  * mode (downsample.rs:99-120, ties to the smallest value as pyr_mode8): the 8 values of both
//    windows as packed 16-bit lanes (v_pk_min_u16 / v_pk_max_u16 sorting network, one issue for
//    both windows), inverted (255 - v) so that one packed max over the keys run * 256 + (255 - v)
//    of the sorted runs picks the longest run and, among equal runs, the smallest value (i8:
//    biased by 0x80 first, so the unsigned order is the signed one).
//    ~44 VALU per window against ~75 for pyr_mode8 on one window.
typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ u16x2 as_u16x2(uint32_t w) { return __builtin_bit_cast(u16x2, w); }
__device__ __forceinline__ uint32_t as_u32(u16x2 v) { return __builtin_bit_cast(uint32_t, v); }

template <bool MODE, bool SGN>
__device__ __forceinline__ uint32_t pyr_u8_pair(const uint32_t (&w)[4]) {
    if constexpr (!MODE && SGN) {
        // i8: v_dot4_i32_i8, then / 8 truncating toward zero (`as i8` of the exact f64 mean)
        int lo = 0, hi = 0;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            lo = __builtin_amdgcn_sdot4((int)w[r], 0x00000101, lo, false);
            hi = __builtin_amdgcn_sdot4((int)w[r], 0x01010000, hi, false);
        }
        return ((uint32_t)(lo / 8) & 0xFFu) | (((uint32_t)(hi / 8) & 0xFFu) << 16);
    } else if constexpr (!MODE) {
        uint32_t lo = 0, hi = 0;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            lo = __builtin_amdgcn_udot4(w[r], 0x00000101u, lo, false);
            hi = __builtin_amdgcn_udot4(w[r], 0x01010000u, hi, false);
        }
        return (lo >> 3) | ((hi >> 3) << 16);
    } else {
        // i8: the bias v ^ 0x80 maps the signed order onto the unsigned one
        constexpr uint32_t kBias = SGN ? 0x80808080u : 0u;
        u16x2 s[8];  // inverted values: lane 0 window lo, lane 1 window hi
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const uint32_t iw = ~(w[r] ^ kBias);
            s[2 * r] = as_u16x2(__builtin_amdgcn_perm(0u, iw, 0x0c020c00u));      // bytes 0, 2
            s[2 * r + 1] = as_u16x2(__builtin_amdgcn_perm(0u, iw, 0x0c030c01u));  // bytes 1, 3
        }
        auto cx = [&](int i, int j) {
            const u16x2 lo = __builtin_elementwise_min(s[i], s[j]);
            const u16x2 hi = __builtin_elementwise_max(s[i], s[j]);
            s[i] = lo;
            s[j] = hi;
        };
        cx(0, 2); cx(1, 3); cx(4, 6); cx(5, 7);
        cx(0, 4); cx(1, 5); cx(2, 6); cx(3, 7);
        cx(0, 1); cx(2, 3); cx(4, 5); cx(6, 7);
        cx(2, 4); cx(3, 5);
        cx(1, 4); cx(3, 6);
        cx(1, 2); cx(3, 4); cx(5, 6);
        // run = length of the run of equal values ending at i; key = run * 256 + (255 - v)
        const u16x2 one = {1, 1}, k256 = {256, 256};
        u16x2 run = one;
        u16x2 best = s[0] + k256;
#pragma unroll
        for (int i = 1; i < 8; ++i) {
            const u16x2 eq = __builtin_elementwise_sub_sat(one, s[i] - s[i - 1]);  // 1 iff equal
            run = run * eq + one;
            best = __builtin_elementwise_max(best, run * k256 + s[i]);
        }
        return (~as_u32(best) & 0x00FF00FFu) ^ (kBias & 0x00FF00FFu);  // 255 - (255 - v), unbiased
    }
}

template <int NL, bool VEC, bool MODE, bool SGN>
__global__ __launch_bounds__(256) void pyramid3_u8_kernel(const uint8_t* __restrict__ in,
                                                          uint8_t* __restrict__ l1,
                                                          uint8_t* __restrict__ l2,
                                                          uint8_t* __restrict__ l3,
                                                          PyrParams p) {
    __shared__ uint32_t lds2[4][64];  // a lane's 4 level-2 values, packed
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int dz = w >> 1, dy = w & 1;
    const int64_t x3 = ((int64_t)blockIdx.x * 64 + lane) * 2;  // first of 2 level-3 columns
    const int64_t by = blockIdx.y;
    const int64_t n0y = p.s[0][1], n0x = p.s[0][2];
    const int64_t n1z = p.s[1][0], n1y = p.s[1][1], n1x = p.s[1][2];
    const int64_t n2z = p.s[2][0], n2y = p.s[2][1], n2x = p.s[2][2];
    const int64_t nz1blocks = (n1z + 3) / 4;
    // bytes 0 and 2 of two pair results -> one word of 4 consecutive outputs
    auto join = [](uint32_t r0, uint32_t r1) { return __builtin_amdgcn_perm(r1, r0, 0x06040200u); };
    for (int64_t bz = blockIdx.z; bz < nz1blocks; bz += gridDim.z) {
        uint32_t v[4][4][4];  // level-0 rows z0b + a, y0b + b: 16 bytes x0b .. x0b + 15
        const int64_t z0b = 8 * bz + 4 * dz, y0b = 8 * by + 4 * dy, x0b = 8 * x3;
        const bool xfull = x0b + 16 <= n0x;
#pragma unroll
        for (int a = 0; a < 4; ++a)
#pragma unroll
            for (int b = 0; b < 4; ++b) {
                const int64_t z0 = z0b + a, y0 = y0b + b;
                const bool rok = z0 < p.s[0][0] && y0 < n0y;  // wave-uniform
                const uint8_t* row = in + (z0 * n0y + y0) * n0x + x0b;
                if (VEC && rok && xfull) {
                    const uint4 q = *reinterpret_cast<const uint4*>(row);
                    v[a][b][0] = q.x; v[a][b][1] = q.y; v[a][b][2] = q.z; v[a][b][3] = q.w;
                } else {
#pragma unroll
                    for (int wd = 0; wd < 4; ++wd) {
                        uint32_t word = 0;
#pragma unroll
                        for (int c = 0; c < 4; ++c) {
                            const int64_t x = x0b + 4 * wd + c;
                            word |= (uint32_t)((rok && x < n0x) ? row[4 * wd + c] : 0) << (8 * c);
                        }
                        v[a][b][wd] = word;
                    }
                }
            }
        // level 1: z1 = 4 bz + 2 dz + i, y1 = 4 by + 2 dy + j, x1 = x1b + k (k < 8): word h of
        // u1[i][j] holds outputs 4h .. 4h + 3; outputs 2q, 2q + 1 come from level-0 word q
        uint32_t u1[2][2][2];
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
            for (int j = 0; j < 2; ++j) {
                uint32_t r[4];
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    const uint32_t win[4] = {v[2 * i][2 * j][q], v[2 * i][2 * j + 1][q],
                                             v[2 * i + 1][2 * j][q], v[2 * i + 1][2 * j + 1][q]};
                    r[q] = pyr_u8_pair<MODE, SGN>(win);
                }
                u1[i][j][0] = join(r[0], r[1]);
                u1[i][j][1] = join(r[2], r[3]);
            }
        const int64_t z1b = 4 * bz + 2 * dz, y1b = 4 * by + 2 * dy, x1b = 4 * x3;
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
            for (int j = 0; j < 2; ++j) {
                const int64_t z1 = z1b + i, y1 = y1b + j;
                if (z1 >= n1z || y1 >= n1y) continue;  // wave-uniform
                uint8_t* o = l1 + (z1 * n1y + y1) * n1x + x1b;
                if (VEC && x1b + 8 <= n1x) {
                    *reinterpret_cast<uint2*>(o) = make_uint2(u1[i][j][0], u1[i][j][1]);
                } else {
#pragma unroll
                    for (int k = 0; k < 8; ++k)
                        if (x1b + k < n1x) o[k] = (uint8_t)(u1[i][j][k >> 2] >> (8 * (k & 3)));
                }
            }
        // level 2: z2 = 2 bz + dz, y2 = 2 by + dy, x2 = x2b + m (m < 4), packed in one word;
        // outputs 2h, 2h + 1 come from level-1 word h
        uint32_t r2[2];
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            const uint32_t win[4] = {u1[0][0][h], u1[0][1][h], u1[1][0][h], u1[1][1][h]};
            r2[h] = pyr_u8_pair<MODE, SGN>(win);
        }
        const uint32_t u2 = join(r2[0], r2[1]);
        const int64_t z2 = 2 * bz + dz, y2 = 2 * by + dy, x2 = 2 * x3;
        if (z2 < n2z && y2 < n2y) {
            uint8_t* o = l2 + (z2 * n2y + y2) * n2x + x2;
#pragma unroll
            for (int m = 0; m < 4; ++m)
                if (x2 + m < n2x) o[m] = (uint8_t)(u2 >> (8 * m));
        }
        if constexpr (NL == 3) {
            lds2[w][lane] = u2;
            __syncthreads();
            if (w == 0) {
                // level 3 x3 + q: level-2 outputs 2q, 2q + 1 of the four waves' words
                const uint32_t win[4] = {lds2[0][lane], lds2[1][lane], lds2[2][lane], lds2[3][lane]};
                const uint32_t r3 = pyr_u8_pair<MODE, SGN>(win);
#pragma unroll
                for (int q = 0; q < 2; ++q)
                    if (bz < p.s[3][0] && by < p.s[3][1] && x3 + q < p.s[3][2])
                        l3[(bz * p.s[3][1] + by) * p.s[3][2] + x3 + q] = (uint8_t)(r3 >> (16 * q));
            }
            __syncthreads();
        }
    }
}

template <typename T, bool MODE>
static hipError_t launch_pyr_fused_t(const void* in, void* const* outs, const PyrParams& p,
                                     int nl, hipStream_t s) {
    if constexpr (sizeof(T) == 1) {  // u8, bool, i8: packed bytes
        constexpr bool SGN = std::is_signed<T>::value;
        const int64_t gx = (p.s[1][2] + 511) / 512, gy = (p.s[1][1] + 3) / 4;
        const int64_t gz = std::min<int64_t>((p.s[1][0] + 3) / 4, 128);
        if (gx > 0x7FFFFFFF || gy > 65535) return hipErrorInvalidValue;  // pyramid_fused_grid_fits
        const bool vec = p.s[0][2] % 16 == 0 && (uintptr_t)in % 16 == 0 &&
                         (uintptr_t)outs[0] % 8 == 0 && p.s[1][2] % 8 == 0;
        const dim3 grid((unsigned)gx, (unsigned)gy, (unsigned)gz);
        const uint8_t* i = static_cast<const uint8_t*>(in);  // i8 as its bytes
        uint8_t* o1 = static_cast<uint8_t*>(outs[0]);
        uint8_t* o2 = static_cast<uint8_t*>(outs[1]);
        uint8_t* o3 = nl == 3 ? static_cast<uint8_t*>(outs[2]) : nullptr;
        if (nl == 3) {
            if (vec) hipLaunchKernelGGL((pyramid3_u8_kernel<3, true, MODE, SGN>), grid, dim3(256), 0, s, i, o1, o2, o3, p);
            else hipLaunchKernelGGL((pyramid3_u8_kernel<3, false, MODE, SGN>), grid, dim3(256), 0, s, i, o1, o2, o3, p);
        } else {
            if (vec) hipLaunchKernelGGL((pyramid3_u8_kernel<2, true, MODE, SGN>), grid, dim3(256), 0, s, i, o1, o2, o3, p);
            else hipLaunchKernelGGL((pyramid3_u8_kernel<2, false, MODE, SGN>), grid, dim3(256), 0, s, i, o1, o2, o3, p);
        }
        return hipGetLastError();
    }
    constexpr int X = kPyrXpl<T>;
    const int64_t gx = (p.s[1][2] + 256 * X - 1) / (256 * X), gy = (p.s[1][1] + 3) / 4;
    // z capped at 128 workgroup layers, each workgroup looping over level-1 z blocks: 4096^3 u16
    // levels 1-3 in 29.2 ms against 31.8 ms for one layer per z block (tools/timepyr.hip)
    const int64_t gz = std::min<int64_t>((p.s[1][0] + 3) / 4, 128);
    if (gx > 0x7FFFFFFF || gy > 65535) return hipErrorInvalidValue;  // pyramid_fused_grid_fits
    const bool vec = p.s[0][2] % (8 * X) == 0 && (uintptr_t)in % (8 * X * sizeof(T)) == 0 &&
                     (uintptr_t)outs[0] % (4 * X * sizeof(T)) == 0 && p.s[1][2] % (4 * X) == 0;
    const dim3 grid((unsigned)gx, (unsigned)gy, (unsigned)gz);
    const T* i = static_cast<const T*>(in);
    T* o1 = static_cast<T*>(outs[0]);
    T* o2 = static_cast<T*>(outs[1]);
    T* o3 = nl == 3 ? static_cast<T*>(outs[2]) : nullptr;
    if (nl == 3) {
        if (vec) hipLaunchKernelGGL((pyramid3_fused_kernel<T, 3, true, MODE>), grid, dim3(256), 0, s, i, o1, o2, o3, p);
        else hipLaunchKernelGGL((pyramid3_fused_kernel<T, 3, false, MODE>), grid, dim3(256), 0, s, i, o1, o2, o3, p);
    } else {
        if (vec) hipLaunchKernelGGL((pyramid3_fused_kernel<T, 2, true, MODE>), grid, dim3(256), 0, s, i, o1, o2, o3, p);
        else hipLaunchKernelGGL((pyramid3_fused_kernel<T, 2, false, MODE>), grid, dim3(256), 0, s, i, o1, o2, o3, p);
    }
    return hipGetLastError();
}

// 3-D 2x2x2 mode (downsample.rs:99-120) for the per-level launches: one output per thread on an
// (x, y, z) grid (no 64-bit index divisions, unlike the N-d kernel), the window's 8 values in
// registers (pyr_mode8).
template <typename TIn, typename TOut>
__global__ __launch_bounds__(256) void downsample3_mode_kernel(const TIn* __restrict__ in,
                                                               TOut* __restrict__ out,
                                                               DSParams p) {
    const int64_t onx = p.out_shape[2], ony = p.out_shape[1], onz = p.out_shape[0];
    const int64_t inx = p.in_shape[2], iny = p.in_shape[1];
    const int64_t x = (int64_t)blockIdx.x * 256 + threadIdx.x, y = blockIdx.y;
    if (x >= onx) return;
    for (int64_t z = blockIdx.z; z < onz; z += gridDim.z) {
        const TIn* src = in + ((z * 2) * iny + y * 2) * inx + x * 2;
        const TIn t[8] = {src[0], src[1], src[inx], src[inx + 1], src[iny * inx],
                          src[iny * inx + 1], src[(iny + 1) * inx], src[(iny + 1) * inx + 1]};
        const TIn best = pyr_mode8<TIn>(t);
        out[(z * ony + y) * onx + x] = int_as<TOut>(best);
    }
}

bool pyramid_fused_grid_fits(const int64_t* s1) {
    return (s1[2] + 255) / 256 <= 0x7FFFFFFF && (s1[1] + 3) / 4 <= 65535;
}

bool pyramid_fused_dtype(int dtype, bool discrete) {
    if (discrete)  // the mode needs Eq + Hash element types (downsample.rs:105): integers, bool
        return dtype == kBool || dtype == kU8 || dtype == kI8 || dtype == kU16 || dtype == kI16 ||
               dtype == kU32 || dtype == kI32 || dtype == kU64 || dtype == kI64;
    return dtype != kBF16 && dtype != kF16 && dtype_size(dtype) > 0;
}

hipError_t launch_pyramid_fused(const void* in, int dtype, const int64_t (*shapes)[3], int nl,
                                void* const* outs, bool discrete, hipStream_t s) {
    if (nl != 2 && nl != 3) return hipErrorInvalidValue;
    PyrParams p{};
    for (int l = 0; l <= nl; ++l)
        for (int d = 0; d < 3; ++d) p.s[l][d] = shapes[l][d];
    if (discrete) {
        switch (dtype) {
        case kBool: case kU8: return launch_pyr_fused_t<uint8_t, true>(in, outs, p, nl, s);
        case kI8: return launch_pyr_fused_t<int8_t, true>(in, outs, p, nl, s);
        case kI16: return launch_pyr_fused_t<int16_t, true>(in, outs, p, nl, s);
        case kU16: return launch_pyr_fused_t<uint16_t, true>(in, outs, p, nl, s);
        case kI32: return launch_pyr_fused_t<int32_t, true>(in, outs, p, nl, s);
        case kU32: return launch_pyr_fused_t<uint32_t, true>(in, outs, p, nl, s);
        case kI64: return launch_pyr_fused_t<int64_t, true>(in, outs, p, nl, s);
        case kU64: return launch_pyr_fused_t<uint64_t, true>(in, outs, p, nl, s);
        default: return hipErrorInvalidValue;
        }
    }
    switch (dtype) {
    case kBool: case kU8: return launch_pyr_fused_t<uint8_t, false>(in, outs, p, nl, s);
    case kI8: return launch_pyr_fused_t<int8_t, false>(in, outs, p, nl, s);
    case kI16: return launch_pyr_fused_t<int16_t, false>(in, outs, p, nl, s);
    case kU16: return launch_pyr_fused_t<uint16_t, false>(in, outs, p, nl, s);
    case kI32: return launch_pyr_fused_t<int32_t, false>(in, outs, p, nl, s);
    case kU32: return launch_pyr_fused_t<uint32_t, false>(in, outs, p, nl, s);
    case kI64: return launch_pyr_fused_t<int64_t, false>(in, outs, p, nl, s);
    case kU64: return launch_pyr_fused_t<uint64_t, false>(in, outs, p, nl, s);
    case kF32: return launch_pyr_fused_t<float, false>(in, outs, p, nl, s);
    case kF64: return launch_pyr_fused_t<double, false>(in, outs, p, nl, s);
    default: return hipErrorInvalidValue;
    }
}

template <typename TIn, typename TOut>
static hipError_t launch_ds_types(const void* in, void* out, const DSParams& p, bool discrete,
                                  hipStream_t s) {
    int64_t blocks64 = (p.out_numel + 255) / 256;
    int blocks = (int)(blocks64 > 256 * 64 ? 256 * 64 : (blocks64 < 1 ? 1 : blocks64));
    const TIn* i = static_cast<const TIn*>(in);
    TOut* o = static_cast<TOut*>(out);
    if (discrete) {
        if constexpr (std::is_integral<TIn>::value) {
            if (p.ndim == 3 && p.win[0] == 2 && p.win[1] == 2 && p.win[2] == 2 &&
                p.out_shape[1] <= 65535) {
                const int64_t gx = (p.out_shape[2] + 255) / 256, gy = p.out_shape[1];
                const int64_t gz = std::max<int64_t>(1, std::min<int64_t>(
                    {p.out_shape[0], (int64_t)65535, 262144 / std::max<int64_t>(1, gx * gy)}));
                hipLaunchKernelGGL((downsample3_mode_kernel<TIn, TOut>),
                                   dim3((unsigned)gx, (unsigned)gy, (unsigned)gz), dim3(256), 0, s,
                                   i, o, p);
            } else {
                hipLaunchKernelGGL((downsample_discrete_kernel<TIn, TOut>), dim3(blocks),
                                   dim3(256), 0, s, i, o, p);
            }
            return hipGetLastError();
        } else {
            return hipErrorInvalidValue;
        }
    }
    if (p.ndim == 3 && p.win[0] == 2 && p.win[1] == 2 && p.win[2] == 2 &&
        p.out_shape[1] <= 65535) {
        const int64_t gx = (p.out_shape[2] + 255) / 256, gy = p.out_shape[1];
        // about 256 K workgroups, z looped inside beyond that
        const int64_t gz = std::max<int64_t>(
            1, std::min<int64_t>({p.out_shape[0], (int64_t)65535, 262144 / std::max<int64_t>(1, gx * gy)}));
        hipLaunchKernelGGL((downsample3_kernel<TIn, TOut, 2, 2, 2>),
                           dim3((unsigned)gx, (unsigned)gy, (unsigned)gz), dim3(256), 0, s, i, o, p);
    } else {
        hipLaunchKernelGGL((downsample_continuous_kernel<TIn, TOut>), dim3(blocks), dim3(256), 0, s,
                           i, o, p);
    }
    return hipGetLastError();
}

hipError_t launch_downsample(const void* in, int dtype_in, void* out, int dtype_out,
                             const DSParams& p, bool discrete, hipStream_t s) {
    if (p.out_numel == 0) return hipSuccess;
    hipError_t err = hipErrorInvalidValue;
    ZT_DISPATCH_DTYPE(dtype_in, TI,
        ZT_DISPATCH_DTYPE(dtype_out, TO, err = (launch_ds_types<TI, TO>(in, out, p, discrete, s))))
    return err;
}

// ---------------------------------------------------------------------------------------------
// Synthetic inputs; identical to oracle_synth_* on the host.
// ---------------------------------------------------------------------------------------------
__device__ __forceinline__ uint64_t splitmix64(uint64_t x) {
    uint64_t z = x + 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

__global__ void synth_step_noise_kernel(float* __restrict__ out, int64_t n, int64_t plane,
                                        int64_t nx_row, int64_t nx_global, int64_t z0,
                                        uint64_t seed) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
         i += (int64_t)gridDim.x * blockDim.x) {
        int64_t gl = (z0 + i / plane) * plane + i % plane;
        int64_t x = i % nx_row;
        uint64_t h = splitmix64(seed ^ (uint64_t)gl);
        float U = (float)(h >> 40) * (1.0f / 16777216.0f);
        float t = __fmul_rn(100.0f, U);
        out[i] = __fadd_rn(t, x >= nx_global / 2 ? 500.0f : 0.0f);
    }
}

__global__ void synth_u16_kernel(uint16_t* __restrict__ out, int64_t n, int64_t plane, int64_t z0,
                                 uint64_t seed) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
         i += (int64_t)gridDim.x * blockDim.x) {
        int64_t gl = (z0 + i / plane) * plane + i % plane;
        uint64_t h = splitmix64(seed ^ (uint64_t)gl);
        out[i] = (uint16_t)(((h >> 40) * 65535ull) >> 24);
    }
}

// The box [start, start + shape) of an N-d global synthetic volume (kind 0: step+noise f32,
// kind 1: u16 noise): element values of the global linear index, as the whole-array generators.
struct SynthBox {
    int ndim;
    int64_t start[kMaxDims], shape[kMaxDims], gshape[kMaxDims];
};

__global__ void synth_box_kernel(void* __restrict__ out, int kind, int64_t n, SynthBox b,
                                 uint64_t seed) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
         i += (int64_t)gridDim.x * blockDim.x) {
        int64_t rem = i, gl = 0, mul = 1, gx = 0;
        for (int d = b.ndim - 1; d >= 0; --d) {
            const int64_t c = rem % b.shape[d] + b.start[d];
            rem /= b.shape[d];
            gl += c * mul;
            mul *= b.gshape[d];
            if (d == b.ndim - 1) gx = c;
        }
        const uint64_t h = splitmix64(seed ^ (uint64_t)gl);
        if (kind == 0) {
            const float U = (float)(h >> 40) * (1.0f / 16777216.0f);
            const float t = __fmul_rn(100.0f, U);
            static_cast<float*>(out)[i] =
                __fadd_rn(t, gx >= b.gshape[b.ndim - 1] / 2 ? 500.0f : 0.0f);
        } else {
            static_cast<uint16_t*>(out)[i] = (uint16_t)(((h >> 40) * 65535ull) >> 24);
        }
    }
}

hipError_t launch_synth_box(void* out, int kind, const int64_t* start, const int64_t* shape,
                            const int64_t* gshape, int ndim, uint64_t seed, hipStream_t s) {
    SynthBox b{};
    b.ndim = ndim;
    int64_t n = 1;
    for (int d = 0; d < ndim; ++d) {
        b.start[d] = start[d];
        b.shape[d] = shape[d];
        b.gshape[d] = gshape[d];
        n *= shape[d];
    }
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(synth_box_kernel, dim3(256 * 64), dim3(256), 0, s, out, kind, n, b, seed);
    return hipGetLastError();
}

hipError_t launch_synth_step_noise_f32(float* out, int64_t n, int64_t plane, int64_t nx_row,
                                       int64_t nx_global, int64_t z0, uint64_t seed,
                                       hipStream_t s) {
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(synth_step_noise_kernel, dim3(256 * 32), dim3(256), 0, s, out, n, plane,
                       nx_row, nx_global, z0, seed);
    return hipGetLastError();
}

hipError_t launch_synth_u16(uint16_t* out, int64_t n, int64_t plane, int64_t z0, uint64_t seed,
                            hipStream_t s) {
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(synth_u16_kernel, dim3(256 * 32), dim3(256), 0, s, out, n, plane, z0, seed);
    return hipGetLastError();
}

}  // namespace zt
