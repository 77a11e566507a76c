// guided_filter.hip — MI355X (gfx950) guided filter for the zarrs_filter per-chunk path.
//
// Reference semantics (LDeakin/zarrs_tools 0.7.2, src/filter/filters/guided_filter.rs:117-164,
// SURVEY.md §0.1): with box_r(.) the mean over the window [i-r, i+r] clamped to the block
// (get_block :166-184, count = product of clamped extents, summed_area_table.rs:401-411):
//     u = box_r(v);  s = (v-u)^2;  a = s/(s+eps);  b = (1-a)*u;  out = v*box_r(a) + box_r(b)
// evaluated in f32 with two roundings in the last line (v *= mean(a); v += mean(b)).
//
// Design: one fused 2.5-D kernel. A workgroup owns a 64 x TY output tile and
// marches along z (the slowest axis) through one chunk's depth. Per z-step it
//   P1 updates a running z-window sum of v on the (64+4r) x (TY+4r) apron (global loads:
//      the entering slice z+r and the leaving slice z-r-1),
//   P2/P3 box-sum that plane in x then y through LDS -> U(z) on the (64+2r) x (TY+2r) apron,
//      and computes a, b pointwise there,
//   P4/P5 box-sum a and b in x then y -> per-slice sums on the 64 x TY tile, kept in a ring of
//      2r+1 slices in registers, and emits out(z-r) from the ring's z-window sum.
// HBM traffic is one read of v and one write of out per voxel (+ the xy apron, served by L2);
// no intermediate field ever leaves the CU. Windows that cross the block edge see zeros (LDS
// and ring are zero-padded) and divide by the clamped count, which is exactly the reference's
// clamped-window mean.
//
// Window sums along x and y use a fixed binary tree per output (pairs, quads, octets, ... plus
// the remainder of 2r+1), so each sum's rounding depends only on its 2r+1 inputs, never on the
// position inside the tile. The z-window of a and b is summed from the ring in the same tree
// order. Only the v z-window is a running (add entering / subtract leaving) f32 sum, restarted
// for every chunk-depth march.

#include <hip/hip_runtime.h>
#include <stdint.h>

#include <type_traits>

#include "zt_device.hpp"
#include "zt_kernels.hpp"
#include "gf_fused.hpp"

namespace zt {

bool fused_supports_radius(int radius) { return radius >= 0 && radius <= kFusedMaxRadius; }

int fused_tile_y(int radius) { return radius <= 4 ? 32 : 16; }  // must match gf_fused_r<R>.hip
bool fused_direct_pair(int dtype_in, int dtype_out) {
    return fused_fast_dtype(dtype_in) && fused_fast_dtype(dtype_out);
}

hipError_t launch_fused_radius_0(const GFParams&, int, int, hipStream_t);
hipError_t launch_fused_radius_1(const GFParams&, int, int, hipStream_t);
hipError_t launch_fused_radius_2(const GFParams&, int, int, hipStream_t);
hipError_t launch_fused_radius_3(const GFParams&, int, int, hipStream_t);
hipError_t launch_fused_radius_4(const GFParams&, int, int, hipStream_t);
hipError_t launch_fused_radius_5(const GFParams&, int, int, hipStream_t);
hipError_t launch_fused_radius_6(const GFParams&, int, int, hipStream_t);
hipError_t launch_fused_radius_7(const GFParams&, int, int, hipStream_t);
hipError_t launch_fused_radius_8(const GFParams&, int, int, hipStream_t);

hipError_t launch_guided_fused(const GFParams& p, int dtype_in, int dtype_out, int radius,
                               hipStream_t stream) {
    switch (radius) {
    case 0: return launch_fused_radius_0(p, dtype_in, dtype_out, stream);
    case 1: return launch_fused_radius_1(p, dtype_in, dtype_out, stream);
    case 2: return launch_fused_radius_2(p, dtype_in, dtype_out, stream);
    case 3: return launch_fused_radius_3(p, dtype_in, dtype_out, stream);
    case 4: return launch_fused_radius_4(p, dtype_in, dtype_out, stream);
    case 5: return launch_fused_radius_5(p, dtype_in, dtype_out, stream);
    case 6: return launch_fused_radius_6(p, dtype_in, dtype_out, stream);
    case 7: return launch_fused_radius_7(p, dtype_in, dtype_out, stream);
    case 8: return launch_fused_radius_8(p, dtype_in, dtype_out, stream);
    default: return hipErrorInvalidValue;
    }
}

// ---------------------------------------------------------------------------------------------
// Separable N-d path (ndim >= 4 or radius > kFusedMaxRadius): one window-sum pass per axis
// through device scratch, the reference's arithmetic with the fused kernel's precision rules.
//   stage 1: box sums of v in f64 (exact for f32 inputs; u = (f32)U / count bit-exact, as
//            the reference's f64 SAT), f64 scratch between passes;
//   stage 2: box sums of a and b with an f64 running sum per pass (exact), rounded to f32 once
//            per pass.
// Every pass is a running window sum over a segment of outputs per thread (add the entering
// element, subtract the leaving one: exact in f64), so a voxel is read (seg + 2r) / seg times
// per pass instead of 2r + 1. The last axis runs one thread per row segment; every other axis
// runs one thread per (outer, segment, inner) with inner (the contiguous positions) across the
// lanes, so loads coalesce. Index math is per block / per thread, never per element.
// ---------------------------------------------------------------------------------------------

constexpr int kSepSeg = 32;   // outputs per thread along the summed axis
constexpr int kSepNT = 256;   // threads per block

template <typename TS, typename TD>
__global__ __launch_bounds__(kSepNT) void nd_col_box_kernel(const TS* __restrict__ src,
                                                            TD* __restrict__ dst, int64_t outer,
                                                            int len, int64_t inner, int r,
                                                            int nseg, int64_t ntile) {
    // block -> (outer o, segment sg, inner tile it); all block-uniform
    const int64_t b = blockIdx.x;
    const int64_t it = b % ntile;
    const int64_t rest = b / ntile;
    const int sg = (int)(rest % nseg);
    const int64_t o = rest / nseg;
    const int64_t i = it * kSepNT + threadIdx.x;
    if (o >= outer || i >= inner) return;
    const int c0 = sg * kSepSeg, c1 = min(c0 + kSepSeg, len);
    const TS* col = src + o * (int64_t)len * inner + i;
    TD* dcol = dst + o * (int64_t)len * inner + i;
    double s = 0.0;
    const int lo = max(c0 - r, 0), hi = min(c0 + r, len - 1);
    for (int c = lo; c <= hi; ++c) s += (double)col[(int64_t)c * inner];
    dcol[(int64_t)c0 * inner] = (TD)s;
    for (int c = c0 + 1; c < c1; ++c) {
        if (c + r < len) s += (double)col[(int64_t)(c + r) * inner];
        if (c - r - 1 >= 0) s -= (double)col[(int64_t)(c - r - 1) * inner];
        dcol[(int64_t)c * inner] = (TD)s;
    }
}

template <typename TS, typename TD>
__global__ __launch_bounds__(kSepNT) void nd_row_box_kernel(const TS* __restrict__ src,
                                                            TD* __restrict__ dst, int64_t rows,
                                                            int len, int r, int nseg) {
    const int64_t t = blockIdx.x * (int64_t)kSepNT + threadIdx.x;
    if (t >= rows * nseg) return;
    const int64_t row = t / nseg;
    const int sg = (int)(t % nseg);
    const int c0 = sg * kSepSeg, c1 = min(c0 + kSepSeg, len);
    const TS* x = src + row * len;
    TD* d = dst + row * len;
    double s = 0.0;
    const int lo = max(c0 - r, 0), hi = min(c0 + r, len - 1);
    for (int c = lo; c <= hi; ++c) s += (double)x[c];
    d[c0] = (TD)s;
    for (int c = c0 + 1; c < c1; ++c) {
        if (c + r < len) s += (double)x[c + r];
        if (c - r - 1 >= 0) s -= (double)x[c - r - 1];
        d[c] = (TD)s;
    }
}

// Radii <= kSepDirectMaxR: direct (2R+1)-term f64 sums with no loop-carried dependence, so
// every load of a thread is independent and in flight together.
constexpr int kSepDirectMaxR = 8;
constexpr int kSepColK = 8;    // outputs per thread, column kernel (4-D T share: 4 -> 164.5 ms, 8 -> 154.8, 16 -> 165.6)
constexpr int kSepRowTile = 1024;  // outputs per block, row kernel (4 per thread)

// Column axis: a thread owns kSepColK consecutive outputs of one (outer, inner) column and loads
// their kSepColK + 2R inputs at once (lanes = consecutive inner positions: coalesced).
template <int R, typename TS, typename TD>
__global__ __launch_bounds__(kSepNT) void nd_col_box_direct_kernel(
    const TS* __restrict__ src, TD* __restrict__ dst, int64_t outer, int len, int64_t inner,
    int nseg, int64_t ntile) {
    const int64_t b = blockIdx.x;
    const int64_t it = b % ntile;
    const int64_t rest = b / ntile;
    const int sg = (int)(rest % nseg);
    const int64_t o = rest / nseg;
    const int64_t i = it * kSepNT + threadIdx.x;
    if (o >= outer || i >= inner) return;
    const int c0 = sg * kSepColK;
    const TS* col = src + o * (int64_t)len * inner + i;
    TD* dcol = dst + o * (int64_t)len * inner + i;
    double x[kSepColK + 2 * R];
#pragma unroll
    for (int j = 0; j < kSepColK + 2 * R; ++j) {
        const int c = c0 - R + j;
        x[j] = (c >= 0 && c < len) ? (double)col[(int64_t)c * inner] : 0.0;
    }
#pragma unroll
    for (int k = 0; k < kSepColK; ++k) {
        double s = x[k];
#pragma unroll
        for (int j = 1; j <= 2 * R; ++j) s += x[k + j];
        if (c0 + k < len) dcol[(int64_t)(c0 + k) * inner] = (TD)s;
    }
}

// Two adjacent inner elements per lane (V2 = float2: stage 2's interleaved (a, b); double2:
// stage 1's f64 sums): one 8- or 16-byte load per lane per row, two f64 sums.
template <int R, typename V2>
__global__ __launch_bounds__(kSepNT) void nd_col_box_pair_kernel(
    const V2* __restrict__ src, V2* __restrict__ dst, int64_t outer, int len,
    int64_t inner2, int nseg, int64_t ntile) {
    const int64_t b = blockIdx.x;
    const int64_t it = b % ntile;
    const int64_t rest = b / ntile;
    const int sg = (int)(rest % nseg);
    const int64_t o = rest / nseg;
    const int64_t i = it * kSepNT + threadIdx.x;
    if (o >= outer || i >= inner2) return;
    const int c0 = sg * kSepColK;
    const V2* col = src + o * (int64_t)len * inner2 + i;
    V2* dcol = dst + o * (int64_t)len * inner2 + i;
    double xa[kSepColK + 2 * R], xb[kSepColK + 2 * R];
#pragma unroll
    for (int j = 0; j < kSepColK + 2 * R; ++j) {
        const int c = c0 - R + j;
        V2 v;
        if (c >= 0 && c < len) v = col[(int64_t)c * inner2];
        else v.x = v.y = 0;
        xa[j] = (double)v.x;
        xb[j] = (double)v.y;
    }
#pragma unroll
    for (int k = 0; k < kSepColK; ++k) {
        double sa = xa[k], sb = xb[k];
#pragma unroll
        for (int j = 1; j <= 2 * R; ++j) {
            sa += xa[k + j];
            sb += xb[k + j];
        }
        if (c0 + k < len) {
            V2 o2;
            o2.x = (decltype(o2.x))sa;
            o2.y = (decltype(o2.y))sb;
            dcol[(int64_t)(c0 + k) * inner2] = o2;
        }
    }
}

// Last axis: a block stages kSepRowTile + 2R elements of one row in LDS (coalesced), then each
// thread sums the windows of 4 outputs from LDS. P interleaved components per element (P = 2:
// the (a, b) pairs of stage 2), each summed on its own.
template <int R, int P, typename TS, typename TD>
__global__ __launch_bounds__(kSepNT) void nd_row_box_direct_kernel(const TS* __restrict__ src,
                                                                   TD* __restrict__ dst,
                                                                   int len, int64_t ntx) {
    __shared__ double sh[(kSepRowTile + 2 * R) * P];
    const int64_t b = blockIdx.x;
    const int64_t row = b / ntx;
    const int c0 = (int)(b % ntx) * kSepRowTile;
    const TS* x = src + row * len * P;
    TD* d = dst + row * len * P;
    for (int j = threadIdx.x; j < (kSepRowTile + 2 * R) * P; j += kSepNT) {
        const int c = c0 - R + j / P;
        sh[j] = (c >= 0 && c < len) ? (double)x[(int64_t)c * P + j % P] : 0.0;
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < kSepRowTile * P / kSepNT; ++k) {
        const int e = threadIdx.x + k * kSepNT;  // element-component index in the tile
        const int t = e / P, comp = e % P;
        double s = sh[t * P + comp];
#pragma unroll
        for (int j = 1; j <= 2 * R; ++j) s += sh[(t + j) * P + comp];
        if (c0 + t < len) d[(int64_t)(c0 + t) * P + comp] = (TD)s;
    }
}

template <int R, typename TS, typename TD>
static hipError_t nd_box_axis_direct(const TS* src, TD* dst, int64_t outer, int len,
                                     int64_t inner, hipStream_t s) {
    if (inner <= 2) {  // last axis (inner = the interleaved components)
        const int64_t ntx = (len + kSepRowTile - 1) / kSepRowTile;
        const int64_t nb = outer * ntx;
        if (nb > 0x7FFFFFFFLL) return hipErrorInvalidValue;
        if (inner == 1)
            hipLaunchKernelGGL((nd_row_box_direct_kernel<R, 1, TS, TD>), dim3((unsigned)nb),
                               dim3(kSepNT), 0, s, src, dst, len, ntx);
        else
            hipLaunchKernelGGL((nd_row_box_direct_kernel<R, 2, TS, TD>), dim3((unsigned)nb),
                               dim3(kSepNT), 0, s, src, dst, len, ntx);
    } else {
        const int nseg = (len + kSepColK - 1) / kSepColK;
        if constexpr (std::is_same<TS, TD>::value &&
                      (std::is_same<TS, float>::value || std::is_same<TS, double>::value)) {
            using V2 = typename std::conditional<std::is_same<TS, float>::value, float2,
                                                 double2>::type;
            if (inner % 2 == 0 && ((uintptr_t)src % sizeof(V2)) == 0 &&
                ((uintptr_t)dst % sizeof(V2)) == 0) {
                const int64_t inner2 = inner / 2;
                const int64_t ntile2 = (inner2 + kSepNT - 1) / kSepNT;
                const int64_t nb2 = outer * nseg * ntile2;
                if (nb2 > 0x7FFFFFFFLL) return hipErrorInvalidValue;
                hipLaunchKernelGGL((nd_col_box_pair_kernel<R, V2>), dim3((unsigned)nb2),
                                   dim3(kSepNT), 0, s, reinterpret_cast<const V2*>(src),
                                   reinterpret_cast<V2*>(dst), outer, len, inner2, nseg, ntile2);
                return hipGetLastError();
            }
        }
        const int64_t ntile = (inner + kSepNT - 1) / kSepNT;
        const int64_t nb = outer * nseg * ntile;
        if (nb > 0x7FFFFFFFLL) return hipErrorInvalidValue;
        hipLaunchKernelGGL((nd_col_box_direct_kernel<R, TS, TD>), dim3((unsigned)nb),
                           dim3(kSepNT), 0, s, src, dst, outer, len, inner, nseg, ntile);
    }
    return hipGetLastError();
}

template <int R0, typename TS, typename TD>
static hipError_t nd_box_axis_direct_dispatch(int r, const TS* src, TD* dst, int64_t outer,
                                              int len, int64_t inner, hipStream_t s) {
    if constexpr (R0 > kSepDirectMaxR) {
        return hipErrorInvalidValue;
    } else {
        if (r == R0) return nd_box_axis_direct<R0, TS, TD>(src, dst, outer, len, inner, s);
        return nd_box_axis_direct_dispatch<R0 + 1, TS, TD>(r, src, dst, outer, len, inner, s);
    }
}

// Window sums of src along `axis` of the C-contiguous array g.shape -> dst.
template <typename TS, typename TD>
static hipError_t nd_box_axis(const TS* src, TD* dst, const NdGeom& g, int axis, int r,
                              hipStream_t s, int P = 1) {
    const int len = (int)g.shape[axis];
    const int nseg = (len + kSepSeg - 1) / kSepSeg;
    int64_t inner = P, outer = 1;
    for (int d = axis + 1; d < g.ndim; ++d) inner *= g.shape[d];
    for (int d = 0; d < axis; ++d) outer *= g.shape[d];
    if (r <= kSepDirectMaxR)
        return nd_box_axis_direct_dispatch<0, TS, TD>(r, src, dst, outer, len, inner, s);
    if (inner == 1) {  // (P = 2 pairs take the column kernel with inner = 2 here: slow, rare)
        const int64_t nthr = outer * nseg;
        const int64_t nb = (nthr + kSepNT - 1) / kSepNT;
        if (nb > 0x7FFFFFFFLL) return hipErrorInvalidValue;
        hipLaunchKernelGGL((nd_row_box_kernel<TS, TD>), dim3((unsigned)nb), dim3(kSepNT), 0, s,
                           src, dst, outer, len, r, nseg);
    } else {
        const int64_t ntile = (inner + kSepNT - 1) / kSepNT;
        const int64_t nb = outer * nseg * ntile;
        if (nb > 0x7FFFFFFFLL) return hipErrorInvalidValue;
        hipLaunchKernelGGL((nd_col_box_kernel<TS, TD>), dim3((unsigned)nb), dim3(kSepNT), 0, s,
                           src, dst, outer, len, inner, r, nseg, ntile);
    }
    return hipGetLastError();
}

// Row-per-block helpers: a "row" is one index of every axis but the last. The row's coordinates
// and its window-count factor are block-uniform; threads walk the last axis.
struct RowCoord {
    int64_t c[kMaxDims];
};
__device__ __forceinline__ void row_coords(int64_t row, const int64_t* shape, int ndim,
                                           RowCoord& rc) {
    for (int d = ndim - 2; d >= 0; --d) {
        rc.c[d] = row % shape[d];
        row /= shape[d];
    }
}

// Gather the (strided, any dtype) block into a contiguous f32 buffer.
template <typename TIn>
__global__ __launch_bounds__(kSepNT) void sep_load_kernel(const TIn* __restrict__ in,
                                                          float* __restrict__ v, NdGeom g) {
    const int nd = g.ndim;
    const int64_t len = g.shape[nd - 1], rows = g.numel / len;
    for (int64_t row = blockIdx.x; row < rows; row += gridDim.x) {
        RowCoord rc;
        row_coords(row, g.shape, nd, rc);
        int64_t off = 0;
        for (int d = 0; d < nd - 1; ++d) off += rc.c[d] * g.in_strides[d];
        for (int64_t x = threadIdx.x; x < len; x += kSepNT)
            v[row * len + x] = Elem<TIn>::to_f32(in[off + x * g.in_strides[nd - 1]]);
    }
}

// u = (f32)U / count; s = (v-u)^2; a = s/(s+eps); b = (1-a)u   (guided_filter.rs:126-137,
// summed_area_table.rs:398-410)
__global__ __launch_bounds__(kSepNT) void sep_pointwise_kernel(const float* __restrict__ v,
                                                               const double* __restrict__ U,
                                                               float2* __restrict__ ab_out,
                                                               NdGeom g, int r, float eps) {
    const int nd = g.ndim;
    const int64_t len = g.shape[nd - 1], rows = g.numel / len;
    for (int64_t row = blockIdx.x; row < rows; row += gridDim.x) {
        RowCoord rc;
        row_coords(row, g.shape, nd, rc);
        int64_t cnt_row = 1;
        for (int d = 0; d < nd - 1; ++d) cnt_row *= clamped_count((int)rc.c[d], (int)g.shape[d], r);
        for (int64_t x = threadIdx.x; x < len; x += kSepNT) {
            const int64_t i = row * len + x;
            const float cnt = (float)(cnt_row * clamped_count((int)x, (int)len, r));
            const float u = (float)U[i] / cnt;
            const float d = v[i] - u;
            const float sq = d * d;
            const float a = sq / (sq + eps);
            ab_out[i] = make_float2(a, (1.0f - a) * u);
        }
    }
}

// out = v*(A/cnt) + B/cnt on the output region, cast to TOut (guided_filter.rs:144-163, :101-102)
template <typename TOut>
__global__ __launch_bounds__(kSepNT) void sep_final_kernel(const float* __restrict__ v,
                                                           const float2* __restrict__ AB,
                                                           TOut* __restrict__ out, NdGeom g,
                                                           int r) {
    const int nd = g.ndim;
    const int64_t olen = g.out_shape[nd - 1], orows = g.out_numel / olen;
    const int64_t len = g.shape[nd - 1];
    for (int64_t row = blockIdx.x; row < orows; row += gridDim.x) {
        RowCoord rc;
        row_coords(row, g.out_shape, nd, rc);
        int64_t src = 0, dst = 0, cnt_row = 1;
        for (int d = 0; d < nd - 1; ++d) {
            const int64_t c = rc.c[d] + g.out_start[d];
            src = src * g.shape[d] + c;
            dst += rc.c[d] * g.out_strides[d];
            cnt_row *= clamped_count((int)c, (int)g.shape[d], r);
        }
        src = src * len + g.out_start[nd - 1];
        for (int64_t x = threadIdx.x; x < olen; x += kSepNT) {
            const int64_t i = src + x;
            const int gx = (int)(x + g.out_start[nd - 1]);
            const float cnt = (float)(cnt_row * clamped_count(gx, (int)len, r));
            const float2 ab = AB[i];
            const float ma = ab.x / cnt;
            const float mb = ab.y / cnt;
            out[dst + x * g.out_strides[nd - 1]] = from_f32<TOut>(__fadd_rn(__fmul_rn(v[i], ma), mb));
        }
    }
}

// Box sums along every axis, last axis first (the order of the reference's SAT build is
// immaterial: f64 sums of f32 values are exact). Returns the buffer holding the result.
template <typename T0, typename T>
static hipError_t box_all_axes(const T0* src0, T* p0, T* p1, const NdGeom& g, int r,
                               hipStream_t s, T** result, int P = 1) {
    hipError_t e = nd_box_axis<T0, T>(src0, p0, g, g.ndim - 1, r, s, P);
    T* cur = p0;
    T* nxt = p1;
    for (int axis = g.ndim - 2; axis >= 0 && e == hipSuccess; --axis) {
        e = nd_box_axis<T, T>(cur, nxt, g, axis, r, s, P);
        T* t = cur; cur = nxt; nxt = t;
    }
    *result = cur;
    return e;
}

hipError_t launch_guided_separable(const void* in, int dtype_in, void* out, int dtype_out,
                                   const NdGeom& g, int radius, float eps, float* scratch,
                                   hipStream_t s) {
    // scratch: separable_scratch_floats(numel) = v (f32) | region X (2n floats) | region Y (2n
    // floats), with n padded to a multiple of 4 so X and Y are 16-byte aligned.
    // Stage 1 ping-pongs f64 sums between X and Y; a, b (and their pass ping-pong) then use the
    // region not holding U: A, B in it, A', B' in the other.
    const int64_t n = g.numel;
    if (n <= 0) return hipSuccess;
    float* v = scratch;
    const int64_t np = separable_pad(n);
    float* X = scratch + np;
    float* Y = scratch + 3 * np;
    const int64_t rows = n / g.shape[g.ndim - 1];
    const unsigned rblocks = (unsigned)std::min<int64_t>(rows, 1 << 20);
    // contiguous f32 input is used in place; anything else is gathered into v
    bool contiguous = dtype_in == kF32;
    {
        int64_t st = 1;
        for (int d = g.ndim - 1; d >= 0; --d) {
            if (g.in_strides[d] != st) contiguous = false;
            st *= g.shape[d];
        }
    }
    const float* vin = static_cast<const float*>(in);
    hipError_t err = hipSuccess;
    if (!contiguous) {
        err = hipErrorInvalidValue;
        ZT_DISPATCH_DTYPE(dtype_in, TI,
            hipLaunchKernelGGL(sep_load_kernel<TI>, dim3(rblocks), dim3(kSepNT), 0, s,
                               static_cast<const TI*>(in), v, g);
            err = hipGetLastError())
        if (err != hipSuccess) return err;
        vin = v;
    }
    double* U = nullptr;
    err = box_all_axes<float, double>(vin, reinterpret_cast<double*>(X),
                                      reinterpret_cast<double*>(Y), g, radius, s, &U);
    if (err != hipSuccess) return err;
    float* free_region = (reinterpret_cast<float*>(U) == X) ? Y : X;
    float* other = (free_region == X) ? Y : X;  // U's region: free once a, b are made
    float* AB = free_region;                    // (a, b) interleaved: 2n floats
    hipLaunchKernelGGL(sep_pointwise_kernel, dim3(rblocks), dim3(kSepNT), 0, s, vin, U,
                       reinterpret_cast<float2*>(AB), g, radius, eps);
    if ((err = hipGetLastError()) != hipSuccess) return err;
    float* ABr = nullptr;
    err = box_all_axes<float, float>(AB, other, AB, g, radius, s, &ABr, 2);
    if (err != hipSuccess) return err;
    const int64_t orows = g.out_numel / std::max<int64_t>(g.out_shape[g.ndim - 1], 1);
    if (g.out_numel <= 0) return hipSuccess;
    const unsigned oblocks = (unsigned)std::min<int64_t>(orows, 1 << 20);
    err = hipErrorInvalidValue;
    ZT_DISPATCH_DTYPE(dtype_out, TO,
        hipLaunchKernelGGL(sep_final_kernel<TO>, dim3(oblocks), dim3(kSepNT), 0, s, vin,
                           reinterpret_cast<const float2*>(ABr), static_cast<TO*>(out), g,
                           radius);
        err = hipGetLastError())
    return err;
}

}  // namespace zt
