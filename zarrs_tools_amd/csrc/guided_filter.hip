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

std::atomic<int>& fused_variant() {
    static std::atomic<int> v{0};
    return v;
}
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
// Separable N-d path (ndim >= 4 or radius > kFusedMaxRadius): the same arithmetic as the fused
// kernel, one pass per axis through device scratch.
// ---------------------------------------------------------------------------------------------

// Gather the (strided, any dtype) block into a contiguous f32 buffer.
template <typename TIn>
__global__ void sep_load_kernel(const TIn* __restrict__ in, float* __restrict__ v, NdGeom g) {
    int64_t n = g.numel;
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
         i += (int64_t)gridDim.x * blockDim.x) {
        int64_t rem = i, off = 0;
        for (int d = g.ndim - 1; d >= 0; --d) {
            int64_t c = rem % g.shape[d];
            rem /= g.shape[d];
            off += c * g.in_strides[d];
        }
        v[i] = Elem<TIn>::to_f32(in[off]);
    }
}

// Window sum of src along `axis` (C-contiguous layout of g.shape), zero-padded outside, in the
// same binary-tree order as the fused kernel. `nsrc` sources are summed with the same rule.
template <int W>
__global__ void sep_box_axis_kernel(const float* __restrict__ src, float* __restrict__ dst,
                                    NdGeom g, int axis) {
    int64_t n = g.numel;
    int64_t stride = 1;
    for (int d = g.ndim - 1; d > axis; --d) stride *= g.shape[d];
    int len = (int)g.shape[axis];
    constexpr int R = (W - 1) / 2;
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
         i += (int64_t)gridDim.x * blockDim.x) {
        int c = (int)((i / stride) % len);
        float vin[W];
#pragma unroll
        for (int t = 0; t < W; ++t) {
            int cc = c - R + t;
            vin[t] = (cc >= 0 && cc < len) ? src[i + (int64_t)(cc - c) * stride] : 0.0f;
        }
        float o[1];
        tree_window_sums<R, 1>(vin, o);
        dst[i] = o[0];
    }
}

__device__ __forceinline__ float nd_count(int64_t i, const NdGeom& g, int r) {
    int64_t rem = i;
    int64_t cnt = 1;
    for (int d = g.ndim - 1; d >= 0; --d) {
        int c = (int)(rem % g.shape[d]);
        rem /= g.shape[d];
        cnt *= clamped_count(c, (int)g.shape[d], r);
    }
    return (float)cnt;
}

// u = S/cnt; s = (v-u)^2; a = s/(s+eps); b = (1-a)u  (guided_filter.rs:127-140)
__global__ void sep_pointwise_kernel(const float* __restrict__ v, const float* __restrict__ S,
                                     float* __restrict__ a_out, float* __restrict__ b_out,
                                     NdGeom g, int r, float eps) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < g.numel;
         i += (int64_t)gridDim.x * blockDim.x) {
        float u = S[i] / nd_count(i, g, r);
        float d = v[i] - u;
        float s = d * d;
        float a = s / (s + eps);
        a_out[i] = a;
        b_out[i] = (1.0f - a) * u;
    }
}

// out = v*(A/cnt) + B/cnt on the output region, cast to TOut (guided_filter.rs:144-163, :101-102)
template <typename TOut>
__global__ void sep_final_kernel(const float* __restrict__ v, const float* __restrict__ A,
                                 const float* __restrict__ B, TOut* __restrict__ out, NdGeom g,
                                 int r) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < g.out_numel;
         i += (int64_t)gridDim.x * blockDim.x) {
        int64_t rem = i, src = 0, dst = 0, mul = 1;
        for (int d = g.ndim - 1; d >= 0; --d) {
            int64_t c = rem % g.out_shape[d];
            rem /= g.out_shape[d];
            src += (c + g.out_start[d]) * mul;
            mul *= g.shape[d];
            dst += c * g.out_strides[d];
        }
        float cnt = nd_count(src, g, r);
        float ma = A[src] / cnt;
        float mb = B[src] / cnt;
        out[dst] = from_f32<TOut>(__fadd_rn(__fmul_rn(v[src], ma), mb));
    }
}

template <int W>
static void box_all_axes(float* buf, float* tmp, const NdGeom& g, hipStream_t s, int blocks) {
    // x (last axis) first, then towards axis 0, ping-ponging through tmp; result lands in buf.
    float* src = buf;
    float* dst = tmp;
    for (int axis = g.ndim - 1; axis >= 0; --axis) {
        hipLaunchKernelGGL(sep_box_axis_kernel<W>, dim3(blocks), dim3(256), 0, s, src, dst, g,
                           axis);
        float* t = src; src = dst; dst = t;
    }
    if (src != buf)
        (void)hipMemcpyAsync(buf, src, sizeof(float) * g.numel, hipMemcpyDeviceToDevice, s);
}

template <int R>
static hipError_t sep_boxes(float* S, float* tmp, float* A, float* B, const NdGeom& g,
                            hipStream_t s, int blocks, int which) {
    constexpr int W = 2 * R + 1;
    if (which == 0) box_all_axes<W>(S, tmp, g, s, blocks);
    else {
        box_all_axes<W>(A, tmp, g, s, blocks);
        box_all_axes<W>(B, tmp, g, s, blocks);
    }
    return hipGetLastError();
}

// Large radii (> kSepTreeMaxRadius): sequential left-to-right window sum.
__global__ void sep_box_axis_seq_kernel(const float* __restrict__ src, float* __restrict__ dst,
                                        NdGeom g, int axis, int R) {
    int64_t n = g.numel;
    int64_t stride = 1;
    for (int d = g.ndim - 1; d > axis; --d) stride *= g.shape[d];
    int len = (int)g.shape[axis];
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
         i += (int64_t)gridDim.x * blockDim.x) {
        int c = (int)((i / stride) % len);
        int lo = c - R < 0 ? 0 : c - R, hi = c + R > len - 1 ? len - 1 : c + R;
        float acc = 0.0f;
        for (int cc = lo; cc <= hi; ++cc) acc += src[i + (int64_t)(cc - c) * stride];
        dst[i] = acc;
    }
}

static void box_all_axes_seq(float* buf, float* tmp, const NdGeom& g, hipStream_t s, int blocks,
                             int R) {
    float* src = buf;
    float* dst = tmp;
    for (int axis = g.ndim - 1; axis >= 0; --axis) {
        hipLaunchKernelGGL(sep_box_axis_seq_kernel, dim3(blocks), dim3(256), 0, s, src, dst, g,
                           axis, R);
        float* t = src; src = dst; dst = t;
    }
    if (src != buf)
        (void)hipMemcpyAsync(buf, src, sizeof(float) * g.numel, hipMemcpyDeviceToDevice, s);
}

template <int R0 = 0>
static hipError_t sep_boxes_dispatch(int r, float* S, float* tmp, float* A, float* B,
                                     const NdGeom& g, hipStream_t s, int blocks, int which) {
    if constexpr (R0 > kSepTreeMaxRadius) {
        if (which == 0) box_all_axes_seq(S, tmp, g, s, blocks, r);
        else {
            box_all_axes_seq(A, tmp, g, s, blocks, r);
            box_all_axes_seq(B, tmp, g, s, blocks, r);
        }
        return hipGetLastError();
    } else {
        if (r == R0) return sep_boxes<R0>(S, tmp, A, B, g, s, blocks, which);
        return sep_boxes_dispatch<R0 + 1>(r, S, tmp, A, B, g, s, blocks, which);
    }
}

hipError_t launch_guided_separable(const void* in, int dtype_in, void* out, int dtype_out,
                                   const NdGeom& g, int radius, float eps, float* scratch,
                                   hipStream_t s) {
    // scratch: 5 * numel floats: v, S(then reused), A, B, tmp
    const int64_t n = g.numel;
    float* v = scratch;
    float* S = scratch + n;
    float* A = scratch + 2 * n;
    float* B = scratch + 3 * n;
    float* tmp = scratch + 4 * n;
    int blocks = (int)((n + 255) / 256);
    if (blocks > 256 * 16) blocks = 256 * 16;
    if (blocks < 1) blocks = 1;
    hipError_t err = hipErrorInvalidValue;
    ZT_DISPATCH_DTYPE(dtype_in, TI,
        hipLaunchKernelGGL(sep_load_kernel<TI>, dim3(blocks), dim3(256), 0, s,
                           static_cast<const TI*>(in), v, g);
        err = hipGetLastError())
    if (err != hipSuccess) return err;
    (void)hipMemcpyAsync(S, v, sizeof(float) * n, hipMemcpyDeviceToDevice, s);
    err = sep_boxes_dispatch(radius, S, tmp, A, B, g, s, blocks, 0);
    if (err != hipSuccess) return err;
    hipLaunchKernelGGL(sep_pointwise_kernel, dim3(blocks), dim3(256), 0, s, v, S, A, B, g,
                       radius, eps);
    err = sep_boxes_dispatch(radius, S, tmp, A, B, g, s, blocks, 1);
    if (err != hipSuccess) return err;
    int oblocks = (int)((g.out_numel + 255) / 256);
    if (oblocks > 256 * 16) oblocks = 256 * 16;
    if (oblocks < 1) oblocks = 1;
    err = hipErrorInvalidValue;
    ZT_DISPATCH_DTYPE(dtype_out, TO,
        hipLaunchKernelGGL(sep_final_kernel<TO>, dim3(oblocks), dim3(256), 0, s, v, A, B,
                           static_cast<TO*>(out), g, radius);
        err = hipGetLastError())
    return err;
}

}  // namespace zt
