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
        // `TIn as TOut` for an integer TIn (downsample.rs:117): integer->integer wraps,
        // integer->float rounds to nearest.
        if constexpr (std::is_integral<TOut>::value) out[o] = (TOut)best;
        else out[o] = from_f64<TOut>((double)best);
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
            hipLaunchKernelGGL((downsample_discrete_kernel<TIn, TOut>), dim3(blocks), dim3(256), 0,
                               s, i, o, p);
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
