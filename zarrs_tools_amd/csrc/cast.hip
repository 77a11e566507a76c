// cast.hip — strided 3-D element conversions used to stage the element-type pairs that have no
// direct fused instantiation through f32 (Rust `as` semantics, zt_device.hpp).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <type_traits>

#include "zt_device.hpp"
#include "zt_kernels.hpp"

namespace zt {

template <typename T>
__global__ void cast_to_f32_3d_kernel(const T* __restrict__ in, int64_t sz, int64_t sy,
                                      float* __restrict__ out, int64_t nz, int64_t ny,
                                      int64_t nx) {
    const int64_t n = nz * ny * nx;
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
         i += (int64_t)gridDim.x * blockDim.x) {
        int64_t x = i % nx, t = i / nx, y = t % ny, z = t / ny;
        out[i] = Elem<T>::to_f32(in[z * sz + y * sy + x]);
    }
}

template <typename T>
__global__ void cast_from_f32_3d_kernel(const float* __restrict__ in, T* __restrict__ out,
                                        int64_t sz, int64_t sy, int64_t nz, int64_t ny,
                                        int64_t nx) {
    const int64_t n = nz * ny * nx;
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
         i += (int64_t)gridDim.x * blockDim.x) {
        int64_t x = i % nx, t = i / nx, y = t % ny, z = t / ny;
        out[z * sz + y * sy + x] = from_f32<T>(in[i]);
    }
}

// ---- Reencode's element conversion: TIn.as_() -> TOut for every pair (reencode.rs:58-77) -----
// num-traits 0.2.19 AsPrimitive and half 2.6.0's impls: a half type converts through f32 (to f64
// directly), any type converts to a half type through `as f32` and from_f32 (f64 through
// from_f64); float -> int saturates (NaN -> 0); int -> int wraps; int -> float rounds to nearest.
template <typename T> constexpr bool kIsHalf = std::is_same_v<T, bf16_t> || std::is_same_v<T, f16_t>;
template <typename T> constexpr bool kIsFloat = std::is_same_v<T, float> || std::is_same_v<T, double>;

template <typename TI, typename TO>
__device__ inline TO as_cast(TI v) {
    if constexpr (std::is_same_v<TI, TO>) {
        return v;
    } else if constexpr (kIsHalf<TI>) {
        if constexpr (std::is_same_v<TO, double>) return Elem<TI>::to_f64(v);
        else return as_cast<float, TO>(Elem<TI>::to_f32(v));
    } else if constexpr (kIsHalf<TO>) {
        if constexpr (std::is_same_v<TI, double>) return from_f64<TO>(v);
        else return from_f32<TO>(as_cast<TI, float>(v));
    } else if constexpr (kIsFloat<TI> && !kIsFloat<TO>) {
        if constexpr (std::is_same_v<TI, float>) return from_f32<TO>(v);
        else return from_f64<TO>(v);
    } else {
        return (TO)v;  // int -> int (two's complement wrap), int -> float (RNE), f32 <-> f64
    }
}

template <typename TI, typename TO>
__global__ void reencode_cast_kernel(const TI* __restrict__ in, TO* __restrict__ out, int64_t n) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
         i += (int64_t)gridDim.x * blockDim.x)
        out[i] = as_cast<TI, TO>(in[i]);
}

static int grid_for(int64_t n);

hipError_t launch_reencode_cast(const void* in, int dtype_in, void* out, int dtype_out, int64_t n,
                                hipStream_t s) {
    if (n == 0) return hipSuccess;
    hipError_t err = hipErrorInvalidValue;
    ZT_DISPATCH_DTYPE(dtype_in, TI,
        ZT_DISPATCH_DTYPE(dtype_out, TO,
            hipLaunchKernelGGL((reencode_cast_kernel<TI, TO>), dim3(grid_for(n)), dim3(256), 0, s,
                               static_cast<const TI*>(in), static_cast<TO*>(out), n);
            err = hipGetLastError()))
    return err;
}

static int grid_for(int64_t n) {
    int64_t b = (n + 255) / 256;
    return (int)(b > 256 * 64 ? 256 * 64 : (b < 1 ? 1 : b));
}

hipError_t launch_cast_to_f32_3d(const void* in, int dtype, int64_t sz, int64_t sy, float* out,
                                 int64_t nz, int64_t ny, int64_t nx, hipStream_t s) {
    if (nz * ny * nx == 0) return hipSuccess;
    hipError_t err = hipErrorInvalidValue;
    ZT_DISPATCH_DTYPE(dtype, T,
        hipLaunchKernelGGL(cast_to_f32_3d_kernel<T>, dim3(grid_for(nz * ny * nx)), dim3(256), 0, s,
                           static_cast<const T*>(in), sz, sy, out, nz, ny, nx);
        err = hipGetLastError())
    return err;
}

hipError_t launch_cast_from_f32_3d(const float* in, int dtype, void* out, int64_t sz, int64_t sy,
                                   int64_t nz, int64_t ny, int64_t nx, hipStream_t s) {
    if (nz * ny * nx == 0) return hipSuccess;
    hipError_t err = hipErrorInvalidValue;
    ZT_DISPATCH_DTYPE(dtype, T,
        hipLaunchKernelGGL(cast_from_f32_3d_kernel<T>, dim3(grid_for(nz * ny * nx)), dim3(256), 0,
                           s, in, static_cast<T*>(out), sz, sy, nz, ny, nx);
        err = hipGetLastError())
    return err;
}

}  // namespace zt
