// cast.hip — strided 3-D element conversions used to stage the element-type pairs that have no
// direct fused instantiation through f32 (Rust `as` semantics, zt_device.hpp).
#include <hip/hip_runtime.h>
#include <stdint.h>

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
