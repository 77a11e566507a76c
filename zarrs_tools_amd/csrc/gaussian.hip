// gaussian.hip — separable Gaussian passes (gaussian.rs:110-119, kernel.rs:17-73).
//
// One launch per axis, in axis order, each an f32 sequential sum over the taps of
// input[min(sat_sub(k + i, mid), n - 1)] * tap[i] (replicate edges; no FMA: the translation unit
// is compiled with -ffp-contract=off), which is the reference's apply_1d_kernel operation for
// operation, so results are bit-identical. Pass d only computes what later passes read: the
// output range on axes <= d and the whole block on axes > d, so the region shrinks pass by pass
// (GaussPass: outer x n x inner input, outer x on x inner output, output k reads input o0 + k).
//
// HBM-bound in principle (4 B read + 4 B write per element per pass, taps re-read from L1/L2);
// one thread per output element, consecutive threads along the contiguous axis of the region.

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "zt_device.hpp"
#include "zt_kernels.hpp"

namespace zt {

template <typename TIn, typename IdxT>
__global__ __launch_bounds__(256) void gauss_pass_kernel(const TIn* __restrict__ in,
                                                         float* __restrict__ out, GaussPass p) {
    const IdxT inner = (IdxT)p.inner, on = (IdxT)p.on, n = (IdxT)p.n, o0 = (IdxT)p.o0;
    const IdxT total = (IdxT)p.outer * on * inner;
    const int len = p.len, mid = p.mid;
    for (IdxT e = blockIdx.x * (IdxT)blockDim.x + threadIdx.x; e < total;
         e += (IdxT)gridDim.x * blockDim.x) {
        const IdxT j = e % inner, t = e / inner;
        const IdxT k = t % on, o = t / on;
        const TIn* base = in + (o * n) * inner + j;
        const IdxT kin = o0 + k;
        float sum = -0.0f;  // Iterator::sum::<f32> (kernel.rs:46, :66)
        for (int i = 0; i < len; ++i) {
            IdxT q = kin + i - mid;  // min(sat_sub(k + i, mid), n - 1)
            q = q < 0 ? 0 : q;
            q = q > n - 1 ? n - 1 : q;
            sum = sum + Elem<TIn>::to_f32(base[q * inner]) * p.w[i];
        }
        out[e] = sum;
    }
}

static int gauss_grid(int64_t n) {
    int64_t b = (n + 255) / 256;
    return (int)(b < 65536 ? (b > 0 ? b : 1) : 65536);
}

hipError_t launch_gaussian_pass(const void* in, int dtype_in, float* out, const GaussPass& p,
                                hipStream_t s) {
    const int64_t total = p.outer * p.on * p.inner;
    if (total == 0) return hipSuccess;
    const bool small = p.outer * p.n * p.inner < (int64_t)INT32_MAX;
    hipError_t err = hipErrorInvalidValue;
    ZT_DISPATCH_DTYPE(dtype_in, T,
        if (small)
            hipLaunchKernelGGL((gauss_pass_kernel<T, int32_t>), dim3(gauss_grid(total)),
                               dim3(256), 0, s, static_cast<const T*>(in), out, p);
        else
            hipLaunchKernelGGL((gauss_pass_kernel<T, int64_t>), dim3(gauss_grid(total)),
                               dim3(256), 0, s, static_cast<const T*>(in), out, p);
        err = hipGetLastError())
    return err;
}

}  // namespace zt
