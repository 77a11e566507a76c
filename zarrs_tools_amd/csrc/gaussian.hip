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

// Threads along the contiguous axis of each pass: for axes with inner > 1 a thread owns one
// (outer, k) line position and consecutive threads consecutive inner offsets (coalesced tap
// reads, one stride of `inner` apart); for the last axis (inner == 1) consecutive threads own
// consecutive k and their tap windows overlap in L1. No integer division per element: the
// grid's y / z dimensions enumerate the other coordinates.
template <typename TIn, bool ALONG_K>
__global__ __launch_bounds__(256) void gauss_pass_kernel(const TIn* __restrict__ in,
                                                         float* __restrict__ out, GaussPass p) {
    const int64_t inner = p.inner, on = p.on, n = p.n, o0 = p.o0;
    const int len = p.len, mid = p.mid;
    const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    // rows enumerated by (blockIdx.y, blockIdx.z): (outer, k) pairs or outer lines
    const int64_t rows = ALONG_K ? p.outer : p.outer * on;
    for (int64_t r = (int64_t)blockIdx.z * gridDim.y + blockIdx.y; r < rows;
         r += (int64_t)gridDim.y * gridDim.z) {
        int64_t o, k, j;
        if constexpr (ALONG_K) {
            o = r;
            k = t;
            j = 0;
            if (k >= on) return;
        } else {
            o = r / on;  // one division per row, not per element
            k = r - o * on;
            j = t;
            if (j >= inner) return;
        }
        const TIn* base = in + (o * n) * inner + j;
        const int64_t kin = o0 + k;
        float sum = -0.0f;  // Iterator::sum::<f32> (kernel.rs:46, :66)
        // taps in groups of 8: the group's loads are all issued before its (in-order) sums
        for (int i0 = 0; i0 < len; i0 += 8) {
            float v[8];
#pragma unroll
            for (int u = 0; u < 8; ++u) {
                int64_t q = kin + i0 + u - mid;  // min(sat_sub(k + i, mid), n - 1)
                q = q < 0 ? 0 : q;
                q = q > n - 1 ? n - 1 : q;
                v[u] = i0 + u < len ? Elem<TIn>::to_f32(base[q * inner]) : 0.0f;
            }
#pragma unroll
            for (int u = 0; u < 8; ++u)
                if (i0 + u < len) sum = sum + v[u] * p.w[i0 + u];
        }
        out[(o * on + k) * inner + j] = sum;
    }
}

hipError_t launch_gaussian_pass(const void* in, int dtype_in, float* out, const GaussPass& p,
                                hipStream_t s) {
    if (p.outer * p.on * p.inner == 0) return hipSuccess;
    const bool along_k = p.inner == 1;
    const int64_t lanes = along_k ? p.on : p.inner;
    const int64_t rows = along_k ? p.outer : p.outer * p.on;
    const int64_t gx = (lanes + 255) / 256;
    if (gx > 0x7FFFFFFF) return hipErrorInvalidValue;
    const int64_t gy = rows < 65535 ? rows : 65535;
    const int64_t gzn = (rows + gy - 1) / gy;
    const int64_t gz = gzn < 65535 ? gzn : 65535;
    const dim3 grid((unsigned)gx, (unsigned)gy, (unsigned)gz);
    hipError_t err = hipErrorInvalidValue;
    ZT_DISPATCH_DTYPE(dtype_in, T,
        if (along_k)
            hipLaunchKernelGGL((gauss_pass_kernel<T, true>), grid, dim3(256), 0, s,
                               static_cast<const T*>(in), out, p);
        else
            hipLaunchKernelGGL((gauss_pass_kernel<T, false>), grid, dim3(256), 0, s,
                               static_cast<const T*>(in), out, p);
        err = hipGetLastError())
    return err;
}

}  // namespace zt
