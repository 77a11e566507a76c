// gaussian.hip — separable Gaussian passes (gaussian.rs:110-119, kernel.rs:17-73).
//
// One launch per axis, in axis order, each an f32 sequential sum over the taps of
// input[min(sat_sub(k + i, mid), n - 1)] * tap[i] (replicate edges; no FMA: the translation unit
// is compiled with -ffp-contract=off), which is the reference's apply_1d_kernel operation for
// operation, so results are bit-identical. Pass d only computes what later passes read: the
// output range on axes <= d and the whole block on axes > d, so the region shrinks pass by pass
// (GaussPass: outer x n x inner input, outer x on x inner output, output k reads input o0 + k).
//
// HBM-bound in principle (4 B read + 4 B write per element per pass): every pass stages its
// input windows in LDS so each element is fetched about once (column and row kernels below).

#include <hip/hip_runtime.h>

#include <cstdlib>
#include <stdint.h>

#include <algorithm>
#include <type_traits>

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

// Column passes (inner > 1): a thread owns one inner offset j and a segment of SEG consecutive
// outputs along the axis; it loads the segment's input window once (SEG + len - 1 values, in
// batches of 8 so the loads overlap) into its own LDS column and sums the taps from there, so
// each input is read about once from memory instead of len times. Only the owning thread
// touches its column: no barrier.
constexpr int kGaussSeg = 16, kGaussColMaxWin = 64;
template <typename TIn>
__global__ __launch_bounds__(256) void gauss_col_kernel(const TIn* __restrict__ in,
                                                        float* __restrict__ out, GaussPass p,
                                                        int64_t nseg) {
    extern __shared__ float win[];  // [window][256]
    const int tid = threadIdx.x, len = p.len, mid = p.mid;
    const int64_t inner = p.inner, on = p.on, n = p.n;
    const int64_t j = (int64_t)blockIdx.x * 256 + tid;
    const bool live = j < inner;
    for (int64_t r = (int64_t)blockIdx.z * gridDim.y + blockIdx.y; r < p.outer * nseg;
         r += (int64_t)gridDim.y * gridDim.z) {
        const int64_t o = r / nseg, s = r - o * nseg;  // uniform per block (scalar)
        const int64_t k0 = s * kGaussSeg;
        const int kc = (int)(on - k0 < kGaussSeg ? on - k0 : kGaussSeg);
        const int nw = kc + len - 1;
        const TIn* base = in + (o * n) * inner + (live ? j : 0);
        const int64_t q0 = p.o0 + k0 - mid;
        for (int w0 = 0; w0 < nw; w0 += 8) {
            float v[8];
#pragma unroll
            for (int u = 0; u < 8; ++u) {
                int64_t q = q0 + w0 + u;  // min(sat_sub(k + i, mid), n - 1)
                q = q < 0 ? 0 : (q > n - 1 ? n - 1 : q);
                v[u] = (w0 + u < nw) ? Elem<TIn>::to_f32(base[q * inner]) : 0.0f;
            }
#pragma unroll
            for (int u = 0; u < 8; ++u)
                if (w0 + u < nw) win[(w0 + u) * 256 + tid] = v[u];
        }
        if (live) {
            for (int kk = 0; kk < kc; ++kk) {
                float sum = -0.0f;  // Iterator::sum::<f32> (kernel.rs:46, :66)
                for (int i = 0; i < len; ++i) sum = sum + win[(kk + i) * 256 + tid] * p.w[i];
                out[(o * on + k0 + kk) * inner + j] = sum;
            }
        }
    }
}

// Row passes (inner == 1, the contiguous axis): a block stages 1024 outputs' input window of one
// line in LDS with coalesced loads, then each thread sums its outputs' taps from LDS.
constexpr int kGaussRowTile = 1024;
template <typename TIn>
__global__ __launch_bounds__(256) void gauss_row_kernel(const TIn* __restrict__ in,
                                                        float* __restrict__ out, GaussPass p) {
    extern __shared__ float tile[];  // kGaussRowTile + len - 1
    const int tid = threadIdx.x, len = p.len, mid = p.mid;
    const int64_t on = p.on, n = p.n;
    const int64_t k0 = (int64_t)blockIdx.x * kGaussRowTile;
    const int kc = (int)(on - k0 < kGaussRowTile ? on - k0 : kGaussRowTile);
    const int nw = kc + len - 1;
    for (int64_t o = (int64_t)blockIdx.z * gridDim.y + blockIdx.y; o < p.outer;
         o += (int64_t)gridDim.y * gridDim.z) {
        const TIn* line = in + o * n;
        const int64_t q0 = p.o0 + k0 - mid;
        __syncthreads();  // the previous line's tile is consumed
        for (int w = tid; w < nw; w += 256) {
            int64_t q = q0 + w;
            q = q < 0 ? 0 : (q > n - 1 ? n - 1 : q);
            tile[w] = Elem<TIn>::to_f32(line[q]);
        }
        __syncthreads();
        for (int kk = tid; kk < kc; kk += 256) {
            float sum = -0.0f;
            for (int i = 0; i < len; ++i) sum = sum + tile[kk + i] * p.w[i];
            out[o * on + k0 + kk] = sum;
        }
    }
}

// The y and x passes of one (outer) plane in one kernel: a block stages the input tile its
// 32 x 64 outputs need, with both coordinates clamped at load (clamping composes: the y pass at
// a clamped column is the y pass of that column), runs the y pass over the tile's columns into
// LDS and the x pass from there. Per element the products and their order are those of the two
// separate passes, so the result is identical; the intermediate never goes to memory.
constexpr int kYXTy = 32, kYXTx = 64;
template <typename TIn>
__global__ __launch_bounds__(256) void gauss_yx_kernel(const TIn* __restrict__ in,
                                                       float* __restrict__ out, int64_t outer,
                                                       GaussPass py, GaussPass px) {
    extern __shared__ float sm[];
    const int tid = threadIdx.x;
    const int ly = py.len, lx = px.len;
    const int th = kYXTy + ly - 1, tw = kYXTx + lx - 1;  // staged input tile
    float* tile = sm;                                     // [th][tw]
    float* ybuf = sm + th * tw;                           // [kYXTy][tw]
    const int64_t ny = py.n, nx = px.n, ony = py.on, onx = px.on;
    const int64_t y0 = (int64_t)blockIdx.y * kYXTy, x0 = (int64_t)blockIdx.x * kYXTx;
    const int hy = (int)(ony - y0 < kYXTy ? ony - y0 : kYXTy);
    const int hx = (int)(onx - x0 < kYXTx ? onx - x0 : kYXTx);
    for (int64_t o = blockIdx.z; o < outer; o += gridDim.z) {
        const TIn* plane = in + o * ny * nx;
        __syncthreads();  // the previous plane's tiles are consumed
        const int64_t qy0 = py.o0 + y0 - py.mid, qx0 = px.o0 + x0 - px.mid;
        for (int e = tid; e < th * tw; e += 256) {
            const int r = e / tw, c = e - r * tw;
            int64_t qy = qy0 + r, qx = qx0 + c;  // min(sat_sub(k + i, mid), n - 1)
            qy = qy < 0 ? 0 : (qy > ny - 1 ? ny - 1 : qy);
            qx = qx < 0 ? 0 : (qx > nx - 1 ? nx - 1 : qx);
            tile[e] = Elem<TIn>::to_f32(plane[qy * nx + qx]);
        }
        __syncthreads();
        for (int e = tid; e < kYXTy * tw; e += 256) {  // y pass
            const int r = e / tw, c = e - r * tw;
            float sum = -0.0f;
            for (int i = 0; i < ly; ++i) sum = sum + tile[(r + i) * tw + c] * py.w[i];
            ybuf[e] = sum;
        }
        __syncthreads();
        for (int e = tid; e < kYXTy * kYXTx; e += 256) {  // x pass
            const int r = e / kYXTx, c = e - r * kYXTx;
            if (r >= hy || c >= hx) continue;
            float sum = -0.0f;
            for (int i = 0; i < lx; ++i) sum = sum + ybuf[r * tw + c + i] * px.w[i];
            out[(o * ony + y0 + r) * onx + x0 + c] = sum;
        }
    }
}

// Same passes for f32 input and one odd tap count L on both axes (the common case): taps in
// registers, staging without divisions, and register windows — a thread makes 4 outputs of a
// column (y pass) or of a row (x pass) from 4 + L - 1 LDS reads instead of 4L. Every output is
// still sum = sum + x[i] * w[i] over i = 0..L-1 from -0.0, so the result is bit-identical.
constexpr int kYXFastTy = 32;  // output rows per block (measured 1024^3: 16 -> 3.86 ms, 32 -> 3.60, 64 -> 5.15)
template <int L>
__global__ __launch_bounds__(256) void gauss_yx_fast_kernel(const float* __restrict__ in,
                                                            float* __restrict__ out,
                                                            int64_t outer, GaussPass py,
                                                            GaussPass px) {
    constexpr int TY = kYXFastTy;
    constexpr int TH = TY + L - 1, TW = kYXTx + L - 1;
    __shared__ float tile[TH * TW];
    __shared__ float ybuf[TY * TW];
    const int tid = threadIdx.x;
    float wy[L], wx[L];
#pragma unroll
    for (int i = 0; i < L; ++i) {
        wy[i] = py.w[i];
        wx[i] = px.w[i];
    }
    const int64_t ny = py.n, nx = px.n, ony = py.on, onx = px.on;
    const int64_t y0 = (int64_t)blockIdx.y * TY, x0 = (int64_t)blockIdx.x * kYXTx;
    const int hy = (int)(ony - y0 < TY ? ony - y0 : TY);
    const int hx = (int)(onx - x0 < kYXTx ? onx - x0 : kYXTx);
    const int64_t qy0 = py.o0 + y0 - py.mid, qx0 = px.o0 + x0 - px.mid;
    const int tc = tid % 64, tr = tid / 64;  // staging: 4 rows x 64 columns per sweep
    int64_t qxa = qx0 + tc, qxb = qx0 + 64 + tc;
    qxa = qxa < 0 ? 0 : (qxa > nx - 1 ? nx - 1 : qxa);
    qxb = qxb < 0 ? 0 : (qxb > nx - 1 ? nx - 1 : qxb);
    for (int64_t o = blockIdx.z; o < outer; o += gridDim.z) {
        const float* plane = in + o * ny * nx;
        __syncthreads();  // the previous plane's tiles are consumed
        for (int r = tr; r < TH; r += 4) {
            int64_t qy = qy0 + r;
            qy = qy < 0 ? 0 : (qy > ny - 1 ? ny - 1 : qy);
            const float* row = plane + qy * nx;
            tile[r * TW + tc] = row[qxa];
            if (64 + tc < TW) tile[r * TW + 64 + tc] = row[qxb];
        }
        __syncthreads();
        for (int item = tid; item < TW * (TY / 4); item += 256) {  // y pass, 4 rows / item
            const int c = item % TW, r0 = (item / TW) * 4;
            float v[4 + L - 1];
#pragma unroll
            for (int j = 0; j < 4 + L - 1; ++j) v[j] = tile[(r0 + j) * TW + c];
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                float sum = -0.0f;
#pragma unroll
                for (int i = 0; i < L; ++i) sum = sum + v[k + i] * wy[i];
                ybuf[(r0 + k) * TW + c] = sum;
            }
        }
        __syncthreads();
        for (int item = tid; item < TY * (kYXTx / 4); item += 256) {  // x pass, 4 columns
            const int r = item / (kYXTx / 4), c0 = (item % (kYXTx / 4)) * 4;
            if (r >= hy || c0 >= hx) continue;
            float v[4 + L - 1];
#pragma unroll
            for (int j = 0; j < 4 + L - 1; ++j) v[j] = ybuf[r * TW + c0 + j];
            float o4[4];
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                float sum = -0.0f;
#pragma unroll
                for (int i = 0; i < L; ++i) sum = sum + v[k + i] * wx[i];
                o4[k] = sum;
            }
            float* dst = out + (o * ony + y0 + r) * onx + x0 + c0;
            if (c0 + 4 <= hx && ((uintptr_t)dst & 15) == 0) {
                *reinterpret_cast<float4*>(dst) = make_float4(o4[0], o4[1], o4[2], o4[3]);
            } else {
#pragma unroll
                for (int k = 0; k < 4; ++k)
                    if (c0 + k < hx) dst[k] = o4[k];
            }
        }
    }
}

template <int L>
static bool try_gauss_yx_fast(const void* in, int dtype_in, float* out, int64_t outer,
                              const GaussPass& py, const GaussPass& px, dim3 grid, hipStream_t s,
                              hipError_t& err) {
    if (dtype_in != kF32 || py.len != L || px.len != L) return false;
    const int64_t gy = (py.on + kYXFastTy - 1) / kYXFastTy;
    hipLaunchKernelGGL(gauss_yx_fast_kernel<L>, dim3(grid.x, (unsigned)gy, grid.z), dim3(256), 0, s,
                       static_cast<const float*>(in), out, outer, py, px);
    err = hipGetLastError();
    return true;
}

hipError_t launch_gaussian_yx(const void* in, int dtype_in, float* out, int64_t outer,
                              const GaussPass& py, const GaussPass& px, hipStream_t s) {
    if (outer * py.on * px.on == 0) return hipSuccess;
    if (py.len > kGaussYXMaxLen || px.len > kGaussYXMaxLen) return hipErrorInvalidValue;
    const int th = kYXTy + py.len - 1, tw = kYXTx + px.len - 1;
    const size_t lds = sizeof(float) * (size_t)(th * tw + kYXTy * tw);
    const int64_t gx = (px.on + kYXTx - 1) / kYXTx, gy = (py.on + kYXTy - 1) / kYXTy;
    if (gx > 0x7FFFFFFF || gy > 65535) return hipErrorInvalidValue;
    const dim3 grid((unsigned)gx, (unsigned)gy, (unsigned)(outer < 65535 ? outer : 65535));
    hipError_t err = hipErrorInvalidValue;
    if (try_gauss_yx_fast<3>(in, dtype_in, out, outer, py, px, grid, s, err) ||
        try_gauss_yx_fast<5>(in, dtype_in, out, outer, py, px, grid, s, err) ||
        try_gauss_yx_fast<7>(in, dtype_in, out, outer, py, px, grid, s, err) ||
        try_gauss_yx_fast<9>(in, dtype_in, out, outer, py, px, grid, s, err) ||
        try_gauss_yx_fast<11>(in, dtype_in, out, outer, py, px, grid, s, err) ||
        try_gauss_yx_fast<13>(in, dtype_in, out, outer, py, px, grid, s, err))
        return err;
    ZT_DISPATCH_DTYPE(dtype_in, T,
        hipLaunchKernelGGL(gauss_yx_kernel<T>, grid, dim3(256), lds, s, static_cast<const T*>(in),
                           out, outer, py, px);
        err = hipGetLastError())
    return err;
}

// ---------------------------------------------------------------------------------------------
// All three passes of a 3-D block in one z-march. A workgroup owns a 32 x 64 output tile of the
// (y, x) plane and a segment of output slices; each thread keeps, for its points of the staged
// (32 + L - 1) x (64 + L - 1) input tile (coordinates clamped as the y / x passes clamp), the L
// input slices of the current z window in registers (a ring whose slot of window position i is
// a compile-time constant: the march is unrolled by L), the next entering slice prefetched a step
// ahead. Per output slice: the z pass from the ring into LDS, then the y and x passes of
// gauss_yx_fast_kernel. Each element's sums are the reference's (sum = sum + x[i] * w[i] from
// -0.0, i ascending, no FMA), pass by pass in axis order, so the result is bit-identical to the
// three separate passes, with one read of the input and one write of the output per element.
// ---------------------------------------------------------------------------------------------
constexpr int kZYXTy = 32, kZYXTx = 64, kZYXSegMin = 32;

template <int B, int E, typename F>
__device__ __forceinline__ void static_for(F&& f) {
    if constexpr (B < E) {
        f(std::integral_constant<int, B>{});
        static_for<B + 1, E>(f);
    }
}

// Buffer (SRD) access for the march: the slice base goes in a wave-uniform descriptor, each
// point keeps a 32-bit byte offset, and an offset past num_records reads 0 / drops the store,
// so the march has no branches around its memory instructions: hipcc's vmcnt accounting then
// waits for exactly the step-old prefetch, instead of draining every load (a guarded prefetch
// and __syncthreads() each forced vmcnt(0) per step).
using zrsrc_t = __amdgpu_buffer_rsrc_t;
constexpr int kZBad = (int)0x80000000;
__device__ __forceinline__ zrsrc_t z_rsrc(const void* base, uint32_t bytes) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, (int)bytes,
                                             0x00020000);
}
template <typename T>
__device__ __forceinline__ float z_load(zrsrc_t r, int off) {
    if constexpr (sizeof(T) == 1) {
        const uint8_t b = __builtin_amdgcn_raw_buffer_load_b8(r, off, 0, 0);
        return Elem<T>::to_f32(__builtin_bit_cast(T, b));
    } else if constexpr (sizeof(T) == 2) {
        const uint16_t b = __builtin_amdgcn_raw_buffer_load_b16(r, off, 0, 0);
        return Elem<T>::to_f32(__builtin_bit_cast(T, b));
    } else if constexpr (sizeof(T) == 4) {
        const uint32_t b = __builtin_amdgcn_raw_buffer_load_b32(r, off, 0, 0);
        return Elem<T>::to_f32(__builtin_bit_cast(T, b));
    } else {
        typedef unsigned int u2 __attribute__((ext_vector_type(2)));
        const u2 b = __builtin_amdgcn_raw_buffer_load_b64(r, off, 0, 0);
        return Elem<T>::to_f32(__builtin_bit_cast(T, b));
    }
}
// LDS hand-off barrier that leaves the global prefetches in flight (see gf_fused.hpp)
__device__ __forceinline__ void z_lds_barrier() {
    __asm__ volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
}

// 4 consecutive elements from one buffer access (16/8/4 bytes for 4/2/1-byte types)
template <typename T>
__device__ __forceinline__ void z_load4(zrsrc_t r, int off, float (&v)[4]) {
    if constexpr (sizeof(T) == 4) {
        typedef unsigned int u4 __attribute__((ext_vector_type(4)));
        const u4 q = __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, 0);
        // elements copied out first: clang's bit_cast of a vector element lvalue reads element 0
        const uint32_t w[4] = {q.x, q.y, q.z, q.w};
#pragma unroll
        for (int e = 0; e < 4; ++e) v[e] = Elem<T>::to_f32(__builtin_bit_cast(T, w[e]));
    } else if constexpr (sizeof(T) == 2) {
        typedef unsigned int u2 __attribute__((ext_vector_type(2)));
        const u2 q = __builtin_amdgcn_raw_buffer_load_b64(r, off, 0, 0);
        v[0] = Elem<T>::to_f32(__builtin_bit_cast(T, (uint16_t)(q.x & 0xffffu)));
        v[1] = Elem<T>::to_f32(__builtin_bit_cast(T, (uint16_t)(q.x >> 16)));
        v[2] = Elem<T>::to_f32(__builtin_bit_cast(T, (uint16_t)(q.y & 0xffffu)));
        v[3] = Elem<T>::to_f32(__builtin_bit_cast(T, (uint16_t)(q.y >> 16)));
    } else {
        static_assert(sizeof(T) == 1, "quad loads of 1/2/4-byte elements");
        const uint32_t q = __builtin_amdgcn_raw_buffer_load_b32(r, off, 0, 0);
#pragma unroll
        for (int e = 0; e < 4; ++e)
            v[e] = Elem<T>::to_f32(__builtin_bit_cast(T, (uint8_t)((q >> (8 * e)) & 0xffu)));
    }
}

// A workgroup stages the (TY + L - 1) x (TX + 2 MG) input tile from x0 - MG, MG = L/2 rounded up
// to a multiple of 4 (whole 4-element quads; columns beyond the window are loaded, never read).
// QUAD (block x extent and x origin multiples of 4, aligned base, <= 4-byte elements): each quad
// is one 4/8/16-byte access at its start clamped to [0, nx - 4]; a quad wholly left / right of
// the block then holds the edge element at position 0 / 3, broadcast when the quad enters the
// ring (edge tiles only), which is the replicate clamping of the y / x passes. Otherwise
// element by element at x clamped to the block.
// Quad marches of short kernels fit 128 VGPRs without spilling: 4 waves per SIMD (4 workgroups
// per CU) instead of the 3 their natural 134 allow, so a 1024^3 launch's 2048 workgroups run in
// 2 full rounds instead of 2.7.
constexpr int zyx_min_waves(int L, bool quad) { return quad && L <= 7 ? 4 : 1; }

// Tile shapes (output rows TY x columns TX, NT threads per workgroup).
struct ZYXNarrow { static constexpr int TY = kZYXTy, TX = kZYXTx, NT = 256; };
template <int L, typename TIn, bool QUAD, typename CFG = ZYXNarrow>
__global__ __launch_bounds__(CFG::NT) __attribute__((amdgpu_waves_per_eu(CFG::NT == 256 ? zyx_min_waves(L, QUAD) : 4))) void gauss_zyx_kernel(const TIn* __restrict__ in,
                                                        float* __restrict__ out, GaussZYX p,
                                                        int tiles_x, int tiles_y, int zseg) {
    constexpr int TY = CFG::TY, TX = CFG::TX, NT = CFG::NT;
    constexpr int TH = TY + L - 1, TW = TX + L - 1, MID = L / 2;
    constexpr int MG = (MID + 3) / 4 * 4;      // x margin of the staged tile (whole quads)
    constexpr int TP = TX + 2 * MG, NQX = TP / 4;  // staged tile pitch (floats), quads per row
    constexpr int NQ = TH * NQX, NPQ = (NQ + NT - 1) / NT;  // quads, per thread
    constexpr int NYI = TW * (TY / 4), NXI = TY * (TX / 4);  // y / x pass items
    constexpr int NYP = (NYI + NT - 1) / NT, NXP = (NXI + NT - 1) / NT;
    __shared__ __attribute__((aligned(16))) float tile[NPQ * NT * 4];  // rows past TH: dummies
    __shared__ float ybuf[TY * TW];
    const int tid = threadIdx.x;
    const int64_t nz = p.n[0], ny = p.n[1], nx = p.n[2];
    const int64_t onz = p.on[0], ony = p.on[1], onx = p.on[2];
    // XCD-aware block -> (tile, z segment): consecutive logical ids (x-adjacent tiles of one
    // segment) share an XCD, so their y / x aprons come from that XCD's L2
    const int nwg = gridDim.x, b = blockIdx.x;
    const int lid = (nwg % 8 == 0) ? (b % 8) * (nwg / 8) + b / 8 : b;
    const int ntiles = tiles_x * tiles_y;
    const int tile_i = lid % ntiles, seg = lid / ntiles;
    const int64_t x0 = (int64_t)(tile_i % tiles_x) * TX, y0 = (int64_t)(tile_i / tiles_x) * TY;
    const int64_t kz0 = (int64_t)seg * zseg, kz1 = kz0 + zseg < onz ? kz0 + zseg : onz;
    const int hy = (int)(ony - y0 < TY ? ony - y0 : TY);
    const int hx = (int)(onx - x0 < TX ? onx - x0 : TX);
    const int64_t qy0 = p.o0[1] + y0 - MID, qx4 = p.o0[2] + x0 - MG;  // staged tile origin
    const int64_t plane = ny * nx;
    const uint32_t plane_bytes = (uint32_t)(plane * (int64_t)sizeof(TIn));
    const uint32_t oplane_bytes = (uint32_t)(ony * onx * 4);
    // x-pass stores: whole quads when the box width and the row pitch keep them inside and
    // 16-byte aligned
    const bool quads = (onx % 4 == 0) && (x0 % 4 == 0) && (((uintptr_t)out & 15) == 0);
    {
        constexpr int NOFF = QUAD ? NPQ : 4 * NPQ;
        int off[NOFF];  // byte offsets in the plane (rows clamped; x clamped per element)
        // QUAD edge tiles: bit k of bl / br = quad k lies wholly left / right of the block
        const bool edgex = qx4 < 0 || qx4 + TP > nx;  // block-uniform
        int bl = 0, br = 0;
#pragma unroll
        for (int k = 0; k < NPQ; ++k) {
            const int q = tid + NT * k;
            const int r = q / NQX, cq = q - r * NQX;
            int64_t qy = qy0 + r;
            qy = qy < 0 ? 0 : (qy > ny - 1 ? ny - 1 : qy);
            if constexpr (QUAD) {
                int64_t xs = qx4 + 4 * cq;
                bl |= xs < 0 ? 1 << k : 0;
                br |= xs > nx - 4 ? 1 << k : 0;
                xs = xs < 0 ? 0 : (xs > nx - 4 ? nx - 4 : xs);
                off[k] = q < NQ ? (int)((qy * nx + xs) * (int64_t)sizeof(TIn)) : kZBad;
            } else {
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    int64_t qx = qx4 + 4 * cq + e;
                    qx = qx < 0 ? 0 : (qx > nx - 1 ? nx - 1 : qx);
                    off[4 * k + e] = q < NQ ? (int)((qy * nx + qx) * (int64_t)sizeof(TIn)) : kZBad;
                }
            }
        }
        for (int64_t o = blockIdx.y; o < p.outer; o += gridDim.y) {
            const char* vol =
                reinterpret_cast<const char*>(in) + o * nz * plane * (int64_t)sizeof(TIn);
            auto ld = [&](int64_t zq, float (&v)[NPQ][4]) {  // input slice zq (clamped)
                zq = zq < 0 ? 0 : (zq > nz - 1 ? nz - 1 : zq);
                const zrsrc_t rs = z_rsrc(vol + zq * plane * (int64_t)sizeof(TIn), plane_bytes);
#pragma unroll
                for (int k = 0; k < NPQ; ++k) {
                    if constexpr (QUAD) {
                        z_load4<TIn>(rs, off[k], v[k]);
                    } else {
#pragma unroll
                        for (int e = 0; e < 4; ++e) v[k][e] = z_load<TIn>(rs, off[4 * k + e]);
                    }
                }
            };
            float ring[L][NPQ][4], pre[NPQ][4];
            // window of the first output slice: position i = input slice o0 + kz0 + i - MID in
            // slot i; position L - 1 arrives through pre
            // edge quads of a QUAD march: the edge element broadcast (no memory instructions,
            // applied where a slice enters the ring, a step after its load)
            auto fix = [&](float (&v)[NPQ][4]) {
                if constexpr (QUAD) {
                    if (edgex) {
#pragma unroll
                        for (int k = 0; k < NPQ; ++k) {
                            const bool l = (bl >> k) & 1, rr = (br >> k) & 1;
#pragma unroll
                            for (int e = 0; e < 4; ++e)
                                v[k][e] = l ? v[k][0] : (rr ? v[k][3] : v[k][e]);
                        }
                    }
                }
            };
#pragma unroll
            for (int i = 0; i < L - 1; ++i) {
                ld(p.o0[0] + kz0 + i - MID, ring[i]);
                fix(ring[i]);
            }
            ld(p.o0[0] + kz0 + L - 1 - MID, pre);
            char* obase = reinterpret_cast<char*>(out) + o * onz * ony * onx * 4;
            for (int64_t kb = kz0; kb < kz1; kb += L) {
                static_for<0, L>([&](auto PH_) {
                    constexpr int PH = decltype(PH_)::value;
                    // no early exit: the last block of L steps runs whole (an exit here put a
                    // vmcnt(0) drain on the loop path); steps past the segment store nothing
                    const int64_t kz = kb + PH;
                    // slot of window position i at this phase: (PH + i) % L; L - 1 is new
#pragma unroll
                    for (int k = 0; k < NPQ; ++k)
#pragma unroll
                        for (int e = 0; e < 4; ++e) ring[(PH + L - 1) % L][k][e] = pre[k][e];
                    fix(ring[(PH + L - 1) % L]);
                    // next step's entering slice, unconditionally (clamped; unused past the end)
                    ld(p.o0[0] + kz + 1 + MID, pre);
#pragma unroll
                    for (int k = 0; k < NPQ; ++k) {
                        float sv[4];
#pragma unroll
                        for (int e = 0; e < 4; ++e) {
                            float sum = -0.0f;  // Iterator::sum::<f32> (kernel.rs:46, :66)
#pragma unroll
                            for (int i = 0; i < L; ++i)
                                sum = sum + ring[(PH + i) % L][k][e] * p.w[0][i];
                            sv[e] = sum;
                        }
                        *reinterpret_cast<float4*>(tile + 4 * (tid + NT * k)) =
                            make_float4(sv[0], sv[1], sv[2], sv[3]);
                    }
                    z_lds_barrier();
#pragma unroll
                    for (int ip = 0; ip < NYP; ++ip) {  // y pass, 4 rows per item
                        const int item = tid + NT * ip;
                        if (NYI % NT == 0 || item < NYI) {
                            // column c of the TW window = staged column c + MG - MID
                            const int c = item % TW, r0 = (item / TW) * 4;
                            float v[4 + L - 1];
#pragma unroll
                            for (int j = 0; j < 4 + L - 1; ++j)
                                v[j] = tile[(r0 + j) * TP + c + MG - MID];
#pragma unroll
                            for (int k = 0; k < 4; ++k) {
                                float sum = -0.0f;
#pragma unroll
                                for (int i = 0; i < L; ++i) sum = sum + v[k + i] * p.w[1][i];
                                ybuf[(r0 + k) * TW + c] = sum;
                            }
                        }
                    }
                    z_lds_barrier();
                    const zrsrc_t ro = z_rsrc(obase + (kz < kz1 ? kz : 0) * ony * onx * 4,
                                              kz < kz1 ? oplane_bytes : 0u);
#pragma unroll
                    for (int ip = 0; ip < NXP; ++ip) {  // x pass, 4 columns per item
                        const int item = tid + NT * ip;
                        const int r = item / (TX / 4), c0 = (item % (TX / 4)) * 4;
                        const bool live = (NXI % NT == 0 || item < NXI) && r < hy;
                        float v[4 + L - 1];
#pragma unroll
                        for (int j = 0; j < 4 + L - 1; ++j)
                            v[j] = ybuf[(live ? r : 0) * TW + c0 + j];
                        float o4[4];
#pragma unroll
                        for (int k = 0; k < 4; ++k) {
                            float sum = -0.0f;
#pragma unroll
                            for (int i = 0; i < L; ++i) sum = sum + v[k + i] * p.w[2][i];
                            o4[k] = sum;
                        }
                        const int ooff = (int)(((y0 + r) * onx + x0 + c0) * 4);
                        if (quads) {
                            typedef unsigned int u4 __attribute__((ext_vector_type(4)));
                            const u4 q = {__float_as_uint(o4[0]), __float_as_uint(o4[1]),
                                          __float_as_uint(o4[2]), __float_as_uint(o4[3])};
                            __builtin_amdgcn_raw_buffer_store_b128(
                                q, ro, live && c0 < hx ? ooff : kZBad, 0, 2);
                        } else {
#pragma unroll
                            for (int k = 0; k < 4; ++k)
                                __builtin_amdgcn_raw_buffer_store_b32(
                                    __float_as_uint(o4[k]), ro,
                                    live && c0 + k < hx ? ooff + 4 * k : kZBad, 0, 2);
                        }
                    }
                    // the next tile / ybuf writes follow this step's barriers
                });
            }
            z_lds_barrier();  // the last step's reads of tile / ybuf before the next volume
        }
    }
}

bool gaussian_zyx_supported(const GaussZYX& p, int dtype_in) {
    (void)dtype_in;
    // slices addressed by 32-bit byte offsets (buffer descriptors)
    return p.len >= 3 && p.len <= kGaussZYXMaxLen && p.len % 2 == 1 &&
           p.n[1] * p.n[2] * (int64_t)dtype_size(dtype_in) < 0x7FFFFFFF &&
           p.on[1] * p.on[2] * 4 < 0x7FFFFFFF && (p.on[1] + kZYXTy - 1) / kZYXTy <= 0xFFFF &&
           (p.on[2] + kZYXTx - 1) / kZYXTx <= 0xFFFF;
}

// Wide tiles for short quad marches (L <= 7): 4x the columns of the narrow tile on 1024 threads
// (one workgroup per CU, 4 waves per SIMD), so the staged tile's x apron shrinks from 72/64 to
// 264/256 columns: 1024^3 sigma = 1 measured 2.43 -> 2.13 ms in tools/timegauss.hip
// (profiles/r03_gauss_variants_*.txt), identical output.
struct ZYXWide { static constexpr int TY = 32, TX = 256, NT = 1024; };

// ---------------------------------------------------------------------------------------------
// gauss_zyx_kernel with the entering slice staged by LDS-DMA (round 4; f32 input, wide tiles,
// whole-quad accesses): each wave issues its share of the staged tile's 1 KiB pieces as
// `buffer_load_dwordx4 ... lds` from inline asm into one of two LDS slots, so the next slice's
// bytes are in flight without holding VGPRs (the L-slice register ring fills them) and hipcc's
// waitcnt pass, which does not see an asm load, never drains them: this kernel counts them with
// its own `s_waitcnt vmcnt(N)` (cdna_hip_programming.md §5.7). Per step k:
//   ring <- pre (slice k + MID, read from its slot during step k-1) ; z pass -> tile ;
//   barrier 1 ; DMA of slice k + 2 + MID into the slot step k-1 read ; y pass -> ybuf ;
//   own DMA of slice k + 1 + MID landed (vmcnt) ; barrier 2 ; pre <- that slot ; x pass, stores.
// Same arithmetic, in the same order, as gauss_zyx_kernel: bit-identical output.
// ---------------------------------------------------------------------------------------------
__device__ __forceinline__ void zdma16(zrsrc_t r, int voff, unsigned lds) {
    unsigned keep;
    asm volatile(
        "s_mov_b32 %0, m0\n\t"
        "s_mov_b32 m0, %2\n\t"
        "s_nop 0\n\t"
        "buffer_load_dwordx4 %1, %3, 0 offen lds\n\t"
        "s_mov_b32 m0, %0"
        : "=&s"(keep)
        : "v"(voff), "s"(lds), "s"(r)
        : "memory");
}
template <int N>
__device__ __forceinline__ void zwait_vm() {
    asm volatile("s_waitcnt vmcnt(%0)" ::"i"(N) : "memory");
}

template <int L>
__global__ __launch_bounds__(1024) void gauss_zyx_dma_kernel(const float* __restrict__ in,
                                                             float* __restrict__ out, GaussZYX p,
                                                             int tiles_x, int tiles_y, int zseg) {
    using CFG = ZYXWide;
    constexpr int TY = CFG::TY, TX = CFG::TX, NT = CFG::NT;
    constexpr int TH = TY + L - 1, TW = TX + L - 1, MID = L / 2;
    constexpr int MG = (MID + 3) / 4 * 4;
    constexpr int TP = TX + 2 * MG, NQX = TP / 4;
    constexpr int NQ = TH * NQX, NPQ = (NQ + NT - 1) / NT;
    constexpr int NJ = (NQ + 63) / 64;  // 1 KiB DMA pieces per slice
    constexpr int NXI = TY * (TX / 4), NXP = (NXI + NT - 1) / NT;
    constexpr int NYI = TW * (TY / 4), NYP = (NYI + NT - 1) / NT;
    static_assert(NXI % NT == 0, "every thread stores NXP quads per step (vmcnt count)");
    static_assert(NPQ == 3 && NJ > 32 && NJ <= 48, "three pieces for waves < NJ - 32, else two");
    __shared__ __attribute__((aligned(16))) float tile[NQ * 4];
    __shared__ float ybuf[TY * TW];
    __shared__ __attribute__((aligned(1024))) float slot[2][NJ * 256];
    const int tid = threadIdx.x;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const bool three = wave + 32 < NJ;  // this wave issues a third piece (wave-uniform)
    const int64_t nz = p.n[0], ny = p.n[1], nx = p.n[2];
    const int64_t onz = p.on[0], ony = p.on[1], onx = p.on[2];
    const int nwg = gridDim.x, b = blockIdx.x;
    const int lid = (nwg % 8 == 0) ? (b % 8) * (nwg / 8) + b / 8 : b;
    const int ntiles = tiles_x * tiles_y;
    const int tile_i = lid % ntiles, seg = lid / ntiles;
    const int64_t x0 = (int64_t)(tile_i % tiles_x) * TX, y0 = (int64_t)(tile_i / tiles_x) * TY;
    const int64_t kz0 = (int64_t)seg * zseg, kz1 = kz0 + zseg < onz ? kz0 + zseg : onz;
    const int hy = (int)(ony - y0 < TY ? ony - y0 : TY);
    const int hx = (int)(onx - x0 < TX ? onx - x0 : TX);
    const int64_t qy0 = p.o0[1] + y0 - MID, qx4 = p.o0[2] + x0 - MG;
    const int64_t plane = ny * nx;
    const uint32_t plane_bytes = (uint32_t)(plane * 4);
    const uint32_t oplane_bytes = (uint32_t)(ony * onx * 4);
    const unsigned slot_base = (unsigned)(uintptr_t)&slot[0][0];
    int off[NPQ];
    const bool edgex = qx4 < 0 || qx4 + TP > nx;
    int bl = 0, br = 0;
#pragma unroll
    for (int k = 0; k < NPQ; ++k) {
        const int q = tid + NT * k;
        const int r = q / NQX, cq = q - r * NQX;
        int64_t qy = qy0 + r;
        qy = qy < 0 ? 0 : (qy > ny - 1 ? ny - 1 : qy);
        int64_t xs = qx4 + 4 * cq;
        bl |= xs < 0 ? 1 << k : 0;
        br |= xs > nx - 4 ? 1 << k : 0;
        xs = xs < 0 ? 0 : (xs > nx - 4 ? nx - 4 : xs);
        off[k] = q < NQ ? (int)((qy * nx + xs) * 4) : kZBad;
    }
    auto fix = [&](float (&v)[NPQ][4]) {
        if (edgex) {
#pragma unroll
            for (int k = 0; k < NPQ; ++k) {
                const bool l = (bl >> k) & 1, rr = (br >> k) & 1;
#pragma unroll
                for (int e = 0; e < 4; ++e) v[k][e] = l ? v[k][0] : (rr ? v[k][3] : v[k][e]);
            }
        }
    };
    for (int64_t o = blockIdx.y; o < p.outer; o += gridDim.y) {
        const char* vol = reinterpret_cast<const char*>(in) + o * nz * plane * 4;
        auto rs_of = [&](int64_t zq) {
            zq = zq < 0 ? 0 : (zq > nz - 1 ? nz - 1 : zq);
            return z_rsrc(vol + zq * plane * 4, plane_bytes);
        };
        // this wave's pieces of slice zq into slot sl: piece j = wave + 16 k carries quads
        // [64 j, 64 j + 64), i.e. lane l's own quad tid + NT k
        auto dma = [&](int64_t zq, int sl) {
            const zrsrc_t rs = rs_of(zq);
            const unsigned base = slot_base + (unsigned)sl * (NJ * 1024u);
            zdma16(rs, off[0], base + (unsigned)wave * 1024u);
            zdma16(rs, off[1], base + (unsigned)(wave + 16) * 1024u);
            if (three) zdma16(rs, off[2], base + (unsigned)(wave + 32) * 1024u);
        };
        auto from_slot = [&](int sl, float (&v)[NPQ][4]) {
            const float* sb = &slot[0][0] + sl * (NJ * 256);
#pragma unroll
            for (int k = 0; k < NPQ; ++k) {
                const int q = tid + NT * k;
                const float4 f = *reinterpret_cast<const float4*>(sb + 4 * (q < NJ * 64 ? q : 0));
                v[k][0] = f.x; v[k][1] = f.y; v[k][2] = f.z; v[k][3] = f.w;
            }
        };
        float ring[L][NPQ][4], pre[NPQ][4];
        // window of the first output slice: slices o0 + kz0 + i - MID, i < L - 1, by plain loads
#pragma unroll
        for (int i = 0; i < L - 1; ++i) {
            const zrsrc_t rs = rs_of(p.o0[0] + kz0 + i - MID);
#pragma unroll
            for (int k = 0; k < NPQ; ++k) z_load4<float>(rs, off[k], ring[i][k]);
            fix(ring[i]);
        }
        // slice of window position L - 1 of step kz0 into slot 0, of step kz0 + 1 into slot 1
        dma(p.o0[0] + kz0 + L - 1 - MID, 0);
        zwait_vm<0>();
        z_lds_barrier();
        from_slot(0, pre);
        dma(p.o0[0] + kz0 + L - MID, 1);
        // NXP dropped stores, so that the first step's wait counts the same ops as every later
        // step's (the previous step's stores, then this step's pieces)
        {
            const zrsrc_t none = z_rsrc(out, 0u);
#pragma unroll
            for (int ip = 0; ip < NXP; ++ip) __builtin_amdgcn_raw_buffer_store_b32(0u, none, kZBad, 0, 2);
        }
        char* obase = reinterpret_cast<char*>(out) + o * onz * ony * onx * 4;
        for (int64_t kb = kz0; kb < kz1; kb += L) {
            static_for<0, L>([&](auto PH_) {
                constexpr int PH = decltype(PH_)::value;  // ring phase
                const int64_t kz = kb + PH;
                const int SL = (int)((kz - kz0) & 1);  // slot that held pre (wave-uniform)
#pragma unroll
                for (int k = 0; k < NPQ; ++k)
#pragma unroll
                    for (int e = 0; e < 4; ++e) ring[(PH + L - 1) % L][k][e] = pre[k][e];
                fix(ring[(PH + L - 1) % L]);
#pragma unroll
                for (int k = 0; k < NPQ; ++k) {
                    float sv[4];
#pragma unroll
                    for (int e = 0; e < 4; ++e) {
                        float sum = -0.0f;  // Iterator::sum::<f32> (kernel.rs:46, :66)
#pragma unroll
                        for (int i = 0; i < L; ++i)
                            sum = sum + ring[(PH + i) % L][k][e] * p.w[0][i];
                        sv[e] = sum;
                    }
                    const int q = tid + NT * k;
                    if (k < NPQ - 1 || q < NQ)
                        *reinterpret_cast<float4*>(tile + 4 * q) = make_float4(sv[0], sv[1], sv[2], sv[3]);
                }
                z_lds_barrier();
                // slot SL (read into pre during the previous step) is free: the slice of window
                // position L - 1 two steps on (clamped; unused past the segment)
                dma(p.o0[0] + kz + 2 + L - 1 - MID, SL);
#pragma unroll
                for (int ip = 0; ip < NYP; ++ip) {
                    const int item = tid + NT * ip;
                    if (NYI % NT == 0 || item < NYI) {
                        const int c = item % TW, r0 = (item / TW) * 4;
                        float v[4 + L - 1];
#pragma unroll
                        for (int j = 0; j < 4 + L - 1; ++j) v[j] = tile[(r0 + j) * TP + c + MG - MID];
#pragma unroll
                        for (int k = 0; k < 4; ++k) {
                            float sum = -0.0f;
#pragma unroll
                            for (int i = 0; i < L; ++i) sum = sum + v[k + i] * p.w[1][i];
                            ybuf[(r0 + k) * TW + c] = sum;
                        }
                    }
                }
                // own pieces of the next step's slice (issued a step ago, slot 1 - SL) landed:
                // younger are the previous step's NXP stores and this step's pieces
                if (three) zwait_vm<NXP + 3>(); else zwait_vm<NXP + 2>();
                z_lds_barrier();
                from_slot(1 - SL, pre);
                const zrsrc_t ro = z_rsrc(obase + (kz < kz1 ? kz : 0) * ony * onx * 4,
                                          kz < kz1 ? oplane_bytes : 0u);
#pragma unroll
                for (int ip = 0; ip < NXP; ++ip) {
                    const int item = tid + NT * ip;
                    const int r = item / (TX / 4), c0 = (item % (TX / 4)) * 4;
                    const bool live = r < hy;
                    float v[4 + L - 1];
#pragma unroll
                    for (int j = 0; j < 4 + L - 1; ++j) v[j] = ybuf[(live ? r : 0) * TW + c0 + j];
                    float o4[4];
#pragma unroll
                    for (int k = 0; k < 4; ++k) {
                        float sum = -0.0f;
#pragma unroll
                        for (int i = 0; i < L; ++i) sum = sum + v[k + i] * p.w[2][i];
                        o4[k] = sum;
                    }
                    const int ooff = (int)(((y0 + r) * onx + x0 + c0) * 4);
                    typedef unsigned int u4 __attribute__((ext_vector_type(4)));
                    const u4 q = {__float_as_uint(o4[0]), __float_as_uint(o4[1]),
                                  __float_as_uint(o4[2]), __float_as_uint(o4[3])};
                    __builtin_amdgcn_raw_buffer_store_b128(q, ro, live && c0 < hx ? ooff : kZBad,
                                                           0, 2);
                }
            });
        }
        zwait_vm<0>();  // no piece may land after the workgroup (or this volume) is done
        z_lds_barrier();
    }
}

template <int L, typename CFG>
static hipError_t launch_zyx_cfg(const void* in, int dtype_in, float* out, const GaussZYX& p,
                                 bool quad, hipStream_t s) {
    const int tiles_x = (int)((p.on[2] + CFG::TX - 1) / CFG::TX);
    const int tiles_y = (int)((p.on[1] + CFG::TY - 1) / CFG::TY);
    const int64_t tiles = (int64_t)tiles_x * tiles_y;
    const int64_t outer = p.outer;
    // z segments: about two rounds of full occupancy (4 waves per SIMD) over the launch, at
    // least kZYXSegMin slices each (a segment re-reads L - 1 slices to fill its window)
    const int64_t per_launch = 2 * 256 * (1024 / CFG::NT);
    const int64_t want = (per_launch + tiles * outer - 1) / (tiles * outer);
    int64_t nseg = std::max<int64_t>(1, std::min<int64_t>(want, (p.on[0] + kZYXSegMin - 1) / kZYXSegMin));
    const int zseg = (int)((p.on[0] + nseg - 1) / nseg);
    nseg = (p.on[0] + zseg - 1) / zseg;
    const int64_t gx = tiles * nseg;
    if (gx > 0x7FFFFFFF) return hipErrorInvalidValue;
    const dim3 grid((unsigned)gx, (unsigned)(outer < 65535 ? outer : 65535));
    hipError_t err = hipErrorInvalidValue;
    ZT_DISPATCH_DTYPE(dtype_in, T,
        // (quad instantiations for the common element types only: build time)
        if constexpr (std::is_same_v<T, float> || std::is_same_v<T, uint16_t> ||
                      std::is_same_v<T, uint8_t>) {
            if (quad)
                hipLaunchKernelGGL((gauss_zyx_kernel<L, T, true, CFG>), grid, dim3(CFG::NT), 0, s,
                                   static_cast<const T*>(in), out, p, tiles_x, tiles_y, zseg);
            else if constexpr (std::is_same_v<CFG, ZYXNarrow>)
                hipLaunchKernelGGL((gauss_zyx_kernel<L, T, false, CFG>), grid, dim3(CFG::NT), 0, s,
                                   static_cast<const T*>(in), out, p, tiles_x, tiles_y, zseg);
        } else if constexpr (std::is_same_v<CFG, ZYXNarrow>) {  // (wide tiles: quad marches only)
            hipLaunchKernelGGL((gauss_zyx_kernel<L, T, false, CFG>), grid, dim3(CFG::NT), 0, s,
                               static_cast<const T*>(in), out, p, tiles_x, tiles_y, zseg);
        }
        err = hipGetLastError())
    return err;
}

template <int L>
static hipError_t launch_zyx_dma(const float* in, float* out, const GaussZYX& p, hipStream_t s) {
    using CFG = ZYXWide;
    const int tiles_x = (int)((p.on[2] + CFG::TX - 1) / CFG::TX);
    const int tiles_y = (int)((p.on[1] + CFG::TY - 1) / CFG::TY);
    const int64_t tiles = (int64_t)tiles_x * tiles_y;
    const int64_t outer = p.outer;
    const int64_t per_launch = 2 * 256;  // as launch_zyx_cfg for one workgroup per CU
    const int64_t want = (per_launch + tiles * outer - 1) / (tiles * outer);
    int64_t nseg = std::max<int64_t>(1, std::min<int64_t>(want, (p.on[0] + kZYXSegMin - 1) / kZYXSegMin));
    const int zseg = (int)((p.on[0] + nseg - 1) / nseg);
    nseg = (p.on[0] + zseg - 1) / zseg;
    const int64_t gx = tiles * nseg;
    if (gx > 0x7FFFFFFF) return hipErrorInvalidValue;
    const dim3 grid((unsigned)gx, (unsigned)(outer < 65535 ? outer : 65535));
    hipLaunchKernelGGL((gauss_zyx_dma_kernel<L>), grid, dim3(CFG::NT), 0, s, in, out, p, tiles_x,
                       tiles_y, zseg);
    return hipGetLastError();
}

template <int L>
static hipError_t launch_zyx_l(const void* in, int dtype_in, float* out, const GaussZYX& p,
                               hipStream_t s) {
    const int esz = dtype_size(dtype_in);
    // quads need a 4-aligned x origin and extent and an aligned base, <= 4-byte elements
    const bool quad = esz <= 4 && p.n[2] % 4 == 0 && p.o0[2] % 4 == 0 &&
                      p.n[2] >= 4 && (uintptr_t)in % (4 * esz) == 0 &&
                      (dtype_in == kF32 || dtype_in == kU16 || dtype_in == kU8 || dtype_in == kBool);
    // wide tiles when the march is a short quad march and the block is wide enough not to
    // leave most of a wide tile idle
    if constexpr (L <= 7) {
        // f32 with whole-quad output rows: the entering slice staged by LDS-DMA
        if (quad && p.on[2] >= ZYXWide::TX && dtype_in == kF32 &&
            p.on[2] % 4 == 0 && ((uintptr_t)out & 15) == 0)
            return launch_zyx_dma<L>(static_cast<const float*>(in), out, p, s);
        if (quad && p.on[2] >= ZYXWide::TX)
            return launch_zyx_cfg<L, ZYXWide>(in, dtype_in, out, p, quad, s);
    }
    return launch_zyx_cfg<L, ZYXNarrow>(in, dtype_in, out, p, quad, s);
}

hipError_t launch_gaussian_zyx(const void* in, int dtype_in, float* out, const GaussZYX& p,
                               hipStream_t s) {
    if (p.outer * p.on[0] * p.on[1] * p.on[2] == 0) return hipSuccess;
    if (!gaussian_zyx_supported(p, dtype_in)) return hipErrorInvalidValue;
    switch (p.len) {
    case 3: return launch_zyx_l<3>(in, dtype_in, out, p, s);
    case 5: return launch_zyx_l<5>(in, dtype_in, out, p, s);
    case 7: return launch_zyx_l<7>(in, dtype_in, out, p, s);
    case 9: return launch_zyx_l<9>(in, dtype_in, out, p, s);
    case 11: return launch_zyx_l<11>(in, dtype_in, out, p, s);
    case 13: return launch_zyx_l<13>(in, dtype_in, out, p, s);
    default: return hipErrorInvalidValue;
    }
}

static dim3 rows_grid(int64_t gx, int64_t rows) {
    const int64_t gy = rows < 65535 ? rows : 65535;
    const int64_t gzn = (rows + gy - 1) / gy;
    return dim3((unsigned)gx, (unsigned)gy, (unsigned)(gzn < 65535 ? gzn : 65535));
}

hipError_t launch_gaussian_pass(const void* in, int dtype_in, float* out, const GaussPass& p,
                                hipStream_t s) {
    if (p.outer * p.on * p.inner == 0) return hipSuccess;
    hipError_t err = hipErrorInvalidValue;
    if (p.inner == 1) {
        const int64_t gx = (p.on + kGaussRowTile - 1) / kGaussRowTile;
        const size_t lds = sizeof(float) * (kGaussRowTile + p.len - 1);
        ZT_DISPATCH_DTYPE(dtype_in, T,
            hipLaunchKernelGGL(gauss_row_kernel<T>, rows_grid(gx, p.outer), dim3(256), lds, s,
                               static_cast<const T*>(in), out, p);
            err = hipGetLastError())
    } else if (kGaussSeg + p.len - 1 <= kGaussColMaxWin) {
        const int64_t nseg = (p.on + kGaussSeg - 1) / kGaussSeg;
        const size_t lds = sizeof(float) * 256 * (kGaussSeg + p.len - 1);
        ZT_DISPATCH_DTYPE(dtype_in, T,
            hipLaunchKernelGGL(gauss_col_kernel<T>, rows_grid((p.inner + 255) / 256,
                                                              p.outer * nseg),
                               dim3(256), lds, s, static_cast<const T*>(in), out, p, nseg);
            err = hipGetLastError())
    } else {  // long kernels: one output per thread
        ZT_DISPATCH_DTYPE(dtype_in, T,
            hipLaunchKernelGGL((gauss_pass_kernel<T, false>),
                               rows_grid((p.inner + 255) / 256, p.outer * p.on), dim3(256), 0, s,
                               static_cast<const T*>(in), out, p);
            err = hipGetLastError())
    }
    return err;
}

}  // namespace zt
