// tools/pyr_variants.hpp — experimental variants of the fused 2x2x2 pyramid kernel
// (downsample.hip: pyramid3_fused_kernel, u16, three levels) for tools/timepyr (not a product
// path). IM = 1: u16 windows summed in 32-bit integers and divided by 8 in integers (the mean of
// 8 u16 is exact in f64 and `as u16` truncates, so sum / 8 is the same value); GZ caps the grid's
// z extent, each workgroup then looping over level-1 z blocks.
#pragma once
#include <hip/hip_runtime.h>

#include <stdint.h>

namespace pyrv {

template <int IM>
__device__ __forceinline__ uint16_t mean8(const uint16_t (&v)[8]) {
    if constexpr (IM == 1) {
        uint32_t s = 0;
#pragma unroll
        for (int i = 0; i < 8; ++i) s += v[i];
        return (uint16_t)(s >> 3);
    } else {
        int64_t s = 0;
#pragma unroll
        for (int i = 0; i < 8; ++i) s += (int64_t)v[i];
        const double m = (double)s / 8.0;
        return m >= 65536.0 ? (uint16_t)65535 : (uint16_t)m;
    }
}

struct P {
    int64_t s[4][3];
};

template <int IM>
__global__ __launch_bounds__(256) void pyr3(const uint16_t* __restrict__ in, uint16_t* __restrict__ l1,
                                            uint16_t* __restrict__ l2, uint16_t* __restrict__ l3,
                                            P p) {
    using T = uint16_t;
    __shared__ T lds2[4][64][2];
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int dz = w >> 1, dy = w & 1;
    const int64_t x3 = (int64_t)blockIdx.x * 64 + lane;
    const int64_t by = blockIdx.y;
    const int64_t n0y = p.s[0][1], n0x = p.s[0][2];
    const int64_t n1z = p.s[1][0], n1y = p.s[1][1], n1x = p.s[1][2];
    const int64_t n2z = p.s[2][0], n2y = p.s[2][1], n2x = p.s[2][2];
    const int64_t nz1blocks = (n1z + 3) / 4;
    for (int64_t bz = blockIdx.z; bz < nz1blocks; bz += gridDim.z) {
        typedef T V8 __attribute__((ext_vector_type(8)));
        V8 v[4][4];
        const int64_t z0b = 8 * bz + 4 * dz, y0b = 8 * by + 4 * dy, x0b = 8 * x3;
        const bool xfull = x0b + 8 <= n0x;
#pragma unroll
        for (int a = 0; a < 4; ++a)
#pragma unroll
            for (int b = 0; b < 4; ++b) {
                const int64_t z0 = z0b + a, y0 = y0b + b;
                const bool rok = z0 < p.s[0][0] && y0 < n0y;
                const T* row = in + (z0 * n0y + y0) * n0x + x0b;
                if (rok && xfull) {
                    v[a][b] = *reinterpret_cast<const V8*>(row);
                } else {
#pragma unroll
                    for (int c = 0; c < 8; ++c) v[a][b][c] = (rok && x0b + c < n0x) ? row[c] : T(0);
                }
            }
        T u1[2][2][4];
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
            for (int j = 0; j < 2; ++j)
#pragma unroll
                for (int k = 0; k < 4; ++k) {
                    const T t[8] = {v[2 * i][2 * j][2 * k],     v[2 * i][2 * j][2 * k + 1],
                                    v[2 * i][2 * j + 1][2 * k], v[2 * i][2 * j + 1][2 * k + 1],
                                    v[2 * i + 1][2 * j][2 * k], v[2 * i + 1][2 * j][2 * k + 1],
                                    v[2 * i + 1][2 * j + 1][2 * k],
                                    v[2 * i + 1][2 * j + 1][2 * k + 1]};
                    u1[i][j][k] = mean8<IM>(t);
                }
        const int64_t z1b = 4 * bz + 2 * dz, y1b = 4 * by + 2 * dy, x1b = 4 * x3;
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
            for (int j = 0; j < 2; ++j) {
                const int64_t z1 = z1b + i, y1 = y1b + j;
                if (z1 >= n1z || y1 >= n1y) continue;
                T* o = l1 + (z1 * n1y + y1) * n1x + x1b;
                typedef T V4 __attribute__((ext_vector_type(4)));
                if (x1b + 4 <= n1x) {
                    const V4 q = {u1[i][j][0], u1[i][j][1], u1[i][j][2], u1[i][j][3]};
                    *reinterpret_cast<V4*>(o) = q;
                    continue;
                }
#pragma unroll
                for (int k = 0; k < 4; ++k)
                    if (x1b + k < n1x) o[k] = u1[i][j][k];
            }
        T u2[2];
#pragma unroll
        for (int m = 0; m < 2; ++m) {
            const T t[8] = {u1[0][0][2 * m], u1[0][0][2 * m + 1], u1[0][1][2 * m],
                            u1[0][1][2 * m + 1], u1[1][0][2 * m], u1[1][0][2 * m + 1],
                            u1[1][1][2 * m], u1[1][1][2 * m + 1]};
            u2[m] = mean8<IM>(t);
        }
        const int64_t z2 = 2 * bz + dz, y2 = 2 * by + dy, x2 = 2 * x3;
        if (z2 < n2z && y2 < n2y) {
            T* o = l2 + (z2 * n2y + y2) * n2x + x2;
            if (x2 < n2x) o[0] = u2[0];
            if (x2 + 1 < n2x) o[1] = u2[1];
        }
        lds2[w][lane][0] = u2[0];
        lds2[w][lane][1] = u2[1];
        __syncthreads();
        if (w == 0) {
            const T t[8] = {lds2[0][lane][0], lds2[0][lane][1], lds2[1][lane][0],
                            lds2[1][lane][1], lds2[2][lane][0], lds2[2][lane][1],
                            lds2[3][lane][0], lds2[3][lane][1]};
            const T u3 = mean8<IM>(t);
            if (bz < p.s[3][0] && by < p.s[3][1] && x3 < p.s[3][2])
                l3[(bz * p.s[3][1] + by) * p.s[3][2] + x3] = u3;
        }
        __syncthreads();
    }
}

inline hipError_t launch(const uint16_t* in, uint16_t* l1, uint16_t* l2, uint16_t* l3,
                         const int64_t (*sh)[3], int im, int gzcap, hipStream_t s) {
    P p{};
    for (int l = 0; l < 4; ++l)
        for (int d = 0; d < 3; ++d) p.s[l][d] = sh[l][d];
    const int64_t gx = (p.s[1][2] + 255) / 256, gy = (p.s[1][1] + 3) / 4;
    int64_t gz = (p.s[1][0] + 3) / 4;
    if (gz > gzcap) gz = gzcap;
    if (gz > 65535) gz = 65535;
    const dim3 grid((unsigned)gx, (unsigned)gy, (unsigned)gz);
    if (im == 1) hipLaunchKernelGGL(pyr3<1>, grid, dim3(256), 0, s, in, l1, l2, l3, p);
    else hipLaunchKernelGGL(pyr3<0>, grid, dim3(256), 0, s, in, l1, l2, l3, p);
    return hipGetLastError();
}

}  // namespace pyrv
