// tools/timegauss.hip — timing harness for variants of the fused Gaussian z/y/x march (a copy of
// gauss_zyx_kernel from zarrs_tools_amd/csrc/gaussian.hip with the tile and workgroup sizes as
// macros: -DGV_TY= -DGV_TX= -DGV_NT= -DGV_WPE=). Not a product path. Times 1024^3 f32, L = 7
// (sigma 1, half-width 3) and prints a checksum so variants can be compared.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <type_traits>
#include <vector>

#include "zt_device.hpp"
#include "zt_kernels.hpp"

namespace zt {
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
#ifndef GV_TY
#define GV_TY 32
#endif
#ifndef GV_TX
#define GV_TX 64
#endif
#ifndef GV_NT
#define GV_NT 256
#endif
#ifndef GV_XQ
#define GV_XQ 0
#endif
#ifndef GV_LAUX
#define GV_LAUX 0
#endif
#ifndef GV_PF2
#define GV_PF2 0
#endif
#ifndef GV_WPE
#define GV_WPE 4
#endif
constexpr int kZYXTy = GV_TY, kZYXTx = GV_TX, kZYXSegMin = 32;

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
        const u4 q = __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, GV_LAUX);
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
constexpr int zyx_min_waves(int L, bool quad) { return quad && L <= 7 ? GV_WPE : 1; }

template <int L, typename TIn, bool QUAD>
__global__ __launch_bounds__(GV_NT) __attribute__((amdgpu_waves_per_eu(zyx_min_waves(L, QUAD)))) void gauss_zyx_kernel(const TIn* __restrict__ in,
                                                        float* __restrict__ out, GaussZYX p,
                                                        int tiles_x, int tiles_y, int zseg) {
    constexpr int TY = kZYXTy, TX = kZYXTx, TH = TY + L - 1, TW = TX + L - 1, MID = L / 2;
    constexpr int MG = (MID + 3) / 4 * 4;      // x margin of the staged tile (whole quads)
    constexpr int TP = TX + 2 * MG, NQX = TP / 4;  // staged tile pitch (floats), quads per row
    constexpr int NQ = TH * NQX, NPQ = (NQ + GV_NT - 1) / GV_NT;  // quads, per thread
    constexpr int NYI = TW * (TY / 4), NXI = TY * (TX / 4);  // y / x pass items
    constexpr int NYP = (NYI + GV_NT - 1) / GV_NT, NXP = (NXI + GV_NT - 1) / GV_NT;
    __shared__ __attribute__((aligned(16))) float tile[NPQ * GV_NT * 4];  // rows past TH: dummies
#if GV_XQ
    // x-pass rows read as 16-byte quads: pitch a multiple of 4 floats (lanes 16 B apart are
    // conflict-free for ds_read_b128; single floats 16 B apart were 4-way bank conflicts)
    constexpr int YP = (TW + 3) / 4 * 4 + 4 * ((((TW + 3) / 4) % 2) == 0 ? 1 : 0);
#else
    constexpr int YP = TW;
#endif
    __shared__ __attribute__((aligned(16))) float ybuf[TY * YP];
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
            const int q = tid + GV_NT * k;
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
#if GV_PF2
            float pre2[NPQ][4];  // prefetch two slices ahead
#endif
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
#if GV_PF2
            ld(p.o0[0] + kz0 + L - MID, pre2);
#endif
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
#if GV_PF2
#pragma unroll
                    for (int k = 0; k < NPQ; ++k)
#pragma unroll
                        for (int e = 0; e < 4; ++e) pre[k][e] = pre2[k][e];
                    ld(p.o0[0] + kz + 2 + MID, pre2);
#else
                    ld(p.o0[0] + kz + 1 + MID, pre);
#endif
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
                        *reinterpret_cast<float4*>(tile + 4 * (tid + GV_NT * k)) =
                            make_float4(sv[0], sv[1], sv[2], sv[3]);
                    }
                    z_lds_barrier();
#pragma unroll
                    for (int ip = 0; ip < NYP; ++ip) {  // y pass, 4 rows per item
                        const int item = tid + GV_NT * ip;
                        if (NYI % GV_NT == 0 || item < NYI) {
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
                                ybuf[(r0 + k) * YP + c] = sum;
                            }
                        }
                    }
                    z_lds_barrier();
                    const zrsrc_t ro = z_rsrc(obase + (kz < kz1 ? kz : 0) * ony * onx * 4,
                                              kz < kz1 ? oplane_bytes : 0u);
#pragma unroll
                    for (int ip = 0; ip < NXP; ++ip) {  // x pass, 4 columns per item
                        const int item = tid + GV_NT * ip;
                        const int r = item / (TX / 4), c0 = (item % (TX / 4)) * 4;
                        const bool live = (NXI % GV_NT == 0 || item < NXI) && r < hy;
                        float v[4 + L - 1];
#if GV_XQ
                        {
                            constexpr int NV = 4 + L - 1, NQ4 = NV / 4;
                            const float* rowp = ybuf + (live ? r : 0) * YP + c0;
#pragma unroll
                            for (int q = 0; q < NQ4; ++q) {
                                const float4 f = *reinterpret_cast<const float4*>(rowp + 4 * q);
                                v[4 * q] = f.x; v[4 * q + 1] = f.y; v[4 * q + 2] = f.z; v[4 * q + 3] = f.w;
                            }
                            if constexpr (NV % 4 >= 2) {
                                const float2 f = *reinterpret_cast<const float2*>(rowp + 4 * NQ4);
                                v[4 * NQ4] = f.x; v[4 * NQ4 + 1] = f.y;
                            }
                            if constexpr (NV % 2 == 1) v[NV - 1] = rowp[NV - 1];
                        }
#else
#pragma unroll
                        for (int j = 0; j < 4 + L - 1; ++j)
                            v[j] = ybuf[(live ? r : 0) * YP + c0 + j];
#endif
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


}  // namespace zt

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { \
    printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

int main(int argc, char** argv) {
    using namespace zt;
    const int n = argc > 1 ? atoi(argv[1]) : 1024;
    const char* tag = argc > 2 ? argv[2] : "";
    const size_t vox = (size_t)n * n * n;
    float *in, *out;
    CK(hipMalloc(&in, vox * 4)); CK(hipMalloc(&out, vox * 4));
    std::vector<float> h((size_t)n * n);
    for (int z = 0; z < n; ++z) {
        for (size_t i = 0; i < h.size(); ++i)
            h[i] = (float)(((i + (size_t)z * 7919u) * 2654435761u) % 1000) * 0.1f;
        CK(hipMemcpy(in + (size_t)z * n * n, h.data(), h.size() * 4, hipMemcpyHostToDevice));
    }
    constexpr int L = 7;
    GaussZYX p{};
    p.outer = 1; p.len = L;
    for (int d = 0; d < 3; ++d) { p.n[d] = n; p.on[d] = n; p.o0[d] = 0; }
    const float w7[7] = {0.00443305f, 0.05400558f, 0.24203623f, 0.39905028f, 0.24203623f, 0.05400558f, 0.00443305f};
    for (int d = 0; d < 3; ++d) for (int i = 0; i < L; ++i) p.w[d][i] = w7[i];
    const int tiles_x = (n + kZYXTx - 1) / kZYXTx, tiles_y = (n + kZYXTy - 1) / kZYXTy;
    const int64_t tiles = (int64_t)tiles_x * tiles_y;
    const int64_t per_cu = 1024 / GV_NT;  // workgroups per CU at 4 waves per SIMD
    const int64_t want = (256 * per_cu * 2 + tiles - 1) / tiles;
    int64_t nseg = std::max<int64_t>(1, std::min<int64_t>(want, (n + kZYXSegMin - 1) / kZYXSegMin));
    if (argc > 3) nseg = atoi(argv[3]);
    const int zseg = (int)((n + nseg - 1) / nseg);
    nseg = (n + zseg - 1) / zseg;
    hipStream_t s; CK(hipStreamCreate(&s));
    auto launch = [&]() {
        hipLaunchKernelGGL((gauss_zyx_kernel<L, float, true>), dim3((unsigned)(tiles * nseg), 1), dim3(GV_NT), 0, s,
                           in, out, p, tiles_x, tiles_y, zseg);
        CK(hipGetLastError());
    };
    hipEvent_t a, b;
    CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
    launch();
    std::vector<float> t;
    for (int r = 0; r < 7; ++r) {
        CK(hipEventRecord(a, s)); launch(); CK(hipEventRecord(b, s)); CK(hipEventSynchronize(b));
        float ms; CK(hipEventElapsedTime(&ms, a, b)); t.push_back(ms);
    }
    std::sort(t.begin(), t.end());
    double sum = 0.0;
    for (int z : {0, 5, n / 2, n - 1}) {
        CK(hipMemcpy(h.data(), out + (size_t)z * n * n, h.size() * 4, hipMemcpyDeviceToHost));
        for (float v : h) sum += v;
    }
    printf("%-16s median %7.3f ms  min %7.3f ms  %6.1f GB/s  nseg %lld  checksum %.9e\n", tag, t[3], t[0],
           8.0 * vox / (t[3] * 1e6), (long long)nseg, sum);
    return 0;
}
