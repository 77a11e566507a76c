// Memory-only skeleton of the fused guided-filter march (gf3d_fused_kernel, gf_fused.hpp) at
// 2048^3 r=4: the same grid (64 x 32 tiles, 1024 threads, z-segments of 512 slices), the same
// XCD-aware block -> tile map (4 x 16 super-tiles) and, per z-step, the same global accesses:
//   entering slice zc+R and leaving slice zc-R-1 over the (64+4R) x (32+4R) stage-1 apron,
//   v at zc over the (64+2R) x (32+2R) stage-2 apron (P3), v at zc-R over the tile (P5),
//   one 64 x 32 output slice store (non-temporal).
// No compute and no LDS: the loads are folded into a running sum that feeds the stores (and an
// opaque never-taken store on the threads that emit nothing), so none of them can be dropped.
// SK_BAR = number of workgroup barriers per step (the product has 2); SK_PF = D issues every load D steps
// ahead (0: none); argv[2] = dynamic LDS bytes per workgroup (96 KiB: one workgroup per CU,
// as the product's 123 VGPRs allow). Prints the time per launch
// and the algorithmic rate (8 B per output voxel) — the floor this access pattern allows.
// Build: hipcc --offload-arch=gfx950 -O3 -DSK_BAR=0 tools/skeleton.hip -o tools/sk_b0
// Run (GPU box): tools/sk_b0 [n=2048] [lds bytes=0]
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#ifndef SK_BAR
#define SK_BAR 0
#endif
#ifndef SK_PF
#define SK_PF 0
#endif
// Ablations: SK_NOLEAVE drops the leaving-slice load, SK_NOP3 the P3 load, SK_NOP5 the P5 load,
// SK_M1 sets the stage-1 apron margin (2R in the product; 0 = the tile only).
#ifndef SK_M1
#define SK_M1 (2 * R)
#endif
#ifndef SK_NOLEAVE
#define SK_NOLEAVE 0
#endif
#ifndef SK_NOP3
#define SK_NOP3 0
#endif
#ifndef SK_NOP5
#define SK_NOP5 0
#endif
#ifndef SK_STAUX
#define SK_STAUX 2  // output store cache bits (2 = nt, 16 = sc1: written through, dropped from L2)
#endif
#ifndef SK_PADX
#define SK_PADX 0  // row pitch n + PADX elements
#endif
#ifndef SK_PADY
#define SK_PADY 0  // slice pitch (n + PADY) rows
#endif
#ifndef SK_LDIST
#define SK_LDIST (2 * R + 1)  // z distance of the leaving-slice re-read (0: the entering slice again)
#endif
#ifndef SK_NOSTORE
#define SK_NOSTORE 0  // 1: no output stores (the loads still feed an opaque never-taken store)
#endif
#ifndef SK_RINGBUF
#define SK_RINGBUF 0  // 1: the leaving slice from a per-workgroup ring of the entering quads in global
                      // memory (16 B per lane per slot, coalesced), written as they enter
#endif
#ifndef SK_TX
#define SK_TX 64
#endif
#ifndef SK_STX
#define SK_STX 4
#endif
#ifndef SK_STY
#define SK_STY 16
#endif
#ifndef SK_TY
#define SK_TY (2048 / SK_TX)  // tile height (64 x 16: half the co-resident L2 footprint per XCD)
#endif
constexpr int R = 4, TX = SK_TX, TY = SK_TY, NT = 1024, STX = SK_STX, STY = SK_STY;

#define CK(x)                                                                              \
    do {                                                                                   \
        hipError_t e_ = (x);                                                               \
        if (e_ != hipSuccess) {                                                            \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));      \
            exit(1);                                                                       \
        }                                                                                  \
    } while (0)

// Branch-free 16-byte buffer loads (as the product's): a slice outside [0, n) gets an empty
// descriptor and an item outside the domain an out-of-range offset, both read 0.
__device__ __forceinline__ float4 ld(const float* base, long slice, int n, int z, int off) {
    typedef unsigned int u4 __attribute__((ext_vector_type(4)));
    const bool ok = (unsigned)z < (unsigned)n;
    const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<float*>(base + (ok ? (long)z * slice : 0)), (short)0,
        ok ? (int)(slice * 4) : 0, 0x00020000);
    const u4 q = __builtin_amdgcn_raw_buffer_load_b128(r, off < 0 ? (int)0x80000000 : off * 4, 0, 0);
    return make_float4(__uint_as_float(q.x), __uint_as_float(q.y), __uint_as_float(q.z),
                       __uint_as_float(q.w));
}

// Quad `q` of a (W + 2m) x (TY + 2m) apron around the tile at (x0, y0): element offset or -1.
template <int M>
__device__ __forceinline__ int apron_off(int q, int x0, int y0, int n) {
    constexpr int QX = (TX + 2 * M) / 4, QY = TY + 2 * M;
    if (q >= QX * QY) return -1;
    const int gx = x0 - M + 4 * (q % QX), gy = y0 - M + q / QX;
    if (gy < 0 || gy >= n || gx < 0 || gx + 3 >= n) return -1;  // n is a multiple of 4
    return gy * (n + SK_PADX) + gx;
}

__global__ __launch_bounds__(NT) void skeleton_kernel(const float* __restrict__ in,
                                                      float* __restrict__ out, int n, int zseg,
                                                      float* dummy, float4* ringbuf) {
    extern __shared__ float sk_lds[];  // occupancy only (argv[2]); never touched
    const int nwg = gridDim.x, b = blockIdx.x;
    const int lid = (nwg % 8 == 0) ? (b % 8) * (nwg / 8) + b / 8 : b;
    const int gtx = n / TX, gty = n / TY, ntiles = gtx * gty;
    const int seg = lid / ntiles;
    int t = lid % ntiles;
    const int per_srow = gtx * STY;
    const int sr = t / per_srow, r = t % per_srow;
    const int tile_x = (r / (STX * STY)) * STX + r % STX;
    const int tile_y = sr * STY + (r / STX) % STY;
    const int x0 = tile_x * TX, y0 = tile_y * TY;
    const long slice = (long)(n + SK_PADX) * (n + SK_PADY);
    const int zo_begin = seg * zseg, zo_end = min(zo_begin + zseg, n);
    const int tid = threadIdx.x;

    // items per thread of the stage-1 and P3 aprons (more than one for tiles wider than 64)
    constexpr int K1 = ((TX + 2 * SK_M1) / 4 * (TY + 2 * SK_M1) + NT - 1) / NT;
    constexpr int K3 = ((TX + 2 * R) / 4 * (TY + 2 * R) + NT - 1) / NT;
    int o1[K1], o1l[K1], o3l[K3];
#pragma unroll
    for (int k = 0; k < K1; ++k) {
        o1[k] = apron_off<SK_M1>(tid + k * NT, x0, y0, n);  // stage-1 apron quad
        o1l[k] = SK_NOLEAVE ? -1 : o1[k];
    }
#pragma unroll
    for (int k = 0; k < K3; ++k) o3l[k] = SK_NOP3 ? -1 : apron_off<R>(tid + k * NT, x0, y0, n);
    const int o5 = apron_off<0>(tid, x0, y0, n);  // tile quad (P5 v and the output)
    const int o5l = SK_NOP5 ? -1 : o5;
    float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
    auto add = [&](const float4& e, float sgn) {
        acc.x += sgn * e.x; acc.y += sgn * e.y; acc.z += sgn * e.z; acc.w += sgn * e.w;
    };
    // seed: the z-window before the first stage-1 slice (2R + 1 slices)
    for (int z = zo_begin - 2 * R - 1; z < zo_begin; ++z)
#pragma unroll
        for (int k = 0; k < K1; ++k) add(ld(in, slice, n, z, o1[k]), 1.f);
    typedef float f4 __attribute__((ext_vector_type(4)));
    struct Step {
        float4 e[K1], l[K1], c[K3], v;
    };
    constexpr int WR = 2 * R + 1;  // ring slots (the leaving slice entered WR steps earlier)
    float4* const myring = ringbuf + (long)b * WR * K1 * NT;
    auto rslot = [&](int zc) { return ((zc % WR) + WR) % WR; };
    auto load = [&](int zc, Step& s) {
#pragma unroll
        for (int k = 0; k < K1; ++k) {
            s.e[k] = ld(in, slice, n, zc + R, o1[k]);
            if (SK_RINGBUF)
                s.l[k] = myring[(rslot(zc) * K1 + k) * NT + tid];
            else
                s.l[k] = ld(in, slice, n, zc + R - SK_LDIST, o1l[k]);
        }
#pragma unroll
        for (int k = 0; k < K3; ++k) s.c[k] = ld(in, slice, n, zc, o3l[k]);
        s.v = ld(in, slice, n, zc - R, o5l);
    };
    auto step = [&](int zc, const Step& s) {
#pragma unroll
        for (int k = 0; k < K1; ++k) { add(s.e[k], 1.f); add(s.l[k], -1.f); }
        if (SK_RINGBUF) {
#pragma unroll
            for (int k = 0; k < K1; ++k) myring[(rslot(zc) * K1 + k) * NT + tid] = s.e[k];
        }
#pragma unroll
        for (int k = 0; k < K3; ++k) add(s.c[k], 1.f);
#if SK_BAR >= 1
        __builtin_amdgcn_s_barrier();
#endif
        const int zo = zc - R;
        if (zo >= zo_begin) {
            const float4 v = s.v;
            const float4 w = make_float4(acc.x * v.x, acc.y * v.y, acc.z * v.z, acc.w * v.w);
            if (o5 >= 0 && !SK_NOSTORE) {
                typedef unsigned int u4 __attribute__((ext_vector_type(4)));
                const u4 wv = {__float_as_uint(w.x), __float_as_uint(w.y), __float_as_uint(w.z),
                               __float_as_uint(w.w)};
                const __amdgpu_buffer_rsrc_t ro = __builtin_amdgcn_make_buffer_rsrc(
                    out + (long)zo * slice, (short)0, (int)(slice * 4), 0x00020000);
                __builtin_amdgcn_raw_buffer_store_b128(wv, ro, o5 * 4, 0, SK_STAUX);
            } else if (w.x == 1.2345e-30f && (SK_NOSTORE || w.y == -7.5e-31f)) {
                dummy[tid] = w.z + w.w;  // never taken: keeps the apron-only threads' loads live
            }
        }
#if SK_BAR >= 2
        __builtin_amdgcn_s_barrier();
#endif
    };
    const int zc0 = zo_begin - R, zc1 = zo_end + R;  // steps; (zc1 - zc0) % max(SK_PF, 1) == 0
#if SK_PF == 0
    for (int zc = zc0; zc < zc1; ++zc) {
        Step s;
        load(zc, s);
        step(zc, s);
    }
#else
    // every load of step zc issued SK_PF steps ahead (slot j of a ring, compile-time index)
    constexpr int D = SK_PF;
    Step ring[D];
#pragma unroll
    for (int j = 0; j < D; ++j) load(zc0 + j, ring[j]);
    for (int zb = zc0; zb < zc1; zb += D) {
#pragma unroll
        for (int j = 0; j < D; ++j) {
            const Step cur = ring[j];
            load(zb + j + D, ring[j]);  // past zc1: harmless extra loads
            step(zb + j, cur);
        }
    }
#endif
}

__global__ void fill_kernel(float* p, long count) {
    for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < count;
         i += (long)gridDim.x * blockDim.x) {
        unsigned h = (unsigned)(i * 2654435761u) ^ (unsigned)(i >> 13);
        p[i] = (float)(h & 0xFFFF);
    }
}

int main(int argc, char** argv) {
    const int n = argc > 1 ? atoi(argv[1]) : 2048;
    const int lds = argc > 2 ? atoi(argv[2]) : 0;
    const int zseg = 512;
    if (n % TX || n % TY || n % zseg) {
        fprintf(stderr, "n must be a multiple of %d\n", zseg);
        return 1;
    }
    const long count = (long)(n + SK_PADX) * (n + SK_PADY) * n;
    float *in, *out, *dummy;
    CK(hipMalloc(&in, count * 4));
    CK(hipMalloc(&out, count * 4));
    CK(hipMalloc(&dummy, NT * 4));
    float4* ringbuf = nullptr;
    {
        constexpr int K1h = ((TX + 2 * SK_M1) / 4 * (TY + 2 * SK_M1) + NT - 1) / NT;
        const long nwg0 = (long)(n / TX) * (n / TY) * (n / 512);
        CK(hipMalloc(&ringbuf, nwg0 * (2 * R + 1) * K1h * NT * sizeof(float4)));
        CK(hipMemset(ringbuf, 0, nwg0 * (2 * R + 1) * K1h * NT * sizeof(float4)));
    }
    fill_kernel<<<4096, 256>>>(in, count);
    CK(hipGetLastError());
    const int nwg = (n / TX) * (n / TY) * (n / zseg);
    if (lds > 0) CK(hipFuncSetAttribute((const void*)skeleton_kernel,
                                        hipFuncAttributeMaxDynamicSharedMemorySize, lds));
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    float best = 1e30f, sum = 0.f;
    const int reps = 7;
    for (int i = 0; i < reps + 1; ++i) {
        CK(hipEventRecord(a));
        skeleton_kernel<<<nwg, NT, lds>>>(in, out, n, zseg, dummy, ringbuf);
        CK(hipEventRecord(b));
        CK(hipEventSynchronize(b));
        CK(hipGetLastError());
        float ms;
        CK(hipEventElapsedTime(&ms, a, b));
        if (i > 0) {  // first launch is warm-up
            sum += ms;
            if (ms < best) best = ms;
        }
    }
    const double gb = (double)count * 8 / 1e9;
    printf("skeleton RINGBUF=%d TY=%d LDIST=%d NOSTORE=%d ST=%dx%d PAD=%d,%d STAUX=%d SK_BAR=%d SK_PF=%d TX=%d M1=%d noleave=%d noP3=%d noP5=%d lds=%d n=%d wg=%d: mean %.3f ms min %.3f ms (%.1f GB/s algorithmic)\n",
           SK_RINGBUF, TY, SK_LDIST, SK_NOSTORE, STX, STY, SK_PADX, SK_PADY, SK_STAUX, SK_BAR, SK_PF, TX, SK_M1, SK_NOLEAVE, SK_NOP3, SK_NOP5, lds, n, nwg, sum / reps, best, gb / (sum / reps) * 1e3);
    CK(hipFree(in));
    CK(hipFree(out));
    CK(hipFree(dummy));
    return 0;
}
