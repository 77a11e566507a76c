// zt_api.hip — the C ABI (include/zarrs_tools_amd.h): validation, geometry and launches.
//
// Host-side restatement of the reference's per-chunk orchestration around the kernels:
//   chunk_subset_bounded + ArraySubsetOverlap::new/extract_subset (guided_filter.rs:87-103,
//   array_subset_overlap.rs:11-51), Downsample::input_subset/output_shape (downsample.rs:64-70,
//   :162-168), is_compatible/memory_per_chunk (guided_filter.rs:203-238, downsample.rs:124-160),
//   and the zarrs_ome level loop's shapes and stop rule (zarrs_ome.rs:515-560, :731-737).

#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <string>
#include <vector>

#include "../../include/zarrs_tools_amd.h"
#include "zt_device.hpp"
#include "zt_kernels.hpp"

namespace {

thread_local std::string g_last_error;

int fail(int code, const char* fmt, ...) {
    char buf[1024];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof(buf), fmt, ap);
    va_end(ap);
    g_last_error = buf;
    return code;
}

int hip_fail(hipError_t e, const char* what) {
    return fail(ZT_ERR_DEVICE, "%s: %s", what, hipGetErrorString(e));
}

#define ZT_HIP(call)                                                                             \
    do {                                                                                         \
        hipError_t _e = (call);                                                                  \
        if (_e != hipSuccess) return hip_fail(_e, #call);                                        \
    } while (0)

bool valid_dtype(int d) { return d >= ZT_BOOL && d <= ZT_FLOAT64; }

const char* dtype_name(int d) {
    static const char* names[] = {"bool",   "int8",   "int16",    "int32",   "int64",
                                  "uint8",  "uint16", "uint32",   "uint64",  "bfloat16",
                                  "float16", "float32", "float64"};
    return valid_dtype(d) ? names[d] : "unknown";
}

}  // namespace

struct zt_ctx {
    int device = 0;
    hipStream_t own = nullptr;
    hipStream_t cur = nullptr;
    hipEvent_t ev0 = nullptr, ev1 = nullptr;
    bool timed = false;
    void* scratch = nullptr;
    size_t scratch_bytes = 0;

    int ensure_scratch(size_t bytes) {
        if (bytes <= scratch_bytes) return ZT_OK;
        if (scratch) {
            (void)hipStreamSynchronize(cur);
            (void)hipFree(scratch);
            scratch = nullptr;
            scratch_bytes = 0;
        }
        hipError_t e = hipMalloc(&scratch, bytes);
        if (e != hipSuccess) {
            (void)hipGetLastError();
            return fail(ZT_ERR_OUT_OF_MEMORY, "device scratch of %zu bytes: %s", bytes,
                        hipGetErrorString(e));
        }
        scratch_bytes = bytes;
        return ZT_OK;
    }
};

namespace {

struct DeviceGuard {
    int prev = -1;
    explicit DeviceGuard(int dev) {
        if (hipGetDevice(&prev) != hipSuccess) prev = -1;
        if (prev != dev) (void)hipSetDevice(dev);
    }
    ~DeviceGuard() {
        int now = -1;
        if (prev >= 0 && hipGetDevice(&now) == hipSuccess && now != prev) (void)hipSetDevice(prev);
    }
};

int check_ctx(zt_ctx* ctx) {
    if (!ctx) return fail(ZT_ERR_INVALID_PARAMETERS, "null context");
    return ZT_OK;
}

int check_shape(const int64_t* shape, int ndim, const char* what) {
    if (ndim < 1 || ndim > ZT_MAX_DIMS)
        return fail(ZT_ERR_INVALID_PARAMETERS, "%s: ndim %d not in [1, %d]", what, ndim,
                    ZT_MAX_DIMS);
    if (!shape) return fail(ZT_ERR_INVALID_PARAMETERS, "%s: null shape", what);
    for (int d = 0; d < ndim; ++d)
        if (shape[d] < 0) return fail(ZT_ERR_INVALID_PARAMETERS, "%s: negative extent", what);
    return ZT_OK;
}

int64_t numel(const int64_t* s, int n) {
    int64_t r = 1;
    for (int i = 0; i < n; ++i) r *= s[i];
    return r;
}

void c_strides(const int64_t* shape, int ndim, int64_t* strides) {
    int64_t s = 1;
    for (int d = ndim - 1; d >= 0; --d) {
        strides[d] = s;
        s *= shape[d];
    }
}

// Choose the z-march length for a fused launch: whole chunk depths when there is enough
// parallelism, shorter segments for a single small block. Segments are a free choice (windows
// are clamped at the array, not the segment), so large launches march two chunk depths while
// they keep >= 4096 workgroups (16 per CU): each segment re-fills its z-windows over 2r + 1
// warm-up slices and pads its steps to a multiple of 2r + 1 (2048^3 r=4: 31.4 -> 30.6 ms;
// 384- and 1024-slice segments measured slower, tools/timek.sh; profiles/r02_ab_harness.txt).
int choose_zseg(int onz, int tiles, int radius, int chunk_depth) {
    const int target_wg = 1024;
    int zseg = chunk_depth > 0 ? std::min(chunk_depth, onz) : onz;
    if (zseg <= 0) zseg = 1;
    if (chunk_depth > 0 && radius <= 2) {
        // short windows (5-slice warm-up): up to 4 chunk depths while >= 512 workgroups (2 per CU)
        // remain (1024^3 r=2: 3.46 -> 3.33 ms for one 1024-slice segment per tile)
        for (int m = 4; m >= 2; m /= 2)
            if ((int64_t)m * chunk_depth <= onz &&
                (int64_t)tiles * ((onz + m * chunk_depth - 1) / (m * chunk_depth)) >= 512) {
                zseg = m * chunk_depth;
                break;
            }
    } else if (chunk_depth > 0 && 2LL * chunk_depth <= onz &&
               (int64_t)tiles * ((onz + 2 * chunk_depth - 1) / (2 * chunk_depth)) >= 4096) {
        zseg = 2 * chunk_depth;
    }
    int64_t wg = (int64_t)tiles * ((onz + zseg - 1) / zseg);
    if (wg < target_wg && chunk_depth <= 0) {
        int nseg = (target_wg + tiles - 1) / std::max(tiles, 1);
        int minseg = std::max(8, 4 * radius);
        zseg = std::max(minseg, (onz + nseg - 1) / nseg);
        zseg = std::min(zseg, onz);
    }
    return zseg;
}

int radius_ok(int radius) {
    if (radius < 0 || radius > zt::kMaxRadius)
        return fail(ZT_ERR_INVALID_PARAMETERS,
                    "radius %d not in [0, %d] (the reference's u8 halo radius*2 overflows)", radius,
                    zt::kMaxRadius);
    return ZT_OK;
}

int dtypes_ok(int dtype_in, int dtype_out) {
    if (!valid_dtype(dtype_in))
        return fail(ZT_ERR_UNSUPPORTED_DATA_TYPE, "Unsupported data type code %d", dtype_in);
    if (!valid_dtype(dtype_out))
        return fail(ZT_ERR_UNSUPPORTED_DATA_TYPE, "Unsupported data type code %d", dtype_out);
    return ZT_OK;
}

// The fused kernel addresses each z-plane through a buffer descriptor with 32-bit byte offsets
// (gf_fused.hpp: slice_rsrc, int row strides): every input plane and output plane it touches must
// span < 2^31 bytes, measured after the f32 staging run_fused3 may insert. Larger planes go to
// the separable path (64-bit indexing) instead of silently reading zeros past the range.
bool fused_planes_fit(const int64_t dom[3], int64_t in_sy, const int64_t oshape[3],
                      int64_t out_sy, int dtype_in, int dtype_out) {
    const bool stage_in = !zt::fused_direct_pair(dtype_in, zt::kF32);
    const bool stage_out = !zt::fused_direct_pair(zt::kF32, dtype_out);
    const int64_t isy = stage_in ? dom[2] : in_sy, osy = stage_out ? oshape[2] : out_sy;
    const int64_t iesz = stage_in ? 4 : (int64_t)zt::dtype_size(dtype_in);
    const int64_t oesz = stage_out ? 4 : (int64_t)zt::dtype_size(dtype_out);
    const int64_t lim = (int64_t)INT32_MAX - 16;  // + one quad of slack past the last element
    if (dom[1] <= 0 || dom[2] <= 0 || oshape[1] <= 0 || oshape[2] <= 0) return true;
    const int64_t ib = ((dom[1] - 1) * isy + dom[2]) * iesz;
    const int64_t ob = ((oshape[1] - 1) * osy + oshape[2]) * oesz;
    return ib <= lim && ob <= lim && dom[1] <= INT32_MAX && dom[2] <= INT32_MAX &&
           dom[0] <= INT32_MAX;
}

// Fused launch on a 3-D view (pad 1-2 D arrays with leading unit axes).
int run_fused3(zt_ctx* ctx, int dtype_in, const void* in, const int64_t dom[3], int64_t in_z0,
               int64_t in_rows, int64_t in_sz, int64_t in_sy, const int64_t ostart[3],
               const int64_t oshape[3], int dtype_out, void* out, int64_t out_sz, int64_t out_sy,
               float eps, int radius, int chunk_depth) {
    for (int d = 0; d < 3; ++d)
        if (dom[d] > INT32_MAX || oshape[d] > INT32_MAX)
            return fail(ZT_ERR_INVALID_PARAMETERS, "extent exceeds 2^31-1");
    if (!fused_planes_fit(dom, in_sy, oshape, out_sy, dtype_in, dtype_out))
        return fail(ZT_ERR_INVALID_PARAMETERS, "fused path: a z-plane spans >= 2 GiB");
    zt::GFParams p{};
    p.in = in;
    p.out = out;
    p.in_sz = in_sz;
    p.in_sy = in_sy;
    p.out_sz = out_sz;
    p.out_sy = out_sy;
    p.in_z0 = (int)in_z0;
    p.zlo = (int)std::max<int64_t>(0, in_z0);
    p.zhi = (int)std::min<int64_t>(dom[0], in_z0 + in_rows);
    p.nz = (int)dom[0];
    p.ny = (int)dom[1];
    p.nx = (int)dom[2];
    p.oz0 = (int)ostart[0];
    p.oy0 = (int)ostart[1];
    p.ox0 = (int)ostart[2];
    p.onz = (int)oshape[0];
    p.ony = (int)oshape[1];
    p.onx = (int)oshape[2];
    p.eps = eps;
    if (p.onz == 0 || p.ony == 0 || p.onx == 0) return ZT_OK;
    // Pairs without a direct instantiation: stage the input rows and/or the output region
    // through contiguous f32 scratch (cast kernels with the same Rust `as` semantics).
    const bool stage_in = !zt::fused_direct_pair(dtype_in, zt::kF32);
    const bool stage_out = !zt::fused_direct_pair(zt::kF32, dtype_out);
    const int64_t in_elems = stage_in ? in_rows * dom[1] * dom[2] : 0;
    const int64_t out_elems = stage_out ? oshape[0] * oshape[1] * oshape[2] : 0;
    if (stage_in || stage_out) {
        int rc = ctx->ensure_scratch(sizeof(float) * (size_t)(in_elems + out_elems));
        if (rc) return rc;
    }
    float* sin = static_cast<float*>(ctx->scratch);
    float* sout = sin + in_elems;
    if (stage_in) {
        hipError_t e = zt::launch_cast_to_f32_3d(in, dtype_in, in_sz, in_sy, sin, in_rows, dom[1],
                                                 dom[2], ctx->cur);
        if (e != hipSuccess) return hip_fail(e, "input staging cast");
        p.in = sin;
        p.in_sz = dom[1] * dom[2];
        p.in_sy = dom[2];
        dtype_in = zt::kF32;
    }
    if (stage_out) {
        p.out = sout;
        p.out_sz = oshape[1] * oshape[2];
        p.out_sy = oshape[2];
    }
    const int ty = zt::fused_tile_y(radius);
    int tiles = (int)(((p.onx + 63) / 64) * ((p.ony + ty - 1) / ty));
    p.zseg = choose_zseg(p.onz, tiles, radius, chunk_depth);
    if (ctx->timed) ZT_HIP(hipEventRecord(ctx->ev0, ctx->cur));
    hipError_t e = zt::launch_guided_fused(p, dtype_in, stage_out ? (int)zt::kF32 : dtype_out,
                                           radius, ctx->cur);
    if (e != hipSuccess) return hip_fail(e, "guided filter fused kernel launch");
    if (ctx->timed) ZT_HIP(hipEventRecord(ctx->ev1, ctx->cur));
    if (stage_out) {
        e = zt::launch_cast_from_f32_3d(sout, dtype_out, out, out_sz, out_sy, oshape[0],
                                        oshape[1], oshape[2], ctx->cur);
        if (e != hipSuccess) return hip_fail(e, "output staging cast");
    }
    return ZT_OK;
}

int run_separable(zt_ctx* ctx, int dtype_in, const void* in, const int64_t* shape,
                  const int64_t* in_strides, int ndim, const int64_t* out_start,
                  const int64_t* out_shape, int dtype_out, void* out, const int64_t* out_strides,
                  float eps, int radius) {
    zt::NdGeom g{};
    g.ndim = ndim;
    g.numel = numel(shape, ndim);
    g.out_numel = numel(out_shape, ndim);
    for (int d = 0; d < ndim; ++d) {
        g.shape[d] = shape[d];
        g.in_strides[d] = in_strides[d];
        g.out_start[d] = out_start[d];
        g.out_shape[d] = out_shape[d];
        g.out_strides[d] = out_strides[d];
    }
    if (g.numel == 0 || g.out_numel == 0) return ZT_OK;
    int rc = ctx->ensure_scratch(sizeof(float) * (size_t)zt::separable_scratch_floats(g.numel));
    if (rc) return rc;
    if (ctx->timed) ZT_HIP(hipEventRecord(ctx->ev0, ctx->cur));
    hipError_t e = zt::launch_guided_separable(in, dtype_in, out, dtype_out, g, radius, eps,
                                               static_cast<float*>(ctx->scratch), ctx->cur);
    if (e != hipSuccess) return hip_fail(e, "guided filter separable launch");
    if (ctx->timed) ZT_HIP(hipEventRecord(ctx->ev1, ctx->cur));
    return ZT_OK;
}

// 4-D blocks (config T): guided4d.hip when the radius fits it and x is the unit-stride axis;
// the scratch holds U3/S3, AB and (for other element types or strides) f32 v.
bool use_guided4d(int ndim, int radius, const int64_t* in_strides, const int64_t* shape) {
    return ndim == 4 && zt::guided4d_supports(radius) && in_strides[3] == 1 && shape[0] <= 32 &&
           shape[1] <= 0x7FFFFFFF && shape[2] <= 65535 && shape[3] <= 0x7FFFFFFF;
}

int run_guided4d(zt_ctx* ctx, int dtype_in, const void* in, const int64_t* shape,
                 const int64_t* in_strides, const int64_t* out_start, const int64_t* out_shape,
                 int dtype_out, void* out, const int64_t* out_strides, float eps, int radius) {
    zt::NdGeom g{};
    g.ndim = 4;
    g.numel = numel(shape, 4);
    g.out_numel = numel(out_shape, 4);
    for (int d = 0; d < 4; ++d) {
        g.shape[d] = shape[d];
        g.in_strides[d] = in_strides[d];
        g.out_start[d] = out_start[d];
        g.out_shape[d] = out_shape[d];
        g.out_strides[d] = out_strides[d];
        if (shape[d] > INT32_MAX) return fail(ZT_ERR_INVALID_PARAMETERS, "extent exceeds 2^31-1");
    }
    if (g.numel == 0 || g.out_numel == 0) return ZT_OK;
    // T <= 4, r <= 2: the one-march kernel (g4_fused.hip)
    if (zt::guided4d_fused_supports(radius, g)) {
        bool contiguous = dtype_in == zt::kF32;
        int64_t st = 1;
        for (int d = 3; d >= 0; --d) {
            if (in_strides[d] != st) contiguous = false;
            st *= shape[d];
        }
        const float* v = static_cast<const float*>(in);
        if (!contiguous) {  // f32 C-order copy of the block in scratch
            if (int rc = ctx->ensure_scratch(sizeof(float) * (size_t)g.numel)) return rc;
            float* vv = static_cast<float*>(ctx->scratch);
            const size_t esz = zt::dtype_size(dtype_in);
            for (int64_t t = 0; t < shape[0]; ++t) {
                hipError_t e = zt::launch_cast_to_f32_3d(
                    static_cast<const char*>(in) + esz * t * in_strides[0], dtype_in, in_strides[1],
                    in_strides[2], vv + t * shape[1] * shape[2] * shape[3], shape[1], shape[2],
                    shape[3], ctx->cur);
                if (e != hipSuccess) return hip_fail(e, "guided filter 4-D input cast");
            }
            v = vv;
        }
        if (ctx->timed) ZT_HIP(hipEventRecord(ctx->ev0, ctx->cur));
        hipError_t e = zt::launch_guided4d_fused(v, out, dtype_out, g, radius, eps, ctx->cur);
        if (e != hipSuccess) return hip_fail(e, "guided filter 4-D fused launch");
        if (ctx->timed) ZT_HIP(hipEventRecord(ctx->ev1, ctx->cur));
        return ZT_OK;
    }
    if (int rc = ctx->ensure_scratch((size_t)zt::guided4d_scratch_bytes(g.numel, true))) return rc;
    if (ctx->timed) ZT_HIP(hipEventRecord(ctx->ev0, ctx->cur));
    hipError_t e = zt::launch_guided4d(in, dtype_in, out, dtype_out, g, radius, eps,
                                       ctx->scratch, ctx->cur);
    if (e != hipSuccess) return hip_fail(e, "guided filter 4-D launch");
    if (ctx->timed) ZT_HIP(hipEventRecord(ctx->ev1, ctx->cur));
    return ZT_OK;
}

}  // namespace

namespace zt {
// Used by the host store / pipeline code (host/*.cpp) to report errors through zt_last_error().
int set_last_error(int code, const char* msg) {
    g_last_error = msg ? msg : "";
    return code;
}
}  // namespace zt

extern "C" {

int zt_abi_version(void) { return ZT_ABI_VERSION; }

const char* zt_last_error(void) { return g_last_error.c_str(); }

size_t zt_dtype_size(int dtype) { return zt::dtype_size(dtype); }

int zt_device_count(int* count) {
    if (!count) return fail(ZT_ERR_INVALID_PARAMETERS, "null count");
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) {
        (void)hipGetLastError();
        n = 0;
    }
    *count = n;
    return ZT_OK;
}

int zt_ctx_create(int device, zt_ctx** out) {
    if (!out) return fail(ZT_ERR_INVALID_PARAMETERS, "null output pointer");
    *out = nullptr;
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n == 0) {
        (void)hipGetLastError();
        return fail(ZT_ERR_DEVICE, "no HIP device available");
    }
    if (device < 0 || device >= n)
        return fail(ZT_ERR_INVALID_PARAMETERS, "device %d not in [0, %d)", device, n);
    ZT_HIP(hipSetDevice(device));
    zt_ctx* c = new zt_ctx();
    c->device = device;
    if (hipStreamCreateWithFlags(&c->own, hipStreamNonBlocking) != hipSuccess ||
        hipEventCreate(&c->ev0) != hipSuccess || hipEventCreate(&c->ev1) != hipSuccess) {
        delete c;
        return fail(ZT_ERR_DEVICE, "stream/event creation failed");
    }
    c->cur = c->own;
    c->timed = true;
    *out = c;
    return ZT_OK;
}

int zt_ctx_destroy(zt_ctx* ctx) {
    if (!ctx) return ZT_OK;
    DeviceGuard g(ctx->device);
    (void)hipStreamSynchronize(ctx->cur);
    if (ctx->scratch) (void)hipFree(ctx->scratch);
    if (ctx->ev0) (void)hipEventDestroy(ctx->ev0);
    if (ctx->ev1) (void)hipEventDestroy(ctx->ev1);
    if (ctx->own) (void)hipStreamDestroy(ctx->own);
    delete ctx;
    return ZT_OK;
}

int zt_ctx_set_stream(zt_ctx* ctx, void* hip_stream) {
    if (int rc = check_ctx(ctx)) return rc;
    // Used verbatim: NULL is the device's default (null) stream, which is what
    // torch.cuda.current_stream().cuda_stream returns for torch's default stream.
    ctx->cur = static_cast<hipStream_t>(hip_stream);
    return ZT_OK;
}

int zt_ctx_use_own_stream(zt_ctx* ctx) {
    if (int rc = check_ctx(ctx)) return rc;
    ctx->cur = ctx->own;
    return ZT_OK;
}

int zt_ctx_get_stream(zt_ctx* ctx, void** hip_stream) {
    if (int rc = check_ctx(ctx)) return rc;
    if (!hip_stream) return fail(ZT_ERR_INVALID_PARAMETERS, "null output pointer");
    *hip_stream = ctx->cur;
    return ZT_OK;
}

int zt_ctx_synchronize(zt_ctx* ctx) {
    if (int rc = check_ctx(ctx)) return rc;
    DeviceGuard g(ctx->device);
    ZT_HIP(hipStreamSynchronize(ctx->cur));
    return ZT_OK;
}

int zt_ctx_scratch_bytes(zt_ctx* ctx, uint64_t* bytes) {
    if (int rc = check_ctx(ctx)) return rc;
    if (!bytes) return fail(ZT_ERR_INVALID_PARAMETERS, "null output pointer");
    *bytes = ctx->scratch_bytes;
    return ZT_OK;
}

int zt_ctx_release_scratch(zt_ctx* ctx) {
    if (int rc = check_ctx(ctx)) return rc;
    DeviceGuard g(ctx->device);
    if (ctx->scratch) {
        ZT_HIP(hipStreamSynchronize(ctx->cur));
        ZT_HIP(hipFree(ctx->scratch));
        ctx->scratch = nullptr;
        ctx->scratch_bytes = 0;
    }
    return ZT_OK;
}

int zt_ctx_last_kernel_ms(zt_ctx* ctx, float* ms) {
    if (int rc = check_ctx(ctx)) return rc;
    if (!ms) return fail(ZT_ERR_INVALID_PARAMETERS, "null output pointer");
    DeviceGuard g(ctx->device);
    ZT_HIP(hipEventElapsedTime(ms, ctx->ev0, ctx->ev1));
    return ZT_OK;
}

// ---- guided filter ---------------------------------------------------------------------------

int zt_guided_filter_is_compatible(int dtype_in, int dtype_out) {
    // guided_filter.rs:208-224: every listed type is accepted for input and output.
    return dtypes_ok(dtype_in, dtype_out);
}

int zt_guided_filter_memory_per_chunk(int dtype_in, int dtype_out, const int64_t* chunk_shape,
                                      int ndim, uint64_t* bytes) {
    if (int rc = dtypes_ok(dtype_in, dtype_out)) return rc;
    if (int rc = check_shape(chunk_shape, ndim, "chunk_shape")) return rc;
    if (!bytes) return fail(ZT_ERR_INVALID_PARAMETERS, "null output pointer");
    // guided_filter.rs:234-237 (element sizes + num_elements * (f64 + 2 f32))
    uint64_t n = (uint64_t)numel(chunk_shape, ndim);
    *bytes = zt::dtype_size(dtype_in) + zt::dtype_size(dtype_out) + n * (8 + 4 * 2);
    return ZT_OK;
}

int zt_subset_overlap(const int64_t* array_shape, int ndim, const int64_t* subset_start,
                      const int64_t* subset_shape, const int64_t* overlap, int64_t* input_start,
                      int64_t* input_shape, int64_t* dst_in_src_start) {
    if (int rc = check_shape(array_shape, ndim, "array_shape")) return rc;
    if (!subset_start || !subset_shape || !overlap || !input_start || !input_shape ||
        !dst_in_src_start)
        return fail(ZT_ERR_INVALID_PARAMETERS, "null pointer argument");
    for (int d = 0; d < ndim; ++d) {
        if (overlap[d] < 0 || subset_start[d] < 0 || subset_shape[d] < 0 ||
            subset_start[d] + subset_shape[d] > array_shape[d])
            return fail(ZT_ERR_INVALID_PARAMETERS, "subset outside the array on axis %d", d);
        // array_subset_overlap.rs:12-29
        int64_t s = subset_start[d] > overlap[d] ? subset_start[d] - overlap[d] : 0;
        int64_t e = std::min(subset_start[d] + subset_shape[d] + overlap[d], array_shape[d]);
        input_start[d] = s;
        input_shape[d] = e - s;
        dst_in_src_start[d] = subset_start[d] - s;
    }
    return ZT_OK;
}

int zt_guided_filter_apply_ndarray(zt_ctx* ctx, int dtype_in, const void* in,
                                   const int64_t* in_shape, const int64_t* in_strides, int ndim,
                                   const int64_t* out_start, const int64_t* out_shape,
                                   int dtype_out, void* out, const int64_t* out_strides,
                                   float epsilon, int radius) {
    if (int rc = check_ctx(ctx)) return rc;
    if (int rc = dtypes_ok(dtype_in, dtype_out)) return rc;
    if (int rc = radius_ok(radius)) return rc;
    if (int rc = check_shape(in_shape, ndim, "in_shape")) return rc;
    if (!out_start || !out_shape) return fail(ZT_ERR_INVALID_PARAMETERS, "null output region");
    for (int d = 0; d < ndim; ++d)
        if (out_start[d] < 0 || out_shape[d] < 0 || out_start[d] + out_shape[d] > in_shape[d])
            return fail(ZT_ERR_INVALID_PARAMETERS, "output region outside the block on axis %d",
                        d);
    if (numel(out_shape, ndim) == 0) return ZT_OK;
    if (!in || !out) return fail(ZT_ERR_INVALID_PARAMETERS, "null data pointer");
    int64_t is[ZT_MAX_DIMS], os[ZT_MAX_DIMS];
    if (in_strides) std::copy(in_strides, in_strides + ndim, is);
    else c_strides(in_shape, ndim, is);
    if (out_strides) std::copy(out_strides, out_strides + ndim, os);
    else c_strides(out_shape, ndim, os);
    DeviceGuard g(ctx->device);
    if (ndim <= 3 && zt::fused_supports_radius(radius) && is[ndim - 1] == 1 &&
        os[ndim - 1] == 1) {
        int64_t dom[3] = {1, 1, 1}, ost[3] = {0, 0, 0}, osh[3] = {1, 1, 1};
        int64_t isz = 0, isy = 0, osz = 0, osy = 0;
        for (int d = 0; d < ndim; ++d) {
            dom[3 - ndim + d] = in_shape[d];
            ost[3 - ndim + d] = out_start[d];
            osh[3 - ndim + d] = out_shape[d];
        }
        if (ndim == 3) { isz = is[0]; isy = is[1]; osz = os[0]; osy = os[1]; }
        if (ndim == 2) { isy = is[0]; osy = os[0]; }
        if (ndim == 1) { isy = dom[2]; osy = osh[2]; }
        if (fused_planes_fit(dom, isy, osh, osy, dtype_in, dtype_out))
            return run_fused3(ctx, dtype_in, in, dom, 0, dom[0], isz, isy, ost, osh, dtype_out,
                              out, osz, osy, epsilon, radius, 0);
    }
    if (use_guided4d(ndim, radius, is, in_shape))
        return run_guided4d(ctx, dtype_in, in, in_shape, is, out_start, out_shape, dtype_out, out,
                            os, epsilon, radius);
    return run_separable(ctx, dtype_in, in, in_shape, is, ndim, out_start, out_shape, dtype_out,
                         out, os, epsilon, radius);
}

int zt_guided_filter_apply_array(zt_ctx* ctx, int dtype_in, const void* in, int dtype_out,
                                 void* out, const int64_t* shape, int ndim,
                                 const int64_t* chunk_shape, float epsilon, int radius,
                                 const int64_t* chunk_grid_start,
                                 const int64_t* chunk_grid_count) {
    if (int rc = check_ctx(ctx)) return rc;
    if (int rc = dtypes_ok(dtype_in, dtype_out)) return rc;
    if (int rc = radius_ok(radius)) return rc;
    if (int rc = check_shape(shape, ndim, "shape")) return rc;
    if (!chunk_shape) return fail(ZT_ERR_INVALID_PARAMETERS, "null chunk_shape");
    int64_t grid[ZT_MAX_DIMS], g0[ZT_MAX_DIMS], gn[ZT_MAX_DIMS];
    for (int d = 0; d < ndim; ++d) {
        if (chunk_shape[d] <= 0)
            return fail(ZT_ERR_INVALID_PARAMETERS, "chunk extent must be positive");
        grid[d] = (shape[d] + chunk_shape[d] - 1) / chunk_shape[d];
        g0[d] = chunk_grid_start ? chunk_grid_start[d] : 0;
        gn[d] = chunk_grid_count ? chunk_grid_count[d] : grid[d];
        if (g0[d] < 0 || gn[d] < 0 || g0[d] + gn[d] > grid[d])
            return fail(ZT_ERR_INVALID_PARAMETERS, "chunk grid range outside the grid on axis %d",
                        d);
    }
    if (numel(gn, ndim) == 0 || numel(shape, ndim) == 0) return ZT_OK;
    if (!in || !out) return fail(ZT_ERR_INVALID_PARAMETERS, "null data pointer");
    // Output region = the box of chunks (chunk_subset_bounded per chunk, guided_filter.rs:87).
    int64_t ostart[ZT_MAX_DIMS], oshape[ZT_MAX_DIMS], strides[ZT_MAX_DIMS];
    for (int d = 0; d < ndim; ++d) {
        ostart[d] = g0[d] * chunk_shape[d];
        oshape[d] = std::min((g0[d] + gn[d]) * chunk_shape[d], shape[d]) - ostart[d];
    }
    c_strides(shape, ndim, strides);
    DeviceGuard g(ctx->device);
    const size_t esz_in = zt::dtype_size(dtype_in), esz_out = zt::dtype_size(dtype_out);
    int64_t fdom[3] = {1, 1, 1}, fosh[3] = {1, 1, 1};
    for (int d = 0; d < ndim && ndim <= 3; ++d) {
        fdom[3 - ndim + d] = shape[d];
        fosh[3 - ndim + d] = oshape[d];
    }
    if (ndim <= 3 && zt::fused_supports_radius(radius) &&
        fused_planes_fit(fdom, fdom[2], fosh, fdom[2], dtype_in, dtype_out)) {
        // One launch for the whole box: every window clamps at the array bounds, which is what
        // the reference's per-chunk 2r halo (clamped to the array) produces.
        int64_t dom[3] = {1, 1, 1}, ost[3] = {0, 0, 0}, osh[3] = {1, 1, 1};
        for (int d = 0; d < ndim; ++d) {
            dom[3 - ndim + d] = shape[d];
            ost[3 - ndim + d] = ostart[d];
            osh[3 - ndim + d] = oshape[d];
        }
        int64_t sz = ndim == 3 ? strides[0] : 0, sy = ndim >= 2 ? strides[ndim - 2] : 0;
        char* obase = static_cast<char*>(out) +
                      esz_out * (ost[0] * (ndim == 3 ? sz : 0) + ost[1] * sy + ost[2]);
        (void)esz_in;
        int chunk_depth = ndim == 3 ? (int)chunk_shape[0] : 0;
        return run_fused3(ctx, dtype_in, in, dom, 0, dom[0], sz, sy, ost, osh, dtype_out, obase,
                          sz, sy, epsilon, radius, chunk_depth > 0 ? chunk_depth : 1);
    }
    int64_t ov[ZT_MAX_DIMS];
    for (int d = 0; d < ndim; ++d) ov[d] = (int64_t)((radius * 2) & 0xFF);
    // Separable / four-kernel 4-D paths: as few launches as the scratch allows. Chunks are
    // grouped along the trailing axes — the whole box when its scratch (plus its 2r halo) fits
    // in half the free device memory, else rows of chunks over axes k..ndim-1 for the smallest k
    // that fits, down to single chunks. Chunked == whole with the halo; rows
    // spare the per-chunk halo recompute of the grouped axes and the launches' tails.
    size_t free_b = 0, total_b = 0;
    const bool have_info = hipMemGetInfo(&free_b, &total_b) == hipSuccess;
    (void)hipGetLastError();
    auto need_of = [&](const int64_t* ish) -> size_t {
        return use_guided4d(ndim, radius, strides, ish)
                   ? (size_t)zt::guided4d_scratch_bytes(numel(ish, ndim), true)
                   : sizeof(float) * (size_t)zt::separable_scratch_floats(numel(ish, ndim));
    };
    // ZT_SCRATCH_LIMIT (bytes, tests): a smaller budget, to exercise the row / chunk grouping
    const char* lim_env = getenv("ZT_SCRATCH_LIMIT");
    const size_t lim = lim_env ? (size_t)strtoull(lim_env, nullptr, 10) : SIZE_MAX;
    auto fits = [&](size_t need) {
        if (need > lim) return false;
        return ctx->scratch_bytes >= need ||
               (have_info && need + ctx->scratch_bytes <= free_b / 2);
    };
    // k = number of leading axes iterated chunk by chunk (0: the whole box in one call). A
    // group's input is at most one chunk plus its two halos along axes < k and the box (plus
    // its halos) along the rest; the budget check uses that largest group.
    int64_t bis0[ZT_MAX_DIMS], bish[ZT_MAX_DIMS], bdst[ZT_MAX_DIMS];
    if (int rc = zt_subset_overlap(shape, ndim, ostart, oshape, ov, bis0, bish, bdst)) return rc;
    int k = 0;
    for (; k < ndim; ++k) {
        int64_t ish[ZT_MAX_DIMS];
        for (int d = 0; d < ndim; ++d)
            ish[d] = d < k ? std::min(chunk_shape[d] + 2 * ov[d], bish[d]) : bish[d];
        if (fits(need_of(ish))) break;
    }
    // iterate the chunk grid of axes < k; each call covers those chunks' full extent along >= k
    int64_t ngroups = 1;
    for (int d = 0; d < k; ++d) ngroups *= gn[d];
    for (int64_t c = 0; c < ngroups; ++c) {
        int64_t rem = c, cs[ZT_MAX_DIMS], csh[ZT_MAX_DIMS];
        for (int d = ndim - 1; d >= 0; --d) {
            if (d >= k) {
                cs[d] = ostart[d];
                csh[d] = oshape[d];
                continue;
            }
            int64_t ci = g0[d] + rem % gn[d];
            rem /= gn[d];
            cs[d] = ci * chunk_shape[d];
            csh[d] = std::min(cs[d] + chunk_shape[d], shape[d]) - cs[d];
        }
        int64_t is0[ZT_MAX_DIMS], ish[ZT_MAX_DIMS], dst[ZT_MAX_DIMS];
        int rc = zt_subset_overlap(shape, ndim, cs, csh, ov, is0, ish, dst);
        if (rc) return rc;
        int64_t ioff = 0, ooff = 0;
        for (int d = 0; d < ndim; ++d) {
            ioff += is0[d] * strides[d];
            ooff += cs[d] * strides[d];
        }
        rc = use_guided4d(ndim, radius, strides, ish)
                 ? run_guided4d(ctx, dtype_in, static_cast<const char*>(in) + esz_in * ioff, ish,
                                strides, dst, csh, dtype_out,
                                static_cast<char*>(out) + esz_out * ooff, strides, epsilon,
                                radius)
                 : run_separable(ctx, dtype_in, static_cast<const char*>(in) + esz_in * ioff, ish,
                                 strides, ndim, dst, csh, dtype_out,
                                 static_cast<char*>(out) + esz_out * ooff, strides, epsilon,
                                 radius);
        if (rc) return rc;
    }
    return ZT_OK;
}

int zt_guided_filter_apply_slab(zt_ctx* ctx, int dtype_in, const void* in, int dtype_out,
                                void* out, const int64_t* global_shape, int64_t in_z0,
                                int64_t in_nz, int64_t out_z0, int64_t out_nz,
                                const int64_t* chunk_shape, float epsilon, int radius) {
    if (int rc = check_ctx(ctx)) return rc;
    if (int rc = dtypes_ok(dtype_in, dtype_out)) return rc;
    if (int rc = radius_ok(radius)) return rc;
    if (int rc = check_shape(global_shape, 3, "global_shape")) return rc;
    if (!zt::fused_supports_radius(radius))
        return fail(ZT_ERR_INVALID_PARAMETERS, "slab form supports radius <= %d",
                    zt::kFusedMaxRadius);
    const int R = radius;
    if (in_z0 < 0 || in_nz < 0 || in_z0 + in_nz > global_shape[0] || out_z0 < in_z0 ||
        out_z0 + out_nz > in_z0 + in_nz)
        return fail(ZT_ERR_INVALID_PARAMETERS, "slab rows outside the array / input slab");
    // the slab must carry the 2r halo or reach the array edge
    if ((out_z0 - 2 * R < in_z0 && in_z0 > 0) ||
        (out_z0 + out_nz + 2 * R > in_z0 + in_nz && in_z0 + in_nz < global_shape[0]))
        return fail(ZT_ERR_INVALID_PARAMETERS, "input slab lacks the 2*radius halo rows");
    if (out_nz == 0) return ZT_OK;
    if (!in || !out) return fail(ZT_ERR_INVALID_PARAMETERS, "null data pointer");
    DeviceGuard g(ctx->device);
    const int64_t sy = global_shape[2], sz = global_shape[1] * global_shape[2];
    int64_t dom[3] = {global_shape[0], global_shape[1], global_shape[2]};
    int64_t ost[3] = {out_z0, 0, 0}, osh[3] = {out_nz, global_shape[1], global_shape[2]};
    if (!fused_planes_fit(dom, sy, osh, sy, dtype_in, dtype_out)) {
        // planes of >= 2 GiB: the separable path on the slab block (it carries the 2r halo, so
        // windows clamped at the block equal windows clamped at the array)
        const int64_t bsh[3] = {in_nz, global_shape[1], global_shape[2]};
        const int64_t bst[3] = {sz, sy, 1};
        const int64_t bos[3] = {out_z0 - in_z0, 0, 0};
        return run_separable(ctx, dtype_in, in, bsh, bst, 3, bos, osh, dtype_out, out, bst,
                             epsilon, radius);
    }
    int depth = chunk_shape && chunk_shape[0] > 0 ? (int)chunk_shape[0] : (int)out_nz;
    return run_fused3(ctx, dtype_in, in, dom, in_z0, in_nz, sz, sy, ost, osh, dtype_out, out, sz,
                      sy, epsilon, radius, depth);
}

// ---- Gaussian (gaussian.rs) -------------------------------------------------------------------

namespace {

// create_sampled_gaussian_kernel (gaussian.rs:252-267), operation for operation: t = sigma^2,
// scale = 1 / sqrt(2 * PI * t), tap(n) = scale * exp(-((n*n) as f32) / (2 * t)) with the
// platform libm expf (as the reference's f32::exp on Linux); taps = tap(half..1), tap(0..half).
int64_t gaussian_taps(float sigma, int64_t half, float* taps) {
    if (sigma == 0.0f) {
        if (taps) taps[0] = 1.0f;
        return 1;
    }
    if (taps) {
        const float pi = 3.14159265358979323846f;  // std::f32::consts::PI
        const float t = sigma * sigma;
        const float scale = 1.0f / sqrtf(2.0f * pi * t);
        for (int64_t n = 0; n <= half; ++n) {
            const float e = scale * expf(-((float)(uint64_t)(n * n) / (2.0f * t)));
            taps[half - n] = e;
            taps[half + n] = e;
        }
    }
    return 2 * half + 1;
}

int gaussian_args_ok(const float* sigma, const int64_t* half, int ndim) {
    if (!sigma || !half) return fail(ZT_ERR_INVALID_PARAMETERS, "null sigma / kernel_half_size");
    for (int d = 0; d < ndim; ++d) {
        if (half[d] < 0) return fail(ZT_ERR_INVALID_PARAMETERS, "negative kernel_half_size");
        if (gaussian_taps(sigma[d], half[d], nullptr) > zt::kGaussMaxTaps)
            return fail(ZT_ERR_INVALID_PARAMETERS, "kernel_half_size %lld on axis %d exceeds %d",
                        (long long)half[d], d, (zt::kGaussMaxTaps - 1) / 2);
    }
    return ZT_OK;
}

// Gaussian::apply_ndarray on a C-order block, writing only the output region: one pass per
// axis (gaussian.hip), each restricted to what the later passes read, through two f32 scratch
// buffers; the last pass writes f32 outputs in place, other types through a cast.
int run_gaussian(zt_ctx* ctx, int dtype_in, const void* in, const int64_t* in_shape, int ndim,
                 const int64_t* out_start, const int64_t* out_shape, int dtype_out, void* out,
                 const float* sigma, const int64_t* half) {
    const int64_t nout = numel(out_shape, ndim);
    if (nout == 0) return ZT_OK;
    int64_t cur[ZT_MAX_DIMS];
    std::copy(in_shape, in_shape + ndim, cur);
    int64_t maxn = 0;
    for (int d = 0; d < ndim; ++d) {
        cur[d] = out_shape[d];
        maxn = std::max(maxn, numel(cur, ndim));
    }
    const bool cast_out = dtype_out != zt::kF32;
    if (int rc = ctx->ensure_scratch(sizeof(float) * 2 * (size_t)maxn)) return rc;
    float* bufs[2] = {static_cast<float*>(ctx->scratch), static_cast<float*>(ctx->scratch) + maxn};
    std::copy(in_shape, in_shape + ndim, cur);
    const void* src = in;
    int sdt = dtype_in;
    if (ctx->timed) ZT_HIP(hipEventRecord(ctx->ev0, ctx->cur));
    // the last three axes in one z-march when they share one tap vector length that fits it
    if (ndim >= 3) {
        zt::GaussZYX pz{};
        pz.outer = numel(in_shape, ndim - 3);
        float w[zt::kGaussMaxTaps];
        bool same = true;
        for (int a = 0; a < 3; ++a) {
            const int d = ndim - 3 + a;
            const int64_t len = gaussian_taps(sigma[d], half[d], w);
            if (a == 0) pz.len = (int)len;
            if (len != pz.len || len > zt::kGaussZYXMaxLen) {
                same = false;
                break;
            }
            std::copy(w, w + len, pz.w[a]);
            pz.n[a] = in_shape[d];
            pz.on[a] = out_shape[d];
            pz.o0[a] = out_start[d];
        }
        if (same && zt::gaussian_zyx_supported(pz, dtype_in)) {
            // earlier axes (ndim > 3) first, pass by pass, then the fused three
            for (int d = 0; d < ndim - 3; ++d) {
                zt::GaussPass p{};
                p.outer = numel(cur, d);
                p.n = cur[d];
                p.on = out_shape[d];
                p.o0 = out_start[d];
                p.inner = numel(cur + d + 1, ndim - d - 1);
                p.len = (int)gaussian_taps(sigma[d], half[d], p.w);
                p.mid = p.len / 2;
                float* dst = bufs[d & 1];
                hipError_t e = zt::launch_gaussian_pass(src, sdt, dst, p, ctx->cur);
                if (e != hipSuccess) return hip_fail(e, "gaussian pass launch");
                src = dst;
                sdt = zt::kF32;
                cur[d] = out_shape[d];
            }
            pz.outer = numel(cur, ndim - 3);
            float* dst = !cast_out ? static_cast<float*>(out) : bufs[(ndim - 3) & 1];
            hipError_t e = zt::launch_gaussian_zyx(src, sdt, dst, pz, ctx->cur);
            if (e != hipSuccess) return hip_fail(e, "gaussian z/y/x march launch");
            if (ctx->timed) ZT_HIP(hipEventRecord(ctx->ev1, ctx->cur));
            if (cast_out) {
                e = zt::launch_cast_from_f32_3d(dst, dtype_out, out, 0, 0, 1, 1, nout, ctx->cur);
                if (e != hipSuccess) return hip_fail(e, "gaussian output cast");
            }
            return ZT_OK;
        }
    }
    // the last two axes in one fused pass when their kernels fit it (and the y extent fits a grid)
    const bool fuse_yx = ndim >= 2 &&
                         gaussian_taps(sigma[ndim - 2], half[ndim - 2], nullptr) <=
                             zt::kGaussYXMaxLen &&
                         gaussian_taps(sigma[ndim - 1], half[ndim - 1], nullptr) <=
                             zt::kGaussYXMaxLen &&
                         (out_shape[ndim - 2] + 31) / 32 <= 65535;
    const int nsep = fuse_yx ? ndim - 2 : ndim;
    for (int d = 0; d < nsep; ++d) {
        zt::GaussPass p{};
        p.outer = numel(cur, d);
        p.n = cur[d];
        p.on = out_shape[d];
        p.o0 = out_start[d];
        p.inner = numel(cur + d + 1, ndim - d - 1);
        p.len = (int)gaussian_taps(sigma[d], half[d], p.w);
        p.mid = p.len / 2;
        float* dst = (d == ndim - 1 && !cast_out) ? static_cast<float*>(out) : bufs[d & 1];
        hipError_t e = zt::launch_gaussian_pass(src, sdt, dst, p, ctx->cur);
        if (e != hipSuccess) return hip_fail(e, "gaussian pass launch");
        src = dst;
        sdt = zt::kF32;
        cur[d] = out_shape[d];
    }
    if (fuse_yx) {
        const int dy = ndim - 2, dx = ndim - 1;
        zt::GaussPass py{}, px{};
        py.n = cur[dy];
        py.on = out_shape[dy];
        py.o0 = out_start[dy];
        py.len = (int)gaussian_taps(sigma[dy], half[dy], py.w);
        py.mid = py.len / 2;
        px.n = cur[dx];
        px.on = out_shape[dx];
        px.o0 = out_start[dx];
        px.len = (int)gaussian_taps(sigma[dx], half[dx], px.w);
        px.mid = px.len / 2;
        float* dst = !cast_out ? static_cast<float*>(out) : bufs[nsep & 1];
        hipError_t e = zt::launch_gaussian_yx(src, sdt, dst, numel(cur, dy), py, px, ctx->cur);
        if (e != hipSuccess) return hip_fail(e, "gaussian y/x pass launch");
        src = dst;
    }
    if (ctx->timed) ZT_HIP(hipEventRecord(ctx->ev1, ctx->cur));
    if (cast_out) {
        hipError_t e = zt::launch_cast_from_f32_3d(static_cast<const float*>(src), dtype_out, out,
                                                   0, 0, 1, 1, nout, ctx->cur);
        if (e != hipSuccess) return hip_fail(e, "gaussian output cast");
    }
    return ZT_OK;
}

}  // namespace

int zt_gaussian_kernel(float sigma, int64_t kernel_half_size, float* taps, int64_t* len) {
    if (!len || kernel_half_size < 0)
        return fail(ZT_ERR_INVALID_PARAMETERS, "null len or negative kernel_half_size");
    *len = gaussian_taps(sigma, kernel_half_size, taps);
    return ZT_OK;
}

int zt_gaussian_is_compatible(int dtype_in, int dtype_out) {
    // gaussian.rs:123-147: every listed type is accepted for input and output.
    return dtypes_ok(dtype_in, dtype_out);
}

int zt_gaussian_memory_per_chunk(int dtype_in, int dtype_out, const int64_t* chunk_shape,
                                 int ndim, const int64_t* kernel_half_size, uint64_t* bytes) {
    if (int rc = dtypes_ok(dtype_in, dtype_out)) return rc;
    if (int rc = check_shape(chunk_shape, ndim, "chunk_shape")) return rc;
    if (!bytes || !kernel_half_size) return fail(ZT_ERR_INVALID_PARAMETERS, "null pointer");
    // gaussian.rs:149-168
    uint64_t nin = 1;
    for (int d = 0; d < ndim; ++d) nin *= (uint64_t)(chunk_shape[d] + 2 * kernel_half_size[d]);
    const uint64_t nout = (uint64_t)numel(chunk_shape, ndim);
    *bytes = nin * (zt::dtype_size(dtype_in) + 4 * 2) + nout * (4 + zt::dtype_size(dtype_out));
    return ZT_OK;
}

int zt_gaussian_apply_ndarray(zt_ctx* ctx, int dtype_in, const void* in, const int64_t* in_shape,
                              int ndim, const int64_t* out_start, const int64_t* out_shape,
                              int dtype_out, void* out, const float* sigma,
                              const int64_t* kernel_half_size) {
    if (int rc = check_ctx(ctx)) return rc;
    if (int rc = dtypes_ok(dtype_in, dtype_out)) return rc;
    if (int rc = check_shape(in_shape, ndim, "in_shape")) return rc;
    if (int rc = gaussian_args_ok(sigma, kernel_half_size, ndim)) return rc;
    if (!out_start || !out_shape) return fail(ZT_ERR_INVALID_PARAMETERS, "null output region");
    for (int d = 0; d < ndim; ++d)
        if (out_start[d] < 0 || out_shape[d] < 0 || out_start[d] + out_shape[d] > in_shape[d])
            return fail(ZT_ERR_INVALID_PARAMETERS, "output region outside the block on axis %d",
                        d);
    if (numel(out_shape, ndim) == 0) return ZT_OK;
    if (!in || !out) return fail(ZT_ERR_INVALID_PARAMETERS, "null data pointer");
    DeviceGuard g(ctx->device);
    return run_gaussian(ctx, dtype_in, in, in_shape, ndim, out_start, out_shape, dtype_out, out,
                        sigma, kernel_half_size);
}

int zt_gaussian_apply_array(zt_ctx* ctx, int dtype_in, const void* in, int dtype_out, void* out,
                            const int64_t* shape, int ndim, const int64_t* chunk_shape,
                            const float* sigma, const int64_t* kernel_half_size) {
    if (int rc = check_ctx(ctx)) return rc;
    if (int rc = dtypes_ok(dtype_in, dtype_out)) return rc;
    if (int rc = check_shape(shape, ndim, "shape")) return rc;
    if (int rc = gaussian_args_ok(sigma, kernel_half_size, ndim)) return rc;
    if (!chunk_shape) return fail(ZT_ERR_INVALID_PARAMETERS, "null chunk_shape");
    for (int d = 0; d < ndim; ++d)
        if (chunk_shape[d] <= 0)
            return fail(ZT_ERR_INVALID_PARAMETERS, "chunk extent must be positive");
    if (numel(shape, ndim) == 0) return ZT_OK;
    if (!in || !out) return fail(ZT_ERR_INVALID_PARAMETERS, "null data pointer");
    // Every chunk with its kernel_half_size halo (clamped to the array) equals the whole array
    // with replicate edges at the array bounds: the taps' mid is the halo, so a window clamps
    // inside a chunk's block only where it clamps at the array.
    int64_t zero[ZT_MAX_DIMS] = {0};
    DeviceGuard g(ctx->device);
    return run_gaussian(ctx, dtype_in, in, shape, ndim, zero, shape, dtype_out, out, sigma,
                        kernel_half_size);
}

// ---- downsample ------------------------------------------------------------------------------

int zt_downsample_is_compatible(int dtype_in, int dtype_out, int discrete) {
    if (int rc = dtypes_ok(dtype_in, dtype_out)) return rc;
    if (discrete && dtype_in >= ZT_BFLOAT16)
        return fail(ZT_ERR_UNSUPPORTED_DATA_TYPE,
                    "Unsupported data type %s for discrete (mode) downsampling",
                    dtype_name(dtype_in));
    return ZT_OK;
}

int zt_downsample_output_shape(const int64_t* in_shape, int ndim, const int64_t* stride,
                               int64_t* out_shape) {
    if (int rc = check_shape(in_shape, ndim, "in_shape")) return rc;
    if (!stride || !out_shape) return fail(ZT_ERR_INVALID_PARAMETERS, "null pointer argument");
    for (int d = 0; d < ndim; ++d) {
        if (stride[d] <= 0) return fail(ZT_ERR_INVALID_PARAMETERS, "stride must be positive");
        out_shape[d] = std::max<int64_t>(in_shape[d] / stride[d], 1);  // downsample.rs:162-168
    }
    return ZT_OK;
}

int zt_downsample_input_subset(const int64_t* in_shape, int ndim, const int64_t* stride,
                               const int64_t* out_start, const int64_t* out_shape,
                               int64_t* in_start, int64_t* in_subset_shape) {
    if (int rc = check_shape(in_shape, ndim, "in_shape")) return rc;
    if (!stride || !out_start || !out_shape || !in_start || !in_subset_shape)
        return fail(ZT_ERR_INVALID_PARAMETERS, "null pointer argument");
    for (int d = 0; d < ndim; ++d) {
        if (stride[d] <= 0) return fail(ZT_ERR_INVALID_PARAMETERS, "stride must be positive");
        // downsample.rs:65-69
        int64_t s = out_start[d] * stride[d];
        int64_t e = std::min((out_start[d] + out_shape[d]) * stride[d], in_shape[d]);
        in_start[d] = s;
        in_subset_shape[d] = std::max<int64_t>(e - s, 0);
    }
    return ZT_OK;
}

int zt_downsample_apply_ndarray(zt_ctx* ctx, int dtype_in, const void* in,
                                const int64_t* in_shape, int ndim, const int64_t* stride,
                                int discrete, int dtype_out, void* out) {
    if (int rc = check_ctx(ctx)) return rc;
    if (int rc = zt_downsample_is_compatible(dtype_in, dtype_out, discrete)) return rc;
    if (int rc = check_shape(in_shape, ndim, "in_shape")) return rc;
    if (!stride) return fail(ZT_ERR_INVALID_PARAMETERS, "null stride");
    zt::DSParams p{};
    p.ndim = ndim;
    p.out_numel = 1;
    p.win_numel = 1;
    for (int d = 0; d < ndim; ++d) {
        if (stride[d] <= 0) return fail(ZT_ERR_INVALID_PARAMETERS, "stride must be positive");
        p.in_shape[d] = in_shape[d];
        p.win[d] = std::min(stride[d], in_shape[d]);       // downsample.rs:83-85
        p.out_shape[d] = p.win[d] > 0 ? in_shape[d] / p.win[d] : 0;  // exact_chunks
        p.out_numel *= p.out_shape[d];
        p.win_numel *= p.win[d];
    }
    if (p.out_numel == 0) return ZT_OK;
    if (!in || !out) return fail(ZT_ERR_INVALID_PARAMETERS, "null data pointer");
    DeviceGuard g(ctx->device);
    if (ctx->timed) ZT_HIP(hipEventRecord(ctx->ev0, ctx->cur));
    hipError_t e = zt::launch_downsample(in, dtype_in, out, dtype_out, p, discrete != 0, ctx->cur);
    if (e != hipSuccess) return hip_fail(e, "downsample launch");
    if (ctx->timed) ZT_HIP(hipEventRecord(ctx->ev1, ctx->cur));
    return ZT_OK;
}

int zt_pyramid_level_shapes(const int64_t* shape, int ndim, const int64_t* factor, int max_levels,
                            int64_t* level_shapes, int* n_levels) {
    if (int rc = check_shape(shape, ndim, "shape")) return rc;
    if (!factor || !level_shapes || !n_levels || max_levels < 0)
        return fail(ZT_ERR_INVALID_PARAMETERS, "bad pyramid arguments");
    int64_t cur[ZT_MAX_DIMS];
    std::copy(shape, shape + ndim, cur);
    int n = 0;
    for (int i = 1; i <= max_levels; ++i) {  // zarrs_ome.rs:515
        int64_t nxt[ZT_MAX_DIMS];
        if (int rc = zt_downsample_output_shape(cur, ndim, factor, nxt)) return rc;
        std::copy(nxt, nxt + ndim, level_shapes + (size_t)n * ndim);
        ++n;
        std::copy(nxt, nxt + ndim, cur);
        bool stop = true;  // zarrs_ome.rs:731-737
        for (int d = 0; d < ndim; ++d)
            if (!(factor[d] == 1 || nxt[d] == 1)) stop = false;
        if (stop) break;
    }
    *n_levels = n;
    return ZT_OK;
}

int zt_pyramid_downsample(zt_ctx* ctx, int dtype, const void* level0, const int64_t* shape,
                          int ndim, const int64_t* factor, int max_levels, int discrete,
                          void* const* level_ptrs, int* levels_written) {
    if (int rc = check_ctx(ctx)) return rc;
    if (!level_ptrs || !levels_written) return fail(ZT_ERR_INVALID_PARAMETERS, "null pointers");
    std::vector<int64_t> shapes((size_t)std::max(max_levels, 1) * ZT_MAX_DIMS);
    int n = 0;
    if (int rc = zt_pyramid_level_shapes(shape, ndim, factor, max_levels, shapes.data(), &n))
        return rc;
    const void* src = level0;
    int64_t cur[ZT_MAX_DIMS];
    std::copy(shape, shape + ndim, cur);
    // 2x2x2 mean or mode levels fuse, up to three per launch, while every extent of a fused
    // level's input is >= 2 (window 2 on every axis); other levels run one launch each
    const bool fusable = ndim == 3 && factor[0] == 2 && factor[1] == 2 && factor[2] == 2 &&
                         zt::pyramid_fused_dtype(dtype, discrete != 0);
    auto level_shape = [&](int i) -> const int64_t* {  // shape of level i (0 = input)
        return i == 0 ? shape : shapes.data() + (size_t)(i - 1) * ndim;
    };
    for (int i = 0; i < n;) {
        int k = 0;
        while (fusable && k < 3 && i + k < n) {
            const int64_t* sh = level_shape(i + k);
            if (sh[0] < 2 || sh[1] < 2 || sh[2] < 2) break;
            ++k;
        }
        // the fused grid's y extent covers level-1 rows in fours: past 65535 workgroups (an
        // input y extent of ~524k) the levels run one launch each instead
        if (k >= 2 && !zt::pyramid_fused_grid_fits(level_shape(i + 1))) k = 0;
        if (k >= 2) {
            int64_t sh3[4][3] = {};
            for (int l = 0; l <= k; ++l) std::copy(level_shape(i + l), level_shape(i + l) + 3, sh3[l]);
            bool any = true;
            for (int d = 0; d < 3; ++d) any = any && sh3[1][d] > 0;
            if (any) {
                if (!src || !level_ptrs[i] || !level_ptrs[i + 1] || (k == 3 && !level_ptrs[i + 2]))
                    return fail(ZT_ERR_INVALID_PARAMETERS, "null level pointer");
                DeviceGuard g(ctx->device);
                if (ctx->timed) ZT_HIP(hipEventRecord(ctx->ev0, ctx->cur));
                hipError_t e = zt::launch_pyramid_fused(src, dtype, sh3, k, level_ptrs + i,
                                                       discrete != 0, ctx->cur);
                if (e != hipSuccess) return hip_fail(e, "fused pyramid launch");
                if (ctx->timed) ZT_HIP(hipEventRecord(ctx->ev1, ctx->cur));
            }
            src = level_ptrs[i + k - 1];
            std::copy(level_shape(i + k), level_shape(i + k) + ndim, cur);
            i += k;
            continue;
        }
        // level i+1 = downsample(level i), same dtype in/out (zarrs_ome.rs:211-234)
        int rc = zt_downsample_apply_ndarray(ctx, dtype, src, cur, ndim, factor, discrete, dtype,
                                             level_ptrs[i]);
        if (rc) return rc;
        src = level_ptrs[i];
        std::copy(shapes.data() + (size_t)i * ndim, shapes.data() + (size_t)(i + 1) * ndim, cur);
        ++i;
    }
    *levels_written = n;
    return ZT_OK;
}

// ---- synthetic inputs ------------------------------------------------------------------------

int zt_synth_step_noise_f32(zt_ctx* ctx, float* out, const int64_t* shape, int ndim,
                            const int64_t* global_shape, int64_t z0, uint64_t seed) {
    if (int rc = check_ctx(ctx)) return rc;
    if (int rc = check_shape(shape, ndim, "shape")) return rc;
    const int64_t* gs = global_shape ? global_shape : shape;
    int64_t n = numel(shape, ndim);
    if (n == 0) return ZT_OK;
    int64_t plane = n / std::max<int64_t>(shape[0], 1);
    DeviceGuard g(ctx->device);
    hipError_t e = zt::launch_synth_step_noise_f32(out, n, plane, shape[ndim - 1], gs[ndim - 1],
                                                   z0, seed, ctx->cur);
    if (e != hipSuccess) return hip_fail(e, "synth launch");
    return ZT_OK;
}

int zt_synth_u16(zt_ctx* ctx, uint16_t* out, const int64_t* shape, int ndim,
                 const int64_t* global_shape, int64_t z0, uint64_t seed) {
    (void)global_shape;
    if (int rc = check_ctx(ctx)) return rc;
    if (int rc = check_shape(shape, ndim, "shape")) return rc;
    int64_t n = numel(shape, ndim);
    if (n == 0) return ZT_OK;
    int64_t plane = n / std::max<int64_t>(shape[0], 1);
    DeviceGuard g(ctx->device);
    hipError_t e = zt::launch_synth_u16(out, n, plane, z0, seed, ctx->cur);
    if (e != hipSuccess) return hip_fail(e, "synth launch");
    return ZT_OK;
}

int zt_reencode_cast(zt_ctx* ctx, int dtype_in, const void* in, int dtype_out, void* out,
                     int64_t n) {
    if (int rc = check_ctx(ctx)) return rc;
    if (zt::dtype_size(dtype_in) == 0 || zt::dtype_size(dtype_out) == 0)
        return fail(ZT_ERR_UNSUPPORTED_DATA_TYPE, "unsupported data type");
    if (n < 0) return fail(ZT_ERR_INVALID_PARAMETERS, "negative element count");
    if (n == 0) return ZT_OK;
    if (!in || !out) return fail(ZT_ERR_INVALID_PARAMETERS, "null data pointer");
    DeviceGuard g(ctx->device);
    hipError_t e = zt::launch_reencode_cast(in, dtype_in, out, dtype_out, n, ctx->cur);
    if (e != hipSuccess) return hip_fail(e, "reencode cast launch");
    return ZT_OK;
}

int zt_synth_box(zt_ctx* ctx, int kind, void* out, const int64_t* start, const int64_t* shape,
                 const int64_t* global_shape, int ndim, uint64_t seed) {
    if (int rc = check_ctx(ctx)) return rc;
    if (int rc = check_shape(shape, ndim, "shape")) return rc;
    if (int rc = check_shape(global_shape, ndim, "global_shape")) return rc;
    if (!start) return fail(ZT_ERR_INVALID_PARAMETERS, "null start");
    if (kind != 0 && kind != 1) return fail(ZT_ERR_INVALID_PARAMETERS, "kind must be 0 or 1");
    for (int d = 0; d < ndim; ++d)
        if (start[d] < 0 || start[d] + shape[d] > global_shape[d])
            return fail(ZT_ERR_INVALID_PARAMETERS, "box outside the global shape on axis %d", d);
    if (numel(shape, ndim) == 0) return ZT_OK;
    if (!out) return fail(ZT_ERR_INVALID_PARAMETERS, "null data pointer");
    DeviceGuard g(ctx->device);
    hipError_t e = zt::launch_synth_box(out, kind, start, shape, global_shape, ndim, seed, ctx->cur);
    if (e != hipSuccess) return hip_fail(e, "synth launch");
    return ZT_OK;
}

}  // extern "C"
