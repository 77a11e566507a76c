// zt_kernels.hpp — kernel parameter blocks and launchers shared by the .hip translation units.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include <atomic>

namespace zt {

constexpr int kMaxDims = 8;
constexpr int kMaxRadius = 127;         // reference: u8 radius, halo (radius*2) as u8 (guided_filter.rs:92)
constexpr int kFusedMaxRadius = 8;      // fused 2.5-D kernel instantiations
constexpr int kSepTreeMaxRadius = 16;   // separable path: tree sums up to here, sequential beyond

// Fused 3-D guided filter. Domain = the block windows clamp to ([0,nz) x [0,ny) x [0,nx)).
// Input element (z,y,x) lives at in + (z - in_z0)*in_sz + y*in_sy + x (x stride 1).
// Output element (z,y,x) of the region [oz0,oz0+onz) x [oy0,..) x [ox0,..) lives at
// out + (z-oz0)*out_sz + (y-oy0)*out_sy + (x-ox0).
struct GFParams {
    const void* in;
    void* out;
    int64_t in_sz, in_sy;
    int64_t out_sz, out_sy;
    int in_z0;
    int zlo, zhi;  // input planes present in `in`: [zlo, zhi) = [in_z0, in_z0 + rows) within [0, nz)
    int nz, ny, nx;
    int oz0, oy0, ox0;
    int onz, ony, onx;
    int zseg;  // output slices per workgroup march (normally the chunk depth)
    int tiles_x, tiles_y, nseg;
    int itx0, itx1, ity0, ity1;  // interior tile range (fused kernel, host-computed)
    float eps;
    float rcp_w3;  // RN(1 / (2r+1)^3): the interior window count's reciprocal (host-computed)
};

// N-d geometry for the separable path and downsample (C-order logical shapes).
struct NdGeom {
    int ndim;
    int64_t numel;
    int64_t shape[kMaxDims];
    int64_t in_strides[kMaxDims];
    int64_t out_start[kMaxDims];
    int64_t out_shape[kMaxDims];
    int64_t out_strides[kMaxDims];
    int64_t out_numel;
};

bool fused_supports_radius(int radius);
int fused_tile_y(int radius);  // output tile height of the fused kernel for this radius
// element-type pairs with a direct fused instantiation; others are staged through f32
bool fused_direct_pair(int dtype_in, int dtype_out);
hipError_t launch_reencode_cast(const void* in, int dtype_in, void* out, int dtype_out, int64_t n,
                                hipStream_t s);
hipError_t launch_cast_to_f32_3d(const void* in, int dtype, int64_t sz, int64_t sy, float* out,
                                 int64_t nz, int64_t ny, int64_t nx, hipStream_t s);
hipError_t launch_cast_from_f32_3d(const float* in, int dtype, void* out, int64_t sz, int64_t sy,
                                   int64_t nz, int64_t ny, int64_t nx, hipStream_t s);
hipError_t launch_guided_fused(const GFParams& p, int dtype_in, int dtype_out, int radius,
                               hipStream_t stream);
// scratch must hold separable_scratch_floats(g.numel) floats: v | X (2n) | Y (2n), each region
// starting on a 16-byte boundary (the f64 / float2 views of X and Y stay aligned for odd n)
inline int64_t separable_pad(int64_t n) { return (n + 3) & ~(int64_t)3; }
inline int64_t separable_scratch_floats(int64_t n) { return 5 * separable_pad(n); }
hipError_t launch_guided_separable(const void* in, int dtype_in, void* out, int dtype_out,
                                   const NdGeom& g, int radius, float eps, float* scratch,
                                   hipStream_t s);

// 4-D guided filter (guided4d.hip): t-window sums of per-timepoint 3-D box sums, four kernels.
bool guided4d_supports(int radius);
int64_t guided4d_scratch_bytes(int64_t numel, bool gather);
// T <= 4 timepoints, r <= 2: both stages of every timepoint in one z-march (g4_fused.hip),
// f32 C-order input, no scratch.
bool guided4d_fused_supports(int radius, const NdGeom& g);
hipError_t launch_guided4d_fused(const float* v, void* out, int dtype_out, const NdGeom& g,
                                 int radius, float eps, hipStream_t s);
hipError_t launch_guided4d(const void* in, int dtype_in, void* out, int dtype_out,
                           const NdGeom& g, int radius, float eps, void* scratch, hipStream_t s);

// Downsample (downsample.rs:72-120). g.shape = input shape, g.out_shape = output shape,
// win = window per axis (min(stride, extent)).
struct DSParams {
    int ndim;
    int64_t in_shape[kMaxDims];
    int64_t out_shape[kMaxDims];
    int64_t win[kMaxDims];
    int64_t out_numel;
    int64_t win_numel;
};
hipError_t launch_downsample(const void* in, int dtype_in, void* out, int dtype_out,
                             const DSParams& p, bool discrete, hipStream_t s);
// nl (2 or 3) fused 2x2x2 mean (or mode: discrete) pyramid levels: shapes[0] = input,
// shapes[1..nl] = levels (each floor(previous / 2), every extent of shapes[0..nl-1] >= 2);
// outs[l-1] = level l.
bool pyramid_fused_dtype(int dtype, bool discrete);
// the fused pyramid grid (launch_pyramid_fused) for a level-1 shape fits the launch limits
bool pyramid_fused_grid_fits(const int64_t* level1_shape);
hipError_t launch_pyramid_fused(const void* in, int dtype, const int64_t (*shapes)[3], int nl,
                                void* const* outs, bool discrete, hipStream_t s);

// Gaussian pass along one axis (gaussian.hip): input region outer x n x inner (C order), output
// outer x on x inner with output k reading input positions around o0 + k (replicate edges).
constexpr int kGaussMaxTaps = 255;  // kernel_half_size <= 127 per axis
struct GaussPass {
    int64_t outer, n, on, o0, inner;
    int len, mid;
    float w[kGaussMaxTaps];
};
hipError_t launch_gaussian_pass(const void* in, int dtype_in, float* out, const GaussPass& p,
                                hipStream_t s);
// The last two axes' passes fused (y then x, tiles staged in LDS): input outer x ny x nx, output
// outer x py.on x px.on; py / px carry the two axes' taps, lengths, output offsets and extents.
constexpr int kGaussYXMaxLen = 33;
hipError_t launch_gaussian_yx(const void* in, int dtype_in, float* out, int64_t outer,
                              const GaussPass& py, const GaussPass& px, hipStream_t s);

// The last three axes' passes fused in one z-march (z, y then x; taps L on all three, odd,
// <= kGaussZYXMaxLen): input outer x nz x ny x nx, f32 output outer x on[0] x on[1] x on[2].
constexpr int kGaussZYXMaxLen = 13;
struct GaussZYX {
    int64_t outer, n[3], on[3], o0[3];
    int len;
    float w[3][kGaussZYXMaxLen];
};
bool gaussian_zyx_supported(const GaussZYX& p, int dtype_in);
hipError_t launch_gaussian_zyx(const void* in, int dtype_in, float* out, const GaussZYX& p,
                               hipStream_t s);

// Synthetic inputs
hipError_t launch_synth_step_noise_f32(float* out, int64_t n, int64_t plane, int64_t nx_row,
                                       int64_t nx_global, int64_t z0, uint64_t seed,
                                       hipStream_t s);
hipError_t launch_synth_u16(uint16_t* out, int64_t n, int64_t plane, int64_t z0, uint64_t seed,
                            hipStream_t s);
hipError_t launch_synth_box(void* out, int kind, const int64_t* start, const int64_t* shape,
                            const int64_t* gshape, int ndim, uint64_t seed, hipStream_t s);

}  // namespace zt
