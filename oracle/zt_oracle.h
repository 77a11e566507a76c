/*
 * zt_oracle.h — TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement of the reference zarrs_filter per-chunk path (LDeakin/zarrs_tools 0.7.2, Rust).
 * The reference cannot be built in this image (no cargo/rustc, crates not vendored), so this C
 * restatement is the parity oracle. It is pinned by the reference's own known-answer tests:
 *   - guided_filter.rs:330-374   (4x4 f32, 2x2 chunks, eps=1, r=2; golden values :364-369)
 *   - summed_area_table.rs:265-318 (6x6 u8 -> u16 integral image; golden values :306-313)
 * Downsample has no reference test: its restatement (downsample.rs:64-97) is "parity unpinned"
 * beyond the integer-exactness argument documented in DESIGN.md.
 *
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load this library,
 * and only as the checker / the timed CPU baseline. The product path (zarrs_tools_amd) never
 * links or calls it.
 */
#ifndef ZT_ORACLE_H
#define ZT_ORACLE_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Data type codes: identical numbering to include/zarrs_tools_amd.h (zt_dtype). */
enum {
    OR_BOOL = 0, OR_INT8, OR_INT16, OR_INT32, OR_INT64,
    OR_UINT8, OR_UINT16, OR_UINT32, OR_UINT64,
    OR_BFLOAT16, OR_FLOAT16, OR_FLOAT32, OR_FLOAT64
};

int oracle_version(void);

/* summed_area_table.rs:339-360 — f64 integral image of an f32 block (C order). */
void oracle_summed_area_table(const float* in, double* sat, const int64_t* shape, int ndim);

/* summed_area_table.rs:365-399 / :401-411 — window sum / mean from a SAT, p0/p1 inclusive. */
float oracle_sat_sum(const double* sat, const int64_t* shape, int ndim,
                     const int64_t* p0, const int64_t* p1);
float oracle_sat_mean(const double* sat, const int64_t* shape, int ndim,
                      const int64_t* p0, const int64_t* p1);

/* guided_filter.rs:117-164 — in-place on a whole (halo'd) block, C order. The dead SAT of
 * (v-u)^2 at :133 is computed when faithful != 0 (timing honesty only; no effect on results). */
void oracle_guided_filter_apply_ndarray(float* v, const int64_t* shape, int ndim,
                                        float epsilon, int radius, int faithful);

/* guided_filter.rs:240-319 + :75-114 — whole-array chunked apply of an f32 array held in memory.
 * Each output chunk reads its 2r halo (array_subset_overlap.rs:11-51), is filtered, and its
 * interior is written. Chunks are processed on `nthreads` threads (rayon analogue). Output is f32. */
int oracle_guided_filter_apply(const float* in, float* out, const int64_t* shape, int ndim,
                               const int64_t* chunk_shape, float epsilon, int radius,
                               int nthreads, int faithful);

/* Same, but only for the chunks with linear chunk-grid index in [chunk_begin, chunk_end)
 * (bench.py's bounded CPU sample). Returns number of chunks processed or <0 on error. */
int64_t oracle_guided_filter_apply_chunks(const float* in, float* out, const int64_t* shape,
                                          int ndim, const int64_t* chunk_shape, float epsilon,
                                          int radius, int nthreads, int faithful,
                                          int64_t chunk_begin, int64_t chunk_end);

/* Rust `as` casts from f32 / f64 into every supported element type (num_traits AsPrimitive,
 * half 2.6.0 f16/bf16 from_f32 / from_f64). `dst` is an element of type `dtype`. */
void oracle_cast_from_f32(const float* src, int dtype, void* dst, int64_t n);
void oracle_cast_from_f64(const double* src, int dtype, void* dst, int64_t n);
/* Element -> f32 / f64 (`as f32` / `as f64`). */
void oracle_cast_to_f32(const void* src, int dtype, float* dst, int64_t n);
void oracle_cast_to_f64(const void* src, int dtype, double* dst, int64_t n);

/* downsample.rs:72-97 — mean over complete stride windows (exact_chunks), f64 sum / count,
 * `as TOut`. in/out are C-order; out shape = floor(in_shape / min(stride, in_shape)). */
int oracle_downsample_continuous(const void* in, int dtype_in, const int64_t* in_shape, int ndim,
                                 const int64_t* stride, void* out, int dtype_out);

/* downsample.rs:99-120 — mode over complete windows. The reference breaks ties by HashMap
 * iteration order (nondeterministic); this restatement breaks ties by the smallest value,
 * the documented deterministic rule of this repo. Integer types (and bool) only. */
int oracle_downsample_discrete(const void* in, int dtype_in, const int64_t* in_shape, int ndim,
                               const int64_t* stride, void* out, int dtype_out);

/* Synthetic inputs: splitmix64(seed ^ linear_index). */
uint64_t oracle_splitmix64(uint64_t x);
/* v = 500*[x >= nx/2] + 100*U, U = (h >> 40) * 2^-24; f32 arithmetic, no FMA. `z0` offsets the
 * first axis (for slabs of a larger global volume); shape is the slab's shape, nx = shape[ndim-1]. */
void oracle_synth_step_noise_f32(float* out, const int64_t* shape, int ndim,
                                 const int64_t* global_shape, int64_t z0, uint64_t seed);
/* The box [start, start+shape) of an N-d global synthetic volume: step+noise f32 / u16 noise,
 * element values as the whole-array generators give them (full-size parity samples). */
void oracle_synth_block_nd_f32(float* out, const int64_t* start, const int64_t* shape,
                               const int64_t* global_shape, int ndim, uint64_t seed);
void oracle_synth_block_nd_u16(uint16_t* out, const int64_t* start, const int64_t* shape,
                               const int64_t* global_shape, int ndim, uint64_t seed);
/* The box [start, start+shape) of the 3-D global synthetic step+noise volume (C order). */
void oracle_synth_block_f32(float* out, const int64_t* start, const int64_t* shape,
                            const int64_t* global_shape, uint64_t seed);

/* bench.py cpu_baseline sample: for each listed chunk (3-D chunk-grid coordinates) build its
 * 2r-halo'd input block of the global synthetic volume (untimed), then run
 * GuidedFilter::apply_ndarray (faithful: includes the reference's dead 4th SAT) on all of them
 * with `nthreads` threads, one chunk per task (rayon analogue). Returns the wall seconds of the
 * filtering alone; *voxels_out receives the output (interior) voxels processed. */
double oracle_guided_filter_time_chunks(const int64_t* global_shape, const int64_t* chunk_shape,
                                        const int64_t* chunk_coords, int n_chunks, float epsilon,
                                        int radius, int nthreads, uint64_t seed,
                                        int64_t* voxels_out);

/* u16 = ((h >> 40) * 65535) >> 24. */
void oracle_synth_u16(uint16_t* out, const int64_t* shape, int ndim,
                      const int64_t* global_shape, int64_t z0, uint64_t seed);


/* gaussian.rs:252-267 create_sampled_gaussian_kernel: sigma == 0 -> [1]; else
 * scale * exp(-(n*n as f32) / (2 t)) for n = half..0..half, t = sigma^2,
 * scale = 1 / sqrt(2 pi t). Writes 2*half+1 taps (1 when sigma == 0); returns the tap count. */
int64_t oracle_gaussian_kernel(float sigma, int64_t half, float* taps);
/* gaussian.rs:110-119 + kernel.rs:17-73: for each axis in order, an f32 sequential sum of
 * input[min(sat_sub(k + i, mid), n - 1)] * tap[i] (replicate edges), in place. */
int oracle_gaussian_apply_ndarray(float* v, const int64_t* shape, int ndim, const float* sigma,
                                  const int64_t* half);
/* gaussian.rs:73-108, :170-249: every chunk of the grid with a kernel_half_size halo
 * (ArraySubsetOverlap), apply_ndarray, extract. */
int oracle_gaussian_apply(const float* in, float* out, const int64_t* shape, int ndim,
                          const int64_t* chunk_shape, const float* sigma, const int64_t* half);

#ifdef __cplusplus
}
#endif
#endif
