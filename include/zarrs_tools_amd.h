/*
 * zarrs_tools_amd.h — the C ABI of the MI355X-native zarrs_filter per-chunk transform path.
 *
 * This is the drop-in boundary for the reference's per-chunk filter apply (LDeakin/zarrs_tools
 * 0.7.2, Rust). A Rust host would bind these symbols through a thin `extern "C"` FFI
 * (INTEGRATION.md shows the binding). In this repo the host side above the ABI is Python over
 * ctypes: the zarrs_filter / zarrs_ome drivers (zarrs_tools_amd/zarrs_filter.py, zarrs_ome.py),
 * the tests and the bench; zarrs_tools_amd/csrc/host holds the C++ Zarr V3 store and the
 * overlapped store -> store pipeline behind the zt_store_* entry points.
 *
 * Conventions
 *  - Plain pointers and sizes only. Array buffers are DEVICE pointers (hipMalloc / torch CUDA
 *    tensors) unless a function says otherwise. Shapes/strides are int64 element counts, C order
 *    (last axis fastest), like ndarray's default layout in the reference.
 *  - Every function returns a zt_status (0 = ok, negative = error); the message of the last error
 *    on the calling thread is available from zt_last_error().
 *  - Compute calls are asynchronous on the context's HIP stream; zt_ctx_synchronize() waits.
 *    Contexts are thread-safe across distinct contexts, not re-entrant on one context.
 *  - The library never frees caller memory.
 */
#ifndef ZARRS_TOOLS_AMD_H
#define ZARRS_TOOLS_AMD_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define ZT_ABI_VERSION 4
#define ZT_MAX_DIMS 8

/* Status codes. Negative values mirror FilterError variants (src/filter/filter_error.rs:10-30). */
typedef enum zt_status {
    ZT_OK = 0,
    ZT_ERR_INVALID_PARAMETERS = -1,   /* FilterError::InvalidParameters */
    ZT_ERR_UNSUPPORTED_DATA_TYPE = -2,/* FilterError::UnsupportedDataType (filter.rs:93-101) */
    ZT_ERR_OUT_OF_MEMORY = -3,        /* calculate_chunk_limit "not enough memory" (filter.rs:52-66) */
    ZT_ERR_DEVICE = -4,               /* HIP runtime error (no reference analogue: CPU-only) */
    ZT_ERR_STORAGE = -5,              /* FilterError::StorageError */
    ZT_ERR_ARRAY = -6,                /* FilterError::ArrayError / ArrayCreateError */
    ZT_ERR_IO = -7,                   /* FilterError::IOError */
    ZT_ERR_JSON = -8,                 /* FilterError::JSONError */
    ZT_ERR_INCOMPATIBLE_FILL_VALUE = -9, /* FilterError::IncompatibleFillValue */
    ZT_ERR_OTHER = -10                /* FilterError::Other */
} zt_status;

/* Element types accepted by the filters (guided_filter.rs:203-227, downsample.rs:124-148).
 * Bool is stored as one byte and processed as u8, exactly as the reference's dispatch does
 * (guided_filter.rs:280, downsample.rs:244). bfloat16/float16 are raw 16-bit storage. */
typedef enum zt_dtype {
    ZT_BOOL = 0, ZT_INT8 = 1, ZT_INT16 = 2, ZT_INT32 = 3, ZT_INT64 = 4,
    ZT_UINT8 = 5, ZT_UINT16 = 6, ZT_UINT32 = 7, ZT_UINT64 = 8,
    ZT_BFLOAT16 = 9, ZT_FLOAT16 = 10, ZT_FLOAT32 = 11, ZT_FLOAT64 = 12
} zt_dtype;

typedef struct zt_ctx zt_ctx;

/* ---- library / context ---------------------------------------------------------------------- */

int zt_abi_version(void);
/* Thread-local message of the last error raised on this thread ("" if none). */
const char* zt_last_error(void);
/* Size in bytes of one element of `dtype` (0 for an unknown code). */
size_t zt_dtype_size(int dtype);
/* Number of HIP devices visible (0 on a host without GPUs; never an error). */
int zt_device_count(int* count);
/* One context per (host thread, device): owns a HIP stream, events and reusable scratch. */
int zt_ctx_create(int device, zt_ctx** out);
int zt_ctx_destroy(zt_ctx* ctx);
/* Run subsequent work on an external stream (e.g. torch.cuda.current_stream().cuda_stream).
 * The handle is used verbatim: NULL is the device's default (null) stream. */
int zt_ctx_set_stream(zt_ctx* ctx, void* hip_stream);
/* Return to the context's own (non-blocking) stream, the state after zt_ctx_create. */
int zt_ctx_use_own_stream(zt_ctx* ctx);
int zt_ctx_get_stream(zt_ctx* ctx, void** hip_stream);
int zt_ctx_synchronize(zt_ctx* ctx);
/* Device scratch held by the context between calls (staging casts, separable passes): its size,
 * and a release that synchronises the stream and frees it (the next call needing scratch
 * allocates again). Scratch allocation failures return ZT_ERR_OUT_OF_MEMORY. */
int zt_ctx_scratch_bytes(zt_ctx* ctx, uint64_t* bytes);
int zt_ctx_release_scratch(zt_ctx* ctx);
/* Device time in ms of the most recent filter launch recorded on this context (hipEvents around
 * the kernel(s) on the context stream). Valid after zt_ctx_synchronize(). */
int zt_ctx_last_kernel_ms(zt_ctx* ctx, float* ms);

/* ---- operator surface: guided filter -------------------------------------------------------- */

/* GuidedFilter::is_compatible (guided_filter.rs:203-227): ZT_OK or ZT_ERR_UNSUPPORTED_DATA_TYPE. */
int zt_guided_filter_is_compatible(int dtype_in, int dtype_out);
/* GuidedFilter::memory_per_chunk (guided_filter.rs:229-238), bytes for one output chunk. */
int zt_guided_filter_memory_per_chunk(int dtype_in, int dtype_out, const int64_t* chunk_shape,
                                      int ndim, uint64_t* bytes);
/* ArraySubsetOverlap::new (array_subset_overlap.rs:11-35) with overlap = 2*radius per axis
 * (guided_filter.rs:88-93): the halo'd input subset of an output subset, clamped to the array,
 * and where the output lies inside it. Host-only, no device work. */
int zt_subset_overlap(const int64_t* array_shape, int ndim, const int64_t* subset_start,
                      const int64_t* subset_shape, const int64_t* overlap,
                      int64_t* input_start, int64_t* input_shape, int64_t* dst_in_src_start);

/*
 * GuidedFilter::apply_ndarray + ArraySubsetOverlap::extract_subset + the TIn->f32 / f32->TOut
 * `as` casts of apply_chunk (guided_filter.rs:98-103, :117-164).
 *   in        : device pointer to the (halo'd) input block of `dtype_in`, shape in_shape[ndim],
 *               element strides in_strides (NULL = C-contiguous). Windows clamp to this block,
 *               as get_block (guided_filter.rs:166-184) clamps to the SAT's shape.
 *   out_start : where the output region starts inside the block (dst_in_src); out_shape its shape.
 *   out       : device pointer, `dtype_out`, shape out_shape, strides out_strides (NULL = C).
 *   epsilon, radius : GuidedFilterArguments (guided_filter.rs:25-33); radius in [0, 127]
 *               (the reference's u8 `radius*2` halo overflows above that).
 * ndim in [1, 8]. 1-3 dims run the fused 2.5-D kernel; 4+ dims run the separable path.
 */
int zt_guided_filter_apply_ndarray(zt_ctx* ctx, int dtype_in, const void* in,
                                   const int64_t* in_shape, const int64_t* in_strides, int ndim,
                                   const int64_t* out_start, const int64_t* out_shape,
                                   int dtype_out, void* out, const int64_t* out_strides,
                                   float epsilon, int radius);

/*
 * GuidedFilter::apply (guided_filter.rs:240-319) over a device-resident array: every output chunk
 * of the chunk grid [chunk_grid_start, chunk_grid_start + chunk_grid_count) is filtered with its
 * 2r halo read from `in` (the whole array, C-contiguous, shape[ndim]) and written into `out`
 * (same shape, C-contiguous). Pass NULL for the grid range to process every chunk. The chunks are
 * batched into as few launches as the grid allows (one launch for a box of chunks of a 1-3 D
 * array); the result equals the reference's chunk-by-chunk result because every window clamps at
 * the array bounds exactly as the reference's clamped 2r halo makes it.
 */
int zt_guided_filter_apply_array(zt_ctx* ctx, int dtype_in, const void* in, int dtype_out,
                                 void* out, const int64_t* shape, int ndim,
                                 const int64_t* chunk_shape, float epsilon, int radius,
                                 const int64_t* chunk_grid_start,
                                 const int64_t* chunk_grid_count);

/* Multi-GPU z-slab form used by the sharded bench/driver: `in` holds the global rows
 * [in_z0, in_z0 + in_nz) of an array whose full shape is global_shape (C-contiguous slab); the
 * output rows [out_z0, out_z0 + out_nz) (global coordinates, a subset of the input rows, chunk
 * aligned or not) are written into `out` (C-contiguous, out_nz rows). Windows clamp at the global
 * array bounds, so the result equals the reference's per-chunk result for those rows as long as
 * the slab carries a 2r halo (or reaches the array edge). 3-D only. */
int zt_guided_filter_apply_slab(zt_ctx* ctx, int dtype_in, const void* in, int dtype_out,
                                void* out, const int64_t* global_shape, int64_t in_z0,
                                int64_t in_nz, int64_t out_z0, int64_t out_nz,
                                const int64_t* chunk_shape, float epsilon, int radius);

/* ---- operator surface: downsample ----------------------------------------------------------- */

/* Downsample::is_compatible (downsample.rs:124-148); discrete requires integer/bool input
 * (downsample.rs:244-256). */
int zt_downsample_is_compatible(int dtype_in, int dtype_out, int discrete);
/* Downsample::output_shape (downsample.rs:162-168): max(shape / stride, 1). */
int zt_downsample_output_shape(const int64_t* in_shape, int ndim, const int64_t* stride,
                               int64_t* out_shape);
/* Downsample::input_subset (downsample.rs:64-70). */
int zt_downsample_input_subset(const int64_t* in_shape, int ndim, const int64_t* stride,
                               const int64_t* out_start, const int64_t* out_shape,
                               int64_t* in_start, int64_t* in_subset_shape);
/*
 * Downsample::apply_ndarray_continuous / apply_ndarray_discrete (downsample.rs:72-120) on a
 * device block: window = min(stride, extent) per axis; only complete windows produce output
 * (exact_chunks); out shape = floor(in_shape / window). Continuous: f64 sum in C order / count,
 * Rust `as` into dtype_out. Discrete (integer/bool input only): the most frequent value, ties
 * broken by the smallest value (documented deterministic rule; the reference's tie order is
 * HashMap iteration order).
 */
int zt_downsample_apply_ndarray(zt_ctx* ctx, int dtype_in, const void* in,
                                const int64_t* in_shape, int ndim, const int64_t* stride,
                                int discrete, int dtype_out, void* out);

/*
 * zarrs_ome mean pyramid on a device-resident level 0 (zarrs_ome.rs:515-738, levels computed
 * on-device without a store round trip): level i = downsample(level i-1) for i in 1..=max_levels,
 * stopping when every axis has factor 1 or output extent 1 (zarrs_ome.rs:731-737).
 * `level_ptrs[i-1]` receive the levels (device buffers sized by zt_pyramid_level_shapes).
 * Returns the number of levels written through *levels_written.
 */
int zt_pyramid_level_shapes(const int64_t* shape, int ndim, const int64_t* factor, int max_levels,
                            int64_t* level_shapes /* [max_levels][ndim] */, int* n_levels);
int zt_pyramid_downsample(zt_ctx* ctx, int dtype, const void* level0, const int64_t* shape,
                          int ndim, const int64_t* factor, int max_levels, int discrete,
                          void* const* level_ptrs, int* levels_written);

/* ---- synthetic inputs ------------------------------------------------------ */

/* v = 500*[x >= nx/2] + 100*U, U = (splitmix64(seed ^ global_index) >> 40) * 2^-24, written for
 * the global rows [z0, z0 + shape[0]) of an array of shape global_shape (C order, f32). */
int zt_synth_step_noise_f32(zt_ctx* ctx, float* out, const int64_t* shape, int ndim,
                            const int64_t* global_shape, int64_t z0, uint64_t seed);
/* u16 = ((splitmix64(seed ^ global_index) >> 40) * 65535) >> 24. */
int zt_synth_u16(zt_ctx* ctx, uint16_t* out, const int64_t* shape, int ndim,
                 const int64_t* global_shape, int64_t z0, uint64_t seed);
/* The box [start, start + shape) of the N-d global synthetic volume (kind 0: float32 step+noise,
 * kind 1: uint16 noise), element for element the values the whole-array generators give it: a
 * rank generates its own octant / slab of a global array (benchmarks, parity samples). */
int zt_synth_box(zt_ctx* ctx, int kind, void* out, const int64_t* start, const int64_t* shape,
                 const int64_t* global_shape, int ndim, uint64_t seed);

/* Reencode::apply_chunk_convert (src/filter/filters/reencode.rs:58-77): out[i] = in[i].as_() for
 * n contiguous elements of any of the 13 types to any other (num-traits AsPrimitive, half 2.6.0:
 * half types through f32, float -> int saturating with NaN -> 0, int -> int wrapping). Used by
 * zarrs_ome's level 0 with --data-type (zarrs_ome.rs:355-363). */
int zt_reencode_cast(zt_ctx* ctx, int dtype_in, const void* in, int dtype_out, void* out,
                     int64_t n);


/* ---- Gaussian (src/filter/filters/gaussian.rs; src/filter/kernel.rs) ----------------------- */

/* create_sampled_gaussian_kernel (gaussian.rs:252-267): writes the taps (2*half+1, or 1 when
 * sigma == 0) to `taps` (may be NULL to query) and their count to *len. Host only. */
int zt_gaussian_kernel(float sigma, int64_t kernel_half_size, float* taps, int64_t* len);
/* Gaussian::is_compatible (gaussian.rs:123-147): all 13 types in and out. */
int zt_gaussian_is_compatible(int dtype_in, int dtype_out);
/* Gaussian::memory_per_chunk (gaussian.rs:149-168). */
int zt_gaussian_memory_per_chunk(int dtype_in, int dtype_out, const int64_t* chunk_shape,
                                 int ndim, const int64_t* kernel_half_size, uint64_t* bytes);
/* Gaussian::apply_ndarray + extract_subset + `as` casts of apply_chunk (gaussian.rs:73-119,
 * kernel.rs:17-73): the separable sampled Gaussian of a C-order device block (per axis, in axis
 * order, f32 sequential tap sums, replicate edges at the block bounds), writing the region
 * [out_start, out_start + out_shape) to `out` (C order, out_shape). sigma / kernel_half_size:
 * ndim entries; kernel_half_size <= 127. Bit-identical to the reference. */
int zt_gaussian_apply_ndarray(zt_ctx* ctx, int dtype_in, const void* in, const int64_t* in_shape,
                              int ndim, const int64_t* out_start, const int64_t* out_shape,
                              int dtype_out, void* out, const float* sigma,
                              const int64_t* kernel_half_size);
/* Gaussian::apply's chunk loop (gaussian.rs:170-249) over a device-resident C-order array: every
 * chunk with its kernel_half_size halo, which equals one pass over the whole array. */
int zt_gaussian_apply_array(zt_ctx* ctx, int dtype_in, const void* in, int dtype_out, void* out,
                            const int64_t* shape, int ndim, const int64_t* chunk_shape,
                            const float* sigma, const int64_t* kernel_half_size);

/* ---- Zarr V3 store -> store path (host storage in and out) ----------------------------------
 * The reference's filters read and write Zarr arrays through zarrs (Array::retrieve_array_subset_
 * ndarray / store_array_subset_ndarray, guided_filter.rs:95-110; zarrs_ome.rs:226-232). These
 * entry points restate that I/O for filesystem stores (zarr.json V3 metadata, regular chunk grid,
 * default/v2 chunk keys, codecs bytes, gzip, zstd (runtime libzstd.so.1), crc32c and
 * sharding_indexed) and drive the device kernels over it with a pipelined chunk-row loop:
 * decode (host threads) -> H2D -> kernel -> D2H -> encode (host threads), each input chunk
 * decoded once. Host buffers here are ordinary host memory. */

/* Per-call statistics (the reference's Progress read/process/write split, progress.rs:15-105,
 * plus the device phases). *_s of host phases are thread-seconds; device phases are event
 * seconds summed over chunk rows; wall_s is the whole call. */
typedef struct zt_store_stats {
    double wall_s;
    double decode_s, encode_s;         /* host thread-seconds: read+decode, encode+write */
    double h2d_s, kernel_s, d2h_s;     /* device seconds */
    uint64_t bytes_read, bytes_written;/* encoded bytes moved to/from storage */
    uint64_t voxels;                   /* output elements produced */
    int64_t rows;                      /* output chunk rows processed */
    int threads;                       /* host worker threads used */
    int rows_in_flight;                /* input chunk rows held decoded (memory-bounded) */
    int double_buffered;               /* 1: device slabs / output rows double buffered */
} zt_store_stats;

/* Per-chunk progress of the store filters (Progress / ProgressCallback, progress.rs:15-119):
 * after every output chunk is written, `fn` receives the step count, the number of steps (output
 * chunks of the call) and the cumulative read (decode thread-seconds), process (device seconds)
 * and write (encode thread-seconds) durations. Called from the host worker threads, serialised;
 * process-wide; NULL disables. */
typedef struct zt_progress {
    int64_t step, num_steps;
    double read_s, process_s, write_s;
} zt_progress;
typedef void (*zt_progress_fn)(const zt_progress* progress, void* user);
void zt_store_set_progress_callback(zt_progress_fn fn, void* user);

/* --chunk-limit (zarrs_ome.rs:136-141; GuidedFilter::apply's chunk_limit, guided_filter.rs:
 * 251-258): the store filters called afterwards FROM THIS THREAD hold at most `max_chunks` chunks
 * in flight (decoded input rows + output rows being computed or encoded) and use at most that many
 * host worker threads; the pipeline never goes below one input slab and one output row without
 * overlap (a chunk row is its unit of device work). 0 (the default) = bounded by memory only.
 * Replaces the reference's per-filter `chunk_limit` argument. */
int zt_store_set_chunk_limit(int64_t max_chunks);

/* flags for the store filters */
#define ZT_STORE_ERASE_OUTPUT_METADATA 1 /* remove OUT/zarr.json first ("not finished" marker,
                                             zarrs_filter.rs:297-300) */
#define ZT_STORE_FINISH_OUTPUT 2         /* write OUT/zarr.json at the end (zarrs_filter.rs:313) */

/* Array metadata of a Zarr V3 array: data type (zt_dtype), rank, shape, chunk (= shard) shape and
 * the inner chunk shape of a sharded array (= chunk shape otherwise). Arrays of ZT_MAX_DIMS. */
int zt_store_array_info(const char* path, int* dtype, int* ndim, int64_t* shape,
                        int64_t* chunk_shape, int64_t* inner_chunk_shape);
/* Create an array and write its zarr.json. codecs_json: a Zarr V3 codec list (NULL = [bytes,
 * little endian]); fill_value_json: Zarr V3 fill_value JSON (NULL = 0 / false / 0.0). */
int zt_store_create_array(const char* path, int dtype, int ndim, const int64_t* shape,
                          const int64_t* chunk_shape, const char* codecs_json,
                          const char* fill_value_json);
/* The output array the filters create: the input's shape, chunking and codecs with data type
 * dtype_out (-1 = the input's) and the input fill value cast to it (filter_traits.rs:47-82). */
int zt_store_create_output_like(const char* in_path, const char* out_path, int dtype_out,
                                const char* encoding_json);
/* The output array of a filter step with an explicit output shape (NULL = the input's): what the
 * store filters create before they run (the downsample output is max(n / stride, 1), so
 * Downsample::output_shape, downsample.rs:162-168), with the same reencoding. Used to give
 * device-resident run-config chains (zarrs_filter.rs:338-381) the arrays the store path would
 * have made, without writing the intermediate data. */
int zt_store_create_output(const char* in_path, const char* out_path, int dtype_out,
                           const int64_t* out_shape, int ndim, const char* encoding_json);
/* Read any subset into a C-order host buffer (missing chunks read as the fill value). */
int zt_store_read_subset(const char* path, const int64_t* start, const int64_t* shape,
                         void* host_out, int nthreads);
/* Write a chunk-aligned subset (may end at the array edge) from a C-order host buffer. */
int zt_store_write_subset(const char* path, const int64_t* start, const int64_t* shape,
                          const void* host_in, int nthreads);
/* Fill an existing array with the SURVEY.md §8(d) synthetic data (kind 0: float32 step+noise,
 * kind 1: uint16 noise), identical to zt_synth_step_noise_f32 / zt_synth_u16. */
int zt_store_write_synth(const char* path, int kind, uint64_t seed, int nthreads);

/* encoding_json (NULL or "" = the input's encoding): a JSON object with the reencoding
 * arguments of the filter commands (ZarrReencodingArgs, lib.rs:274-377; applied as
 * get_array_builder_reencode, lib.rs:408-650): "data_type", "fill_value", "separator",
 * "chunk_shape", "shard_shape", "array_to_array_codecs" (only []), "array_to_bytes_codec" (bytes),
 * "bytes_to_bytes_codecs" (gzip / zstd / crc32c), "dimension_names", "attributes",
 * "attributes_append". A "data_type" there takes precedence over dtype_out. Output arrays whose
 * chunk rows do not fit 80 % of the available host / device memory (with no overlap) fail with
 * ZT_ERR_OUT_OF_MEMORY, as calculate_chunk_limit does (filter.rs:52-66). */
/* zarrs_filter guided-filter IN OUT EPS R [--data-type T] over a store (GuidedFilter::apply,
 * guided_filter.rs:240-319): the output array is IN's shape/chunking/codecs with dtype_out (-1 =
 * input type). Processes the output chunk rows [row_begin, row_end) along axis 0 (row_end < 0 =
 * all), so ranks can split the rows; the array's zarr.json is written only with
 * ZT_STORE_FINISH_OUTPUT. nthreads <= 0: min(16, hardware threads). stats may be NULL. */
int zt_store_guided_filter(const char* in_path, const char* out_path, int dtype_out,
                           const char* encoding_json, float epsilon, int radius, int device,
                           int64_t row_begin, int64_t row_end, int nthreads, int flags,
                           zt_store_stats* stats);
/* zt_store_guided_filter restricted to the output chunk columns [col_begin, col_end) along
 * axis 1 (col_end < 0: all), the input read with the 2r halo along axes 0 and 1: one process's
 * (t, z) block of a multi-GPU split (config T; the reference's per-chunk loop,
 * guided_filter.rs:260-316, over that block's chunks). */
int zt_store_guided_filter_box(const char* in_path, const char* out_path, int dtype_out,
                               const char* encoding_json, float epsilon, int radius, int device,
                               int64_t row_begin, int64_t row_end, int64_t col_begin,
                               int64_t col_end, int nthreads, int flags, zt_store_stats* stats);
/* zarrs_filter downsample / one zarrs_ome level over a store (Downsample::apply,
 * downsample.rs:170-286): output shape max(n / stride, 1), encoding as the input's with the
 * encoding_json overrides (zarrs_ome passes its per-level chunk / shard shapes). */
int zt_store_downsample(const char* in_path, const char* out_path, const int64_t* stride,
                        int discrete, int dtype_out, const char* encoding_json, int device,
                        int64_t row_begin, int64_t row_end, int nthreads, int flags,
                        zt_store_stats* stats);
/* zarrs_filter gaussian IN OUT SIGMA HALF [--data-type T] over a store (Gaussian::apply,
 * gaussian.rs:170-249): as zt_store_guided_filter, halo = kernel_half_size. */
int zt_store_gaussian(const char* in_path, const char* out_path, int dtype_out,
                      const char* encoding_json, const float* sigma,
                      const int64_t* kernel_half_size, int device, int64_t row_begin,
                      int64_t row_end, int nthreads, int flags, zt_store_stats* stats);
/* One zarrs_ome level with --gaussian-sigma (apply_chunk_continuous_gaussian, zarrs_ome.rs:
 * 236-271): the Gaussian of each downsample input subset (plus its kernel_half_size halo), then
 * the mean downsample of that f32 block to the level's data type. */
int zt_store_downsample_gaussian(const char* in_path, const char* out_path, const int64_t* stride,
                                 const float* sigma, const int64_t* kernel_half_size,
                                 int dtype_out, const char* encoding_json, int device,
                                 int64_t row_begin, int64_t row_end, int nthreads, int flags,
                                 zt_store_stats* stats);
/* 1 if the named codec can be read and written here, else 0. */
int zt_store_codec_available(const char* name);
/* Host bytes the store pipeline budgets 80 % of (the available-memory half of
 * calculate_chunk_limit, filter.rs:52-66): ZT_STORE_HOST_MEMORY if set, else MemAvailable capped
 * at the cgroup's limit minus its usage net of reclaimable (inactive) page cache. */
uint64_t zt_store_host_available_bytes(void);

#ifdef __cplusplus
}
#endif
#endif /* ZARRS_TOOLS_AMD_H */
