/*
 * zt_oracle.c — TEST INFRASTRUCTURE ONLY (see zt_oracle.h for the contract).
 *
 * A plain-C restatement of the reference zarrs_filter per-chunk transform path
 * (LDeakin/zarrs_tools 0.7.2). Every function cites the reference file:line it follows.
 * Arithmetic is kept operation-for-operation: f64 integral images built sequentially, 2^d
 * inclusion-exclusion in the reference's corner order, f32 means, two roundings (no FMA) in the
 * final v*mean(a)+mean(b). Build with -ffp-contract=off (oracle/Makefile).
 *
 * Third-party arithmetic restated here (absent from /root/reference, pinned in its Cargo.lock):
 *   - num-traits 0.2.19 `AsPrimitive` = Rust `as`: float->int saturating, NaN->0, truncation.
 *   - half 2.6.0 `f16::from_f32/from_f64`, `bf16::from_f32/from_f64` software conversions.
 */
#include "zt_oracle.h"

#include <math.h>
#include <pthread.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

int oracle_version(void) { return 1; }

/* ------------------------------------------------------------------------------------------ */
/* half 2.6.0 conversions (software paths)                                                    */
/* ------------------------------------------------------------------------------------------ */

static uint32_t f32_bits(float f) { uint32_t u; memcpy(&u, &f, 4); return u; }
static float bits_f32(uint32_t u) { float f; memcpy(&f, &u, 4); return f; }
static uint64_t f64_bits(double f) { uint64_t u; memcpy(&u, &f, 8); return u; }

/* half: f32_to_f16 — round to nearest even, NaN keeps the top payload bits + quiet bit. */
static uint16_t h_f32_to_f16(float value) {
    uint32_t x = f32_bits(value);
    uint32_t sign = x & 0x80000000u, exp = x & 0x7F800000u, man = x & 0x007FFFFFu;
    if (exp == 0x7F800000u) {
        uint32_t nan_bit = man == 0 ? 0 : 0x0200u;
        return (uint16_t)((sign >> 16) | 0x7C00u | nan_bit | (man >> 13));
    }
    uint32_t half_sign = sign >> 16;
    int32_t half_exp = (int32_t)(exp >> 23) - 127 + 15;
    if (half_exp >= 0x1F) return (uint16_t)(half_sign | 0x7C00u);
    if (half_exp <= 0) {
        if (14 - half_exp > 24) return (uint16_t)half_sign;
        uint32_t m = man | 0x00800000u;
        uint32_t half_man = m >> (14 - half_exp);
        uint32_t round_bit = 1u << (13 - half_exp);
        if ((m & round_bit) != 0 && (m & (3 * round_bit - 1)) != 0) half_man += 1;
        return (uint16_t)(half_sign | half_man);
    }
    uint32_t he = (uint32_t)half_exp << 10, half_man = man >> 13, round_bit = 0x1000u;
    if ((man & round_bit) != 0 && (man & (3 * round_bit - 1)) != 0)
        return (uint16_t)((half_sign | he | half_man) + 1);
    return (uint16_t)(half_sign | he | half_man);
}

/* half: f64_to_f16 — works on the upper 32 bits of the f64 (the low 32 mantissa bits are
 * dropped before rounding, exactly as the half crate's software path does). */
static uint16_t h_f64_to_f16(double value) {
    uint64_t val = f64_bits(value);
    uint32_t x = (uint32_t)(val >> 32);
    uint32_t sign = x & 0x80000000u, exp = x & 0x7FF00000u, man = x & 0x000FFFFFu;
    if (exp == 0x7FF00000u) {
        uint32_t nan_bit = (man == 0 && (uint32_t)val == 0) ? 0 : 0x0200u;
        return (uint16_t)((sign >> 16) | 0x7C00u | nan_bit | (man >> 10));
    }
    uint32_t half_sign = sign >> 16;
    int64_t half_exp = (int64_t)(exp >> 20) - 1023 + 15;
    if (half_exp >= 0x1F) return (uint16_t)(half_sign | 0x7C00u);
    if (half_exp <= 0) {
        if (10 - half_exp > 21) return (uint16_t)half_sign;
        uint32_t m = man | 0x00100000u;
        uint32_t half_man = m >> (11 - half_exp);
        uint32_t round_bit = 1u << (10 - half_exp);
        if ((m & round_bit) != 0 && (m & (3 * round_bit - 1)) != 0) half_man += 1;
        return (uint16_t)(half_sign | half_man);
    }
    uint32_t he = (uint32_t)half_exp << 10, half_man = man >> 10, round_bit = 0x0200u;
    if ((man & round_bit) != 0 && (man & (3 * round_bit - 1)) != 0)
        return (uint16_t)((half_sign | he | half_man) + 1);
    return (uint16_t)(half_sign | he | half_man);
}

/* half: f32_to_bf16 — round to nearest even on the top 16 bits; NaN gets the quiet bit. */
static uint16_t h_f32_to_bf16(float value) {
    uint32_t x = f32_bits(value);
    if ((x & 0x7FFFFFFFu) > 0x7F800000u) return (uint16_t)((x >> 16) | 0x0040u);
    uint32_t round_bit = 0x8000u;
    if ((x & round_bit) != 0 && (x & (3 * round_bit - 1)) != 0) return (uint16_t)((x >> 16) + 1);
    return (uint16_t)(x >> 16);
}

/* half: f64_to_bf16 — upper-32-bit restatement as for f16. */
static uint16_t h_f64_to_bf16(double value) {
    uint64_t val = f64_bits(value);
    uint32_t x = (uint32_t)(val >> 32);
    uint32_t sign = x & 0x80000000u, exp = x & 0x7FF00000u, man = x & 0x000FFFFFu;
    if (exp == 0x7FF00000u) {
        uint32_t nan_bit = (man == 0 && (uint32_t)val == 0) ? 0 : 0x0040u;
        return (uint16_t)((sign >> 16) | 0x7F80u | nan_bit | (man >> 13));
    }
    uint32_t half_sign = sign >> 16;
    int64_t half_exp = (int64_t)(exp >> 20) - 1023 + 127;
    if (half_exp >= 0xFF) return (uint16_t)(half_sign | 0x7F80u);
    if (half_exp <= 0) {
        if (7 - half_exp > 21) return (uint16_t)half_sign;
        uint32_t m = man | 0x00100000u;
        uint32_t half_man = m >> (14 - half_exp);
        uint32_t round_bit = 1u << (13 - half_exp);
        if ((m & round_bit) != 0 && (m & (3 * round_bit - 1)) != 0) half_man += 1;
        return (uint16_t)(half_sign | half_man);
    }
    uint32_t he = (uint32_t)half_exp << 7, half_man = man >> 13, round_bit = 0x1000u;
    if ((man & round_bit) != 0 && (man & (3 * round_bit - 1)) != 0)
        return (uint16_t)((half_sign | he | half_man) + 1);
    return (uint16_t)(half_sign | he | half_man);
}

static float h_f16_to_f32(uint16_t h) {
    uint32_t sign = (uint32_t)(h & 0x8000u) << 16;
    uint32_t exp = (h >> 10) & 0x1F, man = h & 0x3FFu;
    if (exp == 0x1F) return bits_f32(sign | 0x7F800000u | (man << 13));
    if (exp == 0) {
        if (man == 0) return bits_f32(sign);
        /* subnormal: value = man * 2^-24 */
        float f = (float)man * (1.0f / 16777216.0f);
        return sign ? -f : f;
    }
    return bits_f32(sign | ((exp - 15 + 127) << 23) | (man << 13));
}
static float h_bf16_to_f32(uint16_t h) { return bits_f32((uint32_t)h << 16); }

/* ------------------------------------------------------------------------------------------ */
/* Rust `as` casts (num-traits AsPrimitive)                                                    */
/* ------------------------------------------------------------------------------------------ */

#define SAT_INT(NAME, T, LO, HI)                                                             \
    static T NAME(double x) {                                                                \
        if (x != x) return 0;                                                                \
        if (x <= (double)(LO)) return (T)(LO);                                               \
        if (x >= (double)(HI)) return (T)(HI);                                               \
        return (T)x; /* C truncation toward zero */                                          \
    }
SAT_INT(sat_i8, int8_t, INT8_MIN, INT8_MAX)
SAT_INT(sat_i16, int16_t, INT16_MIN, INT16_MAX)
SAT_INT(sat_i32, int32_t, INT32_MIN, INT32_MAX)
SAT_INT(sat_u8, uint8_t, 0, UINT8_MAX)
SAT_INT(sat_u16, uint16_t, 0, UINT16_MAX)
SAT_INT(sat_u32, uint32_t, 0, UINT32_MAX)
static int64_t sat_i64(double x) {
    if (x != x) return 0;
    if (x <= -9223372036854775808.0) return INT64_MIN;
    if (x >= 9223372036854775808.0) return INT64_MAX;
    return (int64_t)x;
}
static uint64_t sat_u64(double x) {
    if (x != x) return 0;
    if (x <= 0.0) return 0;
    if (x >= 18446744073709551616.0) return UINT64_MAX;
    return (uint64_t)x;
}

/* f32 -> T. For integer targets the f32 is exactly representable in f64, so saturating through
 * f64 is the same as Rust's f32 `as` int. */
static void cast_one_from_f32(float v, int dtype, void* dst, int64_t i) {
    switch (dtype) {
    case OR_BOOL: case OR_UINT8: ((uint8_t*)dst)[i] = sat_u8(v); break;
    case OR_INT8: ((int8_t*)dst)[i] = sat_i8(v); break;
    case OR_INT16: ((int16_t*)dst)[i] = sat_i16(v); break;
    case OR_INT32: ((int32_t*)dst)[i] = sat_i32(v); break;
    case OR_INT64: ((int64_t*)dst)[i] = sat_i64(v); break;
    case OR_UINT16: ((uint16_t*)dst)[i] = sat_u16(v); break;
    case OR_UINT32: ((uint32_t*)dst)[i] = sat_u32(v); break;
    case OR_UINT64: ((uint64_t*)dst)[i] = sat_u64(v); break;
    case OR_BFLOAT16: ((uint16_t*)dst)[i] = h_f32_to_bf16(v); break;
    case OR_FLOAT16: ((uint16_t*)dst)[i] = h_f32_to_f16(v); break;
    case OR_FLOAT32: ((float*)dst)[i] = v; break;
    case OR_FLOAT64: ((double*)dst)[i] = (double)v; break;
    }
}
static void cast_one_from_f64(double v, int dtype, void* dst, int64_t i) {
    switch (dtype) {
    case OR_BOOL: case OR_UINT8: ((uint8_t*)dst)[i] = sat_u8(v); break;
    case OR_INT8: ((int8_t*)dst)[i] = sat_i8(v); break;
    case OR_INT16: ((int16_t*)dst)[i] = sat_i16(v); break;
    case OR_INT32: ((int32_t*)dst)[i] = sat_i32(v); break;
    case OR_INT64: ((int64_t*)dst)[i] = sat_i64(v); break;
    case OR_UINT16: ((uint16_t*)dst)[i] = sat_u16(v); break;
    case OR_UINT32: ((uint32_t*)dst)[i] = sat_u32(v); break;
    case OR_UINT64: ((uint64_t*)dst)[i] = sat_u64(v); break;
    case OR_BFLOAT16: ((uint16_t*)dst)[i] = h_f64_to_bf16(v); break;
    case OR_FLOAT16: ((uint16_t*)dst)[i] = h_f64_to_f16(v); break;
    case OR_FLOAT32: ((float*)dst)[i] = (float)v; break;
    case OR_FLOAT64: ((double*)dst)[i] = v; break;
    }
}
static double load_as_f64(const void* src, int dtype, int64_t i) {
    switch (dtype) {
    case OR_BOOL: case OR_UINT8: return (double)((const uint8_t*)src)[i];
    case OR_INT8: return (double)((const int8_t*)src)[i];
    case OR_INT16: return (double)((const int16_t*)src)[i];
    case OR_INT32: return (double)((const int32_t*)src)[i];
    case OR_INT64: return (double)((const int64_t*)src)[i];
    case OR_UINT16: return (double)((const uint16_t*)src)[i];
    case OR_UINT32: return (double)((const uint32_t*)src)[i];
    case OR_UINT64: return (double)((const uint64_t*)src)[i];
    case OR_BFLOAT16: return (double)h_bf16_to_f32(((const uint16_t*)src)[i]);
    case OR_FLOAT16: return (double)h_f16_to_f32(((const uint16_t*)src)[i]);
    case OR_FLOAT32: return (double)((const float*)src)[i];
    case OR_FLOAT64: return ((const double*)src)[i];
    }
    return 0.0;
}
static float load_as_f32(const void* src, int dtype, int64_t i) {
    switch (dtype) {
    case OR_BOOL: case OR_UINT8: return (float)((const uint8_t*)src)[i];
    case OR_INT8: return (float)((const int8_t*)src)[i];
    case OR_INT16: return (float)((const int16_t*)src)[i];
    case OR_INT32: return (float)((const int32_t*)src)[i];
    case OR_INT64: return (float)((const int64_t*)src)[i];
    case OR_UINT16: return (float)((const uint16_t*)src)[i];
    case OR_UINT32: return (float)((const uint32_t*)src)[i];
    case OR_UINT64: return (float)((const uint64_t*)src)[i];
    case OR_BFLOAT16: return h_bf16_to_f32(((const uint16_t*)src)[i]);
    case OR_FLOAT16: return h_f16_to_f32(((const uint16_t*)src)[i]);
    case OR_FLOAT32: return ((const float*)src)[i];
    case OR_FLOAT64: return (float)((const double*)src)[i];
    }
    return 0.0f;
}

void oracle_cast_from_f32(const float* src, int dtype, void* dst, int64_t n) {
    for (int64_t i = 0; i < n; ++i) cast_one_from_f32(src[i], dtype, dst, i);
}
void oracle_cast_from_f64(const double* src, int dtype, void* dst, int64_t n) {
    for (int64_t i = 0; i < n; ++i) cast_one_from_f64(src[i], dtype, dst, i);
}
void oracle_cast_to_f32(const void* src, int dtype, float* dst, int64_t n) {
    for (int64_t i = 0; i < n; ++i) dst[i] = load_as_f32(src, dtype, i);
}
void oracle_cast_to_f64(const void* src, int dtype, double* dst, int64_t n) {
    for (int64_t i = 0; i < n; ++i) dst[i] = load_as_f64(src, dtype, i);
}

/* ------------------------------------------------------------------------------------------ */
/* Summed area table (summed_area_table.rs:339-411)                                            */
/* ------------------------------------------------------------------------------------------ */

#define OR_MAXDIM 8

static int64_t numel(const int64_t* shape, int ndim) {
    int64_t n = 1;
    for (int d = 0; d < ndim; ++d) n *= shape[d];
    return n;
}

/* summed_area_table.rs:339-360: cumulative sum along the last axis (input as f64 + acc), then
 * along axes d-2..0 (sat += acc), each lane sequential. */
void oracle_summed_area_table(const float* in, double* sat, const int64_t* shape, int ndim) {
    int64_t n = numel(shape, ndim);
    if (n == 0) return;
    int64_t last = shape[ndim - 1];
    for (int64_t lane = 0; lane < n / last; ++lane) {
        double acc = 0.0;
        const float* src = in + lane * last;
        double* dst = sat + lane * last;
        for (int64_t i = 0; i < last; ++i) {
            dst[i] = (double)src[i] + acc;
            acc = dst[i];
        }
    }
    for (int dim = ndim - 2; dim >= 0; --dim) {
        int64_t stride = 1;
        for (int d = dim + 1; d < ndim; ++d) stride *= shape[d];
        int64_t len = shape[dim];
        int64_t outer = n / (len * stride);
        for (int64_t o = 0; o < outer; ++o) {
            for (int64_t s = 0; s < stride; ++s) {
                double acc = 0.0;
                double* p = sat + o * len * stride + s;
                for (int64_t i = 0; i < len; ++i) {
                    p[i * stride] += acc;
                    acc = p[i * stride];
                }
            }
        }
    }
}

/* summed_area_table.rs:365-399: for i in 0..2^d, bit j (MSB first) picks p0-1 (0) or p1 (1);
 * terms needing p0-1 with p0 == 0 are skipped; sign = 1 - 2*((d - #upper) % 2); f64 sum in
 * that order; `sum as f32`. */
float oracle_sat_sum(const double* sat, const int64_t* shape, int ndim, const int64_t* p0,
                     const int64_t* p1) {
    double sum = 0.0;
    for (int64_t i = 0; i < ((int64_t)1 << ndim); ++i) {
        int64_t off = 0, p_sum = 0;
        int skip = 0;
        for (int j = 0; j < ndim; ++j) {
            int64_t p = (i >> (ndim - 1 - j)) & 1;
            int64_t c;
            if (p == 0) {
                if (p0[j] == 0) { skip = 1; break; }
                c = p0[j] - 1;
            } else {
                c = p1[j];
            }
            off = off * shape[j] + c;
            p_sum += p;
        }
        if (skip) continue;
        int sign = 1 - 2 * (int)((ndim - p_sum) % 2);
        sum += (double)sign * sat[off];
    }
    return (float)sum;
}

/* summed_area_table.rs:401-411: sum / (prod(p1 - p0 + 1) as f32). */
float oracle_sat_mean(const double* sat, const int64_t* shape, int ndim, const int64_t* p0,
                      const int64_t* p1) {
    float sum = oracle_sat_sum(sat, shape, ndim, p0, p1);
    uint64_t n = 1;
    for (int j = 0; j < ndim; ++j) n *= (uint64_t)(p1[j] - p0[j] + 1);
    return sum / (float)n;
}

/* guided_filter.rs:166-184: p0 = min(i.saturating_sub(r), n-1), p1 = min(i + r, n-1). */
static void get_block(const int64_t* idx, const int64_t* shape, int ndim, int r, int64_t* p0,
                      int64_t* p1) {
    for (int j = 0; j < ndim; ++j) {
        int64_t a = idx[j] > r ? idx[j] - r : 0;
        int64_t b = idx[j] + r;
        p0[j] = a < shape[j] - 1 ? a : shape[j] - 1;
        p1[j] = b < shape[j] - 1 ? b : shape[j] - 1;
    }
}

static void unravel(int64_t lin, const int64_t* shape, int ndim, int64_t* idx) {
    for (int j = ndim - 1; j >= 0; --j) {
        idx[j] = lin % shape[j];
        lin /= shape[j];
    }
}

/* guided_filter.rs:186-199 (sat_to_mean) and :147-153/:156-162 (the mean loops). */
static void sat_means(const double* sat, const int64_t* shape, int ndim, int r, float* mean) {
    int64_t n = numel(shape, ndim);
    int64_t idx[OR_MAXDIM], p0[OR_MAXDIM], p1[OR_MAXDIM];
    for (int64_t lin = 0; lin < n; ++lin) {
        unravel(lin, shape, ndim, idx);
        get_block(idx, shape, ndim, r, p0, p1);
        mean[lin] = oracle_sat_mean(sat, shape, ndim, p0, p1);
    }
}

/* guided_filter.rs:117-164 (the pointwise-variance form). */
void oracle_guided_filter_apply_ndarray(float* v, const int64_t* shape, int ndim, float epsilon,
                                        int radius, int faithful) {
    int64_t n = numel(shape, ndim);
    if (n == 0) return;
    double* sat = (double*)malloc(sizeof(double) * n);
    float* u = (float*)malloc(sizeof(float) * n);
    float* s = (float*)malloc(sizeof(float) * n);
    float* mean = (float*)malloc(sizeof(float) * n);
    oracle_summed_area_table(v, sat, shape, ndim);   /* :126 */
    sat_means(sat, shape, ndim, radius, u);           /* :127 u_k */
    for (int64_t i = 0; i < n; ++i) {                  /* :130-132 (v-u).powf(2.0) == d*d */
        float d = v[i] - u[i];
        s[i] = d * d;
    }
    if (faithful) oracle_summed_area_table(s, sat, shape, ndim); /* :133 dead SAT */
    for (int64_t i = 0; i < n; ++i) {                  /* :135-140 */
        float a = s[i] / (s[i] + epsilon);
        float b = (1.0f - a) * u[i];
        u[i] = a;
        s[i] = b;
    }
    oracle_summed_area_table(u, sat, shape, ndim);   /* :144 SAT(a) */
    sat_means(sat, shape, ndim, radius, mean);
    for (int64_t i = 0; i < n; ++i) v[i] *= mean[i];   /* :148-153 */
    oracle_summed_area_table(s, sat, shape, ndim);   /* :155 SAT(b) */
    sat_means(sat, shape, ndim, radius, mean);
    for (int64_t i = 0; i < n; ++i) v[i] += mean[i];   /* :157-162 */
    free(sat); free(u); free(s); free(mean);
}

/* ------------------------------------------------------------------------------------------ */
/* Chunked apply (guided_filter.rs:75-114, :240-319; array_subset_overlap.rs:11-51)            */
/* ------------------------------------------------------------------------------------------ */

typedef struct {
    const float* in;
    float* out;
    const int64_t* shape;
    const int64_t* chunk_shape;
    int ndim;
    float epsilon;
    int radius;
    int faithful;
    int64_t next;   /* shared work counter (guarded by mu) */
    int64_t end;
    pthread_mutex_t mu;
} chunk_job;

static void apply_one_chunk(const chunk_job* job, int64_t chunk_lin) {
    int ndim = job->ndim;
    int64_t grid[OR_MAXDIM], cidx[OR_MAXDIM];
    for (int j = 0; j < ndim; ++j)
        grid[j] = (job->shape[j] + job->chunk_shape[j] - 1) / job->chunk_shape[j];
    unravel(chunk_lin, grid, ndim, cidx);
    /* chunk_subset_bounded (guided_filter.rs:87) */
    int64_t o_start[OR_MAXDIM], o_end[OR_MAXDIM];
    for (int j = 0; j < ndim; ++j) {
        o_start[j] = cidx[j] * job->chunk_shape[j];
        int64_t e = o_start[j] + job->chunk_shape[j];
        o_end[j] = e < job->shape[j] ? e : job->shape[j];
    }
    /* ArraySubsetOverlap::new with overlap (radius*2) as u64 (guided_filter.rs:88-93). The
     * reference computes radius*2 in u8 arithmetic; radius is an u8 argument, so radius >= 128
     * would overflow there. Callers reject that case before reaching here. */
    int64_t h = (int64_t)((job->radius * 2) & 0xFF);
    int64_t i_start[OR_MAXDIM], i_shape[OR_MAXDIM], d_start[OR_MAXDIM];
    for (int j = 0; j < ndim; ++j) {
        i_start[j] = o_start[j] > h ? o_start[j] - h : 0;
        int64_t e = o_end[j] + h;
        int64_t i_end = e < job->shape[j] ? e : job->shape[j];
        i_shape[j] = i_end - i_start[j];
        d_start[j] = o_start[j] - i_start[j];
    }
    int64_t nin = numel(i_shape, ndim);
    float* block = (float*)malloc(sizeof(float) * (nin > 0 ? nin : 1));
    int64_t idx[OR_MAXDIM];
    for (int64_t lin = 0; lin < nin; ++lin) {          /* retrieve_array_subset (:95-96) */
        unravel(lin, i_shape, ndim, idx);
        int64_t off = 0;
        for (int j = 0; j < ndim; ++j) off = off * job->shape[j] + (i_start[j] + idx[j]);
        block[lin] = job->in[off];
    }
    oracle_guided_filter_apply_ndarray(block, i_shape, ndim, job->epsilon, job->radius,
                                       job->faithful);
    int64_t o_shape[OR_MAXDIM];
    for (int j = 0; j < ndim; ++j) o_shape[j] = o_end[j] - o_start[j];
    int64_t nout = numel(o_shape, ndim);
    for (int64_t lin = 0; lin < nout; ++lin) {          /* extract_subset + store (:101-110) */
        unravel(lin, o_shape, ndim, idx);
        int64_t src = 0, dst = 0;
        for (int j = 0; j < ndim; ++j) {
            src = src * i_shape[j] + (d_start[j] + idx[j]);
            dst = dst * job->shape[j] + (o_start[j] + idx[j]);
        }
        job->out[dst] = block[src];
    }
    free(block);
}

static void* chunk_worker(void* arg) {
    chunk_job* job = (chunk_job*)arg;
    for (;;) {
        pthread_mutex_lock(&job->mu);
        int64_t c = job->next < job->end ? job->next++ : -1;
        pthread_mutex_unlock(&job->mu);
        if (c < 0) break;
        apply_one_chunk(job, c);
    }
    return NULL;
}

int64_t oracle_guided_filter_apply_chunks(const float* in, float* out, const int64_t* shape,
                                          int ndim, const int64_t* chunk_shape, float epsilon,
                                          int radius, int nthreads, int faithful,
                                          int64_t chunk_begin, int64_t chunk_end) {
    if (ndim < 1 || ndim > OR_MAXDIM || radius < 0 || radius > 255) return -1;
    for (int j = 0; j < ndim; ++j)
        if (shape[j] < 0 || chunk_shape[j] <= 0) return -1;
    chunk_job job;
    job.in = in; job.out = out; job.shape = shape; job.chunk_shape = chunk_shape;
    job.ndim = ndim; job.epsilon = epsilon; job.radius = radius; job.faithful = faithful;
    job.next = chunk_begin; job.end = chunk_end;
    pthread_mutex_init(&job.mu, NULL);
    if (nthreads < 1) nthreads = 1;
    pthread_t* th = (pthread_t*)malloc(sizeof(pthread_t) * nthreads);
    for (int t = 0; t < nthreads; ++t) pthread_create(&th[t], NULL, chunk_worker, &job);
    for (int t = 0; t < nthreads; ++t) pthread_join(th[t], NULL);
    free(th);
    pthread_mutex_destroy(&job.mu);
    return chunk_end - chunk_begin;
}

int oracle_guided_filter_apply(const float* in, float* out, const int64_t* shape, int ndim,
                               const int64_t* chunk_shape, float epsilon, int radius,
                               int nthreads, int faithful) {
    if (ndim < 1 || ndim > OR_MAXDIM) return -1;
    int64_t nchunks = 1;
    for (int j = 0; j < ndim; ++j) {
        if (chunk_shape[j] <= 0) return -1;
        nchunks *= (shape[j] + chunk_shape[j] - 1) / chunk_shape[j];
    }
    int64_t r = oracle_guided_filter_apply_chunks(in, out, shape, ndim, chunk_shape, epsilon,
                                                  radius, nthreads, faithful, 0, nchunks);
    return r < 0 ? (int)r : 0;
}

/* ------------------------------------------------------------------------------------------ */
/* Downsample (downsample.rs:64-120)                                                           */
/* ------------------------------------------------------------------------------------------ */

static int ds_shapes(const int64_t* in_shape, int ndim, const int64_t* stride, int64_t* win,
                     int64_t* out_shape) {
    if (ndim < 1 || ndim > OR_MAXDIM) return -1;
    for (int j = 0; j < ndim; ++j) {
        if (stride[j] <= 0) return -1;
        /* downsample.rs:83-85: chunk_size = min(stride, shape) */
        win[j] = stride[j] < in_shape[j] ? stride[j] : in_shape[j];
        /* exact_chunks: only complete windows */
        out_shape[j] = win[j] > 0 ? in_shape[j] / win[j] : 0;
    }
    return 0;
}

/* downsample.rs:72-97: for each complete window, sum of `as f64` in C order (f64 fold from 0),
 * / (len as f64), `as TOut`. */
int oracle_downsample_continuous(const void* in, int dtype_in, const int64_t* in_shape, int ndim,
                                 const int64_t* stride, void* out, int dtype_out) {
    int64_t win[OR_MAXDIM], out_shape[OR_MAXDIM];
    if (ds_shapes(in_shape, ndim, stride, win, out_shape)) return -1;
    int64_t nout = numel(out_shape, ndim), nwin = numel(win, ndim);
    int64_t oidx[OR_MAXDIM], widx[OR_MAXDIM];
    for (int64_t o = 0; o < nout; ++o) {
        unravel(o, out_shape, ndim, oidx);
        /* Rust's f64 `Sum` folds from -0.0 (std, since 1.83), so an all -0.0 window stays -0.0. */
        double sum = -0.0;
        for (int64_t w = 0; w < nwin; ++w) {
            unravel(w, win, ndim, widx);
            int64_t off = 0;
            for (int j = 0; j < ndim; ++j) off = off * in_shape[j] + (oidx[j] * win[j] + widx[j]);
            sum += load_as_f64(in, dtype_in, off);
        }
        cast_one_from_f64(sum / (double)nwin, dtype_out, out, o);
    }
    return 0;
}

/* downsample.rs:99-120: mode of each complete window, counted over exact `TIn` keys (the
 * reference's HashMap<TIn, usize>): the raw integer, never an f64 image of it, so distinct 64-bit
 * values past 2^53 stay distinct. Deterministic tie rule: the smallest value in TIn's order (the
 * reference picks whichever HashMap entry iterates first, which is unspecified). */
static int dt_signed(int dt) {
    return dt == OR_INT8 || dt == OR_INT16 || dt == OR_INT32 || dt == OR_INT64;
}
/* the element as a 64-bit key: signed types sign-extended (compare as int64), unsigned and bool
 * zero-extended (compare as uint64) */
static uint64_t load_key(const void* src, int dt, int64_t i) {
    switch (dt) {
    case OR_BOOL: case OR_UINT8: return ((const uint8_t*)src)[i];
    case OR_INT8: return (uint64_t)(int64_t)((const int8_t*)src)[i];
    case OR_INT16: return (uint64_t)(int64_t)((const int16_t*)src)[i];
    case OR_INT32: return (uint64_t)(int64_t)((const int32_t*)src)[i];
    case OR_INT64: return (uint64_t)((const int64_t*)src)[i];
    case OR_UINT16: return ((const uint16_t*)src)[i];
    case OR_UINT32: return ((const uint32_t*)src)[i];
    case OR_UINT64: return ((const uint64_t*)src)[i];
    }
    return 0;
}
static int key_less(uint64_t a, uint64_t b, int sgn) {
    return sgn ? (int64_t)a < (int64_t)b : a < b;
}
int oracle_downsample_discrete(const void* in, int dtype_in, const int64_t* in_shape, int ndim,
                               const int64_t* stride, void* out, int dtype_out) {
    if (dtype_in >= OR_BFLOAT16) return -2;
    int64_t win[OR_MAXDIM], out_shape[OR_MAXDIM];
    if (ds_shapes(in_shape, ndim, stride, win, out_shape)) return -1;
    int64_t nout = numel(out_shape, ndim), nwin = numel(win, ndim);
    int64_t oidx[OR_MAXDIM], widx[OR_MAXDIM];
    const int sgn = dt_signed(dtype_in);
    uint64_t* keys = (uint64_t*)malloc(sizeof(uint64_t) * (nwin > 0 ? nwin : 1));
    for (int64_t o = 0; o < nout; ++o) {
        unravel(o, out_shape, ndim, oidx);
        for (int64_t w = 0; w < nwin; ++w) {
            unravel(w, win, ndim, widx);
            int64_t off = 0;
            for (int j = 0; j < ndim; ++j) off = off * in_shape[j] + (oidx[j] * win[j] + widx[j]);
            keys[w] = load_key(in, dtype_in, off);
        }
        uint64_t best = 0;
        int64_t best_count = -1;
        for (int64_t a = 0; a < nwin; ++a) {
            int64_t count = 0;
            for (int64_t b = 0; b < nwin; ++b) count += keys[b] == keys[a];
            if (count > best_count || (count == best_count && key_less(keys[a], best, sgn))) {
                best_count = count;
                best = keys[a];
            }
        }
        /* `TIn as TOut` (downsample.rs:117): integer -> integer wraps (two's complement bits);
         * integer -> f32 / f64 rounds to nearest in one step; f16 / bf16 through f64 (exact below
         * 2^53, and f16 is infinite beyond it either way). */
        switch (dtype_out) {
        case OR_BOOL: case OR_UINT8: ((uint8_t*)out)[o] = (uint8_t)best; break;
        case OR_INT8: ((int8_t*)out)[o] = (int8_t)best; break;
        case OR_INT16: ((int16_t*)out)[o] = (int16_t)best; break;
        case OR_INT32: ((int32_t*)out)[o] = (int32_t)best; break;
        case OR_INT64: ((int64_t*)out)[o] = (int64_t)best; break;
        case OR_UINT16: ((uint16_t*)out)[o] = (uint16_t)best; break;
        case OR_UINT32: ((uint32_t*)out)[o] = (uint32_t)best; break;
        case OR_UINT64: ((uint64_t*)out)[o] = best; break;
        case OR_FLOAT32:
            ((float*)out)[o] = sgn ? (float)(int64_t)best : (float)best;
            break;
        case OR_FLOAT64:
            ((double*)out)[o] = sgn ? (double)(int64_t)best : (double)best;
            break;
        default:
            cast_one_from_f64(sgn ? (double)(int64_t)best : (double)best, dtype_out, out, o);
            break;
        }
    }
    free(keys);
    return 0;
}

/* ------------------------------------------------------------------------------------------ */
/* Synthetic inputs                                                          */
/* ------------------------------------------------------------------------------------------ */

uint64_t oracle_splitmix64(uint64_t x) {
    uint64_t z = x + 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

void oracle_synth_step_noise_f32(float* out, const int64_t* shape, int ndim,
                                 const int64_t* global_shape, int64_t z0, uint64_t seed) {
    int64_t n = numel(shape, ndim);
    int64_t nx = global_shape[ndim - 1];
    int64_t plane = n / (shape[0] > 0 ? shape[0] : 1); /* elements per first-axis slice */
    for (int64_t i = 0; i < n; ++i) {
        int64_t gl = (z0 + i / plane) * plane + i % plane; /* global linear index */
        int64_t x = i % shape[ndim - 1];
        uint64_t h = oracle_splitmix64(seed ^ (uint64_t)gl);
        float U = (float)(h >> 40) * (1.0f / 16777216.0f);
        float t = 100.0f * U;
        out[i] = t + (x >= nx / 2 ? 500.0f : 0.0f);
    }
}

void oracle_synth_u16(uint16_t* out, const int64_t* shape, int ndim,
                      const int64_t* global_shape, int64_t z0, uint64_t seed) {
    (void)global_shape;
    int64_t n = numel(shape, ndim);
    int64_t plane = n / (shape[0] > 0 ? shape[0] : 1);
    for (int64_t i = 0; i < n; ++i) {
        int64_t gl = (z0 + i / plane) * plane + i % plane;
        uint64_t h = oracle_splitmix64(seed ^ (uint64_t)gl);
        out[i] = (uint16_t)(((h >> 40) * 65535ull) >> 24);
    }
}

void oracle_synth_block_f32(float* out, const int64_t* start, const int64_t* shape,
                            const int64_t* global_shape, uint64_t seed) {
    int64_t nx = global_shape[2];
    int64_t i = 0;
    for (int64_t z = 0; z < shape[0]; ++z)
        for (int64_t y = 0; y < shape[1]; ++y)
            for (int64_t x = 0; x < shape[2]; ++x, ++i) {
                int64_t gz = start[0] + z, gy = start[1] + y, gx = start[2] + x;
                int64_t gl = (gz * global_shape[1] + gy) * nx + gx;
                uint64_t h = oracle_splitmix64(seed ^ (uint64_t)gl);
                float U = (float)(h >> 40) * (1.0f / 16777216.0f);
                float t = 100.0f * U;
                out[i] = t + (gx >= nx / 2 ? 500.0f : 0.0f);
            }
}

/* The box [start, start+shape) of an N-d global synthetic volume (C order), kind 0 = step+noise
 * f32 (as oracle_synth_step_noise_f32), kind 1 = u16 noise (as oracle_synth_u16): element i of
 * the box takes the value of its global linear index. Used by the full-size parity samples. */
static void synth_block_nd(void* out, int kind, const int64_t* start, const int64_t* shape,
                           const int64_t* global_shape, int ndim, uint64_t seed) {
    int64_t n = numel(shape, ndim), nx = global_shape[ndim - 1];
    int64_t idx[16] = {0};
    for (int64_t i = 0; i < n; ++i) {
        int64_t gl = 0;
        for (int d = 0; d < ndim; ++d) gl = gl * global_shape[d] + start[d] + idx[d];
        uint64_t h = oracle_splitmix64(seed ^ (uint64_t)gl);
        if (kind == 0) {
            float U = (float)(h >> 40) * (1.0f / 16777216.0f);
            float t = 100.0f * U;
            ((float*)out)[i] = t + (start[ndim - 1] + idx[ndim - 1] >= nx / 2 ? 500.0f : 0.0f);
        } else {
            ((uint16_t*)out)[i] = (uint16_t)(((h >> 40) * 65535ull) >> 24);
        }
        for (int d = ndim - 1; d >= 0; --d) {
            if (++idx[d] < shape[d]) break;
            idx[d] = 0;
        }
    }
}

void oracle_synth_block_nd_f32(float* out, const int64_t* start, const int64_t* shape,
                               const int64_t* global_shape, int ndim, uint64_t seed) {
    synth_block_nd(out, 0, start, shape, global_shape, ndim, seed);
}

void oracle_synth_block_nd_u16(uint16_t* out, const int64_t* start, const int64_t* shape,
                               const int64_t* global_shape, int ndim, uint64_t seed) {
    synth_block_nd(out, 1, start, shape, global_shape, ndim, seed);
}

typedef struct {
    float** blocks;
    int64_t (*shapes)[3];
    int n;
    float epsilon;
    int radius;
    int next;
    pthread_mutex_t mu;
} sample_job;

static void* sample_worker(void* arg) {
    sample_job* j = (sample_job*)arg;
    for (;;) {
        pthread_mutex_lock(&j->mu);
        int c = j->next < j->n ? j->next++ : -1;
        pthread_mutex_unlock(&j->mu);
        if (c < 0) break;
        oracle_guided_filter_apply_ndarray(j->blocks[c], j->shapes[c], 3, j->epsilon, j->radius, 1);
    }
    return NULL;
}

static double now_s(void) {
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return (double)ts.tv_sec + 1e-9 * (double)ts.tv_nsec;
}

double oracle_guided_filter_time_chunks(const int64_t* global_shape, const int64_t* chunk_shape,
                                        const int64_t* chunk_coords, int n_chunks, float epsilon,
                                        int radius, int nthreads, uint64_t seed,
                                        int64_t* voxels_out) {
    sample_job j;
    j.blocks = (float**)calloc((size_t)n_chunks, sizeof(float*));
    j.shapes = malloc(sizeof(int64_t[3]) * (size_t)n_chunks);
    j.n = n_chunks; j.epsilon = epsilon; j.radius = radius; j.next = 0;
    pthread_mutex_init(&j.mu, NULL);
    int64_t vox = 0, h = (int64_t)((radius * 2) & 0xFF);
    for (int c = 0; c < n_chunks; ++c) {
        int64_t st[3];
        for (int d = 0; d < 3; ++d) {
            int64_t o0 = chunk_coords[3 * c + d] * chunk_shape[d];
            int64_t o1 = o0 + chunk_shape[d] < global_shape[d] ? o0 + chunk_shape[d] : global_shape[d];
            int64_t i0 = o0 > h ? o0 - h : 0;
            int64_t i1 = o1 + h < global_shape[d] ? o1 + h : global_shape[d];
            st[d] = i0;
            j.shapes[c][d] = i1 - i0;
        }
        int64_t o = 1;
        for (int d = 0; d < 3; ++d) {
            int64_t o0 = chunk_coords[3 * c + d] * chunk_shape[d];
            int64_t o1 = o0 + chunk_shape[d] < global_shape[d] ? o0 + chunk_shape[d] : global_shape[d];
            o *= o1 - o0;
        }
        vox += o;
        j.blocks[c] = (float*)malloc(sizeof(float) * (size_t)(j.shapes[c][0] * j.shapes[c][1] * j.shapes[c][2]));
        oracle_synth_block_f32(j.blocks[c], st, j.shapes[c], global_shape, seed);
    }
    if (nthreads < 1) nthreads = 1;
    pthread_t* th = (pthread_t*)malloc(sizeof(pthread_t) * (size_t)nthreads);
    double t0 = now_s();
    for (int t = 0; t < nthreads; ++t) pthread_create(&th[t], NULL, sample_worker, &j);
    for (int t = 0; t < nthreads; ++t) pthread_join(th[t], NULL);
    double t1 = now_s();
    free(th);
    for (int c = 0; c < n_chunks; ++c) free(j.blocks[c]);
    free(j.blocks);
    free(j.shapes);
    pthread_mutex_destroy(&j.mu);
    if (voxels_out) *voxels_out = vox;
    return t1 - t0;
}

/* ------------------------------------------------------------------------------------------ */
/* Gaussian (gaussian.rs:110-119, :252-267; kernel.rs:17-73)                                   */
/* ------------------------------------------------------------------------------------------ */

/* gaussian.rs:252-267. Operation order as written there: t = sigma*sigma;
 * scale = 1 / (2 * PI * t).sqrt(); tap(n) = scale * (-((n*n) as f32 / (2 * t))).exp(). f32::exp
 * is the platform libm expf (glibc here, as for the reference on Linux). */
int64_t oracle_gaussian_kernel(float sigma, int64_t half, float* taps) {
    if (sigma == 0.0f) {
        taps[0] = 1.0f;
        return 1;
    }
    const float pi = 3.14159265358979323846f; /* std::f32::consts::PI */
    const float t = sigma * sigma;
    const float scale = 1.0f / sqrtf(2.0f * pi * t);
    for (int64_t n = 0; n <= half; ++n) {
        const float e = scale * expf(-((float)(uint64_t)(n * n) / (2.0f * t)));
        taps[half - n] = e; /* reversed half, then the half without n = 0 */
        taps[half + n] = e;
    }
    return 2 * half + 1;
}

/* kernel.rs:17-73 apply_1d_kernel along `axis` of a C-order block: out[k] = sum over the taps of
 * in[min(k+i saturating_sub mid, n-1)] * tap[i], summed in tap order as f32 (Iterator::sum,
 * no fused multiply-add). */
static void gauss_1d(const float* in, float* out, const int64_t* shape, int ndim, int axis,
                     const float* taps, int64_t len) {
    int64_t inner = 1, outer = 1;
    for (int j = axis + 1; j < ndim; ++j) inner *= shape[j];
    for (int j = 0; j < axis; ++j) outer *= shape[j];
    const int64_t n = shape[axis], mid = len / 2;
    for (int64_t o = 0; o < outer; ++o)
        for (int64_t jn = 0; jn < inner; ++jn) {
            const int64_t base = o * n * inner + jn;
            for (int64_t k = 0; k < n; ++k) {
                float sum = -0.0f;
                for (int64_t i = 0; i < len; ++i) {
                    int64_t p = k + i >= mid ? k + i - mid : 0;
                    if (p > n - 1) p = n - 1;
                    const float prod = in[base + p * inner] * taps[i];
                    sum = sum + prod;
                }
                out[base + k * inner] = sum;
            }
        }
}

int oracle_gaussian_apply_ndarray(float* v, const int64_t* shape, int ndim, const float* sigma,
                                  const int64_t* half) {
    if (ndim < 1 || ndim > OR_MAXDIM) return -1;
    const int64_t nel = numel(shape, ndim);
    if (nel == 0) return 0;
    float* tmp = (float*)malloc(sizeof(float) * nel);
    float* a = v; /* current input */
    float* b = tmp;
    for (int d = 0; d < ndim; ++d) {
        float* taps = (float*)malloc(sizeof(float) * (2 * half[d] + 1));
        const int64_t len = oracle_gaussian_kernel(sigma[d], half[d], taps);
        gauss_1d(a, b, shape, ndim, d, taps, len);
        free(taps);
        float* t = a; a = b; b = t; /* the pass output becomes the next input */
    }
    if (a != v) memcpy(v, a, sizeof(float) * nel);
    free(tmp);
    return 0;
}

int oracle_gaussian_apply(const float* in, float* out, const int64_t* shape, int ndim,
                          const int64_t* chunk_shape, const float* sigma, const int64_t* half) {
    if (ndim < 1 || ndim > OR_MAXDIM) return -1;
    int64_t grid[OR_MAXDIM], nchunks = 1;
    for (int j = 0; j < ndim; ++j) {
        if (chunk_shape[j] <= 0 || half[j] < 0) return -1;
        grid[j] = (shape[j] + chunk_shape[j] - 1) / chunk_shape[j];
        nchunks *= grid[j];
    }
    for (int64_t c = 0; c < nchunks; ++c) {
        int64_t cidx[OR_MAXDIM], o_start[OR_MAXDIM], o_end[OR_MAXDIM];
        int64_t i_start[OR_MAXDIM], i_shape[OR_MAXDIM], d_start[OR_MAXDIM], o_shape[OR_MAXDIM];
        unravel(c, grid, ndim, cidx);
        for (int j = 0; j < ndim; ++j) {
            o_start[j] = cidx[j] * chunk_shape[j];
            const int64_t e = o_start[j] + chunk_shape[j];
            o_end[j] = e < shape[j] ? e : shape[j];
            /* ArraySubsetOverlap::new(shape, subset, kernel_half_size) (gaussian.rs:86-87) */
            i_start[j] = o_start[j] > half[j] ? o_start[j] - half[j] : 0;
            const int64_t ie = o_end[j] + half[j];
            i_shape[j] = (ie < shape[j] ? ie : shape[j]) - i_start[j];
            d_start[j] = o_start[j] - i_start[j];
            o_shape[j] = o_end[j] - o_start[j];
        }
        const int64_t nin = numel(i_shape, ndim), nout = numel(o_shape, ndim);
        float* block = (float*)malloc(sizeof(float) * (nin > 0 ? nin : 1));
        int64_t idx[OR_MAXDIM];
        for (int64_t lin = 0; lin < nin; ++lin) {
            unravel(lin, i_shape, ndim, idx);
            int64_t off = 0;
            for (int j = 0; j < ndim; ++j) off = off * shape[j] + (i_start[j] + idx[j]);
            block[lin] = in[off];
        }
        oracle_gaussian_apply_ndarray(block, i_shape, ndim, sigma, half);
        for (int64_t lin = 0; lin < nout; ++lin) {
            unravel(lin, o_shape, ndim, idx);
            int64_t src = 0, dst = 0;
            for (int j = 0; j < ndim; ++j) {
                src = src * i_shape[j] + (d_start[j] + idx[j]);
                dst = dst * shape[j] + (o_start[j] + idx[j]);
            }
            out[dst] = block[src];
        }
        free(block);
    }
    return 0;
}
