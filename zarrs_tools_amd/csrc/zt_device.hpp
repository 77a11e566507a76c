// zt_device.hpp — device-side element conversions for the zarrs_filter path (gfx950).
//
// The reference casts every element with Rust `as` (num-traits 0.2.19 AsPrimitive) and the half
// 2.6.0 crate: TIn -> f32 before the guided filter (guided_filter.rs:99), f32 -> TOut after it
// (:102), TIn -> f64 and f64 -> TOut around the downsample mean (downsample.rs:89-92).
//   float -> int : saturating at the type bounds, NaN -> 0, truncation toward zero.
//   f32 -> f16/bf16 : round to nearest even (half's software path restated bit for bit).
//   f64 -> f16/bf16 : half's software path works on the upper 32 bits of the f64.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace zt {

enum DType : int {
    kBool = 0, kI8 = 1, kI16 = 2, kI32 = 3, kI64 = 4, kU8 = 5, kU16 = 6, kU32 = 7, kU64 = 8,
    kBF16 = 9, kF16 = 10, kF32 = 11, kF64 = 12
};

// Storage tags for 16-bit float types (raw bits in memory).
struct bf16_t { uint16_t bits; };
struct f16_t { uint16_t bits; };

__host__ __device__ inline uint32_t f2u(float f) { return __builtin_bit_cast(uint32_t, f); }
__host__ __device__ inline float u2f(uint32_t u) { return __builtin_bit_cast(float, u); }
__host__ __device__ inline uint64_t d2u(double f) { return __builtin_bit_cast(uint64_t, f); }

__host__ __device__ inline uint16_t f32_to_f16_bits(float value) {
    uint32_t x = f2u(value);
    uint32_t sign = x & 0x80000000u, exp = x & 0x7F800000u, man = x & 0x007FFFFFu;
    if (exp == 0x7F800000u) {
        uint32_t nan_bit = man == 0 ? 0u : 0x0200u;
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
    uint32_t r = half_sign | he | half_man;
    if ((man & round_bit) != 0 && (man & (3 * round_bit - 1)) != 0) r += 1;
    return (uint16_t)r;
}

__host__ __device__ inline uint16_t f64_to_f16_bits(double value) {
    uint64_t val = d2u(value);
    uint32_t x = (uint32_t)(val >> 32);
    uint32_t sign = x & 0x80000000u, exp = x & 0x7FF00000u, man = x & 0x000FFFFFu;
    if (exp == 0x7FF00000u) {
        uint32_t nan_bit = (man == 0 && (uint32_t)val == 0) ? 0u : 0x0200u;
        return (uint16_t)((sign >> 16) | 0x7C00u | nan_bit | (man >> 10));
    }
    uint32_t half_sign = sign >> 16;
    int32_t half_exp = (int32_t)(exp >> 20) - 1023 + 15;
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
    uint32_t r = half_sign | he | half_man;
    if ((man & round_bit) != 0 && (man & (3 * round_bit - 1)) != 0) r += 1;
    return (uint16_t)r;
}

__host__ __device__ inline uint16_t f32_to_bf16_bits(float value) {
    uint32_t x = f2u(value);
    if ((x & 0x7FFFFFFFu) > 0x7F800000u) return (uint16_t)((x >> 16) | 0x0040u);
    uint32_t round_bit = 0x8000u;
    uint32_t r = x >> 16;
    if ((x & round_bit) != 0 && (x & (3 * round_bit - 1)) != 0) r += 1;
    return (uint16_t)r;
}

__host__ __device__ inline uint16_t f64_to_bf16_bits(double value) {
    uint64_t val = d2u(value);
    uint32_t x = (uint32_t)(val >> 32);
    uint32_t sign = x & 0x80000000u, exp = x & 0x7FF00000u, man = x & 0x000FFFFFu;
    if (exp == 0x7FF00000u) {
        uint32_t nan_bit = (man == 0 && (uint32_t)val == 0) ? 0u : 0x0040u;
        return (uint16_t)((sign >> 16) | 0x7F80u | nan_bit | (man >> 13));
    }
    uint32_t half_sign = sign >> 16;
    int32_t half_exp = (int32_t)(exp >> 20) - 1023 + 127;
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
    uint32_t r = half_sign | he | half_man;
    if ((man & round_bit) != 0 && (man & (3 * round_bit - 1)) != 0) r += 1;
    return (uint16_t)r;
}

__host__ __device__ inline float f16_bits_to_f32(uint16_t h) {
    uint32_t sign = (uint32_t)(h & 0x8000u) << 16;
    uint32_t exp = (h >> 10) & 0x1Fu, man = h & 0x3FFu;
    if (exp == 0x1F) return u2f(sign | 0x7F800000u | (man << 13));
    if (exp == 0) {
        if (man == 0) return u2f(sign);
        float f = (float)man * (1.0f / 16777216.0f);  // exact: man < 2^10
        return sign ? -f : f;
    }
    return u2f(sign | ((exp - 15 + 127) << 23) | (man << 13));
}
__host__ __device__ inline float bf16_bits_to_f32(uint16_t h) { return u2f((uint32_t)h << 16); }

// ---- element -> f32 / f64 (`as f32` / `as f64`) ----------------------------------------------
template <typename T> struct Elem;
#define ZT_INT_ELEM(T, CODE)                                                                    \
    template <> struct Elem<T> {                                                                \
        static constexpr int code = CODE;                                                       \
        __device__ static inline float to_f32(T v) { return (float)v; }                         \
        __device__ static inline double to_f64(T v) { return (double)v; }                       \
    };
ZT_INT_ELEM(int8_t, kI8)
ZT_INT_ELEM(int16_t, kI16)
ZT_INT_ELEM(int32_t, kI32)
ZT_INT_ELEM(int64_t, kI64)
ZT_INT_ELEM(uint8_t, kU8)
ZT_INT_ELEM(uint16_t, kU16)
ZT_INT_ELEM(uint32_t, kU32)
ZT_INT_ELEM(uint64_t, kU64)
#undef ZT_INT_ELEM
template <> struct Elem<float> {
    static constexpr int code = kF32;
    __device__ static inline float to_f32(float v) { return v; }
    __device__ static inline double to_f64(float v) { return (double)v; }
};
template <> struct Elem<double> {
    static constexpr int code = kF64;
    __device__ static inline float to_f32(double v) { return (float)v; }
    __device__ static inline double to_f64(double v) { return v; }
};
template <> struct Elem<bf16_t> {
    static constexpr int code = kBF16;
    __device__ static inline float to_f32(bf16_t v) { return bf16_bits_to_f32(v.bits); }
    __device__ static inline double to_f64(bf16_t v) { return (double)bf16_bits_to_f32(v.bits); }
};
template <> struct Elem<f16_t> {
    static constexpr int code = kF16;
    __device__ static inline float to_f32(f16_t v) { return f16_bits_to_f32(v.bits); }
    __device__ static inline double to_f64(f16_t v) { return (double)f16_bits_to_f32(v.bits); }
};

// ---- f32 / f64 -> element (Rust `as`, saturating) ----------------------------------------------
template <typename T> __device__ inline T from_f32(float x);
template <typename T> __device__ inline T from_f64(double x);

// Saturating float->int with NaN->0; bounds compared in the source precision. `hi_excl` is the
// smallest representable value >= MAX+1, so x >= hi_excl saturates and every smaller value
// truncates to <= MAX.
#define ZT_SAT(T, SRC, LO, HI_EXCL, MAXV)                                                         \
    {                                                                                           \
        if (!(x == x)) return (T)0;                                                             \
        if (x <= (SRC)(LO)) return (T)(LO);                                                     \
        if (x >= (SRC)(HI_EXCL)) return (T)(MAXV);                                              \
        return (T)x;                                                                            \
    }
template <> __device__ inline int8_t from_f32<int8_t>(float x) ZT_SAT(int8_t, float, -128, 128, 127)
template <> __device__ inline int16_t from_f32<int16_t>(float x) ZT_SAT(int16_t, float, -32768, 32768, 32767)
template <> __device__ inline int32_t from_f32<int32_t>(float x) ZT_SAT(int32_t, float, -2147483648.0, 2147483648.0, 2147483647)
template <> __device__ inline int64_t from_f32<int64_t>(float x) ZT_SAT(int64_t, float, -9223372036854775808.0, 9223372036854775808.0, 9223372036854775807LL)
template <> __device__ inline uint8_t from_f32<uint8_t>(float x) ZT_SAT(uint8_t, float, 0, 256, 255)
template <> __device__ inline uint16_t from_f32<uint16_t>(float x) ZT_SAT(uint16_t, float, 0, 65536, 65535)
template <> __device__ inline uint32_t from_f32<uint32_t>(float x) ZT_SAT(uint32_t, float, 0, 4294967296.0, 4294967295u)
template <> __device__ inline uint64_t from_f32<uint64_t>(float x) ZT_SAT(uint64_t, float, 0, 18446744073709551616.0, 18446744073709551615ull)
template <> __device__ inline float from_f32<float>(float x) { return x; }
template <> __device__ inline double from_f32<double>(float x) { return (double)x; }
template <> __device__ inline bf16_t from_f32<bf16_t>(float x) { return bf16_t{f32_to_bf16_bits(x)}; }
template <> __device__ inline f16_t from_f32<f16_t>(float x) { return f16_t{f32_to_f16_bits(x)}; }

template <> __device__ inline int8_t from_f64<int8_t>(double x) ZT_SAT(int8_t, double, -128, 128, 127)
template <> __device__ inline int16_t from_f64<int16_t>(double x) ZT_SAT(int16_t, double, -32768, 32768, 32767)
template <> __device__ inline int32_t from_f64<int32_t>(double x) ZT_SAT(int32_t, double, -2147483648.0, 2147483648.0, 2147483647)
template <> __device__ inline int64_t from_f64<int64_t>(double x) ZT_SAT(int64_t, double, -9223372036854775808.0, 9223372036854775808.0, 9223372036854775807LL)
template <> __device__ inline uint8_t from_f64<uint8_t>(double x) ZT_SAT(uint8_t, double, 0, 256, 255)
template <> __device__ inline uint16_t from_f64<uint16_t>(double x) ZT_SAT(uint16_t, double, 0, 65536, 65535)
template <> __device__ inline uint32_t from_f64<uint32_t>(double x) ZT_SAT(uint32_t, double, 0, 4294967296.0, 4294967295u)
template <> __device__ inline uint64_t from_f64<uint64_t>(double x) ZT_SAT(uint64_t, double, 0, 18446744073709551616.0, 18446744073709551615ull)
template <> __device__ inline float from_f64<float>(double x) { return (float)x; }
template <> __device__ inline double from_f64<double>(double x) { return x; }
template <> __device__ inline bf16_t from_f64<bf16_t>(double x) { return bf16_t{f64_to_bf16_bits(x)}; }
template <> __device__ inline f16_t from_f64<f16_t>(double x) { return f16_t{f64_to_f16_bits(x)}; }
#undef ZT_SAT

// Dispatch a runtime dtype code to a C++ element type (Bool is processed as u8, like the
// reference's `(Bool, u8)` dispatch arms).
#define ZT_DISPATCH_DTYPE(CODE, T, ...)                                                         \
    switch (CODE) {                                                                             \
    case ::zt::kBool: case ::zt::kU8: { using T = uint8_t; __VA_ARGS__; } break;                \
    case ::zt::kI8: { using T = int8_t; __VA_ARGS__; } break;                                   \
    case ::zt::kI16: { using T = int16_t; __VA_ARGS__; } break;                                 \
    case ::zt::kI32: { using T = int32_t; __VA_ARGS__; } break;                                 \
    case ::zt::kI64: { using T = int64_t; __VA_ARGS__; } break;                                 \
    case ::zt::kU16: { using T = uint16_t; __VA_ARGS__; } break;                                \
    case ::zt::kU32: { using T = uint32_t; __VA_ARGS__; } break;                                \
    case ::zt::kU64: { using T = uint64_t; __VA_ARGS__; } break;                                \
    case ::zt::kBF16: { using T = ::zt::bf16_t; __VA_ARGS__; } break;                           \
    case ::zt::kF16: { using T = ::zt::f16_t; __VA_ARGS__; } break;                             \
    case ::zt::kF32: { using T = float; __VA_ARGS__; } break;                                   \
    case ::zt::kF64: { using T = double; __VA_ARGS__; } break;                                  \
    default: break;                                                                             \
    }

inline size_t dtype_size(int code) {
    switch (code) {
    case kBool: case kI8: case kU8: return 1;
    case kI16: case kU16: case kBF16: case kF16: return 2;
    case kI32: case kU32: case kF32: return 4;
    case kI64: case kU64: case kF64: return 8;
    default: return 0;
    }
}

}  // namespace zt
