// Decimal -> float64 for kernel K0, matching strconv.ParseFloat (and the
// host decoder's correctly rounded strtod) exactly on the inputs it accepts:
//   * Clinger's exact path: mantissa <= 2^53, |exp10| <= 22 -> one IEEE op;
//   * Eisel-Lemire (the algorithm strconv.ParseFloat itself tries first,
//     published by D. Lemire, "Number Parsing at a Gigabyte per Second"):
//     a 64x128-bit product with the table in pow10_128.h, refusing the rare
//     inputs whose rounding it cannot decide.
// Anything refused (more than 19 significant digits, subnormal or overflowing
// results, undecided halfway cases) goes back to the host decoder.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "pow10_128.h"

namespace gd {

__host__ __device__ inline uint64_t mul64hi(uint64_t a, uint64_t b) {
#if defined(__HIP_DEVICE_COMPILE__)
    return __umul64hi(a, b);
#else
    return (uint64_t)(((unsigned __int128)a * b) >> 64);
#endif
}

__host__ __device__ inline uint32_t clz64(uint64_t x) {
#if defined(__HIP_DEVICE_COMPILE__)
    return (uint32_t)__clzll((long long)x);
#else
    return (uint32_t)__builtin_clzll(x);
#endif
}

// man != 0 (the significant digits, <= 19 of them) * 10^exp10 -> float64 bits
__host__ __device__ inline bool eisel_lemire(uint64_t man, int64_t exp10, bool neg, uint64_t* out) {
    if (exp10 < kPow10Min || exp10 > kPow10Max) return false;
    const uint32_t clz = clz64(man);
    man <<= clz;
    uint64_t ret_exp2 = (uint64_t)(((217706 * exp10) >> 16) + 64 + 1023) - clz;
    const uint64_t phi = kPow10[exp10 - kPow10Min][0], plo = kPow10[exp10 - kPow10Min][1];
    uint64_t x_hi = mul64hi(man, phi), x_lo = man * phi;
    if ((x_hi & 0x1FF) == 0x1FF && x_lo + man < man) {  // wider approximation
        const uint64_t y_hi = mul64hi(man, plo), y_lo = man * plo;
        uint64_t m_hi = x_hi, m_lo = x_lo + y_hi;
        if (m_lo < x_lo) m_hi++;
        if ((m_hi & 0x1FF) == 0x1FF && m_lo + 1 == 0 && y_lo + man < man) return false;
        x_hi = m_hi;
        x_lo = m_lo;
    }
    const uint64_t msb = x_hi >> 63;
    uint64_t ret_man = x_hi >> (msb + 9);
    ret_exp2 -= 1 ^ msb;
    if (x_lo == 0 && (x_hi & 0x1FF) == 0 && (ret_man & 3) == 1) return false;  // halfway ambiguity
    ret_man += ret_man & 1;
    ret_man >>= 1;
    if (ret_man >> 53) {
        ret_man >>= 1;
        ret_exp2 += 1;
    }
    if (ret_exp2 - 1 >= 0x7FF - 1) return false;  // subnormal / zero exponent / overflow
    uint64_t bits = (ret_exp2 << 52) | (ret_man & 0x000FFFFFFFFFFFFFull);
    if (neg) bits |= 0x8000000000000000ull;
    *out = bits;
    return true;
}

// sign * man * 10^exp10 (man != 0, <= 19 significant digits) -> float64 bits
__host__ __device__ inline bool decimal_to_double(uint64_t man, int64_t exp10, bool neg, uint64_t* out) {
    if (man <= (1ull << 53) && exp10 >= -22 && exp10 <= 22) {
        constexpr double p10[23] = {1e0,  1e1,  1e2,  1e3,  1e4,  1e5,  1e6,  1e7,  1e8,  1e9,  1e10, 1e11,
                                    1e12, 1e13, 1e14, 1e15, 1e16, 1e17, 1e18, 1e19, 1e20, 1e21, 1e22};
        const double m = (double)man;
        double r = exp10 >= 0 ? m * p10[exp10] : m / p10[-exp10];
        if (neg) r = -r;
        union {
            double d;
            uint64_t u;
        } c;
        c.d = r;
        *out = c.u;
        return true;
    }
    return eisel_lemire(man, exp10, neg, out);
}

}  // namespace gd
