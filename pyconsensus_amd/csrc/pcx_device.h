// pcx_device.h -- device helpers for the single-matrix path: double-double (dd)
// accumulation, order-preserving keys of doubles, exact fixed-point weight limbs,
// wave/block reductions.  Compiled with -ffp-contract=off; every fma() is explicit.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace pcx {

constexpr int WAVE = 64;

// ---------------------------------------------------------------- dd arithmetic
struct dd {
    double hi, lo;
};

__device__ __forceinline__ dd two_sum(double a, double b) {
    const double s = a + b;
    const double z = s - a;
    return {s, (a - (s - z)) + (b - z)};
}

__device__ __forceinline__ dd fast_two_sum(double a, double b) {  // |a| >= |b|
    const double s = a + b;
    return {s, b - (s - a)};
}

__device__ __forceinline__ dd dd_add(dd a, dd b) {
    dd s = two_sum(a.hi, b.hi);
    dd t = two_sum(a.lo, b.lo);
    s.lo += t.hi;
    s = fast_two_sum(s.hi, s.lo);
    s.lo += t.lo;
    return fast_two_sum(s.hi, s.lo);
}

__device__ __forceinline__ dd dd_from(double a) { return {a, 0.0}; }

// compensated accumulator (Dot2 / Sum2): s + c
struct acc2 {
    double s = 0.0, c = 0.0;
    __device__ __forceinline__ void add(double x) {
        const dd t = two_sum(s, x);
        s = t.hi;
        c += t.lo;
    }
    __device__ __forceinline__ void add_prod(double x, double y) {
        const double p = x * y;
        const double pe = fma(x, y, -p);
        const dd t = two_sum(s, p);
        s = t.hi;
        c = c + (pe + t.lo);
    }
    __device__ __forceinline__ dd get() const { return two_sum(s, c); }
};

__device__ __forceinline__ double dd_to_double(dd a) { return a.hi + a.lo; }

// (a.hi+a.lo) / (b.hi+b.lo) rounded to double (one Newton correction)
__device__ __forceinline__ double dd_div(dd a, dd b) {
    const double q = a.hi / b.hi;
    // r = a - q*b in dd
    const double p = q * b.hi;
    const double pe = fma(q, b.hi, -p);
    double r = (a.hi - p);
    r = r - pe;
    r = r + a.lo;
    r = r - q * b.lo;
    return q + r / b.hi;
}

__device__ __forceinline__ dd dd_mul_d(dd a, double b) {
    const double p = a.hi * b;
    const double pe = fma(a.hi, b, -p);
    return fast_two_sum(p, pe + a.lo * b);
}

__device__ __forceinline__ dd dd_sub(dd a, dd b) { return dd_add(a, dd{-b.hi, -b.lo}); }

// the exact product a b as a double-double
__device__ __forceinline__ dd two_prod_dd(double a, double b) {
    const double p = a * b;
    return fast_two_sum(p, fma(a, b, -p));
}

// ---------------------------------------------------------------- keys
// order-preserving map double -> uint64 (-0.0 is folded onto +0.0)
__device__ __forceinline__ uint64_t dkey(double x) {
    if (x == 0.0) x = 0.0;
    const uint64_t u = __double_as_longlong(x);
    return (u >> 63) ? ~u : (u | 0x8000000000000000ull);
}

__device__ __forceinline__ double dkey_inv(uint64_t k) {
    const uint64_t u = (k >> 63) ? (k & 0x7fffffffffffffffull) : ~k;
    return __longlong_as_double(u);
}

// ---------------------------------------------------------------- exact weight limbs
// w (0 <= w < 2^8) as three 43-bit limbs: w = L0*2^-35 + L1*2^-78 + L2*2^-121 (+ tail
// below 2^-121 truncated).  Sums of up to 2^21 limb values fit a uint64.
struct limbs3 {
    uint64_t l0, l1, l2;
};

// Each limb is an integer-valued double f: f + 2^52 holds f in its mantissa bits while f < 2^52, so
// one add and a mask convert it (the generic double -> uint64 conversion takes ~7 fp64 ops, three
// times per element in the selection's weight-mode passes).  A NaN weight gives zero limbs, as the
// generic conversion of NaN does.
// Precondition (the caller's): 0 <= w < 2^8.  Then every limb is below 2^43 and sums of 2^21 limbs
// fit a uint64.  Outside it the limbs are wrong -- f0 = floor(w 2^35) reaches 2^52 at w = 2^17,
// and a negative w has no limbs at all -- so k_sel_start sends any event whose weights leave
// [0, 2^8) (a negative reputation, or one above 256 times the total) to the exact replay in the
// reference's order instead (pcx_matrix.hip, the weight-range test; tests/test_matrix_gpu.py
// negative / large reputation cases).
__device__ __forceinline__ uint64_t limb_bits(double f) {
    return (uint64_t)__double_as_longlong(f + 0x1p52) & 0xFFFFFFFFFFFFFull;
}
__device__ __forceinline__ limbs3 to_limbs(double w) {
    if (__builtin_isnan(w)) w = 0.0;
    const double a = ldexp(w, 35);
    const double f0 = floor(a);
    const double b = ldexp(a - f0, 43);
    const double f1 = floor(b);
    const double c = ldexp(b - f1, 43);
    const double f2 = floor(c);
    return {limb_bits(f0), limb_bits(f1), limb_bits(f2)};
}

// ---------------------------------------------------------------- reductions
__device__ __forceinline__ double wave_sum_d(double v) {
#pragma unroll
    for (int s = 32; s >= 1; s >>= 1) v += __shfl_xor(v, s, WAVE);
    return v;
}

__device__ __forceinline__ dd wave_sum_dd(dd v) {
#pragma unroll
    for (int s = 32; s >= 1; s >>= 1) {
        dd o{__shfl_xor(v.hi, s, WAVE), __shfl_xor(v.lo, s, WAVE)};
        v = dd_add(v, o);
    }
    return v;
}

__device__ __forceinline__ double wave_max_d(double v) {
#pragma unroll
    for (int s = 32; s >= 1; s >>= 1) v = fmax(v, __shfl_xor(v, s, WAVE));
    return v;
}

__device__ __forceinline__ double wave_min_d(double v) {
#pragma unroll
    for (int s = 32; s >= 1; s >>= 1) v = fmin(v, __shfl_xor(v, s, WAVE));
    return v;
}

__device__ __forceinline__ double catch_value(double x, double tol) {  // __init__.py:251-258
    if (x < 1.5 - tol) return 1.0;
    if (x > 1.5 + tol) return 2.0;
    return 1.5;
}

}  // namespace pcx
