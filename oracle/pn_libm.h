/*
 * oracle/pn_libm.h -- TEST INFRASTRUCTURE (parity oracle), never shipped or linked
 * by the product path.  Only tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg may load anything under oracle/.
 *
 * PN-libm v1: the fixed fp32 definition of the GLSL built-ins that
 * shaders/ray_tracing.comp calls and whose precision GLSL leaves to the
 * driver (sin, cos, atan(y,x), asin, log, pow; ray_tracing.comp:184,566-572,
 * 644,655-660,691,700,702).  The GLSL-on-NVIDIA values cannot be reproduced
 * anywhere (vendor transcendentals), so this repository fixes ONE sequence of
 * IEEE-754 binary32 operations (+ - * /, sqrt, floor, integer bit ops; no FMA,
 * no contraction) per function.  The HIP device side implements the same
 * sequence independently in pnraytracing_amd/csrc/pn_math.h; the GPU test
 * tests/test_gpu_parity.py::test_math_bitwise checks the two agree bit for bit.
 *
 * Algorithms: Cody-Waite reduction + minimax polynomials (coefficients from
 * the public Cephes single-precision library: sinf/cosf, atanf, asinf, logf,
 * exp2f).  Accuracy vs glibc double: <= 3 ulp on the ranges the shader uses
 * (tests/test_oracle_kat.py::test_libm_accuracy).
 *
 * Compile with -ffp-contract=off -fno-fast-math.
 */
#ifndef PN_LIBM_H
#define PN_LIBM_H
#include <stdint.h>
#include <string.h>
#include <math.h>

static inline float pnl_bits2f(uint32_t u) { float f; memcpy(&f, &u, 4); return f; }
static inline uint32_t pnl_f2bits(float f) { uint32_t u; memcpy(&u, &f, 4); return u; }
static inline float pnl_nan(void) { return pnl_bits2f(0x7fc00000u); }
static inline float pnl_inf(void) { return pnl_bits2f(0x7f800000u); }
static inline float pnl_fabs(float x) { return pnl_bits2f(pnl_f2bits(x) & 0x7fffffffu); }

/* sin/cos: reduce by pi/2 with a 3-part Cody-Waite constant (exact products
 * for |k| < 2^13, i.e. |x| < ~1.2e4), quadrant select, Cephes polynomials on
 * |r| <= pi/4.  NaN/inf -> NaN; |x| >= 1e6 -> x - x (0 for finite). */
static inline float pnl_sin_kernel(float r) {
    float z = r * r;
    float p = -1.9515295891e-4f;
    p = p * z + 8.3321608736e-3f;
    p = p * z - 1.6666654611e-1f;
    return r + (r * z) * p;
}
static inline float pnl_cos_kernel(float r) {
    float z = r * r;
    float p = 2.443315711809948e-5f;
    p = p * z - 1.388731625493765e-3f;
    p = p * z + 4.166664568298827e-2f;
    float y = (p * z) * z;
    y = y - 0.5f * z;
    return y + 1.0f;
}
static inline float pnl_reduce(float x, int* q) {
    float k = floorf(x * 0.636619772f + 0.5f);
    float r = x - k * 1.5703125f;
    r = r - k * 4.837512969970703125e-4f;
    r = r - k * 7.54978995489188216e-8f;
    *q = ((int)k) & 3;
    return r;
}
static inline float pnl_sin(float x) {
    if (!(pnl_fabs(x) < 1.0e6f)) return x - x;
    int q; float r = pnl_reduce(x, &q);
    float s = pnl_sin_kernel(r), c = pnl_cos_kernel(r);
    return q == 0 ? s : q == 1 ? c : q == 2 ? -s : -c;
}
static inline float pnl_cos(float x) {
    if (!(pnl_fabs(x) < 1.0e6f)) return x - x;
    int q; float r = pnl_reduce(x, &q);
    float s = pnl_sin_kernel(r), c = pnl_cos_kernel(r);
    return q == 0 ? c : q == 1 ? -s : q == 2 ? -c : s;
}

/* atan2(y, x): octant reduction to t = min/max in [0,1], one pi/4 shift for
 * t > tan(pi/8), Cephes atanf polynomial.  atan2(0,0) := 0 (GLSL: undefined). */
static inline float pnl_atan2(float y, float x) {
    if (x != x || y != y) return x + y;
    float ax = pnl_fabs(x), ay = pnl_fabs(y);
    float mx = ax > ay ? ax : ay;
    float mn = ax > ay ? ay : ax;
    if (mx == 0.0f) return 0.0f;
    float t;
    if (mx == pnl_inf()) t = (mn == pnl_inf()) ? 1.0f : 0.0f;
    else t = mn / mx;
    float base = 0.0f;
    if (t > 0.414213562373095f) { base = 0.785398163397448f; t = (t - 1.0f) / (t + 1.0f); }
    float z = t * t;
    float p = 8.05374449538e-2f;
    p = p * z - 1.38776856032e-1f;
    p = p * z + 1.99777106478e-1f;
    p = p * z - 3.33329491539e-1f;
    float r = base + ((p * z) * t + t);
    if (ay > ax) r = 1.57079632679490f - r;
    if (x < 0.0f) r = 3.14159265358979f - r;
    if (y < 0.0f) r = -r;
    return r;
}

/* asin: Cephes asinf (|x| > 0.5 via pi/2 - 2 asin(sqrt((1-|x|)/2))); |x| > 1 -> NaN. */
static inline float pnl_asin(float x) {
    if (x != x) return x;
    float a = pnl_fabs(x);
    if (a > 1.0f) return pnl_nan();
    float z, s; int big = 0;
    if (a > 0.5f) { z = 0.5f * (1.0f - a); s = sqrtf(z); big = 1; }
    else { s = a; z = a * a; }
    float p = 4.2163199048e-2f;
    p = p * z + 2.4181311049e-2f;
    p = p * z + 4.5470025998e-2f;
    p = p * z + 7.4953002686e-2f;
    p = p * z + 1.6666752422e-1f;
    float r = (p * z) * s + s;
    if (big) { r = r + r; r = 1.57079632679490f - r; }
    return x < 0.0f ? -r : r;
}

/* natural log: Cephes logf.  x<0 -> NaN, 0 -> -inf, inf -> inf. */
static inline float pnl_log(float x) {
    if (x != x) return x;
    if (x < 0.0f) return pnl_nan();
    if (x == 0.0f) return -pnl_inf();
    if (x == pnl_inf()) return x;
    int e = 0;
    if (x < 1.17549435e-38f) { x = x * 16777216.0f; e = -24; }
    uint32_t b = pnl_f2bits(x);
    e += (int)((b >> 23) & 0xffu) - 126;
    float m = pnl_bits2f((b & 0x807fffffu) | 0x3f000000u);   /* [0.5, 1) */
    if (m < 0.707106781186547524f) { e -= 1; m = (m + m) - 1.0f; }
    else { m = m - 1.0f; }
    float z = m * m;
    float p = 7.0376836292e-2f;
    p = p * m - 1.1514610310e-1f;
    p = p * m + 1.1676998740e-1f;
    p = p * m - 1.2420140846e-1f;
    p = p * m + 1.4249322787e-1f;
    p = p * m - 1.6668057665e-1f;
    p = p * m + 2.0000714765e-1f;
    p = p * m - 2.4999993993e-1f;
    p = p * m + 3.3333331174e-1f;
    float y = (p * m) * z;
    float fe = (float)e;
    y = y + (-2.12194440e-4f * fe);
    y = y - 0.5f * z;
    float r = m + y;
    r = r + 0.693359375f * fe;
    return r;
}

/* exp2: n = round-half-up(x), Cephes exp2f polynomial on [-0.5,0.5], scale by
 * 2^n built from bits (two steps outside the normal exponent range). */
static inline float pnl_exp2(float x) {
    if (x != x) return x;
    if (x > 128.0f) return pnl_inf();
    if (x < -150.0f) return 0.0f;
    float n = floorf(x + 0.5f);
    float f = x - n;
    float p = 1.535336188319500e-4f;
    p = p * f + 1.339887440266574e-3f;
    p = p * f + 9.618437357674640e-3f;
    p = p * f + 5.550332471162809e-2f;
    p = p * f + 2.402264791363012e-1f;
    p = p * f + 6.931472028550421e-1f;
    float r = 1.0f + f * p;
    int ni = (int)n;
    if (ni > 127) { r = r * 1.70141183e38f; ni -= 127; }
    if (ni < -126) { r = r * 1.17549435e-38f; ni += 126; }
    return r * pnl_bits2f((uint32_t)(ni + 127) << 23);
}

/* GLSL pow is defined as exp2(y * log2(x)) (GLSL 4.50 spec 8.2). */
static inline float pnl_pow(float x, float y) {
    return pnl_exp2(y * (pnl_log(x) * 1.44269504088896341f));
}

#endif
