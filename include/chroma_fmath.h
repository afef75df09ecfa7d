/* chroma_fmath.h -- portable, bit-reproducible single-precision math.
 *
 * The reference builds its kernels with `--use_fast_math` (chroma/gpu/tools.py:17-21),
 * so its logf/sinf/cosf/... are CUDA intrinsics whose last bits are not
 * reproducible anywhere else.  This build defines its own transcendental
 * functions from IEEE-exact primitives only (+ - * /, sqrtf, fmaf, integer bit
 * operations), so the HIP kernels (gfx950) and the CPU oracle (gcc, x86-64)
 * compute the SAME bits.  Both sides are compiled with -ffp-contract=off; every
 * fused multiply-add below is explicit (fmaf is exactly rounded on both).
 *
 * Accuracy: within ~2 ulp of the correctly-rounded result on the ranges the
 * propagator uses (tested in tests/test_fmath.py against float64 numpy).
 * Algorithms: classic Cody-Waite argument reduction + short minimax polynomials
 * (fdlibm/cephes-style public-domain coefficient sets).
 *
 * This header is product code; the oracle (oracle/) includes it so that the
 * parity gate (oracle == HIP) is bit-exact.
 */
#ifndef CHROMA_FMATH_H
#define CHROMA_FMATH_H

#include <stdint.h>

#if defined(__HIPCC__)
#include <hip/hip_runtime.h>
#define CHR_FN __host__ __device__ static inline
#else
#include <math.h>
#include <string.h>
#define CHR_FN static inline
#endif

#define CHR_PI_F 3.141592653589793f
#define CHR_PIO2_F 1.57079632679489661923f

/* float -> uint32 with CUDA's saturating conversion (cvt.rzi.sat.u32.f32:
 * NaN and negatives -> 0, >= 2^32 -> 0xFFFFFFFF); a plain C cast is undefined
 * there (DAQ / PDF charge words, daq.cu:72, pdf.cu:15) */
CHR_FN uint32_t chr_sat_u32(float x) {
    if (!(x > 0.0f)) return 0u;
    if (x >= 4294967296.0f) return 0xFFFFFFFFu;
    return (uint32_t)x;
}

CHR_FN uint32_t chr_f2u(float x) {
#if defined(__HIPCC__)
    return __builtin_bit_cast(uint32_t, x);
#else
    uint32_t u; memcpy(&u, &x, 4); return u;
#endif
}
CHR_FN float chr_u2f(uint32_t u) {
#if defined(__HIPCC__)
    return __builtin_bit_cast(float, u);
#else
    float x; memcpy(&x, &u, 4); return x;
#endif
}

CHR_FN float chr_fmaf(float a, float b, float c) {
#if defined(__HIPCC__)
    return __builtin_fmaf(a, b, c);
#else
    return fmaf(a, b, c);
#endif
}
CHR_FN float chr_sqrtf(float x) {   /* IEEE correctly rounded on both targets */
#if defined(__HIPCC__)
    return __builtin_sqrtf(x);
#else
    return sqrtf(x);
#endif
}
CHR_FN float chr_fabsf(float x) { return chr_u2f(chr_f2u(x) & 0x7fffffffu); }
CHR_FN int chr_isnan(float x) { return (chr_f2u(x) & 0x7fffffffu) > 0x7f800000u; }
CHR_FN int chr_isfinite(float x) { return (chr_f2u(x) & 0x7f800000u) != 0x7f800000u; }
/* round-half-away-free nearest integer via the 1.5*2^23 trick, valid |x| < 2^22 */
CHR_FN float chr_rintf_small(float x) {
    const float magic = 12582912.0f;
    return (x + magic) - magic;
}
/* x * 2^k for integer k (exact whenever the result is representable) */
CHR_FN float chr_ldexpf(float x, int k) {
    if (k > 127) { x *= chr_u2f(0x7f000000u); k -= 127; if (k > 127) k = 127; }
    else if (k < -126) { x *= chr_u2f(0x00800000u) * 16777216.0f; k += 102;  /* 2^-126 * 2^24 = 2^-102 */
        if (k < -126) { x *= chr_u2f(0x00800000u) * 16777216.0f; k += 102; if (k < -126) k = -126; } }
    return x * chr_u2f((uint32_t)(k + 127) << 23);
}

/* ---------------------------------------------------------------- log */
CHR_FN float chr_logf(float x) {
    const float ln2_hi = 6.9313812256e-01f, ln2_lo = 9.0580006145e-06f;
    const float L1 = 0.66666662693f, L2 = 0.40000972152f, L3 = 0.28498786688f, L4 = 0.24279078841f;
    uint32_t ix = chr_f2u(x);
    int k = 0;
    if (ix >= 0x7f800000u || ix < 0x00800000u) {
        if ((ix & 0x7fffffffu) == 0) return -chr_u2f(0x7f800000u);   /* log(+-0) = -inf */
        if (ix >> 31) return chr_u2f(0x7fc00000u);                   /* log(<0) = nan */
        if (ix >= 0x7f800000u) return x;                              /* inf or nan */
        x *= 33554432.0f; k = -25; ix = chr_f2u(x);                   /* subnormal */
    }
    ix += 0x3f800000u - 0x3f3504f3u;
    k += (int)(ix >> 23) - 127;
    ix = (ix & 0x007fffffu) + 0x3f3504f3u;
    float f = chr_u2f(ix) - 1.0f;                 /* f in [sqrt(1/2)-1, sqrt(2)-1) */
    float s = f / (2.0f + f);
    float z = s * s;
    float w = z * z;
    float t1 = w * chr_fmaf(w, L4, L2);
    float t2 = z * chr_fmaf(w, L3, L1);
    float R = t2 + t1;
    float hfsq = 0.5f * f * f;
    float dk = (float)k;
    return chr_fmaf(s, hfsq + R, dk * ln2_lo) - hfsq + f + dk * ln2_hi;
}

/* ---------------------------------------------------------------- exp */
CHR_FN float chr_expf(float x) {
    const float ln2_hi = 6.9314575195e-01f, ln2_lo = 1.4286067653e-06f, inv_ln2 = 1.4426950216e+00f;
    const float P1 = 1.6666625440e-1f, P2 = -2.7667332906e-3f;
    if (chr_isnan(x)) return x;
    if (x > 88.7228393555f) return chr_u2f(0x7f800000u);
    if (x < -103.972084045f) return 0.0f;
    float kf = chr_rintf_small(x * inv_ln2);
    int k = (int)kf;
    float hi = chr_fmaf(-kf, ln2_hi, x);
    float lo = kf * ln2_lo;
    float r = hi - lo;
    float rr = r * r;
    float c = r - rr * chr_fmaf(rr, P2, P1);
    float y = 1.0f - ((lo - (r * c) / (2.0f - c)) - hi);
    return chr_ldexpf(y, k);
}

/* ---------------------------------------------------- sin / cos / tan */
/* reduce x = n*(pi/2) + r, |r| <= ~pi/4; returns n (quadrant) */
CHR_FN int chr_rem_pio2f(float x, float *r) {
    const float two_over_pi = 6.3661974669e-01f;
    const float p1 = 1.5707963705062866e+00f;     /* float(pi/2) */
    const float p2 = -4.3711388286737929e-08f;    /* pi/2 - p1 (float) */
    const float p3 = -1.7151245100059665e-15f;    /* remainder */
    float n = chr_rintf_small(x * two_over_pi);
    float y = chr_fmaf(-n, p1, x);
    y = chr_fmaf(-n, p2, y);
    y = chr_fmaf(-n, p3, y);
    *r = y;
    return (int)n;
}
CHR_FN float chr_ksinf(float x) {   /* |x| <= pi/4 */
    float z = x * x;
    float p = chr_fmaf(chr_fmaf(-1.9515295891e-4f, z, 8.3321608736e-3f), z, -1.6666654611e-1f);
    return chr_fmaf(x * z, p, x);
}
CHR_FN float chr_kcosf(float x) {   /* |x| <= pi/4 */
    float z = x * x;
    float p = chr_fmaf(chr_fmaf(2.443315711809948e-5f, z, -1.388731625493765e-3f), z, 4.166664568298827e-2f);
    return chr_fmaf(z * z, p, chr_fmaf(-0.5f, z, 1.0f));
}
CHR_FN void chr_sincosf(float x, float *s, float *c) {
    if (!chr_isfinite(x)) { *s = x - x; *c = x - x; return; }
    float r;
    int n = chr_rem_pio2f(x, &r);
    float sr = chr_ksinf(r), cr = chr_kcosf(r);
    switch (n & 3) {
    case 0: *s = sr; *c = cr; break;
    case 1: *s = cr; *c = -sr; break;
    case 2: *s = -sr; *c = -cr; break;
    default: *s = -cr; *c = sr; break;
    }
}
CHR_FN float chr_sinf(float x) { float s, c; chr_sincosf(x, &s, &c); return s; }
CHR_FN float chr_cosf(float x) { float s, c; chr_sincosf(x, &s, &c); return c; }
CHR_FN float chr_tanf(float x) { float s, c; chr_sincosf(x, &s, &c); return s / c; }

/* ---------------------------------------------------- asin / acos */
CHR_FN float chr_asin_poly(float z) {
    return chr_fmaf(chr_fmaf(chr_fmaf(chr_fmaf(4.2163199048e-2f, z, 2.4181311049e-2f), z,
                    4.5470025998e-2f), z, 7.4953002686e-2f), z, 1.6666752422e-1f);
}
CHR_FN float chr_asinf(float x) {
    float a = chr_fabsf(x);
    if (a > 1.0f) return chr_u2f(0x7fc00000u);
    float r;
    if (a > 0.5f) {
        float z = 0.5f * (1.0f - a);
        float t = chr_sqrtf(z);
        r = CHR_PIO2_F - 2.0f * chr_fmaf(t * z, chr_asin_poly(z), t);
    } else if (a < 1e-4f) {
        r = a;
    } else {
        float z = a * a;
        r = chr_fmaf(a * z, chr_asin_poly(z), a);
    }
    return (chr_f2u(x) >> 31) ? -r : r;
}
CHR_FN float chr_acosf(float x) {
    if (chr_isnan(x) || chr_fabsf(x) > 1.0f) return chr_u2f(0x7fc00000u);
    if (x < -0.5f) return CHR_PI_F - 2.0f * chr_asinf(chr_sqrtf(0.5f * (1.0f + x)));
    if (x > 0.5f) return 2.0f * chr_asinf(chr_sqrtf(0.5f * (1.0f - x)));
    return CHR_PIO2_F - chr_asinf(x);
}

/* ---------------------------------------------------- atan / atan2 */
CHR_FN float chr_atanf(float x) {
    float a = chr_fabsf(x), y, z;
    if (chr_isnan(x)) return x;
    if (a > 2.414213562373095f) { y = CHR_PIO2_F; a = -1.0f / a; }
    else if (a > 0.4142135623730950f) { y = 0.25f * CHR_PI_F; a = (a - 1.0f) / (a + 1.0f); }
    else y = 0.0f;
    z = a * a;
    float p = chr_fmaf(chr_fmaf(chr_fmaf(8.05374449538e-2f, z, -1.38776856032e-1f), z,
                        1.99777106478e-1f), z, -3.33329491539e-1f);
    y = y + chr_fmaf(p * z, a, a);
    return (chr_f2u(x) >> 31) ? -y : y;
}
CHR_FN float chr_atan2f(float y, float x) {
    if (chr_isnan(x) || chr_isnan(y)) return x + y;
    int ysign = (int)(chr_f2u(y) >> 31);
    if (x == 0.0f) {
        if (y == 0.0f) return (chr_f2u(x) >> 31) ? (ysign ? -CHR_PI_F : CHR_PI_F) : y;
        return ysign ? -CHR_PIO2_F : CHR_PIO2_F;
    }
    float r;
    if (!chr_isfinite(x) || !chr_isfinite(y)) {
        /* rare: fall back on quadrant limits */
        if (!chr_isfinite(x) && !chr_isfinite(y)) r = (x > 0.0f) ? 0.25f * CHR_PI_F : 0.75f * CHR_PI_F;
        else if (!chr_isfinite(y)) r = CHR_PIO2_F;
        else r = (x > 0.0f) ? 0.0f : CHR_PI_F;
        return ysign ? -r : r;
    }
    r = chr_atanf(chr_fabsf(y / x));
    if (x < 0.0f) r = CHR_PI_F - r;
    return ysign ? -r : r;
}

/* ---------------------------------------------------------------- erf
 * Used by the kernel-density PDF normalisation (reference pdf.cu:311-362,
 * erff under --use_fast_math).  |x| < 0.5: Maclaurin series to x^13
 * (truncation < 5e-10 relative); 0.5 <= |x| < 4: Abramowitz & Stegun 7.1.26
 * (absolute error <= 1.5e-7; <= 2.5e-7 measured in float32); |x| >= 4: +-1.  Parity with CUDA's erff is
 * unpinned (a few 1e-7 absolute), identical between HIP and the oracle. */
CHR_FN float chr_erff(float x) {
    if (chr_isnan(x)) return x;
    const float a = chr_fabsf(x);
    if (a < 0.5f) {
        const float z = x * x;
        float p = chr_fmaf(1.0683760684e-4f, z, -7.5757575758e-4f);
        p = chr_fmaf(p, z, 4.6296296296e-3f);
        p = chr_fmaf(p, z, -2.3809523810e-2f);
        p = chr_fmaf(p, z, 1.0000000000e-1f);
        p = chr_fmaf(p, z, -3.3333333333e-1f);
        p = chr_fmaf(p, z, 1.0f);
        return (x * 1.1283791671f) * p;
    }
    float r = 1.0f;
    if (a < 4.0f) {
        const float t = 1.0f / chr_fmaf(0.3275911f, a, 1.0f);
        float p = chr_fmaf(1.061405429f, t, -1.453152027f);
        p = chr_fmaf(p, t, 1.421413741f);
        p = chr_fmaf(p, t, -0.284496736f);
        p = chr_fmaf(p, t, 0.254829592f);
        r = 1.0f - (p * t) * chr_expf(-(a * a));
    }
    return (chr_f2u(x) >> 31) ? -r : r;
}

#endif /* CHROMA_FMATH_H */
