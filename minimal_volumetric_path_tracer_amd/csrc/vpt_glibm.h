/*
 * vpt_glibm.h -- the reference's transcendentals, bit for bit, on the GPU.
 *
 * The reference calls glibc's libm (include/samplingFunctions.h:47-82 acos/sin/cos,
 * include/vptSamplingFunctions.h:11-62 log/acos/sin/cos/tan, include/microFacetUtilities.h:34-84
 * atan/log/exp, include/volumetricBasicFunctions.h:14-21,209-223 exp/atan2), and several
 * branches of its estimators flip on the last bit of those results, so per-channel
 * parity with the reference's own images needs glibc's exact results.  glibc 2.35 on x86-64 hosts
 * with FMA + AVX2 (the container and the GPU box) runs the FMA builds of
 * sysdeps/ieee754/dbl-64/{s_sin.c, e_asin.c, ...}; this file restates those algorithms with every
 * rounding step of that build: where GCC contracted a*b+c into one fused multiply-add the code
 * below calls fma(), everywhere else it rounds each operation (the file is compiled with
 * -ffp-contract=off on both sides).  Coefficient tables are glibc's own (vpt_glibm_tables.h,
 * extracted by scripts/gen_glibc_tables.py); scalar constants are spelled as hex literals.
 * tests/test_glibc_libm.py checks every function against the host's libm bit for bit.
 *
 * The restatement is GPU-shaped, not a transcription: glibc picks one of 4-9 argument ranges per
 * call with branches, and a wave whose 64 lanes hold arguments from different ranges would run
 * every taken branch in turn.  Here the range decides only a few operands -- the reduced
 * argument, its correction term, table offsets, the polynomial degree, a sign -- chosen with
 * selects, and one straight-line evaluation serves all lanes.  Because the selected operations
 * are exactly the ones glibc performs for that lane's range, the bits are unchanged.
 *
 * Domain: everything glibc handles, except sin/cos/tan arguments with |x| >= 105414350, where
 * glibc calls its multi-word reduction (__branred); those return NaN here.  The tracer's angles
 * lie in [-2 pi, 2 pi].
 *
 * Needs VM_QUAL, vm_k, vm_as_u64/vm_as_f64, vm_fabs, vm_copysign (vpt_math.h).
 */
#ifndef VPT_GLIBM_H
#define VPT_GLIBM_H

#if defined(__HIPCC__)
#define GM_TABLE(name, n) __device__ static const double name[n]
#else
#define GM_TABLE(name, n) static const double name[n]
#endif
#include "vpt_glibm_tables.h"

VM_QUAL int32_t gm_hi(double x) { return (int32_t)(vm_as_u64(x) >> 32); }
VM_QUAL uint32_t gm_lo(double x) { return (uint32_t)vm_as_u64(x); }
VM_QUAL double gm_fma(double a, double b, double c) { return fma(a, b, c); }
/* c - a*b with one rounding (x86 vfnmadd) */
VM_QUAL double gm_fnma(double a, double b, double c) { return fma(-a, b, c); }

/* ------------------------------------------------------------------ sin / cos (s_sin.c) */
#define GM_HP0 0x1.921fb54442d18p+0     /* pi/2 high part */
#define GM_HP1 0x1.1a62633145c07p-54    /* pi/2 low part */
#define GM_BIG 0x1.8p+45                /* big: rounds |x| to k/128 */

/* do_sin / do_cos / TAYLOR_SIN of s_sin.c, one evaluation for either.  (a, da) is the reduced
 * argument and its correction; cosine selects do_cos.  do_sin takes the Taylor form when
 * |a| < 0.126, otherwise both read sin(k/128), its tail, cos(k/128), its tail from __sincostab
 * (k = round(128 |a|)) and add a short polynomial in the remainder. */
VM_QUAL double gm_sincos_eval(double a, double da, int cosine)
{
    const double aa = vm_fabs(a);
    /* TAYLOR_SIN(xx, a, da) */
    const double xx0 = a * a;
    double p = gm_fma(vm_k(-0x1.addffc2fcdf59p-26), xx0, vm_k(0x1.71de27b9a7ed9p-19));
    p = gm_fma(p, xx0, vm_k(-0x1.a01a019db08b8p-13));
    p = gm_fma(p, xx0, vm_k(0x1.1111111110ecep-7));
    p = gm_fma(p, xx0, vm_k(-0x1.5555555555555p-3));
    const double taylor = gm_fma(xx0, fma(p, a, -(0.5 * da)), da) + a;
    /* table forms: do_sin negates da for a <= 0, do_cos for a < 0 (same lanes: a == 0 takes
     * the Taylor form in do_sin) */
    const double dx = a < 0 ? -da : da;
    const double u = aa + vm_k(GM_BIG);
    uint32_t k = gm_lo(u) << 2;
    k = k < 436u ? k : 436u;   /* lanes outside the table forms (Taylor, |a| >= 0.855, NaN) */
    const double r = aa - (u - vm_k(GM_BIG));
    const double x = cosine ? r + dx : r;
    const double xx = x * x;
    const double ps = gm_fma(vm_k(0x1.11110e829872fp-7), xx, vm_k(-0x1.5555555555515p-3));
    double pc = gm_fma(vm_k(0x1.6c16bedd9e239p-10), xx, vm_k(-0x1.5555555555535p-5));
    pc = gm_fma(pc, xx, 0.5);
    const double c2 = xx * pc;
    const double sn = GM_SINCOSTAB[k], ssn = GM_SINCOSTAB[k + 1];
    const double cs = GM_SINCOSTAB[k + 2], ccs = GM_SINCOSTAB[k + 3];
    double res;
    if (cosine) {
        const double s = gm_fma(x * xx, ps, x);
        const double cor = gm_fnma(s, sn, gm_fnma(c2, cs, gm_fnma(s, ssn, ccs)));
        res = cs + cor;
    } else {
        const double s = x + gm_fma(x * xx, ps, dx);
        const double c = gm_fma(x, dx, c2);
        const double cor = gm_fma(s, cs, gm_fnma(c, sn, gm_fma(s, ccs, ssn)));
        res = vm_copysign(sn + cor, a);
        if (aa < 0.126) res = taylor;
    }
    return res;
}

/* the operands s_sin.c's __sin (cosine = 0) or __cos (cosine = 1) hands to do_sin / do_cos for x,
 * and what it does with the result: *flip negates it; *direct = 1 / 2 returns x / 1.0 instead
 * (tiny |x|), 3 returns NaN (inf, NaN, and |x| >= 105414350 where glibc uses __branred) */
VM_QUAL void gm_sincos_prep(double x, int cosine, double* a, double* da, int* use_cos, int* flip, int* direct)
{
    const uint32_t k = (uint32_t)gm_hi(x) & 0x7fffffffu;
    const double ax = vm_fabs(x);
    /* reduce_sincos: x - n pi/2 as a + da, n = round(x 2/pi) */
    const double t = gm_fma(x, vm_k(0x1.45f306dc9c883p-1), vm_k(0x1.8p52));
    const double xn = t - vm_k(0x1.8p52);
    const int n = (int)(gm_lo(t) & 3u);
    const double y = gm_fnma(xn, vm_k(-0x1.dde973c000000p-27), gm_fnma(xn, vm_k(0x1.921fb58000000p+0), x));
    const double t2 = gm_fnma(xn, vm_k(-0x1.cb3b398000000p-55), y);
    double db = gm_fnma(vm_k(-0x1.cb3b398000000p-55), xn, y - t2);
    const double b = gm_fnma(xn, vm_k(-0x1.d747f23e32ed7p-83), t2);
    db = db + gm_fnma(xn, vm_k(-0x1.d747f23e32ed7p-83), t2 - b);
    /* 0.855469 <= |x| < 2.426265: pi/2 - |x| */
    const double h = vm_k(GM_HP0) - ax;
    const double hs = h + vm_k(GM_HP1);
    const int nn = n + cosine;
    *direct = 0;
    if (k < 0x3feb6000u) {              /* |x| < 0.855469: do_sin(x, 0) / do_cos(x, 0) */
        *a = x;
        *da = 0.0;
        *use_cos = cosine;
        *flip = 0;
    } else if (k < 0x400368fdu) {       /* sin: copysign(do_cos(hp0 - |x|, hp1), x);
                                           cos: do_sin(hp0 - |x| + hp1, ...) */
        if (cosine) {
            *a = hs;
            *da = (h - hs) + vm_k(GM_HP1);
        } else {
            *a = h;
            *da = vm_k(GM_HP1);
        }
        *use_cos = !cosine;
        *flip = !cosine && x < 0;
    } else {                            /* reduce_sincos + do_sincos(a, da, n (+1 for cos)) */
        *a = b;
        *da = db;
        *use_cos = nn & 1;
        *flip = (nn & 2) != 0;
    }
    if (k < (cosine ? 0x3e400000u : 0x3e500000u)) *direct = cosine ? 2 : 1;
    if (k >= 0x419921fbu) *direct = 3;
}

VM_QUAL double gm_sincos_finish(double x, double v, int flip, int direct)
{
    v = flip ? -v : v;
    if (direct == 1) v = x;
    if (direct == 2) v = 1.0;
    if (direct == 3) v = x - x + __builtin_nan("");
    return v;
}

VM_QUAL double gm_sin(double x)
{
    double a, da;
    int c, f, d;
    gm_sincos_prep(x, 0, &a, &da, &c, &f, &d);
    return gm_sincos_finish(x, gm_sincos_eval(a, da, c), f, d);
}

VM_QUAL double gm_cos(double x)
{
    double a, da;
    int c, f, d;
    gm_sincos_prep(x, 1, &a, &da, &c, &f, &d);
    return gm_sincos_finish(x, gm_sincos_eval(a, da, c), f, d);
}

VM_QUAL void gm_sincos(double x, double* s, double* c)
{
    *s = gm_sin(x);
    *c = gm_cos(x);
}

/* ------------------------------------------------------------------ acos (e_asin.c) */
/* __ieee754_acos.  For 0.125 <= |x| < 0.96875 glibc splits [0.125, 1) into intervals
 * (32 + 64 of width 2^-8 / 2^-7 below 0.5, then 2^-6 ... ) and evaluates, around each interval's
 * node asncs[n], a polynomial whose degree grows towards 1 (6, 7, 8, 9, 10 for the five ranges);
 * here one Horner loop of the largest degree runs for every lane and a lane joins it at its own
 * degree.  |x| < 0.125 is an odd polynomial, 0.96875 <= |x| < 1 goes through sqrt((1 - |x|)/2)
 * (inroot seed, Newton steps, a Dekker split). */
VM_QUAL double gm_acos(double x)
{
    const int32_t m = gm_hi(x);
    const uint32_t k = (uint32_t)m & 0x7fffffffu;
    const double xa = m > 0 ? x : -x;
    double res;
    if (k >= 0x3fc00000u && k < 0x3fef0000u) {
        int n, d;
        if (k < 0x3fd00000u) { n = 11 * (int)((k >> 15) & 0x1f); d = 6; }
        else if (k < 0x3fe00000u) { n = 11 * (int)((k >> 14) & 0x3f) + 352; d = 6; }
        else if (k < 0x3fe80000u) { n = 12 * (int)((k >> 13) & 0x7f) + 1056; d = 7; }
        else if (k < 0x3fed8000u) { n = 13 * (int)((k >> 13) & 0x7f) + 992; d = 8; }
        else if (k < 0x3fee8000u) { n = 14 * (int)((k >> 13) & 0x7f) + 884; d = 9; }
        else { n = 15 * (int)((k >> 13) & 0x7f) + 768; d = 10; }
        const double* T = GM_ASNCS + n;
        const double xx = xa - T[0];
        double p = T[d];
#pragma unroll
        for (int j = 9; j >= 2; --j)
            if (j < d) p = gm_fma(p, xx, T[j]);
        p = gm_fma(p, xx * xx, T[d + 1]);
        const double t = gm_fma(xx, T[1], p);
        const double y = T[d + 2];
        res = m > 0 ? (vm_k(GM_HP1) - t) + (vm_k(GM_HP0) - y) : (t + vm_k(GM_HP1)) + (y + vm_k(GM_HP0));
    } else if (k < 0x3fc00000u) {
        /* |x| < 0.125 (and hp0 for |x| < 2^-55) */
        const double x2 = x * x;
        double p = gm_fma(vm_k(0x1.292d80f453c72p-6), x2, vm_k(0x1.6e442c822d419p-6));
        p = gm_fma(p, x2, vm_k(0x1.f1c7e04f4ad99p-6));
        p = gm_fma(p, x2, vm_k(0x1.6db6dae42c0e4p-5));
        p = gm_fma(p, x2, vm_k(0x1.333333336127dp-4));
        p = gm_fma(p, x2, vm_k(0x1.55555555554f9p-3));
        const double r = vm_k(GM_HP0) - x;
        const double c = (((vm_k(GM_HP0) - r) - x) + vm_k(GM_HP1));
        res = r + gm_fnma(p, x * x2, c);
        if (k < 0x3c880000u) res = vm_k(GM_HP0);
    } else if (k < 0x3ff00000u) {
        /* 0.96875 <= |x| < 1: acos = 2 asin(sqrt(z)) or pi - that, z = (1 - |x|)/2 */
        const double z = (m > 0 ? 1.0 - x : x + 1.0) * 0.5;
        const uint64_t zb = vm_as_u64(z);
        const double two = vm_as_f64((uint64_t)(511 - (int)(zb >> 53) + 1023) << 52);  /* powtwo[] */
        double t = GM_INROOT[(zb >> 46) & 0x7f] * two;
        const double r = gm_fnma(t * t, z, 1.0);
        double q = gm_fma(vm_k(0x1.4006318d1dab9p-2), r, vm_k(0x1.800496769c91ap-2));
        q = gm_fma(q, r, vm_k(0x1.fffffff757304p-2));
        q = gm_fma(q, r, vm_k(0x1.fffffffecc1ddp-1));
        t = q * t;
        const double c = z * t;
        const double h = gm_fnma(t * 0.5, c, 1.5);
        const double y = gm_fnma(vm_k(0x1p27), c, gm_fma(c, vm_k(0x1p27), c));
        const double cc = gm_fnma(y, y, z) / gm_fma(h, c, y);
        double p = gm_fma(vm_k(0x1.292d80f453c72p-6), z, vm_k(0x1.6e442c822d419p-6));
        p = gm_fma(p, z, vm_k(0x1.f1c7e04f4ad99p-6));
        p = gm_fma(p, z, vm_k(0x1.6db6dae42c0e4p-5));
        p = gm_fma(p, z, vm_k(0x1.333333336127dp-4));
        p = gm_fma(p, z, vm_k(0x1.55555555554f9p-3));
        const double pr = (p * z) * (y + cc);
        const double s = m >= 0 ? (cc + pr) + y : ((vm_k(GM_HP1) - cc) - pr) + (vm_k(GM_HP0) - y);
        res = s + s;
    } else if (k == 0x3ff00000u && gm_lo(x) == 0) {
        res = m > 0 ? 0.0 : vm_k(0x1.921fb54442d18p+1);
    } else {
        res = x - x + __builtin_nan("");   /* |x| > 1, NaN */
    }
    return res;
}

/* Out-of-line entry points for the kernel.  The tracer's direction samplers call acos and four
 * sin/cos at ~10 sites per stage; inlined, each site carries its own copy (code size, and
 * registers held across the expansion).  On the device these are real calls (VPT_GM_CALL=1),
 * returning their results in registers. */
#ifndef VPT_GM_CALL
#define VPT_GM_CALL 1
#endif
#if defined(__HIP_DEVICE_COMPILE__) && VPT_GM_CALL
#define GM_CALLQ __host__ __device__ static __attribute__((noinline))
#else
#define GM_CALLQ VM_QUAL
#endif

typedef struct {
    double s0, c0, s1, c1;
} gm_sc2;

VM_QUAL gm_sc2 gm_sincos2_inl(double x0, double x1)
{
    gm_sc2 r;
    r.s0 = gm_sin(x0);
    r.c0 = gm_cos(x0);
    r.s1 = gm_sin(x1);
    r.c1 = gm_cos(x1);
    return r;
}

/* sin and cos of x0 and of x1 */
GM_CALLQ gm_sc2 gm_sincos2(double x0, double x1) { return gm_sincos2_inl(x0, x1); }

/* sin(acos c), cos(acos c), sin(phi), cos(phi): the five calls of the reference's direction
 * samplers (include/samplingFunctions.h:47-82, include/vptSamplingFunctions.h:34-47) */
GM_CALLQ gm_sc2 gm_sincos_acos_phi(double c, double phi) { return gm_sincos2_inl(gm_acos(c), phi); }

/* sin(x), cos(x) */
GM_CALLQ gm_sc2 gm_sincos1(double x)
{
    gm_sc2 r;
    r.s0 = gm_sin(x);
    r.c0 = gm_cos(x);
    r.s1 = r.c1 = 0.0;
    return r;
}

#endif /* VPT_GLIBM_H */
