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
 * Needs VM_QUAL, VM_TABLE / vm_tab / VM_T / VM_HORNER_T, vm_as_u64/vm_as_f64, vm_fabs, vm_copysign
 * (vpt_math.h).
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
/* s_sin.c's constants (usncs.h, s_sin.c), read through vm_tab: on the device a few merged scalar
 * loads instead of two scalar moves per use */
VM_TABLE(gm_sc_tab, {
    -0x1.addffc2fcdf59p-26, 0x1.71de27b9a7ed9p-19, -0x1.a01a019db08b8p-13, 0x1.1111111110ecep-7,
    -0x1.5555555555555p-3,                               /* 0-4 s5 .. s1 (TAYLOR_SIN) */
    0x1.11110e829872fp-7, -0x1.5555555555515p-3,         /* 5-6 sn5, sn3 */
    0x1.6c16bedd9e239p-10, -0x1.5555555555535p-5,        /* 7-8 cs6, cs4 (cs2 = 0.5) */
    0x1.8p+45,                                           /* 9 big: rounds |x| to k/128 */
    0x1.45f306dc9c883p-1, 0x1.8p52,                      /* 10-11 hpinv, toint */
    0x1.921fb58000000p+0, -0x1.dde973c000000p-27,        /* 12-13 mp1, mp2 */
    -0x1.cb3b398000000p-55, -0x1.d747f23e32ed7p-83,      /* 14-15 pp3, pp4 */
    0x1.921fb54442d18p+0, 0x1.1a62633145c07p-54,         /* 16-17 hp0, hp1: pi/2 */
    0.126})                                              /* 18 */
enum { GS_S5 = 0, GS_SN5 = 5, GS_SN3, GS_CS6, GS_CS4, GS_BIG, GS_HPINV, GS_TOINT, GS_MP1, GS_MP2, GS_PP3, GS_PP4,
       GS_HP0, GS_HP1, GS_TAYLOR };

/* do_sin / do_cos / TAYLOR_SIN of s_sin.c, one evaluation for either, without branches.  (a, da)
 * is the reduced argument and its correction; cosine selects do_cos.  do_sin takes the Taylor form
 * when |a| < 0.126, otherwise both read sin(k/128), its tail, cos(k/128), its tail from
 * __sincostab (k = round(128 |a|)) and add a short polynomial in the remainder. */
VM_QUAL double gm_sc_eval(vm_ct* K, double a, double da, int cosine)
{
    const double aa = vm_fabs(a);
    /* table forms: do_sin negates da for a <= 0, do_cos for a < 0 (same lanes: a == 0 takes
     * the Taylor form in do_sin) */
    const double dx = a < 0 ? -da : da;
    const double u = aa + VM_T(K, GS_BIG);
    uint32_t k = gm_lo(u) << 2;
    k = k < 436u ? k : 436u;   /* lanes outside the table forms (Taylor, |a| >= 0.855, NaN) */
    const double r = aa - (u - VM_T(K, GS_BIG));
    const double x = cosine ? r + dx : r;
    const double xx = x * x;
    const double ps = gm_fma(VM_T(K, GS_SN5), xx, VM_T(K, GS_SN3));
    double pc = gm_fma(VM_T(K, GS_CS6), xx, VM_T(K, GS_CS4));
    pc = gm_fma(pc, xx, 0.5);
    const double c2 = xx * pc;
    const double sn = GM_SINCOSTAB[k], ssn = GM_SINCOSTAB[k + 1];
    const double cs = GM_SINCOSTAB[k + 2], ccs = GM_SINCOSTAB[k + 3];
    const double q = x * xx;
    /* do_cos: s = x + x xx P, cor = ((ccs - s ssn) - cs c) - sn s, result cs + cor */
    const double s_c = gm_fma(q, ps, x);
    const double r_c = cs + gm_fnma(s_c, sn, gm_fnma(c2, cs, gm_fnma(s_c, ssn, ccs)));
    /* do_sin: s = x + (dx + x xx P), c = x dx + xx C, cor = (ssn + s ccs - sn c) + cs s,
     * result copysign(sn + cor, a) */
    const double s_s = x + gm_fma(q, ps, dx);
    const double c_s = gm_fma(x, dx, c2);
    const double r_s = vm_copysign(sn + gm_fma(s_s, cs, gm_fnma(c_s, sn, gm_fma(s_s, ccs, ssn))), a);
    /* TAYLOR_SIN(xx, a, da) */
    const double xx0 = a * a;
    double p = gm_fma(VM_T(K, GS_S5), xx0, VM_T(K, GS_S5 + 1));
    p = gm_fma(p, xx0, VM_T(K, GS_S5 + 2));
    p = gm_fma(p, xx0, VM_T(K, GS_S5 + 3));
    p = gm_fma(p, xx0, VM_T(K, GS_S5 + 4));
    const double r_t = gm_fma(xx0, fma(p, a, -(0.5 * da)), da) + a;
    return cosine ? r_c : (aa < VM_T(K, GS_TAYLOR) ? r_t : r_s);
}

/* s_sin.c's __sin (cosine = 0) or __cos (cosine = 1) of x: the operands it hands to do_sin /
 * do_cos for x's range, the evaluation, and what it does with the result (negation; x or 1.0 for
 * tiny |x|; NaN for inf, NaN and |x| >= 105414350, where glibc uses __branred) -- all as selects */
VM_QUAL double gm_sc(vm_ct* K, double x, int cosine)
{
    const uint32_t k = (uint32_t)gm_hi(x) & 0x7fffffffu;
    const double ax = vm_fabs(x);
    /* reduce_sincos: x - n pi/2 as b + db, n = round(x 2/pi) */
    const double t = gm_fma(x, VM_T(K, GS_HPINV), VM_T(K, GS_TOINT));
    const double xn = t - VM_T(K, GS_TOINT);
    const int nn = (int)(gm_lo(t) & 3u) + cosine;
    const double y = gm_fnma(xn, VM_T(K, GS_MP2), gm_fnma(xn, VM_T(K, GS_MP1), x));
    const double t2 = gm_fnma(xn, VM_T(K, GS_PP3), y);
    double db = gm_fnma(VM_T(K, GS_PP3), xn, y - t2);
    const double b = gm_fnma(xn, VM_T(K, GS_PP4), t2);
    db = db + gm_fnma(xn, VM_T(K, GS_PP4), t2 - b);
    /* 0.855469 <= |x| < 2.426265 -- sin: copysign(do_cos(hp0 - |x|, hp1), x);
     * cos: do_sin(hp0 - |x| + hp1, (hp0 - |x| - that) + hp1) */
    const double hp1 = VM_T(K, GS_HP1);
    const double h = VM_T(K, GS_HP0) - ax;
    const double hs = h + hp1;
    const int r2 = k < 0x3feb6000u, r3 = k < 0x400368fdu;
    const double a = r2 ? x : r3 ? (cosine ? hs : h) : b;
    const double da = r2 ? 0.0 : r3 ? (cosine ? (h - hs) + hp1 : hp1) : db;
    const int use_cos = r2 ? cosine : r3 ? !cosine : (nn & 1);
    const int flip = r2 ? 0 : r3 ? (!cosine && x < 0) : (nn & 2) != 0;
    double v = gm_sc_eval(K, a, da, use_cos);
    v = flip ? -v : v;
    v = k < (cosine ? 0x3e400000u : 0x3e500000u) ? (cosine ? 1.0 : x) : v;
    return k >= 0x419921fbu ? x - x + __builtin_nan("") : v;
}

VM_QUAL double gm_sin(double x) { return gm_sc(vm_tab(gm_sc_tab), x, 0); }
VM_QUAL double gm_cos(double x) { return gm_sc(vm_tab(gm_sc_tab), x, 1); }

/* ------------------------------------------------------------------ acos (e_asin.c) */
/* __ieee754_acos.  For 0.125 <= |x| < 0.96875 glibc splits [0.125, 1) into intervals
 * (32 + 64 of width 2^-8 / 2^-7 below 0.5, then 2^-6 ... ) and evaluates, around each interval's
 * node asncs[n], a polynomial whose degree grows towards 1 (6, 7, 8, 9, 10 for the five ranges);
 * here one Horner loop of the largest degree runs for every lane and a lane joins it at its own
 * degree.  |x| < 0.125 is an odd polynomial, 0.96875 <= |x| < 1 goes through sqrt((1 - |x|)/2)
 * (inroot seed, Newton steps, a Dekker split). */
VM_TABLE(gm_acos_tab, {
    0x1.292d80f453c72p-6, 0x1.6e442c822d419p-6, 0x1.f1c7e04f4ad99p-6, 0x1.6db6dae42c0e4p-5,
    0x1.333333336127dp-4, 0x1.55555555554f9p-3,          /* 0-5 f6 .. f1 (asin odd polynomial) */
    0x1.4006318d1dab9p-2, 0x1.800496769c91ap-2, 0x1.fffffff757304p-2, 0x1.fffffffecc1ddp-1,  /* 6-9 rt3..rt0 */
    0x1p27,                                              /* 10 t27 (Dekker split) */
    0x1.921fb54442d18p+0, 0x1.1a62633145c07p-54, 0x1.921fb54442d18p+1})  /* 11-13 hp0, hp1, pi */
enum { GA_F6 = 0, GA_RT3 = 6, GA_T27 = 10, GA_HP0, GA_HP1, GA_PI };

VM_QUAL double gm_acos(double x)
{
    vm_ct* K = vm_tab(gm_acos_tab);
    const int32_t m = gm_hi(x);
    const uint32_t k = (uint32_t)m & 0x7fffffffu;
    const double xa = m > 0 ? x : -x;
    double res;
    if (k >= 0x3fc00000u && k < 0x3fef0000u) {
        /* interval i of width 2^-8 / 2^-7 / 2^-6 ..., node table of d + 5 doubles per interval */
        const int d = k < 0x3fe00000u ? 6 : k < 0x3fe80000u ? 7 : k < 0x3fed8000u ? 8 : k < 0x3fee8000u ? 9 : 10;
        const int i = (int)(k < 0x3fd00000u ? (k >> 15) & 0x1f : k < 0x3fe00000u ? (k >> 14) & 0x3f : (k >> 13) & 0x7f);
        const int base = k < 0x3fd00000u ? 0 : k < 0x3fe00000u ? 352 : d == 7 ? 1056 : d == 8 ? 992 : d == 9 ? 884 : 768;
        const int n = (d + 5) * i + base;
        const double* T = GM_ASNCS + n;
        const double xx = xa - T[0];
        double p = T[d];
#pragma unroll
        for (int j = 9; j >= 2; --j)
            if (j < d) p = gm_fma(p, xx, T[j]);
        p = gm_fma(p, xx * xx, T[d + 1]);
        const double t = gm_fma(xx, T[1], p);
        const double y = T[d + 2];
        res = m > 0 ? (VM_T(K, GA_HP1) - t) + (VM_T(K, GA_HP0) - y) : (t + VM_T(K, GA_HP1)) + (y + VM_T(K, GA_HP0));
    } else if (k >= 0x3fef0000u && k < 0x3ff00000u) {
        /* 0.96875 <= |x| < 1: acos = 2 asin(sqrt(z)) or pi - that, z = (1 - |x|)/2 */
        const double z = (m > 0 ? 1.0 - x : x + 1.0) * 0.5;
        const uint64_t zb = vm_as_u64(z);
        const double two = vm_as_f64((uint64_t)(511 - (int)(zb >> 53) + 1023) << 52);  /* powtwo[] */
        double t = GM_INROOT[(zb >> 46) & 0x7f] * two;
        const double r = gm_fnma(t * t, z, 1.0);
        double q;
        VM_HORNER_T(q, K + GA_RT3, 4, r);
        t = q * t;
        const double c = z * t;
        const double h = gm_fnma(t * 0.5, c, 1.5);
        const double t27 = VM_T(K, GA_T27);
        const double y = gm_fnma(t27, c, gm_fma(c, t27, c));
        const double cc = gm_fnma(y, y, z) / gm_fma(h, c, y);
        double p;
        VM_HORNER_T(p, K + GA_F6, 6, z);
        const double pr = (p * z) * (y + cc);
        const double s = m >= 0 ? (cc + pr) + y : ((VM_T(K, GA_HP1) - cc) - pr) + (VM_T(K, GA_HP0) - y);
        res = s + s;
    } else {
        /* |x| < 0.125 (and hp0 for |x| < 2^-55); |x| = 1; |x| > 1 and NaN */
        const double x2 = x * x;
        double p;
        VM_HORNER_T(p, K + GA_F6, 6, x2);
        const double hp0 = VM_T(K, GA_HP0);
        const double r = hp0 - x;
        const double c = (((hp0 - r) - x) + VM_T(K, GA_HP1));
        res = r + gm_fnma(p, x * x2, c);
        res = k < 0x3c880000u ? hp0 : res;
        if (k >= 0x3ff00000u)
            res = k == 0x3ff00000u && gm_lo(x) == 0 ? (m > 0 ? 0.0 : VM_T(K, GA_PI)) : x - x + __builtin_nan("");
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
    vm_ct* K = vm_tab(gm_sc_tab);
    gm_sc2 r;
    r.s0 = gm_sc(K, x0, 0);
    r.c0 = gm_sc(K, x0, 1);
    r.s1 = gm_sc(K, x1, 0);
    r.c1 = gm_sc(K, x1, 1);
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
    vm_ct* K = vm_tab(gm_sc_tab);
    gm_sc2 r;
    r.s0 = gm_sc(K, x, 0);
    r.c0 = gm_sc(K, x, 1);
    r.s1 = r.c1 = 0.0;
    return r;
}

#endif /* VPT_GLIBM_H */
