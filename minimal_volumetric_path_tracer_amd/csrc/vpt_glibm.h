/*
 * vpt_glibm.h -- the reference's transcendentals, bit for bit, on the GPU.
 *
 * Restates algorithms of the GNU C Library (glibc 2.35, sysdeps/ieee754/dbl-64): LGPL-2.1-or-later,
 * see LICENSE-glibc-derived.md (how libvpt.so is rebuilt from these sources).
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

/* the rare arguments' branches (the translated library functions) marked unlikely, so that the
 * register allocator and the block layout serve the common path */
#define GM_UNLIKELY(c) __builtin_expect(!!(c), 0)

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

/* sin(x) and cos(x) together: exactly gm_sc(K, x, 0) and gm_sc(K, x, 1), with the work they share
 * done once.  For every argument range glibc's __sin and __cos call, between them, ONE do_sin (or
 * TAYLOR_SIN) and ONE do_cos:
 *     |x| < 0.855469        sin = do_sin(x, 0)          cos = do_cos(x, 0)
 *     |x| < 2.426265        sin = +-do_cos(h, hp1)      cos = do_sin(hs, (h - hs) + hp1)
 *     otherwise, n = x 2/pi sin and cos = +-do_sin(b, db) and +-do_cos(b, db), by the parity of n
 * (h = hp0 - |x|, hs = h + hp1; b + db = x - n pi/2, reduced once).  So the reduction runs once,
 * one do_sin/Taylor and one do_cos are evaluated (gm_sc evaluates all three forms per call), and
 * in the first and last ranges both read the same __sincostab entries (k = round(128 |a|)); in the
 * middle range the two indices differ only when 128 |h| is within an ulp of a half-integer.  Both
 * entry sets are read unconditionally (same cache lines; re-reading them only when some lane of
 * the wave needed it, behind a ballot, was 21 % slower on the pool kernel: A/B 58.6 vs 70.9 ms).
 * FF 1024^2 x 256: 61.9 ms with two gm_sc calls -> 58.6 ms. */
VM_QUAL void gm_sincos_fused_r(vm_ct* K, double x, double* sn_out, double* cs_out, const int small, const int taylor)
{
    /* small: every lane of the wave has |x| < 0.855469 (glibc's first range: no reduction, no swap);
     * taylor: and |x| < 0.126 (sin by TAYLOR_SIN, the do_sin table form unused).  Constant arguments
     * at the call sites below, so each specialisation drops the work the range makes dead. */
    const uint32_t kx = (uint32_t)gm_hi(x) & 0x7fffffffu;
    const double ax = vm_fabs(x);
    /* reduce_sincos, as in gm_sc */
    const double t = gm_fma(x, VM_T(K, GS_HPINV), VM_T(K, GS_TOINT));
    const double xn = t - VM_T(K, GS_TOINT);
    const int n0 = (int)(gm_lo(t) & 3u);
    const double y = gm_fnma(xn, VM_T(K, GS_MP2), gm_fnma(xn, VM_T(K, GS_MP1), x));
    const double t2 = gm_fnma(xn, VM_T(K, GS_PP3), y);
    double db = gm_fnma(VM_T(K, GS_PP3), xn, y - t2);
    const double b = gm_fnma(xn, VM_T(K, GS_PP4), t2);
    db = db + gm_fnma(xn, VM_T(K, GS_PP4), t2 - b);
    const double hp1 = VM_T(K, GS_HP1);
    const double h = VM_T(K, GS_HP0) - ax;
    const double hs = h + hp1;
    const int r2 = small ? 1 : kx < 0x3feb6000u, r3 = kx < 0x400368fdu;
    /* operands of the do_sin/Taylor evaluation (S) and of the do_cos evaluation (C) */
    const double aS = r2 ? x : r3 ? hs : b;
    const double daS = r2 ? 0.0 : r3 ? (h - hs) + hp1 : db;
    const double aC = r2 ? x : r3 ? h : b;
    const double daC = r2 ? 0.0 : r3 ? hp1 : db;
    /* S: do_sin(aS, daS), or TAYLOR_SIN for |aS| < 0.126 */
    const double aaS = vm_fabs(aS);
    const double dxS = aS < 0 ? -daS : daS;
    const double uS = aaS + VM_T(K, GS_BIG);
    uint32_t kS = gm_lo(uS) << 2;
    kS = kS < 436u ? kS : 436u;
    const double xS = aaS - (uS - VM_T(K, GS_BIG));
    /* C: do_cos(aC, daC) */
    const double aaC = vm_fabs(aC);
    const double dxC = aC < 0 ? -daC : daC;
    const double uC = aaC + VM_T(K, GS_BIG);
    uint32_t kC = gm_lo(uC) << 2;
    kC = kC < 436u ? kC : 436u;
    const double xC = (aaC - (uC - VM_T(K, GS_BIG))) + dxC;
    const double snS = GM_SINCOSTAB[kS], ssnS = GM_SINCOSTAB[kS + 1];
    const double csS = GM_SINCOSTAB[kS + 2], ccsS = GM_SINCOSTAB[kS + 3];
    const double snC = GM_SINCOSTAB[kC], ssnC = GM_SINCOSTAB[kC + 1];
    const double csC = GM_SINCOSTAB[kC + 2], ccsC = GM_SINCOSTAB[kC + 3];
    /* do_sin: s = x + (dx + x xx P), c = x dx + xx C, copysign(sn + cor, a) */
    const double xxS = xS * xS;
    const double psS = gm_fma(VM_T(K, GS_SN5), xxS, VM_T(K, GS_SN3));
    double pcS = gm_fma(VM_T(K, GS_CS6), xxS, VM_T(K, GS_CS4));
    pcS = gm_fma(pcS, xxS, 0.5);
    const double s_s = xS + gm_fma(xS * xxS, psS, dxS);
    const double c_s = gm_fma(xS, dxS, xxS * pcS);
    const double vS = vm_copysign(snS + gm_fma(s_s, csS, gm_fnma(c_s, snS, gm_fma(s_s, ccsS, ssnS))), aS);
    /* TAYLOR_SIN(aS^2, aS, daS) */
    const double xx0 = aS * aS;
    double p = gm_fma(VM_T(K, GS_S5), xx0, VM_T(K, GS_S5 + 1));
    p = gm_fma(p, xx0, VM_T(K, GS_S5 + 2));
    p = gm_fma(p, xx0, VM_T(K, GS_S5 + 3));
    p = gm_fma(p, xx0, VM_T(K, GS_S5 + 4));
    const double vT = gm_fma(xx0, fma(p, aS, -(0.5 * daS)), daS) + aS;
    const double vSin = (taylor || aaS < VM_T(K, GS_TAYLOR)) ? vT : vS;
    /* do_cos: s = x + x xx P, cs + (((ccs - s ssn) - cs c) - sn s) */
    const double xxC = xC * xC;
    const double psC = gm_fma(VM_T(K, GS_SN5), xxC, VM_T(K, GS_SN3));
    double pcC = gm_fma(VM_T(K, GS_CS6), xxC, VM_T(K, GS_CS4));
    pcC = gm_fma(pcC, xxC, 0.5);
    const double s_c = gm_fma(xC * xxC, psC, xC);
    const double vCos = csC + gm_fnma(s_c, snC, gm_fnma(xxC * pcC, csC, gm_fnma(s_c, ssnC, ccsC)));
    /* which evaluation is whose, and the signs */
    const int odd = n0 & 1;
    double s = (r2 || (!r3 && !odd)) ? vSin : vCos;
    double c = (r2 || (!r3 && !odd)) ? vCos : vSin;
    const int sflip = r2 ? 0 : r3 ? (x < 0) : (n0 & 2) != 0;
    const int cflip = (r2 || r3) ? 0 : ((n0 + 1) & 2) != 0;
    s = sflip ? -s : s;
    c = cflip ? -c : c;
    s = kx < 0x3e500000u ? x : s;
    c = kx < 0x3e400000u ? 1.0 : c;
    const double nan = x - x + __builtin_nan("");
    *sn_out = (!small && kx >= 0x419921fbu) ? nan : s;
    *cs_out = (!small && kx >= 0x419921fbu) ? nan : c;
}

/* gm_sincos_fused_r for any x */
VM_QUAL void gm_sincos_fused(vm_ct* K, double x, double* sn_out, double* cs_out)
{
    gm_sincos_fused_r(K, x, sn_out, cs_out, 0, 0);
}

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

/* gm_acos outside glibc's table range (|x| < 0.125, |x| >= 0.96875, NaN): straight-line, every
 * such argument (the cone samplers' cosines are all > 0.9925) */
VM_QUAL double gm_acos_bc(double x);

VM_QUAL double gm_acos(double x)
{
    vm_ct* K = vm_tab(gm_acos_tab);
    const double HP0 = VM_T(K, GA_HP0), HP1 = VM_T(K, GA_HP1);
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
        res = m > 0 ? (HP1 - t) + (HP0 - y) : (t + HP1) + (y + HP0);
    } else {
        res = gm_acos_bc(x);
    }
    return res;
}

VM_QUAL double gm_acos_bc(double x)
{
    vm_ct* K = vm_tab(gm_acos_tab);
    const double HP0 = VM_T(K, GA_HP0), HP1 = VM_T(K, GA_HP1);
    const int32_t m = gm_hi(x);
    const uint32_t k = (uint32_t)m & 0x7fffffffu;
    double res;
    {
        /* 0.96875 <= |x| < 1 (B): acos = 2 asin(sqrt(z)) or pi - that, z = (1 - |x|)/2;
         * |x| < 0.125 (C; hp0 for |x| < 2^-55); |x| = 1; |x| > 1 and NaN.  B and C evaluate the same
         * odd asin polynomial (in z, in x^2): one path, one Horner loop, the result selected (a
         * wave of the cosine-hemisphere or isotropic samplers usually holds lanes of both) */
        const int isB = k >= 0x3fef0000u && k < 0x3ff00000u;
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
        const double x2 = x * x;
        double p;
        const double zp = isB ? z : x2;
        VM_HORNER_T(p, K + GA_F6, 6, zp);
        const double pr = (p * z) * (y + cc);
        const double s = m >= 0 ? (cc + pr) + y : ((HP1 - cc) - pr) + (HP0 - y);
        const double rc = HP0 - x;
        const double c0 = (((HP0 - rc) - x) + HP1);
        double resC = rc + gm_fnma(p, x * x2, c0);
        resC = k < 0x3c880000u ? HP0 : resC;
        const double pi = VM_T(K, GA_PI);
        resC = k >= 0x3ff00000u ? (k == 0x3ff00000u && gm_lo(x) == 0 ? (m > 0 ? 0.0 : pi)
                                                                      : x - x + __builtin_nan(""))
                                : resC;
        res = isB ? s + s : resC;
    }
    return res;
}

/* gm_acos_bc for x in (0.9925, 1] only -- the cone samplers' cosines (every lane of the wave, checked by
 * the caller): glibc's range B (0.96875 <= x < 1: 2 asin(sqrt((1 - x)/2))) and x == 1 (+0), the same
 * operations as gm_acos_bc's B lanes without range C's evaluation and the selects between them
 * (VPT_ACOS_CONE) */
VM_QUAL double gm_acos_cone(double x)
{
    vm_ct* K = vm_tab(gm_acos_tab);
    const double z = (1.0 - x) * 0.5;
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
    const double s = (cc + pr) + y;
    return x == 1.0 ? 0.0 : s + s;
}

/* ------------------------------------------------------------------ exp / log (e_exp.c, e_log.c)
 * glibc 2.35's exp and log (the table-driven ones of sysdeps/ieee754/dbl-64, N = 128), FMA build.
 * The common paths are restated here as straight-line code reading the library's own tables (the
 * image in vpt_glibc.h: gl_tab); the rare arguments -- exp: |x| >= 512 or |x| < 2^-54, NaN, inf;
 * log: x <= 0, subnormal, inf, NaN -- go to the translated functions gl_exp / gl_log, in a branch
 * that a wave enters only when one of its lanes has such an argument.  log's two common paths (|x - 1|
 * < 0x1.09p-4, and the table path) are both evaluated and selected: log(1 - xi) of a uniform draw
 * takes the first in ~6 % of lanes, i.e. in most waves. */
VM_TABLE(gm_exp_tab, {
    0x1.71547652b82fep7, 0x1.8p52, -0x1.62e42fefa0000p-8, -0x1.cf79abc9e3b3ap-47,  /* 0-3 InvLn2N, Shift, NegLn2hiN/loN */
    0x1.ffffffffffdbdp-2, 0x1.555555555543cp-3, 0x1.55555cf172b91p-5, 0x1.1111167a4d017p-7})  /* 4-7 C2..C5 */
VM_TABLE(gm_log_tab, {
    /* 0-10 the |x - 1| < 0x1.09p-4 polynomial (B), in the order the FMA build uses them */
    -0x1.ffffffffffdcbp-3, 0x1.5555555555577p-2, 0x1.24924a344de3p-3, -0x1.55555556745a7p-3,
    -0x1.999eb43b068ffp-4, 0x1.c7184282ad6cap-4, 0x1.999999995dd0cp-3, -0x1.fffffa4423d65p-4,
    0x1.78182f7afd085p-4, -0x1.5521375d145cdp-4, 0x1p27,
    /* 11-18 the table path: Ln2hi, Ln2lo, A (in use order) */
    0x1.62e42fefa3800p-1, 0x1.ef35793c76730p-45, -0x1.fffffffeb4590p-3, 0x1.555555551305bp-2,
    -0x1.55575e506c89fp-3, 0x1.999b324f10111p-3, -0x1.0000000000001p-1})
enum { GE_INVLN2N = 0, GE_SHIFT, GE_NLN2HI, GE_NLN2LO, GE_C2, GE_C3, GE_C4, GE_C5 };
enum { GL_B0 = 0, GL_TWO27 = 10, GL_LN2HI, GL_LN2LO, GL_A0, GL_A1, GL_A2, GL_A3, GL_AH };

/* __exp_data.tab (tail, scale bits) and __log_data.tab (invc, logc), 128 pairs each, in gl_tab */
#define GM_EXP_T(i) gl_tab[(0xAF9D0ull - GL_TAB_LO) / 8 + (i)]
#define GM_LOG_T(i) gl_tab[(0xB0270ull - GL_TAB_LO) / 8 + (i)]

VM_QUAL double gm_exp(double x)
{
    vm_ct* K = vm_tab(gm_exp_tab);
    const uint32_t abstop = (uint32_t)(vm_as_u64(x) >> 52) & 0x7ffu;
    const double z = gm_fma(x, VM_T(K, GE_INVLN2N), VM_T(K, GE_SHIFT));
    const uint64_t ki = vm_as_u64(z);
    const double kd = z - VM_T(K, GE_SHIFT);
    double r = gm_fma(kd, VM_T(K, GE_NLN2HI), x);
    r = gm_fma(kd, VM_T(K, GE_NLN2LO), r);
    const uint32_t idx = 2u * (uint32_t)(ki & 0x7fu);
    const double tail = vm_as_f64(GM_EXP_T(idx));
    const uint64_t sbits = GM_EXP_T(idx + 1) + (ki << 45);
    const double r2 = r * r;
    const double p23 = gm_fma(r, VM_T(K, GE_C3), VM_T(K, GE_C2));
    const double p45 = gm_fma(r, VM_T(K, GE_C5), VM_T(K, GE_C4));
    const double tmp = gm_fma(r2 * r2, p45, gm_fma(p23, r2, r + tail));
    const double scale = vm_as_f64(sbits);
    double v = gm_fma(scale, tmp, scale);
    VM_RARE_FIX(abstop - 0x3c9u >= 0x3fu, v, gl_exp(x));
    return v;
}

VM_QUAL double gm_log(double x)
{
    vm_ct* K = vm_tab(gm_log_tab);
    const uint64_t ix = vm_as_u64(x);
    const uint32_t top = (uint32_t)(ix >> 48);
    /* |x - 1| < 0x1.09p-4: log1p-style polynomial with an exact head */
    const double r1 = x - 1.0;
    const double rr = r1 * r1;
    const double r3 = r1 * rr;
    double a = gm_fma(r1, VM_T(K, GL_B0), VM_T(K, GL_B0 + 1));
    double b = gm_fma(r1, VM_T(K, GL_B0 + 2), VM_T(K, GL_B0 + 3));
    double c = gm_fma(r1, VM_T(K, GL_B0 + 4), VM_T(K, GL_B0 + 5));
    a = gm_fma(rr, VM_T(K, GL_B0 + 6), a);
    b = gm_fma(rr, VM_T(K, GL_B0 + 7), b);
    c = gm_fma(rr, VM_T(K, GL_B0 + 8), c);
    c = gm_fma(r3, VM_T(K, GL_B0 + 9), c);
    c = gm_fma(c, r3, b);
    c = gm_fma(c, r3, a);
    const double two27 = VM_T(K, GL_TWO27);
    const double rhi = gm_fnma(two27, r1, gm_fma(r1, two27, r1));
    const double rhi2 = rhi * rhi;
    const double ah = -0.5;  /* B0 of glibc's table */
    const double hi1 = gm_fma(rhi2, ah, r1);
    double lo1 = gm_fma(rhi2, ah, r1 - hi1);
    lo1 = gm_fma(ah * (r1 - rhi), r1 + rhi, lo1);
    double v1 = hi1 + gm_fma(c, r3, lo1);
    v1 = ix == 0x3ff0000000000000ull ? 0.0 : v1;
    /* table path: x = 2^k z, z near 1/invc, log x = k ln2 + logc + log(z invc) */
    const uint64_t tmp = ix + 0xc01a000000000000ull;
    const uint32_t i = (uint32_t)(tmp >> 45) & 0x7fu;
    const int k = (int)((int64_t)tmp >> 52);
    const double zz = vm_as_f64(ix - (tmp & 0xfff0000000000000ull));
    const double kd = (double)k;
    const double invc = vm_as_f64(GM_LOG_T(2 * i)), logc = vm_as_f64(GM_LOG_T(2 * i + 1));
    const double r = gm_fma(zz, invc, -1.0);
    const double w = gm_fma(kd, VM_T(K, GL_LN2HI), logc);
    const double hi = r + w;
    const double r2 = r * r;
    double lo = gm_fma(kd, VM_T(K, GL_LN2LO), (w - hi) + r);
    lo = gm_fma(r2, VM_T(K, GL_AH), lo);
    double q = gm_fma(r, VM_T(K, GL_A2), VM_T(K, GL_A3));
    q = gm_fma(q, r2, gm_fma(r, VM_T(K, GL_A0), VM_T(K, GL_A1)));
    const double v2 = gm_fma(r * r2, q, lo) + hi;
    double v = ix + 0xc012000000000000ull <= 0x308ffffffffffull ? v1 : v2;
    VM_RARE_FIX(top - 0x0010u >= 0x7ff0u - 0x0010u, v, gl_log(x));
    return v;
}

/* ------------------------------------------------------------------ atan2 (e_atan2.c)
 * glibc 2.35's __ieee754_atan2, FMA build, for x > 0: atan(|y|/x) (|y| < x) or pi/2 - atan(x/|y|)
 * (x <= |y|) from u = min/max and its correction du, by an odd polynomial (u < 1/16) or around a
 * node of the cij table (7 doubles per node), sign of y.  The four forms are evaluated branch-free
 * and selected; |y|/x above 2^57 gives +-hpi.  Everything else -- x <= 0, y = 0, NaN, inf, |y|/x
 * below 2^-57, operands the library rescales (below 2^-500 or above 2^500) -- goes to the
 * translated gl_atan2.  The equi-angular setup (include/volumetricBasicFunctions.h:
 * 209-223) calls atan2(-proj, D) and atan2(tMax - proj, D) with D > 0. */
VM_TABLE(gm_atan2_tab, {
    0x1.375f08b31cbcep-4, -0x1.7458022b13c25p-4, 0x1.c71c6e5129a3bp-4, -0x1.24924923f7603p-3,
    0x1.99999999997fdp-3, -0x1.5555555555555p-2,          /* 0-5 d13 .. d3 */
    0x1.921fb54442d18p+0, 0x1.1a62633145c07p-54,          /* 6-7 hpi, hpi1 */
    0x1p-500, 0x1p500, 0x1p52})                           /* 8-10 */
enum { GT_D13 = 0, GT_HPI = 6, GT_HPI1, GT_TM500, GT_T500, GT_TWO52 };
#define GM_CIJ(i, j) vm_as_f64(gl_tab[(0xBE0E0ull - GL_TAB_LO) / 8 + 7 * (i) + (j)])

VM_QUAL double gm_atan2(double y, double x)
{
    vm_ct* K = vm_tab(gm_atan2_tab);
    const double ax = vm_fabs(x), ay = vm_fabs(y);
    const int de = (int)((uint32_t)gm_hi(y) & 0x7ff00000u) - (int)((uint32_t)gm_hi(x) & 0x7ff00000u);
    const int ci = ax > ay;  /* case (i): atan(ay/ax); else (ii): pi/2 - atan(ax/ay) */
    const double num = ci ? ay : ax, den = ci ? ax : ay;
    const double u = num / den;
    const double v5 = den * u;
    const double v7 = gm_fma(den, u, -v5);
    const double du = ((num - v5) - v7) / den;
    /* u < 1/16: odd polynomial in u */
    const double v = u * u;
    double p;
    VM_HORNER_T(p, K + GT_D13, 6, v);
    const double uv = u * v;
    const double hpi = VM_T(K, GT_HPI), hpi1 = VM_T(K, GT_HPI1);
    const double z_i_poly = u + gm_fma(uv, p, du);
    const double t2 = hpi - u;
    const double z_ii_poly = ((((hpi - t2) - u) + hpi1) - du) - uv * p + t2;
    /* u >= 1/16: around the node i = round(256 u) - 16 */
    int i = (int)(gm_fma(u, 256.0, VM_T(K, GT_TWO52)) - VM_T(K, GT_TWO52)) - 16;
    i = i < 0 ? 0 : i > 240 ? 240 : i;
    const double c0 = GM_CIJ(i, 0), c1 = GM_CIJ(i, 1), c2 = GM_CIJ(i, 2), c3 = GM_CIJ(i, 3);
    const double c4 = GM_CIJ(i, 4), c5 = GM_CIJ(i, 5), c6 = GM_CIJ(i, 6);
    const double t3 = u - c0;
    const double w = du + t3;  /* case (i): EADD(t3, du) */
    const double dw = vm_fabs(t3) > vm_fabs(du) ? (t3 - w) + du : (du - w) + t3;
    double q = gm_fma(w, c6, c5);
    q = gm_fma(w, q, c4);
    q = gm_fma(w, q, c3);
    const double z_i_tab = gm_fma(w, c2, gm_fma(dw, c2, (w * w) * q)) + c1;
    const double w2 = t3 + du;  /* case (ii) */
    double q2 = gm_fma(w2, c6, c5);
    q2 = gm_fma(w2, q2, c4);
    q2 = gm_fma(w2, q2, c3);
    q2 = gm_fma(w2, q2, c2);
    const double z_ii_tab = (hpi - c1) + gm_fnma(w2, q2, hpi1);
    const int small = u < 0.0625;
    const double z = ci ? (small ? z_i_poly : z_i_tab) : (small ? z_ii_poly : z_ii_tab);
    /* |y| / x above 2^57 (exponent difference; tMax = MAXFLOAT of a ray that leaves the scene):
     * atan2 = pi/2 - (less than 2^-57), whose correctly rounded value -- glibc's result there -- is
     * the double hpi (pi/2 - hpi = 6.1e-17 < half an ulp), with y's sign */
    double r = vm_copysign(de > 0x38fffff ? hpi : z, y);
    const double tm500 = VM_T(K, GT_TM500), t500 = VM_T(K, GT_T500);
    const int rare = !(x > 0.0) || !(ay > 0.0) || !(x < __builtin_inf()) || !(ay < __builtin_inf()) ||
                     de < -0x38fffff || ax < tm500 || ay < tm500 || ax > t500 || ay > t500;
    VM_RARE_FIX(rare, r, gl_atan2(y, x));
    return r;
}

/* ------------------------------------------------------------------ tan (s_tan.c)
 * glibc 2.35's __tan, FMA build, for |x| <= 25 (the equi-angular sampler's angle lies in
 * (-pi/2, pi/2), include/volumetricBasicFunctions.h:221): x itself below 0x1.b096cp-27; an odd
 * polynomial up to 0.0608; around a node of the library's table (xi, fi, gi per 1/256, gl_tab) up to
 * 0.787; above, x - n pi/2 as a + da (three pieces of pi/2) and, by the parity of n, tan or -1/tan of
 * it -- by the same polynomial (-1/tan with glibc's double-double division) or around a table node.
 * The forms are evaluated straight-line and selected (the polynomial and the table form once each,
 * on the argument of the lane's range); |x| > 25, inf and NaN go to the translated gl_tan. */
VM_TABLE(gm_tan_tab, {
    0x1.2385a3cf2e4eap-7, 0x1.664ed49cfc666p-6, 0x1.ba1ba1cdb8745p-5, 0x1.11111111107c6p-3,
    0x1.5555555555555p-2,                                /* 0-4 the odd polynomial */
    0x1.11112e0a6b45fp-3, 0x1.5555555554dbdp-2,          /* 5-6 the table form's polynomial */
    0x1.45f306dc9c883p-1, 0x1.8p+52,                     /* 7-8 2/pi, toint */
    0x1.921fb58000000p+0, -0x1.dde973c000000p-27, -0x1.cb3b399d747f2p-55,  /* 9-11 pi/2 in three pieces */
    0x1.b096cp-27, 0x1.f212dp-5, 0x1.92f1ap-1, 25.0})     /* 12-15 range bounds */
enum { GN_P0 = 0, GN_Q1 = 5, GN_Q0, GN_HPINV, GN_TOINT, GN_MP1, GN_MP2, GN_PP3, GN_TINY, GN_SMALL, GN_MID, GN_BIG };
#define GM_TAN_T(i, j) vm_as_f64(gl_tab[(0xC15C0ull - GL_TAB_LO) / 8 + 4 * (i) + (j)])

VM_QUAL double gm_tan(double x)
{
    vm_ct* K = vm_tab(gm_tan_tab);
    const double ax = vm_fabs(x);
    /* |x| in (0.787, 25]: a + da = x - n pi/2 */
    const double t = gm_fma(x, VM_T(K, GN_HPINV), VM_T(K, GN_TOINT));
    const double xn = t - VM_T(K, GN_TOINT);
    const int odd = (int)(gm_lo(t) & 1u);
    double a0 = gm_fnma(xn, VM_T(K, GN_MP1), x);
    a0 = gm_fnma(xn, VM_T(K, GN_MP2), a0);
    const double pp3 = VM_T(K, GN_PP3);
    const double a = gm_fnma(xn, pp3, a0);
    const double da = gm_fnma(xn, pp3, a0 - a);
    const int inR = ax > VM_T(K, GN_MID);
    const int neg = a < 0;
    /* the polynomial form: tan(x) = fma(x^3, P, x) below 0.0608; above, y = a + fma(a^3, P, da), and
     * for odd n -1/y with y's tail yy (glibc's EADD + DIV2) */
    const double v = inR ? a : x;
    const double v2 = v * v;
    double p = gm_fma(v2, VM_T(K, GN_P0), VM_T(K, GN_P0 + 1));
    p = gm_fma(v2, p, VM_T(K, GN_P0 + 2));
    p = gm_fma(v2, p, VM_T(K, GN_P0 + 3));
    p = gm_fma(v2, p, VM_T(K, GN_P0 + 4));
    const double v3 = v * v2;
    const double rP = gm_fma(v3, p, x);
    const double c = gm_fma(v3, p, da);
    const double y = a + c;
    const double yy = vm_fabs(a) > vm_fabs(c) ? (a - y) + c : (c - y) + a;
    const double r = 1.0 / y;
    const double h = r * y;
    const double e = gm_fma(r, y, -h);
    double w = ((1.0 - h) - e) + 0.0;
    w = gm_fnma(yy, r, w);
    const double q = w / y;
    const double s1 = r + q;
    const double rPoly = odd ? -(((r - s1) + q) + s1) : y;
    /* the table form around xi = (i + 16) / 256 -- (fi + gi) p / (gi - p) + fi, or for odd n
     * gi - (fi + gi) p / (p + fi) -- on |x| (0.0608 < |x| <= 0.787) or |a| + sign(a) da */
    const double u = inR ? (neg ? -a : a) : ax;
    const double du = inR ? (neg ? -da : da) : 0.0;
    const int todd = inR && odd;
    const double sg = (inR ? neg : x < 0) ? -1.0 : 1.0;
    const double ti = gm_fma(u, 256.0, -15.5);
    const int i = ti > 0.0 ? (ti < 186.5 ? (int)ti : 186) : 0;  /* (lanes of the other forms: any node) */
    const double z = (u - GM_TAN_T(i, 0)) + du;
    const double z2 = z * z;
    const double z3 = z * z2;
    const double pz = gm_fma(z3, gm_fma(z2, VM_T(K, GN_Q1), VM_T(K, GN_Q0)), z);
    const double fi = GM_TAN_T(i, 1), gi = GM_TAN_T(i, 2);
    const double num = (fi + gi) * pz;
    const double qt = num / (todd ? pz + fi : gi - pz);
    const double rTab = todd ? (gi - qt) * -sg : (qt + fi) * sg;
    const double small = VM_T(K, GN_SMALL);
    double res = ax <= VM_T(K, GN_TINY) ? x : ax <= small ? rP : !inR ? rTab : u <= small ? rPoly : rTab;
    VM_RARE_FIX(!(ax <= VM_T(K, GN_BIG)), res, gl_tan(x));
    return res;
}

/* Out-of-line entry points for the kernel.  The tracer's direction samplers call acos and four
 * sin/cos at ~10 sites per stage; inlined, each site carries its own copy (code size, and
 * registers held across the expansion).  On the device these are real calls, returning their
 * results in registers (inlined, round 2: FF 57.7 -> 91.9 ms, occupancy 1). */
#if defined(__HIP_DEVICE_COMPILE__)
#define GM_CALLQ __host__ __device__ static __attribute__((noinline))
#else
#define GM_CALLQ VM_QUAL
#endif

typedef struct {
    double s0, c0, s1, c1;
} gm_sc2;

/* sin and cos of one argument: one reduction (gm_sincos_fused) */
VM_QUAL void gm_sincos_k(vm_ct* K, double x, double* s, double* c) { gm_sincos_fused(K, x, s, c); }

VM_QUAL gm_sc2 gm_sincos2_inl(double x0, double x1)
{
    vm_ct* K = vm_tab(gm_sc_tab);
    gm_sc2 r;
    gm_sincos_k(K, x0, &r.s0, &r.c0);
    gm_sincos_k(K, x1, &r.s1, &r.c1);
    return r;
}

/* sin and cos of x0 and of x1 */
GM_CALLQ gm_sc2 gm_sincos2(double x0, double x1) { return gm_sincos2_inl(x0, x1); }

/* sin(acos c), cos(acos c), sin(phi), cos(phi): the five calls of the reference's direction
 * samplers (include/samplingFunctions.h:47-82, include/vptSamplingFunctions.h:34-47) */
GM_CALLQ gm_sc2 gm_sincos_acos_phi(double c, double phi)
{
    return gm_sincos2_inl(gm_acos(c), phi);
}

/* gm_sincos_acos_phi for a wave whose every c > 0.9925 (the cone toward a sphere light): acos(c) <
 * 0.1226 < 0.126 in every lane (glibc's acos is within an ulp), so sin of the polar angle is
 * TAYLOR_SIN -- the specialised evaluation, the same bits -- and cos(acos c) is c itself, without
 * evaluating it (VPT_COS_ACOS_C).  Why that is exact: for c in (0.9925, 1], theta = acos(c) < 0.1226 and
 * glibc's acos returns theta' within half an ulp of theta (|theta' - theta| <= 2^-57), so
 * |cos(theta') - c| <= sin(theta) |theta' - theta| < 2^-60, an eighth of a half-ulp of c (2^-54);
 * glibc's do_cos there (table value + double-double correction, error ~2^-68 before its final rounding)
 * therefore rounds to c.  Checked against glibc's own cos(acos(c)) on 2e8 random c in [0.9925, 1) and on
 * every one of the 2^32 doubles below 1 (scripts-free: tests/test_glibc_libm.py repeats a sample), and
 * on the device against glibc (tests/test_gpu_parity.py).  The do_cos evaluation skipped is ~15 FP64
 * operations and four dependent __sincostab reads per direction. */
#ifndef VPT_COS_ACOS_C
#define VPT_COS_ACOS_C 1
#endif
#ifndef VPT_ACOS_CONE
#define VPT_ACOS_CONE 1
#endif
GM_CALLQ gm_sc2 gm_sincos_acos_phi_cone(double c, double phi)
{
    vm_ct* K = vm_tab(gm_sc_tab);
    gm_sc2 r;
    gm_sincos_fused_r(K, VPT_ACOS_CONE ? gm_acos_cone(c) : gm_acos_bc(c), &r.s0, &r.c0, 1, 1);  /* c > 0.9925: range B */
    if (VPT_COS_ACOS_C) r.c0 = c;
    gm_sincos_k(K, phi, &r.s1, &r.c1);
    return r;
}

/* two cone directions at once (MISv2's two light samples, include/samplingFunctions.h:163-206): the
 * same evaluations as two gm_sincos_acos_phi_cone calls, straight-line, so that the two independent
 * chains (and their table reads) overlap */
typedef struct {
    gm_sc2 a, b;
} gm_sc4;
GM_CALLQ gm_sc4 gm_sincos_acos_phi_cone2(double c0, double phi0, double c1, double phi1)
{
    vm_ct* K = vm_tab(gm_sc_tab);
    gm_sc4 r;
    const double t0 = VPT_ACOS_CONE ? gm_acos_cone(c0) : gm_acos_bc(c0), t1 = VPT_ACOS_CONE ? gm_acos_cone(c1) : gm_acos_bc(c1);
    gm_sincos_fused_r(K, t0, &r.a.s0, &r.a.c0, 1, 1);
    gm_sincos_fused_r(K, t1, &r.b.s0, &r.b.c0, 1, 1);
    if (VPT_COS_ACOS_C) {  /* cos(acos c) == c for c > 0.9925 (gm_sincos_acos_phi_cone) */
        r.a.c0 = c0;
        r.b.c0 = c1;
    }
    gm_sincos_k(K, phi0, &r.a.s1, &r.a.c1);
    gm_sincos_k(K, phi1, &r.b.s1, &r.b.c1);
    return r;
}

/* sin(x), cos(x) */
GM_CALLQ gm_sc2 gm_sincos1(double x)
{
    vm_ct* K = vm_tab(gm_sc_tab);
    gm_sc2 r;
    gm_sincos_k(K, x, &r.s0, &r.c0);
    r.s1 = r.c1 = 0.0;
    return r;
}

#endif /* VPT_GLIBM_H */
