/*
 * crmath.c -- correctly rounded sin/cos (TEST INFRASTRUCTURE ONLY, see oracle.h).
 *
 * The reference evaluates sin/cos through libm: Chipmunk's cpBodySetAngle ->
 * cpvforangle (cos, sin), render.py:58-60 Transform.create_rotation_matrix
 * (math.cos/math.sin), pymunk Vec2d.rotated (math.cos/math.sin).  glibc <= 2.27
 * returned the correctly rounded result; glibc >= 2.28 is within 0.548 ulp and
 * misrounds ~0.15% of arguments (measured here).  We restate the correctly
 * rounded function: Cody-Waite reduction by pi/2 split in four doubles, then
 * Taylor series evaluated in double-double arithmetic (~104 bits), rounded once.
 */
#include <math.h>
#include "oracle.h"

typedef struct { double hi, lo; } dd;

static dd two_sum(double a, double b) {
    double s = a + b, bb = s - a;
    dd r = {s, (a - (s - bb)) + (b - bb)};
    return r;
}
static dd fast_two_sum(double a, double b) {
    double s = a + b;
    dd r = {s, b - (s - a)};
    return r;
}
static dd two_prod(double a, double b) {
    double p = a * b;
    dd r = {p, fma(a, b, -p)};
    return r;
}
static dd dd_add(dd a, dd b) {
    dd s = two_sum(a.hi, b.hi), t = two_sum(a.lo, b.lo);
    s.lo += t.hi;
    s = fast_two_sum(s.hi, s.lo);
    s.lo += t.lo;
    return fast_two_sum(s.hi, s.lo);
}
static dd dd_mul(dd a, dd b) {
    dd p = two_prod(a.hi, b.hi);
    p.lo += a.hi * b.lo + a.lo * b.hi;
    return fast_two_sum(p.hi, p.lo);
}
static dd dd_neg(dd a) { dd r = {-a.hi, -a.lo}; return r; }

/* 1/n! as double-double, n = 0..27 (exact to ~2^-107) */
static const dd INVF[28] = {
    {1.0, 0.0},
    {1.0, 0.0},
    {0.5, 0.0},
    {0.16666666666666666, 9.25185853854297e-18},
    {0.041666666666666664, 2.3129646346357427e-18},
    {0.008333333333333333, 1.1564823173178714e-19},
    {0.001388888888888889, -5.300543954373577e-20},
    {0.0001984126984126984, 1.7209558293420705e-22},
    {2.48015873015873e-05, 2.1511947866775882e-23},
    {2.7557319223985893e-06, -1.858393274046472e-22},
    {2.755731922398589e-07, 2.3767714622250297e-23},
    {2.505210838544172e-08, -1.448814070935912e-24},
    {2.08767569878681e-09, -1.20734505911326e-25},
    {1.6059043836821613e-10, 1.2585294588752098e-26},
    {1.1470745597729725e-11, 2.0655512752830745e-28},
    {7.647163731819816e-13, 7.03872877733453e-30},
    {4.779477332387385e-14, 4.399205485834081e-31},
    {2.8114572543455206e-15, 1.6508842730861433e-31},
    {1.5619206968586225e-16, 1.1910679660273754e-32},
    {8.22063524662433e-18, 2.2141894119604265e-34},
    {4.110317623312165e-19, 1.4412973378659527e-36},
    {1.9572941063391263e-20, -1.3643503830087908e-36},
    {8.896791392450574e-22, -7.911402614872376e-38},
    {3.868170170630684e-23, -8.843177655482344e-40},
    {1.6117375710961184e-24, -3.6846573564509766e-41},
    {6.446950284384474e-26, -1.9330404233703465e-42},
    {2.4795962632247976e-27, -1.2953730964765229e-43},
    {9.183689863795546e-29, 1.4303150396787322e-45},
};

/* pi/2 = P1 + P2 + P3 + P4 (each the double nearest the remainder) */
static const double P1 = 1.5707963267948966, P2 = 6.123233995736766e-17,
                    P3 = -1.4973849048591698e-33, P4 = 5.562271104316826e-50;

static void reduce(double x, int *q, dd *r) {
    double k = nearbyint(x * 0.63661977236758134308);
    dd a = two_prod(k, P1), b = two_prod(k, P2), c = two_prod(k, P3);
    dd t = two_sum(x, -a.hi);
    t = dd_add(t, (dd){-a.lo, 0.0});
    t = dd_add(t, dd_neg(b));
    t = dd_add(t, (dd){-c.hi, -c.lo - k * P4});
    *r = t;
    *q = (int)((long long)k & 3);
}

#define NTERMS 13
static dd ksin(dd r) {
    dd r2 = dd_mul(r, r);
    dd p = (NTERMS & 1) ? dd_neg(INVF[2 * NTERMS + 1]) : INVF[2 * NTERMS + 1];
    for (int n = NTERMS - 1; n >= 0; n--) {
        p = dd_mul(p, r2);
        p = dd_add(p, (n & 1) ? dd_neg(INVF[2 * n + 1]) : INVF[2 * n + 1]);
    }
    return dd_mul(p, r);
}
static dd kcos(dd r) {
    dd r2 = dd_mul(r, r);
    dd p = (NTERMS & 1) ? dd_neg(INVF[2 * NTERMS]) : INVF[2 * NTERMS];
    for (int n = NTERMS - 1; n >= 0; n--) {
        p = dd_mul(p, r2);
        p = dd_add(p, (n & 1) ? dd_neg(INVF[2 * n]) : INVF[2 * n]);
    }
    return p;
}

static double cr_sin(double x) {
    if (fabs(x) < 1.4901161193847656e-08) return x; /* |x| < 2^-26: sin x rounds to x */
    int q; dd r, v;
    reduce(x, &q, &r);
    switch (q) {
    case 0: v = ksin(r); break;
    case 1: v = kcos(r); break;
    case 2: v = dd_neg(ksin(r)); break;
    default: v = dd_neg(kcos(r)); break;
    }
    return v.hi + v.lo;
}

static double cr_cos(double x) {
    if (fabs(x) < 7.450580596923828e-09) return 1.0; /* |x| < 2^-27 */
    int q; dd r, v;
    reduce(x, &q, &r);
    switch (q) {
    case 0: v = kcos(r); break;
    case 1: v = dd_neg(ksin(r)); break;
    case 2: v = dd_neg(kcos(r)); break;
    default: v = ksin(r); break;
    }
    return v.hi + v.lo;
}

static dd dd_mul_d(dd a, double b) {
    dd p = two_prod(a.hi, b);
    p.lo += a.lo * b;
    return fast_two_sum(p.hi, p.lo);
}
static dd dd_div(dd a, dd b) {
    double q1 = a.hi / b.hi;
    dd r = dd_add(a, dd_neg(dd_mul_d(b, q1)));
    double q2 = r.hi / b.hi;
    r = dd_add(r, dd_neg(dd_mul_d(b, q2)));
    double q3 = r.hi / b.hi;
    dd q = fast_two_sum(q1, q2);
    return dd_add(q, (dd){q3, 0.0});
}

/* math.tan (geom.py:22 regular_poly_circ_rad_to_side_length): sin/cos in
 * double-double, one division, rounded once */
static double cr_tan(double x) {
    if (fabs(x) < 1.4901161193847656e-08) return x;
    int q; dd r, s, c;
    reduce(x, &q, &r);
    dd ks = ksin(r), kc = kcos(r);
    switch (q) {
    case 0: s = ks; c = kc; break;
    case 1: s = kc; c = dd_neg(ks); break;
    case 2: s = dd_neg(ks); c = dd_neg(kc); break;
    default: s = dd_neg(kc); c = ks; break;
    }
    dd t = dd_div(s, c);
    return t.hi + t.lo;
}

/* the exported functions: correctly rounded, or this image's libm in the measurement build
 * (make libm -> _build/libmg_oracle_libm.so, tools/libm_vs_cr.py) */
#ifdef ORACLE_LIBM_TRIG
double o_crsin(double x) { return sin(x); }
double o_crcos(double x) { return cos(x); }
double o_crtan(double x) { return tan(x); }
#else
double o_crsin(double x) { return cr_sin(x); }
double o_crcos(double x) { return cr_cos(x); }
double o_crtan(double x) { return cr_tan(x); }
#endif
