// mg_math.h -- device arithmetic that must reproduce the reference bit for bit.
//
// * sin/cos/tan: correctly rounded (double-double Cody-Waite + Taylor), i.e.
//   the libm results of the reference's era (glibc <= 2.27); used for body
//   transforms (Chipmunk cpBodySetAngle), render.py Transform rotations and
//   pymunk Vec2d.rotated during resets.
// * mat3: numpy float64 matmul as measured for the reference's render.py
//   (OpenBLAS dgemm): each element is fma(a2,b2, fma(a1,b1, a0*b0)).
// Everything else is plain IEEE double; the library is built with
// -ffp-contract=off so the compiler never fuses a multiply-add.
#pragma once
#include <hip/hip_runtime.h>

#define MG_DEV __device__ __forceinline__

struct dd_t { double hi, lo; };

MG_DEV dd_t dd_two_sum(double a, double b) {
    double s = a + b, bb = s - a;
    return {s, (a - (s - bb)) + (b - bb)};
}
MG_DEV dd_t dd_fast_two_sum(double a, double b) {
    double s = a + b;
    return {s, b - (s - a)};
}
MG_DEV dd_t dd_two_prod(double a, double b) {
    double p = a * b;
    return {p, __fma_rn(a, b, -p)};
}
MG_DEV dd_t dd_add(dd_t a, dd_t b) {
    dd_t s = dd_two_sum(a.hi, b.hi), t = dd_two_sum(a.lo, b.lo);
    s.lo += t.hi;
    s = dd_fast_two_sum(s.hi, s.lo);
    s.lo += t.lo;
    return dd_fast_two_sum(s.hi, s.lo);
}
MG_DEV dd_t dd_mul(dd_t a, dd_t b) {
    dd_t p = dd_two_prod(a.hi, b.hi);
    p.lo += a.hi * b.lo + a.lo * b.hi;
    return dd_fast_two_sum(p.hi, p.lo);
}
MG_DEV dd_t dd_neg(dd_t a) { return {-a.hi, -a.lo}; }

// 1/n!, n = 0..27, as double-double
__constant__ static const double MG_INVF_HI[28] = {
    1.0, 1.0, 0.5, 0.16666666666666666, 0.041666666666666664, 0.008333333333333333,
    0.001388888888888889, 0.0001984126984126984, 2.48015873015873e-05, 2.7557319223985893e-06,
    2.755731922398589e-07, 2.505210838544172e-08, 2.08767569878681e-09, 1.6059043836821613e-10,
    1.1470745597729725e-11, 7.647163731819816e-13, 4.779477332387385e-14, 2.8114572543455206e-15,
    1.5619206968586225e-16, 8.22063524662433e-18, 4.110317623312165e-19, 1.9572941063391263e-20,
    8.896791392450574e-22, 3.868170170630684e-23, 1.6117375710961184e-24, 6.446950284384474e-26,
    2.4795962632247976e-27, 9.183689863795546e-29};
__constant__ static const double MG_INVF_LO[28] = {
    0.0, 0.0, 0.0, 9.25185853854297e-18, 2.3129646346357427e-18, 1.1564823173178714e-19,
    -5.300543954373577e-20, 1.7209558293420705e-22, 2.1511947866775882e-23, -1.858393274046472e-22,
    2.3767714622250297e-23, -1.448814070935912e-24, -1.20734505911326e-25, 1.2585294588752098e-26,
    2.0655512752830745e-28, 7.03872877733453e-30, 4.399205485834081e-31, 1.6508842730861433e-31,
    1.1910679660273754e-32, 2.2141894119604265e-34, 1.4412973378659527e-36, -1.3643503830087908e-36,
    -7.911402614872376e-38, -8.843177655482344e-40, -3.6846573564509766e-41, -1.9330404233703465e-42,
    -1.2953730964765229e-43, 1.4303150396787322e-45};

MG_DEV void mg_reduce_pio2(double x, int &q, dd_t &r) {
    const double P1 = 1.5707963267948966, P2 = 6.123233995736766e-17, P3 = -1.4973849048591698e-33,
                 P4 = 5.562271104316826e-50;
    double k = rint(x * 0.63661977236758134308);
    dd_t a = dd_two_prod(k, P1), b = dd_two_prod(k, P2), c = dd_two_prod(k, P3);
    dd_t t = dd_two_sum(x, -a.hi);
    t = dd_add(t, {-a.lo, 0.0});
    t = dd_add(t, dd_neg(b));
    t = dd_add(t, {-c.hi, -c.lo - k * P4});
    r = t;
    q = (int)((long long)k & 3);
}

MG_DEV dd_t mg_ksin(dd_t r) {
    dd_t r2 = dd_mul(r, r);
    dd_t p = dd_neg({MG_INVF_HI[27], MG_INVF_LO[27]}); // (-1)^13 / 27!
#pragma unroll
    for (int n = 12; n >= 0; n--) {
        p = dd_mul(p, r2);
        dd_t c = {MG_INVF_HI[2 * n + 1], MG_INVF_LO[2 * n + 1]};
        p = dd_add(p, (n & 1) ? dd_neg(c) : c);
    }
    return dd_mul(p, r);
}
MG_DEV dd_t mg_kcos(dd_t r) {
    dd_t r2 = dd_mul(r, r);
    dd_t p = dd_neg({MG_INVF_HI[26], MG_INVF_LO[26]}); // (-1)^13 / 26!
#pragma unroll
    for (int n = 12; n >= 0; n--) {
        p = dd_mul(p, r2);
        dd_t c = {MG_INVF_HI[2 * n], MG_INVF_LO[2 * n]};
        p = dd_add(p, (n & 1) ? dd_neg(c) : c);
    }
    return p;
}

// Ziv-style fast path: sin(r), cos(r) for the reduced r = rh + rl with the leading terms in
// double-double and the tail r^7.. / r^8.. in double (absolute error < 2^-66 |result|), then a
// rounding test: the double nearest to the double-double is returned only when the exact value
// provably rounds to it; otherwise the caller falls back to the full double-double series.  Both
// paths therefore return the correctly rounded value (as the oracle does).
MG_DEV double mg_ifh(int n) { return MG_INVF_HI[n]; }
MG_DEV dd_t mg_ifd(int n) { return {MG_INVF_HI[n], MG_INVF_LO[n]}; }

MG_DEV bool mg_certify(dd_t y, double &out) {
    y = dd_fast_two_sum(y.hi, y.lo);
    const uint64_t bits = (uint64_t)__double_as_longlong(y.hi);
    const int ex = (int)((bits >> 52) & 0x7FF);
    if (ex < 64 || (bits & 0xFFFFFFFFFFFFFull) == 0) return false; // tiny, or a power of two (ulp changes)
    const double half_ulp = __longlong_as_double((long long)((uint64_t)(ex - 53) << 52));
    const double eps = fabs(y.hi) * 2.168404344971009e-19;          // 2^-62 |y| (error bound 2^-65)
    if (fabs(y.lo) + eps < half_ulp) { out = y.hi; return true; }
    return false;
}

MG_DEV bool mg_fast_sin(dd_t r, double &out) {
    const dd_t r2 = dd_mul(r, r);
    const double t = r2.hi;
    double p = mg_ifh(21);
    p = __fma_rn(p, t, -mg_ifh(19)); p = __fma_rn(p, t, mg_ifh(17)); p = __fma_rn(p, t, -mg_ifh(15));
    p = __fma_rn(p, t, mg_ifh(13));  p = __fma_rn(p, t, -mg_ifh(11)); p = __fma_rn(p, t, mg_ifh(9));
    p = __fma_rn(p, t, -mg_ifh(7));                                    // T7 = sum_{k>=3} (-1)^k t^(k-3) / (2k+1)!
    dd_t q = dd_add(mg_ifd(5), {t * p, 0.0});                          // 1/5! + r^2 T7
    q = dd_add(dd_neg(mg_ifd(3)), dd_mul(r2, q));                      // -1/3! + r^2 (...)
    q = dd_add({1.0, 0.0}, dd_mul(r2, q));
    return mg_certify(dd_mul(r, q), out);
}

MG_DEV bool mg_fast_cos(dd_t r, double &out) {
    const dd_t r2 = dd_mul(r, r);
    const double t = r2.hi;
    double p = -mg_ifh(22);
    p = __fma_rn(p, t, mg_ifh(20)); p = __fma_rn(p, t, -mg_ifh(18)); p = __fma_rn(p, t, mg_ifh(16));
    p = __fma_rn(p, t, -mg_ifh(14)); p = __fma_rn(p, t, mg_ifh(12)); p = __fma_rn(p, t, -mg_ifh(10));
    p = __fma_rn(p, t, mg_ifh(8));                                     // T8 = sum_{k>=4} (-1)^k t^(k-4) / (2k)!
    dd_t q = dd_add(dd_neg(mg_ifd(6)), {t * p, 0.0});                  // -1/6! + r^2 T8
    q = dd_add(mg_ifd(4), dd_mul(r2, q));
    q = dd_add(dd_neg(mg_ifd(2)), dd_mul(r2, q));
    return mg_certify(dd_add({1.0, 0.0}, dd_mul(r2, q)), out);
}

// full double-double series: the rare arguments the fast path cannot certify (kept out of line)
__device__ __noinline__ void mg_sincos_slow(double rh, double rl, int q, double *s, double *c) {
    dd_t r = {rh, rl};
    dd_t ks = mg_ksin(r), kc = mg_kcos(r), vs, vc;
    switch (q) {
    case 0: vs = ks; vc = kc; break;
    case 1: vs = kc; vc = dd_neg(ks); break;
    case 2: vs = dd_neg(ks); vc = dd_neg(kc); break;
    default: vs = dd_neg(kc); vc = ks; break;
    }
    *s = vs.hi + vs.lo;
    *c = vc.hi + vc.lo;
}

// correctly rounded (cos x, sin x)
MG_DEV void mg_sincos(double x, double &s, double &c) {
    if (fabs(x) < 7.450580596923828e-09) { s = x; c = 1.0; return; }
    int q; dd_t r;
    mg_reduce_pio2(x, q, r);
    double fs, fc;
    const bool ok_s = mg_fast_sin(r, fs), ok_c = mg_fast_cos(r, fc);
    if (ok_s && ok_c) {
        double vs, vc;
        switch (q) {
        case 0: vs = fs; vc = fc; break;
        case 1: vs = fc; vc = -fs; break;
        case 2: vs = -fs; vc = -fc; break;
        default: vs = -fc; vc = fs; break;
        }
        s = vs; c = vc;
    } else {
        double ss, cc;
        mg_sincos_slow(r.hi, r.lo, q, &ss, &cc);
        s = ss; c = cc;
    }
    if (fabs(x) < 1.4901161193847656e-08) s = x; // |x| < 2^-26: sin rounds to x
}

// numpy float64 3x3 matmul (fma chain, see header)
MG_DEV void mg_mat3_mul(const double *a, const double *b, double *out) {
    double t[9];
#pragma unroll
    for (int i = 0; i < 3; i++)
#pragma unroll
        for (int j = 0; j < 3; j++)
            t[i * 3 + j] = __fma_rn(a[i * 3 + 2], b[6 + j], __fma_rn(a[i * 3 + 1], b[3 + j], a[i * 3 + 0] * b[j]));
#pragma unroll
    for (int i = 0; i < 9; i++) out[i] = t[i];
}

// render.py Transform(translation=(tx,ty), rotation) with unit scale: (T @ R) @ S, from the rotation's
// (sin, cos)
MG_DEV void mg_transform_tr_sc(double tx, double ty, double s, double c, double *out) {
    const double T[9] = {1.0, 0.0, tx, 0.0, 1.0, ty, 0.0, 0.0, 1.0};
    const double R[9] = {c, -s, 0.0, s, c, 0.0, 0.0, 0.0, 1.0};
    const double S[9] = {1.0, 0.0, 0.0, 0.0, 1.0, 0.0, 0.0, 0.0, 1.0};
    double TR[9];
    mg_mat3_mul(T, R, TR);
    mg_mat3_mul(TR, S, out);
}

// render.py Transform(translation=(tx,ty), rotation) with unit scale: (T @ R) @ S
MG_DEV void mg_transform_tr(double tx, double ty, double rot, double *out) {
    double s, c;
    mg_sincos(rot, s, c);
    const double T[9] = {1.0, 0.0, tx, 0.0, 1.0, ty, 0.0, 0.0, 1.0};
    const double R[9] = {c, -s, 0.0, s, c, 0.0, 0.0, 0.0, 1.0};
    const double S[9] = {1.0, 0.0, 0.0, 0.0, 1.0, 0.0, 0.0, 0.0, 1.0};
    double TR[9];
    mg_mat3_mul(T, R, TR);
    mg_mat3_mul(TR, S, out);
}
