// mg_step.h -- one env-step of physics per lane: Robot.update + cpSpaceStep x10.
//
// base_env.py:267-276 (action -> Robot.set_action), entities.py:435-476
// (Robot.set_action / Robot.update), base_env.py:248-255 (10 substeps).
#pragma once
#include "mg_phys.h"
#include "mg_prof.h"

// ---- body access with the static body as zeros --------------------------
struct BodyR { int b; double minv, iinv; };
MG_DEV BodyR bodyr(const MGState &S, int e, int b) {
    if (b < 0) return {b, 0.0, 0.0};
    return {b, AT(S.bminv, b), AT(S.biinv, b)};
}
MG_DEV V2 bv(const MGState &S, int e, int b) { return b < 0 ? v2(0.0, 0.0) : v2(AT(S.bvx, b), AT(S.bvy, b)); }
MG_DEV double bwv(const MGState &S, int e, int b) { return b < 0 ? 0.0 : AT(S.bw, b); }
MG_DEV V2 bvb(const MGState &S, int e, int b) { return b < 0 ? v2(0.0, 0.0) : v2(AT(S.bvbx, b), AT(S.bvby, b)); }
MG_DEV double bwb(const MGState &S, int e, int b) { return b < 0 ? 0.0 : AT(S.bwb, b); }
MG_DEV V2 bp(const MGState &S, int e, int b) { return b < 0 ? v2(0.0, 0.0) : v2(AT(S.bpx, b), AT(S.bpy, b)); }
MG_DEV double ban(const MGState &S, int e, int b) { return b < 0 ? 0.0 : AT(S.ba, b); }

MG_DEV void apply_impulse(const MGState &S, int e, const BodyR &B, V2 j, V2 r) {
    if (B.b < 0) return;
    AT(S.bvx, B.b) = AT(S.bvx, B.b) + j.x * B.minv;
    AT(S.bvy, B.b) = AT(S.bvy, B.b) + j.y * B.minv;
    AT(S.bw, B.b) += B.iinv * vcross(r, j);
}
MG_DEV void apply_impulses(const MGState &S, int e, const BodyR &A, const BodyR &B, V2 r1, V2 r2, V2 j) {
    apply_impulse(S, e, A, vneg(j), r1);
    apply_impulse(S, e, B, j, r2);
}
MG_DEV void apply_bias_impulse(const MGState &S, int e, const BodyR &B, V2 j, V2 r) {
    if (B.b < 0) return;
    AT(S.bvbx, B.b) = AT(S.bvbx, B.b) + j.x * B.minv;
    AT(S.bvby, B.b) = AT(S.bvby, B.b) + j.y * B.minv;
    AT(S.bwb, B.b) += B.iinv * vcross(r, j);
}
MG_DEV V2 relative_velocity(const MGState &S, int e, int a, int b, V2 r1, V2 r2) {
    V2 v1 = vadd(bv(S, e, a), vmult(vperp(r1), bwv(S, e, a)));
    V2 v2_ = vadd(bv(S, e, b), vmult(vperp(r2), bwv(S, e, b)));
    return vsub(v2_, v1);
}
MG_DEV double k_scalar_body(const BodyR &B, V2 r, V2 n) {
    double rcn = vcross(r, n);
    return B.minv + B.iinv * rcn * rcn;
}

// ---- constraints ----------------------------------------------------------
MG_DEV void cons_prestep_impl(const MGState &S, int e, int c, int a, int b, int type, double dt) {
    BodyR A = bodyr(S, e, a), B = bodyr(S, e, b);
    switch (type) {
    case MG_C_PIVOT: {
        double ac = a < 0 ? 1.0 : AT(S.brc, a), as = a < 0 ? 0.0 : AT(S.brs, a);
        double bc = AT(S.brc, b), bs = AT(S.brs, b);
        V2 aa = vsub(v2(CPA(CP_AAX, c), CPA(CP_AAY, c)), v2(0.0, 0.0));
        V2 ab = vsub(v2(CPA(CP_ABX, c), CPA(CP_ABY, c)), v2(0.0, 0.0));
        V2 r1 = v2(ac * aa.x + (-as) * aa.y, as * aa.x + ac * aa.y);
        V2 r2 = v2(bc * ab.x + (-bs) * ab.y, bs * ab.x + bc * ab.y);
        CPA(CP_R1X, c) = r1.x; CPA(CP_R1Y, c) = r1.y; CPA(CP_R2X, c) = r2.x; CPA(CP_R2Y, c) = r2.y;
        double m_sum = A.minv + B.minv;
        double k11 = m_sum, k12 = 0.0, k21 = 0.0, k22 = m_sum;
        double r1xsq = r1.x * r1.x * A.iinv, r1ysq = r1.y * r1.y * A.iinv, r1nxy = -r1.x * r1.y * A.iinv;
        k11 += r1ysq; k12 += r1nxy; k21 += r1nxy; k22 += r1xsq;
        double r2xsq = r2.x * r2.x * B.iinv, r2ysq = r2.y * r2.y * B.iinv, r2nxy = -r2.x * r2.y * B.iinv;
        k11 += r2ysq; k12 += r2nxy; k21 += r2nxy; k22 += r2xsq;
        double det = k11 * k22 - k12 * k21;
        double det_inv = 1.0 / det;
        CPA(CP_K11, c) = k22 * det_inv; CPA(CP_K12, c) = -k12 * det_inv;
        CPA(CP_K21, c) = -k21 * det_inv; CPA(CP_K22, c) = k11 * det_inv;
        V2 delta = vsub(vadd(bp(S, e, b), r2), vadd(bp(S, e, a), r1));
        V2 bias = vclamp(vmult(delta, -CPA(CP_BCOEF, c) / dt), CPA(CP_MAXB, c));
        CPA(CP_BIAS, c) = bias.x; CPA(CP_BIAS2, c) = bias.y;
        break;
    }
    case MG_C_GEAR: {
        CPA(CP_ISUM, c) = 1.0 / (A.iinv * CPA(CP_RATIO_INV, c) + CPA(CP_RATIO, c) * B.iinv);
        double maxBias = CPA(CP_MAXB, c);
        CPA(CP_BIAS, c) = cpclamp(-CPA(CP_BCOEF, c) * (ban(S, e, b) * CPA(CP_RATIO, c) - ban(S, e, a) - CPA(CP_PHASE, c)) / dt,
                                  -maxBias, maxBias);
        break;
    }
    case MG_C_ROTLIMIT: {
        double dist = ban(S, e, b) - ban(S, e, a), pdist = 0.0;
        double mx = CPA(CP_MAX, c), mn = CPA(CP_MIN, c);
        if (dist > mx) pdist = mx - dist;
        else if (dist < mn) pdist = mn - dist;
        CPA(CP_ISUM, c) = 1.0 / (A.iinv + B.iinv);
        double maxBias = CPA(CP_MAXB, c);
        double bias = cpclamp(-CPA(CP_BCOEF, c) * pdist / dt, -maxBias, maxBias);
        CPA(CP_BIAS, c) = bias;
        if (!bias) CPA(CP_JACC, c) = 0.0;
        break;
    }
    case MG_C_MOTOR:
        CPA(CP_ISUM, c) = 1.0 / (A.iinv + B.iinv);
        break;
    case MG_C_SPRING: {
        double moment = A.iinv + B.iinv;
        CPA(CP_ISUM, c) = 1.0 / moment;
        CPA(CP_TWRN, c) = 0.0;
        double j_spring = ((ban(S, e, a) - ban(S, e, b)) - CPA(CP_REST, c)) * CPA(CP_STIFF, c) * dt;
        CPA(CP_JACC, c) = j_spring;
        if (a >= 0) AT(S.bw, a) -= j_spring * A.iinv;
        if (b >= 0) AT(S.bw, b) += j_spring * B.iinv;
        break;
    }
    }
}

MG_DEV void cons_cached_impl(const MGState &S, int e, int c, int a, int b, int type, double dt_coef) {
    BodyR A = bodyr(S, e, a), B = bodyr(S, e, b);
    switch (type) {
    case MG_C_PIVOT:
        apply_impulses(S, e, A, B, v2(CPA(CP_R1X, c), CPA(CP_R1Y, c)), v2(CPA(CP_R2X, c), CPA(CP_R2Y, c)),
                       vmult(v2(CPA(CP_JACC, c), CPA(CP_JACC2, c)), dt_coef));
        break;
    case MG_C_GEAR: {
        double j = CPA(CP_JACC, c) * dt_coef;
        if (a >= 0) AT(S.bw, a) -= j * A.iinv * CPA(CP_RATIO_INV, c);
        if (b >= 0) AT(S.bw, b) += j * B.iinv;
        break;
    }
    case MG_C_ROTLIMIT:
    case MG_C_MOTOR: {
        double j = CPA(CP_JACC, c) * dt_coef;
        if (a >= 0) AT(S.bw, a) -= j * A.iinv;
        if (b >= 0) AT(S.bw, b) += j * B.iinv;
        break;
    }
    default: break;
    }
}

MG_DEV void cons_apply_impl(const MGState &S, int e, int c, int a, int b, int type, double dt) {
    BodyR A = bodyr(S, e, a), B = bodyr(S, e, b);
    switch (type) {
    case MG_C_PIVOT: {
        V2 r1 = v2(CPA(CP_R1X, c), CPA(CP_R1Y, c)), r2 = v2(CPA(CP_R2X, c), CPA(CP_R2Y, c));
        V2 vr = relative_velocity(S, e, a, b, r1, r2);
        V2 d = vsub(v2(CPA(CP_BIAS, c), CPA(CP_BIAS2, c)), vr);
        V2 j = v2(d.x * CPA(CP_K11, c) + d.y * CPA(CP_K12, c), d.x * CPA(CP_K21, c) + d.y * CPA(CP_K22, c));
        V2 jOld = v2(CPA(CP_JACC, c), CPA(CP_JACC2, c));
        V2 jAcc = vclamp(vadd(jOld, j), CPA(CP_MAXF, c) * dt);
        CPA(CP_JACC, c) = jAcc.x; CPA(CP_JACC2, c) = jAcc.y;
        apply_impulses(S, e, A, B, r1, r2, vsub(jAcc, jOld));
        break;
    }
    case MG_C_GEAR: {
        double ratio = CPA(CP_RATIO, c);
        double wr = bwv(S, e, b) * ratio - bwv(S, e, a);
        double jMax = CPA(CP_MAXF, c) * dt;
        double j = (CPA(CP_BIAS, c) - wr) * CPA(CP_ISUM, c);
        double jOld = CPA(CP_JACC, c);
        double jAcc = cpclamp(jOld + j, -jMax, jMax);
        CPA(CP_JACC, c) = jAcc;
        j = jAcc - jOld;
        if (a >= 0) AT(S.bw, a) -= j * A.iinv * CPA(CP_RATIO_INV, c);
        if (b >= 0) AT(S.bw, b) += j * B.iinv;
        break;
    }
    case MG_C_ROTLIMIT: {
        double bias = CPA(CP_BIAS, c);
        if (!bias) return;
        double wr = bwv(S, e, b) - bwv(S, e, a);
        double jMax = CPA(CP_MAXF, c) * dt;
        double j = -(bias + wr) * CPA(CP_ISUM, c);
        double jOld = CPA(CP_JACC, c);
        double jAcc = bias < 0.0 ? cpclamp(jOld + j, 0.0, jMax) : cpclamp(jOld + j, -jMax, 0.0);
        CPA(CP_JACC, c) = jAcc;
        j = jAcc - jOld;
        if (a >= 0) AT(S.bw, a) -= j * A.iinv;
        if (b >= 0) AT(S.bw, b) += j * B.iinv;
        break;
    }
    case MG_C_MOTOR: {
        double wr = bwv(S, e, b) - bwv(S, e, a) + CPA(CP_RATE, c);
        double jMax = CPA(CP_MAXF, c) * dt;
        double j = -wr * CPA(CP_ISUM, c);
        double jOld = CPA(CP_JACC, c);
        double jAcc = cpclamp(jOld + j, -jMax, jMax);
        CPA(CP_JACC, c) = jAcc;
        j = jAcc - jOld;
        if (a >= 0) AT(S.bw, a) -= j * A.iinv;
        if (b >= 0) AT(S.bw, b) += j * B.iinv;
        break;
    }
    case MG_C_SPRING: {
        double wrn = bwv(S, e, a) - bwv(S, e, b);
        double w_damp = (CPA(CP_TWRN, c) - wrn) * CPA(CP_WCOEF, c);
        CPA(CP_TWRN, c) = wrn + w_damp;
        double j_damp = w_damp * CPA(CP_ISUM, c);
        CPA(CP_JACC, c) += j_damp;
        if (a >= 0) AT(S.bw, a) += j_damp * A.iinv;
        if (b >= 0) AT(S.bw, b) -= j_damp * B.iinv;
        break;
    }
    }
}

MG_DEV void cons_prestep(const MGState &S, int e, int c, double dt) {
    cons_prestep_impl(S, e, c, AT(S.ca, c), AT(S.cb, c), AT(S.ctype, c), dt);
}
MG_DEV void cons_cached(const MGState &S, int e, int c, double dt_coef) {
    cons_cached_impl(S, e, c, AT(S.ca, c), AT(S.cb, c), AT(S.ctype, c), dt_coef);
}
MG_DEV void cons_apply(const MGState &S, int e, int c, double dt) {
    cons_apply_impl(S, e, c, AT(S.ca, c), AT(S.cb, c), AT(S.ctype, c), dt);
}

// Constraint lists known at compile time (the LDS step variants): the robot's ten joints in
// add_robot order (entities.py:238-433) with body slots 0 body, 1 control, 2-3 eyes, 4-5 fingers,
// then, for one block, its two ground-friction joints (static body -1, block body 6).
struct ConsDesc { int type, a, b; };
__host__ __device__ constexpr ConsDesc static_cons(int c) {
    constexpr ConsDesc T[12] = {{MG_C_PIVOT, 1, 0},   {MG_C_GEAR, 1, 0},     {MG_C_SPRING, 0, 2},  {MG_C_SPRING, 0, 3},
                                {MG_C_PIVOT, 0, 4},   {MG_C_ROTLIMIT, 0, 4}, {MG_C_MOTOR, 0, 4},   {MG_C_PIVOT, 0, 5},
                                {MG_C_ROTLIMIT, 0, 5}, {MG_C_MOTOR, 0, 5},   {MG_C_PIVOT, -1, 6},  {MG_C_GEAR, -1, 6}};
    return T[c];
}
// ---- arbiters ------------------------------------------------------------
// (ta, ba) / (tb, bb): world-shape type and body of the pair's shapes A / B in broadphase order
// arbiter_update_t with the slot search done by the caller: slot = the first slot holding key (-1: none),
// free_slot = the first empty slot (used only when slot < 0)
MG_DEV void arbiter_update_found(const MGState &S, const mg_library *L, int e, int key, int ta, int ba, int tb,
                                 int bb, double ua, double ub, const Collision &info, int slot, int free_slot);
MG_DEV void arbiter_update_t(const MGState &S, const mg_library *L, int e, int key, int ta, int ba, int tb, int bb,
                             double ua, double ub, const Collision &info) {
    int na = S.arb_cap, slot = -1, free_slot = -1;
    for (int i = 0; i < na; i++) {
        int k = AT(S.akey, i);
        if (k == key) { slot = i; break; }
        if (k < 0 && free_slot < 0) free_slot = i;
    }
    arbiter_update_found(S, L, e, key, ta, ba, tb, bb, ua, ub, info, slot, free_slot);
}
MG_DEV void arbiter_update_found(const MGState &S, const mg_library *L, int e, int key, int ta, int ba, int tb,
                                 int bb, double ua, double ub, const Collision &info, int slot, int free_slot) {
    if (slot < 0) {
        if (free_slot < 0) { S.overflow[e] |= 1; return; }
        slot = free_slot;
        AT(S.akey, slot) = key; AT(S.astate, slot) = ARB_FIRST; AT(S.acount, slot) = 0; AT(S.astamp, slot) = 0;
    }
    // info is in collision order: swapped => (a, b) = (B, A)
    const bool sw = ta > tb;
    const int sa_body = sw ? bb : ba, sb_body = sw ? ba : bb;
    double u_a = sw ? ub : ua, u_b = sw ? ua : ub;
    V2 pa = bp(S, e, sa_body), pb = bp(S, e, sb_body);
    int oldc = AT(S.acount, slot);
    uint64_t oh0 = AHASH(0, slot), oh1 = AHASH(1, slot);
    double ojn0 = ACON(0, AC_JN, slot), ojt0 = ACON(0, AC_JT, slot);
    double ojn1 = ACON(1, AC_JN, slot), ojt1 = ACON(1, AC_JT, slot);
#pragma unroll
    for (int k = 0; k < 2; k++) {   // constant indices: the Collision can stay in registers
        if (k >= info.count) break;
        V2 r1 = vsub(info.p1[k], pa), r2 = vsub(info.p2[k], pb);
        double jn = 0.0, jt = 0.0;
        uint64_t h = info.hash[k];
        if (oldc > 0 && h == oh0) { jn = ojn0; jt = ojt0; }
        if (oldc > 1 && h == oh1) { jn = ojn1; jt = ojt1; }
        ACON(k, AC_R1X, slot) = r1.x; ACON(k, AC_R1Y, slot) = r1.y;
        ACON(k, AC_R2X, slot) = r2.x; ACON(k, AC_R2Y, slot) = r2.y;
        ACON(k, AC_JN, slot) = jn; ACON(k, AC_JT, slot) = jt;
        AHASH(k, slot) = h;
    }
    AT(S.acount, slot) = info.count;
    AT(S.anx, slot) = info.n.x; AT(S.any, slot) = info.n.y;
    AT(S.au, slot) = u_a * u_b;
    AT(S.asa, slot) = sa_body; AT(S.asb, slot) = sb_body;
    if (AT(S.astate, slot) == ARB_CACHED) AT(S.astate, slot) = ARB_FIRST;
    int na_ = S.nactive[e];
    if (na_ < S.arb_cap) { AT(S.active, na_) = slot; S.nactive[e] = na_ + 1; }
    else S.overflow[e] |= 1;
    AT(S.astamp, slot) = S.stamp[e];
}

MG_DEV void arbiter_update(const MGState &S, const mg_library *L, int e, int key, const ShapeW &A, const ShapeW &B,
                           double ua, double ub, const Collision &info) {
    arbiter_update_t(S, L, e, key, A.type, A.body, B.type, B.body, ua, ub, info);
}

MG_DEV void arbiter_prestep(const MGState &S, const mg_library *L, int e, int slot, double dt) {
    int a = AT(S.asa, slot), b = AT(S.asb, slot);
    BodyR A = bodyr(S, e, a), B = bodyr(S, e, b);
    V2 n = v2(AT(S.anx, slot), AT(S.any, slot));
    V2 body_delta = vsub(bp(S, e, b), bp(S, e, a));
    int cnt = AT(S.acount, slot);
    for (int k = 0; k < cnt; k++) {
        V2 r1 = v2(ACON(k, AC_R1X, slot), ACON(k, AC_R1Y, slot)), r2 = v2(ACON(k, AC_R2X, slot), ACON(k, AC_R2Y, slot));
        ACON(k, AC_NMASS, slot) = 1.0 / (k_scalar_body(A, r1, n) + k_scalar_body(B, r2, n));
        V2 pn = vperp(n);
        ACON(k, AC_TMASS, slot) = 1.0 / (k_scalar_body(A, r1, pn) + k_scalar_body(B, r2, pn));
        double dist = vdot(vadd(vsub(r2, r1), body_delta), n);
        ACON(k, AC_BIAS, slot) = -L->collision_bias_coef * cpmin(0.0, dist + L->slop) / dt;
        ACON(k, AC_JB, slot) = 0.0;
    }
}

MG_DEV void arbiter_cached(const MGState &S, int e, int slot, double dt_coef) {
    if (AT(S.astate, slot) == ARB_FIRST) return;
    int a = AT(S.asa, slot), b = AT(S.asb, slot);
    BodyR A = bodyr(S, e, a), B = bodyr(S, e, b);
    V2 n = v2(AT(S.anx, slot), AT(S.any, slot));
    int cnt = AT(S.acount, slot);
    for (int k = 0; k < cnt; k++) {
        V2 j = vrotate(n, v2(ACON(k, AC_JN, slot), ACON(k, AC_JT, slot)));
        apply_impulses(S, e, A, B, v2(ACON(k, AC_R1X, slot), ACON(k, AC_R1Y, slot)),
                       v2(ACON(k, AC_R2X, slot), ACON(k, AC_R2Y, slot)), vmult(j, dt_coef));
    }
}

MG_DEV void arbiter_apply(const MGState &S, int e, int slot) {
    int a = AT(S.asa, slot), b = AT(S.asb, slot);
    BodyR A = bodyr(S, e, a), B = bodyr(S, e, b);
    V2 n = v2(AT(S.anx, slot), AT(S.any, slot));
    double friction = AT(S.au, slot);
    int cnt = AT(S.acount, slot);
    for (int k = 0; k < cnt; k++) {
        double nMass = ACON(k, AC_NMASS, slot);
        V2 r1 = v2(ACON(k, AC_R1X, slot), ACON(k, AC_R1Y, slot)), r2 = v2(ACON(k, AC_R2X, slot), ACON(k, AC_R2Y, slot));
        V2 vb1 = vadd(bvb(S, e, a), vmult(vperp(r1), bwb(S, e, a)));
        V2 vb2 = vadd(bvb(S, e, b), vmult(vperp(r2), bwb(S, e, b)));
        V2 vr = relative_velocity(S, e, a, b, r1, r2);
        double vbn = vdot(vsub(vb2, vb1), n);
        double vrn = vdot(vr, n);
        double vrt = vdot(vr, vperp(n));
        double jbn = (ACON(k, AC_BIAS, slot) - vbn) * nMass;
        double jbnOld = ACON(k, AC_JB, slot);
        double jBias = cpmax(jbnOld + jbn, 0.0);
        ACON(k, AC_JB, slot) = jBias;
        double jn = -(0.0 + vrn) * nMass;
        double jnOld = ACON(k, AC_JN, slot);
        double jnAcc = cpmax(jnOld + jn, 0.0);
        ACON(k, AC_JN, slot) = jnAcc;
        double jtMax = friction * jnAcc;
        double jt = -vrt * ACON(k, AC_TMASS, slot);
        double jtOld = ACON(k, AC_JT, slot);
        double jtAcc = cpclamp(jtOld + jt, -jtMax, jtMax);
        ACON(k, AC_JT, slot) = jtAcc;
        V2 jb = vmult(n, jBias - jbnOld);
        apply_bias_impulse(S, e, A, vneg(jb), r1);
        apply_bias_impulse(S, e, B, jb, r2);
        apply_impulses(S, e, A, B, r1, r2, vrotate(n, v2(jnAcc - jnOld, jtAcc - jtOld)));
    }
}

// ---- register-resident solver sweep (LDS variants) -----------------------
// With the constraint list known at compile time, applyCachedImpulse and the 10 solver
// iterations run on body velocities and constraint terms held in VGPRs: constraints index
// bodies by constants, arbiters (runtime body slots) through select chains.  Same operations
// in the same order as cons_cached_impl / cons_apply_impl / arbiter_cached / arbiter_apply.
template <int NB>
struct RegBodies { double vx[NB], vy[NB], w[NB], vbx[NB], vby[NB], wb[NB], minv[NB], iinv[NB]; };

struct RegCons {
    double r1x, r1y, r2x, r2y, k11, k12, k21, k22, bias, bias2, jacc, jacc2, jmax, ratio, ratio_inv, isum, rate, twrn,
        wcoef;
};

// compile-time body slot (constraints; b < 0 = the static body)
template <int NB>
MG_DEV void rapply(RegBodies<NB> &R, int b, V2 j, V2 r) {
    if (b < 0) return;
    R.vx[b] = R.vx[b] + j.x * R.minv[b];
    R.vy[b] = R.vy[b] + j.y * R.minv[b];
    R.w[b] += R.iinv[b] * vcross(r, j);
}
template <int NB> MG_DEV V2 rv(const RegBodies<NB> &R, int b) { return b < 0 ? v2(0.0, 0.0) : v2(R.vx[b], R.vy[b]); }
template <int NB> MG_DEV double rw(const RegBodies<NB> &R, int b) { return b < 0 ? 0.0 : R.w[b]; }
template <int NB> MG_DEV double rii(const RegBodies<NB> &R, int b) { return b < 0 ? 0.0 : R.iinv[b]; }

template <int NB>
MG_DEV void rb_load(RegBodies<NB> &R, const MGState &S, int e) {
#pragma unroll
    for (int b = 0; b < NB; b++) {
        R.vx[b] = AT(S.bvx, b); R.vy[b] = AT(S.bvy, b); R.w[b] = AT(S.bw, b);
        R.vbx[b] = AT(S.bvbx, b); R.vby[b] = AT(S.bvby, b); R.wb[b] = AT(S.bwb, b);
        R.minv[b] = AT(S.bminv, b); R.iinv[b] = AT(S.biinv, b);
    }
}
template <int NB>
MG_DEV void rb_store(const RegBodies<NB> &R, const MGState &S, int e) {
#pragma unroll
    for (int b = 0; b < NB; b++) {
        AT(S.bvx, b) = R.vx[b]; AT(S.bvy, b) = R.vy[b]; AT(S.bw, b) = R.w[b];
        AT(S.bvbx, b) = R.vbx[b]; AT(S.bvby, b) = R.vby[b]; AT(S.bwb, b) = R.wb[b];
    }
}

MG_DEV void rc_load(RegCons &q, const MGState &S, int e, int c, int type, double dt) {
    q.jacc = CPA(CP_JACC, c); q.jacc2 = 0.0; q.jmax = CPA(CP_MAXF, c) * dt;
    q.isum = CPA(CP_ISUM, c); q.bias = CPA(CP_BIAS, c);
    if (type == MG_C_PIVOT) {
        q.jacc2 = CPA(CP_JACC2, c); q.bias2 = CPA(CP_BIAS2, c);
        q.r1x = CPA(CP_R1X, c); q.r1y = CPA(CP_R1Y, c); q.r2x = CPA(CP_R2X, c); q.r2y = CPA(CP_R2Y, c);
        q.k11 = CPA(CP_K11, c); q.k12 = CPA(CP_K12, c); q.k21 = CPA(CP_K21, c); q.k22 = CPA(CP_K22, c);
    }
    if (type == MG_C_GEAR) { q.ratio = CPA(CP_RATIO, c); q.ratio_inv = CPA(CP_RATIO_INV, c); }
    if (type == MG_C_MOTOR) q.rate = CPA(CP_RATE, c);
    if (type == MG_C_SPRING) { q.twrn = CPA(CP_TWRN, c); q.wcoef = CPA(CP_WCOEF, c); }
}
MG_DEV void rc_store(const RegCons &q, const MGState &S, int e, int c, int type) {
    CPA(CP_JACC, c) = q.jacc;
    if (type == MG_C_PIVOT) CPA(CP_JACC2, c) = q.jacc2;
    if (type == MG_C_SPRING) CPA(CP_TWRN, c) = q.twrn;
}

template <int NB>
MG_DEV void rcons_cached(RegBodies<NB> &R, const RegCons &q, int a, int b, int type, double dt_coef) {
    switch (type) {
    case MG_C_PIVOT: {
        V2 j = vmult(v2(q.jacc, q.jacc2), dt_coef);
        rapply(R, a, vneg(j), v2(q.r1x, q.r1y));
        rapply(R, b, j, v2(q.r2x, q.r2y));
        break;
    }
    case MG_C_GEAR: {
        double j = q.jacc * dt_coef;
        if (a >= 0) R.w[a] -= j * R.iinv[a] * q.ratio_inv;
        if (b >= 0) R.w[b] += j * R.iinv[b];
        break;
    }
    case MG_C_ROTLIMIT:
    case MG_C_MOTOR: {
        double j = q.jacc * dt_coef;
        if (a >= 0) R.w[a] -= j * R.iinv[a];
        if (b >= 0) R.w[b] += j * R.iinv[b];
        break;
    }
    default: break;
    }
}

template <int NB>
MG_DEV void rcons_apply(RegBodies<NB> &R, RegCons &q, int a, int b, int type) {
    switch (type) {
    case MG_C_PIVOT: {
        V2 r1 = v2(q.r1x, q.r1y), r2 = v2(q.r2x, q.r2y);
        V2 v1 = vadd(rv(R, a), vmult(vperp(r1), rw(R, a)));
        V2 v2_ = vadd(rv(R, b), vmult(vperp(r2), rw(R, b)));
        V2 vr = vsub(v2_, v1);
        V2 d = vsub(v2(q.bias, q.bias2), vr);
        V2 j = v2(d.x * q.k11 + d.y * q.k12, d.x * q.k21 + d.y * q.k22);
        V2 jOld = v2(q.jacc, q.jacc2);
        V2 jAcc = vclamp(vadd(jOld, j), q.jmax);
        q.jacc = jAcc.x; q.jacc2 = jAcc.y;
        V2 dj = vsub(jAcc, jOld);
        rapply(R, a, vneg(dj), r1);
        rapply(R, b, dj, r2);
        break;
    }
    case MG_C_GEAR: {
        double wr = rw(R, b) * q.ratio - rw(R, a);
        double j = (q.bias - wr) * q.isum;
        double jOld = q.jacc;
        double jAcc = cpclamp(jOld + j, -q.jmax, q.jmax);
        q.jacc = jAcc;
        j = jAcc - jOld;
        if (a >= 0) R.w[a] -= j * R.iinv[a] * q.ratio_inv;
        if (b >= 0) R.w[b] += j * R.iinv[b];
        break;
    }
    case MG_C_ROTLIMIT: {
        double bias = q.bias;
        if (!bias) return;
        double wr = rw(R, b) - rw(R, a);
        double j = -(bias + wr) * q.isum;
        double jOld = q.jacc;
        double jAcc = bias < 0.0 ? cpclamp(jOld + j, 0.0, q.jmax) : cpclamp(jOld + j, -q.jmax, 0.0);
        q.jacc = jAcc;
        j = jAcc - jOld;
        if (a >= 0) R.w[a] -= j * R.iinv[a];
        if (b >= 0) R.w[b] += j * R.iinv[b];
        break;
    }
    case MG_C_MOTOR: {
        double wr = rw(R, b) - rw(R, a) + q.rate;
        double j = -wr * q.isum;
        double jOld = q.jacc;
        double jAcc = cpclamp(jOld + j, -q.jmax, q.jmax);
        q.jacc = jAcc;
        j = jAcc - jOld;
        if (a >= 0) R.w[a] -= j * R.iinv[a];
        if (b >= 0) R.w[b] += j * R.iinv[b];
        break;
    }
    case MG_C_SPRING: {
        double wrn = rw(R, a) - rw(R, b);
        double w_damp = (q.twrn - wrn) * q.wcoef;
        q.twrn = wrn + w_damp;
        double j_damp = w_damp * q.isum;
        q.jacc += j_damp;
        if (a >= 0) R.w[a] += j_damp * R.iinv[a];
        if (b >= 0) R.w[b] -= j_damp * R.iinv[b];
        break;
    }
    }
}

// Arbiter body slots of the compile-time scenes: only the bodies that carry shapes (robot 0, fingers 4-5,
// block 6) can be in contact, so a runtime slot is a one-hot over those (all false: the static body) and
// reads / writes select among 3-4 registers instead of all NB (the step kernel checks that every shape
// of such a scene is on one of those bodies).
__host__ __device__ constexpr bool shape_body_slot(int k) { return k == 0 || k == 4 || k == 5 || k == 6; }
template <int NB>
struct ArbBody { bool m[NB]; };
template <int NB>
MG_DEV ArbBody<NB> arb_body(int b) {
    ArbBody<NB> h;
#pragma unroll
    for (int k = 0; k < NB; k++) h.m[k] = shape_body_slot(k) && b == k;
    return h;
}
template <int NB>
MG_DEV double hsel(const double (&x)[NB], const ArbBody<NB> &h) {
    double r = 0.0;
#pragma unroll
    for (int k = 0; k < NB; k++)
        if (shape_body_slot(k)) r = h.m[k] ? x[k] : r;
    return r;
}
template <int NB>
MG_DEV void hput(double (&x)[NB], const ArbBody<NB> &h, double v) {
#pragma unroll
    for (int k = 0; k < NB; k++)
        if (shape_body_slot(k)) x[k] = h.m[k] ? v : x[k];
}
template <int NB>
MG_DEV void happly(RegBodies<NB> &R, const ArbBody<NB> &h, double minv, double iinv, V2 j, V2 r) {
    hput(R.vx, h, hsel(R.vx, h) + j.x * minv);
    hput(R.vy, h, hsel(R.vy, h) + j.y * minv);
    hput(R.w, h, hsel(R.w, h) + iinv * vcross(r, j));
}
template <int NB>
MG_DEV void happly_bias(RegBodies<NB> &R, const ArbBody<NB> &h, double minv, double iinv, V2 j, V2 r) {
    hput(R.vbx, h, hsel(R.vbx, h) + j.x * minv);
    hput(R.vby, h, hsel(R.vby, h) + j.y * minv);
    hput(R.wb, h, hsel(R.wb, h) + iinv * vcross(r, j));
}
template <int NB>
MG_DEV void harb_cached(RegBodies<NB> &R, const MGState &S, int e, int slot, double dt_coef) {
    if (AT(S.astate, slot) == ARB_FIRST) return;
    const ArbBody<NB> ha = arb_body<NB>(AT(S.asa, slot)), hb = arb_body<NB>(AT(S.asb, slot));
    const double am = hsel(R.minv, ha), ai = hsel(R.iinv, ha), bm = hsel(R.minv, hb), bi = hsel(R.iinv, hb);
    V2 n = v2(AT(S.anx, slot), AT(S.any, slot));
    int cnt = AT(S.acount, slot);
    for (int k = 0; k < cnt; k++) {
        V2 j = vmult(vrotate(n, v2(ACON(k, AC_JN, slot), ACON(k, AC_JT, slot))), dt_coef);
        happly(R, ha, am, ai, vneg(j), v2(ACON(k, AC_R1X, slot), ACON(k, AC_R1Y, slot)));
        happly(R, hb, bm, bi, j, v2(ACON(k, AC_R2X, slot), ACON(k, AC_R2Y, slot)));
    }
}
template <int NB>
MG_DEV void harb_apply(RegBodies<NB> &R, const MGState &S, int e, int slot) {
    const int sa = AT(S.asa, slot), sb = AT(S.asb, slot);
    const ArbBody<NB> ha = arb_body<NB>(sa), hb = arb_body<NB>(sb);
    const double am = hsel(R.minv, ha), ai = hsel(R.iinv, ha), bm = hsel(R.minv, hb), bi = hsel(R.iinv, hb);
    // a side whose body is static in every lane running this row (a wall: velocity +0.0 exactly, impulses
    // applied to nothing) skips its selects -- a wave-uniform branch
    const bool wa = __ballot(sa >= 0) != 0, wb = __ballot(sb >= 0) != 0;
    V2 n = v2(AT(S.anx, slot), AT(S.any, slot));
    double friction = AT(S.au, slot);
    int cnt = AT(S.acount, slot);
    for (int k = 0; k < cnt; k++) {
        double nMass = ACON(k, AC_NMASS, slot);
        V2 r1 = v2(ACON(k, AC_R1X, slot), ACON(k, AC_R1Y, slot)), r2 = v2(ACON(k, AC_R2X, slot), ACON(k, AC_R2Y, slot));
        V2 vb1 = v2(0.0, 0.0), v1 = v2(0.0, 0.0), vb2 = v2(0.0, 0.0), v2_ = v2(0.0, 0.0);
        if (wa) {
            vb1 = vadd(v2(hsel(R.vbx, ha), hsel(R.vby, ha)), vmult(vperp(r1), hsel(R.wb, ha)));
            v1 = vadd(v2(hsel(R.vx, ha), hsel(R.vy, ha)), vmult(vperp(r1), hsel(R.w, ha)));
        }
        if (wb) {
            vb2 = vadd(v2(hsel(R.vbx, hb), hsel(R.vby, hb)), vmult(vperp(r2), hsel(R.wb, hb)));
            v2_ = vadd(v2(hsel(R.vx, hb), hsel(R.vy, hb)), vmult(vperp(r2), hsel(R.w, hb)));
        }
        V2 vr = vsub(v2_, v1);
        double vbn = vdot(vsub(vb2, vb1), n);
        double vrn = vdot(vr, n);
        double vrt = vdot(vr, vperp(n));
        double jbn = (ACON(k, AC_BIAS, slot) - vbn) * nMass;
        double jbnOld = ACON(k, AC_JB, slot);
        double jBias = cpmax(jbnOld + jbn, 0.0);
        ACON(k, AC_JB, slot) = jBias;
        double jn = -(0.0 + vrn) * nMass;
        double jnOld = ACON(k, AC_JN, slot);
        double jnAcc = cpmax(jnOld + jn, 0.0);
        ACON(k, AC_JN, slot) = jnAcc;
        double jtMax = friction * jnAcc;
        double jt = -vrt * ACON(k, AC_TMASS, slot);
        double jtOld = ACON(k, AC_JT, slot);
        double jtAcc = cpclamp(jtOld + jt, -jtMax, jtMax);
        ACON(k, AC_JT, slot) = jtAcc;
        V2 jb = vmult(n, jBias - jbnOld);
        if (wa) happly_bias(R, ha, am, ai, vneg(jb), r1);
        if (wb) happly_bias(R, hb, bm, bi, jb, r2);
        V2 j = vrotate(n, v2(jnAcc - jnOld, jtAcc - jtOld));
        if (wa) happly(R, ha, am, ai, vneg(j), r1);
        if (wb) happly(R, hb, bm, bi, j, r2);
    }
}

// harb_apply with compile-time body slots A / B (< 0: the static body): the arbiter pairs the compile-time
// scenes produce (robot body / finger / block against a wall or the block) touch body registers by constant
// index instead of through one-hot selects (harb_apply: ~230 selects per contact).  The same operations in the
// same order as harb_apply: a static side contributes velocity +0.0 and receives nothing, as there.
template <int NB, int A, int B>
MG_DEV void harb_apply_k(RegBodies<NB> &R, const MGState &S, int e, int slot) {
    const double am = A >= 0 ? R.minv[A] : 0.0, ai = A >= 0 ? R.iinv[A] : 0.0;
    const double bm = B >= 0 ? R.minv[B] : 0.0, bi = B >= 0 ? R.iinv[B] : 0.0;
    V2 n = v2(AT(S.anx, slot), AT(S.any, slot));
    double friction = AT(S.au, slot);
    int cnt = AT(S.acount, slot);
    for (int k = 0; k < cnt; k++) {
        double nMass = ACON(k, AC_NMASS, slot);
        V2 r1 = v2(ACON(k, AC_R1X, slot), ACON(k, AC_R1Y, slot)), r2 = v2(ACON(k, AC_R2X, slot), ACON(k, AC_R2Y, slot));
        V2 vb1 = v2(0.0, 0.0), v1 = v2(0.0, 0.0), vb2 = v2(0.0, 0.0), v2_ = v2(0.0, 0.0);
        if constexpr (A >= 0) {
            vb1 = vadd(v2(R.vbx[A], R.vby[A]), vmult(vperp(r1), R.wb[A]));
            v1 = vadd(v2(R.vx[A], R.vy[A]), vmult(vperp(r1), R.w[A]));
        }
        if constexpr (B >= 0) {
            vb2 = vadd(v2(R.vbx[B], R.vby[B]), vmult(vperp(r2), R.wb[B]));
            v2_ = vadd(v2(R.vx[B], R.vy[B]), vmult(vperp(r2), R.w[B]));
        }
        V2 vr = vsub(v2_, v1);
        double vbn = vdot(vsub(vb2, vb1), n);
        double vrn = vdot(vr, n);
        double vrt = vdot(vr, vperp(n));
        double jbn = (ACON(k, AC_BIAS, slot) - vbn) * nMass;
        double jbnOld = ACON(k, AC_JB, slot);
        double jBias = cpmax(jbnOld + jbn, 0.0);
        ACON(k, AC_JB, slot) = jBias;
        double jn = -(0.0 + vrn) * nMass;
        double jnOld = ACON(k, AC_JN, slot);
        double jnAcc = cpmax(jnOld + jn, 0.0);
        ACON(k, AC_JN, slot) = jnAcc;
        double jtMax = friction * jnAcc;
        double jt = -vrt * ACON(k, AC_TMASS, slot);
        double jtOld = ACON(k, AC_JT, slot);
        double jtAcc = cpclamp(jtOld + jt, -jtMax, jtMax);
        ACON(k, AC_JT, slot) = jtAcc;
        V2 jb = vmult(n, jBias - jbnOld);
        if constexpr (A >= 0) {
            const V2 m = vneg(jb);
            R.vbx[A] = R.vbx[A] + m.x * am; R.vby[A] = R.vby[A] + m.y * am; R.wb[A] = R.wb[A] + ai * vcross(r1, m);
        }
        if constexpr (B >= 0) {
            R.vbx[B] = R.vbx[B] + jb.x * bm; R.vby[B] = R.vby[B] + jb.y * bm; R.wb[B] = R.wb[B] + bi * vcross(r2, jb);
        }
        V2 j = vrotate(n, v2(jnAcc - jnOld, jtAcc - jtOld));
        if constexpr (A >= 0) {
            const V2 m = vneg(j);
            R.vx[A] = R.vx[A] + m.x * am; R.vy[A] = R.vy[A] + m.y * am; R.w[A] = R.w[A] + ai * vcross(r1, m);
        }
        if constexpr (B >= 0) {
            R.vx[B] = R.vx[B] + j.x * bm; R.vy[B] = R.vy[B] + j.y * bm; R.w[B] = R.w[B] + bi * vcross(r2, j);
        }
    }
}

// harb_cached with compile-time body slots (applyCachedImpulse of one arbiter; see harb_apply_k)
template <int NB, int A, int B>
MG_DEV void harb_cached_k(RegBodies<NB> &R, const MGState &S, int e, int slot, double dt_coef) {
    const double am = A >= 0 ? R.minv[A] : 0.0, ai = A >= 0 ? R.iinv[A] : 0.0;
    const double bm = B >= 0 ? R.minv[B] : 0.0, bi = B >= 0 ? R.iinv[B] : 0.0;
    V2 n = v2(AT(S.anx, slot), AT(S.any, slot));
    int cnt = AT(S.acount, slot);
    for (int k = 0; k < cnt; k++) {
        V2 j = vmult(vrotate(n, v2(ACON(k, AC_JN, slot), ACON(k, AC_JT, slot))), dt_coef);
        if constexpr (A >= 0) {
            const V2 m = vneg(j), r1 = v2(ACON(k, AC_R1X, slot), ACON(k, AC_R1Y, slot));
            R.vx[A] = R.vx[A] + m.x * am; R.vy[A] = R.vy[A] + m.y * am; R.w[A] = R.w[A] + ai * vcross(r1, m);
        }
        if constexpr (B >= 0) {
            const V2 r2 = v2(ACON(k, AC_R2X, slot), ACON(k, AC_R2Y, slot));
            R.vx[B] = R.vx[B] + j.x * bm; R.vy[B] = R.vy[B] + j.y * bm; R.w[B] = R.w[B] + bi * vcross(r2, j);
        }
    }
}

// applyCachedImpulse of one arbiter of the compile-time scenes, dispatched as harb_row
template <int NB>
MG_DEV void harb_cached_row(RegBodies<NB> &R, const MGState &S, int e, int slot, double dt_coef) {
    if (AT(S.astate, slot) == ARB_FIRST) return;
    const int sa = AT(S.asa, slot), sb = AT(S.asb, slot);
    if (sa == 0 && sb < 0) { harb_cached_k<NB, 0, -1>(R, S, e, slot, dt_coef); return; }
    if (sa < 0 && sb == 4) { harb_cached_k<NB, -1, 4>(R, S, e, slot, dt_coef); return; }
    if (sa < 0 && sb == 5) { harb_cached_k<NB, -1, 5>(R, S, e, slot, dt_coef); return; }
    if constexpr (NB > 6) {
        if (sa < 0 && sb == 6) { harb_cached_k<NB, -1, 6>(R, S, e, slot, dt_coef); return; }
        if (sa == 0 && sb == 6) { harb_cached_k<NB, 0, 6>(R, S, e, slot, dt_coef); return; }
        if (sa == 4 && sb == 6) { harb_cached_k<NB, 4, 6>(R, S, e, slot, dt_coef); return; }
        if (sa == 5 && sb == 6) { harb_cached_k<NB, 5, 6>(R, S, e, slot, dt_coef); return; }
    }
    harb_cached(R, S, e, slot, dt_coef);
}

// one arbiter row of the compile-time scenes: dispatched on its (body A, body B) pair -- robot body 0 (a circle,
// ordered before a wall), fingers 4 / 5 and the block 6 (polygons, ordered after a wall), each against a wall
// or the block (shape_body_slot) -- to harb_apply_k; any other pair takes the select form
template <int NB>
MG_DEV void harb_row(RegBodies<NB> &R, const MGState &S, int e, int slot) {
    const int sa = AT(S.asa, slot), sb = AT(S.asb, slot);
    if (sa == 0 && sb < 0) { harb_apply_k<NB, 0, -1>(R, S, e, slot); return; }
    if (sa < 0 && sb == 4) { harb_apply_k<NB, -1, 4>(R, S, e, slot); return; }
    if (sa < 0 && sb == 5) { harb_apply_k<NB, -1, 5>(R, S, e, slot); return; }
    if constexpr (NB > 6) {
        if (sa < 0 && sb == 6) { harb_apply_k<NB, -1, 6>(R, S, e, slot); return; }
        if (sa == 0 && sb == 6) { harb_apply_k<NB, 0, 6>(R, S, e, slot); return; }
        if (sa == 4 && sb == 6) { harb_apply_k<NB, 4, 6>(R, S, e, slot); return; }
        if (sa == 5 && sb == 6) { harb_apply_k<NB, 5, 6>(R, S, e, slot); return; }
    }
    harb_apply(R, S, e, slot);
}

// The first NARB active arbiters of a substep in registers for the 10 iterations (the compile-time scenes
// rarely hold more: MoveToRegion has live arbiters in 3.5% of env-substeps, MoveToCorner 10%): their pair code,
// normal, friction and contacts' pre-stepped terms are read from LDS once per substep instead of once per
// iteration, the accumulated impulses stay in registers and are written back after the sweep.  Same operations
// in the same order as harb_apply.
struct RegArb {
    int code, cnt;
    double nx, ny, fr, nm[2], r1x[2], r1y[2], r2x[2], r2y[2], bias[2], tm[2], jb[2], jn[2], jt[2];
};
// pair code of an arbiter's (body A, body B) in the compile-time scenes (harb_row's cases), -1: other
MG_DEV int arb_pair_code(int sa, int sb) {
    if (sa == 0 && sb < 0) return 0;
    if (sa < 0 && sb == 4) return 1;
    if (sa < 0 && sb == 5) return 2;
    if (sa < 0 && sb == 6) return 3;
    if (sa == 0 && sb == 6) return 4;
    if (sa == 4 && sb == 6) return 5;
    if (sa == 5 && sb == 6) return 6;
    return -1;
}
MG_DEV void rarb_load(RegArb &a, const MGState &S, int e, int slot) {
    a.code = arb_pair_code(AT(S.asa, slot), AT(S.asb, slot));
    a.cnt = AT(S.acount, slot);
    a.nx = AT(S.anx, slot); a.ny = AT(S.any, slot); a.fr = AT(S.au, slot);
#pragma unroll
    for (int k = 0; k < 2; k++) {
        a.nm[k] = ACON(k, AC_NMASS, slot); a.bias[k] = ACON(k, AC_BIAS, slot); a.tm[k] = ACON(k, AC_TMASS, slot);
        a.r1x[k] = ACON(k, AC_R1X, slot); a.r1y[k] = ACON(k, AC_R1Y, slot);
        a.r2x[k] = ACON(k, AC_R2X, slot); a.r2y[k] = ACON(k, AC_R2Y, slot);
        a.jb[k] = ACON(k, AC_JB, slot); a.jn[k] = ACON(k, AC_JN, slot); a.jt[k] = ACON(k, AC_JT, slot);
    }
}
MG_DEV void rarb_store(const RegArb &a, const MGState &S, int e, int slot) {
#pragma unroll
    for (int k = 0; k < 2; k++)
        if (k < a.cnt) { ACON(k, AC_JB, slot) = a.jb[k]; ACON(k, AC_JN, slot) = a.jn[k]; ACON(k, AC_JT, slot) = a.jt[k]; }
}
template <int NB, int A, int B>
MG_DEV void rarb_apply_k(RegBodies<NB> &R, RegArb &a) {
    const double am = A >= 0 ? R.minv[A] : 0.0, ai = A >= 0 ? R.iinv[A] : 0.0;
    const double bm = B >= 0 ? R.minv[B] : 0.0, bi = B >= 0 ? R.iinv[B] : 0.0;
    const V2 n = v2(a.nx, a.ny);
#pragma unroll
    for (int k = 0; k < 2; k++) {
        if (k >= a.cnt) break;
        const double nMass = a.nm[k];
        V2 r1 = v2(a.r1x[k], a.r1y[k]), r2 = v2(a.r2x[k], a.r2y[k]);
        V2 vb1 = v2(0.0, 0.0), v1 = v2(0.0, 0.0), vb2 = v2(0.0, 0.0), v2_ = v2(0.0, 0.0);
        if constexpr (A >= 0) {
            vb1 = vadd(v2(R.vbx[A], R.vby[A]), vmult(vperp(r1), R.wb[A]));
            v1 = vadd(v2(R.vx[A], R.vy[A]), vmult(vperp(r1), R.w[A]));
        }
        if constexpr (B >= 0) {
            vb2 = vadd(v2(R.vbx[B], R.vby[B]), vmult(vperp(r2), R.wb[B]));
            v2_ = vadd(v2(R.vx[B], R.vy[B]), vmult(vperp(r2), R.w[B]));
        }
        V2 vr = vsub(v2_, v1);
        double vbn = vdot(vsub(vb2, vb1), n);
        double vrn = vdot(vr, n);
        double vrt = vdot(vr, vperp(n));
        double jbn = (a.bias[k] - vbn) * nMass;
        double jbnOld = a.jb[k];
        double jBias = cpmax(jbnOld + jbn, 0.0);
        a.jb[k] = jBias;
        double jn = -(0.0 + vrn) * nMass;
        double jnOld = a.jn[k];
        double jnAcc = cpmax(jnOld + jn, 0.0);
        a.jn[k] = jnAcc;
        double jtMax = a.fr * jnAcc;
        double jt = -vrt * a.tm[k];
        double jtOld = a.jt[k];
        double jtAcc = cpclamp(jtOld + jt, -jtMax, jtMax);
        a.jt[k] = jtAcc;
        V2 jb = vmult(n, jBias - jbnOld);
        if constexpr (A >= 0) {
            const V2 m = vneg(jb);
            R.vbx[A] = R.vbx[A] + m.x * am; R.vby[A] = R.vby[A] + m.y * am; R.wb[A] = R.wb[A] + ai * vcross(r1, m);
        }
        if constexpr (B >= 0) {
            R.vbx[B] = R.vbx[B] + jb.x * bm; R.vby[B] = R.vby[B] + jb.y * bm; R.wb[B] = R.wb[B] + bi * vcross(r2, jb);
        }
        V2 j = vrotate(n, v2(jnAcc - jnOld, jtAcc - jtOld));
        if constexpr (A >= 0) {
            const V2 m = vneg(j);
            R.vx[A] = R.vx[A] + m.x * am; R.vy[A] = R.vy[A] + m.y * am; R.w[A] = R.w[A] + ai * vcross(r1, m);
        }
        if constexpr (B >= 0) {
            R.vx[B] = R.vx[B] + j.x * bm; R.vy[B] = R.vy[B] + j.y * bm; R.w[B] = R.w[B] + bi * vcross(r2, j);
        }
    }
}
// a register arbiter's row (its code is one of arb_pair_code's: rarb_ok checked it at load)
template <int NB>
MG_DEV void rarb_row(RegBodies<NB> &R, RegArb &a) {
    switch (a.code) {
    case 0: rarb_apply_k<NB, 0, -1>(R, a); break;
    case 1: rarb_apply_k<NB, -1, 4>(R, a); break;
    case 2: rarb_apply_k<NB, -1, 5>(R, a); break;
    default:
        if constexpr (NB > 6) {
            switch (a.code) {
            case 3: rarb_apply_k<NB, -1, 6>(R, a); break;
            case 4: rarb_apply_k<NB, 0, 6>(R, a); break;
            case 5: rarb_apply_k<NB, 4, 6>(R, a); break;
            default: rarb_apply_k<NB, 5, 6>(R, a); break;
            }
        }
        break;
    }
}

template <int NCS, int C = 0>
MG_DEV void rstatic_load(RegCons *q, const MGState &S, int e, double dt) {
    if constexpr (C < NCS) {
        rc_load(q[C], S, e, C, static_cons(C).type, dt);
        rstatic_load<NCS, C + 1>(q, S, e, dt);
    }
}
template <int NCS, int C = 0>
MG_DEV void rstatic_store(const RegCons *q, const MGState &S, int e) {
    if constexpr (C < NCS) {
        rc_store(q[C], S, e, C, static_cons(C).type);
        rstatic_store<NCS, C + 1>(q, S, e);
    }
}
template <int NCS, int NB, int C = 0>
MG_DEV void rstatic_cached(RegBodies<NB> &R, const RegCons *q, double dt_coef) {
    if constexpr (C < NCS) {
        constexpr ConsDesc d = static_cons(C);
        rcons_cached(R, q[C], d.a, d.b, d.type, dt_coef);
        rstatic_cached<NCS, NB, C + 1>(R, q, dt_coef);
    }
}
template <int NCS, int NB, int C = 0>
MG_DEV void rstatic_apply(RegBodies<NB> &R, RegCons *q) {
    if constexpr (C < NCS) {
        constexpr ConsDesc d = static_cons(C);
        rcons_apply(R, q[C], d.a, d.b, d.type);
        rstatic_apply<NCS, NB, C + 1>(R, q);
    }
}

// bodies of the compile-time scenes: the robot's six, plus the block's
__host__ __device__ constexpr int static_nbodies(int ncs) { return ncs > 10 ? 7 : 6; }

// applyCachedImpulse + 10 iterations of the LDS variants, register-resident; NARB arbiters in registers (the
// 8-env form: 1 -- MoveToRegion 0.414 -> 0.392 ms, MoveToCorner 0.757 -> 0.740 ms per 2048-env chunk; 2 made
// the MoveToCorner form spill and measured slower, and the 16-env forms spill already at 1: 0 there)
template <int NCS, int NARB>
MG_DEV void static_solve(const MGState &S, int e, double dt, double dt_coef, int nact, MGProf &P) {
    constexpr int NB = static_nbodies(NCS);
    RegBodies<NB> R;
    RegCons q[NCS];
    rb_load(R, S, e);
    rstatic_load<NCS>(q, S, e, dt);
    for (int i = 0; i < nact; i++) harb_cached_row(R, S, e, AT(S.active, i), dt_coef);
    rstatic_cached<NCS>(R, q, dt_coef);
    MG_PP(P, 5);
    // the first NARB arbiters in registers when their pairs are compile-time ones (the rest through LDS)
    RegArb ra[NARB > 0 ? NARB : 1];
    int nreg = 0;
    if constexpr (NARB > 0) {
#pragma unroll
        for (int i = 0; i < NARB; i++) {
            ra[i].code = -1; ra[i].cnt = 0;
            if (i < nact) rarb_load(ra[i], S, e, AT(S.active, i));
        }
        bool ok = true;
#pragma unroll
        for (int i = 0; i < NARB; i++) {
            if (i < nact && ok && ra[i].code >= 0 && (NB > 6 || ra[i].code <= 2)) nreg = i + 1;
            else ok = false;
        }
    }
#pragma unroll 1
    for (int it = 0; it < MG_ITERATIONS; it++) {
        if constexpr (NARB > 0) {
#pragma unroll
            for (int i = 0; i < NARB; i++)
                if (i < nreg) rarb_row(R, ra[i]);
        }
        for (int i = nreg; i < nact; i++) harb_row(R, S, e, AT(S.active, i));
        rstatic_apply<NCS>(R, q);
    }
    if constexpr (NARB > 0) {
#pragma unroll
        for (int i = 0; i < NARB; i++)
            if (i < nreg) rarb_store(ra[i], S, e, AT(S.active, i));
    }
    rb_store(R, S, e);
    rstatic_store<NCS>(q, S, e);
}

#ifndef MG_COOP_COMPACT
#define MG_COOP_COMPACT 1
#endif
// ---- cpSpaceStep -----------------------------------------------------------
// one lane per env on the HBM state (variant 0, scenes beyond the LDS forms' caps): runtime constraint lists
MG_DEV void space_step(const MGState &S, const mg_library *L, int e, double dt, MGProf &P) {
    uint32_t stamp = S.stamp[e] + 1;
    S.stamp[e] = stamp;
    double prev_dt = S.curr_dt[e];
    S.curr_dt[e] = dt;
    int nact = S.nactive[e];
    for (int i = 0; i < nact; i++) AT(S.astate, AT(S.active, i)) = ARB_NORMAL;
    S.nactive[e] = 0;
    int nb = S.nbodies[e];
    for (int b = 0; b < nb; b++) {
        AT(S.bpx, b) = AT(S.bpx, b) + (AT(S.bvx, b) + AT(S.bvbx, b)) * dt;
        AT(S.bpy, b) = AT(S.bpy, b) + (AT(S.bvy, b) + AT(S.bvby, b)) * dt;
        body_set_angle_step(S, e, b, AT(S.ba, b) + (AT(S.bw, b) + AT(S.bwb, b)) * dt);
        AT(S.bvbx, b) = 0.0; AT(S.bvby, b) = 0.0; AT(S.bwb, b) = 0.0;
    }
    int ns = S.nshapes[e];
    for (int k = 0; k < ns; k++) shape_update_bb(S, L, e, k);
    MG_PP(P, 1);
    // broadphase + narrowphase, canonical order
    ShapeW A, W, B;   // narrowphase operands (per-lane scratch)
    for (int i = 0; i < ns; i++) {
        // BB tests on the cached BBs; the world-space shape is built only for pairs that pass
        const double al = AT(S.sbbl, i), ab = AT(S.sbbb, i), ar = AT(S.sbbr, i), at = AT(S.sbbt, i);
        bool have_a = false;
        const int gi = AT(S.sgroup, i), bi = AT(S.sbody, i);
        const double ui = AT(S.su, i);
        for (int w = 0; w < 4 && !(gi & MG_GROUP_OFF); w++) { // categories 0 collide with nothing
            double wl, wb, wr, wt;
            wall_bb(w, wl, wb, wr, wt);
            if (!(al <= wr && wl <= ar && ab <= wt && wb <= at)) continue;
            if (!have_a) { load_shape(S, L, e, i, (uint64_t)AT(S.shash, i), A); have_a = true; }
            load_wall(w, W);
            Collision info;
            collide(A, W, info);
            if (info.count) arbiter_update(S, L, e, i * 128 + 100 + w, A, W, ui, 0.8, info);
        }
        for (int j = i + 1; j < ns; j++) {
            if (!(al <= AT(S.sbbr, j) && AT(S.sbbl, j) <= ar && ab <= AT(S.sbbt, j) && AT(S.sbbb, j) <= at))
                continue;
            if (AT(S.sbody, j) == bi) continue;
            int gj = AT(S.sgroup, j);
            if ((gi != 0 && gi == gj) || ((gi | gj) & MG_GROUP_OFF)) continue; // cpShapeFilterReject
            if (surely_apart(S, L, e, i, j)) continue;                          // no contact (exact skip)
            if (!have_a) { load_shape(S, L, e, i, (uint64_t)AT(S.shash, i), A); have_a = true; }
            load_shape(S, L, e, j, (uint64_t)AT(S.shash, j), B);
            Collision info;
            collide(A, B, info);
            if (info.count) arbiter_update(S, L, e, i * 128 + j, A, B, ui, AT(S.su, j), info);
        }
    }
    MG_PP(P, 2);
    // cached arbiter filter
    for (int i = 0; i < S.arb_cap; i++) {
        if (AT(S.akey, i) < 0) continue;
        uint32_t ticks = stamp - AT(S.astamp, i);
        if (ticks >= 1 && AT(S.astate, i) != ARB_CACHED) AT(S.astate, i) = ARB_CACHED;
        if (ticks >= 3) { AT(S.akey, i) = -1; AT(S.acount, i) = 0; }
    }
    MG_PP(P, 3);
    nact = S.nactive[e];
    int nc = S.ncons[e];
    for (int i = 0; i < nact; i++) arbiter_prestep(S, L, e, AT(S.active, i), dt);
    for (int c = 0; c < nc; c++) cons_prestep(S, e, c, dt);
    MG_PP(P, 4);
    // velocity integration is the identity here (no gravity, damping 1, no forces)
    double dt_coef = (prev_dt == 0.0 ? 0.0 : dt / prev_dt);
    for (int i = 0; i < nact; i++) arbiter_cached(S, e, AT(S.active, i), dt_coef);
    for (int c = 0; c < nc; c++) cons_cached(S, e, c, dt_coef);
    MG_PP(P, 5);
    for (int it = 0; it < MG_ITERATIONS; it++) {
        for (int i = 0; i < nact; i++) arbiter_apply(S, e, AT(S.active, i));
        for (int c = 0; c < nc; c++) cons_apply(S, e, c, dt);
    }
    MG_PP(P, 6);
}

// ---- cooperative cpSpaceStep: one env per wavefront ---------------------------
// The env's state is an LDS view (N = 1, e = 0) shared by the 64 lanes of its wavefront.  The
// order-free parts run across lanes: position integration and rotation caches (one body per lane),
// shape BBs, the broadphase BB tests and narrowphase of all candidate pairs (one pair per lane, in
// chunks of 64 pairs in canonical order), the stale-arbiter filter and the pre-steps of arbiters and
// constraints.  Everything whose result depends on order runs on lane 0 in the serial code's order:
// arbiter updates (pairs taken from the lanes in canonical pair order, so arbiter slots, the active
// list and warm starts are those of space_step), the springs' pre-step impulses, applyCachedImpulse
// and the 10 solver iterations.
MG_DEV double rl_d(double v, int src) {
    const uint64_t u = (uint64_t)__double_as_longlong(v);
    const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)u, src);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(u >> 32), src);
    return __longlong_as_double((long long)(((uint64_t)hi << 32) | lo));
}
MG_DEV uint64_t rl_u64(uint64_t v, int src) {
    const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)v, src);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(v >> 32), src);
    return ((uint64_t)hi << 32) | lo;
}

// first pair index of shape i's row: for each shape i the 4 walls, then shapes j > i
MG_DEV int pair_row_off(int i, int ns) { return i * (ns + 3) - (i * (i - 1)) / 2; }

// The serial sweep of the cooperative step keeps the body velocities in the wavefront's VGPRs, spread
// over the lanes (lane b holds body b): every lane runs the sweep on the same (uniform) values, reading
// a body with readlane by its wave-uniform slot and writing it with a lane-select, so no body state
// makes an LDS round trip.  Same operations in the same order as cons_*_impl / arbiter_*.
struct LaneBodies { double vx, vy, w, vbx, vby, wb, minv, iinv; };
MG_DEV int ufirst(int v) { return __builtin_amdgcn_readfirstlane(v); }
MG_DEV double lget(double f, int b) { return b < 0 ? 0.0 : rl_d(f, b); }
MG_DEV void lput(double &f, int b, int lane, double v) { f = lane == b ? v : f; }
MG_DEV void lapply(LaneBodies &R, int lane, int b, V2 j, V2 r) {
    if (b < 0) return;
    const double minv = lget(R.minv, b), iinv = lget(R.iinv, b);
    lput(R.vx, b, lane, lget(R.vx, b) + j.x * minv);
    lput(R.vy, b, lane, lget(R.vy, b) + j.y * minv);
    lput(R.w, b, lane, lget(R.w, b) + iinv * vcross(r, j));
}
MG_DEV void lapply_bias(LaneBodies &R, int lane, int b, V2 j, V2 r) {
    if (b < 0) return;
    const double minv = lget(R.minv, b), iinv = lget(R.iinv, b);
    lput(R.vbx, b, lane, lget(R.vbx, b) + j.x * minv);
    lput(R.vby, b, lane, lget(R.vby, b) + j.y * minv);
    lput(R.wb, b, lane, lget(R.wb, b) + iinv * vcross(r, j));
}
MG_DEV void ladd_w(LaneBodies &R, int lane, int b, double dw) { // AT(S.bw, b) += dw
    if (b >= 0) lput(R.w, b, lane, lget(R.w, b) + dw);
}
MG_DEV void lsub_w(LaneBodies &R, int lane, int b, double dw) { // AT(S.bw, b) -= dw
    if (b >= 0) lput(R.w, b, lane, lget(R.w, b) - dw);
}

MG_DEV void lcons_cached(LaneBodies &R, int lane, const MGState &S, int e, int c, int a, int b, int type,
                         double dt_coef) {
    switch (type) {
    case MG_C_PIVOT: {
        V2 j = vmult(v2(CPA(CP_JACC, c), CPA(CP_JACC2, c)), dt_coef);
        lapply(R, lane, a, vneg(j), v2(CPA(CP_R1X, c), CPA(CP_R1Y, c)));
        lapply(R, lane, b, j, v2(CPA(CP_R2X, c), CPA(CP_R2Y, c)));
        break;
    }
    case MG_C_GEAR: {
        double j = CPA(CP_JACC, c) * dt_coef;
        lsub_w(R, lane, a, j * lget(R.iinv, a) * CPA(CP_RATIO_INV, c));
        ladd_w(R, lane, b, j * lget(R.iinv, b));
        break;
    }
    case MG_C_ROTLIMIT:
    case MG_C_MOTOR: {
        double j = CPA(CP_JACC, c) * dt_coef;
        lsub_w(R, lane, a, j * lget(R.iinv, a));
        ladd_w(R, lane, b, j * lget(R.iinv, b));
        break;
    }
    default: break;
    }
}

MG_DEV void lcons_apply(LaneBodies &R, int lane, const MGState &S, int e, int c, int a, int b, int type, double dt) {
    switch (type) {
    case MG_C_PIVOT: {
        V2 r1 = v2(CPA(CP_R1X, c), CPA(CP_R1Y, c)), r2 = v2(CPA(CP_R2X, c), CPA(CP_R2Y, c));
        V2 v1 = vadd(v2(lget(R.vx, a), lget(R.vy, a)), vmult(vperp(r1), lget(R.w, a)));
        V2 v2_ = vadd(v2(lget(R.vx, b), lget(R.vy, b)), vmult(vperp(r2), lget(R.w, b)));
        V2 vr = vsub(v2_, v1);
        V2 d = vsub(v2(CPA(CP_BIAS, c), CPA(CP_BIAS2, c)), vr);
        V2 j = v2(d.x * CPA(CP_K11, c) + d.y * CPA(CP_K12, c), d.x * CPA(CP_K21, c) + d.y * CPA(CP_K22, c));
        V2 jOld = v2(CPA(CP_JACC, c), CPA(CP_JACC2, c));
        V2 jAcc = vclamp(vadd(jOld, j), CPA(CP_MAXF, c) * dt);
        if (lane == 0) { CPA(CP_JACC, c) = jAcc.x; CPA(CP_JACC2, c) = jAcc.y; }
        V2 dj = vsub(jAcc, jOld);
        lapply(R, lane, a, vneg(dj), r1);
        lapply(R, lane, b, dj, r2);
        break;
    }
    case MG_C_GEAR: {
        double ratio = CPA(CP_RATIO, c);
        double wr = lget(R.w, b) * ratio - lget(R.w, a);
        double jMax = CPA(CP_MAXF, c) * dt;
        double j = (CPA(CP_BIAS, c) - wr) * CPA(CP_ISUM, c);
        double jOld = CPA(CP_JACC, c);
        double jAcc = cpclamp(jOld + j, -jMax, jMax);
        if (lane == 0) CPA(CP_JACC, c) = jAcc;
        j = jAcc - jOld;
        lsub_w(R, lane, a, j * lget(R.iinv, a) * CPA(CP_RATIO_INV, c));
        ladd_w(R, lane, b, j * lget(R.iinv, b));
        break;
    }
    case MG_C_ROTLIMIT: {
        double bias = CPA(CP_BIAS, c);
        if (!bias) return;
        double wr = lget(R.w, b) - lget(R.w, a);
        double jMax = CPA(CP_MAXF, c) * dt;
        double j = -(bias + wr) * CPA(CP_ISUM, c);
        double jOld = CPA(CP_JACC, c);
        double jAcc = bias < 0.0 ? cpclamp(jOld + j, 0.0, jMax) : cpclamp(jOld + j, -jMax, 0.0);
        if (lane == 0) CPA(CP_JACC, c) = jAcc;
        j = jAcc - jOld;
        lsub_w(R, lane, a, j * lget(R.iinv, a));
        ladd_w(R, lane, b, j * lget(R.iinv, b));
        break;
    }
    case MG_C_MOTOR: {
        double wr = lget(R.w, b) - lget(R.w, a) + CPA(CP_RATE, c);
        double jMax = CPA(CP_MAXF, c) * dt;
        double j = -wr * CPA(CP_ISUM, c);
        double jOld = CPA(CP_JACC, c);
        double jAcc = cpclamp(jOld + j, -jMax, jMax);
        if (lane == 0) CPA(CP_JACC, c) = jAcc;
        j = jAcc - jOld;
        lsub_w(R, lane, a, j * lget(R.iinv, a));
        ladd_w(R, lane, b, j * lget(R.iinv, b));
        break;
    }
    case MG_C_SPRING: {
        double wrn = lget(R.w, a) - lget(R.w, b);
        double w_damp = (CPA(CP_TWRN, c) - wrn) * CPA(CP_WCOEF, c);
        double j_damp = w_damp * CPA(CP_ISUM, c);
        double jacc = CPA(CP_JACC, c) + j_damp;
        if (lane == 0) { CPA(CP_TWRN, c) = wrn + w_damp; CPA(CP_JACC, c) = jacc; }
        ladd_w(R, lane, a, j_damp * lget(R.iinv, a));
        lsub_w(R, lane, b, j_damp * lget(R.iinv, b));
        break;
    }
    }
}

MG_DEV void larb_cached(LaneBodies &R, int lane, const MGState &S, int e, int slot, double dt_coef) {
    if (ufirst(AT(S.astate, slot)) == ARB_FIRST) return;
    const int a = ufirst(AT(S.asa, slot)), b = ufirst(AT(S.asb, slot));
    V2 n = v2(AT(S.anx, slot), AT(S.any, slot));
    const int cnt = ufirst(AT(S.acount, slot));
    for (int k = 0; k < cnt; k++) {
        V2 j = vmult(vrotate(n, v2(ACON(k, AC_JN, slot), ACON(k, AC_JT, slot))), dt_coef);
        lapply(R, lane, a, vneg(j), v2(ACON(k, AC_R1X, slot), ACON(k, AC_R1Y, slot)));
        lapply(R, lane, b, j, v2(ACON(k, AC_R2X, slot), ACON(k, AC_R2Y, slot)));
    }
}

MG_DEV void larb_apply(LaneBodies &R, int lane, const MGState &S, int e, int slot) {
    const int a = ufirst(AT(S.asa, slot)), b = ufirst(AT(S.asb, slot));
    V2 n = v2(AT(S.anx, slot), AT(S.any, slot));
    double friction = AT(S.au, slot);
    const int cnt = ufirst(AT(S.acount, slot));
    for (int k = 0; k < cnt; k++) {
        double nMass = ACON(k, AC_NMASS, slot);
        V2 r1 = v2(ACON(k, AC_R1X, slot), ACON(k, AC_R1Y, slot)), r2 = v2(ACON(k, AC_R2X, slot), ACON(k, AC_R2Y, slot));
        V2 vb1 = vadd(v2(lget(R.vbx, a), lget(R.vby, a)), vmult(vperp(r1), lget(R.wb, a)));
        V2 vb2 = vadd(v2(lget(R.vbx, b), lget(R.vby, b)), vmult(vperp(r2), lget(R.wb, b)));
        V2 v1 = vadd(v2(lget(R.vx, a), lget(R.vy, a)), vmult(vperp(r1), lget(R.w, a)));
        V2 v2_ = vadd(v2(lget(R.vx, b), lget(R.vy, b)), vmult(vperp(r2), lget(R.w, b)));
        V2 vr = vsub(v2_, v1);
        double vbn = vdot(vsub(vb2, vb1), n);
        double vrn = vdot(vr, n);
        double vrt = vdot(vr, vperp(n));
        double jbn = (ACON(k, AC_BIAS, slot) - vbn) * nMass;
        double jbnOld = ACON(k, AC_JB, slot);
        double jBias = cpmax(jbnOld + jbn, 0.0);
        double jn = -(0.0 + vrn) * nMass;
        double jnOld = ACON(k, AC_JN, slot);
        double jnAcc = cpmax(jnOld + jn, 0.0);
        double jtMax = friction * jnAcc;
        double jt = -vrt * ACON(k, AC_TMASS, slot);
        double jtOld = ACON(k, AC_JT, slot);
        double jtAcc = cpclamp(jtOld + jt, -jtMax, jtMax);
        if (lane == 0) { ACON(k, AC_JB, slot) = jBias; ACON(k, AC_JN, slot) = jnAcc; ACON(k, AC_JT, slot) = jtAcc; }
        V2 jb = vmult(n, jBias - jbnOld);
        lapply_bias(R, lane, a, vneg(jb), r1);
        lapply_bias(R, lane, b, jb, r2);
        V2 j = vrotate(n, v2(jnAcc - jnOld, jtAcc - jtOld));
        lapply(R, lane, a, vneg(j), r1);
        lapply(R, lane, b, j, r2);
    }
}

// A block's ground joints (Pivot + Gear to the static body, entities.py:580-754) touch only the
// block's body.  When no other constraint touches that body, they commute exactly with every other
// constraint row of the sweep (disjoint bodies; the static body's velocity is never read or written),
// so the lane holding the body applies them itself, in list order, while the rest of the constraint
// list runs in the serial sweep: bit-identical to the serial order, with the 2 x nblocks ground rows
// of an iteration costing two row evaluations instead of 2 x nblocks.
struct GroundRows { int n, c0, c1; uint64_t mask; };
MG_DEV GroundRows ground_rows(const MGState &S, int e, int lane, int nb, int nc) {
    int n = 0, c0 = -1, c1 = -1;
    bool bad = lane >= nb;
    for (int c = 0; c < nc && !bad; c++) {
        const int a = AT(S.ca, c), b = AT(S.cb, c), t = AT(S.ctype, c);
        if (a != lane && b != lane) continue;
        if (a < 0 && (t == MG_C_PIVOT || t == MG_C_GEAR) && n < 2) {
            if (n == 0) c0 = c; else c1 = c;
            n++;
        } else {
            bad = true;
        }
    }
    GroundRows g;
    g.n = bad ? 0 : n; g.c0 = c0; g.c1 = c1;
    g.mask = __ballot(g.n > 0);
    return g;
}
MG_DEV bool is_ground_row(const GroundRows &G, int b) { return b >= 0 && ((G.mask >> b) & 1ull); }

// lcons_cached / lcons_apply of a ground row on the lane that holds body b (body a static)
MG_DEV void lground_cached(LaneBodies &R, const MGState &S, int e, int c, double dt_coef) {
    if (AT(S.ctype, c) == MG_C_PIVOT) {
        V2 j = vmult(v2(CPA(CP_JACC, c), CPA(CP_JACC2, c)), dt_coef);
        V2 r2 = v2(CPA(CP_R2X, c), CPA(CP_R2Y, c));
        R.vx = R.vx + j.x * R.minv;
        R.vy = R.vy + j.y * R.minv;
        R.w = R.w + R.iinv * vcross(r2, j);
    } else { // MG_C_GEAR
        double j = CPA(CP_JACC, c) * dt_coef;
        R.w = R.w + j * R.iinv;
    }
}
MG_DEV void lground_apply(LaneBodies &R, const MGState &S, int e, int c, double dt) {
    if (AT(S.ctype, c) == MG_C_PIVOT) {
        V2 r1 = v2(CPA(CP_R1X, c), CPA(CP_R1Y, c)), r2 = v2(CPA(CP_R2X, c), CPA(CP_R2Y, c));
        V2 v1 = vadd(v2(0.0, 0.0), vmult(vperp(r1), 0.0));
        V2 v2_ = vadd(v2(R.vx, R.vy), vmult(vperp(r2), R.w));
        V2 vr = vsub(v2_, v1);
        V2 d = vsub(v2(CPA(CP_BIAS, c), CPA(CP_BIAS2, c)), vr);
        V2 j = v2(d.x * CPA(CP_K11, c) + d.y * CPA(CP_K12, c), d.x * CPA(CP_K21, c) + d.y * CPA(CP_K22, c));
        V2 jOld = v2(CPA(CP_JACC, c), CPA(CP_JACC2, c));
        V2 jAcc = vclamp(vadd(jOld, j), CPA(CP_MAXF, c) * dt);
        CPA(CP_JACC, c) = jAcc.x; CPA(CP_JACC2, c) = jAcc.y;
        V2 dj = vsub(jAcc, jOld);
        R.vx = R.vx + dj.x * R.minv;
        R.vy = R.vy + dj.y * R.minv;
        R.w = R.w + R.iinv * vcross(r2, dj);
    } else { // MG_C_GEAR
        double ratio = CPA(CP_RATIO, c);
        double wr = R.w * ratio - 0.0;
        double jMax = CPA(CP_MAXF, c) * dt;
        double j = (CPA(CP_BIAS, c) - wr) * CPA(CP_ISUM, c);
        double jOld = CPA(CP_JACC, c);
        double jAcc = cpclamp(jOld + j, -jMax, jMax);
        CPA(CP_JACC, c) = jAcc;
        j = jAcc - jOld;
        R.w = R.w + j * R.iinv;
    }
}

// Robot rows of the cooperative sweep on wave-uniform registers.  One env per wavefront: the robot's six
// bodies (rb0 .. rb0 + 5) and its ten joints' terms live in every lane's registers as in static_solve, so
// the robot rows (3/4 of the sweep's time when read through readlane / lane-select) index bodies by
// constants; block bodies stay in their lanes; arbiter rows reach a robot body through a uniform select.
// Same operations in the same order as lcons_* / larb_*.
MG_DEV bool is_rob(int b, int rb0) { return b >= rb0 && b < rb0 + 6; }
// the robot's velocities, masses and joint accumulators (wave-uniform); the bias velocities (touched by
// arbiter rows only) stay in the bodies' lanes.  Every access to RobotV uses a compile-time slot: a runtime
// index (even through a select chain, which the compiler folds back into one) puts the whole struct in
// per-lane scratch memory -- measured in round 3 as ~4 GB of scratch writes per launch at 8192 envs.
struct RobotV { double vx[6], vy[6], w[6], minv[6], iinv[6], jacc[10], jacc2[10], twrn[10]; };
// body side of an arbiter row: K >= 0 the robot's body slot K (in RobotV), K < 0 a block body (in its lane) or
// the static body (b < 0)
template <int K> MG_DEV double xget(double lf, const double (&rf)[6], int b) {
    if constexpr (K >= 0) return rf[K];
    else return b < 0 ? 0.0 : rl_d(lf, b);
}
template <int K> MG_DEV void xput(double &lf, double (&rf)[6], int b, int lane, double v) {
    if constexpr (K >= 0) rf[K] = v;
    else if (b >= 0) lput(lf, b, lane, v);
}
template <int K>
MG_DEV void xapply(LaneBodies &R, RobotV &V, int lane, int b, V2 j, V2 r) {
    if (K < 0 && b < 0) return;
    const double minv = xget<K>(R.minv, V.minv, b), iinv = xget<K>(R.iinv, V.iinv, b);
    xput<K>(R.vx, V.vx, b, lane, xget<K>(R.vx, V.vx, b) + j.x * minv);
    xput<K>(R.vy, V.vy, b, lane, xget<K>(R.vy, V.vy, b) + j.y * minv);
    xput<K>(R.w, V.w, b, lane, xget<K>(R.w, V.w, b) + iinv * vcross(r, j));
}
template <int K>
MG_DEV void xapply_bias(LaneBodies &R, RobotV &V, int lane, int b, V2 j, V2 r) {
    if (b < 0) return;
    const double minv = xget<K>(R.minv, V.minv, b), iinv = xget<K>(R.iinv, V.iinv, b);
    lput(R.vbx, b, lane, lget(R.vbx, b) + j.x * minv);
    lput(R.vby, b, lane, lget(R.vby, b) + j.y * minv);
    lput(R.wb, b, lane, lget(R.wb, b) + iinv * vcross(r, j));
}
template <int KA, int KB>
MG_DEV void xarb_cached_k(LaneBodies &R, RobotV &V, int lane, const MGState &S, int e, int slot, int a, int b,
                          int cnt, double dt_coef) {
    V2 n = v2(AT(S.anx, slot), AT(S.any, slot));
    for (int k = 0; k < cnt; k++) {
        V2 j = vmult(vrotate(n, v2(ACON(k, AC_JN, slot), ACON(k, AC_JT, slot))), dt_coef);
        xapply<KA>(R, V, lane, a, vneg(j), v2(ACON(k, AC_R1X, slot), ACON(k, AC_R1Y, slot)));
        xapply<KB>(R, V, lane, b, j, v2(ACON(k, AC_R2X, slot), ACON(k, AC_R2Y, slot)));
    }
}
// one side of an arbiter row, gathered once per row (not per contact) into wave-uniform registers: velocities and
// masses of a robot body (RobotV slot K >= 0) or of a block body (readlane from its lane), zeros for the static
// body (b < 0, never written back); bias velocities always live in the body's lane
struct XSide { double vx, vy, w, vbx, vby, wb, minv, iinv; };
template <int K>
MG_DEV XSide xside_get(const LaneBodies &R, const RobotV &V, int b) {
    XSide x;
    x.vx = xget<K>(R.vx, V.vx, b); x.vy = xget<K>(R.vy, V.vy, b); x.w = xget<K>(R.w, V.w, b);
    x.minv = xget<K>(R.minv, V.minv, b); x.iinv = xget<K>(R.iinv, V.iinv, b);
    x.vbx = lget(R.vbx, b); x.vby = lget(R.vby, b); x.wb = lget(R.wb, b);
    return x;
}
template <int K>
MG_DEV void xside_put(LaneBodies &R, RobotV &V, int b, int lane, const XSide &x) {
    if (K < 0 && b < 0) return;
    xput<K>(R.vx, V.vx, b, lane, x.vx); xput<K>(R.vy, V.vy, b, lane, x.vy); xput<K>(R.w, V.w, b, lane, x.w);
    lput(R.vbx, b, lane, x.vbx); lput(R.vby, b, lane, x.vby); lput(R.wb, b, lane, x.wb);
}
template <int KA, int KB>
MG_DEV void xarb_apply_k(LaneBodies &R, RobotV &V, int lane, const MGState &S, int e, int slot, int a, int b,
                         int cnt) {
    V2 n = v2(AT(S.anx, slot), AT(S.any, slot));
    double friction = AT(S.au, slot);
    // a and b are distinct bodies (or the static body), so each side's values can be carried across the row's
    // contacts in registers: the same reads and writes as per-contact lget / lput, in the same order
    XSide A = xside_get<KA>(R, V, a), B = xside_get<KB>(R, V, b);
    const bool da = KA >= 0 || a >= 0, db = KB >= 0 || b >= 0;   // sides that receive impulses
    for (int k = 0; k < cnt; k++) {
        double nMass = ACON(k, AC_NMASS, slot);
        V2 r1 = v2(ACON(k, AC_R1X, slot), ACON(k, AC_R1Y, slot)), r2 = v2(ACON(k, AC_R2X, slot), ACON(k, AC_R2Y, slot));
        V2 vb1 = vadd(v2(A.vbx, A.vby), vmult(vperp(r1), A.wb));
        V2 vb2 = vadd(v2(B.vbx, B.vby), vmult(vperp(r2), B.wb));
        V2 v1 = vadd(v2(A.vx, A.vy), vmult(vperp(r1), A.w));
        V2 v2_ = vadd(v2(B.vx, B.vy), vmult(vperp(r2), B.w));
        V2 vr = vsub(v2_, v1);
        double vbn = vdot(vsub(vb2, vb1), n);
        double vrn = vdot(vr, n);
        double vrt = vdot(vr, vperp(n));
        double jbn = (ACON(k, AC_BIAS, slot) - vbn) * nMass;
        double jbnOld = ACON(k, AC_JB, slot);
        double jBias = cpmax(jbnOld + jbn, 0.0);
        double jn = -(0.0 + vrn) * nMass;
        double jnOld = ACON(k, AC_JN, slot);
        double jnAcc = cpmax(jnOld + jn, 0.0);
        double jtMax = friction * jnAcc;
        double jt = -vrt * ACON(k, AC_TMASS, slot);
        double jtOld = ACON(k, AC_JT, slot);
        double jtAcc = cpclamp(jtOld + jt, -jtMax, jtMax);
        if (lane == 0) { ACON(k, AC_JB, slot) = jBias; ACON(k, AC_JN, slot) = jnAcc; ACON(k, AC_JT, slot) = jtAcc; }
        V2 jb = vmult(n, jBias - jbnOld);
        if (a >= 0) {   // xapply_bias: bias velocities of a non-static side
            const V2 m = vneg(jb);
            A.vbx = A.vbx + m.x * A.minv; A.vby = A.vby + m.y * A.minv; A.wb = A.wb + A.iinv * vcross(r1, m);
        }
        if (b >= 0) { B.vbx = B.vbx + jb.x * B.minv; B.vby = B.vby + jb.y * B.minv; B.wb = B.wb + B.iinv * vcross(r2, jb); }
        V2 j = vrotate(n, v2(jnAcc - jnOld, jtAcc - jtOld));
        if (da) {
            const V2 m = vneg(j);
            A.vx = A.vx + m.x * A.minv; A.vy = A.vy + m.y * A.minv; A.w = A.w + A.iinv * vcross(r1, m);
        }
        if (db) { B.vx = B.vx + j.x * B.minv; B.vy = B.vy + j.y * B.minv; B.w = B.w + B.iinv * vcross(r2, j); }
    }
    xside_put<KA>(R, V, a, lane, A);
    xside_put<KB>(R, V, b, lane, B);
}
// Arbiter rows dispatched on their bodies' robot slots (uniform branches, so every RobotV access has a constant
// slot): only the bodies that carry shapes can be in contact -- the robot body (slot 0) and the fingers (4, 5)
// -- and robot shapes never collide with each other (one shape group), so (a, b) is one of block / robot
// body / finger with a block or the static body.  Any other pair would be a scene outside the compiled robot
// rows: flagged (error 32), never expected.
// Active arbiter i's slot, bodies, contact count and first-step flag packed into one int held by lane i
// (arb_pack, built once per substep after the arbiter updates): a row reads them with one readlane instead of
// two dependent LDS round trips (active[i], then the slot's fields) per row and iteration.
MG_DEV int arb_pack(const MGState &S, int e, int i) {
    const int slot = AT(S.active, i);
    return slot | ((AT(S.asa, slot) + 1) << 8) | ((AT(S.asb, slot) + 1) << 12) | (AT(S.acount, slot) << 16) |
           ((AT(S.astate, slot) == ARB_FIRST ? 1 : 0) << 20);
}
template <bool CACHED>
MG_DEV void xarb_row(LaneBodies &R, RobotV &V, int rb0, int lane, const MGState &S, int e, int pk, double x) {
    if (CACHED && ((pk >> 20) & 1)) return;
    const int slot = pk & 255, a = ((pk >> 8) & 15) - 1, b = ((pk >> 12) & 15) - 1, cnt = (pk >> 16) & 15;
    const int ka = is_rob(a, rb0) ? a - rb0 : -1, kb = is_rob(b, rb0) ? b - rb0 : -1;
#define XROW(KA, KB) do { if (CACHED) xarb_cached_k<KA, KB>(R, V, lane, S, e, slot, a, b, cnt, x); \
                          else xarb_apply_k<KA, KB>(R, V, lane, S, e, slot, a, b, cnt); } while (0)
    if (ka < 0 && kb < 0) XROW(-1, -1);
    else if (kb < 0 && ka == 0) XROW(0, -1);
    else if (kb < 0 && ka == 4) XROW(4, -1);
    else if (kb < 0 && ka == 5) XROW(5, -1);
    else if (ka < 0 && kb == 0) XROW(-1, 0);
    else if (ka < 0 && kb == 4) XROW(-1, 4);
    else if (ka < 0 && kb == 5) XROW(-1, 5);
    else if (lane == 0) S.overflow[e] |= 32;
#undef XROW
}
// robot joint K (static_cons(K): compile-time type and body slots) at list index c: lcons_cached /
// lcons_apply with the bodies and accumulators in registers and the pre-stepped terms read from LDS
template <int K>
MG_DEV void rrow_apply(RobotV &V, const MGState &S, int e, int c, double dt) {
    constexpr ConsDesc d = static_cons(K);
    constexpr int a = d.a, b = d.b;
    if constexpr (d.type == MG_C_PIVOT) {
        V2 r1 = v2(CPA(CP_R1X, c), CPA(CP_R1Y, c)), r2 = v2(CPA(CP_R2X, c), CPA(CP_R2Y, c));
        V2 v1 = vadd(v2(V.vx[a], V.vy[a]), vmult(vperp(r1), V.w[a]));
        V2 v2_ = vadd(v2(V.vx[b], V.vy[b]), vmult(vperp(r2), V.w[b]));
        V2 vr = vsub(v2_, v1);
        V2 dd = vsub(v2(CPA(CP_BIAS, c), CPA(CP_BIAS2, c)), vr);
        V2 j = v2(dd.x * CPA(CP_K11, c) + dd.y * CPA(CP_K12, c), dd.x * CPA(CP_K21, c) + dd.y * CPA(CP_K22, c));
        V2 jOld = v2(V.jacc[K], V.jacc2[K]);
        V2 jAcc = vclamp(vadd(jOld, j), CPA(CP_MAXF, c) * dt);
        V.jacc[K] = jAcc.x; V.jacc2[K] = jAcc.y;
        V2 dj = vsub(jAcc, jOld);
        const V2 ja = vneg(dj);
        V.vx[a] = V.vx[a] + ja.x * V.minv[a]; V.vy[a] = V.vy[a] + ja.y * V.minv[a];
        V.w[a] = V.w[a] + V.iinv[a] * vcross(r1, ja);
        V.vx[b] = V.vx[b] + dj.x * V.minv[b]; V.vy[b] = V.vy[b] + dj.y * V.minv[b];
        V.w[b] = V.w[b] + V.iinv[b] * vcross(r2, dj);
    } else if constexpr (d.type == MG_C_GEAR) {
        double ratio = CPA(CP_RATIO, c);
        double wr = V.w[b] * ratio - V.w[a];
        double jMax = CPA(CP_MAXF, c) * dt;
        double j = (CPA(CP_BIAS, c) - wr) * CPA(CP_ISUM, c);
        double jOld = V.jacc[K];
        double jAcc = cpclamp(jOld + j, -jMax, jMax);
        V.jacc[K] = jAcc;
        j = jAcc - jOld;
        V.w[a] = V.w[a] - j * V.iinv[a] * CPA(CP_RATIO_INV, c);
        V.w[b] = V.w[b] + j * V.iinv[b];
    } else if constexpr (d.type == MG_C_ROTLIMIT) {
        double bias = CPA(CP_BIAS, c);
        if (!bias) return;
        double wr = V.w[b] - V.w[a];
        double jMax = CPA(CP_MAXF, c) * dt;
        double j = -(bias + wr) * CPA(CP_ISUM, c);
        double jOld = V.jacc[K];
        double jAcc = bias < 0.0 ? cpclamp(jOld + j, 0.0, jMax) : cpclamp(jOld + j, -jMax, 0.0);
        V.jacc[K] = jAcc;
        j = jAcc - jOld;
        V.w[a] = V.w[a] - j * V.iinv[a];
        V.w[b] = V.w[b] + j * V.iinv[b];
    } else if constexpr (d.type == MG_C_MOTOR) {
        double wr = V.w[b] - V.w[a] + CPA(CP_RATE, c);
        double jMax = CPA(CP_MAXF, c) * dt;
        double j = -wr * CPA(CP_ISUM, c);
        double jOld = V.jacc[K];
        double jAcc = cpclamp(jOld + j, -jMax, jMax);
        V.jacc[K] = jAcc;
        j = jAcc - jOld;
        V.w[a] = V.w[a] - j * V.iinv[a];
        V.w[b] = V.w[b] + j * V.iinv[b];
    } else if constexpr (d.type == MG_C_SPRING) {
        double wrn = V.w[a] - V.w[b];
        double w_damp = (V.twrn[K] - wrn) * CPA(CP_WCOEF, c);
        V.twrn[K] = wrn + w_damp;
        double j_damp = w_damp * CPA(CP_ISUM, c);
        V.jacc[K] = V.jacc[K] + j_damp;
        V.w[a] = V.w[a] + j_damp * V.iinv[a];
        V.w[b] = V.w[b] - j_damp * V.iinv[b];
    }
}
template <int K>
MG_DEV void rrow_cached(RobotV &V, const MGState &S, int e, int c, double dt_coef) {
    constexpr ConsDesc d = static_cons(K);
    constexpr int a = d.a, b = d.b;
    if constexpr (d.type == MG_C_PIVOT) {
        V2 j = vmult(v2(V.jacc[K], V.jacc2[K]), dt_coef);
        const V2 r1 = v2(CPA(CP_R1X, c), CPA(CP_R1Y, c)), r2 = v2(CPA(CP_R2X, c), CPA(CP_R2Y, c));
        const V2 ja = vneg(j);
        V.vx[a] = V.vx[a] + ja.x * V.minv[a]; V.vy[a] = V.vy[a] + ja.y * V.minv[a];
        V.w[a] = V.w[a] + V.iinv[a] * vcross(r1, ja);
        V.vx[b] = V.vx[b] + j.x * V.minv[b]; V.vy[b] = V.vy[b] + j.y * V.minv[b];
        V.w[b] = V.w[b] + V.iinv[b] * vcross(r2, j);
    } else if constexpr (d.type == MG_C_GEAR) {
        double j = V.jacc[K] * dt_coef;
        V.w[a] = V.w[a] - j * V.iinv[a] * CPA(CP_RATIO_INV, c);
        V.w[b] = V.w[b] + j * V.iinv[b];
    } else if constexpr (d.type == MG_C_ROTLIMIT || d.type == MG_C_MOTOR) {
        double j = V.jacc[K] * dt_coef;
        V.w[a] = V.w[a] - j * V.iinv[a];
        V.w[b] = V.w[b] + j * V.iinv[b];
    }
}
template <int K = 0>
MG_DEV void rrows_cached(RobotV &V, const MGState &S, int e, int rc0, double dt_coef) {
    if constexpr (K < 10) { rrow_cached<K>(V, S, e, rc0 + K, dt_coef); rrows_cached<K + 1>(V, S, e, rc0, dt_coef); }
}
template <int K = 0>
MG_DEV void rrows_apply(RobotV &V, const MGState &S, int e, int rc0, double dt) {
    if constexpr (K < 10) { rrow_apply<K>(V, S, e, rc0 + K, dt); rrows_apply<K + 1>(V, S, e, rc0, dt); }
}

// the env's constraint list is the blocks' ground rows (G) plus the robot's ten joints at rc0 in
// static_cons order on bodies rb0 + slot: the robot rows can run on registers
MG_DEV bool robot_rows_static(const MGState &S, int e, const GroundRows &G, int unc, int rb0, int rc0) {
    if (rb0 < 0 || rc0 < 0 || rc0 + 10 > unc) return false;
    bool ok = true;
    // static_cons is indexed by compile-time constants only (a runtime index into its local table could be
    // speculated out of range)
#pragma unroll
    for (int k = 0; k < 10; k++) {
        const ConsDesc d = static_cons(k);
        const int c = rc0 + k;
        ok = ok && ufirst(AT(S.ctype, c)) == d.type && ufirst(AT(S.ca, c)) == rb0 + d.a &&
             ufirst(AT(S.cb, c)) == rb0 + d.b;
    }
    for (int c = 0; c < unc; c++)
        if (c < rc0 || c >= rc0 + 10) ok = ok && is_ground_row(G, ufirst(AT(S.cb, c)));
    return ok;
}

// the sweep's structure (which rows are ground rows, whether the robot rows can run on registers): fixed for
// an env-step (robot_update changes the motors' rates, not the list), so built once before the 10 substeps
struct CoopPlan { GroundRows G; int rb0, rc0; bool rstatic; };
MG_DEV CoopPlan coop_plan(const MGState &S, int lane) {
    const int e = 0;
    CoopPlan Q;
    Q.G = ground_rows(S, e, lane, S.nbodies[e], S.ncons[e]);
    Q.rb0 = ufirst(S.robot_body0[e]); Q.rc0 = ufirst(S.robot_cons0[e]);
    Q.rstatic = robot_rows_static(S, e, Q.G, ufirst(S.ncons[e]), Q.rb0, Q.rc0);
    return Q;
}

MG_DEV void space_step_coop(const MGState &S, const mg_library *L, double dt, int lane, const CoopPlan &Q, MGProf &P) {
    const int e = 0;
    const uint32_t stamp = S.stamp[e] + 1;
    const double prev_dt = S.curr_dt[e];
    const int nact0 = S.nactive[e], nb = S.nbodies[e], ns = S.nshapes[e];
    __syncthreads();
    if (lane == 0) {
        S.stamp[e] = stamp;
        S.curr_dt[e] = dt;
        for (int i = 0; i < nact0; i++) AT(S.astate, AT(S.active, i)) = ARB_NORMAL;
        S.nactive[e] = 0;
    }
    for (int b = lane; b < nb; b += 64) {
        AT(S.bpx, b) = AT(S.bpx, b) + (AT(S.bvx, b) + AT(S.bvbx, b)) * dt;
        AT(S.bpy, b) = AT(S.bpy, b) + (AT(S.bvy, b) + AT(S.bvby, b)) * dt;
        body_set_angle_step(S, e, b, AT(S.ba, b) + (AT(S.bw, b) + AT(S.bwb, b)) * dt);
        AT(S.bvbx, b) = 0.0; AT(S.bvby, b) = 0.0; AT(S.bwb, b) = 0.0;
    }
    __syncthreads();
    for (int k = lane; k < ns; k += 64) shape_update_bb(S, L, e, k);
    __syncthreads();
    MG_PP(P, 1);
    // broadphase + narrowphase in canonical pair order (shape i's walls 0..3, then shapes j > i).
#if MG_COOP_COMPACT
    // Pass 1 tests every candidate pair, pair p on lane p mod 64 (BB, filters, exact separating-axis skip); the
    // pairs that need collide() are compacted in canonical order -- the q-th such pair to lane q (lane q selects
    // the bit of its rank in the chunk's ballot mask) -- so pass 2 runs collide() once for up to 64 of them (one call site) instead of once per 64-pair chunk
    // that holds any.  Lane 0 then applies the arbiter updates in canonical order, as before.
    const int total = pair_row_off(ns, ns);
    auto decode = [&](int p, int &i, int &r) {
        int lo = 0, hi = ns - 1;
        while (lo < hi) {
            const int mid = (lo + hi + 1) >> 1;
            if (pair_row_off(mid, ns) <= p) lo = mid; else hi = mid - 1;
        }
        i = lo;
        r = p - pair_row_off(i, ns);
    };
    // a round that fills up stops its pass 1 at the chunk holding its last hit; the next round resumes there
    // (it used to rescan every chunk from pair 0)
    int base0 = 0, seen0 = 0;
    for (int round0 = 0;; round0 += 64) {   // hits [round0, round0 + 64) of the substep's canonical hit list
        int mine = 0;                        // 1 + the pair index of this lane's hit in the round (0: none)
        int seen = seen0;                    // hits of the chunks before `base` (wave-uniform)
        bool more = false;                   // this round is full: another one follows
        int base = base0;
        for (; base < total; base += 64) {
            const int p = base + lane;
            bool hit = false;
            if (p < total) {
                int i, r;
                decode(p, i, r);
                const double al = AT(S.sbbl, i), ab = AT(S.sbbb, i), ar = AT(S.sbbr, i), at = AT(S.sbbt, i);
                if (r < 4) {
                    double wl, wb, wr, wt;
                    wall_bb(r, wl, wb, wr, wt);
                    hit = al <= wr && wl <= ar && ab <= wt && wb <= at && !(AT(S.sgroup, i) & MG_GROUP_OFF);
                } else {
                    const int j = i + 1 + (r - 4);
                    const int gi = AT(S.sgroup, i), gj = AT(S.sgroup, j);
                    hit = al <= AT(S.sbbr, j) && AT(S.sbbl, j) <= ar && ab <= AT(S.sbbt, j) && AT(S.sbbb, j) <= at &&
                          AT(S.sbody, j) != AT(S.sbody, i) && !(gi != 0 && gi == gj) && !((gi | gj) & MG_GROUP_OFF) &&
                          !surely_apart(S, L, e, i, j);
                }
            }
            const uint64_t m = __ballot(hit);
            const int nm = (int)__popcll(m);
            // lane q takes the hit of rank round0 + q: the k-th set bit of this chunk's mask, if it is here
            const int k = round0 + lane - seen;
            if (k >= 0 && k < nm) {
                int lo = 0, hi = 63;   // smallest bit position whose prefix holds k + 1 hits
#pragma unroll
                for (int it = 0; it < 6; it++) {
                    const int mid = (lo + hi) >> 1;
                    const uint64_t pre = mid == 63 ? ~0ull : ((2ull << mid) - 1ull);
                    if ((int)__popcll(m & pre) > k) hi = mid; else lo = mid + 1;
                }
                mine = base + lo + 1;
            }
            if (seen + nm >= round0 + 64) { more = true; break; }   // the next round's hits start in this chunk
            seen += nm;
        }
        base0 = base; seen0 = seen;
        int i = 0, j = 0;
        Collision info;
        info.count = 0;
        if (mine) {
            int r;
            decode(mine - 1, i, r);
            ShapeW A, B;
            load_shape(S, L, e, i, (uint64_t)AT(S.shash, i), A);
            if (r < 4) { j = -1 - r; load_wall(r, B); }
            else { j = i + 1 + (r - 4); load_shape(S, L, e, j, (uint64_t)AT(S.shash, j), B); }
            collide(A, B, info);   // the one call site
        }
        uint64_t m = __ballot(info.count > 0);
#ifdef MG_PROFILE
        P.acc[10] += (unsigned long long)__popcll(__ballot(mine != 0));
        P.acc[11] += (unsigned long long)__popcll(m);
#endif
        MG_PP(P, 8);
        while (m) { // hits in lane order = canonical pair order
            const int src = __ffsll((long long)m) - 1;
            m &= m - 1;
            Collision c;
            c.count = __builtin_amdgcn_readlane(info.count, src);
            c.n = v2(rl_d(info.n.x, src), rl_d(info.n.y, src));
            for (int k = 0; k < 2; k++) {
                c.p1[k] = v2(rl_d(info.p1[k].x, src), rl_d(info.p1[k].y, src));
                c.p2[k] = v2(rl_d(info.p2[k].x, src), rl_d(info.p2[k].y, src));
                c.hash[k] = rl_u64(info.hash[k], src);
            }
            const int si = __builtin_amdgcn_readlane(i, src), sj = __builtin_amdgcn_readlane(j, src);
            const int key = sj < 0 ? si * 128 + 100 + (-1 - sj) : si * 128 + sj;
            // the arbiter slot search across the wavefront (the serial search's first match / first empty slot;
            // lane 0's update of the previous hit is ordered before these reads by the wave's in-order LDS)
            const int ak = lane < S.arb_cap ? AT(S.akey, lane) : 0;
            const uint64_t hm = __ballot(lane < S.arb_cap && ak == key), fm = __ballot(lane < S.arb_cap && ak < 0);
            const int fslot = hm ? __ffsll((long long)hm) - 1 : -1, ffree = fm ? __ffsll((long long)fm) - 1 : -1;
            if (lane == 0) {
                // arbiter_update reads the shapes' types and bodies only
                const int ta = AT(S.spoly, si) < 0 ? WS_CIRCLE : WS_POLY, ba = AT(S.sbody, si);
                int tb, bb;
                double ub;
                if (sj < 0) { tb = WS_SEGMENT; bb = -1; ub = 0.8; }
                else { tb = AT(S.spoly, sj) < 0 ? WS_CIRCLE : WS_POLY; bb = AT(S.sbody, sj); ub = AT(S.su, sj); }
                arbiter_update_found(S, L, e, key, ta, ba, tb, bb, AT(S.su, si), ub, c, fslot, ffree);
            }
        }
        MG_PP(P, 9);
        if (!more) break;   // every hit of the substep has been collided
    }
#else
    // pair p (canonical order) on lane p mod 64
    const int total = pair_row_off(ns, ns);
    for (int base = 0; base < total; base += 64) {
        const int p = base + lane;
        int i = 0, j = 0;
        Collision info;
        info.count = 0;
        int called = 0;
        if (p < total) {
            int lo = 0, hi = ns - 1;
            while (lo < hi) {
                const int mid = (lo + hi + 1) >> 1;
                if (pair_row_off(mid, ns) <= p) lo = mid; else hi = mid - 1;
            }
            i = lo;
            const int r = p - pair_row_off(i, ns);
            const double al = AT(S.sbbl, i), ab = AT(S.sbbb, i), ar = AT(S.sbbr, i), at = AT(S.sbbt, i);
            if (r < 4) {
                j = -1 - r;
                double wl, wb, wr, wt;
                wall_bb(r, wl, wb, wr, wt);
                if (al <= wr && wl <= ar && ab <= wt && wb <= at && !(AT(S.sgroup, i) & MG_GROUP_OFF)) {
                    ShapeW A, W;
                    load_shape(S, L, e, i, (uint64_t)AT(S.shash, i), A);
                    load_wall(r, W);
                    collide(A, W, info);
                    called = 1;
                }
            } else {
                j = i + 1 + (r - 4);
                const int gi = AT(S.sgroup, i), gj = AT(S.sgroup, j);
                if (al <= AT(S.sbbr, j) && AT(S.sbbl, j) <= ar && ab <= AT(S.sbbt, j) && AT(S.sbbb, j) <= at &&
                    AT(S.sbody, j) != AT(S.sbody, i) && !(gi != 0 && gi == gj) && !((gi | gj) & MG_GROUP_OFF) &&
                    !surely_apart(S, L, e, i, j)) {
                    ShapeW A, B;
                    load_shape(S, L, e, i, (uint64_t)AT(S.shash, i), A);
                    load_shape(S, L, e, j, (uint64_t)AT(S.shash, j), B);
                    collide(A, B, info);
                    called = 1;
                }
            }
        }
        uint64_t m = __ballot(info.count > 0);
#ifdef MG_PROFILE
        P.acc[10] += (unsigned long long)__popcll(__ballot(called));
        P.acc[11] += (unsigned long long)__popcll(m);
#endif
        (void)called;
        MG_PP(P, 8);
        while (m) { // hits in lane order = canonical pair order
            const int src = __ffsll((long long)m) - 1;
            m &= m - 1;
            Collision c;
            c.count = __builtin_amdgcn_readlane(info.count, src);
            c.n = v2(rl_d(info.n.x, src), rl_d(info.n.y, src));
            for (int k = 0; k < 2; k++) {
                c.p1[k] = v2(rl_d(info.p1[k].x, src), rl_d(info.p1[k].y, src));
                c.p2[k] = v2(rl_d(info.p2[k].x, src), rl_d(info.p2[k].y, src));
                c.hash[k] = rl_u64(info.hash[k], src);
            }
            const int si = __builtin_amdgcn_readlane(i, src), sj = __builtin_amdgcn_readlane(j, src);
            if (lane == 0) {
                ShapeW A, B; // arbiter_update reads the shapes' types and bodies only
                A.type = AT(S.spoly, si) < 0 ? WS_CIRCLE : WS_POLY;
                A.body = AT(S.sbody, si);
                double ub;
                int key;
                if (sj < 0) {
                    B.type = WS_SEGMENT; B.body = -1; ub = 0.8; key = si * 128 + 100 + (-1 - sj);
                } else {
                    B.type = AT(S.spoly, sj) < 0 ? WS_CIRCLE : WS_POLY; B.body = AT(S.sbody, sj);
                    ub = AT(S.su, sj); key = si * 128 + sj;
                }
                arbiter_update(S, L, e, key, A, B, AT(S.su, si), ub, c);
            }
        }
        MG_PP(P, 9);
    }
#endif
    __syncthreads();
    MG_PP(P, 2);
    for (int i = lane; i < S.arb_cap; i += 64) { // cached arbiter filter
        if (AT(S.akey, i) < 0) continue;
        const uint32_t ticks = stamp - AT(S.astamp, i);
        if (ticks >= 1 && AT(S.astate, i) != ARB_CACHED) AT(S.astate, i) = ARB_CACHED;
        if (ticks >= 3) { AT(S.akey, i) = -1; AT(S.acount, i) = 0; }
    }
    __syncthreads();
    MG_PP(P, 3);
    const int nact = S.nactive[e], nc = S.ncons[e];
    for (int i = lane; i < nact; i += 64) arbiter_prestep(S, L, e, AT(S.active, i), dt);
    for (int c = lane; c < nc; c += 64)
        if (AT(S.ctype, c) != MG_C_SPRING) cons_prestep(S, e, c, dt); // touch only their own terms
    __syncthreads();
    if (lane == 0)
        for (int c = 0; c < nc; c++) // the springs apply their impulses to body velocities: in order
            if (AT(S.ctype, c) == MG_C_SPRING) cons_prestep(S, e, c, dt);
    __syncthreads();
    MG_PP(P, 4);
    // applyCachedImpulse + 10 iterations with the bodies in the lanes' registers
    LaneBodies R = {0.0, 0.0, 0.0, 0.0, 0.0, 0.0, 0.0, 0.0};
    if (lane < nb) {
        R.vx = AT(S.bvx, lane); R.vy = AT(S.bvy, lane); R.w = AT(S.bw, lane);
        R.vbx = AT(S.bvbx, lane); R.vby = AT(S.bvby, lane); R.wb = AT(S.bwb, lane);
        R.minv = AT(S.bminv, lane); R.iinv = AT(S.biinv, lane);
    }
    const double dt_coef = (prev_dt == 0.0 ? 0.0 : dt / prev_dt);
    const int unact = ufirst(nact), unc = ufirst(nc);
    const GroundRows &G = Q.G;
    const int rb0 = Q.rb0, rc0 = Q.rc0;
    if (Q.rstatic) {
        RobotV V;
#pragma unroll
        for (int k = 0; k < 6; k++) {
            const int b = rb0 + k;
            V.vx[k] = AT(S.bvx, b); V.vy[k] = AT(S.bvy, b); V.w[k] = AT(S.bw, b);
            V.minv[k] = AT(S.bminv, b); V.iinv[k] = AT(S.biinv, b);
        }
#pragma unroll
        for (int k = 0; k < 10; k++) {
            V.jacc[k] = CPA(CP_JACC, rc0 + k);
            V.jacc2[k] = static_cons(k).type == MG_C_PIVOT ? CPA(CP_JACC2, rc0 + k) : 0.0;
            V.twrn[k] = static_cons(k).type == MG_C_SPRING ? CPA(CP_TWRN, rc0 + k) : 0.0;
        }
        const int apk = lane < unact ? arb_pack(S, e, lane) : 0;   // active arbiter `lane` (arb_pack)
        for (int i = 0; i < unact; i++) xarb_row<true>(R, V, rb0, lane, S, e, __builtin_amdgcn_readlane(apk, i), dt_coef);
        if (G.n > 0) {
            lground_cached(R, S, e, G.c0, dt_coef);
            if (G.n > 1) lground_cached(R, S, e, G.c1, dt_coef);
        }
        rrows_cached(V, S, e, rc0, dt_coef);
        MG_PP(P, 5);
#pragma unroll 1
        for (int it = 0; it < MG_ITERATIONS; it++) {
            for (int i = 0; i < unact; i++) xarb_row<false>(R, V, rb0, lane, S, e, __builtin_amdgcn_readlane(apk, i), 0.0);
            if (G.n > 0) {
                lground_apply(R, S, e, G.c0, dt);
                if (G.n > 1) lground_apply(R, S, e, G.c1, dt);
            }
            rrows_apply(V, S, e, rc0, dt);
        }
        // robot lanes: velocities from V (their bias velocities stayed in the lanes)
        if (lane < nb) {
            double vx = R.vx, vy = R.vy, w = R.w;
#pragma unroll
            for (int k = 0; k < 6; k++)   // constant slots (see RobotV)
                if (lane == rb0 + k) { vx = V.vx[k]; vy = V.vy[k]; w = V.w[k]; }
            AT(S.bvx, lane) = vx; AT(S.bvy, lane) = vy; AT(S.bw, lane) = w;
            AT(S.bvbx, lane) = R.vbx; AT(S.bvby, lane) = R.vby; AT(S.bwb, lane) = R.wb;
        }
        if (lane == 0) {
#pragma unroll
            for (int k = 0; k < 10; k++) {
                CPA(CP_JACC, rc0 + k) = V.jacc[k];
                if (static_cons(k).type == MG_C_PIVOT) CPA(CP_JACC2, rc0 + k) = V.jacc2[k];
                if (static_cons(k).type == MG_C_SPRING) CPA(CP_TWRN, rc0 + k) = V.twrn[k];
            }
        }
        MG_PP(P, 6);
        __syncthreads();
        return;
    }
    for (int i = 0; i < unact; i++) larb_cached(R, lane, S, e, ufirst(AT(S.active, i)), dt_coef);
    if (G.n > 0) {
        lground_cached(R, S, e, G.c0, dt_coef);
        if (G.n > 1) lground_cached(R, S, e, G.c1, dt_coef);
    }
    for (int c = 0; c < unc; c++) {
        const int cb = ufirst(AT(S.cb, c));
        if (is_ground_row(G, cb)) continue;
        lcons_cached(R, lane, S, e, c, ufirst(AT(S.ca, c)), cb, ufirst(AT(S.ctype, c)), dt_coef);
    }
    MG_PP(P, 5);
#pragma unroll 1
    for (int it = 0; it < MG_ITERATIONS; it++) {
        for (int i = 0; i < unact; i++) larb_apply(R, lane, S, e, ufirst(AT(S.active, i)));
        if (G.n > 0) {
            lground_apply(R, S, e, G.c0, dt);
            if (G.n > 1) lground_apply(R, S, e, G.c1, dt);
        }
        for (int c = 0; c < unc; c++) {
            const int cb = ufirst(AT(S.cb, c));
            if (is_ground_row(G, cb)) continue;
            lcons_apply(R, lane, S, e, c, ufirst(AT(S.ca, c)), cb, ufirst(AT(S.ctype, c)), dt);
        }
    }
    if (lane < nb) {
        AT(S.bvx, lane) = R.vx; AT(S.bvy, lane) = R.vy; AT(S.bw, lane) = R.w;
        AT(S.bvbx, lane) = R.vbx; AT(S.bvby, lane) = R.vby; AT(S.bwb, lane) = R.wb;
    }
    MG_PP(P, 6);
    __syncthreads();
}

// ---- robot control ---------------------------------------------------------
MG_DEV void robot_set_action(const MGState &S, const mg_library *L, int e, int action) {
    const int ud = action % 3, lr = (action / 3) % 3;
    double radius = L->robot_radius;
    double ts = 0.0, turn = 0.0;
    if (ud == 1) ts += 4.0 * radius;
    if (ud == 2) ts -= 3.0 * radius;
    if (lr == 1) turn += 1.5;
    if (lr == 2) turn -= 1.5;
    S.target_speed[e] = ts;
    S.rel_turn[e] = turn;
    S.target_finger[e] = action < 9 ? L->finger_angle_off[0] : -0.0; // OPEN: pi/8, CLOSE: -finger_rot_limit_inner
}

// STATIC: the compile-time scenes (step forms 5 / 6: robot bodies at slots 0-5, its joints at 0-9, checked by
// the step kernel) -- constant slots, no dependent LDS reads before the first access
template <bool STATIC = false>
MG_DEV void robot_update(const MGState &S, const mg_library *L, int e) {
    const int body = STATIC ? 0 : S.robot_body0[e], control = body + 1, cons0 = STATIC ? 0 : S.robot_cons0[e];
    AT(S.ba, control) = AT(S.ba, body) + S.rel_turn[e]; // transform unused (body_rot_unused)
    double c = AT(S.brc, body), s = AT(S.brs, body), ts = S.target_speed[e];
    AT(S.bvx, control) = c * 0.0 - s * ts;
    AT(S.bvy, control) = c * ts + s * 0.0;
    double tf = S.target_finger[e];
    for (int k = 0; k < 2; k++) {
        double side = k == 0 ? -1.0 : 1.0;
        double rel = AT(S.ba, body + 4 + k) - AT(S.ba, body);
        double x = (rel + side * tf) * 10;
        double tr = (x < 1) ? x : 1.0;
        tr = (tr > -1) ? tr : -1.0;
        if (fabs(tr) < 1e-4) tr = 0.0;
        CPA(CP_RATE, cons0 + 6 + 3 * k) = tr;
    }
}
