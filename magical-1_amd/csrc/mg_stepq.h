// mg_stepq.h -- cpSpaceStep with QL lanes per env (the compile-time robot scenes, step forms 5 and 6).
//
// The forms 1 / 2 run one env per lane, 16 envs in a 16-lane wave per CU: every phase of an env's
// substep is one lane's serial chain.  Here each env owns QL = 64 / BLK lanes of the workgroup's one
// wavefront (16 envs x 4 lanes) and the order-free phases are split over them:
//   * position integration and rotation caches (body b on lane b mod QL; the correctly rounded sincos of
//     the robot body and fingers run side by side), cached shape BBs (shape k on lane k mod QL);
//   * broadphase + narrowphase: shape i's candidate list (walls 0..3, then shapes j > i) in chunks of QL,
//     candidate c on lane c mod QL (BB test, filters, exact skip, world shapes, collide);
//   * the stale-arbiter filter (slot on lane slot mod QL), arbiter pre-steps (active entry on lane
//     entry mod QL) and the non-spring constraint pre-steps (constraint C on lane C mod QL).
// The order-dependent parts stay on the env's lane 0 in the reference order: the arbiter updates (slot
// search, warm-start matching, active-list append) take the chunk's contacts from lanes 0..QL-1 in
// candidate order through cross-lane reads, the two DampedRotarySpring pre-steps (both write the robot
// body's angular velocity) run in list order, and the solver sweep is static_solve.  Every body, shape,
// arbiter and constraint is computed by exactly the operations of space_step<NCS>, so results are
// bit-identical to it (and to the oracle).
#pragma once
#include "mg_step.h"

// 64-bit values across lanes (ds_bpermute on the two halves)
MG_DEV double qshfl(double v, int src) {
    const uint64_t u = __double_as_longlong(v);
    const uint32_t lo = (uint32_t)__shfl((int)(uint32_t)u, src, 64), hi = (uint32_t)__shfl((int)(uint32_t)(u >> 32), src, 64);
    return __longlong_as_double((long long)(((uint64_t)hi << 32) | lo));
}
MG_DEV uint64_t qshfl_u64(uint64_t u, int src) {
    const uint32_t lo = (uint32_t)__shfl((int)(uint32_t)u, src, 64), hi = (uint32_t)__shfl((int)(uint32_t)(u >> 32), src, 64);
    return ((uint64_t)hi << 32) | lo;
}

// constraint pre-steps split over the env's lanes; the springs apply their impulse to the body's angular
// velocity, so they run on lane 0 in list order (nothing else in the pre-step reads or writes velocities)
template <int NC, int QL, int C = 0>
MG_DEV void static_prestep_quad(const MGState &S, int e, int sub, double dt) {
    if constexpr (C < NC) {
        constexpr ConsDesc d = static_cons(C);
        constexpr int owner = d.type == MG_C_SPRING ? 0 : C % QL;
        if (sub == owner) cons_prestep_impl(S, e, C, d.a, d.b, d.type, dt);
        static_prestep_quad<NC, QL, C + 1>(S, e, sub, dt);
    }
}

// broadphase + narrowphase of env e (canonical pair order), QL lanes per env.  Called with every lane of
// the env active (the trip counts depend on the env's shape count only).
template <int NCS, int QL, bool LDS_SHAPES>
MG_DEV void narrowphase_quad(const MGState &S, const mg_library *L, int e, int sub, int ns) {
    ShapeW locA, locB;
    ShapeW &A = LDS_SHAPES ? S.shw[2 * QL * e + 2 * sub] : locA;
    ShapeW &B = LDS_SHAPES ? S.shw[2 * QL * e + 2 * sub + 1] : locB;
    const int base = (int)(threadIdx.x & 63) - sub;   // the env's lane 0
    for (int i = 0; i < ns; i++) {
        const double al = AT(S.sbbl, i), ab = AT(S.sbbb, i), ar = AT(S.sbbr, i), at = AT(S.sbbt, i);
        const int gi = AT(S.sgroup, i), bi = AT(S.sbody, i);
        const double ui = AT(S.su, i);
        const int ta = AT(S.spoly, i) < 0 ? WS_CIRCLE : WS_POLY;
        const int ncand = 4 + ns - i - 1;   // walls 0..3, then shapes i+1 .. ns-1
        for (int c0 = 0; c0 < ncand; c0 += QL) {
            const int c = c0 + sub;
            Collision info;
            info.count = 0;
            int key = 0, tb = 0, bb = -1;
            double ub = 0.0;
            if (c < 4) {
                if (!(gi & MG_GROUP_OFF)) {   // categories 0 collide with nothing
                    double wl, wb, wr, wt;
                    wall_bb(c, wl, wb, wr, wt);
                    if (al <= wr && wl <= ar && ab <= wt && wb <= at) {
                        load_shape(S, L, e, i, (uint64_t)AT(S.shash, i), A);
                        load_wall(c, B);
                        collide(A, B, info);
                        key = i * 128 + 100 + c; ub = 0.8; tb = WS_SEGMENT; bb = -1;
                    }
                }
            } else if (c < ncand) {
                const int j = i + 1 + (c - 4);
                const int gj = AT(S.sgroup, j);
                if (al <= AT(S.sbbr, j) && AT(S.sbbl, j) <= ar && ab <= AT(S.sbbt, j) && AT(S.sbbb, j) <= at &&
                    AT(S.sbody, j) != bi && !((gi != 0 && gi == gj) || ((gi | gj) & MG_GROUP_OFF)) &&
                    !surely_apart(S, L, e, i, j)) {
                    load_shape(S, L, e, i, (uint64_t)AT(S.shash, i), A);
                    load_shape(S, L, e, j, (uint64_t)AT(S.shash, j), B);
                    collide(A, B, info);
                    key = i * 128 + j; ub = AT(S.su, j); tb = B.type; bb = B.body;
                }
            }
            // the chunk's contacts to lane 0, in candidate order
            const uint32_t m = (uint32_t)(__ballot(info.count > 0) >> base) & ((1u << QL) - 1u);
            for (int s = 0; s < QL; s++) {
                if (!((m >> s) & 1u)) continue;   // uniform over the env's lanes
                const int src = base + s;
                Collision q;
                q.count = __shfl(info.count, src, 64);
                q.n = v2(qshfl(info.n.x, src), qshfl(info.n.y, src));
#pragma unroll
                for (int k = 0; k < 2; k++) {
                    q.p1[k] = v2(qshfl(info.p1[k].x, src), qshfl(info.p1[k].y, src));
                    q.p2[k] = v2(qshfl(info.p2[k].x, src), qshfl(info.p2[k].y, src));
                    q.hash[k] = qshfl_u64(info.hash[k], src);
                }
                const int qkey = __shfl(key, src, 64), qtb = __shfl(tb, src, 64), qbb = __shfl(bb, src, 64);
                const double qub = qshfl(ub, src);
                if (sub == 0) arbiter_update_t(S, L, e, qkey, ta, bi, qtb, qbb, ui, qub, q);
            }
        }
    }
}

template <int NCS, int QL, bool LDS_SHAPES>
MG_DEV void space_step_quad(const MGState &S, const mg_library *L, int e, int sub, double dt, MGProf &P) {
    __syncthreads();   // the previous substep's solver / robot update are done
    const double prev_dt = S.curr_dt[e];
    const uint32_t stamp = S.stamp[e] + 1;
    const int nact0 = S.nactive[e], nb = S.nbodies[e], ns = S.nshapes[e];
    for (int i = sub; i < nact0; i += QL) AT(S.astate, AT(S.active, i)) = ARB_NORMAL;
    for (int b = sub; b < nb; b += QL) {
        AT(S.bpx, b) = AT(S.bpx, b) + (AT(S.bvx, b) + AT(S.bvbx, b)) * dt;
        AT(S.bpy, b) = AT(S.bpy, b) + (AT(S.bvy, b) + AT(S.bvby, b)) * dt;
        body_set_angle_step(S, e, b, AT(S.ba, b) + (AT(S.bw, b) + AT(S.bwb, b)) * dt);
        AT(S.bvbx, b) = 0.0; AT(S.bvby, b) = 0.0; AT(S.bwb, b) = 0.0;
    }
    __syncthreads();   // every lane has read the scalars; bodies before the shape BBs
    if (sub == 0) { S.stamp[e] = stamp; S.curr_dt[e] = dt; S.nactive[e] = 0; }
    for (int k = sub; k < ns; k += QL) shape_update_bb(S, L, e, k);
    __syncthreads();
    MG_PP(P, 1);
#ifndef MG_EXP_NO_NARROW    // timing experiments only (tools/build_unit_variant.sh): no collisions at all
    narrowphase_quad<NCS, QL, LDS_SHAPES>(S, L, e, sub, ns);
#endif
    __syncthreads();
    MG_PP(P, 2);
    for (int i = sub; i < S.arb_cap; i += QL) {   // cached arbiter filter
        if (AT(S.akey, i) < 0) continue;
        const uint32_t ticks = stamp - AT(S.astamp, i);
        if (ticks >= 1 && AT(S.astate, i) != ARB_CACHED) AT(S.astate, i) = ARB_CACHED;
        if (ticks >= 3) { AT(S.akey, i) = -1; AT(S.acount, i) = 0; }
    }
    __syncthreads();
    MG_PP(P, 3);
    const int nact = S.nactive[e];
    for (int i = sub; i < nact; i += QL) arbiter_prestep(S, L, e, AT(S.active, i), dt);
    static_prestep_quad<NCS, QL>(S, e, sub, dt);
    __syncthreads();
    MG_PP(P, 4);
    // velocity integration is the identity here (no gravity, damping 1, no forces)
    const double dt_coef = (prev_dt == 0.0 ? 0.0 : dt / prev_dt);
    if (sub == 0) static_solve<NCS>(S, e, dt, dt_coef, nact, P);
    MG_PP(P, 6);
}

// Robot.set_action + 10 x (Robot.update, cpSpaceStep) with QL lanes per env
template <int NCS, int QL, bool LDS_SHAPES>
__device__ __forceinline__ void env_substeps_quad(const MGState &V, const mg_library *L, int ev, int sub, int a,
                                                  MGProf &P) {
    if (sub == 0) robot_set_action(V, L, ev, a < 18 ? a : 0);
    const double dt = L->dt;
    for (int i = 0; i < 10; i++) {
        __syncthreads();
        if (sub == 0) robot_update(V, L, ev);
        MG_PP(P, 0);
        space_step_quad<NCS, QL, LDS_SHAPES>(V, L, ev, sub, dt, P);
    }
    __syncthreads();
}
