// mg_stepq.h -- cpSpaceStep with QL lanes per env (the compile-time robot scenes, step forms 5 and 6).
//
// The forms 1 / 2 run one env per lane, 16 envs in a 16-lane wave per CU: every phase of an env's
// substep is one lane's serial chain.  Here each env owns QL = 64 / BLK lanes of the workgroup's one
// wavefront (16 envs x 4 lanes) and the order-free phases are split over them:
//   * position integration and rotation caches (quad_body: the robot body, fingers and block -- the bodies
//     that need the correctly rounded sincos -- one per lane, side by side), cached shape BBs (shape k on
//     lane k mod QL);
//   * broadphase + narrowphase: the candidate list (shape i's walls 0..3, then shapes j > i) tested QL at a
//     time into a mask of hits, then the hits QL at a time (world shapes, collide);
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

// Lane layout: env ev (0 .. 64/QL - 1) of the wavefront owns lanes ev * QL .. ev * QL + QL - 1 (a layout with
// the serial sub-lane-0 lanes packed first in the wave measured the same, round 4: FP64 instructions cost the
// same whatever the number of active lanes -- tools/ubench/exec_f64.hip)
template <int QL> MG_DEV int qlane(int ev, int s) { return ev * QL + s; }

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

// body of integration slot p (p < nb) in the compile-time scenes (robot: body 0, control 1, eyes 2-3, fingers
// 4-5; block 6): the bodies whose rotation caches need the correctly rounded sincos (0, 4, 5, 6) first, so the
// first round of slots (one per lane) runs them side by side and the second has none (body_rot_unused)
MG_DEV int quad_body(int p, int nb) {
    if (p == 0) return 0;
    if (p == 1) return 4;
    if (p == 2) return 5;
    if (nb == 7) return p == 3 ? 6 : p - 3;
    return p - 2;
}

MG_DEV uint64_t qshfl_xor_u64(uint64_t u, int m) {
    const uint32_t lo = (uint32_t)__shfl_xor((int)(uint32_t)u, m, 64), hi = (uint32_t)__shfl_xor((int)(uint32_t)(u >> 32), m, 64);
    return ((uint64_t)hi << 32) | lo;
}

// candidate k of shape i in the canonical order (walls 0..3, then shapes j = i + 1 + (k - 4)): the broadphase
// tests that decide whether collide() runs -- cached BBs, shape filters (categories 0: MG_GROUP_OFF), same
// body / same group, and the exact separating-axis skip
MG_DEV bool quad_candidate(const MGState &S, const mg_library *L, int e, int i, int k) {
    const double al = AT(S.sbbl, i), ab = AT(S.sbbb, i), ar = AT(S.sbbr, i), at = AT(S.sbbt, i);
    const int gi = AT(S.sgroup, i);
    if (k < 4) {
        if (gi & MG_GROUP_OFF) return false;   // categories 0 collide with nothing
        double wl, wb, wr, wt;
        wall_bb(k, wl, wb, wr, wt);
        return al <= wr && wl <= ar && ab <= wt && wb <= at;
    }
    const int j = i + 1 + (k - 4), gj = AT(S.sgroup, j);
    return al <= AT(S.sbbr, j) && AT(S.sbbl, j) <= ar && ab <= AT(S.sbbt, j) && AT(S.sbbb, j) <= at &&
           AT(S.sbody, j) != AT(S.sbody, i) && !((gi != 0 && gi == gj) || ((gi | gj) & MG_GROUP_OFF)) &&
           !surely_apart(S, L, e, i, j);
}

// broadphase + narrowphase of env e (canonical pair order), QL lanes per env.  Called with every lane of
// the env active (the trip counts depend on the env's shape count and hits only).
// Pass 1: the env's candidates (shape i's walls 0..3, then shapes j > i, for i = 0 .. ns-1) are tested QL at
// a time (candidate c on lane c mod QL) and the ones that need collide() form a mask in canonical order.  In
// most substeps it is empty (the robot scenes touch a wall or the block now and then).  Pass 2: the hits, QL
// at a time in mask order (the q-th lowest on lane q): collide(), then lane 0 applies the arbiter updates in
// canonical order from its siblings' results (cross-lane reads).  The same collide() calls and the same
// arbiter updates in the same order as a serial sweep of the candidates, so bit-identical.
template <int NCS, int QL, bool LDS_SHAPES>
MG_DEV void narrowphase_quad(const MGState &S, const mg_library *L, int e, int sub, int ns) {
    ShapeW locA, locB;
    ShapeW &A = LDS_SHAPES ? S.shw[2 * QL * e + 2 * sub] : locA;
    ShapeW &B = LDS_SHAPES ? S.shw[2 * QL * e + 2 * sub + 1] : locB;
    const int ntot = 4 * ns + (ns * (ns - 1)) / 2;
    for (int w0 = 0; w0 < ntot; w0 += 64) {
        const int wn = ntot - w0 < 64 ? ntot - w0 : 64;
        uint64_t hits = 0;
        {   // pass 1 (decode c -> (i, k) incrementally: candidates of one lane are QL apart)
            int i = 0, k = w0 + sub;
            while (i < ns && k >= 4 + ns - 1 - i) { k -= 4 + ns - 1 - i; i++; }
            for (int c = sub; c < wn; c += QL) {
                if (quad_candidate(S, L, e, i, k)) hits |= 1ull << c;
                k += QL;
                while (i < ns && k >= 4 + ns - 1 - i) { k -= 4 + ns - 1 - i; i++; }
            }
        }
#pragma unroll
        for (int off = 1; off < QL; off <<= 1)   // the env's lanes: disjoint bits
            hits |= qshfl_xor_u64(hits, off);
        // pass 2
        while (hits) {   // uniform over the env's lanes
            uint64_t rest = hits;
            int mine = -1;
#pragma unroll
            for (int q = 0; q < QL; q++) {
                if (!rest) break;
                const int b = __ffsll((long long)rest) - 1;
                rest &= rest - 1;
                if (q == sub) mine = b;
            }
            hits = rest;
            Collision info;
            info.count = 0;
            int key = 0, ta = 0, bi = 0, tb = 0, bb = -1;
            double ui = 0.0, ub = 0.0;
            if (mine >= 0) {
                int i = 0, k = w0 + mine;
                while (k >= 4 + ns - 1 - i) { k -= 4 + ns - 1 - i; i++; }
                bi = AT(S.sbody, i); ui = AT(S.su, i);
                ta = AT(S.spoly, i) < 0 ? WS_CIRCLE : WS_POLY;
                load_shape(S, L, e, i, (uint64_t)AT(S.shash, i), A);
                if (k < 4) {
                    load_wall(k, B);
                    key = i * 128 + 100 + k; ub = 0.8; tb = WS_SEGMENT; bb = -1;
                } else {
                    const int j = i + 1 + (k - 4);
                    load_shape(S, L, e, j, (uint64_t)AT(S.shash, j), B);
                    key = i * 128 + j; ub = AT(S.su, j); tb = B.type; bb = B.body;
                }
                collide(A, B, info);   // one call site: the narrowphase is inlined once
            }
            // the contacts to lane 0, in candidate order (= lane order: lane q holds the q-th hit)
            const uint64_t bal = __ballot(info.count > 0);
            uint32_t m = 0;
#pragma unroll
            for (int s = 0; s < QL; s++) m |= (uint32_t)((bal >> qlane<QL>(e, s)) & 1ull) << s;
            for (int s = 0; s < QL; s++) {
                if (!((m >> s) & 1u)) continue;   // uniform over the env's lanes
                const int src = qlane<QL>(e, s);
                Collision q;
                q.count = __shfl(info.count, src, 64);
                q.n = v2(qshfl(info.n.x, src), qshfl(info.n.y, src));
#pragma unroll
                for (int kk = 0; kk < 2; kk++) {
                    q.p1[kk] = v2(qshfl(info.p1[kk].x, src), qshfl(info.p1[kk].y, src));
                    q.p2[kk] = v2(qshfl(info.p2[kk].x, src), qshfl(info.p2[kk].y, src));
                    q.hash[kk] = qshfl_u64(info.hash[kk], src);
                }
                const int qkey = __shfl(key, src, 64), qta = __shfl(ta, src, 64), qbi = __shfl(bi, src, 64);
                const int qtb = __shfl(tb, src, 64), qbb = __shfl(bb, src, 64);
                const double qui = qshfl(ui, src), qub = qshfl(ub, src);
                if (sub == 0) arbiter_update_t(S, L, e, qkey, qta, qbi, qtb, qbb, qui, qub, q);
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
    for (int p = sub; p < nb; p += QL) {
        const int b = quad_body(p, nb);
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
    narrowphase_quad<NCS, QL, LDS_SHAPES>(S, L, e, sub, ns);
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
    if (sub == 0) static_solve<NCS, (QL >= 8 ? 1 : 0)>(S, e, dt, dt_coef, nact, P);   // NARB: see static_solve
    MG_PP(P, 6);
}

// Robot.set_action + 10 x (Robot.update, cpSpaceStep) with QL lanes per env
template <int NCS, int QL, bool LDS_SHAPES>
__device__ __forceinline__ void env_substeps_quad(const MGState &V, const mg_library *L, int ev, int sub, int a,
                                                  MGProf &P) {
    // robot.update() before every space.step() (base_env.py:248-255).  From the second substep on it runs on
    // sub-lane 0 right after that lane's solver sweep of the previous substep, in the same phase: it reads
    // angles and rotation caches (the sweep changes velocities only) and writes the control body's velocity
    // and the finger springs' rates, which the next phase's barrier publishes -- one barrier phase fewer per
    // substep, the same operations in the same order.  The first update reads rows (angles, rotation caches)
    // and writes rows (the finger motors' rates) that the env's sibling lanes loaded into LDS in xfer_state:
    // one barrier orders them, once per env-step.
    __syncthreads();
    if (sub == 0) {
        robot_set_action(V, L, ev, a < 18 ? a : 0);
        robot_update<true>(V, L, ev);
    }
    const double dt = L->dt;
    for (int i = 0; i < 10; i++) {
        MG_PP(P, 0);
        space_step_quad<NCS, QL, LDS_SHAPES>(V, L, ev, sub, dt, P);   // starts with a workgroup barrier
        if (sub == 0 && i < 9) robot_update<true>(V, L, ev);
    }
    __syncthreads();
}
