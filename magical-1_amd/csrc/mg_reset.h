// mg_reset.h -- per-lane episode reset: task on_reset, entity setup, randomisers.
//
// base_env.py:190-246 (reset: new Space, PhysicsVariables.sample, arena,
// on_reset), entities.py:238-433 / 580-754 / 762-801 (entity setup),
// geom.py:116-384 (pm_randomise_pose rejection sampling with shape queries,
// pm_randomise_all_poses, randomise_hw, pm_shift_bodies), task files
// move_to_region.py:30-83, move_to_corner.py:125-159, cluster.py:67-164,
// match_regions.py:44-191.  RNG: numpy legacy RandomState (MT19937) per env,
// drawn in the reference's order so parity mode replays the reference stream.
#pragma once
#include "mg_launch.h"
#include "mg_phys.h"
#include "mg_prof.h"

#define MT(i) S.mt_key[(size_t)(i) * (size_t)S.N + (size_t)e]

MG_DEV void mt_seed(const MGState &S, int e, uint32_t seed) {
    uint32_t v = seed;
    for (int i = 0; i < 624; i++) {
        MT(i) = v;
        v = 1812433253u * (v ^ (v >> 30)) + (uint32_t)(i + 1);
    }
    S.mt_pos[e] = 624;
}
// The twist over the LDS copy (a cooperative reset: the wave's 64 lanes call mt_next32 together with the same
// state).  Word i's new value reads the old words i, i + 1 and, for i < 227, the old word i + 397, else the NEW
// word i - 227; so the words are updated in order in chunks of 64 lanes -- each chunk's loads precede its stores
// (one wave, in-order LDS), its i + 1 / i + 397 words are not yet rewritten and its i - 227 words were rewritten
// by an earlier chunk -- and word 623 last (new words 396 and 0).  Same values as the serial loop below.
MG_DEV void mt_twist_lds(uint32_t *m) {
    const uint32_t UPPER = 0x80000000u, LOWER = 0x7fffffffu, MA = 0x9908b0dfu;
    if (__builtin_amdgcn_read_exec() == ~0ull) {
        const int lane = (int)(threadIdx.x & 63);
        for (int b = 0; b < 623; b += 64) {
            const int i = b + lane;
            uint32_t v = 0u;
            if (i < 623) {
                const uint32_t y = (m[i] & UPPER) | (m[i + 1] & LOWER);
                v = m[i < 227 ? i + 397 : i - 227] ^ (y >> 1) ^ (-(y & 1u) & MA);
            }
            __builtin_amdgcn_wave_barrier();
            if (i < 623) m[i] = v;
            __builtin_amdgcn_wave_barrier();
        }
    } else {   // (not every lane active: each runs the serial twist, writing the same values)
        for (int i = 0; i < 623; i++) {
            const uint32_t y = (m[i] & UPPER) | (m[i + 1] & LOWER);
            m[i] = m[i < 227 ? i + 397 : i - 227] ^ (y >> 1) ^ (-(y & 1u) & MA);
        }
    }
    const uint32_t y = (m[623] & UPPER) | (m[0] & LOWER);
    m[623] = m[396] ^ (y >> 1) ^ (-(y & 1u) & MA);
}
MG_DEV uint32_t mt_next32(const MGState &S, int e) {
    if (S.mt_lds) {   // the cooperative reset's LDS copy (every lane reads and writes the same words)
        uint32_t *m = S.mt_lds;
        int pos = (int)m[624];
        if (pos == 624) { mt_twist_lds(m); pos = 0; }
        uint32_t y = m[pos];
        __builtin_amdgcn_wave_barrier();
        m[624] = (uint32_t)(pos + 1);
        y ^= (y >> 11);
        y ^= (y << 7) & 0x9d2c5680u;
        y ^= (y << 15) & 0xefc60000u;
        y ^= (y >> 18);
        return y;
    }
    int pos = S.mt_pos[e];
    if (pos == 624) {
        const uint32_t UPPER = 0x80000000u, LOWER = 0x7fffffffu, MA = 0x9908b0dfu;
        uint32_t y;
        int i;
        for (i = 0; i < 624 - 397; i++) {
            y = (MT(i) & UPPER) | (MT(i + 1) & LOWER);
            MT(i) = MT(i + 397) ^ (y >> 1) ^ (-(y & 1u) & MA);
        }
        for (; i < 623; i++) {
            y = (MT(i) & UPPER) | (MT(i + 1) & LOWER);
            MT(i) = MT(i - 227) ^ (y >> 1) ^ (-(y & 1u) & MA);
        }
        y = (MT(623) & UPPER) | (MT(0) & LOWER);
        MT(623) = MT(396) ^ (y >> 1) ^ (-(y & 1u) & MA);
        pos = 0;
    }
    uint32_t y = MT(pos);
    S.mt_pos[e] = pos + 1;
    y ^= (y >> 11);
    y ^= (y << 7) & 0x9d2c5680u;
    y ^= (y << 15) & 0xefc60000u;
    y ^= (y >> 18);
    return y;
}
MG_DEV double mt_double(const MGState &S, int e) {
    int32_t a = (int32_t)(mt_next32(S, e) >> 5);
    int32_t b = (int32_t)(mt_next32(S, e) >> 6);
    return (a * 67108864.0 + b) / 9007199254740992.0;
}
MG_DEV double mt_uniform(const MGState &S, int e, double lo, double hi) {
    double range = hi - lo;
    return lo + range * mt_double(S, e);
}
MG_DEV uint32_t mt_masked(const MGState &S, int e, uint32_t rng) { // uniform in [0, rng]
    if (rng == 0) return 0;
    uint32_t m = rng;
    m |= m >> 1; m |= m >> 2; m |= m >> 4; m |= m >> 8; m |= m >> 16;
    uint32_t v;
    while ((v = (mt_next32(S, e) & m)) > rng) {}
    return v;
}
MG_DEV int mt_randint(const MGState &S, int e, int lo, int hi) { return lo + (int)mt_masked(S, e, (uint32_t)(hi - 1 - lo)); }

// ---- entity instantiation -------------------------------------------------
struct Builder { int nb, ns, nc, hash; };

MG_DEV int add_body(const MGState &S, int e, Builder &B, bool kin, double m, double i, double px, double py, double a) {
    int b = B.nb++;
    AT(S.bkin, b) = kin ? 1 : 0;
    AT(S.bminv, b) = kin ? 0.0 : 1.0 / m;
    AT(S.biinv, b) = kin ? 0.0 : 1.0 / i;
    AT(S.bpx, b) = px; AT(S.bpy, b) = py;
    AT(S.bvx, b) = 0.0; AT(S.bvy, b) = 0.0; AT(S.bw, b) = 0.0;
    AT(S.bvbx, b) = 0.0; AT(S.bvby, b) = 0.0; AT(S.bwb, b) = 0.0;
    AT(S.bacache, b) = NAN;
    body_set_angle(S, e, b, a);
    return b;
}
MG_DEV int add_shape(const MGState &S, int e, Builder &B, int body, int poly, double r, double u, int group, int ent) {
    int k = B.ns++;
    AT(S.sbody, k) = (int8_t)body; AT(S.spoly, k) = (int8_t)poly; AT(S.sent, k) = (int8_t)ent;
    AT(S.sgroup, k) = (int16_t)group; AT(S.shash, k) = (int16_t)(B.hash++);
    AT(S.scat, k) = 1; AT(S.sr, k) = r; AT(S.su, k) = u;
    return k;
}
MG_DEV int add_cons(const MGState &S, int e, Builder &B, int type, int a, int b, double maxF, double maxB, double bcoef) {
    int c = B.nc++;
    AT(S.ctype, c) = (int8_t)type; AT(S.ca, c) = (int8_t)a; AT(S.cb, c) = (int8_t)b;
    for (int k = 0; k < CP_NUM; k++) CPA(k, c) = 0.0;
    CPA(CP_MAXF, c) = maxF; CPA(CP_MAXB, c) = maxB; CPA(CP_BCOEF, c) = bcoef;
    return c;
}

// cpBodyWorldToLocal via cpTransformRigidInverse
MG_DEV V2 world_to_local(const MGState &S, int e, int b, V2 pt) {
    double c = AT(S.brc, b), s = AT(S.brs, b), tx = AT(S.bpx, b), ty = AT(S.bpy, b);
    double ta = c, tb = s, tc = -s, td = c;
    double ia = td, ic = -tc, itx = tc * ty - tx * td;
    double ib = -tb, id = ta, ity = tx * tb - ta * ty;
    return v2(ia * pt.x + ic * pt.y + itx, ib * pt.x + id * pt.y + ity);
}

MG_DEV V2 rotated(V2 v, double ang) {
    double s, c;
    mg_sincos(ang, s, c);
    return v2(v.x * c - v.y * s, v.x * s + v.y * c);
}

MG_DEV void add_robot(const MGState &S, const mg_library *L, int e, Builder &B, int ent, double px, double py, double ang) {
    const double *pv = S.pv;
    size_t N = (size_t)S.N;
    double radius = L->robot_radius;
    int body = add_body(S, e, B, false, L->robot_mass, L->robot_inertia, px, py, ang);
    int control = add_body(S, e, B, true, 0, 0, px, py, ang);
    S.robot_body0[e] = body;
    S.robot_cons0[e] = B.nc;
    int c = add_cons(S, e, B, MG_C_PIVOT, control, body, pv[0 * N + e], 0.0, L->default_bias_coef);
    c = add_cons(S, e, B, MG_C_GEAR, control, body, pv[1 * N + e], 2.5, 1.0);
    CPA(CP_PHASE, c) = 0.0; CPA(CP_RATIO, c) = 1.0; CPA(CP_RATIO_INV, c) = 1.0 / 1.0;
    for (int k = 0; k < 2; k++) {
        int eye = add_body(S, e, B, false, L->eye_mass, L->eye_inertia, 0.0, 0.0, ang);
        c = add_cons(S, e, B, MG_C_SPRING, body, eye, 0.001, 3.0, L->default_bias_coef);
        CPA(CP_REST, c) = 0.0; CPA(CP_STIFF, c) = 0.1; CPA(CP_WCOEF, c) = L->spring_w_coef;
    }
    int fingers[2];
    for (int k = 0; k < 2; k++) {
        V2 rel = v2(L->finger_rel[k][0], L->finger_rel[k][1]);
        V2 relr = rotated(rel, ang);
        V2 fp = v2(AT(S.bpx, body) + relr.x, AT(S.bpy, body) + relr.y);
        int fb = add_body(S, e, B, false, L->finger_mass, L->finger_inertia[k], fp.x, fp.y, ang + L->finger_angle_off[k]);
        fingers[k] = fb;
        V2 pivot = v2(AT(S.bpx, fb), AT(S.bpy, fb));
        V2 aa = world_to_local(S, e, body, pivot), ab = world_to_local(S, e, fb, pivot);
        c = add_cons(S, e, B, MG_C_PIVOT, body, fb, INFINITY, INFINITY, 1.0);
        CPA(CP_AAX, c) = aa.x; CPA(CP_AAY, c) = aa.y; CPA(CP_ABX, c) = ab.x; CPA(CP_ABY, c) = ab.y;
        c = add_cons(S, e, B, MG_C_ROTLIMIT, body, fb, INFINITY, INFINITY, 1.0);
        CPA(CP_MIN, c) = L->finger_lim[k][0]; CPA(CP_MAX, c) = L->finger_lim[k][1];
        c = add_cons(S, e, B, MG_C_MOTOR, body, fb, pv[2 * N + e], 0.0, L->default_bias_coef);
        CPA(CP_RATE, c) = 0.0;
    }
    add_shape(S, e, B, body, -1, radius, 0.5, 1, ent);
    for (int k = 0; k < 2; k++)
        for (int p = 0; p < 2; p++) {
            int poly = L->finger_poly[2 * k + p];
            add_shape(S, e, B, fingers[k], poly, L->poly_r[poly], 5.0, 1, ent);
        }
}

MG_DEV void add_block(const MGState &S, const mg_library *L, int e, Builder &B, int ent, int type, double px, double py,
                      double ang, int star_group) {
    size_t N = (size_t)S.N;
    int body = add_body(S, e, B, false, L->block_mass[type], L->block_inertia[type], px, py, ang);
    int group = type == MG_SHAPE_STAR ? star_group : 0;
    for (int i = 0; i < L->block_nshapes[type]; i++) {
        int poly = L->block_poly[type][i];
        double r = poly < 0 ? L->block_circle_r : L->poly_r[poly];
        add_shape(S, e, B, body, poly, r, 0.5, group, ent);
    }
    int c = add_cons(S, e, B, MG_C_PIVOT, -1, body, S.pv[3 * N + e], 0.0, L->default_bias_coef);
    c = add_cons(S, e, B, MG_C_GEAR, -1, body, S.pv[4 * N + e], 0.0, L->default_bias_coef);
    CPA(CP_PHASE, c) = 0.0; CPA(CP_RATIO, c) = 1.0; CPA(CP_RATIO_INV, c) = 1.0 / 1.0;
}

// ---- shape queries (cpSpaceShapeQuery semantics, sensors reported) --------
// A is entity self_ent's shape (or goal); ign = bit mask of entities whose shapes are ignored
// (pm_randomise_pose ignore_shapes, geom.py:116-264).
MG_DEV bool query_hits(const MGState &S, const mg_library *L, int e, const ShapeW &A, int self_k, int group, int self_ent,
                       uint32_t ign, bool self_on, int lane) {
    if (!self_on) return false; // the queried shape's categories are 0: cpShapeFilterReject for every pair
    // candidates: 4 arena walls, the entities' goal sensors (enabled: categories != 0), the other shapes.
    // The answer is "any hit", so in a cooperative reset (lane >= 0) lane l tests candidates l, l + 64, ...
    // and the wave ORs the results; serially (lane < 0) one thread tests them all.
    const int nents = S.nents[e], ns = S.nshapes[e];
    const int total = 4 + nents + ns;
    bool hit = false;
    for (int c = lane < 0 ? 0 : lane; c < total && !hit; c += lane < 0 ? 1 : 64) {
        if (c < 4) {
            ShapeW W;
            load_wall(c, W);
            if (!bb_intersects(A, W)) continue;
            Collision info;
            collide(A, W, info);
            hit = info.count != 0;
        } else if (c < 4 + nents) {
            const int g = c - 4;
            if (AT(S.ekind, g) != MG_ENT_GOAL || g == self_ent || ((ign >> g) & 1u) || AT(S.eshape0, g) == 0) continue;
            ShapeW G;
            load_goal(AT(S.ex, g), AT(S.ey, g), AT(S.ew, g), AT(S.eh, g), 0, G);
            if (!bb_intersects(A, G)) continue;
            Collision info;
            collide(A, G, info);
            hit = info.count != 0;
        } else {
            const int j = c - 4 - nents;
            if (j == self_k || !AT(S.scat, j) || ((ign >> AT(S.sent, j)) & 1u)) continue;
            int gj = AT(S.sgroup, j);
            if (group != 0 && group == gj) continue;
            ShapeW O;
            load_shape(S, L, e, j, 0, O);
            if (!bb_intersects(A, O)) continue;
            Collision info;
            collide(A, O, info);
            hit = info.count != 0;
        }
    }
    if (lane >= 0) hit = __ballot(hit) != 0ull;
    return hit;
}

MG_DEV int ent_enabled(const MGState &S, int e, int ent) {
    return AT(S.ekind, ent) == MG_ENT_GOAL ? AT(S.eshape0, ent) : AT(S.scat, AT(S.eshape0, ent));
}
MG_DEV void ent_set_enabled(const MGState &S, int e, int ent, int on) {
    if (AT(S.ekind, ent) == MG_ENT_GOAL) { AT(S.eshape0, ent) = (int8_t)on; return; }
    int s0 = AT(S.eshape0, ent), n = AT(S.enshapes, ent);
    for (int k = s0; k < s0 + n; k++) AT(S.scat, k) = (uint8_t)on;
}

// pm_shift_bodies (geom.py:362-384)
MG_DEV void shift_entity(const MGState &S, int e, int ent, V2 pos, double ang) {
    if (AT(S.ekind, ent) == MG_ENT_GOAL) {
        V2 root = v2(AT(S.ex, ent), AT(S.ey, ent));
        V2 d = v2(AT(S.ex, ent) - root.x, AT(S.ey, ent) - root.y);
        V2 r = rotated(d, ang - 0.0);
        AT(S.ex, ent) = pos.x + r.x; AT(S.ey, ent) = pos.y + r.y;
        return;
    }
    int b0 = AT(S.ebody0, ent);
    int nb = AT(S.ekind, ent) == MG_ENT_ROBOT ? 6 : 1;
    double root_a = AT(S.ba, b0);
    V2 root_p = v2(AT(S.bpx, b0), AT(S.bpy, b0));
    for (int b = b0; b < b0 + nb; b++) {
        double lad = AT(S.ba, b) - root_a;
        V2 lpd = v2(AT(S.bpx, b) - root_p.x, AT(S.bpy, b) - root_p.y);
        body_set_angle(S, e, b, ang + lad);
        V2 r = rotated(lpd, ang - root_a);
        // cpBodySetPosition: p = T(cog = 0) + position
        double c = AT(S.brc, b), s = AT(S.brs, b);
        V2 t0 = v2(c * 0.0 + (-s) * 0.0, s * 0.0 + c * 0.0);
        AT(S.bpx, b) = t0.x + (pos.x + r.x);
        AT(S.bpy, b) = t0.y + (pos.y + r.y);
    }
}

MG_DEV bool entity_collides(const MGState &S, const mg_library *L, int e, int ent, uint32_t ign, int lane) {
    if (AT(S.ekind, ent) == MG_ENT_GOAL) {
        ShapeW G;
        load_goal(AT(S.ex, ent), AT(S.ey, ent), AT(S.ew, ent), AT(S.eh, ent), 0, G);
        return query_hits(S, L, e, G, -1, 0, ent, ign, AT(S.eshape0, ent) != 0, lane);
    }
    int s0 = AT(S.eshape0, ent), n = AT(S.enshapes, ent);
    for (int k = s0; k < s0 + n; k++) {
        ShapeW A;
        load_shape(S, L, e, k, 0, A);
        if (query_hits(S, L, e, A, k, AT(S.sgroup, k), ent, ign, AT(S.scat, k) != 0, lane)) return true;
    }
    return false;
}

// pm_randomise_pose (geom.py:116-264); pos_limit / rot_limit < 0 mean None
MG_DEV int randomise_pose(const MGState &S, const mg_library *L, int e, int lane, int ent, bool rand_rot,
                          double pos_limit, double rot_limit, uint32_t ign = 0u) {
    bool goal = AT(S.ekind, ent) == MG_ENT_GOAL;
    int b0 = goal ? -1 : AT(S.ebody0, ent);
    double orig_a = goal ? 0.0 : AT(S.ba, b0);
    V2 orig_p = goal ? v2(AT(S.ex, ent), AT(S.ey, ent)) : v2(AT(S.bpx, b0), AT(S.bpy, b0));
    double xlo = -1, xhi = 1, ylo = -1, yhi = 1;
    if (pos_limit >= 0) {
        xlo = fmax(-1.0, orig_p.x - pos_limit); xhi = fmin(1.0, orig_p.x + pos_limit);
        ylo = fmax(-1.0, orig_p.y - pos_limit); yhi = fmin(1.0, orig_p.y + pos_limit);
    }
    double rmin = -3.141592653589793, rmax = 3.141592653589793;
    if (rot_limit >= 0) { rmin = orig_a - rot_limit; rmax = orig_a + rot_limit; }
    double saved_x[6], saved_y[6], saved_a[6]; // geom.py:174-176 saved_positions / saved_angles
    if (!goal) {
        const int nb = AT(S.ekind, ent) == MG_ENT_ROBOT ? 6 : 1;
#pragma unroll
        for (int k = 0; k < 6; k++) {
            const int b = b0 + (k < nb ? k : 0);
            saved_x[k] = AT(S.bpx, b); saved_y[k] = AT(S.bpy, b); saved_a[k] = AT(S.ba, b);
        }
    }
    for (int tries = 0; tries < S.max_tries; tries++) {
        double x = mt_uniform(S, e, xlo, xhi);
        double y = mt_uniform(S, e, ylo, yhi);
        double a = rand_rot ? mt_uniform(S, e, rmin, rmax) : orig_a;
        shift_entity(S, e, ent, v2(x, y), a);
        if (!entity_collides(S, L, e, ent, ign, lane)) return 0;
    }
    // PlacementError: every body back to its saved absolute pose (geom.py:250-254: Body.position and
    // Body.angle setters), not a rigid shift relative to the last try
    if (goal) {
        AT(S.ex, ent) = orig_p.x; AT(S.ey, ent) = orig_p.y;
    } else {
        const int nb = AT(S.ekind, ent) == MG_ENT_ROBOT ? 6 : 1;
        for (int k = 0; k < nb; k++) {
            const int b = b0 + k;
            body_set_angle(S, e, b, saved_a[k]);
            const double c = AT(S.brc, b), sn = AT(S.brs, b);
            AT(S.bpx, b) = (c * 0.0 + (-sn) * 0.0) + saved_x[k]; // cpBodySetPosition: p = T(cog = 0) + position
            AT(S.bpy, b) = (sn * 0.0 + c * 0.0) + saved_y[k];
        }
    }
    return -1;
}

MG_DEV void randomise_all(const MGState &S, const mg_library *L, int e, int lane, const int *ents, int n,
                          const bool *rand_rot, double pos_limit, const double *rot_limits, uint32_t ign = 0u) {
    for (int retry = 0; retry < 10; retry++) {
        // geom.py:300-319: each entity's filter is captured at the start of every retry and restored when
        // its turn comes, so entities left disabled by a failed retry stay disabled (categories 0)
        uint32_t saved = 0u;
        for (int k = 0; k < n; k++) {
            saved |= (uint32_t)(ent_enabled(S, e, ents[k]) != 0) << k;
            ent_set_enabled(S, e, ents[k], 0);
        }
        bool failed = false;
        for (int k = 0; k < n && !failed; k++) {
            ent_set_enabled(S, e, ents[k], (saved >> k) & 1u);
            if (randomise_pose(S, L, e, lane, ents[k], rand_rot[k], pos_limit, rot_limits[k], ign) != 0) failed = true;
        }
        if (!failed) return;
    }
    S.overflow[e] |= 2 | 64; // PlacementError after 10 retries (bit 2: this reset; bit 64: sticky, any reset)
}

// ---- tasks -----------------------------------------------------------------
__constant__ static const int MG_SHAPE_COLOURS[4] = {MG_COL_RED, MG_COL_GREEN, MG_COL_BLUE, MG_COL_YELLOW};
__constant__ static const int MG_SHAPE_TYPES[4] = {MG_SHAPE_SQUARE, MG_SHAPE_PENTAGON, MG_SHAPE_STAR, MG_SHAPE_CIRCLE};

MG_DEV int new_entity(const MGState &S, int e, int kind, int type, int colour, int role, double x, double y, double a) {
    int i = S.nents[e]++;
    AT(S.ekind, i) = (int8_t)kind; AT(S.etype, i) = (int8_t)type; AT(S.ecol, i) = (int8_t)colour;
    AT(S.erole, i) = (int8_t)role;
    AT(S.ex, i) = x; AT(S.ey, i) = y; AT(S.eang, i) = a; AT(S.eh, i) = 0.0; AT(S.ew, i) = 0.0;
    AT(S.ebody0, i) = 0; AT(S.eshape0, i) = 0; AT(S.enshapes, i) = 0;
    return i;
}

MG_DEV void inst_robot(const MGState &S, const mg_library *L, int e, Builder &B, double x, double y, double a) {
    int ent = new_entity(S, e, MG_ENT_ROBOT, 0, MG_COL_GREY, 0, x, y, a);
    AT(S.ebody0, ent) = (int8_t)B.nb; AT(S.eshape0, ent) = (int8_t)B.ns;
    add_robot(S, L, e, B, ent, x, y, a);
    AT(S.enshapes, ent) = (int8_t)(B.ns - AT(S.eshape0, ent));
}
MG_DEV void inst_block(const MGState &S, const mg_library *L, int e, Builder &B, int type, int colour, int role, double x,
                       double y, double a, int &star_groups) {
    int ent = new_entity(S, e, MG_ENT_BLOCK, type, colour, role, x, y, a);
    AT(S.ebody0, ent) = (int8_t)B.nb; AT(S.eshape0, ent) = (int8_t)B.ns;
    int group = 0;
    if (type == MG_SHAPE_STAR) group = 1000 + (++star_groups);
    add_block(S, L, e, B, ent, type, x, y, a, group);
    AT(S.enshapes, ent) = (int8_t)(B.ns - AT(S.eshape0, ent));
}
MG_DEV void inst_goal(const MGState &S, int e, Builder &B, double x, double y, double h, double w, int colour) {
    int ent = new_entity(S, e, MG_ENT_GOAL, 0, colour, 0, x, y, 0.0);
    AT(S.eh, ent) = h; AT(S.ew, ent) = w;
    AT(S.eshape0, ent) = 1; // enabled flag for goals
    AT(S.ex, ent) = x + w / 2; AT(S.ey, ent) = y - h / 2; // the sensor body's position
    S.goal_ent[e] = ent;
    B.hash++;
}

#define JITTER_POS_BOUND (1 * 0.05 / 2.0)
#define JITTER_ROT_BOUND (0.05 * 3.141592653589793)
#define JITTER_TARGET_BOUND (0.05 * (0.8 - 0.5) / 2)

MG_DEV void randomise_hw(const MGState &S, int e, double ch, double cw, double linf, double &h, double &w,
                         double mn = 0.5, double mx = 0.8) { // RAND_GOAL_MIN/MAX_SIZE by default
    double lo0 = mn, lo1 = mn, hi0 = mx, hi1 = mx;
    if (linf >= 0) {
        lo0 = fmax(lo0, ch - linf); lo1 = fmax(lo1, cw - linf);
        hi0 = fmin(hi0, ch + linf); hi1 = fmin(hi1, cw + linf);
    }
    h = mt_uniform(S, e, lo0, hi0);
    w = mt_uniform(S, e, lo1, hi1);
}

__constant__ static const int CC_COLOURS[2][8] = {
    {MG_COL_BLUE, MG_COL_BLUE, MG_COL_BLUE, MG_COL_GREEN, MG_COL_GREEN, MG_COL_RED, MG_COL_YELLOW, MG_COL_YELLOW},
    {MG_COL_YELLOW, MG_COL_BLUE, MG_COL_RED, MG_COL_RED, MG_COL_GREEN, MG_COL_YELLOW, MG_COL_BLUE, MG_COL_GREEN}};
__constant__ static const int CC_TYPES[2][8] = {
    {MG_SHAPE_CIRCLE, MG_SHAPE_STAR, MG_SHAPE_SQUARE, MG_SHAPE_PENTAGON, MG_SHAPE_PENTAGON, MG_SHAPE_SQUARE, MG_SHAPE_STAR,
     MG_SHAPE_PENTAGON},
    {MG_SHAPE_SQUARE, MG_SHAPE_PENTAGON, MG_SHAPE_PENTAGON, MG_SHAPE_PENTAGON, MG_SHAPE_CIRCLE, MG_SHAPE_STAR, MG_SHAPE_STAR,
     MG_SHAPE_CIRCLE}};
__constant__ static const double CC_POSES[2][8][3] = {
    {{-0.5147, 0.14149, -0.38871}, {-0.1347, -0.71414, 1.0533}, {-0.74247, -0.097592, 1.1571},
     {-0.077363, -0.42964, -0.64379}, {0.51978, 0.1853, -1.1762}, {-0.5278, -0.21642, 2.9356},
     {-0.54039, 0.48292, 0.072818}, {-0.16761, 0.64303, -2.3255}},
    {{-0.414, 0.297, -1.731}, {0.068, 0.705, 2.184}, {0.821, 0.220, 0.650}, {-0.461, -0.749, -2.673},
     {0.867, -0.149, -2.215}, {-0.785, -0.140, -0.405}, {-0.305, -0.226, 1.341}, {0.758, -0.708, -2.140}}};
__constant__ static const double CC_ROBOT[2][3] = {{0.71692, -0.34374, 0.83693}, {0.286, -0.202, -1.878}};

// make_line.py:13-27
__constant__ static const int ML_COLOURS[4] = {MG_COL_BLUE, MG_COL_YELLOW, MG_COL_RED, MG_COL_GREEN};
__constant__ static const int ML_TYPES[4] = {MG_SHAPE_STAR, MG_SHAPE_CIRCLE, MG_SHAPE_STAR, MG_SHAPE_PENTAGON};
__constant__ static const double ML_POSES[4][3] = {{0.790, -0.820, -0.721}, {-0.177, 0.383, -1.733},
                                                   {-0.051, -0.128, 2.696}, {-0.292, -0.745, -0.159}};

// find_dupe.py:7-37
__constant__ static const int FD_OUT_TYPES[6] = {MG_SHAPE_PENTAGON, MG_SHAPE_CIRCLE, MG_SHAPE_CIRCLE,
                                                 MG_SHAPE_SQUARE, MG_SHAPE_STAR, MG_SHAPE_PENTAGON};
__constant__ static const int FD_OUT_COLOURS[6] = {MG_COL_GREEN, MG_COL_RED, MG_COL_RED, MG_COL_YELLOW, MG_COL_BLUE,
                                                   MG_COL_YELLOW};
__constant__ static const double FD_OUT_POSES[6][3] = {{-0.066751, 0.7552, -2.9266}, {-0.05195, 0.31468, 1.5418},
                                                       {0.57528, -0.46865, -2.2141},  {0.40594, -0.74977, 0.24582},
                                                       {0.45254, 0.3681, -1.0834},    {0.76849, -0.10652, 0.10028}};
// fix_colour.py:12-41
__constant__ static const int FC_BLOCK_COLOURS[3] = {MG_COL_GREEN, MG_COL_GREEN, MG_COL_BLUE};
__constant__ static const int FC_BLOCK_TYPES[3] = {MG_SHAPE_PENTAGON, MG_SHAPE_SQUARE, MG_SHAPE_PENTAGON};
__constant__ static const double FC_BLOCK_POSES[3][3] = {{0.289, 0.030, 0.307}, {0.133, -0.561, 1.699},
                                                         {-0.336, 0.000, -1.529}};
__constant__ static const double FC_REGIONS[3][4] = {{-0.032, 0.348, 0.427, 0.468}, {0.019, -0.391, 0.460, 0.458},
                                                     {-0.681, 0.196, 0.498, 0.418}};
__constant__ static const int FC_REGION_COLOURS[3] = {MG_COL_GREEN, MG_COL_GREEN, MG_COL_RED};

// TASK >= 0: a reset kernel compiled for that task alone; LAYOUT == 0: for variants without layout
// randomisation (flags without MG_RAND_LAYOUT_*) -- the other tasks' and the rejection samplers' code is
// dropped, so the kernel needs far fewer registers (mg_launch_reset)
template <int TASK> MG_DEV constexpr bool task_is(int runtime_task, int t) { return TASK >= 0 ? TASK == t : runtime_task == t; }
template <int TASK = -1, int LAYOUT = -1>
MG_DEV void reset_env(const MGState &S, const mg_library *L, int e, TaskCfg cfg) {
    size_t N = (size_t)S.N;
    // cooperative reset (reset_kernel_coop): the wave's 64 lanes all run this env's reset with the same
    // values; the shape queries of the rejection samplers are split across them (query_hits)
    const int lane = cfg.coop ? (int)(threadIdx.x & 63) : -1;
    const int f = cfg.flags;
    S.episode_steps[e] = 0;
    // bit 2 reports the PlacementError of THIS reset (geom.py:335-336 raises out of reset(); the next reset
    // draws a new layout from the advancing RNG), so it is cleared here; bit 64 keeps the history
    S.overflow[e] &= ~2;
    for (int i = 0; i < MG_MAX_ARB; i++) { AT(S.akey, i) = -1; AT(S.acount, i) = 0; AT(S.astate, i) = ARB_FIRST; }
    S.nactive[e] = 0; S.stamp[e] = 0; S.curr_dt[e] = 0.0; S.nents[e] = 0; S.goal_ent[e] = -1;
    S.target_speed[e] = 0.0; S.rel_turn[e] = 0.0; S.target_finger[e] = 0.0;
    const double PV_DEF[5] = {3, 1, 4, 1.5, 0.1}, PV_LO[5] = {2.2, 0.7, 2.5, 1.0, 0.07}, PV_HI[5] = {3.5, 1.5, 4.5, 1.8, 0.15};
    for (int i = 0; i < 5; i++)
        S.pv[i * N + e] = (f & MG_RAND_DYNAMICS) ? mt_uniform(S, e, PV_LO[i], PV_HI[i]) : PV_DEF[i];
    Builder B = {0, 0, 0, 4}; // arena segments hold hashids 0..3
    new_entity(S, e, MG_ENT_ARENA, 0, MG_COL_GREY, 0, 0, 0, 0);
    int star_groups = 0;
    const bool any_layout = LAYOUT == 0 ? false : (f & (MG_RAND_LAYOUT_MINOR | MG_RAND_LAYOUT_FULL)) != 0;
    const bool minor = LAYOUT == 0 ? false : (f & MG_RAND_LAYOUT_MINOR) != 0;
    int ents[16]; bool rr[16]; double rl[16]; int n = 0;
    if (task_is<TASK>(cfg.task, MG_TASK_MOVE_TO_REGION)) {
        double gx = -0.62, gy = -0.17, gh = 0.76, gw = 0.75;
        if (any_layout) randomise_hw(S, e, gh, gw, minor ? JITTER_TARGET_BOUND : -1.0, gh, gw);
        int colour = MG_COL_BLUE;
        if (f & MG_RAND_COLOUR) colour = MG_SHAPE_COLOURS[mt_randint(S, e, 0, 4)];
        inst_goal(S, e, B, gx, gy, gh, gw, colour);
        inst_robot(S, L, e, B, 0.058, 0.53, -2.13);
        if (any_layout) {
            ents[0] = 1; ents[1] = 2; rr[0] = false; rr[1] = true;
            rl[0] = -1; rl[1] = minor ? JITTER_ROT_BOUND : -1;
            n = 2;
            S.nbodies[e] = B.nb; S.nshapes[e] = B.ns; S.ncons[e] = B.nc;
            randomise_all(S, L, e, lane, ents, n, rr, minor ? JITTER_POS_BOUND : -1.0, rl);
        }
    } else if (task_is<TASK>(cfg.task, MG_TASK_MOVE_TO_CORNER)) {
        double rx = mt_double(S, e), ry = mt_double(S, e);
        inst_robot(S, L, e, B, rx, ry, 0.55 * 3.141592653589793);
        int colour = MG_COL_RED, type = MG_SHAPE_SQUARE;
        if (f & MG_RAND_COLOUR) colour = MG_SHAPE_COLOURS[mt_randint(S, e, 0, 4)];
        if (f & MG_RAND_SHAPE_TYPE) type = MG_SHAPE_TYPES[mt_randint(S, e, 0, 4)];
        inst_block(S, L, e, B, type, colour, 0, 0.1, -0.65, 0.13 * 3.141592653589793, star_groups);
        if (minor) {
            ents[0] = 1; ents[1] = 2; rr[0] = rr[1] = true; rl[0] = rl[1] = JITTER_ROT_BOUND; n = 2;
            S.nbodies[e] = B.nb; S.nshapes[e] = B.ns; S.ncons[e] = B.nc;
            randomise_all(S, L, e, lane, ents, n, rr, JITTER_POS_BOUND, rl);
        }
    } else if (task_is<TASK>(cfg.task, MG_TASK_CLUSTER_COLOUR) || task_is<TASK>(cfg.task, MG_TASK_CLUSTER_SHAPE)) {
        int by = task_is<TASK>(cfg.task, MG_TASK_CLUSTER_SHAPE) ? 1 : 0;
        int nblk = 8;
        bool count = (f & MG_RAND_SHAPE_COUNT) != 0;
        if (count) nblk = mt_randint(S, e, 7, 10 + 1);
        int cols[10], types[10];
        if (f & MG_RAND_COLOUR) {
            for (int i = 0; i < 4; i++) cols[i] = MG_SHAPE_COLOURS[i];
            for (int i = 4; i < nblk; i++) cols[i] = MG_SHAPE_COLOURS[mt_randint(S, e, 0, 4)];
            for (int i = nblk - 1; i >= 1; i--) { int j = (int)mt_masked(S, e, (uint32_t)i); int t = cols[i]; cols[i] = cols[j]; cols[j] = t; }
        } else for (int i = 0; i < 8; i++) cols[i] = CC_COLOURS[by][i];
        if (f & MG_RAND_SHAPE_TYPE) {
            for (int i = 0; i < 4; i++) types[i] = MG_SHAPE_TYPES[i];
            for (int i = 4; i < nblk; i++) types[i] = MG_SHAPE_TYPES[mt_randint(S, e, 0, 4)];
            for (int i = nblk - 1; i >= 1; i--) { int j = (int)mt_masked(S, e, (uint32_t)i); int t = types[i]; types[i] = types[j]; types[j] = t; }
        } else for (int i = 0; i < 8; i++) types[i] = CC_TYPES[by][i];
        for (int i = 0; i < nblk; i++) {
            double x = count ? 0.0 : CC_POSES[by][i][0], y = count ? 0.0 : CC_POSES[by][i][1], a = count ? 0.0 : CC_POSES[by][i][2];
            inst_block(S, L, e, B, types[i], cols[i], 0, x, y, a, star_groups);
        }
        inst_robot(S, L, e, B, CC_ROBOT[by][0], CC_ROBOT[by][1], CC_ROBOT[by][2]);
        if (any_layout) {
            bool full = LAYOUT == 0 ? false : (f & MG_RAND_LAYOUT_FULL) != 0;
            ents[0] = 1 + nblk;
            for (int i = 0; i < nblk; i++) ents[1 + i] = 1 + i;
            n = nblk + 1;
            for (int i = 0; i < n; i++) { rr[i] = true; rl[i] = full ? -1.0 : JITTER_ROT_BOUND; }
            S.nbodies[e] = B.nb; S.nshapes[e] = B.ns; S.ncons[e] = B.nc;
            randomise_all(S, L, e, lane, ents, n, rr, full ? -1.0 : JITTER_POS_BOUND, rl);
        }
    } else if (task_is<TASK>(cfg.task, MG_TASK_MAKE_LINE)) { // make_line.py:86-132
        int nblk = 4;
        const bool count = (f & MG_RAND_SHAPE_COUNT) != 0;
        if (count) nblk = mt_randint(S, e, 3, 4 + 1);
        int cols[4], types[4];
        for (int i = 0; i < 4; i++) { cols[i] = ML_COLOURS[i]; types[i] = ML_TYPES[i]; }
        if (f & MG_RAND_COLOUR) for (int i = 0; i < nblk; i++) cols[i] = MG_SHAPE_COLOURS[mt_randint(S, e, 0, 4)];
        if (f & MG_RAND_SHAPE_TYPE) for (int i = 0; i < nblk; i++) types[i] = MG_SHAPE_TYPES[mt_randint(S, e, 0, 4)];
        for (int i = 0; i < nblk; i++) { // with a random count every block starts at the first default pose
            const int k = count ? 0 : i;
            inst_block(S, L, e, B, types[i], cols[i], 0, ML_POSES[k][0], ML_POSES[k][1], ML_POSES[k][2], star_groups);
        }
        inst_robot(S, L, e, B, 0.702, -0.255, 0.347);
        if (any_layout) {
            ents[0] = 1 + nblk; // robot, then the blocks
            for (int i = 0; i < nblk; i++) ents[1 + i] = 1 + i;
            n = nblk + 1;
            for (int i = 0; i < n; i++) { rr[i] = true; rl[i] = minor ? JITTER_ROT_BOUND : -1.0; }
            S.nbodies[e] = B.nb; S.nshapes[e] = B.ns; S.ncons[e] = B.nc;
            randomise_all(S, L, e, lane, ents, n, rr, minor ? JITTER_POS_BOUND : -1.0, rl);
        }
    } else if (task_is<TASK>(cfg.task, MG_TASK_FIND_DUPE)) { // find_dupe.py:62-199
        int qcol = MG_COL_YELLOW, qtype = MG_SHAPE_PENTAGON, cols[6], types[6];
        for (int i = 0; i < 6; i++) { cols[i] = FD_OUT_COLOURS[i]; types[i] = FD_OUT_TYPES[i]; }
        const bool count = (f & MG_RAND_SHAPE_COUNT) != 0;
        const int n_out = count ? mt_randint(S, e, 1, 5 + 1) + 1 : 6, nd = n_out - 1;
        if (f & MG_RAND_COLOUR) {
            qcol = MG_SHAPE_COLOURS[mt_randint(S, e, 0, 4)];
            for (int i = 0; i < nd; i++) cols[i] = MG_SHAPE_COLOURS[mt_randint(S, e, 0, 4)];
            cols[nd] = qcol;
        }
        if (f & MG_RAND_SHAPE_TYPE) {
            qtype = MG_SHAPE_TYPES[mt_randint(S, e, 0, 4)];
            for (int i = 0; i < nd; i++) types[i] = MG_SHAPE_TYPES[mt_randint(S, e, 0, 4)];
            types[nd] = qtype;
        }
        double th = 0.67, tw = 0.72;
        if (any_layout) randomise_hw(S, e, th, tw, minor ? JITTER_TARGET_BOUND : -1.0, th, tw);
        inst_goal(S, e, B, -0.72, -0.22, th, tw, qcol); // entity 1
        for (int i = 0; i < n_out; i++) // role 1: same colour and shape as the query (target set), 2: distractor
            inst_block(S, L, e, B, types[i], cols[i], (cols[i] == qcol && types[i] == qtype) ? 1 : 2,
                       count ? 0.0 : FD_OUT_POSES[i][0], count ? 0.0 : FD_OUT_POSES[i][1],
                       count ? 0.0 : FD_OUT_POSES[i][2], star_groups);
        inst_block(S, L, e, B, qtype, qcol, 1, -0.33, -0.49, -0.51, star_groups);
        const int query = S.nents[e] - 1;
        inst_robot(S, L, e, B, -0.57, 0.25, 3.83);
        if (any_layout) {
            n = 0;
            ents[n++] = 1;                 // sensor
            ents[n++] = S.nents[e] - 1;    // robot
            for (int i = 0; i < n_out; i++) ents[n++] = 2 + i;
            for (int i = 0; i < n; i++) { rr[i] = i != 0; rl[i] = minor ? JITTER_ROT_BOUND : -1.0; }
            S.nbodies[e] = B.nb; S.nshapes[e] = B.ns; S.ncons[e] = B.nc;
            randomise_all(S, L, e, lane, ents, n, rr, minor ? JITTER_POS_BOUND : -1.0, rl, 1u << query);
            if (!(S.overflow[e] & 2)) { // the query block last, mostly inside the placed sensor
                double lim = fmin(th, tw) / 2 - L->robot_radius * 0.6 / 2;
                lim = lim > 0 ? lim : 0.0;
                if (minor) lim = fmin(JITTER_POS_BOUND, lim);
                shift_entity(S, e, query, v2(AT(S.ex, 1), AT(S.ey, 1)), AT(S.ba, AT(S.ebody0, query)));
                if (randomise_pose(S, L, e, lane, query, true, lim, minor ? JITTER_ROT_BOUND : -1.0, 1u << 1) != 0)
                    S.overflow[e] |= 2 | 64;
            }
        }
    } else if (task_is<TASK>(cfg.task, MG_TASK_FIX_COLOUR)) { // fix_colour.py:67-176
        const bool count = (f & MG_RAND_SHAPE_COUNT) != 0;
        const int nr = count ? mt_randint(S, e, 2, 3 + 1) : 3;
        int rcols[3], bcols[3], types[3];
        double rh[3], rw[3];
        for (int i = 0; i < 3; i++) {
            const int k = count ? 0 : i;
            rcols[i] = FC_REGION_COLOURS[i]; bcols[i] = FC_BLOCK_COLOURS[i]; types[i] = FC_BLOCK_TYPES[i];
            rh[i] = FC_REGIONS[k][2]; rw[i] = FC_REGIONS[k][3];
        }
        if (f & MG_RAND_COLOUR) {
            for (int i = 0; i < nr; i++) rcols[i] = MG_SHAPE_COLOURS[mt_randint(S, e, 0, 4)];
            for (int i = 0; i < nr; i++) bcols[i] = rcols[i];
            const int odd = mt_randint(S, e, 0, nr);
            int nc = mt_randint(S, e, 0, 4 - 1);
            if (MG_SHAPE_COLOURS[nc] == bcols[odd]) nc++;
            bcols[odd] = MG_SHAPE_COLOURS[nc];
        }
        if (f & MG_RAND_SHAPE_TYPE) for (int i = 0; i < nr; i++) types[i] = MG_SHAPE_TYPES[mt_randint(S, e, 0, 4)];
        if (any_layout)
            for (int i = 0; i < nr; i++)
                randomise_hw(S, e, rh[i], rw[i], minor ? JITTER_TARGET_BOUND : -1.0, rh[i], rw[i], 0.4, 0.5);
        for (int i = 0; i < nr; i++) { // regions: entities 1 .. nr
            const int k = count ? 0 : i;
            inst_goal(S, e, B, FC_REGIONS[k][0], FC_REGIONS[k][1], rh[i], rw[i], rcols[i]);
        }
        for (int i = 0; i < nr; i++) { // blocks: entities nr+1 .. 2nr; role 1: matches its region's colour
            const int k = count ? 0 : i;
            inst_block(S, L, e, B, types[i], bcols[i], bcols[i] == rcols[i] ? 1 : 2, FC_BLOCK_POSES[k][0],
                       FC_BLOCK_POSES[k][1], FC_BLOCK_POSES[k][2], star_groups);
        }
        inst_robot(S, L, e, B, 0.368, 0.586, 0.718);
        if (any_layout) {
            n = 0;
            uint32_t blocks = 0u;
            for (int i = 0; i < nr; i++) { ents[n++] = 1 + i; blocks |= 1u << (1 + nr + i); }
            ents[n++] = S.nents[e] - 1;
            for (int i = 0; i < n; i++) { rr[i] = i == nr; rl[i] = minor ? JITTER_ROT_BOUND : -1.0; }
            S.nbodies[e] = B.nb; S.nshapes[e] = B.ns; S.ncons[e] = B.nc;
            randomise_all(S, L, e, lane, ents, n, rr, minor ? JITTER_POS_BOUND : -1.0, rl, blocks);
            if (!(S.overflow[e] & 2)) {
                for (int i = 0; i < nr; i++) {
                    const int b = 1 + nr + i;
                    shift_entity(S, e, b, v2(AT(S.ex, 1 + i), AT(S.ey, 1 + i)), AT(S.ba, AT(S.ebody0, b)));
                }
                for (int i = 0; i < nr; i++) {
                    double lim = fmin(rh[i], rw[i]) / 2 - L->robot_radius * 0.6;
                    lim = lim > 0 ? lim : 0.0;
                    if (minor) lim = fmin(JITTER_POS_BOUND, lim);
                    if (randomise_pose(S, L, e, lane, 1 + nr + i, true, lim, minor ? JITTER_ROT_BOUND : -1.0, 1u << (1 + i)) != 0) {
                        S.overflow[e] |= 2 | 64;
                        break;
                    }
                }
            }
        }
    } else if (task_is<TASK>(cfg.task, MG_TASK_PICK_AND_PLACE)) { // pick_and_place.py:30-85
        inst_robot(S, L, e, B, 0.0, 0.0, 0.55 * 3.141592653589793); // entity 1: added before the shapes
        int cols[3], types[3];
        for (int i = 0; i < 3; i++) { // per shape: colour draw, then type draw
            cols[i] = MG_COL_RED; types[i] = MG_SHAPE_SQUARE;
            if (f & MG_RAND_COLOUR) cols[i] = MG_SHAPE_COLOURS[mt_randint(S, e, 0, 4)];
            if (f & MG_RAND_SHAPE_TYPE) types[i] = MG_SHAPE_TYPES[mt_randint(S, e, 0, 4)];
        }
        for (int i = 0; i < 3; i++)
            inst_block(S, L, e, B, types[i], cols[i], 0, 0.1, -0.65, 0.13 * 3.141592653589793, star_groups);
        int tid = 0, cid = 0;
        for (int k = 0; k < 4; k++) {
            if (MG_SHAPE_TYPES[k] == types[0]) tid = k;
            if (MG_SHAPE_COLOURS[k] == cols[0]) cid = k;
        }
        const double tx = mt_double(S, e), ty = mt_double(S, e); // rng.rand(2) * 2 - 1
        S.tgt_x[e] = tx * 2 - 1; S.tgt_y[e] = ty * 2 - 1;
        S.tgt_ids[e] = tid; S.tgt_ids[N + e] = cid;
        int valid[3], nv = 0;
        for (int i = 0; i < 3; i++) if (types[i] == types[0] && cols[i] == cols[0]) valid[nv++] = 2 + i;
        S.tgt_ent[e] = valid[mt_randint(S, e, 0, nv)]; // rng.choice(valid_target_shapes)
        if (any_layout) { // rand_poses: robot and shapes, unrestricted
            n = 4;
            for (int i = 0; i < 4; i++) { ents[i] = 1 + i; rr[i] = true; rl[i] = -1.0; }
            S.nbodies[e] = B.nb; S.nshapes[e] = B.ns; S.ncons[e] = B.nc;
            randomise_all(S, L, e, lane, ents, n, rr, -1.0, rl);
        }
        if (S.target_out) {
            double *t = S.target_out + 4 * (size_t)e;
            t[0] = tid; t[1] = cid; t[2] = S.tgt_x[e]; t[3] = S.tgt_y[e];
        }
    } else { // MatchRegions
        int target = MG_COL_GREEN;
        if (f & MG_RAND_COLOUR) target = MG_SHAPE_COLOURS[mt_randint(S, e, 0, 4)];
        int dcols[3], nd = 0;
        for (int i = 0; i < 4; i++) if (MG_SHAPE_COLOURS[i] != target) dcols[nd++] = MG_SHAPE_COLOURS[i];
        double th = 0.7, tw = 0.6;
        if (any_layout) randomise_hw(S, e, th, tw, minor ? JITTER_TARGET_BOUND : -1.0, th, tw);
        inst_goal(S, e, B, 0.1, 0.7, th, tw, target);
        const int dtt[2] = {MG_SHAPE_STAR, MG_SHAPE_SQUARE};
        const int ddt[3][2] = {{0, 0}, {MG_SHAPE_PENTAGON, 0}, {MG_SHAPE_CIRCLE, MG_SHAPE_PENTAGON}};
        const double dtp[2][3] = {{0.8, -0.7, 2.37}, {-0.68, 0.72, 1.28}};
        const double ddp[3][2][3] = {{{0, 0, 0}, {0, 0, 0}}, {{-0.05, -0.2, -1.09}, {0, 0, 0}},
                                     {{-0.75, -0.55, 2.78}, {0.3, -0.82, -1.15}}};
        int tcount = 2, dcount[3] = {0, 1, 2};
        if (f & MG_RAND_SHAPE_COUNT) {
            tcount = mt_randint(S, e, 1, 3);
            for (int i = 0; i < 3; i++) dcount[i] = mt_randint(S, e, 0, 3);
        }
        int ttypes[2], dtypes[3][2];
        if (f & MG_RAND_SHAPE_TYPE) {
            for (int i = 0; i < tcount; i++) ttypes[i] = MG_SHAPE_TYPES[mt_randint(S, e, 0, 4)];
            for (int c = 0; c < 3; c++)
                for (int i = 0; i < dcount[c]; i++) dtypes[c][i] = MG_SHAPE_TYPES[mt_randint(S, e, 0, 4)];
        } else {
            ttypes[0] = dtt[0]; ttypes[1] = dtt[1];
            for (int c = 0; c < 3; c++) { dtypes[c][0] = ddt[c][0]; dtypes[c][1] = ddt[c][1]; }
        }
        bool full = LAYOUT == 0 ? false : (f & MG_RAND_LAYOUT_FULL) != 0;
        int first = S.nents[e];
        for (int i = 0; i < tcount; i++)
            inst_block(S, L, e, B, ttypes[i], target, 1, full ? 0.0 : dtp[i][0], full ? 0.0 : dtp[i][1], full ? 0.0 : dtp[i][2],
                       star_groups);
        for (int c = 0; c < 3; c++)
            for (int i = 0; i < dcount[c]; i++)
                inst_block(S, L, e, B, dtypes[c][i], dcols[c], 2, full ? 0.0 : ddp[c][i][0], full ? 0.0 : ddp[c][i][1],
                           full ? 0.0 : ddp[c][i][2], star_groups);
        int nblk = S.nents[e] - first;
        inst_robot(S, L, e, B, -0.5, 0.1, -3.141592653589793 * 1.2);
        if (any_layout) {
            n = 0;
            ents[n++] = 1;                 // sensor
            ents[n++] = S.nents[e] - 1;    // robot
            for (int i = 0; i < nblk; i++) ents[n++] = first + i;
            for (int i = 0; i < n; i++) { rr[i] = i != 0; rl[i] = minor ? JITTER_ROT_BOUND : -1.0; }
            S.nbodies[e] = B.nb; S.nshapes[e] = B.ns; S.ncons[e] = B.nc;
            randomise_all(S, L, e, lane, ents, n, rr, minor ? JITTER_POS_BOUND : -1.0, rl);
        }
    }
    S.nbodies[e] = B.nb; S.nshapes[e] = B.ns; S.ncons[e] = B.nc;
    // shapes left with categories 0 by the randomiser collide with nothing for the episode (step broadphase,
    // goal queries): folded into the group the step kernels already read
    for (int k = 0; k < B.ns; k++)
        if (!AT(S.scat, k)) AT(S.sgroup, k) = (int16_t)(AT(S.sgroup, k) | MG_GROUP_OFF);
}
