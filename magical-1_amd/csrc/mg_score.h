// mg_score.h -- score_on_end_of_traj of the four hot-path tasks, per lane.
//
// move_to_region.py:85-94 (goal point query), move_to_corner.py:161-171
// (robot distance to (-1, 1)), cluster.py:166-216 (centroid margins),
// match_regions.py:193-213 + entities.py:803-863 (goal shape query, COM
// filter, all-shapes-of-entity rule).
#pragma once
#include "mg_reset.h"

MG_DEV double poly_point_query(const ShapeW &sh, V2 p) {
    int count = sh.count;
    V2 v0 = sh.v[count - 1];
    double minDist = INFINITY;
    bool outside = false;
    for (int i = 0; i < count; i++) {
        V2 v1 = sh.v[i];
        outside = outside || (vdot(sh.pn[i], vsub(p, v1)) > 0.0);
        V2 delta = vsub(v0, v1);
        double t = cpclamp01(vdot(delta, vsub(p, v1)) / vlengthsq(delta));
        V2 closest = vadd(v1, vmult(delta, t));
        double dist = vlength(vsub(p, closest));
        if (dist < minDist) minDist = dist;
        v0 = v1;
    }
    double dist = outside ? minDist : -minDist;
    return dist - sh.r;
}

#define MG_MAX_LINE 8
// make_line.py:33-74 longest_line in the reference's numpy arithmetic (oracle/scene.c o_longest_line):
// norm of one 2-vector = sqrt(ddot) = sqrt(fma(y, y, x*x)); offs @ unit (gemv) = fma(x, ux, y*uy);
// norm(axis=1) = sqrt(x*x + y*y)
MG_DEV int longest_line(const double *px, const double *py, int n, double inlier_dist, double max_sep) {
    int best = n < 1 ? n : 1;
    for (int i = 0; i < n - 1; i++)
        for (int j = i + 1; j < n; j++) {
            double inl[MG_MAX_LINE];
            const double jx = px[j] - px[i], jy = py[j] - py[i];
            const double nrm = sqrt(__fma_rn(jy, jy, jx * jx));
            const double ux = jx / nrm, uy = jy / nrm;
            int ni = 0;
            for (int k = 0; k < n; k++) {
                const double ox = px[k] - px[i], oy = py[k] - py[i];
                const double proj = __fma_rn(ox, ux, oy * uy);
                const double dx = ox - proj * ux, dy = oy - proj * uy;
                if (sqrt(dx * dx + dy * dy) <= inlier_dist) inl[ni++] = proj;
            }
            if (ni <= best) continue;
            for (int a = 1; a < ni; a++) {
                const double v = inl[a];
                int b = a - 1;
                while (b >= 0 && inl[b] > v) { inl[b + 1] = inl[b]; b--; }
                inl[b + 1] = v;
            }
            int run = 0, max_run = 0;
            for (int k = 0; k + 1 < ni; k++) {
                if (fabs(inl[k + 1] - inl[k]) <= max_sep) { run++; max_run = run > max_run ? run : max_run; }
                else run = 0;
            }
            best = max_run + 1 > best ? max_run + 1 : best;
        }
    return best;
}

// entities.py:803-863 get_overlapping_ents(com_overlap=True) of goal entity ge over the blocks: bit i set
// when every shape of block i overlaps the goal with its body's position inside the goal's BB
MG_DEV uint32_t goal_overlap_blocks(const MGState &S, const mg_library *L, int e, int ge) {
    if (AT(S.eshape0, ge) == 0) return 0u; // the goal's categories are 0 (MG_GROUP_OFF): the query rejects all
    ShapeW G;
    load_goal(AT(S.ex, ge), AT(S.ey, ge), AT(S.ew, ge), AT(S.eh, ge), 0, G);
    const int nents = S.nents[e];
    uint32_t in = 0u;
    for (int i = 0; i < nents; i++) {
        if (AT(S.ekind, i) != MG_ENT_BLOCK) continue;
        int s0 = AT(S.eshape0, i), ns = AT(S.enshapes, i);
        bool any = false, all = true;
        for (int k = s0; k < s0 + ns; k++) {
            ShapeW A;
            load_shape(S, L, e, k, 0, A);
            bool hit = false;
            if (bb_intersects(G, A) && !(AT(S.sgroup, k) & MG_GROUP_OFF)) {
                Collision info;
                collide(G, A, info);
                if (info.count) {
                    V2 p = v2(AT(S.bpx, A.body), AT(S.bpy, A.body));
                    hit = G.bbl <= p.x && G.bbr >= p.x && G.bbb <= p.y && G.bbt >= p.y;
                }
            }
            if (hit) any = true; else all = false;
        }
        if (any && all) in |= 1u << i;
    }
    return in;
}

MG_DEV double score_env(const MGState &S, const mg_library *L, int e, int task) {
    int rb = S.robot_body0[e];
    V2 rp = v2(AT(S.bpx, rb), AT(S.bpy, rb));
    if (task == MG_TASK_MOVE_TO_REGION) {
        int ge = S.goal_ent[e];
        ShapeW G;
        load_goal(AT(S.ex, ge), AT(S.ey, ge), AT(S.ew, ge), AT(S.eh, ge), 0, G);
        return poly_point_query(G, rp) <= 0 ? 1.0 : 0.0;
    }
    if (task == MG_TASK_MOVE_TO_CORNER) {
        double dx = -1.0 - rp.x, dy = 1.0 - rp.y;
        double dist = sqrt(__fma_rn(dy, dy, dx * dx)); // np.linalg.norm -> BLAS ddot
        double succeed = sqrt(2.0) / 2, furthest = sqrt(2.0);
        double drange = furthest - succeed;
        double v = furthest - dist;
        double sc = (v > 0.0 ? v : 0.0) / drange;
        return sc < 1.0 ? sc : 1.0;
    }
    const int nents = S.nents[e];
    if (task == MG_TASK_CLUSTER_COLOUR || task == MG_TASK_CLUSTER_SHAPE) {
        bool by_type = task == MG_TASK_CLUSTER_SHAPE;
        // np.unique order of the str-enum values
        const int CORD[4] = {MG_COL_BLUE, MG_COL_GREEN, MG_COL_RED, MG_COL_YELLOW};
        const int TORD[4] = {MG_SHAPE_CIRCLE, MG_SHAPE_PENTAGON, MG_SHAPE_SQUARE, MG_SHAPE_STAR};
        int vals[4], nv = 0;
        for (int k = 0; k < 4; k++) {
            int want = by_type ? TORD[k] : CORD[k];
            for (int i = 0; i < nents; i++)
                if (AT(S.ekind, i) == MG_ENT_BLOCK && (by_type ? AT(S.etype, i) : AT(S.ecol, i)) == want) { vals[nv++] = want; break; }
        }
        double cx[4], cy[4];
        for (int c = 0; c < nv; c++) {
            double sx = 0, sy = 0; int cnt = 0;
            for (int i = 0; i < nents; i++) {
                if (AT(S.ekind, i) != MG_ENT_BLOCK || (by_type ? AT(S.etype, i) : AT(S.ecol, i)) != vals[c]) continue;
                int b = AT(S.ebody0, i);
                if (cnt == 0) { sx = AT(S.bpx, b); sy = AT(S.bpy, b); } else { sx += AT(S.bpx, b); sy += AT(S.bpy, b); }
                cnt++;
            }
            cx[c] = sx / cnt; cy[c] = sy / cnt;
        }
        int n_blocks = 0, n_correct = 0;
        for (int c = 0; c < nv; c++)
            for (int i = 0; i < nents; i++) {
                if (AT(S.ekind, i) != MG_ENT_BLOCK || (by_type ? AT(S.etype, i) : AT(S.ecol, i)) != vals[c]) continue;
                n_blocks++;
                int b = AT(S.ebody0, i);
                double px = AT(S.bpx, b), py = AT(S.bpy, b);
                double true_sse = 0, nearest_bad = INFINITY;
                for (int k = 0; k < nv; k++) {
                    double dx = px - cx[k], dy = py - cy[k];
                    double sse = dx * dx + dy * dy;
                    if (k == c) true_sse = sse;
                    else if (sse < nearest_bad) nearest_bad = sse;
                }
                double margin = 2.0 * true_sse;
                n_correct += (sqrt(true_sse) < sqrt(nearest_bad) - margin) ? 1 : 0;
            }
        double frac = (double)n_correct / (n_blocks > 1 ? n_blocks : 1);
        double v = frac - 0.75;
        return (v > 0 ? v : 0) / (1 - 0.75);
    }
    if (task == MG_TASK_MAKE_LINE) { // make_line.py:140-152
        double px[MG_MAX_LINE], py[MG_MAX_LINE];
        int n = 0;
        for (int i = 0; i < nents && n < MG_MAX_LINE; i++) {
            if (AT(S.ekind, i) != MG_ENT_BLOCK) continue;
            const int b = AT(S.ebody0, i);
            px[n] = AT(S.bpx, b); py[n] = AT(S.bpy, b); n++;
        }
        const double rad = L->robot_radius * 0.6; // BaseEnv.SHAPE_RAD
        const int line_len = longest_line(px, py, n, rad * 1.5, rad * 3.5);
        const int min_len = n - 2 > 2 ? n - 2 : 2, d = line_len - min_len;
        return (double)(d > 0 ? d : 0) / (double)(n - min_len);
    }
    if (task == MG_TASK_PICK_AND_PLACE) { // pick_and_place.py:87-101
        const int tb = AT(S.ebody0, S.tgt_ent[e]);
        const double dx = S.tgt_x[e] - AT(S.bpx, tb), dy = S.tgt_y[e] - AT(S.bpy, tb);
        const double dist = sqrt(__fma_rn(dy, dy, dx * dx)); // np.linalg.norm -> BLAS ddot
        const double succeed = L->robot_radius * 0.6, furthest = sqrt(2.0);
        const double drange = furthest - succeed;
        const double v = furthest - dist;
        const double sc = (v > 0.0 ? v : 0.0) / drange;
        return sc < 1.0 ? sc : 1.0;
    }
    if (task == MG_TASK_FIND_DUPE) { // find_dupe.py:202-216
        const uint32_t in = goal_overlap_blocks(S, L, e, S.goal_ent[e]);
        int n_t = 0, n_d = 0, n_in = 0;
        for (int i = 0; i < nents; i++) {
            if (!((in >> i) & 1u)) continue;
            n_in++;
            if (AT(S.erole, i) == 1) n_t++; else n_d++;
        }
        const double have_two = n_t >= 2 ? 1.0 : 0.0;
        const double contamination = n_in == 0 ? 0.0 : (double)n_d / n_in;
        return have_two * (1 - contamination);
    }
    if (task == MG_TASK_FIX_COLOUR) { // fix_colour.py:181-192: region r holds exactly block r iff it matches
        int goals[MG_MAX_ENTS], blocks[MG_MAX_ENTS], ng = 0, nb = 0;
        for (int i = 0; i < nents; i++) {
            if (AT(S.ekind, i) == MG_ENT_GOAL) goals[ng++] = i;
            if (AT(S.ekind, i) == MG_ENT_BLOCK) blocks[nb++] = i;
        }
        for (int r = 0; r < ng && r < nb; r++) {
            const uint32_t in = goal_overlap_blocks(S, L, e, goals[r]);
            const bool want = AT(S.erole, blocks[r]) == 1;
            if (want ? in != (1u << blocks[r]) : in != 0u) return 0.0;
        }
        return 1.0;
    }
    // MatchRegions
    const uint32_t in = goal_overlap_blocks(S, L, e, S.goal_ent[e]);
    int n_t = 0, n_d = 0, n_in = 0, total_t = 0;
    for (int i = 0; i < nents; i++) {
        if (AT(S.ekind, i) != MG_ENT_BLOCK) continue;
        if (AT(S.erole, i) == 1) total_t++;
        if ((in >> i) & 1u) {
            n_in++;
            if (AT(S.erole, i) == 1) n_t++; else n_d++;
        }
    }
    double frac = (double)n_t / total_t;
    double contamination = n_in == 0 ? 0.0 : (double)n_d / n_in;
    return frac * (1 - contamination);
}

// debug_shaped_reward (debug_reward=True): move_to_corner.py:85-100, pick_and_place.py:114-124
MG_DEV double debug_reward(const MGState &S, const mg_library *L, int e, int task) {
    const int rb = S.robot_body0[e];
    const double rx = AT(S.bpx, rb), ry = AT(S.bpy, rb);
    if (task == MG_TASK_PICK_AND_PLACE) {
        const int tb = AT(S.ebody0, S.tgt_ent[e]);
        const double px = AT(S.bpx, tb), py = AT(S.bpy, tb);
        const double ax = px - S.tgt_x[e], ay = py - S.tgt_y[e];
        const double s2t = sqrt(__fma_rn(ay, ay, ax * ax));
        const double bx = rx - px, by = ry - py;
        const double r2s = sqrt(__fma_rn(by, by, bx * bx));
        const double rad = L->robot_radius * 0.6;
        const double shaping = -s2t / 5 - (r2s > rad ? r2s : rad) / 10;
        return shaping + score_env(S, L, e, task);
    }
    int shape = -1; // MoveToCorner: the block
    for (int i = 0; i < S.nents[e] && shape < 0; i++) if (AT(S.ekind, i) == MG_ENT_BLOCK) shape = i;
    const int sb = AT(S.ebody0, shape);
    const double px = AT(S.bpx, sb), py = AT(S.bpy, sb);
    const double ax = px - 0.0, ay = py - 1.0;
    const double s2c = sqrt(__fma_rn(ay, ay, ax * ax));
    const double bx = rx - px, by = ry - py;
    const double r2s = sqrt(__fma_rn(by, by, bx * bx));
    const double shaping = -s2c / 5 - (r2s > 0.2 ? r2s : 0.2) / 20;
    return shaping + score_env(S, L, e, task);
}
