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

MG_DEV double score_env(const MGState &S, const mg_library *L, int e, int task) {
    int rb = S.robot_body0[e];
    V2 rp = v2(AT(S.bpx, rb), AT(S.bpy, rb));
    if (task == MG_TASK_MOVE_TO_REGION) {
        int ge = S.goal_ent[e];
        ShapeW G;
        load_goal(S.gpx[e], S.gpy[e], AT(S.ew, ge), AT(S.eh, ge), 0, G);
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
    // MatchRegions
    int ge = S.goal_ent[e];
    ShapeW G;
    load_goal(S.gpx[e], S.gpy[e], AT(S.ew, ge), AT(S.eh, ge), 0, G);
    int n_t = 0, n_d = 0, n_in = 0, total_t = 0;
    for (int i = 0; i < nents; i++) {
        if (AT(S.ekind, i) != MG_ENT_BLOCK) continue;
        if (AT(S.erole, i) == 1) total_t++;
        int s0 = AT(S.eshape0, i), ns = AT(S.enshapes, i);
        bool any = false, all = true;
        for (int k = s0; k < s0 + ns; k++) {
            ShapeW A;
            load_shape(S, L, e, k, 0, A);
            bool hit = false;
            if (bb_intersects(G, A)) {
                Collision info;
                collide(G, A, info);
                if (info.count) {
                    V2 p = v2(AT(S.bpx, A.body), AT(S.bpy, A.body));
                    hit = G.bbl <= p.x && G.bbr >= p.x && G.bbb <= p.y && G.bbt >= p.y;
                }
            }
            if (hit) any = true; else all = false;
        }
        if (any && all) {
            n_in++;
            if (AT(S.erole, i) == 1) n_t++; else n_d++;
        }
    }
    double frac = (double)n_t / total_t;
    double contamination = n_in == 0 ? 0.0 : (double)n_d / n_in;
    return frac * (1 - contamination);
}
