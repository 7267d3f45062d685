// mg_render.h -- headless Viewer raster + LoRes downsample, one workgroup per (env, view).
//
// Replaces render.py:151-287 / 385-395 (Geom.render, Poly._render ->
// pygame.draw.polygon + width-2 lines + dashed width-4 goal outlines,
// surfarray) and benchmarks/__init__.py:150-190 (cv2.resize INTER_AREA 4x).
// The 384x384 frame never leaves the CU: it is produced in 8-row bands in LDS
// where each covered pixel receives atomicMax(draw ordinal) -- the painter's
// algorithm is "the last primitive drawn wins", i.e. the maximum ordinal -- so
// every fill span and outline pixel can be rasterised concurrently.  Each
// finished band is reduced 4x4 -> 2 output rows (round half to even of
// sum/16, OpenCV resizeAreaFast) and written straight to HBM.
#pragma once
#include "mg_step.h"

#define RG_MAXG 160
#define RG_MAXVERT 2048
#define RG_MAXSPAN 6144
#define RG_MAXDASH 512
#define RG_BAND 8
#define RG_THREADS 256
#define RG_LOROW (MG_LORES * 3)         // bytes of one 96-px RGB row
#define RG_BANDLO (2 * RG_LOROW)        // bytes of the 2 LoRes rows one band produces
#define RG_BANDLO16 (RG_BANDLO / 16)    // ... in 16-byte chunks (36)

struct RenderOut {
    uint8_t *full;      // [N][2][384][384][3] (full-resolution mode) or null
    uint8_t *obs_allo;  // LoRes outputs (layout per preproc), or null
    uint8_t *obs_ego;
    uint8_t *obs_past;
    const uint8_t *mask;  // reset mask: envs with mask[e] == 0 are left untouched (null: all)
    int preproc;
};

// LDS: the setup stages (matrices) and the band stages (band buffer + LoRes
// staging) never live at the same time, so they share storage.
struct RenderSmem {
    union {
        struct {
            double g_m[RG_MAXG][6];
            double e_xf[MG_MAX_ENTS][5][9];
            double view[9];
        } pre;
        struct {
            uint32_t band[RG_BAND][MG_RES];
            uint4 lo[RG_BANDLO16];          // current frame, 2 LoRes rows
            uint4 past[3][RG_BANDLO16];     // frames t-3, t-2, t-1 of the same rows
        } post;
    } u;
    int16_t g_rpoly[RG_MAXG], g_voff[RG_MAXG], g_nv[RG_MAXG];
    int16_t g_ymin[RG_MAXG], g_ymax[RG_MAXG], g_xmin[RG_MAXG], g_xmax[RG_MAXG];
    int8_t g_ent[RG_MAXG];
    int32_t g_soff[RG_MAXG + 1];
    int16_t e_g0[MG_MAX_ENTS + 1];
    int16_t vx[RG_MAXVERT], vy[RG_MAXVERT];   // int pixel vertices (fill, line ends)
    int16_t fx[RG_MAXVERT], fy[RG_MAXVERT];   // float->int first points of solid outline edges
    uint8_t v_geom[RG_MAXVERT];
    int16_t sedge[RG_MAXVERT];                // solid outline edges (start vertex)
    int16_t span_l[RG_MAXSPAN], span_r[RG_MAXSPAN];
    int16_t dash[RG_MAXDASH][4];              // clipped dashed-outline lines
    int16_t dash_o[RG_MAXDASH];
    uint32_t col[2 * RG_MAXG + 2];
    int32_t ngeom, nvert, nspan, nsedge, ndash, err;
};

MG_DEV uint32_t pack_rgb(const uint8_t *c) { return (uint32_t)c[0] | ((uint32_t)c[1] << 8) | ((uint32_t)c[2] << 16); }

MG_DEV uint32_t ref_colour(const mg_library *L, int ref, int ecol) {
    switch (ref) {
    case MG_RC_ENT_BASE: return pack_rgb(L->palette[ecol][0]);
    case MG_RC_ENT_DARK: return pack_rgb(L->palette[ecol][1]);
    case MG_RC_ENT_LIGHT2: return pack_rgb(L->palette[ecol][2]);
    case MG_RC_GREY_BASE: return pack_rgb(L->palette[MG_COL_GREY][0]);
    case MG_RC_GREY_DARK: return pack_rgb(L->palette[MG_COL_GREY][1]);
    case MG_RC_GREY_LIGHT4: return pack_rgb(L->palette[MG_COL_GREY][3]);
    case MG_RC_WHITE: return pack_rgb(L->white);
    default: return pack_rgb(L->pupil);
    }
}

// ---- pygame line clipping (Cohen-Sutherland with a float32 slope) ----------
MG_DEV int cs_encode(int x, int y) {
    int code = 0;
    if (x < 0) code |= 1;
    if (x > MG_RES - 1) code |= 2;
    if (y < 0) code |= 8;
    if (y > MG_RES - 1) code |= 4;
    return code;
}
MG_DEV bool clipline(int &x1, int &y1, int &x2, int &y2) {
    const int left = 0, top = 0, right = MG_RES - 1, bottom = MG_RES - 1;
    for (int guard = 0; guard < 16; guard++) {
        int code1 = cs_encode(x1, y1), code2 = cs_encode(x2, y2);
        if (!(code1 | code2)) return true;
        if (code1 & code2) return false;
        if (!code1) {
            int t = x2; x2 = x1; x1 = t;
            t = y2; y2 = y1; y1 = t;
            t = code2; code2 = code1; code1 = t;
        }
        float m = (x2 != x1) ? (float)(y2 - y1) / (float)(x2 - x1) : 1.0f;
        if (code1 & 1) { y1 += (int)((float)(left - x1) * m); x1 = left; }
        else if (code1 & 2) { y1 += (int)((float)(right - x1) * m); x1 = right; }
        else if (code1 & 4) { if (x2 != x1) x1 += (int)((float)(bottom - y1) / m); y1 = bottom; }
        else if (code1 & 8) { if (x2 != x1) x1 += (int)((float)(top - y1) / m); y1 = top; }
    }
    return false;
}

MG_DEV void push_line(RenderSmem &sm, int x1, int y1, int x2, int y2, int ord) {
    if (!clipline(x1, y1, x2, y2)) return;
    int i = atomicAdd(&sm.ndash, 1);
    if (i >= RG_MAXDASH) { sm.err = 1; return; }
    sm.dash[i][0] = (int16_t)x1; sm.dash[i][1] = (int16_t)y1; sm.dash[i][2] = (int16_t)x2; sm.dash[i][3] = (int16_t)y2;
    sm.dash_o[i] = (int16_t)ord;
}

// clip_and_draw_line_width (pygame 1.9.6): base line + offsets 1, -1, 2, ...
MG_DEV void push_wide_line(RenderSmem &sm, int x1, int y1, int x2, int y2, int width, int ord) {
    int xinc = 0, yinc = 0;
    if (abs(x1 - x2) > abs(y1 - y2)) yinc = 1; else xinc = 1;
    push_line(sm, x1, y1, x2, y2, ord);
    for (int loop = 1; loop < width; loop += 2) {
        int k = loop / 2 + 1;
        push_line(sm, x1 + xinc * k, y1 + yinc * k, x2 + xinc * k, y2 + yinc * k, ord);
        if (loop + 1 < width) push_line(sm, x1 - xinc * k, y1 - yinc * k, x2 - xinc * k, y2 - yinc * k, ord);
    }
}

// numpy arange(start, stop, step) element i (PyArray_ArangeObj + DOUBLE_fill)
MG_DEV int np_arange_len(double start, double stop, double step) {
    double l = ceil((stop - start) / step);
    return l > 0 ? (int)fmin(l, 4096.0) : 0;
}
MG_DEV double np_arange_at(double start, double step, int i) {
    if (i == 0) return start;
    double next = start + step;
    if (i == 1) return next;
    return start + i * (next - start);
}

// render.py:232-255 dashed goal outline, one polygon edge
MG_DEV void push_dashes(RenderSmem &sm, double x1, double y1, double x2, double y2, int ord) {
    const double dl = 10;
    double sx, stx, sy, sty;
    int nx, ny;
    bool constx = false, consty = false;
    if (x1 == x2) {
        sy = y1; sty = y1 < y2 ? dl : -dl; ny = np_arange_len(y1, y2, sty); nx = ny; constx = true; sx = x1; stx = 0;
    } else if (y1 == y2) {
        sx = x1; stx = x1 < x2 ? dl : -dl; nx = np_arange_len(x1, x2, stx); ny = nx; consty = true; sy = y1; sty = 0;
    } else {
        double a = fabs(x2 - x1), b = fabs(y2 - y1);
        double c = rint(sqrt(a * a + b * b));
        double dx = dl * a / c, dy = dl * b / c;
        sx = x1; stx = x1 < x2 ? dx : -dx; nx = np_arange_len(x1, x2, stx);
        sy = y1; sty = y1 < y2 ? dy : -dy; ny = np_arange_len(y1, y2, sty);
    }
    int n = nx < ny ? nx : ny;
    for (int k = 0; 2 * k + 1 < n; k++) {
        double xa = constx ? sx : np_arange_at(sx, stx, 2 * k + 1);
        double ya = consty ? sy : np_arange_at(sy, sty, 2 * k + 1);
        double xb = constx ? sx : np_arange_at(sx, stx, 2 * k);
        double yb = consty ? sy : np_arange_at(sy, sty, 2 * k);
        push_wide_line(sm, (int)rint(xa), (int)rint(ya), (int)rint(xb), (int)rint(yb), 4, ord);
    }
}

MG_DEV void band_put(RenderSmem &sm, int x, int y, int y0, uint32_t ord) {
    int r = y - y0;
    if (r >= 0 && r < RG_BAND && x >= 0 && x < MG_RES) atomicMax(&sm.u.post.band[r][x], ord);
}

// all pixels of a clipped line (pygame drawline) within rows [y0, y0 + RG_BAND)
MG_DEV void raster_line_band(RenderSmem &sm, int x1, int y1, int x2, int y2, uint32_t ord, int y0) {
    int y1b = y0 + RG_BAND - 1;
    if (y1 == y2) {
        if (y1 < y0 || y1 > y1b) return;
        int xa = x1 < x2 ? x1 : x2, xb = x1 < x2 ? x2 : x1;
        for (int x = xa; x <= xb; x++) band_put(sm, x, y1, y0, ord);
        return;
    }
    if (x1 == x2) {
        int ya = y1 < y2 ? y1 : y2, yb = y1 < y2 ? y2 : y1;
        ya = ya > y0 ? ya : y0; yb = yb < y1b ? yb : y1b;
        for (int y = ya; y <= yb; y++) band_put(sm, x1, y, y0, ord);
        return;
    }
    // drawline: major axis has (|d|+1) pixels; minor offset of pixel k = floor(k * dminor / dmajor)
    int dx = x2 - x1, dy = y2 - y1;
    int sgx = dx < 0 ? -1 : 1, sgy = dy < 0 ? -1 : 1;
    int DX = sgx * dx + 1, DY = sgy * dy + 1;
    if (DX >= DY) { // x major
        // rows y1 + sgy*m, m = floor(k*DY/DX); keep m with row in band
        int mlo, mhi;
        if (sgy > 0) { mlo = y0 - y1; mhi = y1b - y1; } else { mlo = y1 - y1b; mhi = y1 - y0; }
        if (mlo < 0) mlo = 0;
        if (mhi > DY - 1) mhi = DY - 1;
        if (mlo > mhi) return;
        int klo = (mlo * DX + DY - 1) / DY;            // smallest k with k*DY >= mlo*DX
        int khi = ((mhi + 1) * DX + DY - 1) / DY - 1;  // largest k with k*DY < (mhi+1)*DX
        if (khi > DX - 1) khi = DX - 1;
        for (int k = klo; k <= khi; k++) band_put(sm, x1 + sgx * k, y1 + sgy * ((k * DY) / DX), y0, ord);
    } else { // y major: pixel k at row y1 + sgy*k
        int klo, khi;
        if (sgy > 0) { klo = y0 - y1; khi = y1b - y1; } else { klo = y1 - y1b; khi = y1 - y0; }
        if (klo < 0) klo = 0;
        if (khi > DY - 1) khi = DY - 1;
        for (int k = klo; k <= khi; k++) band_put(sm, x1 + sgx * ((k * DX) / DY), y1 + sgy * k, y0, ord);
    }
}

// one sub-line of a width-2 outline: clip (pygame clipline) then raster in band
MG_DEV void clip_raster_band(RenderSmem &sm, int x1, int y1, int x2, int y2, uint32_t ord, int y0) {
    if (!clipline(x1, y1, x2, y2)) return;
    raster_line_band(sm, x1, y1, x2, y2, ord, y0);
}

// render polygon point i (local coordinates); the goal rect is make_rect(w, h) of its entity
MG_DEV void rpoly_pt(const MGState &S, const mg_library *L, int e, const mg_rpoly &rp, int ent, int i, double &x, double &y) {
    if (rp.pts_off >= 0) { x = L->rpts[rp.pts_off + i][0]; y = L->rpts[rp.pts_off + i][1]; return; }
    double rad_h = AT(S.eh, ent) / 2, rad_w = AT(S.ew, ent) / 2;
    x = (i == 0 || i == 3) ? -rad_w : rad_w;
    y = (i == 0 || i == 1) ? rad_h : -rad_h;
}

// render.py Transform matrices of one entity (pre_draw: entities.py:478-491, 751-754, 865-868)
MG_DEV void entity_xforms(const MGState &S, int e, int ent, double (*xf)[9]) {
    int kind = AT(S.ekind, ent);
    if (kind == MG_ENT_ROBOT) {
        int b = AT(S.ebody0, ent);
        mg_transform_tr(AT(S.bpx, b), AT(S.bpy, b), AT(S.ba, b), xf[MG_XF_MAIN]);
        for (int k = 0; k < 2; k++) {
            int fb = b + 4 + k;
            mg_transform_tr(AT(S.bpx, fb), AT(S.bpy, fb), AT(S.ba, fb), xf[MG_XF_FINGER_L + k]);
            mg_transform_tr(0.0, 0.0, AT(S.ba, b + 2 + k) - AT(S.ba, b), xf[MG_XF_PUPIL_L + k]);
        }
    } else if (kind == MG_ENT_BLOCK) {
        int b = AT(S.ebody0, ent);
        mg_transform_tr(AT(S.bpx, b), AT(S.bpy, b), AT(S.ba, b), xf[MG_XF_MAIN]);
    } else if (kind == MG_ENT_GOAL) {
        mg_transform_tr(S.gpx[e], S.gpy[e], 0.0, xf[MG_XF_MAIN]);
    }
}

// One (env, view) per workgroup.  mode 0: LoRes outputs; mode 1: full-resolution frames.
__global__ void __launch_bounds__(RG_THREADS) render_kernel(MGState S, const mg_library *__restrict__ L, RenderOut out,
                                                            int mode) {
    __shared__ RenderSmem sm;
    const int e = blockIdx.x, view = blockIdx.y, tid = threadIdx.x;
    if (e >= S.n_envs || (out.mask && !out.mask[e])) return;
    const int nents = S.nents[e];
    // ---- 1. geometry list (entity add order x render polys), colour table, view ----
    int my_r0 = 0, my_nr = 0;
    if (tid < nents) {
        int kind = AT(S.ekind, tid);
        if (kind == MG_ENT_ARENA) { my_r0 = L->arena_rpoly0; my_nr = L->arena_nrpoly; }
        else if (kind == MG_ENT_GOAL) { my_r0 = L->goal_rpoly0; my_nr = L->goal_nrpoly; }
        else if (kind == MG_ENT_ROBOT) { my_r0 = L->robot_rpoly0; my_nr = L->robot_nrpoly; }
        else { int t = AT(S.etype, tid); my_r0 = L->block_rpoly0[t]; my_nr = L->block_nrpoly[t]; }
        sm.e_g0[tid + 1] = (int16_t)my_nr;
    }
    if (tid == 0) {
        sm.err = 0; sm.ndash = 0; sm.nsedge = 0;
        sm.col[0] = pack_rgb(L->background);
        sm.e_g0[0] = 0;
    }
    if (view == 0 && tid == 32) { // Viewer.render: stack.push(self.transform) -> eye(3) @ view
        const double I3[9] = {1, 0, 0, 0, 1, 0, 0, 0, 1};
        mg_mat3_mul(I3, L->allo_view, sm.u.pre.view);
    }
    if (view == 1 && tid == 32) {
        // Viewer.set_cam_follow / ego_cam_matrix: P @ (scale @ (tr1 @ (rot @ tr2)))
        int rb = S.robot_body0[e];
        double rot[9], tr2[9], m1[9], m2[9], m3[9];
        mg_transform_tr(0.0, 0.0, -AT(S.ba, rb), rot);
        mg_transform_tr(-AT(S.bpx, rb), -AT(S.bpy, rb), 0.0, tr2);
        mg_mat3_mul(rot, tr2, m1);
        mg_mat3_mul(L->ego_tr1_m, m1, m2);
        mg_mat3_mul(L->ego_scale_m, m2, m3);
        mg_mat3_mul(L->pygame_m, m3, m1);
        const double I3[9] = {1, 0, 0, 0, 1, 0, 0, 0, 1};
        mg_mat3_mul(I3, m1, sm.u.pre.view);
    }
    if (tid >= 64 && tid - 64 < nents) entity_xforms(S, e, tid - 64, sm.u.pre.e_xf[tid - 64]);
    __syncthreads();
    if (tid == 0) {
        for (int k = 0; k < nents; k++) sm.e_g0[k + 1] += sm.e_g0[k];
        sm.ngeom = sm.e_g0[nents];
        if (sm.ngeom > RG_MAXG) sm.err = 2;
    }
    __syncthreads();
    if (sm.err) { if (tid == 0) S.overflow[e] |= 4 << view; return; }
    const int G = sm.ngeom;
    if (tid < nents) {
        int ecol = AT(S.ecol, tid);
        for (int k = 0, g = sm.e_g0[tid]; k < my_nr; k++, g++) {
            const mg_rpoly &rp = L->rpoly[my_r0 + k];
            sm.g_rpoly[g] = (int16_t)(my_r0 + k);
            sm.g_ent[g] = (int8_t)tid;
            sm.g_nv[g] = (int16_t)rp.npts;
            sm.col[2 * g + 1] = ref_colour(L, rp.col_ref, ecol);
            sm.col[2 * g + 2] = rp.outline ? ref_colour(L, rp.ocol_ref, ecol) : 0u;
        }
    }
    __syncthreads();
    if (tid == 0) {
        int nv = 0;
        for (int g = 0; g < G; g++) { sm.g_voff[g] = (int16_t)nv; nv += sm.g_nv[g]; }
        sm.nvert = nv;
        if (nv > RG_MAXVERT) sm.err = 2;
    }
    // ---- 2. per-geom matrix: view @ T_last @ ... @ T_first (Geom.render stack) ----
    for (int g = tid; g < G; g += RG_THREADS) {
        const mg_rpoly &rp = L->rpoly[sm.g_rpoly[g]];
        int ent = sm.g_ent[g];
        double M[9];
        for (int i = 0; i < 9; i++) M[i] = sm.u.pre.view[i];
        for (int k = rp.nxf - 1; k >= 0; k--) {
            int x = rp.xf[k];
            const double *T = x >= MG_XF_STATIC0 ? L->static_xf[x - MG_XF_STATIC0] : sm.u.pre.e_xf[ent][x];
            mg_mat3_mul(M, T, M);
        }
        for (int i = 0; i < 6; i++) sm.u.pre.g_m[g][i] = M[i];
    }
    __syncthreads();
    if (sm.err) { if (tid == 0) S.overflow[e] |= 4 << view; return; }
    const int NV = sm.nvert;
    for (int g = tid; g < G; g += RG_THREADS)
        for (int i = 0, v0 = sm.g_voff[g]; i < sm.g_nv[g]; i++) sm.v_geom[v0 + i] = (uint8_t)g;
    __syncthreads();
    // ---- 3. vertices -> int pixel coordinates (pygame (int) truncation); outline edges ----
    for (int v = tid; v < NV; v += RG_THREADS) {
        int g = sm.v_geom[v], i = v - sm.g_voff[g];
        const mg_rpoly &rp = L->rpoly[sm.g_rpoly[g]];
        double x, y;
        rpoly_pt(S, L, e, rp, sm.g_ent[g], i, x, y);
        const double *M = sm.u.pre.g_m[g];
        double gx = __fma_rn(M[1], y, M[0] * x) + M[2];
        double gy = __fma_rn(M[4], y, M[3] * x) + M[5];
        sm.vx[v] = (int16_t)(int)gx;
        sm.vy[v] = (int16_t)(int)gy;
        if (rp.outline == MG_OUTLINE_SOLID) {
            // lines(): first point via float (pg FloatFromObj), second via int
            sm.fx[v] = (int16_t)(int)(float)gx;
            sm.fy[v] = (int16_t)(int)(float)gy;
            sm.sedge[atomicAdd(&sm.nsedge, 1)] = (int16_t)v;
        } else if (rp.outline == MG_OUTLINE_DASHED) {
            int j = i + 1 == rp.npts ? 0 : i + 1;
            double xb, yb;
            rpoly_pt(S, L, e, rp, sm.g_ent[g], j, xb, yb);
            double gxb = __fma_rn(M[1], yb, M[0] * xb) + M[2], gyb = __fma_rn(M[4], yb, M[3] * xb) + M[5];
            push_dashes(sm, gx, gy, gxb, gyb, 2 * g + 2);
        }
    }
    __syncthreads();
    // ---- 4. per-geom bounding rows / columns; span table offsets ----
    for (int g = tid; g < G; g += RG_THREADS) {
        int v0 = sm.g_voff[g], n = sm.g_nv[g];
        int ymin = sm.vy[v0], ymax = ymin, xmin = sm.vx[v0], xmax = xmin;
        for (int i = 1; i < n; i++) {
            int y = sm.vy[v0 + i], x = sm.vx[v0 + i];
            ymin = y < ymin ? y : ymin; ymax = y > ymax ? y : ymax;
            xmin = x < xmin ? x : xmin; xmax = x > xmax ? x : xmax;
        }
        sm.g_ymin[g] = (int16_t)ymin; sm.g_ymax[g] = (int16_t)ymax;
        sm.g_xmin[g] = (int16_t)(xmin > 0 ? xmin : 0);
        sm.g_xmax[g] = (int16_t)(xmax < MG_RES - 1 ? xmax : MG_RES - 1);
        int r0 = ymin > 0 ? ymin : 0, r1 = ymax < MG_RES - 1 ? ymax : MG_RES - 1;
        sm.g_soff[g + 1] = r1 >= r0 ? r1 - r0 + 1 : 0;
    }
    __syncthreads();
    if (tid == 0) {
        sm.g_soff[0] = 0;
        for (int g = 0; g < G; g++) sm.g_soff[g + 1] += sm.g_soff[g];
        sm.nspan = sm.g_soff[G];
        if (sm.nspan > RG_MAXSPAN) sm.err = 3;
    }
    __syncthreads();
    if (sm.err) { if (tid == 0) S.overflow[e] |= 4 << view; return; }
    // ---- 5. fill spans: pygame draw_fillpoly intersections per row (2 per row for these convex polys) ----
    for (int s = tid; s < sm.nspan; s += RG_THREADS) {
        int lo_g = 0, hi_g = G - 1; // last g with g_soff[g] <= s
        while (lo_g < hi_g) {
            int mid = (lo_g + hi_g + 1) >> 1;
            if (sm.g_soff[mid] <= s) lo_g = mid; else hi_g = mid - 1;
        }
        const int g = lo_g;
        int ymin = sm.g_ymin[g], ymax = sm.g_ymax[g];
        int y = (ymin > 0 ? ymin : 0) + s - sm.g_soff[g];
        int v0 = sm.g_voff[g], n = sm.g_nv[g];
        int lo = 32767, hi = -32768, cnt = 0;
        for (int i = 0; i < n; i++) {
            int ip = i ? i - 1 : n - 1;
            int ya = sm.vy[v0 + ip], yb = sm.vy[v0 + i], xa, xb;
            if (ya < yb) { xa = sm.vx[v0 + ip]; xb = sm.vx[v0 + i]; }
            else if (ya > yb) { int t = ya; ya = yb; yb = t; xa = sm.vx[v0 + i]; xb = sm.vx[v0 + ip]; }
            else continue;
            if ((y >= ya && y < yb) || (y == ymax && y > ya && y <= yb)) {
                int x = (y - ya) * (xb - xa) / (yb - ya) + xa;
                lo = x < lo ? x : lo; hi = x > hi ? x : hi;
                cnt++;
            }
        }
        if (cnt != 0 && cnt != 2) sm.err = 4;
        if (cnt == 0) { lo = 32767; hi = -32768; }
        sm.span_l[s] = (int16_t)lo;
        sm.span_r[s] = (int16_t)hi;
    }
    __syncthreads();
    if (sm.err) { if (tid == 0) S.overflow[e] |= 4 << view; return; }
    const int ndash = sm.ndash, nsedge = sm.nsedge;
    // ---- 6. bands ----
    uint8_t *ring = view == 0 ? S.hist_allo : S.hist_ego;
    const size_t FR = (size_t)MG_LORES * MG_LORES * 3;
    const bool fresh = S.episode_steps[e] == 0;
    const int head = S.hist_head[view * S.N + e];
    const int nh = fresh ? 0 : ((head + 1) & 3);
    const int pp = out.preproc;
    const bool stacked = pp == MG_PREPROC_LORESSTACK || (pp == MG_PREPROC_LORES4E && view == 1) ||
                         (pp == MG_PREPROC_LORES4A && view == 0);
    const bool plain = pp != MG_PREPROC_LORESSTACK;   // the view's own current-frame output
    uint8_t *o_plain = view == 0 ? out.obs_allo : out.obs_ego;
    uint8_t *o_stack = pp == MG_PREPROC_LORESSTACK ? o_plain : out.obs_past;
    for (int y0 = 0; y0 < MG_RES; y0 += RG_BAND) {
        const size_t lrow = (size_t)(y0 / 4) * RG_LOROW;  // byte offset of this band's LoRes rows
        // prefetch frames t-3..t-1 of these rows (ring slots nh+1..nh+3, never written this step)
        uint4 pf = make_uint4(0, 0, 0, 0);
        const bool do_pf = mode == 0 && stacked && !fresh && tid < 3 * RG_BANDLO16;
        if (do_pf) {
            int k = tid / RG_BANDLO16, c = tid % RG_BANDLO16, sl = (nh + 1 + k) & 3;
            pf = *(const uint4 *)(ring + ((size_t)sl * S.N + e) * FR + lrow + 16 * c);
        }
        for (int i = tid; i < RG_BAND * MG_RES; i += RG_THREADS) (&sm.u.post.band[0][0])[i] = 0u;
        __syncthreads();
        for (int g = 0; g < G; g++) {
            int ymin = sm.g_ymin[g], ymax = sm.g_ymax[g];
            int ra = ymin > y0 ? ymin : y0, rb = ymax < y0 + RG_BAND - 1 ? ymax : y0 + RG_BAND - 1;
            if (ra > rb) continue;
            int xmin = sm.g_xmin[g], xmax = sm.g_xmax[g];
            if (xmin > xmax) continue;
            int w = xmax - xmin + 1, total = (rb - ra + 1) * w;
            int r0 = ymin > 0 ? ymin : 0;
            uint32_t ord = 2 * g + 1;
            for (int i = tid; i < total; i += RG_THREADS) {
                int y = ra + i / w, x = xmin + i % w;
                int s = sm.g_soff[g] + y - r0;
                if (x >= sm.span_l[s] && x <= sm.span_r[s]) atomicMax(&sm.u.post.band[y - y0][x], ord);
            }
        }
        // solid width-2 outlines (clip_and_draw_line_width: base line + one offset copy)
        for (int k = tid; k < nsedge; k += RG_THREADS) {
            int v = sm.sedge[k], g = sm.v_geom[v];
            int nx = v + 1 == sm.g_voff[g] + sm.g_nv[g] ? sm.g_voff[g] : v + 1;
            int x1 = sm.fx[v], y1 = sm.fy[v], x2 = sm.vx[nx], y2 = sm.vy[nx];
            int ylo = (y1 < y2 ? y1 : y2) - 1, yhi = (y1 > y2 ? y1 : y2) + 1;
            if (yhi < y0 || ylo >= y0 + RG_BAND) continue;
            uint32_t ord = 2 * g + 2;
            clip_raster_band(sm, x1, y1, x2, y2, ord, y0);
            if (abs(x1 - x2) > abs(y1 - y2)) clip_raster_band(sm, x1, y1 + 1, x2, y2 + 1, ord, y0);
            else clip_raster_band(sm, x1 + 1, y1, x2 + 1, y2, ord, y0);
        }
        for (int i = tid; i < ndash; i += RG_THREADS)
            raster_line_band(sm, sm.dash[i][0], sm.dash[i][1], sm.dash[i][2], sm.dash[i][3], (uint32_t)sm.dash_o[i], y0);
        __syncthreads();
        if (mode == 1) {
            uint8_t *dst = out.full + (((size_t)e * 2 + view) * MG_RES + y0) * MG_RES * 3;
            for (int i = tid; i < RG_BAND * MG_RES; i += RG_THREADS) {
                uint32_t c = sm.col[(&sm.u.post.band[0][0])[i]];
                dst[3 * i] = (uint8_t)(c & 255); dst[3 * i + 1] = (uint8_t)((c >> 8) & 255); dst[3 * i + 2] = (uint8_t)(c >> 16);
            }
            __syncthreads();
            continue;
        }
        // 4x4 area downsample (round half to even of sum/16) into LDS staging
        uint8_t *lo8 = (uint8_t *)sm.u.post.lo;
        for (int t = tid; t < (RG_BAND / 4) * MG_LORES; t += RG_THREADS) {
            int oyl = t / MG_LORES, ox = t % MG_LORES;
            int sr = 0, sg = 0, sb = 0;
            for (int dy = 0; dy < 4; dy++)
                for (int dx = 0; dx < 4; dx++) {
                    uint32_t c = sm.col[sm.u.post.band[oyl * 4 + dy][ox * 4 + dx]];
                    sr += c & 255; sg += (c >> 8) & 255; sb += c >> 16;
                }
            int ss[3] = {sr, sg, sb};
            for (int ch = 0; ch < 3; ch++) {
                int q = ss[ch] >> 4, r = ss[ch] & 15;
                lo8[t * 3 + ch] = (uint8_t)(q + (r > 8 || (r == 8 && (q & 1))));
            }
        }
        if (do_pf) sm.u.post.past[tid / RG_BANDLO16][tid % RG_BANDLO16] = pf;
        __syncthreads();
        // ring of the last 4 LoRes frames: slot nh (all 4 slots at episode start)
        for (int t = tid; t < (fresh ? 4 : 1) * RG_BANDLO16; t += RG_THREADS) {
            int sl = fresh ? t / RG_BANDLO16 : nh, c = t % RG_BANDLO16;
            *(uint4 *)(ring + ((size_t)sl * S.N + e) * FR + lrow + 16 * c) = sm.u.post.lo[c];
        }
        if (plain)
            for (int c = tid; c < RG_BANDLO16; c += RG_THREADS)
                *(uint4 *)(o_plain + (size_t)e * FR + lrow + 16 * c) = sm.u.post.lo[c];
        if (stacked) {
            // FlattenFrameStack: [96][96][12] = frames oldest..newest concatenated per pixel
            const uint8_t *p8 = (const uint8_t *)sm.u.post.past;
            for (int c = tid; c < 4 * RG_BANDLO16; c += RG_THREADS) {
                uint8_t b[16];
                for (int j = 0; j < 16; j++) {
                    int byte = 16 * c + j, px = byte / 12, k = (byte % 12) / 3, ch = byte % 3;
                    int src = px * 3 + ch;
                    b[j] = (k == 3 || fresh) ? lo8[src] : p8[k * RG_BANDLO + src];
                }
                uint4 w;
                w.x = b[0] | (b[1] << 8) | (b[2] << 16) | ((uint32_t)b[3] << 24);
                w.y = b[4] | (b[5] << 8) | (b[6] << 16) | ((uint32_t)b[7] << 24);
                w.z = b[8] | (b[9] << 8) | (b[10] << 16) | ((uint32_t)b[11] << 24);
                w.w = b[12] | (b[13] << 8) | (b[14] << 16) | ((uint32_t)b[15] << 24);
                *(uint4 *)(o_stack + (size_t)e * FR * 4 + lrow * 4 + 16 * c) = w;
            }
        }
        __syncthreads();
    }
    if (mode == 0 && tid == 0) S.hist_head[view * S.N + e] = nh;
}
