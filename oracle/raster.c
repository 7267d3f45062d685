/*
 * raster.c -- headless Viewer rendering + cv2 INTER_AREA 4x downsample, restated.
 * TEST INFRASTRUCTURE ONLY (see oracle.h).
 *
 * Follows render.py:151-287 (Geom.render, Poly._render, draw_outline incl. the
 * dashed branch), render.py:385-395 (Viewer.render), base_env.py:309-343
 * (views).  Upstream semantics: pygame 1.9.6 draw.c
 * draw_fillpoly / drawhorzlineclip / lines / line / clip_and_draw_line_width /
 * clipline / drawline, and OpenCV resizeAreaFast (round-half-even of sum/16).
 */
#include <math.h>
#include <stdlib.h>
#include <string.h>
#include "oscene.h"

#define W O_RES
#define H O_RES
static const uint8_t BG[3] = {231, 231, 234}; /* lighten_rgb(grey, 4), base_env.py:199 */

static inline void put(uint8_t *fr, int x, int y, const uint8_t *c) {
    uint8_t *p = fr + ((size_t)y * W + x) * 3;
    p[0] = c[0]; p[1] = c[1]; p[2] = c[2];
}

/* drawhorzlineclip */
static void hline_clip(uint8_t *fr, int x1, int y, int x2, const uint8_t *c) {
    if (y < 0 || y >= H) return;
    if (x2 < x1) { int t = x1; x1 = x2; x2 = t; }
    x1 = x1 > 0 ? x1 : 0;
    x2 = x2 < W - 1 ? x2 : W - 1;
    if (x2 < 0 || x1 >= W) return;
    for (int x = x1; x <= x2; x++) put(fr, x, y, c);
}

static int cmp_int(const void *a, const void *b) {
    int x = *(const int *)a, y = *(const int *)b;
    return (x > y) - (x < y);
}

/* draw_fillpoly (pygame 1.9.6) */
static void fill_poly(uint8_t *fr, const int *vx, const int *vy, int n, const uint8_t *c) {
    int miny = vy[0], maxy = vy[0];
    for (int i = 1; i < n; i++) {
        if (vy[i] < miny) miny = vy[i];
        if (vy[i] > maxy) maxy = vy[i];
    }
    int ints[256];
    for (int y = miny; y <= maxy; y++) {
        int nints = 0;
        for (int i = 0; i < n; i++) {
            int ip = i ? i - 1 : n - 1;
            int y1 = vy[ip], y2 = vy[i], x1, x2;
            if (y1 < y2) { x1 = vx[ip]; x2 = vx[i]; }
            else if (y1 > y2) { y2 = vy[ip]; y1 = vy[i]; x2 = vx[ip]; x1 = vx[i]; }
            else continue;
            if ((y >= y1 && y < y2) || (y == maxy && y > y1 && y <= y2))
                ints[nints++] = (y - y1) * (x2 - x1) / (y2 - y1) + x1;
        }
        qsort(ints, (size_t)nints, sizeof(int), cmp_int);
        for (int i = 0; i + 1 < nints; i += 2) hline_clip(fr, ints[i], y, ints[i + 1], c);
    }
}

/* Cohen-Sutherland clipline (float32 slope) */
enum { LEFT_EDGE = 1, RIGHT_EDGE = 2, BOTTOM_EDGE = 4, TOP_EDGE = 8 };
static int encode(int x, int y, int left, int top, int right, int bottom) {
    int code = 0;
    if (x < left) code |= LEFT_EDGE;
    if (x > right) code |= RIGHT_EDGE;
    if (y < top) code |= TOP_EDGE;
    if (y > bottom) code |= BOTTOM_EDGE;
    return code;
}
static int clipline(int *pts, int left, int top, int right, int bottom) {
    int x1 = pts[0], y1 = pts[1], x2 = pts[2], y2 = pts[3];
    int code1, code2, draw = 0, t;
    float m;
    for (;;) {
        code1 = encode(x1, y1, left, top, right, bottom);
        code2 = encode(x2, y2, left, top, right, bottom);
        if (!(code1 | code2)) { draw = 1; break; }
        else if (code1 & code2) break;
        else {
            if (!code1) {
                t = x2; x2 = x1; x1 = t;
                t = y2; y2 = y1; y1 = t;
                t = code2; code2 = code1; code1 = t;
            }
            if (x2 != x1) m = (float)(y2 - y1) / (float)(x2 - x1);
            else m = 1.0f;
            if (code1 & LEFT_EDGE) { y1 += (int)((float)(left - x1) * m); x1 = left; }
            else if (code1 & RIGHT_EDGE) { y1 += (int)((float)(right - x1) * m); x1 = right; }
            else if (code1 & BOTTOM_EDGE) {
                if (x2 != x1) x1 += (int)((float)(bottom - y1) / m);
                y1 = bottom;
            } else if (code1 & TOP_EDGE) {
                if (x2 != x1) x1 += (int)((float)(top - y1) / m);
                y1 = top;
            }
        }
    }
    if (draw) { pts[0] = x1; pts[1] = y1; pts[2] = x2; pts[3] = y2; }
    return draw;
}

/* drawline: Bresenham with deltax = |dx|+1 major steps */
static void drawline(uint8_t *fr, const uint8_t *c, int x1, int y1, int x2, int y2) {
    int deltax = x2 - x1, deltay = y2 - y1;
    int signx = deltax < 0 ? -1 : 1, signy = deltay < 0 ? -1 : 1;
    deltax = signx * deltax + 1;
    deltay = signy * deltay + 1;
    int px = x1, py = y1;
    int majx = signx, majy = 0, minx = 0, miny = signy;
    if (deltax < deltay) {
        int t = deltax; deltax = deltay; deltay = t;
        majx = 0; majy = signy; minx = signx; miny = 0;
    }
    int y = 0;
    for (int x = 0; x < deltax; x++) {
        put(fr, px, py, c);
        px += majx; py += majy;
        y += deltay;
        if (y >= deltax) { y -= deltax; px += minx; py += miny; }
    }
}

static int clip_and_draw_line(uint8_t *fr, const uint8_t *c, int *pts) {
    if (!clipline(pts, 0, 0, W - 1, H - 1)) return 0;
    if (pts[1] == pts[3]) hline_clip(fr, pts[0], pts[1], pts[2], c);
    else if (pts[0] == pts[2]) {
        int ya = pts[1] < pts[3] ? pts[1] : pts[3], yb = pts[1] < pts[3] ? pts[3] : pts[1];
        for (int y = ya; y <= yb; y++) put(fr, pts[0], y, c);
    } else drawline(fr, c, pts[0], pts[1], pts[2], pts[3]);
    return 1;
}

static void clip_and_draw_line_width(uint8_t *fr, const uint8_t *c, int width, const int *pts) {
    int xinc = 0, yinc = 0, np[4];
    if (abs(pts[0] - pts[2]) > abs(pts[1] - pts[3])) yinc = 1;
    else xinc = 1;
    memcpy(np, pts, sizeof(np));
    clip_and_draw_line(fr, c, np);
    for (int loop = 1; loop < width; loop += 2) {
        int k = loop / 2 + 1;
        np[0] = pts[0] + xinc * k; np[1] = pts[1] + yinc * k;
        np[2] = pts[2] + xinc * k; np[3] = pts[3] + yinc * k;
        clip_and_draw_line(fr, c, np);
        if (loop + 1 < width) {
            np[0] = pts[0] - xinc * k; np[1] = pts[1] - yinc * k;
            np[2] = pts[2] - xinc * k; np[3] = pts[3] - yinc * k;
            clip_and_draw_line(fr, c, np);
        }
    }
}

/* numpy arange(start, stop, step) for float64 (PyArray_ArangeObj + DOUBLE_fill) */
static int np_arange(double start, double stop, double step, double *out, int maxn) {
    double len_f = ceil((stop - start) / step);
    if (!(len_f > 0)) return 0;
    int len = (int)len_f;
    if (len > maxn) len = maxn;
    out[0] = start;
    if (len == 1) return 1;
    double next = start + step;
    out[1] = next;
    double delta = next - start;
    for (int i = 2; i < len; i++) out[i] = start + i * delta;
    return len;
}

/* render.py:230-255 dashed branch: the (start, end) integer endpoints of each
 * pygame.draw.line(..., 4) call, in call order; returns the number of dashes */
static int dash_segments(double x1, double y1, double x2, double y2, int *seg, int maxseg) {
    double xs[512], ys[512];
    int nx, ny;
    const double dl = 10;
    if (x1 == x2) {
        ny = np_arange(y1, y2, y1 < y2 ? dl : -dl, ys, 512);
        for (int i = 0; i < ny; i++) xs[i] = x1;
        nx = ny;
    } else if (y1 == y2) {
        nx = np_arange(x1, x2, x1 < x2 ? dl : -dl, xs, 512);
        for (int i = 0; i < nx; i++) ys[i] = y1;
        ny = nx;
    } else {
        double a = fabs(x2 - x1), b = fabs(y2 - y1);
        double c_ = nearbyint(sqrt(a * a + b * b)); /* Python round(): half-even */
        double dx = dl * a / c_, dy = dl * b / c_;
        nx = np_arange(x1, x2, x1 < x2 ? dx : -dx, xs, 512);
        ny = np_arange(y1, y2, y1 < y2 ? dy : -dy, ys, 512);
    }
    int n = nx < ny ? nx : ny, k;
    /* next = odd indices, last = even indices; zip truncates */
    for (k = 0; 2 * k + 1 < n && k < maxseg; k++) {
        seg[4 * k + 0] = (int)nearbyint(xs[2 * k + 1]);
        seg[4 * k + 1] = (int)nearbyint(ys[2 * k + 1]);
        seg[4 * k + 2] = (int)nearbyint(xs[2 * k]);
        seg[4 * k + 3] = (int)nearbyint(ys[2 * k]);
    }
    return k;
}

static void draw_dashed(uint8_t *fr, double x1, double y1, double x2, double y2, const uint8_t *c) {
    int seg[4 * 256];
    int n = dash_segments(x1, y1, x2, y2, seg, 256);
    for (int k = 0; k < n; k++) clip_and_draw_line_width(fr, c, 4, seg + 4 * k);
}

static void render_geom(const OEnv *e, const OGeom *g, const double *view, uint8_t *fr) {
    double M[9];
    memcpy(M, view, sizeof(M));
    for (int k = g->nxf - 1; k >= 0; k--) o_mat3_mul(M, e->xf[g->xf[k]].m, M);
    double gx[O_MAX_PTS], gy[O_MAX_PTS];
    int n = g->npts;
    for (int i = 0; i < n; i++) {
        double x = g->pts[i].x, y = g->pts[i].y;
        gx[i] = fma(M[2], 1.0, fma(M[1], y, M[0] * x));
        gy[i] = fma(M[5], 1.0, fma(M[4], y, M[3] * x));
    }
    /* pygame.draw.polygon(surface, color, ps + [ps[0]]): float -> int truncation */
    int vx[O_MAX_PTS + 1], vy[O_MAX_PTS + 1];
    for (int i = 0; i < n; i++) { vx[i] = (int)gx[i]; vy[i] = (int)gy[i]; }
    vx[n] = vx[0]; vy[n] = vy[0];
    fill_poly(fr, vx, vy, n + 1, g->col);
    if (g->outline == OUTLINE_SOLID) {
        for (int i = 0; i < n; i++) {
            int j = (i + 1) % n;
            /* pygame 1.9.6 lines(): first point via float, later points via int */
            int pts[4] = {(int)(float)gx[i], (int)(float)gy[i], (int)gx[j], (int)gy[j]};
            clip_and_draw_line_width(fr, g->ocol, 2, pts);
        }
    } else if (g->outline == OUTLINE_DASHED) {
        for (int i = 0; i < n; i++) {
            int j = (i + 1) % n;
            draw_dashed(fr, gx[i], gy[i], gx[j], gy[j], g->ocol);
        }
    }
}

void oraster_render(const OEnv *e, int ego, uint8_t *fr) {
    double view[9], eye[9] = {1, 0, 0, 0, 1, 0, 0, 0, 1}, top[9];
    if (ego) {
        const OBody *b = &e->space.bodies[e->ents[e->robot].body0];
        o_ego_view(b->p.x, b->p.y, b->a, view);
    } else {
        o_allo_view(view);
    }
    o_mat3_mul(eye, view, top); /* Stack.push(self.transform) */
    for (int i = 0; i < W * H; i++) memcpy(fr + 3 * i, BG, 3);
    for (int g = 0; g < e->ngeoms; g++) render_geom(e, &e->geoms[g], top, fr);
}

/* cv2.resize(..., (96, 96), INTER_AREA): resizeAreaFast, saturate_cast(sum * 1/16) */
void oraster_downsample(const uint8_t *in, uint8_t *out) {
    for (int oy = 0; oy < O_LORES; oy++)
        for (int ox = 0; ox < O_LORES; ox++)
            for (int ch = 0; ch < 3; ch++) {
                int s = 0;
                for (int dy = 0; dy < 4; dy++)
                    for (int dx = 0; dx < 4; dx++) s += in[((size_t)(oy * 4 + dy) * W + ox * 4 + dx) * 3 + ch];
                int q = s >> 4, r = s & 15;
                out[((size_t)oy * O_LORES + ox) * 3 + ch] = (uint8_t)(q + (r > 8 || (r == 8 && (q & 1))));
            }
}

/* ---- pieces exported for the raster known-answer tests (tests/test_oracle_known_answers.py) ---- */
void o_fill_poly(uint8_t *fr, const int *vx, const int *vy, int n, const uint8_t *c) { fill_poly(fr, vx, vy, n, c); }
int o_clipline(int *pts) { return clipline(pts, 0, 0, W - 1, H - 1); }
void o_line_width(uint8_t *fr, const uint8_t *c, int width, const int *pts) { clip_and_draw_line_width(fr, c, width, pts); }
int o_dash_segments(double x1, double y1, double x2, double y2, int *seg, int maxseg) {
    return dash_segments(x1, y1, x2, y2, seg, maxseg);
}
