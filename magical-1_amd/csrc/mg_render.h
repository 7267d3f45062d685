// mg_render.h -- headless Viewer raster + LoRes downsample, one workgroup per (env, view).
//
// Replaces render.py:151-287 / 385-395 (Geom.render, Poly._render ->
// pygame.draw.polygon + width-2 lines + dashed width-4 goal outlines,
// surfarray) and benchmarks/__init__.py:150-190 (cv2.resize INTER_AREA 4x).
//
// The 384x384 frame never leaves the CU.  Setup (per workgroup) turns the
// scene into integer vertices (pygame truncation), the two y-monotone vertex
// chains of every convex polygon, and per-band lists of outline items.  The
// frame is then produced in 8-row bands: fill spans of the band's rows are found
// by binary search on the chains (pygame draw_fillpoly's intersection rule),
// outline pixels go to an LDS layer by atomicMax(draw ordinal) -- the painter's
// rule "last primitive drawn wins" is "largest ordinal wins" -- and one thread
// per 4x4 block resolves fills (geoms in draw order), takes the max with the
// outline layer, looks up colours and sums the block (cv2 INTER_AREA 4x:
// round-half-even of sum/16).  Each band yields RG_BAND / 4 LoRes rows written to HBM
// with 16-byte stores, together with the frame-stack ring.
#pragma once
#include "mg_launch.h"
#include "mg_step.h"
#include "mg_prof.h"
#include <type_traits>

// capacity classes (template parameters of the LDS layout): geoms, vertices, dash lines, bin entries
// (outline items + fill edges, binned per band), solid outline edges, entities, outline-mask type (one bit
// per entity), rows per band (default 8), outline-mask bits per pixel (default: the type's).  The large class
// fits every task; the small one fits robot + arena + goal or one block (MoveToRegion / MoveToCorner: at most
// 26 geoms (star block), 636 vertices (circle block), 204 solid outline edges, 3 entities) in 16-row bands with
// a 4-bit outline mask: 17.4 KB, 9 workgroups/CU (round 6: the 8-row class took 16.2 KB at 9 per CU; 16-row bands
// halve the bands' barriers, band lists and per-band edge / segment set-up, render 0.628 -> 0.553 ms per 2048-env
// chunk, MoveToRegion 3.16 -> 3.37 M env-steps/s, profiles/r06_b16).  Medium-0 / medium-1 stay at 8 rows: at 16 (6 / 5
// per CU) they measured 15% / 6% slower (ClusterColour / MatchRegions), their launches being throughput-bound.  The
// medium-2 launch renders only the pairs the earlier classes hand over (MatchRegions-TestAll: ~8%) and is bound by
// its slowest workgroups, so the shorter 16-row workgroups pay there: MatchRegions 1.449 -> 1.462 M (profiles/r06_m2b16).
#define RG_LARGE 160, 1600, 256, 3072, 1600, MG_MAX_ENTS, uint32_t
#ifndef RG_MEDIUM0
#define RG_MEDIUM0 44, 784, 128, 1280, 512, MG_MAX_ENTS, uint16_t   // 20.3 KB: 8 workgroups/CU
#endif
#ifndef RG_MEDIUM1
#define RG_MEDIUM1 48, 896, 160, 1536, 512, MG_MAX_ENTS, uint16_t
#endif
#ifndef RG_MEDIUM2
#define RG_MEDIUM2 96, 1280, 160, 2560, 768, MG_MAX_ENTS, uint16_t, 16   // 16-row bands: see below
#endif
#ifndef RG_SMALL
#define RG_SMALL 28, 640, 160, 1536, 208, 4, uint8_t, 16, 4
#endif
#define RG_MAXLONG 16
#define RG_MAXDE 16                     // dashed edges whose dashes are split over the workgroup
#define RG_THREADS 192                  // = one thread per 4x4 block of a band's first 2 block rows (2 x 96)
#ifndef RG_SHORT
#define RG_SHORT 12                     // segments with <= RG_SHORT * RG_SEGLANES pixels in a band: drawn by
#endif
#ifndef RG_SEGLANES
#define RG_SEGLANES 4                   // their own group of RG_SEGLANES lanes
#endif
#ifndef RG_SPANW
#define RG_SPANW 1                      // band spans converted once per slot row to (l, width) before the resolve
#endif
#ifndef RG_OFS
#define RG_OFS 1                        // resolve ordinals carried as byte offsets into the colour table (x8)
#endif
#ifndef RG_XF_LATE
#define RG_XF_LATE 1                    // entity transforms / view matrix overlap the geometry table (one barrier fewer)
#endif
#ifndef RG_DASH_SPLIT
#define RG_DASH_SPLIT 1                 // dashes of dashed edges split over the workgroup (0: per edge thread)
#endif
#ifndef RG_SCACHE
#define RG_SCACHE 1                     // allocentric static layer (S.scache): see render_kernel, section 5
#endif
#define RG_DMARGIN 4                    // px a geom's pixels can reach beyond its vertex bounds (outline width
                                        // offsets, float/int end points)
#define RG_EMPTY 32767
#define RG_OSH (RG_OFS ? 3 : 0)         // resolve/outline-layer ordinal values are ordinal << RG_OSH
#define RG_LOROW (MG_LORES * 3)         // bytes of one 96-px RGB row

// q = n / d and r = n % d for 0 <= n < 2^31, 1 <= d: a float reciprocal estimate (relative error below
// 2^-22, so q is off by at most one for n < 2^22) corrected by one step; larger n take the integer divide
MG_DEV int udivmod(int n, int d, int &r) {
    int q;
    if (n >= (1 << 22)) q = n / d;
    else q = (int)((float)n * __builtin_amdgcn_rcpf((float)d));
    r = n - q * d;
    if (r < 0) { q--; r += d; }
    else if (r >= d) { q++; r -= d; }
    return q;
}

// A pygame drawline pixel run in k-form: the major axis has n = max(|dx|,|dy|) + 1
// pixels and the minor offset of pixel k is m = floor(k * dminor / dmajor) with
// DX = |dx| + 1, DY = |dy| + 1 (horizontal and vertical lines are the cases
// DY = 1 / DX = 1).  x-major (DX >= DY): pixel (x1 + sgx*k, y1 + sgy*m);
// y-major: (x1 + sgx*m, y1 + sgy*k).
struct LineK { int x1, y1, sgx, sgy, DX, DY, xmaj; };

// LDS: the setup matrices / scratch and the band buffers are never live at the same time, so they
// share storage.  Small class: 9 workgroups per CU (17.4 KB); large class: 3.
//
// Outline layer, MT = u32: the largest outline ordinal drawn at each pixel (atomicMax).  MT = u8: every
// entity draws at most one outlined polygon (the library builder checks it), and entities are drawn in
// add order, so "largest outline ordinal at a pixel" is "highest entity bit set at the pixel": the
// layer holds one bit per entity (atomicOr on words of 4 pixels; 8 pixels of 4 bits for the small class's
// <= 4 entities) and oord[] maps the entity back to its outline's ordinal -- a quarter (an eighth) of the LDS.
template <int MAXG_, int MAXVERT_, int MAXDASH_, int MAXBIN_, int MAXSEDGE_, int MAXE_, typename MT_, int BAND_ = 8,
          int MBITS_ = 8 * (int)sizeof(MT_)>
struct RenderSmem {
    static constexpr int RG_MAXG = MAXG_, RG_MAXVERT = MAXVERT_, RG_MAXDASH = MAXDASH_, RG_MAXBIN = MAXBIN_,
                         RG_MAXSEDGE = MAXSEDGE_, RG_MAXE = MAXE_;
    static constexpr int MBITS = MBITS_, MPW = 32 / MBITS_;   // bits / pixels per word of the outline layer
    static_assert(BAND_ == 8 || BAND_ == 16, "bands of 8 or 16 rows");
    static_assert(MAXVERT_ <= 0x2000, "solid-edge entries hold the vertex in 13 bits");
    static constexpr int BAND = BAND_, NBANDS = MG_RES / BAND_, BROWS = BAND_ / 4;   // rows, bands, LoRes rows per band
    static constexpr int BANDLO16 = BROWS * RG_LOROW / 16;   // 16-byte chunks of a band's LoRes rows (36 / 72)
    static constexpr uint32_t MMASK = (1u << MBITS) - 1u;
    static constexpr bool ORDMAX = MBITS == 32;                                      // layer of ordinals
    static_assert(ORDMAX || (MAXE_ <= MBITS && MAXE_ <= MG_MAX_ENTS), "one outline-mask bit per entity");
    union alignas(16) {
        struct {
            double g_m[RG_MAXG][6];
            double e_xf[RG_MAXE + 4][9];   // main transform per entity, then the robot's 4 others (xf_slot)
            double view[9];
            // setup scratch (dead before the bands)
            int32_t gbb[RG_MAXG][4];                 // per-geom ymin, ymax, xmin, xmax while built (atomics)
            int32_t gchg[RG_MAXG];                   // direction changes of the y sequence around each polygon
            int32_t bin_cnt[NBANDS], ebin_cnt[NBANDS];
            int16_t g_rpoly[RG_MAXG];
            int16_t e_g0[RG_MAXE + 1];
            int16_t e_r0[RG_MAXE];                   // first render poly of each entity
            int32_t ocnt[RG_MAXE];                   // outlined polygons per entity (must be <= 1)
            double dedge[RG_MAXDE][4];               // dashed outline edges (pixel-space end points) ...
            int32_t dedge_o[RG_MAXDE];               // ... and their outline-layer value
            int32_t ndedge;
            int32_t nconv;                           // line-list slots taken by pre-clipped solid edges
        } pre;
        struct {
            uint32_t band[BAND][MG_RES / MPW]; // outline layer of the current band (entity bits per pixel)
            uint4 lo[BANDLO16];          // current frame, the band's LoRes rows
            union {
                struct {
                    int32_t lk[RG_MAXLONG][7];      // long segments of this band (LineK)
                    int32_t lkr[RG_MAXLONG][3];     // klo, khi, ordinal
                };
                uint4 los[BANDLO16];     // the band's static-layer rows (episode's first allo frame; written
                                            // after the long segments are drawn, read in the band's tail)
            };
        } post;
    } u;
    uint2 ginfo[RG_MAXG];                     // (ymin | ymax << 16, xmin | xmax << 16), int16 halves
    uint32_t bspan[RG_MAXG][BAND];         // spans of the band's rows, per band-list slot: l | r << 16
    uint64_t col[2 * RG_MAXG + 2];            // R | G << 16 | B << 32 per ordinal
    int16_t g_voff[RG_MAXG + 1], g_nv[RG_MAXG];
    int16_t vx[RG_MAXVERT], vy[RG_MAXVERT];   // int pixel vertices (pygame (int) truncation)
    uint8_t fdelta[RG_MAXVERT];               // float->int minus double->int of x (bits 0-1) / y (2-3), +1
    uint8_t v_geom[RG_MAXVERT];
    uint16_t sedge[RG_MAXSEDGE];              // solid outline edges: start vertex | lines << 13 | last << 14 | inside << 15
    int16_t blist[RG_MAXG];                   // geoms overlapping the current band, in draw order
    uint32_t bxr[RG_MAXG];                    // x range of each band-list slot's geom (ginfo.y)
    int16_t dash[RG_MAXDASH][4];              // clipped dashed-outline lines
    uint16_t dash_o[RG_MAXDASH];              // outline-layer value of each dash line
    int8_t g_ent[RG_MAXG];
    uint16_t oord1[17];                       // [k + 1]: ordinal of entity k's outlined polygon (0: none)
    int16_t bin_off[NBANDS + 1];           // per-band outline item lists (in bin[])
    int16_t ebin_off[NBANDS + 1];          // per-band fill edge lists (in bin[], after the outline items)
    uint16_t bin[RG_MAXBIN];                  // outline item index, or fill edge: vertex | closing << 14 | last-row << 15
    int16_t gslot[RG_MAXG];                   // band-list slot of each geom overlapping the current band
    int32_t ngeom, nsedge, ndash, nlong, nblist, err;
    uint32_t smask;                           // entities without a body (arena, goals): the static layer
    uint32_t dmask[2][3];                     // LoRes columns of a band that a body's geometry can reach (by band parity)
    int32_t brng[2];                          // bands [brng[0], brng[1]) the band loop runs over
#ifdef MG_PROFILE
    unsigned int pw[4];
#endif
};

// Workgroup barrier ordering LDS only (s_waitcnt lgkmcnt(0); s_barrier): unlike
// __syncthreads it does not wait for outstanding global loads/stores, so the
// frame-stack prefetch and the output stores stay in flight across bands.  No
// thread of a workgroup reads global memory another thread of it wrote.
#define RG_SYNC() asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory")

// exclusive prefix sum over in[0, n) (n <= 256) into out[0, n]; out[n] = total.
// Called by the 64 lanes of wave 0; in and out may alias.
template <typename TI, typename TO>
MG_DEV void wave_exclusive_scan(const TI *in, TO *out, int n, int lane) {
    int v[4], s = 0;
    for (int k = 0; k < 4; k++) { int i = 4 * lane + k; v[k] = i < n ? (int)in[i] : 0; s += v[k]; }
    int incl = s;
    for (int off = 1; off < 64; off <<= 1) {
        int t = __shfl_up(incl, off, 64);
        if (lane >= off) incl += t;
    }
    int ex = incl - s;
    for (int k = 0; k < 4; k++) { int i = 4 * lane + k; if (i < n) out[i] = (TO)ex; ex += v[k]; }
    if (lane == 63) out[n] = (TO)incl;
}

MG_DEV uint64_t pack_rgb(const uint8_t *c) { return (uint64_t)c[0] | ((uint64_t)c[1] << 16) | ((uint64_t)c[2] << 32); }

MG_DEV uint64_t ref_colour(const mg_library *L, int ref, int ecol) {
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
#pragma unroll 1
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

template <class SM>
MG_DEV void push_line(SM &sm, int x1, int y1, int x2, int y2, int ord) {
    if (!clipline(x1, y1, x2, y2)) return;
    int i = atomicAdd(&sm.ndash, 1);
    if (i >= SM::RG_MAXDASH) { sm.err = 1; return; }
    sm.dash[i][0] = (int16_t)x1; sm.dash[i][1] = (int16_t)y1; sm.dash[i][2] = (int16_t)x2; sm.dash[i][3] = (int16_t)y2;
    sm.dash_o[i] = (uint16_t)ord;
}

// clip_and_draw_line_width (pygame 1.9.6): base line + offsets 1, -1, 2, ...
template <class SM>
MG_DEV void push_wide_line(SM &sm, int x1, int y1, int x2, int y2, int width, int ord) {
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

// render.py:232-255 dashed goal outline of one polygon edge: the two np.arange point sequences
struct DashSeq { double sx, stx, sy, sty; int n; bool constx, consty; };
MG_DEV DashSeq dash_seq(double x1, double y1, double x2, double y2) {
    const double dl = 10;
    DashSeq d;
    int nx, ny;
    d.constx = false; d.consty = false;
    if (x1 == x2) {
        d.sy = y1; d.sty = y1 < y2 ? dl : -dl; ny = np_arange_len(y1, y2, d.sty); nx = ny; d.constx = true;
        d.sx = x1; d.stx = 0;
    } else if (y1 == y2) {
        d.sx = x1; d.stx = x1 < x2 ? dl : -dl; nx = np_arange_len(x1, x2, d.stx); ny = nx; d.consty = true;
        d.sy = y1; d.sty = 0;
    } else {
        double a = fabs(x2 - x1), b = fabs(y2 - y1);
        double c = rint(sqrt(a * a + b * b));
        double dx = dl * a / c, dy = dl * b / c;
        d.sx = x1; d.stx = x1 < x2 ? dx : -dx; nx = np_arange_len(x1, x2, d.stx);
        d.sy = y1; d.sty = y1 < y2 ? dy : -dy; ny = np_arange_len(y1, y2, d.sty);
    }
    d.n = nx < ny ? nx : ny;
    return d;
}
// dash k of the edge: the width-4 line from point 2k + 1 to point 2k (exists when 2k + 1 < n)
template <class SM>
MG_DEV void push_dash(SM &sm, const DashSeq &d, int k, int ord) {
    double xa = d.constx ? d.sx : np_arange_at(d.sx, d.stx, 2 * k + 1);
    double ya = d.consty ? d.sy : np_arange_at(d.sy, d.sty, 2 * k + 1);
    double xb = d.constx ? d.sx : np_arange_at(d.sx, d.stx, 2 * k);
    double yb = d.consty ? d.sy : np_arange_at(d.sy, d.sty, 2 * k);
    push_wide_line(sm, (int)rint(xa), (int)rint(ya), (int)rint(xb), (int)rint(yb), 4, ord);
}

template <class SM>
MG_DEV void band_put(SM &sm, int x, int y, int y0, uint32_t obit) {
    int r = y - y0;
    if (r >= 0 && r < SM::BAND && x >= 0 && x < MG_RES) {
        if constexpr (SM::ORDMAX) atomicMax(&sm.u.post.band[r][x], obit);
        else atomicOr(&sm.u.post.band[r][x / SM::MPW], obit << (SM::MBITS * (x % SM::MPW)));
    }
}

// pygame drawline of a clipped segment in k-form (major axis has |d|+1 pixels,
// minor offset of pixel k = floor(k * dminor / dmajor))
MG_DEV LineK line_k(int x1, int y1, int x2, int y2) {
    const int dx = x2 - x1, dy = y2 - y1;
    const int sgx = dx < 0 ? -1 : 1, sgy = dy < 0 ? -1 : 1;
    const int DX = sgx * dx + 1, DY = sgy * dy + 1;
    return {x1, y1, sgx, sgy, DX, DY, DX >= DY ? 1 : 0};
}

// the k-range [klo, khi] of a segment's pixels inside rows [y0, y0 + BAND)
template <int BAND>
MG_DEV void band_krange(const LineK &L, int y0, int &klo, int &khi) {
    // row index along the segment (m for x-major, k for y-major) in [0, DY)
    int mlo = L.sgy > 0 ? y0 - L.y1 : L.y1 - (y0 + BAND - 1);
    int mhi = mlo + BAND - 1;
    mlo = mlo > 0 ? mlo : 0;
    mhi = mhi < L.DY - 1 ? mhi : L.DY - 1;
    if (L.xmaj) {
        int rem;
        const int kl = udivmod(mlo * L.DX + L.DY - 1, L.DY, rem);            // smallest k with k*DY >= mlo*DX
        const int kh = udivmod((mhi + 1) * L.DX + L.DY - 1, L.DY, rem) - 1;  // largest k with k*DY < (mhi+1)*DX
        klo = kl; khi = kh < L.DX - 1 ? kh : L.DX - 1;
    } else {
        klo = mlo; khi = mhi;
    }
    if (mlo > mhi) { klo = 0; khi = -1; }
}

// pixels k in [ka, kb] of a segment; the minor offset is stepped incrementally
template <class SM>
MG_DEV void raster_krange(SM &sm, const LineK &L, int ka, int kb, int y0, uint32_t ord) {
    const int dmaj = L.xmaj ? L.DX : L.DY, dmin = L.xmaj ? L.DY : L.DX;
    const int ax = L.xmaj ? L.sgx : 0, ay = L.xmaj ? 0 : L.sgy;   // per k
    const int bx = L.xmaj ? 0 : L.sgx, by = L.xmaj ? L.sgy : 0;   // per m
    int acc, m = udivmod(ka * dmin, dmaj, acc);
    for (int k = ka; k <= kb; k++) {
        band_put(sm, L.x1 + ax * k + bx * m, L.y1 + ay * k + by * m, y0, ord);
        acc += dmin;
        if (acc >= dmaj) { acc -= dmaj; m++; }
    }
}

// one clipped segment, drawn by a group of RG_SEGLANES lanes (lane sub of the group takes one
// contiguous part of the band's pixel run); long runs are queued for the whole workgroup
template <class SM>
MG_DEV void segment_band(SM &sm, int x1, int y1, int x2, int y2, uint32_t ord, int y0, int sub) {
    int klo, khi;
    const LineK L = line_k(x1, y1, x2, y2);
    band_krange<SM::BAND>(L, y0, klo, khi);
    if (khi < klo) return;
    const int n = khi - klo + 1;
    if (n <= RG_SHORT * RG_SEGLANES) {
        const int chunk = (n + RG_SEGLANES - 1) / RG_SEGLANES;
        const int ka = klo + sub * chunk, kb = ka + chunk - 1 < khi ? ka + chunk - 1 : khi;
        if (ka <= kb) raster_krange(sm, L, ka, kb, y0, ord);
        return;
    }
    if (sub == 0) {
        int q = atomicAdd(&sm.nlong, 1);
        if (q < RG_MAXLONG) {
            int32_t *d = sm.u.post.lk[q];
            d[0] = L.x1; d[1] = L.y1; d[2] = L.sgx; d[3] = L.sgy; d[4] = L.DX; d[5] = L.DY; d[6] = L.xmaj;
            sm.u.post.lkr[q][0] = klo; sm.u.post.lkr[q][1] = khi; sm.u.post.lkr[q][2] = (int32_t)ord;
            return;
        }
        raster_krange(sm, L, klo, khi, y0, ord);   // queue full: drawn here
    }
}

// end points of solid outline edge k: (float->int first point) -> (int next vertex)
template <class SM>
MG_DEV void edge_ends(const SM &sm, int k, int &x1, int &y1, int &x2, int &y2, uint32_t &ord, bool &inside) {
    const uint32_t se = sm.sedge[k];
    const int v = se & 0x1FFF, g = sm.v_geom[v];
    const int fd = sm.fdelta[v];
    x1 = sm.vx[v] + (fd & 3) - 1; y1 = sm.vy[v] + ((fd >> 2) & 3) - 1;
    if (se & 0x4000u) { const int nx = sm.g_voff[g]; x2 = sm.vx[nx]; y2 = sm.vy[nx]; } // closing edge
    else { x2 = sm.vx[v + 1]; y2 = sm.vy[v + 1]; }
    ord = SM::ORDMAX ? (2u * g + 2) << RG_OSH : 1u << sm.g_ent[g];   // the outline layer's value
    inside = (se & 0x8000u) != 0;
}

// rows covered by outline item i (solid edge sub-lines or a dash line), before clipping
template <class SM>
MG_DEV void item_rows(const SM &sm, int i, int &ylo, int &yhi) {
    if (i < sm.nsedge) {
        if (sm.sedge[i] & 0x2000u) { ylo = 1; yhi = 0; return; }   // drawn from the line list (pre-clipped)
        int x1, y1, x2, y2;
        uint32_t ord;
        bool inside;
        edge_ends(sm, i, x1, y1, x2, y2, ord, inside);
        ylo = y1 < y2 ? y1 : y2;
        yhi = (y1 > y2 ? y1 : y2) + 1;  // the width-2 copy may sit one row lower
    } else {
        const int16_t *d = sm.dash[i - sm.nsedge];
        ylo = d[1] < d[3] ? d[1] : d[3];
        yhi = d[1] > d[3] ? d[1] : d[3];
    }
}

// rows of fill edge (ip -> v) under pygame draw_fillpoly's rule: with (ya, xa) the upper end, the
// edge meets rows ya <= y < yb, plus y == yb when yb is the polygon's last row; horizontal edges none
template <class SM>
MG_DEV void fill_edge(const SM &sm, int ve, int &xa, int &ya, int &xb, int &yb, int &side, int &r0, int &r1,
                      bool &lastrow) {
    const int v = ve & 0x3FFF, g = sm.v_geom[v];
    const int ip = (ve & 0x4000) ? v + sm.g_nv[g] - 1 : v - 1;
    const uint2 gi = sm.ginfo[g];
    const int gymin = (int16_t)(gi.x & 0xFFFF), gymax = (int16_t)(gi.x >> 16);
    const bool onscreen = (int16_t)(gi.y & 0xFFFF) <= (int16_t)(gi.y >> 16); // else never in a band list
    int y1 = sm.vy[ip], y2 = sm.vy[v];
    side = y1 < y2 ? 0 : 1;
    if (y1 < y2) { xa = sm.vx[ip]; ya = y1; xb = sm.vx[v]; yb = y2; }
    else { xa = sm.vx[v]; ya = y2; xb = sm.vx[ip]; yb = y1; }
    r0 = ya > 0 ? ya : 0;
    lastrow = yb == gymax;
    r1 = lastrow ? yb : yb - 1;
    r1 = r1 < MG_RES - 1 ? r1 : MG_RES - 1;
    if (y1 == y2 || !onscreen) r1 = r0 - 1;
    (void)gymin;
}

// render polygon point i (local coordinates); the goal rect is make_rect(w, h) of its entity
MG_DEV void rpoly_pt(const MGState &S, const mg_library *L, int e, const mg_rpoly &rp, int ent, int i, double &x, double &y) {
    if (rp.pts_off >= 0) { x = L->rpts[rp.pts_off + i][0]; y = L->rpts[rp.pts_off + i][1]; return; }
    double rad_h = AT(S.eh, ent) / 2, rad_w = AT(S.ew, ent) / 2;
    x = (i == 0 || i == 3) ? -rad_w : rad_w;
    y = (i == 0 || i == 1) ? rad_h : -rad_h;
}

// (sin, cos) of body b's angle: the physics' rotation cache (body_set_angle: the same correctly rounded
// sincos of the same angle) when it is current, else computed
MG_DEV void body_sincos(const MGState &S, int e, int b, double &s, double &c) {
    const double a = AT(S.ba, b);
    if (AT(S.bacache, b) == a) { s = AT(S.brs, b); c = AT(S.brc, b); }
    else mg_sincos(a, s, c);
}

// render.py Transform matrix x of one entity (pre_draw: entities.py:478-491, 751-754, 865-868); one
// thread per (entity, transform)
MG_DEV void entity_xform(const MGState &S, int e, int ent, int x, double *xf) {
    const int kind = AT(S.ekind, ent);
    double s, c;
    if (kind == MG_ENT_ROBOT) {
        const int b = AT(S.ebody0, ent);
        if (x == MG_XF_MAIN) {
            body_sincos(S, e, b, s, c);
            mg_transform_tr_sc(AT(S.bpx, b), AT(S.bpy, b), s, c, xf);
        } else if (x == MG_XF_FINGER_L || x == MG_XF_FINGER_R) {
            const int fb = b + 4 + (x - MG_XF_FINGER_L);
            body_sincos(S, e, fb, s, c);
            mg_transform_tr_sc(AT(S.bpx, fb), AT(S.bpy, fb), s, c, xf);
        } else if (x == MG_XF_PUPIL_L || x == MG_XF_PUPIL_R) {
            mg_transform_tr(0.0, 0.0, AT(S.ba, b + 2 + (x - MG_XF_PUPIL_L)) - AT(S.ba, b), xf);
        }
    } else if (kind == MG_ENT_BLOCK && x == MG_XF_MAIN) {
        const int b = AT(S.ebody0, ent);
        body_sincos(S, e, b, s, c);
        mg_transform_tr_sc(AT(S.bpx, b), AT(S.bpy, b), s, c, xf);
    } else if (kind == MG_ENT_GOAL && x == MG_XF_MAIN) {
        mg_transform_tr(AT(S.ex, ent), AT(S.ey, ent), 0.0, xf);
    }
}

// LDS slot of entity ent's transform x: the main transforms by entity, the robot's fingers and pupils after
template <class SM>
MG_DEV int xf_slot(int ent, int x) { return x == MG_XF_MAIN ? ent : SM::RG_MAXE + x - 1; }

// One (env, view) per workgroup.  MODE 0: LoRes outputs; 1: full-resolution frames; 2: LoRes outputs with the
// stacked views as window rings (RenderOut::wring) -- its own instantiation, so the materialising kernels carry
// none of its code (a shared build measured 4% slower render kernels, round 5).
#ifndef RG_SMALL_WPE
#define RG_SMALL_WPE 7                  // waves per SIMD the small class is compiled for: 72 VGPRs, 9 workgroups/CU
                                        // (measured: 7 -> 2.5% faster than the default 6; 8 = 64 VGPRs slower)
#endif
template <class SM, int MODE>
__global__ void __launch_bounds__(RG_THREADS)
__attribute__((amdgpu_waves_per_eu((SM::RG_MAXG <= 32 && RG_SMALL_WPE) ? RG_SMALL_WPE : 1)))
render_kernel(MGState S, const mg_library *__restrict__ L, RenderOut out) {
    __shared__ SM sm;
    // band geometry of the class: rows per band, LoRes rows per band (a thread resolves RG_BROWS / 2 blocks),
    // frame-stack threads (4 pixels each), first ring / plain writer thread, the band's LoRes bytes and 16-byte
    // chunks, first static-layer prefetch thread
    constexpr int RG_BAND = SM::BAND, RG_NBANDS = SM::NBANDS, RG_BROWS = SM::BROWS;
    constexpr int RG_STKT = RG_BROWS * MG_LORES / 4, RG_RING0 = RG_STKT > 64 ? RG_STKT : 64;
    constexpr int RG_BANDLO = RG_BROWS * RG_LOROW, RG_BANDLO16 = SM::BANDLO16;
    constexpr int RG_CPF0 = RG_THREADS - RG_BANDLO16 < 128 ? RG_THREADS - RG_BANDLO16 : 128;
    constexpr int mode = MODE == 2 ? 0 : MODE;
    constexpr bool WIN = MODE == 2;
    const int e = blockIdx.x, view = blockIdx.y, tid = threadIdx.x, lane = tid & 63;
    if (e >= S.n_envs || (out.mask && !out.mask[e])) return;
    // class chain (many-block tasks): S.rg_retry[e][view] holds the chain level that holds this (env, view)
    // in the current episode -- scenes keep their entities for an episode, so a pair that overflowed a class
    // skips it on later frames instead of rebuilding its setup there first.  An episode's first frame starts
    // again at the chain's first level.  Each class renders the pairs at its own level only.
    if (out.retry_in) {
        const bool restart = out.cls_level == out.first_level && S.episode_steps[e] == 0;
        const int stored = S.rg_retry[2 * e + view];
        const int lvl = restart || stored < out.first_level ? out.first_level : stored;
        if (lvl != out.cls_level) return;
        if (tid == 0 && stored != lvl) S.rg_retry[2 * e + view] = (uint8_t)lvl;
    }
    // an episode's first allo frame invalidates the static layer of the previous episode before anything can
    // fail: a frame that a class hands over (or gives up on) must not leave the old layer marked valid
    // (ADVICE r3); a successful first frame of the layer's class sets it again at the end
    if (mode == 0 && view == 0 && tid == 0 && S.scache_ok && S.episode_steps[e] == 0) S.scache_ok[e] = 0;
    MG_PROF_BEGIN(tid == 0);
    // capacity overflow: a class with a successor hands the (env, view) to it, else an env error
#define RG_FAIL() do { \
        if (tid == 0) { if (out.retry_out) S.rg_retry[2 * e + view] = (uint8_t)(out.cls_level + 1); \
                        else S.overflow[e] |= 4 << view; } \
        return; } while (0)
    const int nents = S.nents[e];
    if (nents > SM::RG_MAXE || (out.retry_out && out.force_retry > out.cls_level - out.first_level)) RG_FAIL();
    // ---- 1. geometry list (entity add order x render polys), colour table, view ----
    int my_r0 = 0, my_nr = 0;
    if (tid < nents) {
        int kind = AT(S.ekind, tid);
        if (kind == MG_ENT_ARENA) { my_r0 = L->arena_rpoly0; my_nr = L->arena_nrpoly; }
        else if (kind == MG_ENT_GOAL) { my_r0 = L->goal_rpoly0; my_nr = L->goal_nrpoly; }
        else if (kind == MG_ENT_ROBOT) { my_r0 = L->robot_rpoly0; my_nr = L->robot_nrpoly; }
        else { int t = AT(S.etype, tid); my_r0 = L->block_rpoly0[t]; my_nr = L->block_nrpoly[t]; }
        sm.u.pre.e_g0[tid + 1] = (int16_t)my_nr;
        sm.u.pre.e_r0[tid] = (int16_t)my_r0;
        sm.u.pre.ocnt[tid] = 0;
    }
    if (tid == 0) {
        sm.err = 0; sm.ndash = 0; sm.nsedge = 0; sm.nlong = 0; sm.u.pre.ndedge = 0; sm.u.pre.nconv = 0;
        sm.col[0] = pack_rgb(L->background);
        sm.u.pre.e_g0[0] = 0;
    }
    if (tid < RG_NBANDS) { sm.u.pre.bin_cnt[tid] = 0; sm.u.pre.ebin_cnt[tid] = 0; }
    if (tid < 17) sm.oord1[tid] = 0;
    if (tid < 64) {   // entities without a body (arena, goals): the static layer
        const int k = tid < nents ? AT(S.ekind, tid) : MG_ENT_ROBOT;
        const uint64_t b = __ballot(k == MG_ENT_ARENA || k == MG_ENT_GOAL);
        if (tid == 0) sm.smask = (uint32_t)b;
    }
#if !RG_XF_LATE
    if (view == 0 && tid == 32) { // Viewer.render: stack.push(self.transform) -> eye(3) @ view
        const double I3[9] = {1, 0, 0, 0, 1, 0, 0, 0, 1};
        mg_mat3_mul(I3, L->allo_view, sm.u.pre.view);
    }
    if (view == 1 && tid == 32) {
        // Viewer.set_cam_follow / ego_cam_matrix: P @ (scale @ (tr1 @ (rot @ tr2)))
        int rb = S.robot_body0[e];
        double rot[9], tr2[9], m1[9], m2[9], m3[9], sn, cs;
        body_sincos(S, e, rb, sn, cs); // sincos(-a) = (-sin a, cos a): a correctly rounded sin is odd
        mg_transform_tr_sc(0.0, 0.0, -sn, cs, rot);
        mg_transform_tr(-AT(S.bpx, rb), -AT(S.bpy, rb), 0.0, tr2);
        mg_mat3_mul(rot, tr2, m1);
        mg_mat3_mul(L->ego_tr1_m, m1, m2);
        mg_mat3_mul(L->ego_scale_m, m2, m3);
        mg_mat3_mul(L->pygame_m, m3, m1);
        const double I3[9] = {1, 0, 0, 0, 1, 0, 0, 0, 1};
        mg_mat3_mul(I3, m1, sm.u.pre.view);
    }
    if (tid >= 64 && tid - 64 < 5 * nents) {
        const int ent = (tid - 64) / 5, x = (tid - 64) % 5;
        if (x == MG_XF_MAIN || AT(S.ekind, ent) == MG_ENT_ROBOT)   // one robot per scene
            entity_xform(S, e, ent, x, sm.u.pre.e_xf[xf_slot<SM>(ent, x)]);
    }
#endif
    RG_SYNC();
    MG_PROF(10);
#if RG_XF_LATE
    // every thread forms the entities' first-geom offsets itself from the per-entity counts (independent
    // LDS reads, no barrier); the entity transforms and the view matrix (long serial f64 chains, correctly
    // rounded sincos for the pupils) run here, beside the geometry table's global loads
    int goff[SM::RG_MAXE + 1];
    goff[0] = 0;
#pragma unroll
    for (int k = 0; k < SM::RG_MAXE; k++) goff[k + 1] = goff[k] + (k < nents ? (int)sm.u.pre.e_g0[k + 1] : 0);
    const int G = goff[SM::RG_MAXE];
    if (G > SM::RG_MAXG) RG_FAIL();
    if (view == 0 && tid == RG_THREADS - 1) { // Viewer.render: stack.push(self.transform) -> eye(3) @ view
        const double I3[9] = {1, 0, 0, 0, 1, 0, 0, 0, 1};
        mg_mat3_mul(I3, L->allo_view, sm.u.pre.view);
    }
    if (view == 1 && tid == RG_THREADS - 1) {
        // Viewer.set_cam_follow / ego_cam_matrix: P @ (scale @ (tr1 @ (rot @ tr2)))
        int rb = S.robot_body0[e];
        double rot[9], tr2[9], m1[9], m2[9], m3[9], sn, cs;
        body_sincos(S, e, rb, sn, cs); // sincos(-a) = (-sin a, cos a): a correctly rounded sin is odd
        mg_transform_tr_sc(0.0, 0.0, -sn, cs, rot);
        mg_transform_tr(-AT(S.bpx, rb), -AT(S.bpy, rb), 0.0, tr2);
        mg_mat3_mul(rot, tr2, m1);
        mg_mat3_mul(L->ego_tr1_m, m1, m2);
        mg_mat3_mul(L->ego_scale_m, m2, m3);
        mg_mat3_mul(L->pygame_m, m3, m1);
        const double I3[9] = {1, 0, 0, 0, 1, 0, 0, 0, 1};
        mg_mat3_mul(I3, m1, sm.u.pre.view);
    }
    if (tid >= 64 && tid - 64 < 5 * nents) {
        const int ent = (tid - 64) / 5, x = (tid - 64) % 5;
        if (x == MG_XF_MAIN || AT(S.ekind, ent) == MG_ENT_ROBOT)   // one robot per scene
            entity_xform(S, e, ent, x, sm.u.pre.e_xf[xf_slot<SM>(ent, x)]);
    }
#else
    if (tid == 0) {
        for (int k = 0; k < nents; k++) sm.u.pre.e_g0[k + 1] += sm.u.pre.e_g0[k];
        sm.ngeom = sm.u.pre.e_g0[nents];
        if (sm.ngeom > SM::RG_MAXG) sm.err = 2;
    }
    RG_SYNC();
    if (sm.err) RG_FAIL();
    const int G = sm.ngeom;
#endif
    // one thread per geom: its entity (the last with a first geom <= g; the reads are independent), render
    // poly, colours
    for (int g = tid; g < G; g += RG_THREADS) {
        int ent = 0, g0 = 0;
#pragma unroll
        for (int k = 1; k < SM::RG_MAXE; k++) {
#if RG_XF_LATE
            const int gk = goff[k];
#else
            const int gk = sm.u.pre.e_g0[k];
#endif
            if (k < nents && gk <= g) { ent = k; g0 = gk; }
        }
        const int r = sm.u.pre.e_r0[ent] + g - g0;
        const mg_rpoly &rp = L->rpoly[r];
        const int ecol = AT(S.ecol, ent);
        sm.u.pre.g_rpoly[g] = (int16_t)r;
        sm.g_ent[g] = (int8_t)ent;
        if (rp.outline) {
            // two outlined polygons in one entity: the outline mask has one bit per entity
            if (atomicAdd(&sm.u.pre.ocnt[ent], 1) != 0) sm.err = 6;
            sm.oord1[ent + 1] = (uint16_t)((2 * g + 2) << RG_OSH);
        }
        sm.g_nv[g] = (int16_t)rp.npts;
        sm.col[2 * g + 1] = ref_colour(L, rp.col_ref, ecol);
        sm.col[2 * g + 2] = rp.outline ? ref_colour(L, rp.ocol_ref, ecol) : 0ull;
    }
    RG_SYNC();
    if (tid < 64) wave_exclusive_scan(sm.g_nv, sm.g_voff, G, lane);
    MG_PROF(11);
    // ---- 2. per-geom matrix: view @ T_last @ ... @ T_first (Geom.render stack) ----
    for (int g = tid; g < G; g += RG_THREADS) {
        const mg_rpoly &rp = L->rpoly[sm.u.pre.g_rpoly[g]];
        int ent = sm.g_ent[g];
        double M[9];
        for (int i = 0; i < 9; i++) M[i] = sm.u.pre.view[i];
        for (int k = rp.nxf - 1; k >= 0; k--) {
            int x = rp.xf[k];
            const double *T = x >= MG_XF_STATIC0 ? L->static_xf[x - MG_XF_STATIC0] : sm.u.pre.e_xf[xf_slot<SM>(ent, x)];
            mg_mat3_mul(M, T, M);
        }
        for (int i = 0; i < 6; i++) sm.u.pre.g_m[g][i] = M[i];
    }
    RG_SYNC();
    const int NV = sm.g_voff[G];
    if (NV > SM::RG_MAXVERT) RG_FAIL();
    for (int g = tid; g < G; g += RG_THREADS)
        for (int i = 0, v0 = sm.g_voff[g]; i < sm.g_nv[g]; i++) sm.v_geom[v0 + i] = (uint8_t)g;
    RG_SYNC();
    MG_PROF(12);
    // ---- 3. vertices -> int pixel coordinates (pygame (int) truncation); outline edges ----
    for (int v = tid; v < NV; v += RG_THREADS) {
        int g = sm.v_geom[v], i = v - sm.g_voff[g];
        const mg_rpoly &rp = L->rpoly[sm.u.pre.g_rpoly[g]];
        double x, y;
        rpoly_pt(S, L, e, rp, sm.g_ent[g], i, x, y);
        const double *M = sm.u.pre.g_m[g];
        double gx = __fma_rn(M[1], y, M[0] * x) + M[2];
        double gy = __fma_rn(M[4], y, M[3] * x) + M[5];
        const int ix = (int)gx, iy = (int)gy;
        sm.vx[v] = (int16_t)ix;
        sm.vy[v] = (int16_t)iy;
        // lines(): first point via float (pg FloatFromObj), second via int
        sm.fdelta[v] = (uint8_t)(((int)(float)gx - ix + 1) | (((int)(float)gy - iy + 1) << 2));
        if (rp.outline == MG_OUTLINE_SOLID) {
            const int k = atomicAdd(&sm.nsedge, 1);
            if (k < SM::RG_MAXSEDGE) sm.sedge[k] = (uint16_t)(v | (i + 1 == rp.npts ? 0x4000 : 0));
        } else if (rp.outline == MG_OUTLINE_DASHED) {
            int j = i + 1 == rp.npts ? 0 : i + 1;
            double xb, yb;
            rpoly_pt(S, L, e, rp, sm.g_ent[g], j, xb, yb);
            double gxb = __fma_rn(M[1], yb, M[0] * xb) + M[2], gyb = __fma_rn(M[4], yb, M[3] * xb) + M[5];
            const int ord = SM::ORDMAX ? (2 * g + 2) << RG_OSH : 1 << sm.g_ent[g];
            const int q = RG_DASH_SPLIT ? atomicAdd(&sm.u.pre.ndedge, 1) : RG_MAXDE;
            if (q < RG_MAXDE) {   // dashes drawn below, one thread per dash
                double *de = sm.u.pre.dedge[q];
                de[0] = gx; de[1] = gy; de[2] = gxb; de[3] = gyb;
                sm.u.pre.dedge_o[q] = ord;
            } else {              // list full: this thread draws the edge's dashes
                const DashSeq d = dash_seq(gx, gy, gxb, gyb);
                for (int k = 0; 2 * k + 1 < d.n; k++) push_dash(sm, d, k, ord);
            }
        }
    }
    RG_SYNC();
    MG_PROF(13);
    // ---- 4. per-geom bounds (vertex-parallel atomics) and the convexity premise of the fill: going
    //         round a polygon the sign of dy changes exactly twice (both vertex chains y-monotone) ----
    for (int g = tid; g < G; g += RG_THREADS) {
        int32_t *b = sm.u.pre.gbb[g];
        b[0] = 32767; b[1] = -32768; b[2] = 32767; b[3] = -32768;
        sm.u.pre.gchg[g] = 0;
    }
    {   // the dashes of the listed dashed edges: 32 threads per edge, dash k by thread k mod 32
        const int nde = sm.u.pre.ndedge < RG_MAXDE ? sm.u.pre.ndedge : RG_MAXDE;
        for (int i = tid; i < 32 * nde; i += RG_THREADS) {
            const double *de = sm.u.pre.dedge[i >> 5];
            const DashSeq d = dash_seq(de[0], de[1], de[2], de[3]);
            for (int k = i & 31; 2 * k + 1 < d.n; k += 32) push_dash(sm, d, k, sm.u.pre.dedge_o[i >> 5]);
        }
    }
    RG_SYNC();
    // solid outline edges that leave the surface: clip_and_draw_line_width's two sub-lines (the base line and the
    // +1 copy across the major axis) clipped once here into the line list, where they are drawn as the dash lines
    // are, instead of clipped again in every band they cross.  The list's free slots are taken in pairs; an edge
    // that finds none stays a solid edge clipped per band.  Invisible sub-lines keep their slot with rows -1.
    const int ndash0 = sm.ndash, dfree = SM::RG_MAXDASH - (ndash0 < SM::RG_MAXDASH ? ndash0 : SM::RG_MAXDASH);
    for (int i = tid; i < sm.nsedge && i < SM::RG_MAXSEDGE; i += RG_THREADS) {
        int x1, y1, x2, y2;
        uint32_t ord;
        bool inside;
        edge_ends(sm, i, x1, y1, x2, y2, ord, inside);
        const int ylo = y1 < y2 ? y1 : y2, yhi = (y1 > y2 ? y1 : y2) + 1;
        const int xl = x1 < x2 ? x1 : x2, xh = x1 > x2 ? x1 : x2;
        if (xl >= 0 && xh + 1 <= MG_RES - 1 && ylo >= 0 && yhi <= MG_RES - 1) { sm.sedge[i] |= 0x8000u; continue; }
        const int q = atomicAdd(&sm.u.pre.nconv, 2);
        if (q + 2 > dfree) continue;
        const bool xmaj = abs(x1 - x2) > abs(y1 - y2);
        for (int c = 0; c < 2; c++) {
            int a1 = x1 + ((c && !xmaj) ? 1 : 0), b1 = y1 + ((c && xmaj) ? 1 : 0);
            int a2 = x2 + ((c && !xmaj) ? 1 : 0), b2 = y2 + ((c && xmaj) ? 1 : 0);
            int16_t *d = sm.dash[ndash0 + q + c];
            if (!clipline(a1, b1, a2, b2)) { a1 = a2 = -1; b1 = b2 = -1; }
            d[0] = (int16_t)a1; d[1] = (int16_t)b1; d[2] = (int16_t)a2; d[3] = (int16_t)b2;
            sm.dash_o[ndash0 + q + c] = (uint16_t)ord;
        }
        sm.sedge[i] |= 0x2000u;
    }
    for (int v = tid; v < NV; v += RG_THREADS) {
        const int g = sm.v_geom[v], v0 = sm.g_voff[g], n = sm.g_nv[g];
        int32_t *b = sm.u.pre.gbb[g];
        const int x = sm.vx[v], y = sm.vy[v];
        atomicMin(&b[0], y); atomicMax(&b[1], y); atomicMin(&b[2], x); atomicMax(&b[3], x);
        const int nx = v + 1 == v0 + n ? v0 : v + 1;
        const int d = sm.vy[nx] - y;
        if (d == 0) continue;
        int p = v, dp = 0;
        for (int k = 0; k < n && dp == 0; k++) { // previous edge with dy != 0
            const int pp = p == v0 ? v0 + n - 1 : p - 1;
            dp = sm.vy[p] - sm.vy[pp];
            p = pp;
        }
        if ((dp > 0) != (d > 0)) atomicAdd(&sm.u.pre.gchg[g], 1);
    }
    RG_SYNC();
    for (int g = tid; g < G; g += RG_THREADS) {
        const int32_t *b = sm.u.pre.gbb[g];
        const int ymin = b[0], ymax = b[1];
        const int xmin = b[2] > 0 ? b[2] : 0, xmax = b[3] < MG_RES - 1 ? b[3] : MG_RES - 1;
        if (sm.u.pre.gchg[g] != 2 && sm.u.pre.gchg[g] != 0) sm.err = 4;
        sm.ginfo[g] = make_uint2((uint32_t)(uint16_t)ymin | ((uint32_t)(uint16_t)ymax << 16),
                                 (uint32_t)(uint16_t)xmin | ((uint32_t)(uint16_t)xmax << 16));
    }
    if (sm.ndash > SM::RG_MAXDASH) sm.err = 1;
    if (sm.nsedge > SM::RG_MAXSEDGE) sm.err = 5;
    const int nlines = ndash0 + min(sm.u.pre.nconv, dfree & ~1);   // dash lines + pre-clipped solid sub-lines
    const int nitems = sm.nsedge + (nlines < SM::RG_MAXDASH ? nlines : SM::RG_MAXDASH);
    for (int i = tid; i < nitems; i += RG_THREADS) {
        int ylo, yhi;
        item_rows(sm, i, ylo, yhi);
        ylo = ylo > 0 ? ylo : 0; yhi = yhi < MG_RES - 1 ? yhi : MG_RES - 1;
        for (int b = ylo / RG_BAND; b <= yhi / RG_BAND && ylo <= yhi; b++) atomicAdd(&sm.u.pre.bin_cnt[b], 1);
    }
    for (int i = tid; i < SM::RG_MAXG * RG_BAND; i += RG_THREADS)
        (&sm.bspan[0][0])[i] = (uint32_t)RG_EMPTY | ((uint32_t)RG_EMPTY << 16);
    RG_SYNC();
    MG_PROF(14);
    for (int v = tid; v < NV; v += RG_THREADS) { // fill edges per band (needs the geoms' row ranges)
        const int ve = v | (v == sm.g_voff[sm.v_geom[v]] ? 0x4000 : 0);
        int xa, ya, xb, yb, side, r0, r1;
        bool lastrow;
        fill_edge(sm, ve, xa, ya, xb, yb, side, r0, r1, lastrow);
        for (int b = r0 / RG_BAND; b <= r1 / RG_BAND && r0 <= r1; b++) atomicAdd(&sm.u.pre.ebin_cnt[b], 1);
    }
    RG_SYNC();
    if (tid < 64) {
        wave_exclusive_scan(sm.u.pre.bin_cnt, sm.bin_off, RG_NBANDS, lane);
        wave_exclusive_scan(sm.u.pre.ebin_cnt, sm.ebin_off, RG_NBANDS, lane);
    }
    RG_SYNC();
    const int nout = sm.bin_off[RG_NBANDS];
    if (nout + sm.ebin_off[RG_NBANDS] > SM::RG_MAXBIN) sm.err = 3;
#ifdef MG_PROFILE
    if (tid == 0) {   // scene sizes (tools/gpu_phase.py --sizes): maxima, then counts above candidate caps
        const unsigned long long nb = (unsigned long long)(nout + sm.ebin_off[RG_NBANDS]);
        atomicMax(&g_prof[52], (unsigned long long)G); atomicMax(&g_prof[53], (unsigned long long)NV);
        atomicMax(&g_prof[54], (unsigned long long)sm.ndash); atomicMax(&g_prof[55], (unsigned long long)sm.nsedge);
        atomicMax(&g_prof[56], nb);
        if (G > 48) atomicAdd(&g_prof[57], 1ull);
        if (G > 64) atomicAdd(&g_prof[58], 1ull);
        if (G > 72) atomicAdd(&g_prof[59], 1ull);
        if (NV > 1168) atomicAdd(&g_prof[60], 1ull);
        if (nb > 2080) atomicAdd(&g_prof[61], 1ull);
        if (sm.ndash > 128 || sm.nsedge > 712) atomicAdd(&g_prof[62], 1ull);
        atomicAdd(&g_prof[63], 1ull);
    }
#endif
    if (tid < RG_NBANDS) { sm.u.pre.bin_cnt[tid] = sm.bin_off[tid]; sm.u.pre.ebin_cnt[tid] = nout + sm.ebin_off[tid]; }
    RG_SYNC();
    if (sm.err) RG_FAIL();
    MG_PROF(15);
    for (int i = tid; i < nitems; i += RG_THREADS) {
        int ylo, yhi;
        item_rows(sm, i, ylo, yhi);
        ylo = ylo > 0 ? ylo : 0; yhi = yhi < MG_RES - 1 ? yhi : MG_RES - 1;
        for (int b = ylo / RG_BAND; b <= yhi / RG_BAND && ylo <= yhi; b++)
            sm.bin[atomicAdd(&sm.u.pre.bin_cnt[b], 1)] = (uint16_t)i;
    }
    for (int v = tid; v < NV; v += RG_THREADS) {
        const int ve = v | (v == sm.g_voff[sm.v_geom[v]] ? 0x4000 : 0);
        int xa, ya, xb, yb, side, r0, r1;
        bool lastrow;
        fill_edge(sm, ve, xa, ya, xb, yb, side, r0, r1, lastrow);
        for (int b = r0 / RG_BAND; b <= r1 / RG_BAND && r0 <= r1; b++)
            sm.bin[atomicAdd(&sm.u.pre.ebin_cnt[b], 1)] = (uint16_t)(ve | (lastrow ? 0x8000 : 0));
    }
    const int nsedge = sm.nsedge;
    MG_PROF(0);
#ifdef MG_PROFILE
    if (out.debug_skip & 16) return;  // setup only
#endif
    // ---- 5. bands ----
    uint8_t *ring = view == 0 ? S.hist_allo : S.hist_ego;
    const size_t FR = (size_t)MG_LORES * MG_LORES * 3;
    const bool fresh = S.episode_steps[e] == 0;
    const int head = S.hist_head[view * S.N + e];
    const int nh = fresh ? 0 : ((head + 1) & 3);
    const int pp = out.preproc;
    // frames-only outputs (compact multi-GPU gather): the current frame of each view, no stacks, no ring
    // (the receivers rebuild the stacks: mg_restack)
    const bool fo = out.frames_only != 0;
    const bool stacked0 = !fo && (pp == MG_PREPROC_LORESSTACK || (pp == MG_PREPROC_LORES4E && view == 1) ||
                                  (pp == MG_PREPROC_LORES4A && view == 0));
    // window ring (mg_bind_window): the stack of this view is a strided view of a ring the current frame is
    // written into once, channel-planar (as mg_restack_window's rings) -- no [96][96][12] stack, no frame ring
    uint8_t *const wring = (WIN && stacked0) ? out.wring[view] : nullptr;
    const bool win = WIN && wring != nullptr;
    const bool stacked = stacked0 && !win;
    const bool plain = fo || pp != MG_PREPROC_LORESSTACK;   // the view's own current-frame output
    // frame ring kept only where a stack reads it (LoRes3EA: ego ring, read by compose3ea_kernel)
    const bool keep_ring = stacked || (!fo && pp == MG_PREPROC_LORES3EA && view == 1);
    // Allocentric static layer.  The body-less entities (arena, goals) and the allo view matrix are fixed
    // for the whole episode, so the episode's first allo frame also resolves every block with those
    // entities alone (entity-bit classes: the outline layer tells the entities apart) and writes that frame
    // to S.scache; every later allo frame copies it into each 4x4 block that no geom of a body can reach
    // (its vertex bounds + RG_DMARGIN) and resolves only the others -- bands that no body reaches skip the
    // fill edges, outline lines and resolve altogether.  A block outside every body geom's reach has the
    // same pixels in the full scene as in the static-only scene, so the frame is bit-identical.
    // (allo frames whose only output is the plain current frame: LoRes4E, LoRes3EA, frames-only; a stacked
    // allo view writes ring and stack rows in every band anyway, and measured slower with the layer)
    // The many-block tasks' classes are compiled without it: their scenes' blocks reach most bands, and
    // the layer's code measured slower there (ClusterColour 2.72 -> 3.00 ms, MatchRegions 3.37 -> 3.41 ms).
    constexpr bool kLayer = RG_SCACHE && SM::RG_MAXG <= 32;
    const bool cview = kLayer && mode == 0 && view == 0 && out.scache_mode != 1 && !keep_ring && !stacked0 && plain;
    const bool mk_cache = cview && fresh && !SM::ORDMAX;
    const bool use_cache = cview && !fresh && S.scache_ok[e] != 0;
    uint8_t *const scache = S.scache + (size_t)e * FR;
    uint4 cpf = make_uint4(0, 0, 0, 0);   // wave 2, lanes 0-35: the next band's static-layer rows
    uint8_t *o_plain = view == 0 ? out.obs_allo : out.obs_ego;
    uint8_t *o_stack = pp == MG_PREPROC_LORESSTACK ? o_plain : out.obs_past;
    // 4x4 block of this thread: wave w covers block columns [32w, 32w + 32) of both block rows, so a
    // geom's x-range meets few waves and the per-geom fill test is skipped wave-wide elsewhere
    // (16-row bands: block rows oyl and oyl + 2)
    const int oyl = lane >> 5, ox = 32 * (tid >> 6) + (lane & 31), x0 = 4 * ox;
    // frame-stack threads (4 pixels each) hold frames t-3..t-1 of their pixels in registers
    const bool do_pf = mode == 0 && stacked && !fresh && tid < RG_STKT;
#ifdef MG_PROFILE
    const int dskip = out.debug_skip;
#else
    const int dskip = 0;
#endif
    // prefetch frames t-3..t-1 of this thread's 4 pixels of band y0 (ring slots nh+1..nh+3, never
    // written this step): 3 dwords per frame
    uint32_t pf[3][3];
    auto prefetch = [&](int y0) {
#pragma unroll
        for (int k = 0; k < 3; k++) {
            const int sl = (nh + 1 + k) & 3;
            const uint32_t *src = (const uint32_t *)(ring + ((size_t)sl * S.N + e) * FR + (size_t)(y0 / 4) * RG_LOROW) + 3 * tid;
#pragma unroll
            for (int w = 0; w < 3; w++) pf[k][w] = src[w];
        }
    };
    // geoms whose rows meet band y0, in draw order (ballot compaction by one wave)
    auto band_list = [&](int y0) {
        int cnt = 0;
        uint32_t *dm = sm.dmask[(y0 / RG_BAND) & 1];
        if (use_cache && lane < 3) dm[lane] = 0u;   // same wave: ordered before the atomics below
        for (int base = 0; base < G; base += 64) {
            const int g = base + lane;
            bool ov = false;
            if (g < G) {
                const uint2 gi = sm.ginfo[g];
                const int ymin = (int16_t)(gi.x & 0xFFFF), ymax = (int16_t)(gi.x >> 16);
                const int xmin = (int16_t)(gi.y & 0xFFFF), xmax = (int16_t)(gi.y >> 16);
                ov = ymax >= y0 && ymin < y0 + RG_BAND && xmin <= xmax;
                // LoRes columns of this band that a body geom can reach
                if (use_cache && !((sm.smask >> sm.g_ent[g]) & 1u) && ymax + RG_DMARGIN >= y0 &&
                    ymin - RG_DMARGIN < y0 + RG_BAND) {
                    const int c0 = (xmin - RG_DMARGIN > 0 ? xmin - RG_DMARGIN : 0) >> 2;
                    const int c1 = (xmax + RG_DMARGIN < MG_RES - 1 ? xmax + RG_DMARGIN : MG_RES - 1) >> 2;
#pragma unroll
                    for (int w = 0; w < 3; w++) {
                        const int lo = c0 > 32 * w ? c0 : 32 * w, hi = c1 < 32 * w + 31 ? c1 : 32 * w + 31;
                        if (lo <= hi) atomicOr(&dm[w], (hi - lo == 31 ? 0xFFFFFFFFu : ((1u << (hi - lo + 1)) - 1u)) << (lo - 32 * w));
                    }
                }
            }
            const uint64_t m = __ballot(ov);
            if (ov) {
                const int slot = cnt + __popcll(m & ((1ull << lane) - 1ull));
                sm.blist[slot] = (int16_t)g;
                sm.bxr[slot] = sm.ginfo[g].y;
                sm.gslot[g] = (int16_t)slot;
            }
            cnt += __popcll(m);
        }
        if (lane == 0) sm.nblist = cnt;
    };
    // Allocentric frame whose only output is its plain current frame (LoRes4E, LoRes3EA, frames-only): the
    // bands outside the rows a body geom can reach are the static layer's rows, copied in bulk; the band
    // loop runs over [band0, band1) only.  Elsewhere (frame rings / stacks to write) it runs over every band.
    const bool brange = use_cache;
    auto body_rows = [&](int &b0, int &b1) {   // wave 2: the bands a body geom can reach
        int y0 = MG_RES, y1 = -1;
        for (int g = lane; g < G; g += 64) {
            if ((sm.smask >> sm.g_ent[g]) & 1u) continue;
            const uint2 gi = sm.ginfo[g];
            const int ymin = (int16_t)(gi.x & 0xFFFF) - RG_DMARGIN, ymax = (int16_t)(gi.x >> 16) + RG_DMARGIN;
            y0 = ymin < y0 ? ymin : y0; y1 = ymax > y1 ? ymax : y1;
        }
#pragma unroll
        for (int off = 1; off < 64; off <<= 1) {
            const int a = __shfl_xor(y0, off), b = __shfl_xor(y1, off);
            y0 = a < y0 ? a : y0; y1 = b > y1 ? b : y1;
        }
        y0 = y0 > 0 ? y0 : 0; y1 = y1 < MG_RES - 1 ? y1 : MG_RES - 1;
        b0 = y0 <= y1 ? y0 / RG_BAND : 0;
        b1 = y0 <= y1 ? y1 / RG_BAND + 1 : 0;
    };
    auto cache_prefetch = [&](int y0) {
        if (use_cache && tid >= RG_CPF0 && tid < RG_CPF0 + RG_BANDLO16)
            cpf = *(const uint4 *)(scache + (size_t)(y0 / 4) * RG_LOROW + 16 * (tid - RG_CPF0));
    };
    // band 0 prologue: outline layer cleared (it overlays the setup scratch: after the binning's
    // counters are done with), band list, prefetch (later bands: in the previous band's tail)
    if (do_pf) prefetch(0);
    RG_SYNC();
    for (int i = tid; i < (int)(sizeof(sm.u.post.band) / 16); i += RG_THREADS)
        ((uint4 *)&sm.u.post.band[0][0])[i] = make_uint4(0, 0, 0, 0);
    if (tid == 0) sm.nlong = 0;
    if (tid >= 128) {
        int b0 = 0, b1 = RG_NBANDS;
        if (brange) body_rows(b0, b1);
        if (lane == 0) { sm.brng[0] = b0; sm.brng[1] = b1; }
        if (b0 < b1) band_list(RG_BAND * b0);
        if (b0 < b1) cache_prefetch(RG_BAND * b0);
    }
#ifdef MG_PROFILE
    if (tid < 4) sm.pw[tid] = 0u;
#endif
    RG_SYNC();
    const int band0 = __builtin_amdgcn_readfirstlane(sm.brng[0]), band1 = __builtin_amdgcn_readfirstlane(sm.brng[1]);
    if (RG_CPF0 < 128 && tid < 128 && band0 < band1) cache_prefetch(RG_BAND * band0);   // the prefetch threads below wave 2
    if (brange) {   // the static layer's rows outside [band0, band1): RG_BANDLO16 x 16 B per band, 4 per thread per round
        const int nst = (RG_NBANDS - (band1 - band0)) * RG_BANDLO16;
        for (int i0 = tid; i0 < nst; i0 += 4 * RG_THREADS) {
            uint4 v[4];
#pragma unroll
            for (int k = 0; k < 4; k++) {
                const int i = i0 + k * RG_THREADS;
                const int b = i / RG_BANDLO16, bb = b < band0 ? b : b + (band1 - band0);
                const size_t o = (size_t)bb * RG_BANDLO + 16 * (i % RG_BANDLO16);
                v[k] = i < nst ? *(const uint4 *)(scache + o) : make_uint4(0, 0, 0, 0);
                if (out.scache_mode == 2) v[k] = make_uint4(0x55555555u, 0x55555555u, 0x55555555u, 0x55555555u);
            }
#pragma unroll
            for (int k = 0; k < 4; k++) {
                const int i = i0 + k * RG_THREADS;
                const int b = i / RG_BANDLO16, bb = b < band0 ? b : b + (band1 - band0);
                if (i < nst) *(uint4 *)(o_plain + (size_t)e * FR + (size_t)bb * RG_BANDLO + 16 * (i % RG_BANDLO16)) = v[k];
            }
        }
    }
    for (int y0 = RG_BAND * band0, band_i = band0; band_i < band1; y0 += RG_BAND, band_i++) {
        const size_t lrow = (size_t)(y0 / 4) * RG_LOROW;  // byte offset of this band's LoRes rows
        MG_PROF(1);
        MG_PROF_MARK(t_lines);
        // fill spans of this band's rows: each binned fill edge writes its chain's intersection
        // (side 0: edges going down the vertex order, side 1: going up) of the rows it meets here
        const int nbl = sm.nblist;
        // static layer: this band's rows first (blocks that need a resolve overwrite theirs after the
        // barrier below); a band that no body geom reaches is the static layer's rows
        const uint32_t *dmb = sm.dmask[band_i & 1];
        const bool sband = use_cache && __builtin_amdgcn_readfirstlane(dmb[0] | dmb[1] | dmb[2]) == 0u;
        if (use_cache && tid >= RG_CPF0 && tid < RG_CPF0 + RG_BANDLO16)
            sm.u.post.lo[tid - RG_CPF0] = out.scache_mode == 2 ? make_uint4(0x55555555u, 0x55555555u, 0x55555555u, 0x55555555u) : cpf;
        // (wave 1; the outline items run on waves 0 and 2 at the same time)
        const bool fwave = tid >= 64 && tid < 128;
        const int lt = tid < 64 ? tid : tid - 64;   // outline-item thread index (waves 0, 2)
        for (int j = sm.ebin_off[band_i] + nout + tid - 64; fwave && !sband && j < sm.ebin_off[band_i + 1] + nout && !(dskip & 8); j += 64) {
            // fill_edge without the geom-bounds lookup: the bin entry carries the closing and last-row flags
            const int ve = sm.bin[j];
            const int v = ve & 0x3FFF, g = sm.v_geom[v];
            const int yv = sm.vy[v], xv = sm.vx[v];
            int yp, xp;
            if (ve & 0x4000) { const int ip = v + sm.g_nv[g] - 1; yp = sm.vy[ip]; xp = sm.vx[ip]; }
            else { yp = sm.vy[v - 1]; xp = sm.vx[v - 1]; }
            const int side = yp < yv ? 0 : 1;
            const int xa = side ? xv : xp, ya = side ? yv : yp, xb = side ? xp : xv, yb = side ? yp : yv;
            const int r0 = ya > 0 ? ya : 0;
            int r1 = (ve & 0x8000) ? yb : yb - 1;
            r1 = r1 < MG_RES - 1 ? r1 : MG_RES - 1;
            const int slot = sm.gslot[g];
            int16_t *col = (int16_t *)&sm.bspan[slot][0] + side;
            const int ra = r0 > y0 ? r0 : y0, rb = r1 < y0 + RG_BAND - 1 ? r1 : y0 + RG_BAND - 1;
            if (ra > rb) continue;
            // x = xa + trunc((y - ya) * (xb - xa) / (yb - ya)), stepped row by row (y >= ya, yb > ya)
            const int d = yb - ya, adx = xb > xa ? xb - xa : xa - xb, sg = xb >= xa ? 1 : -1;
            const int n0 = (ra - ya) * adx;
            int r, rs;
            int q = udivmod(n0, d, r);
            const int qs = udivmod(adx, d, rs);
            for (int y = ra; y <= rb; y++) {
                col[2 * (y - y0)] = (int16_t)(xa + sg * q);
                q += qs; r += rs;
                if (r >= d) { r -= d; q++; }
            }
        }
        if (RG_SPANW && fwave && !sband) {
            // each row's two chain intersections -> (l, w = r - l); a row missing either intersection is
            // empty: l = RG_EMPTY, w = 0 (no pixel has x = 32767).  Only this wave writes bspan in the band.
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // this wave's span writes are done
            for (int i = tid - 64; i < nbl * RG_BAND; i += 64) {
                uint32_t *sp = &sm.bspan[0][0] + i;
                const uint32_t v = *sp;
                const int sa = (int16_t)(v & 0xFFFF), sb = (int16_t)(v >> 16);
                const int l = sa < sb ? sa : sb, rr = sa < sb ? sb : sa;
                *sp = rr == RG_EMPTY ? (uint32_t)RG_EMPTY : ((uint32_t)(uint16_t)l | ((uint32_t)min(rr - l, 0xFFFF) << 16));
            }
        }
        // outline items of this band: solid width-2 edges (clip_and_draw_line_width: base line plus one
        // offset copy, each clipped) and clipped dashed-goal lines
        // (one thread per segment: solid edges contribute two, dash lines one)
        for (int j2 = 2 * sm.bin_off[band_i] + lt / RG_SEGLANES; !fwave && !sband && j2 < 2 * sm.bin_off[band_i + 1] && !(dskip & 1);
             j2 += 128 / RG_SEGLANES) {
            const int i = sm.bin[j2 >> 1], c = j2 & 1;
            int x1, y1, x2, y2;
            uint32_t ord;
            bool clip = false;
            if (i < nsedge) {
                bool inside;
                edge_ends(sm, i, x1, y1, x2, y2, ord, inside);
                const bool xmaj = abs(x1 - x2) > abs(y1 - y2);
                const int ox = (c && !xmaj) ? 1 : 0, oy = (c && xmaj) ? 1 : 0;
                x1 += ox; x2 += ox; y1 += oy; y2 += oy;
                clip = !inside;
            } else {
                if (c) continue;
                const int16_t *d = sm.dash[i - nsedge];
                x1 = d[0]; y1 = d[1]; x2 = d[2]; y2 = d[3];
                ord = (uint32_t)sm.dash_o[i - nsedge];
            }
            if (clip && !clipline(x1, y1, x2, y2)) continue;
            segment_band(sm, x1, y1, x2, y2, ord, y0, lt % RG_SEGLANES);
        }
        MG_PROF_MAXW(sm.pw[0], t_lines);
        if (!sband) RG_SYNC();   // sband is uniform (LDS read after a barrier)
        const int nlong = sm.nlong;
        if (nlong > 0) {
            for (int q = 0; q < nlong && q < RG_MAXLONG; q++) {
                const int32_t *d = sm.u.post.lk[q];
                LineK Lk = {d[0], d[1], d[2], d[3], d[4], d[5], d[6]};
                const uint32_t ord = (uint32_t)sm.u.post.lkr[q][2];
                const int klo = sm.u.post.lkr[q][0], khi = sm.u.post.lkr[q][1];
                const int chunk = (khi - klo + RG_THREADS) / RG_THREADS;  // ceil(n / threads)
                const int ka = klo + tid * chunk, kb = ka + chunk - 1 < khi ? ka + chunk - 1 : khi;
                if (ka <= kb) raster_krange(sm, Lk, ka, kb, y0, ord);
            }
            RG_SYNC();
        }
        MG_PROF(2);
        // fill + resolve, one thread per 4x4 block: painter's order over the band's geoms (later
        // fill wins), max with the outline layer, colour, then the area sum of the block
        uint8_t *lo8 = (uint8_t *)sm.u.post.lo;
        MG_PROF_MARK(t_fill);
        const bool need = !use_cache || ((dmb[ox >> 5] >> (ox & 31)) & 1u);
        // pass 0: the frame (skipped where the static layer stands); pass 1 (the episode's first allo frame):
        // the static layer, the body-less entities alone
        auto resolve = [&](auto sonly_c, int oy) {
            constexpr bool sonly = decltype(sonly_c)::value;
            const int yb = 4 * oy, ya = y0 + yb, lpix = oy * MG_LORES + ox;
            uint32_t o[4][4];
#pragma unroll
            for (int r = 0; r < 4; r++)
#pragma unroll
                for (int c = 0; c < 4; c++) o[r][c] = 0u;
            // every LDS read of a slot is indexed by the slot alone (no blist -> ginfo chain), so the
            // reads of successive slots are independent
#pragma unroll 2
            for (int slot = 0; slot < ((dskip & 2) ? 0 : nbl); slot++) {
                const uint32_t xr = sm.bxr[slot];
                const int xmin = (int16_t)(xr & 0xFFFF), xmax = (int16_t)(xr >> 16);
                if (xmax < x0 || xmin > x0 + 3) continue;
                if constexpr (sonly)
                    if (!((sm.smask >> sm.g_ent[sm.blist[slot]]) & 1u)) continue;
                const uint4 s4 = *(const uint4 *)&sm.bspan[slot][yb];
                const uint32_t ord = (2 * (uint32_t)sm.blist[slot] + 1) << RG_OSH;
#pragma unroll
                for (int r = 0; r < 4; r++) {
                    const uint32_t spr = r == 0 ? s4.x : r == 1 ? s4.y : r == 2 ? s4.z : s4.w;
                    if constexpr (RG_SPANW) {
                        // pixel x covered iff 0 <= x - l <= w (unsigned compare; empty rows: l = 32767, w = 0)
                        const int l = (int16_t)(spr & 0xFFFF);
                        const uint32_t w = spr >> 16;
#pragma unroll
                        for (int c = 0; c < 4; c++)
                            o[r][c] = (uint32_t)(x0 + c - l) <= w ? ord : o[r][c];
                    } else {
                        const int sa = (int16_t)(spr & 0xFFFF), sb = (int16_t)(spr >> 16);
                        const int l = sa < sb ? sa : sb, rr = sa < sb ? sb : sa;
                        if (rr == RG_EMPTY) continue;   // a row needs an intersection on both chains
#pragma unroll
                        for (int c = 0; c < 4; c++)
                            if (x0 + c >= l && x0 + c <= rr) o[r][c] = ord;
                    }
                }
            }
            (void)ya;
#pragma unroll
            for (int r = 0; r < ((dskip & 32) ? 0 : 4); r++) {
                if constexpr (SM::ORDMAX) {
                    const uint4 lv = *(const uint4 *)&sm.u.post.band[yb + r][x0];
                    o[r][0] = o[r][0] > lv.x ? o[r][0] : lv.x;
                    o[r][1] = o[r][1] > lv.y ? o[r][1] : lv.y;
                    o[r][2] = o[r][2] > lv.z ? o[r][2] : lv.z;
                    o[r][3] = o[r][3] > lv.w ? o[r][3] : lv.w;
                } else {
                    // the highest entity bit of each pixel -> that entity's outline ordinal (oord1[0] = 0)
                    uint32_t w0, w1;
                    if constexpr (SM::MPW == 8) { w0 = sm.u.post.band[yb + r][ox >> 1] >> (16 * (ox & 1)); w1 = 0u; }
                    else if constexpr (SM::MPW == 4) { w0 = sm.u.post.band[yb + r][ox]; w1 = 0u; }
                    else { const uint2 t = *(const uint2 *)&sm.u.post.band[yb + r][2 * ox]; w0 = t.x; w1 = t.y; }
                    if (w0 | w1) {
#pragma unroll
                        for (int c = 0; c < 4; c++) {
                            const uint32_t wc = (SM::MPW >= 4 || c < 2) ? w0 : w1;
                            const uint32_t m = (wc >> (SM::MBITS * (c % SM::MPW))) & (sonly ? sm.smask : SM::MMASK);
                            const uint32_t oo = sm.oord1[m ? 32 - __clz((int)m) : 0];
                            o[r][c] = o[r][c] > oo ? o[r][c] : oo;
                        }
                    }
                }
            }
            // area sum of the block's 16 colours (a one-lookup path for blocks of one ordinal measured 2% slower:
            // the 15 compares cost more than the 16 LDS reads they save)
            uint64_t sum = 0;
#pragma unroll
            for (int r = 0; r < 4; r++)
#pragma unroll
                for (int c = 0; c < 4; c++) sum += *(const uint64_t *)((const char *)sm.col + (o[r][c] << (3 - RG_OSH)));
            if (mode == 1) {
                for (int r = 0; r < 4; r++) {
                    uint8_t *dst = out.full + ((((size_t)e * 2 + view) * MG_RES + y0 + yb + r) * MG_RES + x0) * 3;
                    for (int c = 0; c < 4; c++) {
                        const uint64_t cc = *(const uint64_t *)((const char *)sm.col + (o[r][c] << (3 - RG_OSH)));
                        dst[3 * c] = (uint8_t)cc; dst[3 * c + 1] = (uint8_t)(cc >> 16); dst[3 * c + 2] = (uint8_t)(cc >> 32);
                    }
                }
            } else {
                uint8_t *dst8 = sonly ? (uint8_t *)sm.u.post.los : lo8;
                // window views: the same bytes channel-planar in `los` ([3][2 x 96]; a window view never uses the
                // static layer that otherwise holds it), so the tail stores 16-byte chunks with no byte shuffle
                uint8_t *pl8 = (WIN && win && !sonly) ? (uint8_t *)sm.u.post.los : nullptr;
                for (int ch = 0; ch < ((dskip & 256) ? 0 : 3); ch++) {
                    const int ss = (int)((sum >> (16 * ch)) & 0xFFFF);
                    // round half to even of ss / 16: + 7, + 1 more when ss / 16 is odd
                    uint8_t v8;
                    if (RG_OFS) v8 = (uint8_t)((ss + 7 + ((ss >> 4) & 1)) >> 4);
                    else { const int q = ss >> 4, rm = ss & 15; v8 = (uint8_t)(q + (rm > 8 || (rm == 8 && (q & 1)))); }
                    dst8[lpix * 3 + ch] = v8;
                    if (WIN && pl8) pl8[ch * (RG_BROWS * MG_LORES) + lpix] = v8;
                }
            }
        };
        if constexpr (RG_BROWS == 2) {
            if (need) resolve(std::false_type{}, oyl);
            if (mk_cache) resolve(std::true_type{}, oyl);
        } else {   // 16-row bands: block rows oyl and oyl + 2, one after the other (registers)
#pragma unroll 1
            for (int oy = oyl; oy < RG_BROWS; oy += 2) {
                if (need) resolve(std::false_type{}, oy);
                if (mk_cache) resolve(std::true_type{}, oy);
            }
        }
        MG_PROF_MAXW(sm.pw[1], t_fill);
        RG_SYNC();
        MG_PROF(3);
#ifdef MG_PROFILE
        _pacc[5] += sm.pw[0]; _pacc[6] += sm.pw[1]; _pacc[7] += nlong; _pacc[8] += sm.bin_off[band_i + 1] - sm.bin_off[band_i];
        _pacc[9] += nbl;
        if (tid < 4) sm.pw[tid] = 0u;
#endif
        // tail: this band's outputs (wave 0: frame stack, waves 1-2: ring + current frame), and the
        // next band's empty spans, cleared outline layer, band list (wave 2) and prefetch
        for (int i = tid; i < nbl * RG_BAND; i += RG_THREADS)
            (&sm.bspan[0][0])[i] = (uint32_t)RG_EMPTY | ((uint32_t)RG_EMPTY << 16);
        for (int i = tid; i < ((dskip & 128) ? 0 : (int)(sizeof(sm.u.post.band) / 16)); i += RG_THREADS)
            ((uint4 *)&sm.u.post.band[0][0])[i] = make_uint4(0, 0, 0, 0);
        if (tid == 0) sm.nlong = 0;
        if (mode == 0 && !(dskip & 4)) {
            if (tid >= RG_RING0) {
                // ring of the last 4 LoRes frames: slot nh (all 4 slots at episode start)
                const int nring = keep_ring ? (fresh ? 4 : 1) * RG_BANDLO16 : 0;
                const int nplain = nring + (plain ? RG_BANDLO16 : 0);
                for (int t = tid - RG_RING0; t < nplain + (mk_cache ? RG_BANDLO16 : 0); t += RG_THREADS - RG_RING0) {
                    if (t < nring) {
                        const int sl = fresh ? t / RG_BANDLO16 : nh, c = t % RG_BANDLO16;
                        *(uint4 *)(ring + ((size_t)sl * S.N + e) * FR + lrow + 16 * c) = sm.u.post.lo[c];
                    } else if (t < nplain) {
                        const int c = t - nring;
                        *(uint4 *)(o_plain + (size_t)e * FR + lrow + 16 * c) = sm.u.post.lo[c];
                    } else {
                        const int c = t - nplain;
                        *(uint4 *)(scache + lrow + 16 * c) = sm.u.post.los[c];
                    }
                }
            } else if (win) {
                // window ring: the band's LoRes rows of each colour plane (RG_BROWS x 96 B, planar in `los` since the
                // resolve) into every slot of this step's frame (fresh: of frames t-3 .. t; the slot lists come
                // from the host, RenderOut::wsl), by the stack's threads: RG_BANDLO16 x 16 B per slot
                const int lst = fresh ? 1 : 0, nwin = out.wnsl[lst] * RG_BANDLO16;
                for (int t = tid; t < nwin; t += RG_RING0) {
                    const int slot = out.wsl[lst][t / RG_BANDLO16];
                    const int c = t % RG_BANDLO16, pl = c / (RG_BANDLO16 / 3), j = c % (RG_BANDLO16 / 3);   // plane, its 16-byte chunk
                    *(uint4 *)(wring + ((size_t)e * (out.wK + 3) + slot) * FR + (size_t)pl * (MG_LORES * MG_LORES) +
                               (size_t)(y0 / 4) * MG_LORES + 16 * j) = sm.u.post.los[c];
                }
            } else if (stacked && tid < RG_STKT && !(dskip & 64)) {
                // FlattenFrameStack: [96][96][12] = frames oldest..newest concatenated per pixel; one thread
                // per 4 pixels: 3 dwords of each frame in, 12 dwords (3 x 16 B) out
                const uint32_t *c32 = (const uint32_t *)sm.u.post.lo;
                uint32_t f[4][3];
#pragma unroll
                for (int w = 0; w < 3; w++) {
                    f[3][w] = c32[3 * tid + w];
#pragma unroll
                    for (int k = 0; k < 3; k++) f[k][w] = fresh ? f[3][w] : pf[k][w];
                }
                uint32_t o[12];
#pragma unroll
                for (int b = 0; b < 48; b++) {   // output byte b: pixel b / 12, frame (b % 12) / 3, channel b % 3
                    const int px = b / 12, k = (b % 12) / 3, sb = 3 * px + b % 3;  // source byte within 12
                    const uint32_t byte = (f[k][sb / 4] >> (8 * (sb % 4))) & 255u;
                    if (b % 4 == 0) o[b / 4] = byte; else o[b / 4] |= byte << (8 * (b % 4));
                }
                uint4 *dst = (uint4 *)(o_stack + (size_t)e * FR * 4 + lrow * 4) + 3 * tid;
                dst[0] = make_uint4(o[0], o[1], o[2], o[3]);
                dst[1] = make_uint4(o[4], o[5], o[6], o[7]);
                dst[2] = make_uint4(o[8], o[9], o[10], o[11]);
            }
        }
        if (band_i + 1 < band1) {
            if (tid >= 128) band_list(y0 + RG_BAND);
            if (do_pf) prefetch(y0 + RG_BAND);
            cache_prefetch(y0 + RG_BAND);
        }
        RG_SYNC();
        MG_PROF(4);
    }
    if (sm.err) { if (tid == 0) S.overflow[e] |= 4 << view; }
    if (mode == 0 && tid == 0) S.hist_head[view * S.N + e] = nh;
    if (cview && fresh && tid == 0) S.scache_ok[e] = mk_cache ? 1 : 0;
    MG_PROF_END(16 * view);
}
#undef RG_FAIL
