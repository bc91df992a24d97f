/*
 * ns_oracle.c -- CPU restatement of the reference hot path (TEST INFRASTRUCTURE).
 * See ns_oracle.h for provenance and the rules on who may call this code.
 * Citations: /root/reference/SRC/<file>:<line>.
 */
#include "ns_oracle.h"

#include <math.h>
#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

static char og_err[512];
const char* og_last_error(void) { return og_err; }

/* OpenMP threads of the per-cell loops (1 unless og_set_threads: the checker stays serial;
 * bench.py's cpu_baseline times 1 thread and the host's cores).  Loops write disjoint
 * cells; a reduction's order depends only on the thread count. */
static int og_nt = 1;
void og_set_threads(int n) { og_nt = n > 0 ? n : 1; }
int og_get_threads(void) { return og_nt; }
static void set_err(const char* fmt, ...) {
    va_list ap; va_start(ap, fmt); vsnprintf(og_err, sizeof og_err, fmt, ap); va_end(ap);
}

#define TOL 1e-8 /* Grid.h:7 */
static int equals_(double a, double b) { return fabs(a - b) > TOL ? 0 : 1; } /* Grid.cpp:292 */

typedef struct {
    int nx, ny;     /* normal (Grid.cpp:40-61) */
    double loc[3];  /* Grid.cpp:36-59 */
    int btype;
    double binfo;
    double c[2];    /* ghost[0].constant, FluidSolver.cpp:89-96 */
} og_edge;

struct og_grid {
    int nx, ny, N;
    double *hx, *hy;
    double *xc, *yc;     /* by compact id */
    int *id;             /* nx*ny, i*ny+j */
    int *tag;            /* nx*ny*4: W,E,S,N edge index or -1 (Grid.h:33) */
    int *ci, *cj;        /* id -> (i,j) */
    int ne;
    og_edge* e;
};

static inline int IDX(const og_grid* g, int i, int j) { return i * g->ny + j; }
/* Grid::inDomain Grid.cpp:214-218 */
static inline int in_dom(const og_grid* g, int i, int j) {
    if (i < 0 || i >= g->nx || j < 0 || j >= g->ny) return 0;
    return g->id[IDX(g, i, j)] >= 0;
}
static inline int CID(const og_grid* g, int i, int j) { return g->id[IDX(g, i, j)]; }
static inline int TAG(const og_grid* g, int i, int j, int k) { return g->tag[4 * IDX(g, i, j) + k]; }

void og_grid_free(og_grid* g) {
    if (!g) return;
    free(g->hx); free(g->hy); free(g->xc); free(g->yc); free(g->id); free(g->tag);
    free(g->ci); free(g->cj); free(g->e); free(g);
}
int og_grid_N(const og_grid* g) { return g->N; }
int og_grid_nx(const og_grid* g) { return g->nx; }
int og_grid_ny(const og_grid* g) { return g->ny; }

void og_grid_info(const og_grid* g, double* hx, double* hy, int* id, int* tag, double* xc, double* yc) {
    if (hx) memcpy(hx, g->hx, sizeof(double) * g->nx);
    if (hy) memcpy(hy, g->hy, sizeof(double) * g->ny);
    if (id) memcpy(id, g->id, sizeof(int) * g->nx * g->ny);
    if (tag) memcpy(tag, g->tag, sizeof(int) * 4 * g->nx * g->ny);
    if (xc) memcpy(xc, g->xc, sizeof(double) * g->N);
    if (yc) memcpy(yc, g->yc, sizeof(double) * g->N);
}

/* GenerateFaces' per-direction loop, Grid.cpp:78-120.  Returns count or -1. */
static int gen_faces(double start, int ns, const double* spec, double** F, double** H) {
    int cap = 64, n = 0;
    double* f = malloc(sizeof(double) * (cap + 1));
    double* h = malloc(sizeof(double) * cap);
    f[0] = start;
    double hh = 0.0;
    for (int s = 0; s < ns; s++) {
        double a = spec[4 * s + 0], b = spec[4 * s + 1], cnt = spec[4 * s + 2], r = spec[4 * s + 3];
        if (!equals_(a, f[n]) || (n == 0 && cnt <= 0)) goto bad;
        if (r > 0) {
            if (cnt <= 0) cnt = ceil(log((b - a) * (r - 1) / hh + 1) / log(r));
            hh = (b - a) * (r - 1) / (pow(r, cnt) - 1);
        } else if (r == -1) {
            if (cnt <= 0) cnt = ceil((b - a) / hh);
            hh = (b - a) / cnt;
        } else goto bad;
        double x = a;
        for (int j = 0; j < cnt; j++) { /* int vs double compare, Grid.cpp:91,97 */
            if (n + 1 >= cap) {
                cap *= 2;
                f = realloc(f, sizeof(double) * (cap + 1));
                h = realloc(h, sizeof(double) * cap);
            }
            x += hh;
            f[n + 1] = x; h[n] = hh; n++;
            if (r > 0) hh *= r;
        }
    }
    *F = f; *H = h;
    return n;
bad:
    free(f); free(h);
    return -1;
}

og_grid* og_grid_polygon(int nv, const double* vx, const double* vy, int nsx, const double* xspec,
                         int nsy, const double* yspec, const int* btype, const double* binfo) {
    og_grid* g = calloc(1, sizeof *g);
    double xr0 = 1e15, xr1 = -1e15, yr0 = 1e15, yr1 = -1e15;
    g->ne = nv;
    g->e = calloc(nv, sizeof(og_edge));
    /* GenerateEdges Grid.cpp:28-72 (polygon closed back to vertex 0) */
    for (int k = 0; k < nv; k++) {
        double x0 = vx[k], y0 = vy[k], x1 = vx[(k + 1) % nv], y1 = vy[(k + 1) % nv];
        og_edge* e = &g->e[k];
        if (x1 == x0) {
            e->loc[0] = x1;
            if (y1 > y0) { e->loc[1] = y0; e->loc[2] = y1; e->nx = -1; xr0 = x1 < xr0 ? x1 : xr0; }
            else         { e->loc[2] = y0; e->loc[1] = y1; e->nx = 1;  xr1 = x1 > xr1 ? x1 : xr1; }
        } else if (y1 == y0) {
            e->loc[0] = y1;
            if (x1 > x0) { e->loc[1] = x0; e->loc[2] = x1; e->ny = 1;  yr1 = y1 > yr1 ? y1 : yr1; }
            else         { e->loc[2] = x0; e->loc[1] = x1; e->ny = -1; yr0 = y1 < yr0 ? y1 : yr0; }
        } else { set_err("Edges should be parallel to the x-axis or y-axis"); og_grid_free(g); return NULL; }
    }
    double *X, *Y;
    int nx = gen_faces(xr0, nsx, xspec, &X, &g->hx);
    if (nx < 0) { set_err("Invalid specification for number of cells"); og_grid_free(g); return NULL; }
    int ny = gen_faces(yr0, nsy, yspec, &Y, &g->hy);
    if (ny < 0) { free(X); set_err("Invalid specification for number of cells"); og_grid_free(g); return NULL; }
    if (!equals_(xr1, X[nx]) || !equals_(yr1, Y[ny])) { /* Grid.cpp:122-125 */
        free(X); free(Y); set_err("Invalid specification for number of cells"); og_grid_free(g); return NULL;
    }
    g->nx = nx; g->ny = ny;
    g->id = malloc(sizeof(int) * nx * ny);
    g->tag = malloc(sizeof(int) * 4 * nx * ny);
    /* GenerateCells + Cleanup + Interior, Grid.cpp:131-185 */
    int n = 0;
    for (int i = 0; i < nx; i++)
        for (int j = 0; j < ny; j++) {
            double X0 = X[i], X1 = X[i + 1], Y0 = Y[j], Y1 = Y[j + 1];
            double cx = 0.5 * (X0 + X1), cy = 0.5 * (Y0 + Y1);
            int* t = &g->tag[4 * (i * ny + j)];
            t[0] = t[1] = t[2] = t[3] = -1;
            int intersect = 0;
            for (int k = 0; k < nv; k++) {
                const og_edge* e = &g->e[k];
                if (e->nx != 0) {
                    if (cy > e->loc[1] && cy < e->loc[2]) {
                        if (e->loc[0] > cx) intersect++;
                        if (e->nx == -1 && equals_(X0, e->loc[0])) t[0] = k;
                        if (e->nx == 1 && equals_(X1, e->loc[0])) t[1] = k;
                    }
                } else {
                    if (cx > e->loc[1] && cx < e->loc[2]) {
                        if (e->ny == -1 && equals_(Y0, e->loc[0])) t[2] = k;
                        if (e->ny == 1 && equals_(Y1, e->loc[0])) t[3] = k;
                    }
                }
            }
            g->id[i * ny + j] = (intersect % 2) ? n++ : -1;
        }
    g->N = n;
    g->xc = malloc(sizeof(double) * n); g->yc = malloc(sizeof(double) * n);
    g->ci = malloc(sizeof(int) * n); g->cj = malloc(sizeof(int) * n);
    for (int i = 0; i < nx; i++)
        for (int j = 0; j < ny; j++) {
            int c = g->id[i * ny + j];
            if (c < 0) continue;
            g->xc[c] = 0.5 * (X[i] + X[i + 1]); g->yc[c] = 0.5 * (Y[j] + Y[j + 1]);
            g->ci[c] = i; g->cj[c] = j;
        }
    free(X); free(Y);
    /* BCs + ConstructGhostStencils FluidSolver.cpp:84-103 */
    for (int k = 0; k < nv; k++) {
        og_edge* e = &g->e[k];
        e->btype = btype[k]; e->binfo = binfo[k];
        e->c[0] = e->c[1] = 0.0;
        if (e->btype == OG_INLET_UNI) {
            if (e->nx == 0) e->c[1] = 2 * e->binfo; else e->c[0] = 2 * e->binfo;
        } else if (e->btype == OG_WALL) {
            if (e->nx != 0) e->c[1] = 2 * e->binfo; else e->c[0] = 2 * e->binfo;
        } else if (e->btype != OG_NEUMANN) {
            /* INLET_PARABOLIC / unset read an empty constant vector (UB,
             * FluidSolver.cpp:86-87,171); PRESSURE has no ghost (:150,168). */
            set_err("edge %d: unsupported boundary condition type %d", k, e->btype);
            og_grid_free(g); return NULL;
        }
    }
    /* one-cell-thick geometry would index j-1 = -1 (FluidSolver.cpp:470-477) */
    for (int c = 0; c < n; c++) {
        int i = g->ci[c], j = g->cj[c];
        if ((!in_dom(g, i, j + 1) && !in_dom(g, i, j - 1)) || (!in_dom(g, i + 1, j) && !in_dom(g, i - 1, j))) {
            set_err("one-cell-thick geometry at cell (%d,%d) is not supported", i, j);
            og_grid_free(g); return NULL;
        }
    }
    return g;
}

/* ---------------------------------------------------------------------- */
/* ghosts: EvaluateGhostStencil_V / _P, FluidSolver.cpp:166-181            */

static inline double ghost_v(const og_grid* g, const double* q, int i, int j, int e, int d) {
    const og_edge* E = &g->e[e];
    double r = 0.0;
    if (E->btype == OG_NEUMANN) { r += 1.0 * q[CID(g, i, j)]; r += 0.0; }
    else { r += -1.0 * q[CID(g, i, j)]; r += E->c[d]; }
    return r;
}
static inline double ghost_p(const og_grid* g, const double* p, int i, int j, int e) {
    const og_edge* E = &g->e[e];
    double r = 0.0;
    if (E->btype == OG_NEUMANN) {
        r += 2.5 * p[CID(g, i, j)];
        r += -2.0 * p[CID(g, i - E->nx, j - E->ny)];
        r += 0.5 * p[CID(g, i - 2 * E->nx, j - 2 * E->ny)];
    } else r += 1.0 * p[CID(g, i, j)];
    return r;
}

/* minmode FluidSolver.cpp:671-674 */
static inline double minmode(double a, double b) {
    if (a * b > 0) return a * fmin(1.0, fabs(b / a));
    return 0;
}

/* SlopeLimiter FluidSolver.cpp:283-325 */
static void slope(const og_grid* g, const double* u, const double* v, int i, int j, int d, double* s) {
    const double* h = d == 0 ? g->hx : g->hy;
    int c = CID(g, i, j);
    double a0, a1, b0, b1;
    if (d == 0) {
        if (in_dom(g, i + 1, j)) {
            a0 = 2 * (u[CID(g, i + 1, j)] - u[c]) / (h[i + 1] + h[i]);
            a1 = 2 * (v[CID(g, i + 1, j)] - v[c]) / (h[i + 1] + h[i]);
        } else {
            a0 = (ghost_v(g, u, i, j, TAG(g, i, j, 1), 0) - u[c]) / h[i];
            a1 = (ghost_v(g, v, i, j, TAG(g, i, j, 1), 1) - v[c]) / h[i];
        }
        if (in_dom(g, i - 1, j)) {
            b0 = 2 * (u[c] - u[CID(g, i - 1, j)]) / (h[i - 1] + h[i]);
            b1 = 2 * (v[c] - v[CID(g, i - 1, j)]) / (h[i - 1] + h[i]);
        } else {
            b0 = (u[c] - ghost_v(g, u, i, j, TAG(g, i, j, 0), 0)) / h[i];
            b1 = (v[c] - ghost_v(g, v, i, j, TAG(g, i, j, 0), 1)) / h[i];
        }
    } else {
        if (in_dom(g, i, j + 1)) {
            a0 = 2 * (u[CID(g, i, j + 1)] - u[c]) / (h[j + 1] + h[j]);
            a1 = 2 * (v[CID(g, i, j + 1)] - v[c]) / (h[j + 1] + h[j]);
        } else {
            a0 = (ghost_v(g, u, i, j, TAG(g, i, j, 3), 0) - u[c]) / h[j];
            a1 = (ghost_v(g, v, i, j, TAG(g, i, j, 3), 1) - v[c]) / h[j];
        }
        if (in_dom(g, i, j - 1)) {
            b0 = 2 * (u[c] - u[CID(g, i, j - 1)]) / (h[j - 1] + h[j]);
            b1 = 2 * (v[c] - v[CID(g, i, j - 1)]) / (h[j - 1] + h[j]);
        } else {
            b0 = (u[c] - ghost_v(g, u, i, j, TAG(g, i, j, 2), 0)) / h[j];
            b1 = (v[c] - ghost_v(g, v, i, j, TAG(g, i, j, 2), 1)) / h[j];
        }
    }
    s[0] = minmode(a0, b0);
    s[1] = minmode(a1, b1);
}

static inline double fnn(double l, double r) { return 0.5 * (l * l + r * r - fabs(l + r) * (r - l)); }
static inline double fuv(double u1, double v1, double u2, double v2) {
    return 0.5 * (u1 * v1 + u2 * v2 - 0.5 * fabs(v1 + v2) * (u2 - u1) - 0.5 * fabs(u2 + u1) * (v2 - v1));
}

/* ConvectiveFlux FluidSolver.cpp:205-281 */
static void conv_flux(const og_grid* g, const double* u, const double* v, int i, int j, double* C) {
    const double *hx = g->hx, *hy = g->hy;
    int c = CID(g, i, j);
    double SL[2], sl[2], u1, u2, v1, v2;
    slope(g, u, v, i, j, 0, SL);
    u2 = u[c] - hx[i] / 2 * SL[0];
    v2 = v[c] - hx[i] / 2 * SL[1];
    if (TAG(g, i, j, 0) == -1) {
        slope(g, u, v, i - 1, j, 0, sl);
        u1 = u[CID(g, i - 1, j)] + hx[i - 1] / 2 * sl[0];
        v1 = v[CID(g, i - 1, j)] + hx[i - 1] / 2 * sl[1];
    } else {
        u1 = 0.5 * (u[c] + ghost_v(g, u, i, j, TAG(g, i, j, 0), 0));
        v1 = 0.5 * (v[c] + ghost_v(g, v, i, j, TAG(g, i, j, 0), 1));
    }
    C[0] = fnn(u1, u2);
    C[1] = fuv(u1, v1, u2, v2);
    u1 = u[c] + hx[i] / 2 * SL[0];
    v1 = v[c] + hx[i] / 2 * SL[1];
    if (TAG(g, i, j, 1) == -1) {
        slope(g, u, v, i + 1, j, 0, sl);
        u2 = u[CID(g, i + 1, j)] - hx[i + 1] / 2 * sl[0];
        v2 = v[CID(g, i + 1, j)] - hx[i + 1] / 2 * sl[1];
    } else {
        u2 = 0.5 * (u[c] + ghost_v(g, u, i, j, TAG(g, i, j, 1), 0));
        v2 = 0.5 * (v[c] + ghost_v(g, v, i, j, TAG(g, i, j, 1), 1));
    }
    C[2] = fnn(u1, u2);
    C[3] = fuv(u1, v1, u2, v2);
    slope(g, u, v, i, j, 1, SL);
    u2 = u[c] - hy[j] / 2 * SL[0];
    v2 = v[c] - hy[j] / 2 * SL[1];
    if (TAG(g, i, j, 2) == -1) {
        slope(g, u, v, i, j - 1, 1, sl);
        u1 = u[CID(g, i, j - 1)] + hy[j - 1] / 2 * sl[0];
        v1 = v[CID(g, i, j - 1)] + hy[j - 1] / 2 * sl[1];
    } else {
        u1 = 0.5 * (u[c] + ghost_v(g, u, i, j, TAG(g, i, j, 2), 0));
        v1 = 0.5 * (v[c] + ghost_v(g, v, i, j, TAG(g, i, j, 2), 1));
    }
    C[5] = fnn(v1, v2);
    C[4] = fuv(u1, v1, u2, v2);
    u1 = u[c] + hy[j] / 2 * SL[0];
    v1 = v[c] + hy[j] / 2 * SL[1];
    if (TAG(g, i, j, 3) == -1) {
        slope(g, u, v, i, j + 1, 1, sl);
        u2 = u[CID(g, i, j + 1)] - hy[j + 1] / 2 * sl[0];
        v2 = v[CID(g, i, j + 1)] - hy[j + 1] / 2 * sl[1];
    } else {
        u2 = 0.5 * (u[c] + ghost_v(g, u, i, j, TAG(g, i, j, 3), 0));
        v2 = 0.5 * (v[c] + ghost_v(g, v, i, j, TAG(g, i, j, 3), 1));
    }
    C[7] = fnn(v1, v2);
    C[6] = fuv(u1, v1, u2, v2);
}

/* DiffusiveFlux FluidSolver.cpp:183-203 */
static void diff_flux(const og_grid* g, double re, const double* q, int i, int j, int d, double* D) {
    const double *hx = g->hx, *hy = g->hy;
    int c = CID(g, i, j);
    if (in_dom(g, i - 1, j)) D[0] = (1 / re) * (q[c] - q[CID(g, i - 1, j)]) / (hx[i] + hx[i - 1]);
    else D[0] = (0.5 / re / hx[i]) * (q[c] - ghost_v(g, q, i, j, TAG(g, i, j, 0), d));
    if (in_dom(g, i + 1, j)) D[1] = (1 / re) * (q[CID(g, i + 1, j)] - q[c]) / (hx[i] + hx[i + 1]);
    else D[1] = -(0.5 / re / hx[i]) * (q[c] - ghost_v(g, q, i, j, TAG(g, i, j, 1), d));
    if (in_dom(g, i, j - 1)) D[2] = (1 / re) * (q[c] - q[CID(g, i, j - 1)]) / (hy[j] + hy[j - 1]);
    else D[2] = (0.5 / re / hy[j]) * (q[c] - ghost_v(g, q, i, j, TAG(g, i, j, 2), d));
    if (in_dom(g, i, j + 1)) D[3] = (1 / re) * (q[CID(g, i, j + 1)] - q[c]) / (hy[j] + hy[j + 1]);
    else D[3] = -(0.5 / re / hy[j]) * (q[c] - ghost_v(g, q, i, j, TAG(g, i, j, 3), d));
}

/* ApplyBoundaryConditions FluidSolver.cpp:458-510 */
static void apply_bc(const og_grid* g, double dt, double re, int i, int j, const double* gx,
                     const double* gy, double* ru, double* rv) {
    const double *hx = g->hx, *hy = g->hy;
    int c = CID(g, i, j);
    int calc = 0;
    double w, W, D = 0.0;
    for (int k = 0; k < 4; k++) {
        int t = TAG(g, i, j, k);
        if (t == -1) continue;
        const og_edge* e = &g->e[t];
        if (!calc) {
            if (e->nx != 0) {
                if (!in_dom(g, i, j + 1)) D = 2.0 * (gx[c] - gx[CID(g, i, j - 1)]) / (hy[j] + hy[j - 1]);
                else if (!in_dom(g, i, j - 1)) D = 2.0 * (gx[CID(g, i, j + 1)] - gx[c]) / (hy[j] + hy[j + 1]);
                else D = gx[CID(g, i, j + 1)] / (hy[j] + hy[j + 1]) - gx[CID(g, i, j - 1)] / (hy[j] + hy[j - 1])
                         - gx[c] * (1 / (hy[j] + hy[j + 1]) - 1 / (hy[j] + hy[j - 1]));
            } else {
                if (!in_dom(g, i + 1, j)) D = 2.0 * (gy[c] - gy[CID(g, i - 1, j)]) / (hx[i] + hx[i - 1]);
                else if (!in_dom(g, i - 1, j)) D = 2.0 * (gy[CID(g, i + 1, j)] - gy[c]) / (hx[i] + hx[i + 1]);
                else D = gy[CID(g, i + 1, j)] / (hx[i] + hx[i + 1]) - gy[CID(g, i - 1, j)] / (hx[i] + hx[i - 1])
                         - gy[c] * (1 / (hx[i] + hx[i + 1]) - 1 / (hx[i] + hx[i - 1]));
            }
            calc = 1;
        }
        if (e->btype == OG_NEUMANN) {
            if (e->nx != 0) {
                w = dt * e->nx * hx[i] * D;
                W = dt * (0.5 / re / pow(hx[i], 2)) * w;
                rv[c] += W;
            } else {
                w = dt * e->ny * hy[j] * D;
                W = dt * (0.5 / re / pow(hy[j], 2)) * w;
                ru[c] += W;
            }
        } else {
            if (e->nx != 0) {
                W = dt * (0.5 / re / pow(hx[i], 2)) * e->c[0];
                ru[c] += W;
                w = 2 * dt * (gy[c] + e->nx * hx[i] * D / 2);
                W = dt * (0.5 / re / pow(hx[i], 2)) * (e->c[1] + w);
                rv[c] += W;
            } else {
                W = dt * (0.5 / re / pow(hy[j], 2)) * e->c[1];
                rv[c] += W;
                w = 2 * dt * (gx[c] + e->ny * hy[j] * D / 2);
                W = dt * (0.5 / re / pow(hy[j], 2)) * (e->c[0] + w);
                ru[c] += W;
            }
        }
    }
}

/* ConstructRHS_V FluidSolver.cpp:327-363 */
void og_rhs_velocity(const og_grid* g, double dt, double re, const double* u, const double* v,
                     const double* gx, const double* gy, double* cu, double* cv, double* ru, double* rv) {
    const double *hx = g->hx, *hy = g->hy;
    /* VecSet(0) ; VecAXPY(1, u) ; VecAXPY(0.5dt, conv0)  (:335-340) */
#pragma omp parallel for schedule(static) num_threads(og_nt)
    for (int c = 0; c < g->N; c++) {
        ru[c] = 0.0 + 1.0 * u[c]; ru[c] += 0.5 * dt * cu[c];
        rv[c] = 0.0 + 1.0 * v[c]; rv[c] += 0.5 * dt * cv[c];
    }
#pragma omp parallel for schedule(static) num_threads(og_nt)
    for (int i = 0; i < g->nx; i++)
        for (int j = 0; j < g->ny; j++) {
            double D[4], C[8], val;
            int c = CID(g, i, j);
            if (c < 0) continue;
            diff_flux(g, re, u, i, j, 0, D);
            val = dt * ((D[1] - D[0]) / hx[i] + (D[3] - D[2]) / hy[j]);
            ru[c] += val;
            diff_flux(g, re, v, i, j, 1, D);
            val = dt * ((D[1] - D[0]) / hx[i] + (D[3] - D[2]) / hy[j]);
            rv[c] += val;
            conv_flux(g, u, v, i, j, C);
            val = (C[2] - C[0]) / hx[i] + (C[6] - C[4]) / hy[j];
            cu[c] = val;
            val *= -1.5 * dt;
            ru[c] += val;
            val = (C[3] - C[1]) / hx[i] + (C[7] - C[5]) / hy[j];
            cv[c] = val;
            val *= -1.5 * dt;
            rv[c] += val;
            apply_bc(g, dt, re, i, j, gx, gy, ru, rv);
        }
}

/* face interpolation used by Div_V and GradP (FluidSolver.cpp:390-412, 429-451) */
static inline double face_w(const og_grid* g, const double* q, int i, int j) {
    double r = g->hx[i] / (g->hx[i - 1] + g->hx[i]);
    return q[CID(g, i - 1, j)] * r + q[CID(g, i, j)] * (1 - r);
}
static inline double face_e(const og_grid* g, const double* q, int i, int j) {
    double r = g->hx[i] / (g->hx[i + 1] + g->hx[i]);
    return q[CID(g, i + 1, j)] * r + q[CID(g, i, j)] * (1 - r);
}
static inline double face_s(const og_grid* g, const double* q, int i, int j) {
    double r = g->hy[j] / (g->hy[j - 1] + g->hy[j]);
    return q[CID(g, i, j - 1)] * r + q[CID(g, i, j)] * (1 - r);
}
static inline double face_n(const og_grid* g, const double* q, int i, int j) {
    double r = g->hy[j] / (g->hy[j + 1] + g->hy[j]);
    return q[CID(g, i, j + 1)] * r + q[CID(g, i, j)] * (1 - r);
}

/* Div_V FluidSolver.cpp:380-418 */
static double div_v(const og_grid* g, const double* u, const double* v, int i, int j) {
    int c = CID(g, i, j);
    double V0 = TAG(g, i, j, 0) == -1 ? face_w(g, u, i, j) : 0.5 * (u[c] + ghost_v(g, u, i, j, TAG(g, i, j, 0), 0));
    double V1 = TAG(g, i, j, 1) == -1 ? face_e(g, u, i, j) : 0.5 * (u[c] + ghost_v(g, u, i, j, TAG(g, i, j, 1), 0));
    double V2 = TAG(g, i, j, 2) == -1 ? face_s(g, v, i, j) : 0.5 * (v[c] + ghost_v(g, v, i, j, TAG(g, i, j, 2), 1));
    double V3 = TAG(g, i, j, 3) == -1 ? face_n(g, v, i, j) : 0.5 * (v[c] + ghost_v(g, v, i, j, TAG(g, i, j, 3), 1));
    return (V1 - V0) / g->hx[i] + (V3 - V2) / g->hy[j];
}

void og_divergence(const og_grid* g, double dt, const double* us, const double* vs, double* rhs) {
#pragma omp parallel for schedule(static) num_threads(og_nt)
    for (int c = 0; c < g->N; c++) rhs[c] = div_v(g, us, vs, g->ci[c], g->cj[c]) / dt;
}

/* GradP FluidSolver.cpp:420-456 */
static void grad_p(const og_grid* g, const double* p, int i, int j, double* gr) {
    int c = CID(g, i, j);
    double V0 = TAG(g, i, j, 0) == -1 ? face_w(g, p, i, j) : 0.5 * (p[c] + ghost_p(g, p, i, j, TAG(g, i, j, 0)));
    double V1 = TAG(g, i, j, 1) == -1 ? face_e(g, p, i, j) : 0.5 * (p[c] + ghost_p(g, p, i, j, TAG(g, i, j, 1)));
    double V2 = TAG(g, i, j, 2) == -1 ? face_s(g, p, i, j) : 0.5 * (p[c] + ghost_p(g, p, i, j, TAG(g, i, j, 2)));
    double V3 = TAG(g, i, j, 3) == -1 ? face_n(g, p, i, j) : 0.5 * (p[c] + ghost_p(g, p, i, j, TAG(g, i, j, 3)));
    gr[0] = (V1 - V0) / g->hx[i];
    gr[1] = (V3 - V2) / g->hy[j];
}

void og_grad_phi(const og_grid* g, const double* phi, double* gx, double* gy) {
#pragma omp parallel for schedule(static) num_threads(og_nt)
    for (int c = 0; c < g->N; c++) {
        double gr[2];
        grad_p(g, phi, g->ci[c], g->cj[c], gr);
        gx[c] = gr[0]; gy[c] = gr[1];
    }
}

/* CorrectVelocities FluidSolver.cpp:512-534 */
void og_correct(const og_grid* g, double dt, const double* us, const double* vs, const double* phi,
                double* u, double* v, double* gx, double* gy) {
#pragma omp parallel for schedule(static) num_threads(og_nt)
    for (int c = 0; c < g->N; c++) {
        double gr[2];
        grad_p(g, phi, g->ci[c], g->cj[c], gr);
        gx[c] = gr[0]; gy[c] = gr[1];
        u[c] = us[c] - dt * gr[0];
        v[c] = vs[c] - dt * gr[1];
    }
}

/* ---------------------------------------------------------------------- */
/* operators, ConstructLHS FluidSolver.cpp:105-145 + AddGhostStencils :147-164 */

static const int NXk[4] = {-1, 1, 0, 0}, NYk[4] = {0, 0, -1, 1};

static inline double face_w8(const og_grid* g, int i, int j, int k, int nb) {
    /* nb: neighbour weight 2/(h(h+h_nb)); else boundary weight 1/h^2 (:119-126) */
    if (NXk[k] != 0) return nb ? 2.0 / (g->hx[i] * (g->hx[i] + g->hx[i + NXk[k]])) : 1.0 / pow(g->hx[i], 2);
    return nb ? 2.0 / (g->hy[j] * (g->hy[j] + g->hy[j + NYk[k]])) : 1.0 / pow(g->hy[j], 2);
}

void og_apply_poisson(const og_grid* g, const double* p, double* out) {
    for (int c = 0; c < g->N; c++) {
        int i = g->ci[c], j = g->cj[c];
        double s = 0.0;
        for (int k = 0; k < 4; k++) {
            int ii = i + NXk[k], jj = j + NYk[k];
            if (in_dom(g, ii, jj)) s += face_w8(g, i, j, k, 1) * (p[CID(g, ii, jj)] - p[c]);
            else s += face_w8(g, i, j, k, 0) * (ghost_p(g, p, i, j, TAG(g, i, j, k)) - p[c]);
        }
        out[c] = s;
    }
}

/* L_V q without the ghost constants (those go to the RHS, :495-506) */
static void apply_lv(const og_grid* g, const double* q, double* out) {
    for (int c = 0; c < g->N; c++) {
        int i = g->ci[c], j = g->cj[c];
        double s = 0.0;
        for (int k = 0; k < 4; k++) {
            int ii = i + NXk[k], jj = j + NYk[k];
            if (in_dom(g, ii, jj)) s += face_w8(g, i, j, k, 1) * (q[CID(g, ii, jj)] - q[c]);
            else {
                double wself = g->e[TAG(g, i, j, k)].btype == OG_NEUMANN ? 1.0 : -1.0;
                s += face_w8(g, i, j, k, 0) * (wself * q[c] - q[c]);
            }
        }
        out[c] = s;
    }
}

void og_apply_helmholtz(const og_grid* g, double alpha, const double* q, double* out) {
    apply_lv(g, q, out);
    for (int c = 0; c < g->N; c++) out[c] = q[c] - alpha * out[c];
}

void og_pressure(const og_grid* g, double alpha, const double* phi, double* P) {
    og_apply_poisson(g, phi, P);
    for (int c = 0; c < g->N; c++) P[c] = phi[c] - alpha * P[c];
}

/* diagonal of the operators (for the Jacobi preconditioner / sweeps) */
static void diag_poisson(const og_grid* g, double* d) {
    for (int c = 0; c < g->N; c++) {
        int i = g->ci[c], j = g->cj[c];
        double s = 0.0;
        for (int k = 0; k < 4; k++) {
            int ii = i + NXk[k], jj = j + NYk[k];
            if (in_dom(g, ii, jj)) s -= face_w8(g, i, j, k, 1);
            else if (g->e[TAG(g, i, j, k)].btype == OG_NEUMANN) s += 1.5 * face_w8(g, i, j, k, 0);
        }
        d[c] = s;
    }
}
static void diag_helmholtz(const og_grid* g, double alpha, double* d) {
    for (int c = 0; c < g->N; c++) {
        int i = g->ci[c], j = g->cj[c];
        double s = 0.0;
        for (int k = 0; k < 4; k++) {
            int ii = i + NXk[k], jj = j + NYk[k];
            if (in_dom(g, ii, jj)) s -= face_w8(g, i, j, k, 1);
            else if (g->e[TAG(g, i, j, k)].btype != OG_NEUMANN) s -= 2.0 * face_w8(g, i, j, k, 0);
        }
        d[c] = 1.0 - alpha * s;
    }
}

/* ---------------------------------------------------------------------- */
/* GPU-path sweeps restated (rectangle, Dirichlet-type faces): Poisson
 *   (L phi)_c = cW phi_W + cE phi_E + cS phi_S + cN phi_N + d phi_c,
 *   cX = 2/(h (h + h_nb)) if the neighbour exists else 0, d = -(cW+cE+cS+cN).
 * This is ConstructLHS's matrix for wall/inlet faces, whose phi ghost = phi_c
 * makes each boundary face contribute 0 (FluidSolver.cpp:124-131,159-163). */

static int rect_dirichlet(const og_grid* g) {
    if (g->N != g->nx * g->ny) return 0;
    for (int k = 0; k < g->ne; k++) if (g->e[k].btype == OG_NEUMANN) return 0;
    return 1;
}

static inline void pcoef(const og_grid* g, int i, int j, double* cw, double* ce, double* cs, double* cn) {
    const double *hx = g->hx, *hy = g->hy;
    *cw = i > 0 ? 2.0 / (hx[i] * (hx[i] + hx[i - 1])) : 0.0;
    *ce = i < g->nx - 1 ? 2.0 / (hx[i] * (hx[i] + hx[i + 1])) : 0.0;
    *cs = j > 0 ? 2.0 / (hy[j] * (hy[j] + hy[j - 1])) : 0.0;
    *cn = j < g->ny - 1 ? 2.0 / (hy[j] * (hy[j] + hy[j + 1])) : 0.0;
}

static inline double lap_rect(const og_grid* g, const double* p, int i, int j) {
    int ny = g->ny;
    double cw, ce, cs, cn;
    pcoef(g, i, j, &cw, &ce, &cs, &cn);
    double c0 = p[i * ny + j];
    double s = -(cw + ce + cs + cn) * c0;
    if (i > 0) s += cw * p[(i - 1) * ny + j];
    if (i < g->nx - 1) s += ce * p[(i + 1) * ny + j];
    if (j > 0) s += cs * p[i * ny + j - 1];
    if (j < ny - 1) s += cn * p[i * ny + j + 1];
    return s;
}

double og_poisson_jacobi_sweep(const og_grid* g, const double* in, double* out, const double* b,
                               double shift, double omega) {
    if (!rect_dirichlet(g)) { set_err("sweeps need a rectangle with Dirichlet-type faces"); return -1; }
    double r2 = 0.0;
    for (int i = 0; i < g->nx; i++)
        for (int j = 0; j < g->ny; j++) {
            double cw, ce, cs, cn;
            pcoef(g, i, j, &cw, &ce, &cs, &cn);
            double d = -(cw + ce + cs + cn);
            int c = i * g->ny + j;
            double r = (b[c] - shift) - lap_rect(g, in, i, j);
            r2 += r * r;
            out[c] = in[c] + omega * r / d;
        }
    return r2;
}

double og_poisson_rbsor_sweep(const og_grid* g, double* p, const double* b, double shift, double omega) {
    if (!rect_dirichlet(g)) { set_err("sweeps need a rectangle with Dirichlet-type faces"); return -1; }
    double r2 = 0.0;
    for (int i = 0; i < g->nx; i++)
        for (int j = 0; j < g->ny; j++) {
            double r = (b[i * g->ny + j] - shift) - lap_rect(g, p, i, j);
            r2 += r * r;
        }
    for (int color = 0; color < 2; color++)
        for (int i = 0; i < g->nx; i++)
            for (int j = (i + color) & 1; j < g->ny; j += 2) {
                double cw, ce, cs, cn;
                pcoef(g, i, j, &cw, &ce, &cs, &cn);
                double d = -(cw + ce + cs + cn);
                int c = i * g->ny + j;
                double r = (b[c] - shift) - lap_rect(g, p, i, j);
                p[c] += omega * r / d;
            }
    return r2;
}

/* Helmholtz (I - a L_V): Dirichlet boundary faces add 2/h^2 to -L_V's diagonal */
static inline double helm_rect(const og_grid* g, double a, const double* q, int i, int j, double* diag) {
    const double *hx = g->hx, *hy = g->hy;
    int ny = g->ny;
    double cw, ce, cs, cn;
    pcoef(g, i, j, &cw, &ce, &cs, &cn);
    double bx = (i == 0 ? 2.0 / (hx[i] * hx[i]) : 0.0) + (i == g->nx - 1 ? 2.0 / (hx[i] * hx[i]) : 0.0);
    double by = (j == 0 ? 2.0 / (hy[j] * hy[j]) : 0.0) + (j == ny - 1 ? 2.0 / (hy[j] * hy[j]) : 0.0);
    double d = 1.0 + a * (cw + ce + cs + cn + bx + by);
    *diag = d;
    double s = d * q[i * ny + j];
    if (i > 0) s -= a * cw * q[(i - 1) * ny + j];
    if (i < g->nx - 1) s -= a * ce * q[(i + 1) * ny + j];
    if (j > 0) s -= a * cs * q[i * ny + j - 1];
    if (j < ny - 1) s -= a * cn * q[i * ny + j + 1];
    return s;
}

/* the GPU path's wall-band relaxation (k_helm_band, ns_kernels.hip): `sweeps` red-black SOR
 * sweeps of u and v restricted to the cells within `w` of a wall, every other cell held (the
 * residual of the guess u^n lies in the walls' boundary layers) */
static void helm_band_sweeps(const og_grid* g, double a, double* u, double* v, const double* ru, const double* rv,
                             double omega, int w, int sweeps) {
    const int nx = g->nx, ny = g->ny;
    for (int k = 0; k < sweeps; k++)
        for (int color = 0; color < 2; color++)
#pragma omp parallel for schedule(static) num_threads(og_nt)
            for (int i = 0; i < nx; i++) {
                const int side = i < w || i >= nx - w;
                for (int j = (i + color) & 1; j < ny; j += 2) {
                    if (!side && j >= w && j < ny - w) continue;
                    double d;
                    int c = i * ny + j;
                    double r1 = ru[c] - helm_rect(g, a, u, i, j, &d);
                    u[c] += omega * r1 / d;
                    double r2v = rv[c] - helm_rect(g, a, v, i, j, &d);
                    v[c] += omega * r2v / d;
                }
            }
}

int og_helm_band(const og_grid* g, double a, double* u, double* v, const double* ru, const double* rv, double omega,
                 int w, int sweeps) {
    if (!rect_dirichlet(g)) { set_err("band sweeps need a rectangle with Dirichlet-type faces"); return -1; }
    helm_band_sweeps(g, a, u, v, ru, rv, omega, w, sweeps);
    return 0;
}

/* ||ru - (I - a L_V) u||^2 and the same for v (rectangle), in one pass */
static void helm_resid2(const og_grid* g, double a, const double* u, const double* v, const double* ru,
                        const double* rv, double* ru2, double* rv2) {
    double su = 0.0, sv = 0.0;
#pragma omp parallel for schedule(static) reduction(+ : su, sv) num_threads(og_nt)
    for (int i = 0; i < g->nx; i++)
        for (int j = 0; j < g->ny; j++) {
            double d;
            int c = i * g->ny + j;
            double r1 = ru[c] - helm_rect(g, a, u, i, j, &d);
            double r2v = rv[c] - helm_rect(g, a, v, i, j, &d);
            su += r1 * r1;
            sv += r2v * r2v;
        }
    *ru2 = su;
    *rv2 = sv;
}

/* the two colour passes of one red-black SOR sweep of u and v */
static void helm_rbsor_colours(const og_grid* g, double a, double* u, double* v, const double* ru,
                               const double* rv, double omega) {
    for (int color = 0; color < 2; color++)
#pragma omp parallel for schedule(static) num_threads(og_nt)
        for (int i = 0; i < g->nx; i++)
            for (int j = (i + color) & 1; j < g->ny; j += 2) {
                double d;
                int c = i * g->ny + j;
                double r1 = ru[c] - helm_rect(g, a, u, i, j, &d);
                u[c] += omega * r1 / d;
                double r2v = rv[c] - helm_rect(g, a, v, i, j, &d);
                v[c] += omega * r2v / d;
            }
}

double og_helmholtz_rbsor_sweep(const og_grid* g, double a, double* u, double* v, const double* ru,
                                const double* rv, double omega) {
    if (!rect_dirichlet(g)) { set_err("sweeps need a rectangle with Dirichlet-type faces"); return -1; }
    double r2 = 0.0;
#pragma omp parallel for schedule(static) reduction(+ : r2) num_threads(og_nt)
    for (int i = 0; i < g->nx; i++)
        for (int j = 0; j < g->ny; j++) {
            double d;
            int c = i * g->ny + j;
            double r1 = ru[c] - helm_rect(g, a, u, i, j, &d);
            double r2v = rv[c] - helm_rect(g, a, v, i, j, &d);
            r2 += r1 * r1 + r2v * r2v;
        }
    for (int color = 0; color < 2; color++)
#pragma omp parallel for schedule(static) num_threads(og_nt)
        for (int i = 0; i < g->nx; i++)
            for (int j = (i + color) & 1; j < g->ny; j += 2) {
                double d;
                int c = i * g->ny + j;
                double r1 = ru[c] - helm_rect(g, a, u, i, j, &d);
                u[c] += omega * r1 / d;
                double r2v = rv[c] - helm_rect(g, a, v, i, j, &d);
                v[c] += omega * r2v / d;
            }
    return r2;
}

/* ---------------------------------------------------------------------- */
/* Krylov solves (the oracle's stand-in for PETSc's KSPs; converged tight)  */

typedef void (*op_fn)(const og_grid*, double, const double*, double*);

static double dot(int n, const double* a, const double* b) {
    double s = 0.0;
    for (int k = 0; k < n; k++) s += a[k] * b[k];
    return s;
}

static void op_helm(const og_grid* g, double a, const double* x, double* y) { og_apply_helmholtz(g, a, x, y); }
static void op_pois(const og_grid* g, double a, const double* x, double* y) { (void)a; og_apply_poisson(g, x, y); }

/* PCG on the area-scaled symmetric system  S A x = S b  (S = diag(hx_i hy_j)),
 * symmetric for Helmholtz always and for Poisson without Neumann faces.
 * proj: remove the (scaled) null space component -- constants. */
static int pcg(const og_grid* g, op_fn A, double a, const double* b, double* x, const double* dg,
               double sgn, int proj, double rtol, int maxit) {
    int n = g->N;
    double *r = malloc(sizeof(double) * n), *z = malloc(sizeof(double) * n);
    double *p = malloc(sizeof(double) * n), *q = malloc(sizeof(double) * n), *S = malloc(sizeof(double) * n);
    for (int c = 0; c < n; c++) S[c] = sgn * g->hx[g->ci[c]] * g->hy[g->cj[c]];
    /* r = S(b - A x) */
    A(g, a, x, q);
    double bn = 0.0;
    for (int c = 0; c < n; c++) { r[c] = S[c] * (b[c] - q[c]); bn += (S[c] * b[c]) * (S[c] * b[c]); }
    if (proj) {
        double m = 0.0, mb = 0.0;
        for (int c = 0; c < n; c++) { m += r[c]; mb += S[c] * b[c]; }
        m /= n; mb /= n;
        for (int c = 0; c < n; c++) r[c] -= m;
        bn = 0.0;
        for (int c = 0; c < n; c++) bn += (S[c] * b[c] - mb) * (S[c] * b[c] - mb);
    }
    bn = sqrt(bn);
    int it = 0;
    if (bn == 0.0) { free(r); free(z); free(p); free(q); free(S); return 0; }
    for (int c = 0; c < n; c++) z[c] = r[c] / (S[c] * dg[c]);
    memcpy(p, z, sizeof(double) * n);
    double rz = dot(n, r, z);
    while (it < maxit) {
        if (sqrt(dot(n, r, r)) <= rtol * bn) break;
        A(g, a, p, q);
        for (int c = 0; c < n; c++) q[c] *= S[c];
        double al = rz / dot(n, p, q);
        for (int c = 0; c < n; c++) { x[c] += al * p[c]; r[c] -= al * q[c]; }
        for (int c = 0; c < n; c++) z[c] = r[c] / (S[c] * dg[c]);
        double rz2 = dot(n, r, z);
        double be = rz2 / rz;
        rz = rz2;
        for (int c = 0; c < n; c++) p[c] = z[c] + be * p[c];
        it++;
    }
    free(r); free(z); free(p); free(q); free(S);
    return it;
}

/* One row of the assembled Poisson matrix LHS_phi (ConstructLHS FluidSolver.cpp:105-131 with
 * AddGhostStencils :147-163): (col, val) pairs, at most 1 + 4 * 3. */
static int poisson_row(const og_grid* g, int c, int* col, double* val) {
    int i = g->ci[c], j = g->cj[c], m = 0;
    double dg = 0.0;
    for (int k = 0; k < 4; k++) {
        int ii = i + NXk[k], jj = j + NYk[k];
        if (in_dom(g, ii, jj)) {
            double w = face_w8(g, i, j, k, 1);
            col[m] = CID(g, ii, jj); val[m++] = w; dg -= w;
        } else {
            double w = face_w8(g, i, j, k, 0);
            const og_edge* E = &g->e[TAG(g, i, j, k)];
            if (E->btype == OG_NEUMANN) {   /* ghost 2.5 p_c - 2 p_1 + 0.5 p_2 (:98-101) */
                dg += 2.5 * w;
                col[m] = CID(g, i - E->nx, j - E->ny); val[m++] = -2.0 * w;
                col[m] = CID(g, i - 2 * E->nx, j - 2 * E->ny); val[m++] = 0.5 * w;
            } else dg += w;                 /* ghost p_c */
            dg -= w;
        }
    }
    col[m] = c; val[m++] = dg;
    return m;
}

/* NEUMANN outflow sides make LHS_phi non-symmetric and not diagonally dominant; Krylov
 * iterations with a Jacobi preconditioner stall or diverge on it, so the oracle solves it
 * DIRECTLY: P A x = P b (P = mean projection, the null-space handling of :142-144, 550) is
 * A x = P b + c 1 for a scalar c.  With row z of A replaced by e_z (x_z = 0; the constant
 * null space pinned) the banded matrix Abar is regular, x = x1 + c x2 for Abar x1 = (P b)',
 * Abar x2 = 1' (row z zeroed), and c follows from the dropped row z.  z must carry a nonzero
 * entry of A's LEFT null vector, which with an outflow side lives next to the outflow (in 1-D
 * it is (.., 0, -1/2, 1) on the last two cells): z = the first cell with a NEUMANN face.
 * Banded Gaussian elimination with partial pivoting; returns 1 (one "iteration"), -1 if
 * singular. */
static int neu_direct(const og_grid* g, const double* b, double* x) {
    const int n = g->N;
    int col[16], kl = 0;
    double val[16];
    for (int c = 0; c < n; c++) {
        int m = poisson_row(g, c, col, val);
        for (int q = 0; q < m; q++) kl = abs(col[q] - c) > kl ? abs(col[q] - c) : kl;
    }
    int z = 0;
    for (int c = n - 1; c >= 0; c--)
        for (int k = 0; k < 4; k++) {
            int e = in_dom(g, g->ci[c] + NXk[k], g->cj[c] + NYk[k]) ? -1 : TAG(g, g->ci[c], g->cj[c], k);
            if (e >= 0 && g->e[e].btype == OG_NEUMANN) z = c;
        }
    const int ku = kl, W = 2 * kl + ku + 1;
    double* ab = calloc((size_t)n * W, sizeof(double));
    double *f1 = malloc(sizeof(double) * n), *f2 = malloc(sizeof(double) * n);
#define AB(r, cc) ab[(size_t)(r) * W + ((cc) - (r) + kl)]
    for (int c = 0; c < n; c++) {
        if (c == z) { AB(z, z) = 1.0; f1[z] = 0.0; f2[z] = 0.0; continue; }
        int m = poisson_row(g, c, col, val);
        for (int q = 0; q < m; q++) AB(c, col[q]) += val[q];
        f1[c] = b[c]; f2[c] = 1.0;
    }
    int rc = 1;
    for (int k = 0; k < n && rc > 0; k++) {
        int last = k + kl < n - 1 ? k + kl : n - 1, hi = k + kl + ku < n - 1 ? k + kl + ku : n - 1, p = k;
        for (int r = k + 1; r <= last; r++) if (fabs(AB(r, k)) > fabs(AB(p, k))) p = r;
        if (AB(p, k) == 0.0) { rc = -1; break; }
        if (p != k) {
            for (int cc = k; cc <= hi; cc++) { double t = AB(k, cc); AB(k, cc) = AB(p, cc); AB(p, cc) = t; }
            double t = f1[k]; f1[k] = f1[p]; f1[p] = t;
            t = f2[k]; f2[k] = f2[p]; f2[p] = t;
        }
        for (int r = k + 1; r <= last; r++) {
            double fct = AB(r, k) / AB(k, k);
            if (fct == 0.0) continue;
            AB(r, k) = 0.0;
            for (int cc = k + 1; cc <= hi; cc++) AB(r, cc) -= fct * AB(k, cc);
            f1[r] -= fct * f1[k];
            f2[r] -= fct * f2[k];
        }
    }
    if (rc > 0) {
        for (int k = n - 1; k >= 0; k--) {
            int hi = k + kl + ku < n - 1 ? k + kl + ku : n - 1;
            double s1 = f1[k], s2 = f2[k];
            for (int cc = k + 1; cc <= hi; cc++) { s1 -= AB(k, cc) * f1[cc]; s2 -= AB(k, cc) * f2[cc]; }
            f1[k] = s1 / AB(k, k);
            f2[k] = s2 / AB(k, k);
        }
        /* the dropped row z: a_z . (x1 + c x2) - c = (P b)_z */
        int m = poisson_row(g, z, col, val);
        double a1 = 0.0, a2 = 0.0;
        for (int q = 0; q < m; q++) { a1 += val[q] * f1[col[q]]; a2 += val[q] * f2[col[q]]; }
        double cc = (b[z] - a1) / (a2 - 1.0);
        for (int c = 0; c < n; c++) x[c] = f1[c] + cc * f2[c];
    }
#undef AB
    free(ab); free(f1); free(f2);
    return rc;
}

int og_solve_helmholtz(const og_grid* g, double alpha, const double* rhs, double* x, double rtol, int maxit) {
    double* d = malloc(sizeof(double) * g->N);
    diag_helmholtz(g, alpha, d);
    int it = pcg(g, op_helm, alpha, rhs, x, d, 1.0, 0, rtol, maxit);
    free(d);
    return it;
}

int og_solve_poisson(const og_grid* g, double* rhs, double* x, double rtol, int maxit) {
    int n = g->N;
    /* MatNullSpaceRemove(NSP, RHS_phi) FluidSolver.cpp:550: subtract the plain mean */
    double m = 0.0;
    for (int c = 0; c < n; c++) m += rhs[c];
    m /= n;
    for (int c = 0; c < n; c++) rhs[c] -= m;
    double* d = malloc(sizeof(double) * n);
    diag_poisson(g, d);
    int neu = 0;
    for (int k = 0; k < g->ne; k++) neu |= g->e[k].btype == OG_NEUMANN;
    int it = neu ? neu_direct(g, rhs, x) : pcg(g, op_pois, 0.0, rhs, x, d, -1.0, 1, rtol, maxit);
    free(d);
    return it;
}

/* ---------------------------------------------------------------------- */
/* geometric multigrid (rectangle, Dirichlet-type faces)                   */

static void coef1(int n, const double* h, double* cm, double* cp) {
    for (int i = 0; i < n; i++) {
        cm[i] = i > 0 ? 2.0 / (h[i] * (h[i] + h[i - 1])) : 0.0;
        cp[i] = i < n - 1 ? 2.0 / (h[i] * (h[i] + h[i + 1])) : 0.0;
    }
}

typedef struct {
    int nx, ny;
    double *hx, *hy, *cw, *ce, *cs, *cn, *x, *b;
} mg_level;

static double lap_at(const mg_level* L, const double* p, int i, int j) {
    const int ny = L->ny;
    const double q = p[i * ny + j];
    const double s = L->cw[i] * p[(i > 0 ? i - 1 : i) * ny + j] + L->ce[i] * p[(i < L->nx - 1 ? i + 1 : i) * ny + j] +
                     L->cs[j] * p[i * ny + (j > 0 ? j - 1 : j)] + L->cn[j] * p[i * ny + (j < ny - 1 ? j + 1 : j)];
    const double dg = -((L->cw[i] + L->ce[i]) + (L->cs[j] + L->cn[j]));
    return s + dg * q;
}

/* The GPU path's last-level solve when that level has <= 64 cells (k_coarse_vcycle, CV_DIRECT):
 * x = M b with M the n x n block of the inverse of the bordered system [A 1; w^T 0] (w = cell
 * areas), i.e. A x = b - (w.b / w.1) 1 with w.x = 0.  Returns M (malloc'd) or NULL. */
static double* mg_direct_matrix(const mg_level* L) {
    const int n = L->nx * L->ny, m = n + 1;
    double* a = calloc((size_t)m * m, sizeof(double));
    double* inv = calloc((size_t)m * m, sizeof(double));
    for (int i = 0; i < L->nx; i++)
        for (int j = 0; j < L->ny; j++) {
            const int r = i * L->ny + j;
            a[(size_t)r * m + r] = -((L->cw[i] + L->ce[i]) + (L->cs[j] + L->cn[j]));
            if (i > 0) a[(size_t)r * m + r - L->ny] += L->cw[i];
            if (i < L->nx - 1) a[(size_t)r * m + r + L->ny] += L->ce[i];
            if (j > 0) a[(size_t)r * m + r - 1] += L->cs[j];
            if (j < L->ny - 1) a[(size_t)r * m + r + 1] += L->cn[j];
            a[(size_t)r * m + n] = 1.0;
            a[(size_t)n * m + r] = L->hx[i] * L->hy[j];
        }
    for (int k = 0; k < m; k++) inv[(size_t)k * m + k] = 1.0;
    /* Gauss-Jordan, partial pivoting */
    for (int c = 0; c < m; c++) {
        int p = c;
        for (int r = c + 1; r < m; r++)
            if (fabs(a[(size_t)r * m + c]) > fabs(a[(size_t)p * m + c])) p = r;
        if (a[(size_t)p * m + c] == 0.0) { free(a); free(inv); return NULL; }
        if (p != c)
            for (int k = 0; k < m; k++) {
                double t = a[(size_t)p * m + k]; a[(size_t)p * m + k] = a[(size_t)c * m + k]; a[(size_t)c * m + k] = t;
                t = inv[(size_t)p * m + k]; inv[(size_t)p * m + k] = inv[(size_t)c * m + k]; inv[(size_t)c * m + k] = t;
            }
        const double d = 1.0 / a[(size_t)c * m + c];
        for (int k = 0; k < m; k++) { a[(size_t)c * m + k] *= d; inv[(size_t)c * m + k] *= d; }
        for (int r = 0; r < m; r++) {
            if (r == c) continue;
            const double f = a[(size_t)r * m + c];
            if (f == 0.0) continue;
            for (int k = 0; k < m; k++) {
                a[(size_t)r * m + k] -= f * a[(size_t)c * m + k];
                inv[(size_t)r * m + k] -= f * inv[(size_t)c * m + k];
            }
        }
    }
    double* M = malloc(sizeof(double) * (size_t)n * n);
    for (int r = 0; r < n; r++)
        for (int k = 0; k < n; k++) M[(size_t)r * n + k] = inv[(size_t)r * m + k];
    free(a); free(inv);
    return M;
}

/* The GPU path's exact solve of its coarsest level (r4, ns_solver.cpp direct_setup / k_direct):
 * the level's first coarse level of <= og_direct_cells cells (sides <= 128; 0 = off) is the
 * last one, and L x = b is solved through the eigen-decompositions of the separable 1-D
 * operators: L1 = tridiag(w_i, -(w_i + e_i), e_i) with H L1 symmetric, S = H^1/2 L1 H^-1/2 =
 * U diag(lam) U^T (cyclic Jacobi rotations), C = Vx^-1 b Vy^-T, Y = C / (lx_k + ly_m) with the
 * null mode (both sides singular) set to 0, x = Vx Y Vy^T -- i.e. w.x = 0 (w the cell areas), as
 * mg_direct_matrix's bordered system. */
static long og_direct_cells = 128L * 128L;
void og_mg_set_direct(long cells) { og_direct_cells = cells < 0 ? 0 : cells; }
static int mg_direct_fits(int nx, int ny) {
    return og_direct_cells > 0 && (long)nx * ny <= og_direct_cells && nx <= 128 && ny <= 128;
}

static void eig_jacobi(int n, double* a, double* lam, double* v) {
    for (int i = 0; i < n * n; i++) v[i] = 0.0;
    for (int i = 0; i < n; i++) v[i * n + i] = 1.0;
    for (int sweep = 0; sweep < 100; sweep++) {
        double off = 0.0, dg = 0.0;
        for (int p = 0; p < n; p++) {
            dg += a[p * n + p] * a[p * n + p];
            for (int q = p + 1; q < n; q++) off += a[p * n + q] * a[p * n + q];
        }
        if (off <= 1e-34 * dg) break;
        for (int p = 0; p < n; p++)
            for (int q = p + 1; q < n; q++) {
                const double apq = a[p * n + q];
                if (apq == 0.0) continue;
                const double tau = (a[q * n + q] - a[p * n + p]) / (2.0 * apq);
                const double t = (tau >= 0.0 ? 1.0 : -1.0) / (fabs(tau) + sqrt(1.0 + tau * tau));
                const double c = 1.0 / sqrt(1.0 + t * t), sn = t * c;
                for (int k = 0; k < n; k++) {
                    const double x = a[k * n + p], y = a[k * n + q];
                    a[k * n + p] = c * x - sn * y; a[k * n + q] = sn * x + c * y;
                }
                for (int k = 0; k < n; k++) {
                    const double x = a[p * n + k], y = a[q * n + k];
                    a[p * n + k] = c * x - sn * y; a[q * n + k] = sn * x + c * y;
                }
                for (int k = 0; k < n; k++) {
                    const double x = v[k * n + p], y = v[k * n + q];
                    v[k * n + p] = c * x - sn * y; v[k * n + q] = sn * x + c * y;
                }
            }
    }
    for (int i = 0; i < n; i++) lam[i] = a[i * n + i];
}

/* one side: V (n x n, column k = eigenvector k scaled by H^-1/2), Vi = V^-1, lam; returns the
 * index of the null mode (walls at both ends) or -1 */
static int mg_direct_side(int n, const double* h, const double* w, const double* e, double* V, double* Vi,
                          double* lam) {
    double* S = calloc((size_t)n * n, sizeof(double));
    double* U = malloc(sizeof(double) * (size_t)n * n);
    for (int i = 0; i < n; i++) {
        S[i * n + i] = -(w[i] + e[i]);
        if (i + 1 < n) S[i * n + i + 1] = S[(i + 1) * n + i] = 2.0 / (sqrt(h[i] * h[i + 1]) * (h[i] + h[i + 1]));
    }
    eig_jacobi(n, S, lam, U);
    for (int i = 0; i < n; i++)
        for (int k = 0; k < n; k++) {
            V[i * n + k] = U[i * n + k] / sqrt(h[i]);
            Vi[k * n + i] = U[i * n + k] * sqrt(h[i]);
        }
    free(S); free(U);
    if (w[0] != 0.0 || e[n - 1] != 0.0) return -1;
    int k0 = 0;
    for (int k = 1; k < n; k++)
        if (fabs(lam[k]) < fabs(lam[k0])) k0 = k;
    lam[k0] = 0.0;
    return k0;
}

typedef struct {
    int nx, ny;
    double *Vx, *Vxi, *Vy, *Vyi, *D, *T;
} mg_direct;

static mg_direct* mg_direct_new(int nx, int ny, const double* hx, const double* hy, const double* cw,
                                const double* ce, const double* cs, const double* cn) {
    mg_direct* d = calloc(1, sizeof *d);
    d->nx = nx; d->ny = ny;
    d->Vx = malloc(sizeof(double) * nx * nx); d->Vxi = malloc(sizeof(double) * nx * nx);
    d->Vy = malloc(sizeof(double) * ny * ny); d->Vyi = malloc(sizeof(double) * ny * ny);
    d->D = malloc(sizeof(double) * nx * ny); d->T = malloc(sizeof(double) * nx * ny);
    double* lx = malloc(sizeof(double) * nx);
    double* ly = malloc(sizeof(double) * ny);
    const int kx0 = mg_direct_side(nx, hx, cw, ce, d->Vx, d->Vxi, lx);
    const int ky0 = mg_direct_side(ny, hy, cs, cn, d->Vy, d->Vyi, ly);
    for (int k = 0; k < nx; k++)
        for (int m = 0; m < ny; m++) {
            const double s = lx[k] + ly[m];
            d->D[k * ny + m] = (k == kx0 && m == ky0) || s == 0.0 ? 0.0 : 1.0 / s;
        }
    free(lx); free(ly);
    return d;
}

static void mg_direct_free(mg_direct* d) {
    if (!d) return;
    free(d->Vx); free(d->Vxi); free(d->Vy); free(d->Vyi); free(d->D); free(d->T); free(d);
}

/* x = L^-1 b (w.x = 0 when L is singular) */
static void mg_direct_solve(const mg_direct* d, const double* b, double* x) {
    const int nx = d->nx, ny = d->ny;
    double* T = d->T;
    /* T = Vx^-1 b, then Y = D o (T Vy^-T) into x */
    for (int k = 0; k < nx; k++)
        for (int j = 0; j < ny; j++) {
            double acc = 0.0;
            for (int i = 0; i < nx; i++) acc += d->Vxi[k * nx + i] * b[i * ny + j];
            T[k * ny + j] = acc;
        }
    for (int k = 0; k < nx; k++)
        for (int m = 0; m < ny; m++) {
            double acc = 0.0;
            for (int j = 0; j < ny; j++) acc += T[k * ny + j] * d->Vyi[m * ny + j];   /* Vy^-T[j][m] = Vyi[m][j] */
            x[k * ny + m] = acc * d->D[k * ny + m];
        }
    /* x = Vx Y Vy^T */
    for (int i = 0; i < nx; i++)
        for (int m = 0; m < ny; m++) {
            double acc = 0.0;
            for (int k = 0; k < nx; k++) acc += d->Vx[i * nx + k] * x[k * ny + m];
            T[i * ny + m] = acc;
        }
    for (int i = 0; i < nx; i++)
        for (int j = 0; j < ny; j++) {
            double acc = 0.0;
            for (int m = 0; m < ny; m++) acc += T[i * ny + m] * d->Vy[j * ny + m];   /* Vy^T[m][j] = Vy[j][m] */
            x[i * ny + j] = acc;
        }
}

/* one red-black sweep in place (red = (i+j) even first) */
static void mg_rb(const mg_level* L, double* p, const double* b, double shift, double omega) {
    const int nt = (size_t)L->nx * L->ny >= 65536 ? og_nt : 1;
    for (int color = 0; color < 2; color++)
#pragma omp parallel for schedule(static) num_threads(nt)
        for (int i = 0; i < L->nx; i++)
            for (int j = (i + color) & 1; j < L->ny; j += 2) {
                const double dg = -((L->cw[i] + L->ce[i]) + (L->cs[j] + L->cn[j]));
                const double r = (b[i * L->ny + j] - shift) - lap_at(L, p, i, j);
                p[i * L->ny + j] += omega * r / dg;
            }
}

static double mg_restrict_lv(const mg_level* F, const double* phi, const double* b, double shift, const mg_level* C,
                             double* bc) {
    double r2 = 0.0;
    const int nt = (size_t)F->nx * F->ny >= 65536 ? og_nt : 1;
#pragma omp parallel for schedule(static) reduction(+ : r2) num_threads(nt)
    for (int I = 0; I < C->nx; I++)
        for (int J = 0; J < C->ny; J++) {
            double sum = 0.0;
            for (int a = 0; a < 2; a++)
                for (int q = 0; q < 2; q++) {
                    const int i = 2 * I + a, j = 2 * J + q;
                    const double r = (b[i * F->ny + j] - shift) - lap_at(F, phi, i, j);
                    sum += (F->hx[i] * F->hy[j]) * r;
                    r2 += r * r;
                }
            bc[I * C->ny + J] = sum / (C->hx[I] * C->hy[J]);
        }
    return r2;
}

void og_mg_prolong(int nx, int ny, const double* ec, double* phi) {
    const int cnx = nx / 2, cny = ny / 2;
    const int nt = (size_t)nx * ny >= 65536 ? og_nt : 1;
#pragma omp parallel for schedule(static) num_threads(nt)
    for (int i = 0; i < nx; i++)
        for (int j = 0; j < ny; j++) {
            const int I = i >> 1, J = j >> 1;
            int In = (i & 1) ? I + 1 : I - 1, Jn = (j & 1) ? J + 1 : J - 1;
            if (In < 0 || In >= cnx) In = I;   /* wall: reflect onto the parent */
            if (Jn < 0 || Jn >= cny) Jn = J;
            phi[i * ny + j] += (9.0 * ec[I * cny + J] + 3.0 * ec[In * cny + J] + 3.0 * ec[I * cny + Jn] +
                                ec[In * cny + Jn]) * 0.0625;
        }
}

static mg_level* mg_build(int nx, int ny, const double* hx, const double* hy, int* nlev) {
    int cap = 32, n = 0;
    mg_level* L = calloc(cap, sizeof(mg_level));
    for (;;) {
        mg_level* l = &L[n];
        l->nx = nx; l->ny = ny;
        l->hx = malloc(sizeof(double) * nx); l->hy = malloc(sizeof(double) * ny);
        if (n == 0) { memcpy(l->hx, hx, sizeof(double) * nx); memcpy(l->hy, hy, sizeof(double) * ny); }
        else {
            for (int i = 0; i < nx; i++) l->hx[i] = L[n - 1].hx[2 * i] + L[n - 1].hx[2 * i + 1];
            for (int j = 0; j < ny; j++) l->hy[j] = L[n - 1].hy[2 * j] + L[n - 1].hy[2 * j + 1];
        }
        l->cw = malloc(sizeof(double) * nx); l->ce = malloc(sizeof(double) * nx);
        l->cs = malloc(sizeof(double) * ny); l->cn = malloc(sizeof(double) * ny);
        coef1(nx, l->hx, l->cw, l->ce);
        coef1(ny, l->hy, l->cs, l->cn);
        l->x = calloc((size_t)nx * ny, sizeof(double));
        l->b = calloc((size_t)nx * ny, sizeof(double));
        n++;
        /* same rule as the GPU hierarchy (global levels + the LDS V-cycle, mg_can_coarsen in
         * ns_internal.h): halve while both sizes are even, >= 4, and the level has > 16 cells;
         * (r4) stop at the first coarse level the exact direct solve takes */
        if (nx % 2 || ny % 2 || nx < 4 || ny < 4 || nx * ny <= 16 || n == cap) break;
        if (n >= 2 && mg_direct_fits(nx, ny)) break;
        nx /= 2; ny /= 2;
    }
    *nlev = n;
    return L;
}

static void mg_free(mg_level* L, int n) {
    for (int k = 0; k < n; k++) {
        free(L[k].hx); free(L[k].hy); free(L[k].cw); free(L[k].ce); free(L[k].cs); free(L[k].cn);
        free(L[k].x); free(L[k].b);
    }
    free(L);
}

void og_mg_restrict(int nx, int ny, const double* hx, const double* hy, const double* phi, const double* b,
                    double shift, double* bc) {
    int n;
    mg_level* L = mg_build(nx, ny, hx, hy, &n);
    mg_level F = L[0];
    mg_level C = {0};
    C.nx = nx / 2; C.ny = ny / 2;
    C.hx = malloc(sizeof(double) * C.nx); C.hy = malloc(sizeof(double) * C.ny);
    for (int i = 0; i < C.nx; i++) C.hx[i] = hx[2 * i] + hx[2 * i + 1];
    for (int j = 0; j < C.ny; j++) C.hy[j] = hy[2 * j] + hy[2 * j + 1];
    mg_restrict_lv(&F, phi, b, shift, &C, bc);
    free(C.hx); free(C.hy);
    mg_free(L, n);
}

int og_mg_solve(const og_grid* g, double* rhs, double* x, double rtol, int pre, int post, int maxcycles) {
    return og_mg_solve_w(g, rhs, x, rtol, pre, post, maxcycles, 1.0);
}

int og_mg_solve_w(const og_grid* g, double* rhs, double* x, double rtol, int pre, int post, int maxcycles,
                  double omega) {
    if (!rect_dirichlet(g)) { set_err("multigrid needs a rectangle with Dirichlet-type faces"); return -1; }
    const int N = g->N;
    double m = 0.0, b2 = 0.0;
    for (int c = 0; c < N; c++) m += rhs[c];
    m /= N;
    for (int c = 0; c < N; c++) { rhs[c] -= m; b2 += rhs[c] * rhs[c]; }
    int nl;
    mg_level* L = mg_build(g->nx, g->ny, g->hx, g->hy, &nl);
    if (nl < 2) { mg_free(L, nl); set_err("grid cannot be coarsened"); return -1; }
    const mg_level* Lc = &L[nl - 1];
    const int nc = Lc->nx > Lc->ny ? Lc->nx : Lc->ny;
    const double omc = 2.0 / (1.0 + sin(3.14159265358979323846 / nc));
    const int itc = 2 * nc + 10;
    const int ncell = Lc->nx * Lc->ny;
    mg_direct* Dd = mg_direct_fits(Lc->nx, Lc->ny)
                        ? mg_direct_new(Lc->nx, Lc->ny, Lc->hx, Lc->hy, Lc->cw, Lc->ce, Lc->cs, Lc->cn) : NULL;
    double* Md = !Dd && ncell <= 64 ? mg_direct_matrix(Lc) : NULL;
    int cycles = 0;
    for (;;) {
        /* down */
        double* xf = x;
        const double* bf = rhs;
        int done = 0;
        for (int l = 0; l < nl - 1; l++) {
            for (int k = 0; k < pre; k++) mg_rb(&L[l], xf, bf, 0.0, omega);
            mg_restrict_lv(&L[l], xf, bf, 0.0, &L[l + 1], L[l + 1].b);
            memset(L[l + 1].x, 0, sizeof(double) * (size_t)L[l + 1].nx * L[l + 1].ny);
            xf = L[l + 1].x;
            bf = L[l + 1].b;
        }
        if (Dd) {
            mg_direct_solve(Dd, L[nl - 1].b, L[nl - 1].x);
        } else if (Md) {
            for (int r = 0; r < ncell; r++) {
                double x = 0.0;
                for (int k = 0; k < ncell; k++) x += Md[(size_t)r * ncell + k] * L[nl - 1].b[k];
                L[nl - 1].x[r] = x;
            }
        } else {
            for (int k = 0; k < itc; k++) mg_rb(Lc, L[nl - 1].x, L[nl - 1].b, 0.0, omc);
        }
        for (int l = nl - 2; l >= 0; l--) {
            double* xl = l == 0 ? x : L[l].x;
            const double* bl = l == 0 ? rhs : L[l].b;
            og_mg_prolong(L[l].nx, L[l].ny, L[l + 1].x, xl);
            for (int k = 0; k < post; k++) mg_rb(&L[l], xl, bl, 0.0, omega);
        }
        cycles++;
        /* the convergence test on the cycle's output residual (the GPU's fused prolongation
         * pass sums it; the restriction written here is overwritten by the next cycle's) */
        const double r2 = mg_restrict_lv(&L[0], x, rhs, 0.0, &L[1], L[1].b);
        if (r2 <= rtol * rtol * b2 || r2 == 0.0 || cycles >= maxcycles) done = 1;
        if (done) break;
    }
    free(Md);
    mg_direct_free(Dd);
    mg_free(L, nl);
    return cycles;
}

/* ---------------------------------------------------------------------- */
/* the GPU's direct Poisson solve restated (ns_fps.hip, r4).  On a rectangle with Dirichlet-type
 * (zero-flux phi) faces and uniform spacings, L = Lx (x) I + I (x) Ly; the DCT-II along y
 * (j, contiguous) diagonalises Ly (mu_k = -(4/hy^2) sin^2(pi k / 2ny)), leaving one tridiagonal
 * system (Lx + mu_k) x_k = f_k along x per mode, solved by Thomas' recurrences; mode 0 is
 * singular (Lx 1 = 0) and its last unknown is pinned to 0; then the DCT-III.  This restatement
 * runs the plain sequential recurrences and a textbook radix-2 FFT: it checks the GPU's chunked
 * scans and Stockham transforms, not their arithmetic order (agreement ~1e-13, not bitwise). */

/* (r6) hy uniform: Ly's eigenvectors are the DCT-II basis whatever hx (L = Lx (x) I + I (x) Ly with Lx's per-row
 * coefficients pcoef -- ConstructLHS, FluidSolver.cpp:113-131, on Grid.cpp:87-92's stretched faces) */
int og_fps_ok(const og_grid* g) {
    if (!rect_dirichlet(g)) return 0;
    for (int j = 1; j < g->ny; j++) if (g->hy[j] != g->hy[0]) return 0;
    /* (r6) any even ny in [16, 8192] with prime factors 2, 3, 5, 7 too -- the GPU's mixed-radix transforms
     * (ns_fps.hip fps_gen_ok); restated here with a plain O(N^2) DFT */
    int m = g->ny;
    if (m % 2 == 0 && m <= 8192)
        for (int q = 2; q <= 7; q++)
            while (m % q == 0) m /= q;
    const int gen = g->ny % 2 == 0 && g->ny <= 8192 && m == 1;
    return g->ny >= 16 && g->ny <= 16384 && ((g->ny & (g->ny - 1)) == 0 || gen) && g->nx >= 2;
}

/* in-place forward DFT of any n (the plain O(n^2) sum; cw / sw: cos / sin (2 pi m / n), m < n) */
static void dft_plain(int n, double* re, double* im, const double* cw, const double* sw) {
    double* xr = malloc(sizeof(double) * n);
    double* xi = malloc(sizeof(double) * n);
    for (int k = 0; k < n; k++) {
        double ar = 0.0, ai = 0.0;
        for (int j = 0; j < n; j++) {
            const int m = (int)(((long)j * k) % n);
            const double c = cw[m], s = -sw[m];   /* e^{-2 pi i j k / n} */
            ar += re[j] * c - im[j] * s;
            ai += re[j] * s + im[j] * c;
        }
        xr[k] = ar; xi[k] = ai;
    }
    for (int k = 0; k < n; k++) { re[k] = xr[k]; im[k] = xi[k]; }
    free(xr); free(xi);
}

/* in-place forward DFT of n = 2^p complex points (iterative radix-2, bit-reversed input order) */
static void fft_inplace(int n, double* re, double* im, const double* cw, const double* sw) {
    for (int i = 1, j = 0; i < n; i++) {
        int bit = n >> 1;
        for (; j & bit; bit >>= 1) j ^= bit;
        j ^= bit;
        if (i < j) {
            double t = re[i]; re[i] = re[j]; re[j] = t;
            t = im[i]; im[i] = im[j]; im[j] = t;
        }
    }
    for (int len = 2; len <= n; len <<= 1) {
        const int st = n / len;
        for (int i = 0; i < n; i += len)
            for (int k = 0; k < len / 2; k++) {
                const double c = cw[k * st], s = -sw[k * st];   /* e^{-2 pi i k / len} */
                const int a = i + k, b = a + len / 2;
                const double xr = re[b] * c - im[b] * s, xi = re[b] * s + im[b] * c;
                re[b] = re[a] - xr; im[b] = im[a] - xi;
                re[a] += xr; im[a] += xi;
            }
    }
}

int og_fps_solve(const og_grid* g, double* rhs, double* x) {
    if (!og_fps_ok(g)) { set_err("the direct solve needs a rectangle with zero-flux faces, uniform hy, ny = 2^p in [16, 16384]"); return -1; }
    const int nx = g->nx, N = g->ny;
    const size_t n = (size_t)nx * N;
    double m = 0.0;
    for (size_t c = 0; c < n; c++) m += rhs[c];
    m /= (double)n;
    for (size_t c = 0; c < n; c++) rhs[c] -= m;
    /* (r6) stretched along x: MatNullSpaceRemove's plain mean (FluidSolver.cpp:550) leaves sum A b != 0, the
     * system inconsistent; the area projection b_c -= (sum A b / N) / A_c (the Krylov solves' converged
     * solution, the GPU's k_area_fix) makes mode 0's singular system along x solvable */
    int xuni = 1;
    for (int i = 1; i < nx; i++) xuni &= g->hx[i] == g->hx[0];
    if (!xuni) {
        double sab = 0.0;
        for (int i = 0; i < nx; i++)
            for (int j = 0; j < N; j++) sab += g->hx[i] * g->hy[j] * rhs[(size_t)i * N + j];
        const double mm = sab / (double)n;
        for (int i = 0; i < nx; i++)
            for (int j = 0; j < N; j++) rhs[(size_t)i * N + j] -= mm / (g->hx[i] * g->hy[j]);
    }
    const double PI = 3.14159265358979323846;
    double* cw = malloc(sizeof(double) * N); double* sw = malloc(sizeof(double) * N);
    double* ck = malloc(sizeof(double) * N); double* sk = malloc(sizeof(double) * N);
    double* mu = malloc(sizeof(double) * N);
    double* re = malloc(sizeof(double) * N); double* im = malloc(sizeof(double) * N);
    double* F = malloc(sizeof(double) * n);
    for (int k = 0; k < N; k++) {
        cw[k] = cos(2.0 * PI * ((double)k / N)); sw[k] = sin(2.0 * PI * ((double)k / N));
        const double u = PI * ((double)k / (2.0 * N));
        ck[k] = cos(u); sk[k] = sin(u);
        mu[k] = -4.0 / (g->hy[0] * g->hy[0]) * sk[k] * sk[k];
    }
    /* DCT-II of each row (Makhoul: v_n = x_2n, v_{N-1-n} = x_{2n+1}; X_k = Re(e^{-i pi k/2N} V_k)) */
    for (int i = 0; i < nx; i++) {
        const double* r = rhs + (size_t)i * N;
        for (int j = 0; j < N; j++) {
            const int q = (j & 1) ? N - 1 - (j >> 1) : (j >> 1);
            re[q] = r[j]; im[q] = 0.0;
        }
        if (N & (N - 1)) dft_plain(N, re, im, cw, sw); else fft_inplace(N, re, im, cw, sw);
        for (int k = 0; k < N; k++) F[(size_t)i * N + k] = ck[k] * re[k] + sk[k] * im[k];
    }
    /* Thomas per mode along x: a_i = cw_i, c_i = ce_i, d_i = -(cw_i + ce_i) + mu_k */
    double* p = malloc(sizeof(double) * nx);
    double* y = malloc(sizeof(double) * nx);
    for (int k = 0; k < N; k++) {
        for (int i = 0; i < nx; i++) {
            double a, c, cs, cn;
            pcoef(g, i, 0, &a, &c, &cs, &cn);
            const double d = -(a + c) + mu[k];
            if (i == 0) { p[0] = d; y[0] = F[k]; continue; }
            double ap, cp, csp, cnp;
            pcoef(g, i - 1, 0, &ap, &cp, &csp, &cnp);
            const double gg = a / p[i - 1];
            p[i] = d - gg * cp;
            y[i] = F[(size_t)i * N + k] - gg * y[i - 1];
        }
        double xn = (k == 0) ? 0.0 : y[nx - 1] / p[nx - 1];
        F[(size_t)(nx - 1) * N + k] = xn;
        for (int i = nx - 2; i >= 0; i--) {
            double a, c, cs, cn;
            pcoef(g, i, 0, &a, &c, &cs, &cn);
            xn = (y[i] - c * xn) / p[i];
            F[(size_t)i * N + k] = xn;
        }
    }
    /* DCT-III: V_k = e^{i pi k/2N}(X_k - i X_{N-k}), v = IFFT(V) = conj(FFT(conj V)) / N */
    for (int i = 0; i < nx; i++) {
        const double* X = F + (size_t)i * N;
        for (int k = 0; k < N; k++) {
            const double a = X[k], b = k ? X[N - k] : 0.0;
            re[k] = ck[k] * a + sk[k] * b;
            im[k] = -(sk[k] * a - ck[k] * b);
        }
        if (N & (N - 1)) dft_plain(N, re, im, cw, sw); else fft_inplace(N, re, im, cw, sw);
        double* o = x + (size_t)i * N;
        for (int j = 0; j < N; j++) {
            const int q = (j & 1) ? N - 1 - (j >> 1) : (j >> 1);
            o[j] = re[q] / N;
        }
    }
    free(cw); free(sw); free(ck); free(sk); free(mu); free(re); free(im); free(F); free(p); free(y);
    return 1;
}

/* ---------------------------------------------------------------------- */
/* time stepper, FluidSolver::Solve FluidSolver.cpp:536-567                */

struct og_solver {
    og_grid* g;
    double dt, re, rtol;
    int gpu_alg;
    double omega_v, omega_mg;
    int band_w, band_sweeps;   /* GPU algorithm: the Helmholtz wall-band relaxation (0: none) */
    double *u, *v, *phi, *cu, *cv, *gx, *gy, *ru, *rv, *us, *vs, *rp;
};

og_solver* og_solver_new(og_grid* g, double dt, double re, double rtol) {
    og_solver* s = calloc(1, sizeof *s);
    s->g = g; s->dt = dt; s->re = re; s->rtol = rtol;
    int n = g->N;
    double** arr[] = {&s->u, &s->v, &s->phi, &s->cu, &s->cv, &s->gx, &s->gy, &s->ru, &s->rv, &s->us, &s->vs, &s->rp};
    for (unsigned k = 0; k < sizeof arr / sizeof arr[0]; k++) *arr[k] = calloc(n, sizeof(double));
    return s;
}

void og_solver_set_algorithm(og_solver* s, int gpu_algorithm, double omega_v, double omega_mg) {
    s->gpu_alg = gpu_algorithm;
    s->omega_v = omega_v;
    s->omega_mg = omega_mg;
}

void og_solver_set_band(og_solver* s, int width, int sweeps) {
    s->band_w = width;
    s->band_sweeps = sweeps;
}

void og_solver_free(og_solver* s) {
    if (!s) return;
    double* arr[] = {s->u, s->v, s->phi, s->cu, s->cv, s->gx, s->gy, s->ru, s->rv, s->us, s->vs, s->rp};
    for (unsigned k = 0; k < sizeof arr / sizeof arr[0]; k++) free(arr[k]);
    free(s);
}

int og_solver_step(og_solver* s, double* mm, int* its) {
    const og_grid* g = s->g;
    int n = g->N, maxit = 100000;
    double alpha = s->dt / (2 * s->re);
    og_rhs_velocity(g, s->dt, s->re, s->u, s->v, s->gx, s->gy, s->cu, s->cv, s->ru, s->rv);
    int iu, iv, ip;
    if (s->gpu_alg) {
        /* the GPU path's algorithm: RB-SOR Helmholtz from u^n, checked every sweep; MG Poisson */
        memcpy(s->us, s->u, sizeof(double) * n);
        memcpy(s->vs, s->v, sizeof(double) * n);
        if (s->band_w > 0)
            helm_band_sweeps(g, alpha, s->us, s->vs, s->ru, s->rv, s->omega_v, s->band_w, s->band_sweeps);
        double bu = dot(n, s->ru, s->ru), bv = dot(n, s->rv, s->rv);
        iu = 0;
        do {
            double ru2 = 0, rv2 = 0;
            helm_resid2(g, alpha, s->us, s->vs, s->ru, s->rv, &ru2, &rv2);
            if ((ru2 <= s->rtol * s->rtol * bu || ru2 == 0) && (rv2 <= s->rtol * s->rtol * bv || rv2 == 0)) break;
            helm_rbsor_colours(g, alpha, s->us, s->vs, s->ru, s->rv, s->omega_v);
            iu++;
        } while (iu < maxit);
        iv = iu;
        og_divergence(g, s->dt, s->us, s->vs, s->rp);
        ip = s->gpu_alg == 2 && og_fps_ok(g) ? og_fps_solve(g, s->rp, s->phi)
                                             : og_mg_solve_w(g, s->rp, s->phi, s->rtol, 2, 2, 1000, s->omega_mg);
    } else {
        /* KSPSolve(uSolver, ...) x2 with zero initial guess (:547-548) */
        memset(s->us, 0, sizeof(double) * n);
        memset(s->vs, 0, sizeof(double) * n);
        iu = og_solve_helmholtz(g, alpha, s->ru, s->us, s->rtol, maxit);
        iv = og_solve_helmholtz(g, alpha, s->rv, s->vs, s->rtol, maxit);
        og_divergence(g, s->dt, s->us, s->vs, s->rp);
        ip = og_solve_poisson(g, s->rp, s->phi, s->rtol, maxit); /* warm start (:54) */
    }
    og_correct(g, s->dt, s->us, s->vs, s->phi, s->u, s->v, s->gx, s->gy);
    double umin = s->u[0], umax = s->u[0], vmin = s->v[0], vmax = s->v[0];
    for (int c = 1; c < n; c++) {
        umin = fmin(umin, s->u[c]); umax = fmax(umax, s->u[c]);
        vmin = fmin(vmin, s->v[c]); vmax = fmax(vmax, s->v[c]);
    }
    if (mm) { mm[0] = umin; mm[1] = umax; mm[2] = vmin; mm[3] = vmax; }
    if (its) { its[0] = iu; its[1] = iv; its[2] = ip; }
    return (iu >= maxit || iv >= maxit || ip >= maxit) ? 1 : 0;
}

void og_solver_get(const og_solver* s, double* u, double* v, double* phi, double* cu, double* cv,
                   double* gx, double* gy) {
    size_t b = sizeof(double) * s->g->N;
    if (u) memcpy(u, s->u, b);
    if (v) memcpy(v, s->v, b);
    if (phi) memcpy(phi, s->phi, b);
    if (cu) memcpy(cu, s->cu, b);
    if (cv) memcpy(cv, s->cv, b);
    if (gx) memcpy(gx, s->gx, b);
    if (gy) memcpy(gy, s->gy, b);
}

void og_solver_set(og_solver* s, const double* u, const double* v, const double* phi, const double* cu,
                   const double* cv, const double* gx, const double* gy) {
    size_t b = sizeof(double) * s->g->N;
    if (u) memcpy(s->u, u, b);
    if (v) memcpy(s->v, v, b);
    if (phi) memcpy(s->phi, phi, b);
    if (cu) memcpy(s->cu, cu, b);
    if (cv) memcpy(s->cv, cv, b);
    if (gx) memcpy(s->gx, gx, b);
    if (gy) memcpy(s->gy, gy, b);
}
