/*
 * gpad_oracle.c -- CPU ORACLE for the GPAD inner loop.  TEST INFRASTRUCTURE ONLY
 * (the checker, never the thing measured or shipped).  See gpad_oracle.h for the
 * parity pins.  Compiled with -ffp-contract=off: every fused multiply-add below is
 * an explicit fmaf()/fma() mirroring what the reference's FMA-contracted build does.
 */
#include "gpad_oracle.h"

#include <math.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

/* 8a -- seq_functions.cpp:45-51.  g++ contracts y + beta*(y - ym1) to fma(beta, y-ym1, y). */
void orc_step1_f32(const float* y, const float* ym1, float* w, float beta, int m) {
    for (int i = 0; i < m; i++) w[i] = fmaf(beta, y[i] - ym1[i], y[i]);
}

/* 8b -- seq_functions.cpp:54-66.  Row-major n x m, sequential fmaf chain from +0. */
void orc_step2_f32(const float* MGneg, const float* w, const float* gP, float* zhat, int n, int m) {
    for (int i = 0; i < n; i++) {
        float sum = 0.0f;
        const float* row = MGneg + (size_t)i * m;
        for (int j = 0; j < m; j++) sum = fmaf(row[j], w[j], sum);
        zhat[i] = sum - gP[i];
    }
}

/* 8c -- seq_functions.cpp:68-72 (= step3.cu:24-28).  g++ emits
 * t = theta*zhat; z = fma(1-theta, zm1, t). */
void orc_step3_f32(float theta, int n, const float* zm1, const float* zhat, float* z) {
    const float omt = 1.0f - theta;
    for (int i = 0; i < n; i++) z[i] = fmaf(omt, zm1[i], theta * zhat[i]);
}

/* 8d -- seq_functions.cpp:75-87.  s = (w + pD) + sum;  y+ = (|s| + s) / 2 (exact relu). */
void orc_step4_f32(const float* GL, float* yp1, const float* w, const float* pD, const float* zhat,
                   int n, int m) {
    for (int i = 0; i < m; i++) {
        float sum = 0.0f;
        const float* row = GL + (size_t)i * n;
        for (int j = 0; j < n; j++) sum = fmaf(row[j], zhat[j], sum);
        float s = (w[i] + pD[i]) + sum;
        yp1[i] = (fabsf(s) + s) * 0.5f;
    }
}

/* acceldualgrad.m:20-23: M_G = inv(H)*A', G_L = (1/L)*A, p_D = (-1/L)*b.  The C path's
 * file stores M_G sign-folded (main.cu:43-44 + seq_functions.cpp:61 compute +M_G.w), so
 * MGneg = -ML.  The scalings are done in fp64 as MATLAB does, then rounded to fp32. */
void orc_scale_f32(const float* ML, const float* G, const float* g, float L, int n, int m,
                   float* MGneg, float* GL, float* pD) {
    const double inv = 1.0 / (double)L, ninv = -1.0 / (double)L;
    if (MGneg) for (size_t k = 0; k < (size_t)n * m; k++) MGneg[k] = -ML[k];
    if (GL) for (size_t k = 0; k < (size_t)n * m; k++) GL[k] = (float)(inv * (double)G[k]);
    if (pD) for (int i = 0; i < m; i++) pD[i] = (float)(ninv * (double)g[i]);
}

/* acceldualgrad.m:18,27,55-56 (MATLAB, beta lagged) or eq. (8e) of the paper. */
void orc_schedule(int N, int kind, double* theta, double* beta) {
    double th = 1.0, thm1 = 1.0, b = 0.0;
    for (int v = 0; v < N; v++) {
        const double thn = (sqrt(pow(th, 4.0) + 4.0 * pow(th, 2.0)) - pow(th, 2.0)) / 2.0;
        if (kind == ORC_SCHEDULE_PAPER) {
            theta[v] = th;
            beta[v] = th * (1.0 / thm1 - 1.0);
        } else {
            theta[v] = th;
            beta[v] = b;                      /* value computed in the previous iteration */
            b = th * (1.0 / thm1 - 1.0);      /* acceldualgrad.m:56, used next iteration  */
        }
        thm1 = th;
        th = thn;
    }
}

/* Algorithm 1 test (nmpc12-gpad.pdf sec. 4.2; acceldualgrad.m:66-79 restricted to the
 * branches computable from (ML, M, G, g, L); the value-function branches :73,76 need H and q):
 *   (A) max_i (G z - g)_i <= tol                                   -> stop, return z     (1)
 *   (B) max_i (G zhat - g)_i <= tol, w >= 0, -w'(G zhat - g) <= tol_gap -> stop, return zhat (2)
 * with G x - g = L (GL x + pD) (tol = e_g, tol_gap = e_V of acceldualgrad.m:12-13).
 *
 * Certified on the constraint itself.  GL zhat is the step-4 chain.  GL z is carried by the
 * affine recursion of 8c, u_v = (1-theta_v) u_{v-1} + theta_v (GL zhat_v) -- equal to GL z_v
 * in exact arithmetic, but its f32 rounding drifts from the f32 z (measured: ~10 units of
 * 2^-24 of max|G z|+|g| after 300 iterations, 400 after 20000).  So the recursion only
 * NOMINATES: when it passes (A), GL z is evaluated directly (one chain per row, the step-4
 * chain on z), u is reset to it, and (A) is decided on the direct value.  Both decisions keep a
 * rounding margin: accept when L max(s) + ORC_MARGIN L max_i(|a_i| + |pD_i|) <= tol, where
 * s = a + pD and a is the chain (GL z or GL zhat): the f32 chain error measured against fp64
 * G x - g stays below 3.3 units of 2^-24 of that scale, the margin is 16 units.  The paper
 * (sec. 4.2) returns whichever candidate passed; the commented MATLAB returns z_v in both
 * branches, which for (B) hands back a point that was never certified. */
static float orc_chain(const float* row, const float* x, int n) {
    float sum = 0.0f;
    for (int j = 0; j < n; j++) sum = fmaf(row[j], x[j], sum);
    return sum;
}

/* chain of row i of G_L on x: full rows (row-major m x n) or the flat battery rows */
typedef float (*orc_row_fn)(const void* ctx, int i, const float* x);

/* ---- value-function branches (acceldualgrad.m:30-33, 73, 76) ---------------------------
 * With the QP Hessian H bound (gpad_setup_hessian), the QP is min 1/2 z'Hz + f'z, G z <= g with
 * f = H M (M = g_P = H^-1 f is what the caller passes), and
 *   valuefcn(x)  V(x) = (1/2 x'H + f) x = sum_i (x_i / 2 + M_i) (H x)_i
 *   dualfcn(y)   D(y) = lagrangian(z(y), y) = V(z(y)) + y'(G z(y) - g),  z(y) = -ML y - M
 * evaluated in fp64 on the solve's own (f32 or f64) data: every product (H x)_i, (MGneg y)_i,
 * (G_L x)_i is one fp64 fma chain over ascending k, G x - g = L (G_L x + p_D); the sums over rows
 * are fp64 (the kernels sum them in a wave/workgroup tree: the same value to ~1e-16 relative).
 * Evaluated only where the MATLAB test reaches them: after test (B)'s violation part passed,
 *   w >= 0 and -w'g(zhat) > e_V:  -w'g(zhat) <= V(zhat) e_V / (1 + e_V)   -> code 3  (:73)
 *   w not >= 0:                    V(zhat) - D(y+) <= e_V max(D(y+), 1)     -> code 4  (:76)
 * both returning zhat (as test (B)). */
struct orc_value_ctx {
    const double* H;      /* n x n row-major (fp64 copy of the bound H) */
    const float* MGneg;   /* f32 path: -ML, n x m */
    const float* GL;      /* f32 path: G_L, m x n */
    const float* gP;      /* M */
    const float* pD;
    const float* zhat;
    const float* yp;      /* y_{v+1} */
    int n, m;
    double L;
};

static double orc_valuefcn(const double* H, const float* gP, const double* x, int n) {
    double v = 0.0;
    for (int i = 0; i < n; i++) {
        double hx = 0.0;
        for (int j = 0; j < n; j++) hx = fma(H[(size_t)i * n + j], x[j], hx);
        v += (0.5 * x[i] + (double)gP[i]) * hx;
    }
    return v;
}

static double orc_dualfcn_f32(const struct orc_value_ctx* c) {
    const int n = c->n, m = c->m;
    double* zp = (double*)malloc(sizeof(double) * (size_t)(n > 0 ? n : 1));
    for (int i = 0; i < n; i++) {  /* z(y+) = -ML y+ - M */
        double a = 0.0;
        for (int j = 0; j < m; j++) a = fma((double)c->MGneg[(size_t)i * m + j], (double)c->yp[j], a);
        zp[i] = a - (double)c->gP[i];
    }
    double lin = 0.0;  /* y+'(G z - g) / L */
    for (int k = 0; k < m; k++) {
        double a = 0.0;
        for (int j = 0; j < n; j++) a = fma((double)c->GL[(size_t)k * n + j], zp[j], a);
        lin += (double)c->yp[k] * (a + (double)c->pD[k]);
    }
    const double d = orc_valuefcn(c->H, c->gP, zp, n) + c->L * lin;
    free(zp);
    return d;
}

/* value branches after the violation part of (B) passed: 3, 4 or 0 */
static int orc_value_branch_f32(const struct orc_value_ctx* c, int w_ok, double gapL, double e_V) {
    double* x = (double*)malloc(sizeof(double) * (size_t)(c->n > 0 ? c->n : 1));
    for (int i = 0; i < c->n; i++) x[i] = (double)c->zhat[i];
    const double V = orc_valuefcn(c->H, c->gP, x, c->n);
    free(x);
    if (w_ok) return gapL <= V * e_V / (1.0 + e_V) ? 3 : 0;                    /* :73 */
    const double D = orc_dualfcn_f32(c);
    return V - D <= e_V * (D > 1.0 ? D : 1.0) ? 4 : 0;                          /* :76 */
}

static int orc_check_f32(float* u, const float* ch, const float* pD, const float* w, const float* z,
                         int m, orc_row_fn rowf, const void* ctx, double L, double tol, double tol_gap,
                         const struct orc_value_ctx* vc_ctx) {
    float viol = -INFINITY;
    for (int i = 0; i < m; i++) viol = fmaxf(viol, u[i] + pD[i]);
    if ((double)viol * L <= tol) {  /* (A) nominated by the recursion: decide on G_L z itself */
        float vc = -INFINITY, mag = 0.0f;
        for (int i = 0; i < m; i++) {
            const float c = rowf(ctx, i, z);
            u[i] = c;
            vc = fmaxf(vc, c + pD[i]);
            mag = fmaxf(mag, fabsf(c) + fabsf(pD[i]));
        }
        if ((double)vc * L + ORC_MARGIN_F32 * (double)mag * L <= tol) return 1;
    }
    float violh = -INFINITY, magh = 0.0f, wmin = INFINITY;
    double gap = 0.0;
    for (int i = 0; i < m; i++) {
        const float t = ch[i] + pD[i];
        violh = fmaxf(violh, t);
        magh = fmaxf(magh, fabsf(ch[i]) + fabsf(pD[i]));
        wmin = fminf(wmin, w[i]);
        gap -= (double)w[i] * (double)t;
    }
    const int vh_ok = (double)violh * L + ORC_MARGIN_F32 * (double)magh * L <= tol;
    if (vh_ok && wmin >= 0.0f && gap * L <= tol_gap) return 2;
    if (vh_ok && vc_ctx) return orc_value_branch_f32(vc_ctx, wmin >= 0.0f, gap * L, tol_gap);
    return 0;
}

struct orc_full_rows { const float* GL; int n; };
static float orc_full_row(const void* ctx, int i, const float* x) {
    const struct orc_full_rows* c = (const struct orc_full_rows*)ctx;
    return orc_chain(c->GL + (size_t)i * c->n, x, c->n);
}

static double orc_tol_gap(double tol, double tol_gap) { return tol_gap > 0.0 ? tol_gap : tol; }

static int orc_solve_f32_h(float* z, float* y, const float* MGneg, const float* gP, const float* GL,
                           const float* pD, const float* H, int n, int m, int N, float L, double tol,
                           double tol_gap, int check_every, const float* theta, const float* beta,
                           int* converged);

int orc_solve_f32(float* z, float* y, const float* MGneg, const float* gP, const float* GL,
                  const float* pD, int n, int m, int N, float L, double tol, double tol_gap,
                  int check_every, const float* theta, const float* beta, int* converged) {
    return orc_solve_f32_h(z, y, MGneg, gP, GL, pD, NULL, n, m, N, L, tol, tol_gap, check_every, theta, beta,
                           converged);
}

int orc_solve_value_f32(float* z, float* y, const float* MGneg, const float* gP, const float* GL,
                        const float* pD, const float* H, int n, int m, int N, float L, double tol,
                        double tol_gap, int check_every, const float* theta, const float* beta, int* converged) {
    return orc_solve_f32_h(z, y, MGneg, gP, GL, pD, H, n, m, N, L, tol, tol_gap, check_every, theta, beta,
                           converged);
}

static int orc_solve_f32_h(float* z, float* y, const float* MGneg, const float* gP, const float* GL,
                           const float* pD, const float* H, int n, int m, int N, float L, double tol,
                           double tol_gap, int check_every, const float* theta, const float* beta,
                           int* converged) {
    const int mm = m > 0 ? m : 1;
    float* base = (float*)malloc(sizeof(float) * (size_t)mm * 6);
    float* ycur = base;
    float* yprev = ycur + mm;
    float* w = yprev + mm;
    float* ynew = w + mm;
    float* u = ynew + mm;   /* GL z, by recursion */
    float* ch = u + mm;     /* GL zhat (step-4 chains) */
    float* zhat = (float*)malloc(sizeof(float) * (size_t)(n > 0 ? n : 1));
    if (check_every <= 0) check_every = 10;
    memcpy(ycur, y, sizeof(float) * m);
    memcpy(yprev, y, sizeof(float) * m); /* acceldualgrad.m:16: y_0 = y_{-1} */
    const int use_tol = tol > 0.0;
    const double tgap = orc_tol_gap(tol, tol_gap);
    const struct orc_full_rows rows = {GL, n};
    double* Hd = NULL;
    if (H) {
        Hd = (double*)malloc(sizeof(double) * (size_t)n * n + 1);
        for (size_t k = 0; k < (size_t)n * n; k++) Hd[k] = (double)H[k];
    }
    if (use_tol)
        for (int i = 0; i < m; i++) u[i] = orc_chain(GL + (size_t)i * n, z, n);
    int it = 0, conv = 0;
    for (int v = 0; v < N; v++) {
        orc_step1_f32(ycur, yprev, w, beta[v], m);          /* main.cu:163 */
        orc_step2_f32(MGneg, w, gP, zhat, n, m);            /* main.cu:166 */
        orc_step3_f32(theta[v], n, z, zhat, z);             /* main.cu:170 */
        orc_step4_f32(GL, ynew, w, pD, zhat, n, m);         /* main.cu:171 */
        float* t = yprev; yprev = ycur; ycur = ynew; ynew = t; /* main.cu:167 + MATLAB :60-64 */
        it = v + 1;
        if (use_tol) {
            const float th = theta[v], omt = 1.0f - th;
            for (int i = 0; i < m; i++) {
                ch[i] = orc_chain(GL + (size_t)i * n, zhat, n);  /* = step 4's sum */
                u[i] = fmaf(omt, u[i], th * ch[i]);
            }
            if ((it % check_every) == 0) {
                const struct orc_value_ctx vctx = {Hd, MGneg, GL, gP, pD, zhat, ycur, n, m, (double)L};
                const int c = orc_check_f32(u, ch, pD, w, z, m, orc_full_row, &rows, (double)L, tol, tgap,
                                            Hd ? &vctx : NULL);
                if (c) {
                    if (c >= 2) memcpy(z, zhat, sizeof(float) * n);
                    conv = c;
                    break;
                }
            }
        }
    }
    memcpy(y, ycur, sizeof(float) * m);
    free(base);
    free(zhat);
    free(Hd);
    if (converged) *converged = conv;
    return it;
}

/* ---- fp64, acceldualgrad.m operation order ------------------------------------- */
/* the fp64 twin of orc_check_f32 (margin ORC_MARGIN_F64 = 16 units of 2^-53) */
/* fp64 twins of the value functions (orc_valuefcn's sums; ML is +H^-1 G' here) */
static double orc_valuefcn_d(const double* H, const double* gP, const double* x, int n) {
    double v = 0.0;
    for (int i = 0; i < n; i++) {
        double hx = 0.0;
        for (int j = 0; j < n; j++) hx = fma(H[(size_t)i * n + j], x[j], hx);
        v += (0.5 * x[i] + gP[i]) * hx;
    }
    return v;
}

struct orc_value_ctx_d {
    const double *H, *ML, *GL, *gP, *pD, *zhat, *yp;
    int n, m;
    double L;
};

static int orc_value_branch_f64(const struct orc_value_ctx_d* c, int w_ok, double gapL, double e_V) {
    const int n = c->n, m = c->m;
    const double V = orc_valuefcn_d(c->H, c->gP, c->zhat, n);
    if (w_ok) return gapL <= V * e_V / (1.0 + e_V) ? 3 : 0;
    double* zp = (double*)malloc(sizeof(double) * (size_t)(n > 0 ? n : 1));
    for (int i = 0; i < n; i++) {
        double a = 0.0;
        for (int j = 0; j < m; j++) a = fma(-c->ML[(size_t)i * m + j], c->yp[j], a);
        zp[i] = a - c->gP[i];
    }
    double lin = 0.0;
    for (int k = 0; k < m; k++) {
        double a = 0.0;
        for (int j = 0; j < n; j++) a = fma(c->GL[(size_t)k * n + j], zp[j], a);
        lin += c->yp[k] * (a + c->pD[k]);
    }
    const double D = orc_valuefcn_d(c->H, c->gP, zp, n) + c->L * lin;
    free(zp);
    return V - D <= e_V * (D > 1.0 ? D : 1.0) ? 4 : 0;
}

static int orc_check_f64(double* u, const double* ch, const double* pD, const double* w, const double* z,
                         const double* GL, int n, int m, double L, double tol, double tol_gap,
                         const struct orc_value_ctx_d* vc_ctx) {
    double viol = -INFINITY;
    for (int i = 0; i < m; i++) viol = fmax(viol, u[i] + pD[i]);
    if (viol * L <= tol) {
        double vc = -INFINITY, mag = 0.0;
        for (int i = 0; i < m; i++) {
            double c = 0.0;
            for (int j = 0; j < n; j++) c = fma(GL[(size_t)i * n + j], z[j], c);
            u[i] = c;
            vc = fmax(vc, c + pD[i]);
            mag = fmax(mag, fabs(c) + fabs(pD[i]));
        }
        if (vc * L + ORC_MARGIN_F64 * mag * L <= tol) return 1;
    }
    double violh = -INFINITY, magh = 0.0, wmin = INFINITY, gap = 0.0;
    for (int i = 0; i < m; i++) {
        const double t = ch[i] + pD[i];
        violh = fmax(violh, t);
        magh = fmax(magh, fabs(ch[i]) + fabs(pD[i]));
        wmin = fmin(wmin, w[i]);
        gap -= w[i] * t;
    }
    const int vh_ok = violh * L + ORC_MARGIN_F64 * magh * L <= tol;
    if (vh_ok && wmin >= 0.0 && gap * L <= tol_gap) return 2;
    if (vh_ok && vc_ctx) return orc_value_branch_f64(vc_ctx, wmin >= 0.0, gap * L, tol_gap);
    return 0;
}

static int orc_solve_f64_h(double* z, double* y, const double* ML, const double* gP, const double* G,
                           const double* g, const double* H, int n, int m, int N, double L, double tol,
                           double tol_gap, int check_every, int schedule, int* converged);

int orc_solve_f64(double* z, double* y, const double* ML, const double* gP, const double* G,
                  const double* g, int n, int m, int N, double L, double tol, double tol_gap,
                  int check_every, int schedule, int* converged) {
    return orc_solve_f64_h(z, y, ML, gP, G, g, NULL, n, m, N, L, tol, tol_gap, check_every, schedule, converged);
}

int orc_solve_value_f64(double* z, double* y, const double* ML, const double* gP, const double* G,
                        const double* g, const double* H, int n, int m, int N, double L, double tol,
                        double tol_gap, int check_every, int schedule, int* converged) {
    return orc_solve_f64_h(z, y, ML, gP, G, g, H, n, m, N, L, tol, tol_gap, check_every, schedule, converged);
}

static int orc_solve_f64_h(double* z, double* y, const double* ML, const double* gP, const double* G,
                           const double* g, const double* H, int n, int m, int N, double L, double tol,
                           double tol_gap, int check_every, int schedule, int* converged) {
    const size_t nm = (size_t)n * m;
    double* GL = (double*)malloc(sizeof(double) * (nm + 1));
    double* pD = (double*)malloc(sizeof(double) * (m + 1));
    double* yv = (double*)malloc(sizeof(double) * (m + 1));
    double* yvm1 = (double*)malloc(sizeof(double) * (m + 1));
    double* w = (double*)malloc(sizeof(double) * (m + 1));
    double* yp1 = (double*)malloc(sizeof(double) * (m + 1));
    double* zhat = (double*)malloc(sizeof(double) * (n + 1));
    double* th = (double*)malloc(sizeof(double) * (N + 1));
    double* be = (double*)malloc(sizeof(double) * (N + 1));
    double* u = (double*)malloc(sizeof(double) * (m + 1));
    double* ch = (double*)malloc(sizeof(double) * (m + 1));
    const double inv = 1.0 / L, ninv = -1.0 / L;
    for (size_t k = 0; k < nm; k++) GL[k] = inv * G[k];           /* acceldualgrad.m:22 */
    for (int i = 0; i < m; i++) pD[i] = ninv * g[i];              /* acceldualgrad.m:23 */
    orc_schedule(N, schedule, th, be);
    if (check_every <= 0) check_every = 10;
    memcpy(yv, y, sizeof(double) * m);
    memcpy(yvm1, y, sizeof(double) * m);
    const int use_tol = tol > 0.0;
    if (use_tol)
        for (int i = 0; i < m; i++) {
            double sum = 0.0;
            for (int j = 0; j < n; j++) sum = fma(GL[(size_t)i * n + j], z[j], sum);
            u[i] = sum;
        }
    int it = 0, conv = 0;
    for (int v = 0; v < N; v++) {
        for (int i = 0; i < m; i++) w[i] = yv[i] + be[v] * (yv[i] - yvm1[i]);      /* :43 */
        for (int i = 0; i < n; i++) {                                               /* :46 */
            double sum = 0.0;
            for (int j = 0; j < m; j++) sum = fma(-ML[(size_t)i * m + j], w[j], sum);
            zhat[i] = sum - gP[i];
        }
        for (int i = 0; i < n; i++) z[i] = (1.0 - th[v]) * z[i] + th[v] * zhat[i]; /* :49 */
        for (int i = 0; i < m; i++) {                                               /* :52 */
            double sum = 0.0;
            for (int j = 0; j < n; j++) sum = fma(GL[(size_t)i * n + j], zhat[j], sum);
            double s = (w[i] + sum) + pD[i];
            yp1[i] = s > 0.0 ? s : 0.0;
            ch[i] = sum;
            if (use_tol) u[i] = (1.0 - th[v]) * u[i] + th[v] * sum;
        }
        double* t = yvm1; yvm1 = yv; yv = yp1; yp1 = t;                               /* :60-64 */
        it = v + 1;
        if (use_tol && (it % check_every) == 0) {
            const struct orc_value_ctx_d vctx = {H, ML, GL, gP, pD, zhat, yv, n, m, L};
            const int c = orc_check_f64(u, ch, pD, w, z, GL, n, m, L, tol, orc_tol_gap(tol, tol_gap),
                                        H ? &vctx : NULL);
            if (c) {
                if (c >= 2) memcpy(z, zhat, sizeof(double) * n);
                conv = c;
                break;
            }
        }
    }
    memcpy(y, yv, sizeof(double) * m);
    free(GL); free(pD); free(yv); free(yvm1); free(w); free(yp1); free(zhat); free(th); free(be);
    free(u); free(ch);
    if (converged) *converged = conv;
    return it;
}

long long orc_solve_batch_f32(float* z, float* y, const float* MGneg, const float* gP,
                              const float* GL, const float* pD, int n, int m, int batch,
                              int shared, int N, float L, double tol, double tol_gap, int check_every,
                              const float* theta, const float* beta, int* iters, int threads) {
    long long total = 0;
    const size_t nm = (size_t)n * m;
#ifdef _OPENMP
    if (threads <= 0) threads = 0;
#pragma omp parallel for schedule(dynamic, 1) reduction(+ : total) num_threads(threads > 0 ? threads : omp_get_max_threads())
#endif
    for (int b = 0; b < batch; b++) {
        const float* mg = shared ? MGneg : MGneg + (size_t)b * nm;
        const float* gl = shared ? GL : GL + (size_t)b * nm;
        int conv = 0;
        int it = orc_solve_f32(z + (size_t)b * n, y + (size_t)b * m, mg, gP + (size_t)b * n, gl,
                               pD + (size_t)b * m, n, m, N, L, tol, tol_gap, check_every, theta, beta, &conv);
        if (iters) iters[b] = it;
        total += it;
    }
    (void)threads;
    return total;
}

/* ---- per-state data and closed loop (gpad.m:79-95) ------------------------------------ */
void orc_affine_f32(const float* P, const float* c0, const float* x, float* out, int rows, int nx) {
    for (int i = 0; i < rows; i++) {
        float acc = c0 ? c0[i] : 0.0f;
        for (int k = 0; k < nx; k++) acc = fmaf(P[(size_t)i * nx + k], x[k], acc);
        out[i] = acc;
    }
}

void orc_plant_step_f32(const float* A, const float* B, const float* x, const float* u, float* xn,
                        int nx, int nu) {
    for (int i = 0; i < nx; i++) {
        float acc = 0.0f;
        for (int k = 0; k < nx; k++) acc = fmaf(A[(size_t)i * nx + k], x[k], acc);
        for (int j = 0; j < nu; j++) acc = fmaf(B[(size_t)i * nu + j], u[j], acc);
        xn[i] = acc;
    }
}

long long orc_closed_loop_f32(float* x, float* z, float* y, const float* MGneg, const float* GL,
                              float L, int n, int m, const float* PM, const float* M0,
                              const float* Pg, const float* g0, const float* A, const float* B,
                              int nx, int nu, int steps, int N, double tol, double tol_gap,
                              int check_every, const float* theta, const float* beta, int warm, float* xs,
                              float* us, int* iters) {
    float* gP = (float*)malloc(sizeof(float) * (n + 1));
    float* g = (float*)malloc(sizeof(float) * (m + 1));
    float* pD = (float*)malloc(sizeof(float) * (m + 1));
    float* xn = (float*)malloc(sizeof(float) * (nx + 1));
    const double ninv = -1.0 / (double)L;
    long long total = 0;
    for (int t = 0; t < steps; t++) {
        orc_affine_f32(PM, M0, x, gP, n, nx);                 /* gpad.m:81 + acceldualgrad.m:21 */
        orc_affine_f32(Pg, g0, x, g, m, nx);                  /* gpad.m:85 */
        for (int i = 0; i < m; i++) pD[i] = (float)(ninv * (double)g[i]);  /* acceldualgrad.m:23 */
        if (!warm) {                                          /* acceldualgrad.m:16-17 */
            memset(z, 0, sizeof(float) * n);
            memset(y, 0, sizeof(float) * m);
        }
        int conv = 0;
        const int it = orc_solve_f32(z, y, MGneg, gP, GL, pD, n, m, N, L, tol, tol_gap, check_every, theta,
                                     beta, &conv);
        total += it;
        if (iters) iters[t] = it;
        if (xs) memcpy(xs + (size_t)t * nx, x, sizeof(float) * nx);
        if (us) memcpy(us + (size_t)t * nu, z, sizeof(float) * nu);
        orc_plant_step_f32(A, B, x, z, xn, nx, nu);           /* gpad.m:91-93 */
        memcpy(x, xn, sizeof(float) * nx);
    }
    free(gP);
    free(g);
    free(pD);
    free(xn);
    return total;
}

/* ---- flat battery steps (seq_functions.cpp:5-43) -------------------------------------- */
void orc_step2_flat_f32(const float* MGf, const float* w, const float* gP, float* zhat, int Nh,
                        int n_u, int m) {
    const int mc = 4 * n_u * Nh;
    for (int i = 0; i < Nh; i++)
        for (int j = 0; j < n_u; j++) {
            float sum = 0.0f;
            for (int k = j; k < mc; k += n_u) sum = fmaf(MGf[(size_t)i * m + k], w[k], sum);
            for (int k = mc; k < m; k++) sum = fmaf(MGf[(size_t)i * m + k], w[k], sum);
            zhat[i * n_u + j] = sum - gP[i * n_u + j];
        }
}

static float orc_flat_row4(const float* GLf, const float* zhat, int r, int Nh, int n_u, int mc) {
    float sum = 0.0f;
    for (int t = 0; t < Nh; t++) {
        const float g = GLf[(size_t)r * Nh + t];
        if (r < mc) {
            sum = fmaf(g, zhat[t * n_u + (r % n_u)], sum);
        } else {
            for (int k = 0; k < n_u; k++) sum = fmaf(g, zhat[t * n_u + k], sum);
        }
    }
    return sum;
}

void orc_step4_flat_f32(const float* GLf, float* yp1, const float* w, const float* pD,
                        const float* zhat, int Nh, int n_u, int m) {
    const int mc = 4 * n_u * Nh;
    for (int r = 0; r < m; r++) {
        const float s = (orc_flat_row4(GLf, zhat, r, Nh, n_u, mc) + w[r]) + pD[r];
        yp1[r] = s < 0.0f ? 0.0f : s;
    }
}

struct orc_flat_rows { const float* GLf; int Nh, n_u, mc; };
static float orc_flat_row(const void* ctx, int i, const float* x) {
    const struct orc_flat_rows* c = (const struct orc_flat_rows*)ctx;
    return orc_flat_row4(c->GLf, x, i, c->Nh, c->n_u, c->mc);
}

int orc_solve_flat_f32(float* z, float* y, const float* MGf, const float* gP, const float* GLf,
                       const float* pD, int Nh, int n_u, int m, int N, float L, double tol, double tol_gap,
                       int check_every, const float* theta, const float* beta, int* converged) {
    const int n = n_u * Nh, mc = 4 * n_u * Nh;
    const int mm = m > 0 ? m : 1;
    float* base = (float*)malloc(sizeof(float) * (size_t)mm * 6);
    float* ycur = base;
    float* yprev = ycur + mm;
    float* w = yprev + mm;
    float* ynew = w + mm;
    float* u = ynew + mm;
    float* ch = u + mm;
    float* zhat = (float*)malloc(sizeof(float) * (size_t)(n > 0 ? n : 1));
    if (check_every <= 0) check_every = 10;
    memcpy(ycur, y, sizeof(float) * m);
    memcpy(yprev, y, sizeof(float) * m);
    const int use_tol = tol > 0.0;
    const double tgap = orc_tol_gap(tol, tol_gap);
    const struct orc_flat_rows rows = {GLf, Nh, n_u, mc};
    if (use_tol)
        for (int r = 0; r < m; r++) u[r] = orc_flat_row4(GLf, z, r, Nh, n_u, mc);
    int it = 0, conv = 0;
    for (int v = 0; v < N; v++) {
        orc_step1_f32(ycur, yprev, w, beta[v], m);
        orc_step2_flat_f32(MGf, w, gP, zhat, Nh, n_u, m);
        orc_step3_f32(theta[v], n, z, zhat, z);
        orc_step4_flat_f32(GLf, ynew, w, pD, zhat, Nh, n_u, m);
        float* t = yprev; yprev = ycur; ycur = ynew; ynew = t;
        it = v + 1;
        if (use_tol) {
            const float th = theta[v], omt = 1.0f - th;
            for (int r = 0; r < m; r++) {
                ch[r] = orc_flat_row4(GLf, zhat, r, Nh, n_u, mc);
                u[r] = fmaf(omt, u[r], th * ch[r]);
            }
            if ((it % check_every) == 0) {
                const int c = orc_check_f32(u, ch, pD, w, z, m, orc_flat_row, &rows, (double)L, tol, tgap, NULL);
                if (c) {
                    if (c == 2) memcpy(z, zhat, sizeof(float) * n);
                    conv = c;
                    break;
                }
            }
        }
    }
    memcpy(y, ycur, sizeof(float) * m);
    free(base);
    free(zhat);
    if (converged) *converged = conv;
    return it;
}
