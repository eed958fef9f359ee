/*
 * gpad_oracle.h -- CPU ORACLE for the GPAD inner loop.  TEST INFRASTRUCTURE ONLY.
 *
 * This is a plain-C restatement of the reference's CPU path
 * (Code/CUDA/FinalProject/src/seq_functions.cpp, composed in the loop order of
 * Code/CUDA/FinalProject/main.cu:160-175, with the theta/beta schedule of
 * Code/MATLAB/acceldualgrad.m:18,27,55-56).  It is the checker that the HIP
 * product path (libgpad.so) is compared against.  Only tests/,
 * __graft_entry__.smoke() and bench.py's cpu_baseline leg may load it; the
 * product path never links or calls it.
 *
 * Parity pins (see DESIGN.md "Oracle"):
 *   - fp32 steps are bit-exact against the reference's own seq_functions.cpp
 *     compiled from /root/reference by oracle/Makefile (target `ref`) with
 *     -O2 -mfma -ffp-contract=fast (what -O3 -march=native gives on any FMA
 *     x86): every `sum += a*b` is an fmaf chain, step 1 is fmaf(beta, y-ym1, y),
 *     step 3 is fmaf(1-theta, zm1, theta*zhat), step 4 is ((w+pD)+sum) then
 *     (|s|+s)*0.5.  The restatement spells those contractions out with fmaf()
 *     and is itself compiled with -ffp-contract=off so they cannot drift.
 *   - the fp64 path follows Code/MATLAB/acceldualgrad.m:43-56 operation order
 *     and is pinned against a numpy restatement of acceldualgrad.m
 *     (tests/golden/make_golden.py) and the reference's step3 fixtures.
 */
#ifndef GPAD_ORACLE_H
#define GPAD_ORACLE_H

#ifdef __cplusplus
extern "C" {
#endif

/* theta/beta schedules (acceldualgrad.m:18,27,55-56; paper eq. 8e) */
#define ORC_SCHEDULE_MATLAB 0 /* beta lagged one iteration, as acceldualgrad.m */
#define ORC_SCHEDULE_PAPER 1  /* beta_v = theta_v (1/theta_{v-1} - 1), eq. (8e) */

/* ---- fp32 steps: one function per reference step (seq_functions.cpp) ---- */
/* 8a  seq_functions.cpp:45-51   w = y + beta (y - ym1)                       */
void orc_step1_f32(const float* y, const float* ym1, float* w, float beta, int m);
/* 8b  seq_functions.cpp:54-66   zhat = MGneg . w - gP   (MGneg = -H^-1 G^T, n x m row-major) */
void orc_step2_f32(const float* MGneg, const float* w, const float* gP, float* zhat, int n, int m);
/* 8c  seq_functions.cpp:68-72   z = (1-theta) zm1 + theta zhat               */
void orc_step3_f32(float theta, int n, const float* zm1, const float* zhat, float* z);
/* 8d  seq_functions.cpp:75-87   y+ = max(0, w + GL . zhat + pD) (GL m x n row-major) */
void orc_step4_f32(const float* GL, float* yp1, const float* w, const float* pD, const float* zhat,
                   int n, int m);

/* Input scaling shared by oracle and product path (acceldualgrad.m:20-23):
 * MGneg = -ML, GL = fl32((1/L)_64 * G), pD = fl32((-1/L)_64 * g).            */
void orc_scale_f32(const float* ML, const float* G, const float* g, float L, int n, int m,
                   float* MGneg, float* GL, float* pD);

/* theta[v] multiplies zhat in iteration v, beta[v] extrapolates w in iteration v (fp64). */
void orc_schedule(int N, int kind, double* theta, double* beta);

/* Rounding margin of the Algorithm 1 decisions (see orc_check_f32 in gpad_oracle.c): a test
 * passes when L max(chain + pD) + MARGIN L max(|chain| + |pD|) <= tol; 16 units of the f32
 * (2^-24) / f64 (2^-53) rounding unit.  The kernels use the same constants (gpad_internal.h). */
#define ORC_MARGIN_F32 0x1p-20
#define ORC_MARGIN_F64 0x1p-49

/* Full solve in main.cu:160-175 order.  z: in z_{-1}, out z*; y: in y0 (= y_{-1}), out y*.
 * tol <= 0: exactly N iterations (Algorithm 2).  tol > 0: Algorithm 1 check every
 * check_every iterations (acceldualgrad.m:66-79; test (A) certifies z, test (B) certifies
 * zhat, which is then returned as z*); tol = e_g (constraint violation), tol_gap = e_V (the
 * duality-gap term of (B); <= 0: = tol).  theta/beta: fp32 schedule tables of length N.
 * Returns the number of iterations executed; *converged = 0 (no), 1 (test A), 2 (test B). */
int orc_solve_f32(float* z, float* y, const float* MGneg, const float* gP, const float* GL,
                  const float* pD, int n, int m, int N, float L, double tol, double tol_gap,
                  int check_every, const float* theta, const float* beta, int* converged);

/* orc_solve_f32 with the value-function branches of Algorithm 1 (acceldualgrad.m:73,76; see
 * orc_value_branch_f32 in gpad_oracle.c): H is the QP Hessian (n x n row-major, f32), the linear
 * term is f = H gP.  *converged additionally 3 (:73, relative gap) or 4 (:76, value - dual gap),
 * both returning zhat. */
int orc_solve_value_f32(float* z, float* y, const float* MGneg, const float* gP, const float* GL,
                        const float* pD, const float* H, int n, int m, int N, float L, double tol,
                        double tol_gap, int check_every, const float* theta, const float* beta, int* converged);
int orc_solve_value_f64(double* z, double* y, const double* ML, const double* gP, const double* G,
                        const double* g, const double* H, int n, int m, int N, double L, double tol,
                        double tol_gap, int check_every, int schedule, int* converged);

/* fp64 solve in acceldualgrad.m:43-64 order: inputs are ML (+H^-1 G^T), gP, G, g, L. */
int orc_solve_f64(double* z, double* y, const double* ML, const double* gP, const double* G,
                  const double* g, int n, int m, int N, double L, double tol, double tol_gap,
                  int check_every, int schedule, int* converged);

/* Batch of independent instances (shared ML/G when shared != 0), `threads` OpenMP
 * threads (<= 0: all).  Per-instance vectors are packed [batch][n] / [batch][m].
 * iters (optional) receives per-instance iteration counts.  Returns total iterations. */
long long orc_solve_batch_f32(float* z, float* y, const float* MGneg, const float* gP,
                              const float* GL, const float* pD, int n, int m, int batch,
                              int shared, int N, float L, double tol, double tol_gap, int check_every,
                              const float* theta, const float* beta, int* iters, int threads);

/* ---- "flat" battery steps (equal cell capacities; seq_functions.cpp:5-43) --------------
 * n_u cells, horizon Nh: n = n_u*Nh primal rows, m = 4 n_u Nh + 2 Nh constraints.  MGf is the
 * flat Nh x m sign-folded M_G, GLf the flat m x Nh G_L (the reference's ENABLE_FLATTEN_MATRICES
 * data).  Step 2: zhat[i n_u + j] = chain(k = j, j+n_u, .. < 4 n_u Nh; then k = 4 n_u Nh .. m-1)
 * of MGf[i][k] w[k], minus gP.  Step 4: row r < 4 n_u Nh: chain over t of GLf[r][t] *
 * zhat[t n_u + r % n_u]; row r >= 4 n_u Nh: chain over t, k of GLf[r][t] * zhat[t n_u + k];
 * y = (sum + w) + pD, then y < 0 -> 0 (NOT the non-flat ((w + pD) + sum, (|s|+s)/2)). */
void orc_step2_flat_f32(const float* MGf, const float* w, const float* gP, float* zhat, int Nh,
                        int n_u, int m);
void orc_step4_flat_f32(const float* GLf, float* yp1, const float* w, const float* pD,
                        const float* zhat, int Nh, int n_u, int m);
/* main_prof.cu flat loop order (steps 1, 2-flat, 3, 4-flat) + the same Algorithm 1 test. */
int orc_solve_flat_f32(float* z, float* y, const float* MGf, const float* gP, const float* GLf,
                       const float* pD, int Nh, int n_u, int m, int N, float L, double tol, double tol_gap,
                       int check_every, const float* theta, const float* beta, int* converged);

/* ---- per-state data and closed loop (gpad_setup_plant / gpad_closed_loop) ----------
 * gpad.m:79-95 restated: the state-dependent QP data are affine in x and the plant is LTI.
 * These define the fp32 evaluation order the product path must match bit for bit.      */
/* out[i] = c0[i] + sum_k P[i][k] x[k]: acc = c0[i] (0 if c0 == NULL); acc = fmaf(P, x, acc) */
void orc_affine_f32(const float* P, const float* c0, const float* x, float* out, int rows, int nx);
/* xn[i] = sum_k A[i][k] x[k] + sum_j B[i][j] u[j]: one fmaf chain from 0, A terms then B */
void orc_plant_step_f32(const float* A, const float* B, const float* x, const float* u, float* xn,
                        int nx, int nu);
/* One instance, `steps` MPC steps of gpad.m:79-95: M = M(x), g = g(x); pD = fl32((-1/L)_64 g);
 * (z, y) = 0 unless warm; orc_solve_f32; xs[t] = x; us[t] = z[0:nu]; x = A x + B u.
 * MGneg/GL as orc_scale_f32 produces them.  xs [steps][nx], us [steps][nu], iters [steps]
 * are optional.  Returns the total iteration count. */
long long orc_closed_loop_f32(float* x, float* z, float* y, const float* MGneg, const float* GL,
                              float L, int n, int m, const float* PM, const float* M0,
                              const float* Pg, const float* g0, const float* A, const float* B,
                              int nx, int nu, int steps, int N, double tol, double tol_gap,
                              int check_every, const float* theta, const float* beta, int warm, float* xs,
                              float* us, int* iters);

#ifdef __cplusplus
}
#endif
#endif
