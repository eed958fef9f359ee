/*
 * gpad.h -- C-ABI of the MI355X-native GPAD solver (libgpad.so).
 *
 * GPAD = accelerated dual gradient-projection for the condensed linear-MPC QP
 *     min 1/2 z'Hz + q'z   s.t.  G z <= g
 * (Bemporad & Patrinos, NMPC'12, eq. 8; reference Code/MATLAB/acceldualgrad.m).
 *
 * Plain C: pointers, sizes and status codes only; no C++ or torch types cross this boundary.
 * Every entry point names the reference interface it replaces (file:line, relative to
 * /root/reference).  Reference-side bindings (C/CUDA driver, ctypes) are in INTEGRATION.md.
 *
 * Conventions
 *   - Matrices are row-major in their mathematical orientation: ML is n x m, G is m x n.
 *   - Batches pack per-instance vectors contiguously: z [batch][n], y/g [batch][m], M [batch][n];
 *     per-instance matrices (dims.shared == 0) are packed [batch][n][m] / [batch][m][n].
 *   - dims.dtype selects float (GPAD_DTYPE_F32) or double (GPAD_DTYPE_F64) for EVERY pointer.
 *   - dims.memory says whether the caller's pointers are host or device (HIP) memory.
 *   - Status: 0 = OK, < 0 = error (gpad_strerror()).  No exceptions cross the ABI.
 *   - Thread safety: distinct handles may be used concurrently; one handle is not reentrant.
 */
#ifndef GPAD_H
#define GPAD_H

#ifdef __cplusplus
extern "C" {
#endif

#define GPAD_VERSION_MAJOR 0
#define GPAD_VERSION_MINOR 1

/* status codes */
#define GPAD_OK 0
#define GPAD_ERR_INVALID (-1)      /* bad argument / inconsistent dims                  */
#define GPAD_ERR_HIP (-2)          /* HIP runtime error (gpad_last_error() has details) */
#define GPAD_ERR_NOMEM (-3)        /* device allocation failed                          */
#define GPAD_ERR_UNSUPPORTED (-4)  /* shape/kernel combination not supported            */
#define GPAD_ERR_NOT_SETUP (-5)    /* gpad_run before gpad_setup                        */
#define GPAD_ERR_NO_DEVICE (-6)    /* no HIP device visible                             */

/* theta/beta schedule (acceldualgrad.m:18,27,55-56 vs paper eq. 8e) */
#define GPAD_SCHEDULE_MATLAB 0 /* beta lagged one iteration, as the reference's MATLAB  */
#define GPAD_SCHEDULE_PAPER 1  /* beta_v = theta_v (1/theta_{v-1} - 1)                   */

#define GPAD_MEM_HOST 0
#define GPAD_MEM_DEVICE 1

#define GPAD_DTYPE_F32 0
#define GPAD_DTYPE_F64 1

/* kernel families (GPAD_KERNEL_AUTO picks; the others force one, for tests and benches) */
#define GPAD_KERNEL_AUTO 0
#define GPAD_KERNEL_STREAM 1   /* matrices streamed (k-major) from HBM/L2; one workgroup/instance */
#define GPAD_KERNEL_RESIDENT 2 /* matrix rows held in VGPRs; one workgroup/instance; n,m <= 208  */
#define GPAD_KERNEL_PANEL 3    /* shared ML/G, f32 MFMA 16x16x4 panels; one wave per 16 instances */

typedef struct gpad_dims {
    int n;           /* primal variables, n = n_u * N                                   */
    int m;           /* inequality constraints (battery: m = 4 n_u N + 2 N)             */
    int batch;       /* independent instances, >= 1                                     */
    int shared;      /* 1: ML, G shared by every instance; 0: per-instance matrices     */
    int dtype;       /* GPAD_DTYPE_*                                                    */
    int memory;      /* GPAD_MEM_*: where the caller's pointers live                    */
    int schedule;    /* GPAD_SCHEDULE_*                                                 */
    int check_every; /* termination test period K when tol > 0 (<= 0 -> 10)            */
    int kernel;      /* GPAD_KERNEL_*                                                   */
} gpad_dims_t;

typedef struct gpad_stats {
    int iterations;              /* max iterations over the batch                       */
    int converged;               /* instances that met tol (0 when tol <= 0)            */
    long long total_iterations;  /* sum of per-instance iterations                      */
    int kernel;                  /* GPAD_KERNEL_* that ran                               */
    double kernel_ms;            /* device time of the solve launch (HIP events)        */
    int* iters;                  /* optional caller array [batch] (host) or NULL        */
} gpad_stats_t;

typedef struct gpad_handle_s* gpad_handle_t;

const char* gpad_version(void);
const char* gpad_strerror(int status);
const char* gpad_last_error(void); /* thread-local detail of the last failure */

/* Handle bound to one device and one HIP stream; every launch and copy of the handle is
 * ordered on that stream.  NULL = the device's default (null) stream, as in every HIP API.
 * Replaces the implicit device/default-stream state of main.cu:116-147. */
int gpad_create(gpad_handle_t* h, int device, void* hip_stream);
int gpad_destroy(gpad_handle_t h);
int gpad_set_stream(gpad_handle_t h, void* hip_stream);

/* Bind the problem shape and the (constant) matrices: ML = H^-1 G' and G, with Lipschitz L.
 * Packs them into the device layouts the kernels read (MGneg = -ML and G_L = G/L,
 * acceldualgrad.m:20-22).  Replaces the off-line precompute + H2D copy of main.cu:29-67,
 * 126-147.  Reusable across many gpad_run calls (an LTI plant has constant ML/G). */
int gpad_setup(gpad_handle_t h, const gpad_dims_t* dims, const void* ML, const void* G, double L);

/* Same, for the reference's data-file boundary (main.cu:29-67): MGneg holds -H^-1 G'
 * (sign-folded as the file does) and GL = G/L already; L only scales tol. */
int gpad_setup_scaled(gpad_handle_t h, const gpad_dims_t* dims, const void* MGneg, const void* GL,
                      double L);

/* Run GPAD on the bound problem for every instance of the batch.
 *   z0: in z_{-1}, out z*      [batch][n]   (acceldualgrad.m:17, :83)
 *   y0: in y_0 = y_{-1}, out y* [batch][m]  (acceldualgrad.m:16)
 *   M : H^-1 q per instance    [batch][n]   (g_P, acceldualgrad.m:21)
 *   g : constraint rhs         [batch][m]   (b_i; p_D = -g/L, acceldualgrad.m:23)
 *   N : max iterations (reference: N_v = 100, main.cu:87)
 *   tol <= 0: exactly N iterations (paper Algorithm 2, main.cu behaviour);
 *   tol  > 0: Algorithm 1 test every check_every iterations (acceldualgrad.m:66-79).
 * Host memory: synchronous.  Device memory: enqueued on the handle's stream; synchronous only
 * when st != NULL (stats need the per-instance counters). */
int gpad_run(gpad_handle_t h, void* z0, void* y0, const void* M, const void* g, int N, double tol,
             gpad_stats_t* st);

/* gpad_run for gpad_setup_scaled problems: gP (g_P) and pD (p_D = -g/L) as in the data file,
 * optional per-iteration theta/beta tables (main.cu:61-64; float or double per dtype, length N;
 * NULL -> dims.schedule). */
int gpad_run_scaled(gpad_handle_t h, void* z0, void* y0, const void* gP, const void* pD, int N,
                    double tol, const void* theta, const void* beta, gpad_stats_t* st);

/* Per-instance iteration counts / convergence flags of the last run (device work finished). */
int gpad_last_stats(gpad_handle_t h, gpad_stats_t* st);

/* One-shot north-star surface: solve(z0, y0, ML, M, G, g, N, L, tol).  Equivalent to
 * create + setup + run + destroy (the handle is cached per thread and device). */
int gpad_solve(void* z0, void* y0, const void* ML, const void* M, const void* G, const void* g,
               int N, double L, double tol, const gpad_dims_t* dims, gpad_stats_t* st);

/* ---- per-step device entry points (float, device pointers, handle stream) ---------------
 * Mirror the reference kernels of kernel_functions.h:9-41 one for one, with the CPU
 * semantics of seq_functions.h:4-17 (row-major matrices).  For integration and per-step
 * known-answer tests; the fused gpad_run path is the fast one. */
/* 8a: w = y + beta (y - ym1)               -- StepOneGPADKernel, kernel_functions.cu:7-14   */
int gpad_step1_extrapolate(gpad_handle_t h, const float* y, const float* ym1, float* w, float beta,
                           int m);
/* 8b: zhat = MGneg w - gP (MGneg n x m)    -- StepTwoGPADKernel, kernel_functions.cu:16-64  */
int gpad_step2_primal(gpad_handle_t h, const float* MGneg, const float* w, const float* gP,
                      float* zhat, int n, int m);
/* 8c: z = (1-theta) zm1 + theta zhat        -- StepThreeGPADKernel, kernel_functions.cu:66-72 */
int gpad_step3_average(gpad_handle_t h, float theta, const float* zm1, const float* zhat, float* z,
                       int n);
/* 8d: yp1 = max(0, w + GL zhat + pD)        -- StepFourGPADFlippedParRows, kernel_functions.cu:142-200 */
int gpad_step4_project(gpad_handle_t h, const float* GL, float* yp1, const float* w,
                       const float* pD, const float* zhat, int n, int m);
/* 8e (host): theta[v], beta[v] for v < N   -- acceldualgrad.m:18,27,55-56 / main.cu:61-64    */
int gpad_schedule(int N, int kind, double* theta, double* beta);

/* Synchronise the handle's stream (for callers using device memory + async runs). */
int gpad_sync(gpad_handle_t h);

#ifdef __cplusplus
}
#endif
#endif /* GPAD_H */
