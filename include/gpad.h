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
#define GPAD_VERSION_MINOR 5 /* 0.3: gpad_stats_t gained tol_floor / flags, gpad_dims_t an explicit reserved
                              * word (layouts changed: rebuild callers against this header);
                              * 0.4: the condensed operator (kernel 5, option 14) removed, the device
                              * error word sticky until reported; layouts as in 0.3;
                              * 0.5: options 20, 21 removed; layouts as in 0.3 */

/* status codes */
#define GPAD_OK 0
#define GPAD_ERR_INVALID (-1)      /* bad argument / inconsistent dims                  */
#define GPAD_ERR_HIP (-2)          /* HIP runtime error (gpad_last_error() has details) */
#define GPAD_ERR_NOMEM (-3)        /* device allocation failed                          */
#define GPAD_ERR_UNSUPPORTED (-4)  /* shape/kernel combination not supported            */
#define GPAD_ERR_NOT_SETUP (-5)    /* gpad_run before gpad_setup                        */
#define GPAD_ERR_NO_DEVICE (-6)    /* no HIP device visible                             */
#define GPAD_ERR_DEVICE (-7)       /* a kernel reported a failure on the device (e.g. a chain
                                    * hand-off that never arrived): the run's z, y are invalid.
                                    * Returned by the call that collects the run's stats or
                                    * synchronises it (gpad_run with st, gpad_last_stats,
                                    * gpad_sync, host-memory runs) -- never GPAD_OK; the error
                                    * is kept on the device until one of those reports it, so
                                    * asynchronous runs queued behind a failed one do not
                                    * hide it, and once reported every later sync / stats call
                                    * on the handle returns it again until the next run starts */

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
#define GPAD_KERNEL_FLAT 4     /* reported only: the flat battery path bound by gpad_setup_flat      */
/* 5: the opt-in condensed operator (not the reference's arithmetic), removed in 0.4; dims.kernel = 5
 * returns GPAD_ERR_INVALID */

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
    int reserved;    /* must be 0 (explicit padding before tol_gap; reserved for extensions) */
    double tol_gap;  /* e_V of acceldualgrad.m:13: tolerance of test (B)'s duality-gap term
                      * -w'(G zhat - g); <= 0 (e.g. a zeroed struct): the run's tol (= e_g) */
} gpad_dims_t;

typedef struct gpad_stats {
    int iterations;              /* max iterations over the batch                       */
    int converged;               /* instances that met tol (0 when tol <= 0)            */
    long long total_iterations;  /* sum of per-instance iterations                      */
    int kernel;                  /* GPAD_KERNEL_* that ran                               */
    double kernel_ms;            /* device time of the solve launch (HIP events)        */
    int* iters;                  /* optional caller array (host) or NULL: [batch]; gpad_closed_loop:
                                  * [steps][batch]                                        */
    double tol_floor;            /* tol > 0: the certification floor of this run's data, see
                                  * gpad_run (0 when tol <= 0)                             */
    int flags;                   /* GPAD_FLAG_* of the run                                  */
    int* codes;                  /* optional caller array (host) or NULL, sized as iters:
                                  * [batch]; gpad_closed_loop: [steps][batch].  Per-instance
                                  * termination code, 0 = ran to N, 1..4 = the test that
                                  * stopped it (gpad_run)                                   */
} gpad_stats_t;

/* gpad_stats_t.flags */
#define GPAD_FLAG_TOL_FLOOR 1 /* 0 < tol < tol_floor: no instance with an active constraint can be
                               * certified; expect converged == 0 (use f64 or a larger tol)   */
#define GPAD_FLAG_NONFINITE_G 2 /* tol > 0 and g holds a NaN or an infinity: tol_floor is not
                                 * finite (NaN when g has a NaN) and TOL_FLOOR is set too        */

typedef struct gpad_handle_s* gpad_handle_t;

const char* gpad_version(void);
/* HIP devices visible to this process (>= 0), or a negative GPAD_ERR_* status; the device list
 * of gpad_group_create / gpad_solve_sharded (main.cu picks device 0, :116) */
int gpad_device_count(void);
const char* gpad_strerror(int status);
/* thread-local detail of the last failure; HIP runtime failures carry the HIP status name and
 * number ("hipErrorNoDevice (code 100): ...") */
const char* gpad_last_error(void);

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

/* The reference's "flat" battery data (ENABLE_FLATTEN_MATRICES, main.cu:39-56; valid for equal
 * cell capacities): MGf is the N x m flat sign-folded M_G, GLf the m x N flat G_L (row-major as
 * seq_functions.cpp:5-43 index them), n = dims.n = n_u N, m = dims.m >= 4 n_u N.  Subsequent
 * gpad_run / gpad_run_scaled use the structure-exploiting kernel with the arithmetic of
 * StepTwoGPADFlatSequential / StepFourGPADFlatSequential (f32, shared matrices only). */
int gpad_setup_flat(gpad_handle_t h, const gpad_dims_t* dims, int n_u, const float* MGf,
                    const float* GLf, double L);

/* Bind the QP Hessian H (n x n row-major; dims.shared: one for the batch, else [batch][n][n];
 * dims.dtype / dims.memory of the bound problem; symmetric positive definite) and so enable the
 * value-function branches of Algorithm 1 (acceldualgrad.m:30-33,73,76) in later gpad_run /
 * gpad_run_state calls with tol > 0.  The QP is then min 1/2 z'Hz + f'z, G z <= g with f = H M
 * (M = H^-1 f is the vector gpad_run takes).  Which kernel evaluates the value functions:
 *   f64, shared matrices, n, m <= 256: the f64 MFMA panels (gpad_panel64.hip) when forced
 *     (GPAD_KERNEL_PANEL) or under AUTO from 16 instances per CU on (gpad_host.cpp, the f64
 *     panel branch of gpad_run); bit-identical to the f64 stream kernel, codes 3 / 4 included;
 *   otherwise (f32, f64 below that batch, distinct matrices, larger n or m): the stream kernel.
 * The f32 panel and the latency (resident / duo / flat) kernels do not evaluate the value
 * functions: with H bound, forcing GPAD_KERNEL_RESIDENT, or GPAD_KERNEL_PANEL where the f64
 * panels do not apply (f32, distinct matrices, n or m > 256), returns GPAD_ERR_UNSUPPORTED.
 * H = NULL unbinds.  gpad_setup / gpad_setup_scaled unbind as well.
 * Replaces acceldualgrad.m's own H (the MATLAB function receives H, :1). */
int gpad_setup_hessian(gpad_handle_t h, const void* H);

/* Run GPAD on the bound problem for every instance of the batch.
 *   z0: in z_{-1}, out z*      [batch][n]   (acceldualgrad.m:17, :83)
 *   y0: in y_0 = y_{-1}, out y* [batch][m]  (acceldualgrad.m:16)
 *   M : H^-1 q per instance    [batch][n]   (g_P, acceldualgrad.m:21)
 *   g : constraint rhs         [batch][m]   (b_i; p_D = -g/L, acceldualgrad.m:23)
 *   N : max iterations (reference: N_v = 100, main.cu:87)
 *   tol <= 0: exactly N iterations (paper Algorithm 2, main.cu behaviour);
 *   tol  > 0: Algorithm 1 test every check_every iterations (acceldualgrad.m:66-79), tol = e_g:
 *     (A) max(G z - g) <= tol                                  -> z* = z,    converged = 1
 *     (B) max(G zhat - g) <= tol, w >= 0, -w'(G zhat - g) <= e_V -> z* = zhat, converged = 2
 *     e_V = dims.tol_gap (default tol).  Both violation tests are decided on directly evaluated
 *     chains (G/L z, G/L zhat) with a rounding margin of 16 units of 2^-24 (f32) / 2^-53 (f64)
 *     of max_i |(G x)_i| + |g_i| / L, so a reported convergence holds for G z* - g evaluated
 *     exactly on the returned z*.  With H bound (gpad_setup_hessian) the value-function branches
 *     of acceldualgrad.m:73,76 follow where the MATLAB test reaches them -- after (B)'s
 *     violation part passed -- with valuefcn V(x) = (1/2 x'H + f) x and dualfcn D(y) = V(z(y)) +
 *     y'(G z(y) - g), z(y) = -ML y - M, evaluated in fp64 on the run's data:
 *     (B') w >= 0, -w'(G zhat - g) > e_V, -w'(G zhat - g) <= V(zhat) e_V/(1+e_V) -> z* = zhat, 3
 *     (B'') w not >= 0, V(zhat) - D(y+) <= e_V max(D(y+), 1)                  -> z* = zhat, 4
 *     Without H (the solve(...) surface carries no H, q) they are not evaluated.
 *   Certification floor: the margin above is at least 2^-20 max_i |g_i| (f32; f64: 2^-49), so
 *     a tol below tol_floor = 2^-20 max_{b,i} |g_{b,i}| can never certify an instance whose
 *     solution has an active constraint (G z* - g = 0 in some row) -- e.g. the reference's own
 *     e_g = 1e-6 (acceldualgrad.m:12) on data with |g| of order 10.  Such a run is not rejected
 *     (an instance with no active constraint can still pass) but flagged: st->tol_floor holds
 *     the floor of the run's data and st->flags GPAD_FLAG_TOL_FLOOR is set when tol < it.
 * Host memory: synchronous.  Device memory: enqueued on the handle's stream; synchronous only
 * when st != NULL (stats need the per-instance counters). */
int gpad_run(gpad_handle_t h, void* z0, void* y0, const void* M, const void* g, int N, double tol,
             gpad_stats_t* st);

/* gpad_run for gpad_setup_scaled problems: gP (g_P) and pD (p_D = -g/L) as in the data file,
 * optional per-iteration theta/beta tables (main.cu:61-64; float or double per dtype, length N;
 * NULL -> dims.schedule).  theta/beta are HOST arrays whatever dims.memory says (as main.cu:163,
 * 170 pass them by value per launch); the library copies them to the device. */
int gpad_run_scaled(gpad_handle_t h, void* z0, void* y0, const void* gP, const void* pD, int N,
                    double tol, const void* theta, const void* beta, gpad_stats_t* st);

/* ---- one-time QP precompute on the device ---------------------------
 * acceldualgrad.m:11,20-21 in fp64:  L = ||H||_F^2,  ML = inv(H) A' (n x m),  gP = inv(H) f' (n).
 * Replaces the MATLAB-side precompute (and the off-line data-file generator) that the reference
 * runs before main.cu:29-67 reads M_G, g_P.  shared = 1: one H (n x n) and one A (m x n) for the
 * whole batch (LTI) -> one ML, one L, and gP for each of the batch rows of f; shared = 0: H
 * [batch][n][n], A [batch][m][n] -> ML [batch][n][m], L [batch], gP [batch][n].  f (and gP) may
 * be NULL.  One workgroup per elimination of [H | A' | f'] (shared: [H | A' | I], then
 * gP = inv(H) f' row by row); H must be symmetric positive definite (no pivoting).  memory =
 * GPAD_MEM_HOST or GPAD_MEM_DEVICE for every pointer (device: on the handle's stream).
 * Synchronous.  The outputs feed gpad_setup (ML, A as G, L) and gpad_run (gP as M). */
int gpad_precompute(gpad_handle_t h, int n, int m, int batch, int shared, int memory, const double* H,
                    const double* A, const double* f, double* ML, double* gP, double* L);

/* ---- per-state QP data and closed-loop MPC -------------------
 * For an LTI plant the state-dependent QP data are affine in the state x (nx):
 *   M(x) = M0 + PM x   (n;  PM = H^-1 F': the reference forms f = x0'F, gpad.m:81, and
 *                            g_P = H^-1 f', acceldualgrad.m:21, on the host every MPC step)
 *   g(x) = g0 + Pg x   (m;  b_i(x0), gpad.m:85)
 * and the receding-horizon update is x+ = A x + B u with u = z*[0:nu] (gpad.m:91-93).
 * gpad_setup_plant binds PM (n x nx), Pg (m x nx), optional M0 (n) / g0 (m) (NULL = 0) and,
 * for closed-loop runs, A (nx x nx) and B (nx x nu).  Row-major, dims.dtype / dims.memory of
 * the preceding gpad_setup, whose ML/G/L the solves use.  The fp32 evaluation order is
 * acc = c0; acc = fma(P[i][k], x[k], acc) for k = 0..nx-1 (and A then B for the update). */
int gpad_setup_plant(gpad_handle_t h, int nx, int nu, const void* PM, const void* M0, const void* Pg,
                     const void* g0, const void* A, const void* B);

/* gpad_run with M = M(x), g = g(x) evaluated on the device for every instance's state
 * x [batch][nx] (no host round trip for the per-state precompute). */
int gpad_run_state(gpad_handle_t h, const void* x, void* z0, void* y0, int N, double tol,
                   gpad_stats_t* st);

/* Closed-loop simulation of gpad.m:79-95 on the device, for every instance of the batch:
 *   for t < steps:  M, g <- M(x), g(x);  z, y <- 0 (warm == 0, acceldualgrad.m:16-17) or kept
 *                   from the previous step (warm != 0);  GPAD(N, tol);
 *                   xs[t] = x;  us[t] = u = z*[0:nu];  x <- A x + B u
 * x [batch][nx]: in x_0, out x_steps.  z [batch][n], y [batch][m]: the last step's solution.
 * xs [steps][batch][nx], us [steps][batch][nu]: optional trajectories (NULL to skip).
 * st->iters and st->codes, when given, receive [steps][batch] iteration counts and termination
 * codes (size both arrays steps * batch); the other stats aggregate over every (step, instance);
 * kernel_ms times the whole loop. */
int gpad_closed_loop(gpad_handle_t h, void* x, void* z, void* y, int steps, int N, double tol, int warm,
                     void* xs, void* us, gpad_stats_t* st);

/* ---- reference data-file boundary (main.cu:29-67 readData) ------------------------------
 * Text file: "n_u N m num_iterations L", then M_G (n*m), g_P (n), G_L (n*m), p_D (m),
 * theta (num_iterations), beta (num_iterations), n = n_u*N, whitespace-separated floats.
 * M_G = -H^-1 G' (sign-folded), G_L = G/L, p_D = -g/L: the gpad_setup_scaled/run_scaled
 * inputs.  The file's matrix layout is the reference build's choice: GPAD_FILE_ROWMAJOR is
 * seq_functions.cpp's (M_G[i*m+j], G_L[i*n+j]); GPAD_FILE_FLIPPED is kernel_functions.cu's
 * ENABLE_FLIPPING layout (M_G[j*n+i], G_L[j*m+i]).  The struct always holds the row-major
 * mathematical orientation (M_G n x m, G_L m x n). */
#define GPAD_FILE_ROWMAJOR 0
#define GPAD_FILE_FLIPPED 1
#define GPAD_FILE_FLAT 2 /* ENABLE_FLATTEN_MATRICES files: M_G is N x m, G_L is m x N (flat) */

typedef struct gpad_datafile {
    int n_u, N, m, num_iterations;
    float L;
    float* M_G;   /* n x m  (GPAD_FILE_FLAT: N x m) */
    float* g_P;   /* n */
    float* G_L;   /* m x n  (GPAD_FILE_FLAT: m x N) */
    float* p_D;   /* m */
    float* theta; /* num_iterations */
    float* beta;  /* num_iterations */
} gpad_datafile_t;

/* Allocates the arrays (release with gpad_datafile_free).  GPAD_ERR_INVALID on a malformed or
 * truncated file (the reference's readData only perror()s and continues). */
int gpad_datafile_read(const char* path, int layout, gpad_datafile_t* out);
int gpad_datafile_write(const char* path, int layout, const gpad_datafile_t* f);
void gpad_datafile_free(gpad_datafile_t* f);

/* Per-instance iteration counts / convergence flags of the last run (device work finished). */
int gpad_last_stats(gpad_handle_t h, gpad_stats_t* st);

/* Enqueue, on the handle's stream, acc[0] += the sum of the last run's per-instance iteration
 * counts (acc: one device int64).  Lets a caller count the work of back-to-back asynchronous
 * runs without a host synchronisation per run (bench.py's timed loop). */
int gpad_accumulate_iterations(gpad_handle_t h, long long* acc);

/* Diagnostics (no reference counterpart): the phase plan the next phased panel solve of this
 * handle will follow, made from the previous solve's iteration counts by gpad_last_stats / a
 * stats-collecting run.  Writes up to cap phase ends (iterations; the last is N) and finisher
 * thresholds, and the modelled solve time in us; returns the number of phases (0: no plan,
 * the default schedule applies). */
int gpad_phase_plan(gpad_handle_t h, int* ends, int* fins, int cap, double* cost_us);
/* Diagnostics: the survivors each boundary of the last phased panel solve listed -- counts[ph] =
 * instances still running after phase ph (the next phase's input) -- for up to cap phases
 * (synchronises the handle's stream).  Returns the number written, 0 when the last run was not a
 * phased panel solve. */
int gpad_phase_counts(gpad_handle_t h, int* counts, int cap);
/* Diagnostics: the phases the last phased panel solve of this handle actually launched -- ends[ph]
 * (iterations), fins[ph] (the finisher threshold at the start of phase ph: the finisher takes phase
 * ph's list when counts[ph - 1] <= fins[ph]; 0 = none) and counts[ph] (survivors after phase ph, as
 * gpad_phase_counts) -- for up to cap phases (any array may be NULL; counts synchronises the stream);
 * *prior (may be NULL) = 1 when the solve followed the shape's plan prior (a handle without a plan
 * of its own: gpad_run).  Returns the number of phases written, 0 when the last run was not a phased
 * panel solve. */
int gpad_last_phases(gpad_handle_t h, int* ends, int* fins, int* counts, int cap, int* prior);
/* The planner itself on given iteration counts (host only, no device work; for tests/tools). */
int gpad_plan_phases(const int* iters, int batch, int n, int m, int N, int check_every, int num_cus,
                     int* ends, int* fins, int cap, double* cost_us);

/* One-shot north-star surface: solve(z0, y0, ML, M, G, g, N, L, tol).  Equivalent to
 * create + setup + run + destroy (the handle is cached per thread and device). */
int gpad_solve(void* z0, void* y0, const void* ML, const void* M, const void* G, const void* g,
               int N, double L, double tol, const gpad_dims_t* dims, gpad_stats_t* st);
/* Free the calling thread's cached gpad_solve handle and gpad_solve_sharded group (device memory,
 * streams, RCCL communicators).  Call it before a thread that used them exits; the caches are
 * never freed from a thread-exit destructor (at process exit the OS reclaims them). */
void gpad_release_cached(void);

/* ---- multi-device: instance shards, RCCL scatter/gather ------------------
 * A group drives several devices from ONE C process (the reference's caller is a single C
 * program, main.cu:79-203; north_star: "partition across the 8 GPUs of one node by sharding
 * independent MPC problem instances with a single RCCL gather of solutions").  One handle and
 * HIP stream per device; the batch splits into contiguous shards (sizes differ by at most one,
 * larger first) solved with no communication.  dims.memory == GPAD_MEM_DEVICE: every pointer is
 * device memory on devices[0] (the root); shared ML/G are broadcast at setup (ncclBroadcast),
 * per-instance matrices and each non-root shard of M, g, z0, y0 go out by one grouped
 * ncclSend/ncclRecv, and (z*, y*) come back into the root buffers by another.  GPAD_MEM_HOST:
 * every device copies its own shard in and out.  With distinct devices the group holds one RCCL
 * clique (ncclCommInitAll); a device listed twice (one GPU standing in for several) moves the
 * same bytes by peer copies instead (gpad_group_transport tells which).  librccl is loaded on the
 * first group over distinct devices (not linked: single-GPU users need no RCCL); when it cannot
 * be loaded such a group uses the peer copies too. */
typedef struct gpad_group_s* gpad_group_t;
#define GPAD_GROUP_RCCL 1
#define GPAD_GROUP_PEER 2
int gpad_group_create(gpad_group_t* g, int ndev, const int* devices);
int gpad_group_destroy(gpad_group_t g);
int gpad_group_transport(gpad_group_t g); /* GPAD_GROUP_RCCL or GPAD_GROUP_PEER */
/* Integration / test hook: groups created after this call (gpad_group_create, gpad_solve_sharded)
 * take their RCCL entry points (ncclCommInitAll, ncclCommDestroy, ncclGroupStart / End, ncclSend,
 * ncclRecv, ncclBroadcast, ncclGetErrorString) from the shared library at `path` (NULL: the default
 * librccl).  force_rccl != 0: they use the RCCL transport even when a device is listed twice (for a
 * library that accepts it -- real RCCL refuses duplicate devices, so the group creation then fails).
 * Returns GPAD_OK, or GPAD_ERR_UNSUPPORTED when the library or one of the symbols cannot be loaded;
 * such groups then use the peer copies.  Existing groups keep the library they were created with. */
int gpad_group_rccl_library(const char* path, int force_rccl);
/* Device memory: the stream of devices[0] on which the caller produces / consumes the buffers it
 * passes (NULL, the default: the null stream).  Setup and run first make every device stream of
 * the group wait for the work queued on it so far; runs are synchronous, so the results are
 * complete when gpad_group_run returns. */
int gpad_group_set_stream(gpad_group_t g, void* hip_stream);
/* dims.batch is the WHOLE batch (as for gpad_setup); ML, G as gpad_setup's. */
int gpad_group_setup(gpad_group_t g, const gpad_dims_t* dims, const void* ML, const void* G, double L);
/* The whole batch's vectors (gpad_run's meaning).  Synchronous.  st aggregates every shard
 * (kernel_ms: the slowest shard's device time); st->iters, when given, receives [batch] counts. */
int gpad_group_run(gpad_group_t g, void* z0, void* y0, const void* M, const void* g_rhs, int N, double tol,
                   gpad_stats_t* st);
/* One-shot solve(...) over several devices (the group is cached per thread and device list). */
int gpad_solve_sharded(int ndev, const int* devices, void* z0, void* y0, const void* ML, const void* M,
                       const void* G, const void* g, int N, double L, double tol, const gpad_dims_t* dims,
                       gpad_stats_t* st);

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
/* flat battery steps (device pointers; MGf N x m, GLf m x N):
 * StepTwoGPADFlatSequential seq_functions.cpp:5-20 / StepFourGPADFlatParRows kernel_functions.cu:74-109
 * (with the CPU step's projection y < 0 -> 0, seq_functions.cpp:40-42). */
int gpad_step2_primal_flat(gpad_handle_t h, const float* MGf, const float* w, const float* gP,
                           float* zhat, int N, int n_u, int m);
int gpad_step4_project_flat(gpad_handle_t h, const float* GLf, float* yp1, const float* w,
                            const float* pD, const float* zhat, int N, int n_u, int m);
/* 8e (host): theta[v], beta[v] for v < N   -- acceldualgrad.m:18,27,55-56 / main.cu:61-64    */
int gpad_schedule(int N, int kind, double* theta, double* beta);

/* ---- schedule / launch tuning (no reference counterpart) ---------------------------------
 * Per-handle options for tests, diagnostics and A/B tools.  None changes any result: they move
 * phase boundaries, cap grids, reorder the finisher's queue or choose where operands are staged.
 * value GPAD_OPT_DEFAULT restores the default.  Returns GPAD_ERR_INVALID for an unknown option
 * or an out-of-range value. */
#define GPAD_OPT_DEFAULT (-1)
#define GPAD_OPT_PHASE_LEN 1       /* panel phase length in iterations (default 4 * check_every,
                                    * doubling after the 10th phase; set: uniform, with PLAN 0);
                                    * flat panels: the first phase                                  */
#define GPAD_OPT_FINISH_THRESH 2   /* survivors at which the finisher takes over (default 2/CU)    */
#define GPAD_OPT_PLAN 3            /* 1: plan phases from the previous solve's counts (default)    */
#define GPAD_OPT_PHASED 4          /* 1: phased compaction of tol > 0 panel solves (default; flat
                                    * panels: from 4 panels per CU), 2: always, 0: one launch       */
/* 5 (finisher kind), 13 (solo finisher workgroups), 15 (plan finisher cost): retired in 0.3 after
 * measuring no gain; 14 (condensed panels): removed with the condensed operator in
 * 0.4; 17: the round-4 pair layouts (W32, TailPair) measured slower and left out of 0.4; 20 (panel
 * dataflow GEMM boundaries, 2-4 % slower) and 21 (finisher slot hand-off mailbox, even at the step
 * level): built and measured in round 5, removed in 0.5; setting any of them
 * returns GPAD_ERR_INVALID                                                                       */
#define GPAD_OPT_LPT 6             /* 1: longest-predicted-first finisher queue (default)          */
#define GPAD_OPT_PANEL_MAX_GRID 7  /* cap on the panel grid, workgroups (0 = none, default)        */
#define GPAD_OPT_DUO_MAX_GRID 8    /* cap on the finisher grid (0 = none, default)                 */
#define GPAD_OPT_FLAT_PANEL_MIN 9  /* batch from which flat setups run the flat panels (default 8/CU) */
#define GPAD_OPT_FLAT_PANELS 10    /* panels per flat-panel workgroup, 1..4 (0 = auto, default)    */
#define GPAD_OPT_FLAT_WAVES 11     /* flat-panel workgroup waves: 0 auto (default), 8 or 16         */
#define GPAD_OPT_FLAT_A_LDS 12     /* 1: flat fragment image staged in LDS when it fits (default)  */
#define GPAD_OPT_DEBUG_DROP_HANDOFF 16 /* test only (fault injection): 1 = every panel solve that
                                    * uses the chain hand-off withholds its first post, so the
                                    * receiver's bounded wait expires and the run ends in
                                    * GPAD_ERR_DEVICE; 0 (default) = off.  Honoured by the
                                    * 193..208-row shapes (the C3/C4 tiling, T = 13), which run
                                    * a separate test-only kernel instantiation while it is set */
#define GPAD_OPT_P64_RELAY 18      /* 1: f64 panels at T = 9, 13 (n, m in (128, 144], (192, 208]) run
                                    * the 16-wave relay layout (default); 0: one wave per tile */
#define GPAD_OPT_P64_REFILL 19     /* 1: f64 panel solves with tol > 0, N a multiple of check_every and
                                    * more panels than workgroups refill a finished column with the
                                    * next instance (default); 0: each panel runs to its slowest column */
int gpad_set_option(gpad_handle_t h, int option, int value);

/* Synchronise the handle's stream (for callers using device memory + async runs). */
int gpad_sync(gpad_handle_t h);

#ifdef __cplusplus
}
#endif
#endif /* GPAD_H */
