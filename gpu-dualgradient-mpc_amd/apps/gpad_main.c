/*
 * gpad_main.c -- the reference's host driver (Code/CUDA/FinalProject/main.cu:79-203) on
 * libgpad: read one data file (main.cu:29-67 format), run N_v GPAD iterations from
 * y = y_{-1} = 0, z_{-1} = 0 (main.cu:69-77), print the result and the device time.
 *
 * usage: gpad_main <datafile> [--flipped] [--iters N_v] [--tol eps] [--device d]
 *                           [--one-shot] [--repeat R]
 *   --flipped : the file stores kernel_functions.cu ENABLE_FLIPPING layouts
 *   --iters   : iteration count (reference: N_v = 100, main.cu:87); must be <= the file's
 *               num_iterations, whose theta/beta tables drive the run as in main.cu:163,170
 *   --tol     : > 0 enables the Algorithm 1 termination test (the reference has none)
 *   --one-shot: call the north-star gpad_solve(z0, y0, ML, M, G, g, N, L, tol) instead of the
 *               handle API, on the unscaled problem recovered from the file (ML = -M_G,
 *               M = g_P, G = L G_L, g = -L p_D, in fp64 then rounded to float) with the
 *               library's own theta/beta schedule (the same recursion as the file's tables)
 *   --repeat R: one-shot only: call gpad_solve R more times on the same inputs and print the
 *               mean wall time per call ("solve_us", host clock around each synchronous call)
 *   --scenarios B [--devices D | --devices a,b,c]: a battery-scenario batch of B instances of the
 *               file's problem (shared ML, G; instance b's g_P scaled by 1 + 1e-3 ((31 b + i) mod 17))
 *               solved over D devices (default: every visible one) with gpad_solve_sharded -- the
 *               main.cu-shaped C caller using all GPUs of a node, no Python; prints the batch's
 *               iteration total, converged count, wall ms and an FNV-1a hash of the z*, y* bits
 * Output: "n_u N m", "iterations", "kernel_ms", then "z" and "y" lines with %.9g values.
 */
#define _POSIX_C_SOURCE 199309L
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "gpad.h"

static int die(int rc, const char* where) {
    fprintf(stderr, "gpad_main: %s: %s (%s)\n", where, gpad_strerror(rc), gpad_last_error());
    return 1;
}

int main(int argc, char** argv) {
    if (argc < 2) {
        fprintf(stderr, "usage: %s <datafile> [--flipped] [--iters N] [--tol eps] [--device d]\n", argv[0]);
        return 2;
    }
    const char* path = argv[1];
    int layout = GPAD_FILE_ROWMAJOR, N_v = 100, device = 0, one_shot = 0, repeat = 0, scenarios = 0;
    int devs[64], ndev = 0;
    double tol = 0.0;
    for (int a = 2; a < argc; a++) {
        if (!strcmp(argv[a], "--flipped")) layout = GPAD_FILE_FLIPPED;
        else if (!strcmp(argv[a], "--iters") && a + 1 < argc) N_v = atoi(argv[++a]);
        else if (!strcmp(argv[a], "--tol") && a + 1 < argc) tol = atof(argv[++a]);
        else if (!strcmp(argv[a], "--device") && a + 1 < argc) device = atoi(argv[++a]);
        else if (!strcmp(argv[a], "--one-shot")) one_shot = 1;
        else if (!strcmp(argv[a], "--repeat") && a + 1 < argc) repeat = atoi(argv[++a]);
        else if (!strcmp(argv[a], "--scenarios") && a + 1 < argc) scenarios = atoi(argv[++a]);
        else if (!strcmp(argv[a], "--devices") && a + 1 < argc) {
            const char* s = argv[++a];
            if (!strchr(s, ',')) {  /* a count: devices 0 .. D-1 */
                ndev = atoi(s);
                for (int k = 0; k < ndev && k < 64; k++) devs[k] = k;
            } else {                 /* an explicit list (may repeat a device) */
                for (char* p = (char*)s; *p && ndev < 64;) {
                    devs[ndev++] = (int)strtol(p, &p, 10);
                    if (*p == ',') p++;
                }
            }
        }
        else {
            fprintf(stderr, "gpad_main: unknown argument %s\n", argv[a]);
            return 2;
        }
    }
    gpad_datafile_t f;
    int rc = gpad_datafile_read(path, layout, &f);
    if (rc) return die(rc, "read");
    if (N_v < 0 || N_v > f.num_iterations) {
        fprintf(stderr, "gpad_main: --iters %d exceeds the file's %d theta/beta entries\n", N_v,
                f.num_iterations);
        gpad_datafile_free(&f);
        return 2;
    }
    const int n = f.n_u * f.N, m = f.m;
    float* z = (float*)calloc((size_t)n, sizeof(float)); /* z_{-1} = 0      (main.cu:69-77) */
    float* y = (float*)calloc((size_t)m, sizeof(float)); /* y_0 = y_{-1} = 0                */
    gpad_dims_t d;
    memset(&d, 0, sizeof(d));
    d.n = n;
    d.m = m;
    d.batch = 1;
    d.shared = 1;
    d.dtype = GPAD_DTYPE_F32;
    d.memory = GPAD_MEM_HOST;
    d.schedule = GPAD_SCHEDULE_MATLAB;
    d.check_every = 10;
    d.kernel = GPAD_KERNEL_AUTO;
    gpad_handle_t h = NULL;
    gpad_stats_t st;
    memset(&st, 0, sizeof(st));
    int ret = 0;
    double solve_us = -1.0;
    if (scenarios > 0) {  /* the scenario batch over several devices (gpad_solve_sharded) */
        if (ndev <= 0) {
            ndev = gpad_device_count();
            if (ndev <= 0) return die(ndev < 0 ? ndev : GPAD_ERR_NO_DEVICE, "device count");
            if (ndev > 64) ndev = 64;
            for (int k = 0; k < ndev; k++) devs[k] = k;
        }
        const int B = scenarios;
        const size_t nm = (size_t)n * m;
        float* ML = (float*)malloc(sizeof(float) * nm);
        float* G = (float*)malloc(sizeof(float) * nm);
        float* M = (float*)malloc(sizeof(float) * (size_t)B * n);
        float* g = (float*)malloc(sizeof(float) * (size_t)B * m);
        float* Z = (float*)calloc((size_t)B * n, sizeof(float));
        float* Y = (float*)calloc((size_t)B * m, sizeof(float));
        for (size_t k = 0; k < nm; k++) {
            ML[k] = -f.M_G[k];
            G[k] = (float)((double)f.L * (double)f.G_L[k]);
        }
        for (int b = 0; b < B; b++) {
            for (int i = 0; i < n; i++)
                M[(size_t)b * n + i] = (float)((double)f.g_P[i] * (1.0 + 1e-3 * (double)((31 * b + i) % 17)));
            for (int i = 0; i < m; i++) g[(size_t)b * m + i] = (float)(-(double)f.L * (double)f.p_D[i]);
        }
        d.batch = B;
        struct timespec t0, t1;
        clock_gettime(CLOCK_MONOTONIC, &t0);
        rc = gpad_solve_sharded(ndev, devs, Z, Y, ML, M, G, g, N_v, (double)f.L, tol, &d, &st);
        clock_gettime(CLOCK_MONOTONIC, &t1);
        if (rc) ret = die(rc, "gpad_solve_sharded");
        else {
            unsigned long long hsh = 1469598103934665603ull;
            const unsigned char* pz = (const unsigned char*)Z;
            const unsigned char* py = (const unsigned char*)Y;
            for (size_t k = 0; k < sizeof(float) * (size_t)B * n; k++) hsh = (hsh ^ pz[k]) * 1099511628211ull;
            for (size_t k = 0; k < sizeof(float) * (size_t)B * m; k++) hsh = (hsh ^ py[k]) * 1099511628211ull;
            printf("scenarios %d devices %d\n", B, ndev);
            printf("total_iterations %lld converged %d\n", st.total_iterations, st.converged);
            printf("wall_ms %.3f\n", (double)(t1.tv_sec - t0.tv_sec) * 1e3 + (double)(t1.tv_nsec - t0.tv_nsec) * 1e-6);
            printf("hash %016llx\n", hsh);
        }
        free(ML);
        free(G);
        free(M);
        free(g);
        free(Z);
        free(Y);
        gpad_datafile_free(&f);
        free(z);
        free(y);
        return ret;
    }
    if (one_shot) {
        /* the unscaled problem: ML = -M_G, G = L G_L, g = -L p_D (acceldualgrad.m:20-23 undone) */
        const size_t nm = (size_t)n * m;
        float* ML = (float*)malloc(sizeof(float) * nm);
        float* G = (float*)malloc(sizeof(float) * nm);
        float* g = (float*)malloc(sizeof(float) * (size_t)m);
        float* z1 = (float*)malloc(sizeof(float) * (size_t)n);
        float* y1 = (float*)malloc(sizeof(float) * (size_t)m);
        for (size_t k = 0; k < nm; k++) {
            ML[k] = -f.M_G[k];
            G[k] = (float)((double)f.L * (double)f.G_L[k]);
        }
        for (int i = 0; i < m; i++) g[i] = (float)(-(double)f.L * (double)f.p_D[i]);
        if ((rc = gpad_solve(z, y, ML, f.g_P, G, g, N_v, (double)f.L, tol, &d, &st))) ret = die(rc, "gpad_solve");
        if (!ret && repeat > 0) {
            struct timespec t0, t1;
            double tot = 0.0;
            for (int r = 0; r < repeat && !ret; r++) {
                memset(z1, 0, sizeof(float) * (size_t)n);
                memset(y1, 0, sizeof(float) * (size_t)m);
                clock_gettime(CLOCK_MONOTONIC, &t0);
                rc = gpad_solve(z1, y1, ML, f.g_P, G, g, N_v, (double)f.L, tol, &d, NULL);
                clock_gettime(CLOCK_MONOTONIC, &t1);
                if (rc) ret = die(rc, "gpad_solve (repeat)");
                else if (memcmp(z1, z, sizeof(float) * (size_t)n) || memcmp(y1, y, sizeof(float) * (size_t)m)) {
                    fprintf(stderr, "gpad_main: repeated gpad_solve differs from the first call\n");
                    ret = 1;
                }
                tot += (double)(t1.tv_sec - t0.tv_sec) * 1e6 + (double)(t1.tv_nsec - t0.tv_nsec) * 1e-3;
            }
            solve_us = tot / repeat;
        }
        free(ML);
        free(G);
        free(g);
        free(z1);
        free(y1);
    } else if ((rc = gpad_create(&h, device, NULL))) ret = die(rc, "create");
    else if ((rc = gpad_setup_scaled(h, &d, f.M_G, f.G_L, (double)f.L))) ret = die(rc, "setup");
    else if ((rc = gpad_run_scaled(h, z, y, f.g_P, f.p_D, N_v, tol, f.theta, f.beta, &st)))
        ret = die(rc, "run");
    if (!ret) {
        printf("%d %d %d\n", f.n_u, f.N, f.m);
        printf("iterations %d converged %d\n", st.iterations, st.converged);
        printf("kernel_ms %.6f\n", st.kernel_ms);
        if (solve_us >= 0.0) printf("solve_us %.3f\n", solve_us);
        printf("z");
        for (int i = 0; i < n; i++) printf(" %.9g", (double)z[i]);
        printf("\ny");
        for (int i = 0; i < m; i++) printf(" %.9g", (double)y[i]);
        printf("\n");
    }
    if (h) gpad_destroy(h);
    gpad_datafile_free(&f);
    free(z);
    free(y);
    return ret;
}
