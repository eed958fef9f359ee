/*
 * gpad_main.c -- the reference's host driver (Code/CUDA/FinalProject/main.cu:79-203) on
 * libgpad: read one data file (main.cu:29-67 format), run N_v GPAD iterations from
 * y = y_{-1} = 0, z_{-1} = 0 (main.cu:69-77), print the result and the device time.
 *
 * usage: gpad_main <datafile> [--flipped] [--iters N_v] [--tol eps] [--device d]
 *   --flipped : the file stores kernel_functions.cu ENABLE_FLIPPING layouts
 *   --iters   : iteration count (reference: N_v = 100, main.cu:87); must be <= the file's
 *               num_iterations, whose theta/beta tables drive the run as in main.cu:163,170
 *   --tol     : > 0 enables the Algorithm 1 termination test (the reference has none)
 * Output: "n_u N m", "iterations", "kernel_ms", then "z" and "y" lines with %.9g values.
 */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

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
    int layout = GPAD_FILE_ROWMAJOR, N_v = 100, device = 0;
    double tol = 0.0;
    for (int a = 2; a < argc; a++) {
        if (!strcmp(argv[a], "--flipped")) layout = GPAD_FILE_FLIPPED;
        else if (!strcmp(argv[a], "--iters") && a + 1 < argc) N_v = atoi(argv[++a]);
        else if (!strcmp(argv[a], "--tol") && a + 1 < argc) tol = atof(argv[++a]);
        else if (!strcmp(argv[a], "--device") && a + 1 < argc) device = atoi(argv[++a]);
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
    if ((rc = gpad_create(&h, device, NULL))) ret = die(rc, "create");
    else if ((rc = gpad_setup_scaled(h, &d, f.M_G, f.G_L, (double)f.L))) ret = die(rc, "setup");
    else if ((rc = gpad_run_scaled(h, z, y, f.g_P, f.p_D, N_v, tol, f.theta, f.beta, &st)))
        ret = die(rc, "run");
    if (!ret) {
        printf("%d %d %d\n", f.n_u, f.N, f.m);
        printf("iterations %d converged %d\n", st.iterations, st.converged);
        printf("kernel_ms %.6f\n", st.kernel_ms);
        printf("z");
        for (int i = 0; i < n; i++) printf(" %.9g", (double)z[i]);
        printf("\ny");
        for (int i = 0; i < m; i++) printf(" %.9g", (double)y[i]);
        printf("\n");
    }
    gpad_destroy(h);
    gpad_datafile_free(&f);
    free(z);
    free(y);
    return ret;
}
