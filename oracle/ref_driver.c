/*
 * ref_driver.c -- loop driver around the REFERENCE's own CPU steps (TEST INFRASTRUCTURE).
 *
 * Linked by `make -C oracle ref` together with the reference's seq_functions.cpp (compiled in
 * place from /root/reference, never copied) into oracle/_ref/libref_seq.so.  It composes the
 * reference's StepOne..StepFour functions in the loop order of main.cu:160-175 (fixed N
 * iterations, y-history rotation of main.cu:167) so bench.py can time the reference's own
 * arithmetic on the host (cpu_baseline kind "reference") without Python per-step overhead.
 */
#include <stdlib.h>
#include <string.h>

#include "seq_functions.h"

#ifdef _OPENMP
#include <omp.h>
#endif

/* One instance: z in z_{-1} / out z; y in y0 / out y.  MGneg is n x m (sign-folded M_G as
 * main.cu reads it), GL is m x n; theta/beta are the per-iteration tables (main.cu:61-64). */
void ref_solve_f32(float* z, float* y, const float* MGneg, const float* gP, const float* GL,
                   const float* pD, int n, int m, int N, const float* theta, const float* beta) {
    float* buf = (float*)malloc(sizeof(float) * ((size_t)4 * m + n + 4));
    float* ycur = buf;
    float* yprev = ycur + m;
    float* w = yprev + m;
    float* ynew = w + m;
    float* zhat = ynew + m;
    memcpy(ycur, y, sizeof(float) * m);
    memcpy(yprev, y, sizeof(float) * m);
    for (int v = 0; v < N; v++) {
        StepOneGPADSequential(ycur, yprev, w, beta[v], m);
        StepTwoGPADSequential(MGneg, w, gP, zhat, n, 1, m);
        StepThreeGPADSequential(theta[v], n, z, zhat, z);
        StepFourGPADSequential(GL, ynew, w, pD, zhat, n, 1, m);
        float* t = yprev;
        yprev = ycur;
        ycur = ynew;
        ynew = t;
    }
    memcpy(y, ycur, sizeof(float) * m);
    free(buf);
}

/* Batch of instances sharing MGneg/GL (shared != 0) or with per-instance matrices, spread over
 * `threads` OpenMP threads (one instance per thread at a time). */
void ref_solve_batch_f32(float* Z, float* Y, const float* MGneg, const float* GP, const float* GL,
                         const float* PD, int n, int m, int batch, int shared, int N,
                         const float* theta, const float* beta, int threads) {
    const size_t nm = (size_t)n * m;
#ifdef _OPENMP
#pragma omp parallel for schedule(dynamic, 1) num_threads(threads > 0 ? threads : omp_get_max_threads())
#endif
    for (int b = 0; b < batch; b++) {
        ref_solve_f32(Z + (size_t)b * n, Y + (size_t)b * m, shared ? MGneg : MGneg + b * nm,
                      GP + (size_t)b * n, shared ? GL : GL + b * nm, PD + (size_t)b * m, n, m, N,
                      theta, beta);
    }
    (void)threads;
}

/* The reference's FLAT battery steps (seq_functions.cpp:5-43, ENABLE_FLATTEN_MATRICES) in the
 * main_prof.cu loop order: MGf is Nh x m, GLf is m x Nh. */
void ref_solve_flat_f32(float* z, float* y, const float* MGf, const float* gP, const float* GLf,
                        const float* pD, int Nh, int n_u, int m, int N, const float* theta,
                        const float* beta) {
    const int n = n_u * Nh;
    float* buf = (float*)malloc(sizeof(float) * ((size_t)4 * m + n + 4));
    float* ycur = buf;
    float* yprev = ycur + m;
    float* w = yprev + m;
    float* ynew = w + m;
    float* zhat = ynew + m;
    memcpy(ycur, y, sizeof(float) * m);
    memcpy(yprev, y, sizeof(float) * m);
    for (int v = 0; v < N; v++) {
        StepOneGPADSequential(ycur, yprev, w, beta[v], m);
        StepTwoGPADFlatSequential(MGf, w, gP, zhat, Nh, n_u, m);
        StepThreeGPADSequential(theta[v], n, z, zhat, z);
        StepFourGPADFlatSequential(GLf, ynew, w, pD, zhat, Nh, n_u, m);
        float* t = yprev;
        yprev = ycur;
        ycur = ynew;
        ynew = t;
    }
    memcpy(y, ycur, sizeof(float) * m);
    free(buf);
}
