/* mapchain_oracle.c — TEST INFRASTRUCTURE ONLY (see pqd_oracle.h).
 * One-to-one C restatement of the reference's Fortran sweep kernels. Index arithmetic keeps the
 * Fortran 1-based indices where it matters, so each loop can be read next to its source line.
 * Layouts: map stacks and ops are Fortran column-major exactly as the reference callers pass them.
 */
#include "pqd_oracle.h"
#include <math.h>
#include <stdlib.h>
#include <string.h>

#define FMAP(base, N2, m1) ((base) + (size_t)((m1) - 1) * (N2) * (N2)) /* 1-based map index */

/* y = A x, A column-major N2 x N2 (zgemv 'N') */
static void gemv(int N2, const ocplx* A, const ocplx* x, ocplx* y) {
    for (int r = 0; r < N2; ++r) y[r] = 0;
    for (int c = 0; c < N2; ++c) {
        ocplx xc = x[c];
        const ocplx* col = A + (size_t)c * N2;
        for (int r = 0; r < N2; ++r) y[r] += col[r] * xc;
    }
}

/* C = A B for column-major dim x dim (Fortran matmul) */
static void matmul(int n, const ocplx* A, const ocplx* B, ocplx* Cm) {
    for (int j = 0; j < n; ++j)
        for (int i = 0; i < n; ++i) {
            ocplx s = 0;
            for (int k = 0; k < n; ++k) s += A[i + k * n] * B[k + j * n];
            Cm[i + j * n] = s;
        }
}

static ocplx trace(int n, const ocplx* A) {
    ocplx s = 0;
    for (int l = 0; l < n; ++l) s += A[l + l * n];
    return s;
}

/* Tr(opA * opB * opC * rho): tmp = C rho; tmp = B tmp; tmp = A tmp   (propagate_tau.f90:154-158) */
static ocplx tr_abc_rho(int dim, const ocplx* A, const ocplx* B, const ocplx* Cm, const ocplx* rho,
                        ocplx* t1, ocplx* t2) {
    matmul(dim, Cm, rho, t1);
    matmul(dim, B, t1, t2);
    matmul(dim, A, t2, t1);
    return trace(dim, t1);
}

/* propagate_tau.f90:3-19 */
void or_propagate_tau(const ocplx* dm_tl, const ocplx* rho_init, int n_tau, int dim, int j_start,
                      ocplx* rho_out) {
    int N2 = dim * dim;
    memcpy(rho_out, rho_init, sizeof(ocplx) * N2);
    for (int k = 1; k <= n_tau; ++k)
        gemv(N2, FMAP(dm_tl, N2, j_start + k), rho_out + (size_t)(k - 1) * N2, rho_out + (size_t)k * N2);
}

/* propagate_tau.f90:110-187 */
void or_calc_onetime_parallel(const ocplx* dm_tl, const ocplx* rho_init, int n_tau, int n_t, int n_tfull,
                              int dim, const ocplx* opA, const ocplx* opB, const ocplx* opC,
                              const double* time, const double* time_sparse, ocplx* result, int nthreads) {
    int N2 = dim * dim;
    ocplx* rho_vec = malloc(sizeof(ocplx) * N2);
    ocplx* rho_res = malloc(sizeof(ocplx) * N2);
    ocplx* t1 = malloc(sizeof(ocplx) * N2);
    ocplx* t2 = malloc(sizeof(ocplx) * N2);
    ocplx* rho_buffer = malloc(sizeof(ocplx) * N2 * (size_t)n_t);
    int* j_array = malloc(sizeof(int) * n_t);
    memcpy(rho_vec, rho_init, sizeof(ocplx) * N2);
    result[0] = tr_abc_rho(dim, opA, opB, opC, rho_vec, t1, t2);
    int j = 1;
    for (int i = 1; i <= n_t; ++i) {
        while (j <= n_tfull && time[j - 1] < time_sparse[i - 1]) { /* :144 */
            gemv(N2, FMAP(dm_tl, N2, j), rho_vec, rho_res);
            memcpy(rho_vec, rho_res, sizeof(ocplx) * N2);
            ++j;
        }
        result[(i - 1)] = tr_abc_rho(dim, opA, opB, opC, rho_vec, t1, t2); /* :154-158 */
        matmul(dim, opC, rho_vec, t1); /* :161-162: C rho A */
        matmul(dim, t1, opA, rho_buffer + (size_t)(i - 1) * N2);
        j_array[i - 1] = j;
    }
#pragma omp parallel for num_threads(nthreads > 0 ? nthreads : 1) schedule(dynamic)
    for (int i = 1; i <= n_t; ++i) { /* :170-184 */
        ocplx rr[1296], tmpv[1296], tm[1296];
        memcpy(rr, rho_buffer + (size_t)(i - 1) * N2, sizeof(ocplx) * N2);
        int jj = j_array[i - 1];
        for (int k = 2; k <= n_tau + 1; ++k) {
            gemv(N2, FMAP(dm_tl, N2, jj - 2 + k), rr, tmpv);
            matmul(dim, opB, tmpv, tm);
            result[(i - 1) + (size_t)(k - 1) * n_t] = trace(dim, tm);
            memcpy(rr, tmpv, sizeof(ocplx) * N2);
        }
    }
    free(rho_vec); free(rho_res); free(t1); free(t2); free(rho_buffer); free(j_array);
}

/* propagate_tau.f90:189-295 */
void or_calc_onetime_parallel_block(const ocplx* dm_block, const ocplx* dm_s, const ocplx* rho_init,
                                    int n_tb, int nx_tau, int n_map, int n_t, int n_tfull, int dim,
                                    const ocplx* opA, const ocplx* opB, const ocplx* opC,
                                    const double* time, const double* time_sparse, ocplx* result) {
    int N2 = dim * dim;
    ocplx rho_vec[1296], rho_res[1296], t1[1296], t2[1296];
    ocplx* rho_buffer = malloc(sizeof(ocplx) * N2 * (size_t)n_t);
    int* j_array = malloc(sizeof(int) * n_t);
    memcpy(rho_vec, rho_init, sizeof(ocplx) * N2);
    result[0] = tr_abc_rho(dim, opA, opB, opC, rho_vec, t1, t2);
    int j = 1;
    for (int i = 1; i <= n_t; ++i) {
        while (j <= n_tfull && time[j - 1] < time_sparse[i - 1]) {
            gemv(N2, (j <= n_map) ? FMAP(dm_block, N2, j) : dm_s, rho_vec, rho_res);
            memcpy(rho_vec, rho_res, sizeof(ocplx) * N2);
            ++j;
        }
        result[i - 1] = tr_abc_rho(dim, opA, opB, opC, rho_vec, t1, t2);
        matmul(dim, opC, rho_vec, t1);
        matmul(dim, t1, opA, rho_buffer + (size_t)(i - 1) * N2);
        j_array[i - 1] = j;
    }
    int ncol = n_tb * nx_tau + 1;
    for (int i = 1; i <= n_t; ++i) {
        ocplx rr[1296], tmpv[1296], tm[1296];
        memcpy(rr, rho_buffer + (size_t)(i - 1) * N2, sizeof(ocplx) * N2);
        int jj = j_array[i - 1];
        for (int k = 2; k <= ncol; ++k) {
            gemv(N2, (jj <= n_map) ? FMAP(dm_block, N2, jj) : dm_s, rr, tmpv);
            matmul(dim, opB, tmpv, tm);
            result[(i - 1) + (size_t)(k - 1) * n_t] = trace(dim, tm);
            memcpy(rr, tmpv, sizeof(ocplx) * N2);
            jj = jj + 1;
            if (jj == n_tb + 1) jj = 1; /* :282-284 */
        }
    }
    free(rho_buffer); free(j_array);
}

/* propagate_tau.f90:374-536 */
void or_calc_twotime_phonon_block(const ocplx* dm_taucs2, const ocplx* dm_sep1, const ocplx* dm_sep2,
                                  const ocplx* dm_s, const ocplx* rho_init, int n_tb, int nx_tau, int n_map,
                                  int n_t, int n_tfull, int n_tauc, int dim,
                                  const ocplx* opA, const ocplx* opB, const ocplx* opC,
                                  const double* time, const double* time_sparse, ocplx* result) {
    int N2 = dim * dim;
    ocplx rho_vec[1296], rho_res[1296], t1[1296], t2[1296], opBT[36 * 36];
    ocplx* rho_buffer = malloc(sizeof(ocplx) * N2 * (size_t)(n_t > n_tauc ? n_t : n_tauc));
    int* j_array = malloc(sizeof(int) * (n_t > n_tauc ? n_t : n_tauc));
    for (int a = 0; a < dim; ++a)
        for (int b = 0; b < dim; ++b) opBT[a + b * dim] = opB[b + a * dim];
    memcpy(rho_vec, rho_init, sizeof(ocplx) * N2);
    /* :418-429 (value overwritten by i=1 below; kept for fidelity) */
    matmul(dim, opB, opC, t1);
    matmul(dim, opA, t1, t2);
    matmul(dim, t2, rho_vec, t1);
    result[0] = trace(dim, t1);
    int j = 1;
    for (int i = 1; i <= n_t; ++i) {
        while (j <= n_tfull && time[j - 1] < time_sparse[i - 1]) {
            gemv(N2, (j <= n_map) ? FMAP(dm_sep1, N2, j) : dm_s, rho_vec, rho_res);
            memcpy(rho_vec, rho_res, sizeof(ocplx) * N2);
            ++j;
        }
        result[i - 1] = tr_abc_rho(dim, opA, opB, opC, rho_vec, t1, t2);
        memcpy(rho_buffer + (size_t)(i - 1) * N2, rho_vec, sizeof(ocplx) * N2); /* :462: no MTO */
        j_array[i - 1] = j;
    }
    int ncol = n_tb * nx_tau + 1;
    for (int phase = 0; phase < 2; ++phase) {
        int i0 = phase == 0 ? 1 : n_tauc + 1, i1 = phase == 0 ? n_tauc : n_t;
        for (int i = i0; i <= i1; ++i) {
            ocplx rr[1296], tmpv[1296], tm[1296];
            memcpy(rr, rho_buffer + (size_t)(i - 1) * N2, sizeof(ocplx) * N2);
            int jj = 1, j_start = j_array[i - 1], use_dm2 = 1;
            for (int k = 2; k <= ncol; ++k) {
                const ocplx* map;
                if (jj <= n_map) {
                    if (use_dm2)
                        map = (phase == 0)
                                  ? dm_taucs2 + (size_t)N2 * N2 * ((size_t)(i - 1) + (size_t)n_tauc * (jj - 1))
                                  : FMAP(dm_sep2, N2, jj);
                    else
                        map = FMAP(dm_sep1, N2, jj);
                } else {
                    map = dm_s;
                }
                gemv(N2, map, rr, tmpv);
                memcpy(rr, tmpv, sizeof(ocplx) * N2);
                matmul(dim, opBT, rr, tm); /* :484 transpose(opB) */
                result[(i - 1) + (size_t)(k - 1) * n_t] = trace(dim, tm);
                jj = jj + 1;
                if (jj + j_start == n_tb + 1) { j_start = 0; jj = 1; use_dm2 = 0; }
            }
        }
    }
    free(rho_buffer); free(j_array);
}

/* ---- timebin_tl.f90 ---- */
static double round_to_6(double x) { /* timebin_tl.f90:13-20 nint(x*1e6,8)/1e6 */
    return (double)llround(x * 1000000.0) / 1000000.0;
}

/* timebin_tl.f90:23-47 */
static void fast_propagate(ocplx* rho, const ocplx* precalc, int n_steps, int N2, ocplx* tmp) {
    int n = n_steps, i = 0;
    while (n > 0) {
        if (n & 1) {
            gemv(N2, precalc + (size_t)i * N2 * N2, rho, tmp);
            memcpy(rho, tmp, sizeof(ocplx) * N2);
        }
        n >>= 1;
        ++i;
    }
}

/* timebin_tl.f90:50-77 (in place on rho) */
static void propagate_tb(double t_start, double t_stop, double dt, ocplx* rho, const ocplx* dm_tl,
                         const ocplx* precalc, int N2, int n_dm) {
    ocplx tmp[1296];
    int n_start = (int)(round_to_6(t_start) / dt);
    int n_stop = (int)(round_to_6(t_stop) / dt);
    int n_steps = n_stop - n_start;
    int steps_dm = (n_dm - n_start) < n_steps ? (n_dm - n_start) : n_steps;
    while (steps_dm > 0) {
        gemv(N2, dm_tl + (size_t)n_start * N2 * N2, rho, tmp); /* dm_tl(:,:,n_start+1) */
        memcpy(rho, tmp, sizeof(ocplx) * N2);
        n_steps--; n_start++; steps_dm--;
    }
    if (n_steps > 0) fast_propagate(rho, precalc, n_steps, N2, tmp);
}

static void apply_left(ocplx* rho, const ocplx* op, int dim) {
    ocplx t[1296];
    matmul(dim, op, rho, t);
    memcpy(rho, t, sizeof(ocplx) * dim * dim);
}
static void apply_right(ocplx* rho, const ocplx* op, int dim) {
    ocplx t[1296];
    matmul(dim, rho, op, t);
    memcpy(rho, t, sizeof(ocplx) * dim * dim);
}

/* timebin_tl.f90:216-303 */
void or_four_time_8op(const ocplx* dm_1, const ocplx* dm_2, const ocplx* rho_init, const double* t1,
                      const ocplx* precalc, int n_t, double dt, int n_map, int dim, const ocplx* ops8,
                      int early_only, int late_t1_only, double tb, int n_precalc, ocplx* result) {
    (void)n_precalc;
    int N2 = dim * dim;
    const ocplx *et1l = ops8, *et1r = ops8 + N2, *et2l = ops8 + 2 * N2, *et2r = ops8 + 3 * N2;
    const ocplx *lt1l = ops8 + 4 * N2, *lt1r = ops8 + 5 * N2, *lt2l = ops8 + 6 * N2, *lt2r = ops8 + 7 * N2;
    memset(result, 0, sizeof(ocplx) * (size_t)n_t * n_t);
#pragma omp parallel for schedule(dynamic)
    for (int i = 0; i < n_t; ++i) {
        ocplx rho_vec[1296], r[1296];
        double t1_now = t1[i];
        memcpy(rho_vec, rho_init, sizeof(ocplx) * N2);
        propagate_tb(0.0, t1_now, dt, rho_vec, dm_1, precalc, N2, n_map);
        for (int j = 0; j <= n_t - 1 - i; ++j) {
            double t2 = t1[i + j];
            memcpy(r, rho_vec, sizeof(ocplx) * N2);
            apply_right(r, et1r, dim); apply_left(r, et1l, dim);
            propagate_tb(t1_now, t2, dt, r, dm_1, precalc, N2, n_map);
            apply_right(r, et2r, dim); apply_left(r, et2l, dim);
            if (early_only) { result[i + (size_t)(i + j) * n_t] = trace(dim, r); continue; }
            propagate_tb(t2, tb, dt, r, dm_1, precalc, N2, n_map);
            propagate_tb(0.0, t1_now, dt, r, dm_2, precalc, N2, n_map);
            apply_right(r, lt1r, dim); apply_left(r, lt1l, dim);
            if (late_t1_only) { result[i + (size_t)(i + j) * n_t] = trace(dim, r); continue; }
            propagate_tb(t1_now, t2, dt, r, dm_2, precalc, N2, n_map);
            apply_right(r, lt2r, dim); apply_left(r, lt2l, dim);
            result[i + (size_t)(i + j) * n_t] = trace(dim, r);
        }
    }
}

/* timebin_tl.f90:145-214 */
void or_four_time(const ocplx* dm_1, const ocplx* dm_2, const ocplx* rho_init, const double* t1,
                  const ocplx* precalc, int n_t, double dt, int n_map, int dim, const ocplx* ops4,
                  double tb, int n_precalc, ocplx* result) {
    (void)n_precalc;
    int N2 = dim * dim;
    memset(result, 0, sizeof(ocplx) * (size_t)n_t * n_t);
#pragma omp parallel for schedule(dynamic)
    for (int i = 0; i < n_t; ++i) {
        ocplx rho_vec[1296], r[1296];
        double t1_now = t1[i];
        memcpy(rho_vec, rho_init, sizeof(ocplx) * N2);
        propagate_tb(0.0, t1_now, dt, rho_vec, dm_1, precalc, N2, n_map);
        for (int j = 0; j <= n_t - 1 - i; ++j) {
            double t2 = t1[i + j];
            memcpy(r, rho_vec, sizeof(ocplx) * N2);
            apply_right(r, ops4, dim);
            propagate_tb(t1_now, t2, dt, r, dm_1, precalc, N2, n_map);
            apply_right(r, ops4 + N2, dim);
            propagate_tb(t2, tb, dt, r, dm_1, precalc, N2, n_map);
            propagate_tb(0.0, t1_now, dt, r, dm_2, precalc, N2, n_map);
            apply_left(r, ops4 + 2 * N2, dim);
            propagate_tb(t1_now, t2, dt, r, dm_2, precalc, N2, n_map);
            apply_left(r, ops4 + 3 * N2, dim);
            result[i + (size_t)(i + j) * n_t] = trace(dim, r);
        }
    }
}

/* timebin_tl.f90:305-342 */
void or_dynamics_t1(const ocplx* dm_1, const ocplx* dm_2, const ocplx* rho_init, const double* t1,
                    const ocplx* precalc, int n_t, double dt, int n_map, int dim, double tb,
                    int n_precalc, ocplx* result) {
    (void)tb; (void)n_precalc;
    int N2 = dim * dim;
    memcpy(result, rho_init, sizeof(ocplx) * N2);
    for (int i = 0; i <= n_t - 2; ++i) {
        memcpy(result + (size_t)(i + 1) * N2, result + (size_t)i * N2, sizeof(ocplx) * N2);
        propagate_tb(t1[i], t1[i + 1], dt, result + (size_t)(i + 1) * N2, dm_1, precalc, N2, n_map);
    }
    for (int i = 0; i <= n_t - 2; ++i) {
        ocplx* dst = result + (size_t)(i + 1 + n_t - 1) * N2;
        memcpy(dst, result + (size_t)(i + n_t - 1) * N2, sizeof(ocplx) * N2);
        propagate_tb(t1[i], t1[i + 1], dt, dst, dm_2, precalc, N2, n_map);
    }
}
