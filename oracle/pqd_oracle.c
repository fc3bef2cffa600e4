/* pqd_oracle.c — TEST INFRASTRUCTURE ONLY (see pqd_oracle.h for the parity status).
 *
 * CPU restatement of the propagation the reference hands to ACE (general_system.py:227-290,
 * 337-343): per step n (t_n = ta + n dt):
 *     [MTOs "applyBefore true" at n] -> output(n) -> [MTOs "applyBefore false" at n]
 *     -> state <- M_a(n) state -> PT contraction with slice sched[n] -> state <- M_b(n) state
 * (use_symmetric_Trotter true, general_system.py:234; MTO timing general_system.py:283-285).
 * M_a/M_b are the free propagators exp(L dt/2) of the first/second half step, each as a product of
 * n_sub exponential-midpoint factors; L is the Lindblad Liouvillian of
 *     H(t) = H0 + sum_p ( f_p(t) X_p + conj(f_p(t)) X_p^dagger )   (add_Pulse + h.c., general_system.py:245,279)
 * with dissipators gamma (L rho L^dag - 1/2 {L^dag L, rho})          (add_Lindblad, general_system.py:260).
 * The state of one trajectory is the augmented density matrix Q[alpha][d] (alpha Liouville index,
 * d PT bond index); the PT slice acts diagonally in alpha through the dictionary map g(alpha)
 * (diagonal system-bath coupling: tls.py:56, four_level_system/linear.py:17, six_level_system/linear.py:50).
 */
#include "pqd_oracle.h"
#include <math.h>
#include <stdlib.h>
#include <string.h>

static void mm(int n, const ocplx* A, const ocplx* B, ocplx* C) { /* row-major C = A B */
    for (int i = 0; i < n; ++i) {
        ocplx* ci = C + (size_t)i * n;
        for (int j = 0; j < n; ++j) ci[j] = 0;
        for (int k = 0; k < n; ++k) {
            ocplx a = A[(size_t)i * n + k];
            const ocplx* bk = B + (size_t)k * n;
            for (int j = 0; j < n; ++j) ci[j] += a * bk[j];
        }
    }
}

void or_expm(int n, const ocplx* A, ocplx* E) {
    size_t nn = (size_t)n * n;
    double norm = 0.0;
    for (int c = 0; c < n; ++c) {
        double s = 0.0;
        for (int r = 0; r < n; ++r) s += cabs(A[(size_t)r * n + c]);
        if (s > norm) norm = s;
    }
    int e = 0;
    frexp(norm / 0.5, &e);
    int s = e > 0 ? e : 0;
    double scale = ldexp(1.0, -s);
    ocplx* As = malloc(sizeof(ocplx) * nn);
    ocplx* P = malloc(sizeof(ocplx) * nn);
    ocplx* T = malloc(sizeof(ocplx) * nn);
    for (size_t k = 0; k < nn; ++k) As[k] = A[k] * scale;
    /* Horner: P = I + As/18 (I + As/17 (...)) */
    for (size_t k = 0; k < nn; ++k) P[k] = As[k] / 18.0;
    for (int i = 0; i < n; ++i) P[(size_t)i * n + i] += 1.0;
    for (int m = 17; m >= 1; --m) {
        mm(n, As, P, T);
        for (size_t k = 0; k < nn; ++k) P[k] = T[k] / (double)m;
        for (int i = 0; i < n; ++i) P[(size_t)i * n + i] += 1.0;
    }
    for (int q = 0; q < s; ++q) {
        mm(n, P, P, T);
        memcpy(P, T, sizeof(ocplx) * nn);
    }
    memcpy(E, P, sizeof(ocplx) * nn);
    free(As); free(P); free(T);
}

static ocplx sample(const or_system* sys, int p, double t) {
    const ocplx* f = sys->chan_samples + (size_t)p * sys->n_samples;
    int ns = sys->n_samples;
    double u = (t - sys->sample_t0) / sys->sample_dt;
    if (!(u > 0.0)) return f[0];
    if (u >= (double)(ns - 1)) return f[ns - 1];
    int k = (int)floor(u);
    double w = u - (double)k;
    return f[k] + w * (f[k + 1] - f[k]);
}

void or_liouvillian(const or_system* sys, double t, ocplx* L) {
    int N = sys->dim, N2 = N * N;
    ocplx* H = malloc(sizeof(ocplx) * N2);
    memcpy(H, sys->H0, sizeof(ocplx) * N2);
    for (int p = 0; p < sys->n_chan; ++p) {
        ocplx f = sample(sys, p, t);
        const ocplx* X = sys->chan_ops + (size_t)p * N2;
        for (int i = 0; i < N; ++i)
            for (int j = 0; j < N; ++j) H[i * N + j] += f * X[i * N + j] + conj(f) * conj(X[j * N + i]);
    }
    const ocplx mih = -I / sys->hbar;
    for (int i = 0; i < N; ++i)
        for (int j = 0; j < N; ++j)
            for (int k = 0; k < N; ++k)
                for (int l = 0; l < N; ++l) {
                    ocplx v = 0;
                    if (j == l) v += mih * H[i * N + k];
                    if (i == k) v -= mih * H[l * N + j];
                    L[(size_t)(i * N + j) * N2 + (k * N + l)] = v;
                }
    for (int q = 0; q < sys->n_lind; ++q) {
        const ocplx* Lk = sys->lind_ops + (size_t)q * N2;
        double g = sys->lind_rates[q];
        ocplx LdL[36 * 36];
        for (int i = 0; i < N; ++i)
            for (int j = 0; j < N; ++j) {
                ocplx s = 0;
                for (int k = 0; k < N; ++k) s += conj(Lk[k * N + i]) * Lk[k * N + j];
                LdL[i * N + j] = s;
            }
        for (int i = 0; i < N; ++i)
            for (int j = 0; j < N; ++j)
                for (int k = 0; k < N; ++k)
                    for (int l = 0; l < N; ++l) {
                        ocplx v = Lk[i * N + k] * conj(Lk[j * N + l]);
                        if (j == l) v -= 0.5 * LdL[i * N + k];
                        if (i == k) v -= 0.5 * LdL[l * N + j];
                        L[(size_t)(i * N + j) * N2 + (k * N + l)] += g * v;
                    }
    }
    free(H);
}

int or_free_propagators(const or_system* sys, const or_grid* g, ocplx* M) {
    int N2 = sys->dim * sys->dim;
    size_t mm2 = (size_t)N2 * N2;
    int nsub = g->n_sub > 0 ? g->n_sub : 1;
#pragma omp parallel for schedule(static)
    for (int m = 0; m < 2 * g->n_steps; ++m) {
        int n = m >> 1, h = m & 1;
        double w = 0.5 * g->dt / nsub;
        ocplx* L = malloc(sizeof(ocplx) * mm2);
        ocplx* Ej = malloc(sizeof(ocplx) * mm2);
        ocplx* acc = malloc(sizeof(ocplx) * mm2);
        ocplx* tmp = malloc(sizeof(ocplx) * mm2);
        for (int j = 0; j < nsub; ++j) {
            double t = g->ta + n * g->dt + h * 0.5 * g->dt + (j + 0.5) * w;
            or_liouvillian(sys, t, L);
            for (size_t k = 0; k < mm2; ++k) L[k] *= w;
            or_expm(N2, L, Ej);
            if (j == 0) memcpy(acc, Ej, sizeof(ocplx) * mm2);
            else { mm(N2, Ej, acc, tmp); memcpy(acc, tmp, sizeof(ocplx) * mm2); }
        }
        memcpy(M + (size_t)m * mm2, acc, sizeof(ocplx) * mm2);
        free(L); free(Ej); free(acc); free(tmp);
    }
    return 0;
}

/* apply the MTO to every bond column of the augmented state (as N x N matrices, not superops) */
static void apply_mto(int N, int chi, ocplx* st, int kind, const ocplx* A) {
    int N2 = N * N;
    ocplx r[36 * 36], t[36 * 36];
    for (int d = 0; d < chi; ++d) {
        for (int a = 0; a < N2; ++a) r[a] = st[(size_t)a * chi + d];
        if (kind == 1 || kind == 0) { /* A rho */
            for (int i = 0; i < N; ++i)
                for (int j = 0; j < N; ++j) {
                    ocplx s = 0;
                    for (int k = 0; k < N; ++k) s += A[i * N + k] * r[k * N + j];
                    t[i * N + j] = s;
                }
            memcpy(r, t, sizeof(ocplx) * N2);
        }
        if (kind == 2) { /* rho A */
            for (int i = 0; i < N; ++i)
                for (int j = 0; j < N; ++j) {
                    ocplx s = 0;
                    for (int k = 0; k < N; ++k) s += r[i * N + k] * A[k * N + j];
                    t[i * N + j] = s;
                }
            memcpy(r, t, sizeof(ocplx) * N2);
        }
        if (kind == 0) { /* (A rho) A^dagger */
            for (int i = 0; i < N; ++i)
                for (int j = 0; j < N; ++j) {
                    ocplx s = 0;
                    for (int k = 0; k < N; ++k) s += r[i * N + k] * conj(A[j * N + k]);
                    t[i * N + j] = s;
                }
            memcpy(r, t, sizeof(ocplx) * N2);
        }
        for (int a = 0; a < N2; ++a) st[(size_t)a * chi + d] = r[a];
    }
}

static void apply_free(int N2, int chi, const ocplx* M, const ocplx* st, ocplx* nw) {
    for (int a2 = 0; a2 < N2; ++a2) {
        ocplx* o = nw + (size_t)a2 * chi;
        for (int d = 0; d < chi; ++d) o[d] = 0;
        for (int a = 0; a < N2; ++a) {
            ocplx m = M[(size_t)a2 * N2 + a];
            const ocplx* s = st + (size_t)a * chi;
            for (int d = 0; d < chi; ++d) o[d] += m * s[d];
        }
    }
}

static void apply_pt(int N2, int chi, const ocplx* Qs, const int32_t* gmap, const ocplx* st, ocplx* nw) {
    for (int a = 0; a < N2; ++a) {
        const ocplx* Qg = Qs + (size_t)gmap[a] * chi * chi;
        ocplx* o = nw + (size_t)a * chi;
        for (int d = 0; d < chi; ++d) o[d] = 0;
        for (int d = 0; d < chi; ++d) {
            ocplx x = st[(size_t)a * chi + d];
            const ocplx* q = Qg + (size_t)d * chi;
            for (int e = 0; e < chi; ++e) o[e] += x * q[e];
        }
    }
}

int or_propagate(const or_system* sys, const or_grid* g, const or_pt* pt, const ocplx* rho0,
                 int n_out, const ocplx* out_ops, const or_traj* tr, const ocplx* Min,
                 ocplx* out, int nthreads) {
    int N = sys->dim, N2 = N * N;
    size_t mm2 = (size_t)N2 * N2;
    const ocplx* M = Min;
    ocplx* Mown = NULL;
    if (!M) {
        Mown = malloc(sizeof(ocplx) * mm2 * 2 * (size_t)g->n_steps);
        or_free_propagators(sys, g, Mown);
        M = Mown;
    }
    int chi = pt ? pt->chi : 1;
#pragma omp parallel for schedule(dynamic) num_threads(nthreads > 0 ? nthreads : 1)
    for (int it = 0; it < tr->n_traj; ++it) {
        ocplx* st = malloc(sizeof(ocplx) * N2 * (size_t)chi);
        ocplx* nw = malloc(sizeof(ocplx) * N2 * (size_t)chi);
        ocplx r[36];
        for (int a = 0; a < N2; ++a)
            for (int d = 0; d < chi; ++d) st[(size_t)a * chi + d] = rho0[a] * (pt ? pt->bond0[d] : 1.0);
        int nb = tr->out_begin[it], ne = tr->out_end[it];
        for (int n = 0; n <= ne; ++n) {
            for (int q = 0; q < tr->n_mto; ++q)
                if (tr->mto_traj[q] == it && tr->mto_step[q] == n && tr->mto_before[q])
                    apply_mto(N, chi, st, tr->mto_kind[q], tr->mto_ops + (size_t)q * N2);
            if (n >= nb) {
                const ocplx* c = NULL;
                if (pt) c = (n == 0) ? pt->closure0 : pt->closure + (size_t)pt->sched[n - 1] * chi;
                for (int a = 0; a < N2; ++a) {
                    ocplx s = 0;
                    for (int d = 0; d < chi; ++d) s += st[(size_t)a * chi + d] * (c ? c[d] : 1.0);
                    r[a] = s;
                }
                ocplx* o = out + tr->out_offset[it] + (size_t)(n - nb) * n_out;
                for (int k = 0; k < n_out; ++k) {
                    const ocplx* O = out_ops + (size_t)k * N2;
                    ocplx s = 0;
                    for (int i = 0; i < N; ++i)
                        for (int j = 0; j < N; ++j) s += O[j * N + i] * r[i * N + j];
                    o[k] = s;
                }
            }
            for (int q = 0; q < tr->n_mto; ++q)
                if (tr->mto_traj[q] == it && tr->mto_step[q] == n && !tr->mto_before[q])
                    apply_mto(N, chi, st, tr->mto_kind[q], tr->mto_ops + (size_t)q * N2);
            if (n == ne) break;
            apply_free(N2, chi, M + (size_t)(2 * n) * mm2, st, nw);
            if (pt) {
                apply_pt(N2, chi, pt->Q + (size_t)pt->sched[n] * pt->D * chi * chi, pt->gmap, nw, st);
            } else {
                memcpy(st, nw, sizeof(ocplx) * N2 * chi);
            }
            apply_free(N2, chi, M + (size_t)(2 * n + 1) * mm2, st, nw);
            memcpy(st, nw, sizeof(ocplx) * N2 * chi);
        }
        free(st); free(nw);
    }
    free(Mown);
    return 0;
}
