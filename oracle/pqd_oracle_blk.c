/* oracle/pqd_oracle_blk.c — TEST INFRASTRUCTURE ONLY (never shipped, never measured as the product).
 *
 * The CPU baseline of bench.py: the same algorithm as or_propagate (pqd_oracle.c, which restates the ACE step
 * order behind pyaceqd/general_system/general_system.py:215-331), arranged for the host caches instead of as a
 * one-trajectory-at-a-time checker. Trajectories of one system advance in lockstep in blocks of `bt`:
 *   - the augmented states of a block are stored as st[alpha][t][d], so each PT row is a (bt x chi) x (chi x chi)
 *     product whose slice rows are reused bt times from L1 (the plain port streams the whole N^2 chi^2 slice set
 *     once per trajectory-step: L2/L3-bound at ~25 GFLOP/s per core);
 *   - the free propagator of a half step is applied to the whole block as one (N^2 x N^2) x (N^2 x bt chi) product;
 *   - each trajectory's MTOs are looked up in a list sorted by step instead of scanning every MTO at every step.
 * Summation order inside the products differs from or_propagate (four slice rows per pass), so results agree to
 * rounding, not bit for bit (tests/test_oracle_blocked.py). */
#include <stdlib.h>
#include <string.h>

#include "pqd_oracle.h"

#pragma GCC optimize("fp-contract=fast")

/* or_propagate's apply_mto on one trajectory of a block (row stride rs between the N^2 rows of its state) */
static void mto_strided(int N, int chi, ocplx* st, size_t rs, int kind, const ocplx* A) {
    int N2 = N * N;
    ocplx r[36], t[36];
    for (int d = 0; d < chi; ++d) {
        for (int a = 0; a < N2; ++a) r[a] = st[(size_t)a * rs + d];
        if (kind == 1 || kind == 0) {
            for (int i = 0; i < N; ++i)
                for (int j = 0; j < N; ++j) {
                    ocplx s = 0;
                    for (int k = 0; k < N; ++k) s += A[i * N + k] * r[k * N + j];
                    t[i * N + j] = s;
                }
            memcpy(r, t, sizeof(ocplx) * N2);
        }
        if (kind == 2) {
            for (int i = 0; i < N; ++i)
                for (int j = 0; j < N; ++j) {
                    ocplx s = 0;
                    for (int k = 0; k < N; ++k) s += r[i * N + k] * A[k * N + j];
                    t[i * N + j] = s;
                }
            memcpy(r, t, sizeof(ocplx) * N2);
        }
        if (kind == 0) {
            for (int i = 0; i < N; ++i)
                for (int j = 0; j < N; ++j) {
                    ocplx s = 0;
                    for (int k = 0; k < N; ++k) s += r[i * N + k] * conj(A[j * N + k]);
                    t[i * N + j] = s;
                }
            memcpy(r, t, sizeof(ocplx) * N2);
        }
        for (int a = 0; a < N2; ++a) st[(size_t)a * rs + d] = r[a];
    }
}

/* nw[a2][:] = sum_a M[a2][a] st[a][:], rows of len = bt chi contiguous; in column chunks of FB so the N^2 input
 * and output row pieces of a chunk stay in L1 (a pass over whole rows per output row would stream the block state
 * from L2 N^2 times per half step) */
#define FB 64
static void free_block(int N2, size_t len, const ocplx* M, const ocplx* st, ocplx* nw) {
    for (size_t j0 = 0; j0 < len; j0 += FB) {
        const size_t jn = (len - j0) < FB ? (len - j0) : FB;
        for (int a2 = 0; a2 < N2; ++a2) {
            ocplx* o = nw + (size_t)a2 * len + j0;
            const ocplx* m = M + (size_t)a2 * N2;
            {
                const ocplx m0 = m[0];
                const ocplx* s0 = st + j0;
                for (size_t j = 0; j < jn; ++j) o[j] = m0 * s0[j];
            }
            int a = 1;
            for (; a + 3 <= N2; a += 3) {
                const ocplx m0 = m[a], m1 = m[a + 1], m2 = m[a + 2];
                const ocplx *s0 = st + (size_t)a * len + j0, *s1 = s0 + len, *s2 = s1 + len;
                for (size_t j = 0; j < jn; ++j) o[j] += m0 * s0[j] + m1 * s1[j] + m2 * s2[j];
            }
            for (; a < N2; ++a) {
                const ocplx m0 = m[a];
                const ocplx* s0 = st + (size_t)a * len + j0;
                for (size_t j = 0; j < jn; ++j) o[j] += m0 * s0[j];
            }
        }
    }
}

/* o_r/o_i[e] += sum_{j<4} x_j Q[d + j][e] for e < chi (QR/QI: slice rows d..d+3, real and imaginary parts) */
static inline void cmac4(int chi, double* restrict orr, double* restrict oii, const double* restrict QR,
                         const double* restrict QI, const double* restrict xt) {
    const double x0r = xt[0], x0i = xt[1], x1r = xt[2], x1i = xt[3];
    const double x2r = xt[4], x2i = xt[5], x3r = xt[6], x3i = xt[7];
    const size_t c = (size_t)chi;
    for (int e = 0; e < chi; ++e) {
        const double r0 = QR[e], r1 = QR[c + e], r2 = QR[2 * c + e], r3 = QR[3 * c + e];
        const double i0 = QI[e], i1 = QI[c + e], i2 = QI[2 * c + e], i3 = QI[3 * c + e];
        orr[e] += x0r * r0 - x0i * i0 + x1r * r1 - x1i * i1 + x2r * r2 - x2i * i2 + x3r * r3 - x3i * i3;
        oii[e] += x0r * i0 + x0i * r0 + x1r * i1 + x1i * r1 + x2r * i2 + x2i * r2 + x3r * i3 + x3i * r3;
    }
}

/* st[a][t][:] = nw[a][t][:] Q_{gmap[a]} for the nt trajectories of a block. The slice of a row is split into real
 * and imaginary parts once (qr/qi, reused by every trajectory of the block and by the rows sharing the slice) and the
 * accumulators are split likewise, so the inner loop is plain FMAs over contiguous doubles; four slice rows per pass
 * stay in L1 while every trajectory of the block uses them. ws: 2 chi^2 + 2 nt chi doubles. */
static void pt_block(int N2, int chi, int nt, const ocplx* Qs, const int32_t* gmap, const ocplx* nw, ocplx* st,
                     double* ws) {
    const size_t len = (size_t)nt * chi;
    double* qr = ws;
    double* qi = qr + (size_t)chi * chi;
    double* ar = qi + (size_t)chi * chi;
    double* ai = ar + len;
    int g_split = -1;
    for (int a = 0; a < N2; ++a) {
        if (gmap[a] != g_split) {
            const double* Q = (const double*)(Qs + (size_t)gmap[a] * chi * chi);
            for (size_t e = 0; e < (size_t)chi * chi; ++e) { qr[e] = Q[2 * e]; qi[e] = Q[2 * e + 1]; }
            g_split = gmap[a];
        }
        const double* x = (const double*)(nw + (size_t)a * len);
        memset(ar, 0, sizeof(double) * len);
        memset(ai, 0, sizeof(double) * len);
        int d = 0;
        for (; d + 4 <= chi; d += 4) {
            for (int t = 0; t < nt; ++t)
                cmac4(chi, ar + (size_t)t * chi, ai + (size_t)t * chi, qr + (size_t)d * chi, qi + (size_t)d * chi,
                      x + 2 * ((size_t)t * chi + d));
        }
        for (; d < chi; ++d) {
            const double *r0 = qr + (size_t)d * chi, *i0 = qi + (size_t)d * chi;
            for (int t = 0; t < nt; ++t) {
                const double x0r = x[2 * ((size_t)t * chi + d)], x0i = x[2 * ((size_t)t * chi + d) + 1];
                double* otr = ar + (size_t)t * chi;
                double* oti = ai + (size_t)t * chi;
                for (int e = 0; e < chi; ++e) {
                    otr[e] += x0r * r0[e] - x0i * i0[e];
                    oti[e] += x0r * i0[e] + x0i * r0[e];
                }
            }
        }
        double* o = (double*)(st + (size_t)a * len);
        for (size_t j = 0; j < len; ++j) { o[2 * j] = ar[j]; o[2 * j + 1] = ai[j]; }
    }
}

int or_propagate_blocked(const or_system* sys, const or_grid* g, const or_pt* pt, const ocplx* rho0, int n_out,
                         const ocplx* out_ops, const or_traj* tr, const ocplx* Min, ocplx* out, int nthreads, int bt) {
    const int N = sys->dim, N2 = N * N;
    const size_t mm2 = (size_t)N2 * N2;
    if (bt < 1) bt = 1;
    const ocplx* M = Min;
    ocplx* Mown = NULL;
    if (!M) {
        Mown = malloc(sizeof(ocplx) * mm2 * 2 * (size_t)g->n_steps);
        if (!Mown) return 2;
        or_free_propagators(sys, g, Mown);
        M = Mown;
    }
    const int chi = pt ? pt->chi : 1;
    const int nT = tr->n_traj;
    /* each trajectory's MTOs in list order, then stably by step (or_propagate applies them in list order) */
    int* first = calloc((size_t)nT + 1, sizeof(int));
    int* ord = malloc(sizeof(int) * (size_t)(tr->n_mto > 0 ? tr->n_mto : 1));
    if (!first || !ord) { free(first); free(ord); free(Mown); return 2; }
    for (int q = 0; q < tr->n_mto; ++q) first[tr->mto_traj[q] + 1]++;
    for (int i = 0; i < nT; ++i) first[i + 1] += first[i];
    {
        int* fill = malloc(sizeof(int) * ((size_t)nT + 1));
        memcpy(fill, first, sizeof(int) * ((size_t)nT + 1));
        for (int q = 0; q < tr->n_mto; ++q) ord[fill[tr->mto_traj[q]]++] = q;
        free(fill);
        for (int i = 0; i < nT; ++i)
            for (int u = first[i] + 1; u < first[i + 1]; ++u)
                for (int v = u; v > first[i] && tr->mto_step[ord[v - 1]] > tr->mto_step[ord[v]]; --v) {
                    int tmp = ord[v]; ord[v] = ord[v - 1]; ord[v - 1] = tmp;
                }
    }
    const int n_blk = (nT + bt - 1) / bt;
#pragma omp parallel for schedule(dynamic) num_threads(nthreads > 0 ? nthreads : 1)
    for (int b = 0; b < n_blk; ++b) {
        const int t0 = b * bt, nt = (nT - t0) < bt ? (nT - t0) : bt;
        const size_t len = (size_t)nt * chi;
        ocplx* st = malloc(sizeof(ocplx) * N2 * len);
        ocplx* nw = malloc(sizeof(ocplx) * N2 * len);
        int* evp = malloc(sizeof(int) * (size_t)nt);
        double* ws = malloc(sizeof(double) * (2 * (size_t)chi * chi + 2 * len));
        ocplx r[36];
        int nmax = 0;
        for (int t = 0; t < nt; ++t) {
            evp[t] = first[t0 + t];
            if (tr->out_end[t0 + t] > nmax) nmax = tr->out_end[t0 + t];
        }
        for (int a = 0; a < N2; ++a)
            for (int t = 0; t < nt; ++t)
                for (int d = 0; d < chi; ++d) st[(size_t)a * len + (size_t)t * chi + d] = rho0[a] * (pt ? pt->bond0[d] : 1.0);
        for (int n = 0; n <= nmax; ++n) {
            const ocplx* c = NULL;
            if (pt) c = (n == 0) ? pt->closure0 : pt->closure + (size_t)pt->sched[n - 1] * chi;
            for (int t = 0; t < nt; ++t) {
                const int it = t0 + t, nb = tr->out_begin[it], ne = tr->out_end[it];
                if (n > ne) continue;
                ocplx* s = st + (size_t)t * chi;
                const int e1 = first[it + 1];
                for (int u = evp[t]; u < e1 && tr->mto_step[ord[u]] == n; ++u)
                    if (tr->mto_before[ord[u]])
                        mto_strided(N, chi, s, len, tr->mto_kind[ord[u]], tr->mto_ops + (size_t)ord[u] * N2);
                if (n >= nb) {
                    for (int a = 0; a < N2; ++a) {
                        ocplx acc = 0;
                        const ocplx* sa = s + (size_t)a * len;
                        for (int d = 0; d < chi; ++d) acc += sa[d] * (c ? c[d] : 1.0);
                        r[a] = acc;
                    }
                    ocplx* o = out + tr->out_offset[it] + (size_t)(n - nb) * n_out;
                    for (int k = 0; k < n_out; ++k) {
                        const ocplx* O = out_ops + (size_t)k * N2;
                        ocplx acc = 0;
                        for (int i = 0; i < N; ++i)
                            for (int j = 0; j < N; ++j) acc += O[j * N + i] * r[i * N + j];
                        o[k] = acc;
                    }
                }
                int u = evp[t];
                for (; u < e1 && tr->mto_step[ord[u]] == n; ++u)
                    if (!tr->mto_before[ord[u]])
                        mto_strided(N, chi, s, len, tr->mto_kind[ord[u]], tr->mto_ops + (size_t)ord[u] * N2);
                evp[t] = u;
            }
            if (n == nmax) break;
            /* trajectories past their last step keep stepping with the block (their states are not read again) */
            free_block(N2, len, M + (size_t)(2 * n) * mm2, st, nw);
            if (pt)
                pt_block(N2, chi, nt, pt->Q + (size_t)pt->sched[n] * pt->D * chi * chi, pt->gmap, nw, st, ws);
            else
                memcpy(st, nw, sizeof(ocplx) * N2 * len);
            free_block(N2, len, M + (size_t)(2 * n + 1) * mm2, st, nw);
            ocplx* sw = st; st = nw; nw = sw;
        }
        free(st); free(nw); free(evp); free(ws);
    }
    free(first); free(ord); free(Mown);
    return 0;
}
