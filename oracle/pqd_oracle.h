/* pqd_oracle.h — TEST INFRASTRUCTURE ONLY.
 *
 * Plain-C CPU restatement of the hot path, used as the CHECKER by tests/, __graft_entry__.smoke()
 * and bench.py's cpu_baseline leg. Never linked into, loaded by, or called from the product
 * (pyaceqd_amd / libpqd.so). The product must fail loudly when its HIP extension is missing.
 *
 * Parity status
 *   - map-chain sweeps (mapchain_oracle.c): PINNED against golden vectors produced by the
 *     reference's own Fortran (tests/golden/fortran_*.npz, oracle/_ref built from
 *     /root/reference/pyaceqd/two_time/propagate_tau.f90 and timebin/timebin_tl.f90).
 *   - PT propagator (pqd_oracle.c): the reference delegates this arithmetic to the external ACE
 *     binary, which is absent. Pinned by analytic known-answer tests (Rabi
 *     rotation, spontaneous decay, pure dephasing) and PT invariants (chi=1 identity PT ==
 *     no-PT result; PT-encoded Markovian dephasing == Lindblad dephasing); parity with ACE
 *     itself is UNPINNED.
 *
 * Conventions (frozen):
 *   - complex numbers are interleaved doubles (re, im) = C99 double _Complex;
 *   - N x N operators are row-major; Liouville vectors are row-major vec(rho)[i*N+j] = rho[i][j]
 *     (tools.py:583-588, correlations.py:517-524);
 *   - Fortran-layout map stacks are column-major (N2, N2, n): element (r,c) of map m at
 *     [m*N2*N2 + c*N2 + r]  (correlations.py:781 np.asfortranarray(dm_tl.transpose(1,2,0))).
 */
#ifndef PQD_ORACLE_H
#define PQD_ORACLE_H
#include <complex.h>
#include <stdint.h>
#ifdef __cplusplus
extern "C" {
#endif

typedef double _Complex ocplx;

/* ---- system description (same meaning as pqd_system in include/pqd.h) ---- */
typedef struct {
    int dim;                     /* N */
    double hbar;                 /* meV ps (constants.py:1) */
    const ocplx* H0;             /* N*N */
    int n_lind;
    const double* lind_rates;    /* n_lind */
    const ocplx* lind_ops;       /* n_lind*N*N */
    int n_chan;                  /* pulse channels: H += f(t) X + conj(f(t)) X^dagger */
    const ocplx* chan_ops;       /* n_chan*N*N (X, already scaled, e.g. -0.5*pi*hbar*op) */
    const ocplx* chan_samples;   /* n_chan*n_samples */
    int n_samples;
    double sample_t0, sample_dt; /* samples at sample_t0 + k*sample_dt, linear interpolation, clamped */
} or_system;

typedef struct {
    double ta, dt;
    int n_steps;
    int n_sub;                   /* exponential-midpoint sub-steps per half step (>=1) */
} or_grid;

typedef struct {
    int chi, D, n_slices;
    const ocplx* Q;              /* n_slices * D * chi * chi, Q[s][g][d][d'] */
    const ocplx* closure;        /* n_slices * chi */
    const ocplx* closure0;       /* chi: closure for the output at step 0 */
    const ocplx* bond0;          /* chi: initial bond vector */
    const int32_t* gmap;         /* N2: Liouville index -> dictionary slice g */
    const int32_t* sched;        /* n_steps: PT slice applied in step n */
} or_pt;

typedef struct {
    int n_traj;
    const int32_t* out_begin;    /* inclusive */
    const int32_t* out_end;      /* inclusive; the trajectory is propagated up to this step */
    const int64_t* out_offset;   /* complex offset of each trajectory's window in out[] */
    int n_mto;
    const int32_t* mto_traj;
    const int32_t* mto_step;
    const int32_t* mto_before;   /* 1: applied before the output of that step (applyBefore true) */
    const int32_t* mto_kind;     /* 0: A rho A^dagger ("") 1: A rho ("_left") 2: rho A ("_right") */
    const ocplx* mto_ops;        /* n_mto * N * N */
} or_traj;

/* free propagators: M[(2n+h)*N2*N2 ...] for step n, half h (h=0 first half), row-major */
int or_free_propagators(const or_system* sys, const or_grid* g, ocplx* M);
/* Liouvillian at time t (row-major N2 x N2) */
void or_liouvillian(const or_system* sys, double t, ocplx* L);
/* matrix exponential (scaling & squaring + degree-18 Taylor) of an n x n complex matrix */
void or_expm(int n, const ocplx* A, ocplx* E);

/* full propagation of all trajectories; pt may be NULL (no environment).
 * M may be NULL (computed internally) or the precomputed free propagators.
 * n_out output operators (row-major N x N); out receives <O_k> per window step.
 * nthreads: OpenMP threads over trajectories (<=0: runtime default). */
int or_propagate(const or_system* sys, const or_grid* g, const or_pt* pt, const ocplx* rho0,
                 int n_out, const ocplx* out_ops, const or_traj* tr, const ocplx* M,
                 ocplx* out, int nthreads);

/* the same propagation with trajectories advanced in lockstep blocks of bt (pqd_oracle_blk.c): bench.py's CPU
 * baseline; agrees with or_propagate to rounding */
int or_propagate_blocked(const or_system* sys, const or_grid* g, const or_pt* pt, const ocplx* rho0, int n_out,
                         const ocplx* out_ops, const or_traj* tr, const ocplx* M, ocplx* out, int nthreads, int bt);

/* ---- Fortran map-chain sweeps (restated one-to-one, mapchain_oracle.c) ---- */
void or_propagate_tau(const ocplx* dm_tl, const ocplx* rho_init, int n_tau, int dim, int j_start,
                      ocplx* rho_out);
void or_calc_onetime_parallel(const ocplx* dm_tl, const ocplx* rho_init, int n_tau, int n_t, int n_tfull,
                              int dim, const ocplx* opA, const ocplx* opB, const ocplx* opC,
                              const double* time, const double* time_sparse, ocplx* result, int nthreads);
void or_calc_onetime_parallel_block(const ocplx* dm_block, const ocplx* dm_s, const ocplx* rho_init,
                                    int n_tb, int nx_tau, int n_map, int n_t, int n_tfull, int dim,
                                    const ocplx* opA, const ocplx* opB, const ocplx* opC,
                                    const double* time, const double* time_sparse, ocplx* result);
void or_calc_twotime_phonon_block(const ocplx* dm_taucs2, const ocplx* dm_sep1, const ocplx* dm_sep2,
                                  const ocplx* dm_s, const ocplx* rho_init, int n_tb, int nx_tau, int n_map,
                                  int n_t, int n_tfull, int n_tauc, int dim,
                                  const ocplx* opA, const ocplx* opB, const ocplx* opC,
                                  const double* time, const double* time_sparse, ocplx* result);
void or_four_time_8op(const ocplx* dm_1, const ocplx* dm_2, const ocplx* rho_init, const double* t1,
                      const ocplx* precalc, int n_t, double dt, int n_map, int dim, const ocplx* ops8,
                      int early_only, int late_t1_only, double tb, int n_precalc, ocplx* result);
void or_four_time(const ocplx* dm_1, const ocplx* dm_2, const ocplx* rho_init, const double* t1,
                  const ocplx* precalc, int n_t, double dt, int n_map, int dim, const ocplx* ops4,
                  double tb, int n_precalc, ocplx* result);
void or_dynamics_t1(const ocplx* dm_1, const ocplx* dm_2, const ocplx* rho_init, const double* t1,
                    const ocplx* precalc, int n_t, double dt, int n_map, int dim, double tb,
                    int n_precalc, ocplx* result);

#ifdef __cplusplus
}
#endif
#endif
