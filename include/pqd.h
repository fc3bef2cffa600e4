/* pqd.h — C-ABI of libpqd, the MI355X-native process-tensor propagator behind pyaceqd's
 * `system_ace_stream` driver and its two-time sweeps.
 *
 * Drop-in boundary. Each entry point replaces one reference interface:
 *
 *   pqd_propagate / pqd_plan_*      replace the ACE engine process boundary
 *                                   `subprocess.check_output(["ACE", param_file])` + outfile parse
 *                                   (pyaceqd/general_system/general_system.py:337-343, params :227-290,
 *                                   parse read_result :104-110), batched over trajectories so the
 *                                   ThreadPoolExecutor fan-out of two_time/correlations.py:153-169 becomes
 *                                   one launch.
 *   pqd_pt_create                   replaces `add_PT <file>` + the PT files ACE writes
 *                                   (general_system.py:146-197, 236); device-resident, shared per context.
 *   pqd_ace_pt_shape / _read        read ACE's own PT files (general_system.py:153-157, 194-197) under a
 *                                   stated layout assumption (ACE_PTB_V0)
 *   pqd_free_propagators            exposes the free propagator ACEutils.FreePropagator.update(t,dt).M
 *                                   (general_system.py:324-327, `get_M_t`).
 *   pqd_propagate_tau               f2py propagate_tau_module.propagate_tau   (two_time/propagate_tau.f90:3)
 *   pqd_calc_onetime_parallel       ... .calc_onetime_parallel                 (propagate_tau.f90:110)
 *   pqd_calc_onetime_parallel_block ... .calc_onetime_parallel_block           (propagate_tau.f90:189)
 *   pqd_calc_twotime_phonon_block   ... .calc_twotime_phonon_block             (propagate_tau.f90:374)
 *   pqd_four_time_8op               f2py timebin_tl.four_time_8op              (timebin/timebin_tl.f90:216)
 *   pqd_four_time                   ... .four_time                             (timebin_tl.f90:145)
 *   pqd_dynamics_t1                 ... .dynamics_t1                           (timebin_tl.f90:305)
 *
 * Conventions: complex numbers are interleaved doubles {re, im}; N x N operators row-major;
 * Liouville vectors row-major vec(rho)[i*N+j] = rho[i][j]; map-chain arguments keep the
 * reference's Fortran (column-major) layouts and index semantics, with the f2py-hidden
 * dimensions passed explicitly. All host buffers are caller-owned. Every function returns 0 on
 * success or a PQD_ERR_* code; pqd_last_error() (thread-local) describes the last failure.
 * Nothing here ever calls exit().
 */
#ifndef PQD_H
#define PQD_H
#include <stdint.h>
#ifdef __cplusplus
extern "C" {
#endif

#define PQD_OK 0
#define PQD_ERR_ARG 1
#define PQD_ERR_HIP 2
#define PQD_ERR_UNSUPPORTED 3
#define PQD_ERR_NOMEM 4
#define PQD_ERR_NUMERIC 5

typedef struct { double re, im; } pqd_c128;
typedef struct pqd_ctx pqd_ctx;
typedef struct pqd_pt pqd_pt;
typedef struct pqd_plan pqd_plan;

/* The system: what the param file's add_Hamiltonian / add_Lindblad / add_Pulse lines say
 * (general_system.py:241-279). H(t) = H0 + sum_p (f_p(t) X_p + conj(f_p(t)) X_p^dagger). */
typedef struct {
    int32_t dim;                 /* N (Hilbert-space dimension) */
    double hbar;                 /* meV ps, constants.py:1 */
    const pqd_c128* H0;          /* N*N */
    int32_t n_lind;
    const double* lind_rates;    /* n_lind       (add_Lindblad <rate> {L}) */
    const pqd_c128* lind_ops;    /* n_lind*N*N */
    int32_t n_chan;              /* pulse / rotating-frame channels */
    const pqd_c128* chan_ops;    /* n_chan*N*N: X_p (already scaled, e.g. -0.5*pi*hbar*op) */
    const pqd_c128* chan_samples;/* n_chan*n_samples: f_p at sample_t0 + k*sample_dt */
    int32_t n_samples;
    double sample_t0, sample_dt; /* linear interpolation, clamped at both ends */
} pqd_system;

/* dt / ta / te of the param file; n_steps = round((te-ta)/dt). Output rows are steps 0..n_steps. */
typedef struct {
    double ta, dt;
    int32_t n_steps;
    int32_t n_sub;               /* exponential-midpoint sub-steps per half step (>= 1) */
} pqd_grid;

/* Process-tensor MPO for a diagonal system-bath coupling: per slice s and dictionary index g a
 * chi x chi matrix Q[s][g][d][d']; g = gmap[alpha] for Liouville index alpha. */
typedef struct {
    int32_t chi, D, n_slices;
    const pqd_c128* Q;           /* n_slices*D*chi*chi */
    const pqd_c128* closure;     /* n_slices*chi: bond closure after a step that used slice s */
    const pqd_c128* closure0;    /* chi: closure for the output at step 0 */
    const pqd_c128* bond0;       /* chi: initial bond vector */
    const int32_t* gmap;         /* N*N */
} pqd_pt_desc;

/* A batch of trajectories sharing system, grid, PT and initial state. Trajectory t is propagated
 * from step 0 to out_end[t] and writes n_out expectation values per step of [out_begin, out_end]
 * to out[out_offset[t] + (n - out_begin[t])*n_out + k]. MTOs = apply_Operator lines
 * (general_system.py:281-286): kind 0 "" (A rho A^dag), 1 "_left" (A rho), 2 "_right" (rho A);
 * before=1 is applyBefore true (visible at step), 0 visible one step later; same (traj, step,
 * before) operators apply in array order. */
typedef struct {
    int32_t n_traj;
    const int32_t* out_begin;
    const int32_t* out_end;
    const int64_t* out_offset;
    int32_t n_mto;
    const int32_t* mto_traj;
    const int32_t* mto_step;
    const int32_t* mto_before;
    const int32_t* mto_kind;
    const pqd_c128* mto_ops;     /* n_mto*N*N */
} pqd_traj;

int32_t pqd_version(void);
const char* pqd_last_error(void);
/* HIP version libpqd was built against (HIP_VERSION) and the one its loaded runtime reports (hipRuntimeGetVersion);
 * the Python loader warns when their major.minor differ (the process may have loaded another runtime first) */
int pqd_hip_versions(int32_t* build, int32_t* runtime);

int pqd_ctx_create(int32_t device, pqd_ctx** out);
void pqd_ctx_destroy(pqd_ctx* ctx);
int pqd_ctx_synchronize(pqd_ctx* ctx);

int pqd_pt_create(pqd_ctx* ctx, int32_t dim, const pqd_pt_desc* desc, pqd_pt** out);
void pqd_pt_destroy(pqd_pt* pt);

/* Reading the PT files ACE writes with `write_PT <name>`: <name>_initial, <name>_initial_0, <name>_repeated,
 * <name>_repeated_0 (reference general_system.py:146-157, 190, 194-197; detection :153-156). ACE's layout is
 * undocumented offline; the reader implements ONE stated assumption, "ACE_PTB_V0" (csrc/ace_pt.cpp header,
 * INTEGRATION.md), and returns PQD_ERR_UNSUPPORTED, naming the file and the mismatch, for anything else
 * (PQD_ERR_ARG when a file is missing). Host-only, no context. pqd_ace_pt_shape sizes the buffers;
 * pqd_ace_pt_read fills a pqd_pt_desc-shaped set of caller buffers (Q: n_slices*D*chi*chi, closure:
 * n_slices*chi, closure0/bond0: chi, gmap: dim*dim) with slices [0, n_init) from _initial and slice n_init (the
 * repeated slice) from _repeated; smaller bonds are zero-padded to chi. */
typedef struct {
    int32_t n_init, n_slices, chi, D;
} pqd_ace_pt_dims;
int pqd_ace_pt_shape(const char* name, int32_t dim, pqd_ace_pt_dims* shape);
int pqd_ace_pt_read(const char* name, int32_t dim, const pqd_ace_pt_dims* shape, pqd_c128* Q, pqd_c128* closure,
                    pqd_c128* closure0, pqd_c128* bond0, int32_t* gmap);

/* M_out: 2*n_steps matrices (N^2 x N^2, row-major): [2n] first half step, [2n+1] second. */
int pqd_free_propagators(pqd_ctx* ctx, const pqd_system* sys, const pqd_grid* grid, pqd_c128* M_out);

/* one-shot: upload, propagate, download. pt may be NULL (no phonons); sched[n_steps] selects the
 * PT slice per step (NULL: min(n, n_slices-1)). rho0: N*N. out_ops: n_out*N*N. */
int pqd_propagate(pqd_ctx* ctx, const pqd_system* sys, const pqd_grid* grid, const pqd_pt* pt,
                  const int32_t* sched, const pqd_c128* rho0, int32_t n_out, const pqd_c128* out_ops,
                  const pqd_traj* traj, pqd_c128* out, int64_t out_len);

/* multi-system batch (pulse / field parameter scans): n_sys systems of equal dim share
 * grid, PT, initial state and output operators; trajectory t uses systems[traj_sys[t]]. This replaces the
 * caller-side scan loops over ACE runs (rabi_rotations.py:172-198, the C5 pulse/B-field scan). */
int pqd_propagate_multi(pqd_ctx* ctx, int32_t n_sys, const pqd_system* systems, const int32_t* traj_sys,
                        const pqd_grid* grid, const pqd_pt* pt, const int32_t* sched, const pqd_c128* rho0,
                        int32_t n_out, const pqd_c128* out_ops, const pqd_traj* traj, pqd_c128* out,
                        int64_t out_len);

/* pqd_propagate_multi returning ACE's output table instead of the flat output buffer: per trajectory t, at offset
 * sum_{u<t} (1 + n_out) * L_u (L = out_end - out_begin + 1), (1 + n_out) rows of L values, row 0 = the times
 * ta + dt * step (imaginary part 0), row 1 + k = output k. Replaces reading the ACE outfile
 * (general_system.py:343: `np.loadtxt(outfile, dtype=complex).T`, one table per ACE run); the transposition runs on
 * the device, so a caller gets every trajectory's table as a view of one buffer. table_len >= sum of the tables. */
int pqd_propagate_table(pqd_ctx* ctx, int32_t n_sys, const pqd_system* systems, const int32_t* traj_sys,
                        const pqd_grid* grid, const pqd_pt* pt, const int32_t* sched, const pqd_c128* rho0,
                        int32_t n_out, const pqd_c128* out_ops, const pqd_traj* traj, pqd_c128* table,
                        int64_t table_len);

/* pqd_propagate_table's run reduced on the device to trapezoid integrals over each trajectory's output window, in
 * place of the tables: with y_k(s) = output k at window step s (s = 0 .. L_t - 1) and a uniform spacing dx,
 *   res[t * n_pairs + q] = dx * (y_{k_head[q]}(0) / 2 + sum_{s=1}^{L_t-2} y_{k_tail[q]}(s) + y_{k_tail[q]}(L_t - 1) / 2)
 * (0 when L_t < 2). This is the tau integral of G2_reuse (pol_entanglement/G2.py:484-505: tau = 0 from
 * <op1 op2 op3 op4> at t1, tau > 0 from <op2 op3>, np.trapz over t2) for every t1 trajectory at once; only
 * n_traj * n_pairs values leave the device. pqd_plan_trapz: the same reduction of an executed plan's outputs. */
int pqd_propagate_trapz(pqd_ctx* ctx, int32_t n_sys, const pqd_system* systems, const int32_t* traj_sys,
                        const pqd_grid* grid, const pqd_pt* pt, const int32_t* sched, const pqd_c128* rho0,
                        int32_t n_out, const pqd_c128* out_ops, const pqd_traj* traj, int32_t n_pairs,
                        const int32_t* k_head, const int32_t* k_tail, double dx, pqd_c128* res);

/* device-resident plan for repeated execution (bench, scans): same arguments as pqd_propagate(_multi). */
int pqd_plan_create(pqd_ctx* ctx, const pqd_system* sys, const pqd_grid* grid, const pqd_pt* pt,
                    const int32_t* sched, const pqd_c128* rho0, int32_t n_out, const pqd_c128* out_ops,
                    const pqd_traj* traj, int64_t out_len, pqd_plan** out);
int pqd_plan_create_multi(pqd_ctx* ctx, int32_t n_sys, const pqd_system* systems, const int32_t* traj_sys,
                          const pqd_grid* grid, const pqd_pt* pt, const int32_t* sched, const pqd_c128* rho0,
                          int32_t n_out, const pqd_c128* out_ops, const pqd_traj* traj, int64_t out_len,
                          pqd_plan** out);
/* enqueue free-propagator build (if rebuild_free) + sweep on the context stream (asynchronous) */
int pqd_plan_execute(pqd_plan* plan, int32_t rebuild_free);
/* device pointer of the plan's output buffer (out_len complex values); valid after pqd_plan_synchronize */
void* pqd_plan_output_device(pqd_plan* plan);
/* wait for the last execute and check it: a split-group launch (PQD_PATH_SPLIT) that timed out because its
 * workgroups could not all be resident (device shared with other work) is re-run on the batched kernel, and
 * the plan stays batched; a NaN/Inf output returns PQD_ERR_NUMERIC. Replaces the reference's
 * CalledProcessError on a failed ACE run (general_system.py:339-341). */
int pqd_plan_synchronize(pqd_plan* plan);
/* pqd_plan_synchronize + copy of the outputs (also on PQD_ERR_NUMERIC, which is still returned) */
int pqd_plan_download(pqd_plan* plan, pqd_c128* out, int64_t out_len);
/* pqd_plan_synchronize + copy of the outputs into `dst`, a device buffer of the plan's device (or host memory) of
 * out_len complex values, e.g. a torch tensor that a collective then gathers over xGMI (scan.py). Replaces the
 * reference's result lists assembled from per-process CSV files (correlations.py:171-183). */
int pqd_plan_copy_output(pqd_plan* plan, void* dst, int64_t out_len);
/* the plan's ACE-table length (complex values, layout of pqd_propagate_table) and pqd_plan_synchronize + the tables */
int pqd_plan_table_len(const pqd_plan* plan, int64_t* table_len);
int pqd_plan_download_table(pqd_plan* plan, pqd_c128* table, int64_t table_len);
int pqd_plan_trapz(pqd_plan* plan, int32_t n_pairs, const int32_t* k_head, const int32_t* k_tail, double dx,
                   pqd_c128* res);
#define PQD_PATH_NOPT 0     /* no PT: one wave per trajectory */
#define PQD_PATH_BATCHED 1  /* lock-step PT sweep, bt trajectories per workgroup */
#define PQD_PATH_SPLIT 2    /* one trajectory over N^2 workgroups (latency path) */
#define PQD_PATH_QUAD 3     /* two-level system: four trajectories per wave set, state in registers (pt_quad.hip) */
#define PQD_PATH_MSPLIT 4   /* several trajectories per split group: row g of TB trajectories per workgroup (pt_msplit.hip) */
/* the path the plan runs now, its trajectories per workgroup, how many split launches fell back, and the
 * trajectory-steps one execute propagates (trajectories of one system that share a lock-step workgroup propagate
 * their common MTO-free trunk once: PQD_BRANCH) */
int pqd_plan_info(const pqd_plan* plan, int32_t* path, int32_t* bt, int32_t* split_fallbacks, int64_t* traj_steps);
/* 1 when the plan builds its free propagators through pulse windows (half steps outside a system's first..last driven
 * half step are not built; its kernels read the idle operators there: DESIGN.md §4.2, PQD_WIN), else 0 */
int pqd_plan_windows(const pqd_plan* plan, int32_t* on);
/* average kernel durations (ms) of the executions since the last reset (the most recent 64 at most),
 * from HIP events on the launch stream: [0] free-propagator kernel, [1] sweep kernel; n = executions */
int pqd_plan_timing(pqd_plan* plan, double* ms_free, double* ms_sweep, int32_t* n, int32_t reset);
void pqd_plan_destroy(pqd_plan* plan);

/* ---- map-chain sweeps: reference Fortran signatures, hidden dims explicit, Fortran layouts ---- */
int pqd_propagate_tau(pqd_ctx* ctx, const pqd_c128* dm_tl, int32_t n_maps, const pqd_c128* rho_init,
                      int32_t n_tau, int32_t dim, int32_t j_start, pqd_c128* rho_out);
int pqd_calc_onetime_parallel(pqd_ctx* ctx, const pqd_c128* dm_tl, const pqd_c128* rho_init, int32_t n_tau,
                              int32_t n_t, int32_t n_tfull, int32_t dim, const pqd_c128* opA,
                              const pqd_c128* opB, const pqd_c128* opC, const double* time,
                              const double* time_sparse, pqd_c128* result);
int pqd_calc_onetime_parallel_block(pqd_ctx* ctx, const pqd_c128* dm_block, const pqd_c128* dm_s,
                                    const pqd_c128* rho_init, int32_t n_tb, int32_t nx_tau, int32_t n_map,
                                    int32_t n_t, int32_t n_tfull, int32_t dim, const pqd_c128* opA,
                                    const pqd_c128* opB, const pqd_c128* opC, const double* time,
                                    const double* time_sparse, pqd_c128* result);
int pqd_calc_twotime_phonon_block(pqd_ctx* ctx, const pqd_c128* dm_taucs2, const pqd_c128* dm_sep1,
                                  const pqd_c128* dm_sep2, const pqd_c128* dm_s, const pqd_c128* rho_init,
                                  int32_t n_tb, int32_t nx_tau, int32_t n_map, int32_t n_t, int32_t n_tfull,
                                  int32_t n_tauc, int32_t dim, const pqd_c128* opA, const pqd_c128* opB,
                                  const pqd_c128* opC, const double* time, const double* time_sparse,
                                  pqd_c128* result);
int pqd_four_time_8op(pqd_ctx* ctx, const pqd_c128* dm_1, const pqd_c128* dm_2, const pqd_c128* rho_init,
                      const double* t1, const pqd_c128* precalc, int32_t n_t, double dt, int32_t n_map,
                      int32_t dim, const pqd_c128* ops8, int32_t early_only, int32_t late_t1_only, double tb,
                      int32_t n_precalc, pqd_c128* result);
/* pqd_four_time_8op restricted to the rows i in [row_lo, row_hi) of the (t1, t2 >= t1) triangle: result(i, i + j)
 * for those rows, every other element 0. One rank's share of the pair grid split over GPUs (a
 * load-balanced triangular row split of timebin_tl.f90:255-302's loop over i; python: scan.triangular_rows). */
int pqd_four_time_8op_rows(pqd_ctx* ctx, const pqd_c128* dm_1, const pqd_c128* dm_2, const pqd_c128* rho_init,
                           const double* t1, const pqd_c128* precalc, int32_t n_t, double dt, int32_t n_map,
                           int32_t dim, const pqd_c128* ops8, int32_t early_only, int32_t late_t1_only, double tb,
                           int32_t n_precalc, int32_t row_lo, int32_t row_hi, pqd_c128* result);
int pqd_four_time(pqd_ctx* ctx, const pqd_c128* dm_1, const pqd_c128* dm_2, const pqd_c128* rho_init,
                  const double* t1, const pqd_c128* precalc, int32_t n_t, double dt, int32_t n_map, int32_t dim,
                  const pqd_c128* ops4, double tb, int32_t n_precalc, pqd_c128* result);
int pqd_dynamics_t1(pqd_ctx* ctx, const pqd_c128* dm_1, const pqd_c128* dm_2, const pqd_c128* rho_init,
                    const double* t1, const pqd_c128* precalc, int32_t n_t, double dt, int32_t n_map,
                    int32_t dim, double tb, int32_t n_precalc, pqd_c128* result);

/* ---- tau tails on one constant map (the `for j: X = tl_map2 @ X; G[:, n_tauc + j + 1] = Bt @ X` loops of
 * tl_three_op_two_time_phonons / tl_threeoptwotime_phonons_dm, reference two_time/correlations.py:866-1186) ----
 * out[i][j] = w . M^{j+1} x_i for i < n_x, j < n_steps. M: N2 x N2 row-major, X: [n_x][N2] row-major, w: N2,
 * out: [n_x][n_steps] row-major. N2 in {4, 9, 16, 25, 36}. */
int pqd_map_tail(pqd_ctx* ctx, const pqd_c128* M, int32_t N2, const pqd_c128* X, int32_t n_x, const pqd_c128* w,
                 int32_t n_steps, pqd_c128* out);

/* ---- time-local dynamical maps (replaces tools.calc_tl_dynmap_pseudo, reference tools.py:446-484) ----
 * dm: n_maps row-major n x n maps, dm[i] = E(t_{i+1}, t0). out (n_maps maps): out[0] = dm[0],
 * out[i] = dm[i] pinv(dm[i-1]) with singular values <= rcond * max(s) dropped (numpy pinv, rcond
 * 1e-12 in the reference). n <= 36 (N <= 6). */
int pqd_tl_dynmap_pseudo(pqd_ctx* ctx, const pqd_c128* dm, int32_t n_maps, int32_t n, double rcond,
                         pqd_c128* out);

/* ---- PT generator factorizations (replaces the factorizations inside `ACE <generate.param>` with
 * `dont_propagate true` + `write_PT`, reference general_system.py:152-211; driven by pyaceqd_amd/ptgen_gpu.py,
 * whose host restatement is pyaceqd_amd/ptgen.py). Device pointers, column-major matrices (ld = rows), all work
 * enqueued on `stream` (a hipStream_t). pqd_ptg_qr with pivot = 0 returns with its work still queued (its rank is
 * min(m, n)); with pivot = 1, and pqd_ptg_jacobi, it synchronises with the stream (the rank / sweep count decides
 * what the caller does next).
 *
 * pqd_ptg_qr: Householder QR of W (m x n, overwritten). pivot = 0: W = Q R with rank = min(m, n) (LAPACK zgeqrf
 * reflectors, R real diagonal). pivot = 1: column pivoting on the trailing column norms, stopping at the first step
 * whose largest trailing column norm is <= tol (a rank-revealing truncation): W P ~= Q R; tol < 0 means |tol| times
 * the largest column norm of W (found on the device: no host pass over W). pivot = 2: the same, with R returned in
 * W's own column order (R P^T: column perm[j] of the output is column j of R), so that W ~= Q R directly. Outputs: Q (m x rank),
 * R (rank x n, columns in pivoted order), perm (n: column j of W P is column perm[j] of W), *rank (host).
 * Kernel choice (environment, read per call; every combination is parity-tested): PQD_PTG_SMALL=0 (no
 * single-workgroup LDS kernel), PQD_PTG_WG=0 (per-wave column steps instead of workgroup-per-column steps with the
 * columns in registers), PQD_PTG_PAIR=0 (one reflector per launch), PQD_PTG_BLOCKED=1 (plain QRs factorized in
 * panels of 32 columns with a compact-WY trailing update), PQD_PTG_QFB=0 (Q by the per-wave reflector kernel
 * instead of blocks of 32 reflectors). */
int pqd_ptg_qr(void* stream, pqd_c128* W, int32_t m, int32_t n, int32_t pivot, double tol, pqd_c128* Q,
               pqd_c128* R, int32_t* perm, int32_t* rank);
/* pqd_ptg_jacobi: one-sided Jacobi SVD of a square n x n X (overwritten): X V = U diag(sigma), columns rotated
 * until every pair satisfies |x_p^H x_q| <= tol |x_p| |x_q|; a column with |x_j| < zero_tol ||X||_F is treated as
 * zero (never rotated). Outputs: X <- U (unit columns, unsorted), V (n x n), sigma (n, unsorted), *sweeps (host):
 * the sweeps run, the last one without a rotation, or max_sweeps + 1 when max_sweeps sweeps did not converge.
 * Scratch is kept per (device, stream): calls on different streams or devices never share a buffer. */
int pqd_ptg_jacobi(void* stream, pqd_c128* X, int32_t n, pqd_c128* V, double* sigma, double tol, double zero_tol,
                   int32_t max_sweeps, int32_t* sweeps);
/* pqd_ptg_jacobi runs its sweeps in one persistent launch (a grid barrier per round) when n <= 1024; if a barrier
 * wait times out (the workgroups were not all resident), the launch is rerun from a saved copy of X with one launch
 * per round. pqd_ptg_counters: how many times that happened in this process (diagnostics, tests). */
int pqd_ptg_counters(int32_t* jacobi_fallbacks);
/* With PQD_PTG_QPERSIST=1, pqd_ptg_qr runs a column-pivoted QR whose columns fit in registers (m <= 4096) in one
 * persistent launch (workgroup g holds physical column g; a grid barrier per step) when its n workgroups can all be
 * resident; a timed-out barrier wait reruns it from a saved copy with one launch per step (the default path, which
 * measured faster: profiles/r04/ptgen/qpersist/). PQD_PTG_QPERSIST=2 also takes plain QRs.
 * pqd_ptg_qr_counters: how many reruns happened in this process (diagnostics, tests). */
int pqd_ptg_qr_counters(int32_t* qrcp_fallbacks);

#ifdef __cplusplus
}
#endif
#endif
