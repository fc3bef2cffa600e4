// pqd_common.h — shared device/host definitions for libpqd (gfx950 / CDNA4 only).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <climits>

#define PQD_WAVE 64

// ---------------------------------------------------------------------------------------------
// complex double helpers (interleaved re, im == pqd_c128 == double2)
// ---------------------------------------------------------------------------------------------
__device__ __forceinline__ double2 c_zero() { return make_double2(0.0, 0.0); }
__device__ __forceinline__ double2 c_add(double2 a, double2 b) { return make_double2(a.x + b.x, a.y + b.y); }
__device__ __forceinline__ double2 c_sub(double2 a, double2 b) { return make_double2(a.x - b.x, a.y - b.y); }
__device__ __forceinline__ double2 c_scale(double2 a, double s) { return make_double2(a.x * s, a.y * s); }
__device__ __forceinline__ double2 c_conj(double2 a) { return make_double2(a.x, -a.y); }
__device__ __forceinline__ double2 c_mul(double2 a, double2 b) {
    return make_double2(fma(a.x, b.x, -a.y * b.y), fma(a.x, b.y, a.y * b.x));
}
// acc += a * b  (4 FMAs)
__device__ __forceinline__ void c_fma(double2& acc, double2 a, double2 b) {
    acc.x = fma(a.x, b.x, acc.x);
    acc.x = fma(-a.y, b.y, acc.x);
    acc.y = fma(a.x, b.y, acc.y);
    acc.y = fma(a.y, b.x, acc.y);
}
__device__ __forceinline__ double2 c_shfl_xor(double2 v, int m) {
    return make_double2(__shfl_xor(v.x, m), __shfl_xor(v.y, m));
}
// one DPP move of a double inside a 16-lane row (two 32-bit moves; no LDS round trip, unlike __shfl_xor's ds_bpermute)
template <int CTRL>
__device__ __forceinline__ double dpp_d(double v) {
    const long long b = __double_as_longlong(v);
    const int lo = __builtin_amdgcn_update_dpp(0, (int)b, CTRL, 0xF, 0xF, false);
    const int hi = __builtin_amdgcn_update_dpp(0, (int)(b >> 32), CTRL, 0xF, 0xF, false);
    return __longlong_as_double(((long long)hi << 32) | (unsigned)lo);
}
// sum over each group of W (4 or 16) consecutive lanes, left in every lane of the group with the same bits (each step
// adds the same pair in either order): quad_perm [1,0,3,2], quad_perm [2,3,0,1], then row_half_mirror, row_mirror.
// Every lane of the wave must be active.
template <int W>
__device__ __forceinline__ double2 c_group_sum(double2 v) {
    static_assert(W == 4 || W == 16, "lane groups of 4 or 16");
    v = c_add(v, make_double2(dpp_d<0xB1>(v.x), dpp_d<0xB1>(v.y)));
    v = c_add(v, make_double2(dpp_d<0x4E>(v.x), dpp_d<0x4E>(v.y)));
    if constexpr (W == 16) {
        v = c_add(v, make_double2(dpp_d<0x141>(v.x), dpp_d<0x141>(v.y)));
        v = c_add(v, make_double2(dpp_d<0x140>(v.x), dpp_d<0x140>(v.y)));
    }
    return v;
}
// acc += pv(lane J of this lane's 16-lane row) * s, as c_fma (same order of the four products): v_fmac_f64 with its
// first source taken by DPP row_newbcast, so a row value held once per row feeds the 16 lanes of the row. Every lane of
// the wave must be active (the PT runs whole waves)
template <int J>
__device__ __forceinline__ void pq_cmac_bcast(double2& acc, const double2 pv, const double2 s) {
    asm volatile(
        "v_fmac_f64_dpp %0, %2, %4 row_newbcast:%c6 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %0, -%3, %5 row_newbcast:%c6 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %1, %2, %5 row_newbcast:%c6 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %1, %3, %4 row_newbcast:%c6 row_mask:0xf bank_mask:0xf"
        : "+v"(acc.x), "+v"(acc.y)
        : "v"(pv.x), "v"(pv.y), "v"(s.x), "v"(s.y), "i"(J));
}
// sum over j < KP of pv[j / 16](lane j % 16) * sreg[j]
template <int J, int KP, int NPV, int NS>
__device__ __forceinline__ void pq_row_bcast_mac(double2& acc, const double2 (&pv)[NPV], const double2 (&sreg)[NS]) {
    if constexpr (J < KP) {
        pq_cmac_bcast<J % 16>(acc, pv[J / 16], sreg[J]);
        pq_row_bcast_mac<J + 1, KP>(acc, pv, sreg);
    }
}
// a DPP source must not be written by a VALU instruction in the two cycles before it (the row values come from LDS
// reads; this keeps two wait states after whatever the compiler puts between them and the products)
template <int NPV>
__device__ __forceinline__ void pq_dpp_src_ready(const double2 (&pv)[NPV]) {
#pragma unroll
    for (int c = 0; c < NPV; ++c) asm volatile("" ::"v"(pv[c].x), "v"(pv[c].y));
    asm volatile("s_nop 1");
}

// x[l] + x[l ^ W] for W = 32 or 16 in every lane l, the same bits in both partners (each adds the same pair): gfx950's
// v_permlane32_swap / v_permlane16_swap, one VALU move per 32-bit half instead of an LDS round trip. Whichever half
// each swap moves, its two results hold x[l] and x[l ^ W] in some order, so their sum is the pair's.
template <int W>
__device__ __forceinline__ double xor_add(double x) {
    static_assert(W == 32 || W == 16, "permlane swaps pair lanes 32 or 16 apart");
    const long long b = __double_as_longlong(x);
    const unsigned lo = (unsigned)b, hi = (unsigned)(b >> 32);
    unsigned l0, l1, h0, h1;
    if constexpr (W == 32) {
        const auto sl = __builtin_amdgcn_permlane32_swap(lo, lo, false, false);
        const auto sh = __builtin_amdgcn_permlane32_swap(hi, hi, false, false);
        l0 = sl[0]; l1 = sl[1]; h0 = sh[0]; h1 = sh[1];
    } else {
        const auto sl = __builtin_amdgcn_permlane16_swap(lo, lo, false, false);
        const auto sh = __builtin_amdgcn_permlane16_swap(hi, hi, false, false);
        l0 = sl[0]; l1 = sl[1]; h0 = sh[0]; h1 = sh[1];
    }
    return __longlong_as_double(((long long)h0 << 32) | l0) + __longlong_as_double(((long long)h1 << 32) | l1);
}

// ---------------------------------------------------------------------------------------------
// kernel parameter blocks (passed by value)
// ---------------------------------------------------------------------------------------------
struct FreePropSys {           // one system of a (possibly multi-system) plan
    const double2* L0;       // N2*N2 constant Liouvillian (H0 commutator + dissipators), row-major
    const double2* S;        // n_chan*N2*N2 superoperator of -i/hbar [X_p, .]
    const double2* T;        // n_chan*N2*N2 superoperator of -i/hbar [X_p^dagger, .]
    const double2* samples;  // n_chan*n_samples
    int n_chan, n_samples;
    double s_t0, s_dt;
};

struct FreePropParams {
    const FreePropSys* systems;  // device table, n_sys entries
    int n_sys;
    double ta, dt;
    int n_steps, n_sub;
    double2* M;              // out: n_sys*2*n_steps*N2*N2
    int packed4;             // N2 = 4: 16 matrices per workgroup (free_prop4_kernel); 0: the general kernel (A/B)
    double2* Midle;          // n_sys*N2*N2: exp(L0 w)^n_sub, the propagator of a half step whose pulse samples are all
                             //   exactly zero (built first, copied for every such half step); NULL: always compute
    int idle_pass;           // 1: this launch builds Midle (one matrix per system, samples taken as 0)
    int2* win;               // n_sys pulse windows (lo, hi): every half step h < lo or h > hi is idle and is NOT stored
                             //   (readers take Midle, see fw_M); NULL: every half step stored (copies of Midle)
    int chunk;               // free_prop4_kernel: half steps per workgroup (set by its launcher)
    int mfma;                // N2 = 25, 36: products on the matrix cores (free_prop_mfma_kernel; PQD_FPM=0: LDS kernel)
};

struct SweepParams {
    const double2* M;        // 2*n_steps*N2*N2 free propagators
    const double2* Q;        // PT slices n_slices*D*CHI*CHI (chi padded to CHI)
    const double* Qsum;      // Re + Im of Q (N2 = 4 PTs: the quad kernel's 3M operand), else NULL
    int D;
    const int* sched;        // n_steps
    const double2* closure;  // n_slices*CHI
    const double2* closure0; // CHI
    const double2* bond0;    // CHI
    const int* gmap;         // N2
    const double2* rho0;     // N2 (row-major vec)
    int n_out;
    const double2* ovec;     // n_out*N2: ovec[k][i*N+j] = O_k[j][i]  => <O_k> = sum_a ovec[k][a] r[a]
    const int* blk_traj;     // n_blocks*BT trajectory ids (-1: empty slot)
    const int* blk_end;      // n_blocks: last step of the block (max out_end)
    const int* blk_sys;      // n_blocks: system of the block's first trajectory (waves index traj_sys)
    const int* blk_act;      // n_blocks*BT: step at which the slot becomes active (shared trunk, see pqd_host.cpp
                             //   branch_slots; 0 = from the start, INT_MAX = empty slot)
    const int* blk_src;      // n_blocks*BT: at activation copy the (state, fused flag) of this slot (>= 0), or load
                             //   checkpoint -2 - src of the trunk pre-pass (<= -2; fused flag 1); -1: fresh start
    double2* ck;             // trunk checkpoints [n_ck][N2][CHI] (dense rows): augmented state at the top of a step
    const int* ck_map;       // trunk pre-pass only: ck_map[t * ck_stride + n] = checkpoint written at the top of step
    long long ck_stride;     //   n by trajectory t (-1: none); NULL in the main sweep
    const int* traj_sys;     // n_traj: system of each trajectory (chi = 1 kernel)
    long long m_stride;      // complex elements between the free propagators of consecutive systems
    const int* wbeg;         // per trajectory
    const int* wend;
    const long long* woff;
    const int* ev_start;     // n_traj+1
    const int4* ev;          // (step, after?1:0, superop index, 0), sorted per trajectory
    const double2* sop;      // MTO superoperators N2*N2 each
    double2* out;
    const double2* F;        // fused half steps F(m) = M_a(m) M_b(m-1)   [n_sys][n_steps][N2 x N2]
    const double2* W;        // output rows through M_b(m-1): W(m) = ovec . M_b(m-1)   [n_sys][n_steps+1][n_out][N2]
    long long f_stride, w_stride;
    int fuse;                // 1: steps without MTOs apply F(m) once instead of M_b(m-1) then M_a(m)
    int pt_mode;             // PT contraction: 0 VALU, 1 matrix cores (4x4x4_4b), 2 mixed per wave,
                             //   3 split-complex 16x16x4 (BT = 8), 4 matrix cores with 3 real products (3M)
    int cmul3;               // column phases with 3 real products per complex product (3M)
    const int4* units;       // 3M PT rows per wave: [waves][umax] (slice, row 0, row 1 or -1, row 2 | row 3 << 16 or -1;
                             //   a missing row 3 is 0x7FFF),
    int umax;                //   a unit with slice < 0 ends a wave's list; NULL: rows a = wave + k BT
    int trpre;               // 1: traces one lane per (trajectory, output, row), W rows fetched a step ahead
    int ablate;              // diagnostics only (PQD_ABLATE): 1 skip PT, 2 skip column phases, 4 skip outputs
    int split_gran;          // split groups: data-tagged granule exchange (PQD_SPLIT_GRAN=1; default 0: counter form)
    int split_ow;            // split groups, counter form: one output workgroup per group (default 1; PQD_SPLIT_OW=0 off)
    unsigned* flags;         // bit 0: a non-finite output value (set by launch_check_finite at synchronize)
    unsigned spin_limit;     // split groups: polls before a wait for the peers times out (PQD_SPLIT_SPIN, tests)
    int traj_base;           // split groups: trajectory of group 0 (a batch run as several co-resident launches)
    int split_xcd;           // split groups, set per launch: > 0 = trajectories in this launch, each group's workgroups
                             //   dealt onto one XCD (blocks b with equal b % 8; speed only, PQD_SPLIT_XCD=0 off)
    int split_l2;            // split groups on the XCD-grouped grid: exchange lines kept in the group's L2 (placement
                             //   checked at the first poll; PQD_SPLIT_L2=0: sc1 stores)
    int n_steps;             // grid steps (operand prefetch bound)
    int n_blk;               // blocks of the launch (quad kernel: quads; tail workgroups check it)
    int qprio;               // quad kernel wave priorities (PQD_QPRIO, A/B): bit 0 first half of the grid above the
                             //   second, bit 1 raised outside the PT contraction
    const int2* win;         // per-system pulse windows (FreePropParams::win) or NULL; outside them M, F, W are the
    const double2* Midle;    //   system's idle operators: Midle [n_sys][N2 x N2], Fidle = Midle Midle [n_sys][N2 x N2],
    const double2* Fidle;    //   Widle = ovec . Midle [n_sys][n_out][N2]
    const double2* Widle;
    int colbig;              // N2 > 16 column phases: one pass over k for all of a wave's tiles (1, PQD_COLBIG; 0: per tile)
};

// split groups with several trajectories per group (pt_msplit.hip)
struct MsplitParams {
    const int* gtraj;        // n_groups * TB trajectory ids (-1: empty slot)
    const int* gend;         // n_groups: last step of the group (max out_end of its trajectories)
    const int* cev_start;    // n_traj + 1: composite events of trajectory t are cev[cev_start[t] .. cev_start[t + 1])
    const int4* cev;         // (step, MTO superoperator before or -1, after or -1, system), steps ascending per trajectory
    double2* Fev;            // [n_cev][N2 x N2]: M_a(s) S_after S_before M_b(s - 1) (M_b(-1) = 1; zero at s = n_steps)
    double2* Wev;            // [n_cev][n_out][N2]: ovec S_before M_b(s - 1)
    int TB, n_groups;        // trajectories per group, groups
    int xcd;                 // > 0: XCD-grouped grid with this many groups per XCD slot; 0: plain grid
    int l2keep;              // 1: payload stores keep their L2 lines (XCD-grouped grid only; placement checked in-kernel)
    int ptm;                 // 1: PT contraction on the matrix cores (3M, 4 trajectories per row block), 0: FP64 VALU
};

// ---- free propagators through the pulse windows: M(h), F(n) = M(2n) M(2n-1) and W(n) = ovec . M(2n-1) of system sys
// are stored only where the half steps involved lie inside the system's window [lo, hi]; outside, the propagator is
// the idle one (the same bits the builder copied there before windows: Midle, and Fidle / Widle computed from it by
// the fuse kernels' own arithmetic)
__device__ __forceinline__ int2 fw_win(const SweepParams& p, int sys) {
    return p.win ? p.win[sys] : make_int2(INT_MIN, INT_MAX);
}
__device__ __forceinline__ bool fw_out(int2 w, int h) { return h < w.x || h > w.y; }
__device__ __forceinline__ const double2* fw_M(const SweepParams& p, int sys, int2 w, int h, int m2) {
    return fw_out(w, h) ? p.Midle + (size_t)sys * m2 : p.M + (size_t)sys * p.m_stride + (size_t)h * m2;
}
__device__ __forceinline__ const double2* fw_F(const SweepParams& p, int sys, int2 w, int n, int m2) {
    return (fw_out(w, 2 * n - 1) && fw_out(w, 2 * n)) ? p.Fidle + (size_t)sys * m2
                                                      : p.F + (size_t)sys * p.f_stride + (size_t)n * m2;
}
// the n_out rows of W(n) (n_out * N2 elements)
__device__ __forceinline__ const double2* fw_W(const SweepParams& p, int sys, int2 w, int n, int N2) {
    return fw_out(w, 2 * n - 1) ? p.Widle + (size_t)sys * p.n_out * N2
                                : p.W + (size_t)sys * p.w_stride + (size_t)n * p.n_out * N2;
}



// map-chain (Fortran f2py equivalents)
struct MapChainParams {
    int mode;                // 0 onetime, 1 onetime_block, 2 twotime_phonon_block
    int dim, N2;
    const double2* dmA;      // mode0: dm_tl   mode1: dm_block   mode2: dm_sep1
    const double2* dmB;      // mode2: dm_sep2
    const double2* dmT;      // mode2: dm_taucs2 (N2,N2,n_tauc,n_map)
    const double2* dm_s;     // mode1/2 stationary map
    int n_map, n_tb, nx_tau, n_tauc;
    const double2* rho_init;
    const double2* opA; const double2* opB; const double2* opC;   // Fortran column-major dim x dim
    const double* time; const double* time_sparse;
    int n_t, n_tfull, n_tau;  // n_tau: number of tau columns after the first (ncol-1)
    double2* rho_buf;        // scratch n_t*N2
    int* j_arr;              // scratch n_t
    double2* result;         // (n_t, n_tau+1) column-major
    // blocked tau sweep (mode 0, mapchain.hip "blocked"): positions q = map index 0.., blocks of L positions
    int L, n_blk, Q;         // block length, blocks, positions with maps [0, Q)
    int q_s;                 // mode 1: positions >= q_s map to dm_s (trajectories whose trunk ends past n_tb)
    const int* pos;          // n_t: p_i = j_i - 1, host-computed trunk end (first tau map)
    double2* U;              // Q*N2: U[q] = w^T E[q] ... E[cL] (c = q / L)
    double2* Rend;           // n_blk*N2*N2: E[end of block c] ... E[cL], column-major
    double2* P;              // n_blk*N2: trunk state before block c
    double2* X;              // n_blk*n_t*N2: trajectory i's tau state before block c
};

struct FourTimeParams {
    int dim, N2, n_t, n_map, n_precalc;
    double dt, tb;
    const double2* dm1; const double2* dm2; const double2* precalc;  // Fortran layouts
    const double2* rho_init;
    const double* t1;
    const double2* ops;      // 8 (or 4) Fortran dim x dim
    int variant;             // 0: four_time_8op, 1: four_time (4 ops)
    int early_only, late_t1_only;
    const int2* pairs;       // (i, j) list
    int n_pairs;
    double2* result;         // (n_t, n_t) column-major
};

// launchers (defined in the .hip translation units)
struct FuseParams {          // F(m) = M_a(m) M_b(m-1) (1 <= m < n_steps), W(m) = ovec . M_b(m-1) (1 <= m <= n_steps)
    const double2* M;
    double2* F;
    double2* W;
    const double2* ovec;
    int n_sys, n_steps, n_out;
    const int2* win;         // FreePropParams::win or NULL: F(m) / W(m) whose half steps are all outside are not stored
    const double2* Midle;    // with win: the idle pass writes Fidle = Midle Midle and Widle = ovec . Midle per system
    double2* Fidle;
    double2* Widle;
    int mfma;                // N2 = 25, 36: F(m) on the matrix cores (fuse_steps_mfma_kernel; follows PQD_FPM)
};

hipError_t launch_free_prop(int N2, const FreePropParams& p, hipStream_t s);
hipError_t launch_free_win(const FreePropParams& p, hipStream_t s);
// flags |= 1 if any of the n complex values is NaN or Inf (one pass over the output buffer at synchronize: the sweep
// kernels carry no per-store check, which cost 1.7% of the headline kernel)
hipError_t launch_check_finite(const double2* v, int64_t n, unsigned* flags, hipStream_t s);
hipError_t launch_table(const double2* out, const long long* woff, const int* wbeg, const int* wend,
                        const long long* toff, int n_traj, int n_out, double t_start, double dt, double2* table,
                        hipStream_t s);
hipError_t launch_fuse_steps(int N2, const FuseParams& p, hipStream_t s);
hipError_t launch_trapz(const double2* out, const long long* woff, const int* wbeg, const int* wend, int n_traj,
                        int n_out, int n_pairs, const int* kh, const int* kt, double dx, double2* res, hipStream_t s);
// waves per trajectory in the PT sweep: a 4-trajectory workgroup (N2 > 16 or chi = 128) runs 8 waves, two per
// trajectory (each owns half of the bond columns in the column phases), so every SIMD holds two waves
// (N2 = 4 included: one wave per trajectory there, four waves per workgroup and two workgroups per CU, measured
// slower on the TLS scan, 38.4 -> 68.8 ms, profiles/r02/cfg_c2_bt4.log)
constexpr int sweep_wpt(int N2, int BT, int CHI) { return (BT == 4 && CHI >= 32) ? 2 : 1; }
// rows per PT unit (rows sharing one dictionary slice contracted together): 3 R (BT/4) (CHI/16) accumulators <= 48
// (quads only at N2 > 16, where the 4-trajectory slice stream is L2-bound; smaller N2 keep pairs)
constexpr int sweep_rmax(int N2, int BT, int CHI) {
    const int acc = (BT >= 8 ? BT / 4 : 1) * (CHI >= 16 ? CHI / 16 : 1);  // accumulators per row and product
    const int r = 16 / acc >= 4 ? 4 : (16 / acc >= 2 ? 2 : 1);
    return N2 > 16 ? r : (r > 2 ? 2 : r);
}
hipError_t launch_sweep(int N2, int CHI, int BT, int n_blocks, const SweepParams& p, hipStream_t s);
int sweep_max_bt(int N2);
hipError_t launch_sweep_nopt(int N2, int n_blocks, const SweepParams& p, hipStream_t s);
hipError_t launch_mapchain(const MapChainParams& p, hipStream_t s);
hipError_t launch_mapchain_blocked(const MapChainParams& p, int n_chain, hipStream_t s);
hipError_t launch_four_time(const FourTimeParams& p, hipStream_t s);
hipError_t launch_propagate_tau(int N2, const double2* dm, const double2* rho0, int n_tau, int j_start,
                                double2* out, hipStream_t s);
hipError_t launch_dynamics_t1(const FourTimeParams& p, double2* out, hipStream_t s);
hipError_t launch_map_tail(int N2, const double2* M, const double2* X, int n_x, const double2* w, int n_steps,
                           double2* out, hipStream_t s);
hipError_t launch_tl_dynmap(const double2* dm, int n_maps, int n, double rcond, double2* out, hipStream_t s);
int tl_dynmap_nmax();
bool split_supported(int N2, int CHI, int n_traj, int n_cu);
int split_group_size(int N2);  // workgroups per split group (N2, or N2 + 1 with the output workgroup)
bool split_ow_env();
int split_blocks_per_cu(int N2, int CHI);
hipError_t launch_split(int N2, int CHI, int n_traj, const SweepParams& p, double2* X, unsigned* cnt,
                        unsigned* err, hipStream_t s, int chunk = 0);
bool sweep_supported(int N2, int CHI);
// split groups carrying TB trajectories each (pt_msplit.hip)
bool msplit_supported(int N2, int CHI, int n_out);
int msplit_tbmax(int N2, int CHI);
int msplit_cev_max();  // composite MTO steps per group (held in LDS)
int msplit_group_size(int N2, int CHI);  // workgroups per group (each owns up to R PT rows of every trajectory)
int msplit_blocks_per_cu(int N2, int CHI);
hipError_t launch_evcomp(int N2, const SweepParams& p, const MsplitParams& q, int n_cev, int n_steps, hipStream_t s);
hipError_t launch_msplit(int N2, int CHI, const SweepParams& p, const MsplitParams& q, double2* X, unsigned* cnt,
                         unsigned* err, hipStream_t s);
// the register-resident TLS sweep (pt_quad.hip): four trajectories per block, CHI/16 waves each
bool quad_supported(int N2, int CHI);
// ncg: 4-column groups per wave, 4 (strips of 16 columns, one wave per SIMD) or 2 (strips of 8, two waves per SIMD)
int quad_qpw(int CHI, int qpw, int ncg);  // quads per workgroup launch_quad instantiates
hipError_t launch_quad(int CHI, int n_quads, int qpw, int ncg, const SweepParams& p, hipStream_t s);

// thread-local last error shared by the host translation units (pqd_host.cpp owns it); returns code
extern "C" int pqd_fail_msg(int code, const char* msg);
