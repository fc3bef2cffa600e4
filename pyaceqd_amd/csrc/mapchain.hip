// mapchain.hip — GPU restatement of the reference's Fortran dynamical-map sweeps:
//   calc_onetime_parallel (two_time/propagate_tau.f90:110-187), calc_onetime_parallel_block
//   (:189-295), calc_twotime_phonon_block (:374-536), propagate_tau (:3-19),
//   four_time / four_time_8op / dynamics_t1 (timebin/timebin_tl.f90:145-342).
// Index semantics are the Fortran ones (column-major maps and operators, 1-based map counters,
// truncating int(round_to_6(t)/dt), exact `time(j) < time_sparse(i)` comparisons); the reference's
// OpenMP "one trajectory per thread" loops become packed lanes: a 64-lane wave carries
// 64 / N2 trajectories, lane (traj, r) owns row r of that trajectory's Liouville vector.
// One wave per workgroup, so every __syncthreads() is a single s_barrier.
#include "pqd_common.h"
#include <cstdlib>

namespace {

// y = A x for a column-major N2 x N2 map; x/y in LDS; lane r of its trajectory group
__device__ __forceinline__ double2 cm_row(const double2* __restrict__ A, const double2* x, int r, int N2) {
    double2 acc = c_zero();
    for (int c = 0; c < N2; ++c) c_fma(acc, A[r + c * N2], x[c]);
    return acc;
}

// Z(e) for e = a + b*dim: sum_k X(a,k) Y(k,b) (column-major dim x dim)
__device__ __forceinline__ double2 cm_mat(const double2* X, const double2* Y, int e, int dim) {
    const int a = e % dim, b = e / dim;
    double2 acc = c_zero();
    for (int k = 0; k < dim; ++k) c_fma(acc, X[a + k * dim], Y[k + b * dim]);
    return acc;
}

__device__ __forceinline__ const double2* trunk_map(const MapChainParams& p, int j) {
    const size_t m2 = (size_t)p.N2 * p.N2;
    if (p.mode == 0) return p.dmA + (size_t)(j - 1) * m2;
    return (j <= p.n_map) ? p.dmA + (size_t)(j - 1) * m2 : p.dm_s;  // dm_block / dm_sep1, else dm_s
}

// serial trunk (propagate_tau.f90:144-165 and its block / phonon-block siblings): one wave
__global__ __launch_bounds__(64) void mc_trunk_kernel(MapChainParams p) {
    __shared__ double2 x[64], t1[64], t2[64];
    const int lane = threadIdx.x;
    const int N2 = p.N2, dim = p.dim;
    const bool on = lane < N2;
    if (on) x[lane] = p.rho_init[lane];
    __syncthreads();
    int j = 1;
    for (int i = 0; i < p.n_t; ++i) {
        while (j <= p.n_tfull && p.time[j - 1] < p.time_sparse[i]) {
            const double2* A = trunk_map(p, j);
            double2 y = on ? cm_row(A, x, lane, N2) : c_zero();
            __syncthreads();
            if (on) x[lane] = y;
            __syncthreads();
            ++j;
        }
        // result(i,1) = Tr(A (B (C rho)))
        if (on) t1[lane] = cm_mat(p.opC, x, lane, dim);
        __syncthreads();
        if (on) t2[lane] = cm_mat(p.opB, t1, lane, dim);
        __syncthreads();
        if (on) t1[lane] = cm_mat(p.opA, t2, lane, dim);
        __syncthreads();
        if (lane == 0) {
            double2 s = c_zero();
            for (int l = 0; l < dim; ++l) s = c_add(s, t1[l + l * dim]);
            p.result[i] = s;
            p.j_arr[i] = j;
        }
        __syncthreads();
        if (p.mode == 2) {
            if (on) p.rho_buf[(size_t)i * N2 + lane] = x[lane];  // :462 (MTO baked into the maps)
        } else {
            if (on) t1[lane] = cm_mat(p.opC, x, lane, dim);    // :161-163: C rho A
            __syncthreads();
            if (on) p.rho_buf[(size_t)i * N2 + lane] = cm_mat(t1, p.opA, lane, dim);
        }
        __syncthreads();
    }
}

// tau sweeps: trajectories packed TPW per wave
__global__ __launch_bounds__(64) void mc_tau_kernel(MapChainParams p) {
    __shared__ double2 xs[64], ws[64];
    const int lane = threadIdx.x;
    const int N2 = p.N2, dim = p.dim;
    const int TPW = 64 / N2;
    const int tl = lane / N2, r = lane - (lane / N2) * N2;
    const int i = blockIdx.x * TPW + tl;  // 0-based trajectory (Fortran i-1)
    const bool act = (tl < TPW) && (i < p.n_t);
    const size_t m2 = (size_t)N2 * N2;
    if (act) {
        // weights for Tr(opB R) with R(a,b) = rho[a + b dim]: lane r = b + a dim gets opB(a,b);
        // phonon block uses transpose(opB) (propagate_tau.f90:484): lane r gets opB(b,a) = opB[r]
        const int a = r / dim, b = r % dim;
        ws[lane] = (p.mode == 2) ? p.opB[r] : p.opB[a + b * dim];
        xs[lane] = p.rho_buf[(size_t)i * N2 + r];
    }
    int jj = act ? p.j_arr[i] : 1;
    int j_start = 0, use_dm2 = 1;
    if (p.mode == 2) { j_start = jj; jj = 1; }
    __syncthreads();
    const int ncol = p.n_tau + 1;
    for (int k = 2; k <= ncol; ++k) {
        double2 y = c_zero();
        if (act) {
            const double2* A;
            if (p.mode == 0) {
                A = p.dmA + (size_t)(jj - 2 + k - 1) * m2;
            } else if (p.mode == 1) {
                A = (jj <= p.n_map) ? p.dmA + (size_t)(jj - 1) * m2 : p.dm_s;
            } else {
                if (jj <= p.n_map) {
                    if (use_dm2)
                        A = (i < p.n_tauc) ? p.dmT + m2 * ((size_t)i + (size_t)p.n_tauc * (jj - 1))
                                           : p.dmB + (size_t)(jj - 1) * m2;
                    else
                        A = p.dmA + (size_t)(jj - 1) * m2;
                } else {
                    A = p.dm_s;
                }
            }
            y = cm_row(A, xs + tl * N2, r, N2);
        }
        __syncthreads();
        if (act) xs[lane] = y;
        __syncthreads();
        if (act && r == 0) {
            double2 s = c_zero();
            for (int q = 0; q < N2; ++q) c_fma(s, ws[tl * N2 + q], xs[tl * N2 + q]);
            p.result[(size_t)i + (size_t)(k - 1) * p.n_t] = s;
        }
        if (p.mode == 1) {
            jj = jj + 1;
            if (jj == p.n_tb + 1) jj = 1;
        } else if (p.mode == 2) {
            jj = jj + 1;
            if (jj + j_start == p.n_tb + 1) { j_start = 0; jj = 1; use_dm2 = 0; }
        }
    }
}

// tau sweeps, software-pipelined: the map rows of step k + PFD are loaded into registers while step k computes
// (the sweep is a chain of dependent map-vector products whose maps are inputs, so their L2/HBM latency is hidden
// behind PFD steps of arithmetic); the loop is unrolled by PFD so the register ring needs no moves, and every load is
// unconditional (past the last step the lookahead state re-reads a valid map) so the compiler's wait counts stay
// exact. x is double-buffered in LDS (one barrier per step); lane r keeps its own weighted term, lane 0 of each
// trajectory sums them. Same map sequence and arithmetic as mc_tau_kernel (kept as PQD_MC_PIPE=0).
template <int N2, int PFD>
__global__ __launch_bounds__(64) void mc_tau_pipe_kernel(MapChainParams p) {
    constexpr int TPW = 64 / N2;
    __shared__ double2 xs[2][64], ts[64];
    const int lane = threadIdx.x;
    const int dim = p.dim;
    const int tl = lane / N2, r = lane - (lane / N2) * N2;
    const int i = blockIdx.x * TPW + tl;
    const bool act = (tl < TPW) && (i < p.n_t);
    const size_t m2 = (size_t)N2 * N2;
    double2 w = c_zero();
    if (act) {
        const int a = r / dim, b = r % dim;
        w = (p.mode == 2) ? p.opB[r] : p.opB[a + b * dim];
        xs[0][lane] = p.rho_buf[(size_t)i * N2 + r];
    }
    // lookahead map state (the Fortran counters), advanced once per issued map
    int jj = act ? p.j_arr[i] : 1;
    int j_start = 0, use_dm2 = 1, kl = 2;
    if (p.mode == 2) { j_start = jj; jj = 1; }
    const int ncol = p.n_tau + 1;
    auto map_now = [&]() -> const double2* {
        if (!act || kl > ncol) return p.mode == 0 ? p.dmA : (p.mode == 1 ? p.dm_s : p.dm_s);
        if (p.mode == 0) return p.dmA + (size_t)(jj - 2 + kl - 1) * m2;
        if (p.mode == 1) return (jj <= p.n_map) ? p.dmA + (size_t)(jj - 1) * m2 : p.dm_s;
        if (jj <= p.n_map) {
            if (use_dm2)
                return (i < p.n_tauc) ? p.dmT + m2 * ((size_t)i + (size_t)p.n_tauc * (jj - 1))
                                      : p.dmB + (size_t)(jj - 1) * m2;
            return p.dmA + (size_t)(jj - 1) * m2;
        }
        return p.dm_s;
    };
    auto advance = [&]() {
        if (p.mode == 1) {
            jj = jj + 1;
            if (jj == p.n_tb + 1) jj = 1;
        } else if (p.mode == 2) {
            jj = jj + 1;
            if (jj + j_start == p.n_tb + 1) { j_start = 0; jj = 1; use_dm2 = 0; }
        }
        ++kl;
    };
    double2 am[PFD][N2];
    auto load_row = [&](int sl) {
        const double2* A = map_now() + r;
#pragma unroll
        for (int c = 0; c < N2; ++c) am[sl][c] = A[c * N2];
        advance();
    };
#pragma unroll
    for (int sl = 0; sl < PFD; ++sl) load_row(sl);
    __syncthreads();
    int cur = 0;
    // padding lanes (tl == TPW when N2 does not divide 64) read trajectory 0's vector: no LDS access past xs[.][63]
    const int tlx = tl < TPW ? tl : 0;
    auto step = [&](int sl, int k) {
        const double2* x = xs[cur] + tlx * N2;
        double2 y = c_zero();
#pragma unroll
        for (int c = 0; c < N2; ++c) c_fma(y, am[sl][c], x[c]);
        load_row(sl);  // the map of step k + PFD into the slot just used
        xs[cur ^ 1][lane] = y;
        ts[lane] = c_mul(w, y);
        __syncthreads();
        if (act && r == 0) {
            double2 s = c_zero();
#pragma unroll
            for (int q = 0; q < N2; ++q) s = c_add(s, ts[tl * N2 + q]);
            p.result[(size_t)i + (size_t)(k - 1) * p.n_t] = s;
        }
        cur ^= 1;
    };
    int k = 2;
    for (; k + PFD - 1 <= ncol; k += PFD) {
#pragma unroll
        for (int sl = 0; sl < PFD; ++sl) step(sl, k + sl);
    }
#pragma unroll
    for (int sl = 0; sl < PFD; ++sl)
        if (k + sl <= ncol) step(sl, k + sl);
}

__global__ __launch_bounds__(64) void propagate_tau_kernel(const double2* dm, const double2* rho0, int N2,
                                                           int n_tau, int j_start, double2* out) {
    __shared__ double2 x[64];
    const int lane = threadIdx.x;
    const bool on = lane < N2;
    if (on) { x[lane] = rho0[lane]; out[lane] = rho0[lane]; }
    __syncthreads();
    for (int k = 1; k <= n_tau; ++k) {
        const double2* A = dm + (size_t)(j_start + k - 1) * N2 * N2;
        double2 y = on ? cm_row(A, x, lane, N2) : c_zero();
        __syncthreads();
        if (on) { x[lane] = y; out[(size_t)k * N2 + lane] = y; }
        __syncthreads();
    }
}

// ---------------------------------------------------------------------------------------------
// timebin_tl.f90: propagate_tb with uniform control flow across the packed pairs of a wave
// ---------------------------------------------------------------------------------------------
__device__ __forceinline__ double round6(double x) { return (double)llround(x * 1000000.0) / 1000000.0; }

struct PairCtx {
    int lane, tl, r, N2, dim;
    bool act;
    double2* xs;  // LDS base of this wave's packed vectors
};

__device__ int wave_max(int v, int* red) {
    // one-wave workgroup: reduce through LDS
    __syncthreads();
    if (threadIdx.x == 0) *red = INT_MIN;
    __syncthreads();
    atomicMax(red, v);
    __syncthreads();
    const int m = *red;
    __syncthreads();
    return m;
}

// in-place on this pair's vector xs[tl*N2 ...]; maps column-major, dm index 0-based n_start
__device__ void prop_tb(const PairCtx& c, double ts, double te, double dt, const double2* dm, int n_dm,
                        const double2* precalc, int n_precalc, int* red) {
    const size_t m2 = (size_t)c.N2 * c.N2;
    int n_start = (int)(round6(ts) / dt);
    const int n_stop = (int)(round6(te) / dt);
    int n_steps = n_stop - n_start;
    int steps_dm = (n_dm - n_start) < n_steps ? (n_dm - n_start) : n_steps;
    if (!c.act) { steps_dm = 0; n_steps = 0; }
    const int mx = wave_max(steps_dm, red);
    for (int s = 0; s < mx; ++s) {
        const bool go = c.act && s < steps_dm;
        double2 y = go ? cm_row(dm + (size_t)(n_start + s) * m2, c.xs + c.tl * c.N2, c.r, c.N2) : c_zero();
        __syncthreads();
        if (go) c.xs[c.lane] = y;
        __syncthreads();
    }
    if (steps_dm > 0) n_steps -= steps_dm;
    const int rem = n_steps > 0 ? n_steps : 0;
    const int mrem = wave_max(rem, red);
    for (int bit = 0; bit < n_precalc && (mrem >> bit) > 0; ++bit) {
        const bool go = c.act && ((rem >> bit) & 1);
        double2 y = go ? cm_row(precalc + (size_t)bit * m2, c.xs + c.tl * c.N2, c.r, c.N2) : c_zero();
        __syncthreads();
        if (go) c.xs[c.lane] = y;
        __syncthreads();
    }
}

__device__ void pair_op(const PairCtx& c, const double2* op, bool right, double2* tmp) {
    double2 y = c_zero();
    if (c.act) {
        const double2* X = c.xs + c.tl * c.N2;
        y = right ? cm_mat(X, op, c.r, c.dim) : cm_mat(op, X, c.r, c.dim);
    }
    __syncthreads();
    if (c.act) c.xs[c.lane] = y;
    __syncthreads();
    (void)tmp;
}

__device__ double2 pair_trace(const PairCtx& c) {
    double2 s = c_zero();
    for (int l = 0; l < c.dim; ++l) s = c_add(s, c.xs[c.tl * c.N2 + l + l * c.dim]);
    return s;
}

// rho_vec(i) = propagate_tb(0, t1(i), dm_1, rho_init) for all i (the per-i prologue of four_time*)
__global__ __launch_bounds__(64) void ft_prologue_kernel(FourTimeParams p, double2* rho_i) {
    __shared__ double2 xs[64];
    __shared__ int red;
    PairCtx c;
    c.lane = threadIdx.x; c.N2 = p.N2; c.dim = p.dim;
    const int TPW = 64 / p.N2;
    c.tl = c.lane / p.N2; c.r = c.lane - c.tl * p.N2;
    const int i = blockIdx.x * TPW + c.tl;
    c.act = c.tl < TPW && i < p.n_t;
    c.xs = xs;
    if (c.act) xs[c.lane] = p.rho_init[c.r];
    __syncthreads();
    prop_tb(c, 0.0, c.act ? p.t1[i] : 0.0, p.dt, p.dm1, p.n_map, p.precalc, p.n_precalc, &red);
    if (c.act) rho_i[(size_t)i * p.N2 + c.r] = xs[c.lane];
}

__global__ __launch_bounds__(64) void ft_pairs_kernel(FourTimeParams p, const double2* rho_i) {
    __shared__ double2 xs[64];
    __shared__ int red;
    PairCtx c;
    c.lane = threadIdx.x; c.N2 = p.N2; c.dim = p.dim;
    const int TPW = 64 / p.N2;
    c.tl = c.lane / p.N2; c.r = c.lane - c.tl * p.N2;
    const int pidx = blockIdx.x * TPW + c.tl;
    c.act = c.tl < TPW && pidx < p.n_pairs;
    c.xs = xs;
    int i = 0, j = 0;
    if (c.act) { const int2 ij = p.pairs[pidx]; i = ij.x; j = ij.y; }
    const double t1n = c.act ? p.t1[i] : 0.0;
    const double t2 = c.act ? p.t1[i + j] : 0.0;
    if (c.act) xs[c.lane] = rho_i[(size_t)i * p.N2 + c.r];
    __syncthreads();
    const size_t o2 = (size_t)p.N2;
    const double2* O = p.ops;
    bool done = false;
    double2 res = c_zero();
    if (p.variant == 0) {
        pair_op(c, O + 1 * o2, true, nullptr);   // op_et1r
        pair_op(c, O + 0 * o2, false, nullptr);  // op_et1l
        prop_tb(c, t1n, t2, p.dt, p.dm1, p.n_map, p.precalc, p.n_precalc, &red);
        pair_op(c, O + 3 * o2, true, nullptr);   // op_et2r
        pair_op(c, O + 2 * o2, false, nullptr);  // op_et2l
        if (p.early_only) { res = pair_trace(c); done = true; }
        if (!p.early_only) {
            prop_tb(c, t2, p.tb, p.dt, p.dm1, p.n_map, p.precalc, p.n_precalc, &red);
            prop_tb(c, 0.0, t1n, p.dt, p.dm2, p.n_map, p.precalc, p.n_precalc, &red);
            pair_op(c, O + 5 * o2, true, nullptr);   // op_lt1r
            pair_op(c, O + 4 * o2, false, nullptr);  // op_lt1l
            if (p.late_t1_only) { res = pair_trace(c); done = true; }
            if (!p.late_t1_only) {
                prop_tb(c, t1n, t2, p.dt, p.dm2, p.n_map, p.precalc, p.n_precalc, &red);
                pair_op(c, O + 7 * o2, true, nullptr);   // op_lt2r
                pair_op(c, O + 6 * o2, false, nullptr);  // op_lt2l
                res = pair_trace(c); done = true;
            }
        }
    } else {
        pair_op(c, O + 0 * o2, true, nullptr);
        prop_tb(c, t1n, t2, p.dt, p.dm1, p.n_map, p.precalc, p.n_precalc, &red);
        pair_op(c, O + 1 * o2, true, nullptr);
        prop_tb(c, t2, p.tb, p.dt, p.dm1, p.n_map, p.precalc, p.n_precalc, &red);
        prop_tb(c, 0.0, t1n, p.dt, p.dm2, p.n_map, p.precalc, p.n_precalc, &red);
        pair_op(c, O + 2 * o2, false, nullptr);
        prop_tb(c, t1n, t2, p.dt, p.dm2, p.n_map, p.precalc, p.n_precalc, &red);
        pair_op(c, O + 3 * o2, false, nullptr);
        res = pair_trace(c); done = true;
    }
    if (c.act && c.r == 0 && done) p.result[(size_t)i + (size_t)(i + j) * p.n_t] = res;
}

__global__ __launch_bounds__(64) void dyn_t1_kernel(FourTimeParams p, double2* out) {
    __shared__ double2 xs[64];
    __shared__ int red;
    PairCtx c;
    c.lane = threadIdx.x; c.N2 = p.N2; c.dim = p.dim;
    c.tl = 0; c.r = c.lane; c.act = c.lane < p.N2; c.xs = xs;
    if (c.act) { xs[c.lane] = p.rho_init[c.lane]; out[c.lane] = p.rho_init[c.lane]; }
    __syncthreads();
    for (int half = 0; half < 2; ++half) {
        const double2* dm = half == 0 ? p.dm1 : p.dm2;
        for (int i = 0; i <= p.n_t - 2; ++i) {
            prop_tb(c, p.t1[i], p.t1[i + 1], p.dt, dm, p.n_map, p.precalc, p.n_precalc, &red);
            if (c.act) out[(size_t)(i + 1 + half * (p.n_t - 1)) * p.N2 + c.lane] = xs[c.lane];
            __syncthreads();
        }
    }
}

}  // namespace

hipError_t launch_mapchain(const MapChainParams& p, hipStream_t s) {
    hipLaunchKernelGGL(mc_trunk_kernel, dim3(1), dim3(64), 0, s, p);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    const int TPW = 64 / p.N2;
    const int nblk = (p.n_t + TPW - 1) / TPW;
    if (nblk <= 0 || p.n_tau <= 0) return hipGetLastError();
    const char* pe = getenv("PQD_MC_PIPE");
    if (!(pe && atoi(pe) == 0)) {
        switch (p.N2) {
            case 4: hipLaunchKernelGGL((mc_tau_pipe_kernel<4, 4>), dim3(nblk), dim3(64), 0, s, p); return hipGetLastError();
            case 9: hipLaunchKernelGGL((mc_tau_pipe_kernel<9, 2>), dim3(nblk), dim3(64), 0, s, p); return hipGetLastError();
            case 16: hipLaunchKernelGGL((mc_tau_pipe_kernel<16, 2>), dim3(nblk), dim3(64), 0, s, p); return hipGetLastError();
            case 25: hipLaunchKernelGGL((mc_tau_pipe_kernel<25, 1>), dim3(nblk), dim3(64), 0, s, p); return hipGetLastError();
            case 36: hipLaunchKernelGGL((mc_tau_pipe_kernel<36, 1>), dim3(nblk), dim3(64), 0, s, p); return hipGetLastError();
            default: break;
        }
    }
    hipLaunchKernelGGL(mc_tau_kernel, dim3(nblk), dim3(64), 0, s, p);
    return hipGetLastError();
}

hipError_t launch_propagate_tau(int N2, const double2* dm, const double2* rho0, int n_tau, int j_start,
                                double2* out, hipStream_t s) {
    hipLaunchKernelGGL(propagate_tau_kernel, dim3(1), dim3(64), 0, s, dm, rho0, N2, n_tau, j_start, out);
    return hipGetLastError();
}

// scratch rho_i (n_t*N2) is carried in p.result's tail by the host (see pqd_host.cpp)
hipError_t launch_four_time(const FourTimeParams& p, hipStream_t s) {
    const int TPW = 64 / p.N2;
    double2* rho_i = p.result + (size_t)p.n_t * p.n_t;
    hipLaunchKernelGGL(ft_prologue_kernel, dim3((p.n_t + TPW - 1) / TPW), dim3(64), 0, s, p, rho_i);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    if (p.n_pairs > 0)
        hipLaunchKernelGGL(ft_pairs_kernel, dim3((p.n_pairs + TPW - 1) / TPW), dim3(64), 0, s, p,
                           (const double2*)rho_i);
    return hipGetLastError();
}

hipError_t launch_dynamics_t1(const FourTimeParams& p, double2* out, hipStream_t s) {
    hipLaunchKernelGGL(dyn_t1_kernel, dim3(1), dim3(64), 0, s, p, out);
    return hipGetLastError();
}
