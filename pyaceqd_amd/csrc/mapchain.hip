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
#include <algorithm>
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

// ---------------------------------------------------------------------------------------------
// Blocked sweep for calc_onetime_parallel (mode 0). Every trajectory i runs along the same map sequence E[q]
// (q = map index, 0-based): the trunk applies E[0 .. p_i - 1], the tau sweep E[p_i .. p_i + n_tau - 1]
// (p_i = j_i - 1, propagate_tau.f90:144-181). The sequence is cut into blocks of L positions and, per block c,
// the products R_c(q) = E[q] ... E[cL] are formed once (mcb_prefix_kernel, blocks in parallel) and kept as
// U[q] = w^T R_c(q) (the trace functional) and Rend[c] = R_c(last). A trajectory then needs only a short
// dependent chain: the map-by-map steps up to its first block boundary (outputs written directly) and one
// Rend matvec per later block (mcb_tau_kernel); every later output is the dot U[q] . X_i[c]
// (mcb_out_kernel, all (i, tau) in parallel). Same products as the reference's chain, associated per block:
// results agree to rounding (the Fortran goldens and the pipelined kernel, PQD_MC_BLOCKED=0).
// ---------------------------------------------------------------------------------------------
// the map at position q of the shared sequence: mode 0 dm_tl(:, :, q + 1); mode 1 (calc_onetime_parallel_block) the
// periodic sequence jj = q mod n_tb + 1 -> dm_block(:, :, jj) for jj <= n_map, else dm_s (propagate_tau.f90:270-287).
// The blocked mode-1 path treats every position past q_s as dm_s: that holds only for n_map <= n_tb, and the host
// (pqd_host.cpp, blocked-kernel choice) runs the map-by-map kernels when n_map > n_tb.
__device__ __forceinline__ const double2* map_at(const MapChainParams& p, int q, int M2) {
    if (p.mode == 0) return p.dmA + (size_t)q * M2;
    if (q >= p.q_s) return p.dm_s;
    const int jj = q % p.n_tb + 1;
    return jj <= p.n_map ? p.dmA + (size_t)(jj - 1) * M2 : p.dm_s;
}

__device__ __forceinline__ double2 trace_weight(const MapChainParams& p, int r) {
    // Tr(opB R) over the column-major view of R (propagate_tau.f90:176): lane r = b + a dim gets opB(a, b)
    const int a = r / p.dim, b = r % p.dim;
    return p.opB[a + b * p.dim];
}

template <int N2>
__global__ __launch_bounds__(256) void mcb_prefix_kernel(MapChainParams p) {
    constexpr int M2 = N2 * N2;
    constexpr int PER = (M2 + 255) / 256;
    __shared__ double2 R[2][M2];
    __shared__ double2 E[M2];
    __shared__ double2 w[N2];
    const int tid = threadIdx.x, c = blockIdx.x;
    const int q0 = c * p.L, q1 = min(q0 + p.L, p.Q);
    if (tid < N2) w[tid] = trace_weight(p, tid);
    double2 nx[PER];
    auto fetch = [&](int q) {
        const double2* A = map_at(p, q, M2);
#pragma unroll
        for (int u = 0; u < PER; ++u) {
            const int e = tid + 256 * u;
            nx[u] = (e < M2) ? A[e] : c_zero();
        }
    };
    fetch(q0);
    int cur = 0;
    for (int q = q0; q < q1; ++q) {
        __syncthreads();  // the previous product and U read R / E
#pragma unroll
        for (int u = 0; u < PER; ++u) {
            const int e = tid + 256 * u;
            if (e < M2) E[e] = nx[u];
        }
        if (q + 1 < q1) fetch(q + 1);
        __syncthreads();
        if (q == q0) {
#pragma unroll
            for (int u = 0; u < PER; ++u) {
                const int e = tid + 256 * u;
                if (e < M2) R[cur][e] = E[e];
            }
        } else {
#pragma unroll
            for (int u = 0; u < PER; ++u) {
                const int e = tid + 256 * u;
                if (e < M2) {
                    const int rr = e % N2, cc = e / N2;
                    double2 acc = c_zero();
#pragma unroll 4
                    for (int k = 0; k < N2; ++k) c_fma(acc, E[rr + k * N2], R[cur][k + cc * N2]);
                    R[cur ^ 1][e] = acc;
                }
            }
            cur ^= 1;
        }
        __syncthreads();
        if (tid < N2) {  // U[q][col] = sum_k w[k] R(k, col)
            double2 acc = c_zero();
            for (int k = 0; k < N2; ++k) c_fma(acc, w[k], R[cur][k + tid * N2]);
            p.U[(size_t)q * N2 + tid] = acc;
        }
    }
    __syncthreads();
#pragma unroll
    for (int u = 0; u < PER; ++u) {
        const int e = tid + 256 * u;
        if (e < M2) p.Rend[(size_t)c * M2 + e] = R[cur][e];
    }
}

// trunk states at the block starts: P[0] = rho_init, P[c + 1] = Rend[c] P[c] (one wave, c < n_chain)
template <int N2>
__global__ __launch_bounds__(64) void mcb_chain_kernel(MapChainParams p, int n_chain) {
    __shared__ double2 x[64];
    const int lane = threadIdx.x;
    const bool on = lane < N2;
    if (on) { x[lane] = p.rho_init[lane]; p.P[lane] = p.rho_init[lane]; }
    __syncthreads();
    constexpr int M2 = N2 * N2;
    double2 am[N2];
    auto load = [&](int c) {
        const double2* A = p.Rend + (size_t)c * M2 + (on ? lane : 0);
#pragma unroll
        for (int k = 0; k < N2; ++k) am[k] = A[k * N2];
    };
    if (n_chain > 0) load(0);
    for (int c = 0; c < n_chain; ++c) {
        double2 y = c_zero();
#pragma unroll
        for (int k = 0; k < N2; ++k) c_fma(y, am[k], x[k]);
        if (c + 1 < n_chain) load(c + 1);
        __syncthreads();
        if (on) { x[lane] = y; p.P[(size_t)(c + 1) * N2 + lane] = y; }
        __syncthreads();
    }
}

__device__ __forceinline__ int wave_max_int(int v) {
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) v = max(v, __shfl_xor(v, o, 64));
    return v;
}

// per trajectory: rho(j_i) = E[p_i - 1] ... E[cL] P[c] (c = p_i / L, < L steps), then G(i, 1) = Tr(A B C rho) and
// the tau start C rho A (propagate_tau.f90:154-163), as mc_trunk_kernel computes them
template <int N2>
__global__ __launch_bounds__(64) void mcb_trunk_kernel(MapChainParams p) {
    constexpr int TPW = 64 / N2;
    constexpr int M2 = N2 * N2;
    __shared__ double2 xs[2][64], t1[64], t2[64];
    const int lane = threadIdx.x, dim = p.dim;
    const int tl = lane / N2, r = lane - (lane / N2) * N2;
    const int i = blockIdx.x * TPW + tl;
    const bool act = (tl < TPW) && (i < p.n_t);
    const int tlx = tl < TPW ? tl : 0;
    const int p0 = act ? p.pos[i] : 0;
    const int c = p0 / p.L;
    const int ns = act ? p0 - c * p.L : 0;
    xs[0][lane] = act ? p.P[(size_t)c * N2 + r] : c_zero();
    const int mx = wave_max_int(ns);
    double2 am[N2];
    auto load = [&](int s) {
        const double2* A = p.dmA + (size_t)(s < ns ? c * p.L + s : 0) * M2 + r;
#pragma unroll
        for (int k = 0; k < N2; ++k) am[k] = A[k * N2];
    };
    if (mx > 0) load(0);
    __syncthreads();
    int cur = 0;
    for (int s = 0; s < mx; ++s) {
        const double2* x = xs[cur] + tlx * N2;
        double2 y = c_zero();
#pragma unroll
        for (int k = 0; k < N2; ++k) c_fma(y, am[k], x[k]);
        if (s + 1 < mx) load(s + 1);
        xs[cur ^ 1][lane] = (s < ns) ? y : xs[cur][lane];
        __syncthreads();
        cur ^= 1;
    }
    const double2* X = xs[cur] + tlx * N2;
    double2* T1 = t1 + tlx * N2;
    double2* T2 = t2 + tlx * N2;
    // G(i, 1) = Tr(A (B (C rho)))
    if (act) T1[r] = cm_mat(p.opC, X, r, dim);
    __syncthreads();
    if (act) T2[r] = cm_mat(p.opB, T1, r, dim);
    __syncthreads();
    if (act) T1[r] = cm_mat(p.opA, T2, r, dim);
    __syncthreads();
    if (act && r == 0) {
        double2 s = c_zero();
        for (int l = 0; l < dim; ++l) s = c_add(s, T1[l + l * dim]);
        p.result[i] = s;
    }
    __syncthreads();
    if (act) T1[r] = cm_mat(p.opC, X, r, dim);
    __syncthreads();
    if (act) p.rho_buf[(size_t)i * N2 + r] = cm_mat(T1, p.opA, r, dim);
}

// per trajectory: the map-by-map steps up to its first block boundary (outputs written) and one Rend matvec per later
// block (states X_i[c] stored); the loop is pipelined like mc_tau_pipe_kernel
template <int N2, int PFD>
__global__ __launch_bounds__(64) void mcb_tau_kernel(MapChainParams p) {
    constexpr int TPW = 64 / N2;
    constexpr int M2 = N2 * N2;
    __shared__ double2 xs[2][64], ts[64];
    const int lane = threadIdx.x;
    const int tl = lane / N2, r = lane - (lane / N2) * N2;
    const int i = blockIdx.x * TPW + tl;
    const bool act = (tl < TPW) && (i < p.n_t);
    const int tlx = tl < TPW ? tl : 0;
    const int L = p.L;
    const int p0 = act ? p.pos[i] : 0;
    const int nf = act ? min(p.n_tau, (L - p0 % L) % L) : 0;
    const bool full = act && nf < p.n_tau;
    const int cs = (p0 + nf) / L;
    const int nb = full ? (p0 + p.n_tau - 1) / L - cs : 0;
    const int ns = nf + nb;
    const int mx = wave_max_int(ns);
    const double2 w = act ? trace_weight(p, r) : c_zero();
    const double2 x0 = act ? p.rho_buf[(size_t)i * N2 + r] : c_zero();
    xs[0][lane] = x0;
    if (full && nf == 0) p.X[((size_t)cs * p.n_t + i) * N2 + r] = x0;
    double2 am[PFD][N2];
    int sl_next = 0;  // lookahead step index
    auto load_row = [&](int sl) {
        const int s = sl_next++;
        const double2* A = s < nf ? map_at(p, p0 + s, M2)
                                  : (s < ns ? p.Rend + (size_t)(cs + s - nf) * M2 : p.Rend);
        A += r;
#pragma unroll
        for (int k = 0; k < N2; ++k) am[sl][k] = A[k * N2];
    };
#pragma unroll
    for (int sl = 0; sl < PFD; ++sl) load_row(sl);
    __syncthreads();
    int cur = 0;
    auto step = [&](int sl, int s) {
        const double2* x = xs[cur] + tlx * N2;
        double2 y = c_zero();
#pragma unroll
        for (int k = 0; k < N2; ++k) c_fma(y, am[sl][k], x[k]);
        load_row(sl);
        xs[cur ^ 1][lane] = (s < ns) ? y : xs[cur][lane];
        ts[lane] = c_mul(w, y);
        if (s >= nf && s < ns) p.X[((size_t)(cs + s - nf + 1) * p.n_t + i) * N2 + r] = y;
        else if (full && s == nf - 1) p.X[((size_t)cs * p.n_t + i) * N2 + r] = y;
        __syncthreads();
        if (act && r == 0 && s < nf) {
            double2 g = c_zero();
#pragma unroll
            for (int q = 0; q < N2; ++q) g = c_add(g, ts[tl * N2 + q]);
            p.result[(size_t)i + (size_t)(s + 1) * p.n_t] = g;
        }
        cur ^= 1;
    };
    int s = 0;
    for (; s + PFD - 1 < mx; s += PFD) {
#pragma unroll
        for (int sl = 0; sl < PFD; ++sl) step(sl, s + sl);
    }
#pragma unroll
    for (int sl = 0; sl < PFD; ++sl)
        if (s + sl < mx) step(sl, s + sl);
}

// every output past a trajectory's first block boundary: G(i, s + 2) = U[p_i + s] . X_i[(p_i + s) / L]
template <int N2>
__global__ __launch_bounds__(256) void mcb_out_kernel(MapChainParams p) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= p.n_t) return;
    const int L = p.L;
    const int p0 = p.pos[i];
    const int nf = min(p.n_tau, (L - p0 % L) % L);
    for (int col = blockIdx.y + 1; col <= p.n_tau; col += gridDim.y) {
        const int s = col - 1;
        if (s < nf) continue;
        const int q = p0 + s;
        const double2* u = p.U + (size_t)q * N2;
        const double2* x = p.X + ((size_t)(q / L) * p.n_t + i) * N2;
        double2 g = c_zero();
#pragma unroll
        for (int k = 0; k < N2; ++k) c_fma(g, u[k], x[k]);
        p.result[(size_t)i + (size_t)col * p.n_t] = g;
    }
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
// tau tails of the phonon dynamical-map correlations (reference two_time/correlations.py:866-1186:
// `for j: X = tl_map2 @ X; G[:, n_tauc + j + 1] = Bt @ X`): every row's vector x_i is propagated by ONE constant
// map, out[i][j] = w . M^{j+1} x_i. Rows are independent: 64 / N2 rows packed per wave (lane = row r of M, held in
// registers), the vector double-buffered in LDS, the trace w . y summed by lane 0 of the row's lanes.
// ---------------------------------------------------------------------------------------------
template <int N2>
__global__ __launch_bounds__(64) void map_tail_kernel(const double2* __restrict__ M, const double2* __restrict__ X,
                                                      int n_x, const double2* __restrict__ w, int n_steps,
                                                      double2* __restrict__ out) {
    constexpr int TPW = 64 / N2;
    __shared__ double2 xs[2][64], ts[64];
    const int lane = threadIdx.x;
    const int tl = lane / N2, r = lane - (lane / N2) * N2;
    const int i = blockIdx.x * TPW + tl;
    const bool act = tl < TPW && i < n_x;
    double2 mrow[N2];
#pragma unroll
    for (int c = 0; c < N2; ++c) mrow[c] = act ? M[(size_t)r * N2 + c] : c_zero();
    const double2 wr = act ? w[r] : c_zero();
    xs[0][lane] = act ? X[(size_t)i * N2 + r] : c_zero();
    const int tlx = tl < TPW ? tl : 0;
    __syncthreads();
    int cur = 0;
    for (int j = 0; j < n_steps; ++j) {
        const double2* x = xs[cur] + tlx * N2;
        double2 y = c_zero();
#pragma unroll
        for (int c = 0; c < N2; ++c) c_fma(y, mrow[c], x[c]);
        xs[cur ^ 1][lane] = y;
        ts[lane] = c_mul(wr, y);
        __syncthreads();
        if (act && r == 0) {
            double2 s = c_zero();
#pragma unroll
            for (int q = 0; q < N2; ++q) s = c_add(s, ts[tl * N2 + q]);
            out[(size_t)i * n_steps + j] = s;
        }
        cur ^= 1;
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

template <int N2, int PFD>
static hipError_t launch_blocked_n(const MapChainParams& p, int n_chain, hipStream_t s) {
    if (p.n_blk > 0) hipLaunchKernelGGL((mcb_prefix_kernel<N2>), dim3(p.n_blk), dim3(256), 0, s, p);
    constexpr int TPW = 64 / N2;
    const int nblk = (p.n_t + TPW - 1) / TPW;
    if (p.mode == 0) {
        hipLaunchKernelGGL((mcb_chain_kernel<N2>), dim3(1), dim3(64), 0, s, p, n_chain);
        hipLaunchKernelGGL((mcb_trunk_kernel<N2>), dim3(nblk), dim3(64), 0, s, p);
    } else {
        // mode 1: the trunk runs dm_block then dm_s without wrapping (propagate_tau.f90:235-241), a different
        // sequence from the periodic tau maps: the serial trunk kernel
        hipLaunchKernelGGL(mc_trunk_kernel, dim3(1), dim3(64), 0, s, p);
    }
    if (p.n_tau > 0) {
        hipLaunchKernelGGL((mcb_tau_kernel<N2, PFD>), dim3(nblk), dim3(64), 0, s, p);
        const int gy = std::min(p.n_tau, 65535);
        hipLaunchKernelGGL((mcb_out_kernel<N2>), dim3((p.n_t + 255) / 256, gy), dim3(256), 0, s, p);
    }
    return hipGetLastError();
}

// modes 0 and 1 on the blocked sweep; p.pos, p.L, p.n_blk, p.Q and the U / Rend / P / X buffers set by the host;
// n_chain = max_i p_i / L block starts of the trunk (mode 0)
hipError_t launch_mapchain_blocked(const MapChainParams& p, int n_chain, hipStream_t s) {
    switch (p.N2) {
        case 4: return launch_blocked_n<4, 4>(p, n_chain, s);
        case 9: return launch_blocked_n<9, 2>(p, n_chain, s);
        case 16: return launch_blocked_n<16, 2>(p, n_chain, s);
        case 25: return launch_blocked_n<25, 1>(p, n_chain, s);
        case 36: return launch_blocked_n<36, 1>(p, n_chain, s);
        default: return hipErrorInvalidValue;
    }
}

hipError_t launch_map_tail(int N2, const double2* M, const double2* X, int n_x, const double2* w, int n_steps,
                           double2* out, hipStream_t s) {
    const int TPW = 64 / N2;
    const dim3 grid((n_x + TPW - 1) / TPW);
    switch (N2) {
        case 4: hipLaunchKernelGGL(map_tail_kernel<4>, grid, dim3(64), 0, s, M, X, n_x, w, n_steps, out); break;
        case 9: hipLaunchKernelGGL(map_tail_kernel<9>, grid, dim3(64), 0, s, M, X, n_x, w, n_steps, out); break;
        case 16: hipLaunchKernelGGL(map_tail_kernel<16>, grid, dim3(64), 0, s, M, X, n_x, w, n_steps, out); break;
        case 25: hipLaunchKernelGGL(map_tail_kernel<25>, grid, dim3(64), 0, s, M, X, n_x, w, n_steps, out); break;
        case 36: hipLaunchKernelGGL(map_tail_kernel<36>, grid, dim3(64), 0, s, M, X, n_x, w, n_steps, out); break;
        default: return hipErrorInvalidValue;
    }
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
