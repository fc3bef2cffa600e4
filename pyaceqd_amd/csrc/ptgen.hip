// ptgen.hip — device factorizations of the Gaussian-bath PT generator (pyaceqd_amd/ptgen_gpu.py).
//
// The generator (ACE's `dont_propagate` + `write_PT` step, reference general_system.py:152-211; host restatement
// pyaceqd_amd/ptgen.py) compresses, twice per PT step, a "future influence" MPS of K = t_mem/dt sites: a
// right-to-left QR sweep (right-canonical form), one SVD at the boundary (its isometry IS the PT slice) and a
// left-to-right truncating sweep. Every factorization of a sweep depends on the previous one, so there is no batch
// to spread over the chip; the matrices are tall complex blocks of up to a few thousand rows and several hundred
// columns. The kernels here are built for that shape:
//
//   * Householder QR (optionally column-pivoted, stopping at a norm tolerance: a rank-revealing truncation),
//     ONE LAUNCH PER COLUMN over the whole chip: every wave recomputes the step's reflector from the pivot column
//     (a redundant length-m reduction, no inter-workgroup hand-off) and applies it to one trailing column. The
//     pivot search reads the previous launch's column norms, written by the waves that updated those columns (exact
//     norms of the trailing rows, no downdating). A launch boundary (~1.5-3.5 us) is the only synchronisation.
//   * Q formation: reflectors applied in blocks of QF_RB per launch, one wave per column of Q.
//   * one-sided (Hestenes) Jacobi SVD of the square R factor, one launch per round of a round-robin tournament
//     (n/2 disjoint column pairs, one wave each), accumulating V; the host stops at the first sweep without a
//     rotation. One-sided Jacobi computes every singular value to high relative accuracy, so the threshold
//     truncation (1e-10 relative) sees the same spectrum LAPACK's SVD does.
//   * single-workgroup variants of all three for matrices that fit in LDS (the far, small-bond sites).
//
// Layout: every matrix is column-major with leading dimension = rows (a row-major torch tensor of shape
// (cols, rows) whose row j is column j). Complex numbers are double2 (pqd_c128).
#include "pqd_common.h"
#include "../../include/pqd.h"

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <mutex>
#include <vector>

namespace {

__device__ __forceinline__ double wsum(double v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
    return v;
}
__device__ __forceinline__ double2 wsum2(double2 v) { return make_double2(wsum(v.x), wsum(v.y)); }
__device__ __forceinline__ double c_abs2(double2 a) { return a.x * a.x + a.y * a.y; }
// conj(a) * b
__device__ __forceinline__ double2 c_cmul(double2 a, double2 b) {
    return make_double2(fma(a.x, b.x, a.y * b.y), fma(a.x, b.y, -a.y * b.x));
}
__device__ __forceinline__ double2 c_div(double2 a, double2 b) {
    const double d = 1.0 / (b.x * b.x + b.y * b.y);
    return make_double2((a.x * b.x + a.y * b.y) * d, (a.y * b.x - a.x * b.y) * d);
}

// LAPACK zlarfg: H^H (alpha; x) = (beta; 0) with H = I - tau v v^H, v = (1; x * scale), beta real.
struct Refl {
    double2 tau, scale;
    double beta;
};
__device__ __forceinline__ Refl make_refl(double2 alpha, double xn2) {
    Refl r;
    if (xn2 == 0.0 && alpha.y == 0.0) {
        r.tau = c_zero();
        r.scale = c_zero();
        r.beta = alpha.x;
        return r;
    }
    const double nrm = sqrt(alpha.x * alpha.x + alpha.y * alpha.y + xn2);
    const double beta = alpha.x >= 0.0 ? -nrm : nrm;
    r.beta = beta;
    r.tau = make_double2((beta - alpha.x) / beta, -alpha.y / beta);
    r.scale = c_div(make_double2(1.0, 0.0), make_double2(alpha.x - beta, alpha.y));
    return r;
}

struct QRArgs {
    double2* W;        // m x n column-major (ld = m), factorized in place: rows < k of a column hold R, column k's
                       //   rows > k keep x_k (v_k = (1; x_k * scale_k))
    double2* X;        // the reflector columns: column k as it was when reflector k was made (rows < k: R, row k:
                       //   alpha, rows > k: x_k). X == W for one-column steps; the two-column step keeps its own copy
    int m, n, kmax;    // kmax = min(m, n)
    int pivot;
    double tol2;       // pivot: stop when the largest trailing column norm^2 <= tol2
    double2* tau;      // kmax
    double2* scale;    // kmax
    double* beta;      // kmax
    int* perm;         // 2 x n (double-buffered by step parity)
    double* norms;     // 2 x n, indexed by PHYSICAL column
    int* ctrl;         // [0] = rank (kmax until a pivot step finds the trailing block below tol)
};

__global__ void qr_init_kernel(QRArgs a) {
    const int lane = threadIdx.x & 63;
    const int wave = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    if (wave == 0 && lane == 0) a.ctrl[0] = a.kmax;
    if (wave < a.n) {
        const int c = wave;
        if (lane == 0) a.perm[c] = c;
        if (a.pivot) {
            const double2* col = a.W + (size_t)c * a.m;
            double s = 0.0;
            for (int i = lane; i < a.m; i += 64) s += c_abs2(col[i]);
            s = wsum(s);
            if (lane == 0) a.norms[c] = s;
        }
    }
}

// step k: reflector from logical column k (after the pivot swap), applied to logical columns k+1.. (one wave each)
__global__ __launch_bounds__(256) void qr_step_kernel(QRArgs a, int k) {
    if (a.ctrl[0] <= k) return;
    const int lane = threadIdx.x & 63;
    const int wave = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    const int* pin = a.perm + (size_t)(k & 1) * a.n;
    int* pout = a.perm + (size_t)((k + 1) & 1) * a.n;
    const double* nin = a.norms + (size_t)(k & 1) * a.n;
    double* nout = a.norms + (size_t)((k + 1) & 1) * a.n;
    int p = k;
    if (a.pivot) {
        double best = -1.0;
        int bj = k;
        for (int j = k + lane; j < a.n; j += 64) {
            const double v = nin[pin[j]];
            if (v > best) { best = v; bj = j; }
        }
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) {
            const double ob = __shfl_xor(best, o);
            const int oj = __shfl_xor(bj, o);
            if (ob > best || (ob == best && oj < bj)) { best = ob; bj = oj; }
        }
        p = bj;
        if (best <= a.tol2) {
            if (wave == 0 && lane == 0) a.ctrl[0] = k;
            return;
        }
    }
    auto phys = [&](int j) {
        if (!a.pivot) return j;
        return j == k ? pin[p] : (j == p ? pin[k] : pin[j]);
    };
    const int pk = phys(k);
    const double2* x = a.W + (size_t)pk * a.m;
    double xn = 0.0;
    for (int i = k + 1 + lane; i < a.m; i += 64) xn += c_abs2(x[i]);
    xn = wsum(xn);
    const double2 alpha = x[k];
    const Refl R = make_refl(alpha, xn);
    if (wave == 0) {
        if (lane == 0) {
            a.tau[k] = R.tau;
            a.scale[k] = R.scale;
            a.beta[k] = R.beta;
        }
        if (a.pivot)
            for (int j = lane; j < a.n; j += 64) pout[j] = j < k ? pin[j] : phys(j);
        if (a.X != a.W)
            for (int i = lane; i < a.m; i += 64) a.X[(size_t)k * a.m + i] = x[i];
    }
    const int j = k + 1 + wave;
    if (j >= a.n) return;
    const int c = phys(j);
    double2* col = a.W + (size_t)c * a.m;
    const double2 ck = col[k];
    double2 s = c_zero();
    for (int i = k + 1 + lane; i < a.m; i += 64) {
        const double2 v = c_mul(x[i], R.scale);
        const double2 ci = col[i];
        s.x += v.x * ci.x + v.y * ci.y;
        s.y += v.x * ci.y - v.y * ci.x;
    }
    s = wsum2(s);
    s = c_add(s, ck);
    const double2 ct = c_cmul(R.tau, s);  // conj(tau) * (v^H c)
    double nn = 0.0;
    for (int i = k + 1 + lane; i < a.m; i += 64) {
        const double2 v = c_mul(x[i], R.scale);
        double2 ci = col[i];
        ci = c_sub(ci, c_mul(ct, v));
        col[i] = ci;
        nn += c_abs2(ci);
    }
    if (lane == 0) col[k] = c_sub(ck, ct);
    if (a.pivot) {
        nn = wsum(nn);
        if (lane == 0) nout[c] = nn;
    }
}

// two reflectors per launch (plain QR only): every wave makes reflector k from column k, applies it to column k+1
// on the fly and makes reflector k+1 from that (redundantly, no hand-off), then applies both to its own column in three
// passes. Waves 0 and 1 store the two panel columns as the reflectors saw them into X (W's panel columns are read by
// every wave of this launch, so they stay untouched). Half the launches of qr_step_kernel for the same arithmetic.
__global__ __launch_bounds__(256) void qr_step2_kernel(QRArgs a, int k) {
    const int lane = threadIdx.x & 63;
    const int wave = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    const int m = a.m;
    const double2* c0 = a.W + (size_t)k * m;
    const double2* c1 = a.W + (size_t)(k + 1) * m;
    double xn0 = 0.0;
    double2 w01 = c_zero();
    for (int i = k + 1 + lane; i < m; i += 64) {
        const double2 u = c0[i], v = c1[i];
        xn0 += c_abs2(u);
        w01.x += u.x * v.x + u.y * v.y;
        w01.y += u.x * v.y - u.y * v.x;
    }
    xn0 = wsum(xn0);
    w01 = wsum2(w01);
    const Refl R0 = make_refl(c0[k], xn0);
    // v0 = (1; c0 sc0): v0^H c1 = c1[k] + conj(sc0) sum conj(c0) c1
    const double2 w0 = c_add(c1[k], c_cmul(R0.scale, w01));
    const double2 ct01 = c_cmul(R0.tau, w0);
    // c1' = c1 - ct01 v0 (rows >= k); reflector k+1 from rows >= k+1 of c1'
    const double2 f01 = c_mul(ct01, R0.scale);  // c1'_i = c1_i - f01 c0_i for i > k
    const double2 alpha1 = c_sub(c1[k + 1], c_mul(f01, c0[k + 1]));
    double xn1 = 0.0;
    for (int i = k + 2 + lane; i < m; i += 64) xn1 += c_abs2(c_sub(c1[i], c_mul(f01, c0[i])));
    xn1 = wsum(xn1);
    const Refl R1 = make_refl(alpha1, xn1);
    if (wave == 0) {
        if (lane == 0) {
            a.tau[k] = R0.tau; a.scale[k] = R0.scale; a.beta[k] = R0.beta;
            a.tau[k + 1] = R1.tau; a.scale[k + 1] = R1.scale; a.beta[k + 1] = R1.beta;
        }
        for (int i = lane; i < m; i += 64) a.X[(size_t)k * m + i] = c0[i];
        return;
    }
    if (wave == 1) {
        for (int i = lane; i < m; i += 64) {
            double2 v = c1[i];
            if (i == k) v = c_sub(v, ct01);
            else if (i > k) v = c_sub(v, c_mul(f01, c0[i]));
            a.X[(size_t)(k + 1) * m + i] = v;
        }
        return;
    }
    const int j = k + wave;  // waves 2.. -> columns k+2..
    if (j >= a.n) return;
    double2* col = a.W + (size_t)j * m;
    // pass A: w = v0^H c_j
    double2 sA = c_zero();
    for (int i = k + 1 + lane; i < m; i += 64) {
        const double2 u = c0[i], v = col[i];
        sA.x += u.x * v.x + u.y * v.y;
        sA.y += u.x * v.y - u.y * v.x;
    }
    sA = wsum2(sA);
    const double2 ck = col[k], ck1 = col[k + 1];
    const double2 ctA = c_cmul(R0.tau, c_add(ck, c_cmul(R0.scale, sA)));
    const double2 fA = c_mul(ctA, R0.scale);  // (H_k^H c_j)_i = c_i - fA c0_i for i > k
    // pass B: w = v1^H (H_k^H c_j), v1 = (1 at k+1; (c1_i - f01 c0_i) sc1 for i > k+1)
    double2 sB = c_zero();
    for (int i = k + 2 + lane; i < m; i += 64) {
        const double2 u0 = c0[i];
        const double2 v1 = c_sub(c1[i], c_mul(f01, u0));
        const double2 y = c_sub(col[i], c_mul(fA, u0));
        sB.x += v1.x * y.x + v1.y * y.y;
        sB.y += v1.x * y.y - v1.y * y.x;
    }
    sB = wsum2(sB);
    const double2 yk1 = c_sub(ck1, c_mul(fA, c0[k + 1]));
    const double2 ctB = c_cmul(R1.tau, c_add(yk1, c_cmul(R1.scale, sB)));
    const double2 fB = c_mul(ctB, R1.scale);
    // pass C: c_j <- H_{k+1}^H H_k^H c_j
    for (int i = k + 2 + lane; i < m; i += 64) {
        const double2 u0 = c0[i];
        const double2 v1 = c_sub(c1[i], c_mul(f01, u0));
        col[i] = c_sub(c_sub(col[i], c_mul(fA, u0)), c_mul(fB, v1));
    }
    if (lane == 0) {
        col[k] = c_sub(ck, ctA);
        col[k + 1] = c_sub(yk1, ctB);
    }
}

// R (rank x n, column-major, ld = rank) in pivoted column order; perm_out = the final permutation
__global__ void qr_extract_r_kernel(QRArgs a, int rank, double2* R, int* perm_out) {
    const int idx = blockIdx.x * blockDim.x + threadIdx.x;
    const int* pf = a.perm + (size_t)(rank & 1) * a.n;
    if (idx < a.n) perm_out[idx] = a.pivot ? pf[idx] : idx;
    if (idx >= rank * a.n) return;
    const int j = idx / rank, i = idx - j * rank;
    const int c = a.pivot ? pf[j] : j;
    double2 v;
    // reflector columns (j < rank) as their reflector saw them (X); columns past the rank only in W
    if (i < j) v = (j < rank ? a.X : a.W)[(size_t)c * a.m + i];
    else if (i == j) v = make_double2(a.beta[i], 0.0);
    else v = c_zero();
    R[(size_t)j * rank + i] = v;
}

// Q = H_0 ... H_{rank-1} [I; 0]  (m x rank): init, then blocks of QF_RB reflectors applied in descending order
constexpr int QF_RB = 8;
__global__ void qf_init_kernel(double2* Q, int m, int rank) {
    const size_t idx = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (idx >= (size_t)m * rank) return;
    const int j = (int)(idx / m), i = (int)(idx - (size_t)j * m);
    Q[idx] = make_double2(i == j ? 1.0 : 0.0, 0.0);
}

__global__ __launch_bounds__(256) void qf_apply_kernel(QRArgs a, int rank, const int* perm_final, double2* Q,
                                                       int i0, int i1) {
    const int lane = threadIdx.x & 63;
    const int wave = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    const int j = i0 + wave;
    if (j >= rank) return;
    double2* col = Q + (size_t)j * a.m;
    for (int i = min(j, i1 - 1); i >= i0; --i) {
        const int pc = a.pivot ? perm_final[i] : i;
        const double2* x = a.X + (size_t)pc * a.m;
        const double2 sc = a.scale[i], tau = a.tau[i];
        const double2 ci0 = col[i];
        double2 s = c_zero();
        for (int r = i + 1 + lane; r < a.m; r += 64) {
            const double2 v = c_mul(x[r], sc);
            const double2 cr = col[r];
            s.x += v.x * cr.x + v.y * cr.y;
            s.y += v.x * cr.y - v.y * cr.x;
        }
        s = wsum2(s);
        s = c_add(s, ci0);
        const double2 t = c_mul(tau, s);
        for (int r = i + 1 + lane; r < a.m; r += 64) col[r] = c_sub(col[r], c_mul(t, c_mul(x[r], sc)));
        if (lane == 0) col[i] = c_sub(ci0, t);
    }
}

// -------------------------------------------------------------------------------------------------------------
// single-workgroup QR for matrices that fit in LDS (m * n <= QS_MAX): the same arithmetic, one barrier per step
// -------------------------------------------------------------------------------------------------------------
constexpr int QS_MAX = 8192;  // 128 KiB of complex doubles
constexpr int QS_THREADS = 1024;

__global__ __launch_bounds__(QS_THREADS) void qr_small_kernel(const double2* Win, int m, int n, int pivot, double tol2,
                                                             double2* Q, double2* R, int* perm_out, int* rank_out) {
    extern __shared__ double2 sm[];
    double2* A = sm;                       // m x n
    __shared__ double2 s_tau[256], s_scale[256];
    __shared__ double s_beta[256], s_norm[256];
    __shared__ int s_perm[256];
    __shared__ int s_p, s_rank;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, nw = QS_THREADS / 64;
    const int kmax = min(m, n);
    for (int idx = tid; idx < m * n; idx += QS_THREADS) A[idx] = Win[idx];
    for (int j = tid; j < n; j += QS_THREADS) s_perm[j] = j;
    if (tid == 0) s_rank = kmax;
    __syncthreads();
    if (pivot)
        for (int c = wave; c < n; c += nw) {
            double s = 0.0;
            for (int i = lane; i < m; i += 64) s += c_abs2(A[c * m + i]);
            s = wsum(s);
            if (lane == 0) s_norm[c] = s;
        }
    __syncthreads();
    for (int k = 0; k < kmax; ++k) {
        if (tid < 64) {
            int p = k;
            if (pivot) {
                double best = -1.0;
                int bj = k;
                for (int j = k + lane; j < n; j += 64) {
                    const double v = s_norm[s_perm[j]];
                    if (v > best) { best = v; bj = j; }
                }
#pragma unroll
                for (int o = 32; o > 0; o >>= 1) {
                    const double ob = __shfl_xor(best, o);
                    const int oj = __shfl_xor(bj, o);
                    if (ob > best || (ob == best && oj < bj)) { best = ob; bj = oj; }
                }
                p = bj;
                if (best <= tol2) p = -1;
            }
            if (lane == 0) {
                if (p < 0) {
                    s_rank = k;
                } else if (p != k) {
                    const int t = s_perm[k];
                    s_perm[k] = s_perm[p];
                    s_perm[p] = t;
                }
                s_p = p;
            }
        }
        __syncthreads();
        if (s_p < 0) break;
        const int pk = s_perm[k];
        const double2* x = A + pk * m;
        if (tid < 64) {
            double xn = 0.0;
            for (int i = k + 1 + lane; i < m; i += 64) xn += c_abs2(x[i]);
            xn = wsum(xn);
            const Refl Rf = make_refl(x[k], xn);
            if (lane == 0) { s_tau[k] = Rf.tau; s_scale[k] = Rf.scale; s_beta[k] = Rf.beta; }
        }
        __syncthreads();
        const double2 sc = s_scale[k], tau = s_tau[k];
        for (int j = k + 1 + wave; j < n; j += nw) {
            double2* col = A + s_perm[j] * m;
            const double2 ck = col[k];
            double2 s = c_zero();
            for (int i = k + 1 + lane; i < m; i += 64) {
                const double2 v = c_mul(x[i], sc);
                const double2 ci = col[i];
                s.x += v.x * ci.x + v.y * ci.y;
                s.y += v.x * ci.y - v.y * ci.x;
            }
            s = wsum2(s);
            s = c_add(s, ck);
            const double2 ct = c_cmul(tau, s);
            double nn = 0.0;
            for (int i = k + 1 + lane; i < m; i += 64) {
                const double2 ci = c_sub(col[i], c_mul(ct, c_mul(x[i], sc)));
                col[i] = ci;
                nn += c_abs2(ci);
            }
            nn = wsum(nn);
            if (lane == 0) {
                col[k] = c_sub(ck, ct);
                s_norm[s_perm[j]] = nn;
            }
        }
        __syncthreads();
    }
    const int rank = s_rank;
    // R (rank x n), perm
    for (int idx = tid; idx < rank * n; idx += QS_THREADS) {
        const int j = idx / rank, i = idx - j * rank;
        const int c = s_perm[j];
        R[idx] = i < j ? A[c * m + i] : (i == j ? make_double2(s_beta[i], 0.0) : c_zero());
    }
    for (int j = tid; j < n; j += QS_THREADS) perm_out[j] = s_perm[j];
    if (tid == 0) *rank_out = rank;
    // Q (m x rank) in global memory, one wave per column, reflectors descending
    for (int j = wave; j < rank; j += nw) {
        double2* col = Q + (size_t)j * m;
        for (int i = lane; i < m; i += 64) col[i] = make_double2(i == j ? 1.0 : 0.0, 0.0);
        for (int i = j; i >= 0; --i) {
            const double2* x = A + s_perm[i] * m;
            const double2 sc = s_scale[i], tau = s_tau[i];
            const double2 ci0 = col[i];
            double2 s = c_zero();
            for (int r = i + 1 + lane; r < m; r += 64) {
                const double2 v = c_mul(x[r], sc);
                const double2 cr = col[r];
                s.x += v.x * cr.x + v.y * cr.y;
                s.y += v.x * cr.y - v.y * cr.x;
            }
            s = wsum2(s);
            s = c_add(s, ci0);
            const double2 t = c_mul(tau, s);
            for (int r = i + 1 + lane; r < m; r += 64) col[r] = c_sub(col[r], c_mul(t, c_mul(x[r], sc)));
            if (lane == 0) col[i] = c_sub(ci0, t);
        }
    }
}

// -------------------------------------------------------------------------------------------------------------
// one-sided Jacobi SVD of a square n x n matrix X (column-major): X V = W with orthogonal columns
// -------------------------------------------------------------------------------------------------------------
struct JacArgs {
    double2* X;   // n x n, rotated in place
    double2* V;   // n x n, accumulated
    int n, nn;    // nn = n rounded up to even (index n is a dummy player)
    double tol;
    const double* zero2; // device word: a column with |x|^2 < *zero2 is numerically zero, never rotated
    int* count;   // rotations in this sweep
};

// *zero2 = zero_tol^2 ||X||_F^2 (one workgroup; rotations leave ||X||_F unchanged)
__global__ __launch_bounds__(1024) void jac_zero2_kernel(const double2* X, int n, double zt2, double* zero2) {
    __shared__ double part[16];
    double s = 0.0;
    for (size_t i = threadIdx.x; i < (size_t)n * n; i += 1024) s += c_abs2(X[i]);
    s = wsum(s);
    if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = s;
    __syncthreads();
    if (threadIdx.x == 0) {
        double t = 0.0;
        for (int w = 0; w < 16; ++w) t += part[w];
        *zero2 = zt2 * t;
    }
}

__device__ __forceinline__ void jac_pair(int t, int i, int nn, int& p, int& q) {
    auto L = [&](int s) { return s == 0 ? 0 : ((s - 1 + t) % (nn - 1)) + 1; };
    const int a = L(i), b = L(nn - 1 - i);
    p = min(a, b);
    q = max(a, b);
}

__global__ void jac_init_kernel(double2* V, int n) {
    const size_t idx = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (idx >= (size_t)n * n) return;
    const int j = (int)(idx / n), i = (int)(idx - (size_t)j * n);
    V[idx] = make_double2(i == j ? 1.0 : 0.0, 0.0);
}

// rotate the pair (p, q): [xp xq] J with J = [[cs, sn], [-sn e^{-i phi}, cs e^{-i phi}]], c = xp^H xq = |c| e^{i phi}
__device__ __forceinline__ bool jac_rotate(double2* xp, double2* xq, double2* vp, double2* vq, int len, int vlen,
                                           double tol, double zero2, int lane) {
    double a = 0.0, b = 0.0;
    double2 c = c_zero();
    for (int r = lane; r < len; r += 64) {
        const double2 u = xp[r], w = xq[r];
        a += c_abs2(u);
        b += c_abs2(w);
        c.x += u.x * w.x + u.y * w.y;
        c.y += u.x * w.y - u.y * w.x;
    }
    a = wsum(a);
    b = wsum(b);
    c = wsum2(c);
    const double ac = sqrt(c.x * c.x + c.y * c.y);
    // a column at the rounding floor of the matrix (|x|^2 < zero2) holds no information: rotating it against the
    // others only shrinks it by eps per pass towards the denormals, where its relative inner products stay noisy
    // and the sweep would never end (LAPACK's zgesvj skips such columns the same way)
    if (a < zero2 || b < zero2) return false;
    if (!(ac > tol * sqrt(a * b)) || ac == 0.0) return false;
    const double2 eph = make_double2(c.x / ac, -c.y / ac);  // e^{-i phi}
    const double zeta = (b - a) / (2.0 * ac);
    const double t = (zeta >= 0.0 ? 1.0 : -1.0) / (fabs(zeta) + sqrt(1.0 + zeta * zeta));
    const double cs = 1.0 / sqrt(1.0 + t * t), sn = cs * t;
    for (int r = lane; r < len; r += 64) {
        const double2 u = xp[r], w = c_mul(xq[r], eph);
        xp[r] = make_double2(cs * u.x - sn * w.x, cs * u.y - sn * w.y);
        xq[r] = make_double2(sn * u.x + cs * w.x, sn * u.y + cs * w.y);
    }
    for (int r = lane; r < vlen; r += 64) {
        const double2 u = vp[r], w = c_mul(vq[r], eph);
        vp[r] = make_double2(cs * u.x - sn * w.x, cs * u.y - sn * w.y);
        vq[r] = make_double2(sn * u.x + cs * w.x, sn * u.y + cs * w.y);
    }
    return true;
}

__global__ __launch_bounds__(256) void jac_round_kernel(JacArgs a, int t) {
    const int lane = threadIdx.x & 63;
    const int i = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    if (i >= a.nn / 2) return;
    int p, q;
    jac_pair(t, i, a.nn, p, q);
    if (q >= a.n) return;
    const bool rot = jac_rotate(a.X + (size_t)p * a.n, a.X + (size_t)q * a.n, a.V + (size_t)p * a.n,
                                a.V + (size_t)q * a.n, a.n, a.n, a.tol, *a.zero2, lane);
    if (rot && lane == 0) atomicAdd(a.count, 1);
}

// single workgroup: X and V in LDS (2 n^2 <= QS_MAX), all sweeps in one launch
__global__ __launch_bounds__(QS_THREADS) void jac_small_kernel(double2* Xg, double2* Vg, int n, double tol,
                                                              const double* zero2p, int max_sweeps, int* sweeps_out) {
    extern __shared__ double2 sm[];
    double2* X = sm;
    double2* V = sm + n * n;
    __shared__ int s_cnt;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, nw = QS_THREADS / 64;
    const int nn = n + (n & 1);
    const double zero2 = *zero2p;
    for (int idx = tid; idx < n * n; idx += QS_THREADS) {
        X[idx] = Xg[idx];
        const int j = idx / n, i = idx - j * n;
        V[idx] = make_double2(i == j ? 1.0 : 0.0, 0.0);
    }
    int sweep = 0;
    for (; sweep < max_sweeps; ++sweep) {
        if (tid == 0) s_cnt = 0;
        __syncthreads();
        for (int t = 0; t < nn - 1; ++t) {
            for (int i = wave; i < nn / 2; i += nw) {
                int p, q;
                jac_pair(t, i, nn, p, q);
                if (q >= n) continue;
                const bool rot = jac_rotate(X + p * n, X + q * n, V + p * n, V + q * n, n, n, tol, zero2, lane);
                if (rot && lane == 0) atomicAdd(&s_cnt, 1);
            }
            __syncthreads();
        }
        if (s_cnt == 0) { ++sweep; break; }
        __syncthreads();
    }
    for (int idx = tid; idx < n * n; idx += QS_THREADS) {
        Xg[idx] = X[idx];
        Vg[idx] = V[idx];
    }
    if (tid == 0) *sweeps_out = sweep;
}

// sigma_j = |x_j|, x_j <- x_j / sigma_j (zero columns stay zero)
__global__ void jac_finish_kernel(double2* X, int n, double* sigma) {
    const int lane = threadIdx.x & 63;
    const int j = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    if (j >= n) return;
    double2* col = X + (size_t)j * n;
    double s = 0.0;
    for (int r = lane; r < n; r += 64) s += c_abs2(col[r]);
    s = sqrt(wsum(s));
    if (lane == 0) sigma[j] = s;
    const double inv = s > 0.0 ? 1.0 / s : 0.0;
    for (int r = lane; r < n; r += 64) col[r] = c_scale(col[r], inv);
}

// ------------------------------------------------------------------------------------------------------------
thread_local char g_err[512];
int perr(int code, const char* msg) {
    snprintf(g_err, sizeof g_err, "%s", msg);
    pqd_fail_msg(code, g_err);
    return code;
}
#define PCHK(x)                                                                                  \
    do {                                                                                         \
        hipError_t e_ = (x);                                                                     \
        if (e_ != hipSuccess) {                                                                  \
            char b_[400];                                                                        \
            snprintf(b_, sizeof b_, "%s: %s (%s:%d)", #x, hipGetErrorString(e_), __FILE__, __LINE__); \
            return perr(PQD_ERR_HIP, b_);                                                        \
        }                                                                                        \
    } while (0)

// per-process scratch (the generator runs one factorization at a time per stream; guarded for safety)
std::mutex g_mu;
struct Scratch {
    void* p = nullptr;
    size_t bytes = 0;
} g_scr;
hipError_t scratch(size_t bytes, void** out) {
    if (bytes > g_scr.bytes) {
        if (g_scr.p) {
            hipError_t e = hipDeviceSynchronize();
            if (e != hipSuccess) return e;
            e = hipFree(g_scr.p);
            if (e != hipSuccess) return e;
            g_scr.p = nullptr;
        }
        hipError_t e = hipMalloc(&g_scr.p, bytes);
        if (e != hipSuccess) { g_scr.bytes = 0; return e; }
        g_scr.bytes = bytes;
    }
    *out = g_scr.p;
    return hipSuccess;
}
inline size_t al(size_t x) { return (x + 255) & ~(size_t)255; }

bool g_attr_done = false;
hipError_t small_attrs() {
    if (g_attr_done) return hipSuccess;
    const int lds = QS_MAX * (int)sizeof(double2);
    hipError_t e = hipFuncSetAttribute((const void*)qr_small_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, lds);
    if (e != hipSuccess) return e;
    e = hipFuncSetAttribute((const void*)jac_small_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, lds);
    if (e != hipSuccess) return e;
    g_attr_done = true;
    return hipSuccess;
}

// PQD_PTG_SMALL=0: every factorization on the multi-workgroup kernels (A/B and tests of both paths)
bool small_ok() {
    const char* e = getenv("PQD_PTG_SMALL");
    return !(e && atoi(e) == 0);
}

}  // namespace

extern "C" int pqd_ptg_qr(void* stream, pqd_c128* Wp, int32_t m, int32_t n, int32_t pivot, double tol,
                          pqd_c128* Qp, pqd_c128* Rp, int32_t* perm_out, int32_t* rank_out) {
    if (!Wp || !Qp || !Rp || !perm_out || !rank_out) return perr(PQD_ERR_ARG, "pqd_ptg_qr: NULL argument");
    if (m < 1 || n < 1) return perr(PQD_ERR_ARG, "pqd_ptg_qr: empty matrix");
    std::lock_guard<std::mutex> lk(g_mu);
    hipStream_t s = (hipStream_t)stream;
    double2* W = reinterpret_cast<double2*>(Wp);
    double2* Q = reinterpret_cast<double2*>(Qp);
    double2* R = reinterpret_cast<double2*>(Rp);
    const int kmax = std::min(m, n);
    const double tol2 = pivot ? tol * tol : -1.0;
    void* base = nullptr;
    // two reflectors per launch for plain QRs on the multi-workgroup path (PQD_PTG_PAIR=0: one per launch)
    const char* ep = getenv("PQD_PTG_PAIR");
    const bool small = small_ok() && (size_t)m * n <= (size_t)QS_MAX && n <= 256;
    const bool pairs = !pivot && !small && kmax >= 2 && !(ep && atoi(ep) == 0);
    const size_t b_tau = al(kmax * sizeof(double2)), b_beta = al(kmax * sizeof(double)),
                 b_perm = al(2 * (size_t)n * sizeof(int)), b_norm = al(2 * (size_t)n * sizeof(double)),
                 b_ctrl = al(64 * sizeof(int)), b_x = pairs ? al((size_t)m * kmax * sizeof(double2)) : 0;
    PCHK(scratch(2 * b_tau + b_beta + b_perm + b_norm + b_ctrl + b_x, &base));
    char* c = static_cast<char*>(base);
    QRArgs a;
    a.W = W; a.m = m; a.n = n; a.kmax = kmax; a.pivot = pivot ? 1 : 0; a.tol2 = tol2;
    a.tau = reinterpret_cast<double2*>(c); c += b_tau;
    a.scale = reinterpret_cast<double2*>(c); c += b_tau;
    a.beta = reinterpret_cast<double*>(c); c += b_beta;
    a.perm = reinterpret_cast<int*>(c); c += b_perm;
    a.norms = reinterpret_cast<double*>(c); c += b_norm;
    a.ctrl = reinterpret_cast<int*>(c); c += b_ctrl;
    a.X = pairs ? reinterpret_cast<double2*>(c) : W;
    int* d_rank = a.ctrl + 8;
    if (small) {
        PCHK(small_attrs());
        hipLaunchKernelGGL(qr_small_kernel, dim3(1), dim3(QS_THREADS), (size_t)m * n * sizeof(double2), s, W, m, n,
                           a.pivot, tol2, Q, R, perm_out, d_rank);
        PCHK(hipGetLastError());
        if (!pivot) {  // the rank of a plain QR is min(m, n): no host round trip, the caller's work stays queued
            *rank_out = kmax;
            return PQD_OK;
        }
        int rank = 0;
        PCHK(hipMemcpyAsync(&rank, d_rank, sizeof(int), hipMemcpyDeviceToHost, s));
        PCHK(hipStreamSynchronize(s));
        *rank_out = rank;
        return PQD_OK;
    }
    const int wpb = 4;
    hipLaunchKernelGGL(qr_init_kernel, dim3((n + wpb - 1) / wpb), dim3(64 * wpb), 0, s, a);
    for (int k = 0; k < kmax;) {
        if (pairs && k + 1 < kmax) {
            const int nw = 2 + std::max(0, n - k - 2);
            hipLaunchKernelGGL(qr_step2_kernel, dim3((nw + wpb - 1) / wpb), dim3(64 * wpb), 0, s, a, k);
            k += 2;
        } else {
            const int nw = std::max(1, n - k - 1);
            hipLaunchKernelGGL(qr_step_kernel, dim3((nw + wpb - 1) / wpb), dim3(64 * wpb), 0, s, a, k);
            k += 1;
        }
    }
    PCHK(hipGetLastError());
    int rank = kmax;
    if (pivot) {  // the stopping step decides the rank: one host round trip
        PCHK(hipMemcpyAsync(&rank, a.ctrl, sizeof(int), hipMemcpyDeviceToHost, s));
        PCHK(hipStreamSynchronize(s));
    }
    const int tot = std::max(rank * n, n);
    hipLaunchKernelGGL(qr_extract_r_kernel, dim3((tot + 255) / 256), dim3(256), 0, s, a, rank, R, perm_out);
    if (rank > 0) {
        const size_t mq = (size_t)m * rank;
        hipLaunchKernelGGL(qf_init_kernel, dim3((unsigned)((mq + 255) / 256)), dim3(256), 0, s, Q, m, rank);
        for (int i1 = rank; i1 > 0; i1 -= QF_RB) {
            const int i0 = std::max(0, i1 - QF_RB);
            const int ncol = rank - i0;
            hipLaunchKernelGGL(qf_apply_kernel, dim3((ncol + wpb - 1) / wpb), dim3(64 * wpb), 0, s, a, rank,
                               perm_out, Q, i0, i1);
        }
    }
    PCHK(hipGetLastError());
    *rank_out = rank;
    return PQD_OK;
}

extern "C" int pqd_ptg_jacobi(void* stream, pqd_c128* Xp, int32_t n, pqd_c128* Vp, double* sigma, double tol,
                              double zero_tol, int32_t max_sweeps, int32_t* sweeps_out) {
    if (!Xp || !Vp || !sigma || !sweeps_out) return perr(PQD_ERR_ARG, "pqd_ptg_jacobi: NULL argument");
    if (n < 1) return perr(PQD_ERR_ARG, "pqd_ptg_jacobi: empty matrix");
    std::lock_guard<std::mutex> lk(g_mu);
    hipStream_t s = (hipStream_t)stream;
    double2* X = reinterpret_cast<double2*>(Xp);
    double2* V = reinterpret_cast<double2*>(Vp);
    void* base = nullptr;
    PCHK(scratch(al(64 * sizeof(int)), &base));
    int* cnt = static_cast<int*>(base);
    double* zero2 = reinterpret_cast<double*>(cnt + 8);
    int sweeps = 0;
    // zero threshold relative to the Frobenius norm (rotation-invariant): |x_j| < zero_tol * ||X||_F
    hipLaunchKernelGGL(jac_zero2_kernel, dim3(1), dim3(1024), 0, s, X, n, zero_tol * zero_tol, zero2);
    if (small_ok() && 2 * (size_t)n * n <= (size_t)QS_MAX) {
        PCHK(small_attrs());
        hipLaunchKernelGGL(jac_small_kernel, dim3(1), dim3(QS_THREADS), 2 * (size_t)n * n * sizeof(double2), s, X, V,
                           n, tol, zero2, max_sweeps, cnt);
        PCHK(hipGetLastError());
        PCHK(hipMemcpyAsync(&sweeps, cnt, sizeof(int), hipMemcpyDeviceToHost, s));
        PCHK(hipStreamSynchronize(s));
    } else {
        JacArgs a;
        a.X = X; a.V = V; a.n = n; a.nn = n + (n & 1); a.tol = tol; a.zero2 = zero2; a.count = cnt;
        const size_t nv = (size_t)n * n;
        hipLaunchKernelGGL(jac_init_kernel, dim3((unsigned)((nv + 255) / 256)), dim3(256), 0, s, V, n);
        const int npair = a.nn / 2, wpb = 4;
        for (; sweeps < max_sweeps;) {
            PCHK(hipMemsetAsync(cnt, 0, sizeof(int), s));
            for (int t = 0; t < a.nn - 1; ++t)
                hipLaunchKernelGGL(jac_round_kernel, dim3((npair + wpb - 1) / wpb), dim3(64 * wpb), 0, s, a, t);
            PCHK(hipGetLastError());
            int h = 0;
            PCHK(hipMemcpyAsync(&h, cnt, sizeof(int), hipMemcpyDeviceToHost, s));
            PCHK(hipStreamSynchronize(s));
            ++sweeps;
            if (h == 0) break;
        }
    }
    hipLaunchKernelGGL(jac_finish_kernel, dim3((n + 3) / 4), dim3(256), 0, s, X, n, sigma);
    PCHK(hipGetLastError());
    *sweeps_out = sweeps;
    return PQD_OK;
}
