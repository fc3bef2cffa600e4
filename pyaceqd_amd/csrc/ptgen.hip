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
#include <map>
#include "../../include/pqd.h"

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <atomic>
#include <mutex>
#include <vector>

namespace {

// wave sum, the same bits in every lane: DPP within each 16-lane row (quad_perm 1032, quad_perm 2301, half-mirror,
// mirror: every lane of a row then holds the row sum, bitwise equal, since each step adds the same two values),
// then the four row sums read from lanes 0/16/32/48 (v_readlane) and added in a fixed order. __shfl_xor compiles to
// six ds_bpermute round trips per double; this is four DPP moves and eight readlanes.
template <int CTRL>
__device__ __forceinline__ double dppd(double v) {
    const long long b = __double_as_longlong(v);
    const int lo = __builtin_amdgcn_update_dpp(0, (int)b, CTRL, 0xF, 0xF, false);
    const int hi = __builtin_amdgcn_update_dpp(0, (int)(b >> 32), CTRL, 0xF, 0xF, false);
    return __longlong_as_double(((long long)hi << 32) | (unsigned)lo);
}
__device__ __forceinline__ double lane_d(double v, int l) {
    const long long b = __double_as_longlong(v);
    const int lo = __builtin_amdgcn_readlane((int)b, l);
    const int hi = __builtin_amdgcn_readlane((int)(b >> 32), l);
    return __longlong_as_double(((long long)hi << 32) | (unsigned)lo);
}
__device__ __forceinline__ double wsum(double v) {
    v += dppd<0xB1>(v);   // quad_perm [1,0,3,2]
    v += dppd<0x4E>(v);   // quad_perm [2,3,0,1]
    v += dppd<0x141>(v);  // row_half_mirror
    v += dppd<0x140>(v);  // row_mirror
    return (lane_d(v, 0) + lane_d(v, 16)) + (lane_d(v, 32) + lane_d(v, 48));
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
    double tol2;       // pivot: stop when the largest trailing column norm^2 <= tol2 (tol2 < 0: relative mode, below)
    double rel2;       // relative mode (> 0): stop at rel2 x the largest column norm^2 of W, found by step 0's pivot
                       //   search and kept in *thr for the later steps
    double* thr;
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
    if (a.ctrl && a.ctrl[0] <= k) return;  // ctrl == nullptr: a panel of the blocked QR (plain, full rank)
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
        double lim = a.tol2;
        if (a.rel2 > 0.0) {
            if (k == 0) {
                lim = a.rel2 * best;
                if (wave == 0 && lane == 0) *a.thr = lim;
            } else {
                lim = *a.thr;
            }
        }
        if (best <= lim) {
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
// unperm: column j of R (pivoted order) is written as column perm[j] (R P^T, the original column order)
__global__ void qr_extract_r_kernel(QRArgs a, int rank, double2* R, int* perm_out, int unperm) {
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
    R[(size_t)(unperm ? c : j) * rank + i] = v;
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
// workgroup-per-column step kernels (m <= 256 * EPT): the per-wave kernels above walk a column of m rows 64 at a
// time in a dependent loop, three passes per step, so a launch costs 20-50 us of memory latency at m ~ 3000
// (rocprofv3, profiles/r04/ptgen/). Here a column is spread over 256 threads and held in registers for the whole
// step: one round of loads, two workgroup reductions (LDS), one round of stores. Same arithmetic, same outputs.
// -------------------------------------------------------------------------------------------------------------
constexpr int WG_T = 256;

// sum NV doubles over the workgroup; every thread gets the totals (red: 4 x NV scratch, one barrier pair)
template <int NV>
__device__ __forceinline__ void wg_reduce(double (&v)[NV], double* red) {
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
#pragma unroll
    for (int q = 0; q < NV; ++q) v[q] = wsum(v[q]);
    if (lane == 0)
#pragma unroll
        for (int q = 0; q < NV; ++q) red[wv * NV + q] = v[q];
    __syncthreads();
#pragma unroll
    for (int q = 0; q < NV; ++q) v[q] = red[q] + red[NV + q] + red[2 * NV + q] + red[3 * NV + q];
}

// two reflectors per launch, plain QR: workgroup 0 stores column k into X, workgroup 1 column k+1 after H_k,
// workgroup g >= 2 updates column k + g (qr_step2_kernel's arithmetic)
template <int EPT>
__global__ __launch_bounds__(WG_T) void qr_step2_wg_kernel(QRArgs a, int k) {
    __shared__ double red[2][4 * 5];
    const int tid = threadIdx.x, jw = blockIdx.x, m = a.m;
    const int j = k + jw;
    if (jw >= 2 && j >= a.n) return;
    const double2* c0 = a.W + (size_t)k * m;
    const double2* c1 = a.W + (size_t)(k + 1) * m;
    double2* col = a.W + (size_t)j * m;
    const bool upd = jw >= 2;
    double2 u0[EPT], u1[EPT], cj[EPT];
#pragma unroll
    for (int e = 0; e < EPT; ++e) {
        const int i = tid + WG_T * e;
        const bool in = i < m;
        u0[e] = in ? c0[i] : c_zero();
        u1[e] = in ? c1[i] : c_zero();
        cj[e] = (in && upd) ? col[i] : c_zero();
    }
    const double2 c0k = c0[k], c0k1 = c0[k + 1], c1k = c1[k], c1k1 = c1[k + 1];
    const double2 ck = upd ? col[k] : c_zero(), ck1 = upd ? col[k + 1] : c_zero();
    double r1[5] = {0.0, 0.0, 0.0, 0.0, 0.0};  // |c0|^2, c0^H c1, c0^H c_j over rows > k
#pragma unroll
    for (int e = 0; e < EPT; ++e) {
        const int i = tid + WG_T * e;
        if (i > k && i < m) {
            const double2 u = u0[e], v = u1[e], w = cj[e];
            r1[0] += c_abs2(u);
            r1[1] += u.x * v.x + u.y * v.y;
            r1[2] += u.x * v.y - u.y * v.x;
            r1[3] += u.x * w.x + u.y * w.y;
            r1[4] += u.x * w.y - u.y * w.x;
        }
    }
    wg_reduce<5>(r1, red[0]);
    const Refl R0 = make_refl(c0k, r1[0]);
    const double2 w0 = c_add(c1k, c_cmul(R0.scale, make_double2(r1[1], r1[2])));
    const double2 ct01 = c_cmul(R0.tau, w0);
    const double2 f01 = c_mul(ct01, R0.scale);
    const double2 alpha1 = c_sub(c1k1, c_mul(f01, c0k1));
    const double2 ctA = c_cmul(R0.tau, c_add(ck, c_cmul(R0.scale, make_double2(r1[3], r1[4]))));
    const double2 fA = c_mul(ctA, R0.scale);
    double r2[3] = {0.0, 0.0, 0.0};  // |c1'|^2 over rows > k+1, v1^H (H_k^H c_j)
#pragma unroll
    for (int e = 0; e < EPT; ++e) {
        const int i = tid + WG_T * e;
        if (i > k + 1 && i < m) {
            const double2 v1 = c_sub(u1[e], c_mul(f01, u0[e]));
            const double2 y = c_sub(cj[e], c_mul(fA, u0[e]));
            r2[0] += c_abs2(v1);
            r2[1] += v1.x * y.x + v1.y * y.y;
            r2[2] += v1.x * y.y - v1.y * y.x;
        }
    }
    wg_reduce<3>(r2, red[1]);
    const Refl R1 = make_refl(alpha1, r2[0]);
    if (jw == 0) {
        if (tid == 0) {
            a.tau[k] = R0.tau; a.scale[k] = R0.scale; a.beta[k] = R0.beta;
            a.tau[k + 1] = R1.tau; a.scale[k + 1] = R1.scale; a.beta[k + 1] = R1.beta;
        }
#pragma unroll
        for (int e = 0; e < EPT; ++e) {
            const int i = tid + WG_T * e;
            if (i < m) a.X[(size_t)k * m + i] = u0[e];
        }
        return;
    }
    if (jw == 1) {
#pragma unroll
        for (int e = 0; e < EPT; ++e) {
            const int i = tid + WG_T * e;
            if (i >= m) continue;
            double2 v = u1[e];
            if (i == k) v = c_sub(v, ct01);
            else if (i > k) v = c_sub(v, c_mul(f01, u0[e]));
            a.X[(size_t)(k + 1) * m + i] = v;
        }
        return;
    }
    const double2 yk1 = c_sub(ck1, c_mul(fA, c0k1));
    const double2 ctB = c_cmul(R1.tau, c_add(yk1, c_cmul(R1.scale, make_double2(r2[1], r2[2]))));
    const double2 fB = c_mul(ctB, R1.scale);
#pragma unroll
    for (int e = 0; e < EPT; ++e) {
        const int i = tid + WG_T * e;
        if (i > k + 1 && i < m) {
            const double2 v1 = c_sub(u1[e], c_mul(f01, u0[e]));
            col[i] = c_sub(c_sub(cj[e], c_mul(fA, u0[e])), c_mul(fB, v1));
        }
    }
    if (tid == 0) {
        col[k] = c_sub(ck, ctA);
        col[k + 1] = c_sub(yk1, ctB);
    }
}

// one reflector per launch (column pivoting optional): workgroup 0 records the reflector / permutation (and the X
// copy), workgroup g >= 1 updates logical column k + g and its trailing norm (qr_step_kernel's arithmetic)
template <int EPT>
__global__ __launch_bounds__(WG_T) void qr_step_wg_kernel(QRArgs a, int k) {
    __shared__ double red[2][4 * 3];
    __shared__ int s_p;
    __shared__ double s_best;
    if (a.ctrl && a.ctrl[0] <= k) return;
    const int tid = threadIdx.x, jw = blockIdx.x, m = a.m;
    const int* pin = a.pivot ? a.perm + (size_t)(k & 1) * a.n : nullptr;
    int* pout = a.pivot ? a.perm + (size_t)((k + 1) & 1) * a.n : nullptr;
    const double* nin = a.pivot ? a.norms + (size_t)(k & 1) * a.n : nullptr;
    double* nout = a.pivot ? a.norms + (size_t)((k + 1) & 1) * a.n : nullptr;
    int p = k;
    if (a.pivot) {
        if (tid < 64) {
            double best = -1.0;
            int bj = k;
            for (int jj = k + tid; jj < a.n; jj += 64) {
                const double v = nin[pin[jj]];
                if (v > best) { best = v; bj = jj; }
            }
#pragma unroll
            for (int o = 32; o > 0; o >>= 1) {
                const double ob = __shfl_xor(best, o);
                const int oj = __shfl_xor(bj, o);
                if (ob > best || (ob == best && oj < bj)) { best = ob; bj = oj; }
            }
            if (tid == 0) { s_p = bj; s_best = best; }
        }
        __syncthreads();
        p = s_p;
        double lim = a.tol2;
        if (a.rel2 > 0.0) {
            if (k == 0) {
                lim = a.rel2 * s_best;
                if (jw == 0 && tid == 0) *a.thr = lim;
            } else {
                lim = *a.thr;
            }
        }
        if (s_best <= lim) {
            if (jw == 0 && tid == 0) a.ctrl[0] = k;
            return;
        }
    }
    auto phys = [&](int jj) {
        if (!a.pivot) return jj;
        return jj == k ? pin[p] : (jj == p ? pin[k] : pin[jj]);
    };
    const int j = k + jw;
    if (jw >= 1 && j >= a.n) return;
    const bool upd = jw >= 1;
    const double2* x = a.W + (size_t)phys(k) * m;
    const int c = upd ? phys(j) : 0;
    double2* col = a.W + (size_t)c * m;
    double2 u[EPT], cj[EPT];
#pragma unroll
    for (int e = 0; e < EPT; ++e) {
        const int i = tid + WG_T * e;
        const bool in = i < m;
        u[e] = in ? x[i] : c_zero();
        cj[e] = (in && upd) ? col[i] : c_zero();
    }
    const double2 alpha = x[k];
    const double2 ck = upd ? col[k] : c_zero();
    double r1[3] = {0.0, 0.0, 0.0};
#pragma unroll
    for (int e = 0; e < EPT; ++e) {
        const int i = tid + WG_T * e;
        if (i > k && i < m) {
            const double2 v = u[e], w = cj[e];
            r1[0] += c_abs2(v);
            r1[1] += v.x * w.x + v.y * w.y;
            r1[2] += v.x * w.y - v.y * w.x;
        }
    }
    wg_reduce<3>(r1, red[0]);
    const Refl R = make_refl(alpha, r1[0]);
    if (jw == 0) {
        if (tid == 0) { a.tau[k] = R.tau; a.scale[k] = R.scale; a.beta[k] = R.beta; }
        if (a.pivot)
            for (int jj = tid; jj < a.n; jj += WG_T) pout[jj] = jj < k ? pin[jj] : phys(jj);
        if (a.X != a.W)
#pragma unroll
            for (int e = 0; e < EPT; ++e) {
                const int i = tid + WG_T * e;
                if (i < m) a.X[(size_t)k * m + i] = u[e];
            }
        return;
    }
    const double2 s = c_add(ck, c_cmul(R.scale, make_double2(r1[1], r1[2])));
    const double2 ct = c_cmul(R.tau, s);
    const double2 f = c_mul(ct, R.scale);  // c_i -= ct v_i = f x_i for i > k
    double r2[1] = {0.0};
#pragma unroll
    for (int e = 0; e < EPT; ++e) {
        const int i = tid + WG_T * e;
        if (i > k && i < m) {
            const double2 ci = c_sub(cj[e], c_mul(f, u[e]));
            col[i] = ci;
            r2[0] += c_abs2(ci);
        }
    }
    if (tid == 0) col[k] = c_sub(ck, ct);
    if (a.pivot) {
        wg_reduce<1>(r2, red[1]);
        if (tid == 0) nout[c] = r2[0];
    }
}

// -------------------------------------------------------------------------------------------------------------
// blocked Q formation / trailing update helpers
// -------------------------------------------------------------------------------------------------------------
// Vc (nb x (m - i0), row-major) of reflectors i0 .. i0+nb-1: row b = v_{i0+b} from row i0 on (0 above its own row,
// 1 at it, x * scale below); reflector i's column is X[perm[i]] (perm == nullptr: i)
__global__ __launch_bounds__(256) void refl_block_kernel(const double2* X, int m, const int* perm, int i0, int nb,
                                                        const double2* scale, double2* Vc) {
    const int lane = threadIdx.x & 63;
    const int w = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    if (w >= nb) return;
    const int i = i0 + w, mm = m - i0;
    const int pc = perm ? perm[i] : i;
    const double2* x = X + (size_t)pc * m;
    double2* v = Vc + (size_t)w * mm;
    const double2 sc = scale[i];
    for (int r = i0 + lane; r < m; r += 64)
        v[r - i0] = r < i ? c_zero() : (r == i ? make_double2(1.0, 0.0) : c_mul(x[r], sc));
}

// Yp[chunk][j][b] = sum over the chunk's rows r of A[j][r] conj(Vc[b][r]) (A: ncol rows of length mm, stride lda;
// VHA_RC rows per chunk; the caller sums the chunks): the long-inner-dimension product V^H A of the blocked
// updates, spread over (ncol / VHA_J) x (mm / VHA_RC) workgroups with 64-row tiles staged in LDS
constexpr int VHA_J = 64, VHA_RC = 128, VHA_TR = 32, VHA_NB = 32;
__global__ __launch_bounds__(256) void vha_kernel(const double2* A, int lda, int ncol, const double2* Vc, int mm,
                                                 int nb, double2* Yp) {
    __shared__ double2 sV[VHA_NB][VHA_TR + 1];
    __shared__ double2 sA[VHA_J][VHA_TR + 1];
    constexpr int NV = VHA_NB * VHA_TR / 256, NA = VHA_J * VHA_TR / 256;  // elements per thread and tile
    const int tid = threadIdx.x;
    const int j0 = blockIdx.x * VHA_J, r0 = blockIdx.y * VHA_RC;
    const int tb = tid & 7, tj = tid >> 3;  // outputs (tb + 8p, j0 + tj + 32q), p < 4, q < 2
    const int rend = min(mm, r0 + VHA_RC);
    double2 acc[4][2];
#pragma unroll
    for (int p = 0; p < 4; ++p) acc[p][0] = acc[p][1] = c_zero();
    double2 pv[NV], pa[NA];  // the next tile, in flight while the current one is multiplied
    auto fetch = [&](int rt) {
#pragma unroll
        for (int u = 0; u < NV; ++u) {
            const int q = tid + 256 * u, bb = q / VHA_TR, rr = q - bb * VHA_TR;
            pv[u] = (bb < nb && rt + rr < rend) ? Vc[(size_t)bb * mm + rt + rr] : c_zero();
        }
#pragma unroll
        for (int u = 0; u < NA; ++u) {
            const int q = tid + 256 * u, jj = q / VHA_TR, rr = q - jj * VHA_TR;
            pa[u] = (j0 + jj < ncol && rt + rr < rend) ? A[(size_t)(j0 + jj) * lda + rt + rr] : c_zero();
        }
    };
    fetch(r0);
    for (int rt = r0; rt < rend; rt += VHA_TR) {
        __syncthreads();
#pragma unroll
        for (int u = 0; u < NV; ++u) {
            const int q = tid + 256 * u, bb = q / VHA_TR, rr = q - bb * VHA_TR;
            sV[bb][rr] = pv[u];
        }
#pragma unroll
        for (int u = 0; u < NA; ++u) {
            const int q = tid + 256 * u, jj = q / VHA_TR, rr = q - jj * VHA_TR;
            sA[jj][rr] = pa[u];
        }
        __syncthreads();
        if (rt + VHA_TR < rend) fetch(rt + VHA_TR);
#pragma unroll 4
        for (int rr = 0; rr < VHA_TR; ++rr) {
            double2 v[4], av[2];
#pragma unroll
            for (int p = 0; p < 4; ++p) v[p] = sV[tb + 8 * p][rr];
            av[0] = sA[tj][rr];
            av[1] = sA[tj + 32][rr];
#pragma unroll
            for (int p = 0; p < 4; ++p)
#pragma unroll
                for (int q = 0; q < 2; ++q) {  // a conj(v)
                    acc[p][q].x = fma(av[q].x, v[p].x, fma(av[q].y, v[p].y, acc[p][q].x));
                    acc[p][q].y = fma(av[q].y, v[p].x, fma(-av[q].x, v[p].y, acc[p][q].y));
                }
        }
    }
#pragma unroll
    for (int p = 0; p < 4; ++p)
#pragma unroll
        for (int q = 0; q < 2; ++q) {
            const int b = tb + 8 * p, j = j0 + tj + 32 * q;
            if (b < nb && j < ncol) Yp[((size_t)blockIdx.y * ncol + j) * nb + b] = acc[p][q];
        }
}

// Zt[j][b] = (op(T) Y)[b][j] with Y[c][j] = sum over chunks of Yp[ch][j][c]; herm = 0: op(T) = T (Q formation,
// Q <- Q - V T V^H Q), herm = 1: op(T) = T^H (trailing update, A <- A - V T^H V^H A). T is never formed: its inverse is
// diag(1/tau) + striu(S) with S = V^H V (the UT transform; LAPACK zlarft's T is its inverse), so op(T) Y is one
// triangular substitution per column (lane b holds y_b). A reflector with tau = 0 is the identity: z_b = 0.
__global__ __launch_bounds__(64) void zt_kernel(const double2* Yp, int nch, int ncol, int nb, const double2* S,
                                               const double2* tau, int i0, int herm, double2* Zt) {
    const int j = blockIdx.x, b = threadIdx.x;
    double2 y = c_zero();
    if (b < nb)
        for (int ch = 0; ch < nch; ++ch) y = c_add(y, Yp[((size_t)ch * ncol + j) * nb + b]);
    const double2 tb = b < nb ? tau[i0 + b] : c_zero();
    double2 z = c_zero();
    if (!herm) {  // T^-1 z = y, back substitution
        for (int c = nb - 1; c >= 0; --c) {
            if (b == c) z = c_mul(tb, y);
            const double2 zc = make_double2(__shfl(z.x, c), __shfl(z.y, c));
            if (b < c) y = c_sub(y, c_mul(S[(size_t)b * nb + c], zc));
        }
    } else {      // T^-H z = y, forward substitution
        for (int c = 0; c < nb; ++c) {
            if (b == c) z = c_mul(c_conj(tb), y);
            const double2 zc = make_double2(__shfl(z.x, c), __shfl(z.y, c));
            if (b > c && b < nb) y = c_sub(y, c_mul(c_conj(S[(size_t)c * nb + b]), zc));
        }
    }
    if (b < nb) Zt[(size_t)j * nb + b] = z;
}

// A[j][r] -= sum_b Zt[j][b] Vc[b][r] (r < mm): workgroup (r-chunk, j)
__global__ __launch_bounds__(256) void rank_update_kernel(double2* A, int lda, int mm, const double2* Vc, int nb,
                                                         const double2* Zt) {
    __shared__ double2 sz[64];
    const int j = blockIdx.y, r = blockIdx.x * 256 + threadIdx.x;
    if (threadIdx.x < nb) sz[threadIdx.x] = Zt[(size_t)j * nb + threadIdx.x];
    __syncthreads();
    if (r >= mm) return;
    double2 acc = c_zero();
    for (int b = 0; b < nb; ++b) c_fma(acc, sz[b], Vc[(size_t)b * mm + r]);
    double2* p = A + (size_t)j * lda + r;
    *p = c_sub(*p, acc);
}

// -------------------------------------------------------------------------------------------------------------
// blocked (compact-WY) plain QR: the panel's columns are factorized by the column kernels above with a.n = the
// panel end; the kernels below turn the panel's reflectors into V (unit lower trapezoidal, rows >= k0) and the
// upper triangular T of LAPACK's zlarft (H_k0 ... H_k0+nb-1 = I - V T V^H), applied to the trailing columns and,
// in every QR on the multi-workgroup path, to Q (blocks of QB = 32 reflectors: vha_kernel, zt_kernel,
// rank_update_kernel).
// -------------------------------------------------------------------------------------------------------------
// S[i][l] = v_i^H v_l for i < l (row-major nb x nb), one wave per pair; v_l is zero above its row l - k0
__global__ __launch_bounds__(256) void panel_gram_kernel(const double2* Vc, int mm, int nb, double2* S) {
    const int lane = threadIdx.x & 63;
    const int w = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    if (w >= nb * nb) return;
    const int i = w / nb, l = w - i * nb;
    if (i >= l) return;
    const double2* vi = Vc + (size_t)i * mm;
    const double2* vl = Vc + (size_t)l * mm;
    double2 s = c_zero();
    for (int r = l + lane; r < mm; r += 64) {
        const double2 a = vi[r], b = vl[r];
        s.x += a.x * b.x + a.y * b.y;
        s.y += a.x * b.y - a.y * b.x;
    }
    s = wsum2(s);
    if (lane == 0) S[(size_t)i * nb + l] = s;
}

// -------------------------------------------------------------------------------------------------------------
// single-workgroup QR for matrices that fit in LDS (m * n <= QS_MAX): the same arithmetic, one barrier per step
// -------------------------------------------------------------------------------------------------------------
constexpr int QS_MAX = 8192;  // 128 KiB of complex doubles
constexpr int QS_THREADS = 1024;

template <int QE>
__global__ __launch_bounds__(QS_THREADS) void qr_small_kernel(const double2* Win, int m, int n, int pivot, double tol2,
                                                             double rel2, double2* Q, double2* R, int* perm_out,
                                                             int* rank_out, int unperm, int diag) {
    // one barrier per column step: every wave finds the pivot and builds the reflector itself (redundantly, from
    // LDS), then updates its trailing columns; the permutation is double-buffered by step parity (wave 0 writes the
    // next one), so no wave waits for a serial pivot / reflector phase
    extern __shared__ double2 sm[];
    double2* A = sm;                       // m x n
    __shared__ double2 s_tau[256], s_scale[256];
    __shared__ double s_beta[256], s_norm[2][256];  // norms by physical column, double-buffered like the perm
    __shared__ int s_perm[2][256];
    __shared__ int s_rank;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, nw = QS_THREADS / 64;
    const int kmax = min(m, n);
    for (int idx = tid; idx < m * n; idx += QS_THREADS) A[idx] = Win[idx];
    for (int j = tid; j < n; j += QS_THREADS) s_perm[0][j] = j;
    if (tid == 0) s_rank = kmax;
    __syncthreads();
    if (pivot)
        for (int c = wave; c < n; c += nw) {
            double sacc = 0.0;
            for (int i = lane; i < m; i += 64) sacc += c_abs2(A[c * m + i]);
            sacc = wsum(sacc);
            if (lane == 0) s_norm[0][c] = sacc;
        }
    __syncthreads();
    int k = 0;
    for (; k < ((diag & 2) ? 0 : kmax); ++k) {  // diag (PQD_PTG_DIAG, timing only): 2 = no column steps
        const int* pin = s_perm[k & 1];
        int* pout = s_perm[(k + 1) & 1];
        const double* nin = s_norm[k & 1];
        double* nout = s_norm[(k + 1) & 1];
        int p = k;
        if (pivot) {
            double best = -1.0;
            int bj = k;
            for (int j = k + lane; j < n; j += 64) {
                const double v = nin[pin[j]];
                if (v > best) { best = v; bj = j; }
            }
#pragma unroll
            for (int o = 32; o > 0; o >>= 1) {
                const double ob = __shfl_xor(best, o);
                const int oj = __shfl_xor(bj, o);
                if (ob > best || (ob == best && oj < bj)) { best = ob; bj = oj; }
            }
            if (k == 0 && rel2 > 0.0) tol2 = rel2 * best;  // relative mode: step 0 sees the largest column norm
            if (best <= tol2) break;  // the same decision in every wave (same LDS values, same reduction)
            p = bj;
        }
        auto phys = [&](int j) { return j == k ? pin[p] : (j == p ? pin[k] : pin[j]); };
        const double2* x = A + phys(k) * m;
        if constexpr (QE > 0) {
            // the pivot column in registers for the whole step; each trailing column: one round of LDS loads
            double2 xr[QE];
            double xn = 0.0;
#pragma unroll
            for (int e = 0; e < QE; ++e) {
                const int r = lane + 64 * e;
                xr[e] = r < m ? x[r] : c_zero();
                if (r > k && r < m) xn += c_abs2(xr[e]);
            }
            xn = wsum(xn);
            const Refl Rf = make_refl(x[k], xn);
            if (wave == 0) {
                if (lane == 0) { s_tau[k] = Rf.tau; s_scale[k] = Rf.scale; s_beta[k] = Rf.beta; }
                for (int j = lane; j < n; j += 64) pout[j] = j < k ? pin[j] : phys(j);
            }
#pragma unroll
            for (int e = 0; e < QE; ++e) {
                const int r = lane + 64 * e;
                xr[e] = r > k && r < m ? c_mul(xr[e], Rf.scale) : c_zero();  // v below the diagonal
            }
            for (int j = k + 1 + wave; j < n; j += nw) {
                const int cidx = phys(j);
                double2* col = A + cidx * m;
                double2 cv[QE];
#pragma unroll
                for (int e = 0; e < QE; ++e) {
                    const int r = lane + 64 * e;
                    cv[e] = r < m ? col[r] : c_zero();
                }
                const double2 ck = col[k];
                double2 sacc = c_zero();
#pragma unroll
                for (int e = 0; e < QE; ++e) {
                    sacc.x += xr[e].x * cv[e].x + xr[e].y * cv[e].y;
                    sacc.y += xr[e].x * cv[e].y - xr[e].y * cv[e].x;
                }
                sacc = c_add(wsum2(sacc), ck);
                const double2 ct = c_cmul(Rf.tau, sacc);
                double nn = 0.0;
#pragma unroll
                for (int e = 0; e < QE; ++e) {
                    const int r = lane + 64 * e;
                    if (r > k && r < m) {
                        const double2 ci = c_sub(cv[e], c_mul(ct, xr[e]));
                        col[r] = ci;
                        nn += c_abs2(ci);
                    }
                }
                if (pivot) nn = wsum(nn);  // trailing norms only steer the pivot search
                if (lane == 0) {
                    col[k] = c_sub(ck, ct);
                    nout[cidx] = nn;
                }
            }
        } else {
            double xn = 0.0;
            for (int i = k + 1 + lane; i < m; i += 64) xn += c_abs2(x[i]);
            xn = wsum(xn);
            const Refl Rf = make_refl(x[k], xn);
            if (wave == 0) {
                if (lane == 0) { s_tau[k] = Rf.tau; s_scale[k] = Rf.scale; s_beta[k] = Rf.beta; }
                for (int j = lane; j < n; j += 64) pout[j] = j < k ? pin[j] : phys(j);
            }
            const double2 sc = Rf.scale, tau = Rf.tau;
            for (int j = k + 1 + wave; j < n; j += nw) {
                const int cidx = phys(j);
                double2* col = A + cidx * m;
                const double2 ck = col[k];
                double2 sacc = c_zero();
                for (int i = k + 1 + lane; i < m; i += 64) {
                    const double2 v = c_mul(x[i], sc);
                    const double2 ci = col[i];
                    sacc.x += v.x * ci.x + v.y * ci.y;
                    sacc.y += v.x * ci.y - v.y * ci.x;
                }
                sacc = wsum2(sacc);
                sacc = c_add(sacc, ck);
                const double2 ct = c_cmul(tau, sacc);
                double nn = 0.0;
                for (int i = k + 1 + lane; i < m; i += 64) {
                    const double2 ci = c_sub(col[i], c_mul(ct, c_mul(x[i], sc)));
                    col[i] = ci;
                    nn += c_abs2(ci);
                }
                if (pivot) nn = wsum(nn);  // trailing norms only steer the pivot search
                if (lane == 0) {
                    col[k] = c_sub(ck, ct);
                    nout[cidx] = nn;
                }
            }
        }
        __syncthreads();
    }
    if (tid == 0) s_rank = k;
    __syncthreads();
    const int* s_pf = s_perm[k & 1];
    const int rank = s_rank;
    // R (rank x n), perm
    for (int idx = tid; idx < rank * n; idx += QS_THREADS) {
        const int j = idx / rank, i = idx - j * rank;
        const int c = s_pf[j];
        R[unperm ? c * rank + i : idx] = i < j ? A[c * m + i] : (i == j ? make_double2(s_beta[i], 0.0) : c_zero());
    }
    for (int j = tid; j < n; j += QS_THREADS) perm_out[j] = s_pf[j];
    if (tid == 0) *rank_out = rank;
    if (diag & 1) return;  // timing only: no Q
    // Q (m x rank), one wave per column, reflectors descending. QE > 0: the column lives in registers (QE rows per
    // lane, m <= 64 QE) and goes to global memory once; QE == 0: in global memory (a round trip per reflector)
    for (int j = wave; j < rank; j += nw) {
        double2* col = Q + (size_t)j * m;
        if constexpr (QE > 0) {
            double2 q[QE];
#pragma unroll
            for (int e = 0; e < QE; ++e) q[e] = make_double2(lane + 64 * e == j ? 1.0 : 0.0, 0.0);
            for (int i = j; i >= 0; --i) {
                const double2* x = A + s_pf[i] * m;
                const double2 sc = s_scale[i], tau = s_tau[i];
                double2 sacc = c_zero();
                double2 v[QE];
#pragma unroll
                for (int e = 0; e < QE; ++e) {
                    const int r = lane + 64 * e;
                    v[e] = r > i && r < m ? c_mul(x[r], sc) : (r == i ? make_double2(1.0, 0.0) : c_zero());
                    sacc.x += v[e].x * q[e].x + v[e].y * q[e].y;
                    sacc.y += v[e].x * q[e].y - v[e].y * q[e].x;
                }
                sacc = wsum2(sacc);
                const double2 t = c_mul(tau, sacc);
#pragma unroll
                for (int e = 0; e < QE; ++e) q[e] = c_sub(q[e], c_mul(t, v[e]));
            }
#pragma unroll
            for (int e = 0; e < QE; ++e) {
                const int r = lane + 64 * e;
                if (r < m) col[r] = q[e];
            }
        } else {
            for (int i = lane; i < m; i += 64) col[i] = make_double2(i == j ? 1.0 : 0.0, 0.0);
            for (int i = j; i >= 0; --i) {
                const double2* x = A + s_pf[i] * m;
                const double2 sc = s_scale[i], tau = s_tau[i];
                const double2 ci0 = col[i];
                double2 sacc = c_zero();
                for (int r = i + 1 + lane; r < m; r += 64) {
                    const double2 v = c_mul(x[r], sc);
                    const double2 cr = col[r];
                    sacc.x += v.x * cr.x + v.y * cr.y;
                    sacc.y += v.x * cr.y - v.y * cr.x;
                }
                sacc = wsum2(sacc);
                sacc = c_add(sacc, ci0);
                const double2 t = c_mul(tau, sacc);
                for (int r = i + 1 + lane; r < m; r += 64) col[r] = c_sub(col[r], c_mul(t, c_mul(x[r], sc)));
                if (lane == 0) col[i] = c_sub(ci0, t);
            }
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
    bool conv = false;
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
        if (s_cnt == 0) { ++sweep; conv = true; break; }
        __syncthreads();
    }
    for (int idx = tid; idx < n * n; idx += QS_THREADS) {
        Xg[idx] = X[idx];
        Vg[idx] = V[idx];
    }
    if (tid == 0) *sweeps_out = conv ? sweep : max_sweeps + 1;  // > max_sweeps: no convergence
}

// persistent one-sided Jacobi: every round of every sweep in ONE launch. Wave i of the grid owns tournament slot i;
// its two columns of X (and, when it rotates, of V) are loaded into registers, rotated and stored back, then the
// grid meets at a barrier (a monotonic counter) before the next round. Hand-off as in pt_split.hip (the guide's
// valid form): payload loads/stores are 16-B sc1 buffer accesses (coherent across the XCDs), each storing wave drains with
// s_waitcnt vmcnt(0) before one lane per workgroup adds to the counter; the wait is a bounded poll. The rotation
// count of a sweep goes to cnt[sweep] before the sweep's last arrive; every workgroup reads it after that barrier
// and all leave together at the first sweep without a rotation. Needs all ceil(n/8) workgroups co-resident
// (n <= 1024: at most 128 of 256 threads) and n <= 64 * EPL.
typedef unsigned long long __attribute__((address_space(1))) gu64;
typedef unsigned int __attribute__((address_space(1))) gu32;
// 16-B element e of a buffer, sc1 (aux bit 16): coherent across the XCDs' L2s like the 8-B atomics above
typedef unsigned int v4u32 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ double2 ld16(__amdgpu_buffer_rsrc_t r, int e) {
    const v4u32 v = __builtin_amdgcn_raw_buffer_load_b128(r, e * 16, 0, 16);
    return make_double2(__hiloint2double((int)v.y, (int)v.x), __hiloint2double((int)v.w, (int)v.z));
}
__device__ __forceinline__ void st16(__amdgpu_buffer_rsrc_t r, int e, double2 d) {
    const long long x = __double_as_longlong(d.x), y = __double_as_longlong(d.y);
    v4u32 v;
    v.x = (unsigned)x; v.y = (unsigned)(x >> 32); v.z = (unsigned)y; v.w = (unsigned)(y >> 32);
    __builtin_amdgcn_raw_buffer_store_b128(v, r, e * 16, 0, 16);
}

struct JacPersist {
    unsigned* bar;        // arrivals (zeroed by the host)
    int* cnt;             // rotations per sweep (max_sweeps, zeroed)
    unsigned* err;        // 1: a barrier wait timed out
    int* sweeps;          // out
    int max_sweeps;
    unsigned spin_limit;
};

template <int EPL>
__global__ __launch_bounds__(256) void jac_persist_kernel(JacArgs a, JacPersist q) {
    __shared__ int s_rot, s_abort, s_done;
    const int tid = threadIdx.x, lane = tid & 63;
    const int slot = (blockIdx.x * blockDim.x + tid) >> 6;
    const int n = a.n, nn = a.nn, npair = nn / 2;
    const unsigned G = gridDim.x;
    const double zero2 = *a.zero2;
    const __amdgpu_buffer_rsrc_t rX = __builtin_amdgcn_make_buffer_rsrc(a.X, 0, n * n * 16, 0x00020000);
    const __amdgpu_buffer_rsrc_t rV = __builtin_amdgcn_make_buffer_rsrc(a.V, 0, n * n * 16, 0x00020000);
    unsigned epoch = 0;
    int sweep = 0;
    bool conv = false;
    if (tid == 0) s_abort = 0;
    for (; sweep < q.max_sweeps; ++sweep) {
        if (tid == 0) s_rot = 0;
        __syncthreads();
        for (int t = 0; t < nn - 1; ++t) {
            int p = 0, qq = n;
            if (slot < npair) jac_pair(t, slot, nn, p, qq);
            if (slot < npair && qq < n) {
                // X and V columns in one round of 16-B sc1 loads (V speculatively: one memory latency per round)
                const int xo = p * n, yo = qq * n;
                double2 up[EPL], uq[EPL], wp[EPL], wq[EPL];
#pragma unroll
                for (int e = 0; e < EPL; ++e) {
                    const int r = lane + 64 * e;
                    const bool in = r < n;
                    up[e] = in ? ld16(rX, xo + r) : c_zero();
                    uq[e] = in ? ld16(rX, yo + r) : c_zero();
                    wp[e] = in ? ld16(rV, xo + r) : c_zero();
                    wq[e] = in ? ld16(rV, yo + r) : c_zero();
                }
                double sa = 0.0, sb = 0.0;
                double2 c = c_zero();
#pragma unroll
                for (int e = 0; e < EPL; ++e) {
                    sa += c_abs2(up[e]);
                    sb += c_abs2(uq[e]);
                    c.x += up[e].x * uq[e].x + up[e].y * uq[e].y;
                    c.y += up[e].x * uq[e].y - up[e].y * uq[e].x;
                }
                sa = wsum(sa);
                sb = wsum(sb);
                c = wsum2(c);
                const double ac = sqrt(c.x * c.x + c.y * c.y);
                const bool rot = !(sa < zero2 || sb < zero2) && (ac > a.tol * sqrt(sa * sb)) && ac != 0.0;
                if (rot) {
                    const double2 eph = make_double2(c.x / ac, -c.y / ac);
                    const double zeta = (sb - sa) / (2.0 * ac);
                    const double tt = (zeta >= 0.0 ? 1.0 : -1.0) / (fabs(zeta) + sqrt(1.0 + zeta * zeta));
                    const double cs = 1.0 / sqrt(1.0 + tt * tt), sn = cs * tt;
#pragma unroll
                    for (int e = 0; e < EPL; ++e) {
                        const int r = lane + 64 * e;
                        if (r >= n) continue;
                        const double2 u = up[e], w = c_mul(uq[e], eph);
                        st16(rX, xo + r, make_double2(cs * u.x - sn * w.x, cs * u.y - sn * w.y));
                        st16(rX, yo + r, make_double2(sn * u.x + cs * w.x, sn * u.y + cs * w.y));
                        const double2 u2 = wp[e], w2 = c_mul(wq[e], eph);
                        st16(rV, xo + r, make_double2(cs * u2.x - sn * w2.x, cs * u2.y - sn * w2.y));
                        st16(rV, yo + r, make_double2(sn * u2.x + cs * w2.x, sn * u2.y + cs * w2.y));
                    }
                    if (lane == 0) atomicAdd(&s_rot, 1);
                }
            }
            // ---- grid barrier (and, after a sweep's last round, the sweep's rotation count)
            ++epoch;
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            __syncthreads();
            if (tid == 0) {
                if (t == nn - 2 && s_rot)
                    __hip_atomic_fetch_add((gu32*)(q.cnt + sweep), (unsigned)s_rot, __ATOMIC_RELAXED,
                                           __HIP_MEMORY_SCOPE_AGENT);
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                __hip_atomic_fetch_add((gu32*)q.bar, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
            if (tid < 64) {
                const unsigned target = G * epoch;
                unsigned spins = 0;
                bool ok = true;
                while (__hip_atomic_load((gu32*)q.bar, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < target) {
                    __builtin_amdgcn_s_sleep(1);
                    if (++spins > q.spin_limit) { ok = false; break; }
                }
                if (tid == 0 && !ok) {
                    s_abort = 1;
                    __hip_atomic_store((gu32*)q.err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                }
            }
            __syncthreads();
            if (s_abort) return;
        }
        if (tid == 0)
            s_done = __hip_atomic_load((gu32*)(q.cnt + sweep), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0u;
        __syncthreads();
        if (s_done) { ++sweep; conv = true; break; }
    }
    if (blockIdx.x == 0 && tid == 0) *q.sweeps = conv ? sweep : q.max_sweeps + 1;  // > max_sweeps: no convergence
}

// block one-sided Jacobi, persistent: columns dealt into blocks of JB = 4; workgroup i takes block pair i of a
// round-robin tournament over the blocks each round, loads the pair's 2 JB columns of X and V into LDS (every load of
// a wave in flight at once), runs one inner sweep over the 2 JB (2 JB - 1) / 2 local pairs (2 JB - 1 sub-rounds, one
// wave per pair, each rotation on register copies of its four column slices), stores the columns back and meets the
// grid at jac_persist_kernel's barrier (16-B sc1 accesses, one counter add per workgroup, bounded polls). A sweep is
// ceil(n / JB) - 1 grid barriers instead of n - 1. Stops at the first sweep without a rotation. LDS 4 JB n complex.
constexpr int JB = 4;

template <int EPL>
__device__ __forceinline__ bool jac_rotate_regs(double2* xp, double2* xq, double2* vp, double2* vq, int n, double tol,
                                                double zero2, int lane) {
    double2 up[EPL], uq[EPL], wp[EPL], wq[EPL];
#pragma unroll
    for (int e = 0; e < EPL; ++e) {
        const int r = lane + 64 * e;
        const bool in = r < n;
        up[e] = in ? xp[r] : c_zero();
        uq[e] = in ? xq[r] : c_zero();
        wp[e] = in ? vp[r] : c_zero();
        wq[e] = in ? vq[r] : c_zero();
    }
    double sa = 0.0, sb = 0.0;
    double2 c = c_zero();
#pragma unroll
    for (int e = 0; e < EPL; ++e) {
        sa += c_abs2(up[e]);
        sb += c_abs2(uq[e]);
        c.x += up[e].x * uq[e].x + up[e].y * uq[e].y;
        c.y += up[e].x * uq[e].y - up[e].y * uq[e].x;
    }
    sa = wsum(sa);
    sb = wsum(sb);
    c = wsum2(c);
    const double ac = sqrt(c.x * c.x + c.y * c.y);
    if (sa < zero2 || sb < zero2) return false;
    if (!(ac > tol * sqrt(sa * sb)) || ac == 0.0) return false;
    const double2 eph = make_double2(c.x / ac, -c.y / ac);
    const double zeta = (sb - sa) / (2.0 * ac);
    const double tt = (zeta >= 0.0 ? 1.0 : -1.0) / (fabs(zeta) + sqrt(1.0 + zeta * zeta));
    const double cs = 1.0 / sqrt(1.0 + tt * tt), sn = cs * tt;
#pragma unroll
    for (int e = 0; e < EPL; ++e) {
        const int r = lane + 64 * e;
        if (r >= n) continue;
        const double2 u = up[e], w = c_mul(uq[e], eph);
        xp[r] = make_double2(cs * u.x - sn * w.x, cs * u.y - sn * w.y);
        xq[r] = make_double2(sn * u.x + cs * w.x, sn * u.y + cs * w.y);
        const double2 u2 = wp[e], w2 = c_mul(wq[e], eph);
        vp[r] = make_double2(cs * u2.x - sn * w2.x, cs * u2.y - sn * w2.y);
        vq[r] = make_double2(sn * u2.x + cs * w2.x, sn * u2.y + cs * w2.y);
    }
    return true;
}

template <int EPL>
__global__ __launch_bounds__(256) void jac_block_kernel(JacArgs a, JacPersist q, int nblk) {
    extern __shared__ double2 sm[];  // X columns [2 JB][n], then V columns [2 JB][n]
    __shared__ int s_rot, s_abort, s_done;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int n = a.n;
    const unsigned G = gridDim.x;
    const double zero2 = *a.zero2;
    const __amdgpu_buffer_rsrc_t rX = __builtin_amdgcn_make_buffer_rsrc(a.X, 0, n * n * 16, 0x00020000);
    const __amdgpu_buffer_rsrc_t rV = __builtin_amdgcn_make_buffer_rsrc(a.V, 0, n * n * 16, 0x00020000);
    double2* sX = sm;
    double2* sV = sm + 2 * JB * n;
    unsigned epoch = 0;
    int sweep = 0;
    bool conv = false;
    if (tid == 0) s_abort = 0;
    for (; sweep < q.max_sweeps; ++sweep) {
        if (tid == 0) s_rot = 0;
        __syncthreads();
        for (int t = 0; t < nblk - 1; ++t) {
            int bp, bq;
            jac_pair(t, blockIdx.x, nblk, bp, bq);
            // wave w owns local columns w and w + 4 for the load and the store
            int gcs[2];
#pragma unroll
            for (int cc = 0; cc < 2; ++cc) {
                const int c = wave + 4 * cc;
                gcs[cc] = c < JB ? bp * JB + c : bq * JB + (c - JB);
            }
            {
                double2 rx[2][EPL], rv[2][EPL];
#pragma unroll
                for (int cc = 0; cc < 2; ++cc)
#pragma unroll
                    for (int e = 0; e < EPL; ++e) {
                        const int r = lane + 64 * e;
                        const bool in = gcs[cc] < n && r < n;
                        rx[cc][e] = in ? ld16(rX, gcs[cc] * n + r) : c_zero();
                        rv[cc][e] = in ? ld16(rV, gcs[cc] * n + r) : c_zero();
                    }
#pragma unroll
                for (int cc = 0; cc < 2; ++cc)
#pragma unroll
                    for (int e = 0; e < EPL; ++e) {
                        const int r = lane + 64 * e;
                        if (r < n) {
                            sX[(wave + 4 * cc) * n + r] = rx[cc][e];
                            sV[(wave + 4 * cc) * n + r] = rv[cc][e];
                        }
                    }
            }
            __syncthreads();
            for (int st = 0; st < 2 * JB - 1; ++st) {  // inner sweep: wave w rotates local pair w of sub-round st
                int lp, lq;
                jac_pair(st, wave, 2 * JB, lp, lq);
                const int gp = lp < JB ? bp * JB + lp : bq * JB + (lp - JB);
                const int gq = lq < JB ? bp * JB + lq : bq * JB + (lq - JB);
                if (gp < n && gq < n) {
                    const bool rot = jac_rotate_regs<EPL>(sX + lp * n, sX + lq * n, sV + lp * n, sV + lq * n, n, a.tol,
                                                          zero2, lane);
                    if (rot && lane == 0) atomicAdd(&s_rot, 1);
                }
                __syncthreads();
            }
#pragma unroll
            for (int cc = 0; cc < 2; ++cc) {
                if (gcs[cc] >= n) continue;
                double2 rx[EPL], rv[EPL];
#pragma unroll
                for (int e = 0; e < EPL; ++e) {
                    const int r = lane + 64 * e;
                    rx[e] = r < n ? sX[(wave + 4 * cc) * n + r] : c_zero();
                    rv[e] = r < n ? sV[(wave + 4 * cc) * n + r] : c_zero();
                }
#pragma unroll
                for (int e = 0; e < EPL; ++e) {
                    const int r = lane + 64 * e;
                    if (r < n) {
                        st16(rX, gcs[cc] * n + r, rx[e]);
                        st16(rV, gcs[cc] * n + r, rv[e]);
                    }
                }
            }
            // ---- grid barrier (and, after a sweep's last round, the sweep's rotation count)
            ++epoch;
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            __syncthreads();
            if (tid == 0) {
                if (t == nblk - 2 && s_rot)
                    __hip_atomic_fetch_add((gu32*)(q.cnt + sweep), (unsigned)s_rot, __ATOMIC_RELAXED,
                                           __HIP_MEMORY_SCOPE_AGENT);
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                __hip_atomic_fetch_add((gu32*)q.bar, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
            if (tid < 64) {
                const unsigned target = G * epoch;
                unsigned spins = 0;
                bool ok = true;
                while (__hip_atomic_load((gu32*)q.bar, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < target) {
                    __builtin_amdgcn_s_sleep(1);
                    if (++spins > q.spin_limit) { ok = false; break; }
                }
                if (tid == 0 && !ok) {
                    s_abort = 1;
                    __hip_atomic_store((gu32*)q.err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                }
            }
            __syncthreads();
            if (s_abort) return;
        }
        if (tid == 0)
            s_done = __hip_atomic_load((gu32*)(q.cnt + sweep), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0u;
        __syncthreads();
        if (s_done) { ++sweep; conv = true; break; }
    }
    if (blockIdx.x == 0 && tid == 0) *q.sweeps = conv ? sweep : q.max_sweeps + 1;  // > max_sweeps: no convergence
}

// persistent Householder QR (column-pivoted, or plain: a.pivot == 0, no search, no stop, no norms): every step in ONE
// launch, qr_step_wg_kernel's arithmetic. Workgroup g owns PHYSICAL
// column g for the whole factorization and holds it in registers; the permutation lives in each workgroup's LDS (every
// workgroup makes the same swap). Step k: the pivot search over the trailing norms (sc1 loads, the same scan and tie
// rule as the launch path), the stop test, the swap; the pivot column's owner records the reflector, the trailing
// workgroups read the pivot column (16-B sc1 loads), update their column in registers, store its rows >= k (sc1,
// for a later pivot read and for R) and its trailing norm, then the grid meets at jac_persist_kernel's barrier.
// Workgroups whose column is eliminated only keep the barrier count. Results equal the launch path's bit for bit.
// Needs all n workgroups co-resident (the host checks the occupancy; a timed-out barrier wait sets *q.err and every
// workgroup leaves, and the host reruns the factorization one launch per step from a saved copy).
struct QRPersist {
    unsigned* bar;
    unsigned* err;
    unsigned spin_limit;
};
template <int EPT>
__global__ __launch_bounds__(WG_T) void qrcp_persist_kernel(QRArgs a, QRPersist q) {
    extern __shared__ int s_perm[];  // n
    __shared__ double red[2][4 * 3];
    __shared__ int s_p, s_abort;
    __shared__ double s_best;
    __shared__ double2 s_ck;
    const int tid = threadIdx.x, g = blockIdx.x, m = a.m, n = a.n;
    const unsigned G = gridDim.x;
    const __amdgpu_buffer_rsrc_t rW = __builtin_amdgcn_make_buffer_rsrc(a.W, 0, m * n * 16, 0x00020000);
    for (int j = tid; j < n; j += WG_T) s_perm[j] = j;
    if (tid == 0) s_abort = 0;
    double2 cj[EPT];
#pragma unroll
    for (int e = 0; e < EPT; ++e) {
        const int i = tid + WG_T * e;
        cj[e] = i < m ? a.W[(size_t)g * m + i] : c_zero();
    }
    bool done = false;  // this column is a reflector column (eliminated)
    double lim = a.tol2;
    int k = 0;
    unsigned epoch = 0;
    __syncthreads();
    for (; k < a.kmax; ++k) {
        const double* nin = a.norms + (size_t)(k & 1) * n;
        double* nout = a.norms + (size_t)((k + 1) & 1) * n;
        if (a.pivot && tid < 64) {
            double best = -1.0;
            int bj = k;
            for (int jj = k + tid; jj < n; jj += 64) {
                const unsigned long long b = __hip_atomic_load((gu64*)(nin + s_perm[jj]), __ATOMIC_RELAXED,
                                                               __HIP_MEMORY_SCOPE_AGENT);
                const double v = __longlong_as_double((long long)b);
                if (v > best) { best = v; bj = jj; }
            }
#pragma unroll
            for (int o = 32; o > 0; o >>= 1) {
                const double ob = __shfl_xor(best, o);
                const int oj = __shfl_xor(bj, o);
                if (ob > best || (ob == best && oj < bj)) { best = ob; bj = oj; }
            }
            if (tid == 0) { s_p = bj; s_best = best; }
        }
        __syncthreads();
        const int p = a.pivot ? s_p : k;  // plain QR: no search, no stop (s_perm stays the identity)
        if (a.pivot) {
            const double sb = s_best;
            if (a.rel2 > 0.0 && k == 0) {
                lim = a.rel2 * sb;
                if (g == 0 && tid == 0) *a.thr = lim;
            }
            if (sb <= lim) {
                if (g == 0 && tid == 0) a.ctrl[0] = k;
                break;
            }
        }
        const int cp = s_perm[p];  // the pivot's physical column
        __syncthreads();           // every thread has read s_perm[p] before the swap
        if (tid == 0) { s_perm[p] = s_perm[k]; s_perm[k] = cp; }
        if (!done) {
            const bool own = cp == g;  // this workgroup's column is the pivot: it records the reflector
            // row k of this column (own: alpha; trailing: c_k) to every thread through LDS (ordered by wg_reduce's
            // barrier); the trailing workgroups read the pivot column's rows >= k
#pragma unroll
            for (int e = 0; e < EPT; ++e)
                if (tid + WG_T * e == k) s_ck = cj[e];
            double2 u[EPT];
#pragma unroll
            for (int e = 0; e < EPT; ++e) {
                const int i = tid + WG_T * e;
                u[e] = own ? cj[e] : ((i > k && i < m) ? ld16(rW, cp * m + i) : c_zero());
            }
            const double2 alpha_g = own ? c_zero() : ld16(rW, cp * m + k);
            double r1[3] = {0.0, 0.0, 0.0};
#pragma unroll
            for (int e = 0; e < EPT; ++e) {
                const int i = tid + WG_T * e;
                if (i > k && i < m) {
                    const double2 v = u[e], w = own ? c_zero() : cj[e];
                    r1[0] += c_abs2(v);
                    r1[1] += v.x * w.x + v.y * w.y;
                    r1[2] += v.x * w.y - v.y * w.x;
                }
            }
            wg_reduce<3>(r1, red[0]);
            const Refl R = make_refl(own ? s_ck : alpha_g, r1[0]);
            if (own) {
                if (tid == 0) { a.tau[k] = R.tau; a.scale[k] = R.scale; a.beta[k] = R.beta; }
                done = true;
            } else {
                const double2 ck = s_ck;
                const double2 sv = c_add(ck, c_cmul(R.scale, make_double2(r1[1], r1[2])));
                const double2 ct = c_cmul(R.tau, sv);
                const double2 f = c_mul(ct, R.scale);  // c_i -= ct v_i = f x_i for i > k
                double r2[1] = {0.0};
#pragma unroll
                for (int e = 0; e < EPT; ++e) {
                    const int i = tid + WG_T * e;
                    if (i > k && i < m) {
                        const double2 ci = c_sub(cj[e], c_mul(f, u[e]));
                        cj[e] = ci;
                        st16(rW, g * m + i, ci);
                        r2[0] += c_abs2(ci);
                    } else if (i == k) {
                        cj[e] = c_sub(ck, ct);
                        st16(rW, g * m + k, cj[e]);
                    }
                }
                if (a.pivot) {
                    wg_reduce<1>(r2, red[1]);
                    if (tid == 0)
                        __hip_atomic_store((gu64*)(nout + g), (unsigned long long)__double_as_longlong(r2[0]),
                                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                }
            }
        }
        // ---- grid barrier
        ++epoch;
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        if (tid == 0) {
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            __hip_atomic_fetch_add((gu32*)q.bar, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        if (tid < 64) {
            const unsigned target = G * epoch;
            unsigned spins = 0;
            bool ok = true;
            while (__hip_atomic_load((gu32*)q.bar, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < target) {
                __builtin_amdgcn_s_sleep(1);
                if (++spins > q.spin_limit) { ok = false; break; }
            }
            if (tid == 0 && !ok) {
                s_abort = 1;
                __hip_atomic_store((gu32*)q.err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
        }
        __syncthreads();
        if (s_abort) return;
    }
    // the final permutation where the launch path leaves it (the buffer of parity rank & 1)
    if (g == 0)
        for (int j = tid; j < n; j += WG_T) a.perm[(size_t)(k & 1) * n + j] = s_perm[j];
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

std::atomic<int> g_jac_fallbacks{0};  // persistent Jacobi launches rerun per round (barrier timeout)
std::atomic<int> g_qr_fallbacks{0};   // persistent QRCP launches rerun one launch per step (barrier timeout)

// scratch per (device, stream): a factorization's kernels stay queued after the call returns (pqd_ptg_qr without
// pivoting does not synchronise), so a call on another stream or device must not reuse the same buffer.
// Calls are serialised by g_mu; the buffer of a stream grows (after synchronising that stream) and is kept. At most
// SCR_KEEP buffers are kept: past that the least recently used one is freed after synchronising its device (its stream
// handle may be gone by then), so a caller cycling through many streams does not accumulate buffers.
std::mutex g_mu;
struct Scratch {
    void* p = nullptr;
    size_t bytes = 0;
    unsigned long long used = 0;
};
std::map<std::pair<int, hipStream_t>, Scratch> g_scr;
unsigned long long g_scr_tick = 0;
constexpr size_t SCR_KEEP = 8;
hipError_t scratch(hipStream_t s, size_t bytes, void** out) {
    int dev = 0;
    hipError_t e = hipGetDevice(&dev);
    if (e != hipSuccess) return e;
    const auto key = std::make_pair(dev, s);
    Scratch& sc = g_scr[key];
    sc.used = ++g_scr_tick;
    if (g_scr.size() > SCR_KEEP) {
        auto lru = g_scr.end();
        for (auto it = g_scr.begin(); it != g_scr.end(); ++it)
            if (it->first != key && (lru == g_scr.end() || it->second.used < lru->second.used)) lru = it;
        if (lru != g_scr.end()) {
            if (lru->second.p) {
                if ((e = hipSetDevice(lru->first.first)) != hipSuccess) return e;
                e = hipDeviceSynchronize();
                if (e == hipSuccess) e = hipFree(lru->second.p);
                const hipError_t e2 = hipSetDevice(dev);
                if (e != hipSuccess) return e;
                if (e2 != hipSuccess) return e2;
            }
            g_scr.erase(lru);
        }
    }
    if (bytes > sc.bytes) {
        if (sc.p) {
            e = hipStreamSynchronize(s);
            if (e != hipSuccess) return e;
            e = hipFree(sc.p);
            if (e != hipSuccess) return e;
            sc.p = nullptr;
        }
        e = hipMalloc(&sc.p, bytes);
        if (e != hipSuccess) { sc.bytes = 0; return e; }
        sc.bytes = bytes;
    }
    *out = sc.p;
    return hipSuccess;
}
// the current device (function attributes and occupancy answers are per device)
int cur_dev() {
    int d = 0;
    return hipGetDevice(&d) == hipSuccess && d >= 0 && d < 64 ? d : 0;
}
inline size_t al(size_t x) { return (x + 255) & ~(size_t)255; }

unsigned long long g_attr_done = 0;  // bit d: the attributes are set on device d
hipError_t small_attrs() {
    const int dev = cur_dev();
    if (g_attr_done >> dev & 1ull) return hipSuccess;
    const int lds = QS_MAX * (int)sizeof(double2);
    hipError_t e = hipSuccess;
    for (const void* f : {(const void*)qr_small_kernel<0>, (const void*)qr_small_kernel<1>,
                          (const void*)qr_small_kernel<2>, (const void*)qr_small_kernel<4>,
                          (const void*)qr_small_kernel<8>}) {
        e = hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, lds);
        if (e != hipSuccess) return e;
    }
    e = hipFuncSetAttribute((const void*)jac_small_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, lds);
    if (e != hipSuccess) return e;
    g_attr_done |= 1ull << dev;
    return hipSuccess;
}

// PQD_PTG_SMALL=0: every factorization on the multi-workgroup kernels (A/B and tests of both paths)
bool small_ok() {
    const char* e = getenv("PQD_PTG_SMALL");
    return !(e && atoi(e) == 0);
}
int env_int(const char* name, int dflt) {
    const char* e = getenv(name);
    return (e && *e) ? atoi(e) : dflt;
}

// registers per thread of the workgroup-per-column kernels: the smallest EPT with 256 * EPT >= m (0: too tall)
int wg_ept(int m) {
    for (int e : {1, 2, 4, 8, 16})
        if (WG_T * e >= m) return e;
    return 0;
}
void launch_step2_wg(int ept, const QRArgs& a, int k, int grid, hipStream_t s) {
    switch (ept) {
        case 1: hipLaunchKernelGGL(qr_step2_wg_kernel<1>, dim3(grid), dim3(WG_T), 0, s, a, k); break;
        case 2: hipLaunchKernelGGL(qr_step2_wg_kernel<2>, dim3(grid), dim3(WG_T), 0, s, a, k); break;
        case 4: hipLaunchKernelGGL(qr_step2_wg_kernel<4>, dim3(grid), dim3(WG_T), 0, s, a, k); break;
        case 8: hipLaunchKernelGGL(qr_step2_wg_kernel<8>, dim3(grid), dim3(WG_T), 0, s, a, k); break;
        default: hipLaunchKernelGGL(qr_step2_wg_kernel<16>, dim3(grid), dim3(WG_T), 0, s, a, k); break;
    }
}
void launch_step_wg(int ept, const QRArgs& a, int k, int grid, hipStream_t s) {
    switch (ept) {
        case 1: hipLaunchKernelGGL(qr_step_wg_kernel<1>, dim3(grid), dim3(WG_T), 0, s, a, k); break;
        case 2: hipLaunchKernelGGL(qr_step_wg_kernel<2>, dim3(grid), dim3(WG_T), 0, s, a, k); break;
        case 4: hipLaunchKernelGGL(qr_step_wg_kernel<4>, dim3(grid), dim3(WG_T), 0, s, a, k); break;
        case 8: hipLaunchKernelGGL(qr_step_wg_kernel<8>, dim3(grid), dim3(WG_T), 0, s, a, k); break;
        default: hipLaunchKernelGGL(qr_step_wg_kernel<16>, dim3(grid), dim3(WG_T), 0, s, a, k); break;
    }
}

// the persistent QRCP kernel for ept, and whether its n workgroups (256 threads, n ints of LDS) can all be resident
const void* qrcp_persist_fn(int ept) {
    switch (ept) {
        case 1: return (const void*)qrcp_persist_kernel<1>;
        case 2: return (const void*)qrcp_persist_kernel<2>;
        case 4: return (const void*)qrcp_persist_kernel<4>;
        case 8: return (const void*)qrcp_persist_kernel<8>;
        default: return (const void*)qrcp_persist_kernel<16>;
    }
}
bool qrcp_persist_fits(int ept, int n) {
    static int cus_d[64] = {0};
    static int per_cu_d[64][17] = {{0}};
    const int dev = cur_dev();
    int& cus = cus_d[dev];
    int* per_cu = per_cu_d[dev];
    if (!cus) {
        if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
            return false;
    }
    if (!per_cu[ept]) {
        int nb = 0;
        // LDS: the permutation (n ints) at the largest n taken (4096), so the answer holds for every n below it
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, qrcp_persist_fn(ept), WG_T, 4096 * sizeof(int)) !=
            hipSuccess)
            return false;
        per_cu[ept] = nb > 0 ? nb : -1;
    }
    return n <= 4096 && per_cu[ept] > 0 && (long long)per_cu[ept] * cus >= n;
}

// column steps k .. k_end-1 of a (updating logical columns < a.n): pairs on plain QRs, workgroup-per-column kernels
// when the column fits in registers (ept > 0), else the wave-per-column kernels
void column_steps(const QRArgs& a, int k, int k_end, bool pairs, int ept, hipStream_t s) {
    const int wpb = 4;
    while (k < k_end) {
        if (pairs && k + 1 < k_end) {
            if (ept) {
                launch_step2_wg(ept, a, k, std::max(2, a.n - k), s);
            } else {
                const int nw = 2 + std::max(0, a.n - k - 2);
                hipLaunchKernelGGL(qr_step2_kernel, dim3((nw + wpb - 1) / wpb), dim3(64 * wpb), 0, s, a, k);
            }
            k += 2;
        } else {
            if (ept) {
                launch_step_wg(ept, a, k, std::max(1, a.n - k), s);
            } else {
                const int nw = std::max(1, a.n - k - 1);
                hipLaunchKernelGGL(qr_step_kernel, dim3((nw + wpb - 1) / wpb), dim3(64 * wpb), 0, s, a, k);
            }
            k += 1;
        }
    }
}

// blocked-update scratch: Vc (QB x m), S and T (QB x QB), Yp (chunks x n x QB), Zt (n x QB)
constexpr int QB = VHA_NB;
struct BlockBufs {
    double2 *Vc, *S, *T, *Yp, *Zt;
};
size_t block_bytes(int m, int n) {
    const size_t nch = (size_t)(m + VHA_RC - 1) / VHA_RC;
    return al((size_t)QB * m * 16) + 2 * al((size_t)QB * QB * 16) + al(nch * n * QB * 16) + al((size_t)n * QB * 16);
}
BlockBufs carve_block(char*& c, int m, int n) {
    BlockBufs b;
    const size_t nch = (size_t)(m + VHA_RC - 1) / VHA_RC;
    b.Vc = reinterpret_cast<double2*>(c); c += al((size_t)QB * m * 16);
    b.S = reinterpret_cast<double2*>(c); c += al((size_t)QB * QB * 16);
    b.T = reinterpret_cast<double2*>(c); c += al((size_t)QB * QB * 16);
    b.Yp = reinterpret_cast<double2*>(c); c += al(nch * n * QB * 16);
    b.Zt = reinterpret_cast<double2*>(c); c += al((size_t)n * QB * 16);
    return b;
}

// V and S = V^H V (strict upper part) of reflectors i0 .. i0+nb-1 (X columns perm[i], perm == nullptr: i)
void block_vt(const QRArgs& a, const int* perm, int i0, int nb, const BlockBufs& b, hipStream_t s) {
    const int wpb = 4;
    hipLaunchKernelGGL(refl_block_kernel, dim3((nb + wpb - 1) / wpb), dim3(64 * wpb), 0, s, a.X, a.m, perm, i0, nb,
                       a.scale, b.Vc);
    if (nb > 1)
        hipLaunchKernelGGL(panel_gram_kernel, dim3((nb * nb + wpb - 1) / wpb), dim3(64 * wpb), 0, s, b.Vc, a.m - i0,
                           nb, b.S);
}

// A <- A - V op(T) V^H A on ncol columns of length mm = m - i0 (A column j at A0 + j * lda)
void block_apply(double2* A0, int lda, int ncol, int mm, int i0, int nb, int herm, const double2* tau,
                 const BlockBufs& b, hipStream_t s) {
    if (ncol <= 0) return;
    const int nch = (mm + VHA_RC - 1) / VHA_RC;
    hipLaunchKernelGGL(vha_kernel, dim3((ncol + VHA_J - 1) / VHA_J, nch), dim3(256), 0, s, A0, lda, ncol, b.Vc, mm,
                       nb, b.Yp);
    hipLaunchKernelGGL(zt_kernel, dim3(ncol), dim3(64), 0, s, b.Yp, nch, ncol, nb, b.S, tau, i0, herm, b.Zt);
    hipLaunchKernelGGL(rank_update_kernel, dim3((mm + 255) / 256, ncol), dim3(256), 0, s, A0, lda, mm, b.Vc, nb, b.Zt);
}

}  // namespace

// Switches (read per call, for A/B runs and tests): PQD_PTG_SMALL=0 (no single-workgroup kernel), PQD_PTG_WG=0 (wave-
// per-column step kernels), PQD_PTG_PAIR=0 (one reflector per launch), PQD_PTG_BLOCKED=1 (blocked factorization of
// plain QRs: panels of 32 columns, trailing update V T^H V^H A), PQD_PTG_QFB=0 (Q from the per-wave reflector kernel
// instead of blocks of 32 reflectors).
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
    // tol >= 0: absolute; tol < 0: relative to the largest column norm of W (found on the device, no host pass)
    const double tol2 = pivot && tol >= 0.0 ? tol * tol : -1.0;
    const bool unperm = pivot == 2;  // R returned in the original column order (R P^T)
    const double rel2 = pivot && tol < 0.0 ? tol * tol : 0.0;
    void* base = nullptr;
    const bool small = small_ok() && (size_t)m * n <= (size_t)QS_MAX && n <= 256;
    const int ept = env_int("PQD_PTG_WG", 1) ? wg_ept(m) : 0;
    // blocked factorization: PQD_PTG_BLOCKED=1 always, 0 never, default from 10^6 elements (the size where the
    // per-step trailing traffic of the column kernels starts to exceed the panels' extra launches; profiles/r04/ptgen)
    const int blk_env = env_int("PQD_PTG_BLOCKED", -1);
    // QRs whose columns fit in registers: every step in one persistent launch (PQD_PTG_QPERSIST=1: pivoted QRs, 2:
    // pivoted and plain QRs; default 0: one launch per step). A plain QR then takes one reflector per step (no pairs).
    // Measured slower than the launches (profiles/r04/ptgen/qpersist/: QRCP phases +8-13%, plain QRs +40%): each step
    // is three dependent coherent round trips (the norm scan, the barrier, the pivot column), where back-to-back
    // launches read the same data from L2
    const int qp_env = env_int("PQD_PTG_QPERSIST", 0);
    const bool qpersist = !small && ept > 0 && kmax >= 2 && (pivot ? qp_env >= 1 : (qp_env >= 2 && blk_env != 1)) &&
                          qrcp_persist_fits(ept, n);
    const bool pairs = !pivot && !small && !qpersist && kmax >= 2 && env_int("PQD_PTG_PAIR", 1) != 0;
    const bool blocked = !pivot && !small && !qpersist && m >= n && n > QB &&
                         (blk_env == 1 || (blk_env < 0 && (size_t)m * n >= (size_t)1000000));
    const bool qfb = !small && env_int("PQD_PTG_QFB", 1) != 0;
    const bool sepx = pairs || blocked;  // reflector columns in their own buffer X
    const size_t b_tau = al(kmax * sizeof(double2)), b_beta = al(kmax * sizeof(double)),
                 b_perm = al(2 * (size_t)n * sizeof(int)), b_norm = al(2 * (size_t)n * sizeof(double)),
                 b_ctrl = al(64 * sizeof(int)), b_x = sepx ? al((size_t)m * kmax * sizeof(double2)) : 0,
                 b_blk = (blocked || qfb) ? block_bytes(m, n) : 0,
                 b_bak = qpersist ? al((size_t)m * n * sizeof(double2)) : 0;
    PCHK(scratch(s, 2 * b_tau + b_beta + b_perm + b_norm + b_ctrl + b_x + b_blk + b_bak, &base));
    char* c = static_cast<char*>(base);
    QRArgs a;
    a.W = W; a.m = m; a.n = n; a.kmax = kmax; a.pivot = pivot ? 1 : 0; a.tol2 = tol2; a.rel2 = rel2;
    a.tau = reinterpret_cast<double2*>(c); c += b_tau;
    a.scale = reinterpret_cast<double2*>(c); c += b_tau;
    a.beta = reinterpret_cast<double*>(c); c += b_beta;
    a.perm = reinterpret_cast<int*>(c); c += b_perm;
    a.norms = reinterpret_cast<double*>(c); c += b_norm;
    a.ctrl = reinterpret_cast<int*>(c); c += b_ctrl;
    a.X = sepx ? reinterpret_cast<double2*>(c) : W;
    c += b_x;
    BlockBufs bb{};
    if (b_blk) bb = carve_block(c, m, n);
    double2* Wbak = b_bak ? reinterpret_cast<double2*>(c) : nullptr;  // after the blocks: carve_block advanced c
    c += b_bak;
    int* d_rank = a.ctrl + 8;
    a.thr = reinterpret_cast<double*>(a.ctrl + 16);
    if (small) {
        PCHK(small_attrs());
        const size_t lds = (size_t)m * n * sizeof(double2);
        const int diag = env_int("PQD_PTG_DIAG", 0);
        const int qe = m <= 64 ? 1 : m <= 128 ? 2 : m <= 256 ? 4 : m <= 512 ? 8 : 0;
#define PQD_QS(QEV) hipLaunchKernelGGL(qr_small_kernel<QEV>, dim3(1), dim3(QS_THREADS), lds, s, W, m, n, a.pivot, \
                                       tol2, rel2, Q, R, perm_out, d_rank, unperm ? 1 : 0, diag)
        switch (qe) {
            case 1: PQD_QS(1); break;
            case 2: PQD_QS(2); break;
            case 4: PQD_QS(4); break;
            case 8: PQD_QS(8); break;
            default: PQD_QS(0); break;
        }
#undef PQD_QS
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
    if (blocked) {
        for (int k0 = 0; k0 < kmax; k0 += QB) {
            const int nb = std::min(QB, kmax - k0);
            QRArgs ap = a;
            ap.n = k0 + nb;  // the panel's column steps update the panel only
            column_steps(ap, k0, k0 + nb, true, ept, s);
            if (k0 + nb < n) {
                block_vt(a, nullptr, k0, nb, bb, s);
                block_apply(W + (size_t)(k0 + nb) * m + k0, m, n - k0 - nb, m - k0, k0, nb, 1, a.tau, bb, s);
            }
        }
    } else if (qpersist) {
        QRPersist q;
        q.bar = reinterpret_cast<unsigned*>(a.ctrl + 32);
        q.err = reinterpret_cast<unsigned*>(a.ctrl + 40);
        q.spin_limit = (unsigned)env_int("PQD_PTG_QSPIN", 1 << 22);  // polls per barrier wait (tests: 1)
        PCHK(hipMemsetAsync(a.ctrl + 32, 0, 16 * sizeof(int), s));
        PCHK(hipMemcpyAsync(Wbak, W, (size_t)m * n * sizeof(double2), hipMemcpyDeviceToDevice, s));
        const size_t lds = (size_t)n * sizeof(int);
        switch (ept) {
            case 1: hipLaunchKernelGGL(qrcp_persist_kernel<1>, dim3(n), dim3(WG_T), lds, s, a, q); break;
            case 2: hipLaunchKernelGGL(qrcp_persist_kernel<2>, dim3(n), dim3(WG_T), lds, s, a, q); break;
            case 4: hipLaunchKernelGGL(qrcp_persist_kernel<4>, dim3(n), dim3(WG_T), lds, s, a, q); break;
            case 8: hipLaunchKernelGGL(qrcp_persist_kernel<8>, dim3(n), dim3(WG_T), lds, s, a, q); break;
            default: hipLaunchKernelGGL(qrcp_persist_kernel<16>, dim3(n), dim3(WG_T), lds, s, a, q); break;
        }
        PCHK(hipGetLastError());
        unsigned e = 0;
        PCHK(hipMemcpyAsync(&e, q.err, sizeof(unsigned), hipMemcpyDeviceToHost, s));
        PCHK(hipStreamSynchronize(s));
        if (e) {  // a barrier wait timed out: every workgroup has left; start over from the copy, one launch per step
            PCHK(hipMemcpyAsync(W, Wbak, (size_t)m * n * sizeof(double2), hipMemcpyDeviceToDevice, s));
            hipLaunchKernelGGL(qr_init_kernel, dim3((n + wpb - 1) / wpb), dim3(64 * wpb), 0, s, a);
            column_steps(a, 0, kmax, false, ept, s);
            g_qr_fallbacks.fetch_add(1);
        }
    } else {
        column_steps(a, 0, kmax, pairs, ept, s);
    }
    PCHK(hipGetLastError());
    int rank = kmax;
    if (pivot) {  // the stopping step decides the rank: one host round trip
        PCHK(hipMemcpyAsync(&rank, a.ctrl, sizeof(int), hipMemcpyDeviceToHost, s));
        PCHK(hipStreamSynchronize(s));
    }
    const int tot = std::max(rank * n, n);
    hipLaunchKernelGGL(qr_extract_r_kernel, dim3((tot + 255) / 256), dim3(256), 0, s, a, rank, R, perm_out,
                       unperm ? 1 : 0);
    if (rank > 0) {
        const size_t mq = (size_t)m * rank;
        hipLaunchKernelGGL(qf_init_kernel, dim3((unsigned)((mq + 255) / 256)), dim3(256), 0, s, Q, m, rank);
        if (qfb && rank > 2 * QB) {
            // Q = H_0 ... H_{rank-1} [I; 0], blocks of QB reflectors from the last: Q[i0:, i0:] <- (I - V T V^H) Q[i0:, i0:]
            const int* pf = a.pivot ? perm_out : nullptr;
            for (int i0 = ((rank - 1) / QB) * QB; i0 >= 0; i0 -= QB) {
                const int nb = std::min(QB, rank - i0);
                block_vt(a, pf, i0, nb, bb, s);
                block_apply(Q + (size_t)i0 * m + i0, m, rank - i0, m - i0, i0, nb, 0, a.tau, bb, s);
            }
        } else {
            for (int i1 = rank; i1 > 0; i1 -= QF_RB) {
                const int i0 = std::max(0, i1 - QF_RB);
                const int ncol = rank - i0;
                hipLaunchKernelGGL(qf_apply_kernel, dim3((ncol + wpb - 1) / wpb), dim3(64 * wpb), 0, s, a, rank,
                                   perm_out, Q, i0, i1);
            }
        }
    }
    PCHK(hipGetLastError());
    *rank_out = rank;
    return PQD_OK;
}

extern "C" int pqd_ptg_counters(int32_t* jacobi_fallbacks) {
    if (!jacobi_fallbacks) return perr(PQD_ERR_ARG, "pqd_ptg_counters: NULL argument");
    *jacobi_fallbacks = g_jac_fallbacks.load();
    return PQD_OK;
}

extern "C" int pqd_ptg_qr_counters(int32_t* qrcp_fallbacks) {
    if (!qrcp_fallbacks) return perr(PQD_ERR_ARG, "pqd_ptg_qr_counters: NULL argument");
    *qrcp_fallbacks = g_qr_fallbacks.load();
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
    // counters, then a copy of X: a persistent launch whose grid barrier times out (workgroups not co-resident, e.g.
    // under contention from other work on the device) is rerun from this copy with one launch per round
    const size_t b_cnt = al((64 + 200) * sizeof(int));
    PCHK(scratch(s, b_cnt + al((size_t)n * n * sizeof(double2)), &base));
    int* cnt = static_cast<int*>(base);
    double2* Xbak = reinterpret_cast<double2*>(static_cast<char*>(base) + b_cnt);
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
        const int epl = n <= 64 ? 1 : n <= 128 ? 2 : n <= 256 ? 4 : n <= 512 ? 8 : n <= 1024 ? 16 : 0;
        bool persist = epl && env_int("PQD_PTG_JPERSIST", 1) != 0 && max_sweeps <= 200;
        if (persist) {
            PCHK(hipMemcpyAsync(Xbak, X, nv * sizeof(double2), hipMemcpyDeviceToDevice, s));
            JacPersist q;
            q.bar = reinterpret_cast<unsigned*>(cnt + 16);
            q.err = reinterpret_cast<unsigned*>(cnt + 32);
            q.sweeps = cnt + 48;
            q.cnt = cnt + 64;
            q.max_sweeps = max_sweeps;
            q.spin_limit = (unsigned)env_int("PQD_PTG_JSPIN", 1 << 22);  // polls per barrier wait (tests: 1)
            PCHK(hipMemsetAsync(cnt + 16, 0, (64 + 200) * sizeof(int) - 16 * sizeof(int), s));
            const dim3 g((npair + wpb - 1) / wpb), b(64 * wpb);
            int nblk = (n + JB - 1) / JB;
            nblk += nblk & 1;  // even: the round-robin pairs every block each round (a block past n is all dummies)
            const size_t lds_blk = (size_t)4 * JB * n * sizeof(double2);
            constexpr int JB_LDS_MAX = 160 * 1024 - 256;  // the kernel's own static LDS words come on top
            // PQD_PTG_JBLOCK=0: the column-pair kernel (one grid barrier per tournament round of single columns)
            const bool jblock = env_int("PQD_PTG_JBLOCK", 1) != 0 && epl <= 8 && lds_blk <= (size_t)JB_LDS_MAX &&
                                nblk >= 2;
            if (jblock) {
                static unsigned long long attr = 0;  // bit d: set on device d
                const int dev = cur_dev();
                if (!(attr >> dev & 1ull)) {
                    for (const void* f : {(const void*)jac_block_kernel<1>, (const void*)jac_block_kernel<2>,
                                          (const void*)jac_block_kernel<4>, (const void*)jac_block_kernel<8>})
                        PCHK(hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, JB_LDS_MAX));
                    attr |= 1ull << dev;
                }
                const dim3 gb(nblk / 2);
                switch (epl) {
                    case 1: hipLaunchKernelGGL(jac_block_kernel<1>, gb, b, lds_blk, s, a, q, nblk); break;
                    case 2: hipLaunchKernelGGL(jac_block_kernel<2>, gb, b, lds_blk, s, a, q, nblk); break;
                    case 4: hipLaunchKernelGGL(jac_block_kernel<4>, gb, b, lds_blk, s, a, q, nblk); break;
                    default: hipLaunchKernelGGL(jac_block_kernel<8>, gb, b, lds_blk, s, a, q, nblk); break;
                }
            } else switch (epl) {
                case 1: hipLaunchKernelGGL(jac_persist_kernel<1>, g, b, 0, s, a, q); break;
                case 2: hipLaunchKernelGGL(jac_persist_kernel<2>, g, b, 0, s, a, q); break;
                case 4: hipLaunchKernelGGL(jac_persist_kernel<4>, g, b, 0, s, a, q); break;
                case 8: hipLaunchKernelGGL(jac_persist_kernel<8>, g, b, 0, s, a, q); break;
                default: hipLaunchKernelGGL(jac_persist_kernel<16>, g, b, 0, s, a, q); break;
            }
            PCHK(hipGetLastError());
            int h[2] = {0, 0};
            PCHK(hipMemcpyAsync(&h[0], q.sweeps, sizeof(int), hipMemcpyDeviceToHost, s));
            PCHK(hipMemcpyAsync(&h[1], q.err, sizeof(int), hipMemcpyDeviceToHost, s));
            PCHK(hipStreamSynchronize(s));
            if (h[1]) {  // a barrier wait timed out: every workgroup has left; start over from X, one launch per round
                PCHK(hipMemcpyAsync(X, Xbak, nv * sizeof(double2), hipMemcpyDeviceToDevice, s));
                hipLaunchKernelGGL(jac_init_kernel, dim3((unsigned)((nv + 255) / 256)), dim3(256), 0, s, V, n);
                persist = false;
                g_jac_fallbacks.fetch_add(1);
            } else {
                sweeps = h[0];
            }
        }
        if (!persist) {
            bool conv = false;
            for (; sweeps < max_sweeps;) {
                PCHK(hipMemsetAsync(cnt, 0, sizeof(int), s));
                for (int t = 0; t < a.nn - 1; ++t)
                    hipLaunchKernelGGL(jac_round_kernel, dim3((npair + wpb - 1) / wpb), dim3(64 * wpb), 0, s, a, t);
                PCHK(hipGetLastError());
                int h = 0;
                PCHK(hipMemcpyAsync(&h, cnt, sizeof(int), hipMemcpyDeviceToHost, s));
                PCHK(hipStreamSynchronize(s));
                ++sweeps;
                if (h == 0) { conv = true; break; }
            }
            if (!conv) sweeps = max_sweeps + 1;
        }
    }
    hipLaunchKernelGGL(jac_finish_kernel, dim3((n + 3) / 4), dim3(256), 0, s, X, n, sigma);
    PCHK(hipGetLastError());
    *sweeps_out = sweeps;
    return PQD_OK;
}
