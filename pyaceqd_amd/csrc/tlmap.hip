// tlmap.hip — time-local dynamical maps from cumulative ones, on the GPU:
//   out[0] = dm[0];  out[i] = dm[i] · pinv(dm[i-1], rcond)   for i = 1 .. n_maps-1
// restating calc_tl_dynmap_pseudo (reference pyaceqd/tools.py:446-484), whose pinv is numpy's
// (SVD, singular values <= rcond * max(s) dropped). The SVD here is a one-sided (Hestenes) Jacobi
// on the columns of dm[i-1]: A·V = W with orthogonal columns w_j = s_j u_j, so
//   pinv(A) = V diag(1/s_j^2) W^H   (s_j > rcond * max s, else 0),
// and out[i] = (dm[i] V) diag(1/s_j^2) W^H without forming U. One-sided Jacobi is accurate to
// eps relative in every singular value, so the rcond cut-off lands where LAPACK's does.
//
// One workgroup (one 64-lane wave, so every __syncthreads() is a single s_barrier) per map.
// A, V and the product stay in LDS (column-major, n <= 36 = N^2 at N = 6). Each Jacobi round
// rotates n/2 disjoint column pairs (round-robin tournament): lane k computes pair k's Gram
// entries, then all lanes apply the rotations element-wise.
#include "pqd_common.h"

namespace {

constexpr int TL_NMAX = 36;
constexpr int TL_LD = TL_NMAX + 1;
constexpr int TL_MAX_SWEEPS = 40;

// round-robin tournament: m players (m even), player m-1 fixed; round k, slot j
__device__ __forceinline__ void rr_pair(int m, int k, int j, int& p, int& q) {
    if (j == 0) { p = k; q = m - 1; return; }
    p = (k + j) % (m - 1);
    q = (k - j + (m - 1)) % (m - 1);
}

__global__ __launch_bounds__(64) void tl_dynmap_kernel(const double2* __restrict__ dm, int n, double rcond,
                                                       double2* __restrict__ out) {
    __shared__ double2 A[TL_NMAX * TL_LD], V[TL_NMAX * TL_LD], B[TL_NMAX * TL_LD];
    __shared__ double rc[TL_NMAX / 2 + 1], rs[TL_NMAX / 2 + 1], wsc[TL_NMAX];
    __shared__ double2 rph[TL_NMAX / 2 + 1];
    __shared__ int rp[TL_NMAX / 2 + 1], rq[TL_NMAX / 2 + 1];
    __shared__ int rotated;
    const int lane = threadIdx.x;
    const int i = blockIdx.x + 1;  // out[0] = dm[0] is copied by the host
    const size_t m2 = (size_t)n * n;
    const double2* __restrict__ Ai = dm + (size_t)(i - 1) * m2;  // row-major dm[i-1]
    const double2* __restrict__ Ei = dm + (size_t)i * m2;
    for (int e = lane; e < n * n; e += 64) {
        const int r = e / n, c = e % n;
        A[c * TL_LD + r] = Ai[e];
        V[c * TL_LD + r] = (r == c) ? make_double2(1.0, 0.0) : c_zero();
    }
    const int m = n + (n & 1);  // odd n: player n is a dummy (its pairs are skipped)
    const int half = m / 2;
    const double tol = 2.220446049250313e-16 * n;
    __syncthreads();
    for (int sweep = 0; sweep < TL_MAX_SWEEPS; ++sweep) {
        if (lane == 0) rotated = 0;
        __syncthreads();
        for (int k = 0; k < m - 1; ++k) {
            if (lane < half) {
                int p, q;
                rr_pair(m, k, lane, p, q);
                if (p > q) { const int t = p; p = q; q = t; }
                double c = 1.0, s = 0.0;
                double2 ph = make_double2(1.0, 0.0);
                bool act = false;
                if (q < n) {
                    double al = 0.0, be = 0.0;
                    double2 g = c_zero();
                    const double2* ap = A + p * TL_LD;
                    const double2* aq = A + q * TL_LD;
                    for (int r = 0; r < n; ++r) {
                        const double2 x = ap[r], y = aq[r];
                        al = fma(x.x, x.x, fma(x.y, x.y, al));
                        be = fma(y.x, y.x, fma(y.y, y.y, be));
                        c_fma(g, c_conj(x), y);
                    }
                    const double ga = hypot(g.x, g.y);
                    if (ga > tol * sqrt(al) * sqrt(be) && ga > 0.0) {
                        const double zeta = (be - al) / (2.0 * ga);
                        const double t = (zeta >= 0.0 ? 1.0 : -1.0) / (fabs(zeta) + sqrt(1.0 + zeta * zeta));
                        c = 1.0 / sqrt(1.0 + t * t);
                        s = c * t;
                        ph = make_double2(g.x / ga, -g.y / ga);  // e^{-i phi}, phi = arg(a_p^H a_q)
                        act = true;
                        rotated = 1;
                    }
                }
                rp[lane] = p; rq[lane] = q; rc[lane] = c; rs[lane] = s; rph[lane] = ph;
                if (!act) rq[lane] = -1;
            }
            __syncthreads();
            // a_p' = c a_p - s e^{-i phi} a_q ;  a_q' = s a_p + c e^{-i phi} a_q   (same on V)
            for (int e = lane; e < half * n; e += 64) {
                const int j = e / n, r = e % n;
                const int q = rq[j];
                if (q < 0) continue;
                const int p = rp[j];
                const double c = rc[j], s = rs[j];
                const double2 ph = rph[j];
                double2 x = A[p * TL_LD + r], y = c_mul(ph, A[q * TL_LD + r]);
                A[p * TL_LD + r] = c_sub(c_scale(x, c), c_scale(y, s));
                A[q * TL_LD + r] = c_add(c_scale(x, s), c_scale(y, c));
                x = V[p * TL_LD + r]; y = c_mul(ph, V[q * TL_LD + r]);
                V[p * TL_LD + r] = c_sub(c_scale(x, c), c_scale(y, s));
                V[q * TL_LD + r] = c_add(c_scale(x, s), c_scale(y, c));
            }
            __syncthreads();
        }
        if (!rotated) break;
        __syncthreads();
    }
    // s_j^2 = |w_j|^2; weights 1/s_j^2 above the cut-off (numpy: s > rcond * max(s))
    if (lane < n) {
        double al = 0.0;
        for (int r = 0; r < n; ++r) {
            const double2 x = A[lane * TL_LD + r];
            al = fma(x.x, x.x, fma(x.y, x.y, al));
        }
        wsc[lane] = al;
    }
    __syncthreads();
    double smax2 = 0.0;
    for (int j = 0; j < n; ++j) smax2 = fmax(smax2, wsc[j]);
    const double smax = sqrt(smax2);
    __syncthreads();
    if (lane < n) {
        const double sj = sqrt(wsc[lane]);
        wsc[lane] = (sj > rcond * smax) ? 1.0 / wsc[lane] : 0.0;
    }
    __syncthreads();
    // B = dm[i] V diag(w)
    for (int e = lane; e < n * n; e += 64) {
        const int r = e / n, j = e % n;
        double2 acc = c_zero();
        for (int k = 0; k < n; ++k) c_fma(acc, Ei[r * n + k], V[j * TL_LD + k]);
        B[j * TL_LD + r] = c_scale(acc, wsc[j]);
    }
    __syncthreads();
    // out[i] = B W^H,  W^H[j][c] = conj(A[c][j])
    double2* __restrict__ o = out + (size_t)i * m2;
    for (int e = lane; e < n * n; e += 64) {
        const int r = e / n, c = e % n;
        double2 acc = c_zero();
        for (int j = 0; j < n; ++j) c_fma(acc, B[j * TL_LD + r], c_conj(A[j * TL_LD + c]));
        o[e] = acc;
    }
}

}  // namespace

int tl_dynmap_nmax() { return TL_NMAX; }

hipError_t launch_tl_dynmap(const double2* dm, int n_maps, int n, double rcond, double2* out, hipStream_t s) {
    if (n_maps > 1)
        hipLaunchKernelGGL(tl_dynmap_kernel, dim3(n_maps - 1), dim3(64), 0, s, dm, n, rcond, out);
    return hipGetLastError();
}
