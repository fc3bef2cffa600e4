// free_prop.hip — batched free propagators M(n,h) = prod_j exp(L(t_j) w), one workgroup per matrix.
//
// Replaces the free-propagator construction ACE performs for every step from the param lines
// add_Hamiltonian / add_Pulse (+h.c.) / add_Lindblad (general_system.py:241-279, symmetric Trotter
// :234) and that ACEutils exposes as FreePropagator.update(t, dt).M (general_system.py:324-327).
// All trajectories at the same absolute step share these matrices, so they are built once per
// step here (2 * n_steps independent N2 x N2 expm's: 16x16 at N=4, 36x36 at N=6).
//
// Algorithm per matrix (the oracle's or_expm, with the degree cut to the precision): A = L(t) w,
// s = max(0, e) with frexp(||A||_1 / 0.5) = m 2^e, Taylor polynomial by Horner on A 2^-s of the smallest
// degree <= 18 whose remainder bound is below 2^-56 (the oracle always uses 18), then s squarings.
// The N2 x N2 operands live in LDS; each of the 256 threads owns ceil(N2^2/256) output entries.
#include "pqd_common.h"
#include <algorithm>
#include <cstdlib>

// blocks per launch: 256-thread blocks keep the dispatch grid (work-items, 32 bits) below 2^32; larger
// batches loop (grid-stride)
constexpr long long FP_MAX_BLOCKS = 1LL << 22;

namespace {

__device__ __forceinline__ double2 sample_ch(const FreePropSys& p, int c, double t) {
    const double2* f = p.samples + (size_t)c * p.n_samples;
    const int ns = p.n_samples;
    const double u = (t - p.s_t0) / p.s_dt;
    if (!(u > 0.0)) return f[0];
    if (u >= (double)(ns - 1)) return f[ns - 1];
    const int k = (int)floor(u);
    const double w = u - (double)k;
    const double2 a = f[k], b = f[k + 1];
    return make_double2(a.x + w * (b.x - a.x), a.y + w * (b.y - a.y));
}

// a half step is idle when every channel sample at every sub-step midpoint is exactly zero: then
// L(t) = L0 + 0 S + 0 T is bitwise L0, and its propagator is the system's Midle (built by the idle pass with the
// same code and zero samples), so it is copied instead of recomputed. Pulses are localised: the TLS scans
//  have zero drive after ~135 ps of a 100/1000 ps window.
__device__ __forceinline__ bool idle_half_step(const FreePropSys& sy, double t0, double w, int nsub) {
    for (int j = 0; j < nsub; ++j) {
        const double t = t0 + (j + 0.5) * w;
        for (int c = 0; c < sy.n_chan && c < 4; ++c) {
            const double2 f = sample_ch(sy, c, t);
            if (f.x != 0.0 || f.y != 0.0) return false;
        }
    }
    return true;
}

// 1 / mm for the Horner steps of the matrix-core builders: a wave-uniform index reads it with a scalar load, where a
// division is a dozen FP64 VALU instructions per element (and FP64 VALU does not co-issue with the matrix cores).
// x * (1 / mm) may differ from x / mm in the last place; parity vs the oracle is at 1e-12 relative
__constant__ double k_rinv[19] = {0.0, 1.0, 1.0 / 2, 1.0 / 3, 1.0 / 4, 1.0 / 5, 1.0 / 6, 1.0 / 7, 1.0 / 8, 1.0 / 9,
                                  1.0 / 10, 1.0 / 11, 1.0 / 12, 1.0 / 13, 1.0 / 14, 1.0 / 15, 1.0 / 16, 1.0 / 17, 1.0 / 18};

template <int N2>
__device__ __forceinline__ void lds_matmul(const double2* A, const double2* B, double2* C, int tid) {
    if constexpr (N2 == 36) {
        // 3 x 3 register blocks on 144 threads: one LDS read feeds 3 complex MACs instead of 1/2 (the 1x1 form is
        // LDS-bandwidth bound, ≈16 TF/s chip-wide); every element keeps the k = 0..N2-1 summation order
        if (tid < 144) {
            const int r0 = 3 * (tid / 12), c0 = 3 * (tid % 12);
            double2 acc[3][3];
#pragma unroll
            for (int r = 0; r < 3; ++r)
#pragma unroll
                for (int c = 0; c < 3; ++c) acc[r][c] = c_zero();
#pragma unroll 4
            for (int k = 0; k < N2; ++k) {
                double2 a[3], b[3];
#pragma unroll
                for (int r = 0; r < 3; ++r) a[r] = A[(r0 + r) * N2 + k];
#pragma unroll
                for (int c = 0; c < 3; ++c) b[c] = B[k * N2 + c0 + c];
#pragma unroll
                for (int r = 0; r < 3; ++r)
#pragma unroll
                    for (int c = 0; c < 3; ++c) c_fma(acc[r][c], a[r], b[c]);
            }
#pragma unroll
            for (int r = 0; r < 3; ++r)
#pragma unroll
                for (int c = 0; c < 3; ++c) C[(r0 + r) * N2 + c0 + c] = acc[r][c];
        }
        return;
    }
    for (int e = tid; e < N2 * N2; e += 256) {
        const int i = e / N2, j = e - i * N2;
        double2 acc = c_zero();
#pragma unroll 4
        for (int k = 0; k < N2; ++k) c_fma(acc, A[i * N2 + k], B[k * N2 + j]);
        C[e] = acc;
    }
}

template <int N2>
__global__ __launch_bounds__(256) void free_prop_kernel(FreePropParams p) {
    extern __shared__ __attribute__((aligned(16))) double2 smem[];
    double2* A = smem;
    double2* P = A + N2 * N2;
    double2* T = P + N2 * N2;
    double2* Acc = T + N2 * N2;
    __shared__ double colsum[N2];
    __shared__ int s_sh, s_deg;

    const int tid = threadIdx.x;
    const long long nblk = p.idle_pass ? (long long)p.n_sys : (long long)p.n_sys * 2 * p.n_steps;
    // grid-stride: the dispatch grid counts work-items in 32 bits, so a launch is capped (FP_MAX_BLOCKS)
    for (long long blk = blockIdx.x; blk < nblk; blk += gridDim.x) {
    const int si = p.idle_pass ? (int)blk : (int)(blk / (2 * p.n_steps));
    const int m = p.idle_pass ? 0 : (int)(blk - (long long)si * 2 * p.n_steps);
    const int n = m >> 1, h = m & 1;
    const FreePropSys sy = p.systems[si];
    const int nsub = p.n_sub > 0 ? p.n_sub : 1;
    const double w = 0.5 * p.dt / nsub;
    double2* out = p.idle_pass ? p.Midle + (size_t)si * N2 * N2 : p.M + ((size_t)si * 2 * p.n_steps + m) * N2 * N2;
    if (!p.idle_pass && p.win) {  // outside the pulse window: not stored (readers take Midle)
        const int2 wn = p.win[si];
        if (m < wn.x || m > wn.y) continue;
    }
    if (!p.idle_pass && p.Midle && idle_half_step(sy, p.ta + n * p.dt + h * 0.5 * p.dt, w, nsub)) {
        const double2* src = p.Midle + (size_t)si * N2 * N2;
        for (int e = tid; e < N2 * N2; e += 256) out[e] = src[e];
        continue;  // block-uniform: LDS untouched
    }

    for (int j = 0; j < nsub; ++j) {
        const double t = p.ta + n * p.dt + h * 0.5 * p.dt + (j + 0.5) * w;
        double2 f[4], fc[4];
#pragma unroll
        for (int c = 0; c < 4; ++c) {
            if (c < sy.n_chan) {
                f[c] = p.idle_pass ? c_zero() : sample_ch(sy, c, t);
                fc[c] = c_conj(f[c]);
            }
        }
        for (int e = tid; e < N2 * N2; e += 256) {
            double2 v = sy.L0[e];
            for (int c = 0; c < sy.n_chan; ++c) {
                c_fma(v, f[c], sy.S[(size_t)c * N2 * N2 + e]);
                c_fma(v, fc[c], sy.T[(size_t)c * N2 * N2 + e]);
            }
            A[e] = c_scale(v, w);
        }
        __syncthreads();
        if (tid < N2) {
            double s = 0.0;
            for (int r = 0; r < N2; ++r) { const double2 a = A[r * N2 + tid]; s += hypot(a.x, a.y); }
            colsum[tid] = s;
        }
        __syncthreads();
        if (tid == 0) {
            double norm = 0.0;
            for (int c = 0; c < N2; ++c) norm = colsum[c] > norm ? colsum[c] : norm;
            int e2 = 0;
            frexp(norm / 0.5, &e2);
            const int s = e2 > 0 ? e2 : 0;
            // Taylor degree: the smallest m <= 18 whose remainder bound theta^(m+1)/(m+1)! e^theta on the
            // scaled matrix (theta <= 0.5) is below 2^-56, so the series stops at double precision instead of
            // always running 18 terms (theta = 0.5 needs 15 terms, smaller norms fewer)
            const double theta = ldexp(norm, -s);
            double rem = 0.5 * theta * theta;  // theta^(deg+1)/(deg+1)! for deg = 1
            int deg = 1;
            while (deg < 18 && rem * 1.7 > 1.4e-17) { ++deg; rem *= theta / (deg + 1); }
            s_sh = s;
            s_deg = deg;
        }
        __syncthreads();
        const int s = s_sh, deg = s_deg;
        const double scale = ldexp(1.0, -s);
        for (int e = tid; e < N2 * N2; e += 256) {
            const double2 a = c_scale(A[e], scale);
            A[e] = a;
            double2 pv = make_double2(a.x / (double)deg, a.y / (double)deg);
            const int i = e / N2;
            if (e == i * N2 + i) pv.x += 1.0;
            P[e] = pv;
        }
        __syncthreads();
        for (int mm = deg - 1; mm >= 1; --mm) {
            lds_matmul<N2>(A, P, T, tid);
            __syncthreads();
            for (int e = tid; e < N2 * N2; e += 256) {
                const double2 tv = T[e];
                double2 pv = make_double2(tv.x / (double)mm, tv.y / (double)mm);
                const int i = e / N2;
                if (e == i * N2 + i) pv.x += 1.0;
                P[e] = pv;
            }
            __syncthreads();
        }
        for (int q = 0; q < s; ++q) {
            lds_matmul<N2>(P, P, T, tid);
            __syncthreads();
            for (int e = tid; e < N2 * N2; e += 256) P[e] = T[e];
            __syncthreads();
        }
        if (nsub == 1) {
            // single factor: P is the propagator (no Acc buffer allocated, so two workgroups fit a CU at N2 = 36)
        } else if (j == 0) {
            for (int e = tid; e < N2 * N2; e += 256) Acc[e] = P[e];
        } else {
            lds_matmul<N2>(P, Acc, T, tid);
            __syncthreads();
            for (int e = tid; e < N2 * N2; e += 256) Acc[e] = T[e];
        }
        __syncthreads();
    }
    const double2* res = (nsub == 1) ? P : Acc;
    for (int e = tid; e < N2 * N2; e += 256) out[e] = res[e];
    __syncthreads();  // Acc is rewritten by the next matrix
    }
}

// ---------------------------------------------------------------------------------------------------------------
// Large N2 (25, 36: the six-level and five-level systems) on the FP64 matrix cores. The same algorithm and degree
// choice as free_prop_kernel, with every N2 x N2 complex product C = A B done as 4 x 4 blocks on
// v_mfma_f64_4x4x4_4b (N2 = 36 is 9 x 9 blocks exactly; 25 is padded to 7 x 7): one instruction computes four
// blocks D[blk] += A[blk] B[blk] (lane l = 16 k + 4 blk + x holds A[blk][x][k], B[blk][k][x], D[blk][l >> 4][x]),
// so the 81 output blocks are 21 instruction slots of four, dealt to the four waves, each accumulating its slots over
// the 9 k-blocks with 3 real products per complex product (3M). Operands stay in LDS with rows padded to an odd
// stride; the result of a product stays in registers until the step that consumes it (Horner: P = A P / m + I,
// squarings: P = P P, sub-steps: Acc = P Acc) writes it back after a barrier. The general kernel's 3 x 3 LDS blocks
// ran the C5 scan's 132 k six-level propagators in 26.5 ms (≈30 TF/s).
template <int N2>
struct FPM {
    static constexpr int NB = (N2 + 3) / 4;          // 4 x 4 blocks per dimension
    static constexpr int NP = 4 * NB;                // padded dimension
    static constexpr int LS = NP + 1;                // LDS row stride (complex)
    static constexpr int NSLOT = NB * NB;            // output blocks
    static constexpr int NG = (NSLOT + 3) / 4;       // instruction groups
    static constexpr int GPW = (NG + 3) / 4;         // groups per wave (4 waves)
    static constexpr size_t MAT = (size_t)NP * LS;   // complex elements per LDS matrix
};

// this lane's share of C = A B (A, B in LDS, padded, row stride LS): R[q] = element (row, col) of slot group
// g = wave + 4 q, in the D-layout (row = 4 I + (l >> 4), col = 4 J + (l & 3)); rows/cols of dummy slots are not stored
template <int N2>
__device__ __forceinline__ void fpm_product(const double2* A, const double2* B, double2 (&R)[FPM<N2>::GPW], int wave,
                                            int lane) {
    using F = FPM<N2>;
    const int k = lane >> 4, blk = (lane >> 2) & 3, x = lane & 3;
    double p1[F::GPW], p2[F::GPW], p3[F::GPW];
    int arow[F::GPW], bcol[F::GPW];
#pragma unroll
    for (int q = 0; q < F::GPW; ++q) {
        p1[q] = 0.0; p2[q] = 0.0; p3[q] = 0.0;
        int s = 4 * (wave + 4 * q) + blk;
        s = s < F::NSLOT ? s : F::NSLOT - 1;   // dummy slots recompute the last block (not stored)
        const int I = s / F::NB, J = s - (s / F::NB) * F::NB;
        arow[q] = (4 * I + x) * F::LS + k;      // A[4 I + x][4 K + k]
        bcol[q] = k * F::LS + 4 * J + x;        // B[4 K + k][4 J + x]
    }
#pragma unroll 3
    for (int K = 0; K < F::NB; ++K) {
#pragma unroll
        for (int q = 0; q < F::GPW; ++q) {
            if (wave + 4 * q >= F::NG) break;   // wave-uniform
            const double2 a = A[arow[q] + 4 * K];
            const double2 b = B[bcol[q] + 4 * K * F::LS];
            p1[q] = __builtin_amdgcn_mfma_f64_4x4x4f64(a.x, b.x, p1[q], 0, 0, 0);
            p2[q] = __builtin_amdgcn_mfma_f64_4x4x4f64(a.y, b.y, p2[q], 0, 0, 0);
            p3[q] = __builtin_amdgcn_mfma_f64_4x4x4f64(a.x + a.y, b.x + b.y, p3[q], 0, 0, 0);
        }
    }
#pragma unroll
    for (int q = 0; q < F::GPW; ++q) R[q] = make_double2(p1[q] - p2[q], p3[q] - p1[q] - p2[q]);
}

// the D-layout element of slot group q of this lane: its LDS index, or -1 (dummy slot, or padding beyond N2)
template <int N2>
__device__ __forceinline__ int fpm_index(int q, int wave, int lane, int& row, int& col) {
    using F = FPM<N2>;
    const int s = 4 * (wave + 4 * q) + ((lane >> 2) & 3);
    if (wave + 4 * q >= F::NG || s >= F::NSLOT) return -1;
    const int I = s / F::NB, J = s - (s / F::NB) * F::NB;
    row = 4 * I + (lane >> 4);
    col = 4 * J + (lane & 3);
    return (row < N2 && col < N2) ? row * F::LS + col : -1;
}

template <int N2>
__global__ __launch_bounds__(256) void free_prop_mfma_kernel(FreePropParams p) {
    using F = FPM<N2>;
    extern __shared__ __attribute__((aligned(16))) double2 smem[];
    double2* A = smem;
    double2* P = A + F::MAT;
    double2* Acc = P + F::MAT;   // n_sub > 1 only
    __shared__ double colsum[N2];
    __shared__ int s_sh, s_deg;
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    // padding rows / columns stay zero for the whole launch (every product reads them, none writes them)
    const int nmat = (p.n_sub > 1) ? 3 : 2;
    for (int e = tid; e < (int)(nmat * F::MAT); e += 256) smem[e] = c_zero();
    __syncthreads();
    const long long nblk = p.idle_pass ? (long long)p.n_sys : (long long)p.n_sys * 2 * p.n_steps;
    for (long long blk = blockIdx.x; blk < nblk; blk += gridDim.x) {
        const int si = p.idle_pass ? (int)blk : (int)(blk / (2 * p.n_steps));
        const int m = p.idle_pass ? 0 : (int)(blk - (long long)si * 2 * p.n_steps);
        const int n = m >> 1, h = m & 1;
        const FreePropSys sy = p.systems[si];
        const int nsub = p.n_sub > 0 ? p.n_sub : 1;
        const double w = 0.5 * p.dt / nsub;
        double2* out = p.idle_pass ? p.Midle + (size_t)si * N2 * N2 : p.M + ((size_t)si * 2 * p.n_steps + m) * N2 * N2;
        if (!p.idle_pass && p.win) {
            const int2 wn = p.win[si];
            if (m < wn.x || m > wn.y) continue;
        }
        if (!p.idle_pass && p.Midle && idle_half_step(sy, p.ta + n * p.dt + h * 0.5 * p.dt, w, nsub)) {
            const double2* src = p.Midle + (size_t)si * N2 * N2;
            for (int e = tid; e < N2 * N2; e += 256) out[e] = src[e];
            continue;
        }
        double2 R[F::GPW];
        for (int j = 0; j < nsub; ++j) {
            const double t = p.ta + n * p.dt + h * 0.5 * p.dt + (j + 0.5) * w;
            double2 f[4], fc[4];
#pragma unroll
            for (int c = 0; c < 4; ++c) {
                if (c < sy.n_chan) {
                    f[c] = p.idle_pass ? c_zero() : sample_ch(sy, c, t);
                    fc[c] = c_conj(f[c]);
                }
            }
            for (int e = tid; e < N2 * N2; e += 256) {
                double2 v = sy.L0[e];
                for (int c = 0; c < sy.n_chan; ++c) {
                    c_fma(v, f[c], sy.S[(size_t)c * N2 * N2 + e]);
                    c_fma(v, fc[c], sy.T[(size_t)c * N2 * N2 + e]);
                }
                const int i = e / N2, jj = e - i * N2;
                A[i * F::LS + jj] = c_scale(v, w);
            }
            __syncthreads();
            if (tid < N2) {
                double s = 0.0;
                for (int r = 0; r < N2; ++r) { const double2 a = A[r * F::LS + tid]; s += hypot(a.x, a.y); }
                colsum[tid] = s;
            }
            __syncthreads();
            if (tid == 0) {
                double norm = 0.0;
                for (int c = 0; c < N2; ++c) norm = colsum[c] > norm ? colsum[c] : norm;
                int e2 = 0;
                frexp(norm / 0.5, &e2);
                const int s = e2 > 0 ? e2 : 0;
                const double theta = ldexp(norm, -s);
                double rem = 0.5 * theta * theta;
                int deg = 1;
                while (deg < 18 && rem * 1.7 > 1.4e-17) { ++deg; rem *= theta / (deg + 1); }
                s_sh = s;
                s_deg = deg;
            }
            __syncthreads();
            const int s = s_sh, deg = s_deg;
            const double scale = ldexp(1.0, -s);
            for (int e = tid; e < N2 * N2; e += 256) {
                const int i = e / N2, jj = e - i * N2;
                const double2 a = c_scale(A[i * F::LS + jj], scale);
                A[i * F::LS + jj] = a;
                double2 pv = make_double2(a.x / (double)deg, a.y / (double)deg);
                if (i == jj) pv.x += 1.0;
                P[i * F::LS + jj] = pv;
            }
            __syncthreads();
            // Horner: P <- A P / mm + I
            for (int mm = deg - 1; mm >= 1; --mm) {
                const double rm = k_rinv[mm];
                fpm_product<N2>(A, P, R, wave, lane);
                __syncthreads();
#pragma unroll
                for (int q = 0; q < F::GPW; ++q) {
                    int r, c;
                    const int ix = fpm_index<N2>(q, wave, lane, r, c);
                    if (ix >= 0) {
                        double2 pv = make_double2(R[q].x * rm, R[q].y * rm);
                        if (r == c) pv.x += 1.0;
                        P[ix] = pv;
                    }
                }
                __syncthreads();
            }
            for (int qq = 0; qq < s; ++qq) {  // squarings
                fpm_product<N2>(P, P, R, wave, lane);
                __syncthreads();
#pragma unroll
                for (int q = 0; q < F::GPW; ++q) {
                    int r, c;
                    const int ix = fpm_index<N2>(q, wave, lane, r, c);
                    if (ix >= 0) P[ix] = R[q];
                }
                __syncthreads();
            }
            if (nsub > 1) {
                if (j == 0) {
                    for (int e = tid; e < N2 * N2; e += 256) {
                        const int i = e / N2, jj = e - i * N2;
                        Acc[i * F::LS + jj] = P[i * F::LS + jj];
                    }
                } else {
                    fpm_product<N2>(P, Acc, R, wave, lane);
                    __syncthreads();
#pragma unroll
                    for (int q = 0; q < F::GPW; ++q) {
                        int r, c;
                        const int ix = fpm_index<N2>(q, wave, lane, r, c);
                        if (ix >= 0) Acc[ix] = R[q];
                    }
                }
                __syncthreads();
            }
        }
        const double2* res = (nsub == 1) ? P : Acc;
        for (int e = tid; e < N2 * N2; e += 256) {
            const int i = e / N2, jj = e - i * N2;
            out[e] = res[i * F::LS + jj];
        }
        __syncthreads();
    }
}

template <int N2>
hipError_t launch_fpm(const FreePropParams& p, hipStream_t s) {
    using F = FPM<N2>;
    const size_t lds = (p.n_sub > 1 ? 3 : 2) * F::MAT * sizeof(double2);
    static bool attr = false;
    if (!attr) {
        hipError_t e = hipFuncSetAttribute((const void*)free_prop_mfma_kernel<N2>,
                                           hipFuncAttributeMaxDynamicSharedMemorySize, (int)(3 * F::MAT * sizeof(double2)));
        if (e != hipSuccess) return e;
        attr = true;
    }
    const long long nblk = p.idle_pass ? (long long)p.n_sys : 2LL * p.n_steps * p.n_sys;
    if (nblk <= 0) return hipSuccess;
    hipLaunchKernelGGL(free_prop_mfma_kernel<N2>, dim3((unsigned)std::min<long long>(nblk, FP_MAX_BLOCKS)), dim3(256),
                       lds, s, p);
    return hipGetLastError();
}

// N2 = 4 (two-level system): a 4 x 4 matrix is 16 lanes, so a wave carries 4 matrices
// and a 256-thread workgroup 16 — the general kernel would give each one a whole workgroup with 16 of
// its 256 threads busy and a barrier per matmul. Lane (matrix, i, j) holds element (i, j) of A, P and
// the accumulated product; products gather their row/column operands by lane shuffles inside the
// 16-lane group (same matrix, so the same degree and squaring count: the group never diverges
// internally). The arithmetic (sum orders included) is the general kernel's.
__device__ __forceinline__ double2 c_shfl(double2 v, int src) {
    return make_double2(__shfl(v.x, src), __shfl(v.y, src));
}

// C(i,j) = sum_k A(i,k) B(k,j) within the 16-lane group starting at lane gb
__device__ __forceinline__ double2 grp_matmul4(double2 a, double2 b, int gb, int i, int j) {
    double2 acc = c_zero();
#pragma unroll
    for (int k = 0; k < 4; ++k) c_fma(acc, c_shfl(a, gb + i * 4 + k), c_shfl(b, gb + k * 4 + j));
    return acc;
}

// one 4 x 4 propagator per 16-lane group: matrix (si, m) (m = half step; the idle pass: Midle of si). Dead groups
// (live = false) shadow a live matrix of the same workgroup and store nothing
__device__ __forceinline__ void fp4_matrix(const FreePropParams& p, int si, int m, bool live, int lane) {
    const int n = m >> 1, h = m & 1;
    const int gb = lane & ~15, e = lane & 15, i = e >> 2, j = e & 3;
    const FreePropSys sy = p.systems[si];
    const int nsub = p.n_sub > 0 ? p.n_sub : 1;
    const double w = 0.5 * p.dt / nsub;
    double2* out = p.idle_pass ? p.Midle + (size_t)si * 16 : p.M + ((size_t)si * 2 * p.n_steps + m) * 16;
    // an idle half step copies Midle; the test is uniform within the 16-lane group (one matrix), so the group's
    // shuffles below never mix copied and computed matrices of different groups
    if (!p.idle_pass && p.Midle && idle_half_step(sy, p.ta + n * p.dt + h * 0.5 * p.dt, w, nsub)) {
        if (live) out[e] = p.Midle[(size_t)si * 16 + e];
        return;
    }
    double2 acc = c_zero();
    for (int js = 0; js < nsub; ++js) {
        const double t = p.ta + n * p.dt + h * 0.5 * p.dt + (js + 0.5) * w;
        double2 v = sy.L0[e];
        for (int c = 0; c < sy.n_chan && c < 4; ++c) {
            const double2 f = p.idle_pass ? c_zero() : sample_ch(sy, c, t);
            c_fma(v, f, sy.S[(size_t)c * 16 + e]);
            c_fma(v, c_conj(f), sy.T[(size_t)c * 16 + e]);
        }
        double2 a = c_scale(v, w);
        // 1-norm: column sums in row order (as the general kernel), then the max over columns
        double cs = 0.0;
#pragma unroll
        for (int r = 0; r < 4; ++r) { const double2 x = c_shfl(a, gb + r * 4 + j); cs += hypot(x.x, x.y); }
        double norm = 0.0;
#pragma unroll
        for (int c = 0; c < 4; ++c) { const double x = __shfl(cs, gb + c); norm = x > norm ? x : norm; }
        int e2 = 0;
        frexp(norm / 0.5, &e2);
        const int sh = e2 > 0 ? e2 : 0;
        const double theta = ldexp(norm, -sh);
        double rem = 0.5 * theta * theta;
        int deg = 1;
        while (deg < 18 && rem * 1.7 > 1.4e-17) { ++deg; rem *= theta / (deg + 1); }
        a = c_scale(a, ldexp(1.0, -sh));
        double2 pm = make_double2(a.x / (double)deg, a.y / (double)deg);
        if (i == j) pm.x += 1.0;
        for (int mm = deg - 1; mm >= 1; --mm) {
            const double2 tv = grp_matmul4(a, pm, gb, i, j);
            pm = make_double2(tv.x / (double)mm, tv.y / (double)mm);
            if (i == j) pm.x += 1.0;
        }
        for (int q = 0; q < sh; ++q) pm = grp_matmul4(pm, pm, gb, i, j);
        acc = (js == 0) ? pm : grp_matmul4(pm, acc, gb, i, j);
    }
    if (live) out[e] = acc;
}

// main pass: one workgroup per p.chunk consecutive half steps of one system (16..128: 8 groups of 16 when the launch
// has thousands of workgroups to spare, 1 for a single system), clipped to the system's pulse window once (one window
// load per workgroup: a load per 16-matrix group made the out-of-window groups latency-bound, 1.5 ms of the TLS area
// scan's 4 ms)
static int fp4_chunk(const FreePropParams& p) {
    const long long groups = (long long)p.n_sys * ((2LL * p.n_steps + 15) / 16);
    long long g = groups / 8192;
    if (const char* e = getenv("PQD_FP4_CHUNK")) return atoi(e);  // A/B (a multiple of 16)
    return 16 * (int)(g < 1 ? 1 : (g > 8 ? 8 : g));
}

// The same propagator on the FP64 matrix cores: one v_mfma_f64_4x4x4_4b carries the 4 x 4 products of the wave's
// four matrices (block g = matrix), three instructions per complex product (3M). Lane l = 16 i + 4 g + j holds
// element (i, j) of matrix g: the instruction's D-layout, which is also the B-layout of the next product, so Horner
// steps chain without data movement; the A operand (lane 16 k + 4 g + i holds element (i, k)) is one shuffle of a
// D-layout value, done once per sub-step for the scaled generator and once per squaring. Degrees and squaring counts
// stay per matrix (the wave runs to its largest and each matrix keeps its value past its own count), so a matrix
// gets exactly the polynomial and squarings of fp4_matrix; only the rounding of the products differs (3M).
__device__ __forceinline__ double2 mm4_mfma(double2 aA, double2 b) {
    const double p1 = __builtin_amdgcn_mfma_f64_4x4x4f64(aA.x, b.x, 0.0, 0, 0, 0);
    const double p2 = __builtin_amdgcn_mfma_f64_4x4x4f64(aA.y, b.y, 0.0, 0, 0, 0);
    const double p3 = __builtin_amdgcn_mfma_f64_4x4x4f64(aA.x + aA.y, b.x + b.y, 0.0, 0, 0, 0);
    return make_double2(p1 - p2, p3 - p1 - p2);
}
// D-layout -> A-layout: lane (k, g, i) takes element (i, k) of matrix g, held by lane 16 i + 4 g + k
__device__ __forceinline__ double2 to_a4(double2 v, int lane) {
    return c_shfl(v, 16 * (lane & 3) + (lane & 12) + (lane >> 4));
}
__device__ __forceinline__ int wave_max_i(int v) {
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) { const int y = __shfl_xor(v, o); v = y > v ? y : v; }
    return __builtin_amdgcn_readfirstlane(v);
}

// all 64 lanes of the wave call this together (the MFMAs read every lane); matrix g = (lane >> 2) & 3
__device__ __forceinline__ void fp4m_matrix(const FreePropParams& p, int si, int m, bool live, int lane) {
    const int n = m >> 1, h = m & 1;
    const int i = lane >> 4, j = lane & 3, e = 4 * i + j;
    const FreePropSys sy = p.systems[si];
    const int nsub = p.n_sub > 0 ? p.n_sub : 1;
    const double w = 0.5 * p.dt / nsub;
    double2* out = p.idle_pass ? p.Midle + (size_t)si * 16 : p.M + ((size_t)si * 2 * p.n_steps + m) * 16;
    const bool idle = !p.idle_pass && p.Midle && idle_half_step(sy, p.ta + n * p.dt + h * 0.5 * p.dt, w, nsub);
    if (idle && live) out[e] = p.Midle[(size_t)si * 16 + e];
    if (__ballot(!idle) == 0) return;  // wave-uniform
    double2 acc = c_zero();
    for (int js = 0; js < nsub; ++js) {
        const double t = p.ta + n * p.dt + h * 0.5 * p.dt + (js + 0.5) * w;
        double2 v = sy.L0[e];
        for (int c = 0; c < sy.n_chan && c < 4; ++c) {
            const double2 f = p.idle_pass ? c_zero() : sample_ch(sy, c, t);
            c_fma(v, f, sy.S[(size_t)c * 16 + e]);
            c_fma(v, c_conj(f), sy.T[(size_t)c * 16 + e]);
        }
        double2 a = c_scale(v, w);
        // 1-norm as fp4_matrix: column sums in row order, then the max over columns
        double cs = 0.0;
#pragma unroll
        for (int r = 0; r < 4; ++r) { const double2 x = c_shfl(a, 16 * r + (lane & 15)); cs += hypot(x.x, x.y); }
        double norm = 0.0;
#pragma unroll
        for (int c = 0; c < 4; ++c) { const double x = __shfl(cs, (lane & ~3) + c); norm = x > norm ? x : norm; }
        int e2 = 0;
        frexp(norm / 0.5, &e2);
        const int sh = e2 > 0 ? e2 : 0;
        const double theta = ldexp(norm, -sh);
        double rem = 0.5 * theta * theta;
        int deg = 1;
        while (deg < 18 && rem * 1.7 > 1.4e-17) { ++deg; rem *= theta / (deg + 1); }
        a = c_scale(a, ldexp(1.0, -sh));
        const double2 aA = to_a4(a, lane);
        double2 pm = make_double2(a.x / (double)deg, a.y / (double)deg);
        if (i == j) pm.x += 1.0;
        const int dmax = wave_max_i(deg), smax = wave_max_i(sh);
        for (int mm = dmax - 1; mm >= 1; --mm) {
            const double2 tv = mm4_mfma(aA, pm);
            const double rm = k_rinv[mm];
            double2 u = make_double2(tv.x * rm, tv.y * rm);
            if (i == j) u.x += 1.0;
            const bool up = mm < deg;  // per-component selects (a select of double2 values went through scratch)
            pm.x = up ? u.x : pm.x;
            pm.y = up ? u.y : pm.y;
        }
        for (int q = 0; q < smax; ++q) {
            const double2 tv = mm4_mfma(to_a4(pm, lane), pm);
            const bool up = q < sh;
            pm.x = up ? tv.x : pm.x;
            pm.y = up ? tv.y : pm.y;
        }
        if (js == 0) acc = pm;
        else acc = mm4_mfma(to_a4(pm, lane), acc);
    }
    if (live && !idle) out[e] = acc;
}

template <bool MF>
__global__ __launch_bounds__(256) void free_prop4_kernel(FreePropParams p) {
    const int tid = threadIdx.x, lane = tid & 63;
    // matrix of this lane within the workgroup's 16: 16-lane groups (fp4_matrix) or block g of the wave (fp4m_matrix)
    const int mw = MF ? 4 * (tid >> 6) + ((lane >> 2) & 3) : tid >> 4;
    if (p.idle_pass) {
        for (long long base = (long long)blockIdx.x * 16; base < p.n_sys; base += (long long)gridDim.x * 16) {
            const long long mat = base + mw;
            const bool live = mat < p.n_sys;
            if constexpr (MF) fp4m_matrix(p, (int)(live ? mat : p.n_sys - 1), 0, live, lane);
            else fp4_matrix(p, (int)(live ? mat : p.n_sys - 1), 0, live, lane);
        }
        return;
    }
    const int nh = 2 * p.n_steps, CH = p.chunk, cps = (nh + CH - 1) / CH;
    const long long nblk = (long long)p.n_sys * cps;
    for (long long b = blockIdx.x; b < nblk; b += gridDim.x) {
        // chunks rotate with the system: workgroups go to the 8 XCDs round-robin, so with cps a multiple of 8 the
        // chunk at one time position (pulse centre: larger norms, more squarings) would land on one XCD for every
        // system (C1 free propagators 3.8 -> 5.7 ms at 64/128-step chunks without the rotation)
        const int si = (int)(b / cps), r = (int)(b - (long long)si * cps), ch = (r + si) % cps;
        int lo = ch * CH, hi = (lo + CH < nh ? lo + CH : nh) - 1;
        if (p.win) {  // outside the pulse window: not stored (readers take Midle)
            const int2 wn = p.win[si];
            lo = lo > wn.x ? lo : wn.x;
            hi = hi < wn.y ? hi : wn.y;
        }
        for (int base = lo; base <= hi; base += 16) {
            const int m = base + mw;
            const bool live = m <= hi;
            if constexpr (MF) fp4m_matrix(p, si, live ? m : hi, live, lane);
            else fp4_matrix(p, si, live ? m : hi, live, lane);
        }
    }
}

// Pulse windows: win[s] = (first, last) half step of system s that is not idle (INT_MAX, -1 when all are). The idle
// test is the builders' own, so a half step outside the window is exactly one the builders would have copied Midle
// into. One workgroup per 256 consecutive half steps of one system: a block reduction, then one atomic min / max.
__global__ __launch_bounds__(256) void free_win_init_kernel(int2* win, int n_sys) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i < n_sys) win[i] = make_int2(INT_MAX, -1);
}

__global__ __launch_bounds__(256) void free_win_kernel(FreePropParams p) {
    __shared__ int s_lo[4], s_hi[4];
    const int nh = 2 * p.n_steps, chunks = (nh + 255) / 256;
    const long long nblk = (long long)p.n_sys * chunks;
    const int nsub = p.n_sub > 0 ? p.n_sub : 1;
    const double w = 0.5 * p.dt / nsub;
    for (long long blk = blockIdx.x; blk < nblk; blk += gridDim.x) {
        const int si = (int)(blk / chunks);
        const int m = (int)(blk - (long long)si * chunks) * 256 + (int)threadIdx.x;
        int lo = INT_MAX, hi = -1;
        if (m < nh) {
            const FreePropSys sy = p.systems[si];
            const int n = m >> 1, h = m & 1;
            if (!idle_half_step(sy, p.ta + n * p.dt + h * 0.5 * p.dt, w, nsub)) lo = hi = m;
        }
#pragma unroll
        for (int o = 32; o >= 1; o >>= 1) {
            const int a = __shfl_xor(lo, o), b = __shfl_xor(hi, o);
            lo = a < lo ? a : lo;
            hi = b > hi ? b : hi;
        }
        const int wv = threadIdx.x >> 6;
        if ((threadIdx.x & 63) == 0) { s_lo[wv] = lo; s_hi[wv] = hi; }
        __syncthreads();
        if (threadIdx.x == 0) {
            for (int k = 1; k < 4; ++k) { lo = s_lo[k] < lo ? s_lo[k] : lo; hi = s_hi[k] > hi ? s_hi[k] : hi; }
            if (hi >= 0) {
                atomicMin(&p.win[si].x, lo);
                atomicMax(&p.win[si].y, hi);
            }
        }
        __syncthreads();
    }
}

template <int N2>
hipError_t launch_fp(const FreePropParams& p, hipStream_t s) {
    const size_t lds = 4ull * N2 * N2 * sizeof(double2);
    static bool attr = false;
    if (!attr) {
        hipError_t e = hipFuncSetAttribute((const void*)free_prop_kernel<N2>,
                                           hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
        if (e != hipSuccess) return e;
        attr = true;
    }
    const long long nblk = p.idle_pass ? (long long)p.n_sys : 2LL * p.n_steps * p.n_sys;
    if (nblk <= 0) return hipSuccess;
    // A, P, T (+ Acc only for n_sub > 1): at N2 = 36, 62 KiB instead of 83 KiB lets two workgroups share a CU
    const size_t lds_run = (p.n_sub > 1 ? 4ull : 3ull) * N2 * N2 * sizeof(double2);
    hipLaunchKernelGGL(free_prop_kernel<N2>, dim3((unsigned)std::min<long long>(nblk, FP_MAX_BLOCKS)), dim3(256),
                       lds_run, s, p);
    return hipGetLastError();
}

// Fused free half steps of consecutive PT steps. Between PT(m-1) and PT(m) a trajectory without MTOs at
// step m applies M_b(m-1), reads its outputs, then applies M_a(m): one N2 x N2 operator F(m) = M_a(m) M_b(m-1)
// does the same work with half the column-phase flops, and the outputs at step m are read from the state
// before M_b(m-1) through W(m)[k] = ovec[k] . M_b(m-1) (a row vector per output operator).
template <int N2>
__global__ __launch_bounds__(256) void fuse_steps_kernel(FuseParams p) {
    const long long nblk = (long long)p.n_sys * p.n_steps;
    for (long long blk = blockIdx.x; blk < nblk; blk += gridDim.x) {
    const int si = (int)(blk / p.n_steps), m = (int)(blk - (long long)si * p.n_steps) + 1;  // m = 1..n_steps
    const int tid = threadIdx.x;
    int2 wn = make_int2(INT_MIN, INT_MAX);
    if (p.win) wn = p.win[si];
    const bool out_b = 2 * m - 1 < wn.x || 2 * m - 1 > wn.y, out_a = 2 * m < wn.x || 2 * m > wn.y;
    if (out_b && out_a) continue;  // F(m) and W(m) are the idle ones (block-uniform)
    // a half step outside the window is not stored: its propagator is Midle
    const double2* Mb = out_b ? p.Midle + (size_t)si * N2 * N2
                              : p.M + ((size_t)si * 2 * p.n_steps + 2 * (m - 1) + 1) * N2 * N2;
    if (m < p.n_steps) {
        const double2* Ma = out_a ? p.Midle + (size_t)si * N2 * N2
                                  : p.M + ((size_t)si * 2 * p.n_steps + 2 * m) * N2 * N2;
        double2* F = p.F + ((size_t)si * p.n_steps + m) * N2 * N2;
        for (int e = tid; e < N2 * N2; e += 256) {
            const int r = e / N2, c = e - (e / N2) * N2;
            double2 acc = c_zero();
#pragma unroll
            for (int k = 0; k < N2; ++k) c_fma(acc, Ma[r * N2 + k], Mb[k * N2 + c]);
            F[e] = acc;
        }
    }
    double2* W = p.W + ((size_t)si * (p.n_steps + 1) + m) * p.n_out * N2;
    if (!out_b)
    for (int e = tid; e < p.n_out * N2; e += 256) {
        const int k = e / N2, a = e - (e / N2) * N2;
        double2 acc = c_zero();
#pragma unroll
        for (int b = 0; b < N2; ++b) c_fma(acc, p.ovec[k * N2 + b], Mb[b * N2 + a]);
        W[e] = acc;
    }
    }
}

// N2 = 25, 36: F(m) = M_a(m) M_b(m-1) as one matrix-core product (fpm_product) on the two operators staged in LDS;
// W(m) = ovec . M_b(m-1) from the staged M_b. Same skips as fuse_steps_kernel.
template <int N2>
__global__ __launch_bounds__(256) void fuse_steps_mfma_kernel(FuseParams p) {
    using F = FPM<N2>;
    extern __shared__ __attribute__((aligned(16))) double2 smem[];
    double2* Sa = smem;
    double2* Sb = Sa + F::MAT;
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    for (int e = tid; e < (int)(2 * F::MAT); e += 256) smem[e] = c_zero();
    __syncthreads();
    const long long nblk = (long long)p.n_sys * p.n_steps;
    for (long long blk = blockIdx.x; blk < nblk; blk += gridDim.x) {
        const int si = (int)(blk / p.n_steps), m = (int)(blk - (long long)si * p.n_steps) + 1;  // m = 1..n_steps
        int2 wn = make_int2(INT_MIN, INT_MAX);
        if (p.win) wn = p.win[si];
        const bool out_b = 2 * m - 1 < wn.x || 2 * m - 1 > wn.y, out_a = 2 * m < wn.x || 2 * m > wn.y;
        if (out_b && out_a) continue;
        const double2* Mb = out_b ? p.Midle + (size_t)si * N2 * N2
                                  : p.M + ((size_t)si * 2 * p.n_steps + 2 * (m - 1) + 1) * N2 * N2;
        const bool hasF = m < p.n_steps;
        const double2* Ma = (!hasF) ? Mb
                          : out_a ? p.Midle + (size_t)si * N2 * N2 : p.M + ((size_t)si * 2 * p.n_steps + 2 * m) * N2 * N2;
        for (int e = tid; e < N2 * N2; e += 256) {
            const int i = e / N2, j = e - i * N2;
            Sb[i * F::LS + j] = Mb[e];
            if (hasF) Sa[i * F::LS + j] = Ma[e];
        }
        __syncthreads();
        if (hasF) {
            double2 R[F::GPW];
            fpm_product<N2>(Sa, Sb, R, wave, lane);
            double2* Fo = p.F + ((size_t)si * p.n_steps + m) * N2 * N2;
#pragma unroll
            for (int q = 0; q < F::GPW; ++q) {
                int r, c;
                if (fpm_index<N2>(q, wave, lane, r, c) >= 0) Fo[r * N2 + c] = R[q];
            }
        }
        if (!out_b) {
            double2* W = p.W + ((size_t)si * (p.n_steps + 1) + m) * p.n_out * N2;
            for (int e = tid; e < p.n_out * N2; e += 256) {
                const int k = e / N2, a = e - (e / N2) * N2;
                double2 acc = c_zero();
#pragma unroll 4
                for (int b = 0; b < N2; ++b) c_fma(acc, p.ovec[k * N2 + b], Sb[b * F::LS + a]);
                W[e] = acc;
            }
        }
        __syncthreads();
    }
}

// small N2: one thread per output element — F(m) entries, then W(m) entries — instead of a 256-thread workgroup per
// step with N2^2 + n_out N2 of its threads busy (N2 = 4: 24 of 256). A workgroup takes FS_CHUNK steps of one system,
// clipped to the steps whose F or W is stored (the pulse window) with one window load
constexpr int FS_CHUNK = 64;

template <int N2>
__global__ __launch_bounds__(256) void fuse_steps_flat_kernel(FuseParams p) {
    const int E = N2 * N2 + p.n_out * N2;
    const int cps = (p.n_steps + FS_CHUNK - 1) / FS_CHUNK;
    const long long nblk = (long long)p.n_sys * cps;
    for (long long bk = blockIdx.x; bk < nblk; bk += gridDim.x) {
        const int si = (int)(bk / cps), ch = (int)(bk - (long long)si * cps);
        int m_lo = 1 + ch * FS_CHUNK, m_hi = m_lo + FS_CHUNK - 1 < p.n_steps ? m_lo + FS_CHUNK - 1 : p.n_steps;
        int2 wn = make_int2(INT_MIN, INT_MAX);
        if (p.win) {
            wn = p.win[si];
            if (wn.y < 0) continue;  // no pulse at all: every F and W is the idle one
            // F(m) is stored when 2m - 1 or 2m lies in [lo, hi], W(m) when 2m - 1 does: m in [ceil(lo/2), (hi+1)/2]
            const int a = (wn.x + 1) >> 1, b = (wn.y + 1) >> 1;
            m_lo = m_lo > a ? m_lo : a;
            m_hi = m_hi < b ? m_hi : b;
        }
        const int cnt = m_hi - m_lo + 1;
        for (int i = threadIdx.x; i < cnt * E; i += 256) {
            const int m = m_lo + i / E, e = i - (i / E) * E;
            const bool out_b = 2 * m - 1 < wn.x || 2 * m - 1 > wn.y, out_a = 2 * m < wn.x || 2 * m > wn.y;
            // a half step outside the window is not stored: its propagator is Midle
            const double2* Mb = out_b ? p.Midle + (size_t)si * N2 * N2
                                      : p.M + ((size_t)si * 2 * p.n_steps + 2 * (m - 1) + 1) * N2 * N2;
            double2 acc = c_zero();
            if (e < N2 * N2) {
                if (m >= p.n_steps) continue;
                if (out_b && out_a) continue;  // F(m) is Fidle: not stored
                const double2* Ma = out_a ? p.Midle + (size_t)si * N2 * N2
                                          : p.M + ((size_t)si * 2 * p.n_steps + 2 * m) * N2 * N2;
                const int r = e / N2, c = e - (e / N2) * N2;
#pragma unroll
                for (int k = 0; k < N2; ++k) c_fma(acc, Ma[r * N2 + k], Mb[k * N2 + c]);
                p.F[((size_t)si * p.n_steps + m) * N2 * N2 + e] = acc;
            } else {
                if (out_b) continue;  // W(m) is Widle: not stored
                const int q = e - N2 * N2, k = q / N2, a = q - (q / N2) * N2;
#pragma unroll
                for (int b = 0; b < N2; ++b) c_fma(acc, p.ovec[k * N2 + b], Mb[b * N2 + a]);
                p.W[((size_t)si * (p.n_steps + 1) + m) * p.n_out * N2 + q] = acc;
            }
        }
    }
}

// the idle operators of every system, with the fuse kernels' arithmetic (same summation order): Fidle = Midle Midle,
// Widle = ovec . Midle — so a step outside the window reads the bits a stored copy would have held
template <int N2>
__global__ __launch_bounds__(256) void fuse_idle_kernel(FuseParams p) {
    const int E = N2 * N2 + p.n_out * N2;
    const long long total = (long long)p.n_sys * E;
    for (long long idx = (long long)blockIdx.x * 256 + threadIdx.x; idx < total; idx += (long long)gridDim.x * 256) {
        const int si = (int)(idx / E), e = (int)(idx - (long long)si * E);
        const double2* Mi = p.Midle + (size_t)si * N2 * N2;
        double2 acc = c_zero();
        if (e < N2 * N2) {
            const int r = e / N2, c = e - (e / N2) * N2;
#pragma unroll
            for (int k = 0; k < N2; ++k) c_fma(acc, Mi[r * N2 + k], Mi[k * N2 + c]);
            p.Fidle[(size_t)si * N2 * N2 + e] = acc;
        } else {
            const int q = e - N2 * N2, k = q / N2, a = q - (q / N2) * N2;
#pragma unroll
            for (int b = 0; b < N2; ++b) c_fma(acc, p.ovec[k * N2 + b], Mi[b * N2 + a]);
            p.Widle[(size_t)si * p.n_out * N2 + q] = acc;
        }
    }
}

template <int N2>
hipError_t launch_fs(const FuseParams& p, hipStream_t s) {
    const long long nblk = (long long)p.n_sys * p.n_steps;
    if (nblk <= 0) return hipSuccess;
    if (p.win) {
        const long long total = (long long)p.n_sys * (N2 * N2 + p.n_out * N2);
        hipLaunchKernelGGL(fuse_idle_kernel<N2>, dim3((unsigned)std::min<long long>((total + 255) / 256, FP_MAX_BLOCKS)),
                           dim3(256), 0, s, p);
        if (hipError_t e = hipGetLastError(); e != hipSuccess) return e;
    }
    if constexpr (N2 <= 9) {
        const long long nb = (long long)p.n_sys * ((p.n_steps + FS_CHUNK - 1) / FS_CHUNK);
        hipLaunchKernelGGL(fuse_steps_flat_kernel<N2>, dim3((unsigned)std::min<long long>(nb, FP_MAX_BLOCKS)), dim3(256),
                           0, s, p);
        return hipGetLastError();
    }
    if constexpr (N2 >= 25) {
        if (p.mfma) {
            hipLaunchKernelGGL(fuse_steps_mfma_kernel<N2>, dim3((unsigned)std::min<long long>(nblk, FP_MAX_BLOCKS)),
                               dim3(256), 2 * FPM<N2>::MAT * sizeof(double2), s, p);
            return hipGetLastError();
        }
    }
    hipLaunchKernelGGL(fuse_steps_kernel<N2>, dim3((unsigned)std::min<long long>(nblk, FP_MAX_BLOCKS)), dim3(256), 0,
                       s, p);
    return hipGetLastError();
}

}  // namespace

hipError_t launch_fuse_steps(int N2, const FuseParams& p, hipStream_t s) {
    switch (N2) {
        case 4: return launch_fs<4>(p, s);
        case 9: return launch_fs<9>(p, s);
        case 16: return launch_fs<16>(p, s);
        case 25: return launch_fs<25>(p, s);
        case 36: return launch_fs<36>(p, s);
        default: return hipErrorInvalidValue;
    }
}

static hipError_t launch_free_prop_pass(int N2, const FreePropParams& p, hipStream_t s) {
    if (N2 == 4 && p.packed4) {  // packed4 = 0 (PQD_FP4=0 at plan creation): the general kernel (A/B)
        FreePropParams q = p;
        q.chunk = fp4_chunk(p);
        const long long nblk = p.idle_pass ? ((long long)p.n_sys + 15) / 16
                                           : (long long)p.n_sys * ((2LL * p.n_steps + q.chunk - 1) / q.chunk);
        if (nblk <= 0) return hipSuccess;
        // p.mfma (PQD_FPM, default 1): the matrix-core products; 0: the shuffle products (A/B)
        if (p.mfma)
            hipLaunchKernelGGL(free_prop4_kernel<true>, dim3((unsigned)std::min<long long>(nblk, FP_MAX_BLOCKS)), dim3(256),
                               0, s, q);
        else
            hipLaunchKernelGGL(free_prop4_kernel<false>, dim3((unsigned)std::min<long long>(nblk, FP_MAX_BLOCKS)),
                               dim3(256), 0, s, q);
        return hipGetLastError();
    }
    switch (N2) {
        case 4: return launch_fp<4>(p, s);
        case 9: return launch_fp<9>(p, s);
        case 16: return p.mfma ? launch_fpm<16>(p, s) : launch_fp<16>(p, s);
        case 25: return p.mfma ? launch_fpm<25>(p, s) : launch_fp<25>(p, s);
        case 36: return p.mfma ? launch_fpm<36>(p, s) : launch_fp<36>(p, s);
        default: return hipErrorInvalidValue;
    }
}

// the pulse windows alone (plan creation decides from them whether windows pay, pqd_host.cpp)
hipError_t launch_free_win(const FreePropParams& p, hipStream_t s) {
    if (!p.win || p.n_steps <= 0 || p.n_sys <= 0) return hipSuccess;
    hipLaunchKernelGGL(free_win_init_kernel, dim3((p.n_sys + 255) / 256), dim3(256), 0, s, p.win, p.n_sys);
    const long long nblk = (long long)p.n_sys * ((2LL * p.n_steps + 255) / 256);
    hipLaunchKernelGGL(free_win_kernel, dim3((unsigned)std::min<long long>(nblk, FP_MAX_BLOCKS)), dim3(256), 0, s, p);
    return hipGetLastError();
}

// with p.Midle: the idle propagators first (one per system), then (with p.win) the pulse windows, then every half step
// inside its window (idle ones copy Midle)
hipError_t launch_free_prop(int N2, const FreePropParams& p, hipStream_t s) {
    FreePropParams q = p;
    if (p.Midle && p.n_steps > 0) {
        q.idle_pass = 1;
        hipError_t e = launch_free_prop_pass(N2, q, s);
        if (e != hipSuccess) return e;
    }
    q.idle_pass = 0;
    if (!p.Midle) q.win = nullptr;  // windows need the idle propagator
    if (q.win && p.n_steps > 0) {
        hipLaunchKernelGGL(free_win_init_kernel, dim3((p.n_sys + 255) / 256), dim3(256), 0, s, q.win, p.n_sys);
        const long long nblk = (long long)p.n_sys * ((2LL * p.n_steps + 255) / 256);
        hipLaunchKernelGGL(free_win_kernel, dim3((unsigned)std::min<long long>(nblk, FP_MAX_BLOCKS)), dim3(256), 0, s,
                           q);
        if (hipError_t e = hipGetLastError(); e != hipSuccess) return e;
    }
    return launch_free_prop_pass(N2, q, s);
}
