// pqd_util.hip — small device utilities of libpqd (gfx950).
#include "pqd_common.h"
#include <algorithm>

namespace {

// one flag per launch: any non-finite real or imaginary part among n complex values sets flags bit 0. Grid-stride,
// 16-B loads; a wave that found one raises the flag once (vector atomic).
__global__ __launch_bounds__(256) void check_finite_kernel(const double2* __restrict__ v, int64_t n,
                                                           unsigned* __restrict__ flags) {
    bool bad = false;
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
        const double2 x = v[i];
        bad |= !(__builtin_isfinite(x.x) && __builtin_isfinite(x.y));
    }
    if (__any(bad) && (threadIdx.x & 63) == 0) atomicOr(flags, 1u);
}

// ACE's output table per trajectory (general_system.py:343, `np.loadtxt(outfile).T`): row 0 the times
// t_start + dt * step, rows 1 + k the outputs, for the steps of the trajectory's window. One workgroup per trajectory
// (grid-stride), lanes over steps; the time is dt * step then + t_start in two roundings, as numpy forms it.
__global__ __launch_bounds__(256) void table_kernel(const double2* __restrict__ out, const long long* __restrict__ woff,
                                                    const int* __restrict__ wbeg, const int* __restrict__ wend,
                                                    const long long* __restrict__ toff, int n_traj, int n_out,
                                                    double t_start, double dt, double2* __restrict__ table) {
    for (int t = blockIdx.x; t < n_traj; t += gridDim.x) {
        const int b = wbeg[t], L = wend[t] - wbeg[t] + 1;
        const double2* o = out + woff[t];
        double2* tb = table + toff[t];
        for (int i = threadIdx.x; i < L; i += 256) {
#pragma clang fp contract(off)  // no FMA: the product rounds before the sum, as in numpy
            tb[i] = make_double2(dt * (double)(b + i) + t_start, 0.0);
            for (int k = 0; k < n_out; ++k) tb[(size_t)(1 + k) * L + i] = o[(size_t)i * n_out + k];
        }
    }
}

// trapezoid integrals over each trajectory's window (pqd_plan_trapz): one wave per (trajectory, pair), lanes over the
// interior steps 1 .. L-2 of the tail output, a 64-lane tree sum; res = dx (y_head(0) / 2 + interior + y_tail(L-1) / 2)
__global__ __launch_bounds__(256) void trapz_kernel(const double2* __restrict__ out, const long long* __restrict__ woff,
                                                    const int* __restrict__ wbeg, const int* __restrict__ wend,
                                                    int n_traj, int n_out, int n_pairs, const int* __restrict__ kh,
                                                    const int* __restrict__ kt, double dx, double2* __restrict__ res) {
    const int lane = threadIdx.x & 63;
    const long long n_items = (long long)n_traj * n_pairs;
    for (long long it = (long long)blockIdx.x * 4 + (threadIdx.x >> 6); it < n_items; it += (long long)gridDim.x * 4) {
        const int t = (int)(it / n_pairs), q = (int)(it - (long long)t * n_pairs);
        const int L = wend[t] - wbeg[t] + 1;
        const double2* o = out + woff[t];
        const int a = kh[q], b = kt[q];
        double2 acc = c_zero();
        for (int i = 1 + lane; i < L - 1; i += 64) acc = c_add(acc, o[(size_t)i * n_out + b]);
#pragma unroll
        for (int m = 32; m >= 1; m >>= 1) acc = c_add(acc, c_shfl_xor(acc, m));
        if (lane == 0) {
            double2 v = c_zero();
            if (L >= 2) {
                const double2 h = o[a], e = o[(size_t)(L - 1) * n_out + b];
                v = c_scale(make_double2(0.5 * h.x + acc.x + 0.5 * e.x, 0.5 * h.y + acc.y + 0.5 * e.y), dx);
            }
            res[it] = v;
        }
    }
}

}  // namespace

hipError_t launch_trapz(const double2* out, const long long* woff, const int* wbeg, const int* wend, int n_traj,
                        int n_out, int n_pairs, const int* kh, const int* kt, double dx, double2* res, hipStream_t s) {
    const long long items = (long long)n_traj * n_pairs;
    if (items <= 0) return hipSuccess;
    hipLaunchKernelGGL(trapz_kernel, dim3((unsigned)std::min<long long>((items + 3) / 4, 1 << 16)), dim3(256), 0, s, out,
                       woff, wbeg, wend, n_traj, n_out, n_pairs, kh, kt, dx, res);
    return hipGetLastError();
}

hipError_t launch_table(const double2* out, const long long* woff, const int* wbeg, const int* wend,
                        const long long* toff, int n_traj, int n_out, double t_start, double dt, double2* table,
                        hipStream_t s) {
    if (n_traj <= 0) return hipSuccess;
    hipLaunchKernelGGL(table_kernel, dim3((unsigned)std::min(n_traj, 1 << 16)), dim3(256), 0, s, out, woff, wbeg,
                       wend, toff, n_traj, n_out, t_start, dt, table);
    return hipGetLastError();
}

hipError_t launch_check_finite(const double2* v, int64_t n, unsigned* flags, hipStream_t s) {
    if (n <= 0) return hipSuccess;
    const int64_t blocks = std::min<int64_t>((n + 255) / 256, 4096);
    hipLaunchKernelGGL(check_finite_kernel, dim3((unsigned)blocks), dim3(256), 0, s, v, n, flags);
    return hipGetLastError();
}
