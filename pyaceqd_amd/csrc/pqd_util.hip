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

}  // namespace

hipError_t launch_check_finite(const double2* v, int64_t n, unsigned* flags, hipStream_t s) {
    if (n <= 0) return hipSuccess;
    const int64_t blocks = std::min<int64_t>((n + 255) / 256, 4096);
    hipLaunchKernelGGL(check_finite_kernel, dim3((unsigned)blocks), dim3(256), 0, s, v, n, flags);
    return hipGetLastError();
}
