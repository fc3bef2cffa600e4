// Microbenchmark: do FP64 VALU (v_fma_f64) and FP64 MFMA (v_mfma_f64_16x16x4_f64) waves overlap on
// gfx950? 256 workgroups x 8 waves (2 per SIMD). mode 0: all waves VALU, 1: all waves MFMA,
// 2: waves 0-3 VALU + waves 4-7 MFMA (one of each per SIMD), 3: all waves alternate both.
// Prints kernel ms per mode (HIP events) and the implied per-wave instruction cycle costs.
#include <hip/hip_runtime.h>
#include <cstdio>
typedef double dbl4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ void valu_work(double* out, int iters, double seed) {
    double a[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) a[i] = seed + i;
    const double x = seed * 1e-9, y = 1.0 - 1e-12;
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int i = 0; i < 16; ++i) a[i] = fma(a[i], y, x);
#pragma unroll
        for (int i = 0; i < 16; ++i) a[i] = fma(a[i], y, x);
    }
    double s = 0;
#pragma unroll
    for (int i = 0; i < 16; ++i) s += a[i];
    out[0] = s;
}

__device__ __forceinline__ void mfma_work(double* out, int iters, double seed) {
    dbl4 c[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) c[i] = dbl4{seed, 0, 0, 0};
    const double a = 1e-9 * seed, b = 1.0 - 1e-12;
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int i = 0; i < 4; ++i) c[i] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c[i], 0, 0, 0);
#pragma unroll
        for (int i = 0; i < 4; ++i) c[i] = __builtin_amdgcn_mfma_f64_16x16x4f64(b, a, c[i], 0, 0, 0);
    }
    out[0] = c[0][0] + c[1][1] + c[2][2] + c[3][3];
}

__global__ __launch_bounds__(512) void k(double* out, int mode, int iv, int im) {
    const int wave = threadIdx.x >> 6;
    double* o = out + blockIdx.x * 512 + threadIdx.x;
    const double seed = 1.0 + threadIdx.x * 1e-3;
    if (mode == 0) valu_work(o, iv, seed);
    else if (mode == 1) mfma_work(o, im, seed);
    else if (mode == 2) { if (wave < 4) valu_work(o, iv, seed); else mfma_work(o, im, seed); }
    else { valu_work(o, iv / 2, seed); mfma_work(o, im / 2, seed); }
}

int main() {
    double* d;
    hipMalloc(&d, 256 * 512 * sizeof(double));
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    const int iv = 4000, im = 2000;  // per-wave: 32*iv v_fma_f64 ; 8*im MFMA
    for (int rep = 0; rep < 2; ++rep)
        for (int mode = 0; mode < 4; ++mode) {
            hipLaunchKernelGGL(k, dim3(256), dim3(512), 0, 0, d, mode, iv, im);
            hipEventRecord(a);
            for (int r = 0; r < 5; ++r) hipLaunchKernelGGL(k, dim3(256), dim3(512), 0, 0, d, mode, iv, im);
            hipEventRecord(b);
            hipEventSynchronize(b);
            float ms;
            hipEventElapsedTime(&ms, a, b);
            ms /= 5;
            const double valu_flops = (mode == 0 ? 8 : mode == 2 ? 4 : mode == 3 ? 4 : 0) * 256.0 * 64 * 32.0 * iv * 2;
            const double mfma_flops = (mode == 1 ? 8 : mode == 2 ? 4 : mode == 3 ? 4 : 0) * 256.0 * 8.0 * im * 2048;
            printf("mode %d: %.3f ms  valu %.1f TF/s  mfma %.1f TF/s  total %.1f TF/s\n", mode, ms,
                   valu_flops / ms / 1e9, mfma_flops / ms / 1e9, (valu_flops + mfma_flops) / ms / 1e9);
        }
    hipFree(d);
    return 0;
}
