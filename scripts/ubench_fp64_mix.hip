// Microbenchmark: FP64 pipe co-issue on gfx950 for the PT-contraction instruction mix.
// 256 workgroups x 8 waves (2 per SIMD). Modes:
//   0: all waves v_mfma_f64_4x4x4_4b (8 independent accumulators)
//   1: all waves v_mfma_f64_4x4x4_4b (16 independent accumulators)
//   2: all waves v_fma_f64
//   3: waves 0-3 v_fma_f64, waves 4-7 4x4x4_4b (one of each per SIMD)
//   4: waves 0-3 v_fma_f64, waves 4-7 16x16x4 (reference: known to overlap)
//   5: every wave interleaves 4x4x4_4b and v_fma_f64 in one instruction stream
#include <hip/hip_runtime.h>
#include <cstdio>
typedef double dbl4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ double valu_work(int iters, double seed) {
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
    return s;
}

template <int NA>
__device__ __forceinline__ double m44_work(int iters, double seed) {  // 8 MFMAs per iteration
    double c[NA];
#pragma unroll
    for (int i = 0; i < NA; ++i) c[i] = seed + i;
    const double a = 1e-9 * seed, b = 1.0 - 1e-12;
    for (int it = 0; it < iters; it += NA / 8) {
#pragma unroll
        for (int i = 0; i < NA; ++i) c[i] = __builtin_amdgcn_mfma_f64_4x4x4f64(a, b, c[i], 0, 0, 0);
    }
    double s = 0;
#pragma unroll
    for (int i = 0; i < NA; ++i) s += c[i];
    return s;
}

__device__ __forceinline__ double m16_work(int iters, double seed) {  // 8 MFMAs per iteration
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
    return c[0][0] + c[1][1] + c[2][2] + c[3][3];
}

__device__ __forceinline__ double mixed_work(int iters, double seed) {  // per iteration: 8 MFMA 4x4x4 + 32 v_fma
    double c[8], a[16];
#pragma unroll
    for (int i = 0; i < 8; ++i) c[i] = seed + i;
#pragma unroll
    for (int i = 0; i < 16; ++i) a[i] = seed - i;
    const double x = 1e-9 * seed, y = 1.0 - 1e-12;
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            c[i] = __builtin_amdgcn_mfma_f64_4x4x4f64(x, y, c[i], 0, 0, 0);
            a[2 * i] = fma(a[2 * i], y, x);
            a[2 * i + 1] = fma(a[2 * i + 1], y, x);
            a[2 * i] = fma(a[2 * i], y, x);
            a[2 * i + 1] = fma(a[2 * i + 1], y, x);
        }
    }
    double s = 0;
#pragma unroll
    for (int i = 0; i < 8; ++i) s += c[i];
#pragma unroll
    for (int i = 0; i < 16; ++i) s += a[i];
    return s;
}

__global__ __launch_bounds__(512) void k(double* out, int mode, int iv, int im) {
    const int wave = threadIdx.x >> 6;
    const double seed = 1.0 + threadIdx.x * 1e-3;
    double r = 0;
    if (mode == 0) r = m44_work<8>(im, seed);
    else if (mode == 1) r = m44_work<16>(im, seed);
    else if (mode == 2) r = valu_work(iv, seed);
    else if (mode == 3) r = wave < 4 ? valu_work(iv, seed) : m44_work<8>(im, seed);
    else if (mode == 4) r = wave < 4 ? valu_work(iv, seed) : m16_work(im / 4, seed);
    else r = mixed_work(im, seed);
    out[blockIdx.x * 512 + threadIdx.x] = r;
}

int main() {
    double* d;
    (void)hipMalloc(&d, 256 * 512 * sizeof(double));
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    const int iv = 2000, im = 4000;
    // flops per wave: valu 64*32*iv*2 ; 4x4x4: 8*im*512 ; 16x16x4: 8*(im/4)*2048*2... (=m44 flops)
    const double fv = 64.0 * 32 * iv * 2, f44 = 8.0 * im * 512, f16 = 8.0 * (im / 4) * 4096;
    const char* names[] = {"4x4x4 (8 acc)", "4x4x4 (16 acc)", "valu", "valu|4x4x4 waves", "valu|16x16x4 waves",
                           "4x4x4+valu interleaved"};
    for (int rep = 0; rep < 2; ++rep)
        for (int mode = 0; mode < 6; ++mode) {
            hipLaunchKernelGGL(k, dim3(256), dim3(512), 0, 0, d, mode, iv, im);
            (void)hipEventRecord(a);
            for (int r = 0; r < 5; ++r) hipLaunchKernelGGL(k, dim3(256), dim3(512), 0, 0, d, mode, iv, im);
            (void)hipEventRecord(b);
            (void)hipEventSynchronize(b);
            float ms;
            (void)hipEventElapsedTime(&ms, a, b);
            ms /= 5;
            double fl = 0;
            if (mode == 0 || mode == 1) fl = 8 * f44;
            else if (mode == 2) fl = 8 * fv;
            else if (mode == 3) fl = 4 * fv + 4 * f44;
            else if (mode == 4) fl = 4 * fv + 4 * f16;
            else fl = 8 * (f44 + 64.0 * 32 * im * 2);
            printf("mode %d %-24s %.3f ms  %.1f TF/s\n", mode, names[mode], ms, 256.0 * fl / ms / 1e9);
        }
    (void)hipFree(d);
    return 0;
}
