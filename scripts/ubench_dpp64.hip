// Microbenchmark: FP64 VALU FMAs whose first operand is broadcast from another lane of the 16-lane row by the DPP64
// modifier (v_fmac_f64_dpp ... row_newbcast:n), alone and beside v_mfma_f64_16x16x4 in the other wave of each SIMD.
// This is the instruction a VALU PT row needs when every lane owns one output column and the row's state elements
// X[b][k] are broadcast from the lanes that read them (no LDS broadcast reads). 256 workgroups x 8 waves
// (2 per SIMD: waves w and w + 4 share SIMD w). Modes:
//   0: all waves DPP FMAs          1: all waves plain v_fmac_f64
//   2: waves 0-3 16x16x4, 4-7 DPP FMAs    3: waves 0-3 16x16x4, 4-7 plain FMAs
//   4: waves 0-3 16x16x4, 4-7 exit        5: waves 0-3 exit, 4-7 DPP FMAs
// Per wave class: shader cycles (s_memtime) of its loop and the TF/s it reaches over the whole chip.
#include <hip/hip_runtime.h>
#include <cstdio>
typedef double dbl4 __attribute__((ext_vector_type(4)));

#define FD(I) asm volatile("v_fmac_f64_dpp %0, %1, %2 row_newbcast:" #I " row_mask:0xf bank_mask:0xf" : "+v"(a[I]) : "v"(x), "v"(q))
#define FP(I) asm volatile("v_fmac_f64 %0, %1, %2" : "+v"(a[I]) : "v"(x), "v"(q))

template <bool DPP>
__device__ __forceinline__ double valu_work(int iters, double seed) {
    double a[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) a[i] = seed + i;
    double x = seed * 1e-9, q = 1.0 - 1e-12;
    asm volatile("s_nop 4" ::: "memory");
    for (int it = 0; it < iters; ++it) {
        if constexpr (DPP) {
            FD(0); FD(1); FD(2); FD(3); FD(4); FD(5); FD(6); FD(7);
            FD(8); FD(9); FD(10); FD(11); FD(12); FD(13); FD(14); FD(15);
            FD(0); FD(1); FD(2); FD(3); FD(4); FD(5); FD(6); FD(7);
            FD(8); FD(9); FD(10); FD(11); FD(12); FD(13); FD(14); FD(15);
        } else {
            FP(0); FP(1); FP(2); FP(3); FP(4); FP(5); FP(6); FP(7);
            FP(8); FP(9); FP(10); FP(11); FP(12); FP(13); FP(14); FP(15);
            FP(0); FP(1); FP(2); FP(3); FP(4); FP(5); FP(6); FP(7);
            FP(8); FP(9); FP(10); FP(11); FP(12); FP(13); FP(14); FP(15);
        }
    }
    double s = 0;
#pragma unroll
    for (int i = 0; i < 16; ++i) s += a[i];
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

__global__ __launch_bounds__(512) void k(double* out, unsigned long long* cyc, int mode, int iv, int im) {
    const int wave = threadIdx.x >> 6;
    const double seed = 1.0 + threadIdx.x * 1e-3;
    double r = 0;
    const bool lo = wave < 4;
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    if (mode == 0) r = valu_work<true>(iv, seed);
    else if (mode == 1) r = valu_work<false>(iv, seed);
    else if (mode == 2) r = lo ? m16_work(im, seed) : valu_work<true>(iv, seed);
    else if (mode == 3) r = lo ? m16_work(im, seed) : valu_work<false>(iv, seed);
    else if (mode == 4) { if (lo) r = m16_work(im, seed); }
    else { if (!lo) r = valu_work<true>(iv, seed); }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    out[blockIdx.x * 512 + threadIdx.x] = r;
    if ((threadIdx.x & 63) == 0) cyc[blockIdx.x * 8 + wave] = t1 - t0;
}

int main() {
    double* d;
    unsigned long long* c;
    (void)hipMalloc(&d, 256 * 512 * sizeof(double));
    (void)hipMalloc(&c, 256 * 8 * sizeof(unsigned long long));
    unsigned long long hc[256 * 8];
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    const int iv = 4000, im = 4000;
    // per wave: VALU 32 FMAs x 64 lanes x 2 flops per iteration; 16x16x4 8 MFMAs x 16x16x4 x 2 flops per iteration
    const double fv = 64.0 * 32 * 2 * iv, fm = 8.0 * 16 * 16 * 4 * 2 * im;
    const char* names[] = {"all DPP FMA", "all plain FMA", "16x16x4 | DPP FMA", "16x16x4 | plain FMA",
                           "16x16x4 alone (1/SIMD)", "DPP FMA alone (1/SIMD)"};
    for (int rep = 0; rep < 2; ++rep)
        for (int mode = 0; mode < 6; ++mode) {
            hipLaunchKernelGGL(k, dim3(256), dim3(512), 0, 0, d, c, mode, iv, im);
            (void)hipEventRecord(a);
            hipLaunchKernelGGL(k, dim3(256), dim3(512), 0, 0, d, c, mode, iv, im);
            (void)hipEventRecord(b);
            (void)hipEventSynchronize(b);
            float ms;
            (void)hipEventElapsedTime(&ms, a, b);
            (void)hipMemcpy(hc, c, sizeof(hc), hipMemcpyDeviceToHost);
            double clo = 0, chi = 0;
            for (int w = 0; w < 256 * 8; ++w) ((w & 7) < 4 ? clo : chi) += (double)hc[w];
            clo /= 1024; chi /= 1024;
            const bool mlo = mode >= 2 && mode <= 4, vlo = mode <= 1, vhi = mode <= 3 || mode == 5;
            double flo = mlo ? fm : (vlo ? fv : 0), fhi = vhi ? fv : 0;
            const double tf = (1024 * flo + 1024 * fhi) / (ms * 1e-3) / 1e12;
            // per-class rate: the class's own loop time = wall x (its s_memtime cycles / the longer class's)
            const double cm = clo > chi ? clo : chi;
            const double tlo = ms * 1e-3 * clo / cm, thi = ms * 1e-3 * chi / cm;
            printf("%-26s %8.3f ms  total %6.1f TF/s | waves 0-3: %9.0f cyc %6.1f TF/s | waves 4-7: %9.0f cyc %6.1f TF/s\n",
                   names[mode], ms, tf, clo, clo > 0 && flo > 0 ? 1024 * flo / tlo / 1e12 : 0.0, chi,
                   chi > 0 && fhi > 0 ? 1024 * fhi / thi / 1e12 : 0.0);
        }
    return 0;
}
