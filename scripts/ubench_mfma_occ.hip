// Microbenchmark: FP64 MFMA issue rate at ONE vs TWO waves per SIMD (ubench_mfma44 measured two), for
// v_mfma_f64_4x4x4_4b and v_mfma_f64_16x16x4, NCH independent accumulator chains per wave, optionally with one
// v_add_f64 per MFMA on an operand (the 3M operand sums of pt_quad). All 256 CUs, 4 or 8 waves per CU.
// Prints TF/s and shader cycles per MFMA per wave (s_memtime).
#include <hip/hip_runtime.h>
#include <cstdio>
typedef double dbl4 __attribute__((ext_vector_type(4)));

template <int NCH, bool ADD>
__global__ void k44(double* out, unsigned long long* cyc, int iters) {
    double c[NCH];
    double a = 1e-9 * threadIdx.x, b = 1.0 - 1e-12;
#pragma unroll
    for (int i = 0; i < NCH; ++i) c[i] = i;
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int i = 0; i < NCH; ++i) {
            if constexpr (ADD) a = a + 1e-30;
            c[i] = __builtin_amdgcn_mfma_f64_4x4x4f64(a, b, c[i], 0, 0, 0);
        }
    }
    double s = 0;
#pragma unroll
    for (int i = 0; i < NCH; ++i) s += c[i];
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
    if ((threadIdx.x & 63) == 0) cyc[blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64] = t1 - t0;
}

template <int NCH, bool ADD>
__global__ void k16(double* out, unsigned long long* cyc, int iters) {
    dbl4 c[NCH];
    double a = 1e-9 * threadIdx.x, b = 1.0 - 1e-12;
#pragma unroll
    for (int i = 0; i < NCH; ++i) c[i] = dbl4{(double)i, 0, 0, 0};
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int i = 0; i < NCH; ++i) {
            if constexpr (ADD) a = a + 1e-30;
            c[i] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c[i], 0, 0, 0);
        }
    }
    double s = 0;
#pragma unroll
    for (int i = 0; i < NCH; ++i) s += c[i][0] + c[i][3];
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
    if ((threadIdx.x & 63) == 0) cyc[blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64] = t1 - t0;
}

template <typename K>
void run(const char* name, K kern, int wps, int iters, int nch, double flop_per_mfma, double* dout,
         unsigned long long* dcyc) {
    const int threads = 64 * 4 * wps;
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0); (void)hipEventCreate(&e1);
    hipLaunchKernelGGL(kern, dim3(256), dim3(threads), 0, 0, dout, dcyc, iters);
    (void)hipEventRecord(e0);
    hipLaunchKernelGGL(kern, dim3(256), dim3(threads), 0, 0, dout, dcyc, iters);
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    float ms;
    (void)hipEventElapsedTime(&ms, e0, e1);
    unsigned long long h[64];
    (void)hipMemcpy(h, dcyc, sizeof(h), hipMemcpyDeviceToHost);
    double cy = 0;
    for (int i = 0; i < 4 * wps; ++i) cy += (double)h[i];
    cy /= 4 * wps;
    const double n_mfma = (double)iters * nch;
    printf("%-28s waves/SIMD %d: %7.3f ms  %6.1f TF/s  %6.1f cycles per MFMA per wave\n", name, wps, ms,
           256.0 * 4 * wps * n_mfma * flop_per_mfma / ms / 1e9, cy / n_mfma);
}

int main() {
    double* dout;
    unsigned long long* dcyc;
    (void)hipMalloc(&dout, 256 * 512 * 8);
    (void)hipMalloc(&dcyc, 256 * 8 * 8);
    const int it = 4000;
    for (int wps = 1; wps <= 2; ++wps) {
        run("4x4x4_4b nch=8", k44<8, false>, wps, it, 8, 512, dout, dcyc);
        run("4x4x4_4b nch=12", k44<12, false>, wps, it, 12, 512, dout, dcyc);
        run("4x4x4_4b nch=12 +add", k44<12, true>, wps, it, 12, 512, dout, dcyc);
        run("16x16x4 nch=4", k16<4, false>, wps, it / 4, 4, 2048, dout, dcyc);
        run("16x16x4 nch=8", k16<8, false>, wps, it / 4, 8, 2048, dout, dcyc);
        run("16x16x4 nch=8 +add", k16<8, true>, wps, it / 4, 8, 2048, dout, dcyc);
    }
    return 0;
}
