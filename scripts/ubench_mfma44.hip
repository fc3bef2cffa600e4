// (1) lane layout of v_mfma_f64_4x4x4_4b_f64 (dump A, B, D for random inputs; the host script infers the map)
// (2) throughput of 4x4x4_4b vs 16x16x4 f64 MFMA, all CUs, 8 waves per CU.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
typedef double dbl4 __attribute__((ext_vector_type(4)));

__global__ void layout(const double* a, const double* b, double* d) {
    const int l = threadIdx.x;
    double acc = 0;
    acc = __builtin_amdgcn_mfma_f64_4x4x4f64(a[l], b[l], acc, 0, 0, 0);
    d[l] = acc;
}

__global__ __launch_bounds__(512) void tp44(double* out, int iters) {
    double c[8];
    const double a = 1e-9 * threadIdx.x, b = 1.0 - 1e-12;
#pragma unroll
    for (int i = 0; i < 8; ++i) c[i] = i;
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int i = 0; i < 8; ++i) c[i] = __builtin_amdgcn_mfma_f64_4x4x4f64(a, b, c[i], 0, 0, 0);
    }
    double s = 0;
#pragma unroll
    for (int i = 0; i < 8; ++i) s += c[i];
    out[blockIdx.x * 512 + threadIdx.x] = s;
}

__global__ __launch_bounds__(512) void tp16(double* out, int iters) {
    dbl4 c[4];
    const double a = 1e-9 * threadIdx.x, b = 1.0 - 1e-12;
#pragma unroll
    for (int i = 0; i < 4; ++i) c[i] = dbl4{(double)i, 0, 0, 0};
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int i = 0; i < 4; ++i) c[i] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c[i], 0, 0, 0);
    }
    out[blockIdx.x * 512 + threadIdx.x] = c[0][0] + c[1][1] + c[2][2] + c[3][3];
}

int main() {
    double ha[64], hb[64], hd[64];
    srand(7);
    for (int i = 0; i < 64; ++i) { ha[i] = (rand() % 1000) / 100.0; hb[i] = (rand() % 1000) / 100.0; }
    double *da, *db, *dd, *dout;
    (void)hipMalloc(&da, 512); (void)hipMalloc(&db, 512); (void)hipMalloc(&dd, 512);
    (void)hipMalloc(&dout, 256 * 512 * 8);
    (void)hipMemcpy(da, ha, 512, hipMemcpyHostToDevice);
    (void)hipMemcpy(db, hb, 512, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(layout, dim3(1), dim3(64), 0, 0, da, db, dd);
    (void)hipMemcpy(hd, dd, 512, hipMemcpyDeviceToHost);
    printf("A");
    for (int i = 0; i < 64; ++i) printf(" %.2f", ha[i]);
    printf("\nB");
    for (int i = 0; i < 64; ++i) printf(" %.2f", hb[i]);
    printf("\nD");
    for (int i = 0; i < 64; ++i) printf(" %.6f", hd[i]);
    printf("\n");
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0); (void)hipEventCreate(&e1);
    const int iters = 4000;
    for (int rep = 0; rep < 2; ++rep) {
        float ms;
        hipLaunchKernelGGL(tp44, dim3(256), dim3(512), 0, 0, dout, iters);
        (void)hipEventRecord(e0);
        hipLaunchKernelGGL(tp44, dim3(256), dim3(512), 0, 0, dout, iters);
        (void)hipEventRecord(e1); (void)hipEventSynchronize(e1); (void)hipEventElapsedTime(&ms, e0, e1);
        printf("4x4x4_4b: %.3f ms  %.1f TF/s\n", ms, 256.0 * 8 * iters * 8 * 256 * 2 / ms / 1e9);
        hipLaunchKernelGGL(tp16, dim3(256), dim3(512), 0, 0, dout, iters);
        (void)hipEventRecord(e0);
        hipLaunchKernelGGL(tp16, dim3(256), dim3(512), 0, 0, dout, iters);
        (void)hipEventRecord(e1); (void)hipEventSynchronize(e1); (void)hipEventElapsedTime(&ms, e0, e1);
        printf("16x16x4: %.3f ms  %.1f TF/s\n", ms, 256.0 * 8 * iters * 4 * 1024 * 2 / ms / 1e9);
    }
    return 0;
}
