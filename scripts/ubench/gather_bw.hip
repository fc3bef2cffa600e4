// Microbenchmark: the multi-trajectory split gather's load pattern (pt_msplit.hip) in isolation.
// 256 workgroups x 512 threads (one per CU by a 96 KiB LDS request); per iteration each thread issues 16 buffer loads
// of 16 B (4 "trajectories" x 4 rows: thread (w, c, rg) reads row rg + 4 i, column 16 (w % 4) + c of a 16 x 64
// element slot), i.e. 128 KiB per workgroup, then sums them. Modes choose which workgroups share a region:
//   0: the 8 workgroups of a "group" (blocks b with equal b % 8 and (b / 8) / 8) read one 128 KiB region
//   1: every workgroup its own region (32 MiB in all)
//   2: all workgroups of an XCD slot (b % 8) one region
// aux: 0 plain loads, 16 sc1 loads; coalesced 0: lanes 4 c + rg (consecutive lanes 1 KiB apart), 1: lanes c + 16 rg.
// Prints cycles per iteration per workgroup and B/clk/CU.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>

typedef unsigned int v4u __attribute__((ext_vector_type(4)));

template <int AUX, bool COAL>
__global__ __launch_bounds__(512) void gather_k(const double* __restrict__ X, int mode, int iters, double* out,
                                                unsigned long long* cyc) {
    extern __shared__ double lds[];
    const int b = blockIdx.x, tid = threadIdx.x, h = tid / 256, ht = tid & 255, kq = ht / 64, j = ht & 63;
    // COAL: 16 consecutive lanes read 16 consecutive elements of one row (256 B); else lanes 4 c + rg, as pt_msplit's
    // first gather (consecutive lanes 1 KiB apart)
    const int cg = COAL ? (j & 15) : j / 4, rg = COAL ? (j >> 4) : (j & 3), kcol = kq * 16 + cg;
    int region;
    if (mode == 0) region = (b & 7) + 8 * ((b >> 3) >> 3);
    else if (mode == 1) region = b;
    else region = b & 7;
    const char* base = (const char*)X + (size_t)region * 128 * 1024;
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void*)base, 0, 128 * 1024, 0x00020000);
    double acc = 0;
    unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int it = 0; it < iters; ++it) {
        v4u xr[4][4];
#pragma unroll
        for (int bb = 0; bb < 4; ++bb)
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const int traj = h + 2 * bb;
                const int off = ((traj * 16 + rg + 4 * i) * 64 + kcol) * 16;
                xr[bb][i] = __builtin_amdgcn_raw_buffer_load_b128(rs, off, 0, AUX);
            }
#pragma unroll
        for (int bb = 0; bb < 4; ++bb)
#pragma unroll
            for (int i = 0; i < 4; ++i) acc += __uint_as_float(xr[bb][i].x) + __uint_as_float(xr[bb][i].z);
        __syncthreads();
    }
    unsigned long long t1 = __builtin_amdgcn_s_memtime();
    lds[tid] = acc;
    __syncthreads();
    if (tid == 0) {
        double s = 0;
        for (int i = 0; i < 512; ++i) s += lds[i];
        out[b] = s;
        cyc[b] = t1 - t0;
    }
}

int main(int argc, char** argv) {
    const int iters = argc > 1 ? atoi(argv[1]) : 200;
    double* X;
    double* out;
    unsigned long long* cyc;
    const size_t bytes = (size_t)256 * 128 * 1024;
    hipMalloc(&X, bytes);
    hipMemset(X, 0, bytes);
    hipMalloc(&out, 256 * sizeof(double));
    hipMalloc(&cyc, 256 * sizeof(unsigned long long));
    hipFuncSetAttribute((const void*)gather_k<0, false>, hipFuncAttributeMaxDynamicSharedMemorySize, 96 * 1024);
    hipFuncSetAttribute((const void*)gather_k<16, false>, hipFuncAttributeMaxDynamicSharedMemorySize, 96 * 1024);
    hipFuncSetAttribute((const void*)gather_k<0, true>, hipFuncAttributeMaxDynamicSharedMemorySize, 96 * 1024);
    hipFuncSetAttribute((const void*)gather_k<16, true>, hipFuncAttributeMaxDynamicSharedMemorySize, 96 * 1024);
    std::vector<unsigned long long> hc(256);
    for (int coal : {0, 1})
        for (int aux : {16, 0})
            for (int mode : {0, 1, 2}) {
                for (int rep = 0; rep < 2; ++rep) {
                    auto k = coal ? (aux == 16 ? gather_k<16, true> : gather_k<0, true>)
                                  : (aux == 16 ? gather_k<16, false> : gather_k<0, false>);
                    hipLaunchKernelGGL(k, dim3(256), dim3(512), 96 * 1024, 0, X, mode, iters, out, cyc);
                    hipDeviceSynchronize();
                }
                hipMemcpy(hc.data(), cyc, 256 * sizeof(unsigned long long), hipMemcpyDeviceToHost);
                double mean = 0, mx = 0;
                for (auto c : hc) { mean += (double)c; mx = (double)c > mx ? (double)c : mx; }
                mean /= 256;
                // s_memtime counts shader clocks here (msplit stamps: 23,400 per 10.1 us step)
                printf("coalesced %d aux %2d mode %d: %.0f cycles per iteration (mean), max %.0f; %.1f B per cycle per CU\n",
                       coal, aux, mode, mean / iters, mx / iters, 131072.0 / (mean / iters));
            }
    return 0;
}
