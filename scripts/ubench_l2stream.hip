// Microbenchmark: L2 -> CU streaming rate of the PT slice access pattern (pt_row_mfma3): every workgroup reads the
// SAME 1 MiB slice set (16 rows of 64 KiB, chi = 64 complex doubles) once per "step", wave w taking rows w, w + NW, ...;
// lane l reads Q[4 ks + (l >> 4)][16 g + (l & 15)] (g = 0..3: four 16-B loads per k-step, 4 KiB per wave and k-step).
// DEPTH = k-steps in flight per wave (register ring). Prints GB/s per CU and chip-wide: the ceiling the headline
// kernel's PT phase (1 MiB per workgroup-step at BT = 8) and the six-level one (2.25 MiB at BT = 4) stream against.
// build: hipcc --offload-arch=gfx950 -O3 -o ubench_l2stream ubench_l2stream.hip
#include <hip/hip_runtime.h>
#include <cstdio>

template <int DEPTH, int NW>
__global__ __launch_bounds__(64 * NW) void stream(const double2* __restrict__ Q, double* out, int steps, int nrows, int zero) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int kk = lane >> 4, c16 = lane & 15;
    double acc = 0.0;
    for (int s = 0; s < steps; ++s) {
        for (int r = wave; r < nrows; r += NW) {
            const double2* qp = Q + (size_t)(s * zero) + (size_t)r * 64 * 64 + (size_t)kk * 64 + c16;
            double2 ring[DEPTH][4];
#pragma unroll
            for (int f = 0; f < DEPTH; ++f)
#pragma unroll
                for (int g = 0; g < 4; ++g) ring[f][g] = qp[(size_t)4 * f * 64 + 16 * g];
#pragma unroll DEPTH
            for (int ks = 0; ks < 16; ++ks) {
                double2 v[4];
#pragma unroll
                for (int g = 0; g < 4; ++g) v[g] = ring[0][g];
#pragma unroll
                for (int f = 0; f + 1 < DEPTH; ++f)
#pragma unroll
                    for (int g = 0; g < 4; ++g) ring[f][g] = ring[f + 1][g];
                if (ks + DEPTH < 16) {
#pragma unroll
                    for (int g = 0; g < 4; ++g) ring[DEPTH - 1][g] = qp[(size_t)4 * (ks + DEPTH) * 64 + 16 * g];
                }
#pragma unroll
                for (int g = 0; g < 4; ++g) acc += v[g].x * v[g].y;
            }
        }
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
}

template <int DEPTH, int NW>
void run(const double2* Q, double* out, int wg_per_cu, int nrows) {
    const int steps = 400, grid = 256 * wg_per_cu;
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0); (void)hipEventCreate(&e1);
    hipLaunchKernelGGL((stream<DEPTH, NW>), dim3(grid), dim3(64 * NW), 0, 0, Q, out, 20, nrows, 0);
    (void)hipEventRecord(e0);
    hipLaunchKernelGGL((stream<DEPTH, NW>), dim3(grid), dim3(64 * NW), 0, 0, Q, out, steps, nrows, 0);
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    float ms = 0;
    (void)hipEventElapsedTime(&ms, e0, e1);
    const double bytes = (double)grid * steps * nrows * 65536.0;
    printf("rows %2d  waves/WG %2d  WG/CU %d  depth %d: %8.3f ms  %7.1f GB/s per CU  %6.2f TB/s chip  (%.2f us per WG-step)\n",
           nrows, NW, wg_per_cu, DEPTH, ms, bytes / (ms * 1e-3) / 256 / 1e9, bytes / (ms * 1e-3) / 1e12,
           1e3 * ms / steps);
}

int main() {
    double2* Q;
    double* out;
    (void)hipMalloc(&Q, (size_t)36 * 65536);
    (void)hipMalloc(&out, (size_t)512 * 1024 * sizeof(double));
    (void)hipMemset(Q, 0, (size_t)36 * 65536);
    for (int nrows : {16, 36}) {
        run<1, 8>(Q, out, 1, nrows);
        run<2, 8>(Q, out, 1, nrows);
        run<4, 8>(Q, out, 1, nrows);
        run<2, 16>(Q, out, 1, nrows);
        run<4, 16>(Q, out, 1, nrows);
        run<2, 8>(Q, out, 2, nrows);
        run<2, 4>(Q, out, 2, nrows);
    }
    return 0;
}
