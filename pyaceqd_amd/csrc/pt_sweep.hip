// pt_sweep.hip — the hot path: lock-step propagation of a batch of trajectories through the
// process-tensor MPO (PT contraction + symmetric-Trotter free half steps + MTOs + output traces).
//
// Replaces the per-step loop inside the external ACE binary that pyaceqd drives through
// system_ace_stream (general_system.py:227-343) and fans out one OS process per trajectory in the
// two-time sweeps (two_time/correlations.py:135-184, pol_entanglement/G2.py:439-533, ...).
//
// Work decomposition (MI355X: 256 CUs, 160 KiB LDS/CU, 64-wide waves, FP64 VALU = FP64 MFMA peak):
//   * one workgroup owns BT trajectories (8 at N2 <= 16, else 4) for the whole time range (persistent over
//     steps, no inter-workgroup traffic: trajectories are independent); 8 waves per workgroup (one per
//     trajectory at BT = 8, two per trajectory at BT = 4 and chi >= 32, see sweep_wpt);
//   * the augmented states Q_b[alpha][d] (N2 x CHI complex doubles, 16 KiB each at N=4, chi=64) stay
//     resident in LDS, rows padded to CHI+1 so column reads and row reads are bank-conflict free;
//   * free half steps / MTOs (N2 x N2 operator applied to every bond column): the waves of a trajectory
//     run the complex GEMM M . Q on the FP64 matrix cores (v_mfma_f64_16x16x4_f64, 3 real MFMAs per complex
//     tile by default), no cross-wave traffic, no barrier inside the phase; steps without MTOs apply the
//     fused operator F(n) = M_a(n) M_b(n-1) once;
//   * PT contraction (row alpha of all BT trajectories times the chi x chi slice Q[g(alpha)]): waves take the
//     rows (or up to 4 rows sharing a dictionary slice) of a host-built unit list; v_mfma_f64_4x4x4_4b with
//     3 real products per complex product, every slice element read from L2 once per workgroup and step;
//   * closure + output traces only on steps inside some trajectory's output window.
// All PT slices / free propagators are shared by every workgroup at the same absolute step, so the
// dominant traffic is L2/MALL-resident; the kernel is FP64 matrix-core bound.
#include "pqd_common.h"
#include <climits>

namespace {

template <int N2, int CHI, int BT>
struct SweepLayout {
    static constexpr int RS = CHI + 1;          // row stride (double2)
    static constexpr int TS = N2 * RS + 4;      // trajectory stride (+64 B: shifts banks per trajectory)
    static constexpr int KD = CHI / 16;         // PT output columns per lane
    static constexpr int NCOL = BT * CHI;       // column-phase work items
    static constexpr int WPT = sweep_wpt(N2, BT, CHI);  // waves per trajectory
    static constexpr int NW = BT * WPT;             // waves per workgroup
    static constexpr size_t LDS = (size_t)(BT * TS + BT * N2) * sizeof(double2);
};

typedef double dbl4 __attribute__((ext_vector_type(4)));

// Column phase on the matrix cores: one wave applies the N2 x N2 operator Op (row-major, complex) to
// all CHI bond columns of its trajectory's augmented state S (LDS, row stride RS):
//   C[N2 x CHI] = Op[N2 x N2] . S[N2 x CHI]   as v_mfma_f64_16x16x4_f64 tiles,
// complex = 4 real MFMAs (Cr += Ar Br - Ai Bi, Ci += Ar Bi + Ai Br). Fragment maps (gfx950 f64):
// A[i = l&15][k = l>>4], B[k = l>>4][j = l&15], C[i = (l>>4) + 4 r][j = l&15].
// Column tiles are the outer loop, so each 16-column tile is read completely before it is written
// back in place. With WPT waves per trajectory, wave `half` takes every WPT-th tile (columns are
// independent). Rows/k beyond N2 are zero padding (N2 = 4, 9, 25, 36).
template <int N2, int CHI, int RS, int WPT = 1>
__device__ __forceinline__ void col_apply_mfma(const double2* __restrict__ Op, double2* S, int lane, int half = 0) {
    constexpr int MT = (N2 + 15) / 16;   // output row tiles
    constexpr int KS = (N2 + 3) / 4;     // k steps
    constexpr int NTL = CHI / 16;        // column tiles
    constexpr bool CACHE_A = KS * MT <= 8;
    constexpr int KSU = CACHE_A ? KS : 3;   // large N2: bounded unroll keeps the operator loads out of VGPRs
    const int li = lane & 15, lk = lane >> 4;
    double2 ac[CACHE_A ? KS * MT : 1];
    if constexpr (CACHE_A) {
#pragma unroll
        for (int ks = 0; ks < KS; ++ks)
#pragma unroll
            for (int mt = 0; mt < MT; ++mt) {
                const int r = 16 * mt + li, a = 4 * ks + lk;
                ac[ks * MT + mt] = (r < N2 && a < N2) ? Op[r * N2 + a] : c_zero();
            }
    }
#pragma unroll
    for (int j = 0; j < NTL / WPT; ++j) {   // this wave's column tiles: half, half + WPT, ...
        const int nt = j * WPT + half;
        dbl4 cr[MT], ci[MT];
#pragma unroll
        for (int mt = 0; mt < MT; ++mt) { cr[mt] = dbl4{0, 0, 0, 0}; ci[mt] = dbl4{0, 0, 0, 0}; }
#pragma unroll KSU
        for (int ks = 0; ks < KS; ++ks) {
            const int a = 4 * ks + lk;
            const double2 b = (a < N2) ? S[a * RS + 16 * nt + li] : c_zero();
#pragma unroll
            for (int mt = 0; mt < MT; ++mt) {
                double2 m;
                if constexpr (CACHE_A) {
                    m = ac[ks * MT + mt];
                } else {
                    const int r = 16 * mt + li;
                    m = (r < N2 && a < N2) ? Op[r * N2 + a] : c_zero();
                }
                cr[mt] = __builtin_amdgcn_mfma_f64_16x16x4f64(m.x, b.x, cr[mt], 0, 0, 0);
                cr[mt] = __builtin_amdgcn_mfma_f64_16x16x4f64(-m.y, b.y, cr[mt], 0, 0, 0);
                ci[mt] = __builtin_amdgcn_mfma_f64_16x16x4f64(m.x, b.y, ci[mt], 0, 0, 0);
                ci[mt] = __builtin_amdgcn_mfma_f64_16x16x4f64(m.y, b.x, ci[mt], 0, 0, 0);
            }
        }
#pragma unroll
        for (int mt = 0; mt < MT; ++mt)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int row = 16 * mt + lk + 4 * r;
                if (row < N2) S[row * RS + 16 * nt + li] = make_double2(cr[mt][r], ci[mt][r]);
            }
    }
    // the next operator of this wave re-reads what other lanes just wrote
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
}

// Column phase with three real products per complex product ("3M"): P1 = Ar Br, P2 = Ai Bi,
// P3 = (Ar + Ai)(Br + Bi); Cr = P1 - P2, Ci = P3 - P1 - P2. Three MFMA chains instead of four, the sums are
// two VALU adds per operand fragment. Error bound eps (|Ar||Br| + |Ai||Bi| + |Ar + Ai||Br + Bi|) per product,
// i.e. the same order as the 4M form for these O(1) propagators.
template <int N2, int CHI, int RS, int WPT = 1>
__device__ __forceinline__ void col_apply_mfma3(const double2* __restrict__ Op, double2* S, int lane, int half = 0) {
    constexpr int MT = (N2 + 15) / 16;
    constexpr int KS = (N2 + 3) / 4;
    constexpr int NTL = CHI / 16;
    constexpr bool CACHE_A = KS * MT <= 8;
    constexpr int KSU = CACHE_A ? KS : 3;   // large N2: bounded unroll keeps the operator loads out of VGPRs
    const int li = lane & 15, lk = lane >> 4;
    double2 ac[CACHE_A ? KS * MT : 1];
    double as[CACHE_A ? KS * MT : 1];
    if constexpr (CACHE_A) {
#pragma unroll
        for (int ks = 0; ks < KS; ++ks)
#pragma unroll
            for (int mt = 0; mt < MT; ++mt) {
                const int r = 16 * mt + li, a = 4 * ks + lk;
                ac[ks * MT + mt] = (r < N2 && a < N2) ? Op[r * N2 + a] : c_zero();
                as[ks * MT + mt] = ac[ks * MT + mt].x + ac[ks * MT + mt].y;
            }
    }
#pragma unroll
    for (int j = 0; j < NTL / WPT; ++j) {   // this wave's column tiles: half, half + WPT, ...
        const int nt = j * WPT + half;
        dbl4 p1[MT], p2[MT], p3[MT];
#pragma unroll
        for (int mt = 0; mt < MT; ++mt) { p1[mt] = dbl4{0, 0, 0, 0}; p2[mt] = p1[mt]; p3[mt] = p1[mt]; }
#pragma unroll KSU
        for (int ks = 0; ks < KS; ++ks) {
            const int a = 4 * ks + lk;
            const double2 b = (a < N2) ? S[a * RS + 16 * nt + li] : c_zero();
            const double bs = b.x + b.y;
#pragma unroll
            for (int mt = 0; mt < MT; ++mt) {
                double2 m;
                double ms;
                if constexpr (CACHE_A) {
                    m = ac[ks * MT + mt];
                    ms = as[ks * MT + mt];
                } else {
                    const int r = 16 * mt + li;
                    m = (r < N2 && a < N2) ? Op[r * N2 + a] : c_zero();
                    ms = m.x + m.y;
                }
                p1[mt] = __builtin_amdgcn_mfma_f64_16x16x4f64(m.x, b.x, p1[mt], 0, 0, 0);
                p2[mt] = __builtin_amdgcn_mfma_f64_16x16x4f64(m.y, b.y, p2[mt], 0, 0, 0);
                p3[mt] = __builtin_amdgcn_mfma_f64_16x16x4f64(ms, bs, p3[mt], 0, 0, 0);
            }
        }
#pragma unroll
        for (int mt = 0; mt < MT; ++mt)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int row = 16 * mt + lk + 4 * r;
                if (row < N2)
                    S[row * RS + 16 * nt + li] = make_double2(p1[mt][r] - p2[mt][r], p3[mt][r] - p1[mt][r] - p2[mt][r]);
            }
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
}

// col_apply_mfma3 for large N2 (25, 36: the operator's fragments do not fit in VGPRs): all of this wave's column tiles
// in one pass over k, so every operator fragment is loaded from L2 once per call instead of once per tile, with the
// next k-step's fragments in flight while the current one's MFMAs run (the per-tile loop waited on each load:
// six-level scan, column phases ~24 us per step against ~9 us of MFMA work). Accumulators: 3 MT NTW tiles <= 18.
template <int N2, int CHI, int RS, int WPT>
constexpr bool col_big_ok() {
    return (N2 + 3) / 4 * ((N2 + 15) / 16) > 8 && 3 * ((N2 + 15) / 16) * (CHI / 16 / WPT) <= 18;
}
template <int N2, int CHI, int RS, int WPT>
__device__ __forceinline__ void col_apply_mfma3_big(const double2* __restrict__ Op, double2* S, int lane, int half) {
    constexpr int MT = (N2 + 15) / 16;
    constexpr int KS = (N2 + 3) / 4;
    constexpr int NTW = CHI / 16 / WPT;   // this wave's column tiles: half, half + WPT, ...
    const int li = lane & 15, lk = lane >> 4;
    dbl4 p1[MT][NTW], p2[MT][NTW], p3[MT][NTW];
#pragma unroll
    for (int mt = 0; mt < MT; ++mt)
#pragma unroll
        for (int j = 0; j < NTW; ++j) { p1[mt][j] = dbl4{0, 0, 0, 0}; p2[mt][j] = p1[mt][j]; p3[mt][j] = p1[mt][j]; }
    auto ldm = [&](int ks, int mt) {
        const int r = 16 * mt + li, a = 4 * ks + lk;
        return (r < N2 && a < N2) ? Op[r * N2 + a] : c_zero();
    };
    double2 mn[MT];
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) mn[mt] = ldm(0, mt);
#pragma unroll 3
    for (int ks = 0; ks < KS; ++ks) {
        double2 m[MT];
#pragma unroll
        for (int mt = 0; mt < MT; ++mt) m[mt] = mn[mt];
        if (ks + 1 < KS) {
#pragma unroll
            for (int mt = 0; mt < MT; ++mt) mn[mt] = ldm(ks + 1, mt);
        }
        const int a = 4 * ks + lk;
        double2 b[NTW];
        double bs[NTW];
#pragma unroll
        for (int j = 0; j < NTW; ++j) {
            b[j] = (a < N2) ? S[a * RS + 16 * (j * WPT + half) + li] : c_zero();
            bs[j] = b[j].x + b[j].y;
        }
#pragma unroll
        for (int mt = 0; mt < MT; ++mt) {
            const double ms = m[mt].x + m[mt].y;
#pragma unroll
            for (int j = 0; j < NTW; ++j) {
                p1[mt][j] = __builtin_amdgcn_mfma_f64_16x16x4f64(m[mt].x, b[j].x, p1[mt][j], 0, 0, 0);
                p2[mt][j] = __builtin_amdgcn_mfma_f64_16x16x4f64(m[mt].y, b[j].y, p2[mt][j], 0, 0, 0);
                p3[mt][j] = __builtin_amdgcn_mfma_f64_16x16x4f64(ms, bs[j], p3[mt][j], 0, 0, 0);
            }
        }
    }
#pragma unroll
    for (int mt = 0; mt < MT; ++mt)
#pragma unroll
        for (int j = 0; j < NTW; ++j)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int row = 16 * mt + lk + 4 * r;
                if (row < N2)
                    S[row * RS + 16 * (j * WPT + half) + li] =
                        make_double2(p1[mt][j][r] - p2[mt][j][r], p3[mt][j][r] - p1[mt][j][r] - p2[mt][j][r]);
            }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
}

// PT contraction of one Liouville row alpha on the matrix cores (v_mfma_f64_4x4x4_4b_f64):
//   C[BT x CHI] = X[BT x CHI] . Qg[CHI x CHI],  X = rows alpha of the BT trajectories.
// gfx950 lane map of the 4-block f64 MFMA (measured): lane l = 16 k + 4 blk + x holds A[blk][x][k],
// B[blk][k][x], D[blk][l>>4][x]. The 4 blocks of one instruction are 4 consecutive 4-column tiles,
// so lane l reads Qg[4 ks + (l>>4)][16 grp + (l & 15)] (256 contiguous bytes per 16 lanes) and ends up
// owning C[4 rb + (l>>4)][16 grp + (l & 15)]: no cross-lane reduction. Complex = 4 real MFMAs.
template <int CHI, int BT, int RS, int TS>
__device__ __forceinline__ void pt_row_mfma(const double2* __restrict__ Qg, double2* st, int a, int lane) {
    constexpr int RB = BT / 4, NG = CHI / 16, KSN = CHI / 4;
    const int x = lane & 3, kk = lane >> 4, c16 = lane & 15;
    double cr[RB][NG], ci[RB][NG];
#pragma unroll
    for (int rb = 0; rb < RB; ++rb)
#pragma unroll
        for (int g = 0; g < NG; ++g) { cr[rb][g] = 0.0; ci[rb][g] = 0.0; }
    const double2* xr = st + a * RS + kk;          // + b*TS + 4 ks
    const double2* qp = Qg + (size_t)kk * CHI + c16;  // + 4 ks * CHI + 16 g
    double2 qn[NG];
#pragma unroll
    for (int g = 0; g < NG; ++g) qn[g] = qp[16 * g];
#pragma unroll 2
    for (int ks = 0; ks < KSN; ++ks) {
        double2 qv[NG];
#pragma unroll
        for (int g = 0; g < NG; ++g) qv[g] = qn[g];
        if (ks + 1 < KSN) {
#pragma unroll
            for (int g = 0; g < NG; ++g) qn[g] = qp[(size_t)4 * (ks + 1) * CHI + 16 * g];
        }
#pragma unroll
        for (int rb = 0; rb < RB; ++rb) {
            const double2 av = xr[(4 * rb + x) * TS + 4 * ks];
            const double ai_neg = -av.y;
#pragma unroll
            for (int g = 0; g < NG; ++g) {
                cr[rb][g] = __builtin_amdgcn_mfma_f64_4x4x4f64(av.x, qv[g].x, cr[rb][g], 0, 0, 0);
                cr[rb][g] = __builtin_amdgcn_mfma_f64_4x4x4f64(ai_neg, qv[g].y, cr[rb][g], 0, 0, 0);
                ci[rb][g] = __builtin_amdgcn_mfma_f64_4x4x4f64(av.x, qv[g].y, ci[rb][g], 0, 0, 0);
                ci[rb][g] = __builtin_amdgcn_mfma_f64_4x4x4f64(av.y, qv[g].x, ci[rb][g], 0, 0, 0);
            }
        }
    }
    double2* wr = st + a * RS + c16;
#pragma unroll
    for (int rb = 0; rb < RB; ++rb)
#pragma unroll
        for (int g = 0; g < NG; ++g) wr[(4 * rb + kk) * TS + 16 * g] = make_double2(cr[rb][g], ci[rb][g]);
}

// pt_row_mfma with three real products per complex product (3M, see col_apply_mfma3): 3 MFMA chains per
// (row block, column group) instead of 4; (Qr + Qi) and (Xr + Xi) are one VALU add per loaded element.
// PF = how many k-steps of the PT slice are in flight ahead of the MFMAs (L2 latency hiding).
// R > 1 contracts R Liouville rows that share one PT slice (dictionary PTs: rows with the same
// coupling-eigenvalue pair) in one pass, so each slice element loaded from L2 feeds R times the MFMAs.
// a0..a3 = the R row indices (unused ones ignored).
// RBN <= BT / 4: only the first RBN row blocks (4 trajectories each) are contracted — the later ones are dormant
// shared-trunk slots (their rows are left as they are until the slot is activated, pqd_host.cpp branch_slots).
template <int CHI, int BT, int RS, int TS, int PF = 1, int R = 1, int RBN = BT / 4>
__device__ __forceinline__ void pt_row_mfma3(const double2* __restrict__ Qg, double2* st, int a0, int a1, int a2,
                                             int a3, int lane) {
    constexpr int RB = RBN, NG = CHI / 16, KSN = CHI / 4;
    const int x = lane & 3, kk = lane >> 4, c16 = lane & 15;
    double p1[R][RB][NG], p2[R][RB][NG], p3[R][RB][NG];
#pragma unroll
    for (int r = 0; r < R; ++r)
#pragma unroll
        for (int rb = 0; rb < RB; ++rb)
#pragma unroll
            for (int g = 0; g < NG; ++g) { p1[r][rb][g] = 0.0; p2[r][rb][g] = 0.0; p3[r][rb][g] = 0.0; }
    const double2* xr[R];
    xr[0] = st + a0 * RS + kk;
    if constexpr (R >= 2) xr[1] = st + a1 * RS + kk;
    if constexpr (R >= 3) xr[2] = st + a2 * RS + kk;
    if constexpr (R >= 4) xr[3] = st + a3 * RS + kk;
    const double2* qp = Qg + (size_t)kk * CHI + c16;
    double2 qn[PF][NG];
#pragma unroll
    for (int f = 0; f < PF; ++f)
#pragma unroll
        for (int g = 0; g < NG; ++g) qn[f][g] = qp[(size_t)4 * f * CHI + 16 * g];
#pragma unroll PF + 1
    for (int ks = 0; ks < KSN; ++ks) {
        double2 qv[NG];
        double qs[NG];
#pragma unroll
        for (int g = 0; g < NG; ++g) { qv[g] = qn[0][g]; qs[g] = qv[g].x + qv[g].y; }
#pragma unroll
        for (int f = 0; f + 1 < PF; ++f)
#pragma unroll
            for (int g = 0; g < NG; ++g) qn[f][g] = qn[f + 1][g];
        if (ks + PF < KSN) {
#pragma unroll
            for (int g = 0; g < NG; ++g) qn[PF - 1][g] = qp[(size_t)4 * (ks + PF) * CHI + 16 * g];
        }
#pragma unroll
        for (int r = 0; r < R; ++r)
#pragma unroll
            for (int rb = 0; rb < RB; ++rb) {
                const double2 av = xr[r][(4 * rb + x) * TS + 4 * ks];
                const double as = av.x + av.y;
#pragma unroll
                for (int g = 0; g < NG; ++g) {
                    p1[r][rb][g] = __builtin_amdgcn_mfma_f64_4x4x4f64(av.x, qv[g].x, p1[r][rb][g], 0, 0, 0);
                    p2[r][rb][g] = __builtin_amdgcn_mfma_f64_4x4x4f64(av.y, qv[g].y, p2[r][rb][g], 0, 0, 0);
                    p3[r][rb][g] = __builtin_amdgcn_mfma_f64_4x4x4f64(as, qs[g], p3[r][rb][g], 0, 0, 0);
                }
            }
    }
#pragma unroll
    for (int r = 0; r < R; ++r) {
        double2* wr = st + (r == 0 ? a0 : r == 1 ? a1 : r == 2 ? a2 : a3) * RS + c16;
#pragma unroll
        for (int rb = 0; rb < RB; ++rb)
#pragma unroll
            for (int g = 0; g < NG; ++g)
                wr[(4 * rb + kk) * TS + 16 * g] = make_double2(p1[r][rb][g] - p2[r][rb][g],
                                                               p3[r][rb][g] - p1[r][rb][g] - p2[r][rb][g]);
    }
}

// a unit of n rows sharing one slice (n <= sweep_rmax: the accumulators stay within 48 doubles)
template <int N2, int CHI, int BT, int RS, int TS, int PF, int RBN>
__device__ __forceinline__ void pt_rows3_n(const double2* __restrict__ Qg, double2* st, int4 e, int lane) {
    constexpr int RM = sweep_rmax(N2, BT, CHI);
    if constexpr (RM >= 4) {
        if (e.w >= 0) {  // rows 2 (and 3) in the low (high) 16 bits of w
            const int a2 = e.w & 0xFFFF, a3 = e.w >> 16;
            if (a3 != 0x7FFF) pt_row_mfma3<CHI, BT, RS, TS, PF, 4, RBN>(Qg, st, e.y, e.z, a2, a3, lane);
            else pt_row_mfma3<CHI, BT, RS, TS, PF, 3, RBN>(Qg, st, e.y, e.z, a2, a2, lane);
            return;
        }
    }
    if constexpr (RM >= 2) {
        if (e.z >= 0) pt_row_mfma3<CHI, BT, RS, TS, PF, 2, RBN>(Qg, st, e.y, e.z, e.z, e.z, lane);
        else pt_row_mfma3<CHI, BT, RS, TS, PF, 1, RBN>(Qg, st, e.y, e.y, e.y, e.y, lane);
    } else {
        pt_row_mfma3<CHI, BT, RS, TS, PF, 1, RBN>(Qg, st, e.y, e.y, e.y, e.y, lane);
    }
}

// all rows of the workgroup, dormant shared-trunk slots included (their rows are overwritten at activation):
// skipping a dormant row block through a second instance (RBN = 1) cost 0.7% on the bench workload, where blocks
// are dormant for a few steps only (profiles/r02/ab_rbn.log)
template <int N2, int CHI, int BT, int RS, int TS, int PF>
__device__ __forceinline__ void pt_rows3(const double2* __restrict__ Qg, double2* st, int4 e, int lane) {
    pt_rows3_n<N2, CHI, BT, RS, TS, PF, BT / 4>(Qg, st, e, lane);
}

// PT contraction of row alpha for BT = 8 on v_mfma_f64_16x16x4_f64 ("split complex"): the 16 MFMA rows are
// [Re X; Im X] of the 8 trajectories, so two real GEMMs P1 = [Xr; Xi] Qr and P2 = [Xr; Xi] Qi hold all four
// partial products: Cr = P1[top] - P2[bottom], Ci = P2[top] + P1[bottom]. C fragment rows (l>>4) + 4 r put
// row b (r = 0, 1) and row b + 8 (r + 2) in the same lane, so the recombination is lane-local. Same operand
// traffic as the 4x4x4 path, but the 16x16x4 instruction runs at the FP64 matrix peak and co-issues with VALU.
template <int CHI, int RS, int TS>
__device__ __forceinline__ void pt_row_mfma16(const double2* __restrict__ Qg, double2* st, int a, int lane) {
    constexpr int NTL = CHI / 16, KSN = CHI / 4;
    const int li = lane & 15, lk = lane >> 4;
    const bool imag_row = (li & 8) != 0;
    dbl4 p1[NTL], p2[NTL];
#pragma unroll
    for (int t = 0; t < NTL; ++t) { p1[t] = dbl4{0, 0, 0, 0}; p2[t] = dbl4{0, 0, 0, 0}; }
    const double2* xr = st + (li & 7) * TS + a * RS + lk;  // + 4 ks
    const double2* qp = Qg + (size_t)lk * CHI + li;         // + 4 ks * CHI + 16 t
    double2 qn[NTL];
#pragma unroll
    for (int t = 0; t < NTL; ++t) qn[t] = qp[16 * t];
#pragma unroll 2
    for (int ks = 0; ks < KSN; ++ks) {
        double2 qv[NTL];
#pragma unroll
        for (int t = 0; t < NTL; ++t) qv[t] = qn[t];
        if (ks + 1 < KSN) {
#pragma unroll
            for (int t = 0; t < NTL; ++t) qn[t] = qp[(size_t)4 * (ks + 1) * CHI + 16 * t];
        }
        const double2 xv = xr[4 * ks];
        const double av = imag_row ? xv.y : xv.x;
#pragma unroll
        for (int t = 0; t < NTL; ++t) {
            p1[t] = __builtin_amdgcn_mfma_f64_16x16x4f64(av, qv[t].x, p1[t], 0, 0, 0);
            p2[t] = __builtin_amdgcn_mfma_f64_16x16x4f64(av, qv[t].y, p2[t], 0, 0, 0);
        }
    }
    double2* wr = st + a * RS + li;
#pragma unroll
    for (int t = 0; t < NTL; ++t)
#pragma unroll
        for (int r = 0; r < 2; ++r)
            wr[(lk + 4 * r) * TS + 16 * t] = make_double2(p1[t][r] - p2[t][r + 2], p2[t][r] + p1[t][r + 2]);
}

// TRUNK: the trunk pre-pass instance (writes checkpoints through p.ck_map); kept out of the main sweep's instance,
// where the extra live values cost VGPR spills
// Reads every half step's M, F, W as stored: plans running this kernel (main sweep or trunk pre-pass) build the free
// propagators without pulse windows (pqd_host.cpp). A window-select form of these loads measured 1.8% slower on the
// bench launch even with its selects folded away at compile time (202.3 vs 198.1 ms, profiles/r02/windows/).
template <int N2, int CHI, int BT, bool TRUNK>
__global__ __launch_bounds__(64 * BT * sweep_wpt(N2, BT, CHI)) void pt_sweep_kernel(SweepParams p, const double2* __restrict__ Mg,
                                                           const double2* __restrict__ Qg0, double2* __restrict__ outg,
                                                           const double2* __restrict__ Fg, const double2* __restrict__ Wg) {
    using L = SweepLayout<N2, CHI, BT>;
    constexpr int RS = L::RS, TS = L::TS, KD = L::KD, NCOL = L::NCOL;
    constexpr int WPT = L::WPT, NW = L::NW, NT = 64 * NW;  // waves per trajectory, waves, threads
    extern __shared__ __attribute__((aligned(16))) double2 smem[];
    double2* st = smem;
    double2* rbuf = smem + BT * TS;
    __shared__ int s_traj[BT], s_wb[BT], s_we[BT], s_fz[BT], s_sys[BT], s_act[BT], s_src[BT];
    __shared__ long long s_wo[BT];

    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int tw = wave % BT, half = wave / BT;  // column phases: trajectory of this wave, its column half

    if (tid < BT) {
        const int t = p.blk_traj[blockIdx.x * BT + tid];
        s_traj[tid] = t;
        s_wb[tid] = t >= 0 ? p.wbeg[t] : INT_MAX;
        s_we[tid] = t >= 0 ? p.wend[t] : -1;
        s_wo[tid] = t >= 0 ? p.woff[t] : 0;
        s_fz[tid] = 0;
        s_sys[tid] = t >= 0 ? p.traj_sys[t] : 0;
        s_act[tid] = p.blk_act[blockIdx.x * BT + tid];
        s_src[tid] = p.blk_src[blockIdx.x * BT + tid];
    }
    __syncthreads();
    // shared trunk (pqd_host.cpp branch_slots): a slot is dormant before its activation step, then copies the
    // (state, fused flag) of an earlier-activated slot of its workgroup or a trunk checkpoint. next_act: the next step
    // with activations
    const int my_act = __builtin_amdgcn_readfirstlane(s_act[tw]);
    auto next_activation = [&](int after) {
        int m = INT_MAX;
#pragma unroll
        for (int b = 0; b < BT; ++b)
            if (s_act[b] > after && s_act[b] < m) m = s_act[b];
        return m;
    };
    int n0 = INT_MAX;  // first step of the block: its earliest activation (0 unless every slot starts later)
#pragma unroll
    for (int b = 0; b < BT; ++b) n0 = s_act[b] < n0 ? s_act[b] : n0;
    if (n0 == INT_MAX) return;  // no trajectory in this workgroup (the whole block exits together)
    int next_act = n0 > 0 ? n0 : next_activation(0);
    const int n_end = p.blk_end[blockIdx.x];
    // a workgroup may mix systems (per-trajectory drives, e.g. one system per scan point): each wave reads the
    // free propagators of its own trajectory's system
    {
        const int sw = __builtin_amdgcn_readfirstlane(s_sys[tw]);
        Mg += (size_t)sw * p.m_stride;
        Fg += (size_t)sw * p.f_stride;
    }

    // ---- initial augmented states rho0 (x) bond0 (thread -> column)
    for (int c = tid; c < NCOL; c += NT) {
        const int cb = c / CHI, cd = c - (c / CHI) * CHI;
        const double2 b0 = p.bond0[cd];
#pragma unroll
        for (int a = 0; a < N2; ++a) st[cb * TS + a * RS + cd] = c_mul(p.rho0[a], b0);
    }
    __syncthreads();
    // ---- column phases: wave w owns trajectory w % BT (its free propagators, its MTO events), and with two
    // waves per trajectory the column tiles of half w / BT
    double2* stw = st + tw * TS;
    const bool c3 = p.cmul3 != 0;
    const bool cbig = p.colbig != 0;
    auto col = [&](const double2* __restrict__ Op) {
        if (c3) {
            if constexpr (col_big_ok<N2, CHI, RS, WPT>()) {
                if (cbig) { col_apply_mfma3_big<N2, CHI, RS, WPT>(Op, stw, lane, half); return; }
            }
            col_apply_mfma3<N2, CHI, RS, WPT>(Op, stw, lane, half);
        } else {
            col_apply_mfma<N2, CHI, RS, WPT>(Op, stw, lane, half);
        }
    };
    int ev_cur = 0, ev_lim = 0;
    {
        const int t = s_traj[tw];
        if (t >= 0) { ev_cur = p.ev_start[t]; ev_lim = p.ev_start[t + 1]; }
        while (ev_cur < ev_lim) {  // applyBefore-true MTOs at step 0
            const int4 e = p.ev[ev_cur];
            if (e.x != 0 || e.y != 0) break;
            col(p.sop + (size_t)e.z * N2 * N2);
            ++ev_cur;
        }
    }
    __syncthreads();

    const int pj = lane & 15, pq = lane >> 4;
    // traces with one lane per (trajectory, output, row) when N2 is a power of two and they fit the workgroup
    // (16-lane reduction groups); each lane keeps the next step's W row element in a register
    const int ntr = BT * p.n_out * N2;
    const bool lanetr = (N2 == 4 || N2 == 16) && p.trpre && ntr <= NT;
    double2 wpre = c_zero();
    if (n0 > 0 && lanetr && tid < ntr) {  // the step the loop starts at: W(n0) row element, as fetched a step ahead
        const int a = tid % N2, bk = tid / N2, b = bk / p.n_out, k = bk - (bk / p.n_out) * p.n_out;
        wpre = Wg[(size_t)s_sys[b] * p.w_stride + ((size_t)n0 * p.n_out + k) * N2 + a];
    }
    bool fz = false;  // this wave's trajectory sits between M_b(n-1) and M_a(n) unapplied (fused step n)
    for (int n = n0;; ++n) {
        // ------------------------------------------------------------ shared-trunk activations at step n
        if (n == next_act) {
            // a checkpoint (src <= -2) holds the trunk at the top of step n >= 1 with M_b(n-1) deferred (fused)
            if (tid < BT && s_act[tid] == n) s_fz[tid] = s_src[tid] >= 0 ? s_fz[s_src[tid]] : 1;
            for (int b = 0; b < BT; ++b) {
                if (s_act[b] != n) continue;
                double2* dp = st + b * TS;
                if (s_src[b] >= 0) {
                    const double2* sp = st + s_src[b] * TS;
                    for (int e = tid; e < N2 * CHI; e += NT) {
                        const int a = e / CHI, c = e - (e / CHI) * CHI;
                        dp[a * RS + c] = sp[a * RS + c];
                    }
                } else if (s_src[b] <= -2) {
                    const double2* cp = p.ck + (size_t)(-2 - s_src[b]) * N2 * CHI;
                    for (int e = tid; e < N2 * CHI; e += NT) {
                        const int a = e / CHI, c = e - (e / CHI) * CHI;
                        dp[a * RS + c] = cp[e];
                    }
                }
            }
            if (my_act == n) fz = s_src[tw] >= 0 ? (s_fz[s_src[tw]] != 0) : true;
            next_act = next_activation(n);
            __syncthreads();
        }
        // ------------------------------------------------------------ trunk pre-pass: checkpoints at step n
        if constexpr (TRUNK) {
            bool wrote = false;
            for (int b = 0; b < BT; ++b) {
                const int t = s_traj[b];
                const int c = t >= 0 ? p.ck_map[(size_t)t * p.ck_stride + n] : -1;
                if (c < 0) continue;
                wrote = true;
                double2* cp = p.ck + (size_t)c * N2 * CHI;
                for (int e = tid; e < N2 * CHI; e += NT) {
                    const int a = e / CHI, cc = e - (e / CHI) * CHI;
                    cp[e] = st[b * TS + a * RS + cc];
                }
            }
            if (wrote) __syncthreads();
        }
        // ------------------------------------------------------------ outputs at step n
        bool need = false;
#pragma unroll
        for (int b = 0; b < BT; ++b) need |= (s_wb[b] <= n) & (n <= s_we[b]);
        if (need && !(p.ablate & 4)) {
            const double2* cvec = (n == 0) ? p.closure0 : p.closure + (size_t)p.sched[n - 1] * CHI;
            constexpr int NPART = BT * N2 * 4;
            for (int it = 0; it < (NPART + NT - 1) / NT; ++it) {
                const int e = tid + NT * it;
                const int row = e >> 2, qr = e & 3;
                double2 s = c_zero();
                if (e < NPART) {
                    const int b = row / N2, a = row - (row / N2) * N2;
                    const double2* rp = st + b * TS + a * RS + qr;
#pragma unroll 4
                    for (int kk = 0; kk < CHI / 4; ++kk) c_fma(s, rp[4 * kk], cvec[4 * kk + qr]);
                }
                s = c_add(s, c_shfl_xor(s, 1));
                s = c_add(s, c_shfl_xor(s, 2));
                if (e < NPART && qr == 0) rbuf[row] = s;
            }
            __syncthreads();
            if (lanetr) {
                // one lane per (trajectory, output, row): the row element of W(n) was fetched a step ahead
                if (tid < ntr) {
                    const int a = tid % N2, bk = tid / N2, b = bk / p.n_out, k = bk - (bk / p.n_out) * p.n_out;
                    const double2 v = s_fz[b] ? wpre : p.ovec[k * N2 + a];
                    double2 x = c_mul(v, rbuf[b * N2 + a]);
#pragma unroll
                    for (int m = 1; m < N2; m <<= 1) x = c_add(x, c_shfl_xor(x, m));
                    if (a == 0 && s_wb[b] <= n && n <= s_we[b])
                        outg[s_wo[b] + (long long)(n - s_wb[b]) * p.n_out + k] = x;
                }
            } else
            for (int e = tid; e < BT * p.n_out; e += NT) {
                const int b = e / p.n_out, k = e - (e / p.n_out) * p.n_out;
                if (s_wb[b] <= n && n <= s_we[b]) {
                    double2 s = c_zero();
                    // fused trajectories still hold the state before M_b(n-1): read it through W(n)
                    const double2* ov = (s_fz[b] ? Wg + (size_t)s_sys[b] * p.w_stride + (size_t)n * p.n_out * N2
                                                 : p.ovec) + (size_t)k * N2;
                    // all of a chunk's row loads are issued before its first FMA (one memory round trip per
                    // chunk, not one per few elements: the scheduler otherwise interleaves them)
                    constexpr int CK = N2 <= 16 ? N2 : 9;
#pragma unroll
                    for (int a0 = 0; a0 < N2; a0 += CK) {
                        double2 ovr[CK];
#pragma unroll
                        for (int j = 0; j < CK; ++j) ovr[j] = (a0 + j < N2) ? ov[a0 + j] : c_zero();
                        asm volatile("" ::: "memory");
#pragma unroll
                        for (int j = 0; j < CK; ++j)
                            if (a0 + j < N2) c_fma(s, ovr[j], rbuf[b * N2 + a0 + j]);
                    }
                    outg[s_wo[b] + (long long)(n - s_wb[b]) * p.n_out + k] = s;
                }
            }
        }
        if (n >= n_end) break;
        if (lanetr && tid < ntr) {  // W(n + 1) row element for the next step's traces (fused trajectories)
            const int a = tid % N2, bk = tid / N2, b = bk / p.n_out, k = bk - (bk / p.n_out) * p.n_out;
            wpre = Wg[(size_t)s_sys[b] * p.w_stride + ((size_t)(n + 1) * p.n_out + k) * N2 + a];
        }

        // ------------------------------------------------------------ column phase A
        const double2* Ma = Mg + (size_t)(2 * n) * N2 * N2;
        if (!(p.ablate & 2) && n >= my_act) {
            const bool mto_now = ev_cur < ev_lim && p.ev[ev_cur].x == n;
            if (fz && !mto_now) {  // no MTO at step n: M_b(n-1) and M_a(n) in one operator
                col(Fg + (size_t)n * N2 * N2);
            } else {
                // a slot activated at n holds the trunk's state with M_b(n-1) still deferred, but has an MTO at n
                if (fz) col(Mg + (size_t)(2 * n - 1) * N2 * N2);
                while (ev_cur < ev_lim) {  // applyBefore-false MTOs at step n
                    const int4 e = p.ev[ev_cur];
                    if (e.x != n || e.y != 1) break;
                    col(p.sop + (size_t)e.z * N2 * N2);
                    ++ev_cur;
                }
                col(Ma);
            }
        }
        __syncthreads();

        // ------------------------------------------------------------ PT contraction
        if (!(p.ablate & 1)) {
            const double2* Qs = Qg0 + (size_t)p.sched[n] * p.D * CHI * CHI;
            // pt_mode 0: VALU rows, 1: matrix-core rows (4x4x4_4b), 4: matrix-core rows with 3 real products per
            // complex product (default), 3: split-complex 16x16x4 rows (BT = 8), 2: mixed (waves 0..NW/2-1 start on the matrix cores,
            // the others on the VALU, alternating per row), so the two FP64 pipes of a SIMD run concurrently
            int parity = (p.pt_mode == 2) ? ((wave >= NW / 2) ? 1 : 0) : 0;
            if (p.units && (p.pt_mode == 4 || p.pt_mode == 5)) {
                // 3M rows by the host's per-wave unit list: (slice, row 0, row 1 or -1, rows 2 | 3 << 16 or -1)
                const int4* U = p.units + (size_t)wave * p.umax;
                for (int u = 0; u < p.umax; ++u) {
                    const int4 e = U[u];
                    if (e.x < 0) break;
                    const double2* Qg = Qs + (size_t)e.x * CHI * CHI;
                    if (p.pt_mode == 5) pt_rows3<N2, CHI, BT, RS, TS, 2>(Qg, st, e, lane);
                    else pt_rows3<N2, CHI, BT, RS, TS, 1>(Qg, st, e, lane);
                }
            } else
            for (int a = wave; a < N2; a += NW) {
                const double2* Qg = Qs + (size_t)p.gmap[a] * CHI * CHI;
                const bool use_mfma = (p.pt_mode == 1) || (p.pt_mode == 2 && parity == 0);
                parity ^= 1;
                if (p.pt_mode == 4) {
                    pt_row_mfma3<CHI, BT, RS, TS, 1>(Qg, st, a, a, a, a, lane);
                    continue;
                }
                if (p.pt_mode == 5) {   // 3M with two k-steps of the slice in flight
                    pt_row_mfma3<CHI, BT, RS, TS, 2>(Qg, st, a, a, a, a, lane);
                    continue;
                }
                if constexpr (BT == 8) {
                    if (p.pt_mode == 3) {
                        pt_row_mfma16<CHI, RS, TS>(Qg, st, a, lane);
                        continue;
                    }
                }
                // the VALU rows are compiled for BT = 4, chi <= 64 and one wave per trajectory only: elsewhere
                // their accumulators cap the whole kernel's VGPR allocation and spill, so those run modes 0/2 on
                // the 4x4x4 path
                if (BT == 8 || CHI > 64 || WPT > 1 || use_mfma || p.pt_mode == 3) {
                    pt_row_mfma<CHI, BT, RS, TS>(Qg, st, a, lane);
                    continue;
                }
                if constexpr (BT == 4 && CHI <= 64 && WPT == 1) {
                Qg += pj;
                const double2* xr = st + a * RS + pq;
                double2 acc[BT][KD];
#pragma unroll
                for (int b = 0; b < BT; ++b)
#pragma unroll
                    for (int i = 0; i < KD; ++i) acc[b][i] = c_zero();
                double2 qn[KD];
#pragma unroll
                for (int i = 0; i < KD; ++i) qn[i] = Qg[(size_t)pq * CHI + 16 * i];
#pragma unroll 2
                for (int kk = 0; kk < CHI / 4; ++kk) {
                    double2 qv[KD];
#pragma unroll
                    for (int i = 0; i < KD; ++i) qv[i] = qn[i];
                    if (kk + 1 < CHI / 4) {
                        const int dn = 4 * (kk + 1) + pq;
#pragma unroll
                        for (int i = 0; i < KD; ++i) qn[i] = Qg[(size_t)dn * CHI + 16 * i];
                    }
#pragma unroll
                    for (int b = 0; b < BT; ++b) {
                        const double2 x = xr[b * TS + 4 * kk];
#pragma unroll
                        for (int i = 0; i < KD; ++i) c_fma(acc[b][i], x, qv[i]);
                    }
                }
                // reduce the 4 input quarters (lanes j, j+16, j+32, j+48) and scatter the columns
                double2* wr = st + a * RS + pj;
                if constexpr (KD == 4) {
                    const bool q0 = pq & 1, q1 = (pq >> 1) & 1;
#pragma unroll
                    for (int b = 0; b < BT; ++b) {
                        double2 h[2];
#pragma unroll
                        for (int pi = 0; pi < 2; ++pi) {
                            const double2 mine = q0 ? acc[b][2 * pi + 1] : acc[b][2 * pi];
                            const double2 oth = q0 ? acc[b][2 * pi] : acc[b][2 * pi + 1];
                            h[pi] = c_add(mine, c_shfl_xor(oth, 16));
                        }
                        const double2 mine = q1 ? h[1] : h[0];
                        const double2 oth = q1 ? h[0] : h[1];
                        wr[b * TS + 16 * pq] = c_add(mine, c_shfl_xor(oth, 32));
                    }
                } else if constexpr (KD == 2) {
                    const bool q0 = pq & 1;
#pragma unroll
                    for (int b = 0; b < BT; ++b) {
                        const double2 mine = q0 ? acc[b][1] : acc[b][0];
                        const double2 oth = q0 ? acc[b][0] : acc[b][1];
                        double2 h = c_add(mine, c_shfl_xor(oth, 16));
                        h = c_add(h, c_shfl_xor(h, 32));
                        if (pq < 2) wr[b * TS + 16 * pq] = h;
                    }
                } else {
#pragma unroll
                    for (int b = 0; b < BT; ++b) {
                        double2 h = c_add(acc[b][0], c_shfl_xor(acc[b][0], 16));
                        h = c_add(h, c_shfl_xor(h, 32));
                        if (pq == 0) wr[b * TS] = h;
                    }
                }
                }  // VALU rows
            }
        }
        __syncthreads();

        // ------------------------------------------------------------ column phase B
        const double2* Mb = Ma + N2 * N2;
        // fuse M_b(n) into the next step's operator unless this trajectory has an MTO at step n+1
        fz = p.fuse && !(ev_cur < ev_lim && p.ev[ev_cur].x == n + 1);
        if (!(p.ablate & 2) && !fz && n >= my_act) {
            col(Mb);
            while (ev_cur < ev_lim) {  // applyBefore-true MTOs at step n+1
                const int4 e = p.ev[ev_cur];
                if (e.x != n + 1 || e.y != 0) break;
                col(p.sop + (size_t)e.z * N2 * N2);
                ++ev_cur;
            }
        }
        if (lane == 0 && half == 0) s_fz[tw] = fz ? 1 : 0;
        __syncthreads();
    }
}

// ------------------------------------------------------------------------------------------------
// chi = 1 (no environment): one wave per trajectory, lane r owns rho[r]; operators applied through
// cross-lane shuffles (no LDS, no barriers). Latency-bound by construction (C1: 1 trajectory).
// ------------------------------------------------------------------------------------------------
template <int N2>
__device__ __forceinline__ double2 lane_apply(const double2* __restrict__ Op, double2 own, int lane) {
    const int r = lane < N2 ? lane : N2 - 1;
    const double2* Or = Op + r * N2;
    double2 acc = c_zero();
#pragma unroll
    for (int a = 0; a < N2; ++a) {
        const double2 x = make_double2(__shfl(own.x, a), __shfl(own.y, a));
        c_fma(acc, Or[a], x);
    }
    return acc;
}

template <int N2>
__global__ __launch_bounds__(64) void sweep_nopt_kernel(SweepParams p) {
    const int lane = threadIdx.x;
    const int t = blockIdx.x;
    const int wb = p.wbeg[t], we = p.wend[t];
    const long long wo = p.woff[t];
    int ev_cur = p.ev_start[t];
    const int sy = p.traj_sys[t];
    const int2 wn = fw_win(p, sy);  // pulse windows (pqd_host.cpp: only plans whose kernels all read through them)
    const int ev_lim = p.ev_start[t + 1];
    double2 own = lane < N2 ? p.rho0[lane] : c_zero();
    while (ev_cur < ev_lim) {
        const int4 e = p.ev[ev_cur];
        if (e.x != 0 || e.y != 0) break;
        own = lane_apply<N2>(p.sop + (size_t)e.z * N2 * N2, own, lane);
        ++ev_cur;
    }
    for (int n = 0;; ++n) {
        if (wb <= n && n <= we) {
            // every lane gathers the state (all lanes take part in the shuffles), then lane k owns outputs
            // k, k + 64, ... (n_out may exceed the wave)
            double2 x[N2];
#pragma unroll
            for (int a = 0; a < N2; ++a) x[a] = make_double2(__shfl(own.x, a), __shfl(own.y, a));
            for (int k = lane; k < p.n_out; k += 64) {
                double2 s = c_zero();
                const double2* ov = p.ovec + (size_t)k * N2;
#pragma unroll
                for (int a = 0; a < N2; ++a) c_fma(s, ov[a], x[a]);
                p.out[wo + (long long)(n - wb) * p.n_out + k] = s;
            }
        }
        if (n >= we) break;
        while (ev_cur < ev_lim) {
            const int4 e = p.ev[ev_cur];
            if (e.x != n || e.y != 1) break;
            own = lane_apply<N2>(p.sop + (size_t)e.z * N2 * N2, own, lane);
            ++ev_cur;
        }
        own = lane_apply<N2>(fw_M(p, sy, wn, 2 * n, N2 * N2), own, lane);
        own = lane_apply<N2>(fw_M(p, sy, wn, 2 * n + 1, N2 * N2), own, lane);
        while (ev_cur < ev_lim) {
            const int4 e = p.ev[ev_cur];
            if (e.x != n + 1 || e.y != 0) break;
            own = lane_apply<N2>(p.sop + (size_t)e.z * N2 * N2, own, lane);
            ++ev_cur;
        }
    }
}

template <int N2, int CHI, int BT, bool TRUNK>
hipError_t launch_sw(int n_blocks, const SweepParams& p, hipStream_t s) {
    using L = SweepLayout<N2, CHI, BT>;
    static_assert(L::LDS <= 160 * 1024, "LDS budget");
    static bool attr = false;
    if (!attr) {
        hipError_t e = hipFuncSetAttribute((const void*)pt_sweep_kernel<N2, CHI, BT, TRUNK>,
                                           hipFuncAttributeMaxDynamicSharedMemorySize, (int)L::LDS);
        if (e != hipSuccess) return e;
        attr = true;
    }
    hipLaunchKernelGGL((pt_sweep_kernel<N2, CHI, BT, TRUNK>), dim3(n_blocks), dim3(64 * L::NW), L::LDS, s, p, p.M, p.Q,
                       p.out, p.F, p.W);
    return hipGetLastError();
}

template <int N2, int BT, bool TRUNK = false>
hipError_t launch_sw_chi(int CHI, int n_blocks, const SweepParams& p, hipStream_t s) {
    switch (CHI) {
        case 16: return launch_sw<N2, 16, BT, TRUNK>(n_blocks, p, s);
        case 32: return launch_sw<N2, 32, BT, TRUNK>(n_blocks, p, s);
        case 64: return launch_sw<N2, 64, BT, TRUNK>(n_blocks, p, s);
        case 128:
            // chi = 128 keeps 4 augmented states of N2 <= 16 in LDS (132 KiB); larger N2 or BT do not fit
            if constexpr (BT == 4 && N2 <= 16) return launch_sw<N2, 128, BT, TRUNK>(n_blocks, p, s);
            return hipErrorInvalidValue;
        default: return hipErrorInvalidValue;
    }
}

}  // namespace

bool sweep_supported(int N2, int CHI) {
    return (N2 == 4 || N2 == 9 || N2 == 16 || N2 == 25 || N2 == 36) &&
           (CHI == 1 || CHI == 16 || CHI == 32 || CHI == 64 || (CHI == 128 && N2 <= 16));
}

// trajectories per workgroup that fit the LDS for this N2 (8 halves the per-trajectory PT-slice traffic)
int sweep_max_bt(int N2) { return N2 <= 16 ? 8 : 4; }

hipError_t launch_sweep(int N2, int CHI, int BT, int n_blocks, const SweepParams& p, hipStream_t s) {
    if (n_blocks <= 0) return hipSuccess;
    if (p.ck_map) {  // trunk pre-pass: four trunks per workgroup
        if (BT != 4) return hipErrorInvalidValue;
        switch (N2) {
            case 4: return launch_sw_chi<4, 4, true>(CHI, n_blocks, p, s);
            case 9: return launch_sw_chi<9, 4, true>(CHI, n_blocks, p, s);
            case 16: return launch_sw_chi<16, 4, true>(CHI, n_blocks, p, s);
            case 25: return launch_sw_chi<25, 4, true>(CHI, n_blocks, p, s);
            case 36: return launch_sw_chi<36, 4, true>(CHI, n_blocks, p, s);
            default: return hipErrorInvalidValue;
        }
    }
    if (BT == 8) {
        switch (N2) {
            case 4: return launch_sw_chi<4, 8>(CHI, n_blocks, p, s);
            case 9: return launch_sw_chi<9, 8>(CHI, n_blocks, p, s);
            case 16: return launch_sw_chi<16, 8>(CHI, n_blocks, p, s);
            default: return hipErrorInvalidValue;
        }
    }
    if (BT != 4) return hipErrorInvalidValue;
    switch (N2) {
        case 4: return launch_sw_chi<4, 4>(CHI, n_blocks, p, s);
        case 9: return launch_sw_chi<9, 4>(CHI, n_blocks, p, s);
        case 16: return launch_sw_chi<16, 4>(CHI, n_blocks, p, s);
        case 25: return launch_sw_chi<25, 4>(CHI, n_blocks, p, s);
        case 36: return launch_sw_chi<36, 4>(CHI, n_blocks, p, s);
        default: return hipErrorInvalidValue;
    }
}

hipError_t launch_sweep_nopt(int N2, int n_traj, const SweepParams& p, hipStream_t s) {
    if (n_traj <= 0) return hipSuccess;
#define PQD_NOPT(NN) case NN: hipLaunchKernelGGL(sweep_nopt_kernel<NN>, dim3(n_traj), dim3(64), 0, s, p); break;
    switch (N2) {
        PQD_NOPT(4) PQD_NOPT(9) PQD_NOPT(16) PQD_NOPT(25) PQD_NOPT(36)
        default: return hipErrorInvalidValue;
    }
#undef PQD_NOPT
    return hipGetLastError();
}
