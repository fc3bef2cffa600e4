// pt_quad.hip — the PT sweep for the two-level system (N2 = 4), register-resident.
//
// Replaces, for the TLS (reference two_level_system/tls.py -> system_ace_stream, general_system.py:227-343), the same
// per-step ACE loop as pt_sweep.hip. At N2 = 4 the batched kernel's step is short (4 PT rows x chi^2 per trajectory)
// and its eight waves spend it in four workgroup barriers and L2 round trips: 0.25 of the FP64 peak on the
// 2048-point TLS scan (C2). Here:
//   * a "quad" is four trajectories (one host block of BT = 4); it is carried by CHI/16 waves, wave h owning the
//     bond columns [16h, 16h + 16) of all four augmented states, in registers;
//   * ONE v_mfma_f64_4x4x4_4b stream contracts all four Liouville rows of all four trajectories: the instruction's
//     four blocks are the four rows alpha (each its own PT slice Q_g(alpha)), a block's 4 x 4 A tile is (trajectory,
//     bond k) and its B tile (bond k, column): no lanes idle, no row/wave assignment, three real MFMA chains per
//     complex product (3M);
//   * the column phases (free half steps, fused F(n), MTOs: an N2 x N2 operator per trajectory acting on alpha) are the
//     same instruction with blocks = the four trajectories, on the state in its register layout;
//   * the slice operands of step n+1 (CHI/4 x 4 complex per lane) are loaded into registers while step n runs, as are
//     the closure, the fused operator F(n+1) and the output rows W(n+1): nothing on the step's critical path waits on
//     L2;
//   * one LDS exchange per step (the strips' columns -> every wave's full rows for the contraction, plus the closure
//     partial sums), double-buffered by step parity: one workgroup barrier per step (none at CHI = 16).
// Lane maps (gfx950 4x4x4_4b f64, lane l = 16 k + 4 blk + x holds A[blk][x][k], B[blk][k][x], D[blk][l>>4][x]):
//   C-layout (state, column ops)   l = 16 alpha + 4 t + c'  holds S_t[alpha][16 h + 4 cg + c']   (register cg)
//   A-layout (PT input)            l = 16 k' + 4 alpha + t  holds S_t[alpha][4 ks + k']           (register ks)
//   B-layout (PT slice)            l = 16 k' + 4 alpha + c' holds Q_g(alpha)[4 ks + k'][16 h + 4 cg + c']
//   D-layout (PT output)           l = 16 t + 4 alpha + c'  holds (S_t Q)[alpha][16 h + 4 cg + c']
// The D -> C relayout and the C -> A transposition go through the LDS row buffer st[t][alpha][c] (row stride
// CHI + 1: conflict-free for 16-lane phases of both access patterns).
// Semantics and shared-trunk activation (pqd_host.cpp branch_slots) are those of pt_sweep_kernel.
#include "pqd_common.h"
#include <climits>
#include <cstdlib>
#include <type_traits>

#ifndef PQD_QRAISE
#define PQD_QRAISE(KS) (KS)
#endif

namespace {

__device__ __forceinline__ double mfma4(double a, double b, double c) {
    return __builtin_amdgcn_mfma_f64_4x4x4f64(a, b, c, 0, 0, 0);
}

// one column operator per trajectory (block t) applied to the C-layout state: R[cg] <- Op_t R[cg] where `mine`
// (uniform per block t); `a` = this lane's operator element Op_t[alpha' = l & 3][alpha = l >> 4]. Every lane takes
// part in the MFMAs (they read all 64 lanes); slots without an operator this round keep their values exactly.
template <int NCG>
__device__ __forceinline__ void quad_col(double2 a, bool mine, double2 (&R)[NCG]) {
    const double as = a.x + a.y;
#pragma unroll
    for (int cg = 0; cg < NCG; ++cg) {
        const double bs = R[cg].x + R[cg].y;
        const double p1 = mfma4(a.x, R[cg].x, 0.0);
        const double p2 = mfma4(a.y, R[cg].y, 0.0);
        const double p3 = mfma4(as, bs, 0.0);
        if (mine) R[cg] = make_double2(p1 - p2, p3 - p1 - p2);
    }
}

// diagnostics (PQD_ABLATE bit 32, scripts/quad_stamps.py): s_memtime at the phase boundaries of steps
// 1000..1015, workgroup 0, wave 0 (a separate instantiation; the production kernel carries none of it)
__device__ unsigned long long g_quad_stamps[16 * 16];

// a per-lane value the compiler must treat as new at this point: the slow step's operator and event addresses derived
// from it are computed there (a few VALU ops) instead of hoisted out of the step loop and held, as 64-bit pairs,
// across the fast pairs that never use them (C2 instance: 21 -> 8 spilled VGPRs, 64 -> 28 B scratch, sweep
// 14.27 -> 14.21 ms; profiles/r04/quad/ab_v1.log)
template <class T>
__device__ __forceinline__ T opq(T v) {
    asm volatile("" : "+v"(v));
    return v;
}

// s_setprio takes an immediate
__device__ __forceinline__ void set_prio(int k) {
    if (k <= 0) __builtin_amdgcn_s_setprio(0);
    else if (k == 1) __builtin_amdgcn_s_setprio(1);
    else if (k == 2) __builtin_amdgcn_s_setprio(2);
    else __builtin_amdgcn_s_setprio(3);
}

// DPP lane exchange inside groups of four lanes (quad_perm), on a double's two halves: no LDS round trip
template <int CTRL>
__device__ __forceinline__ double dpp_q(double v) {
    const int lo = __builtin_amdgcn_update_dpp(0, __double2loint(v), CTRL, 0xF, 0xF, false);
    const int hi = __builtin_amdgcn_update_dpp(0, __double2hiint(v), CTRL, 0xF, 0xF, false);
    return __hiloint2double(hi, lo);
}
__device__ __forceinline__ double2 quad_sum(double2 v) {  // sum over lanes l ^ 1, l ^ 2 (quad_perm 0xB1, 0x4E)
    v.x += dpp_q<0xB1>(v.x);
    v.y += dpp_q<0xB1>(v.y);
    v.x += dpp_q<0x4E>(v.x);
    v.y += dpp_q<0x4E>(v.y);
    return v;
}

// NCG = 4-column groups per wave: 4 (strips of 16 columns, one wave per SIMD), 2 (strips of 8, twice the waves,
// two per SIMD so one wave's LDS round trips and barrier hide behind the other's MFMAs)
template <int CHI, int QPW, bool STAMP = false, int NCG = 4>
__global__ __launch_bounds__(64 * QPW * (CHI / (4 * NCG)), NCG == 2 ? 2 : (NCG == 1 ? 4 : 1)) void pt_quad_kernel(SweepParams p) {
    constexpr int CW = 4 * NCG;         // columns per wave
    constexpr int NWG = CHI / CW;       // waves per quad (column strips of CW)
    constexpr int KS = CHI / 4;         // k-steps of the contraction
    constexpr int RS = CHI + 1;         // LDS row stride (double2)
    constexpr int QST = 16 * RS;        // one quad's rows (t, alpha)
    extern __shared__ __attribute__((aligned(16))) double2 smem[];
    double2* rp = smem + 2 * QPW * QST;  // closure partials [parity][quad][strip][t][alpha]
    __shared__ int s_lo, s_hi;

    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int q = wave / NWG, h = wave - (wave / NWG) * NWG;
    const int blk = blockIdx.x * QPW + q;
    const bool qvalid = blk < p.n_blk;
    const int ns = p.n_steps, NO = p.n_out;
    const bool fuse = p.fuse != 0;

    // ---- per-lane slot data, C-layout (t = (l >> 2) & 3): state, column operators
    const int la = lane >> 4, lt = (lane >> 2) & 3, lc = lane & 3;
    const int traj = qvalid ? p.blk_traj[blk * 4 + lt] : -1;
    const int act = qvalid ? p.blk_act[blk * 4 + lt] : INT_MAX;
    const int src = qvalid ? p.blk_src[blk * 4 + lt] : -1;
    const int wb = traj >= 0 ? p.wbeg[traj] : INT_MAX, we = traj >= 0 ? p.wend[traj] : -1;
    const int sys = traj >= 0 ? p.traj_sys[traj] : 0;
    int ev_cur = traj >= 0 ? p.ev_start[traj] : 0;
    const int ev_lim = traj >= 0 ? p.ev_start[traj + 1] : 0;
    const int2 wq = fw_win(p, sys);  // pulse window: M, F outside it are the system's idle operators (fw_M, fw_F)
    const int opi = lc * 4 + la;  // this lane's operator element Op[alpha' = lc][alpha = la]
    // ---- T-layout (l = 16 t + 4 k + alpha): the traces, four lanes per (trajectory, output k < 4), reduced over alpha
    // by DPP inside the quad of lanes
    const int t2 = lane >> 4, k2 = (lane >> 2) & 3, a2 = lane & 3;
    const int traj2 = qvalid ? p.blk_traj[blk * 4 + t2] : -1;
    const int act2 = qvalid ? p.blk_act[blk * 4 + t2] : INT_MAX;
    const int wb2 = traj2 >= 0 ? p.wbeg[traj2] : INT_MAX, we2 = traj2 >= 0 ? p.wend[traj2] : -1;
    const long long wo2 = traj2 >= 0 ? p.woff[traj2] : 0;
    const int sys2 = traj2 >= 0 ? p.traj_sys[traj2] : 0;
    const int2 wq2 = fw_win(p, sys2);
    const int k2c = k2 < NO ? k2 : NO - 1;

    // ---- loop bounds: the quad's [first activation, last output], the workgroup's hull (barriers are workgroup-wide)
    int q_lo = INT_MAX, q_hi = -1;
#pragma unroll
    for (int b = 0; b < 4; ++b) {
        const int a_b = __builtin_amdgcn_readlane(act, 4 * b);
        q_lo = a_b < q_lo ? a_b : q_lo;
    }
    if (qvalid) q_hi = p.blk_end[blk];
    if (q_lo == INT_MAX) q_hi = -1;
    if (threadIdx.x == 0) { s_lo = INT_MAX; s_hi = -1; }
    __syncthreads();
    if (lane == 0 && h == 0) { atomicMin(&s_lo, q_lo); atomicMax(&s_hi, q_hi); }
    __syncthreads();
    const int n_lo = s_lo, n_hi = s_hi;
    if (n_hi < 0 || n_lo == INT_MAX) return;  // whole workgroup empty
    const int pbase = (p.qprio & 1) && 2 * (int)blockIdx.x < (int)gridDim.x ? 1 : 0;
    const bool pdyn = (p.qprio & 2) != 0;
    if (p.qprio) set_prio(pbase + (pdyn ? 2 : 0));

    double2* stq = smem + q * QST;        // + parity * QPW * QST
    const int crow = (4 * lt + la) * RS + CW * h + lc;                     // C-layout element (+ 4 cg)
    const int arow = (4 * (lane & 3) + ((lane >> 2) & 3)) * RS + (lane >> 4);  // A-layout element (+ 4 ks)
    const int drow = (4 * (lane >> 4) + ((lane >> 2) & 3)) * RS + CW * h + lc;  // D-layout element (+ 4 cg)

    // ---- initial augmented states (slots active from step 0), before-MTOs at step 0
    double2 R[NCG];
    {
        const double2 r0 = p.rho0[la];
#pragma unroll
        for (int cg = 0; cg < NCG; ++cg)
            R[cg] = (traj >= 0 && act == 0) ? c_mul(r0, p.bond0[CW * h + 4 * cg + lc]) : c_zero();
    }
    int4 evn = ev_cur < ev_lim ? p.ev[ev_cur] : make_int4(INT_MAX, 0, 0, 0);
    {
        const bool has = traj >= 0 && act == 0 && evn.x == 0 && evn.y == 0;
        if (__ballot(has)) {
            const double2 a = has ? p.sop[(size_t)evn.z * 16 + opi] : c_zero();
            quad_col(a, has, R);
            if (has) { ++ev_cur; evn = ev_cur < ev_lim ? p.ev[ev_cur] : make_int4(INT_MAX, 0, 0, 0); }
        }
    }
    bool fz = false;  // this slot holds its state with M_b(n-1) deferred (fused step n)
    int next_act = INT_MAX;
#pragma unroll
    for (int b = 0; b < 4; ++b) {
        const int a_b = __builtin_amdgcn_readlane(act, 4 * b);
        if (a_b > 0 && a_b < next_act) next_act = a_b;
    }

    // ---- operands. Slices (B-layout) and the closure are shared by all trajectories (L2); they are reloaded only
    // when the schedule changes slice (a repeated slice - ACE's _repeated / infinite PTs - stays in registers).
    // F(n), the W(n) rows and the schedule are per system / step (HBM): a two-step ring in registers. The step loop is
    // unrolled by two so the ring needs no register moves (a move from a register whose load is in flight waits for
    // it), and the common path (fused steps, no MTO, no activation) is straight-line, so the compiler's wait counts
    // stay exact and never drain the prefetched loads early.
    const int bl_a = (lane >> 2) & 3, bl_k = lane >> 4;   // B-layout alpha, k'
    const size_t qoff = (size_t)p.gmap[bl_a] * CHI * CHI + (size_t)bl_k * CHI + CW * h + lc;
    const size_t sstride = (size_t)p.D * CHI * CHI;
    double2 B[KS][NCG];
    // Re + Im of B (precomputed per PT: the 3M operand without VALU adds per step) where the registers allow it
    constexpr bool PRESUM = CHI == 16;
    double Bs[PRESUM ? KS : 1][PRESUM ? NCG : 1];
    auto load_slices = [&](int s) {
        const double2* Qs = p.Q + (size_t)s * sstride + qoff;
        const double* Qm = p.Qsum + (size_t)s * sstride + qoff;
#pragma unroll
        for (int ks = 0; ks < KS; ++ks)
#pragma unroll
            for (int cg = 0; cg < NCG; ++cg) {
                B[ks][cg] = Qs[(size_t)4 * ks * CHI + 4 * cg];
                if constexpr (PRESUM) Bs[ks][cg] = Qm[(size_t)4 * ks * CHI + 4 * cg];
            }
    };
    double2 cl[NCG];
    auto load_closure = [&](int s) {  // s < 0: closure0
        const double2* cv = s < 0 ? p.closure0 : p.closure + (size_t)s * CHI;
#pragma unroll
        for (int cg = 0; cg < NCG; ++cg) cl[cg] = cv[CW * h + 4 * cg + lc];
    };
    // unfused plans: the ring reads p.M[0] (unused); the window selects are selects, not branches (the ring loads
    // stay unconditional)
    const size_t fmul = fuse ? 1 : 0;
    auto ldF = [&](int n) {
        const double2* f = fuse ? fw_F(p, sys, wq, n < ns ? n : ns - 1, 16) : p.M;
        return f[fmul * opi];
    };
    auto ldS = [&](int n) { return p.sched[n < ns ? n : ns - 1]; };
    const double2 ov = p.ovec[k2c * 4 + a2];  // T-layout: element (k2, a2) of the output rows (unfused steps)
    double2 fpre[2], wv[2];
    int sr[2];
    auto ldW = [&](int j, int n) {
        const double2* w = fuse ? fw_W(p, sys2, wq2, n <= ns ? n : ns, 4) : p.M;
        wv[j] = w[fmul * ((size_t)k2c * 4 + a2)];
    };
    const int n0 = n_lo;
    int q_cur = __builtin_amdgcn_readfirstlane(ldS(n0));
    int c_cur = n0 == 0 ? -1 : __builtin_amdgcn_readfirstlane(ldS(n0 - 1));
    load_closure(c_cur);
    load_slices(q_cur);
    fpre[0] = ldF(n0); ldW(0, n0); sr[0] = ldS(n0 + 1);
    fpre[1] = ldF(n0 + 1); ldW(1, n0 + 1); sr[1] = ldS(n0 + 2);

    // end of step n: the ring moves one step (slot 0 = step n + 1, loaded a step ago) and slot 1 fetches step n + 2
    auto shift_ring = [&](int n) {
        fpre[0] = fpre[1];
        wv[0] = wv[1];
        sr[0] = sr[1];
        fpre[1] = ldF(n + 2);
        ldW(1, n + 2);
        sr[1] = ldS(n + 3);
    };
    // one step (ring slot 0 = step n). Returns true when the workgroup is done.
    auto step = [&](const int n) -> bool {
        constexpr int S = 0;
        auto stamp = [&](int k) {
            if constexpr (STAMP) {
                if (blockIdx.x == 0 && threadIdx.x == 0 && n >= 1000 && n < 1016)
                    g_quad_stamps[(n - 1000) * 16 + k] = __builtin_amdgcn_s_memtime();
            }
        };
        stamp(0);
        const int par = n & 1;
        double2* st = stq + par * QPW * QST;
        double2* rpp = rp + (par * QPW + q) * NWG * 16;
        const bool qlive = n <= q_hi;  // wave-uniform (per quad)
        // ------------------------------------------------ shared-trunk activations at the top of step n
        if (n == next_act) {
            const int sl = 16 * la + 4 * (src >= 0 ? src : 0) + lc;
            double2 Rs[NCG];
#pragma unroll
            for (int cg = 0; cg < NCG; ++cg) Rs[cg] = make_double2(__shfl(R[cg].x, sl), __shfl(R[cg].y, sl));
            const bool fzs = __shfl((int)fz, sl) != 0;
            if (act == n) {
                if (src >= 0) {
#pragma unroll
                    for (int cg = 0; cg < NCG; ++cg) R[cg] = Rs[cg];
                    fz = fzs;
                } else if (src <= -2) {
                    const double2* ck = p.ck + (size_t)(-2 - src) * 4 * CHI + (size_t)la * CHI + CW * h + lc;
#pragma unroll
                    for (int cg = 0; cg < NCG; ++cg) R[cg] = ck[4 * cg];
                    fz = true;
                }
            }
            next_act = INT_MAX;
#pragma unroll
            for (int b = 0; b < 4; ++b) {
                const int a_b = __builtin_amdgcn_readlane(act, 4 * b);
                if (a_b > n && a_b < next_act) next_act = a_b;
            }
        }
        const bool on = traj >= 0 && n >= act;  // slot active (per lane, uniform per t)
        // ------------------------------------------------ outputs at step n: closure partial of this strip
        const bool win = on && wb <= n && n <= we;
        const bool need = qlive && __ballot(win) != 0 && !(p.ablate & 4);
        const unsigned long long fzb = __ballot(fz);  // bit 4 t: slot t fused (read by the T-layout traces)
        if (need) {
            double2 part = c_zero();
#pragma unroll
            for (int cg = 0; cg < NCG; ++cg) c_fma(part, R[cg], cl[cg]);
            part = quad_sum(part);
            if (lc == 0) rpp[h * 16 + 4 * lt + la] = part;
        }
        if (!qlive) {
            // quad finished: keep the workgroup's barrier count
            if constexpr (NWG > 1 || QPW > 1) __syncthreads();
            return n >= n_hi;
        }
        stamp(1);
        // ------------------------------------------------ column phase A (per slot: F(n), or M_b(n-1), MTOs, M_a(n))
        if (!(p.ablate & 2)) {
            const bool mto_now = evn.x == n;
            if (!__ballot(on && !(fz && !mto_now))) {
                quad_col(fpre[S], on, R);  // every active slot: the fused F(n) alone
            } else {
                // 0 = F(n), 1 = M_b(n-1), 2 = after-MTO at n or else M_a(n); 9 = none left
                int k0 = !on ? 9 : (fz && !mto_now) ? 0 : (fz ? 1 : 2);
                while (__ballot(k0 < 9)) {
                    const bool mine = k0 < 9;
                    double2 a = c_zero();
                    if (k0 == 0) { a = fpre[S]; k0 = 9; }
                    else if (k0 == 1) { a = fw_M(p, opq(sys), wq, 2 * n - 1, 16)[opq(opi)]; k0 = 2; }
                    else if (k0 == 2) {
                        if (evn.x == n && evn.y == 1) {
                            a = p.sop[(size_t)evn.z * 16 + opq(opi)];
                            ++ev_cur;
                            evn = ev_cur < ev_lim ? p.ev[opq(ev_cur)] : make_int4(INT_MAX, 0, 0, 0);
                        } else {
                            a = fw_M(p, opq(sys), wq, 2 * n, 16)[opq(opi)];
                            k0 = 9;
                        }
                    }
                    quad_col(a, mine, R);
                }
            }
        }
        stamp(2);
        // ------------------------------------------------ exchange: this strip's columns -> rows of every wave
#pragma unroll
        for (int cg = 0; cg < NCG; ++cg) st[crow + 4 * cg] = R[cg];
        if constexpr (NWG > 1 || QPW > 1) __syncthreads();
        else asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        stamp(3);
        // ------------------------------------------------ outputs at step n: traces (strip 0), T-layout
        if (need && h == 0) {
            double2 r = rpp[4 * t2 + a2];
#pragma unroll
            for (int g = 1; g < NWG; ++g) r = c_add(r, rpp[g * 16 + 4 * t2 + a2]);
            const bool f2 = (fzb >> (4 * t2)) & 1;
            const bool win2 = traj2 >= 0 && n >= act2 && wb2 <= n && n <= we2;
            const double2 x = quad_sum(c_mul(f2 ? wv[S] : ov, r));
            if (a2 == 0 && win2 && k2 < NO) p.out[wo2 + (long long)(n - wb2) * NO + k2] = x;
            for (int kb = 4; kb < NO; kb += 4) {  // more than four outputs: further passes, rows loaded here
                const int k = kb + k2 < NO ? kb + k2 : NO - 1;
                const double2 w = f2 ? fw_W(p, sys2, wq2, n, 4)[k * 4 + a2] : p.ovec[k * 4 + a2];
                const double2 y = quad_sum(c_mul(w, r));
                if (a2 == 0 && win2 && kb + k2 < NO) p.out[wo2 + (long long)(n - wb2) * NO + kb + k2] = y;
            }
        }
        stamp(4);
        if (n >= n_hi) return true;
        if (n >= q_hi) return false;  // this quad is done; the others still step (next: the !qlive branch)
        // ------------------------------------------------ PT contraction of step n (3M, all rows in one stream)
        double2 D[NCG];
        if (!(p.ablate & 1)) {
            double2 A[KS];
#pragma unroll
            for (int ks = 0; ks < KS; ++ks) A[ks] = st[arow + 4 * ks];
            double p1[NCG] = {}, p2[NCG] = {}, p3[NCG] = {};
#pragma unroll
            for (int ks = 0; ks < KS; ++ks) {
                const double as = A[ks].x + A[ks].y;
#pragma unroll
                for (int cg = 0; cg < NCG; ++cg) {
                    p1[cg] = mfma4(A[ks].x, B[ks][cg].x, p1[cg]);
                    p2[cg] = mfma4(A[ks].y, B[ks][cg].y, p2[cg]);
                    p3[cg] = mfma4(as, PRESUM ? Bs[PRESUM ? ks : 0][PRESUM ? cg : 0] : B[ks][cg].x + B[ks][cg].y, p3[cg]);
                }
            }
#pragma unroll
            for (int cg = 0; cg < NCG; ++cg) D[cg] = make_double2(p1[cg] - p2[cg], p3[cg] - p1[cg] - p2[cg]);
        } else {
            // diagnostics: the rows unchanged (read back in D-layout)
#pragma unroll
            for (int cg = 0; cg < NCG; ++cg) D[cg] = st[drow + 4 * cg];
        }
        if constexpr (STAMP) {  // wait for the contraction's results before the stamp
            if (blockIdx.x == 0 && threadIdx.x == 0 && n >= 1000 && n < 1016 && D[0].x == 12345.678) g_quad_stamps[255] = 1;
        }
        stamp(5);
        // operands ahead, in the order they are needed (loads complete in order): F/W and the schedule of step n + 2
        // into the slot this step used, then (if the slice changes) the closure and the slices of step n + 1
        {
            const int s1 = __builtin_amdgcn_readfirstlane(sr[0]);  // sched[n + 1]
            shift_ring(n);
            if (q_cur != c_cur) { load_closure(q_cur); c_cur = q_cur; }  // closure of step n + 1: sched[n]
            if (s1 != q_cur) { load_slices(s1); q_cur = s1; }
        }
        stamp(6);
        // ------------------------------------------------ D -> C relayout through the next parity's rows
        {
            double2* sn = stq + (par ^ 1) * QPW * QST;
#pragma unroll
            for (int cg = 0; cg < NCG; ++cg) sn[drow + 4 * cg] = D[cg];
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
            for (int cg = 0; cg < NCG; ++cg) R[cg] = sn[crow + 4 * cg];
        }
        stamp(7);
        // ------------------------------------------------ column phase B: M_b(n) and before-MTOs at n+1 unless fused
        const bool fzn = fuse && evn.x != n + 1;
        if (!(p.ablate & 2) && __ballot(on && !fzn)) {
            // 0 = M_b(n), 1 = before-MTO at n+1 (if any); 9 = none left
            int k0 = (on && !fzn) ? 0 : 9;
            while (__ballot(k0 < 9)) {
                bool mine = k0 < 9;
                double2 a = c_zero();
                if (k0 == 0) { a = fw_M(p, opq(sys), wq, 2 * n + 1, 16)[opq(opi)]; k0 = 1; }
                else if (k0 == 1) {
                    if (evn.x == n + 1 && evn.y == 0) {
                        a = p.sop[(size_t)evn.z * 16 + opq(opi)];
                        ++ev_cur;
                        evn = ev_cur < ev_lim ? p.ev[opq(ev_cur)] : make_int4(INT_MAX, 0, 0, 0);
                    } else {
                        mine = false;
                    }
                    k0 = 9;
                }
                quad_col(a, mine, R);
            }
        }
        if (on) fz = fzn;
        stamp(8);
        return false;
    };
    // The common step as one basic block: every active slot fused with no MTO at n or n + 1, no activation at n, the
    // quad still live after n. Its phases are ordered for overlap: the traces of step n and the ring loads of step
    // n + 2 sit between the contraction's MFMAs (the compiler interleaves them within the block), and the closure
    // partial of the next step sits beside its column operator. Critical path per step: D -> C relayout, F(n) on the
    // matrix cores, exchange + barrier, A-operand reads, the contraction.
    // ring slot S (compile time): step n's operands; after use the slot fetches step n + 2 (no register moves,
    // so each fetch has two steps to arrive; see the loop below)
    auto fast = [&](const int n, auto slot, auto reload) {
        constexpr int S = decltype(slot)::value;
        constexpr bool RL = decltype(reload)::value;  // false: the schedule keeps this slice and closure at n + 1
        auto stamp = [&](int k) {
            if constexpr (STAMP) {
                if (blockIdx.x == 0 && threadIdx.x == 0 && n >= 1000 && n < 1016)
                    g_quad_stamps[(n - 1000) * 16 + k] = __builtin_amdgcn_s_memtime();
            }
        };
        stamp(0);
        const int par = n & 1;
        double2* st = stq + par * QPW * QST;
        double2* rpp = rp + (par * QPW + q) * NWG * 16;
        // closure partial of this strip (outputs at step n) beside the column operator F(n)
        {
            double2 part = c_zero();
#pragma unroll
            for (int cg = 0; cg < NCG; ++cg) c_fma(part, R[cg], cl[cg]);
            part = quad_sum(part);
            if (lc == 0) rpp[h * 16 + 4 * lt + la] = part;
        }
        quad_col(fpre[S], true, R);  // every valid slot is active (empty slots hold zeros)
        stamp(1);
#pragma unroll
        for (int cg = 0; cg < NCG; ++cg) st[crow + 4 * cg] = R[cg];
        if constexpr (NWG > 1 || QPW > 1) __syncthreads();
        else asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        stamp(2);
        // contraction of step n
        if (pdyn) set_prio(pbase);
        double2 A[KS];
#pragma unroll
        for (int ks = 0; ks < KS; ++ks) A[ks] = st[arow + 4 * ks];
        double p1[NCG] = {}, p2[NCG] = {}, p3[NCG] = {};
#pragma unroll
        for (int ks = 0; ks < KS; ++ks) {
            if (ks == PQD_QRAISE(KS) && pdyn) set_prio(pbase + 2);
            const double as = A[ks].x + A[ks].y;
#pragma unroll
            for (int cg = 0; cg < NCG; ++cg) {
                p1[cg] = mfma4(A[ks].x, B[ks][cg].x, p1[cg]);
                p2[cg] = mfma4(A[ks].y, B[ks][cg].y, p2[cg]);
                p3[cg] = mfma4(as, PRESUM ? Bs[PRESUM ? ks : 0][PRESUM ? cg : 0] : B[ks][cg].x + B[ks][cg].y, p3[cg]);
            }
        }
        // priority raised again once the MFMAs are issued: the traces, the relayout and the next column operator
        // are the serial chain (C2: 16.0 -> 15.8 ms against raising it after the results, profiles/r03/quad_prio.log)
        if (PQD_QRAISE(KS) >= KS && pdyn) set_prio(pbase + 2);
        // traces of step n (strip 0; every slot is fused: W(n) rows), stored inside each trajectory's window
        if (h == 0) {
            double2 r = rpp[4 * t2 + a2];
#pragma unroll
            for (int g = 1; g < NWG; ++g) r = c_add(r, rpp[g * 16 + 4 * t2 + a2]);
            const double2 x = quad_sum(c_mul(wv[S], r));
            if (a2 == 0 && traj2 >= 0 && n >= act2 && wb2 <= n && n <= we2 && k2 < NO)
                p.out[wo2 + (long long)(n - wb2) * NO + k2] = x;
        }
        // ring loads of step n + 2 into the slot this step used
        const int s1 = RL ? __builtin_amdgcn_readfirstlane(sr[S]) : q_cur;  // sched[n + 1]
        fpre[S] = ldF(n + 2);
        ldW(S, n + 2);
        sr[S] = ldS(n + 3);
        stamp(3);
        double2 D[NCG];
#pragma unroll
        for (int cg = 0; cg < NCG; ++cg) D[cg] = make_double2(p1[cg] - p2[cg], p3[cg] - p1[cg] - p2[cg]);
        if constexpr (STAMP) {  // wait for the contraction's results before the stamp
            if (blockIdx.x == 0 && threadIdx.x == 0 && n >= 1000 && n < 1016 && D[0].x == 12345.678) g_quad_stamps[255] = 1;
        }
        stamp(4);
        // D -> C relayout
        {
            double2* sn = stq + (par ^ 1) * QPW * QST;
#pragma unroll
            for (int cg = 0; cg < NCG; ++cg) sn[drow + 4 * cg] = D[cg];
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
            for (int cg = 0; cg < NCG; ++cg) R[cg] = sn[crow + 4 * cg];
        }
        stamp(5);
        // a new slice (or closure) for step n + 1 only when the schedule changes. The wait sits inside the branch: a
        // load that MAY be in flight at the join makes the compiler wait for every older load at the first use
        // (vmcnt counts in order), i.e. for the ring fetches of step n + 2 just issued, on every step
        if constexpr (RL) {
            if (q_cur != c_cur || s1 != q_cur) {
                if (q_cur != c_cur) { load_closure(q_cur); c_cur = q_cur; }
                if (s1 != q_cur) { load_slices(s1); q_cur = s1; }
                __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0)
            }
        }
        stamp(6);
    };
    // the first step m in (n, lim) whose slice differs from step n's (lim if none): steps n .. m - 2 need no
    // reload check when the closure has caught up (q_cur == c_cur)
    auto same_end = [&](const int n, const int lim) -> int {
        const int s0 = p.sched[n];
        for (int m0 = n + 1; m0 < lim; m0 += 64) {
            const int m = m0 + lane;
            const unsigned long long b = __ballot(m < lim && p.sched[m] != s0);
            if (b) return m0 + (int)__builtin_ctzll(b);
        }
        return lim;
    };
    // step n is fast when n != next_act, n < q_hi, n < n_hi, the plan is fused with <= 4 outputs, and no live
    // trajectory is inactive (n < act), unfused (!fz) or has an MTO at n or n + 1. Fast steps change none of these,
    // so the first step >= n that is not fast is found once, with one wave-wide minimum, instead of two ballots
    // per pair
    auto fast_end = [&](const int n) -> int {
        if (!(fuse && NO <= 4 && !(p.ablate & 31))) return n;
        int e = INT_MAX;
        if (traj >= 0) e = (n < act || !fz) ? n : (evn.x >= n ? (evn.x - 1 > n ? evn.x - 1 : n) : INT_MAX);
#pragma unroll
        for (int o = 32; o >= 1; o >>= 1) {
            const int y = __shfl_xor(e, o);
            e = y < e ? y : e;
        }
        e = __builtin_amdgcn_readfirstlane(e);
        if (next_act >= n && next_act < e) e = next_act;
        if (q_hi < e) e = q_hi;
        if (n_hi < e) e = n_hi;
        return e < n ? n : e;
    };
    for (int n = n0;; ++n) {
        // runs of fast step PAIRS in a loop of their own, one straight-line body over the two ring slots (slot 0
        // holds step n, slot 1 step n + 1 at the top of every pair; each slot fetches two steps ahead, no register
        // moves, so the compiler's wait counts never drain a fetch early); an odd step left over takes step()
        const int fe = fast_end(n);
        while (n + 1 < fe) {
            // a repeated slice (ACE's _repeated / infinite PTs) leaves the schedule constant for long runs: pairs
            // inside such a run skip the reload check and its wait for the schedule fetch
            const int se = q_cur == c_cur ? same_end(n, fe + 1 < ns ? fe + 1 : ns) : n;
            while (n + 2 < se && n + 1 < fe) {
                fast(n, std::integral_constant<int, 0>{}, std::false_type{});
                fast(n + 1, std::integral_constant<int, 1>{}, std::false_type{});
                n += 2;
            }
            if (n + 1 < fe) {
                fast(n, std::integral_constant<int, 0>{}, std::true_type{});
                fast(n + 1, std::integral_constant<int, 1>{}, std::true_type{});
                n += 2;
            }
        }
        if (step(n)) break;
    }
}

template <int CHI, int QPW, int NCG>
hipError_t launch_q(int n_quads, const SweepParams& p, hipStream_t s) {
    constexpr int NWG = CHI / (4 * NCG);
    const size_t lds = (size_t)(2 * QPW * 16 * (CHI + 1) + 2 * QPW * NWG * 16) * sizeof(double2);
    const int grid = (n_quads + QPW - 1) / QPW;
    if (p.ablate & 32)
        hipLaunchKernelGGL((pt_quad_kernel<CHI, QPW, true, NCG>), dim3(grid), dim3(64 * QPW * NWG), lds, s, p);
    else
        hipLaunchKernelGGL((pt_quad_kernel<CHI, QPW, false, NCG>), dim3(grid), dim3(64 * QPW * NWG), lds, s, p);
    return hipGetLastError();
}

}  // namespace

// diagnostics: the stamps of the last PQD_ABLATE=32 launch (16 steps x 16 phase slots)
extern "C" int pqd_debug_quad_stamps(unsigned long long* out) {
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_quad_stamps), sizeof(unsigned long long) * 256) == hipSuccess ? 0 : 4;
}

bool quad_supported(int N2, int CHI) { return N2 == 4 && (CHI == 16 || CHI == 32 || CHI == 64); }

// the instantiated quads per workgroup for a requested qpw: 1 (always at chi = 64) or (chi = 16 with 16-column strips:
// 4 quads of one wave each, a 256-thread workgroup) else 2
int quad_qpw(int CHI, int qpw, int ncg) {
    return (qpw <= 1 || ncg == 1 || CHI == 64) ? 1 : (CHI == 16 && ncg != 2 ? 4 : 2);
}

hipError_t launch_quad(int CHI, int n_quads, int qpw, int ncg, const SweepParams& p, hipStream_t s) {
    if (n_quads <= 0) return hipSuccess;
    const int q = quad_qpw(CHI, qpw, ncg);
    switch (CHI) {
        case 16:
            if (ncg == 2) return q == 2 ? launch_q<16, 2, 2>(n_quads, p, s) : launch_q<16, 1, 2>(n_quads, p, s);
            return q == 4 ? launch_q<16, 4, 4>(n_quads, p, s) : launch_q<16, 1, 4>(n_quads, p, s);
        case 32:
            // ncg = 1 (4-column strips, 8 waves per quad, four waves per SIMD within 128 VGPRs): A/B only (PQD_QCG=1)
            if (ncg == 1) return launch_q<32, 1, 1>(n_quads, p, s);
            if (ncg == 2) return q == 2 ? launch_q<32, 2, 2>(n_quads, p, s) : launch_q<32, 1, 2>(n_quads, p, s);
            return q == 2 ? launch_q<32, 2, 4>(n_quads, p, s) : launch_q<32, 1, 4>(n_quads, p, s);
        case 64:
            // one quad per workgroup: 8-column strips (eight waves, two per SIMD) or 16-column strips (four waves)
            return ncg == 4 ? launch_q<64, 1, 4>(n_quads, p, s) : launch_q<64, 1, 2>(n_quads, p, s);
        default: return hipErrorInvalidValue;
    }
}
