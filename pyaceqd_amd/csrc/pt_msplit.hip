// pt_msplit.hip — split groups that carry several trajectories: a group of G = N2 workgroups propagates TB
// trajectories at once, workgroup g owning PT row alpha = g of every one of them.
//
// Why: the single-trajectory split path (pt_split.hip) fits n_cu / (N2 + 1)
// groups, 15 at N2 = 16, so the 32-t1 rank shard of the C4 sweep and the whole 256-t1 sweep fell to the batched
// kernel: 8 or 64 workgroups, each streaming the whole 1 MiB slice set per step through its CU (≈12.8 µs per
// step). Here every CU streams only its slice row (64 KiB at chi = 64, held in registers while the schedule repeats
// it) and ONE slice read feeds TB trajectories, so 32 trajectories run as 16 groups of 2 on all 256 CUs and 256
// trajectories as 16 groups of 16.
//
// Per step n, row workgroup g of a group:
//   PT(n)     y_b = r_b . S_g(n) for every active trajectory b, r_b = row g of F_b(n) Q_b (from the gather of step
//             n - 1): thread (kq, d) holds S_g[kq KPER + j][d] (j < KPER) in registers, the KG partial sums meet in LDS
//   publish   y_b -> exchange slot n & 1 of trajectory b (8-B sc1 relaxed atomic stores), every storing wave drains
//             (s_waitcnt vmcnt(0)), a barrier, then ONE lane stores the workgroup's arrival word (= n + 1)
//   prefetch  F_b(n + 1) row g, the output rows W_b(n + 1) of the trajectories this workgroup writes, the closure
//             column, then the next slice row when the schedule changes it (issued last: the LDS staging of the small
//             operands waits only for their own loads)
//   poll      wave 0 reads the G arrival words of the group (one relaxed sc1 load per poll), the others wait at a barrier
//   gather    every element of every active state, 16-B sc1 buffer loads of 4 trajectories at a time in flight:
//             thread (kq, c, rg) takes column kq KPER + c of rows rg + 4 i, contracts them with F_b(n + 1)[g][.] and
//             sums the 4 row groups by DPP (quad_perm): r_b for PT(n + 1) lands in the k-range the thread's own
//             k-group contracts (chi <= 64: one wave, no barrier)
//   outputs   trajectory b's outputs are written by workgroup b mod N2 from the state it gathers anyway: <O_k> at
//             step n + 1 = sum W_b(n + 1)[k][beta] Q_b[beta][d] c[d], one wave sum each, the KG wave partials added
//             after the next PT barrier — no output workgroup, so two groups of 16 fit one XCD's 32 CUs
// MTOs: every trajectory-step with an MTO uses a composite operator, F'(n) = M_a(n) S_after S_before M_b(n - 1) and
// W'(n) = ovec S_before M_b(n - 1) (M_b(-1) = 1), built per event on the device after the free propagators
// (evcomp_kernel), so each step of each trajectory is one row operator and one set of output rows (the batched
// kernel's unfused sequence gives the same values to rounding).
// Hand-off and residency as in pt_split.hip (MI355X_MICROARCH.md § visibility "Valid forms" row 1): payload stores
// sc1, drain, barrier, arrival word; polls and payload loads sc1; one workgroup per CU by the LDS request and at most
// n_cu workgroups (host check); every spin is bounded and a timeout ends the kernel with an error word, after which
// the host re-runs the step range on the batched kernel.
#include "pqd_common.h"

namespace {

typedef unsigned long long __attribute__((address_space(1))) mu64;
typedef unsigned int __attribute__((address_space(1))) mu32;
typedef unsigned int v4u32m __attribute__((ext_vector_type(4)));

constexpr int MS_LDS_FORCE = 96 * 1024;  // dynamic LDS request: one workgroup per CU

__device__ __forceinline__ void ms_st_sc1(double2* p, double2 v) {
    __hip_atomic_store((mu64*)&p->x, (unsigned long long)__double_as_longlong(v.x), __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store((mu64*)&p->y, (unsigned long long)__double_as_longlong(v.y), __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_AGENT);
}

// plain global load (global_load, not flat_load: a flat load also counts in lgkmcnt)
__device__ __forceinline__ double2 ms_gld(const double2* p) {
    const __attribute__((address_space(1))) double* q = (const __attribute__((address_space(1))) double*)p;
    return make_double2(q[0], q[1]);
}

__device__ __forceinline__ double2 ms_wave_sum(double2 v) {
    v = c_group_sum<16>(v);
    v = make_double2(xor_add<16>(v.x), xor_add<16>(v.y));
    return make_double2(xor_add<32>(v.x), xor_add<32>(v.y));
}

template <int N2, int CHI>
struct MsLayout {
    static constexpr int KG = 4;                    // k-groups of the row contraction
    static constexpr int KPER = CHI / KG;           // slice rows per thread: 8 / 16 / 32 (chi = 32 / 64 / 128)
    static constexpr int NT = KG * CHI;             // threads: 128 / 256 / 512
    static constexpr int NW = NT / 64;              // waves
    static constexpr int RG = 4;                    // gather row groups: lanes 4 c + rg of a k-group
    static constexpr int EPT = (N2 + RG - 1) / RG;  // state rows per thread and trajectory in the gather
    static constexpr int GCH = CHI == 128 ? 1 : (EPT <= 4 ? 4 : 2);  // trajectories whose gather loads are in flight together
    static constexpr int TBMAX = CHI == 128 ? 16 : 32;
    static constexpr int TBC = CHI == 128 ? 4 : (CHI == 64 ? 16 : 32);  // trajectories per PT pass (LDS partials)
    static constexpr int OMAX = 8;                  // outputs per trajectory
    static constexpr int TMINE = (TBMAX + N2 - 1) / N2;  // trajectories whose outputs one workgroup writes
    static constexpr int FPT = (TBMAX * N2 + NT - 1) / NT;          // F-row entries per thread
    static constexpr int WPT = (TMINE * OMAX * N2 + NT - 1) / NT;   // output-row entries per thread
    static constexpr int PRO = 0;                      // r_b rows [TBMAX][CHI]
    static constexpr int REDO = PRO + TBMAX * CHI;     // PT partials [TBC][NT]
    static constexpr int FRO = REDO + TBC * NT;        // F_b(n + 1) row g [TBMAX][N2]
    static constexpr int WLO = FRO + TBMAX * N2;       // output rows [TMINE][OMAX][N2]
    static constexpr int OPO = WLO + TMINE * OMAX * N2;  // output wave partials [TMINE][OMAX][NW]
    static constexpr int END = OPO + TMINE * OMAX * NW;
    static constexpr int LDS = END * 16 > MS_LDS_FORCE ? END * 16 : MS_LDS_FORCE;
};

template <int N2, int CHI>
__global__ __launch_bounds__(4 * CHI) void pt_msplit_kernel(SweepParams p, MsplitParams q,
                                                                           double2* __restrict__ X,
                                                                           unsigned* __restrict__ cnt,
                                                                           unsigned* __restrict__ err) {
    using L = MsLayout<N2, CHI>;
    constexpr int NT = L::NT, KG = L::KG, KPER = L::KPER, RG = L::RG, EPT = L::EPT, NW = L::NW;
    constexpr int E = N2 * CHI, m2 = N2 * N2;
    static_assert(L::LDS <= 160 * 1024, "LDS budget");
    static_assert(KPER * KG == CHI && CHI / RG == KPER, "gather columns = the k-group's slice rows");
    extern __shared__ __attribute__((aligned(16))) double2 smem[];
    __shared__ int s_abort;
    __shared__ int s_t[L::TBMAX], s_wb[L::TBMAX], s_we[L::TBMAX], s_sy[L::TBMAX];
    __shared__ int s_evs[L::TBMAX], s_evi[L::TBMAX], s_eve[L::TBMAX];
    __shared__ long long s_wo[L::TBMAX];

    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    int grp, g;
    if (q.xcd > 0) {
        // XCD-grouped grid: block b sits in XCD slot b % 8 under the observed round-robin dealing; slot xs holds the
        // groups xs, xs + 8, ... so each group's hand-offs stay in one L2 (speed only, as in pt_split.hip)
        const int xs = blockIdx.x & 7, loc = blockIdx.x >> 3;
        grp = xs + 8 * (loc / N2);
        g = loc - (loc / N2) * N2;
    } else {
        grp = blockIdx.x / N2;
        g = blockIdx.x - grp * N2;
    }
    if (grp >= q.n_groups) return;  // an unused block (before any shared state is touched)
    const int TB = q.TB, n_out = p.n_out;
    const int n_end = q.gend[grp];
    if (tid == 0) s_abort = 0;
    if (tid < TB) {
        const int t = q.gtraj[grp * TB + tid];
        s_t[tid] = t;
        s_wb[tid] = t >= 0 ? p.wbeg[t] : INT_MAX;
        s_we[tid] = t >= 0 ? p.wend[t] : -1;
        s_sy[tid] = t >= 0 ? p.traj_sys[t] : 0;
        s_wo[tid] = t >= 0 ? p.woff[t] : 0;
        const int i0 = t >= 0 ? q.cev_start[t] : 0, i1 = t >= 0 ? q.cev_start[t + 1] : 0;
        s_evi[tid] = i0;
        s_eve[tid] = i1;
        s_evs[tid] = i0 < i1 ? q.cev[i0].x : INT_MAX;
    }
    // exchange of this group: slot (b, parity) of trajectory slot b at X + ((grp TB + b) 2 + parity) E
    double2* __restrict__ Xg = X + (size_t)grp * TB * 2 * E;
    const __amdgpu_buffer_rsrc_t rX = __builtin_amdgcn_make_buffer_rsrc(Xg, 0, TB * 2 * E * 16, 0x00020000);
    unsigned* ct = cnt + (size_t)grp * 64;

    // thread roles: PT (kq, j): slice rows kq KPER + jj, column j; gather (kq, c = j / RG, rg = j % RG): column
    // kcol = kq KPER + c of rows rg + RG i
    const int kq = tid / CHI, j = tid - kq * CHI, cgi = j / RG, rg = j - cgi * RG;
    const int kcol = kq * KPER + cgi;
    const int grow = p.gmap[g];
    double2 sreg[KPER];
    auto fetch_slice = [&](int si) {
        const double2* __restrict__ S = p.Q + ((size_t)si * p.D + grow) * CHI * CHI;
#pragma unroll
        for (int jj = 0; jj < KPER; ++jj) sreg[jj] = ms_gld(S + (size_t)(kq * KPER + jj) * CHI + j);
    };
    // the schedule, 64 entries per VGPR (lane i holds sched[64 c + i]) one chunk ahead, picked with v_readlane
    auto sched_chunk = [&](int ch) {
        const int i = 64 * ch + lane;
        return i < n_end ? *(const __attribute__((address_space(1))) int*)(p.sched + i) : -1;
    };
    int sch_cur = sched_chunk(0), sch_nxt = sched_chunk(1);
    int cur_slice = n_end > 0 ? __builtin_amdgcn_readlane(sch_cur, 0) : -1;
    if (n_end > 0) fetch_slice(cur_slice);
    __syncthreads();

    // ---- step 0: r_b = row g of F_b(0) Q_b(0), Q_b(0) = rho0 (x) bond0, F_b(0) = M_a(0) or the composite at step 0;
    // outputs at step 0 of this workgroup's trajectories directly
    for (int e = tid; e < TB * CHI; e += NT) {
        const int b = e / CHI, k = e - b * CHI;
        if (s_we[b] <= 0) continue;
        const int sy = s_sy[b];
        const double2* __restrict__ Fr =
            (s_evs[b] == 0 ? q.Fev + (size_t)s_evi[b] * m2 : fw_M(p, sy, fw_win(p, sy), 0, m2)) + (size_t)g * N2;
        double2 acc = c_zero();
        for (int be = 0; be < N2; ++be) c_fma(acc, ms_gld(Fr + be), ms_gld(p.rho0 + be));
        smem[L::PRO + b * CHI + k] = c_mul(acc, ms_gld(p.bond0 + k));
    }
    for (int e = tid; e < TB * n_out; e += NT) {
        const int b = e / n_out, k = e - b * n_out;
        if (b % N2 != g || s_wb[b] != 0 || s_we[b] < 0) continue;
        const double2* __restrict__ W0 =
            s_evs[b] == 0 ? q.Wev + (size_t)s_evi[b] * n_out * N2 : p.ovec;
        double2 r = c_zero(), bc = c_zero();
        for (int be = 0; be < N2; ++be) c_fma(r, ms_gld(W0 + (size_t)k * N2 + be), ms_gld(p.rho0 + be));
        for (int d = 0; d < CHI; ++d) c_fma(bc, ms_gld(p.bond0 + d), ms_gld(p.closure0 + d));
        p.out[s_wo[b] + k] = c_mul(r, bc);
    }
    __syncthreads();
    if (tid < TB && s_evs[tid] == 0) {
        const int i = ++s_evi[tid];
        s_evs[tid] = i < s_eve[tid] ? q.cev[i].x : INT_MAX;
    }
    __syncthreads();

    const int tmine = (TB - g + N2 - 1) / N2;  // trajectories b = g + N2 mb whose outputs this workgroup writes
    // the wave partials of the outputs at step n gathered during step n - 1, summed and stored
    auto flush = [&](int n) {
        for (int e = tid; e < tmine * n_out; e += NT) {
            const int mb = e / n_out, k = e - mb * n_out, b = g + N2 * mb;
            if (n < s_wb[b] || n > s_we[b]) continue;
            double2 o = smem[L::OPO + (mb * L::OMAX + k) * NW];
#pragma unroll
            for (int w = 1; w < NW; ++w) o = c_add(o, smem[L::OPO + (mb * L::OMAX + k) * NW + w]);
            p.out[s_wo[b] + (long long)(n - s_wb[b]) * n_out + k] = o;
        }
    };

    double2 fpre[L::FPT], wpre[L::WPT];
#pragma unroll
    for (int i = 0; i < L::FPT; ++i) fpre[i] = c_zero();
#pragma unroll
    for (int i = 0; i < L::WPT; ++i) wpre[i] = c_zero();
    for (int n = 0;; ++n) {
        if (n >= n_end) {
            __syncthreads();
            if (n >= 1) flush(n);
            break;
        }
        // ---- PT(n) for the trajectories that continue past n, TBC at a time (LDS partials)
        for (int b0 = 0; b0 < TB; b0 += L::TBC) {
            const int nb = TB - b0 < L::TBC ? TB - b0 : L::TBC;
            for (int bb = 0; bb < nb; ++bb) {
                const int b = b0 + bb;
                if (n >= s_we[b]) continue;
                double2 acc = c_zero();
#pragma unroll
                for (int j0 = 0; j0 < KPER; j0 += 16) {
                    // at most 16 row values in flight (chi = 128: 32 would add 128 VGPRs to the slice's 128)
#pragma unroll
                    for (int jj = j0; jj < j0 + 16 && jj < KPER; ++jj)
                        c_fma(acc, smem[L::PRO + b * CHI + kq * KPER + jj], sreg[jj]);
                    if (KPER > 16) asm volatile("" ::: "memory");
                }
                smem[L::REDO + bb * NT + tid] = acc;
            }
            __syncthreads();
            if (b0 == 0 && n >= 1) flush(n);
            for (int e = tid; e < nb * CHI; e += NT) {
                const int bb = e / CHI, d = e - bb * CHI, b = b0 + bb;
                if (n >= s_we[b]) continue;
                double2 y = smem[L::REDO + bb * NT + d];
#pragma unroll
                for (int k2 = 1; k2 < KG; ++k2) y = c_add(y, smem[L::REDO + bb * NT + k2 * CHI + d]);
                ms_st_sc1(Xg + ((size_t)b * 2 + (n & 1)) * E + (size_t)g * CHI + d, y);
            }
            if (b0 + L::TBC < TB) __syncthreads();  // REDO reused by the next pass
        }
        // ---- arrive (every storing wave drained, then one lane)
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        if (tid == 0) __hip_atomic_store((mu32*)(ct + g), (unsigned)n + 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        // ---- operands of step m = n + 1: F rows, output rows, closure column, then the slice row
        const int m = n + 1;
#pragma unroll
        for (int i = 0; i < L::FPT; ++i) {
            const int e = tid + NT * i;
            if (e < TB * N2) {
                const int b = e / N2, be = e - b * N2;
                if (m < s_we[b]) {
                    const int sy = s_sy[b];
                    const double2* __restrict__ Fr =
                        s_evs[b] == m ? q.Fev + (size_t)s_evi[b] * m2 : fw_F(p, sy, fw_win(p, sy), m, m2);
                    fpre[i] = ms_gld(Fr + (size_t)g * N2 + be);
                }
            }
        }
        const int wrow = n_out * N2;
#pragma unroll
        for (int i = 0; i < L::WPT; ++i) {
            const int e = tid + NT * i;
            const int mb = e / wrow, r = e - mb * wrow, b = g + N2 * mb;
            if (mb < tmine && m >= s_wb[b] && m <= s_we[b]) {
                const int sy = s_sy[b];
                const double2* __restrict__ Wr =
                    s_evs[b] == m ? q.Wev + (size_t)s_evi[b] * wrow : fw_W(p, sy, fw_win(p, sy), m, N2);
                wpre[i] = ms_gld(Wr + r);
            }
        }
        const double2 cvr = ms_gld(p.closure + (size_t)cur_slice * CHI + kcol);  // sched[n]: the slice PT(n) used
        if (m < n_end) {
            if ((m & 63) == 0) { sch_cur = sch_nxt; sch_nxt = sched_chunk((m >> 6) + 1); }
            const int ns = __builtin_amdgcn_readlane(sch_cur, m & 63);
            if (ns != cur_slice) {
                fetch_slice(ns);
                cur_slice = ns;
            }
        }
#pragma unroll
        for (int i = 0; i < L::FPT; ++i) {
            const int e = tid + NT * i;
            if (e < TB * N2) smem[L::FRO + e] = fpre[i];
        }
#pragma unroll
        for (int i = 0; i < L::WPT; ++i) {
            const int e = tid + NT * i;
            const int mb = e / wrow, r = e - mb * wrow;
            if (mb < tmine) smem[L::WLO + (mb * L::OMAX) * N2 + r] = wpre[i];
        }
        // ---- wait for the group
        if (tid < 64) {
            const unsigned want = (unsigned)n + 1u;
            unsigned spins = 0;
            bool ok = true;
            for (;;) {
                const unsigned v =
                    lane < N2 ? __hip_atomic_load((mu32*)(ct + lane), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : want;
                if (__all(v >= want)) break;
                __builtin_amdgcn_s_sleep(1);
                if (++spins > p.spin_limit) { ok = false; break; }
            }
            if (tid == 0) {
                s_abort = ok ? 0 : 1;
                if (!ok) __hip_atomic_store((mu32*)err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
        }
        __syncthreads();
        if (s_abort) return;
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");  // compiler ordering only: payload loads are sc1
        // composites of step m consumed (every reader of s_evs for m ran before the barrier above)
        if (tid < TB && s_evs[tid] == m) {
            const int i = ++s_evi[tid];
            s_evs[tid] = i < s_eve[tid] ? q.cev[i].x : INT_MAX;
        }
        // ---- gather slot n & 1: r_b(m) into PRO, output partials of this workgroup's trajectories
        for (int b0 = 0; b0 < TB; b0 += L::GCH) {
            v4u32m xr[L::GCH][EPT];
#pragma unroll
            for (int bb = 0; bb < L::GCH; ++bb) {
                const int b = b0 + bb;
                if (b < TB && n < s_we[b]) {
#pragma unroll
                    for (int i = 0; i < EPT; ++i) {
                        const int be = rg + RG * i;
                        const int off = (int)((((size_t)b * 2 + (n & 1)) * E + (size_t)(be < N2 ? be : 0) * CHI + kcol) * 16);
                        xr[bb][i] = __builtin_amdgcn_raw_buffer_load_b128(rX, off, 0, 16);
                    }
                }
            }
#pragma unroll
            for (int bb = 0; bb < L::GCH; ++bb) {
                const int b = b0 + bb;
                if (b >= TB || n >= s_we[b]) continue;
                double2 xv[EPT];
#pragma unroll
                for (int i = 0; i < EPT; ++i)
                    xv[i] = make_double2(__hiloint2double((int)xr[bb][i].y, (int)xr[bb][i].x),
                                         __hiloint2double((int)xr[bb][i].w, (int)xr[bb][i].z));
                if (m < s_we[b]) {
                    double2 part = c_zero();
#pragma unroll
                    for (int i = 0; i < EPT; ++i)
                        if (rg + RG * i < N2) c_fma(part, smem[L::FRO + b * N2 + rg + RG * i], xv[i]);
                    part = c_group_sum<4>(part);
                    if (rg == 0) smem[L::PRO + b * CHI + kcol] = part;
                }
                if (b % N2 == g && m >= s_wb[b]) {
                    const int mb = b / N2;
#pragma unroll
                    for (int i = 0; i < EPT; ++i) xv[i] = c_mul(xv[i], cvr);
                    for (int k = 0; k < n_out; ++k) {
                        double2 o = c_zero();
#pragma unroll
                        for (int i = 0; i < EPT; ++i)
                            if (rg + RG * i < N2) c_fma(o, smem[L::WLO + (mb * L::OMAX + k) * N2 + rg + RG * i], xv[i]);
                        o = ms_wave_sum(o);
                        if (lane == 0) smem[L::OPO + (mb * L::OMAX + k) * NW + wv] = o;
                    }
                }
            }
        }
        if constexpr (CHI > 64) __syncthreads();  // a k-group spans two waves: r_b from both before PT(m)
    }
}

// composite operators of the MTO steps: one workgroup per composite event e (trajectory t at step s)
//   P  = S_before M_b(s - 1)        (M_b(-1) = 1, S = 1 where the slot has no MTO)
//   Wev[e] = ovec P                 (n_out x N2)
//   Fev[e] = M_a(s) S_after P       (s < n_steps; zero otherwise: no PT after the last step)
template <int N2>
__global__ __launch_bounds__(256) void evcomp_kernel(SweepParams p, MsplitParams q, int n_cev, int n_steps) {
    constexpr int m2 = N2 * N2;
    __shared__ double2 A[m2], B[m2], Cm[m2];
    const int tid = threadIdx.x;
    for (int e = blockIdx.x; e < n_cev; e += gridDim.x) {
        const int4 ce = q.cev[e];  // (step, sop before or -1, sop after or -1, system)
        const int s = ce.x, sy = ce.w;
        const int2 wn = fw_win(p, sy);
        __syncthreads();
        for (int i = tid; i < m2; i += 256) {
            const int r = i / N2, c = i - r * N2;
            A[i] = s >= 1 ? ms_gld(fw_M(p, sy, wn, 2 * (s - 1) + 1, m2) + i) : make_double2(r == c ? 1.0 : 0.0, 0.0);
            if (ce.y >= 0) B[i] = ms_gld(p.sop + (size_t)ce.y * m2 + i);
        }
        __syncthreads();
        auto mul = [&](const double2* Lm, const double2* Rm, double2* Out) {  // Out = Lm Rm (LDS, all threads)
            for (int i = tid; i < m2; i += 256) {
                const int r = i / N2, c = i - r * N2;
                double2 acc = c_zero();
                for (int k = 0; k < N2; ++k) c_fma(acc, Lm[r * N2 + k], Rm[k * N2 + c]);
                Out[i] = acc;
            }
            __syncthreads();
        };
        double2* P = A;
        if (ce.y >= 0) { mul(B, A, Cm); P = Cm; }
        for (int i = tid; i < p.n_out * N2; i += 256) {
            const int k = i / N2, c = i - k * N2;
            double2 acc = c_zero();
            for (int b = 0; b < N2; ++b) c_fma(acc, ms_gld(p.ovec + (size_t)k * N2 + b), P[b * N2 + c]);
            q.Wev[(size_t)e * p.n_out * N2 + i] = acc;
        }
        double2* R = P == A ? Cm : A;  // the free buffer
        if (ce.z >= 0) {
            __syncthreads();
            for (int i = tid; i < m2; i += 256) B[i] = ms_gld(p.sop + (size_t)ce.z * m2 + i);
            __syncthreads();
            mul(B, P, R);
            double2* t = P; P = R; R = t;
        }
        __syncthreads();
        for (int i = tid; i < m2; i += 256) B[i] = s < n_steps ? ms_gld(fw_M(p, sy, wn, 2 * s, m2) + i) : c_zero();
        __syncthreads();
        mul(B, P, R);
        for (int i = tid; i < m2; i += 256) q.Fev[(size_t)e * m2 + i] = R[i];
    }
}

template <int N2, int CHI>
hipError_t launch_ms_t(const SweepParams& p, const MsplitParams& q, double2* X, unsigned* cnt, unsigned* err,
                       int n_blocks, hipStream_t s) {
    using L = MsLayout<N2, CHI>;
    static unsigned attr = 0;  // per-device bitmask
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) return hipErrorInvalidDevice;
    if (dev < 32 && !(attr & (1u << dev))) {
        hipError_t e = hipFuncSetAttribute((const void*)pt_msplit_kernel<N2, CHI>,
                                           hipFuncAttributeMaxDynamicSharedMemorySize, (int)L::LDS);
        if (e != hipSuccess) return e;
        attr |= 1u << dev;
    }
    hipLaunchKernelGGL((pt_msplit_kernel<N2, CHI>), dim3(n_blocks), dim3(L::NT), L::LDS, s, p, q, X, cnt, err);
    return hipGetLastError();
}

template <int N2, int CHI>
int ms_occ_t() {
    using L = MsLayout<N2, CHI>;
    if (hipFuncSetAttribute((const void*)pt_msplit_kernel<N2, CHI>, hipFuncAttributeMaxDynamicSharedMemorySize,
                            (int)L::LDS) != hipSuccess)
        return 0;
    int nb = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, pt_msplit_kernel<N2, CHI>, L::NT, L::LDS) != hipSuccess)
        return 0;
    return nb;
}

template <int N2>
hipError_t launch_ms_n(int CHI, const SweepParams& p, const MsplitParams& q, double2* X, unsigned* cnt,
                       unsigned* err, int n_blocks, hipStream_t s) {
    switch (CHI) {
        case 32: return launch_ms_t<N2, 32>(p, q, X, cnt, err, n_blocks, s);
        case 64: return launch_ms_t<N2, 64>(p, q, X, cnt, err, n_blocks, s);
        default: return hipErrorInvalidValue;
    }
}

template <int N2>
int ms_occ_n(int CHI) {
    switch (CHI) {
        case 32: return ms_occ_t<N2, 32>();
        case 64: return ms_occ_t<N2, 64>();
        default: return 0;
    }
}

}  // namespace

int msplit_tbmax(int CHI) { return CHI == 128 ? 16 : 32; }

bool msplit_supported(int N2, int CHI, int n_out) {
    return (N2 == 9 || N2 == 16 || N2 == 25 || N2 == 36) && (CHI == 32 || CHI == 64) &&
           n_out >= 1 && n_out <= 8;
}

int msplit_blocks_per_cu(int N2, int CHI) {
    switch (N2) {
        case 9: return ms_occ_n<9>(CHI);
        case 16: return ms_occ_n<16>(CHI);
        case 25: return ms_occ_n<25>(CHI);
        case 36: return ms_occ_n<36>(CHI);
        default: return 0;
    }
}

hipError_t launch_evcomp(int N2, const SweepParams& p, const MsplitParams& q, int n_cev, int n_steps, hipStream_t s) {
    if (n_cev <= 0) return hipSuccess;
    const dim3 grid((unsigned)(n_cev < 4096 ? n_cev : 4096));
    switch (N2) {
        case 9: hipLaunchKernelGGL((evcomp_kernel<9>), grid, dim3(256), 0, s, p, q, n_cev, n_steps); break;
        case 16: hipLaunchKernelGGL((evcomp_kernel<16>), grid, dim3(256), 0, s, p, q, n_cev, n_steps); break;
        case 25: hipLaunchKernelGGL((evcomp_kernel<25>), grid, dim3(256), 0, s, p, q, n_cev, n_steps); break;
        case 36: hipLaunchKernelGGL((evcomp_kernel<36>), grid, dim3(256), 0, s, p, q, n_cev, n_steps); break;
        default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

// X: n_groups * TB * 2 * N2 * CHI double2; cnt: n_groups * 64 arrival words; err: 4 words (all zeroed here)
hipError_t launch_msplit(int N2, int CHI, const SweepParams& p, const MsplitParams& q, double2* X, unsigned* cnt,
                         unsigned* err, hipStream_t s) {
    hipError_t e = hipMemsetAsync(cnt, 0, (size_t)q.n_groups * 64 * sizeof(unsigned), s);
    if (e != hipSuccess) return e;
    e = hipMemsetAsync(err, 0, 4 * sizeof(unsigned), s);
    if (e != hipSuccess) return e;
    const int n_blocks = q.xcd > 0 ? 8 * q.xcd * N2 : q.n_groups * N2;
    switch (N2) {
        case 9: return launch_ms_n<9>(CHI, p, q, X, cnt, err, n_blocks, s);
        case 16: return launch_ms_n<16>(CHI, p, q, X, cnt, err, n_blocks, s);
        case 25: return launch_ms_n<25>(CHI, p, q, X, cnt, err, n_blocks, s);
        case 36: return launch_ms_n<36>(CHI, p, q, X, cnt, err, n_blocks, s);
        default: return hipErrorInvalidValue;
    }
}
