// pt_msplit.hip — split groups that carry several trajectories: a group of G = ceil(N2 / R) workgroups propagates
// TB trajectories at once, workgroup g owning PT rows alpha = R g + h (h < R) of every one of them.
//
// Why: the single-trajectory split path (pt_split.hip) fits n_cu / (N2 + 1)
// groups, 15 at N2 = 16, so the 32-t1 rank shard of the C4 sweep and the whole 256-t1 sweep fell to the batched
// kernel: 8 or 64 workgroups, each streaming the whole 1 MiB slice set per step through its CU (≈12.3 µs per
// step). Here every CU holds only its R slice rows (R x 64 KiB at chi = 64, in registers while the schedule repeats
// them), ONE slice read feeds TB trajectories, and 32 trajectories run as 32 groups of one on all 256 CUs.
//
// A workgroup is R "halves" of HT = 4 CHI threads; half h owns row alpha_h = R g + h. Per step n:
//   PT(n)     half h: y_b = r_b^h . S_alpha_h(n) for every active trajectory b, r_b^h = row alpha_h of F_b(n) Q_b
//             (from the gather of step n - 1): thread (kq, d) holds S[kq KPER + j][d] (j < KPER) in registers; a
//             wave's four 16-lane rows are the four k-groups of 16 columns, summed by permlane swaps
//   publish   y_b -> exchange slot n & 1 of trajectory b (16-B stores that keep the line in the group's L2, or 8-B
//             sc1 relaxed atomic stores: l2keep), every storing wave drains (s_waitcnt vmcnt(0)), a barrier, then ONE
//             lane stores the workgroup's arrival word (= n + 1, with its XCD id)
//   operands  F_b(n + 1) rows and the output rows W_b(n + 1) were loaded into registers during step n - 1: they go to
//             LDS now and the loads of step n + 2's are issued (an operand load never sits between a publish and a
//             poll); then the next slice rows when the schedule changes them
//   poll      wave 0 reads the G arrival words of the group (one relaxed sc1 load per poll), the others wait at a barrier
//   gather    half h takes the trajectories b = h, h + R, ...: every element of each state by 16-B sc1 buffer loads,
//             up to 4 trajectories' loads in flight per thread; thread (kq, c, rg) takes column kq KPER + c of rows
//             rg + 4 i (consecutive lanes consecutive columns) and contracts them with F_b(n + 1)[alpha][.] for all R
//             rows of the workgroup (each element is loaded once per workgroup), the 4 row groups summed by permlane
//             swaps; one barrier, then PT(n + 1)
//   outputs   trajectory b's outputs are written by workgroup b mod G (the half that gathers b) from the state it
//             loads anyway: <O_k>(n + 1) = sum W_b(n + 1)[k][beta] Q_b[beta][d] c[d], one wave sum each, the wave
//             partials added after the next PT barrier — no output workgroup
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
constexpr int MS_CEV_MAX = 512;          // composite events per group held in LDS (msplit_cev_max)
constexpr unsigned MS_STEP_MASK = 0x0FFFFFFFu;  // arrival word: step n + 1 in bits 0..27, the writer's XCD id above
// s_getreg_b32 hwreg(HW_REG_XCC_ID, 0, 4): register id 20, offset 0, size 4 (simm16 = (size - 1) << 11 | offset << 6 | id)
constexpr int MS_HWREG_XCC_ID = (3 << 11) | (0 << 6) | 20;
template <int V>
struct MsIC {  // compile-time int tag (the gather's chunk variants)
    static constexpr int value = V;
};

__device__ __forceinline__ void ms_st_sc1(double2* p, double2 v) {
    __hip_atomic_store((mu64*)&p->x, (unsigned long long)__double_as_longlong(v.x), __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store((mu64*)&p->y, (unsigned long long)__double_as_longlong(v.y), __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_AGENT);
}

// sum over the 4 row groups of a gather column (lanes 8 / 16 apart at KPER = 8, 16 / 32 apart otherwise), left in all
// four lanes with the same bits (each step adds the same pair: row_ror:8 inside a 16-lane row, then permlane swaps)
template <int KP>
__device__ __forceinline__ double2 ms_rg_sum(double2 v) {
    if constexpr (KP == 8) {
        v = c_add(v, make_double2(dpp_d<0x128>(v.x), dpp_d<0x128>(v.y)));
        return make_double2(xor_add<16>(v.x), xor_add<16>(v.y));
    } else {
        v = make_double2(xor_add<16>(v.x), xor_add<16>(v.y));
        return make_double2(xor_add<32>(v.x), xor_add<32>(v.y));
    }
}

// two sums over the 4 row groups of a gather column at KPER >= 16 (row groups = 16-lane rows): the lanes of the even
// row groups get a's sum, those of the odd ones b's. v_permlane16_swap exchanges the odd 16-lane rows of its first
// operand with the even rows of its second, so after swapping (a, b) an even row holds a and its odd neighbour's a,
// an odd row b and its even neighbour's b; one permlane32 sum then adds the other pair (the same grouping, and bits,
// as two ms_rg_sum calls, at half their instructions)
__device__ __forceinline__ double ms_pair16(double u, double v) {
    const long long U = __double_as_longlong(u), V = __double_as_longlong(v);
    const auto lo = __builtin_amdgcn_permlane16_swap((unsigned)U, (unsigned)V, false, false);
    const auto hi = __builtin_amdgcn_permlane16_swap((unsigned)(U >> 32), (unsigned)(V >> 32), false, false);
    return __longlong_as_double(((long long)hi[0] << 32) | (unsigned)lo[0]) +
           __longlong_as_double(((long long)hi[1] << 32) | (unsigned)lo[1]);
}
__device__ __forceinline__ double2 ms_rg_sum2(double2 a, double2 b) {
    const double2 h = make_double2(ms_pair16(a.x, b.x), ms_pair16(a.y, b.y));
    return make_double2(xor_add<32>(h.x), xor_add<32>(h.y));
}

// plain 16-B global store: the line stays in the XCD's L2 (an sc1 store drops it, and the same-XCD readers then fetch
// it at the cross-XCD rate, MI355X_MICROARCH.md § visibility, store flavours). Used only where every workgroup of the
// group runs on one XCD (checked at the first poll: see l2keep)
__device__ __forceinline__ void ms_st_keep(double2* p, double2 v) {
    typedef double v2f64 __attribute__((ext_vector_type(2)));
    v2f64 w = {v.x, v.y};
    *(__attribute__((address_space(1))) v2f64*)p = w;
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

template <int N2, int CHI, int R>
struct MsLayout {
    static constexpr int KG = 4;                    // k-groups of a row contraction
    static constexpr int KPER = CHI / KG;           // slice rows per thread: 8 / 16 (chi = 32 / 64)
    static constexpr int HT = KG * CHI;             // threads per half (one PT row): 128 / 256
    static constexpr int NT = R * HT;               // threads per workgroup
    static constexpr int NW = NT / 64, NWH = HT / 64;
    static constexpr int G = (N2 + R - 1) / R;      // workgroups per group
    static constexpr int RG = 4;                    // gather row groups: lanes 4 c + rg of a k-group
    static constexpr int EPT = (N2 + RG - 1) / RG;  // state rows per thread and trajectory in the gather
    static constexpr int GCH = CHI > 64 ? 1 : (R >= 4 ? 2 : (EPT <= 4 ? 4 : 1));  // trajectories per half with gather loads in flight
    static constexpr int PVR = (KPER + 15) / 16;   // registers of 16 row values (DPP row broadcast in the PT)
    static constexpr int TBMAX = CHI > 64 ? 8 : (R == 1 ? 32 : (R == 2 ? 16 : 8));
    static constexpr int OMAX = 8;                  // outputs per trajectory
    static constexpr int TMINE = (TBMAX + G - 1) / G;  // trajectories whose outputs one workgroup writes
    static constexpr int FPT = (R * TBMAX * N2 + NT - 1) / NT;      // F-row entries per thread
    static constexpr int WPT = (TMINE * OMAX * N2 + NT - 1) / NT;   // output-row entries per thread
    static constexpr int PRS = CHI + 4;                  // r_b row stride: the MFMA PT's A reads (rows b, k-steps) in distinct banks
    static constexpr int PRO = 0;                        // r_b rows [R][TBMAX][PRS]
    static constexpr int FRO = PRO + R * TBMAX * PRS;    // F_b(n + 1) rows of the workgroup [R][TBMAX][N2]
    static constexpr int WLO = FRO + R * TBMAX * N2;     // output rows [TMINE][OMAX][N2]
    static constexpr int CLO = WLO + TMINE * OMAX * N2;  // closure vector of the outputs the gather writes [CHI]
    static constexpr int OPO = CLO + CHI;                // output columns (W row x state, times the closure) [TMINE][OMAX][CHI]
    static constexpr int DUMMY = OPO + TMINE * OMAX * CHI;  // write target of out-of-range operand entries
    static constexpr int END = DUMMY + 1;
    static constexpr int LDS = END * 16 > MS_LDS_FORCE ? END * 16 : MS_LDS_FORCE;
};

// diagnostics (PQD_ABLATE bit 64, scripts/msplit_stamps.py): s_memtime at the phase boundaries of steps 1000..1015 in
// workgroups 0 and 1 of group 0 (thread 0): [wg][step][slot 0..31]
__device__ unsigned long long g_ms_stamps[2 * 16 * 32];

template <int N2, int CHI, int R, bool STAMP = false>
__global__ __launch_bounds__(4 * CHI * R) void pt_msplit_kernel(SweepParams p, MsplitParams q,
                                                                 double2* __restrict__ X, unsigned* __restrict__ cnt,
                                                                 unsigned* __restrict__ err) {
    using L = MsLayout<N2, CHI, R>;
    constexpr int NT = L::NT, HT = L::HT, KG = L::KG, KPER = L::KPER, RG = L::RG, EPT = L::EPT, NW = L::NW;
    constexpr int G = L::G, E = N2 * CHI, m2 = N2 * N2, TBM = L::TBMAX;
    static_assert(L::LDS + 4 + 32 * L::TBMAX + 4 * MS_CEV_MAX + 8 * (L::FPT + L::WPT) * L::NT <= 160 * 1024,
                  "LDS budget (dynamic + static)");
    static_assert(KPER * KG == CHI && CHI / RG == KPER, "gather columns = the k-group's slice rows");
    extern __shared__ __attribute__((aligned(16))) double2 smem[];
    __shared__ int s_abort;
    __shared__ int s_wb[TBM], s_we[TBM], s_sy[TBM];
    __shared__ int s_evs[TBM], s_evi[TBM], s_eve[TBM];  // first composite step, its index, the end of the list
    __shared__ int s_cvo[TBM];                          // where trajectory slot b's composite steps start in s_cev
    __shared__ int s_cev[MS_CEV_MAX];                   // the group's composite steps (host: at most MS_CEV_MAX)
    __shared__ long long s_wo[TBM];

    const int tid = threadIdx.x, lane = tid & 63;
    const int h = R == 1 ? 0 : __builtin_amdgcn_readfirstlane(tid / HT), ht = tid - h * HT;  // half (wave-uniform), thread in it
    int grp, g;
    if (q.xcd > 0) {
        // XCD-grouped grid: block b sits in XCD slot b % 8 under the observed round-robin dealing; slot xs holds the
        // groups xs, xs + 8, ... so each group's hand-offs stay in one L2 (speed only, as in pt_split.hip)
        const int xs = blockIdx.x & 7, loc = blockIdx.x >> 3;
        grp = xs + 8 * (loc / G);
        g = loc - (loc / G) * G;
    } else {
        grp = blockIdx.x / G;
        g = blockIdx.x - grp * G;
    }
    if (grp >= q.n_groups) return;  // an unused block (before any shared state is touched)
    const int TB = q.TB, n_out = p.n_out;
    const int n_end = q.gend[grp];
    // phase stamps: 0 top, 1 PT partials (barrier), 2 published + arrived, 3 operands staged, 4 peers arrived (poll +
    // barrier), 5 gather loads and operand loads issued, 6 first chunk's loads returned, 7 gather done, 8 end barrier;
    // per wave w < 8: 16 + w first chunk's loads returned, 24 + w gather done
    auto stamp = [&](int n, int k) {
        if constexpr (STAMP) {
            if (grp == 0 && g < 2 && threadIdx.x == 0 && n >= 1000 && n < 1016)
                g_ms_stamps[(g * 16 + (n - 1000)) * 32 + k] = __builtin_amdgcn_s_memtime();
        }
    };
    // per wave (lane 0 of waves 0..7): slot base + wave
    auto wstamp = [&](int n, int base) {
        if constexpr (STAMP) {
            if (grp == 0 && g < 2 && lane == 0 && tid < 8 * 64 && n >= 1000 && n < 1016)
                g_ms_stamps[(g * 16 + (n - 1000)) * 32 + base + (tid >> 6)] = __builtin_amdgcn_s_memtime();
        }
    };
    const int alpha = R * g + h;          // this half's PT row
    const bool live = alpha < N2;         // (the last workgroup of a group may own fewer than R rows)
    if (tid == 0) s_abort = 0;
    if (tid < TB) {
        const int t = q.gtraj[grp * TB + tid];
        s_wb[tid] = t >= 0 ? p.wbeg[t] : INT_MAX;
        s_we[tid] = t >= 0 ? p.wend[t] : -1;
        s_sy[tid] = t >= 0 ? p.traj_sys[t] : 0;
        s_wo[tid] = t >= 0 ? p.woff[t] : 0;
        const int i0 = t >= 0 ? q.cev_start[t] : 0, i1 = t >= 0 ? q.cev_start[t + 1] : 0;
        s_evi[tid] = i0;
        s_eve[tid] = i1;
        s_evs[tid] = i0 < i1 ? q.cev[i0].x : INT_MAX;
    }
    // exchange of this group: slot (b, parity) at Xg + (2 b + parity) E
    double2* __restrict__ Xg = X + (size_t)grp * TB * 2 * E;
    const __amdgpu_buffer_rsrc_t rX = __builtin_amdgcn_make_buffer_rsrc(Xg, 0, TB * 2 * E * 16, 0x00020000);
    unsigned* ct = cnt + (size_t)grp * 64;
    // l2keep (XCD-grouped grid): payload stores keep their lines in the XCD's L2, which is coherent for the readers'
    // sc1 loads only if every workgroup of the group runs on that XCD. Each arrival word carries its writer's XCD id
    // (bits 28..30, HW_REG_XCC_ID) and the first poll checks them; a group spread over XCDs ends the launch before its
    // first gather (error words 0 and 1) and the host re-runs it with sc1 stores. PQD_ABLATE bit 512 fakes a spread
    // group (workgroup 0 reports the next XCD) for the test of that path.
    unsigned xtag = 0;
    if (q.l2keep) {
        unsigned xid = (unsigned)__builtin_amdgcn_s_getreg(MS_HWREG_XCC_ID) & 7u;
        if ((p.ablate & 512) && g == 0) xid = (xid + 1u) & 7u;
        xtag = xid << 28;
    }

    // thread roles in its half: PT column j = 16 (wave in the half) + lane % 16 and the lane's 16-lane row kq. The
    // VALU PT (q.ptm = 0) holds slice rows kq KPER + jj of column j; the matrix-core PT (q.ptm = 1) holds rows
    // 4 jj + kq, the B operand of v_mfma_f64_4x4x4_4b at k-step jj (lane 16 k + 4 blk + x: B[blk][k][x] = S[4 jj + k]
    // [16 w + 4 blk + x]). The gather's roles are set in the step loop
    const int kq = (ht & 63) >> 4, j = 16 * (ht >> 6) + (ht & 15);
    const int grow = live ? p.gmap[alpha] : 0;
    // chi = 128: the VALU path only (its slice row alone is 128 VGPRs; streaming it instead, as at chi = 256, removes
    // the spills but measured slower: single run 51-53 ms against 42-45, profiles/r06/stream128/); chi = 256 (STREAM):
    // the slice row (1 MiB) is streamed from L2 through the matrix-core PT every step, and sreg is unused
    constexpr bool STREAM = CHI > 128;
    const bool ptm = STREAM || (CHI <= 64 && q.ptm != 0);
    double2 sreg[STREAM ? 1 : KPER];
    auto fetch_slice = [&](int si) {
        if constexpr (STREAM) return;
        if (!live) return;
        const double2* __restrict__ S = p.Q + ((size_t)si * p.D + grow) * CHI * CHI;
#pragma unroll
        for (int jj = 0; jj < KPER; ++jj)
            sreg[jj] = ms_gld(S + (size_t)(ptm ? 4 * jj + kq : kq * KPER + jj) * CHI + j);
    };
    // the schedule, 64 entries per VGPR (lane i holds sched[64 c + i]) one chunk ahead, picked with v_readlane
    auto sched_chunk = [&](int ch) {
        const int i = 64 * ch + lane;
        return i < n_end ? *(const __attribute__((address_space(1))) int*)(p.sched + i) : -1;
    };
    int sch_reg = sched_chunk(0);  // the chunk of sched[m] for the coming step's m = n + 1, loaded a step ahead
    int cur_slice = n_end > 0 ? __builtin_amdgcn_readlane(sch_reg, 0) : -1;
    if (n_end > 0) fetch_slice(cur_slice);
    __syncthreads();

    // composite event index of trajectory b at step 0 (-1: none); step 0 only — the loop keeps per-entry cursors
    auto comp0 = [&](int b) { return s_evs[b] == 0 ? s_evi[b] : -1; };

    // ---- step 0: r_b^h = row alpha_h of F_b(0) Q_b(0), Q_b(0) = rho0 (x) bond0, F_b(0) = M_a(0) or the composite at
    // step 0; outputs at step 0 of this workgroup's trajectories directly
    for (int e = tid; e < R * TB * CHI; e += NT) {
        const int r = e / (TB * CHI), b = (e / CHI) % TB, k = e % CHI, a = R * g + r;
        if (s_we[b] <= 0 || a >= N2) continue;
        const int sy = s_sy[b], ci = comp0(b);
        const double2* __restrict__ Fr =
            (ci >= 0 ? q.Fev + (size_t)ci * m2 : fw_M(p, sy, fw_win(p, sy), 0, m2)) + (size_t)a * N2;
        double2 acc = c_zero();
        for (int be = 0; be < N2; ++be) c_fma(acc, ms_gld(Fr + be), ms_gld(p.rho0 + be));
        smem[L::PRO + (r * TBM + b) * L::PRS + k] = c_mul(acc, ms_gld(p.bond0 + k));
    }
    for (int e = tid; e < TB * n_out; e += NT) {
        const int b = e / n_out, k = e - b * n_out;
        if (b % G != g || s_wb[b] != 0 || s_we[b] < 0) continue;
        const int ci = comp0(b);
        const double2* __restrict__ W0 = ci >= 0 ? q.Wev + (size_t)ci * n_out * N2 : p.ovec;
        double2 r = c_zero(), bc = c_zero();
        for (int be = 0; be < N2; ++be) c_fma(r, ms_gld(W0 + (size_t)k * N2 + be), ms_gld(p.rho0 + be));
        for (int d = 0; d < CHI; ++d) c_fma(bc, ms_gld(p.bond0 + d), ms_gld(p.closure0 + d));
        p.out[s_wo[b] + k] = c_mul(r, bc);
    }

    // the group's composite steps into LDS, so an operand entry's cursor advances with LDS reads: a global load there
    // would leave a register pending across the step loop, and the waits for it (in-order vmcnt) would hold the gather
    __syncthreads();
    if (tid == 0) {
        int o = 0;
        for (int b = 0; b < TB; ++b) { s_cvo[b] = o; o += s_eve[b] - s_evi[b]; }
        s_abort = o > MS_CEV_MAX;  // the host never launches such a group (msplit_cev_max); refuse rather than overrun
        if (s_abort) __hip_atomic_store((mu32*)err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    __syncthreads();
    if (s_abort) return;
    for (int b = 0; b < TB; ++b)
        for (int i = tid; i < s_eve[b] - s_evi[b]; i += NT) s_cev[s_cvo[b] + i] = q.cev[s_evi[b] + i].x;
    __syncthreads();

    const int tmine = (TB - g + G - 1) / G;  // trajectories b = g + G mb whose outputs this workgroup writes
    const int wrow = n_out * N2;
    // per-step activity as wave-uniform bit masks (bit b = trajectory slot b): lane b < TB holds its window
    const int my_wb = lane < TB ? s_wb[lane] : INT_MAX, my_we = lane < TB ? s_we[lane] : -1;
    auto mask = [](bool c) { return (unsigned long long)__ballot(c); };

    // operand entries, fixed for the launch: F entry i = (row a, slot b, column be) of F_b(m)[a][be]; W entry i =
    // (output slot mb, element rr) of W_b(m). Each keeps its trajectory's system base, window and a composite cursor
    // (next composite step / index / end) in registers, so the per-step loads need no LDS reads or table lookups. The
    // split paths run without pulse windows (pqd_host.cpp: windows only for the quad and no-PT kernels), so F(m) and
    // W(m) are the stored operators.
    // cursors: ci = position in s_cev, ce = its end, cg = global composite index - position, cs = s_cev[ci] or INT_MAX
    const double2* fbase[L::FPT];
    // the rarely used cursor fields (position, end, global offset, row) live in LDS, one slot per thread and entry:
    // in registers they pushed the gather past the VGPR budget, and the spill reloads' vmcnt waits sat among the
    // gather's loads
    // packed: [0] = position | end << 10 | row << 20 (positions <= MS_CEV_MAX, rows < N2 * N2 or n_out * N2), [1] =
    // global composite index - position
    static_assert(MS_CEV_MAX < 1024 && N2 * N2 < 2048 && L::OMAX * N2 < 2048, "cursor packing");
    __shared__ int s_fcur[2][L::FPT * NT], s_wcur[2][L::WPT * NT];
    int f_we[L::FPT], f_cs[L::FPT];
    const double2* wbase[L::WPT];
    int w_wb[L::WPT], w_we[L::WPT], w_cs[L::WPT];
    auto first_comp = [&](int b, int from, int& cs, int& ci, int& ce, int& cg) {
        int i = s_cvo[b];
        ce = i + s_eve[b] - s_evi[b];
        cg = s_evi[b] - i;
        while (i < ce && s_cev[i] < from) ++i;
        ci = i;
        cs = i < ce ? s_cev[i] : INT_MAX;
    };
#pragma unroll
    for (int i = 0; i < L::FPT; ++i) {
        const int e = tid + NT * i;
        const bool in = e < R * TB * N2;
        const int r = in ? e / (TB * N2) : 0, b = in ? (e / N2) % TB : 0, be = e % N2, a = R * g + r;
        fbase[i] = p.F + (size_t)s_sy[b] * p.f_stride + a * N2 + be;
        f_we[i] = (in && a < N2) ? s_we[b] : -1;
        int ci, ce, cg;
        first_comp(b, 1, f_cs[i], ci, ce, cg);
        s_fcur[0][i * NT + tid] = ci | (ce << 10) | ((a * N2 + be) << 20);
        s_fcur[1][i * NT + tid] = cg;
    }
#pragma unroll
    for (int i = 0; i < L::WPT; ++i) {
        const int e = tid + NT * i;
        const int mb = e / wrow, rr = e - mb * wrow;
        const bool in = mb < tmine;
        const int b = in ? g + G * mb : 0;

        wbase[i] = p.W + (size_t)s_sy[b] * p.w_stride + rr;
        w_wb[i] = in ? s_wb[b] : INT_MAX;
        w_we[i] = in ? s_we[b] : -1;
        int ci, ce, cg;
        first_comp(b, 1, w_cs[i], ci, ce, cg);
        s_wcur[0][i * NT + tid] = ci | (ce << 10) | (rr << 20);
        s_wcur[1][i * NT + tid] = cg;
    }
    // operands of step m into registers (staged into LDS one step later). Every lane issues the same number of loads
    // (entries it does not need read rho0[0]), so the gather's waits can leave them in flight.
    double2 fpre[L::FPT], wpre[L::WPT];
    double2 clv = c_zero();  // the closure vector of the outputs at step m + 1 (the slice PT(m) uses), with step m's operands
    auto load_ops = [&](int m) {
#pragma unroll
        for (int i = 0; i < L::FPT; ++i) {
            const double2* src = p.rho0;
            if (m < f_we[i]) {
                src = fbase[i] + (size_t)m * m2;
                if (m >= f_cs[i]) {  // rare: a composite at m (cursor moved past composites before m)
                    const int pk = s_fcur[0][i * NT + tid];
                    int ci = pk & 1023;
                    const int ce = (pk >> 10) & 1023;
                    while (f_cs[i] < m) { ++ci; f_cs[i] = ci < ce ? s_cev[ci] : INT_MAX; }
                    if (f_cs[i] == m) {
                        src = q.Fev + (size_t)(ci + s_fcur[1][i * NT + tid]) * m2 + (pk >> 20);
                        ++ci;
                        f_cs[i] = ci < ce ? s_cev[ci] : INT_MAX;
                    }
                    s_fcur[0][i * NT + tid] = (pk & ~1023) | ci;
                }
            }
            fpre[i] = ms_gld(src);
        }
#pragma unroll
        for (int i = 0; i < L::WPT; ++i) {
            const double2* src = p.rho0;
            if (m >= w_wb[i] && m <= w_we[i]) {
                src = wbase[i] + (size_t)m * wrow;
                if (m >= w_cs[i]) {
                    const int pk = s_wcur[0][i * NT + tid];
                    int ci = pk & 1023;
                    const int ce = (pk >> 10) & 1023;
                    while (w_cs[i] < m) { ++ci; w_cs[i] = ci < ce ? s_cev[ci] : INT_MAX; }
                    if (w_cs[i] == m) {
                        src = q.Wev + (size_t)(ci + s_wcur[1][i * NT + tid]) * wrow + (pk >> 20);
                        ++ci;
                        w_cs[i] = ci < ce ? s_cev[ci] : INT_MAX;
                    }
                    s_wcur[0][i * NT + tid] = (pk & ~1023) | ci;
                }
            }
            wpre[i] = ms_gld(src);
        }
    };
    // every entry is written (out-of-range ones to a dummy slot): a load consumed on some paths only stays pending in
    // the waitcnt pass across the loop, and a later wait for it would hold the gather's loads (vmcnt is in order)
    auto stage_ops = [&]() {
#pragma unroll
        for (int i = 0; i < L::FPT; ++i) {
            const int e = tid + NT * i;
            const int r = e / (TB * N2), be = e % (TB * N2);
            smem[e < R * TB * N2 ? L::FRO + r * TBM * N2 + be : L::DUMMY] = fpre[i];
        }
#pragma unroll
        for (int i = 0; i < L::WPT; ++i) {
            const int e = tid + NT * i;
            const int mb = e / wrow, rr = e - mb * wrow;
            smem[mb < tmine ? L::WLO + (mb * L::OMAX) * N2 + rr : L::DUMMY] = wpre[i];
        }
        smem[tid < CHI ? L::CLO + tid : L::DUMMY] = clv;
    };
    // outputs at step n: the CHI output columns the gather of step n - 1 left per (trajectory, output), summed by one
    // wave each and stored. Run by waves 1.. while wave 0 polls (first = 1), or by every wave after the last step
    auto flush = [&](int n, int first) {
        const int nw = NW - first, w = (tid >> 6) - first;
        for (int e = w; e < tmine * n_out; e += nw) {
            const int mb = e / n_out, k = e - mb * n_out, b = g + G * mb;
            if (n < s_wb[b] || n > s_we[b]) continue;
            double2 o = c_zero();
#pragma unroll
            for (int c = lane; c < CHI; c += 64) o = c_add(o, smem[L::OPO + (mb * L::OMAX + k) * CHI + c]);
            o = ms_wave_sum(o);
            if (lane == 0) p.out[s_wo[b] + (long long)(n - s_wb[b]) * n_out + k] = o;
        }
    };
    load_ops(1);
    clv = ms_gld(p.closure + (size_t)(n_end > 0 ? cur_slice : 0) * CHI + (tid & (CHI - 1)));
    __syncthreads();

    for (int n = 0;; ++n) {
        stamp(n, 0);
        if (n >= n_end) {
            __syncthreads();
            if (n >= 1) flush(n, 0);
            break;
        }
        const int m = n + 1;
        const unsigned long long act = mask(n < my_we);                      // PT(n), published, gathered
        const unsigned long long nxt = mask(m < my_we);                      // r_b for PT(m)
        const unsigned long long own = mask(lane < TB && lane % G == g && m >= my_wb && m <= my_we);  // outputs at m
        // ---- PT(n), half h: row alpha_h of every trajectory that continues past n. Wave w of the half takes columns
        // 16 w .. 16 w + 15 and its four 16-lane rows the four k-groups (KPER slice rows each): lane i of row kq reads
        // row value kq KPER + 16 c + i (one ds_read_b128 per wave and 64 values), the products take it by DPP
        // row_newbcast, two permlane swaps add the k-groups, and row 0 stores the 16 columns — no LDS partials and no
        // barrier between the PT and the publish. The row values of PF trajectories are read at once
        if (live && ptm) {
            // on the matrix cores, three real products per complex product (3M: P1 = Xr Sr, P2 = Xi Si, P3 = (Xr + Xi)
            // (Sr + Si); y = (P1 - P2, P3 - P1 - P2)), two row blocks of 4 trajectories per pass: lane 16 k + 4 blk + x
            // reads A = X[4 rb + x][4 jj + k] (rows PRS apart: distinct banks) and ends up holding y[4 rb + k][j]. Rows
            // of slots past TB or inactive are contracted too (each output row depends on its own input row only) and
            // not stored
            const int x = lane & 3;
            const double2* __restrict__ xr = smem + L::PRO + h * TBM * L::PRS + kq;
            for (int rb0 = 0; rb0 < TB; rb0 += 8) {
                double p1[2] = {0.0, 0.0}, p2[2] = {0.0, 0.0}, p3[2] = {0.0, 0.0};
                const bool two = rb0 + 4 < TB;
                auto kstep = [&](int jj, double2 bv) {
                    const double qs = bv.x + bv.y;
                    const double2 a0 = xr[(rb0 + x) * L::PRS + 4 * jj];
                    p1[0] = __builtin_amdgcn_mfma_f64_4x4x4f64(a0.x, bv.x, p1[0], 0, 0, 0);
                    p2[0] = __builtin_amdgcn_mfma_f64_4x4x4f64(a0.y, bv.y, p2[0], 0, 0, 0);
                    p3[0] = __builtin_amdgcn_mfma_f64_4x4x4f64(a0.x + a0.y, qs, p3[0], 0, 0, 0);
                    if (two) {
                        const double2 a1 = xr[(rb0 + 4 + x) * L::PRS + 4 * jj];
                        p1[1] = __builtin_amdgcn_mfma_f64_4x4x4f64(a1.x, bv.x, p1[1], 0, 0, 0);
                        p2[1] = __builtin_amdgcn_mfma_f64_4x4x4f64(a1.y, bv.y, p2[1], 0, 0, 0);
                        p3[1] = __builtin_amdgcn_mfma_f64_4x4x4f64(a1.x + a1.y, qs, p3[1], 0, 0, 0);
                    }
                };
                if constexpr (STREAM) {
                    // B = S[4 jj + kq][j] of this row's slice, 4 k-steps of loads at a time (L2-resident: every
                    // workgroup of the step reads the same slices)
                    const double2* __restrict__ Sg =
                        p.Q + ((size_t)cur_slice * p.D + grow) * CHI * CHI + (size_t)kq * CHI + j;
                    constexpr int PFS = CHI > 128 ? 4 : 8;
                    for (int j0 = 0; j0 < KPER; j0 += PFS) {
                        double2 bq[PFS];
#pragma unroll
                        for (int u = 0; u < PFS; ++u) bq[u] = ms_gld(Sg + (size_t)4 * (j0 + u) * CHI);
#pragma unroll
                        for (int u = 0; u < PFS; ++u) kstep(j0 + u, bq[u]);
                    }
                } else {
#pragma unroll
                    for (int jj = 0; jj < KPER; ++jj) kstep(jj, sreg[jj]);
                }
#pragma unroll
                for (int u = 0; u < 2; ++u) {
                    const int b = rb0 + 4 * u + kq;
                    if (b < TB && ((act >> b) & 1)) {
                        double2* dst = Xg + ((size_t)b * 2 + (n & 1)) * E + (size_t)alpha * CHI + j;
                        const double2 y = make_double2(p1[u] - p2[u], p3[u] - p1[u] - p2[u]);
                        if (q.l2keep) ms_st_keep(dst, y); else ms_st_sc1(dst, y);
                    }
                }
            }
        }
        if constexpr (!STREAM) {
            if (live && !ptm) {
                constexpr int PF = CHI <= 32 ? 8 : (CHI <= 64 ? 4 : 1);
                for (int b0 = 0; b0 < TB; b0 += PF) {
                    double2 pv[PF][L::PVR];
#pragma unroll
                    for (int u = 0; u < PF; ++u)
#pragma unroll
                        for (int c = 0; c < L::PVR; ++c) {
                            const int jv = 16 * c + (lane & 15), bu = b0 + u < TBM ? b0 + u : TBM - 1;
                            pv[u][c] = smem[L::PRO + (h * TBM + bu) * L::PRS + kq * KPER + (jv < KPER ? jv : KPER - 1)];
                        }
#pragma unroll
                    for (int u = 0; u < PF; ++u) {
                        const int b = b0 + u;
                        if (b >= TB || !((act >> b) & 1)) continue;
                        double2 acc = c_zero();
                        pq_dpp_src_ready(pv[u]);
                        pq_row_bcast_mac<0, KPER>(acc, pv[u], sreg);
                        acc = make_double2(xor_add<16>(acc.x), xor_add<16>(acc.y));
                        acc = make_double2(xor_add<32>(acc.x), xor_add<32>(acc.y));
                        if (lane < 16) {
                            double2* dst = Xg + ((size_t)b * 2 + (n & 1)) * E + (size_t)alpha * CHI + j;
                            if (q.l2keep) ms_st_keep(dst, acc); else ms_st_sc1(dst, acc);
                        }
                    }
                }
            }
        }
        stamp(n, 1);
        // ---- arrive (every storing wave drained, then one lane). The builtin tells the waitcnt pass that nothing is
        // pending past this point (the operand loads of the last gather included); the asm keeps the wait where it is
        __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0) expcnt(7) lgkmcnt(15)
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        if (tid == 0) {
            // with the group's placement on one XCD verified (first poll, l2keep) the arrival word is a plain store
            // too: its line stays in the group's L2, where the peers' sc1 polls find it without a fabric round trip
            const unsigned av = ((unsigned)n + 1u) | xtag;
            if (q.l2keep && n >= 1) *(__attribute__((address_space(1))) unsigned*)(ct + g) = av;
            else __hip_atomic_store((mu32*)(ct + g), av, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        stamp(n, 2);
        // ---- operands of step n + 1 (loaded during step n - 1's gather) to LDS
        stage_ops();
        stamp(n, 3);
        // step n + 2's operand loads, the closure column of the outputs at step n + 2 (the slice PT(n + 1) uses) and the
        // slice rows of step n + 1 are issued in the gather, behind its first loads (the vmcnt waits are in order: issued
        // here they would sit in front of the gather's)
        // (all of them unconditional but the slice rows: a path with fewer loads after the gather's would make the
        // waitcnt pass wait for the gather with a smaller count on every path)
        auto issue_ops = [&]() {
            if constexpr (STAMP) {  // timing-only ablation (results not used): 128 no operand loads
                if (!(p.ablate & 128)) load_ops(m + 1);
            } else {
                load_ops(m + 1);  // entries past their window read rho0[0]
            }
            const int ns = m < n_end ? __builtin_amdgcn_readlane(sch_reg, m & 63) : cur_slice;
            sch_reg = sched_chunk((m + 1) >> 6);
            clv = ms_gld(p.closure + (size_t)ns * CHI + (tid & (CHI - 1)));
            if (ns != cur_slice) {
                fetch_slice(ns);
                cur_slice = ns;
            }
        };
        // ---- wait for the group (wave 0); the other waves store the outputs of step n meanwhile
        if (tid >= 64 && n >= 1) flush(n, 1);
        if (tid < 64) {
            const unsigned want = (unsigned)n + 1u;
            unsigned spins = 0;
            bool ok = true;
            bool placed = true;
            for (;;) {
                const unsigned v =
                    lane < G ? __hip_atomic_load((mu32*)(ct + lane), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : want;
                if (__all((v & MS_STEP_MASK) >= want)) {
                    // first poll: every peer's XCD id is in its word; the same words reach every workgroup of the group,
                    // so all of them take the same decision
                    if (q.l2keep && n == 0) {
                        const unsigned x0 = __builtin_amdgcn_readfirstlane(v) >> 28;
                        placed = __all(lane >= G || (v >> 28) == x0);
                    }
                    break;
                }
                __builtin_amdgcn_s_sleep(1);
                if (++spins > p.spin_limit) { ok = false; break; }
            }
            if (tid == 0) {
                s_abort = ok && placed ? 0 : 1;
                if (!placed) __hip_atomic_store((mu32*)(err + 1), 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                if (s_abort) __hip_atomic_store((mu32*)err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
        }
        __syncthreads();
        if (s_abort) return;
        stamp(n, 4);
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");  // compiler ordering only: payload loads are sc1
        // ---- gather slot n & 1, half h: trajectories b = h + R i; r_b^{r}(m) for the R rows into PRO, output partials
        // of this workgroup's trajectories
        // the first chunk is peeled (first = true: the operand loads are issued behind its gather loads); a loop body
        // shared by chunks with and without those loads would wait for the gather with the smaller count
        // the gather's thread roles recomputed from an opaque copy of the thread index each step: derived from the
        // launch-time values, the compiler kept a dozen precomputed LDS addresses alive across the loop, spilled
        // them, and each reload's vmcnt wait held the gather behind the operand and slice loads
        // Lanes: 16 (KPER = 8: 8) consecutive lanes take consecutive columns of one row, so a wave's 16-B load is
        // four (eight) contiguous 256-B (128-B) runs; with the row group in the low lane bits every lane was its own
        // request, 16 B per cycle per CU instead of 51.6 (scripts/ubench/gather_bw.hip)
        int tg = tid;
        asm volatile("" : "+v"(tg));
        const int gw = (tg & (HT - 1)) >> 6, gl = tg & 63;
        int rg, kcol;
        if constexpr (KPER == 8) {
            rg = (gl >> 3) & 3;
            kcol = (2 * gw + (gl >> 5)) * KPER + (gl & 7);
        } else if constexpr (KPER == 16) {
            rg = gl >> 4;
            kcol = gw * KPER + (gl & 15);
        } else {  // KPER = 32 / 64: a k-group spans KPER / 16 waves
            rg = gl >> 4;
            kcol = (gw / (KPER / 16)) * KPER + 16 * (gw % (KPER / 16)) + (gl & 15);
        }
        const double2 cv = smem[L::CLO + kcol];
        auto chunk = [&](auto gct, auto firstt, int b0) {
            constexpr int GC = decltype(gct)::value;
            constexpr bool FIRST = decltype(firstt)::value != 0;
            // every slot's loads are issued and waited for on every path (an idle slot reads element 0, one line for the
            // whole wave): loads that are consumed on some paths only stay pending in the waitcnt pass across the loops,
            // and the waits it then puts in front of the next chunk's loads serialised the chunk's round trips
            v4u32m xr[GC][EPT];
            // timing-only variants (STAMP builds): 2048 rotates the chunk's trajectory order by the workgroup index,
            // 1024 points every gather load at element 0, 8192 those of half 1 (results not used)
            int rot = 0;
            if constexpr (STAMP) rot = (p.ablate & 2048) ? g : 0;
            auto slot_b = [&](int bb) { return b0 + R * (GC > 1 ? (bb + rot) % GC : bb); };
#pragma unroll
            for (int bb = 0; bb < GC; ++bb) {
                const int b = slot_b(bb);
                const bool on = b < TB && ((act >> b) & 1);
#pragma unroll
                for (int i = 0; i < EPT; ++i) {
                    const int be = rg + RG * i;
                    int off = on ? (int)((((size_t)b * 2 + (n & 1)) * E + (size_t)(be < N2 ? be : 0) * CHI + kcol) * 16)
                                 : 0;
                    if constexpr (STAMP) off = ((p.ablate & 1024) || ((p.ablate & 8192) && h == 1)) ? 0 : off;
                    xr[bb][i] = __builtin_amdgcn_raw_buffer_load_b128(rX, off, 0, 16);
                }
            }
            if constexpr (FIRST) {
                __builtin_amdgcn_sched_barrier(0);
                issue_ops();
                __builtin_amdgcn_sched_barrier(0);
                stamp(n, 5);
            }
            // each trajectory's loads are waited for right before its arithmetic (in issue order: the counted
            // vmcnt leaves the later trajectories' loads in flight) and on every path, used or not
#pragma unroll
            for (int i = 0; i < EPT; ++i) asm volatile("" ::"v"(xr[0][i]));
            if constexpr (FIRST) { stamp(n, 6); wstamp(n, 16); }
#pragma unroll
            for (int bb = 0; bb < GC; ++bb) {
#pragma unroll
                for (int i = 0; i < EPT; ++i) asm volatile("" ::"v"(xr[bb][i]));
                const int b = slot_b(bb);
                if (b >= TB || !((act >> b) & 1)) continue;
                double2 xv[EPT];
#pragma unroll
                for (int i = 0; i < EPT; ++i)
                    xv[i] = make_double2(__hiloint2double((int)xr[bb][i].y, (int)xr[bb][i].x),
                                         __hiloint2double((int)xr[bb][i].w, (int)xr[bb][i].z));
                // the operand entries of a row are read from LDS together and then used (read one by one next to
                // their products, each read's latency was exposed: ≈9,300 cycles for 8 trajectories' rows)
                if ((nxt >> b) & 1) {
                    if constexpr (R == 2 && KPER >= 16 && EPT <= 4) {
                        // both rows at once: one butterfly sums row 0 into the even row groups and row 1 into the odd
                        // ones (ms_rg_sum2), and one store writes both
                        double2 part[2] = {c_zero(), c_zero()};
#pragma unroll
                        for (int r = 0; r < 2; ++r) {
                            double2 fv[EPT];
#pragma unroll
                            for (int i = 0; i < EPT; ++i) {
                                const int be = rg + RG * i;
                                fv[i] = smem[L::FRO + (r * TBM + b) * N2 + (be < N2 ? be : 0)];
                            }
#pragma unroll
                            for (int i = 0; i < EPT; ++i)
                                if (rg + RG * i < N2) c_fma(part[r], fv[i], xv[i]);
                        }
                        const double2 sum = ms_rg_sum2(part[0], part[1]);
                        if (rg < 2 && 2 * g + rg < N2) smem[L::PRO + (rg * TBM + b) * L::PRS + kcol] = sum;
                    } else {
#pragma unroll
                        for (int r = 0; r < R; ++r) {
                            if (R * g + r >= N2) continue;
                            double2 fv[EPT];
#pragma unroll
                            for (int i = 0; i < EPT; ++i) {
                                const int be = rg + RG * i;
                                fv[i] = smem[L::FRO + (r * TBM + b) * N2 + (be < N2 ? be : 0)];
                            }
                            double2 part = c_zero();
#pragma unroll
                            for (int i = 0; i < EPT; ++i)
                                if (rg + RG * i < N2) c_fma(part, fv[i], xv[i]);
                            part = ms_rg_sum<KPER>(part);
                            if (rg == 0) smem[L::PRO + (r * TBM + b) * L::PRS + kcol] = part;
                        }
                    }
                }
                if ((own >> b) & 1) {
                    // output column kcol of W(m)[k] . Q times the closure: like a row of r_b, the sum over columns
                    // is left to flush (next step, while wave 0 polls)
                    const int mb = b / G;
                    if constexpr (KPER >= 16 && EPT <= 4) {
                        // two outputs per butterfly (k0 in the even row groups, k0 + 1 in the odd ones)
                        for (int k0 = 0; k0 < n_out; k0 += 2) {
                            double2 o[2] = {c_zero(), c_zero()};
#pragma unroll
                            for (int u = 0; u < 2; ++u) {
                                double2 wv[EPT];
#pragma unroll
                                for (int i = 0; i < EPT; ++i) {
                                    const int be = rg + RG * i;
                                    wv[i] = smem[L::WLO + (mb * L::OMAX + k0 + u) * N2 + (be < N2 ? be : 0)];
                                }
#pragma unroll
                                for (int i = 0; i < EPT; ++i)
                                    if (rg + RG * i < N2) c_fma(o[u], wv[i], xv[i]);
                            }
                            const double2 sum = ms_rg_sum2(o[0], o[1]);
                            if (rg < 2 && k0 + rg < n_out)
                                smem[L::OPO + (mb * L::OMAX + k0 + rg) * CHI + kcol] = c_mul(sum, cv);
                        }
                    } else {
                        for (int k = 0; k < n_out; ++k) {
                            double2 wv[EPT];
#pragma unroll
                            for (int i = 0; i < EPT; ++i) {
                                const int be = rg + RG * i;
                                wv[i] = smem[L::WLO + (mb * L::OMAX + k) * N2 + (be < N2 ? be : 0)];
                            }
                            double2 o = c_zero();
#pragma unroll
                            for (int i = 0; i < EPT; ++i)
                                if (rg + RG * i < N2) c_fma(o, wv[i], xv[i]);
                            o = ms_rg_sum<KPER>(o);
                            if (rg == 0) smem[L::OPO + (mb * L::OMAX + k) * CHI + kcol] = c_mul(o, cv);
                        }
                    }
                }
            }
                };
        // the first chunk is peeled and sized to the half's trajectories (idle slots still cost their loads' issue)
        // half hg's trajectories are b = hg, hg + R, ...; at R = 2 odd workgroups swap the halves so that half 0 (whose
        // loads the CU serves first) gathers the trajectories whose outputs this workgroup writes (b = g mod G)
        const int hg = R == 2 ? (h ^ (g & 1)) : h;
        const int nh = hg < TB ? (TB - hg + R - 1) / R : 0;  // trajectories of this half
        int fc = 0;
        if constexpr (L::GCH >= 4) {
            // (three trajectories too: one idle slot, one round trip; a chunk of 2 and one of 4 with 3 idle slots
            // took two, and a third chunk size made the compiler spill ≈1,000 VGPRs)
            if (nh >= 3) { chunk(MsIC<4>{}, MsIC<1>{}, hg); fc = 4; }
        }
        if (fc == 0 && nh >= 2 && L::GCH >= 2) { chunk(MsIC<(L::GCH >= 2 ? 2 : 1)>{}, MsIC<1>{}, hg); fc = L::GCH >= 2 ? 2 : 1; }
        if (fc == 0 && nh >= 1) { chunk(MsIC<1>{}, MsIC<1>{}, hg); fc = 1; }
        if (fc == 0) issue_ops();
        for (int b0 = hg + R * fc; b0 < TB; b0 += R * L::GCH) chunk(MsIC<L::GCH>{}, MsIC<0>{}, b0);
        stamp(n, 7);
        wstamp(n, 24);
        __syncthreads();  // r_b from every half before PT(m)
        stamp(n, 8);
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
        double2* Rb = P == A ? Cm : A;  // the free buffer
        if (ce.z >= 0) {
            __syncthreads();
            for (int i = tid; i < m2; i += 256) B[i] = ms_gld(p.sop + (size_t)ce.z * m2 + i);
            __syncthreads();
            mul(B, P, Rb);
            double2* t = P; P = Rb; Rb = t;
        }
        __syncthreads();
        for (int i = tid; i < m2; i += 256) B[i] = s < n_steps ? ms_gld(fw_M(p, sy, wn, 2 * s, m2) + i) : c_zero();
        __syncthreads();
        mul(B, P, Rb);
        for (int i = tid; i < m2; i += 256) q.Fev[(size_t)e * m2 + i] = Rb[i];
    }
}

template <int N2, int CHI, int R, bool STAMP = false>
hipError_t launch_ms_t(const SweepParams& p, const MsplitParams& q, double2* X, unsigned* cnt, unsigned* err,
                       hipStream_t s) {
    using L = MsLayout<N2, CHI, R>;
    if constexpr (!STAMP && N2 == 16 && CHI == 64) {
        if (p.ablate & 64) return launch_ms_t<N2, CHI, R, true>(p, q, X, cnt, err, s);
    }
    static unsigned attr = 0;  // per-device bitmask
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) return hipErrorInvalidDevice;
    if (dev >= 32 || !(attr & (1u << dev))) {
        hipError_t e = hipFuncSetAttribute((const void*)pt_msplit_kernel<N2, CHI, R, STAMP>,
                                           hipFuncAttributeMaxDynamicSharedMemorySize, (int)L::LDS);
        if (e != hipSuccess) return e;
        if (dev < 32) attr |= 1u << dev;
    }
    const int n_blocks = q.xcd > 0 ? 8 * q.xcd * L::G : q.n_groups * L::G;
    hipLaunchKernelGGL((pt_msplit_kernel<N2, CHI, R, STAMP>), dim3(n_blocks), dim3(L::NT), L::LDS, s, p, q, X, cnt,
                       err);
    return hipGetLastError();
}

template <int N2, int CHI, int R>
int ms_occ_t() {
    using L = MsLayout<N2, CHI, R>;
    if (hipFuncSetAttribute((const void*)pt_msplit_kernel<N2, CHI, R>, hipFuncAttributeMaxDynamicSharedMemorySize,
                            (int)L::LDS) != hipSuccess)
        return 0;
    int nb = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, pt_msplit_kernel<N2, CHI, R>, L::NT, L::LDS) != hipSuccess)
        return 0;
    return nb;
}

// rows per workgroup: 2 (each trajectory's state gathered by half as many workgroups, the slice rows 128 KiB per CU
// at chi = 64 in the registers of 512 threads), 1 at N2 = 9 (G = 9 keeps three groups per XCD)
constexpr int ms_rows(int N2) { return N2 == 9 ? 1 : 2; }

template <int N2>
hipError_t launch_ms_n(int CHI, const SweepParams& p, const MsplitParams& q, double2* X, unsigned* cnt,
                       unsigned* err, hipStream_t s) {
    if constexpr (N2 == 4) {  // chi = 256 only
        return CHI == 256 ? launch_ms_t<4, 256, 1>(p, q, X, cnt, err, s) : hipErrorInvalidValue;
    } else {
    switch (CHI) {
        case 32: return launch_ms_t<N2, 32, ms_rows(N2)>(p, q, X, cnt, err, s);
        case 64:
            if constexpr (N2 != 25) return launch_ms_t<N2, 64, ms_rows(N2)>(p, q, X, cnt, err, s);
            return hipErrorInvalidValue;
        case 128:
            if constexpr (N2 <= 16) return launch_ms_t<N2, 128, 1>(p, q, X, cnt, err, s);
            return hipErrorInvalidValue;
        case 256:
            if constexpr (N2 <= 16) return launch_ms_t<N2, 256, 1>(p, q, X, cnt, err, s);
            return hipErrorInvalidValue;
        default: return hipErrorInvalidValue;
    }
    }
}

template <int N2>
int ms_occ_n(int CHI) {
    if constexpr (N2 == 4) {
        return CHI == 256 ? ms_occ_t<4, 256, 1>() : 0;
    } else {
    switch (CHI) {
        case 32: return ms_occ_t<N2, 32, ms_rows(N2)>();
        case 64:
            if constexpr (N2 != 25) return ms_occ_t<N2, 64, ms_rows(N2)>();
            return 0;
        case 128:
            if constexpr (N2 <= 16) return ms_occ_t<N2, 128, 1>();
            return 0;
        case 256:
            if constexpr (N2 <= 16) return ms_occ_t<N2, 256, 1>();
            return 0;
        default: return 0;
    }
    }
}

}  // namespace

int msplit_rows(int N2, int CHI) { return CHI > 64 ? 1 : ms_rows(N2); }
// (N2 = 4 only at chi = 256: the two-level system's other bonds run on the quad and batched kernels)
int msplit_tbmax(int N2, int CHI) { return CHI > 64 ? 8 : (ms_rows(N2) == 1 ? 32 : 16); }
int msplit_cev_max() { return MS_CEV_MAX; }
int msplit_group_size(int N2, int CHI) { return (N2 + msplit_rows(N2, CHI) - 1) / msplit_rows(N2, CHI); }

bool msplit_supported(int N2, int CHI, int n_out) {
    // N2 = 25 at chi = 64 spills (7 gathered rows per thread for two PT rows): the single split or batched kernels
    // chi = 128 (the bond cap of generated N <= 4 PTs, which the single-trajectory split kernel does not take): one PT
    // row per workgroup of 512 threads, the 256 KiB slice row in their registers
    // chi = 256 (a bond past the batched kernel's LDS: generated PTs whose threshold asks for more than 128, VERDICT r5
    // item 2b): one PT row per workgroup of 1,024 threads, the slice row streamed from L2 each step
    if (CHI == 256) return (N2 == 4 || N2 == 9 || N2 == 16) && n_out >= 1 && n_out <= 8;
    return (N2 == 9 || N2 == 16 || N2 == 25 || N2 == 36) &&
           (CHI == 32 || (CHI == 64 && N2 != 25) || (CHI == 128 && N2 <= 16)) && n_out >= 1 && n_out <= 8;
}

int msplit_blocks_per_cu(int N2, int CHI) {
    switch (N2) {
        case 4: return ms_occ_n<4>(CHI);
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
        case 4: hipLaunchKernelGGL((evcomp_kernel<4>), grid, dim3(256), 0, s, p, q, n_cev, n_steps); break;
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
    switch (N2) {
        case 4: return launch_ms_n<4>(CHI, p, q, X, cnt, err, s);
        case 9: return launch_ms_n<9>(CHI, p, q, X, cnt, err, s);
        case 16: return launch_ms_n<16>(CHI, p, q, X, cnt, err, s);
        case 25: return launch_ms_n<25>(CHI, p, q, X, cnt, err, s);
        case 36: return launch_ms_n<36>(CHI, p, q, X, cnt, err, s);
        default: return hipErrorInvalidValue;
    }
}

// diagnostics: the stamps of the last PQD_ABLATE=64 multi-trajectory split launch (2 workgroups x 16 steps x 32 slots)
extern "C" int pqd_debug_msplit_stamps(unsigned long long* out) {
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_ms_stamps), sizeof(unsigned long long) * 1024) == hipSuccess ? 0 : 4;
}
