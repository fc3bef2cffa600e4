// pt_split.hip — latency path for small batches: ONE trajectory spread over a group of G = N2 (+ 1) workgroups.
//
// The batched sweep (pt_sweep.hip) gives a trajectory one wave of one workgroup, so a single run
// (SURVEY §8d C3 "biexciton, chi 64, 1 MI355X": one trajectory) streams the whole PT slice set
// (N2 chi^2 c128 = 1 MiB per step at N = 4, chi = 64) through ONE CU: ≈13 µs per step.
// Here workgroup g of a trajectory's group owns PT row alpha = g: it contracts that row with its
// slice (64 KiB per step at chi = 64, prefetched into registers while the group exchanges). The
// column phases (M_b(n-1), MTOs, outputs, M_a(n), or the fused F(n) = M_a(n) M_b(n-1)) mix rows, so
// every workgroup gathers the whole state (N2 x chi, 16 KiB at C3) once per step and runs them
// redundantly — ONE exchange per step instead of a row/column transpose pair.
// Hand-off (default): arrival words. Payload stores are 8-B sc1 atomics, the storing wave drains with
// s_waitcnt vmcnt(0), a workgroup barrier, then ONE lane stores the workgroup's arrival word (steps published; groups
// of more than 32 workgroups add to one shared counter instead); wave 0 polls every word of the group with one relaxed
// sc1 load per poll, the other waves wait at a barrier, and every payload load is an sc1 load — so no fences
// (MI355X_MICROARCH.md § visibility "Valid forms" table row 1). With the XCD-grouped grid the counter form beat the
// granule form below (C3 5.02 vs 5.33 us per step, profiles/r04/split/xcd/).
// Output workgroup (default in the counter form, PQD_SPLIT_OW=0 off): the group gets one more workgroup, g = N2, that
// owns no PT row. It gathers the state like its peers, writes the outputs and trunk checkpoints, and arrives at the
// top of each step (it has read the previous slot); without it workgroup 0 ran the output pass between its publish
// and its poll and every peer waited for it (C3 single run 34.7 -> 31.8 ms, profiles/r05/ow/).
// Alternative (PQD_SPLIT_GRAN=1): data-tagged granules (cdna_hip_programming.md §6 Guideline 16 R2: "the data IS
// the flag"). Every 32-bit word of the row a workgroup publishes travels as one naturally aligned 8-B
// {tag = step + 1, word} granule written by ONE relaxed agent-scope atomic store (global_store_dwordx2 sc1); the
// consumers sweep the whole state's granules with sc1 loads and re-read the ones whose tag is not yet the step's,
// until every tag matches: no drain, no counter, no barrier between publishing and reading.
// Either exchange buffer is double-buffered by step parity (a workgroup cannot publish step n+2 before every
// peer has gathered step n: its step n+1 row depends on that gather; the output workgroup's arrival at step n+1
// says it has gathered step n). One workgroup per CU (the LDS request
// forces it) and at most n_cu workgroups (host check), so every workgroup is resident; every spin is bounded
// and a timeout ends the kernel with an error word the host turns into PQD_ERR_HIP (then the batched kernel).
// Semantics are the sweep's: step n applies M_b(n-1), applyBefore MTOs at n,
// output(n), applyAfter MTOs at n, M_a(n), PT(n); steps without MTOs use F(n) and read the outputs
// through W(n) = ovec M_b(n-1), as the batched kernel does.
#include "pqd_common.h"
#include <cstdlib>

namespace {

typedef unsigned long long __attribute__((address_space(1))) gu64;
typedef unsigned int __attribute__((address_space(1))) gu32;

constexpr int SP_NT = 256;
constexpr int SP_LDS_FORCE = 96 * 1024;  // dynamic LDS request: one workgroup per CU

__device__ __forceinline__ void st_sc1(double2* p, double2 v) {
    __hip_atomic_store((gu64*)&p->x, (unsigned long long)__double_as_longlong(v.x), __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store((gu64*)&p->y, (unsigned long long)__double_as_longlong(v.y), __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_AGENT);
}

// plain global load (a generic pointer would become flat_load, which also counts in lgkmcnt: every LDS wait
// would then wait for the register prefetches too)
__device__ __forceinline__ double2 gld(const double2* p) {
    const __attribute__((address_space(1))) double* q = (const __attribute__((address_space(1))) double*)p;
    return make_double2(q[0], q[1]);
}

typedef unsigned int v4u32 __attribute__((ext_vector_type(4)));

// one granule: {tag, word} in ONE aligned 8-B sc1 store
__device__ __forceinline__ void st_granule(unsigned long long* g, unsigned tag, unsigned word) {
    __hip_atomic_store((gu64*)g, ((unsigned long long)tag << 32) | word, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

template <int N2, int CHI>
struct SplitLayout {
    static constexpr int KG = SP_NT / CHI;            // k groups of the row contraction
    static constexpr int KPER = CHI / KG;             // slice rows per thread
    static constexpr int RPT = (N2 + KG - 1) / KG;    // state rows per thread in the column phase
    static constexpr int OPER = (N2 * N2 + SP_NT - 1) / SP_NT;  // operator elements per thread (staging)
    static constexpr int WST = 4 * SP_NT;                     // output-row elements staged in LDS (n_out N2 <= WST)
    static constexpr int LDS_STATE = 2 * N2 * CHI + N2 * N2 + N2 + 2 * SP_NT + CHI + WST;  // complex elements
    static constexpr int LDS = (LDS_STATE * 16 > SP_LDS_FORCE) ? LDS_STATE * 16 : SP_LDS_FORCE;
};

// diagnostics (PQD_ABLATE bit 32, scripts/split_stamps.py): s_memtime at the phase boundaries of steps 1000..1015 in
// workgroups 0 and G-1 of trajectory 0 (thread 0): [wg 0 / 1][step][phase 0..7]
__device__ unsigned long long g_split_stamps[2 * 16 * 8];

template <int N2, int CHI, bool GRAN, bool OWG, bool STAMP = false>
__global__ __launch_bounds__(SP_NT) void pt_split_kernel(SweepParams p, double2* __restrict__ X,
                                                         unsigned* __restrict__ cnt, unsigned* __restrict__ err) {
    using L = SplitLayout<N2, CHI>;
    constexpr int KG = L::KG, KPER = L::KPER, RPT = L::RPT, OPER = L::OPER;
    static_assert(!(OWG && GRAN), "the output workgroup takes part in the counter form only");
    // OWG: one more workgroup per group, g = N2, owns no PT row: it writes the outputs (and trunk checkpoints) from the
    // gathered state while the N2 row workgroups contract and publish the next step, so the output pass leaves the
    // group's critical path (without it workgroup 0 ran it between its publish and its poll, and every peer waited)
    constexpr int G = N2 + (OWG ? 1 : 0), E = N2 * CHI;
    constexpr int OG = OWG ? N2 : 0;  // the workgroup that writes outputs and checkpoints
    extern __shared__ __attribute__((aligned(16))) double2 smem[];
    // smem: full state ping-pong [0, E) and [E, 2E), staged column operator, closure contractions r[beta]
    // (output phase), PT partial sums, the step's closure vector and output rows (workgroup 0) — all indexed off
    // smem so every access stays ds_*
    constexpr int OPO = 2 * E, RRO = OPO + N2 * N2, REDO = RRO + N2, CVO = REDO + SP_NT, WRO = CVO + CHI;
    constexpr int PRT = WRO + L::WST;  // counter form: KG partial sums of the next PT row (see the gather)
    constexpr int WST = L::WST, WPT = WST / SP_NT;
    // chi = 64 fused gather: wave w writes PRT[16 w + lane] and only its own PT k-range (kq KPER ..) reads them, with no
    // barrier between — that holds only while a wave's k-range is exactly those 16 columns
    static_assert(CHI != 64 || (KG == 4 && KPER == 16 && SP_NT == 256), "PRT layout assumes one wave per k-group");
    __shared__ int s_abort;
    if (threadIdx.x == 0) s_abort = 0;

    const int tid = threadIdx.x;
    int tl = blockIdx.x / G, g = blockIdx.x - tl * G;
    if (p.split_xcd > 0) {
        // XCD-grouped grid (launch_split_tg): block b sits in XCD slot b % 8 under the observed round-robin dealing;
        // group tl = slot + 8 (b / 8 / G) keeps all G workgroups of a group in one slot, so the group's hand-offs
        // stay in one L2 when the dealing holds. Placement is speed only: the exchange is the same at any placement.
        const int xs = blockIdx.x & 7, loc = blockIdx.x >> 3;
        tl = xs + 8 * (loc / G);
        g = loc - (loc / G) * G;
        if (tl >= p.split_xcd) return;  // an unused block (before any shared state is touched)
    }
    const bool ow = OWG && g == N2;
    // counter form: the row workgroups get their next PT row from the gather (rowg); workgroup 0 without the output
    // workgroup writes the outputs, so it gathers the whole state and forms its row in the column phase, as the
    // granule form does
    const bool rowg = !GRAN && (OWG || g != 0);
    const int t = p.traj_base + tl;
    const int wb = p.wbeg[t], we = p.wend[t];
    const long long wo = p.woff[t];
    const int sy = p.traj_sys[t];
    const int2 wn = fw_win(p, sy);  // pulse window: M, F, W outside it are the system's idle operators
    // exchange region of this trajectory: 2 slots x E elements x 4 granules x 8 B (GRAN) = 4 E double2; the
    // counter form uses the first 2 E double2 of it
    double2* __restrict__ Xt = X + (size_t)t * 4 * E;
    unsigned long long* __restrict__ Gt = reinterpret_cast<unsigned long long*>(Xt);
    // descriptor over this trajectory's granules, from workgroup-uniform values only (16-B sc1 loads of 2 granules)
    const __amdgpu_buffer_rsrc_t rG = __builtin_amdgcn_make_buffer_rsrc(Xt, 0, 4 * E * 16, 0x00020000);
    // counter form: the group's arrival flags, one word per workgroup (flag g = steps workgroup g has published; the
    // output workgroup's = steps it has gathered + 1), two 128-B lines per group. One word per producer instead of one
    // shared counter: no serialised atomics at the L2, and wave 0 reads every flag with ONE load per poll. A group of
    // more than 32 workgroups (N2 = 36: 37) spans two XCDs and two lines of flags; there one monotonic counter (one
    // add per arrival, G per step) measured faster (C5 single run 43.1 -> 38.6-40.5 ms, profiles/r05/hyb/)
    constexpr bool FLAGS = G <= 32;
    unsigned* ct = cnt + (size_t)t * 64;
    // l2k (counter form with flags, XCD-grouped grid): the payload and, from the second step on, the arrival words are
    // plain stores that keep their lines in the group's L2, where the peers' sc1 loads find them. That is coherent only
    // if the whole group runs on one XCD: every flag carries its writer's XCD id (bits 28..30, HW_REG_XCC_ID) and the
    // first poll checks them; a group spread over XCDs ends the launch before its first gather (error word), and the
    // host re-runs it on the batched kernel. PQD_ABLATE bit 512 fakes a spread group (workgroup 0 reports the next XCD)
    const bool l2k = FLAGS && !GRAN && p.split_xcd > 0 && p.split_l2 != 0;
    unsigned xtag = 0;
    if (l2k) {
        unsigned xid = (unsigned)__builtin_amdgcn_s_getreg((3 << 11) | (0 << 6) | 20) & 7u;  // hwreg(HW_REG_XCC_ID, 0, 4)
        if ((p.ablate & 512) && g == 0) xid = (xid + 1u) & 7u;
        xtag = xid << 28;
    }
    auto arrive = [&](int n) {
        if constexpr (FLAGS) {
            const unsigned av = ((unsigned)n + 1u) | xtag;
            if (l2k && n >= 1) *(__attribute__((address_space(1))) unsigned*)(ct + g) = av;
            else __hip_atomic_store((gu32*)(ct + g), av, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        } else {
            __hip_atomic_fetch_add((gu32*)ct, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
    };
    bool placed_checked = false;
    const int n_end = we;
    constexpr int m2 = N2 * N2;
    const int ev_lim = p.ev_start[t + 1];
    int ev_cur = p.ev_start[t];
    const int dcol = tid % CHI, kq = tid / CHI;

    int qo = 0, to = E;  // current state / scratch offsets
    for (int e = tid; e < E; e += SP_NT) {
        const int a = e / CHI, d = e - (e / CHI) * CHI;
        smem[qo + e] = c_mul(gld(p.rho0 + a), gld(p.bond0 + d));
    }
    // y[a][d] = sum_b Op[a][b] Q[b][d]: thread owns column d and rows kq + KG i
    auto apply_lds = [&]() {
        __syncthreads();  // Op staged, Q complete
        double2 x[N2];
#pragma unroll
        for (int b = 0; b < N2; ++b) x[b] = smem[qo + b * CHI + dcol];
#pragma unroll
        for (int i = 0; i < RPT; ++i) {
            const int a = kq + KG * i;
            if (a < N2) {
                double2 acc = c_zero();
#pragma unroll
                for (int b = 0; b < N2; ++b) c_fma(acc, smem[OPO + a * N2 + b], x[b]);
                smem[to + a * CHI + dcol] = acc;
            }
        }
        __syncthreads();
        const int sw = qo; qo = to; to = sw;
    };
    auto apply_global = [&](const double2* __restrict__ M) {
        __syncthreads();  // previous readers of Op done
#pragma unroll
        for (int i = 0; i < OPER; ++i) {
            const int e = tid + SP_NT * i;
            if (e < m2) smem[OPO + e] = gld(M + e);
        }
        apply_lds();
    };
    // phase stamps: 0 top, 1 column phase done, 2 PT partials in LDS, 3 row published + arrived, 4 output/prefetch
    // done, 5 peers arrived (poll + barrier), 6 state gathered (end of step); 7 output operands staged (workgroup 0)
    auto stamp = [&](int n, int k) {
        if constexpr (STAMP) {
            const int wsel = g == 0 ? 0 : (g == G - 1 ? 1 : -1);
            if (t == 0 && wsel >= 0 && threadIdx.x == 0 && n >= 1000 && n < 1016)
                g_split_stamps[(wsel * 16 + (n - 1000)) * 8 + k] = __builtin_amdgcn_s_memtime();
        }
    };
    // output(n) through rows w[k][.] (ovec, or W(n) on the state before M_b(n-1)): workgroup 0 writes it. The closure
    // vector and the rows are fetched into registers a step ahead (ofetch) and staged in LDS here, so the
    // pass is LDS-only: it sits on the group's critical path every step (workgroup 0 publishes step n + 1 only after
    // it), and with the loads inside it took ~6,500 of a ~12,800-cycle C3 step (profiles/r05/split/stamps_before.log)
    double2 cvr = c_zero(), wrr[WPT];
    bool wdirect = false;  // more output-row elements than the staging area: read them from memory in the pass
    auto ofetch = [&](int n, const double2* __restrict__ w, int sp) {  // sp = sched[n - 1] (n >= 1)
        if (g != OG || n < wb || n > we) return;
        const double2* cv = (n == 0) ? p.closure0 : p.closure + (size_t)sp * CHI;
        if (tid < CHI) cvr = gld(cv + tid);
        wdirect = p.n_out * N2 > WST;
        if (!wdirect) {
#pragma unroll
            for (int i = 0; i < WPT; ++i) {
                const int e = tid + SP_NT * i;
                wrr[i] = e < p.n_out * N2 ? gld(w + e) : c_zero();
            }
        }
    };
    // the fetched operands into LDS: after the poll of the step before (the loads have landed; a barrier before
    // output() makes them visible), so the pass itself has no staging wait or barrier
    auto ostage = [&]() {
        if (g != OG) return;
        if (tid < CHI) smem[CVO + tid] = cvr;
        if (!wdirect) {
#pragma unroll
            for (int i = 0; i < WPT; ++i)
                if (tid + SP_NT * i < p.n_out * N2) smem[WRO + tid + SP_NT * i] = wrr[i];
        }
    };
    auto output = [&](int n, const double2* __restrict__ w) {
        if (g != OG || n < wb || n > we) return;
        stamp(n, 7);
        // closure r[b] = sum_d Q[b][d] c[d], then out[k] = sum_b W[k][b] r[b]: QW consecutive lanes per row or
        // output, summed by DPP moves inside the lane group (c_group_sum), every thread busy
        constexpr int QW = N2 <= 16 ? 16 : 4;
        constexpr int RPP = SP_NT / QW;  // rows (outputs) per pass
        const int q = tid % QW;
        for (int b0 = 0; b0 < N2; b0 += RPP) {
            const int b = b0 + tid / QW;
            double2 sacc = c_zero();
            if (b < N2)
#pragma unroll
                for (int d = q; d < CHI; d += QW) c_fma(sacc, smem[qo + b * CHI + d], smem[CVO + d]);
            sacc = c_group_sum<QW>(sacc);
            if (b < N2 && q == 0) smem[RRO + b] = sacc;
        }
        __syncthreads();
        for (int k0 = 0; k0 < p.n_out; k0 += RPP) {
            const int k = k0 + tid / QW;
            double2 sacc = c_zero();
            // two loops, not one with a select: a global load in the merged loop put an s_waitcnt vmcnt(0) (every
            // outstanding store and prefetch) in front of the staged path's FMAs too
            if (k < p.n_out) {
                if (wdirect) {
                    for (int b = q; b < N2; b += QW) c_fma(sacc, gld(w + (size_t)k * N2 + b), smem[RRO + b]);
                } else {
#pragma unroll
                    for (int b = q; b < N2; b += QW) c_fma(sacc, smem[WRO + k * N2 + b], smem[RRO + b]);
                }
            }
            sacc = c_group_sum<QW>(sacc);
            if (k < p.n_out && q == 0) p.out[wo + (long long)(n - wb) * p.n_out + k] = sacc;
        }
    };
    // the step of the next unconsumed event, kept in a register: the fast path asks it every step and a p.ev load there
    // was a dependent memory round trip on the group's critical path (re-read only when an event is consumed)
    int ev_next = ev_cur < ev_lim ? p.ev[ev_cur].x : INT_MAX;
    auto has_event = [&](int n) { return ev_next == n; };
    auto ev_advance = [&]() { ++ev_cur; ev_next = ev_cur < ev_lim ? p.ev[ev_cur].x : INT_MAX; };

    // slice row of PT(0) and row g of the fused operator of step 1
    double2 sreg[KPER], frow = c_zero();
    // gather layout (counter form): slot i of thread tid holds state element ge(i), -1 past the state. chi = 64: wave w
    // takes the columns 16 w .. 16 w + 15 of every row (its own PT k-range), lane group lane >> 4 the rows
    // lane >> 4 + 4 i; otherwise element tid + SP_NT i
    constexpr int EPT_G = (E + SP_NT - 1) / SP_NT;
    const int lane = tid & 63;
    auto ge = [&](int i) -> int {
        if constexpr (CHI == 64) {
            const int b = (lane >> 4) + 4 * i;
            return b < N2 ? b * CHI + 16 * (tid >> 6) + (lane & 15) : -1;
        } else {
            const int e = tid + SP_NT * i;
            return e < E ? e : -1;
        }
    };
    // counter form, row workgroups: F(n + 1)[g][b] of the thread's gather elements (b = ge(i) / CHI): the gather of
    // step n contracts them with the state as it arrives, so a fused step has no column phase
    double2 fr[EPT_G];
#pragma unroll
    for (int i = 0; i < EPT_G; ++i) fr[i] = c_zero();
    const int grow = ow ? 0 : p.gmap[g];
    auto fetch_slice = [&](int si) {  // si = sched[n], from a register (a p.sched load here was a dependent round trip)
        const double2* __restrict__ S = p.Q + ((size_t)si * p.D + grow) * CHI * CHI;
#pragma unroll
        for (int j = 0; j < KPER; ++j) sreg[j] = gld(S + (size_t)(kq * KPER + j) * CHI + dcol);
    };
    // the schedule, 64 entries at a time in a VGPR (lane i holds sched[64 c + i]) one chunk ahead, picked with
    // v_readlane: a uniform p.sched[n] load in the loop compiles to a vector load + readfirstlane that waits
    // (s_waitcnt vmcnt(0)) for every outstanding vector memory op where it is issued — on every workgroup's critical
    // path each step
    auto sched_chunk = [&](int c) {
        const int i = 64 * c + lane;
        return i < n_end ? *(const __attribute__((address_space(1))) int*)(p.sched + i) : -1;
    };
    int sch_cur = sched_chunk(0), sch_nxt = sched_chunk(1);
    int cur_slice = n_end > 0 ? __builtin_amdgcn_readlane(sch_cur, 0) : -1;  // the slice index sreg holds (sched[n])
    if (n_end > 0 && !ow) fetch_slice(cur_slice);
    ofetch(0, p.ovec, 0);  // step 0 is never fused
    ostage();
    __syncthreads();
    bool pre = false;  // the coming step is fused: frow (granule form) / fr (counter form) hold its F row
    for (int n = 0;; ++n) {
        stamp(n, 0);
        // ---- trunk pre-pass: checkpoint of the state at the top of step n (M_b(n-1) still deferred), workgroup 0
        if (p.ck_map && g == OG && n >= 1) {
            const int c = p.ck_map[(size_t)t * p.ck_stride + n];
            if (c >= 0)
                for (int e = tid; e < E; e += SP_NT) p.ck[(size_t)c * E + e] = smem[qo + e];
        }
        // the output workgroup arrives at the top of the step: it has gathered step n - 1, so the row workgroups may
        // reuse that slot for step n + 1 once their poll of step n has seen this (its word, or its add to the counter)
        if (ow && n < n_end && tid == 0) arrive(n);
        // ---- column phase
        const bool fz = p.fuse && n >= 1 && !has_event(n);
        int rb;  // row g of the state the PT contracts
        if (fz) {
            // only row g of F(n) Q is needed here; Q itself stays for the deferred output(n) through W(n)
            if (n >= n_end) { output(n, fw_W(p, sy, wn, n, N2)); break; }
            rb = to;
            // counter form: the gather of step n - 1 left row g of F(n) Q in PRT (pre was set): chi = 64 as the row
            // itself (each wave wrote its own k-range), else as KG partial sums
            if (!ow && !rowg) {
                if (tid < N2) smem[OPO + tid] = pre ? frow : gld(fw_F(p, sy, wn, n, m2) + (size_t)g * N2 + tid);
                __syncthreads();
                if (tid < CHI) {
                    double2 acc = c_zero();
#pragma unroll
                    for (int b = 0; b < N2; ++b) c_fma(acc, smem[OPO + b], smem[qo + b * CHI + tid]);
                    smem[to + g * CHI + tid] = acc;
                }
                __syncthreads();
                rb = to + g * CHI;
            }
        } else {
            if (n > 0) apply_global(fw_M(p, sy, wn, 2 * (n - 1) + 1, m2));
            while (ev_cur < ev_lim) {  // applyBefore MTOs at n
                const int4 ev = p.ev[ev_cur];
                if (ev.x != n || ev.y != 0) break;
                apply_global(p.sop + (size_t)ev.z * m2);
                ev_advance();
            }
            output(n, p.ovec);
            if (n >= n_end) break;
            while (ev_cur < ev_lim) {  // applyAfter MTOs at n
                const int4 ev = p.ev[ev_cur];
                if (ev.x != n || ev.y != 1) break;
                apply_global(p.sop + (size_t)ev.z * m2);
                ev_advance();
            }
            apply_global(fw_M(p, sy, wn, 2 * n, m2));
            rb = qo + g * CHI;
        }
        stamp(n, 1);
        // ---- PT row g: y = row . S(n) -> exchange buffer (parity n & 1)
        if (!ow) {
            double2 acc = c_zero();
            if (rowg && fz && CHI == 64) {
                // the wave's 16 row values in lanes 0..15 of every 16-lane row, one ds_read_b128, taken by the products
                // through DPP row_newbcast (16 broadcast reads before: one 4-cycle LDS instruction per complex MAC)
                const double2 pv[1] = {smem[PRT + kq * KPER + (lane & 15)]};
                pq_dpp_src_ready(pv);
                pq_row_bcast_mac<0, KPER>(acc, pv, sreg);
            } else if (rowg && fz) {
#pragma unroll
                for (int j = 0; j < KPER; ++j) {
                    const int k = kq * KPER + j;
                    double2 r = smem[PRT + k];
#pragma unroll
                    for (int kg = 1; kg < KG; ++kg) r = c_add(r, smem[PRT + kg * CHI + k]);
                    c_fma(acc, r, sreg[j]);
                }
            } else {
#pragma unroll
                for (int j = 0; j < KPER; ++j) c_fma(acc, smem[rb + kq * KPER + j], sreg[j]);
            }
            smem[REDO + tid] = acc;
            __syncthreads();
            stamp(n, 2);
            if (GRAN) {
                // thread q publishes word (q & 3) of element q >> 2 (every thread one granule when CHI = 64)
                const unsigned ep = (unsigned)n + 1u;
                for (int q = tid; q < 4 * CHI; q += SP_NT) {
                    const int el = q >> 2, wd = q & 3;
                    double2 y = smem[REDO + el];
#pragma unroll
                    for (int kg = 1; kg < KG; ++kg) y = c_add(y, smem[REDO + kg * CHI + el]);
                    const double v = (wd < 2) ? y.x : y.y;
                    const unsigned word = (wd & 1) ? (unsigned)__double2hiint(v) : (unsigned)__double2loint(v);
                    st_granule(Gt + ((size_t)(n & 1) * E + (size_t)g * CHI + el) * 4 + wd, ep, word);
                }
            } else {
                double2* Xn = Xt + (size_t)(n & 1) * E;
                if (tid < CHI) {
                    double2 y = smem[REDO + tid];
#pragma unroll
                    for (int q = 1; q < KG; ++q) y = c_add(y, smem[REDO + q * CHI + tid]);
                    if (l2k) {
                        typedef double v2f64 __attribute__((ext_vector_type(2)));
                        *(__attribute__((address_space(1))) v2f64*)(Xn + (size_t)g * CHI + tid) = v2f64{y.x, y.y};
                    } else {
                        st_sc1(Xn + (size_t)g * CHI + tid, y);
                    }
                }
                // ---- arrive (every storing wave drained, then one lane); the wait for the group is below
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                __syncthreads();
                if (tid == 0) arrive(n);
            }
        }
        stamp(n, 3);
        // ---- prefetch the next step's slice row (only when the schedule changes the slice: the repeated slice of
        // ACE's _repeated / infinite PTs stays in registers), issued right after the arrive so its 64 KiB are in flight
        // during workgroup 0's output pass rather than in front of the poll; then the fused operator row
        const int sn = cur_slice;  // sched[n]
        if (n + 1 < n_end) {
            const int m = n + 1;
            if ((m & 63) == 0) { sch_cur = sch_nxt; sch_nxt = sched_chunk((m >> 6) + 1); }
            const int ns = __builtin_amdgcn_readlane(sch_cur, m & 63);
            if (ns != cur_slice) {
                if (!ow) fetch_slice(ns);
                cur_slice = ns;
            }
        }
        if (fz) output(n, fw_W(p, sy, wn, n, N2));  // workgroup OG only (without OWG it publishes step n + 1 after this)
        pre = p.fuse && n + 1 < n_end && !has_event(n + 1);
        if (!rowg) {
            if (pre && tid < N2 && !ow) frow = gld(fw_F(p, sy, wn, n + 1, m2) + (size_t)g * N2 + tid);
        } else if (pre && !ow) {
            const double2* __restrict__ Fr = fw_F(p, sy, wn, n + 1, m2) + (size_t)g * N2;
#pragma unroll
            for (int i = 0; i < EPT_G; ++i) {
                const int e = ge(i);
                fr[i] = e >= 0 ? gld(Fr + e / CHI) : c_zero();
            }
        }
        // the next step's output operands, a whole step ahead (W(n + 1) is a fresh row from memory every step)
        if (n + 1 <= n_end) {
            const bool fz1 = p.fuse && !has_event(n + 1);
            ofetch(n + 1, fz1 ? fw_W(p, sy, wn, n + 1, N2) : p.ovec, sn);
        }
        stamp(n, 4);
        if (GRAN) {
            // ---- sweep: every element of the state, 2 x 16-B sc1 loads (2 granules each), re-read until its four
            // tags are n + 1; each wave leaves when all its elements have arrived
            constexpr int EPT = (E + SP_NT - 1) / SP_NT;
            const unsigned ep = (unsigned)n + 1u;
            unsigned pend = 0;
#pragma unroll
            for (int i = 0; i < EPT; ++i)
                if (tid + SP_NT * i < E) pend |= 1u << i;
            unsigned spins = 0;
            bool ok = true;
            for (;;) {
                // all of this pass's loads in flight before the first tag check
                v4u32 ga[EPT], gb[EPT];
#pragma unroll
                for (int i = 0; i < EPT; ++i) {
                    const int e = tid + SP_NT * i;
                    const int off = (int)(((size_t)(n & 1) * E + (e < E ? e : 0)) * 32);
                    if (pend & (1u << i)) {
                        ga[i] = __builtin_amdgcn_raw_buffer_load_b128(rG, off, 0, 16);
                        gb[i] = __builtin_amdgcn_raw_buffer_load_b128(rG, off + 16, 0, 16);
                    }
                }
#pragma unroll
                for (int i = 0; i < EPT; ++i) {
                    if (!(pend & (1u << i))) continue;
                    const v4u32 a = ga[i], b = gb[i];
                    if (a.y == ep && a.w == ep && b.y == ep && b.w == ep) {
                        smem[qo + tid + SP_NT * i] = make_double2(__hiloint2double((int)a.z, (int)a.x),
                                                                  __hiloint2double((int)b.z, (int)b.x));
                        pend &= ~(1u << i);
                    }
                }
                if (__all(pend == 0)) break;
                __builtin_amdgcn_s_sleep(1);
                if (++spins > p.spin_limit) { ok = false; break; }
            }
            if (!ok) {
                s_abort = 1;
                __hip_atomic_store((gu32*)err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
            __syncthreads();
            if (s_abort) return;
            ostage();  // visible to output(n + 1) after the column phase's barriers
        } else {
            if (tid < 64) {
                const unsigned want = (unsigned)n + 1u;
                unsigned spins = 0;
                bool ok = true;
                for (;;) {
                    if constexpr (FLAGS) {
                        const unsigned v =
                            lane < G ? __hip_atomic_load((gu32*)(ct + lane), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                                     : want;
                        if (__all((v & 0x0FFFFFFFu) >= want)) {
                            if (l2k && !placed_checked) {  // the same words reach every workgroup: one decision
                                const unsigned x0 = __builtin_amdgcn_readfirstlane(v) >> 28;
                                if (!__all(lane >= G || (v >> 28) == x0)) { ok = false; break; }
                            }
                            break;
                        }
                    } else {
                        if (__hip_atomic_load((gu32*)ct, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >= (unsigned)G * want)
                            break;
                    }
                    __builtin_amdgcn_s_sleep(1);
                    if (++spins > p.spin_limit) { ok = false; break; }
                }
                if (tid == 0) {
                    s_abort = ok ? 0 : 1;
                    if (!ok) __hip_atomic_store((gu32*)err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                }
            }
            placed_checked = true;
            __syncthreads();
            if (s_abort) return;
            stamp(n, 5);
            ostage();  // visible to output(n + 1) after the gather's barrier (or the PT's, chi = 64 fused rows)
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");  // compiler ordering only: payload loads are sc1
            // every element's 16-B sc1 load in flight before the first use (buffer loads, not atomic ones: the compiler
            // kept relaxed atomic loads in order and waited vmcnt(0) on each element, four L2 round trips in a row)
            v4u32 xr[EPT_G];
#pragma unroll
            for (int i = 0; i < EPT_G; ++i) {
                const int e = ge(i);
                xr[i] = __builtin_amdgcn_raw_buffer_load_b128(rG, (int)(((size_t)(n & 1) * E + (e >= 0 ? e : 0)) * 16),
                                                              0, 16);
            }
            auto xel = [&](int i) {
                return make_double2(__hiloint2double((int)xr[i].y, (int)xr[i].x),
                                    __hiloint2double((int)xr[i].w, (int)xr[i].z));
            };
            if (pre && !ow && rowg) {
                // a fused step next: only row g of F(n + 1) Q is needed, y[d] = sum_b F[g][b] Q[b][d]
                double2 part = c_zero();
#pragma unroll
                for (int i = 0; i < EPT_G; ++i)
                    if (ge(i) >= 0) c_fma(part, fr[i], xel(i));
                if constexpr (CHI == 64) {
                    // the four lane groups hold the same columns: add them (permlane swaps); lanes 0..15 keep
                    // y[16 w + lane], which only this wave's PT reads — no barrier
                    part = make_double2(xor_add<32>(part.x), xor_add<32>(part.y));
                    part = make_double2(xor_add<16>(part.x), xor_add<16>(part.y));
                    if (lane < 16) smem[PRT + 16 * (tid >> 6) + lane] = part;
                } else {
                    // the thread's elements share the column d = tid % CHI (SP_NT is a multiple of CHI) and sit in
                    // rows tid / CHI + KG i: PRT[tid] = partial (tid / CHI, d); the PT sums the KG partials
                    smem[PRT + tid] = part;
                    __syncthreads();
                }
            } else {
#pragma unroll
                for (int i = 0; i < EPT_G; ++i)
                    if (ge(i) >= 0) smem[qo + ge(i)] = xel(i);
                __syncthreads();
            }
            stamp(n, 6);
        }
    }
}

template <int N2, int CHI, bool GRAN, bool OWG, bool STAMP = false>
hipError_t launch_split_tg(int n_traj, const SweepParams& p, double2* X, unsigned* cnt, unsigned* err, hipStream_t s) {
    using L = SplitLayout<N2, CHI>;
    static_assert(L::LDS <= 160 * 1024, "LDS budget");
    if constexpr (!STAMP && !GRAN && N2 == 16 && CHI == 64) {
        if (p.ablate & 32) return launch_split_tg<N2, CHI, GRAN, OWG, true>(n_traj, p, X, cnt, err, s);
    }
    static unsigned attr = 0;  // per-device bitmask (a second device needs the attribute set too)
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) return hipErrorInvalidDevice;
    if (dev >= 32 || !(attr & (1u << dev))) {
        hipError_t e = hipFuncSetAttribute((const void*)pt_split_kernel<N2, CHI, GRAN, OWG, STAMP>,
                                           hipFuncAttributeMaxDynamicSharedMemorySize, (int)L::LDS);
        if (e != hipSuccess) return e;
        if (dev < 32) attr |= 1u << dev;
    }
    // XCD-grouped grid when every XCD slot can hold its groups at one workgroup per CU (32 CUs per XCD on MI355X):
    // 8 slots x ceil(n_traj / 8) groups x G blocks, the blocks of missing groups return at once
    const int per_slot = (n_traj + 7) / 8;
    SweepParams q = p;
    constexpr int G = N2 + (OWG ? 1 : 0);
    unsigned nb = (unsigned)(n_traj * G);
    q.split_xcd = 0;
    if (p.split_xcd && per_slot * G <= 32) {
        q.split_xcd = n_traj;
        nb = 8u * (unsigned)(per_slot * G);
    }
    hipLaunchKernelGGL((pt_split_kernel<N2, CHI, GRAN, OWG, STAMP>), dim3(nb), dim3(SP_NT), L::LDS, s, q, X, cnt, err);
    return hipGetLastError();
}

template <int N2, int CHI>
hipError_t launch_split_t(int n_traj, const SweepParams& p, double2* X, unsigned* cnt, unsigned* err, hipStream_t s) {
    // p.split_gran (PQD_SPLIT_GRAN=1): data-tagged granule exchange; default 0 = the counter form, with the output
    // workgroup unless PQD_SPLIT_OW=0 (p.split_ow)
    if (p.split_gran) return launch_split_tg<N2, CHI, true, false>(n_traj, p, X, cnt, err, s);
    return p.split_ow ? launch_split_tg<N2, CHI, false, true>(n_traj, p, X, cnt, err, s)
                      : launch_split_tg<N2, CHI, false, false>(n_traj, p, X, cnt, err, s);
}

template <int N2>
hipError_t launch_split_n(int CHI, int n_traj, const SweepParams& p, double2* X, unsigned* cnt, unsigned* err,
                          hipStream_t s) {
    switch (CHI) {
        case 16: return launch_split_t<N2, 16>(n_traj, p, X, cnt, err, s);
        case 32: return launch_split_t<N2, 32>(n_traj, p, X, cnt, err, s);
        case 64: return launch_split_t<N2, 64>(n_traj, p, X, cnt, err, s);
        default: return hipErrorInvalidValue;
    }
}

template <int N2, int CHI>
int split_occ_t() {
    using L = SplitLayout<N2, CHI>;
    if (hipFuncSetAttribute((const void*)pt_split_kernel<N2, CHI, false, true>, hipFuncAttributeMaxDynamicSharedMemorySize,
                            (int)L::LDS) != hipSuccess)
        return 0;
    int nb = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, pt_split_kernel<N2, CHI, false, true>, SP_NT, L::LDS) != hipSuccess)
        return 0;
    return nb;
}

template <int N2>
int split_occ_n(int CHI) {
    switch (CHI) {
        case 16: return split_occ_t<N2, 16>();
        case 32: return split_occ_t<N2, 32>();
        case 64: return split_occ_t<N2, 64>();
        default: return 0;
    }
}

}  // namespace

// workgroups per group: the N2 row workgroups, plus the output workgroup in the counter form unless PQD_SPLIT_OW=0
// (the same environment the plan's SweepParams.split_gran / split_ow are read from)
bool split_ow_env() {
    const char* g = getenv("PQD_SPLIT_GRAN");
    const char* o = getenv("PQD_SPLIT_OW");
    return !(g && atoi(g) == 1) && !(o && atoi(o) == 0);
}
int split_group_size(int N2) { return N2 + (split_ow_env() ? 1 : 0); }

// workgroups of the split kernel the runtime can keep resident per CU (0: the kernel cannot run)
int split_blocks_per_cu(int N2, int CHI) {
    switch (N2) {
        case 4: return split_occ_n<4>(CHI);
        case 9: return split_occ_n<9>(CHI);
        case 16: return split_occ_n<16>(CHI);
        case 25: return split_occ_n<25>(CHI);
        case 36: return split_occ_n<36>(CHI);
        default: return 0;
    }
}

bool split_supported(int N2, int CHI, int n_traj, int n_cu) {
    return (CHI == 16 || CHI == 32 || CHI == 64) &&
           (N2 == 4 || N2 == 9 || N2 == 16 || N2 == 25 || N2 == 36) && n_traj >= 1 &&
           (long long)n_traj * split_group_size(N2) <= n_cu;
}

// X: n_traj * 4 * N2 * CHI double2 exchange buffer (granules, tags zeroed here); cnt: n_traj * 64 arrival words and err,
// zeroed here before every launch.
// chunk > 0: at most `chunk` trajectories per launch (each launch's groups co-resident), launched one after the other
hipError_t launch_split(int N2, int CHI, int n_traj, const SweepParams& p, double2* X, unsigned* cnt,
                        unsigned* err, hipStream_t s, int chunk) {
    hipError_t e = hipMemsetAsync(cnt, 0, (size_t)n_traj * 64 * sizeof(unsigned), s);
    if (e != hipSuccess) return e;
    if (p.split_gran) {  // every granule tag 0: never a step's epoch (n + 1 >= 1)
        e = hipMemsetAsync(X, 0, (size_t)n_traj * 4 * N2 * CHI * sizeof(double2), s);
        if (e != hipSuccess) return e;
    }
    e = hipMemsetAsync(err, 0, 4 * sizeof(unsigned), s);
    if (e != hipSuccess) return e;
    if (chunk <= 0 || chunk > n_traj) chunk = n_traj;
    for (int base = 0; base < n_traj; base += chunk) {
        SweepParams q = p;
        q.traj_base = base;
        const int n = n_traj - base < chunk ? n_traj - base : chunk;
        switch (N2) {
            case 4: e = launch_split_n<4>(CHI, n, q, X, cnt, err, s); break;
            case 9: e = launch_split_n<9>(CHI, n, q, X, cnt, err, s); break;
            case 16: e = launch_split_n<16>(CHI, n, q, X, cnt, err, s); break;
            case 25: e = launch_split_n<25>(CHI, n, q, X, cnt, err, s); break;
            case 36: e = launch_split_n<36>(CHI, n, q, X, cnt, err, s); break;
            default: return hipErrorInvalidValue;
        }
        if (e != hipSuccess) return e;
    }
    return hipSuccess;
}

// diagnostics: the stamps of the last PQD_ABLATE=32 split launch (2 workgroups x 16 steps x 8 phase slots)
extern "C" int pqd_debug_split_stamps(unsigned long long* out) {
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_split_stamps), sizeof(unsigned long long) * 256) == hipSuccess ? 0 : 4;
}
