// pqd_host.cpp — C-ABI implementation of libpqd (include/pqd.h): validation, Liouvillian /
// superoperator construction, MTO scheduling, trajectory grouping, device buffers, launches.
// No arithmetic of the propagation itself happens on the host: the free propagators, the PT
// sweep, traces and the map-chain sweeps all run in the HIP kernels (free_prop.hip, pt_sweep.hip,
// mapchain.hip). Host code only assembles constant N^2 x N^2 generators from N x N operators.
#include "../../include/pqd.h"
#include "pqd_common.h"

#include <algorithm>
#include <chrono>
#include <climits>
#include <memory>
#include <cmath>
#include <complex>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>
#include <unordered_map>
#include <vector>

using cd = std::complex<double>;

namespace {

thread_local std::string g_err;

int fail(int code, const char* fmt, ...) {
    char buf[1024];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof buf, fmt, ap);
    va_end(ap);
    g_err = buf;
    return code;
}

#define HIPCHK(x)                                                                              \
    do {                                                                                       \
        hipError_t e_ = (x);                                                                   \
        if (e_ != hipSuccess) return fail(PQD_ERR_HIP, "%s: %s (%s:%d)", #x, hipGetErrorString(e_), \
                                          __FILE__, __LINE__);                                 \
    } while (0)

template <class T>
struct DevBuf {
    T* p = nullptr;
    size_t n = 0;
    DevBuf() = default;
    DevBuf(const DevBuf&) = delete;
    DevBuf& operator=(const DevBuf&) = delete;
    ~DevBuf() { release(); }
    void release() {
        if (p) (void)hipFree(p);
        p = nullptr;
        n = 0;
    }
    hipError_t alloc(size_t count) {
        release();
        n = count;
        if (count == 0) return hipSuccess;
        return hipMalloc((void**)&p, count * sizeof(T));
    }
    hipError_t upload(const T* src, size_t count, hipStream_t s) {
        hipError_t e = alloc(count);
        if (e != hipSuccess || count == 0) return e;
        return hipMemcpyAsync(p, src, count * sizeof(T), hipMemcpyHostToDevice, s);
    }
};

const cd* C(const pqd_c128* p) { return reinterpret_cast<const cd*>(p); }

int pad_chi(int chi) {
    if (chi <= 16) return 16;
    if (chi <= 32) return 32;
    if (chi <= 64) return 64;
    if (chi <= 128) return 128;
    if (chi <= 256) return 256;  // multi-trajectory split groups only (pt_msplit.hip, slice rows streamed)
    return -1;
}

// ---- superoperators in the row-major vec convention: vec(A rho B) = (A (x) B^T) vec(rho)
void kron_left(int N, const cd* A, cd* S, cd f) {  // S += f * (A (x) I)
    const int N2 = N * N;
    for (int i = 0; i < N; ++i)
        for (int j = 0; j < N; ++j)
            for (int k = 0; k < N; ++k) S[(size_t)(i * N + j) * N2 + (k * N + j)] += f * A[i * N + k];
}
void kron_right(int N, const cd* B, cd* S, cd f) {  // S += f * (I (x) B^T): rho -> rho B
    const int N2 = N * N;
    for (int i = 0; i < N; ++i)
        for (int j = 0; j < N; ++j)
            for (int l = 0; l < N; ++l) S[(size_t)(i * N + j) * N2 + (i * N + l)] += f * B[l * N + j];
}
void commutator(int N, const cd* H, double hbar, cd* S) {  // S += -i/hbar [H, .]
    const cd f(0.0, -1.0 / hbar);
    kron_left(N, H, S, f);
    kron_right(N, H, S, -f);
}
void dissipator(int N, const cd* Lk, double g, cd* S) {  // S += g (L . L^dag - 1/2 {L^dag L, .})
    const int N2 = N * N;
    std::vector<cd> LdL(N * N);
    for (int i = 0; i < N; ++i)
        for (int j = 0; j < N; ++j) {
            cd s = 0;
            for (int k = 0; k < N; ++k) s += std::conj(Lk[k * N + i]) * Lk[k * N + j];
            LdL[i * N + j] = s;
        }
    for (int i = 0; i < N; ++i)
        for (int j = 0; j < N; ++j)
            for (int k = 0; k < N; ++k)
                for (int l = 0; l < N; ++l)
                    S[(size_t)(i * N + j) * N2 + (k * N + l)] += g * Lk[i * N + k] * std::conj(Lk[j * N + l]);
    kron_left(N, LdL.data(), S, cd(-0.5 * g));
    kron_right(N, LdL.data(), S, cd(-0.5 * g));
}
void matmul_sq(int n, const cd* A, const cd* B, cd* Cm) {
    std::vector<cd> t((size_t)n * n, 0.0);
    for (int i = 0; i < n; ++i)
        for (int k = 0; k < n; ++k) {
            const cd a = A[(size_t)i * n + k];
            for (int j = 0; j < n; ++j) t[(size_t)i * n + j] += a * B[(size_t)k * n + j];
        }
    std::copy(t.begin(), t.end(), Cm);
}

int check_system(const pqd_system* sys) {
    if (!sys) return fail(PQD_ERR_ARG, "system is NULL");
    if (sys->dim < 2 || sys->dim > 6) return fail(PQD_ERR_UNSUPPORTED, "dim %d not in [2, 6]", sys->dim);
    if (!sys->H0) return fail(PQD_ERR_ARG, "H0 is NULL");
    if (!(sys->hbar > 0)) return fail(PQD_ERR_ARG, "hbar must be > 0");
    if (sys->n_lind < 0 || (sys->n_lind > 0 && (!sys->lind_ops || !sys->lind_rates)))
        return fail(PQD_ERR_ARG, "bad Lindblad arguments");
    if (sys->n_chan < 0 || sys->n_chan > 4) return fail(PQD_ERR_UNSUPPORTED, "n_chan %d not in [0, 4]", sys->n_chan);
    if (sys->n_chan > 0 && (!sys->chan_ops || !sys->chan_samples || sys->n_samples < 1 || !(sys->sample_dt > 0)))
        return fail(PQD_ERR_ARG, "bad pulse-channel arguments");
    return PQD_OK;
}

int check_grid(const pqd_grid* g) {
    if (!g) return fail(PQD_ERR_ARG, "grid is NULL");
    if (g->n_steps < 0) return fail(PQD_ERR_ARG, "n_steps < 0");
    if (!(g->dt > 0)) return fail(PQD_ERR_ARG, "dt must be > 0");
    if (g->n_sub < 1 || g->n_sub > 64) return fail(PQD_ERR_ARG, "n_sub %d not in [1, 64]", g->n_sub);
    return PQD_OK;
}

struct Generators {
    std::vector<cd> L0, S, T, samples;
};

void build_generators(const pqd_system* sys, Generators& G) {
    const int N = sys->dim, N2 = N * N;
    const size_t m2 = (size_t)N2 * N2;
    G.L0.assign(m2, 0.0);
    commutator(N, C(sys->H0), sys->hbar, G.L0.data());
    for (int q = 0; q < sys->n_lind; ++q)
        dissipator(N, C(sys->lind_ops) + (size_t)q * N * N, sys->lind_rates[q], G.L0.data());
    const int nc = sys->n_chan;
    G.S.assign(std::max<size_t>(1, nc * m2), 0.0);
    G.T.assign(std::max<size_t>(1, nc * m2), 0.0);
    for (int p = 0; p < nc; ++p) {
        const cd* X = C(sys->chan_ops) + (size_t)p * N * N;
        std::vector<cd> Xd(N * N);
        for (int i = 0; i < N; ++i)
            for (int j = 0; j < N; ++j) Xd[i * N + j] = std::conj(X[j * N + i]);
        commutator(N, X, sys->hbar, G.S.data() + p * m2);
        commutator(N, Xd.data(), sys->hbar, G.T.data() + p * m2);
    }
    if (nc > 0)
        G.samples.assign(C(sys->chan_samples), C(sys->chan_samples) + (size_t)nc * sys->n_samples);
    else
        G.samples.assign(1, 0.0);
}

}  // namespace

// =================================================================================================
struct pqd_ctx {
    int device = 0;
    hipStream_t stream = nullptr;
    // map-chain sweeps: one device arena reused across calls (grown on demand), so a call allocates nothing
    DevBuf<char> mc_arena;
};

namespace {
int Q_of(const std::vector<int>& pos, int n_tau) {
    int q = 0;
    for (int v : pos) q = std::max(q, v + n_tau);
    return q;
}

// write one byte per 4 KiB page of a host output buffer (its contents are overwritten afterwards), on up to 8
// threads for buffers of several MB
void touch_pages(void* buf, size_t bytes) {
    if (bytes < ((size_t)1 << 20)) return;
    char* b = static_cast<char*>(buf);
    const int nth = (int)std::min<size_t>(8, bytes >> 22) + 1;
    const size_t chunk = ((bytes / nth) + 4095) & ~(size_t)4095;
    auto work = [=](int k) {
        volatile char* q = b;
        for (size_t o = (size_t)k * chunk; o < std::min(bytes, (size_t)(k + 1) * chunk); o += 4096) q[o] = 0;
    };
    std::vector<std::thread> th;
    int k_started = 1;
    try {
        for (; k_started < nth; ++k_started) th.emplace_back(work, k_started);
    } catch (...) {  // no thread could be started: touch the remaining chunks here (no exception crosses the C-ABI)
    }
    for (int k = k_started; k < nth; ++k) work(k);
    work(0);
    for (auto& t : th) t.join();
}

// consecutive 256-B aligned sub-buffers of one device allocation (size pass with base == nullptr)
struct Carve {
    char* base = nullptr;
    size_t off = 0;
    template <class T>
    T* take(size_t count) {
        off = (off + 255) & ~(size_t)255;
        T* r = base ? reinterpret_cast<T*>(base + off) : nullptr;
        off += count * sizeof(T);
        return r;
    }
};
}  // namespace

struct pqd_pt {
    pqd_ctx* ctx = nullptr;
    int dim = 0, chi = 0, CHI = 0, D = 0, n_slices = 0;
    DevBuf<double2> Q, closure, closure0, bond0;
    DevBuf<double> Qsum;      // Re + Im of every slice element (the 3M operand of the TLS quad kernel; N2 = 4 only)
    DevBuf<int> gmap;
    std::vector<int> gmap_h;  // host copy: the plan derives its PT row units from it
};

struct pqd_plan {
    pqd_ctx* ctx = nullptr;
    int N2 = 0, CHI = 1, BT = 4, n_traj = 0, n_blocks = 0, n_steps = 0, n_sys = 1;
    bool nopt = true;
    bool split = false;  // small batch: one trajectory over N2 workgroups (pt_split.hip)
    bool quad = false;   // two-level system: register-resident quads (pt_quad.hip), blocks of BT = 4
    int qpw = 2;         // quads per workgroup (PQD_QPW)
    int qcg = 4;         // 4-column groups per wave (PQD_QCG; auto: 2 when the quads do not fill the CUs)
    int split_chunk = 0; // split groups: trajectories per launch when the batch exceeds the device (0: one launch)
    // split groups carrying several trajectories each (pt_msplit.hip): composite MTO operators, groups, exchange
    bool msplit = false;
    MsplitParams mq{};
    int n_cev = 0;
    DevBuf<int> ms_gtraj, ms_gend, cev_start;
    DevBuf<int4> cev;
    DevBuf<double2> Fev, Wev, msX;
    DevBuf<unsigned> ms_cnt;
    DevBuf<double2> Xs;
    DevBuf<unsigned> cnt, err;
    DevBuf<double2> L0, S, T, samples, M, Midle, F, W, rho0, ovec, sop, out;
    DevBuf<double2> Fidle, Widle;  // idle fused operators per system (pulse windows)
    DevBuf<int2> win;              // per-system pulse windows (free_prop.hip free_win_kernel), PQD_WIN=0: none
    int win_mode = 0;              // PQD_WIN: 1 auto (windows when they leave out >= 10% of the half steps), 2 always
    DevBuf<FreePropSys> systab;
    FuseParams fu{};
    DevBuf<int> sched, blk_traj, blk_end, blk_sys, blk_act, blk_src, traj_sys, wbeg, wend, ev_start;
    int64_t traj_steps = 0;       // executed trajectory-steps per execute (shared trunks counted once)
    int branch = 1;               // shared-trunk activation in the batched sweep (PQD_BRANCH)
    // trunk pre-pass (pqd_host.cpp plan_trunks): one MTO-free trajectory per system writes the checkpoints the
    // main sweep's slots start from
    int n_trunk = 0, tk_blocks = 0, tk_BT = 4;
    int tk_chunk = 0;  // split trunks per launch when they do not all fit the device at once (0: one launch)
    bool tk_split = false;
    SweepParams tk{};
    DevBuf<double2> ck, tk_out, tk_Xs;
    DevBuf<int> tk_ckmap, tk_wbeg, tk_wend, tk_evstart, tk_tsys, tk_blk_traj, tk_blk_end, tk_blk_sys, tk_blk_act,
        tk_blk_src;
    DevBuf<long long> tk_woff;
    DevBuf<int4> tk_units;
    DevBuf<unsigned> tk_cnt, tk_err;
    DevBuf<long long> woff;
    DevBuf<int4> ev, units;
    FreePropParams fp{};
    SweepParams sp{};
    int64_t out_len = 0;
    int n_out = 0;
    double t_start = 0.0, dt = 0.0;
    std::vector<long long> toff;  // ACE-table offsets per trajectory ((1 + n_out) rows of its window), + total
    DevBuf<long long> toff_d;
    DevBuf<double2> table;
    DevBuf<unsigned> flags;       // bit 0: non-finite output (PQD_ERR_NUMERIC)
    int split_fallbacks = 0;      // split launches that timed out and were re-run on the batched kernel
    // hipEvent triplets (start, free propagators done, sweep done) of the last RING executes, created once
    static constexpr int RING = 64;
    hipEvent_t ring[3 * RING] = {};
    bool ring_ready = false;
    int ev_head = 0, ev_count = 0;  // next slot; executes recorded since the last timing reset (<= RING kept)
    int32_t execs = 0;
    ~pqd_plan() {
        if (ring_ready)
            for (auto& e : ring) (void)hipEventDestroy(e);
    }
};


// upload the generators of n_sys systems into concatenated device buffers + a device table
static int upload_systems(int n_sys, const pqd_system* systems, hipStream_t s, DevBuf<double2>& L0,
                          DevBuf<double2>& S, DevBuf<double2>& T, DevBuf<double2>& smp, DevBuf<FreePropSys>& tab) {
    const int N = systems[0].dim, N2 = N * N;
    const size_t m2 = (size_t)N2 * N2;
    std::vector<Generators> G(n_sys);
    size_t nS = 0, nT = 0, nsmp = 0;
    for (int k = 0; k < n_sys; ++k) {
        build_generators(&systems[k], G[k]);
        nS += G[k].S.size(); nT += G[k].T.size(); nsmp += G[k].samples.size();
    }
    std::vector<cd> l0((size_t)n_sys * m2), sv, tv, sm;
    sv.reserve(nS); tv.reserve(nT); sm.reserve(nsmp);
    std::vector<size_t> oS, oT, oM;
    for (int k = 0; k < n_sys; ++k) {
        std::copy(G[k].L0.begin(), G[k].L0.end(), l0.begin() + k * m2);
        oS.push_back(sv.size()); sv.insert(sv.end(), G[k].S.begin(), G[k].S.end());
        oT.push_back(tv.size()); tv.insert(tv.end(), G[k].T.begin(), G[k].T.end());
        oM.push_back(sm.size()); sm.insert(sm.end(), G[k].samples.begin(), G[k].samples.end());
    }
    HIPCHK(L0.upload(reinterpret_cast<double2*>(l0.data()), l0.size(), s));
    HIPCHK(S.upload(reinterpret_cast<double2*>(sv.data()), sv.size(), s));
    HIPCHK(T.upload(reinterpret_cast<double2*>(tv.data()), tv.size(), s));
    HIPCHK(smp.upload(reinterpret_cast<double2*>(sm.data()), sm.size(), s));
    std::vector<FreePropSys> t(n_sys);
    for (int k = 0; k < n_sys; ++k) {
        const pqd_system& y = systems[k];
        t[k].L0 = L0.p + k * m2;
        t[k].S = S.p + oS[k];
        t[k].T = T.p + oT[k];
        t[k].samples = smp.p + oM[k];
        t[k].n_chan = y.n_chan;
        t[k].n_samples = std::max(1, y.n_samples);
        t[k].s_t0 = y.sample_t0;
        t[k].s_dt = y.n_chan > 0 ? y.sample_dt : 1.0;
    }
    HIPCHK(tab.upload(t.data(), t.size(), s));
    return PQD_OK;
}

extern "C" {

int32_t pqd_version(void) { return 1; }
const char* pqd_last_error(void) { return g_err.c_str(); }
int pqd_hip_versions(int32_t* build, int32_t* runtime) {
    if (!build || !runtime) return fail(PQD_ERR_ARG, "NULL argument");
    *build = HIP_VERSION;
    int v = 0;
    if (hipRuntimeGetVersion(&v) != hipSuccess) return fail(PQD_ERR_HIP, "hipRuntimeGetVersion failed");
    *runtime = v;
    return PQD_OK;
}

int pqd_ctx_create(int32_t device, pqd_ctx** out) {
    if (!out) return fail(PQD_ERR_ARG, "out is NULL");
    int ndev = 0;
    HIPCHK(hipGetDeviceCount(&ndev));
    if (device < 0 || device >= ndev) return fail(PQD_ERR_ARG, "device %d out of range (%d devices)", device, ndev);
    HIPCHK(hipSetDevice(device));
    hipDeviceProp_t prop;
    HIPCHK(hipGetDeviceProperties(&prop, device));
    if (std::strncmp(prop.gcnArchName, "gfx950", 6) != 0)
        return fail(PQD_ERR_UNSUPPORTED, "libpqd is built for gfx950 (MI355X); device is %s", prop.gcnArchName);
    auto* c = new pqd_ctx;
    c->device = device;
    hipError_t e = hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking);
    if (e != hipSuccess) {
        delete c;
        return fail(PQD_ERR_HIP, "hipStreamCreate: %s", hipGetErrorString(e));
    }
    *out = c;
    return PQD_OK;
}

void pqd_ctx_destroy(pqd_ctx* ctx) {
    if (!ctx) return;
    (void)hipSetDevice(ctx->device);
    (void)hipStreamSynchronize(ctx->stream);
    (void)hipStreamDestroy(ctx->stream);
    delete ctx;
}

int pqd_ctx_synchronize(pqd_ctx* ctx) {
    if (!ctx) return fail(PQD_ERR_ARG, "ctx is NULL");
    HIPCHK(hipStreamSynchronize(ctx->stream));
    return PQD_OK;
}

int pqd_pt_create(pqd_ctx* ctx, int32_t dim, const pqd_pt_desc* d, pqd_pt** out) {
    if (!ctx || !d || !out) return fail(PQD_ERR_ARG, "NULL argument");
    if (dim < 2 || dim > 6) return fail(PQD_ERR_UNSUPPORTED, "dim %d", dim);
    const int N2 = dim * dim;
    const int CHI = pad_chi(d->chi);
    if (d->chi < 1 || CHI < 0) return fail(PQD_ERR_UNSUPPORTED, "chi %d not in [1, 256]", d->chi);
    if (d->D < 1 || d->n_slices < 1) return fail(PQD_ERR_ARG, "D and n_slices must be >= 1");
    if (!d->Q || !d->closure || !d->closure0 || !d->bond0 || !d->gmap) return fail(PQD_ERR_ARG, "NULL PT array");
    for (int a = 0; a < N2; ++a)
        if (d->gmap[a] < 0 || d->gmap[a] >= d->D) return fail(PQD_ERR_ARG, "gmap[%d]=%d out of [0,%d)", a, d->gmap[a], d->D);
    HIPCHK(hipSetDevice(ctx->device));
    const int chi = d->chi;
    const size_t qn = (size_t)d->n_slices * d->D * CHI * CHI;
    std::vector<double2> Q(qn, make_double2(0, 0)), cl((size_t)d->n_slices * CHI, make_double2(0, 0));
    std::vector<double2> c0(CHI, make_double2(0, 0)), b0(CHI, make_double2(0, 0));
    const double2* src = reinterpret_cast<const double2*>(d->Q);
    for (size_t s = 0; s < (size_t)d->n_slices * d->D; ++s)
        for (int r = 0; r < chi; ++r)
            std::memcpy(&Q[(s * CHI + r) * CHI], &src[(s * chi + r) * chi], sizeof(double2) * chi);
    for (int s = 0; s < d->n_slices; ++s)
        std::memcpy(&cl[(size_t)s * CHI], reinterpret_cast<const double2*>(d->closure) + (size_t)s * chi,
                    sizeof(double2) * chi);
    std::memcpy(c0.data(), d->closure0, sizeof(double2) * chi);
    std::memcpy(b0.data(), d->bond0, sizeof(double2) * chi);
    auto* pt = new pqd_pt;
    pt->ctx = ctx; pt->dim = dim; pt->chi = chi; pt->CHI = CHI; pt->D = d->D; pt->n_slices = d->n_slices;
    pt->gmap_h.assign(d->gmap, d->gmap + N2);
    hipError_t e = pt->Q.upload(Q.data(), qn, ctx->stream);
    if (e == hipSuccess && N2 == 4) {
        std::vector<double> qs(qn);
        for (size_t k = 0; k < qn; ++k) qs[k] = Q[k].x + Q[k].y;
        e = pt->Qsum.upload(qs.data(), qn, ctx->stream);
        if (e == hipSuccess) e = hipStreamSynchronize(ctx->stream);  // qs goes out of scope
    }
    if (e == hipSuccess) e = pt->closure.upload(cl.data(), cl.size(), ctx->stream);
    if (e == hipSuccess) e = pt->closure0.upload(c0.data(), CHI, ctx->stream);
    if (e == hipSuccess) e = pt->bond0.upload(b0.data(), CHI, ctx->stream);
    if (e == hipSuccess) e = pt->gmap.upload(d->gmap, N2, ctx->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(ctx->stream);
    if (e != hipSuccess) {
        delete pt;
        return fail(e == hipErrorOutOfMemory ? PQD_ERR_NOMEM : PQD_ERR_HIP, "PT upload: %s", hipGetErrorString(e));
    }
    *out = pt;
    return PQD_OK;
}

void pqd_pt_destroy(pqd_pt* pt) { delete pt; }

int pqd_free_propagators(pqd_ctx* ctx, const pqd_system* sys, const pqd_grid* grid, pqd_c128* M_out) {
    if (!ctx || !M_out) return fail(PQD_ERR_ARG, "NULL argument");
    int rc = check_system(sys);
    if (rc) return rc;
    if ((rc = check_grid(grid))) return rc;
    HIPCHK(hipSetDevice(ctx->device));
    const int N2 = sys->dim * sys->dim;
    DevBuf<double2> L0, S, T, smp, M, Mi;
    DevBuf<FreePropSys> tab;
    hipStream_t s = ctx->stream;
    if ((rc = upload_systems(1, sys, s, L0, S, T, smp, tab))) return rc;
    const size_t nM = (size_t)2 * grid->n_steps * N2 * N2;
    HIPCHK(M.alloc(nM));
    FreePropParams fp{};
    fp.systems = tab.p; fp.n_sys = 1;
    fp.ta = grid->ta; fp.dt = grid->dt; fp.n_steps = grid->n_steps; fp.n_sub = grid->n_sub; fp.M = M.p;
    { const char* f4 = getenv("PQD_FP4"); fp.packed4 = (f4 && atoi(f4) == 0) ? 0 : 1; }
    { const char* fm = getenv("PQD_FPM"); fp.mfma = fm ? atoi(fm) : 1; }
    if (const char* ie = getenv("PQD_IDLE"); !(ie && atoi(ie) == 0)) {
        HIPCHK(Mi.alloc((size_t)N2 * N2));
        fp.Midle = Mi.p;
    }
    HIPCHK(launch_free_prop(N2, fp, s));
    if (nM) HIPCHK(hipMemcpyAsync(M_out, M.p, nM * sizeof(double2), hipMemcpyDeviceToHost, s));
    HIPCHK(hipStreamSynchronize(s));
    return PQD_OK;
}

// PT rows per wave for the 3M sweep. Rows whose coupling-eigenvalue pair maps to the same slice (dictionary
// PTs, e.g. 16 biexciton rows over 9 slices) are contracted together in units of up to rmax rows, so one L2
// read of a slice feeds all of them. Units (cost = rows) go to the least-loaded wave, largest first. A unit is
// (slice, row 0, row 1 or -1, row 2 | row 3 << 16 or -1, a missing row 3 being 0x7FFF); each wave's list ends
// with slice -1.
static std::vector<int4> pt_row_units(const std::vector<int>& gmap, int NW, int rmax) {
    const int N2 = (int)gmap.size();
    std::vector<int4> units;
    std::vector<int> done(N2, 0);
    for (int a = 0; a < N2; ++a) {
        if (done[a]) continue;
        int rows[4] = {-1, -1, -1, -1}, cnt = 0;
        for (int c = a; c < N2 && cnt < rmax; ++c)
            if (!done[c] && gmap[c] == gmap[a]) { done[c] = 1; rows[cnt++] = c; }
        const int w = cnt > 2 ? (rows[2] | ((cnt > 3 ? rows[3] : 0x7FFF) << 16)) : -1;
        units.push_back(make_int4(gmap[a], rows[0], rows[1], w));
    }
    auto cost = [](const int4& e) { return e.z < 0 ? 1 : e.w < 0 ? 2 : (e.w >> 16) == 0x7FFF ? 3 : 4; };
    std::stable_sort(units.begin(), units.end(), [&](const int4& x, const int4& y) { return cost(x) > cost(y); });
    std::vector<std::vector<int4>> per(NW);
    std::vector<int> load(NW, 0);
    // the PT phase lasts as long as the most-loaded wave: aim at T = ceil(rows / waves) rows per wave. Whole units go
    // to the least-loaded wave they fit (largest first); a unit that fits nowhere is split into its rows,
    // which then fill the waves' remaining capacity, rows of one slice kept together per wave (a split slice is read
    // once more from L2 per extra wave). Six-level dictionary PT (9 slices x 4 rows, 8 waves): max 5 rows per wave
    // instead of 8 (one wave held two 4-row units). Least-loaded first, so the two waves of a SIMD (w, w + NW / 2)
    // also stay balanced: their MFMAs share its matrix pipe
    int T = (N2 + NW - 1) / NW;
    if (const char* e = getenv("PQD_UNITBAL"); e && atoi(e) == 0) T = 1 << 20;  // A/B: whole units, least loaded
    std::vector<int> pending;  // rows of split units, slice-ordered
    for (const int4& e : units) {
        int w = -1;
        for (int k = 0; k < NW; ++k)
            if (load[k] + cost(e) <= T && (w < 0 || load[k] < load[w])) w = k;
        if (w >= 0) {
            per[w].push_back(e);
            load[w] += cost(e);
            continue;
        }
        const int rows[4] = {e.y, e.z, e.w >= 0 ? (e.w & 0xFFFF) : -1, e.w >= 0 ? (e.w >> 16) : -1};
        for (int r : rows)
            if (r >= 0 && r != 0x7FFF) pending.push_back(r);
    }
    for (size_t i = 0; i < pending.size();) {
        int w = 0;  // the least-loaded wave takes as many rows of this slice as fit (at most rmax)
        for (int k = 1; k < NW; ++k)
            if (load[k] < load[w]) w = k;
        const int room = std::max(1, std::min(rmax, T - load[w]));
        int rows[4] = {-1, -1, -1, -1}, cnt = 0;
        const int g = gmap[pending[i]];
        while (i < pending.size() && cnt < room && gmap[pending[i]] == g) rows[cnt++] = pending[i++];
        const int wv = cnt > 2 ? (rows[2] | ((cnt > 3 ? rows[3] : 0x7FFF) << 16)) : -1;
        per[w].push_back(make_int4(g, rows[0], rows[1], wv));
        load[w] += cnt;
    }
    size_t umax = 1;
    for (auto& v : per) umax = std::max(umax, v.size() + 1);
    std::vector<int4> out((size_t)NW * umax, make_int4(-1, 0, -1, -1));
    for (int w = 0; w < NW; ++w)
        for (size_t k = 0; k < per[w].size(); ++k) out[(size_t)w * umax + k] = per[w][k];
    return out;
}

// Shared trunks inside a lock-step block (the reference re-propagates 0 -> t1 in every trajectory of a two-time
// sweep: correlations.py:155-169, pol_entanglement/G2.py:486-497). j[t] = the last step at whose top (before its
// outputs) trajectory t still holds the MTO-free state: its first MTO's step if that MTO applies after the output,
// one less if it applies before. Slots are ordered by j; slot k becomes active at
// act[k] = min(j_k, out_begin_k, j_m) by copying the (state, fused flag) of an earlier slot m of the same system that
// is already active then (act[m] < act[k]) and still MTO-free (j_m >= act[k]); before that it is dormant (no column
// phases, its PT rows skipped where a whole row block is dormant). Outputs before act[k] are never needed
// (act[k] <= out_begin_k), so every trajectory's outputs are those of its own full run.
static void branch_slots(int BT, const int* members, const std::vector<int>& jv, const int32_t* out_begin,
                         const std::vector<int>& tsys, bool enable, int* act, int* src) {
    for (int k = 0; k < BT; ++k) {
        const int t = members[k];
        src[k] = -1;
        if (t < 0) { act[k] = INT_MAX; continue; }
        act[k] = 0;
        if (!enable) continue;
        const int a = std::min(jv[t], out_begin[t]);
        int best = 0, bm = -1;
        for (int m = 0; m < k; ++m) {
            const int tm = members[m];
            if (tm < 0 || tsys[tm] != tsys[t]) continue;
            const int cand = std::min(a, jv[tm]);
            if (act[m] < cand && cand > best) { best = cand; bm = m; }
        }
        if (bm >= 0) { act[k] = best; src[k] = bm; }
    }
}

// Trunk pre-pass of a plan: one MTO-free trajectory per system that has checkpoints, propagated from step 0 to
// its last checkpoint step, writing the augmented state at the top of every checkpoint step (ck_steps[y], indices
// ck_base[y] + k). It runs before the main sweep on split groups when those fit (N2 >= 9, as in auto mode), else
// as batched workgroups of four; the batched layout is always built (fallback after a split timeout).
static int plan_trunks(pqd_plan* P, pqd_ctx* ctx, int n_sys, const std::vector<std::vector<int>>& ck_steps,
                       const std::vector<int>& ck_base, int n_ck, int n_cu, int N2, int n_out, const pqd_pt* pt,
                       hipStream_t s) {
    const int ns = P->n_steps, CHI = P->CHI;
    std::vector<int> wb, we, ts, map;
    std::vector<long long> wo;
    for (int y = 0; y < n_sys; ++y) {
        if (ck_steps[y].empty()) continue;
        const int t = (int)ts.size(), L = ck_steps[y].back();
        ts.push_back(y);
        wb.push_back(L);
        we.push_back(L);
        wo.push_back((long long)t * n_out);
        map.resize((size_t)(t + 1) * (ns + 1), -1);
        for (size_t k = 0; k < ck_steps[y].size(); ++k) map[(size_t)t * (ns + 1) + ck_steps[y][k]] = ck_base[y] + (int)k;
        P->traj_steps += L + 1;
    }
    const int nt = (int)ts.size();
    P->n_trunk = nt;
    if (!nt) return PQD_OK;
    std::vector<int> evs0(nt + 1, 0);
    HIPCHK(P->ck.alloc((size_t)n_ck * N2 * CHI));
    HIPCHK(P->tk_out.alloc((size_t)nt * n_out));
    HIPCHK(P->tk_ckmap.upload(map.data(), map.size(), s));
    HIPCHK(P->tk_wbeg.upload(wb.data(), nt, s));
    HIPCHK(P->tk_wend.upload(we.data(), nt, s));
    HIPCHK(P->tk_woff.upload(wo.data(), nt, s));
    HIPCHK(P->tk_tsys.upload(ts.data(), nt, s));
    HIPCHK(P->tk_evstart.upload(evs0.data(), evs0.size(), s));
    // batched layout: four trunks per workgroup
    const int BT = 4;
    std::vector<int> bt, be, bs, ba, bsrc;
    for (int t = 0; t < nt; t += BT) {
        int end = 0;
        for (int q = 0; q < BT; ++q) {
            const int u = t + q < nt ? t + q : -1;
            bt.push_back(u);
            ba.push_back(u >= 0 ? 0 : INT_MAX);
            bsrc.push_back(-1);
            if (u >= 0) end = std::max(end, we[u]);
        }
        be.push_back(end);
        bs.push_back(ts[t]);
    }
    P->tk_BT = BT;
    P->tk_blocks = (int)be.size();
    HIPCHK(P->tk_blk_traj.upload(bt.data(), bt.size(), s));
    HIPCHK(P->tk_blk_end.upload(be.data(), be.size(), s));
    HIPCHK(P->tk_blk_sys.upload(bs.data(), bs.size(), s));
    HIPCHK(P->tk_blk_act.upload(ba.data(), ba.size(), s));
    HIPCHK(P->tk_blk_src.upload(bsrc.data(), bsrc.size(), s));
    {
        const int nw = BT * sweep_wpt(N2, BT, CHI);
        std::vector<int4> u = pt_row_units(pt->gmap_h, nw, sweep_rmax(N2, BT, CHI));
        HIPCHK(P->tk_units.upload(u.data(), u.size(), s));
    }
    const int bpc = split_blocks_per_cu(N2, CHI);
    const char* e = getenv("PQD_SPLIT");
    const int mode = e ? atoi(e) : 1;
    // more trunks than the device holds as co-resident groups: consecutive launches of as many as fit (C5 tomography:
    // 8 six-level trunks = 288 workgroups on 256 CUs -> 7 + 1; a group steps ~7x faster than a batched block)
    const int fit = bpc >= 1 ? (n_cu * bpc) / split_group_size(N2) : 0;
    P->tk_chunk = fit >= 1 && nt > fit ? fit : 0;
    P->tk_split = mode != 0 && N2 >= 9 && bpc >= 1 && fit >= 1 &&
                  split_supported(N2, CHI, std::min(nt, fit), n_cu * bpc) &&
                  nt <= (N2 >= 25 ? 4 : 2) * fit;  // launches in a row still beat one batched pass (§4.6 latencies)
    HIPCHK(P->tk_Xs.alloc((size_t)nt * 4 * N2 * CHI));  // split exchange: 2 slots of granules (pt_split.hip)
    HIPCHK(P->tk_cnt.alloc((size_t)nt * 64));  // split arrival flags: two 128-B lines per group
    HIPCHK(P->tk_err.alloc(4));
    (void)ctx;
    return PQD_OK;
}

// the trunk pre-pass launch parameters: the main sweep's, with the trunk trajectories and checkpoint map
static void finalize_trunks(pqd_plan* P) {
    P->sp.ck = P->ck.p;
    P->sp.ck_map = nullptr;
    if (!P->n_trunk) return;
    SweepParams& k = P->tk;
    k = P->sp;
    k.blk_traj = P->tk_blk_traj.p; k.blk_end = P->tk_blk_end.p; k.blk_sys = P->tk_blk_sys.p;
    k.blk_act = P->tk_blk_act.p; k.blk_src = P->tk_blk_src.p;
    k.traj_sys = P->tk_tsys.p; k.wbeg = P->tk_wbeg.p; k.wend = P->tk_wend.p; k.woff = P->tk_woff.p;
    k.ev_start = P->tk_evstart.p; k.out = P->tk_out.p;
    k.ck_map = P->tk_ckmap.p; k.ck_stride = P->n_steps + 1;
    const int nw = P->tk_BT * sweep_wpt(P->N2, P->tk_BT, P->CHI);
    k.units = (P->sp.units ? P->tk_units.p : nullptr);
    k.umax = (int)(P->tk_units.n / nw);
}

// the main batched sweep of a plan: quads (N2 = 4) or BT-trajectory workgroups
static hipError_t launch_main(pqd_plan* P, hipStream_t s) {
    if (P->quad) return launch_quad(P->CHI, P->n_blocks, P->qpw, P->qcg, P->sp, s);
    return launch_sweep(P->N2, P->CHI, P->BT, P->n_blocks, P->sp, s);
}

static hipError_t launch_trunks(pqd_plan* P, hipStream_t s) {
    if (!P->n_trunk) return hipSuccess;
    if (P->tk_split)
        return launch_split(P->N2, P->CHI, P->n_trunk, P->tk, P->tk_Xs.p, P->tk_cnt.p, P->tk_err.p, s, P->tk_chunk);
    return launch_sweep(P->N2, P->CHI, P->tk_BT, P->tk_blocks, P->tk, s);
}

int pqd_plan_create_multi(pqd_ctx* ctx, int32_t n_sys, const pqd_system* systems, const int32_t* traj_sys,
                          const pqd_grid* grid, const pqd_pt* pt, const int32_t* sched, const pqd_c128* rho0,
                          int32_t n_out, const pqd_c128* out_ops, const pqd_traj* tr, int64_t out_len,
                          pqd_plan** out) {
    if (!ctx || !rho0 || !tr || !out || !systems) return fail(PQD_ERR_ARG, "NULL argument");
    if (n_sys < 1) return fail(PQD_ERR_ARG, "n_sys must be >= 1");
    if (n_sys > 1 && !traj_sys) return fail(PQD_ERR_ARG, "traj_sys is NULL with n_sys > 1");
    int rc = 0;
    for (int k = 0; k < n_sys; ++k) {
        if ((rc = check_system(&systems[k]))) return rc;
        if (systems[k].dim != systems[0].dim) return fail(PQD_ERR_ARG, "system %d: dim %d != %d", k, systems[k].dim, systems[0].dim);
    }
    const pqd_system* sys = systems;
    for (int t = 0; t < tr->n_traj; ++t)
        if (traj_sys && (traj_sys[t] < 0 || traj_sys[t] >= n_sys)) return fail(PQD_ERR_ARG, "traj_sys[%d]=%d out of [0,%d)", t, traj_sys[t], n_sys);
    if ((rc = check_grid(grid))) return rc;
    const int N = sys->dim, N2 = N * N;
    const size_t m2 = (size_t)N2 * N2;
    const int ns = grid->n_steps;
    if (n_out < 1 || n_out > 256 || !out_ops) return fail(PQD_ERR_ARG, "n_out %d not in [1, 256]", n_out);
    if (tr->n_traj < 0 || (tr->n_traj > 0 && (!tr->out_begin || !tr->out_end || !tr->out_offset)))
        return fail(PQD_ERR_ARG, "bad trajectory arrays");
    if (pt) {
        if (pt->ctx != ctx) return fail(PQD_ERR_ARG, "PT belongs to another context");
        if (pt->dim != N) return fail(PQD_ERR_ARG, "PT dim %d != system dim %d", pt->dim, N);
        if (!sweep_supported(N2, pt->CHI) && !(pt->CHI == 256 && msplit_supported(N2, pt->CHI, n_out)))
            return fail(PQD_ERR_UNSUPPORTED, "N2=%d CHI=%d (chi 256: N2 4, 9 or 16 and at most 8 outputs)", N2, pt->CHI);
    }
    for (int t = 0; t < tr->n_traj; ++t) {
        const int b = tr->out_begin[t], e = tr->out_end[t];
        if (b < 0 || e < b || e > ns)
            return fail(PQD_ERR_ARG, "trajectory %d window [%d, %d] outside [0, %d]", t, b, e, ns);
        const int64_t hi = tr->out_offset[t] + (int64_t)(e - b + 1) * n_out;
        if (tr->out_offset[t] < 0 || hi > out_len)
            return fail(PQD_ERR_ARG, "trajectory %d output [%lld, %lld) exceeds out_len %lld", t,
                        (long long)tr->out_offset[t], (long long)hi, (long long)out_len);
    }
    if (tr->n_mto < 0 || (tr->n_mto > 0 && (!tr->mto_traj || !tr->mto_step || !tr->mto_before || !tr->mto_kind || !tr->mto_ops)))
        return fail(PQD_ERR_ARG, "bad MTO arrays");
    for (int q = 0; q < tr->n_mto; ++q) {
        if (tr->mto_traj[q] < 0 || tr->mto_traj[q] >= tr->n_traj) return fail(PQD_ERR_ARG, "MTO %d: bad trajectory", q);
        if (tr->mto_step[q] < 0 || tr->mto_step[q] > ns) return fail(PQD_ERR_ARG, "MTO %d: step %d outside [0, %d]", q, tr->mto_step[q], ns);
        if (tr->mto_kind[q] < 0 || tr->mto_kind[q] > 2) return fail(PQD_ERR_ARG, "MTO %d: kind %d", q, tr->mto_kind[q]);
    }
    std::vector<int32_t> sch(std::max(1, ns), 0);
    if (pt) {
        for (int n = 0; n < ns; ++n) {
            const int s = sched ? sched[n] : std::min(n, pt->n_slices - 1);
            if (s < 0 || s >= pt->n_slices) return fail(PQD_ERR_ARG, "sched[%d]=%d out of [0,%d)", n, s, pt->n_slices);
            sch[n] = s;
        }
    }
    HIPCHK(hipSetDevice(ctx->device));
    hipStream_t s = ctx->stream;
    auto* P = new pqd_plan;
    std::unique_ptr<pqd_plan> guard(P);
    P->ctx = ctx; P->N2 = N2; P->n_traj = tr->n_traj; P->n_steps = ns; P->out_len = out_len;
    P->n_out = n_out; P->t_start = grid->ta; P->dt = grid->dt;
    P->toff.assign(tr->n_traj + 1, 0);
    for (int t = 0; t < tr->n_traj; ++t)
        P->toff[t + 1] = P->toff[t] + (long long)(1 + n_out) * (tr->out_end[t] - tr->out_begin[t] + 1);
    P->nopt = (pt == nullptr);
    P->CHI = pt ? pt->CHI : 1;
    P->n_sys = n_sys;

    // ---- generators for the free propagators (one table entry per system)
    if ((rc = upload_systems(n_sys, systems, s, P->L0, P->S, P->T, P->samples, P->systab))) return rc;
    HIPCHK(P->M.alloc(std::max<size_t>(1, (size_t)n_sys * 2 * ns * m2)));
    std::vector<int> tsys(std::max(1, tr->n_traj), 0);
    for (int t = 0; t < tr->n_traj; ++t) tsys[t] = traj_sys ? traj_sys[t] : 0;
    HIPCHK(P->traj_sys.upload(tsys.data(), tsys.size(), s));

    // ---- MTO events: per trajectory, stable-sorted by (step, phase), same-slot ops composed. Every MTO kind is
    // rho -> L rho R ("": A rho A^dag, _left: A rho, _right: rho A), so a slot's ops compose as N x N products
    // (L = L_k ... L_1, R = R_1 ... R_k) and its superoperator is L (x) R^T; identical (L, R) pairs share one
    // superoperator (a two-time sweep applies the same operators at every t1).
    std::vector<std::vector<int>> per(tr->n_traj);
    for (int q = 0; q < tr->n_mto; ++q) per[tr->mto_traj[q]].push_back(q);
    std::vector<int> ev_start(tr->n_traj + 1, 0);
    std::vector<int4> evs;
    std::vector<cd> sops;
    std::unordered_map<std::string, int> sop_index;
    const size_t nn = (size_t)N * N;
    std::vector<cd> Lm(nn), Rm(nn), Lq(nn), Rq(nn), key_buf(2 * nn);
    auto eye = [&](std::vector<cd>& M) { std::fill(M.begin(), M.end(), cd(0)); for (int i = 0; i < N; ++i) M[(size_t)i * N + i] = 1.0; };
    for (int t = 0; t < tr->n_traj; ++t) {
        auto& v = per[t];
        auto key = [&](int q) { return 2 * tr->mto_step[q] + (tr->mto_before[q] ? 0 : 1); };
        std::stable_sort(v.begin(), v.end(), [&](int a, int b) { return key(a) < key(b); });
        ev_start[t] = (int)evs.size();
        size_t i = 0;
        while (i < v.size()) {
            const int k0 = key(v[i]);
            eye(Lm);
            eye(Rm);
            for (; i < v.size() && key(v[i]) == k0; ++i) {
                const int q = v[i];
                const cd* A = C(tr->mto_ops) + (size_t)q * nn;
                const int kind = tr->mto_kind[q];
                if (kind == 2) eye(Lq); else std::copy(A, A + nn, Lq.begin());
                if (kind == 1) eye(Rq);
                else if (kind == 2) std::copy(A, A + nn, Rq.begin());
                else
                    for (int r = 0; r < N; ++r)
                        for (int c = 0; c < N; ++c) Rq[(size_t)r * N + c] = std::conj(A[(size_t)c * N + r]);
                matmul_sq(N, Lq.data(), Lm.data(), Lm.data());  // L <- L_q L
                matmul_sq(N, Rm.data(), Rq.data(), Rm.data());  // R <- R R_q
            }
            std::copy(Lm.begin(), Lm.end(), key_buf.begin());
            std::copy(Rm.begin(), Rm.end(), key_buf.begin() + nn);
            std::string kb(reinterpret_cast<const char*>(key_buf.data()), key_buf.size() * sizeof(cd));
            auto it = sop_index.find(kb);
            int idx;
            if (it != sop_index.end()) {
                idx = it->second;
            } else {
                idx = (int)(sops.size() / m2);
                sop_index.emplace(std::move(kb), idx);
                sops.resize(sops.size() + m2);
                cd* S = sops.data() + (size_t)idx * m2;
                for (int a = 0; a < N; ++a)
                    for (int j = 0; j < N; ++j)
                        for (int k = 0; k < N; ++k)
                            for (int l = 0; l < N; ++l)
                                S[(size_t)(a * N + j) * N2 + (k * N + l)] = Lm[(size_t)a * N + k] * Rm[(size_t)l * N + j];
            }
            evs.push_back(make_int4(k0 >> 1, k0 & 1, idx, 0));
        }
    }
    ev_start[tr->n_traj] = (int)evs.size();
    if (evs.empty()) evs.push_back(make_int4(-1, -1, 0, 0));
    if (sops.empty()) sops.assign(m2, 0.0);
    HIPCHK(P->ev.upload(evs.data(), evs.size(), s));
    HIPCHK(P->ev_start.upload(ev_start.data(), ev_start.size(), s));
    HIPCHK(P->sop.upload(reinterpret_cast<double2*>(sops.data()), sops.size(), s));

    // ---- output operators: ovec[k][i*N+j] = O_k[j][i]   (<O> = Tr(O rho))
    std::vector<cd> ov((size_t)n_out * N2);
    for (int k = 0; k < n_out; ++k)
        for (int i = 0; i < N; ++i)
            for (int j = 0; j < N; ++j) ov[(size_t)k * N2 + i * N + j] = C(out_ops)[(size_t)k * N2 + j * N + i];
    HIPCHK(P->ovec.upload(reinterpret_cast<double2*>(ov.data()), ov.size(), s));
    HIPCHK(P->rho0.upload(reinterpret_cast<const double2*>(rho0), N2, s));

    // ---- trajectory windows and block grouping (longest first so lock-step blocks end together)
    HIPCHK(P->wbeg.upload(tr->out_begin, std::max(1, tr->n_traj), s));
    HIPCHK(P->wend.upload(tr->out_end, std::max(1, tr->n_traj), s));
    HIPCHK(P->woff.upload(reinterpret_cast<const long long*>(tr->out_offset), std::max(1, tr->n_traj), s));
    std::vector<int> order(tr->n_traj);
    for (int t = 0; t < tr->n_traj; ++t) order[t] = t;
    // j[t]: last step whose top still sees the MTO-free state (branch_slots)
    std::vector<int> jv(std::max(1, tr->n_traj), 0);
    for (int t = 0; t < tr->n_traj; ++t) {
        if (ev_start[t] == ev_start[t + 1]) { jv[t] = tr->out_end[t]; continue; }
        const int4 e = evs[ev_start[t]];
        jv[t] = e.y == 1 ? e.x : e.x - 1;
    }
    // group by system (a workgroup whose trajectories share one system reads one set of free propagators),
    // longest first inside a system, then by branch step (neighbouring slots share the longest trunk)
    std::stable_sort(order.begin(), order.end(), [&](int a, int b) {
        if (tsys[a] != tsys[b]) return tsys[a] < tsys[b];
        if (tr->out_end[a] != tr->out_end[b]) return tr->out_end[a] > tr->out_end[b];
        return jv[a] < jv[b];
    });
    // trajectories per workgroup: 8 (half the PT-slice L2 traffic per trajectory) when the LDS allows it
    // and the batch still fills every CU, else 4
    int n_cu = 256;
    {
        hipDeviceProp_t prop;
        if (hipGetDeviceProperties(&prop, ctx->device) == hipSuccess) n_cu = prop.multiProcessorCount;
    }
    // latency path: a batch whose trajectories fit one group of N2 workgroups each on the device runs
    // each trajectory over N2 workgroups (pt_split.hip). Measured: 2.3-3.6x faster per step
    // at N2 = 16 and 36; at N2 = 4 the batched kernel's single workgroup is as fast, so auto mode skips it.
    // PQD_SPLIT: 0 off, 1 auto, 2 whenever the device holds the groups.
    {
        const char* e = getenv("PQD_SPLIT");
        const int mode = e ? atoi(e) : 1;
        // the spin hand-off needs every workgroup of a group resident: the occupancy the runtime reports for the
        // split kernel (one workgroup per CU by its LDS request) must cover all n_traj * N2 workgroups
        const int bpc = (pt && mode != 0) ? split_blocks_per_cu(N2, P->CHI) : 0;
        // a batch just above what the device holds runs as consecutive co-resident launches (up to 4 at N2 >= 25,
        // 2 below: a group step is 3.6x / 2.4x faster than a batched block's)
        const int fit = bpc >= 1 ? (n_cu * bpc) / split_group_size(N2) : 0;
        // (not where multi-trajectory groups can take the batch: one launch of those beats consecutive launches)
        const char* msa = getenv("PQD_MSPLIT");
        const bool ms_can = !(msa && atoi(msa) == 0) && msplit_supported(N2, P->CHI, n_out) &&
                            [] { const char* f = getenv("PQD_FUSE"); return f ? atoi(f) != 0 : true; }();
        const int max_launches = ms_can ? 1 : (N2 >= 25 ? 4 : 2);
        const char* ms = getenv("PQD_MSPLIT");  // 2: multi-trajectory split groups in place of these (A/B, tests)
        P->split = pt && mode != 0 && !(ms && atoi(ms) == 2) && fit >= 1 && split_supported(N2, P->CHI, std::min(tr->n_traj, fit), n_cu * bpc) &&
                   tr->n_traj <= max_launches * fit && (mode == 2 || N2 >= 9);
        P->split_chunk = P->split && tr->n_traj > fit ? fit : 0;
    }
    int BT = (sweep_max_bt(N2) >= 8 && tr->n_traj >= 8 * n_cu) ? 8 : 4;
    if (const char* e = getenv("PQD_BT")) BT = std::min(atoi(e) >= 8 ? 8 : 4, sweep_max_bt(N2));
    if (P->CHI > 64) BT = 4;  // chi = 128: only four augmented states fit the LDS
    // two-level system: the register-resident quad kernel (pt_quad.hip) unless split groups were forced or
    // PQD_QUAD=0 (A/B); its blocks are quads
    {
        const char* e = getenv("PQD_QUAD");
        // chi = 64 quads only on request (PQD_QUAD=2): their slices do not fit the registers yet and the batched
        // kernel is faster (C2 shape at chi = 64: 19.9 ms batched, 41.9 ms quads; profiles/r03/q64.log)
        P->quad = pt && !P->split && quad_supported(N2, P->CHI) && !(e && atoi(e) == 0) &&
                  (P->CHI != 64 || (e && atoi(e) == 2));
        // chi = 32: one quad per workgroup, so the two 8-column-strip workgroups sharing a CU barrier independently
        // (C2: 19.8 -> 18.4 ms per launch with the strips below, profiles/r02/quad/envab_qpw_qcg.log)
        if (P->CHI == 32) P->qpw = 1;
        if (const char* w = getenv("PQD_QPW")) P->qpw = std::max(1, atoi(w));
        if (P->quad) BT = 4;
    }
    P->BT = BT;
    std::vector<int> bt, be, bs, ba, bsrc;
    {
        const char* e = getenv("PQD_BRANCH");
        P->branch = (e && atoi(e) == 0) ? 0 : 1;
    }
    const bool fuse_on = !P->nopt && ns > 0 && [] { const char* f = getenv("PQD_FUSE"); return f ? atoi(f) != 0 : true; }();
    // batches the single-trajectory split groups do not take: split groups of TB trajectories each (pt_msplit.hip),
    // G = N2 / 2 workgroups per group (N2 = 9: 9), up to 32 / G groups per XCD (their hand-offs in one L2). PQD_MSPLIT: 0 off, 1 auto,
    // 2 whenever supported; PQD_MS_TB forces the trajectories per group
    int ms_groups = 0, ms_TB = 0, ms_xcd = 0;
    {
        const char* e = getenv("PQD_MSPLIT");
        int mode = e ? atoi(e) : 1;
        // PQD_SPLIT=0 (batched kernel only) and a forced trunk pre-pass (PQD_TRUNK=1) keep the batched path
        if (const char* sp0 = getenv("PQD_SPLIT"); sp0 && atoi(sp0) == 0) mode = 0;
        if (const char* tk = getenv("PQD_TRUNK"); tk && atoi(tk) == 1 && mode == 1) mode = 0;
        if (pt && P->CHI == 256) mode = 2;  // no other path holds chi = 256
        const int bpc = (pt && !P->split && mode != 0 && fuse_on && tr->n_traj >= 1 && msplit_supported(N2, P->CHI, n_out))
                            ? msplit_blocks_per_cu(N2, P->CHI) : 0;
        if (bpc >= 1) {
            const int G = msplit_group_size(N2, P->CHI);
            const int resident = n_cu * bpc / G;          // groups the device holds at once
            const int gps = 32 / G;                        // groups per XCD slot (32 CUs per XCD on MI355X)
            // PQD_SPLIT_XCD=0: the plain grid (groups may span XCDs, sc1 exchange), as many groups as are resident
            bool xgrid = [] { const char* x = getenv("PQD_SPLIT_XCD"); return !(x && atoi(x) == 0); }();
            // where the XCD slots hold fewer groups than the device (G > 16: one group of 18 per 32 CUs at N2 = 36)
            // and that leaves more than 8 trajectories per group, the plain grid's extra groups pay for its cross-XCD
            // exchange (six-level, 128 trajectories: 11.6 against 14.6 us per grid step; equal at 64, slower below,
            // profiles/r06/msx2/)
            if (xgrid && gps >= 1 && 8 * gps < resident) {
                const int tbx = (tr->n_traj + 8 * gps - 1) / (8 * gps), tbp = (tr->n_traj + resident - 1) / resident;
                if (tbx > 8 && tbp < tbx) xgrid = false;
            }
            const int max_groups = std::min(resident, (xgrid && gps >= 1) ? 8 * gps : resident);
            int TB = (tr->n_traj + max_groups - 1) / std::max(1, max_groups);
            if (const char* f = getenv("PQD_MS_TB")) TB = std::max(TB, atoi(f));
            const int n_groups = (tr->n_traj + TB - 1) / TB;
            // auto: while a group's per-step work stays below the batched kernel's per-step time
            // (DESIGN.md §4.10); the single-trajectory groups keep the batches they fit
            // and while shared trunks would save little: the batched sweep starts each slot at its branch step (a
            // G2_reuse grid saves about half of its steps there), a split group runs every trajectory from step 0
            // (a system's trunk itself is propagated once: what sharing saves is the activations beyond its longest)
            int64_t shared = 0, total = 0;
            std::vector<int> amax(n_sys, 0);
            for (int t = 0; t < tr->n_traj; ++t) {
                const int a = std::max(0, std::min(jv[t], tr->out_begin[t]));
                shared += a;
                amax[tsys[t]] = std::max(amax[tsys[t]], a);
                total += tr->out_end[t] + 1;
            }
            for (int y = 0; y < n_sys; ++y) shared -= amax[y];
            // (measured, profiles/r06/bfly/c4ntraj.log, µs per grid step vs the batched kernel: 32 trajectories TB = 1
            // 2.8 vs 13.5; 256 TB = 8 6.0 vs 11.8; 384 TB = 12 8.3 vs 11.5; 512 TB = 16 9.8 vs 11.1)
            const bool want = mode == 2 || (TB <= 16 && 4 * shared <= total);
            // a group's composite MTO steps are held in LDS (pt_msplit.hip s_cev): at most msplit_cev_max() per group
            int max_cev = 0;
            for (int k0 = 0; k0 < tr->n_traj; k0 += TB) {
                int c = 0;
                for (int k = k0; k < std::min(tr->n_traj, k0 + TB); ++k) {
                    const int t = order[k];
                    for (int i = ev_start[t]; i < ev_start[t + 1]; ++i)
                        if (i == ev_start[t] || evs[i].x != evs[i - 1].x) ++c;
                }
                max_cev = std::max(max_cev, c);
            }
            if (want && TB <= msplit_tbmax(N2, P->CHI) && n_groups <= resident && max_cev <= msplit_cev_max()) {
                P->msplit = true;
                ms_TB = TB;
                ms_groups = n_groups;
                ms_xcd = (xgrid && gps >= 1 && n_groups <= 8 * gps) ? (n_groups + 7) / 8 : 0;
                if (const char* x = getenv("PQD_SPLIT_XCD"); x && atoi(x) == 0) ms_xcd = 0;
            }
        }
    }
    if (pt && P->CHI == 256 && !P->msplit)
        return fail(PQD_ERR_UNSUPPORTED, "chi 256 runs on multi-trajectory split groups only: %d trajectories at N2=%d do "
                    "not fit one launch of them (at most 8 per group), or the plan has no fused steps (PQD_FUSE=0)",
                    tr->n_traj, N2);
    const bool branch_on = P->branch != 0 && pt != nullptr && !P->split && !P->msplit;
    // blocks are filled in this order and may straddle systems (each wave indexes its own system's propagators),
    // so a scan with one trajectory per system still fills every slot of a workgroup
    for (size_t k = 0; k < order.size();) {
        const int sy = tsys[order[k]];
        int filled = 0, end = 0;
        const size_t b0 = bt.size();
        while (k < order.size() && filled < BT) {
            bt.push_back(order[k]);
            end = std::max(end, tr->out_end[order[k]]);
            ++k; ++filled;
        }
        for (; filled < BT; ++filled) bt.push_back(-1);
        // slots by branch step (empty ones last): the trunk passes from slot to slot
        std::stable_sort(bt.begin() + b0, bt.end(), [&](int a, int b) {
            if (a < 0 || b < 0) return a >= 0 && b < 0;
            return jv[a] < jv[b];
        });
        ba.resize(bt.size());
        bsrc.resize(bt.size());
        branch_slots(BT, bt.data() + b0, jv, tr->out_begin, tsys, branch_on, ba.data() + b0, bsrc.data() + b0);
        be.push_back(end);
        bs.push_back(sy);
    }
    // quad kernel: strips of 8 columns (twice the waves, two per SIMD) overlap one wave's round trips with the
    // other's MFMAs: with no more quads than CUs (C2 single run 17.2 -> 13.1 ms), and at chi = 32 with one quad per
    // workgroup on a full device too (C2 scan 18.9 -> 18.4 ms); chi = 16 full devices keep the 16-column strips.
    // P->qpw is then set to the quads per workgroup launch_quad instantiates for (CHI, qcg), so that the trunk
    // estimate below and PQD_QPW mean what the kernel runs
    if (P->quad) {
        const int nbq = (int)be.size();
        P->qcg = (nbq <= n_cu || (P->CHI == 32 && P->qpw == 1)) ? 2 : 4;
        if (const char* e = getenv("PQD_QCG")) P->qcg = atoi(e) == 2 ? 2 : (atoi(e) == 1 && P->CHI == 32 ? 1 : 4);
        P->qpw = quad_qpw(P->CHI, P->qpw, P->qcg);
    }
    // trunk pre-pass instead of in-workgroup chains: every slot starts at its own branch step from a checkpoint
    // of its system's MTO-free trunk, which one trajectory per system propagates first. Chosen (PQD_TRUNK=-1,
    // auto) when the estimated critical path — trunk latency + the longest block from its first activation — is
    // shorter than the longest block from step 0; PQD_TRUNK=1 forces it, 0 disables it. Needs fused half steps
    // (checkpoints hold the state with M_b(n-1) deferred).
    std::vector<int> ca(bt.size(), 0);                 // per slot: activation with a checkpoint (0 = fresh)
    std::vector<std::vector<int>> ck_steps(n_sys);     // per system: checkpoint steps (sorted, unique)
    int trunk_mode = -1;
    if (const char* e = getenv("PQD_TRUNK")) trunk_mode = atoi(e);
    bool use_trunk = false;
    if (branch_on && fuse_on && trunk_mode != 0 && ns > 0) {
        // estimated main-sweep time in steps of one block: the longest block (critical path) or, with more blocks than
        // the device holds at once, the total block-steps over the resident blocks, whichever is larger. Without the
        // pre-pass a block spans [0, end] (its chain's first slot carries the trunk from step 0, dormant slots cost a
        // lock-step block the same), with it [first activation, end]
        int64_t crit_no = 0, crit_tk = 0, max_ck = 0, sum_no = 0, sum_tk = 0;
        const int nbk = (int)be.size();
        for (int b = 0; b < nbk; ++b) {
            int start = INT_MAX;
            for (int q = 0; q < BT; ++q) {
                const int t = bt[(size_t)b * BT + q];
                if (t < 0) continue;
                const int a = std::max(0, std::min(jv[t], tr->out_begin[t]));
                ca[(size_t)b * BT + q] = a;
                start = std::min(start, a);
                if (a >= 1) { ck_steps[tsys[t]].push_back(a); max_ck = std::max<int64_t>(max_ck, a); }
            }
            crit_no = std::max<int64_t>(crit_no, be[b]);
            sum_no += be[b];
            if (start != INT_MAX) {
                crit_tk = std::max<int64_t>(crit_tk, be[b] - start);
                sum_tk += be[b] - start;
            }
        }
        // blocks resident at once: quads (one workgroup of qpw quads per CU) or BT-workgroups as the LDS allows
        int64_t conc = n_cu;
        if (P->quad) {
            conc = (int64_t)n_cu * (P->CHI == 32 ? 2 : P->qpw);  // chi = 32: two quads per CU either way
        } else {
            const int64_t lds = ((int64_t)BT * (N2 * (P->CHI + 1) + 4) + (int64_t)BT * N2) * 16;
            conc = (int64_t)n_cu * std::max<int64_t>(1, std::min<int64_t>(4, (160 * 1024) / std::max<int64_t>(1, lds)));
        }
        const double t_no = std::max((double)crit_no, (double)sum_no / (double)conc);
        const double t_tk = std::max((double)crit_tk, (double)sum_tk / (double)conc);
        // trunk step latency relative to a lock-step main-sweep step: split groups (N2 >= 9) ~0.5, one batched
        // workgroup ~0.7
        const double r = N2 >= 9 ? 0.5 : 0.7;
        use_trunk = max_ck > 0 && (trunk_mode == 1 || t_tk + r * (double)max_ck < 0.995 * t_no);
    }
    if (use_trunk) {
        std::vector<int> ck_base(n_sys, 0);
        int n_ck = 0;
        for (int y = 0; y < n_sys; ++y) {
            auto& v = ck_steps[y];
            std::sort(v.begin(), v.end());
            v.erase(std::unique(v.begin(), v.end()), v.end());
            ck_base[y] = n_ck;
            n_ck += (int)v.size();
        }
        for (size_t i = 0; i < bt.size(); ++i) {
            const int t = bt[i];
            if (t < 0) continue;
            const int a = ca[i];
            if (a >= 1) {
                const auto& v = ck_steps[tsys[t]];
                const int idx = ck_base[tsys[t]] + (int)(std::lower_bound(v.begin(), v.end(), a) - v.begin());
                ba[i] = a;
                bsrc[i] = -2 - idx;
            } else {
                ba[i] = 0;
                bsrc[i] = -1;
            }
        }
        if ((rc = plan_trunks(P, ctx, n_sys, ck_steps, ck_base, n_ck, n_cu, N2, n_out, pt, s))) return rc;
    }
    for (size_t i = 0; i < bt.size(); ++i)
        if (bt[i] >= 0) P->traj_steps += tr->out_end[bt[i]] - ba[i] + 1;
    const int nb = (int)be.size();
    if (bt.empty()) { bt.assign(BT, -1); be.assign(1, 0); bs.assign(1, 0); ba.assign(BT, INT_MAX); bsrc.assign(BT, -1); }
    P->n_blocks = nb;
    HIPCHK(P->blk_traj.upload(bt.data(), bt.size(), s));
    HIPCHK(P->blk_end.upload(be.data(), be.size(), s));
    HIPCHK(P->blk_sys.upload(bs.data(), bs.size(), s));
    HIPCHK(P->blk_act.upload(ba.data(), ba.size(), s));
    HIPCHK(P->blk_src.upload(bsrc.data(), bsrc.size(), s));
    HIPCHK(P->sched.upload(sch.data(), sch.size(), s));
    HIPCHK(P->out.alloc(std::max<int64_t>(1, out_len)));
    HIPCHK(hipMemsetAsync(P->out.p, 0, std::max<int64_t>(1, out_len) * sizeof(double2), s));

    P->fp.systems = P->systab.p; P->fp.n_sys = n_sys;
    if (const char* ie = getenv("PQD_IDLE"); !(ie && atoi(ie) == 0)) {  // PQD_IDLE=0: compute every half step (A/B)
        HIPCHK(P->Midle.alloc((size_t)n_sys * m2));
        P->fp.Midle = P->Midle.p;
        // pulse windows: half steps outside a system's [first, last] non-idle half step are neither stored nor
        // re-read (kernels take Midle / Fidle / Widle there). PQD_WIN=0 stores every half step, 2 always uses the
        // windows, 1 (default) uses them when they leave out at least a tenth of the half steps
        // Windows only where every kernel of the plan reads through them: the quad and no-PT kernels without a
        // trunk pre-pass (the batched sweep reads every half step as stored; the split path may fall back to it).
        const bool win_ok = (P->nopt || P->quad) && P->n_trunk == 0;
        if (const char* we = getenv("PQD_WIN"); win_ok && !(we && atoi(we) == 0)) {
            HIPCHK(P->win.alloc((size_t)n_sys));
            P->fp.win = P->win.p;
            P->win_mode = we ? atoi(we) : 1;
        }
    }
    P->fp.ta = grid->ta; P->fp.dt = grid->dt; P->fp.n_steps = ns; P->fp.n_sub = grid->n_sub; P->fp.M = P->M.p;
    if (P->win.p && P->win_mode == 1 && ns > 0) {
        HIPCHK(launch_free_win(P->fp, s));
        std::vector<int2> wh(n_sys);
        HIPCHK(hipMemcpyAsync(wh.data(), P->win.p, sizeof(int2) * n_sys, hipMemcpyDeviceToHost, s));
        HIPCHK(hipStreamSynchronize(s));
        int64_t stored = 0;
        for (const int2& w : wh) stored += w.y >= w.x ? (int64_t)(w.y - w.x + 1) : 0;
        if (10 * stored > 9 * (int64_t)n_sys * 2 * ns) {  // windows leave out < 10%: store every half step
            P->win.release();
            P->fp.win = nullptr;
        }
    }

    SweepParams& sp = P->sp;
    sp.M = P->M.p;
    if (pt) {
        sp.Q = pt->Q.p; sp.Qsum = pt->Qsum.p; sp.D = pt->D; sp.closure = pt->closure.p; sp.closure0 = pt->closure0.p;
        sp.bond0 = pt->bond0.p; sp.gmap = pt->gmap.p;
    }
    sp.sched = P->sched.p; sp.rho0 = P->rho0.p; sp.n_out = n_out; sp.ovec = P->ovec.p;
    sp.blk_traj = P->blk_traj.p; sp.blk_end = P->blk_end.p; sp.blk_sys = P->blk_sys.p;
    sp.blk_act = P->blk_act.p; sp.blk_src = P->blk_src.p;
    sp.traj_sys = P->traj_sys.p; sp.m_stride = (long long)2 * ns * m2; sp.wbeg = P->wbeg.p; sp.wend = P->wend.p;
    { const char* ab = getenv("PQD_ABLATE"); sp.ablate = ab ? atoi(ab) : 0; }
    // exchange form: counter (default; with the XCD-grouped grid C3 runs 5.02 us per step against 5.33 for the granules,
    // profiles/r04/split/xcd/) or data-tagged granules (PQD_SPLIT_GRAN=1)
    { const char* b1 = getenv("PQD_SPLIT_GRAN"); sp.split_gran = (b1 && atoi(b1) == 1) ? 1 : 0; }
    sp.split_ow = split_ow_env() ? 1 : 0;  // the output workgroup (pt_split.hip OWG); split_group_size agrees
    { const char* b2 = getenv("PQD_SPLIT_XCD"); sp.split_xcd = (b2 && atoi(b2) == 0) ? 0 : 1; }
    { const char* b3 = getenv("PQD_SPLIT_L2"); sp.split_l2 = (b3 && atoi(b3) == 0) ? 0 : 1; }
    // polls of a split group's counter before the wait counts as a timeout (~0.1 s); PQD_SPLIT_SPIN overrides
    // it (tests provoke the batched fallback with 0)
    { const char* sl = getenv("PQD_SPLIT_SPIN"); sp.spin_limit = sl ? (unsigned)strtoul(sl, nullptr, 10) : (1u << 22); }
    { const char* f4 = getenv("PQD_FP4"); P->fp.packed4 = (f4 && atoi(f4) == 0) ? 0 : 1; }
    { const char* fm = getenv("PQD_FPM"); P->fp.mfma = fm ? atoi(fm) : 1; }
    HIPCHK(P->flags.alloc(4));
    HIPCHK(hipMemsetAsync(P->flags.p, 0, 4 * sizeof(unsigned), s));
    sp.flags = P->flags.p;
    // PT rows: 3M on the matrix cores; at BT = 4 (N2 > 16, chi = 128) with two k-steps of the slice in flight
    // (six-level scan c5: 84.7 -> 79.5 ms per launch, profiles/r03/exp_c/c5_ptmode.log)
    { const char* pm = getenv("PQD_PT_MODE"); sp.pt_mode = pm ? atoi(pm) : (P->BT == 4 ? 5 : 4); }
    { const char* c3 = getenv("PQD_CMUL3"); sp.cmul3 = c3 ? atoi(c3) : 1; }
    { const char* tp = getenv("PQD_TRPRE"); sp.trpre = tp ? atoi(tp) : 1; }
    { const char* cb = getenv("PQD_COLBIG"); sp.colbig = cb ? atoi(cb) : 1; }
    if (pt && (sp.pt_mode == 4 || sp.pt_mode == 5)) {
        const int nw = P->BT * sweep_wpt(P->N2, P->BT, P->CHI);
        int rmax = sweep_rmax(P->N2, P->BT, P->CHI);
        if (const char* e = getenv("PQD_ROWPAIR")) rmax = std::max(1, std::min(rmax, atoi(e) ? rmax : 1));
        std::vector<int4> u = pt_row_units(pt->gmap_h, nw, rmax);
        HIPCHK(P->units.upload(u.data(), u.size(), s));
        sp.units = P->units.p;
        sp.umax = (int)(u.size() / nw);
    }
    { const char* fz = getenv("PQD_FUSE"); sp.fuse = (!P->nopt && ns > 0 && (fz ? atoi(fz) : 1)) ? 1 : 0; }
    if (!sp.fuse) sp.trpre = 0;  // the prefetched rows are W(n), which exists only with fused half steps
    if (sp.fuse) {
        HIPCHK(P->F.alloc((size_t)n_sys * ns * m2));
        HIPCHK(P->W.alloc((size_t)n_sys * (ns + 1) * n_out * N2));
        P->fu = FuseParams{P->M.p, P->F.p, P->W.p, P->ovec.p, n_sys, ns, n_out};
        P->fu.mfma = P->fp.mfma;
        if (P->win.p) {
            HIPCHK(P->Fidle.alloc((size_t)n_sys * m2));
            HIPCHK(P->Widle.alloc((size_t)n_sys * n_out * N2));
            P->fu.win = P->win.p; P->fu.Midle = P->Midle.p; P->fu.Fidle = P->Fidle.p; P->fu.Widle = P->Widle.p;
        }
        sp.f_stride = (long long)ns * m2;
        sp.w_stride = (long long)(ns + 1) * n_out * N2;
    }
    sp.F = P->F.p; sp.W = P->W.p;
    sp.win = P->win.p; sp.Midle = P->Midle.p; sp.Fidle = P->Fidle.p; sp.Widle = P->Widle.p;
    sp.woff = P->woff.p; sp.ev_start = P->ev_start.p; sp.ev = P->ev.p; sp.sop = P->sop.p; sp.out = P->out.p;
    sp.n_steps = ns;
    sp.n_blk = nb;
    // quad kernel: waves raise their priority outside the PT contraction, so a wave on its serial chain (column
    // operator, exchange, relayout) issues ahead of the other quad's MFMA stream on the same SIMD (C2: 17.5 -> 16.1 ms;
    // a static bias between the grid halves gains nothing; profiles/r03/quad_prio.log)
    sp.qprio = 2;
    if (const char* e = getenv("PQD_QPRIO")) sp.qprio = atoi(e) & 3;
    finalize_trunks(P);
    if (P->split) {
        HIPCHK(P->Xs.alloc((size_t)P->n_traj * 4 * N2 * P->CHI));  // split exchange: 2 slots of granules
        HIPCHK(P->cnt.alloc((size_t)P->n_traj * 64));  // split arrival flags: two 128-B lines per group
        HIPCHK(P->err.alloc(4));
    }
    if (P->msplit) {
        // groups: consecutive trajectories of the block order (system, longest first), TB per group
        std::vector<int> gt((size_t)ms_groups * ms_TB, -1), ge(ms_groups, 0);
        for (int k = 0; k < tr->n_traj; ++k) {
            const int gi = k / ms_TB, t = order[k];
            gt[(size_t)gi * ms_TB + k % ms_TB] = t;
            ge[gi] = std::max(ge[gi], tr->out_end[t]);
        }
        // composite MTO events: one per (trajectory, step) with MTOs, the before / after superoperators of that step
        std::vector<int4> ce;
        std::vector<int> cs(tr->n_traj + 1, 0);
        for (int t = 0; t < tr->n_traj; ++t) {
            cs[t] = (int)ce.size();
            for (int i = ev_start[t]; i < ev_start[t + 1]; ++i) {
                const int4 v = evs[i];
                if (ce.size() > (size_t)cs[t] && ce.back().x == v.x) {
                    if (v.y == 0) ce.back().y = v.z; else ce.back().z = v.z;
                } else {
                    ce.push_back(make_int4(v.x, v.y == 0 ? v.z : -1, v.y == 0 ? -1 : v.z, tsys[t]));
                }
            }
        }
        cs[tr->n_traj] = (int)ce.size();
        P->n_cev = (int)ce.size();
        if (ce.empty()) ce.push_back(make_int4(INT_MAX, -1, -1, 0));
        HIPCHK(P->ms_gtraj.upload(gt.data(), gt.size(), s));
        HIPCHK(P->ms_gend.upload(ge.data(), ge.size(), s));
        HIPCHK(P->cev.upload(ce.data(), ce.size(), s));
        HIPCHK(P->cev_start.upload(cs.data(), cs.size(), s));
        HIPCHK(P->Fev.alloc((size_t)std::max(1, P->n_cev) * m2));
        HIPCHK(P->Wev.alloc((size_t)std::max(1, P->n_cev) * n_out * N2));
        HIPCHK(P->msX.alloc((size_t)ms_groups * ms_TB * 2 * N2 * P->CHI));
        HIPCHK(P->ms_cnt.alloc((size_t)ms_groups * 64));
        HIPCHK(P->err.alloc(4));
        // L2-kept exchange lines on the XCD-grouped grid (PQD_MS_L2=0: sc1 stores, as on the plain grid)
        const int l2keep = ms_xcd > 0 && [] { const char* f = getenv("PQD_MS_L2"); return f ? atoi(f) != 0 : true; }();
        // PT contraction on the matrix cores from 3 trajectories per group (a row block of 4 rows per MFMA; below
        // that the VALU path's per-trajectory work is smaller); PQD_MS_PTM=0/1 forces the VALU / matrix-core path
        int ptm = ms_TB >= 3 && P->CHI <= 64;
        if (const char* f = getenv("PQD_MS_PTM")) ptm = atoi(f) != 0;
        P->mq = MsplitParams{P->ms_gtraj.p, P->ms_gend.p, P->cev_start.p, P->cev.p, P->Fev.p, P->Wev.p,
                             ms_TB, ms_groups, ms_xcd, l2keep, ptm};
    }
    HIPCHK(hipStreamSynchronize(s));
    *out = guard.release();
    return PQD_OK;
}

int pqd_plan_create(pqd_ctx* ctx, const pqd_system* sys, const pqd_grid* grid, const pqd_pt* pt,
                    const int32_t* sched, const pqd_c128* rho0, int32_t n_out, const pqd_c128* out_ops,
                    const pqd_traj* tr, int64_t out_len, pqd_plan** out) {
    return pqd_plan_create_multi(ctx, 1, sys, nullptr, grid, pt, sched, rho0, n_out, out_ops, tr, out_len, out);
}

int pqd_plan_execute(pqd_plan* P, int32_t rebuild_free) {
    if (!P) return fail(PQD_ERR_ARG, "plan is NULL");
    HIPCHK(hipSetDevice(P->ctx->device));
    hipStream_t s = P->ctx->stream;
    if (!P->ring_ready) {
        for (auto& e : P->ring) HIPCHK(hipEventCreate(&e));
        P->ring_ready = true;
    }
    hipEvent_t* e = P->ring + 3 * P->ev_head;
    HIPCHK(hipEventRecord(e[0], s));
    if (rebuild_free && P->n_steps > 0) {
        HIPCHK(launch_free_prop(P->N2, P->fp, s));
        if (P->sp.fuse) HIPCHK(launch_fuse_steps(P->N2, P->fu, s));
        if (P->msplit) HIPCHK(launch_evcomp(P->N2, P->sp, P->mq, P->n_cev, P->n_steps, s));
    }
    HIPCHK(hipEventRecord(e[1], s));
    HIPCHK(launch_trunks(P, s));
    if (P->nopt)
        HIPCHK(launch_sweep_nopt(P->N2, P->n_traj, P->sp, s));
    else if (P->split)
        HIPCHK(launch_split(P->N2, P->CHI, P->n_traj, P->sp, P->Xs.p, P->cnt.p, P->err.p, s, P->split_chunk));
    else if (P->msplit)
        HIPCHK(launch_msplit(P->N2, P->CHI, P->sp, P->mq, P->msX.p, P->ms_cnt.p, P->err.p, s));
    else
        HIPCHK(launch_main(P, s));
    HIPCHK(hipEventRecord(e[2], s));
    P->ev_head = (P->ev_head + 1) % pqd_plan::RING;
    P->ev_count++;
    P->execs++;
    return PQD_OK;
}

void* pqd_plan_output_device(pqd_plan* P) { return P ? (void*)P->out.p : nullptr; }

// Wait for the plan's last execute and check it. A split launch whose groups could not all be resident (the device
// is shared with other work, so a peer workgroup never arrived) ends with its error word set: the plan then re-runs
// the same step range on the batched kernel, which needs no co-residency, and stays on it. A non-finite output
// value raises PQD_ERR_NUMERIC.
int pqd_plan_synchronize(pqd_plan* P) {
    if (!P) return fail(PQD_ERR_ARG, "plan is NULL");
    HIPCHK(hipSetDevice(P->ctx->device));
    hipStream_t s = P->ctx->stream;
    HIPCHK(hipMemsetAsync(P->flags.p, 0, sizeof(unsigned), s));
    if (P->n_trunk && P->tk_split) {
        unsigned err = 0;
        HIPCHK(hipMemcpyAsync(&err, P->tk_err.p, sizeof(unsigned), hipMemcpyDeviceToHost, s));
        HIPCHK(hipStreamSynchronize(s));
        if (err) {  // the checkpoints are incomplete: redo the trunks on batched workgroups, then the main sweep
            P->tk_split = false;
            P->split_fallbacks++;
            HIPCHK(hipMemsetAsync(P->tk_err.p, 0, sizeof(unsigned), s));
            HIPCHK(launch_trunks(P, s));
            HIPCHK(launch_main(P, s));
        }
    }
    if (P->split || P->msplit) {
        unsigned err[2] = {0, 0};
        HIPCHK(hipMemcpyAsync(err, P->err.p, 2 * sizeof(unsigned), hipMemcpyDeviceToHost, s));
        HIPCHK(hipStreamSynchronize(s));
        if (err[0] && err[1] && P->msplit && P->mq.l2keep) {
            // a group's workgroups were not all on one XCD (pt_msplit.hip l2keep): again with sc1 exchange stores,
            // which need no placement, and stay there
            P->mq.l2keep = 0;
            P->split_fallbacks++;
            HIPCHK(launch_msplit(P->N2, P->CHI, P->sp, P->mq, P->msX.p, P->ms_cnt.p, P->err.p, s));
            HIPCHK(hipMemcpyAsync(err, P->err.p, sizeof(unsigned), hipMemcpyDeviceToHost, s));
            HIPCHK(hipStreamSynchronize(s));
        }
        if (err[0] && P->msplit && P->CHI > 128)
            return fail(PQD_ERR_HIP, "multi-trajectory split groups timed out at chi %d (no batched fallback holds that "
                        "bond); the device is shared or the groups could not all be resident", P->CHI);
        if (err[0]) {
            P->split = false;
            P->msplit = false;
            P->split_fallbacks++;
            HIPCHK(hipMemsetAsync(P->err.p, 0, sizeof(unsigned), s));
            HIPCHK(launch_main(P, s));
        }
    }
    unsigned flags = 0;
    HIPCHK(launch_check_finite(P->out.p, P->out_len, P->flags.p, s));
    HIPCHK(hipMemcpyAsync(&flags, P->flags.p, sizeof(unsigned), hipMemcpyDeviceToHost, s));
    HIPCHK(hipStreamSynchronize(s));
    if (flags & 1u) return fail(PQD_ERR_NUMERIC, "non-finite value (NaN/Inf) in the propagated outputs");
    return PQD_OK;
}

int pqd_plan_download(pqd_plan* P, pqd_c128* out, int64_t out_len) {
    if (!P || !out) return fail(PQD_ERR_ARG, "NULL argument");
    if (out_len < P->out_len) return fail(PQD_ERR_ARG, "out_len %lld < plan out_len %lld", (long long)out_len, (long long)P->out_len);
    int rc = pqd_plan_synchronize(P);
    if (rc && rc != PQD_ERR_NUMERIC) return rc;
    if (P->out_len > 0) {
        HIPCHK(hipMemcpyAsync(out, P->out.p, P->out_len * sizeof(double2), hipMemcpyDeviceToHost, P->ctx->stream));
        HIPCHK(hipStreamSynchronize(P->ctx->stream));
    }
    return rc;  // PQD_ERR_NUMERIC still hands the values over (they show where the run went bad)
}

int pqd_plan_table_len(const pqd_plan* P, int64_t* table_len) {
    if (!P || !table_len) return fail(PQD_ERR_ARG, "NULL argument");
    *table_len = P->toff.empty() ? 0 : P->toff.back();
    return PQD_OK;
}

int pqd_plan_download_table(pqd_plan* P, pqd_c128* table, int64_t table_len) {
    if (!P || !table) return fail(PQD_ERR_ARG, "NULL argument");
    const long long need = P->toff.empty() ? 0 : P->toff.back();
    if (table_len < need) return fail(PQD_ERR_ARG, "table_len %lld < %lld", (long long)table_len, need);
    int rc = pqd_plan_synchronize(P);
    if (rc && rc != PQD_ERR_NUMERIC) return rc;
    if (need > 0) {
        hipStream_t s = P->ctx->stream;
        if (!P->toff_d.p) HIPCHK(P->toff_d.upload(P->toff.data(), P->toff.size(), s));
        if (!P->table.p) HIPCHK(P->table.alloc((size_t)need));
        HIPCHK(launch_table(P->out.p, P->woff.p, P->wbeg.p, P->wend.p, P->toff_d.p, P->n_traj, P->n_out, P->t_start,
                            P->dt, P->table.p, s));
        HIPCHK(hipMemcpyAsync(table, P->table.p, (size_t)need * sizeof(double2), hipMemcpyDeviceToHost, s));
        HIPCHK(hipStreamSynchronize(s));
    }
    return rc;
}

int pqd_plan_trapz(pqd_plan* P, int32_t n_pairs, const int32_t* k_head, const int32_t* k_tail, double dx,
                   pqd_c128* res) {
    if (!P || (n_pairs > 0 && (!k_head || !k_tail || !res))) return fail(PQD_ERR_ARG, "NULL argument");
    if (n_pairs < 0) return fail(PQD_ERR_ARG, "n_pairs %d < 0", n_pairs);
    for (int q = 0; q < n_pairs; ++q)
        if (k_head[q] < 0 || k_head[q] >= P->n_out || k_tail[q] < 0 || k_tail[q] >= P->n_out)
            return fail(PQD_ERR_ARG, "pair %d: output (%d, %d) not in [0, %d)", q, k_head[q], k_tail[q], P->n_out);
    int rc = pqd_plan_synchronize(P);
    if (rc && rc != PQD_ERR_NUMERIC) return rc;
    const size_t n = (size_t)P->n_traj * n_pairs;
    if (n == 0) return rc;
    hipStream_t s = P->ctx->stream;
    DevBuf<int> kd;
    DevBuf<double2> rd;
    std::vector<int> k(2 * (size_t)n_pairs);
    for (int q = 0; q < n_pairs; ++q) { k[q] = k_head[q]; k[n_pairs + q] = k_tail[q]; }
    HIPCHK(kd.upload(k.data(), k.size(), s));
    HIPCHK(rd.alloc(n));
    HIPCHK(launch_trapz(P->out.p, P->woff.p, P->wbeg.p, P->wend.p, P->n_traj, P->n_out, n_pairs, kd.p, kd.p + n_pairs,
                        dx, rd.p, s));
    HIPCHK(hipMemcpyAsync(res, rd.p, n * sizeof(double2), hipMemcpyDeviceToHost, s));
    HIPCHK(hipStreamSynchronize(s));
    return rc;
}

int pqd_propagate_trapz(pqd_ctx* ctx, int32_t n_sys, const pqd_system* systems, const int32_t* traj_sys,
                        const pqd_grid* grid, const pqd_pt* pt, const int32_t* sched, const pqd_c128* rho0,
                        int32_t n_out, const pqd_c128* out_ops, const pqd_traj* tr, int32_t n_pairs,
                        const int32_t* k_head, const int32_t* k_tail, double dx, pqd_c128* res) {
    if (!tr) return fail(PQD_ERR_ARG, "NULL argument");
    int64_t out_len = 0;
    for (int t = 0; t < tr->n_traj; ++t)
        out_len = std::max<int64_t>(out_len, tr->out_offset[t] + (int64_t)(tr->out_end[t] - tr->out_begin[t] + 1) * n_out);
    pqd_plan* P = nullptr;
    int rc = pqd_plan_create_multi(ctx, n_sys, systems, traj_sys, grid, pt, sched, rho0, n_out, out_ops, tr,
                                   std::max<int64_t>(1, out_len), &P);
    if (rc) return rc;
    rc = pqd_plan_execute(P, 1);
    if (!rc) rc = pqd_plan_trapz(P, n_pairs, k_head, k_tail, dx, res);
    pqd_plan_destroy(P);
    return rc;
}

int pqd_plan_copy_output(pqd_plan* P, void* dst, int64_t out_len) {
    if (!P || !dst) return fail(PQD_ERR_ARG, "NULL argument");
    if (out_len < P->out_len) return fail(PQD_ERR_ARG, "out_len %lld < plan out_len %lld", (long long)out_len, (long long)P->out_len);
    int rc = pqd_plan_synchronize(P);
    if (rc && rc != PQD_ERR_NUMERIC) return rc;
    if (P->out_len > 0) {
        HIPCHK(hipMemcpyAsync(dst, P->out.p, P->out_len * sizeof(double2), hipMemcpyDefault, P->ctx->stream));
        HIPCHK(hipStreamSynchronize(P->ctx->stream));
    }
    return rc;
}

int pqd_plan_windows(const pqd_plan* P, int32_t* on) {
    if (!P || !on) return fail(PQD_ERR_ARG, "NULL argument");
    *on = P->win.p ? 1 : 0;
    return PQD_OK;
}

int pqd_plan_info(const pqd_plan* P, int32_t* path, int32_t* bt, int32_t* split_fallbacks, int64_t* traj_steps) {
    if (!P) return fail(PQD_ERR_ARG, "plan is NULL");
    if (traj_steps) *traj_steps = P->traj_steps;
    if (path)
        *path = P->nopt ? PQD_PATH_NOPT : P->split ? PQD_PATH_SPLIT : P->msplit ? PQD_PATH_MSPLIT
              : P->quad ? PQD_PATH_QUAD : PQD_PATH_BATCHED;
    if (bt) *bt = P->msplit ? P->mq.TB : P->BT;
    if (split_fallbacks) *split_fallbacks = P->split_fallbacks;
    return PQD_OK;
}

int pqd_plan_timing(pqd_plan* P, double* ms_free, double* ms_sweep, int32_t* n, int32_t reset) {
    if (!P) return fail(PQD_ERR_ARG, "plan is NULL");
    HIPCHK(hipSetDevice(P->ctx->device));
    double f = 0, w = 0;
    const int k = std::min(P->ev_count, pqd_plan::RING);  // the most recent k executes
    for (int i = 0; i < k; ++i) {
        const int slot = ((P->ev_head - 1 - i) % pqd_plan::RING + pqd_plan::RING) % pqd_plan::RING;
        hipEvent_t* e = P->ring + 3 * slot;
        float a = 0, b = 0;
        HIPCHK(hipEventSynchronize(e[2]));
        HIPCHK(hipEventElapsedTime(&a, e[0], e[1]));
        HIPCHK(hipEventElapsedTime(&b, e[1], e[2]));
        f += a; w += b;
    }
    if (ms_free) *ms_free = k ? f / k : 0.0;
    if (ms_sweep) *ms_sweep = k ? w / k : 0.0;
    if (n) *n = k;
    if (reset) P->ev_count = 0;
    return PQD_OK;
}

void pqd_plan_destroy(pqd_plan* P) {
    if (!P) return;
    (void)hipSetDevice(P->ctx->device);
    (void)hipStreamSynchronize(P->ctx->stream);
    delete P;
}

int pqd_propagate(pqd_ctx* ctx, const pqd_system* sys, const pqd_grid* grid, const pqd_pt* pt,
                  const int32_t* sched, const pqd_c128* rho0, int32_t n_out, const pqd_c128* out_ops,
                  const pqd_traj* tr, pqd_c128* out, int64_t out_len) {
    return pqd_propagate_multi(ctx, 1, sys, nullptr, grid, pt, sched, rho0, n_out, out_ops, tr, out, out_len);
}

int pqd_propagate_multi(pqd_ctx* ctx, int32_t n_sys, const pqd_system* systems, const int32_t* traj_sys,
                        const pqd_grid* grid, const pqd_pt* pt, const int32_t* sched, const pqd_c128* rho0,
                        int32_t n_out, const pqd_c128* out_ops, const pqd_traj* tr, pqd_c128* out,
                        int64_t out_len) {
    pqd_plan* P = nullptr;
    int rc = pqd_plan_create_multi(ctx, n_sys, systems, traj_sys, grid, pt, sched, rho0, n_out, out_ops, tr, out_len, &P);
    if (rc) return rc;
    rc = pqd_plan_execute(P, 1);
    if (!rc) rc = pqd_plan_download(P, out, out_len);
    pqd_plan_destroy(P);
    return rc;
}

int pqd_propagate_table(pqd_ctx* ctx, int32_t n_sys, const pqd_system* systems, const int32_t* traj_sys,
                        const pqd_grid* grid, const pqd_pt* pt, const int32_t* sched, const pqd_c128* rho0,
                        int32_t n_out, const pqd_c128* out_ops, const pqd_traj* tr, pqd_c128* table,
                        int64_t table_len) {
    if (!tr) return fail(PQD_ERR_ARG, "NULL argument");
    int64_t out_len = 0;
    for (int t = 0; t < tr->n_traj; ++t)
        out_len = std::max<int64_t>(out_len, tr->out_offset[t] + (int64_t)(tr->out_end[t] - tr->out_begin[t] + 1) * n_out);
    pqd_plan* P = nullptr;
    int rc = pqd_plan_create_multi(ctx, n_sys, systems, traj_sys, grid, pt, sched, rho0, n_out, out_ops, tr,
                                   std::max<int64_t>(1, out_len), &P);
    if (rc) return rc;
    rc = pqd_plan_execute(P, 1);
    if (!rc) rc = pqd_plan_download_table(P, table, table_len);
    pqd_plan_destroy(P);
    return rc;
}

int pqd_fail_msg(int code, const char* msg) { return fail(code, "%s", msg); }

// =================================================================================================
// map-chain sweeps
// =================================================================================================
static int mapchain_run(pqd_ctx* ctx, MapChainParams& p, const pqd_c128* dmA, size_t nA, const pqd_c128* dmB,
                        size_t nB, const pqd_c128* dmT, size_t nT, const pqd_c128* dm_s, const pqd_c128* rho_init,
                        const pqd_c128* opA, const pqd_c128* opB, const pqd_c128* opC, const double* time,
                        const double* time_sparse, pqd_c128* result) {
    if (!ctx || !rho_init || !opA || !opB || !opC || !time || !time_sparse || !result || !dmA)
        return fail(PQD_ERR_ARG, "NULL argument");
    if (p.dim < 2 || p.dim > 6) return fail(PQD_ERR_UNSUPPORTED, "dim %d not in [2, 6]", p.dim);
    if (p.n_t < 1 || p.n_tfull < 1 || p.n_tau < 0) return fail(PQD_ERR_ARG, "bad sizes");
    HIPCHK(hipSetDevice(ctx->device));
    hipStream_t s = ctx->stream;
    const int N2 = p.dim * p.dim;
    p.N2 = N2;
    const size_t m2 = (size_t)N2 * N2;
    const size_t nres = (size_t)p.n_t * (p.n_tau + 1);
    // calc_onetime_parallel on the blocked sweep (mapchain.hip): the trunk ends j_i are found here with the
    // Fortran's own comparisons (propagate_tau.f90:144-151), which also bounds every map the sweep reads
    const char* eb = getenv("PQD_MC_BLOCKED");
    bool blocked = (p.mode == 0 || p.mode == 1) && !(eb && atoi(eb) == 0) &&
                   (N2 == 4 || N2 == 9 || N2 == 16 || N2 == 25 || N2 == 36);
    std::vector<int> pos;
    int pmax = 0;
    if (blocked) {
        pos.resize(p.n_t);
        int j = 1;
        for (int i = 0; i < p.n_t; ++i) {
            while (j <= p.n_tfull && time[j - 1] < time_sparse[i]) ++j;
            pos[i] = j - 1;
            pmax = std::max(pmax, j - 1);
        }
        if (p.mode == 1) {
            // a trunk that ends past the first period (j > n_tb) never wraps in the tau loop (:270-287: jj resets
            // only when it equals n_tb + 1), so that trajectory applies dm_s at every tau step: it starts at q_s, the
            // first position of a constant dm_s region placed after the periodic positions (map_at)
            int qp = 0;
            bool any_s = false;
            for (int i = 0; i < p.n_t; ++i) {
                if (pos[i] + 1 <= p.n_tb) qp = std::max(qp, pos[i] + p.n_tau);
                else any_s = true;
            }
            p.q_s = any_s ? qp : INT_MAX;
            for (int i = 0; i < p.n_t; ++i)
                if (pos[i] + 1 > p.n_tb) pos[i] = p.q_s;
            // precondition of that constant region: with n_map > n_tb a trunk ending at n_tb < j <= n_map walks
            // dm_block(j), dm_block(j+1), ..., dm_block(n_map) before dm_s (:270-281), which the blocked position
            // map does not represent; such calls run on the map-by-map kernels
            if (any_s && p.n_map > p.n_tb) blocked = false;
        }
    }
    if (blocked) {
        if (p.mode == 0 && (size_t)std::max(Q_of(pos, p.n_tau), pmax) > nA)
            return fail(PQD_ERR_ARG, "the sweep would read map %d of %zu (time_sparse beyond time, or n_tau too long "
                        "for dm_tl)", std::max(Q_of(pos, p.n_tau), pmax), nA);
        const int Q = Q_of(pos, p.n_tau);
        const char* el = getenv("PQD_MC_L");
        int L = el ? atoi(el) : (int)std::lround(std::sqrt((double)std::max(1, p.n_tau)));
        L = std::max(8, std::min(256, L));
        p.L = L;
        p.Q = std::max(Q, 1);
        p.n_blk = (p.Q + L - 1) / L;
    }
    // every device buffer of the call carved from the context's arena
    auto carve = [&](Carve& c) {
        p.dmA = c.take<double2>(nA * m2);
        p.dmB = dmB ? c.take<double2>(nB * m2) : nullptr;
        p.dmT = dmT ? c.take<double2>(nT * m2) : nullptr;
        p.dm_s = dm_s ? c.take<double2>(m2) : nullptr;
        p.rho_init = c.take<double2>(N2);
        p.opA = c.take<double2>(N2);
        p.opB = c.take<double2>(N2);
        p.opC = c.take<double2>(N2);
        p.time = c.take<double>(p.n_tfull);
        p.time_sparse = c.take<double>(p.n_t);
        p.rho_buf = c.take<double2>((size_t)p.n_t * N2);
        p.j_arr = c.take<int>(p.n_t);
        p.result = c.take<double2>(nres);
        if (blocked) {
            p.pos = c.take<int>(p.n_t);
            p.U = c.take<double2>((size_t)p.Q * N2);
            p.Rend = c.take<double2>((size_t)p.n_blk * m2);
            p.P = c.take<double2>((size_t)(p.n_blk + 1) * N2);
            p.X = c.take<double2>((size_t)p.n_blk * p.n_t * N2);
        }
    };
    Carve sz;
    carve(sz);
    if (ctx->mc_arena.n < sz.off + 256) {
        HIPCHK(hipStreamSynchronize(s));
        HIPCHK(ctx->mc_arena.alloc(sz.off + sz.off / 4 + 256));
    }
    Carve cv;
    cv.base = ctx->mc_arena.p;
    carve(cv);
    auto up = [&](const void* dst, const void* src, size_t bytes) {
        return bytes ? hipMemcpyAsync(const_cast<void*>(dst), src, bytes, hipMemcpyHostToDevice, s) : hipSuccess;
    };
    // PQD_MC_TIMING=1: host-side phase times of this call on stderr (diagnostics)
    const bool tmg = getenv("PQD_MC_TIMING") != nullptr;
    auto now = [] { return std::chrono::steady_clock::now(); };
    const auto t0 = now();
    // the caller's result array is typically fresh (f2py-style: np.zeros, pages not yet mapped): fault its pages in
    // on a few host threads while the maps upload and the kernels run, so the copy back runs at the link rate (a
    // 41 MB copy into fresh pages: 1.7 ms, into mapped ones 0.73 ms; scripts/ubench_h2d.py)
    std::thread toucher;
    try {
        toucher = std::thread(touch_pages, (void*)result, nres * sizeof(double2));
    } catch (...) {  // thread creation failed: skip the pre-touch (the copy back is only slower), never throw
    }
    struct Join {
        std::thread& t;
        ~Join() { if (t.joinable()) t.join(); }
    } join_toucher{toucher};
    HIPCHK(up(p.dmA, dmA, nA * m2 * sizeof(double2)));
    if (dmB) HIPCHK(up(p.dmB, dmB, nB * m2 * sizeof(double2)));
    if (dmT) HIPCHK(up(p.dmT, dmT, nT * m2 * sizeof(double2)));
    if (dm_s) HIPCHK(up(p.dm_s, dm_s, m2 * sizeof(double2)));
    HIPCHK(up(p.rho_init, rho_init, N2 * sizeof(double2)));
    HIPCHK(up(p.opA, opA, N2 * sizeof(double2)));
    HIPCHK(up(p.opB, opB, N2 * sizeof(double2)));
    HIPCHK(up(p.opC, opC, N2 * sizeof(double2)));
    HIPCHK(up(p.time, time, p.n_tfull * sizeof(double)));
    HIPCHK(up(p.time_sparse, time_sparse, p.n_t * sizeof(double)));
    if (blocked) {
        // every result element is written by the blocked kernels (trunk column, partial-block outputs, dots)
        HIPCHK(up(p.pos, pos.data(), p.n_t * sizeof(int)));
        HIPCHK(launch_mapchain_blocked(p, pmax / p.L, s));
    } else {
        HIPCHK(hipMemsetAsync(p.result, 0, nres * sizeof(double2), s));
        HIPCHK(launch_mapchain(p, s));
    }
    const auto t1 = now();
    toucher.join();
    const auto t2 = now();
    if (tmg) HIPCHK(hipStreamSynchronize(s));
    const auto t3 = now();
    HIPCHK(hipMemcpyAsync(result, p.result, nres * sizeof(double2), hipMemcpyDeviceToHost, s));
    HIPCHK(hipStreamSynchronize(s));
    if (tmg) {
        const auto t4 = now();
        auto ms = [](auto a, auto b) { return std::chrono::duration<double, std::milli>(b - a).count(); };
        fprintf(stderr, "pqd mapchain: upload+launch %.3f ms, page touch left %.3f ms, kernels left %.3f ms, download %.3f ms\n",
                ms(t0, t1), ms(t1, t2), ms(t2, t3), ms(t3, t4));
    }
    return PQD_OK;
}

int pqd_calc_onetime_parallel(pqd_ctx* ctx, const pqd_c128* dm_tl, const pqd_c128* rho_init, int32_t n_tau,
                              int32_t n_t, int32_t n_tfull, int32_t dim, const pqd_c128* opA,
                              const pqd_c128* opB, const pqd_c128* opC, const double* time,
                              const double* time_sparse, pqd_c128* result) {
    MapChainParams p{};
    p.mode = 0; p.dim = dim; p.n_t = n_t; p.n_tfull = n_tfull; p.n_tau = n_tau;
    // the tau loop reads maps up to index j_max - 1 + n_tau <= n_tfull - 1 (Fortran bounds)
    return mapchain_run(ctx, p, dm_tl, (size_t)std::max(1, n_tfull - 1), nullptr, 0, nullptr, 0, nullptr, rho_init,
                        opA, opB, opC, time, time_sparse, result);
}

int pqd_calc_onetime_parallel_block(pqd_ctx* ctx, const pqd_c128* dm_block, const pqd_c128* dm_s,
                                    const pqd_c128* rho_init, int32_t n_tb, int32_t nx_tau, int32_t n_map,
                                    int32_t n_t, int32_t n_tfull, int32_t dim, const pqd_c128* opA,
                                    const pqd_c128* opB, const pqd_c128* opC, const double* time,
                                    const double* time_sparse, pqd_c128* result) {
    if (!dm_s) return fail(PQD_ERR_ARG, "dm_s is NULL");
    if (n_map < 1 || n_tb < 1 || nx_tau < 0) return fail(PQD_ERR_ARG, "bad block sizes");
    MapChainParams p{};
    p.mode = 1; p.dim = dim; p.n_t = n_t; p.n_tfull = n_tfull; p.n_tau = n_tb * nx_tau;
    p.n_map = n_map; p.n_tb = n_tb; p.nx_tau = nx_tau;
    return mapchain_run(ctx, p, dm_block, n_map, nullptr, 0, nullptr, 0, dm_s, rho_init, opA, opB, opC, time,
                        time_sparse, result);
}

int pqd_calc_twotime_phonon_block(pqd_ctx* ctx, const pqd_c128* dm_taucs2, const pqd_c128* dm_sep1,
                                  const pqd_c128* dm_sep2, const pqd_c128* dm_s, const pqd_c128* rho_init,
                                  int32_t n_tb, int32_t nx_tau, int32_t n_map, int32_t n_t, int32_t n_tfull,
                                  int32_t n_tauc, int32_t dim, const pqd_c128* opA, const pqd_c128* opB,
                                  const pqd_c128* opC, const double* time, const double* time_sparse,
                                  pqd_c128* result) {
    if (!dm_taucs2 || !dm_sep2 || !dm_s) return fail(PQD_ERR_ARG, "NULL map argument");
    if (n_map < 1 || n_tb < 1 || nx_tau < 0 || n_tauc < 0) return fail(PQD_ERR_ARG, "bad block sizes");
    if (n_tauc > n_t) return fail(PQD_ERR_ARG, "n_tauc %d > n_t %d (reads past rho_buffer in the reference)", n_tauc, n_t);
    MapChainParams p{};
    p.mode = 2; p.dim = dim; p.n_t = n_t; p.n_tfull = n_tfull; p.n_tau = n_tb * nx_tau;
    p.n_map = n_map; p.n_tb = n_tb; p.nx_tau = nx_tau; p.n_tauc = n_tauc;
    return mapchain_run(ctx, p, dm_sep1, n_map, dm_sep2, n_map, dm_taucs2, (size_t)std::max(1, n_tauc) * n_map, dm_s,
                        rho_init, opA, opB, opC, time, time_sparse, result);
}

int pqd_propagate_tau(pqd_ctx* ctx, const pqd_c128* dm_tl, int32_t n_maps, const pqd_c128* rho_init,
                      int32_t n_tau, int32_t dim, int32_t j_start, pqd_c128* rho_out) {
    if (!ctx || !dm_tl || !rho_init || !rho_out) return fail(PQD_ERR_ARG, "NULL argument");
    if (dim < 2 || dim > 6) return fail(PQD_ERR_UNSUPPORTED, "dim %d", dim);
    if (n_tau < 0 || j_start < 0 || j_start + n_tau > n_maps)
        return fail(PQD_ERR_ARG, "maps j_start+1..j_start+n_tau = %d..%d outside 1..%d", j_start + 1, j_start + n_tau, n_maps);
    HIPCHK(hipSetDevice(ctx->device));
    hipStream_t s = ctx->stream;
    const int N2 = dim * dim;
    DevBuf<double2> A, r0, o;
    HIPCHK(A.upload(reinterpret_cast<const double2*>(dm_tl), (size_t)n_maps * N2 * N2, s));
    HIPCHK(r0.upload(reinterpret_cast<const double2*>(rho_init), N2, s));
    HIPCHK(o.alloc((size_t)N2 * (n_tau + 1)));
    HIPCHK(launch_propagate_tau(N2, A.p, r0.p, n_tau, j_start, o.p, s));
    HIPCHK(hipMemcpyAsync(rho_out, o.p, (size_t)N2 * (n_tau + 1) * sizeof(double2), hipMemcpyDeviceToHost, s));
    HIPCHK(hipStreamSynchronize(s));
    return PQD_OK;
}

int pqd_map_tail(pqd_ctx* ctx, const pqd_c128* M, int32_t N2, const pqd_c128* X, int32_t n_x, const pqd_c128* w,
                 int32_t n_steps, pqd_c128* out) {
    if (!ctx || !M || !X || !w || !out) return fail(PQD_ERR_ARG, "NULL argument");
    if (!(N2 == 4 || N2 == 9 || N2 == 16 || N2 == 25 || N2 == 36)) return fail(PQD_ERR_UNSUPPORTED, "N2 %d", N2);
    if (n_x < 0 || n_steps < 0) return fail(PQD_ERR_ARG, "n_x %d n_steps %d", n_x, n_steps);
    if (n_x == 0 || n_steps == 0) return PQD_OK;
    HIPCHK(hipSetDevice(ctx->device));
    hipStream_t s = ctx->stream;
    DevBuf<double2> dM, dX, dw, o;
    HIPCHK(dM.upload(reinterpret_cast<const double2*>(M), (size_t)N2 * N2, s));
    HIPCHK(dX.upload(reinterpret_cast<const double2*>(X), (size_t)n_x * N2, s));
    HIPCHK(dw.upload(reinterpret_cast<const double2*>(w), N2, s));
    HIPCHK(o.alloc((size_t)n_x * n_steps));
    HIPCHK(launch_map_tail(N2, dM.p, dX.p, n_x, dw.p, n_steps, o.p, s));
    HIPCHK(hipMemcpyAsync(out, o.p, (size_t)n_x * n_steps * sizeof(double2), hipMemcpyDeviceToHost, s));
    HIPCHK(hipStreamSynchronize(s));
    return PQD_OK;
}

static int four_time_common(pqd_ctx* ctx, FourTimeParams& p, const pqd_c128* dm_1, const pqd_c128* dm_2,
                            const pqd_c128* rho_init, const double* t1, const pqd_c128* precalc, const pqd_c128* ops,
                            int n_ops, pqd_c128* result, bool dyn, int row_lo = 0, int row_hi = INT_MAX) {
    if (!ctx || !dm_1 || !dm_2 || !rho_init || !t1 || !precalc || !result || (!dyn && !ops))
        return fail(PQD_ERR_ARG, "NULL argument");
    if (p.dim < 2 || p.dim > 6) return fail(PQD_ERR_UNSUPPORTED, "dim %d", p.dim);
    if (p.n_t < 1 || p.n_map < 1 || p.n_precalc < 1 || !(p.dt > 0)) return fail(PQD_ERR_ARG, "bad sizes");
    HIPCHK(hipSetDevice(ctx->device));
    hipStream_t s = ctx->stream;
    const int N2 = p.dim * p.dim;
    p.N2 = N2;
    const size_t m2 = (size_t)N2 * N2;
    DevBuf<double2> d1, d2, pc, r0, op, res;
    DevBuf<double> tt;
    DevBuf<int2> pr;
    HIPCHK(d1.upload(reinterpret_cast<const double2*>(dm_1), p.n_map * m2, s));
    HIPCHK(d2.upload(reinterpret_cast<const double2*>(dm_2), p.n_map * m2, s));
    HIPCHK(pc.upload(reinterpret_cast<const double2*>(precalc), p.n_precalc * m2, s));
    HIPCHK(r0.upload(reinterpret_cast<const double2*>(rho_init), N2, s));
    HIPCHK(tt.upload(t1, p.n_t, s));
    if (!dyn) HIPCHK(op.upload(reinterpret_cast<const double2*>(ops), (size_t)n_ops * N2, s));
    p.dm1 = d1.p; p.dm2 = d2.p; p.precalc = pc.p; p.rho_init = r0.p; p.t1 = tt.p; p.ops = op.p;
    if (dyn) {
        const size_t n = (size_t)N2 * (2 * p.n_t - 1);
        HIPCHK(res.alloc(n));
        HIPCHK(launch_dynamics_t1(p, res.p, s));
        HIPCHK(hipMemcpyAsync(result, res.p, n * sizeof(double2), hipMemcpyDeviceToHost, s));
    } else {
        std::vector<int2> pairs;
        pairs.reserve((size_t)p.n_t * (p.n_t + 1) / 2);
        for (int i = std::max(0, row_lo); i < std::min(p.n_t, row_hi); ++i)
            for (int j = 0; j <= p.n_t - 1 - i; ++j) pairs.push_back(make_int2(i, j));
        HIPCHK(pr.upload(pairs.data(), pairs.size(), s));
        p.pairs = pr.p; p.n_pairs = (int)pairs.size();
        const size_t nres = (size_t)p.n_t * p.n_t;
        HIPCHK(res.alloc(nres + (size_t)p.n_t * N2));  // + prologue scratch
        HIPCHK(hipMemsetAsync(res.p, 0, nres * sizeof(double2), s));
        p.result = res.p;
        HIPCHK(launch_four_time(p, s));
        HIPCHK(hipMemcpyAsync(result, res.p, nres * sizeof(double2), hipMemcpyDeviceToHost, s));
    }
    HIPCHK(hipStreamSynchronize(s));
    return PQD_OK;
}

int pqd_four_time_8op(pqd_ctx* ctx, const pqd_c128* dm_1, const pqd_c128* dm_2, const pqd_c128* rho_init,
                      const double* t1, const pqd_c128* precalc, int32_t n_t, double dt, int32_t n_map,
                      int32_t dim, const pqd_c128* ops8, int32_t early_only, int32_t late_t1_only, double tb,
                      int32_t n_precalc, pqd_c128* result) {
    FourTimeParams p{};
    p.dim = dim; p.n_t = n_t; p.n_map = n_map; p.n_precalc = n_precalc; p.dt = dt; p.tb = tb;
    p.variant = 0; p.early_only = early_only; p.late_t1_only = late_t1_only;
    return four_time_common(ctx, p, dm_1, dm_2, rho_init, t1, precalc, ops8, 8, result, false);
}

int pqd_four_time_8op_rows(pqd_ctx* ctx, const pqd_c128* dm_1, const pqd_c128* dm_2, const pqd_c128* rho_init,
                           const double* t1, const pqd_c128* precalc, int32_t n_t, double dt, int32_t n_map,
                           int32_t dim, const pqd_c128* ops8, int32_t early_only, int32_t late_t1_only, double tb,
                           int32_t n_precalc, int32_t row_lo, int32_t row_hi, pqd_c128* result) {
    if (row_lo < 0 || row_hi < row_lo || row_hi > n_t) return fail(PQD_ERR_ARG, "rows [%d, %d) outside [0, %d)", row_lo, row_hi, n_t);
    FourTimeParams p{};
    p.dim = dim; p.n_t = n_t; p.n_map = n_map; p.n_precalc = n_precalc; p.dt = dt; p.tb = tb;
    p.variant = 0; p.early_only = early_only; p.late_t1_only = late_t1_only;
    return four_time_common(ctx, p, dm_1, dm_2, rho_init, t1, precalc, ops8, 8, result, false, row_lo, row_hi);
}

int pqd_four_time(pqd_ctx* ctx, const pqd_c128* dm_1, const pqd_c128* dm_2, const pqd_c128* rho_init,
                  const double* t1, const pqd_c128* precalc, int32_t n_t, double dt, int32_t n_map, int32_t dim,
                  const pqd_c128* ops4, double tb, int32_t n_precalc, pqd_c128* result) {
    FourTimeParams p{};
    p.dim = dim; p.n_t = n_t; p.n_map = n_map; p.n_precalc = n_precalc; p.dt = dt; p.tb = tb; p.variant = 1;
    return four_time_common(ctx, p, dm_1, dm_2, rho_init, t1, precalc, ops4, 4, result, false);
}

int pqd_dynamics_t1(pqd_ctx* ctx, const pqd_c128* dm_1, const pqd_c128* dm_2, const pqd_c128* rho_init,
                    const double* t1, const pqd_c128* precalc, int32_t n_t, double dt, int32_t n_map,
                    int32_t dim, double tb, int32_t n_precalc, pqd_c128* result) {
    FourTimeParams p{};
    p.dim = dim; p.n_t = n_t; p.n_map = n_map; p.n_precalc = n_precalc; p.dt = dt; p.tb = tb;
    return four_time_common(ctx, p, dm_1, dm_2, rho_init, t1, precalc, nullptr, 0, result, true);
}

int pqd_tl_dynmap_pseudo(pqd_ctx* ctx, const pqd_c128* dm, int32_t n_maps, int32_t n, double rcond,
                         pqd_c128* out) {
    if (!ctx || !dm || !out) return fail(PQD_ERR_ARG, "NULL argument");
    if (n < 1 || n > tl_dynmap_nmax()) return fail(PQD_ERR_UNSUPPORTED, "map size %d (max %d)", n, tl_dynmap_nmax());
    if (n_maps < 0) return fail(PQD_ERR_ARG, "n_maps %d", n_maps);
    if (!(rcond >= 0.0)) return fail(PQD_ERR_ARG, "rcond %g", rcond);
    if (n_maps == 0) return PQD_OK;
    HIPCHK(hipSetDevice(ctx->device));
    hipStream_t s = ctx->stream;
    const size_t m2 = (size_t)n * n;
    DevBuf<double2> d, o;
    HIPCHK(d.upload(reinterpret_cast<const double2*>(dm), (size_t)n_maps * m2, s));
    HIPCHK(o.alloc((size_t)n_maps * m2));
    HIPCHK(hipMemcpyAsync(o.p, d.p, m2 * sizeof(double2), hipMemcpyDeviceToDevice, s));  // out[0] = dm[0]
    HIPCHK(launch_tl_dynmap(d.p, n_maps, n, rcond, o.p, s));
    HIPCHK(hipMemcpyAsync(out, o.p, (size_t)n_maps * m2 * sizeof(double2), hipMemcpyDeviceToHost, s));
    HIPCHK(hipStreamSynchronize(s));
    return PQD_OK;
}

}  // extern "C"
