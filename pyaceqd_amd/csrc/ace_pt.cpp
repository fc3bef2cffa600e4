// ace_pt.cpp — reader for the process-tensor files ACE writes with `write_PT <name>` (reference
// general_system.py:146-157 names them, :190 writes them, :194-197 lists the four files <name>_initial,
// <name>_initial_0, <name>_repeated, <name>_repeated_0 and :153/:156 detects <name>_initial).
//
// ACE's on-disk layout is not documented anywhere in the reference and no ACE-made file exists offline
// (SURVEY.md §8c, §8f rank 2), so this reader implements one explicit ASSUMPTION, layout "ACE_PTB_V0", and
// refuses everything else with PQD_ERR_UNSUPPORTED and a message naming the file and the mismatch:
//
//   The four names are two PT buffers (initial slices, repeated slice), each a header file <buf> plus block
//   files <buf>_0, <buf>_1, ... (buffer_blocksize -1 = one block: exactly the four files the reference lists).
//   Header <buf> (text, whitespace separated):   ACE_PTB_V0  elements <n>  blocks <nb>
//   Block  <buf>_<k> (binary, little endian), its elements back to back, each:
//       char    tag[4] = "PTE0"
//       int32   N2, D                 outer (Liouville) dimension of the system, dictionary size
//       int32   dict[N2]              dictionary entry of Liouville index alpha = i*N + j (diagonal coupling)
//       int32   chi_l, chi_r          bond dimensions into and out of the element
//       c128    M[D][chi_l][chi_r]    the element, row-major (left bond, right bond)
//       c128    closure[chi_r]        bond closure after the element
//   Element s of <name>_initial is PT slice s; <name>_repeated holds one element, the slice used for every step
//   after the initial ones (use_Gaussian_repeat). The first element's left bond is the initial bond (chi_l = 1 in
//   ACE's construction, bond vector e_0); the output closure at step 0 is e_0 of that bond.
//
// The pqd PT has one bond dimension for all slices: chi = max over elements, smaller elements zero-padded (the
// padding rows and columns never receive weight, so the contraction is unchanged).
#include "../../include/pqd.h"
#include "pqd_common.h"

#include <algorithm>
#include <cstdio>
#include <cstring>
#include <fstream>
#include <sstream>
#include <string>
#include <vector>

namespace {

struct Elem {
    int32_t N2 = 0, D = 0, chi_l = 0, chi_r = 0;
    std::vector<int32_t> dict;
    std::vector<double2> M, closure;
};

struct Reader {
    std::string err;
    int code = PQD_OK;
    bool fail(int c, const std::string& m) {
        if (code == PQD_OK) { code = c; err = m; }
        return false;
    }
};

bool read_header(Reader& R, const std::string& buf, int64_t& n_el, int64_t& n_blk) {
    std::ifstream f(buf);
    if (!f) return R.fail(PQD_ERR_ARG, buf + ": cannot open the PT buffer header");
    std::string magic, k1, k2;
    if (!(f >> magic) || magic != "ACE_PTB_V0")
        return R.fail(PQD_ERR_UNSUPPORTED, buf + ": header does not start with ACE_PTB_V0 (the only ACE PT layout "
                                                 "this reader implements; see include/pqd.h pqd_ace_pt_read)");
    if (!(f >> k1 >> n_el >> k2 >> n_blk) || k1 != "elements" || k2 != "blocks" || n_el < 1 || n_blk < 1 ||
        n_blk > n_el)
        return R.fail(PQD_ERR_UNSUPPORTED, buf + ": malformed ACE_PTB_V0 header (expected 'elements <n> blocks <nb>')");
    return true;
}

template <typename T>
bool get(std::ifstream& f, T* p, size_t n) {
    f.read(reinterpret_cast<char*>(p), (std::streamsize)(n * sizeof(T)));
    return (size_t)f.gcount() == n * sizeof(T);
}

bool read_buffer(Reader& R, const std::string& buf, int32_t N2, std::vector<Elem>& out) {
    int64_t n_el = 0, n_blk = 0;
    if (!read_header(R, buf, n_el, n_blk)) return false;
    for (int64_t b = 0; b < n_blk && (int64_t)out.size() < n_el + 0; ++b) {
        const std::string fn = buf + "_" + std::to_string(b);
        std::ifstream f(fn, std::ios::binary);
        if (!f) return R.fail(PQD_ERR_ARG, fn + ": cannot open the PT block file");
        while ((int64_t)out.size() < n_el) {
            char tag[4];
            f.read(tag, 4);
            if (f.gcount() == 0) break;  // end of this block
            if (f.gcount() != 4 || std::memcmp(tag, "PTE0", 4) != 0)
                return R.fail(PQD_ERR_UNSUPPORTED, fn + ": element " + std::to_string(out.size()) +
                                                       " does not start with the PTE0 tag (layout ACE_PTB_V0)");
            Elem e;
            int32_t hd[2];
            if (!get(f, hd, 2)) return R.fail(PQD_ERR_UNSUPPORTED, fn + ": truncated element header");
            e.N2 = hd[0];
            e.D = hd[1];
            if (e.N2 != N2)
                return R.fail(PQD_ERR_UNSUPPORTED, fn + ": element for Liouville dimension " + std::to_string(e.N2) +
                                                       ", the system has " + std::to_string(N2));
            if (e.D < 1 || e.D > N2) return R.fail(PQD_ERR_UNSUPPORTED, fn + ": dictionary size out of range");
            e.dict.resize(N2);
            if (!get(f, e.dict.data(), (size_t)N2)) return R.fail(PQD_ERR_UNSUPPORTED, fn + ": truncated dictionary");
            for (int a = 0; a < N2; ++a)
                if (e.dict[a] < 0 || e.dict[a] >= e.D)
                    return R.fail(PQD_ERR_UNSUPPORTED, fn + ": dictionary entry out of range (non-diagonal couplings "
                                                           "are not supported)");
            int32_t ch[2];
            if (!get(f, ch, 2)) return R.fail(PQD_ERR_UNSUPPORTED, fn + ": truncated bond dimensions");
            e.chi_l = ch[0];
            e.chi_r = ch[1];
            if (e.chi_l < 1 || e.chi_r < 1 || e.chi_l > 128 || e.chi_r > 128)
                return R.fail(PQD_ERR_UNSUPPORTED, fn + ": bond dimension outside [1, 128]");
            e.M.resize((size_t)e.D * e.chi_l * e.chi_r);
            e.closure.resize(e.chi_r);
            if (!get(f, e.M.data(), e.M.size()) || !get(f, e.closure.data(), e.closure.size()))
                return R.fail(PQD_ERR_UNSUPPORTED, fn + ": truncated element data");
            out.push_back(std::move(e));
        }
    }
    if ((int64_t)out.size() != n_el)
        return R.fail(PQD_ERR_UNSUPPORTED, buf + ": header announces " + std::to_string(n_el) + " elements, blocks hold " +
                                               std::to_string(out.size()));
    return true;
}

bool read_all(Reader& R, const char* name, int32_t dim, std::vector<Elem>& ini, std::vector<Elem>& rep) {
    if (!name) return R.fail(PQD_ERR_ARG, "NULL PT name");
    if (dim < 2 || dim > 6) return R.fail(PQD_ERR_UNSUPPORTED, "dim not in [2, 6]");
    const int32_t N2 = dim * dim;
    if (!read_buffer(R, std::string(name) + "_initial", N2, ini)) return false;
    if (!read_buffer(R, std::string(name) + "_repeated", N2, rep)) return false;
    if (rep.size() != 1) return R.fail(PQD_ERR_UNSUPPORTED, std::string(name) + "_repeated: expected one element");
    // bonds chain: right bond of slice s = left bond of slice s+1; the repeated slice maps its own bond to itself
    std::vector<const Elem*> all;
    for (auto& e : ini) all.push_back(&e);
    all.push_back(&rep[0]);
    for (size_t s = 1; s < all.size(); ++s)
        if (all[s]->chi_l != all[s - 1]->chi_r)
            return R.fail(PQD_ERR_UNSUPPORTED, std::string(name) + ": bond dimensions do not chain at slice " +
                                                   std::to_string(s));
    if (rep[0].chi_l != rep[0].chi_r)
        return R.fail(PQD_ERR_UNSUPPORTED, std::string(name) + "_repeated: element is not square in the bond");
    for (size_t s = 1; s < all.size(); ++s)
        if (all[s]->D != all[0]->D || all[s]->dict != all[0]->dict)
            return R.fail(PQD_ERR_UNSUPPORTED, std::string(name) + ": slices use different dictionaries");
    return true;
}

}  // namespace

extern "C" int pqd_ace_pt_shape(const char* name, int32_t dim, pqd_ace_pt_dims* shape) {
    if (!shape) return pqd_fail_msg(PQD_ERR_ARG, "NULL shape");
    Reader R;
    std::vector<Elem> ini, rep;
    if (!read_all(R, name, dim, ini, rep)) return pqd_fail_msg(R.code, R.err.c_str());
    int chi = rep[0].chi_r;
    for (auto& e : ini) chi = std::max(chi, std::max(e.chi_l, e.chi_r));
    shape->n_init = (int32_t)ini.size();
    shape->n_slices = (int32_t)ini.size() + 1;
    shape->chi = chi;
    shape->D = ini[0].D;
    return PQD_OK;
}

extern "C" int pqd_ace_pt_read(const char* name, int32_t dim, const pqd_ace_pt_dims* shape, pqd_c128* Q,
                               pqd_c128* closure, pqd_c128* closure0, pqd_c128* bond0, int32_t* gmap) {
    if (!shape || !Q || !closure || !closure0 || !bond0 || !gmap) return pqd_fail_msg(PQD_ERR_ARG, "NULL argument");
    Reader R;
    std::vector<Elem> ini, rep;
    if (!read_all(R, name, dim, ini, rep)) return pqd_fail_msg(R.code, R.err.c_str());
    const int chi = shape->chi, D = ini[0].D, S = (int)ini.size() + 1;
    if (shape->n_slices != S || shape->D != D || shape->n_init != S - 1)
        return pqd_fail_msg(PQD_ERR_ARG, "shape does not match the files (call pqd_ace_pt_shape first)");
    int mx = rep[0].chi_r;
    for (auto& e : ini) mx = std::max(mx, std::max(e.chi_l, e.chi_r));
    if (chi < mx)
        return pqd_fail_msg(PQD_ERR_ARG, ("shape->chi " + std::to_string(chi) + " below the files' bond dimension " +
                                          std::to_string(mx)).c_str());
    const size_t cc = (size_t)chi * chi;
    std::memset(Q, 0, sizeof(pqd_c128) * (size_t)S * D * cc);
    std::memset(closure, 0, sizeof(pqd_c128) * (size_t)S * chi);
    std::memset(closure0, 0, sizeof(pqd_c128) * chi);
    std::memset(bond0, 0, sizeof(pqd_c128) * chi);
    for (int s = 0; s < S; ++s) {
        const Elem& e = s < S - 1 ? ini[s] : rep[0];
        for (int g = 0; g < D; ++g)
            for (int i = 0; i < e.chi_l; ++i)
                for (int j = 0; j < e.chi_r; ++j) {
                    const double2 v = e.M[((size_t)g * e.chi_l + i) * e.chi_r + j];
                    Q[((size_t)s * D + g) * cc + (size_t)i * chi + j] = {v.x, v.y};
                }
        for (int j = 0; j < e.chi_r; ++j) closure[(size_t)s * chi + j] = {e.closure[j].x, e.closure[j].y};
    }
    closure0[0] = {1.0, 0.0};
    bond0[0] = {1.0, 0.0};
    std::memcpy(gmap, ini[0].dict.data(), sizeof(int32_t) * ini[0].dict.size());
    return PQD_OK;
}
