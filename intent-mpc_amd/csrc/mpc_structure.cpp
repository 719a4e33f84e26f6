// mpc_structure.cpp -- see mpc_structure.hpp.
#include "mpc_structure.hpp"

#include <algorithm>

namespace impc {

std::string MpcStructure::analyse(int64_t n64, int64_t m64, const int64_t *Pp, const int64_t *Pi, const int64_t *Ap,
                                  const int64_t *Ai) {
    if ((n64 + 5) % 13 != 0) return "n is not 13N-5";
    N = (int32_t)((n64 + 5) / 13);
    if (N < 2) return "horizon < 2";
    n = (int32_t)n64;
    m = (int32_t)m64;
    W = N - 1;
    nnzP = (int32_t)Pp[n];
    nnzA = (int32_t)Ap[n];
    // stage-order index of an original variable
    auto sidx = [&](int32_t j) -> int32_t {
        if (j < 8 * N) return 13 * (j / 8) + j % 8;
        int32_t c = j - 8 * N;
        return 13 * (c / 5) + 8 + c % 5;
    };
    var_orig.assign(n, 0);
    for (int32_t j = 0; j < n; j++) var_orig[sidx(j)] = j;
    // P diagonal
    var_pdiag.assign(n, -1);
    for (int32_t j = 0; j < n; j++) {
        for (int64_t k = Pp[j]; k < Pp[j + 1]; k++) {
            if (Pi[k] != j) return "P is not diagonal";
            if (var_pdiag[sidx(j)] >= 0) return "duplicate P entry";
            var_pdiag[sidx(j)] = (int32_t)k;
        }
    }
    // rows of A
    std::vector<std::vector<std::pair<int32_t, int32_t>>> rows(m);  // (stage-order col, CSC slot)
    for (int32_t j = 0; j < n; j++)
        for (int64_t k = Ap[j]; k < Ap[j + 1]; k++) {
            if (Ai[k] < 0 || Ai[k] >= m) return "row index out of range";
            rows[Ai[k]].push_back({sidx(j), (int32_t)k});
        }
    var_boxrow.assign(n, -1);
    var_boxpos.assign(n, -1);
    std::vector<char> is_box(m, 0);
    for (int32_t i = 0; i < m; i++)
        if (rows[i].size() == 1) {
            int32_t v = rows[i][0].first;
            if (var_boxrow[v] < 0) {
                var_boxrow[v] = i;
                var_boxpos[v] = rows[i][0].second;
                is_box[i] = 1;
            }
        }
    for (int32_t v = 0; v < n; v++)
        if (var_boxrow[v] < 0) return "a variable has no single-entry row";
    gen_row.clear();
    gen_col.clear();
    gen_pos.clear();
    std::vector<int32_t> per_stage(N, 0);
    for (int32_t i = 0; i < m; i++) {
        if (is_box[i]) continue;
        auto r = rows[i];
        if (r.size() > 4) return "a general row has more than 4 entries";
        std::sort(r.begin(), r.end());
        int32_t k = r.empty() ? 0 : r.front().first / 13;
        for (auto &e : r) {
            int32_t ke = e.first / 13, re = e.first % 13;
            if (!(ke == k || (ke == k + 1 && re < 8))) return "a row couples non-adjacent stages";
        }
        gen_row.push_back(i);
        for (int e = 0; e < 4; e++) {
            gen_col.push_back(e < (int)r.size() ? r[e].first : -1);
            gen_pos.push_back(e < (int)r.size() ? r[e].second : -1);
        }
        per_stage[k]++;
    }
    mg = (int32_t)gen_row.size();
    max_general_per_stage = *std::max_element(per_stage.begin(), per_stage.end());
    // column gather lists (general entries per variable, increasing row order)
    std::vector<std::vector<int32_t>> cl(n);
    for (int32_t g = 0; g < mg; g++)
        for (int e = 0; e < 4; e++)
            if (gen_col[4 * g + e] >= 0) cl[gen_col[4 * g + e]].push_back(4 * g + e);
    CG = 1;
    for (auto &c : cl) CG = std::max<int32_t>(CG, (int32_t)c.size());
    colg.assign((size_t)n * CG, -1);
    for (int32_t v = 0; v < n; v++)
        for (size_t t = 0; t < cl[v].size(); t++) colg[(size_t)v * CG + t] = cl[v][t];
    HS = 0;
    col_hid.assign((size_t)n, -1);
    for (int32_t v = 0; v < n; v++)
        if ((int32_t)cl[v].size() > kProdTier1) col_hid[(size_t)v] = HS++;
    // factorisation assembly program: per stage k and destination d (M_kk[r][c] at 13r+c,
    // B_k[i][c] at 169+13i+c) the (g, e, f) triples of rho_g a_ge a_gf
    std::vector<std::vector<int32_t>> dest((size_t)N * kStageDests);
    for (int32_t g = 0; g < mg; g++)
        for (int e = 0; e < 4; e++)
            for (int f = 0; f < 4; f++) {
                int32_t ve = gen_col[4 * g + e], vf = gen_col[4 * g + f];
                if (ve < 0 || vf < 0) continue;
                int32_t ke = ve / 13, re = ve % 13, kf = vf / 13, rf = vf % 13;
                int32_t code = (g << 4) | (e << 2) | f;
                if (ke == kf)
                    dest[(size_t)ke * kStageDests + 13 * re + rf].push_back(code);
                else if (ke == kf + 1)
                    dest[(size_t)kf * kStageDests + 169 + 13 * re + rf].push_back(code);
            }
    term_ptr.assign((size_t)N * kStageDests + 1, 0);
    term.clear();
    for (size_t d = 0; d < dest.size(); d++) {
        for (int32_t c : dest[d]) term.push_back(c);
        term_ptr[d + 1] = (int32_t)term.size();
    }
    if (term.empty()) term.push_back(0);
    return "";
}

}  // namespace impc
