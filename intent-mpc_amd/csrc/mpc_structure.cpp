// mpc_structure.cpp -- see mpc_structure.hpp.
#include "mpc_structure.hpp"

#include <algorithm>
#include <cmath>

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
    mgd = mg;
    gen_dst.clear();
    return "";
}

namespace {

// fixed-seed generator: the placement is a function of the pattern and the shape alone
struct Lcg {
    uint64_t s = 0x9E3779B97F4A7C15ull;
    uint32_t next() {
        s = s * 6364136223846793005ull + 1442695040888963407ull;
        return (uint32_t)(s >> 32);
    }
    int below(int n) { return (int)(((uint64_t)next() * (uint64_t)n) >> 32); }
    double unit() { return (next() >> 8) * (1.0 / 16777216.0); }
};

}  // namespace

void MpcStructure::place(int slots, int T1r, int stride, int hsp, int pz, int nmax) {
    const bool spread = slots > mgd;
    // per dense row and entry: products slot (slot t of column v, colg order) and x index
    std::vector<int32_t> wa((size_t)4 * mgd, -1), ra((size_t)4 * mgd, -1);
    for (int32_t v = 0; v < n; v++)
        for (int32_t t = 0; t < CG; t++) {
            const int32_t id = colg[(size_t)v * CG + t];
            if (id < 0) continue;
            wa[id] = t < T1r ? t * stride + v : T1r * stride + (t - T1r) * hsp + col_hid[v];
            ra[id] = v;
        }
    const int L = std::max<int>(slots, mgd);
    std::vector<int32_t> lane(L, -1);  // table slot -> dense row
    for (int32_t g = 0; g < mgd; g++) lane[g] = g;
    // bank occupancy, kept incrementally: per (16-lane group, entry) the write addresses per bank
    // (distinct within a group), per (32-lane pair, entry) the rows reading each column and the
    // distinct columns per bank
    const int G = (L + 15) / 16, H = (L + 31) / 32;
    std::vector<int16_t> cw((size_t)G * 4 * 16, 0), dr((size_t)H * 4 * 32, 0), cr((size_t)H * 4 * n, 0);
    auto upd = [&](int p, int g, int s) {  // row g enters (s = 1) or leaves (s = -1) slot p
        if (g < 0) return;
        const size_t j = (size_t)p / 16, h = (size_t)p / 32;
        for (int e = 0; e < 4; e++) {
            const int32_t w = wa[4 * g + e], r = ra[4 * g + e];
            if (w >= 0) cw[(j * 4 + e) * 16 + (w & 15)] += s;
            if (r >= 0) {
                int16_t &c = cr[(h * 4 + e) * n + r];
                c += s;
                if ((s > 0 && c == 1) || (s < 0 && c == 0)) dr[(h * 4 + e) * 32 + (r & 31)] += s;
            }
        }
    };
    // extra LDS cycles of the write group j / the read pair h, all four entries
    auto wcost = [&](int j) {
        int c = 0;
        for (int e = 0; e < 4; e++) {
            int mx = 0;
            for (int b = 0; b < 16; b++) mx = std::max<int>(mx, cw[((size_t)j * 4 + e) * 16 + b]);
            c += mx > 1 ? mx - 1 : 0;
        }
        return c;
    };
    auto rcost = [&](int h) {
        int c = 0;
        for (int e = 0; e < 4; e++) {
            int mx = 0;
            for (int b = 0; b < 32; b++) mx = std::max<int>(mx, dr[((size_t)h * 4 + e) * 32 + b]);
            c += mx > 1 ? mx - 1 : 0;
        }
        return c;
    };
    place_conflicts[0] = place_conflicts[1] = 0;
    place_iters = 0;
    if (spread && L > mgd) {
        // first fit: each row into the least-filled 16-lane group where none of its entries meets
        // a write bank the group holds or a read bank its 32-lane pair holds with another column
        std::vector<int> fill(G, 0);
        std::fill(lane.begin(), lane.end(), -1);
        for (int32_t g = 0; g < mgd; g++) {
            int best = 0, bk = 1 << 30;
            for (int j = 0; j < G; j++) {
                if (fill[j] >= 16 || 16 * j + fill[j] >= L) continue;
                const size_t h = (size_t)j / 2;
                int c = 0;
                for (int e = 0; e < 4; e++) {
                    const int32_t w = wa[4 * g + e], r = ra[4 * g + e];
                    if (w >= 0 && cw[((size_t)j * 4 + e) * 16 + (w & 15)] > 0) c++;
                    if (r >= 0 && cr[(h * 4 + e) * n + r] == 0 && dr[(h * 4 + e) * 32 + (r & 31)] > 0) c++;
                }
                const int key = c * 64 + fill[j];
                if (key < bk) bk = key, best = j;
            }
            const int p = 16 * best + fill[best]++;
            lane[p] = g;
            upd(p, g, 1);
        }
    } else {
        for (int p = 0; p < L; p++) upd(p, lane[p], 1);
    }
    std::vector<int> Wc(G), Rc(H);
    int tot = 0;
    for (int j = 0; j < G; j++) tot += Wc[j] = wcost(j);
    for (int h = 0; h < H; h++) tot += Rc[h] = rcost(h);
    if (spread && tot > 0 && L > mgd) {
        // annealing over slot swaps from there (a fixed seed and schedule: deterministic); a move
        // takes a slot of a conflicting group and any slot of another group, a row or empty
        Lcg rng;
        const int iters = 200000;
        const double T0 = 0.3, T1 = 0.03, decay = std::pow(T1 / T0, 1.0 / iters);
        double T = T0;
        std::vector<int32_t> best = lane;
        int best_tot = tot;
        auto swp = [&](int a, int b) {
            upd(a, lane[a], -1);
            upd(b, lane[b], -1);
            std::swap(lane[a], lane[b]);
            upd(a, lane[a], 1);
            upd(b, lane[b], 1);
        };
        for (int it = 0; it < iters && tot > 0; it++, T *= decay) {
            int a = rng.below(L);
            for (int k = 0; k < 16 && Wc[a / 16] == 0 && Rc[a / 32] == 0; k++) a = rng.below(L);
            const int b = rng.below(L);
            if (a / 16 == b / 16 || lane[a] == lane[b]) continue;
            const int ja = a / 16, jb = b / 16, ha = a / 32, hb = b / 32;
            const int before = Wc[ja] + Wc[jb] + Rc[ha] + (hb != ha ? Rc[hb] : 0);
            swp(a, b);
            const int wa2 = wcost(ja), wb2 = wcost(jb), ra2 = rcost(ha), rb2 = hb != ha ? rcost(hb) : 0;
            const int d = wa2 + wb2 + ra2 + rb2 - before;
            if (d <= 0 || rng.unit() < std::exp(-d / T)) {
                Wc[ja] = wa2;
                Wc[jb] = wb2;
                Rc[ha] = ra2;
                if (hb != ha) Rc[hb] = rb2;
                tot += d;
                if (tot < best_tot) best_tot = tot, best = lane, place_iters = it;
            } else {
                swp(a, b);
            }
        }
        if (best != lane) {
            for (int p = 0; p < L; p++) upd(p, lane[p], -1);
            lane = best;
            for (int p = 0; p < L; p++) upd(p, lane[p], 1);
        }
    }
    for (int j = 0; j < G; j++) place_conflicts[0] += wcost(j);
    for (int h = 0; h < H; h++) place_conflicts[1] += rcost(h);
    // renumber the tables to the slots; an absent entry (padded, or any entry of an empty slot)
    // writes its zero product to a discard slot pz + k and reads a zero of the x exchange's tail,
    // nmax + k' (gen_col = -1 - k'), each on a bank no present entry of its group uses
    std::vector<int32_t> row2(L, -1), col2((size_t)4 * L, -1), pos2((size_t)4 * L, -1), slot_of(mgd, -1);
    gen_dst.assign((size_t)4 * L, -1);
    for (int p = 0; p < L; p++) {
        const int g = lane[p];
        if (g < 0) continue;
        slot_of[g] = p;
        row2[p] = gen_row[g];
        for (int e = 0; e < 4; e++) pos2[4 * p + e] = gen_pos[4 * g + e];
    }
    for (int p = 0; p < L; p++)
        for (int e = 0; e < 4; e++) {
            const int g = lane[p];
            if (g >= 0 && wa[4 * g + e] >= 0) {
                gen_dst[4 * p + e] = wa[4 * g + e];
                col2[4 * p + e] = ra[4 * g + e];
                continue;
            }
            uint32_t wu = 0, ru = 0;
            for (int i = 16 * (p / 16); i < std::min(L, 16 * (p / 16) + 16); i++)
                if (lane[i] >= 0 && wa[4 * lane[i] + e] >= 0) wu |= 1u << (wa[4 * lane[i] + e] & 15);
            for (int i = 32 * (p / 32); i < std::min(L, 32 * (p / 32) + 32); i++)
                if (lane[i] >= 0 && ra[4 * lane[i] + e] >= 0) ru |= 1u << (ra[4 * lane[i] + e] & 31);
            int bw = 0, br = 0;
            while (bw < 15 && (wu >> bw & 1)) bw++;
            while (br < 31 && (ru >> br & 1)) br++;
            gen_dst[4 * p + e] = pz + ((bw - pz) & 15);
            col2[4 * p + e] = -1 - ((br - nmax) & 31);
        }
    for (auto &id : colg)
        if (id >= 0) id = 4 * slot_of[id >> 2] + (id & 3);
    if (mgd > 0)  // the program on the slots (same term order)
        for (auto &c : term) c = (slot_of[c >> 4] << 4) | (c & 15);
    gen_row.swap(row2);
    gen_col.swap(col2);
    gen_pos.swap(pos2);
    mg = L;
}

}  // namespace impc
