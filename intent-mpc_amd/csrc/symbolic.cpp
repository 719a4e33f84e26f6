// symbolic.cpp -- see symbolic.hpp.
#include "symbolic.hpp"

#include <algorithm>
#include <cstring>
#include <numeric>
#include <set>

namespace impc {
namespace {

// Minimum-degree ordering on an explicit elimination graph (sorted adjacency vectors).
// Ties are broken by the smaller original index, so the ordering is deterministic.
std::vector<int32_t> min_degree(int32_t n, std::vector<std::vector<int32_t>> adj) {
    std::vector<int32_t> order;
    order.reserve(n);
    std::vector<char> alive(n, 1);
    // bucketed priority: std::set of (degree, index)
    std::set<std::pair<int32_t, int32_t>> pq;
    for (int32_t i = 0; i < n; i++) pq.insert({(int32_t)adj[i].size(), i});
    std::vector<int32_t> merged;
    while (!pq.empty()) {
        auto it = pq.begin();
        int32_t v = it->second;
        pq.erase(it);
        alive[v] = 0;
        order.push_back(v);
        const std::vector<int32_t> nb = adj[v];
        for (int32_t u : nb) {
            if (!alive[u]) continue;
            pq.erase({(int32_t)adj[u].size(), u});
            // adj[u] <- (adj[u] U nb) \ {u, v}
            merged.clear();
            std::set_union(adj[u].begin(), adj[u].end(), nb.begin(), nb.end(), std::back_inserter(merged));
            adj[u].clear();
            for (int32_t w : merged)
                if (w != u && w != v && alive[w]) adj[u].push_back(w);
            pq.insert({(int32_t)adj[u].size(), u});
        }
        adj[v].clear();
    }
    return order;
}

}  // namespace

std::string Symbolic::build(int64_t n64, int64_t m64, const int64_t *Pp_, const int64_t *Pi_, const int64_t *Ap_,
                            const int64_t *Ai_) {
    if (n64 <= 0 || m64 < 0) return "n must be > 0 and m >= 0";
    if (n64 > (1 << 24) || m64 > (1 << 24)) return "problem too large for the batched solver";
    n = (int32_t)n64;
    m = (int32_t)m64;
    if (!Pp_ || !Ap_) return "null pattern pointer";
    if (Pp_[0] != 0 || Ap_[0] != 0) return "column pointers must start at 0";
    for (int32_t j = 0; j < n; j++)
        if (Pp_[j + 1] < Pp_[j] || Ap_[j + 1] < Ap_[j]) return "column pointers must be non-decreasing";
    if (Pp_[n] > INT32_MAX || Ap_[n] > INT32_MAX) return "too many nonzeros";
    nnzP = (int32_t)Pp_[n];
    nnzA = (int32_t)Ap_[n];
    Pp.assign(Pp_, Pp_ + n + 1);
    Ap.assign(Ap_, Ap_ + n + 1);
    Pi.resize(nnzP);
    Ai.resize(nnzA);
    for (int32_t k = 0; k < nnzP; k++) {
        Pi[k] = (int32_t)Pi_[k];
    }
    for (int32_t j = 0; j < n; j++)
        for (int32_t k = Pp[j]; k < Pp[j + 1]; k++)
            if (Pi[k] < 0 || Pi[k] > j) return "P must be upper triangular (OSQP validate_data)";
    for (int32_t k = 0; k < nnzA; k++) {
        if (Ai_[k] < 0 || Ai_[k] >= m) return "A row index out of range";
        Ai[k] = (int32_t)Ai_[k];
    }

    // ---- CSR view of A
    Arp.assign(m + 1, 0);
    for (int32_t k = 0; k < nnzA; k++) Arp[Ai[k] + 1]++;
    for (int32_t r = 0; r < m; r++) Arp[r + 1] += Arp[r];
    Arpos.resize(nnzA);
    Arcol.resize(nnzA);
    {
        std::vector<int32_t> next(Arp.begin(), Arp.end() - 1);
        for (int32_t j = 0; j < n; j++)
            for (int32_t k = Ap[j]; k < Ap[j + 1]; k++) {
                int32_t q = next[Ai[k]]++;
                Arpos[q] = k;
                Arcol[q] = j;
            }
    }

    // ---- pattern of M = P + sigma I + A'A (symmetric adjacency, no diagonal)
    std::vector<std::vector<int32_t>> adj(n);
    for (int32_t j = 0; j < n; j++)
        for (int32_t k = Pp[j]; k < Pp[j + 1]; k++)
            if (Pi[k] != j) {
                adj[j].push_back(Pi[k]);
                adj[Pi[k]].push_back(j);
            }
    for (int32_t r = 0; r < m; r++)
        for (int32_t a = Arp[r]; a < Arp[r + 1]; a++)
            for (int32_t b = Arp[r]; b < Arp[r + 1]; b++)
                if (Arcol[a] != Arcol[b]) adj[Arcol[a]].push_back(Arcol[b]);
    for (auto &v : adj) {
        std::sort(v.begin(), v.end());
        v.erase(std::unique(v.begin(), v.end()), v.end());
    }

    // ---- ordering
    perm = min_degree(n, adj);
    iperm.assign(n, 0);
    for (int32_t k = 0; k < n; k++) iperm[perm[k]] = k;
    Arcolf.resize(nnzA);
    for (int32_t q = 0; q < nnzA; q++) Arcolf[q] = iperm[Arcol[q]];

    // ---- upper(M) in factor order: column c holds rows r <= c
    std::vector<std::vector<int32_t>> cols(n);
    for (int32_t v = 0; v < n; v++) {
        int32_t fv = iperm[v];
        cols[fv].push_back(fv);
        for (int32_t u : adj[v]) {
            int32_t fu = iperm[u];
            if (fu < fv) cols[fv].push_back(fu);
        }
    }
    Mp.assign(n + 1, 0);
    for (int32_t c = 0; c < n; c++) {
        std::sort(cols[c].begin(), cols[c].end());
        Mp[c + 1] = Mp[c] + (int32_t)cols[c].size();
    }
    nnzM = Mp[n];
    Mi.resize(nnzM);
    Mdiag.resize(n);
    for (int32_t c = 0; c < n; c++)
        for (size_t t = 0; t < cols[c].size(); t++) {
            Mi[Mp[c] + (int32_t)t] = cols[c][t];
            if (cols[c][t] == c) Mdiag[c] = Mp[c] + (int32_t)t;
        }
    auto slot = [&](int32_t fa, int32_t fb) -> int32_t {  // slot of (min, max) in upper(M)
        int32_t r = std::min(fa, fb), c = std::max(fa, fb);
        const int32_t *b = Mi.data() + Mp[c], *e = Mi.data() + Mp[c + 1];
        const int32_t *it = std::lower_bound(b, e, r);
        return (int32_t)(it - Mi.data());
    };

    // ---- assembly program (sorted by destination slot for locality)
    {
        std::vector<std::pair<int32_t, int32_t>> pt;
        for (int32_t j = 0; j < n; j++)
            for (int32_t k = Pp[j]; k < Pp[j + 1]; k++) pt.push_back({slot(iperm[Pi[k]], iperm[j]), k});
        std::stable_sort(pt.begin(), pt.end());
        Pt_dest.resize(pt.size());
        Pt_src.resize(pt.size());
        for (size_t t = 0; t < pt.size(); t++) {
            Pt_dest[t] = pt[t].first;
            Pt_src[t] = pt[t].second;
        }
        struct ATerm {
            int32_t d, a, b, r;
        };
        std::vector<ATerm> at;
        for (int32_t r = 0; r < m; r++)
            for (int32_t a = Arp[r]; a < Arp[r + 1]; a++)
                for (int32_t b = a; b < Arp[r + 1]; b++)
                    at.push_back({slot(Arcolf[a], Arcolf[b]), Arpos[a], Arpos[b], r});
        std::stable_sort(at.begin(), at.end(), [](const ATerm &x, const ATerm &y) { return x.d < y.d; });
        At_dest.resize(at.size());
        At_a.resize(at.size());
        At_b.resize(at.size());
        At_r.resize(at.size());
        for (size_t t = 0; t < at.size(); t++) {
            At_dest[t] = at[t].d;
            At_a[t] = at[t].a;
            At_b[t] = at[t].b;
            At_r[t] = at[t].r;
        }
    }

    // ---- QDLDL symbolic: elimination tree and column counts (QDLDL_etree)
    std::vector<int32_t> etree(n, -1), Lnz(n, 0), work(n, 0);
    for (int32_t j = 0; j < n; j++) {
        work[j] = j;
        for (int32_t p = Mp[j]; p < Mp[j + 1]; p++) {
            int32_t i = Mi[p];
            while (work[i] != j) {
                if (etree[i] == -1) etree[i] = j;
                Lnz[i]++;
                work[i] = j;
                i = etree[i];
            }
        }
    }
    Lp.assign(n + 1, 0);
    for (int32_t i = 0; i < n; i++) Lp[i + 1] = Lp[i] + Lnz[i];
    nnzL = Lp[n];
    Li.assign(nnzL, 0);

    // ---- replay of QDLDL_factor's pattern traversal -> update program
    upd_ptr.assign(n + 1, 0);
    upd_c.clear();
    upd_js.clear();
    upd_je.clear();
    upd_w.clear();
    {
        std::vector<char> marked(n, 0);
        std::vector<int32_t> yIdx(n), elim(n), next(Lp.begin(), Lp.end() - 1);
        factor_flops = 0;
        for (int32_t k = 0; k < n; k++) {
            int32_t nnzY = 0;
            for (int32_t p = Mp[k]; p < Mp[k + 1]; p++) {
                int32_t bidx = Mi[p];
                if (bidx == k) continue;
                if (!marked[bidx]) {
                    marked[bidx] = 1;
                    elim[0] = bidx;
                    int32_t nnzE = 1;
                    int32_t nx = etree[bidx];
                    while (nx != -1 && nx < k) {
                        if (marked[nx]) break;
                        marked[nx] = 1;
                        elim[nnzE++] = nx;
                        nx = etree[nx];
                    }
                    while (nnzE) yIdx[nnzY++] = elim[--nnzE];
                }
            }
            for (int32_t i = nnzY - 1; i >= 0; i--) {
                int32_t c = yIdx[i];
                upd_c.push_back(c);
                upd_js.push_back(Lp[c]);
                upd_je.push_back(next[c]);
                upd_w.push_back(next[c]);
                factor_flops += 2 * (next[c] - Lp[c]) + 3;
                Li[next[c]] = k;
                next[c]++;
                marked[c] = 0;
            }
            upd_ptr[k + 1] = (int32_t)upd_c.size();
        }
        n_upd = (int64_t)upd_c.size();
    }

    // ---- CSR view of L (row i: entries L(i, c), c < i)
    Lrp.assign(n + 1, 0);
    for (int32_t t = 0; t < nnzL; t++) Lrp[Li[t] + 1]++;
    for (int32_t i = 0; i < n; i++) Lrp[i + 1] += Lrp[i];
    Lrc.resize(nnzL);
    Lrpos.resize(nnzL);
    {
        std::vector<int32_t> nx(Lrp.begin(), Lrp.end() - 1);
        for (int32_t c = 0; c < n; c++)
            for (int32_t t = Lp[c]; t < Lp[c + 1]; t++) {
                int32_t q = nx[Li[t]]++;
                Lrc[q] = c;
                Lrpos[q] = t;
            }
    }
    max_row_L = 0;
    for (int32_t i = 0; i < n; i++) max_row_L = std::max(max_row_L, Lrp[i + 1] - Lrp[i]);
    return "";
}

}  // namespace impc
