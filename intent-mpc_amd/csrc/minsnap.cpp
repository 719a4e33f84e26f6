// minsnap.cpp -- batched assembly of polyTrajSolver's minimum-snap QP (host C++; the solve runs
// on the device through impc_batch_*).  Reference:
// trajectory_planner/include/trajectory_planner/polyTrajSolver.cpp (line ranges in
// include/impc_minsnap.h).
//
// The reference fills an Eigen::SparseMatrix entry by entry and OsqpEigen copies it to CSC
// (rows sorted per column, inserted entries kept even when their value is zero).  Which entries
// are inserted depends only on the degrees and the segment count (an entry is inserted when its
// time-free factor is non-zero), so the entry list is generated once, sorted to CSC order once,
// and each path's values are scattered into their slots.  Values follow the reference's
// expressions and evaluation order (std::pow as the reference calls it; -ffp-contract=off).
//
// Corridor constraints (setCorridorConstraint / updateCorridorParam :960-1012, rows of constructA
// :557-579 and constructBound :815-835): segment i with corridor size r_i != 0 gets one row per
// sample t of `for (t = 0; t <= 1; t += 1.0 / numCorridor_i)`, numCorridor_i =
// ceil((T_{i+1} - T_i) * corridor_res), entries pow(t, d) on the segment's coefficients and bounds
// interpolate(p_i, p_{i+1}, t) -+ r_i.  The reference keeps the samples of a segment in a
// std::unordered_map<double, pose> and emits the rows in that container's iteration order; the
// same container (libstdc++'s, the reference's standard library) fed the same keys in the same
// insertion order gives the same order here.  The sample times -- hence the pattern and the A
// values -- depend only on numCorridor_i, so paths sharing the numCorridor vector share a batch.
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <unordered_map>
#include <vector>

#include "../../include/impc_minsnap.h"

namespace {

struct Shape {
    int deg, diff, cont, W, S;
    int64_t n, m;
    std::vector<int32_t> cnum;              // numCorridor per segment (0: no corridor rows); empty: off
    std::vector<std::vector<double>> ctime;  // per segment: sample times in the container's order
};

// updateCorridorParam's samples of one segment, in std::unordered_map<double, pose> order
std::vector<double> corridor_times(int32_t num_corridor) {
    std::unordered_map<double, int> samples;
    const double dt = (1.0) / num_corridor;
    int k = 0;
    for (double t = 0; t <= 1.0; t += dt) samples[t] = k++;
    std::vector<double> out;
    out.reserve(samples.size());
    for (const auto &it : samples) out.push_back(it.first);
    return out;
}

constexpr int32_t kMaxCorridor = 1 << 16;  // samples per segment (a guard against absurd inputs)

bool make_shape(const impc_minsnap_params *p, int32_t W, const int32_t *corridor_num, Shape *s) {
    if (!p || W < 2 || p->poly_degree < 1 || p->diff_degree < 0 || !(p->desired_vel > 0)) return false;
    s->deg = p->poly_degree;
    s->diff = p->diff_degree;
    s->cont = p->continuity_degree < 2 ? 2 : p->continuity_degree;  // updatePath :56
    if (s->cont > 4) return false;  // constructA / constructBound build rows up to snap only
    s->W = W;
    s->S = W - 1;
    s->n = (int64_t)(s->deg + 1) * s->S;
    const int64_t S = s->S;
    s->m = (2 + 2 * (S - 1)) + (2 + S - 1) + (2 + S - 1) + (S - 1) * (s->cont - 2);  // :156-160
    s->cnum.clear();
    s->ctime.clear();
    if (corridor_num) {  // constraintNum_ = getConstraintNum() + countCorridorConstraint (:1011)
        s->cnum.assign(corridor_num, corridor_num + S);
        s->ctime.resize((size_t)S);
        for (int i = 0; i < S; i++) {
            if (s->cnum[i] < 0 || s->cnum[i] > kMaxCorridor) return false;
            if (s->cnum[i] == 0) continue;
            s->ctime[i] = corridor_times(s->cnum[i]);
            s->m += (int64_t)s->ctime[i].size();
        }
    }
    return true;
}

// numCorridor of segment i (updateCorridorParam :996-998); 0 when its corridor size is 0
int32_t num_corridor(double duration, double size, double res) {
    if (size == 0.0) return 0;
    const double c = std::ceil(duration * res);
    return c >= 1 && c <= kMaxCorridor ? (int32_t)c : -1;
}

// One inserted A entry: the value is coef * dt(seg_dt)^pw, dt taken from the time allocation
// (kind 0: no duration factor, 1: dtRight of junction i, 2: dtLeft of junction i).
struct AEntry {
    int64_t row, col;
    double coef;
    int kind, junction, pw;
};

// Insertion list of constructA (:314-585) without the corridor rows.
std::vector<AEntry> a_entries(const Shape &s) {
    std::vector<AEntry> e;
    const int D = s.deg + 1, S = s.S;
    int64_t r = 0;
    auto endpoint_rows = [&](int order) {  // start (t = 0) and end (t = 1) rows of one derivative order
        for (int side = 0; side < 2; side++) {
            const double t = side == 0 ? 0.0 : 1.0;
            const int64_t base = side == 0 ? 0 : (int64_t)(S - 1) * D;
            for (int d = order; d < D; d++) {
                double f;
                if (order == 0) f = std::pow(t, d);
                else if (order == 1) f = d * std::pow(t, d - 1);
                else f = d * (d - 1) * std::pow(t, d - 2);
                if (f != 0) e.push_back({r, base + d, f, 0, 0, 0});
            }
            r++;
        }
    };
    // position: 2 endpoints, S-1 waypoints (right end of segment i), S-1 C0 continuity
    endpoint_rows(0);
    for (int i = 0; i < S - 1; i++) {
        for (int d = 0; d < D; d++) {
            const double f = std::pow(1.0, d);
            if (f != 0) e.push_back({r, (int64_t)D * i + d, f, 0, 0, 0});
        }
        r++;
    }
    for (int i = 0; i < S - 1; i++) {
        for (int d = 0; d < D; d++) {
            const double lf = std::pow(1.0, d), rf = std::pow(0.0, d);
            if (lf != 0) e.push_back({r, (int64_t)D * i + d, lf, 0, 0, 0});
            if (rf != 0) e.push_back({r, (int64_t)D * (i + 1) + d, -rf, 0, 0, 0});
        }
        r++;
    }
    // velocity, acceleration, jerk, snap: endpoints (orders 1, 2) and continuity rows scaled by
    // the neighbouring durations, left * dtRight^k, -right * dtLeft^k
    for (int order = 1; order <= 4; order++) {
        if (order >= 3 && s.cont < order) break;
        if (order <= 2) endpoint_rows(order);
        for (int i = 0; i < S - 1; i++) {
            for (int d = order; d < D; d++) {
                double lf, rf;
                if (order == 1) {
                    lf = d * std::pow(1.0, d - 1);
                    rf = d * std::pow(0.0, d - 1);
                } else if (order == 2) {
                    lf = d * (d - 1) * std::pow(1.0, d - 2);
                    rf = d * (d - 1) * std::pow(0.0, d - 2);
                } else if (order == 3) {
                    lf = d * (d - 1) * (d - 2) * std::pow(1.0, d - 3);
                    rf = d * (d - 1) * (d - 2) * std::pow(0.0, d - 3);
                } else {
                    lf = d * (d - 1) * (d - 2) * (d - 3) * std::pow(1.0, d - 4);
                    rf = d * (d - 1) * (d - 2) * (d - 3) * std::pow(0.0, d - 4);
                }
                if (lf != 0) e.push_back({r, (int64_t)D * i + d, lf, 1, i, order});
                if (rf != 0) e.push_back({r, (int64_t)D * (i + 1) + d, -rf, 2, i, order});
            }
            r++;
        }
    }
    // corridor rows (:557-579): pow(t, d) on segment i's coefficients, non-zero factors only
    for (int i = 0; i < (int)s.ctime.size(); i++)
        for (double t : s.ctime[(size_t)i]) {
            for (int d = 0; d < D; d++) {
                const double f = std::pow(t, d);
                if (f != 0) e.push_back({r, (int64_t)D * i + d, f, 0, 0, 0});
            }
            r++;
        }
    return e;
}

// CSC order of the entries (column, then row): perm[k] = insertion index of CSC slot k
void a_pattern(const Shape &s, const std::vector<AEntry> &e, int64_t *Ap, int64_t *Ai, std::vector<int64_t> *perm) {
    std::vector<int64_t> idx(e.size());
    for (size_t k = 0; k < e.size(); k++) idx[k] = (int64_t)k;
    std::stable_sort(idx.begin(), idx.end(), [&](int64_t a, int64_t b) {
        return e[a].col != e[b].col ? e[a].col < e[b].col : e[a].row < e[b].row;
    });
    if (Ap) {
        std::fill(Ap, Ap + s.n + 1, 0);
        for (const AEntry &x : e) Ap[x.col + 1]++;
        for (int64_t j = 0; j < s.n; j++) Ap[j + 1] += Ap[j];
    }
    if (Ai)
        for (size_t k = 0; k < idx.size(); k++) Ai[k] = e[idx[k]].row;
    if (perm) *perm = idx;
}

int64_t p_nnz(const Shape &s) {
    const int64_t b = s.deg >= s.diff ? s.deg - s.diff + 1 : 0;
    return s.S * b * (b + 1) / 2;
}

// desiredTime_ of avgTimeAllocation (:125-138)
void time_allocation(const Shape &s, const double *path, double v, double *T) {
    double total = 0;
    T[0] = total;
    for (int i = 1; i < s.W; i++) {
        const double *a = path + 3 * i, *b = path + 3 * (i - 1);
        const double dist = std::sqrt(std::pow(a[0] - b[0], 2) + std::pow(a[1] - b[1], 2) + std::pow(a[2] - b[2], 2));
        const double duration = (double)dist / v;
        total += duration;
        T[i] = total;
    }
}

// constructBound (:587-835) for one path, three axes: l, u [3][m]; csize [S] corridor sizes
void bounds(const Shape &s, const impc_minsnap_params *p, const double *path, const double *iv, const double *ev,
            const double *ia, const double *ea, const double *csize, double *l, double *u) {
    const double zero3[3] = {0, 0, 0};
    iv = iv ? iv : zero3, ev = ev ? ev : zero3, ia = ia ? ia : zero3, ea = ea ? ea : zero3;
    const int S = s.S;
    for (int a = 0; a < 3; a++) {
        double *la = l ? l + (int64_t)a * s.m : nullptr, *ua = u ? u + (int64_t)a * s.m : nullptr;
        int64_t r = 0;
        auto set = [&](double lo, double hi) {
            if (la) la[r] = lo;
            if (ua) ua[r] = hi;
            r++;
        };
        set(path[a], path[a]);
        set(path[3 * (s.W - 1) + a], path[3 * (s.W - 1) + a]);
        for (int i = 0; i < S - 1; i++) {
            const double w = path[3 * (i + 1) + a];
            if (p->soft_constraint)
                set(w - p->sc_deviation[a], w + p->sc_deviation[a]);
            else
                set(w, w);
        }
        for (int i = 0; i < S - 1; i++) set(0.0, 0.0);
        set(iv[a], iv[a]);
        set(ev[a], ev[a]);
        for (int i = 0; i < S - 1; i++) set(0.0, 0.0);
        set(ia[a], ia[a]);
        set(ea[a], ea[a]);
        for (int i = 0; i < S - 1; i++) set(0.0, 0.0);
        for (int k = 3; k <= s.cont; k++)
            for (int i = 0; i < S - 1; i++) set(0.0, 0.0);
        // corridor rows (:815-835): interpolatePose(p_i, p_{i+1}, 0, 1, t) (:1014-1023) -+ r_i
        for (int i = 0; i < (int)s.ctime.size(); i++) {
            const double rr = csize[i];
            const double ps = path[3 * i + a], pe = path[3 * (i + 1) + a];
            for (double t : s.ctime[(size_t)i]) {
                const double mid = ps + (pe - ps) * (t - 0.0) / (1.0 - 0.0);
                set(mid - rr, mid + rr);
            }
        }
    }
}

// every path's numCorridor vector must be the batch's (the corridor rows are part of the pattern)
bool corridor_matches(const Shape &s, const impc_minsnap_params *p, const double *path, const double *csize,
                      double res, std::vector<double> &T) {
    if (s.cnum.empty()) return true;
    time_allocation(s, path, p->desired_vel, T.data());
    for (int i = 0; i < s.S; i++)
        if (num_corridor(T[i + 1] - T[i], csize[i], res) != s.cnum[(size_t)i]) return false;
    return true;
}

}  // namespace

extern "C" int impc_minsnap_corridor_num(const impc_minsnap_params *p, int64_t nb, int32_t num_waypoints,
                                         const double *path, const double *corridor_size, double corridor_res,
                                         int32_t *corridor_num) {
    Shape s;
    if (!make_shape(p, num_waypoints, nullptr, &s) || nb < 0 || !path || !corridor_size || !corridor_num ||
        !(corridor_res > 0))
        return 1;
    std::vector<double> T((size_t)s.W);
    for (int64_t b = 0; b < nb; b++) {
        time_allocation(s, path + (size_t)b * s.W * 3, p->desired_vel, T.data());
        for (int i = 0; i < s.S; i++) {
            const int32_t c = num_corridor(T[i + 1] - T[i], corridor_size[(size_t)b * s.S + i], corridor_res);
            if (c < 0) return 1;
            corridor_num[(size_t)b * s.S + i] = c;
        }
    }
    return 0;
}

extern "C" int impc_minsnap_corridor_dims(const impc_minsnap_params *p, int32_t num_waypoints,
                                          const int32_t *corridor_num, impc_qp_dims *out) {
    Shape s;
    if (!out || !make_shape(p, num_waypoints, corridor_num, &s)) return 1;
    out->n = s.n;
    out->m = s.m;
    out->nnzP = p_nnz(s);
    out->nnzA = (int64_t)a_entries(s).size();
    return 0;
}

extern "C" int impc_minsnap_dims(const impc_minsnap_params *p, int32_t num_waypoints, impc_qp_dims *out) {
    return impc_minsnap_corridor_dims(p, num_waypoints, nullptr, out);
}

extern "C" int impc_minsnap_corridor_pattern(const impc_minsnap_params *p, int32_t num_waypoints,
                                             const int32_t *corridor_num, int64_t *Pp, int64_t *Pi, int64_t *Ap,
                                             int64_t *Ai) {
    Shape s;
    if (!make_shape(p, num_waypoints, corridor_num, &s)) return 1;
    // P upper triangle: column D n + j holds rows D n + i, diff <= i <= j
    const int D = s.deg + 1;
    int64_t k = 0;
    for (int64_t c = 0; c < s.n; c++) {
        if (Pp) Pp[c] = k;
        const int seg = (int)(c / D), j = (int)(c % D);
        if (j < s.diff) continue;
        for (int i = s.diff; i <= j; i++, k++)
            if (Pi) Pi[k] = (int64_t)D * seg + i;
    }
    if (Pp) Pp[s.n] = k;
    a_pattern(s, a_entries(s), Ap, Ai, nullptr);
    return 0;
}

extern "C" int impc_minsnap_build_pattern(const impc_minsnap_params *p, int32_t num_waypoints, int64_t *Pp,
                                          int64_t *Pi, int64_t *Ap, int64_t *Ai) {
    return impc_minsnap_corridor_pattern(p, num_waypoints, nullptr, Pp, Pi, Ap, Ai);
}

extern "C" int impc_minsnap_corridor_values(const impc_minsnap_params *p, int64_t nb, int32_t num_waypoints,
                                            const double *path, const double *init_vel, const double *end_vel,
                                            const double *init_acc, const double *end_acc,
                                            const int32_t *corridor_num, const double *corridor_size,
                                            double corridor_res, double *Px, double *q, double *Ax, double *l,
                                            double *u, double *seg_time) {
    Shape s;
    if (!make_shape(p, num_waypoints, corridor_num, &s) || nb < 0 || !path) return 1;
    if (corridor_num && !corridor_size) return 1;
    const int D = s.deg + 1;
    // P values (path independent): prod_{d<diff} (i-d)(j-d) / (i+j-2 diff+1), constructP :241-272
    std::vector<double> pv;
    for (int64_t c = 0; c < s.n; c++) {
        const int j = (int)(c % D);
        if (j < s.diff) continue;
        for (int i = s.diff; i <= j; i++) {
            double factor = 1.0;
            for (int d = 0; d < s.diff; ++d) factor *= (double)(i - d) * (j - d);
            factor /= (double)(i + j - s.diff * 2 + 1);
            pv.push_back(factor);
        }
    }
    const std::vector<AEntry> e = a_entries(s);
    std::vector<int64_t> perm;
    a_pattern(s, e, nullptr, nullptr, &perm);
    const int64_t nnzA = (int64_t)e.size(), nnzP = (int64_t)pv.size();
    std::vector<double> T((size_t)s.W);
    for (int64_t b = 0; b < nb; b++) {
        const double *pb = path + (size_t)b * s.W * 3;
        const double *cs = corridor_num ? corridor_size + (size_t)b * s.S : nullptr;
        if (!corridor_matches(s, p, pb, cs, corridor_res, T)) return 1;
        time_allocation(s, pb, p->desired_vel, T.data());
        if (seg_time) std::copy(T.begin(), T.end(), seg_time + (size_t)b * s.W);
        std::vector<double> av((size_t)nnzA);
        for (int64_t k = 0; k < nnzA; k++) {
            const AEntry &x = e[(size_t)perm[(size_t)k]];
            if (x.kind == 0) {
                av[(size_t)k] = x.coef;
                continue;
            }
            const int i = x.junction;
            const double dtLeft = T[i + 1] - T[i], dtRight = T[i + 2] - T[i + 1];
            const double dt = x.kind == 1 ? dtRight : dtLeft;
            // velocity rows multiply by dt itself (:432,435), higher orders by pow(dt, k)
            av[(size_t)k] = x.pw == 1 ? x.coef * dt : x.coef * std::pow(dt, x.pw);
        }
        for (int a = 0; a < 3; a++) {
            const int64_t qp = 3 * b + a;
            if (Px) std::copy(pv.begin(), pv.end(), Px + qp * nnzP);
            if (q) std::fill(q + qp * s.n, q + (qp + 1) * s.n, 0.0);
            if (Ax) std::copy(av.begin(), av.end(), Ax + qp * nnzA);
        }
        bounds(s, p, pb, init_vel ? init_vel + 3 * b : nullptr, end_vel ? end_vel + 3 * b : nullptr,
               init_acc ? init_acc + 3 * b : nullptr, end_acc ? end_acc + 3 * b : nullptr, cs,
               l ? l + 3 * b * s.m : nullptr, u ? u + 3 * b * s.m : nullptr);
    }
    return 0;
}

extern "C" int impc_minsnap_build_values(const impc_minsnap_params *p, int64_t nb, int32_t num_waypoints,
                                         const double *path, const double *init_vel, const double *end_vel,
                                         const double *init_acc, const double *end_acc, double *Px, double *q,
                                         double *Ax, double *l, double *u, double *seg_time) {
    return impc_minsnap_corridor_values(p, nb, num_waypoints, path, init_vel, end_vel, init_acc, end_acc, nullptr,
                                        nullptr, 0.0, Px, q, Ax, l, u, seg_time);
}

extern "C" int impc_minsnap_corridor_bounds(const impc_minsnap_params *p, int64_t nb, int32_t num_waypoints,
                                            const double *path, const double *init_vel, const double *end_vel,
                                            const double *init_acc, const double *end_acc,
                                            const int32_t *corridor_num, const double *corridor_size,
                                            double corridor_res, double *l, double *u) {
    Shape s;
    if (!make_shape(p, num_waypoints, corridor_num, &s) || nb < 0 || !path) return 1;
    if (corridor_num && !corridor_size) return 1;
    std::vector<double> T((size_t)s.W);
    for (int64_t b = 0; b < nb; b++) {
        const double *pb = path + (size_t)b * s.W * 3;
        const double *cs = corridor_num ? corridor_size + (size_t)b * s.S : nullptr;
        if (!corridor_matches(s, p, pb, cs, corridor_res, T)) return 1;
        bounds(s, p, pb, init_vel ? init_vel + 3 * b : nullptr, end_vel ? end_vel + 3 * b : nullptr,
               init_acc ? init_acc + 3 * b : nullptr, end_acc ? end_acc + 3 * b : nullptr, cs,
               l ? l + 3 * b * s.m : nullptr, u ? u + 3 * b * s.m : nullptr);
    }
    return 0;
}

extern "C" int impc_minsnap_build_bounds(const impc_minsnap_params *p, int64_t nb, int32_t num_waypoints,
                                         const double *path, const double *init_vel, const double *end_vel,
                                         const double *init_acc, const double *end_acc, double *l, double *u) {
    return impc_minsnap_corridor_bounds(p, nb, num_waypoints, path, init_vel, end_vel, init_acc, end_acc, nullptr,
                                        nullptr, 0.0, l, u);
}

extern "C" int impc_minsnap_unscale(const impc_minsnap_params *p, int64_t nb, int32_t num_waypoints,
                                    const double *seg_time, double *x) {
    Shape s;
    if (!make_shape(p, num_waypoints, nullptr, &s) || nb < 0 || !seg_time || !x) return 1;
    const int D = s.deg + 1;
    for (int64_t b = 0; b < nb; b++) {
        const double *T = seg_time + (size_t)b * s.W;
        for (int a = 0; a < 3; a++) {
            double *xa = x + (3 * b + a) * s.n;
            for (int n = 0; n < s.S; n++)
                for (int d = 0; d <= s.deg; ++d) xa[n * D + d] /= std::pow((T[n + 1] - T[n]), d);  // :873-876
        }
    }
    return 0;
}
