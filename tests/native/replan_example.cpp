// A batched mpcPlanner::makePlanWithPred (reference mpcPlanner.cpp:571-661) for I planning
// instances, in C++ over the C-ABI only -- the integration a planner would write instead of the
// serial candidate loop (:609-628): every candidate of every instance in one grouped solve.
//
//   fan-out       impc_intent_fanout_device      findClosestObstacle + getIntentComb (:663-769)
//   references    impc_repeat_rows_device        each candidate gets its instance's x0, xRef and
//                                                linearisation point (solveTraj arguments)
//   assembly      impc_mpc_build_values_device   castMPCToQP* for the K and K+1 candidate shapes
//   solve         impc_batch_solve_group         OsqpEigen initSolver / setWarmStart / solveProblem
//   selection     impc_fanout_candidates_device  getTrajectoryScore + evaluateTraj (:771-887)
//                 impc_select_best_device
//
// TEST INFRASTRUCTURE: tests/test_replan_pipeline.py writes the inputs of a scenario, runs this
// program on the GPU and compares its outputs bit for bit with impc.replan.DeviceReplan.
//   replan_example <inputs.bin> <outputs.bin>
#include <cstdio>
#include <cstring>
#include <vector>

#include <impc_fanout.h>
#include <impc_mpc.h>
#include <impc_qp.h>
#include <impc_select.h>

#define CK(call)                                                                          \
    do {                                                                                  \
        int rc_ = (call);                                                                 \
        if (rc_) {                                                                        \
            std::fprintf(stderr, "%s failed (%d): %s\n", #call, rc_, impc_last_error()); \
            return 1;                                                                     \
        }                                                                                 \
    } while (0)

namespace {

struct In {
    int32_t I, K, L, N, P;
    impc_mpc_params mp;
    impc_settings st;
    double dyn_safety, static_safety;
    std::vector<double> pos, vel, xref, prev, dyn_cur, pred_pos, pred_size, prob;
    std::vector<int8_t> first_time;
    std::vector<int32_t> prev_count;
};

template <class T>
bool rd(FILE *f, std::vector<T> &v, size_t n) {
    v.resize(n);
    return std::fread(v.data(), sizeof(T), n, f) == n;
}

// device copy of a host vector
struct Dev {
    impc_ctx ctx = nullptr;
    void *p = nullptr;
    int64_t bytes = 0;
    int alloc(impc_ctx c, int64_t b) {
        ctx = c;
        bytes = b;
        return impc_device_alloc(c, b > 0 ? b : 8, &p);
    }
    template <class T>
    int upload(impc_ctx c, const std::vector<T> &v) {
        int rc = alloc(c, (int64_t)(v.size() * sizeof(T)));
        return rc ? rc : impc_copy_to_device(c, p, v.data(), bytes);
    }
    ~Dev() {
        if (p) impc_device_free(ctx, p);
    }
    template <class T>
    T *as() const { return (T *)p; }
};

}  // namespace

int main(int argc, char **argv) {
    if (argc < 3) {
        std::fprintf(stderr, "usage: replan_example <inputs.bin> <outputs.bin>\n");
        return 2;
    }
    In in{};
    FILE *f = std::fopen(argv[1], "rb");
    if (!f) return 2;
    int32_t hdr[5];
    bool ok = std::fread(hdr, sizeof hdr, 1, f) == 1 && std::fread(&in.mp, sizeof in.mp, 1, f) == 1 &&
              std::fread(&in.st, sizeof in.st, 1, f) == 1 && std::fread(&in.dyn_safety, 8, 1, f) == 1 &&
              std::fread(&in.static_safety, 8, 1, f) == 1;
    in.I = hdr[0], in.K = hdr[1], in.L = hdr[2], in.N = hdr[3], in.P = hdr[4];
    const int64_t I = in.I, K = in.K, L = in.L, N = in.N, P = in.P;
    ok = ok && rd(f, in.pos, I * 3) && rd(f, in.vel, I * 3) && rd(f, in.xref, I * N * 8) && rd(f, in.prev, I * P * 8) &&
         rd(f, in.first_time, I) && rd(f, in.prev_count, I) && rd(f, in.dyn_cur, I * K * 3) &&
         rd(f, in.pred_pos, I * K * 4 * L * 3) && rd(f, in.pred_size, I * K * 4 * L * 3) && rd(f, in.prob, I * K * 4);
    std::fclose(f);
    if (!ok) {
        std::fprintf(stderr, "short input file\n");
        return 2;
    }

    impc_ctx ctx = nullptr;
    CK(impc_ctx_create(0, &ctx));
    Dev pos, vel, xref, prev, ft, pc, dcur, ppos, psize, prob;
    CK(pos.upload(ctx, in.pos));
    CK(vel.upload(ctx, in.vel));
    CK(xref.upload(ctx, in.xref));
    CK(prev.upload(ctx, in.prev));
    CK(ft.upload(ctx, in.first_time));
    CK(pc.upload(ctx, in.prev_count));
    CK(dcur.upload(ctx, in.dyn_cur));
    CK(ppos.upload(ctx, in.pred_pos));
    CK(psize.upload(ctx, in.pred_size));
    CK(prob.upload(ctx, in.prob));

    // ---- fan-out: the six candidate obstacle sets of every instance
    Dev ob_idx, cand_type, cand_slot, closest_prob, single_pos, single_size, pair_pos, pair_size;
    CK(ob_idx.alloc(ctx, I * 4));
    CK(cand_type.alloc(ctx, I * 6 * 4));
    CK(cand_slot.alloc(ctx, I * 6 * 4));
    CK(closest_prob.alloc(ctx, I * 4 * 8));
    CK(single_pos.alloc(ctx, I * 4 * K * L * 3 * 8));
    CK(single_size.alloc(ctx, I * 4 * K * L * 3 * 8));
    CK(pair_pos.alloc(ctx, I * 2 * (K + 1) * L * 3 * 8));
    CK(pair_size.alloc(ctx, I * 2 * (K + 1) * L * 3 * 8));
    CK(impc_intent_fanout_device(ctx, I, (int32_t)K, (int32_t)L, (int32_t)P, pos.as<double>(), ft.as<int8_t>(),
                                 prev.as<double>(), pc.as<int32_t>(), dcur.as<double>(), ppos.as<double>(),
                                 psize.as<double>(), prob.as<double>(), ob_idx.as<int32_t>(), cand_type.as<int32_t>(),
                                 cand_slot.as<int32_t>(), closest_prob.as<double>(), single_pos.as<double>(),
                                 single_size.as<double>(), pair_pos.as<double>(), pair_size.as<double>(), nullptr));

    // ---- two candidate shapes: 4 single-intent candidates (K obstacles), 2 two-intent (K + 1)
    struct Shape {
        int32_t K, cnt;
        int64_t nb, n, m;
        impc_mpc_builder bld = nullptr;
        impc_batch batch = nullptr;
        Dev rpos, rvel, rxref, rprev, Px, q, Ax, l, u;
    } sh[2];
    sh[0].K = (int32_t)K, sh[0].cnt = 4;
    sh[1].K = (int32_t)K + 1, sh[1].cnt = 2;
    for (Shape &s : sh) {
        s.nb = I * s.cnt;
        impc_qp_dims dm{};
        CK(impc_mpc_dims(&in.mp, 0, s.K, &dm));
        s.n = dm.n, s.m = dm.m;
        std::vector<int64_t> Pp(dm.n + 1), Pi(dm.nnzP > 0 ? dm.nnzP : 1), Ap(dm.n + 1), Ai(dm.nnzA);
        CK(impc_mpc_build_pattern(&in.mp, 0, s.K, Pp.data(), Pi.data(), Ap.data(), Ai.data()));
        CK(impc_batch_create(ctx, dm.n, dm.m, Pp.data(), Pi.data(), Ap.data(), Ai.data(), s.nb, &s.batch));
        CK(impc_batch_set_settings(s.batch, &in.st));
        CK(impc_mpc_builder_create(ctx, &in.mp, 0, s.K, (int32_t)L, &s.bld));
        // every candidate of an instance is linearised at, and warm-started from, the same plan
        CK(s.rpos.alloc(ctx, s.nb * 3 * 8));
        CK(s.rvel.alloc(ctx, s.nb * 3 * 8));
        CK(s.rxref.alloc(ctx, s.nb * N * 8 * 8));
        CK(s.rprev.alloc(ctx, s.nb * P * 8 * 8));
        CK(impc_repeat_rows_device(ctx, pos.p, I, 3 * 8, s.cnt, s.rpos.p, nullptr));
        CK(impc_repeat_rows_device(ctx, vel.p, I, 3 * 8, s.cnt, s.rvel.p, nullptr));
        CK(impc_repeat_rows_device(ctx, xref.p, I, N * 8 * 8, s.cnt, s.rxref.p, nullptr));
        CK(impc_repeat_rows_device(ctx, prev.p, I, P * 8 * 8, s.cnt, s.rprev.p, nullptr));
        CK(s.Px.alloc(ctx, s.nb * dm.nnzP * 8));
        CK(s.q.alloc(ctx, s.nb * dm.n * 8));
        CK(s.Ax.alloc(ctx, s.nb * dm.nnzA * 8));
        CK(s.l.alloc(ctx, s.nb * dm.m * 8));
        CK(s.u.alloc(ctx, s.nb * dm.m * 8));
        const double *dp = s.cnt == 4 ? single_pos.as<double>() : pair_pos.as<double>();
        const double *ds = s.cnt == 4 ? single_size.as<double>() : pair_size.as<double>();
        CK(impc_mpc_build_values_device(s.bld, s.nb, s.rpos.as<double>(), s.rvel.as<double>(), s.rxref.as<double>(),
                                        s.rprev.as<double>(), nullptr, nullptr, nullptr, dp, ds, s.Px.as<double>(),
                                        s.q.as<double>(), s.Ax.as<double>(), s.l.as<double>(), s.u.as<double>(),
                                        nullptr));
        CK(impc_batch_set_values_device(s.batch, s.Px.as<double>(), s.q.as<double>(), s.Ax.as<double>(),
                                        s.l.as<double>(), s.u.as<double>()));
        // solveTraj's warm start (:485-509): the previous plan's states, zero controls
        std::vector<double> xws((size_t)(s.nb * dm.n), 0.0);
        for (int64_t b = 0; b < s.nb; b++)
            std::memcpy(&xws[(size_t)(b * dm.n)], &in.prev[(size_t)((b / s.cnt) * P * 8)], sizeof(double) * 8 * N);
        CK(impc_batch_warm_start(s.batch, xws.data(), nullptr));
    }
    impc_batch group[2] = {sh[0].batch, sh[1].batch};
    CK(impc_batch_solve_group(group, 2, nullptr));

    // ---- selection on the device
    double *xs[2];
    for (int k = 0; k < 2; k++) CK(impc_batch_device_results(sh[k].batch, &xs[k], nullptr, nullptr));
    Dev x_cand, dyn_count, dyn_pos, dyn_size, valid, best_cand, best_pos, scores, weighted;
    CK(x_cand.alloc(ctx, I * 6 * 8));
    CK(dyn_count.alloc(ctx, I * 6 * 4));
    CK(dyn_pos.alloc(ctx, I * 6 * (K + 1) * L * 3 * 8));
    CK(dyn_size.alloc(ctx, I * 6 * (K + 1) * L * 3 * 8));
    CK(valid.upload(ctx, std::vector<int8_t>((size_t)(I * 6), 1)));
    CK(best_cand.alloc(ctx, I * 4));
    CK(best_pos.alloc(ctx, I * 4));
    CK(scores.alloc(ctx, I * 6 * 3 * 8));
    CK(weighted.alloc(ctx, I * 6 * 8));
    CK(impc_fanout_candidates_device(ctx, I, (int32_t)K, (int32_t)L, cand_slot.as<int32_t>(), single_pos.as<double>(),
                                     single_size.as<double>(), pair_pos.as<double>(), pair_size.as<double>(), xs[0],
                                     sh[0].n, xs[1], sh[1].n, x_cand.as<const double *>(), dyn_count.as<int32_t>(),
                                     dyn_pos.as<double>(), dyn_size.as<double>(), nullptr));
    impc_select_params sp{};
    sp.horizon = (int32_t)N, sp.num_candidates = 6, sp.max_dynamic = (int32_t)K + 1, sp.pred_len = (int32_t)L;
    sp.num_static = 0, sp.prev_len = (int32_t)P;
    sp.dynamic_safety_dist = in.dyn_safety, sp.static_safety_dist = in.static_safety;
    CK(impc_select_best_device(ctx, &sp, I, x_cand.as<const double *const>(), valid.as<int8_t>(), ft.as<int8_t>(),
                               prev.as<double>(), pc.as<int32_t>(), xref.as<double>(), nullptr, nullptr,
                               dyn_count.as<int32_t>(), dyn_pos.as<double>(), dyn_size.as<double>(),
                               closest_prob.as<double>(), best_cand.as<int32_t>(), best_pos.as<int32_t>(),
                               scores.as<double>(), weighted.as<double>(), nullptr));

    // ---- outputs: best candidate per instance, then both shapes' solutions and statuses
    std::vector<int32_t> best((size_t)I);
    CK(impc_copy_to_host(ctx, best.data(), best_cand.p, I * 4));
    FILE *o = std::fopen(argv[2], "wb");
    if (!o) return 2;
    std::fwrite(best.data(), 4, best.size(), o);
    for (Shape &s : sh) {
        std::vector<double> x((size_t)(s.nb * s.n));
        std::vector<impc_info> info((size_t)s.nb);
        CK(impc_batch_get(s.batch, x.data(), nullptr, info.data()));
        std::fwrite(x.data(), 8, x.size(), o);
        for (const impc_info &r : info) std::fwrite(&r.iter, 8, 1, o);
    }
    std::fclose(o);
    for (Shape &s : sh) {
        impc_batch_destroy(s.batch);
        impc_mpc_builder_destroy(s.bld);
    }
    std::printf("replan_example: %lld instances, best candidates written\n", (long long)I);
    return 0;
}
