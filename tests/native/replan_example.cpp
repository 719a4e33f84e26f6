// The batched mpcPlanner::makePlanWithPred (reference mpcPlanner.cpp:571-661) as a C++ planner
// would drive it: one impc_replan object for I planning instances, R chained replans, each ONE
// library call (impc_replan_run) -- branch table, fan-out, assembly, grouped solve, validity,
// selection and commit on the device -- followed by the vehicle following its plan
// (impc_replan_advance_device: currPos / currVel = getPos(dt) / getVel(dt), mpc_node.cpp:216-224)
// and the obstacle predictions moving one step on (the predictor's next output; here the
// previous prediction shifted by one step, as tests/test_replan_branches.py does).
//
// What mpcNavigation.cpp:316-322 calls once per instance per replan becomes:
//     impc_replan_run(rp, &inputs);                        // every instance, one call
//     impc_replan_advance_device(rp, dt, d_pos, d_vel);    // the next x0, on the device
//
// TEST INFRASTRUCTURE: tests/test_replan_native.py writes a scenario, runs this program on the GPU
// and checks every replan against the restatement oracle/replan_ref.py.  After each replan the
// program dumps (outside the timed call) the branch table, the selection, the committed state and
// each shape's QPs and solutions.
//   replan_example <inputs.bin> <outputs.bin>
// inputs.bin: int32 I, K, L, N, R, P, S; impc_mpc_params; impc_settings; pos [I][3], vel [I][3],
// xref [I][N][8], prev [I][N][8], first_time int8 [I], dyn/pred_pos [I][K][4][L][3], pred_size
// [I][K][4][L][3], prob [I][K][4], cur_size [I][K][3], cur_count int32 [I], has_pred int8 [R][I],
// when P = 1 num_pred int32 [R][I] (each instance's obstacle count per replan), and when S > 0
// each instance's S static obstacles (getStaticObstacles): centroid [I][S][3], size [I][S][3],
// yaw [I][S].
#include <chrono>
#include <cstdio>
#include <cstring>
#include <vector>

#include <impc_mpc.h>
#include <impc_qp.h>
#include <impc_replan.h>

#define CK(call)                                                                          \
    do {                                                                                  \
        int rc_ = (call);                                                                 \
        if (rc_) {                                                                        \
            std::fprintf(stderr, "%s failed (%d): %s\n", #call, rc_, impc_last_error()); \
            return 1;                                                                     \
        }                                                                                 \
    } while (0)

namespace {

template <class T>
bool rd(FILE *f, std::vector<T> &v, size_t n) {
    v.resize(n);
    return std::fread(v.data(), sizeof(T), n, f) == n;
}

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
        int rc = p ? 0 : alloc(c, (int64_t)(v.size() * sizeof(T)));
        return rc ? rc : impc_copy_to_device(c, p, v.data(), (int64_t)(v.size() * sizeof(T)));
    }
    ~Dev() {
        if (p) impc_device_free(ctx, p);
    }
    template <class T>
    T *as() const { return (T *)p; }
};

template <class T>
void put(FILE *o, const void *src_dev, int64_t count, impc_ctx ctx) {
    std::vector<T> h((size_t)count);
    if (count) impc_copy_to_host(ctx, h.data(), src_dev, count * (int64_t)sizeof(T));
    std::fwrite(h.data(), sizeof(T), h.size(), o);
}

}  // namespace

int main(int argc, char **argv) {
    if (argc < 3) {
        std::fprintf(stderr, "usage: replan_example <inputs.bin> <outputs.bin>\n");
        return 2;
    }
    FILE *f = std::fopen(argv[1], "rb");
    if (!f) return 2;
    int32_t hdr[7];
    impc_mpc_params mp{};
    impc_settings st{};
    bool ok = std::fread(hdr, sizeof hdr, 1, f) == 1 && std::fread(&mp, sizeof mp, 1, f) == 1 &&
              std::fread(&st, sizeof st, 1, f) == 1;
    const int64_t I = hdr[0], K = hdr[1], L = hdr[2], N = hdr[3], R = hdr[4], P = hdr[5], S = hdr[6];
    std::vector<double> pos, vel, xref, prev, pred, psize, prob, csize, scen, ssize, syaw;
    std::vector<int8_t> first, has_pred;
    std::vector<int32_t> ccount, npred;
    ok = ok && rd(f, pos, I * 3) && rd(f, vel, I * 3) && rd(f, xref, I * N * 8) && rd(f, prev, I * N * 8) &&
         rd(f, first, I) && rd(f, pred, I * K * 4 * L * 3) && rd(f, psize, I * K * 4 * L * 3) && rd(f, prob, I * K * 4) &&
         rd(f, csize, I * K * 3) && rd(f, ccount, I) && rd(f, has_pred, R * I) && (!P || rd(f, npred, R * I)) &&
         (!S || (rd(f, scen, I * S * 3) && rd(f, ssize, I * S * 3) && rd(f, syaw, I * S)));
    std::fclose(f);
    if (!ok || mp.horizon != N) {
        std::fprintf(stderr, "short or inconsistent input file\n");
        return 2;
    }
    const int64_t n = 13 * N - 5;

    impc_ctx ctx = nullptr;
    CK(impc_ctx_create(0, &ctx));
    impc_replan_config cfg{};
    cfg.instances = I, cfg.num_obstacles = (int32_t)K, cfg.pred_len = (int32_t)L;
    cfg.mpc = mp;
    cfg.settings = st;
    cfg.issue_cutoff_s = 0.15;  // makePlanWithPred (:613)
    cfg.queue_order = IMPC_QUEUE_FIFO;
    cfg.num_static = (int32_t)S;  // obclustering_->getStaticObstacles() per instance (:594)
    impc_replan rp = nullptr;
    CK(impc_replan_create(ctx, &cfg, &rp));
    // the planner state the scenario starts from: plan_x = previous states, zero controls
    std::vector<double> plan((size_t)(I * n), 0.0);
    for (int64_t i = 0; i < I; i++) std::memcpy(&plan[(size_t)(i * n)], &prev[(size_t)(i * N * 8)], 8 * 8 * N);
    CK(impc_replan_set_state(rp, plan.data(), first.data()));

    Dev d_pos, d_vel, d_xref, d_dcur, d_pred, d_psize, d_prob, d_csize, d_ccount, d_hp, d_np, d_scen, d_ssize, d_syaw;
    CK(d_pos.upload(ctx, pos));
    CK(d_vel.upload(ctx, vel));
    CK(d_xref.upload(ctx, xref));
    CK(d_psize.upload(ctx, psize));
    CK(d_prob.upload(ctx, prob));
    CK(d_csize.upload(ctx, csize));
    CK(d_ccount.upload(ctx, ccount));
    if (S) {
        CK(d_scen.upload(ctx, scen));
        CK(d_ssize.upload(ctx, ssize));
        CK(d_syaw.upload(ctx, syaw));
    }
    FILE *o = std::fopen(argv[2], "wb");
    if (!o) return 2;
    double call_s = 0.0;
    for (int64_t r = 0; r < R; r++) {
        // the obstacles' current positions = the predictions' first step (predPos[.][0][0])
        std::vector<double> dcur((size_t)(I * K * 3));
        for (int64_t ik = 0; ik < I * K; ik++)
            for (int c = 0; c < 3; c++) dcur[(size_t)(3 * ik + c)] = pred[(size_t)(ik * 4 * L * 3 + c)];
        CK(d_dcur.upload(ctx, dcur));
        CK(d_pred.upload(ctx, pred));
        std::vector<int8_t> hp(has_pred.begin() + r * I, has_pred.begin() + (r + 1) * I);
        CK(d_hp.upload(ctx, hp));
        if (P) {
            std::vector<int32_t> np(npred.begin() + r * I, npred.begin() + (r + 1) * I);
            CK(d_np.upload(ctx, np));
        }
        impc_replan_inputs in{};
        in.pos = d_pos.as<double>(), in.vel = d_vel.as<double>(), in.xref = d_xref.as<double>();
        in.dyn_cur = d_dcur.as<double>(), in.pred_pos = d_pred.as<double>(), in.pred_size = d_psize.as<double>();
        in.prob = d_prob.as<double>(), in.has_pred = d_hp.as<int8_t>();
        in.cur_size = d_csize.as<double>(), in.cur_count = d_ccount.as<int32_t>();
        in.num_pred = P ? d_np.as<int32_t>() : nullptr;
        if (S) in.st_centroid = d_scen.as<double>(), in.st_size = d_ssize.as<double>(), in.st_yaw = d_syaw.as<double>();
        in.solver_time_limit = 0.0;
        CK(impc_ctx_synchronize(ctx));
        const auto t0 = std::chrono::steady_clock::now();
        CK(impc_replan_run(rp, &in));
        CK(impc_ctx_synchronize(ctx));
        call_s += std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();

        // ---- dump this replan (test output; not part of the planner's call)
        impc_replan_view v{};
        CK(impc_replan_view_device(rp, &v));
        put<int8_t>(o, v.branch, I, ctx);
        put<int32_t>(o, v.best_cand, I, ctx);
        put<int32_t>(o, v.ob_idx, I, ctx);
        put<int32_t>(o, v.cand_type, 6 * I, ctx);
        put<int32_t>(o, v.cand_slot, 6 * I, ctx);
        put<double>(o, v.plan_x, I * n, ctx);
        put<int8_t>(o, v.first_time, I, ctx);
        put<int32_t>(o, v.prev_count, I, ctx);
        put<int8_t>(o, v.valid, I, ctx);
        put<int32_t>(o, v.num_obs, I, ctx);
        put<int32_t>(o, v.slot_row, 6 * I, ctx);
        put<int32_t>(o, v.shape, I, ctx);
        // shape s: the QPs with s dynamic-obstacle rows per stage; K + 2: the first plans with statics
        for (int32_t s = 0; s < (int32_t)K + 2 + (S ? 1 : 0); s++) {
            impc_batch b = nullptr;
            int64_t cnt = 0;
            const int32_t *rinst = nullptr;
            const int8_t *rcode = nullptr;
            const double *vals[5] = {};
            CK(impc_replan_shape(rp, s, &b, &cnt, &rinst, &rcode, &vals[0], &vals[1], &vals[2], &vals[3], &vals[4]));
            std::fwrite(&cnt, 8, 1, o);
            if (!cnt) continue;
            put<int32_t>(o, rinst, cnt, ctx);
            put<int8_t>(o, rcode, cnt, ctx);
            impc_batch_stats bs{};
            CK(impc_batch_get_stats(b, &bs));
            std::vector<double> x((size_t)(bs.batch * bs.n)), y((size_t)(bs.batch * bs.m));
            std::vector<impc_info> info((size_t)bs.batch);
            CK(impc_batch_get(b, x.data(), y.data(), info.data()));
            const int64_t dims[4] = {bs.n, bs.m, bs.nnzP, bs.nnzA};
            std::fwrite(dims, 8, 4, o);
            std::fwrite(x.data(), 8, (size_t)(cnt * bs.n), o);
            std::fwrite(y.data(), 8, (size_t)(cnt * bs.m), o);
            std::fwrite(info.data(), sizeof(impc_info), (size_t)cnt, o);
            const int64_t len[5] = {bs.nnzP, bs.n, bs.nnzA, bs.m, bs.m};
            for (int k = 0; k < 5; k++) put<double>(o, vals[k], cnt * len[k], ctx);
        }

        // ---- the vehicle follows its plan; the predictions move one step on
        CK(impc_replan_advance_device(rp, mp.ts, d_pos.as<double>(), d_vel.as<double>()));
        for (int64_t ikm = 0; ikm < I * K * 4; ikm++) {
            double *row = &pred[(size_t)(ikm * L * 3)];
            std::memmove(row, row + 3, sizeof(double) * 3 * (L - 1));  // step s <- s + 1, the last kept
        }
    }
    std::fclose(o);
    impc_replan_stats rs{};
    CK(impc_replan_get_stats(rp, &rs));
    CK(impc_replan_destroy(rp));
    CK(impc_ctx_destroy(ctx));
    std::printf("replan_example: %lld instances, %lld chained replans, %.3f ms per impc_replan_run call\n",
                (long long)I, (long long)R, 1e3 * call_s / (double)R);
    return 0;
}
