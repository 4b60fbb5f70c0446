// CPU timing of LocalBA's per-call host structure build (lba_host.h: build_active +
// build_schur_tiles) on a C4-shaped graph: 22 keyframes (2 fixed), 3000 map points with 3-10
// observations each in point order, as tools/synth localba_problem lays them out.
//   hipcc -O3 -I orb-slam2-noted_amd/csrc tools/microbench/lba_host_bench.cpp -o /tmp/lba_host_bench
#include "lba_host.h"

#include <chrono>
#include <cstdio>
#include <random>

using namespace lbaamd_host;

int main(int argc, char **argv) {
    const int reps = argc > 1 ? std::atoi(argv[1]) : 200;
    const int n_kf = 20, np = n_kf + 2, nq = 3000;
    std::mt19937 rng(4);
    std::vector<int32_t> pose_id(np), point_id(nq), ep, eq;
    std::vector<uint8_t> fixed(np, 0);
    fixed[0] = fixed[np - 1] = 1;
    for (int i = 0; i < np; i++) pose_id[i] = i;
    for (int i = 0; i < nq; i++) point_id[i] = np + i;
    for (int p = 0; p < nq; p++) {
        const int k = 3 + (int)(rng() % 6), first = 1 + (int)(rng() % (n_kf - k + 1));
        std::vector<int> run;
        if (first == 1 && rng() % 2) run.push_back(0);
        for (int j = 0; j < k; j++) run.push_back(first + j);
        if (run.back() == n_kf && rng() % 2) run.push_back(n_kf + 1);
        for (int kf : run) { ep.push_back(kf); eq.push_back(p); }
    }
    HostGraph h{};
    h.np = np; h.nq = nq; h.ne = (int)ep.size();
    h.pose_id = pose_id.data(); h.point_id = point_id.data(); h.fixed = fixed.data();
    h.edge_point = eq.data(); h.edge_pose = ep.data();
    ActiveSet A;
    double t_act = 0, t_til = 0, m_act = 1e30, m_til = 1e30;   // mean and minimum per call
    size_t check = 0;
    for (int r = 0; r < reps + 10; r++) {
        const auto t0 = std::chrono::steady_clock::now();
        build_active(h, A);
        const auto t1 = std::chrono::steady_clock::now();
        build_schur_tiles(A, std::max(4, ((3 * A.Lm + 3) / 4) * 4), 64);
        const auto t2 = std::chrono::steady_clock::now();
        if (r >= 10) {
            const double a = std::chrono::duration<double, std::micro>(t1 - t0).count();
            const double b = std::chrono::duration<double, std::micro>(t2 - t1).count();
            t_act += a;
            t_til += b;
            m_act = std::min(m_act, a);
            m_til = std::min(m_til, b);
        }
        check += A.tp_rows.size() + A.pt_items[A.pt_items.size() / 2];
    }
    std::printf("{\"edges\": %d, \"P\": %d, \"Lm\": %d, \"pairs\": %zu, \"tp_rows\": %zu, \"chunks\": %zu, "
                "\"build_active_us\": %.1f, \"build_schur_tiles_us\": %.1f, \"min_build_active_us\": %.1f, "
                "\"min_build_schur_tiles_us\": %.1f, \"check\": %zu}\n",
                h.ne, A.P, A.Lm, A.tp_ij.size(), A.tp_rows.size(), A.tp_chunk.size(), t_act / reps, t_til / reps, m_act,
                m_til, check);
    return 0;
}
