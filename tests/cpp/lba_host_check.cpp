// Invariants of LocalBA's host structure build (orb-slam2-noted_amd/csrc/lba_host.h) on graphs in
// landmark-major edge order (the fast path) and shuffled order, with unsorted vertex ids and fixed
// poses: the hessian order is the id order of the used, non-fixed vertices (buildIndexMapping),
// pt_items / ps_items list every slot of a landmark / pose in slot order, the inverse maps and the
// lpos arrays agree, and every Schur tile pair lists exactly the landmarks seen from both tiles,
// in landmark order, padded to 4 rows. Prints "ok <graphs>" or the first violation.
#include "lba_host.h"

#include <cstdio>
#include <random>
#include <set>

using namespace lbaamd_host;

static int fail(const char *what, int g) {
    std::printf("FAIL graph %d: %s\n", g, what);
    return 1;
}

int main() {
    int graphs = 0;
    for (int g = 0; g < 8; g++) {
        std::mt19937 rng(100 + g);
        const int n_kf = 6 + 5 * g, np = n_kf + 2, nq = 200 + 400 * g;
        std::vector<int32_t> pose_id(np), point_id(nq), ep, eq;
        std::vector<uint8_t> fixed(np, 0);
        fixed[0] = fixed[np - 1] = 1;
        if (g & 2) fixed[np / 2] = 1;
        for (int i = 0; i < np; i++) pose_id[i] = (g & 4) ? 1000 - 7 * i : i;
        for (int i = 0; i < nq; i++) point_id[i] = (g & 4) ? 900000 - 3 * i : np + i;
        for (int p = 0; p < nq; p++) {
            if (g == 7 && p % 13 == 0) continue;   // unobserved points
            const int k = 2 + (int)(rng() % 6), first = (int)(rng() % (np - k));
            for (int j = 0; j < k; j++) { ep.push_back(first + j); eq.push_back(p); }
        }
        if (g & 1)
            for (size_t i = ep.size() - 1; i > 0; i--) {
                const size_t j = rng() % (i + 1);
                std::swap(ep[i], ep[j]);
                std::swap(eq[i], eq[j]);
            }
        HostGraph h{};
        h.np = np; h.nq = nq; h.ne = (int)ep.size();
        h.pose_id = pose_id.data(); h.point_id = point_id.data(); h.fixed = fixed.data();
        h.edge_point = eq.data(); h.edge_pose = ep.data();
        ActiveSet A;
        build_active(h, A);
        const int ne = h.ne;
        // hessian order: used vertices, poses without the fixed ones, by id
        std::vector<int> used_p(np, 0), used_q(nq, 0);
        for (int k = 0; k < ne; k++) { used_p[ep[k]] = 1; used_q[eq[k]] = 1; }
        std::vector<int> hp, hq;
        for (int i = 0; i < np; i++) if (used_p[i] && !fixed[i]) hp.push_back(i);
        for (int i = 0; i < nq; i++) if (used_q[i]) hq.push_back(i);
        std::stable_sort(hp.begin(), hp.end(), [&](int a, int b) { return pose_id[a] < pose_id[b]; });
        std::stable_sort(hq.begin(), hq.end(), [&](int a, int b) { return point_id[a] < point_id[b]; });
        if (A.hpose != hp || A.hpoint != hq) return fail("hessian order", g);
        if (A.mono != (g % 2 == 0 && !(g & 4))) return fail("landmark-major detection", g);
        for (int s = 0; s < ne; s++) {
            const int l = A.point_hidx[eq[s]], ph = A.pose_hidx[ep[s]];
            if (A.slot_pt[s] != l || A.slot_ph[s] != ph) return fail("slot indices", g);
            const int lpos = A.slot_lpos[s];
            if (lpos < A.pt_start[l] || lpos >= A.pt_start[l + 1] || A.pt_items[lpos] != s) return fail("landmark CSR", g);
            if (A.lpos_ph[lpos] != ph || A.lpos_ppos[lpos] != A.slot_ppos[s]) return fail("lpos arrays", g);
            if (ph >= 0) {
                const int pp = A.slot_ppos[s];
                if (pp < A.ps_start[ph] || pp >= A.ps_start[ph + 1] || A.ps_items[pp] != s) return fail("pose CSR", g);
            } else if (A.slot_ppos[s] != -1) return fail("fixed pose position", g);
        }
        for (int l = 0; l < A.Lm; l++)
            for (int i = A.pt_start[l] + 1; i < A.pt_start[l + 1]; i++)
                if (A.pt_items[i] <= A.pt_items[i - 1]) return fail("slot order inside a landmark", g);
        for (int p = 0; p < A.P; p++)
            for (int i = A.ps_start[p] + 1; i < A.ps_start[p + 1]; i++)
                if (A.ps_items[i] <= A.ps_items[i - 1]) return fail("slot order inside a pose", g);
        const int zero_row = std::max(4, ((3 * A.Lm + 3) / 4) * 4);
        build_schur_tiles(A, zero_row, 64);
        const int ntile = std::max(1, (6 * A.P + 15) / 16);
        for (size_t q = 0; q < A.tp_ij.size(); q++) {
            const int I = A.tp_ij[q].x, J = A.tp_ij[q].y;
            std::vector<int> want;
            for (int l = 0; l < A.Lm; l++) {
                std::set<int> t;
                for (int i = A.pt_start[l]; i < A.pt_start[l + 1]; i++) {
                    const int ph = A.slot_ph[A.pt_items[i]];
                    if (ph >= 0) { t.insert(6 * ph / 16); t.insert((6 * ph + 5) / 16); }
                }
                if (t.count(I) && t.count(J)) { want.push_back(3 * l); want.push_back(3 * l + 1); want.push_back(3 * l + 2); }
            }
            while (want.size() % 4) want.push_back(zero_row);
            const std::vector<int> got(A.tp_rows.begin() + A.tp_start[q], A.tp_rows.begin() + A.tp_start[q + 1]);
            if (I > J || J >= ntile || got != want) return fail("tile pair rows", g);
        }
        graphs++;
    }
    std::printf("ok %d\n", graphs);
    return 0;
}
