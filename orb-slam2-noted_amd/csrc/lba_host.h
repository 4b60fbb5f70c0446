// Host-side block structure of one LocalBA call (lba.hip's lba_solve; tools/microbench/lba_host_bench.cpp
// times it on the CPU): the active set of SparseOptimizer::initializeOptimization + buildIndexMapping
// (build_active) and the Schur product's tile-pair row lists (build_schur_tiles).
#pragma once
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <vector>

namespace lbaamd_host {

struct HostGraph {
    int np, nq, ne;

    const int32_t *pose_id, *point_id;
    const uint8_t *fixed;
    const int32_t *edge_point, *edge_pose;   // the caller's arrays (lba_problem), validated
};

struct ActiveSet {
    int P = 0, Lm = 0;
    bool mono = false;   // landmark-major order = slot order (lpos_* equal slot_*, pt_items the identity)
    std::vector<int> act, pose_hidx, point_hidx, hpose, hpoint, pt_start, pt_items, ps_start, ps_items, slot_pt, slot_ph,
        slot_ppos, slot_lpos, lpos_ph, lpos_ppos;
    std::vector<int2> tp_ij, tp_nch;     // Schur tile pairs (build_schur_tiles)
    std::vector<int> tp_start, tp_rows;
    std::vector<int4> tp_chunk;
    std::vector<char> scratch_p, scratch_q;
    std::vector<int> scratch_l, scratch_f, scratch_cnt, scratch_tiles, scratch_fill;
    std::vector<unsigned long long> scratch_mask;
};

// Block structure of the Schur product Y Y^T over 16-column tiles: for every upper tile pair
// (I <= J) the Y^T rows (3 per landmark, hessian order) of the landmarks with a free pose in both
// tiles' columns, each list padded to a multiple of 4 rows with the zero row `zero_row`
// (block_solver.hpp:354-439 visits the same pose pairs per landmark). Two passes over the
// landmarks (count, fill); a landmark's tiles come from its free poses' 6-column blocks.
inline void build_schur_tiles(ActiveSet &A, int zero_row, int ksch) {
    const int ntile = std::max(1, (6 * A.P + 15) / 16);
    const int npairs = ntile * (ntile + 1) / 2;
    auto pid = [&](int I, int J) { return I * ntile - I * (I - 1) / 2 + (J - I); };
    A.tp_ij.resize(npairs);
    for (int I = 0; I < ntile; I++)
        for (int J = I; J < ntile; J++) A.tp_ij[pid(I, J)] = make_int2(I, J);
    std::vector<int> &cnt = A.scratch_cnt, &tiles = A.scratch_tiles;
    cnt.assign(npairs + 1, 0);
    if (ntile <= 64) {
        // common case (6P <= 1024): a landmark's tiles as one 64-bit mask, formed once and read by
        // both passes; pairs in (I, J) order, I <= J, like the sorted-list path below
        std::vector<unsigned long long> &mask = A.scratch_mask;
        mask.assign(A.Lm, 0ull);
        // pair id of (I, J), I <= J, as a table (raw pointers below: the stores into the int arrays
        // would otherwise reload every vector's data pointer and counter)
        std::vector<int> &pidt = A.scratch_tiles;
        pidt.assign((size_t)ntile * ntile, 0);
        for (int I = 0; I < ntile; I++)
            for (int J = I; J < ntile; J++) pidt[(size_t)I * ntile + J] = pid(I, J);
        const int *__restrict pt = pidt.data(), *__restrict pts = A.pt_start.data(), *__restrict lph = A.lpos_ph.data();
        unsigned long long *__restrict mk = mask.data();
        int *__restrict cn = cnt.data();
        for (int l = 0; l < A.Lm; l++) {
            unsigned long long m = 0;
            for (int i = pts[l]; i < pts[l + 1]; i++) {
                const int ph = lph[i];   // = slot_ph[pt_items[i]]
                if (ph >= 0) m |= 1ull << (6 * ph / 16) | 1ull << ((6 * ph + 5) / 16);
            }
            mk[l] = m;
            for (unsigned long long ma = m; ma; ma &= ma - 1) {
                const int *row = pt + (size_t)__builtin_ctzll(ma) * ntile;
                for (unsigned long long mb = ma; mb; mb &= mb - 1) cn[row[__builtin_ctzll(mb)]] += 3;
            }
        }
        A.tp_start.assign(npairs + 1, 0);
        for (int p = 0; p < npairs; p++) A.tp_start[p + 1] = A.tp_start[p] + ((cnt[p] + 3) & ~3);
        A.tp_rows.assign(std::max(1, A.tp_start[npairs]), zero_row);
        std::vector<int> &fill = A.scratch_fill;
        fill.assign(A.tp_start.begin(), A.tp_start.end() - 1);
        int *__restrict fl = fill.data(), *__restrict rows = A.tp_rows.data();
        for (int l = 0; l < A.Lm; l++)
            for (unsigned long long ma = mk[l]; ma; ma &= ma - 1) {
                const int *row = pt + (size_t)__builtin_ctzll(ma) * ntile;
                for (unsigned long long mb = ma; mb; mb &= mb - 1) {
                    const int q = row[__builtin_ctzll(mb)];
                    const int f = fl[q];
                    rows[f] = 3 * l;
                    rows[f + 1] = 3 * l + 1;
                    rows[f + 2] = 3 * l + 2;
                    fl[q] = f + 3;
                }
            }
    } else {
    auto point_tiles = [&](int l) {
        tiles.clear();
        for (int i = A.pt_start[l]; i < A.pt_start[l + 1]; i++) {
            const int ph = A.slot_ph[A.pt_items[i]];
            if (ph < 0) continue;
            tiles.push_back(6 * ph / 16);
            tiles.push_back((6 * ph + 5) / 16);
        }
        std::sort(tiles.begin(), tiles.end());
        tiles.erase(std::unique(tiles.begin(), tiles.end()), tiles.end());
    };
    for (int l = 0; l < A.Lm; l++) {
        point_tiles(l);
        for (size_t a = 0; a < tiles.size(); a++)
            for (size_t b = a; b < tiles.size(); b++) cnt[pid(tiles[a], tiles[b])] += 3;
    }
    A.tp_start.assign(npairs + 1, 0);
    for (int p = 0; p < npairs; p++) A.tp_start[p + 1] = A.tp_start[p] + ((cnt[p] + 3) & ~3);
    A.tp_rows.assign(std::max(1, A.tp_start[npairs]), zero_row);
    std::vector<int> &fill = A.scratch_fill;
    fill.assign(A.tp_start.begin(), A.tp_start.end() - 1);
    for (int l = 0; l < A.Lm; l++) {
        point_tiles(l);
        for (size_t a = 0; a < tiles.size(); a++)
            for (size_t b = a; b < tiles.size(); b++) {
                int &f = fill[pid(tiles[a], tiles[b])];
                A.tp_rows[f++] = 3 * l;
                A.tp_rows[f++] = 3 * l + 1;
                A.tp_rows[f++] = 3 * l + 2;
            }
    }
    }
    // chunk workgroups: ksch steps each, at least one per pair (empty pairs still write their tile)
    A.tp_chunk.clear();
    A.tp_nch.assign(npairs, make_int2(0, 0));
    for (int p = 0; p < npairs; p++) {
        const int steps = (A.tp_start[p + 1] - A.tp_start[p]) / 4;
        const int nc = std::max(1, (steps + ksch - 1) / ksch);
        A.tp_nch[p] = make_int2((int)A.tp_chunk.size(), nc);
        for (int c = 0; c < nc; c++) A.tp_chunk.push_back(make_int4(p, c * ksch, std::min(ksch, steps - c * ksch), c));
    }
}

// SparseOptimizer::initializeOptimization(level) + buildIndexMapping + block structure
// Every edge starts at level 0, so the active slots of the first optimize() are all edges in edge
// order (the second reuses them: lba_phase2_mark). The vectors of A keep their capacity from call
// to call (lba_solve's thread_local set).
inline void build_active(const HostGraph &h, ActiveSet &A) {
    const int ne = h.ne;
    A.act.resize(ne);   // slot s = edge s: only the size is used
    std::vector<char> &pa = A.scratch_p, &qa = A.scratch_q;
    pa.assign(h.np, 0);
    qa.assign(h.nq, 0);
    {
        char *__restrict pp = pa.data(), *__restrict qq = qa.data();
        for (int k = 0; k < ne; k++) { pp[h.edge_pose[k]] = 1; qq[h.edge_point[k]] = 1; }
    }
    A.hpose.clear();
    A.hpoint.clear();
    for (int i = 0; i < h.np; i++) if (pa[i] && !h.fixed[i]) A.hpose.push_back(i);
    for (int i = 0; i < h.nq; i++) if (qa[i]) A.hpoint.push_back(i);
    // vertex ids order the hessian (g2o's buildIndexMapping); callers usually pass them sorted
    auto by_id = [](std::vector<int> &v, const int32_t *id) {
        for (size_t i = 1; i < v.size(); i++)
            if (id[v[i]] < id[v[i - 1]]) {
                std::stable_sort(v.begin(), v.end(), [&](int a, int b) { return id[a] < id[b]; });
                return;
            }
    };
    by_id(A.hpose, h.pose_id);
    by_id(A.hpoint, h.point_id);
    A.P = (int)A.hpose.size();
    A.Lm = (int)A.hpoint.size();
    A.pose_hidx.assign(h.np, -1);
    A.point_hidx.assign(h.nq, -1);
    for (int i = 0; i < A.P; i++) A.pose_hidx[A.hpose[i]] = i;
    for (int i = 0; i < A.Lm; i++) A.point_hidx[A.hpoint[i]] = i;
    A.pt_start.assign(A.Lm + 1, 0);
    A.ps_start.assign(A.P + 1, 0);
    const size_t ns = std::max<size_t>(1, (size_t)ne);
    // every entry of these is written by the fill loop below (size only, no initialisation pass)
    A.slot_pt.resize(ns);
    A.slot_ph.resize(ns);
    A.slot_ppos.resize(ns);
    A.slot_lpos.resize(ns);
    A.lpos_ph.resize(ns);
    A.lpos_ppos.resize(ns);
    A.pt_items.resize(ns);
    int *__restrict slot_pt = A.slot_pt.data(), *__restrict slot_ph = A.slot_ph.data();
    const int *__restrict phx = A.pose_hidx.data(), *__restrict qhx = A.point_hidx.data();
    int *__restrict pts = A.pt_start.data(), *__restrict pss = A.ps_start.data();
    // counts, and each slot's (landmark, pose) hessian indices, once; `mono`: the edges come
    // landmark by landmark in hessian order (Optimizer.cc:766-848 adds them map point by map point),
    // so the landmark-major order is the slot order itself
    bool mono = true;
    int prev = -1;
    for (int s = 0; s < ne; s++) {
        const int l = qhx[h.edge_point[s]], ph = phx[h.edge_pose[s]];
        slot_pt[s] = l;
        slot_ph[s] = ph;
        pts[l + 1]++;
        if (ph >= 0) pss[ph + 1]++;
        mono &= l >= prev;
        prev = l;
    }
    for (int l = 0; l < A.Lm; l++) pts[l + 1] += pts[l];
    for (int i = 0; i < A.P; i++) pss[i + 1] += pss[i];
    A.ps_items.resize(std::max(1, pss[A.P]));
    std::vector<int> &fp = A.scratch_f;
    fp.assign(A.P + 1, 0);
    int *__restrict pti = A.pt_items.data(), *__restrict psi = A.ps_items.data(), *__restrict fpp = fp.data();
    int *__restrict slpos = A.slot_lpos.data(), *__restrict lph = A.lpos_ph.data();
    int *__restrict sppos = A.slot_ppos.data(), *__restrict lppos = A.lpos_ppos.data();
    if (ne == 0) { slot_pt[0] = 0; slot_ph[0] = -1; sppos[0] = -1; slpos[0] = 0; lph[0] = -1; lppos[0] = -1; pti[0] = 0; }
    // the pose-major position of every slot (slot order inside a pose)
    for (int s = 0; s < ne; s++) {
        const int ph = slot_ph[s];
        int pp = -1;
        if (ph >= 0) {
            pp = pss[ph] + fpp[ph]++;
            psi[pp] = s;
        }
        sppos[s] = pp;
    }
    A.mono = mono;
    if (mono) {   // landmark-major position = slot
        for (int s = 0; s < ne; s++) {
            pti[s] = s;
            slpos[s] = s;
            lph[s] = slot_ph[s];
            lppos[s] = sppos[s];
        }
    } else {
        std::vector<int> &fl = A.scratch_l;
        fl.assign(A.Lm, 0);
        int *__restrict flp = fl.data();
        for (int s = 0; s < ne; s++) {
            const int l = slot_pt[s];
            const int lpos = pts[l] + flp[l]++;
            pti[lpos] = s;
            slpos[s] = lpos;
            lph[lpos] = slot_ph[s];
            lppos[lpos] = sppos[s];
        }
    }
}


}  // namespace lbaamd_host
