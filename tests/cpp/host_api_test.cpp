// C++ host-layer driver (orb-slam2-noted_amd/host/orbslam2_amd.hpp) used by
// tests/test_host_cpp_gpu.py: reads raw inputs written by the test, runs the reference-named
// classes, writes raw outputs for comparison with the CPU oracle.
//   host_api_test extract <img.u8> <w> <h> <nfeat> <out.bin>
//   host_api_test stereo <left.u8> <right.u8> <w> <h> <nfeat> <mbf> <mb> <out.bin>
//   host_api_test lba <problem.bin> <out.bin>
//   host_api_test pose <edges.bin> <out.bin>
//   host_api_test bow <vocab.txt> <desc.u8> <n> <levelsup> <out.bin>
//   host_api_test newpts <problem.bin> <out.bin>
//   host_api_test concurrent <left.u8> <right.u8> <w> <h> <nfeat> <mbf> <mb> <problem.bin> <rounds> <out.bin>
//     Frame.cc:144-153 + LocalMapping.cc:116-118 concurrency: every round runs the left and right
//     ORBextractor on two std::threads while a third thread keeps running
//     Optimizer::LocalBundleAdjustment; each round's keypoints / descriptors / stereo must equal the
//     serial run's bytes, every LocalBA result is written out for the tolerance check.
#include <atomic>
#include <chrono>
#include <cstdio>
#include <thread>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <iostream>
#include <vector>

#include "orbslam2_amd.hpp"

using namespace orbslam2_amd;

static std::vector<uint8_t> read_file(const char *path) {
    std::ifstream f(path, std::ios::binary);
    return std::vector<uint8_t>((std::istreambuf_iterator<char>(f)), std::istreambuf_iterator<char>());
}

template <class T> static void put(std::ofstream &o, const std::vector<T> &v) {
    const int64_t n = (int64_t)v.size();
    o.write((const char *)&n, 8);
    o.write((const char *)v.data(), sizeof(T) * v.size());
}

static lba_problem read_lba(const std::vector<uint8_t> &b) {
    const int32_t *hdr = (const int32_t *)b.data();
    const int np = hdr[0], nq = hdr[1], ne = hdr[2];
    const uint8_t *p = b.data() + 12;
    lba_problem g{};
    g.n_poses = np; g.n_points = nq; g.n_edges = ne;
    g.pose_id = (const int32_t *)p; p += 4 * np;
    g.pose_fixed = p; p += np; p += (4 - (np % 4)) % 4;
    g.pose_Tcw = (const float *)p; p += 4 * 16 * np;
    g.pose_cam = (const float *)p; p += 4 * 5 * np;
    g.point_id = (const int32_t *)p; p += 4 * nq;
    g.point_Xw = (const float *)p; p += 4 * 3 * nq;
    g.edge_point = (const int32_t *)p; p += 4 * ne;
    g.edge_pose = (const int32_t *)p; p += 4 * ne;
    g.edge_obs = (const float *)p; p += 4 * 3 * ne;
    g.edge_inv_sigma2 = (const float *)p;
    return g;
}

static int run_concurrent(char **argv) {
    auto L = read_file(argv[2]), R = read_file(argv[3]);
    const int w = atoi(argv[4]), h = atoi(argv[5]), nf = atoi(argv[6]);
    const float mbf = (float)atof(argv[7]), mb = (float)atof(argv[8]);
    auto pb = read_file(argv[9]);
    const lba_problem g = read_lba(pb);
    const int rounds = atoi(argv[10]);
    ORBextractor exL(nf, 1.2f, 8, 20, 7), exR(nf, 1.2f, 8, 20, 7);
    // serial reference run
    std::vector<KeyPoint> kL0, kR0;
    std::vector<uint8_t> dL0, dR0;
    exL(ImageU8{L.data(), w, h, w}, kL0, dL0);
    exR(ImageU8{R.data(), w, h, w}, kR0, dR0);
    std::vector<float> u0, z0;
    ComputeStereoMatches(exL, exR, (int)kL0.size(), mbf, mb, u0, z0);
    // LocalMapping thread: LocalBA back to back until the tracking rounds are done
    std::atomic<bool> tracking_done{false};
    std::vector<std::vector<float>> lbaT, lbaX;
    std::vector<std::vector<uint8_t>> lbaE;
    std::string lba_err;
    std::thread mapping([&] {
        try {
            do {
                bool stop = false;
                std::vector<float> T, X;
                std::vector<uint8_t> er;
                Optimizer::LocalBundleAdjustment(g, &stop, T, X, er);
                lbaT.push_back(T); lbaX.push_back(X); lbaE.push_back(er);
            } while (!tracking_done.load() || lbaT.size() < 2);
        } catch (const std::exception &e) { lba_err = e.what(); }
    });
    int mismatches = 0;
    double t_total = 0;
    for (int r = 0; r < rounds; r++) {
        std::vector<KeyPoint> kL, kR;
        std::vector<uint8_t> dL, dR;
        std::string errL, errR;
        const auto t0 = std::chrono::steady_clock::now();
        std::thread tl([&] { try { exL(ImageU8{L.data(), w, h, w}, kL, dL); } catch (const std::exception &e) { errL = e.what(); } });
        std::thread tr([&] { try { exR(ImageU8{R.data(), w, h, w}, kR, dR); } catch (const std::exception &e) { errR = e.what(); } });
        tl.join();
        tr.join();
        if (!errL.empty() || !errR.empty()) throw std::runtime_error("extract thread: " + errL + errR);
        std::vector<float> u, z;
        ComputeStereoMatches(exL, exR, (int)kL.size(), mbf, mb, u, z);
        t_total += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
        const bool same = kL.size() == kL0.size() && kR.size() == kR0.size() &&
                          !std::memcmp(kL.data(), kL0.data(), sizeof(KeyPoint) * kL.size()) &&
                          !std::memcmp(kR.data(), kR0.data(), sizeof(KeyPoint) * kR.size()) && dL == dL0 && dR == dR0 &&
                          !std::memcmp(u.data(), u0.data(), 4 * u.size()) && !std::memcmp(z.data(), z0.data(), 4 * z.size());
        mismatches += !same;
    }
    tracking_done = true;
    mapping.join();
    if (!lba_err.empty()) throw std::runtime_error("LocalBA thread: " + lba_err);
    std::ofstream o(argv[11], std::ios::binary);
    put(o, std::vector<int32_t>{mismatches, rounds, (int32_t)lbaT.size()});
    put(o, std::vector<double>{t_total / rounds});
    for (size_t i = 0; i < lbaT.size(); i++) { put(o, lbaT[i]); put(o, lbaX[i]); put(o, lbaE[i]); }
    return 0;
}

int main(int argc, char **argv) {
    try {
        if (argc >= 12 && !strcmp(argv[1], "concurrent")) return run_concurrent(argv);
        if (argc >= 4 && !strcmp(argv[1], "newpts")) {
            // problem.bin: int32 n1, n2, npairs; float ratio; per keyframe: keys[n], keys_un[n]
            // (28 B), u_right[n], depth[n], 23 floats (Tcw, Ow, fx fy cx cy invfx invfy mb mbf),
            // int32 nlevels, float sf[16], s2[16]; then int32 pairs[npairs][2]
            auto buf = read_file(argv[2]);
            const uint8_t *q = buf.data();
            auto take = [&q](void *dst, size_t bytes) { std::memcpy(dst, q, bytes); q += bytes; };
            int32_t nk[2], np;
            float ratio;
            take(&nk[0], 4); take(&nk[1], 4); take(&np, 4); take(&ratio, 4);
            std::vector<orbx_kp> keys[2], keysUn[2];
            std::vector<float> ur[2], dep[2];
            orbn_keyframe kf[2];
            for (int i = 0; i < 2; i++) {
                const size_t n = (size_t)nk[i];
                keys[i].resize(n); keysUn[i].resize(n); ur[i].resize(n); dep[i].resize(n);
                take(keys[i].data(), sizeof(orbx_kp) * n);
                take(keysUn[i].data(), sizeof(orbx_kp) * n);
                take(ur[i].data(), 4 * n);
                take(dep[i].data(), 4 * n);
                orbn_keyframe &k = kf[i];
                k = orbn_keyframe{};
                k.n = nk[i];
                k.keys = keys[i].data(); k.keys_un = keysUn[i].data(); k.u_right = ur[i].data(); k.depth = dep[i].data();
                float h[23];
                take(h, sizeof h);
                std::memcpy(k.Tcw, h, 48); std::memcpy(k.Ow, h + 12, 12);
                k.fx = h[15]; k.fy = h[16]; k.cx = h[17]; k.cy = h[18]; k.invfx = h[19]; k.invfy = h[20];
                k.mb = h[21]; k.mbf = h[22];
                take(&k.nlevels, 4);
                take(k.scale_factors, 64);
                take(k.level_sigma2, 64);
            }
            std::vector<int32_t> pairs((size_t)np * 2);
            take(pairs.data(), 8 * (size_t)np);
            std::vector<float> x3d;
            std::vector<uint8_t> ok;
            const int nnew = LocalMapping::TriangulateMatches(kf[0], kf[1], pairs, ratio, x3d, ok);
            std::ofstream o(argv[3], std::ios::binary);
            put(o, std::vector<int32_t>{nnew});
            put(o, x3d);
            put(o, ok);
            return 0;
        }
        if (argc >= 7 && !strcmp(argv[1], "extract")) {
            auto img = read_file(argv[2]);
            const int w = atoi(argv[3]), h = atoi(argv[4]), nf = atoi(argv[5]);
            ORBextractor ex(nf, 1.2f, 8, 20, 7);
            std::vector<KeyPoint> kps;
            std::vector<uint8_t> desc;
            ex(ImageU8{img.data(), w, h, w}, kps, desc);
            std::ofstream o(argv[6], std::ios::binary);
            put(o, kps);
            put(o, desc);
            std::vector<float> sf = ex.GetScaleFactors();
            put(o, sf);
            return 0;
        }
        if (argc >= 10 && !strcmp(argv[1], "stereo")) {
            auto L = read_file(argv[2]), R = read_file(argv[3]);
            const int w = atoi(argv[4]), h = atoi(argv[5]), nf = atoi(argv[6]);
            const float mbf = (float)atof(argv[7]), mb = (float)atof(argv[8]);
            ORBextractor exL(nf, 1.2f, 8, 20, 7), exR(nf, 1.2f, 8, 20, 7);
            std::vector<KeyPoint> kL, kR;
            std::vector<uint8_t> dL, dR;
            exL(ImageU8{L.data(), w, h, w}, kL, dL);   // Frame.cc:144-153 (two extractors)
            exR(ImageU8{R.data(), w, h, w}, kR, dR);
            std::vector<float> uR, depth;
            ComputeStereoMatches(exL, exR, (int)kL.size(), mbf, mb, uR, depth);
            std::ofstream o(argv[9], std::ios::binary);
            put(o, uR);
            put(o, depth);
            return 0;
        }
        if (argc >= 4 && !strcmp(argv[1], "lba")) {
            auto b = read_file(argv[2]);
            const lba_problem g = read_lba(b);
            bool stop = false;
            std::vector<float> T, X;
            std::vector<uint8_t> erase;
            Optimizer::LocalBundleAdjustment(g, &stop, T, X, erase);
            std::ofstream o(argv[3], std::ios::binary);
            put(o, T);
            put(o, X);
            put(o, erase);
            return 0;
        }
        if (argc >= 4 && !strcmp(argv[1], "pose")) {
            auto b = read_file(argv[2]);   // int32 n | float Tcw[16] | float cam[5] | Xw[n][3] | obs[n][3] | isg[n]
            const int n = *(const int32_t *)b.data();
            const float *p = (const float *)(b.data() + 4);
            orbp_frame f{};
            f.n = n;
            for (int i = 0; i < 16; i++) f.Tcw[i] = p[i];
            f.fx = p[16]; f.fy = p[17]; f.cx = p[18]; f.cy = p[19]; f.bf = p[20];
            f.Xw = p + 21;
            f.obs = p + 21 + 3 * n;
            f.inv_sigma2 = p + 21 + 6 * n;
            std::vector<float> T(16);
            std::vector<uint8_t> out;
            const int nin = Optimizer::PoseOptimization(f, T.data(), out);
            std::ofstream o(argv[3], std::ios::binary);
            put(o, T);
            put(o, out);
            put(o, std::vector<int32_t>{nin});
            return 0;
        }
        if (argc >= 7 && !strcmp(argv[1], "bow")) {
            ORBVocabulary voc;
            if (!voc.loadFromTextFile(argv[2])) throw std::runtime_error("loadFromTextFile");
            auto d = read_file(argv[3]);
            const int n = atoi(argv[4]), levelsup = atoi(argv[5]);
            BowVector v;
            FeatureVector fv;
            voc.transform(d.data(), n, v, fv, levelsup);
            std::vector<uint32_t> words, nodes;
            std::vector<double> vals;
            std::vector<int32_t> start{0}, feats;
            for (auto &kv : v) { words.push_back(kv.first); vals.push_back(kv.second); }
            for (auto &kv : fv) {
                nodes.push_back(kv.first);
                for (unsigned i : kv.second) feats.push_back((int32_t)i);
                start.push_back((int32_t)feats.size());
            }
            std::ofstream o(argv[6], std::ios::binary);
            put(o, words);
            put(o, vals);
            put(o, nodes);
            put(o, start);
            put(o, feats);
            return 0;
        }
    } catch (const std::exception &e) {
        std::cerr << e.what() << "\n";
        return 2;
    }
    std::cerr << "usage: host_api_test extract|stereo|lba|pose|bow ...\n";
    return 1;
}
