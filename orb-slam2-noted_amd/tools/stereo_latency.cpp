// Drop-in latency of the stereo Frame constructor's hot path (SURVEY.md §8d latency mode):
// per frame, exactly as Frame::Frame(imLeft, imRight, ...) runs it (Frame.cc:144-153, 176-178):
//   std::thread threadLeft(&Frame::ExtractORB, this, 0, imLeft);
//   std::thread threadRight(&Frame::ExtractORB, this, 1, imRight);
//   threadLeft.join(); threadRight.join();
//   ... ComputeStereoMatches();
// with host images in and host keypoints / descriptors / mvuRight / mvDepth out, through the C++
// host layer (orbslam2_amd.hpp) over the C-ABI. `serial` runs L then R on the calling thread.
//   stereo_latency <pairs.u8> <n_pairs> <w> <h> <nfeat> <mbf> <mb> <warmup> <frames> <threads|serial>
// Prints one JSON line: per-frame wall time median / mean / p10 / p90 / min / max (ms).
#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <iostream>
#include <thread>
#include <vector>

#include "orbslam2_amd.hpp"

using namespace orbslam2_amd;

int main(int argc, char **argv) {
    if (argc < 11) {
        std::cerr << "usage: stereo_latency <pairs.u8> <n_pairs> <w> <h> <nfeat> <mbf> <mb> <warmup> <frames> <threads|serial>\n";
        return 1;
    }
    try {
        std::ifstream f(argv[1], std::ios::binary);
        std::vector<uint8_t> pool((std::istreambuf_iterator<char>(f)), std::istreambuf_iterator<char>());
        const int np = atoi(argv[2]), w = atoi(argv[3]), h = atoi(argv[4]), nf = atoi(argv[5]);
        const float mbf = (float)atof(argv[6]), mb = (float)atof(argv[7]);
        const int warmup = atoi(argv[8]), frames = atoi(argv[9]);
        const bool threads = !strcmp(argv[10], "threads");
        const size_t img = (size_t)w * h;
        if (np <= 0 || pool.size() < 2 * img * np) throw std::runtime_error("short pairs file");
        ORBextractor exL(nf, 1.2f, 8, 20, 7), exR(nf, 1.2f, 8, 20, 7);   // Tracking.cc:177-190
        std::vector<double> ms;
        long long kp_total = 0, match_total = 0;
        for (int t = 0; t < warmup + frames; t++) {
            const uint8_t *L = pool.data() + 2 * img * (t % np), *R = L + img;
            std::vector<KeyPoint> kL, kR;
            std::vector<uint8_t> dL, dR;
            std::vector<float> uR, depth;
            const auto t0 = std::chrono::steady_clock::now();
            if (threads) {
                std::string eL, eR;
                std::thread tl([&] { try { exL(ImageU8{L, w, h, w}, kL, dL); } catch (const std::exception &e) { eL = e.what(); } });
                std::thread tr([&] { try { exR(ImageU8{R, w, h, w}, kR, dR); } catch (const std::exception &e) { eR = e.what(); } });
                tl.join();
                tr.join();
                if (!eL.empty() || !eR.empty()) throw std::runtime_error(eL + eR);
            } else {
                exL(ImageU8{L, w, h, w}, kL, dL);
                exR(ImageU8{R, w, h, w}, kR, dR);
            }
            ComputeStereoMatches(exL, exR, (int)kL.size(), mbf, mb, uR, depth);
            const double dt = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
            if (t >= warmup) {
                ms.push_back(dt);
                kp_total += (long long)kL.size() + (long long)kR.size();
                for (float u : uR) match_total += u >= 0;
            }
        }
        std::vector<double> s = ms;
        std::sort(s.begin(), s.end());
        double mean = 0;
        for (double v : ms) mean += v;
        mean /= (double)ms.size();
        auto q = [&](double p) { return s[std::min(s.size() - 1, (size_t)(p * (s.size() - 1) + 0.5))]; };
        std::printf("{\"mode\": \"%s\", \"frames\": %d, \"warmup\": %d, \"median_ms\": %.4f, \"mean_ms\": %.4f, "
                    "\"p10_ms\": %.4f, \"p90_ms\": %.4f, \"min_ms\": %.4f, \"max_ms\": %.4f, \"keypoints_per_frame\": %.1f, "
                    "\"stereo_matches_per_frame\": %.1f}\n",
                    threads ? "threads" : "serial", frames, warmup, q(0.5), mean, q(0.1), q(0.9), s.front(), s.back(),
                    (double)kp_total / frames, (double)match_total / frames);
        return 0;
    } catch (const std::exception &e) {
        std::cerr << e.what() << "\n";
        return 2;
    }
}
