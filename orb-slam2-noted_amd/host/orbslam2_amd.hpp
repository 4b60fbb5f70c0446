// C++ host layer over the orbslam2_amd C-ABI, mirroring the reference classes the HIP path
// replaces (same names, argument meaning and call order; OpenCV types swapped for PODs so
// this header builds without OpenCV). INTEGRATION.md shows the cv::Mat adapters that drop
// these into the reference tree unchanged for Tracking.cc / LocalMapping.cc.
//
//   orbslam2_amd::ORBextractor   <- ORB_SLAM2::ORBextractor (include/ORBextractor.h:80-216)
//   orbslam2_amd::ORBmatcher     <- ORB_SLAM2::ORBmatcher   (include/ORBmatcher.h:57-65, 169)
//   orbslam2_amd::ComputeStereoMatches <- Frame::ComputeStereoMatches (Frame.cc:831-1128)
//   orbslam2_amd::Optimizer::LocalBundleAdjustment <- Optimizer.h:112 (graph supplied flat)
//   orbslam2_amd::Optimizer::PoseOptimization     <- Optimizer.h:105 (edges supplied flat)
//   orbslam2_amd::ORBmatcher::SearchByProjection   <- ORBmatcher.h:82 (+ Frame::isInFrustum),
//                                                     ORBmatcher.h:102 (motion model)
//   orbslam2_amd::ORBVocabulary                    <- DBoW2 TemplatedVocabulary<FORB>:
//                                                     loadFromTextFile + transform (ComputeBoW)
//
// Error behaviour: the reference has no error path (it asserts / returns silently); a GPU
// failure here throws std::runtime_error -- there is no CPU fallback.
#pragma once
#include <cstdint>
#include <map>
#include <stdexcept>
#include <string>
#include <vector>

#include "orbslam2_amd.h"

namespace orbslam2_amd {

using KeyPoint = orbx_kp;   // cv::KeyPoint memory layout: pt.x, pt.y, size, angle, response, octave, class_id

struct ImageU8 {            // cv::Mat CV_8UC1 view
    const uint8_t *data = nullptr;
    int cols = 0, rows = 0;
    int step = 0;           // bytes per row
};

inline void check(int rc, const char *what) {
    if (rc != ORBX_OK) throw std::runtime_error(std::string("orbslam2_amd: ") + what + " failed (" + std::to_string(rc) + ")");
}

class ORBextractor {
public:
    ORBextractor(int nfeatures, float scaleFactor, int nlevels, int iniThFAST, int minThFAST)
        : nfeatures_(nfeatures), nlevels_(nlevels), scaleFactor_(scaleFactor) {
        orbx_params p{sizeof(orbx_params), nfeatures, scaleFactor, nlevels, iniThFAST, minThFAST, /*resize_mode*/ 0, /*blur_mode*/ 0};
        check(orbx_create(&p, &h_), "orbx_create");
    }
    ~ORBextractor() { orbx_destroy(h_); }
    ORBextractor(const ORBextractor &) = delete;
    ORBextractor &operator=(const ORBextractor &) = delete;

    // operator()(image, mask, keypoints, descriptors): descriptors is N x 32 bytes, row i
    // belongs to keypoints[i]. Empty image -> returns with outputs untouched (:1547).
    void operator()(const ImageU8 &image, std::vector<KeyPoint> &keypoints, std::vector<uint8_t> &descriptors) {
        if (!image.data || image.cols == 0 || image.rows == 0) return;
        const int cap = 2 * nfeatures_ + 512;
        keypoints.resize(cap);
        descriptors.resize((size_t)cap * 32);
        int n = 0;
        check(orbx_extract(h_, image.data, image.cols, image.rows, image.step, keypoints.data(), descriptors.data(), cap, &n),
              "orbx_extract");
        keypoints.resize(n);
        descriptors.resize((size_t)n * 32);
    }

    int GetLevels() const { return nlevels_; }
    float GetScaleFactor() const { return scaleFactor_; }
    std::vector<float> GetScaleFactors() const { return levels()[0]; }
    std::vector<float> GetInverseScaleFactors() const { return levels()[1]; }
    std::vector<float> GetScaleSigmaSquares() const { return levels()[2]; }
    std::vector<float> GetInverseScaleSigmaSquares() const { return levels()[3]; }

    // mvImagePyramid[level] (host copy of the device level)
    std::vector<uint8_t> ImagePyramidLevel(int level, int *cols, int *rows) {
        check(orbx_pyramid_level(h_, 0, level, nullptr, cols, rows), "orbx_pyramid_level");
        std::vector<uint8_t> out((size_t)(*cols) * (*rows));
        check(orbx_pyramid_level(h_, 0, level, out.data(), nullptr, nullptr), "orbx_pyramid_level");
        return out;
    }

    orbx_engine *engine() const { return h_; }

private:
    std::vector<std::vector<float>> levels() const {
        std::vector<std::vector<float>> v(4, std::vector<float>(nlevels_));
        int L = 0;
        check(orbx_levels(h_, &L, v[0].data(), v[1].data(), v[2].data(), v[3].data(), nullptr), "orbx_levels");
        return v;
    }
    orbx_engine *h_ = nullptr;
    int nfeatures_, nlevels_;
    float scaleFactor_;
};

// Frame::ComputeStereoMatches over the frame whose left/right images were last extracted by
// `left` / `right` (mvKeys = left keypoints, N = their count).
inline void ComputeStereoMatches(ORBextractor &left, ORBextractor &right, int N, float mbf, float mb,
                                 std::vector<float> &mvuRight, std::vector<float> &mvDepth) {
    mvuRight.assign(N, -1.0f);
    mvDepth.assign(N, -1.0f);
    check(orbm_stereo_match(left.engine(), right.engine(), mbf, mb, mvuRight.data(), mvDepth.data(), N),
          "orbm_stereo_match");
}

// The Frame members SearchForInitialization reads (Frame.h): mvKeysUn, mDescriptors (N x 32)
// and the static image bounds mnMinX / mnMaxX / mnMinY / mnMaxY.
struct InitFrame {
    std::vector<KeyPoint> mvKeysUn;
    std::vector<uint8_t> mDescriptors;
    float mnMinX = 0, mnMaxX = 0, mnMinY = 0, mnMaxY = 0;
};

struct Point2f {   // cv::Point2f
    float x, y;
};

class ORBmatcher {
public:
    static const int TH_LOW = 50, TH_HIGH = 100, HISTO_LENGTH = 30;
    explicit ORBmatcher(float nnratio = 0.6f, bool checkOri = true) : mfNNratio(nnratio), mbCheckOrientation(checkOri) {}
    ~ORBmatcher() { orbm_destroy(m_); }
    ORBmatcher(const ORBmatcher &) = delete;
    ORBmatcher &operator=(const ORBmatcher &) = delete;
    // DescriptorDistance (ORBmatcher.cc:2123-2143)
    static int DescriptorDistance(const uint8_t *a, const uint8_t *b) {
        int d = 0;
        for (int i = 0; i < 32; i++) d += __builtin_popcount((unsigned)(a[i] ^ b[i]));
        return d;
    }
    // brute-force best / second-best scan on the GPU
    static void HammingBest2(const std::vector<uint8_t> &q, const std::vector<uint8_t> &db, std::vector<int> &best,
                             std::vector<int> &bestDist, std::vector<int> &secondDist) {
        const int nq = (int)(q.size() / 32), ndb = (int)(db.size() / 32);
        best.resize(nq); bestDist.resize(nq); secondDist.resize(nq);
        check(orbm_hamming_best2(q.data(), nq, db.data(), ndb, best.data(), bestDist.data(), secondDist.data()),
              "orbm_hamming_best2");
    }
    // best / second over caller-built candidate lists (CSR: query i's candidates are
    // candIdx[candOff[i] .. candOff[i+1]) into db), first minimum in list order
    void HammingBest2(const std::vector<uint8_t> &q, const std::vector<uint8_t> &db, const std::vector<int32_t> &candOff,
                      const std::vector<int32_t> &candIdx, std::vector<int32_t> &best, std::vector<int32_t> &bestDist,
                      std::vector<int32_t> &secondDist) {
        const int nq = (int)(q.size() / 32), ndb = (int)(db.size() / 32);
        if ((int)candOff.size() != nq + 1) throw std::invalid_argument("candOff needs nq + 1 entries");
        best.resize(nq); bestDist.resize(nq); secondDist.resize(nq);
        check(orbm_hamming_best2_cand(handle(), q.data(), nq, db.data(), ndb, candOff.data(), candIdx.data(), best.data(),
                                      bestDist.data(), secondDist.data()),
              "orbm_hamming_best2_cand");
    }
    // SearchForInitialization(F1, F2, vbPrevMatched, vnMatches12, windowSize) (ORBmatcher.cc:580-748):
    // vbPrevMatched is read as the window centres and updated with the matched F2 positions.
    int SearchForInitialization(const InitFrame &F1, const InitFrame &F2, std::vector<Point2f> &vbPrevMatched,
                                std::vector<int> &vnMatches12, int windowSize = 10) {
        static_assert(sizeof(Point2f) == 8 && sizeof(int) == 4, "Point2f / int layout");
        const int n1 = (int)F1.mvKeysUn.size();
        vnMatches12.assign(n1, -1);
        if (vbPrevMatched.size() < (size_t)n1) throw std::invalid_argument("vbPrevMatched shorter than F1");
        if (F1.mDescriptors.size() < (size_t)n1 * 32 || F2.mDescriptors.size() < F2.mvKeysUn.size() * 32)
            throw std::invalid_argument("descriptors shorter than keypoints");
        const orbm_frame f1{n1, F1.mvKeysUn.data(), F1.mDescriptors.data(), F1.mnMinX, F1.mnMaxX, F1.mnMinY, F1.mnMaxY};
        const orbm_frame f2{(int32_t)F2.mvKeysUn.size(), F2.mvKeysUn.data(), F2.mDescriptors.data(), F2.mnMinX, F2.mnMaxX,
                            F2.mnMinY, F2.mnMaxY};
        int32_t nmatches = 0;
        check(orbm_search_for_initialization(handle(), &f1, &f2, reinterpret_cast<float *>(vbPrevMatched.data()),
                                             vnMatches12.data(), windowSize, &nmatches),
              "orbm_search_for_initialization");
        return nmatches;
    }
    // SearchByProjection(Frame&, const vector<MapPoint*>&, th) with the in-view selection of
    // Tracking::SearchLocalPoints (isInFrustum(pMP, 0.5)); owner[i] = index into M assigned to
    // keypoint i, -1 untouched. inView (optional) = mbTrackInView per map point.
    int SearchByProjection(const orbt_frame &F, const orbt_mappoints &M, float th, const uint8_t *blocked,
                           std::vector<int32_t> &owner, std::vector<uint8_t> *inView = nullptr) {
        owner.assign(F.n, -1);
        std::vector<uint8_t> iv(M.n);
        orbt_view v{iv.data(), nullptr, nullptr, nullptr, nullptr, nullptr};
        int32_t nm = 0;
        check(orbt_search_local_points(track(), &F, &M, 0.5f, th, mfNNratio, blocked, &v, owner.data(), &nm),
              "orbt_search_local_points");
        if (inView) *inView = iv;
        return nm;
    }
    // SearchByProjection(CurrentFrame, LastFrame, th, bMono); owner[i] == -2: set to NULL by
    // the rotation-consistency check.
    int SearchByProjection(const orbt_frame &cur, const orbt_frame &last, const int32_t *lastMp,
                           const uint8_t *lastOutlier, const orbt_mappoints &M, float th, bool bMono,
                           std::vector<int32_t> &owner) {
        owner.assign(cur.n, -1);
        int32_t nm = 0;
        check(orbt_search_by_projection_frame(track(), &cur, &last, lastMp, lastOutlier, &M, th, bMono ? 1 : 0,
                                              mbCheckOrientation ? 1 : 0, nullptr, owner.data(), &nm),
              "orbt_search_by_projection_frame");
        return nm;
    }
    // SearchByProjection(CurrentFrame, pKF, sAlreadyFound, th, ORBdist) (Tracking::Relocalization):
    // kfMp = pKF->GetMapPointMatches() as indices into M, M.flags ORBT_MP_FOUND = sAlreadyFound
    int SearchByProjection(const orbt_frame &cur, const orbt_frame &kf, const int32_t *kfMp, const orbt_mappoints &M,
                           float th, int ORBdist, const uint8_t *blocked, std::vector<int32_t> &owner) {
        owner.assign(cur.n, -1);
        int32_t nm = 0;
        check(orbt_search_by_projection_keyframe(track(), &cur, &kf, kfMp, &M, th, ORBdist, mbCheckOrientation ? 1 : 0,
                                                 blocked, owner.data(), &nm),
              "orbt_search_by_projection_keyframe");
        return nm;
    }
    // SearchByProjection(pKF, Scw, vpPoints, vpMatched, th) (LoopClosing): vpMatched in/out as indices
    int SearchByProjection(const orbt_frame &kf, const float Scw[16], const orbt_mappoints &vpPoints,
                           std::vector<int32_t> &vpMatched, int th) {
        vpMatched.resize(kf.n, -1);
        int32_t nm = 0;
        check(orbt_search_by_projection_sim3(track(), &kf, Scw, &vpPoints, th, vpMatched.data(), &nm),
              "orbt_search_by_projection_sim3");
        return nm;
    }
    // SearchByBoW(pKF1, pKF2, vpMatches12) (LoopClosing::ComputeSim3)
    int SearchByBoW(const orbb_keyframe &kf1, const orbb_keyframe &kf2, std::vector<int32_t> &vpMatches12) {
        vpMatches12.assign(kf1.n, -1);
        int32_t nm = 0;
        check(orbb_search_by_bow_kf(bow(), &kf1, &kf2, mfNNratio, mbCheckOrientation ? 1 : 0, vpMatches12.data(), &nm),
              "orbb_search_by_bow_kf");
        return nm;
    }
    // SearchBySim3(pKF1, pKF2, vpMatches12, s12, R12, t12, th): vpMatches12 in/out as indices
    int SearchBySim3(const orbt_frame &kf1, const int32_t *kf1Mp, const orbt_frame &kf2, const int32_t *kf2Mp,
                     const orbt_mappoints &M, std::vector<int32_t> &vpMatches12, float s12, const float R12[9],
                     const float t12[3], float th) {
        vpMatches12.resize(kf1.n, -1);
        int32_t nf = 0;
        check(orbt_search_by_sim3(track(), &kf1, kf1Mp, &kf2, kf2Mp, &M, s12, R12, t12, th, vpMatches12.data(), &nf),
              "orbt_search_by_sim3");
        return nf;
    }
    // Fuse(pKF, Scw, vpPoints, th, vpReplacePoint), search half: the caller applies the updates in
    // point order for bestDist <= TH_LOW (ORBmatcher.cc:1437-1453)
    void FuseCandidates(const orbt_frame &kf, const float Scw[16], const orbt_mappoints &vpPoints, float th,
                        std::vector<int32_t> &bestIdx, std::vector<int32_t> &bestDist) {
        bestIdx.resize(vpPoints.n);
        bestDist.resize(vpPoints.n);
        check(orbt_fuse_sim3_candidates(track(), &kf, Scw, &vpPoints, th, bestIdx.data(), bestDist.data()),
              "orbt_fuse_sim3_candidates");
    }
    float mfNNratio;
    bool mbCheckOrientation;

private:
    orbm_matcher *handle() {   // created on first use: matchers are cheap stack objects in the reference
        if (!m_) check(orbm_create(mfNNratio, mbCheckOrientation ? 1 : 0, &m_), "orbm_create");
        return m_;
    }
    orbm_matcher *m_ = nullptr;
    static orbb_engine *bow() {
        struct H {
            orbb_engine *h = nullptr;
            H() { check(orbb_create(&h), "orbb_create"); }
            ~H() { orbb_destroy(h); }
        };
        static thread_local H h;
        return h.h;
    }
    static orbt_engine *track() {
        struct H {
            orbt_engine *h = nullptr;
            H() { check(orbt_create(&h), "orbt_create"); }
            ~H() { orbt_destroy(h); }
        };
        static thread_local H h;
        return h.h;
    }
};

// DBoW2 TemplatedVocabulary<FORB::TDescriptor, FORB> (ORBVocabulary.h) resident in HBM.
using BowVector = std::map<uint32_t, double>;                        // DBoW2::BowVector
using FeatureVector = std::map<uint32_t, std::vector<unsigned int>>; // DBoW2::FeatureVector

class ORBVocabulary {
public:
    ORBVocabulary() = default;
    ~ORBVocabulary() { orbv_destroy(h_); }
    ORBVocabulary(const ORBVocabulary &) = delete;
    ORBVocabulary &operator=(const ORBVocabulary &) = delete;
    bool loadFromTextFile(const std::string &filename) {
        orbv_destroy(h_);
        h_ = nullptr;
        return orbv_load_text(filename.c_str(), &h_) == ORBX_OK;
    }
    // transform(features, BowVector&, FeatureVector&, levelsup): Frame::ComputeBoW uses 4
    void transform(const uint8_t *desc, int n, BowVector &v, FeatureVector &fv, int levelsup) const {
        v.clear();
        fv.clear();
        std::vector<uint32_t> words(n + 1), nodes(n + 1);
        std::vector<double> vals(n + 1);
        std::vector<int32_t> start(n + 2), feats(n + 1);
        int32_t nw = 0, nf = 0;
        check(orbv_transform(h_, desc, n, levelsup, words.data(), vals.data(), &nw, nodes.data(), start.data(),
                             feats.data(), &nf), "orbv_transform");
        for (int j = 0; j < nw; j++) v.emplace_hint(v.end(), words[j], vals[j]);
        for (int j = 0; j < nf; j++)
            fv.emplace_hint(fv.end(), nodes[j], std::vector<unsigned int>(feats.begin() + start[j], feats.begin() + start[j + 1]));
    }
    size_t size() const {
        int nw = 0;
        if (h_) orbv_info(h_, nullptr, &nw, nullptr, nullptr);
        return (size_t)nw;
    }

private:
    orbv_vocab *h_ = nullptr;
};

// Optimizer::LocalBundleAdjustment minus the map walk: the caller flattens the local
// keyframes / fixed keyframes / local map points / observations into lba_problem
// (Optimizer.cc:646-898 order) and applies the result (SetPose / SetWorldPos /
// EraseMapPointMatch, :977-1048).
class Optimizer {
public:
    static lba_result LocalBundleAdjustment(const lba_problem &graph, bool *pbStopFlag, std::vector<float> &poseTcw,
                                            std::vector<float> &pointXw, std::vector<uint8_t> &edgeErase) {
        static thread_local LbaHandle lba;
        poseTcw.resize((size_t)graph.n_poses * 16);
        pointXw.resize((size_t)graph.n_points * 3);
        edgeErase.resize(graph.n_edges);
        lba_result r{};
        r.pose_Tcw = poseTcw.data();
        r.point_Xw = pointXw.data();
        r.edge_erase = edgeErase.data();
        static_assert(sizeof(bool) == 1, "pbStopFlag is passed to the C-ABI as one byte");
        check(lba_solve(lba.h, &graph, &r, reinterpret_cast<const volatile uint8_t *>(pbStopFlag)), "lba_solve");
        return r;
    }

    // PoseOptimization(Frame*): edges = the frame's keypoints with a map point, in keypoint
    // order (Optimizer.cc:412-531). Returns nInitialCorrespondences - nBad; Tcw = SetPose
    // value, outlier[k] = mvbOutlier of edge k.
    static int PoseOptimization(const orbp_frame &f, float Tcw[16], std::vector<uint8_t> &outlier) {
        struct H {
            orbp_engine *h = nullptr;
            H() { check(orbp_create(&h), "orbp_create"); }
            ~H() { orbp_destroy(h); }
        };
        static thread_local H eng;
        outlier.assign(f.n, 0);
        orbp_result r{};
        r.outlier = outlier.data();
        check(orbp_pose_optimization(eng.h, &f, &r), "orbp_pose_optimization");
        for (int i = 0; i < 16; i++) Tcw[i] = r.Tcw[i];
        return r.n_inliers;
    }

private:
    struct LbaHandle {
        lba_engine *h = nullptr;
        LbaHandle() { check(lba_create(&h), "lba_create"); }
        ~LbaHandle() { lba_destroy(h); }
    };
};

// LocalMapping::CreateNewMapPoints (LocalMapping.cc:295-600): per neighbour, the caller keeps
// the baseline test, ComputeF12 and ORBmatcher::SearchForTriangulation (orbb_*), then
// TriangulateMatches runs the per-match body on the GPU; ok[k] = 1 -> create the MapPoint at
// x3D[3k..3k+2] with observations (idx1 in mpCurrentKeyFrame, idx2 in pKF2) as the reference does.
class LocalMapping {
public:
    static int TriangulateMatches(const orbn_keyframe &kf1, const orbn_keyframe &kf2,
                                  const std::vector<int32_t> &vMatchedIndices, float ratioFactor,
                                  std::vector<float> &x3D, std::vector<uint8_t> &ok) {
        struct H {
            orbn_engine *h = nullptr;
            H() { check(orbn_create(&h), "orbn_create"); }
            ~H() { orbn_destroy(h); }
        };
        static thread_local H eng;
        const int32_t n = (int32_t)(vMatchedIndices.size() / 2);
        x3D.assign((size_t)n * 3, 0.0f);
        ok.assign(n, 0);
        int32_t nnew = 0;
        check(orbn_triangulate(eng.h, &kf1, &kf2, vMatchedIndices.data(), n, ratioFactor, x3D.data(), ok.data(), &nnew),
              "orbn_triangulate");
        return nnew;
    }
};

}  // namespace orbslam2_amd
