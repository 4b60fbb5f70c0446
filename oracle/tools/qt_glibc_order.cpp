// ORACLE TOOL — TEST INFRASTRUCTURE ONLY (parity exposure of the quadtree tie pin).
//
// ORBextractor::DistributeOctTree (ORBextractor.cc:696-1042) sorts pair<int, ExtractorNode*>
// (:935) and splits equal-size nodes in descending *heap address* order (:938). The oracle pins
// that tie by node creation sequence (orb_oracle.c:524-539). This harness asks
// what real glibc addresses do: it restates DistributeOctTree over a real std::list<ExtractorNode>
// whose element has ExtractorNode's layout (ORBextractor.h:40-67: vector<KeyPoint> 24 B, four
// Point2i, a list iterator, a bool = 72 B, list node 88 B) with the reference's allocation sequence
// (DivideNode's four reserves, push_front copies, erase, the temporaries' destruction order), sorts
// by the real pointers, and runs each image in a fresh std::thread, two per stereo frame, as
// Frame.cc:144-153 does. Three allocation contexts around it:
//   ctx 0  DistributeOctTree alone (the level's candidates in an exactly sized vector);
//   ctx 1  + ComputeKeyPointsOctTree's vectors (:1051-1169): allKeypoints, vToDistributeKeys
//          reserve(nfeatures*10), one vKeysCell per visited cell grown by push_back to the cell's
//          FAST count (cv::FAST push_backs its output), keypoints.reserve(nfeatures) then the
//          move-assignment of the result;
//   ctx 2  + the cv::Mat traffic of operator() (:1543-1658): per level a new pyramid Mat
//          (a UMatData header of 88 B -- the list node's size class -- and (W+38)(H+38) + 72 B of
//          data, the previous frame's level released on assignment, ComputePyramid :1664-1733), the
//          descriptor Mat and output keypoint vector of the frame (released two frames later by the
//          calling thread, as Tracking drops mLastFrame), and per level a workingMat clone released
//          after the descriptors.
// The element carries its creation sequence in the struct's tail padding (sizeof unchanged), so
// each final-phase sort can report whether address order agreed with creation order for every
// adjacent equal-size pair. With pin=1 the sort uses the creation sequence instead (must equal
// orc_distribute_octtree: tools/qt_glibc_order.py checks it).
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <list>
#include <thread>
#include <utility>
#include <vector>

extern "C" {
#include "../orb_oracle.h"
}

namespace {

struct Point2f { float x, y; };
struct KeyPoint {   // cv::KeyPoint, 28 B
    Point2f pt;
    float size, angle, response;
    int octave, class_id;
};
static_assert(sizeof(KeyPoint) == 28, "cv::KeyPoint layout");
struct Point2i {
    int x = 0, y = 0;
    Point2i() = default;
    Point2i(int a, int b) : x(a), y(b) {}
};

struct ExtractorNode {
    ExtractorNode() : bNoMore(false) {}
    void DivideNode(ExtractorNode &n1, ExtractorNode &n2, ExtractorNode &n3, ExtractorNode &n4);
    std::vector<KeyPoint> vKeys;
    Point2i UL, UR, BL, BR;
    std::list<ExtractorNode>::iterator lit;
    bool bNoMore;
    int seq = 0;   // harness only: lives in the padding after bNoMore
};
static_assert(sizeof(ExtractorNode) == 72, "ExtractorNode layout (ORBextractor.h:40-67)");

void ExtractorNode::DivideNode(ExtractorNode &n1, ExtractorNode &n2, ExtractorNode &n3, ExtractorNode &n4) {
    const int halfX = (int)std::ceil((float)(UR.x - UL.x) / 2);
    const int halfY = (int)std::ceil((float)(BR.y - UL.y) / 2);
    n1.UL = UL;
    n1.UR = Point2i(UL.x + halfX, UL.y);
    n1.BL = Point2i(UL.x, UL.y + halfY);
    n1.BR = Point2i(UL.x + halfX, UL.y + halfY);
    n1.vKeys.reserve(vKeys.size());
    n2.UL = n1.UR;
    n2.UR = UR;
    n2.BL = n1.BR;
    n2.BR = Point2i(UR.x, UL.y + halfY);
    n2.vKeys.reserve(vKeys.size());
    n3.UL = n1.BL;
    n3.UR = n1.BR;
    n3.BL = BL;
    n3.BR = Point2i(n1.BR.x, BL.y);
    n3.vKeys.reserve(vKeys.size());
    n4.UL = n3.UR;
    n4.UR = n2.BR;
    n4.BL = n3.BR;
    n4.BR = BR;
    n4.vKeys.reserve(vKeys.size());
    for (const KeyPoint &kp : vKeys) {
        if (kp.pt.x < n1.UR.x) {
            if (kp.pt.y < n1.BR.y) n1.vKeys.push_back(kp);
            else n3.vKeys.push_back(kp);
        } else if (kp.pt.y < n1.BR.y) {
            n2.vKeys.push_back(kp);
        } else {
            n4.vKeys.push_back(kp);
        }
    }
    if (n1.vKeys.size() == 1) n1.bNoMore = true;
    if (n2.vKeys.size() == 1) n2.bNoMore = true;
    if (n3.vKeys.size() == 1) n3.bNoMore = true;
    if (n4.vKeys.size() == 1) n4.bNoMore = true;
}

struct TieStats { long sorts = 0, pairs = 0, agree = 0, final_levels = 0; };

typedef std::pair<int, ExtractorNode *> SizePtr;

// the list-order quadtree; `pin` replaces the pointer of the :935 sort by the creation sequence
std::vector<KeyPoint> DistributeOctTree(const std::vector<KeyPoint> &keys, int minX, int maxX, int minY, int maxY,
                                        int N, int nfeatures, bool pin, TieStats &st) {
    const int nIni = (int)std::round((float)(maxX - minX) / (maxY - minY));
    const float hX = (float)(maxX - minX) / nIni;
    std::list<ExtractorNode> lNodes;
    std::vector<ExtractorNode *> vpIniNodes;
    vpIniNodes.resize(nIni);
    int seq = 0;
    for (int i = 0; i < nIni; i++) {
        ExtractorNode ni;
        ni.UL = Point2i((int)(hX * (float)i), 0);
        ni.UR = Point2i((int)(hX * (float)(i + 1)), 0);
        ni.BL = Point2i(ni.UL.x, maxY - minY);
        ni.BR = Point2i(ni.UR.x, maxY - minY);
        ni.vKeys.reserve(keys.size());
        lNodes.push_back(ni);
        lNodes.back().seq = seq++;
        vpIniNodes[i] = &lNodes.back();
    }
    for (const KeyPoint &kp : keys) vpIniNodes[(size_t)(kp.pt.x / hX)]->vKeys.push_back(kp);
    for (auto lit = lNodes.begin(); lit != lNodes.end();) {
        if (lit->vKeys.size() == 1) {
            lit->bNoMore = true;
            ++lit;
        } else if (lit->vKeys.empty()) {
            lit = lNodes.erase(lit);
        } else {
            ++lit;
        }
    }
    bool bFinish = false;
    std::vector<SizePtr> vSizeAndPointerToNode;
    vSizeAndPointerToNode.reserve(lNodes.size() * 4);
    auto push_child = [&](ExtractorNode &c, bool track, int &nToExpand) {
        if (c.vKeys.empty()) return;
        lNodes.push_front(c);
        lNodes.front().seq = seq++;
        if (c.vKeys.size() > 1) {
            nToExpand += track;
            vSizeAndPointerToNode.push_back(std::make_pair((int)c.vKeys.size(), &lNodes.front()));
            lNodes.front().lit = lNodes.begin();
        }
    };
    bool reached_final = false;
    while (!bFinish) {
        int prevSize = (int)lNodes.size();
        auto lit = lNodes.begin();
        int nToExpand = 0;
        vSizeAndPointerToNode.clear();
        while (lit != lNodes.end()) {
            if (lit->bNoMore) {
                ++lit;
                continue;
            }
            ExtractorNode n1, n2, n3, n4;
            lit->DivideNode(n1, n2, n3, n4);
            push_child(n1, true, nToExpand);
            push_child(n2, true, nToExpand);
            push_child(n3, true, nToExpand);
            push_child(n4, true, nToExpand);
            lit = lNodes.erase(lit);
        }
        if ((int)lNodes.size() >= N || (int)lNodes.size() == prevSize) {
            bFinish = true;
        } else if ((int)lNodes.size() + nToExpand * 3 > N) {
            reached_final = true;
            while (!bFinish) {
                prevSize = (int)lNodes.size();
                std::vector<SizePtr> vPrev = vSizeAndPointerToNode;
                vSizeAndPointerToNode.clear();
                if (pin)
                    std::sort(vPrev.begin(), vPrev.end(), [](const SizePtr &a, const SizePtr &b) {
                        return a.first != b.first ? a.first < b.first : a.second->seq < b.second->seq;
                    });
                else
                    std::sort(vPrev.begin(), vPrev.end());
                st.sorts++;
                for (size_t j = 1; j < vPrev.size(); j++)
                    if (vPrev[j].first == vPrev[j - 1].first) {
                        st.pairs++;
                        st.agree += vPrev[j].second->seq > vPrev[j - 1].second->seq;
                    }
                int dummy = 0;
                for (int j = (int)vPrev.size() - 1; j >= 0; j--) {
                    ExtractorNode n1, n2, n3, n4;
                    vPrev[j].second->DivideNode(n1, n2, n3, n4);
                    push_child(n1, false, dummy);
                    push_child(n2, false, dummy);
                    push_child(n3, false, dummy);
                    push_child(n4, false, dummy);
                    lNodes.erase(vPrev[j].second->lit);
                    if ((int)lNodes.size() >= N) break;
                }
                if ((int)lNodes.size() >= N || (int)lNodes.size() == prevSize) bFinish = true;
            }
        }
    }
    st.final_levels += reached_final;
    std::vector<KeyPoint> vResultKeys;
    vResultKeys.reserve(nfeatures);
    for (auto &node : lNodes) {
        std::vector<KeyPoint> &v = node.vKeys;
        const KeyPoint *p = &v[0];
        float maxResponse = p->response;
        for (size_t k = 1; k < v.size(); k++)
            if (v[k].response > maxResponse) {
                p = &v[k];
                maxResponse = v[k].response;
            }
        vResultKeys.push_back(*p);
    }
    return vResultKeys;
}

// cv::Mat stand-in: a UMatData header (88 B) and fastMalloc'd data (size + 8 + 64 B)
struct FakeMat {
    void *hdr = nullptr, *data = nullptr;
    void create(size_t bytes) {
        release();
        hdr = std::malloc(88);
        data = std::malloc(bytes + 8 + 64);
        std::memset(hdr, 0, 88);
        static_cast<volatile char *>(data)[0] = 1;
    }
    void release() {
        if (data) std::free(data);
        if (hdr) std::free(hdr);
        hdr = data = nullptr;
    }
};

}  // namespace

extern "C" {

typedef struct {
    const orc_kp *cand;
    int ncand;
    const int *cell_counts;
    int ncells;
    int minX, maxX, minY, maxY, N;
    int lw, lh;
} qtg_level;

typedef struct {
    int nlevels, nfeatures;
    qtg_level lev[ORC_MAX_LEVELS];
    orc_kp *out[ORC_MAX_LEVELS];   // per level, list order, cell-offset coordinates like orc_distribute_octtree
    int out_cap;
    int nout[ORC_MAX_LEVELS];
} qtg_image;

typedef struct { FakeMat pyr[ORC_MAX_LEVELS]; } qtg_extractor_state;

static void run_image(qtg_image *im, int ctx, bool pin, qtg_extractor_state *ext, FakeMat *frame_desc,
                      std::vector<KeyPoint> *frame_kps, TieStats *st) {
    const int nl = im->nlevels;
    if (ctx >= 2)   // ComputePyramid: a new Mat per level, the previous frame's released on assignment
        for (int l = 0; l < nl; l++) {
            FakeMat temp;
            temp.create((size_t)(im->lev[l].lw + 38) * (im->lev[l].lh + 38));
            ext->pyr[l].release();
            ext->pyr[l] = temp;
        }
    std::vector<std::vector<KeyPoint>> allKeypoints;
    if (ctx >= 1) allKeypoints.resize(nl);
    for (int l = 0; l < nl; l++) {
        const qtg_level &L = im->lev[l];
        std::vector<KeyPoint> keypoints;
        std::vector<KeyPoint> vToDistributeKeys;
        if (ctx >= 1) {
            vToDistributeKeys.reserve((size_t)im->nfeatures * 10);
            int k = 0;
            for (int c = 0; c < L.ncells; c++) {
                std::vector<KeyPoint> vKeysCell;
                for (int i = 0; i < L.cell_counts[c]; i++) {
                    const orc_kp &q = L.cand[k + i];
                    vKeysCell.push_back(KeyPoint{{q.x, q.y}, q.size, q.angle, q.response, q.octave, q.class_id});
                }
                for (const KeyPoint &kp : vKeysCell) vToDistributeKeys.push_back(kp);
                k += L.cell_counts[c];
            }
        } else {
            vToDistributeKeys.resize(L.ncand);
            for (int i = 0; i < L.ncand; i++) {
                const orc_kp &q = L.cand[i];
                vToDistributeKeys[i] = KeyPoint{{q.x, q.y}, q.size, q.angle, q.response, q.octave, q.class_id};
            }
        }
        std::vector<KeyPoint> &dst = ctx >= 1 ? allKeypoints[l] : keypoints;
        if (ctx >= 1) dst.reserve(im->nfeatures);
        dst = DistributeOctTree(vToDistributeKeys, L.minX, L.maxX, L.minY, L.maxY, L.N, im->nfeatures, pin, *st);
        const int n = (int)dst.size();
        im->nout[l] = n;
        for (int i = 0; i < n && i < im->out_cap; i++) {
            const KeyPoint &p = dst[i];
            im->out[l][i] = orc_kp{p.pt.x, p.pt.y, p.size, p.angle, p.response, p.octave, p.class_id};
        }
    }
    if (ctx >= 2) {   // operator(): descriptors Mat + output keypoints (kept by the Frame), blur clones
        size_t total = 0;
        for (int l = 0; l < nl; l++) total += allKeypoints[l].size();
        frame_desc->create(total * 32);
        frame_kps->reserve(total);
        for (int l = 0; l < nl; l++) {
            if (allKeypoints[l].empty()) continue;
            FakeMat working;
            working.create((size_t)im->lev[l].lw * im->lev[l].lh);
            frame_kps->insert(frame_kps->end(), allKeypoints[l].begin(), allKeypoints[l].end());
            working.release();
        }
    }
}

// Runs the images frame by frame, images_per_frame fresh std::threads per frame (image i of a frame
// on extractor i, whose pyramid Mats persist across frames); the frame outputs are released by the
// calling thread two frames later. stats: [0] final-phase sorts, [1] adjacent equal-size pairs in
// them, [2] pairs whose address order agreed with creation order, [3] levels reaching the final phase.
int qtg_run_frames(qtg_image *imgs, int n_images, int images_per_frame, int ctx, int pin, long stats[4]) {
    if (!imgs || n_images <= 0 || images_per_frame <= 0 || images_per_frame > 8) return -1;
    std::vector<qtg_extractor_state> ext(images_per_frame);
    const int nframes = (n_images + images_per_frame - 1) / images_per_frame;
    std::vector<std::vector<FakeMat>> desc(nframes, std::vector<FakeMat>(images_per_frame));
    std::vector<std::vector<std::vector<KeyPoint>>> kps(nframes, std::vector<std::vector<KeyPoint>>(images_per_frame));
    std::vector<TieStats> st(n_images);
    for (int f = 0; f < nframes; f++) {
        std::vector<std::thread> th;
        for (int i = 0; i < images_per_frame; i++) {
            const int idx = f * images_per_frame + i;
            if (idx >= n_images) break;
            th.emplace_back(run_image, &imgs[idx], ctx, pin != 0, &ext[i], &desc[f][i], &kps[f][i], &st[idx]);
        }
        for (auto &t : th) t.join();
        if (f >= 2)
            for (int i = 0; i < images_per_frame; i++) {
                desc[f - 2][i].release();
                std::vector<KeyPoint>().swap(kps[f - 2][i]);
            }
    }
    for (auto &fr : desc)
        for (auto &m : fr) m.release();
    for (auto &e : ext)
        for (auto &m : e.pyr) m.release();
    for (int k = 0; k < 4; k++) stats[k] = 0;
    for (const TieStats &s : st) {
        stats[0] += s.sorts;
        stats[1] += s.pairs;
        stats[2] += s.agree;
        stats[3] += s.final_levels;
    }
    return 0;
}

}  // extern "C"
