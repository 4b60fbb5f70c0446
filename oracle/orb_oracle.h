/*
 * ORACLE — TEST INFRASTRUCTURE ONLY.
 *
 * Single-threaded, OpenCV-free C restatement of ORB-SLAM2-noted's per-frame hot path
 * (/root/reference, read-only). It is the checker the HIP path is compared against and
 * the `cpu_baseline` leg of bench.py; it is never linked into the product library.
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load it.
 *
 * Parity status: the reference cannot be compiled in this image (OpenCV / Eigen absent,
 * SURVEY.md §8c) and ships no golden vectors, so this restatement is "parity unpinned"
 * against a real OpenCV build. Pinned pieces: glibc cosf/sinf restatement (validated
 * exhaustively against live libm by oracle/tools/check_sincosf.c), FAST / IC_Angle /
 * BRIEF / Hamming cross-checked against an independent numpy restatement
 * (oracle/np_ref.py).
 */
#ifndef ORB_ORACLE_H
#define ORB_ORACLE_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define ORC_MAX_LEVELS 16

/* cv::KeyPoint memory layout (28 bytes). */
typedef struct {
    float x, y, size, angle, response;
    int octave, class_id;
} orc_kp;

typedef struct {
    int nfeatures;
    double scaleFactor;          /* ORBextractor.h:203 stores it as double */
    int nlevels, iniThFAST, minThFAST;
    int resize_mode;             /* 0 = scalar FixedPtCast (default pin), 1 = SSE2 VResizeLinearVec layout */
    int blur_mode;               /* 0 = OpenCV >= 3.4 fixed point (default pin), 1 = OpenCV 3.2 half-even prefix */
    float mvScaleFactor[ORC_MAX_LEVELS], mvInvScaleFactor[ORC_MAX_LEVELS];
    float mvLevelSigma2[ORC_MAX_LEVELS], mvInvLevelSigma2[ORC_MAX_LEVELS];
    int mnFeaturesPerLevel[ORC_MAX_LEVELS];
    int umax[16];
    int pattern[1024];           /* 512 points (x,y) */
    /* pyramid (unpadded ROI of each level, row stride == width) */
    int lw[ORC_MAX_LEVELS], lh[ORC_MAX_LEVELS];
    uint8_t *level[ORC_MAX_LEVELS];
    uint8_t *blurred[ORC_MAX_LEVELS];
} orc_extractor;

/* ORBextractor::ORBextractor (ORBextractor.cc:471-579). */
int  orc_extractor_init(orc_extractor *ex, int nfeatures, float scaleFactor, int nlevels,
                        int iniThFAST, int minThFAST);
void orc_extractor_free(orc_extractor *ex);

/* ORBextractor::operator() (ORBextractor.cc:1543-1658). Returns the keypoint count, writes
 * at most `cap` keypoints / 32-byte descriptors; returns -1 if cap is too small. */
int  orc_extract(orc_extractor *ex, const uint8_t *img, int w, int h, int stride,
                 orc_kp *kps, uint8_t *desc, int cap);

/* building blocks, exported for unit tests */
void orc_resize_linear(const uint8_t *src, int sw, int sh, int sstride,
                       uint8_t *dst, int dw, int dh, int dstride, int mode);
int  orc_fast_roi(const uint8_t *img, int stride, int rows, int cols, int threshold,
                  int *xs, int *ys, int *scores, int cap);
int  orc_corner_score16(const uint8_t *ptr, int stride, int threshold);
void orc_gaussian_blur9(const uint8_t *src, int w, int h, uint8_t *dst);
void orc_gaussian_blur9_mode(const uint8_t *src, int w, int h, uint8_t *dst, int mode);
float orc_fast_atan2(float y, float x);
float orc_ic_angle(const uint8_t *img, int stride, float px, float py, const int *umax);
void orc_orb_descriptor(const uint8_t *img, int stride, float px, float py, float angle,
                        const int *pattern, uint8_t *desc);
float orc_cosf(float x);
float orc_sinf(float x);
int  orc_descriptor_distance(const uint8_t *a, const uint8_t *b);

/* level-wise candidates: FAST cell grid of one level (ORBextractor.cc:1046-1153).
 * Returns the candidate count (candidate coordinates are cell-offset, origin minBorder). */
int  orc_level_candidates(const orc_extractor *ex, int level, orc_kp *out, int cap);
/* + the candidate count of each visited FAST cell, in visiting order (*ncells of them; cell_counts
 * holds at least nRows * nCols ints): the allocation pattern of the per-cell vKeysCell vectors,
 * for the glibc pointer-order harness (oracle/tools/qt_glibc_order.cpp) */
int  orc_level_candidates_cells(const orc_extractor *ex, int level, orc_kp *out, int cap,
                                int *cell_counts, int *ncells);
/* DistributeOctTree (ORBextractor.cc:696-1042); returns kept count. */
int  orc_distribute_octtree(const orc_kp *keys, int nkeys, int minX, int maxX, int minY,
                            int maxY, int N, orc_kp *out, int cap);

/* Frame::ComputeStereoMatches (Frame.cc:831-1128). Pyramids are the two extractors'
 * mvImagePyramid after the extract calls. */
void orc_stereo_matches(const orc_extractor *exL, const orc_extractor *exR,
                        const orc_kp *kL, const uint8_t *dL, int nL,
                        const orc_kp *kR, const uint8_t *dR, int nR,
                        float mbf, float mb, float *uRight, float *depth);

/* Frame grid (Frame.cc:398-422, 590-698, 780-830) */
#define ORC_GRID_COLS 64
#define ORC_GRID_ROWS 48
typedef struct {
    int N;
    const orc_kp *keysUn;
    const uint8_t *desc;
    float minX, maxX, minY, maxY, gridInvW, gridInvH;
    int *cell_start;     /* [COLS*ROWS+1] CSR over cells, cell = ix*ROWS+iy */
    int *cell_items;     /* [N] */
} orc_frame_grid;
void orc_image_bounds(int cols, int rows, const float K[4] /*fx,fy,cx,cy*/, const float dist[5],
                      float *minX, float *maxX, float *minY, float *maxY);
int  orc_grid_build(orc_frame_grid *g, const orc_kp *keysUn, const uint8_t *desc, int N,
                    float minX, float maxX, float minY, float maxY);
void orc_grid_free(orc_frame_grid *g);
int  orc_features_in_area(const orc_frame_grid *g, float x, float y, float r, int minLevel,
                          int maxLevel, int *out, int cap);

/* ORBmatcher::SearchForInitialization (ORBmatcher.cc:580-748). prev_xy is vbPrevMatched
 * (in/out, 2 floats per F1 keypoint). Returns nmatches. */
int  orc_search_for_initialization(const orc_frame_grid *F1, const orc_frame_grid *F2,
                                   float *prev_xy, int *matches12, int windowSize,
                                   float nnratio, int checkOri);

/* cv::undistortPoints restatement + Frame::UndistortKeyPoints
 * (Frame.cc:725-776) + ComputeStereoFromRGBD (Frame.cc:1131-1169). */
void orc_undistort_points(const float *xy_in, float *xy_out, int n, const float K[4],
                          const float dist[5]);
void orc_stereo_from_rgbd(const orc_kp *keys, const orc_kp *keysUn, int N, const float *depth,
                          int dstride, float mbf, float *uRight, float *depthOut);

/* parity-exposure instruments (test infrastructure): quadtree tie counters of the calling
 * thread ([0] calls, [1] final phase reached, [2] equal-size nodes split (order exposed),
 * [3] cut inside an equal-size run (set exposed)); blur variant (0 = pin, 1 = OpenCV 3.2 SSE2
 * half-even column rounding on the vectorised prefix). */
void orc_qt_tie_stats(long out[4], int reset);
void orc_set_blur_mode(int mode);
/* tie key of the final-phase sort: 0 = creation sequence (pin), 1 = reversed, 2 = hashed */
void orc_set_tie_mode(int mode);

/* batched Hamming best/second-best (the ORBmatcher scan core) */
void orc_hamming_best2(const uint8_t *q, int nq, const uint8_t *db, int ndb,
                       int *best_idx, int *best_d, int *second_d);

#ifdef __cplusplus
}
#endif
#endif
