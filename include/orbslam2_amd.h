/*
 * orbslam2_amd — C-ABI of the MI355X-native ORB-SLAM2 per-frame hot path.
 *
 * Plain pointers, sizes and POD structs only (no OpenCV / Eigen / torch types). Every
 * entry point returns int status: 0 = OK, < 0 = error (never throws across the ABI).
 * Each declaration names the reference interface it replaces (paths relative to the
 * QiuYue-bit/ORB-SLAM2-noted tree). INTEGRATION.md shows the C++ adapters that keep the
 * reference class signatures (ORBextractor / ORBmatcher / Frame / Optimizer) on top.
 */
#ifndef ORBSLAM2_AMD_H
#define ORBSLAM2_AMD_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define ORBX_OK 0
#define ORBX_EINVAL (-1)     /* bad argument / shape */
#define ORBX_EDEVICE (-2)    /* HIP runtime error or no device */
#define ORBX_ECAP (-3)       /* caller buffer too small; *n holds the required count */
#define ORBX_ESTATE (-4)     /* call order (e.g. results before extract) */

/* cv::KeyPoint memory layout (28 bytes): pt.x, pt.y, size, angle, response, octave,
 * class_id. Keypoints cross the ABI in exactly this layout. */
typedef struct {
    float x, y, size, angle, response;
    int32_t octave, class_id;
} orbx_kp;

/* ORBextractor(int nfeatures, float scaleFactor, int nlevels, int iniThFAST, int minThFAST)
 * -- include/ORBextractor.h:89 (ORBextractor.cc:471-579). The two OpenCV-version choices the
 * reference leaves to its OpenCV build, each 0 or 1 (else ORBX_EINVAL):
 *   resize_mode: cv::resize INTER_LINEAR vertical pass -- 0 scalar FixedPtCast (default),
 *                1 the OpenCV 3.2 SSE2 VResizeLinearVec_32s8u layout;
 *   blur_mode:   cv::GaussianBlur(9x9, 2) column pass (ORBextractor.cc:1617-1625) -- 0 the
 *                OpenCV >= 3.4 fixed-point rounding (default), 1 OpenCV 3.2's SSE2
 *                SymmColumnVec_32s8u (round half to even over each row's prefix [0, w & ~3)).
 * resize_mode 1 + blur_mode 1 is the reference's documented platform (OpenCV 3.2.0 on x86-64,
 * /root/reference/README.md:9).
 * Input range (checked by orbx_reserve / orbx_extract, ORBX_EINVAL otherwise): image width and
 * height <= 4000 (keys carry 12-bit coordinates), every pyramid level >= 40 x 40 pixels (the
 * 19-pixel FAST border plus the blur halo; ORBextractor.cc:1084-1100 detects nothing in a
 * smaller level), and scaleFactor <= 2 (the resize kernel's 4 outputs span <= 8 source bytes).
 * struct_size must be sizeof(orbx_params) of the header the caller was built against: orbx_create
 * refuses any other value with ORBX_EINVAL, so a caller built against an older layout (fewer
 * fields) fails at creation instead of having fields read past its struct. */
typedef struct {
    uint32_t struct_size;   /* = sizeof(orbx_params) */
    int32_t nfeatures;
    float scale_factor;
    int32_t nlevels;
    int32_t ini_th_fast;
    int32_t min_th_fast;
    int32_t resize_mode;
    int32_t blur_mode;
} orbx_params;

typedef struct orbx_engine orbx_engine;

/* -------- extractor (replaces ORBextractor, include/ORBextractor.h:80-216) -------- */

/* constructor: ORBextractor::ORBextractor (ORBextractor.h:89). Binds the current HIP
 * device; creates a private stream (one instance per thread, as Frame.cc:144-153 runs the
 * left and right extractors on two threads). */
int orbx_create(const orbx_params *p, orbx_engine **out);
void orbx_destroy(orbx_engine *e);

/* GetLevels / GetScaleFactor(s) / GetInverseScaleFactors / GetScaleSigmaSquares /
 * GetInverseScaleSigmaSquares (ORBextractor.h:115-155). Any pointer may be NULL; arrays
 * hold nlevels entries. features_per_level = mnFeaturesPerLevel (ORBextractor.cc:514-531). */
int orbx_levels(const orbx_engine *e, int *nlevels, float *scale, float *inv_scale,
                float *sigma2, float *inv_sigma2, int *features_per_level);

/* ORBextractor::operator()(image, mask, keypoints, descriptors) (ORBextractor.h:107,
 * ORBextractor.cc:1543-1658) on a host u8 image (row pitch `stride` bytes). Thread-safe across
 * engines: each engine uploads, runs and downloads on its own stream and waits for nothing
 * else, so the left / right extractors of Frame.cc:144-153 run concurrently from two threads. Writes up to
 * `cap` keypoints (level-major, quadtree list order) and N x 32 descriptor bytes; *n gets
 * the count. Empty image (w or h == 0) -> *n = 0 (reference returns untouched). The mask is
 * ignored, as in the reference. The pyramid stays resident on the device for
 * orbm_stereo_match (Frame::ComputeStereoMatches reads mvImagePyramid). */
int orbx_extract(orbx_engine *e, const uint8_t *img, int w, int h, int stride, orbx_kp *kps,
                 uint8_t *desc, int cap, int *n);

/* mvImagePyramid[level] (ORBextractor.h:158) copied to host (dst may be NULL to query w/h). */
int orbx_pyramid_level(orbx_engine *e, int image, int level, uint8_t *dst, int *w, int *h);

/* The blurred working copy of mvImagePyramid[level] that computeDescriptors samples:
 * GaussianBlur(workingMat, workingMat, Size(9, 9), 2, 2, BORDER_REFLECT_101) on a clone of the level
 * (ORBextractor.cc:1617-1625), copied to host (dst may be NULL to query w/h). Not a reference
 * interface (the reference keeps it in a local cv::Mat): exposed so the blur is checked directly. */
int orbx_blurred_level(orbx_engine *e, int image, int level, uint8_t *dst, int *w, int *h);

/* -------- batched device-resident path (many frames per launch) -------- */

/* Size device buffers for up to max_images images of w x h. */
int orbx_reserve(orbx_engine *e, int w, int h, int max_images);
/* Extract n_images frames already resident in device memory (u8, image i at
 * d_imgs + i * image_stride, rows `pitch` bytes apart; image_stride >= pitch*(h-1)+w when
 * n_images > 1). No byte outside the images' pixels is read: the last image may end exactly at
 * the end of the caller's allocation, as a cv::Mat's data does (ORBextractor.cc:1543-1560).
 * Every buffer descriptor over the input carries the level's exact extent, so the hardware
 * range check would return 0 for a byte past it instead of faulting. Asynchronous on `stream`
 * (hipStream_t; NULL = the engine's stream), ordered after the engine's previous work; results
 * stay on the device and orbx_batch_fetch waits for this engine's work only. */
int orbx_extract_batch_device(orbx_engine *e, const uint8_t *d_imgs, int n_images, int w,
                              int h, int pitch, size_t image_stride, void *stream);
/* The same in two halves on one stream, so that two engines can interleave their batches:
 * phase 1 = pyramid + FAST strength map + blur (the VALU-bound half), phase 2 = cell NMS,
 * quadtree, orientation + descriptors (latency-bound); phase 2 must follow phase 1 of the same
 * d_imgs / n_images; phase 3 = both (= orbx_extract_batch_device). */
int orbx_extract_batch_device_phase(orbx_engine *e, const uint8_t *d_imgs, int n_images, int w,
                                    int h, int pitch, size_t image_stride, void *stream, int phase);
/* Device pointers of the last batch: counts[n_images], kps[n_images][cap],
 * desc[n_images][cap][32]. */
int orbx_batch_results(orbx_engine *e, const int **d_counts, const orbx_kp **d_kps,
                       const uint8_t **d_desc, int *cap);
/* Keypoint capacity per image (the row count of the kps / desc result arrays) for the reserved
 * image size; ORBX_ESTATE before the first reserve / extraction. */
int orbx_capacity(const orbx_engine *e, int *cap);
/* Copy one image's results of the last batch to host. Waits for this engine's last launch
 * (an event), never for the device: engines on other threads keep running. */
int orbx_batch_fetch(orbx_engine *e, int image, orbx_kp *kps, uint8_t *desc, int cap, int *n);
/* The engine's HIP stream (hipStream_t). */
void *orbx_stream(orbx_engine *e);

/* -------- stereo / matching (replaces Frame::ComputeStereoMatches and the ORBmatcher
 * Hamming core) -------- */

/* Frame::ComputeStereoMatches (include/Frame.h:249, Frame.cc:831-1128) for the frame whose
 * left image was last extracted by `left` and right image by `right` (orbx_extract).
 * mbf = Camera.bf, mb = mbf / fx. Writes mvuRight[n] and mvDepth[n] (-1 = no match). */
int orbm_stereo_match(orbx_engine *left, orbx_engine *right, float mbf, float mb,
                      float *u_right, float *depth, int n);

/* Batched stereo over the engine's last device batch: image 2p = left, 2p+1 = right of
 * pair p. Results stay on device: u_right / depth [n_pairs][cap]. */
int orbm_stereo_match_batch_device(orbx_engine *e, int n_pairs, float mbf, float mb, void *stream);

/* Provenance: 16 hex digits of SHA-256 over the library's sources (tools/src_hash.py), baked in
 * at build time. Not a reference interface: profiles/ summaries carry it so a benchmark can tell
 * whether committed counter figures were measured on the library it runs. */
const char *orbx_build_id(void);

/* -------- stereo batch pipeline (Frame::Frame stereo constructor, Frame.cc:144-160, over a batch
 * of pairs) -------- */
typedef struct orbx_pipeline orbx_pipeline;
/* n_engines extractors (<= 0: 3), one HIP stream each. A batch is split into n_engines chunks of
 * consecutive pairs; each chunk runs extraction phase 1, phase 2 and ComputeStereoMatches on its
 * engine, and the chunks' phase 1 run in turn so one chunk's VALU-bound pyramid / FAST / blur
 * overlaps the other chunks' latency-bound NMS / quadtree / descriptors / stereo. Results equal
 * one engine over the whole batch. */
int orbx_pipeline_create(const orbx_params *p, int n_engines, orbx_pipeline **out);
void orbx_pipeline_destroy(orbx_pipeline *pl);
int orbx_pipeline_engines(orbx_pipeline *pl);
int orbx_pipeline_reserve(orbx_pipeline *pl, int w, int h, int max_pairs);
/* d_imgs: 2 * n_pairs device images, left / right interleaved (image i at d_imgs + i * image_stride).
 * Starts after the work queued on `stream` (hipStream_t, NULL = legacy default stream) and returns
 * without making `stream` wait for it, so consecutive batches overlap; order consumers (or reuse
 * of d_imgs) with orbx_pipeline_join or a device synchronisation. */
int orbx_pipeline_stereo_batch(orbx_pipeline *pl, const uint8_t *d_imgs, int n_pairs, int w, int h,
                               int pitch, size_t image_stride, float mbf, float mb, void *stream);
/* Engine i and its chunk [first_pair, first_pair + n_pairs) of the last batch: its results are
 * read with orbx_batch_* (images 2p, 2p + 1 of the chunk) and orbm_stereo_*. */
int orbx_pipeline_chunk(orbx_pipeline *pl, int i, orbx_engine **e, int *first_pair, int *n_pairs);
/* Make `stream` wait for every chunk of the last batch. */
int orbx_pipeline_join(orbx_pipeline *pl, void *stream);
/* Host-memory outputs of a stereo batch (the Frame members the boundary returns: mvKeys,
 * mDescriptors of both images, mvuRight, mvDepth). cap = orbx_pipeline_capacity. */
typedef struct {
    int32_t *counts;    /* [2 n_pairs] keypoints of image 2p (left) / 2p+1 (right) */
    orbx_kp *kps;       /* [2 n_pairs][cap] */
    uint8_t *desc;      /* [2 n_pairs][cap][32] */
    float *u_right;     /* [n_pairs][cap] mvuRight of the left image (-1 = none) */
    float *depth;       /* [n_pairs][cap] mvDepth */
} orbx_stereo_host_out;
/* Keypoint capacity per image of the pipeline's engines (after orbx_pipeline_reserve). */
int orbx_pipeline_capacity(orbx_pipeline *pl, int *cap);
/* The stereo batch with HOST images in and host outputs (ORBextractor::operator() takes a host
 * cv::InputArray, ORBextractor.h:107): the batch is uploaded chunk by chunk on the pipeline's H2D
 * stream into one of two device slots (batch k+1's upload overlaps batch k's kernels), each
 * engine starts when its chunk has landed, and its results are copied out on a D2H stream right
 * after its stereo pass. Returns once enqueued; orbx_pipeline_wait blocks until the outputs are
 * in host memory. h_imgs and the outputs should be pinned (orbx_host_alloc) and stay valid until
 * the wait; results equal orbx_pipeline_stereo_batch's. */
int orbx_pipeline_stereo_batch_host(orbx_pipeline *pl, const uint8_t *h_imgs, int n_pairs, int w,
                                    int h, int pitch, size_t image_stride, float mbf, float mb,
                                    const orbx_stereo_host_out *out);
int orbx_pipeline_wait(orbx_pipeline *pl);
/* Page-locked host memory (hipHostMalloc) for the host-mode buffers. */
int orbx_host_alloc(size_t bytes, void **p);
int orbx_host_free(void *p);
int orbm_stereo_results(orbx_engine *e, const float **d_u_right, const float **d_depth);
int orbm_stereo_fetch(orbx_engine *e, int pair, float *u_right, float *depth, int cap);

/* ORBmatcher::DescriptorDistance (ORBmatcher.h:65, ORBmatcher.cc:2123-2143) batched as a
 * brute-force scan: for each query row the first minimum Hamming distance over db, its
 * index and the second-best distance (best/second-best update order of ORBmatcher's
 * matchers). Host pointers. */
int orbm_hamming_best2(const uint8_t *q, int nq, const uint8_t *db, int ndb, int *best_idx,
                       int *best_d, int *second_d);

/* -------- ORBmatcher instance: ORBmatcher(float nnratio = 0.6, bool checkOri = true)
 * (include/ORBmatcher.h:57, ORBmatcher.cc:61). Holds mfNNratio / mbCheckOrientation, a private
 * HIP stream and grow-only device buffers; any number of matchers may be used from different
 * host threads concurrently (each waits only for its own work). -------- */
typedef struct orbm_matcher orbm_matcher;
int orbm_create(float nnratio, int check_ori, orbm_matcher **out);
void orbm_destroy(orbm_matcher *m);

/* The scan core of every ORBmatcher search (ORBmatcher.cc:639-668 and the same loop in the
 * SearchByProjection / SearchByBoW overloads) over caller-built candidate lists: query i's
 * candidates are cand_idx[cand_off[i] .. cand_off[i+1]) into db (CSR, cand_off[0] == 0, indices in
 * [0, ndb)). best_idx = the candidate (db index) of the FIRST minimum distance in list order,
 * best_d its distance, second_d the minimum over the other candidates (INT_MAX when there are
 * none; best_idx -1 / best_d INT_MAX for an empty list). cand_off == NULL scans all of db in index
 * order (= orbm_hamming_best2). Host pointers. SURVEY.md §8b orbm_hamming_best2. */
int orbm_hamming_best2_cand(orbm_matcher *m, const uint8_t *q, int nq, const uint8_t *db, int ndb,
                            const int32_t *cand_off, const int32_t *cand_idx, int32_t *best_idx,
                            int32_t *best_d, int32_t *second_d);
/* Device-pointer form, enqueued on `stream` (NULL = the matcher's stream); outputs stay on device. */
int orbm_hamming_best2_cand_device(orbm_matcher *m, const uint8_t *d_q, int nq, const uint8_t *d_db,
                                   int ndb, const int32_t *d_cand_off, const int32_t *d_cand_idx,
                                   int32_t *d_best_idx, int32_t *d_best_d, int32_t *d_second_d,
                                   void *stream);

/* The Frame members SearchForInitialization reads (include/Frame.h): N, mvKeysUn, mDescriptors
 * and the image bounds of the grid (static mnMinX / mnMaxX / mnMinY / mnMaxY, computed once by
 * Frame::ComputeImageBounds, Frame.cc:780-830; the grid cell inverses follow from them as in
 * Frame.cc:183-184). Host pointers. */
typedef struct {
    int32_t n;
    const orbx_kp *keys_un;   /* n undistorted keypoints, extractor order */
    const uint8_t *desc;      /* n x 32 */
    float min_x, max_x, min_y, max_y;
} orbm_frame;

/* ORBmatcher::SearchForInitialization(Frame &F1, Frame &F2, vector<cv::Point2f> &vbPrevMatched,
 * vector<int> &vnMatches12, int windowSize) (ORBmatcher.h:169, ORBmatcher.cc:580-748) with the
 * matcher's nnratio / checkOri, on two independently built host frames.
 * prev_matched: F1->n (x, y) pairs, in/out -- read as the search-window centre of each octave-0
 * F1 keypoint (:627) and overwritten with the matched F2 keypoint position (:742-745), so the
 * caller carries it from call to call as Tracking::MonocularInitialization does
 * (Tracking.cc:893-897, 929-933). matches12: F1->n entries (vnMatches12, -1 = none). *nmatches =
 * the return value of the reference. F1->n, F2->n <= 4096. Greedy order kept exactly. */
int orbm_search_for_initialization(orbm_matcher *m, const orbm_frame *F1, const orbm_frame *F2,
                                   float *prev_matched, int32_t *matches12, int window,
                                   int32_t *nmatches);

/* -------- RGB-D frame + frame-to-frame matching (C3) -------- */

/* Frame::UndistortKeyPoints (Frame.cc:725-776, cv::undistortPoints with K = {fx, fy, cx, cy}
 * and dist = {k1, k2, p1, p2, k3}; k1 == 0 -> copy) + Frame::ComputeStereoFromRGBD
 * (Frame.cc:1131-1169: depth read at the distorted keypoint, uR = xUn - mbf / d) for the
 * last extraction of `e` (image 0). depth is the CV_32F depth map (metres), dpitch floats per
 * row. Outputs mvKeysUn[n], mvuRight[n], mvDepth[n]. */
int orbf_rgbd(orbx_engine *e, const float *depth, int dpitch, const float K[4], const float dist[5],
              float mbf, orbx_kp *keys_un, float *u_right, float *depth_out, int n);
/* Same for every image of the last device batch: depth image i at d_depth + i*depth_stride
 * floats. Results stay on device (fetch with orbf_rgbd_fetch). */
int orbf_rgbd_batch_device(orbx_engine *e, const float *d_depth, size_t depth_stride, int dpitch,
                           const float K[4], const float dist[5], float mbf, void *stream);
int orbf_rgbd_fetch(orbx_engine *e, int image, orbx_kp *keys_un, float *u_right, float *depth_out,
                    int cap);

/* ORBmatcher::SearchForInitialization(F1, F2, vbPrevMatched, vnMatches12, windowSize)
 * (ORBmatcher.h:169, ORBmatcher.cc:580-748) with ORBmatcher(nnratio, checkOri), over pairs of
 * images of the last device batch: F1 = image f1_base + f1_step*p, F2 = f2_base + f2_step*p,
 * using their undistorted keypoints (orbf_rgbd_batch_device) and the Frame grid of F2
 * (Frame.cc:398-698, bounds from ComputeImageBounds with K/dist). vbPrevMatched starts at F1's
 * undistorted keypoints (Tracking::MonocularInitialization). Greedy order kept exactly. */
int orbm_search_init_batch_device(orbx_engine *e, int n_pairs, int f1_base, int f1_step, int f2_base,
                                  int f2_step, const float K[4], const float dist[5], int window,
                                  float nnratio, int check_ori, void *stream);
int orbm_search_init_fetch(orbx_engine *e, int pair, int *matches12, float *prev_xy, int cap,
                           int *nmatches);

/* -------- tracking matchers (replace Frame::isInFrustum and the two per-frame
 * ORBmatcher::SearchByProjection overloads used by Tracking) -------- */

/* The Frame members the tracking matchers read (include/Frame.h:195-300). Host pointers. */
typedef struct {
    int32_t n;                   /* N */
    const orbx_kp *keys_un;      /* mvKeysUn[N] (octave / angle equal mvKeys') */
    const float *u_right;        /* mvuRight[N]; < 0 = no stereo */
    const uint8_t *desc;         /* mDescriptors, N x 32 */
    float Tcw[12];               /* mTcw rows 0..2 = [Rcw | tcw], CV_32F */
    float Ow[3];                 /* mOw (Frame::UpdatePoseMatrices, Frame.cc:453-473) */
    float fx, fy, cx, cy, mbf, mb;
    float min_x, max_x, min_y, max_y;   /* mnMinX .. mnMaxY (Frame::ComputeImageBounds) */
    int32_t nlevels;             /* mnScaleLevels */
    float log_scale_factor;      /* mfLogScaleFactor = log(mfScaleFactor) */
    float scale_factors[16];     /* mvScaleFactors */
    float inv_level_sigma2[16];  /* mvInvLevelSigma2 (read by orbt_fuse_candidates) */
} orbt_frame;

#define ORBT_MP_BAD 1            /* MapPoint::isBad() */
#define ORBT_MP_HAS_OBS 2        /* MapPoint::Observations() > 0 */
#define ORBT_MP_IN_FRAME 4       /* mnLastFrameSeen == CurrentFrame.mnId (Tracking.cc:1749-1769) */
#define ORBT_MP_FOUND 8          /* in sAlreadyFound (ORBmatcher.cc:1951; Tracking::Relocalization) */

/* The map points a matcher reads (MapPoint getters). Host pointers. */
typedef struct {
    int32_t n;
    const float *Xw;             /* [n][3] GetWorldPos() */
    const float *normal;         /* [n][3] GetNormal() */
    const float *min_dist;       /* [n] mfMinDistance (GetMinDistanceInvariance = 0.8f * this) */
    const float *max_dist;       /* [n] mfMaxDistance (GetMaxDistanceInvariance = 1.2f * this) */
    const uint8_t *desc;         /* [n][32] GetDescriptor() */
    const uint8_t *flags;        /* [n] ORBT_MP_* */
} orbt_mappoints;

/* MapPoint tracking members written by Frame::isInFrustum (Frame.cc:556-574). Any pointer
 * may be NULL. */
typedef struct {
    uint8_t *in_view;            /* mbTrackInView */
    float *proj_x, *proj_y, *proj_xr, *view_cos;   /* mTrackProjX/Y/XR, mTrackViewCos */
    int32_t *level;              /* mnTrackScaleLevel */
} orbt_view;

typedef struct orbt_engine orbt_engine;

int orbt_create(orbt_engine **out);
void orbt_destroy(orbt_engine *e);

/* Tracking::SearchLocalPoints (Tracking.cc:1745-1810) minus the MapPoint counters:
 * mbTrackInView = !(flags & (BAD | IN_FRAME)) && Frame::isInFrustum(pMP, view_cos_limit)
 * (Frame.cc:490-578, PredictScale MapPoint.cc:612-626), then
 * ORBmatcher(nnratio).SearchByProjection(F, vpMapPoints, th) (ORBmatcher.h:82,
 * ORBmatcher.cc:78-176) with the reference's greedy claim order (map points in order; a
 * keypoint owned by a map point with Observations() > 0 is skipped by later ones).
 * kp_blocked[N] (may be NULL): 1 where F.mvpMapPoints[idx] holds a point with
 * Observations() > 0 on entry. owner[N] out: map point index assigned to keypoint idx, or
 * -1 = untouched. view may be NULL. */
int orbt_search_local_points(orbt_engine *e, const orbt_frame *F, const orbt_mappoints *M,
                             float view_cos_limit, float th, float nnratio, const uint8_t *kp_blocked,
                             orbt_view *view, int32_t *owner, int32_t *nmatches);

/* ORBmatcher(nnratio, check_ori).SearchByProjection(CurrentFrame, LastFrame, th, bMono)
 * (ORBmatcher.h:102, ORBmatcher.cc:1741-1904; Tracking::TrackWithMotionModel). last_mp[i]
 * = index into M of LastFrame.mvpMapPoints[i] (-1 = NULL); last_outlier[i] = mvbOutlier[i]
 * (may be NULL). owner[cur->n] out: -1 untouched, >= 0 map point index assigned, -2 =
 * assigned and then cleared by the rotation-consistency check (mvpMapPoints[idx] = NULL).
 * *nmatches = the reference's return value. */
int orbt_search_by_projection_frame(orbt_engine *e, const orbt_frame *cur, const orbt_frame *last,
                                    const int32_t *last_mp, const uint8_t *last_outlier,
                                    const orbt_mappoints *M, float th, int mono, int check_ori,
                                    const uint8_t *kp_blocked, int32_t *owner, int32_t *nmatches);

/* ORBmatcher(0.9, check_ori).SearchByProjection(CurrentFrame, pKF, sAlreadyFound, th, ORBdist)
 * (ORBmatcher.h:116, ORBmatcher.cc:1922-2066; Tracking::Relocalization, th 10 / 3, ORBdist
 * 100 / 64). `kf` carries pKF->mvKeysUn (angles); kf_mp[i] = index into M of
 * pKF->GetMapPointMatches()[i] (-1 = NULL); M->flags ORBT_MP_FOUND = in sAlreadyFound.
 * kp_blocked[cur->n] (may be NULL) = CurrentFrame.mvpMapPoints[i2] != NULL on entry; a keypoint
 * claimed by an earlier point is skipped by later ones (greedy, point order). Frame pose,
 * bounds, grid, scale tables are `cur`'s. owner / nmatches as for
 * orbt_search_by_projection_frame. */
int orbt_search_by_projection_keyframe(orbt_engine *e, const orbt_frame *cur, const orbt_frame *kf,
                                       const int32_t *kf_mp, const orbt_mappoints *M, float th,
                                       int orb_dist, int check_ori, const uint8_t *kp_blocked,
                                       int32_t *owner, int32_t *nmatches);

/* ORBmatcher::Fuse(pKF, vpMapPoints, th) (ORBmatcher.h:208, ORBmatcher.cc:1139-1278; th = 3 from
 * LocalMapping::SearchInNeighbors) -- the search half. `kf` is the KeyFrame (pose, calibration,
 * bounds, grid keypoints, mvuRight, descriptors, mvScaleFactors, mvInvLevelSigma2); flags
 * ORBT_MP_IN_FRAME = pMP->IsInKeyFrame(pKF). For every other non-bad point: projection,
 * IsInImage, scale-invariance and viewing-angle gates, PredictScale(dist, pKF), window,
 * level and chi2 (5.99 / 7.8) gates, first minimum Hamming distance -> best_idx[m] (-1 = no
 * candidate) and best_dist[m]. The search of a point does not depend on the map updates of
 * earlier points, so all points run in parallel; the caller applies the reference's updates
 * (Replace / AddObservation, :1245-1271) in point order for best_dist <= 50, re-checking
 * isBad / IsInKeyFrame, exactly as the reference loop does. */
int orbt_fuse_candidates(orbt_engine *e, const orbt_frame *kf, const orbt_mappoints *M, float th,
                         int32_t *best_idx, int32_t *best_dist);

/* LoopClosing's ORBmatcher::SearchByProjection(pKF, Scw, vpPoints, vpMatched, th) (ORBmatcher.h:126,
 * ORBmatcher.cc:431-560; LoopClosing::ComputeSim3 with th = 10). `kf` = pKF (its Tcw / Ow are ignored:
 * the pose is Scw, row-major 4x4 CV_32F [sR | t], unscaled as the reference does), M = vpPoints
 * (ORBT_MP_BAD = isBad()), matched[kf->n] in/out = vpMatched as indices into M (-1 = NULL, <= -2 =
 * a map point outside vpPoints: the keypoint stays taken). Greedy in point order, every claim
 * blocks later points, first minimum Hamming distance <= TH_LOW. *nmatches = the return value. */
int orbt_search_by_projection_sim3(orbt_engine *e, const orbt_frame *kf, const float Scw[16],
                                   const orbt_mappoints *M, int th, int32_t *matched, int32_t *nmatches);

/* LoopClosing's ORBmatcher::Fuse(pKF, Scw, vpPoints, th, vpReplacePoint) (ORBmatcher.h:215,
 * ORBmatcher.cc:1321-1458; LoopClosing::SearchAndFuse th = 4) -- the search half: pose = Scw
 * unscaled, flags ORBT_MP_IN_FRAME = in pKF->GetMapPoints(); best_idx[m] / best_dist[m] = the
 * first minimum over the window at levels [l - 1, l] (-1 / INT_MAX = no candidate). The caller
 * applies the reference's update for best_dist <= 50 (vpReplacePoint / AddObservation, :1439-1453). */
int orbt_fuse_sim3_candidates(orbt_engine *e, const orbt_frame *kf, const float Scw[16], const orbt_mappoints *M,
                              float th, int32_t *best_idx, int32_t *best_dist);

/* ORBmatcher::SearchBySim3(pKF1, pKF2, vpMatches12, s12, R12, t12, th) (ORBmatcher.h:197,
 * ORBmatcher.cc:1472-1723; LoopClosing::ComputeSim3 th = 7.5): kf1_mp / kf2_mp =
 * GetMapPointMatches() as indices into M (-1 = NULL), matches12[kf1->n] in/out = vpMatches12 (-1 =
 * NULL). Both projection directions run in parallel (no claims), then the mutual-agreement check;
 * *nfound = the return value. R12 row-major CV_32F, t12 CV_32F. */
int orbt_search_by_sim3(orbt_engine *e, const orbt_frame *kf1, const int32_t *kf1_mp, const orbt_frame *kf2,
                        const int32_t *kf2_mp, const orbt_mappoints *M, float s12, const float R12[9],
                        const float t12[3], float th, int32_t *matches12, int32_t *nfound);

/* Batched device-resident form (throughput path): stage independent problems into slots
 * (host -> HBM), run one launch chain over all slots, fetch per slot. `last`, `last_mp`,
 * `last_outlier` may be NULL when only orbt_run_local_batch is used. */
int orbt_reserve(orbt_engine *e, int n_slots, int cap_kp, int cap_mp);
int orbt_stage(orbt_engine *e, int slot, const orbt_frame *F, const orbt_mappoints *M,
               const orbt_frame *last, const int32_t *last_mp, const uint8_t *last_outlier,
               const uint8_t *kp_blocked);
int orbt_run_local_batch(orbt_engine *e, int n_slots, float view_cos_limit, float th, float nnratio,
                         void *stream);
int orbt_run_frame_batch(orbt_engine *e, int n_slots, float th, int mono, int check_ori, void *stream);
/* relocalisation matcher over staged slots: `last` = the keyframe, `last_mp` = its matches */
int orbt_run_reloc_batch(orbt_engine *e, int n_slots, float th, int orb_dist, int check_ori, void *stream);
int orbt_run_fuse_batch(orbt_engine *e, int n_slots, float th, void *stream);
/* loop-closing projection search over slots staged with orbt_stage_sim3; orbt_fetch's owner[i] is
 * the newly matched point of keypoint i (-1 = none: vpMatched[i] unchanged) */
int orbt_stage_sim3(orbt_engine *e, int slot, const orbt_frame *kf, const float Scw[16], const orbt_mappoints *M,
                    const int32_t *matched);
int orbt_run_sim3_batch(orbt_engine *e, int n_slots, int th, void *stream);
/* Fuse(pKF, Scw, ...) search half over slots (fetch with orbt_fetch_fuse) */
int orbt_stage_fuse_sim3(orbt_engine *e, int slot, const orbt_frame *kf, const float Scw[16],
                         const orbt_mappoints *M);
int orbt_run_fuse_sim3_batch(orbt_engine *e, int n_slots, float th, void *stream);
/* SearchBySim3 pair k uses slots 2k and 2k + 1 (one per projection direction) */
int orbt_stage_search_by_sim3(orbt_engine *e, int pair, const orbt_frame *kf1, const int32_t *kf1_mp,
                              const orbt_frame *kf2, const int32_t *kf2_mp, const orbt_mappoints *M, float s12,
                              const float R12[9], const float t12[3], const int32_t *matches12);
int orbt_run_sim3_match_batch(orbt_engine *e, int n_pairs, float th, void *stream);
int orbt_fetch_search_by_sim3(orbt_engine *e, int pair, const int32_t *kf2_mp, int32_t *matches12, int32_t *nfound);
int orbt_fetch_fuse(orbt_engine *e, int slot, int32_t *best_idx, int32_t *best_dist);
int orbt_fetch(orbt_engine *e, int slot, orbt_view *view, int32_t *owner, int32_t *nmatches);

/* -------- bag of words (replaces Frame::ComputeBoW -> DBoW2 TemplatedVocabulary::transform) -------- */

/* A DBoW2 TemplatedVocabulary<FORB::TDescriptor, FORB> (Thirdparty/DBoW2/DBoW2/
 * TemplatedVocabulary.h) in the order loadFromTextFile (:1385-1460) builds it: node 0 is the
 * root, node i >= 1 is the i-th node line of the text file (parent id, isLeaf, 32 descriptor
 * bytes, weight); children keep file order; word ids are given to leaves in file order.
 * scoring = ScoringType (L1_NORM = 0 .. DOT_PRODUCT = 5), weighting = WeightingType
 * (TF_IDF = 0, TF, IDF, BINARY). ORBvoc.txt is k = 10, L = 6, L1_NORM, TF_IDF. */
typedef struct orbv_vocab orbv_vocab;

int orbv_create(int k, int L, int scoring, int weighting, int n_nodes, const int32_t *parent,
                const uint8_t *is_leaf, const uint8_t *desc, const double *weight, orbv_vocab **out);
/* TemplatedVocabulary::loadFromTextFile (TemplatedVocabulary.h:1385-1460). */
int orbv_load_text(const char *path, orbv_vocab **out);
void orbv_destroy(orbv_vocab *v);
/* nodes / words / k / L of a loaded vocabulary (any pointer may be NULL) */
int orbv_info(const orbv_vocab *v, int *n_nodes, int *n_words, int *k, int *L);

/* TemplatedVocabulary::transform(features, BowVector&, FeatureVector&, levelsup)
 * (TemplatedVocabulary.h:1125-1209, per-feature descent :1226-1286; Frame::ComputeBoW calls it
 * with levelsup = 4, Frame.cc:704-719) on n descriptors (N x 32, host). Outputs:
 *   BowVector     words[n_words] ascending with values[n_words] (after the scoring's norm);
 *   FeatureVector fv_nodes[n_fv] ascending, the features of fv_nodes[j] are
 *                 fv_features[fv_start[j] .. fv_start[j+1]) in increasing index order.
 * Capacities: words / values / fv_nodes n entries, fv_start n + 1, fv_features n. */
int orbv_transform(orbv_vocab *v, const uint8_t *desc, int n, int levelsup, uint32_t *words, double *values,
                   int32_t *n_words, uint32_t *fv_nodes, int32_t *fv_start, int32_t *fv_features, int32_t *n_fv);
/* Batched device-resident form: descriptors of frame f at d_desc + f * frame_stride (N x 32
 * bytes, counts in d_counts[f] <= cap); results stay on the device, fetched per frame. */
int orbv_transform_batch_device(orbv_vocab *v, const uint8_t *d_desc, const int32_t *d_counts, int n_frames,
                                int cap, size_t frame_stride, int levelsup, void *stream);
int orbv_batch_fetch(orbv_vocab *v, int frame, uint32_t *words, double *values, int32_t *n_words,
                     uint32_t *fv_nodes, int32_t *fv_start, int32_t *fv_features, int32_t *n_fv);

/* -------- BoW-guided matchers (replace ORBmatcher::SearchByBoW(KeyFrame*, Frame&, ...) and
 * ORBmatcher::SearchForTriangulation) -------- */

/* A KeyFrame (or Frame) as the BoW matchers read it (include/KeyFrame.h). Host pointers. */
typedef struct {
    int32_t n;                   /* N */
    const orbx_kp *keys_un;      /* mvKeysUn (angle / octave / pt) */
    const float *u_right;        /* mvuRight */
    const uint8_t *desc;         /* mDescriptors, N x 32 */
    const int32_t *mp;           /* GetMapPoint(i) as an index into the caller's point table, -1 = NULL */
    const uint8_t *mp_bad;       /* [N] 1 if that map point isBad() (may be NULL = none bad) */
    int32_t n_fv;                /* mFeatVec: n_fv nodes ascending, features of node j are */
    const uint32_t *fv_nodes;    /*   fv_features[fv_start[j] .. fv_start[j+1]) */
    const int32_t *fv_start;
    const int32_t *fv_features;
    float fx, fy, cx, cy;        /* KeyFrame calibration */
    int32_t nlevels;
    float scale_factors[16];     /* mvScaleFactors */
    float level_sigma2[16];      /* mvLevelSigma2 */
} orbb_keyframe;

typedef struct orbb_engine orbb_engine;
int orbb_create(orbb_engine **out);
void orbb_destroy(orbb_engine *e);

/* ORBmatcher(nnratio, check_ori).SearchByBoW(pKF, F, vpMapPointMatches) (ORBmatcher.h:148,
 * ORBmatcher.cc:236-353; Tracking::TrackReferenceKeyFrame / Relocalization). matches[F.n] out:
 * the KF map-point index matched to frame keypoint i, -1 = NULL. Feature-vector nodes are
 * independent (a frame keypoint belongs to one node), so each shared node is one wavefront
 * that keeps the reference's greedy order inside the node. */
int orbb_search_by_bow(orbb_engine *e, const orbb_keyframe *kf, const orbb_keyframe *f, float nnratio,
                       int check_ori, int32_t *matches, int32_t *nmatches);

/* ORBmatcher(0.6, check_ori).SearchForTriangulation(pKF1, pKF2, F12, vMatchedPairs, bOnlyStereo)
 * (ORBmatcher.h:181, ORBmatcher.cc:915-1089; LocalMapping::CreateNewMapPoints). F12 row-major
 * CV_32F (LocalMapping::ComputeF12), Cw1 = pKF1->GetCameraCenter(), T2w = pKF2 [R2w | t2w]
 * rows. pairs[2 * k] = idx1, pairs[2 * k + 1] = idx2 of the k-th vMatchedPairs entry (idx1
 * ascending); capacity kf1->n pairs. */
int orbb_search_for_triangulation(orbb_engine *e, const orbb_keyframe *kf1, const orbb_keyframe *kf2,
                                  const float F12[9], const float Cw1[3], const float T2w[12], int only_stereo,
                                  int check_ori, int32_t *pairs, int32_t *npairs);
/* ORBmatcher(nnratio, check_ori).SearchByBoW(pKF1, pKF2, vpMatches12) (ORBmatcher.h:151,
 * ORBmatcher.cc:760-903; LoopClosing::ComputeSim3 with ORBmatcher(0.75, true)). matches12[kf1->n]
 * out: the kf2 map-point index (kf2->mp) matched to keypoint idx1 of kf1, -1 = NULL. Both
 * sides need a map point that is not bad (mp_bad); KF2 keypoints are claimed (vbMatched2). */
int orbb_search_by_bow_kf(orbb_engine *e, const orbb_keyframe *kf1, const orbb_keyframe *kf2, float nnratio,
                          int check_ori, int32_t *matches12, int32_t *nmatches);

/* Batched device-resident form: stage (a, b) pairs into slots -- SearchByBoW reads a = KeyFrame,
 * b = Frame (or KeyFrame 2); SearchForTriangulation a = KF1, b = KF2 (F12 / Cw1 / T2w may be NULL
 * for SearchByBoW) -- run one launch chain over all slots, fetch per slot (tri = 0:
 * matches[b.n], tri = 1: pairs[2 * n], tri = 2: matches12[a.n] of orbb_run_bowkf_batch). */
int orbb_reserve(orbb_engine *e, int n_slots, int cap_kp);
int orbb_stage(orbb_engine *e, int slot, const orbb_keyframe *a, const orbb_keyframe *b, const float F12[9],
               const float Cw1[3], const float T2w[12]);
int orbb_run_bow_batch(orbb_engine *e, int n_slots, float nnratio, int check_ori, void *stream);
int orbb_run_tri_batch(orbb_engine *e, int n_slots, int only_stereo, int check_ori, void *stream);
int orbb_run_bowkf_batch(orbb_engine *e, int n_slots, float nnratio, int check_ori, void *stream);
int orbb_fetch(orbb_engine *e, int slot, int tri, int32_t *out, int32_t *n);

/* -------- pose-only optimisation (replaces Optimizer::PoseOptimization) -------- */

/* The edges Optimizer::PoseOptimization (Optimizer.h:105, Optimizer.cc:375-622) builds from a
 * Frame: one per keypoint i with pFrame->mvpMapPoints[i] != NULL, in keypoint order
 * (the caller compacts them; edge k <-> keypoint i_k). obs = (mvKeysUn[i].pt, mvuRight[i]):
 * uR < 0 -> EdgeSE3ProjectXYZOnlyPose (mono), else EdgeStereoSE3ProjectXYZOnlyPose. */
typedef struct {
    int32_t n;                   /* edges */
    const float *Xw;             /* [n][3] MapPoint::GetWorldPos() */
    const float *obs;            /* [n][3] u, v, uR */
    const float *inv_sigma2;     /* [n] mvInvLevelSigma2[mvKeysUn[i].octave] */
    float Tcw[16];               /* pFrame->mTcw (row-major, CV_32F), the start of every round */
    float fx, fy, cx, cy, bf;    /* Frame::fx.. and mbf */
} orbp_frame;

typedef struct {
    float Tcw[16];               /* pFrame->SetPose(...) value (unchanged input if < 3 edges) */
    uint8_t *outlier;            /* [n] out: pFrame->mvbOutlier[i_k] */
    int32_t n_inliers;           /* the return value: nInitialCorrespondences - nBad (0 if < 3) */
    int32_t iterations[4];       /* LM iterations per round (-1 = round not run) */
} orbp_result;

typedef struct orbp_engine orbp_engine;

int orbp_create(orbp_engine **out);
void orbp_destroy(orbp_engine *e);
/* Optimizer::PoseOptimization(Frame*): four rounds of optimize(10) from the frame's pose with
 * Huber kernels in rounds 0-2, outliers (chi2 > 5.991 mono / 7.815 stereo on g2o's last
 * _error) moved to level 1 between rounds. The whole Levenberg-Marquardt loop runs on the GPU
 * (one workgroup per frame, no host round trips). */
int orbp_pose_optimization(orbp_engine *e, const orbp_frame *f, orbp_result *r);
/* Batched device-resident form: stage frames into slots, one launch solves every slot. */
int orbp_reserve(orbp_engine *e, int n_slots, int cap_edges);
int orbp_stage(orbp_engine *e, int slot, const orbp_frame *f);
int orbp_run_batch(orbp_engine *e, int n_slots, void *stream);
int orbp_fetch(orbp_engine *e, int slot, orbp_result *r);

/* -------- new map points (replaces the triangulation loop of LocalMapping::CreateNewMapPoints) -------- */

/* A KeyFrame as LocalMapping::CreateNewMapPoints (LocalMapping.cc:295-600) reads it. Host pointers. */
typedef struct {
    int32_t n;                   /* N */
    const orbx_kp *keys;         /* mvKeys (KeyFrame::UnprojectStereo reads the distorted pt) */
    const orbx_kp *keys_un;      /* mvKeysUn */
    const float *u_right;        /* mvuRight */
    const float *depth;          /* mvDepth */
    float Tcw[12];               /* GetPose() rows 0..2 = [Rcw | tcw], CV_32F */
    float Ow[3];                 /* GetCameraCenter() (= Twc translation, KeyFrame::SetPose) */
    float fx, fy, cx, cy, invfx, invfy, mb, mbf;
    int32_t nlevels;
    float scale_factors[16];     /* mvScaleFactors */
    float level_sigma2[16];      /* mvLevelSigma2 */
} orbn_keyframe;

typedef struct orbn_engine orbn_engine;
int orbn_create(orbn_engine **out);
void orbn_destroy(orbn_engine *e);

/* The per-match body of LocalMapping::CreateNewMapPoints (LocalMapping.cc:396-600) for one
 * (mpCurrentKeyFrame = kf1, pKF2 = kf2) neighbour: pairs[2k], pairs[2k+1] = vMatchedIndices[k]
 * (orbb_search_for_triangulation's output). Parallax test, linear triangulation by
 * cv::SVD(A, MODIFY_A | FULL_UV) (OpenCV's float Jacobi SVD) or KeyFrame::UnprojectStereo,
 * positive depth, reprojection chi2 (5.991 / 7.8) in both keyframes, scale consistency with
 * ratio_factor = 1.5f * mpCurrentKeyFrame->mfScaleFactor. ok[k] = 1 where the reference creates
 * a MapPoint at x3d[3k..3k+2]; *nnew = their count. The baseline test and F12 before the
 * matcher, and the MapPoint bookkeeping after, stay with the caller (per keyframe, not per
 * match). */
int orbn_triangulate(orbn_engine *e, const orbn_keyframe *kf1, const orbn_keyframe *kf2, const int32_t *pairs,
                     int32_t npairs, float ratio_factor, float *x3d, uint8_t *ok, int32_t *nnew);
/* Batched device-resident form: stage (kf1, kf2, pairs) into slots, one launch for all. */
int orbn_reserve(orbn_engine *e, int n_slots, int cap_kp, int cap_pairs);
int orbn_stage(orbn_engine *e, int slot, const orbn_keyframe *kf1, const orbn_keyframe *kf2, const int32_t *pairs,
               int32_t npairs, float ratio_factor);
int orbn_run_batch(orbn_engine *e, int n_slots, void *stream);
int orbn_fetch(orbn_engine *e, int slot, float *x3d, uint8_t *ok, int32_t *nnew);

/* -------- local bundle adjustment (replaces Optimizer::LocalBundleAdjustment) -------- */

/* The graph Optimizer::LocalBundleAdjustment (Optimizer.cc:646-898) builds from the map,
 * flattened by the caller's graph walk (local KFs, fixed KFs, local map points and their
 * observations). Poses cross the boundary as cv::Mat CV_32F Tcw, points as CV_32F Xw
 * (Converter::toSE3Quat / toVector3d, Converter.cc:63-139). Edges are in g2o insertion
 * order: local map points in list order, each point's observations in map order
 * (Optimizer.cc:806-898). edge_obs = (u, v, uR) of the undistorted keypoint; uR < 0 ->
 * monocular EdgeSE3ProjectXYZ, else EdgeStereoSE3ProjectXYZ. */
typedef struct {
    int32_t n_poses;
    const int32_t *pose_id;      /* vertex id (KeyFrame::mnId) */
    const uint8_t *pose_fixed;   /* mnId == 0 or a fixed (non-local) camera */
    const float *pose_Tcw;       /* [n_poses][16] row-major 4x4 */
    const float *pose_cam;       /* [n_poses][5] fx, fy, cx, cy, bf (KeyFrame members) */
    int32_t n_points;
    const int32_t *point_id;     /* vertex id = MapPoint::mnId + maxKFid + 1 */
    const float *point_Xw;       /* [n_points][3] */
    int32_t n_edges;
    const int32_t *edge_point;   /* index into points */
    const int32_t *edge_pose;    /* index into poses */
    const float *edge_obs;       /* [n_edges][3] */
    const float *edge_inv_sigma2;/* mvInvLevelSigma2[octave] */
} lba_problem;

typedef struct {
    float *pose_Tcw;             /* [n_poses][16] out: SetPose(Converter::toCvMat(...)) */
    float *point_Xw;             /* [n_points][3] out: SetWorldPos */
    uint8_t *edge_erase;         /* [n_edges] out: 1 = pair in vToErase (Optimizer.cc:977-1008) */
    int32_t iterations[2];       /* LM iterations run in optimize(5) / optimize(10) */
    double chi2[2];              /* active robust chi2 after each phase */
    int32_t stopped;             /* 2 = *stop set before optimising: early return, outputs =
                                    inputs, nothing to write back (Optimizer.cc:902-904);
                                    1 = raised during the optimisation: phase 2 skipped (:913-917)
                                    or cut short; 0 = both phases ran to their own end */
    int32_t trials[2];           /* LM trials (solve + update + chi2 evaluations) per phase */
} lba_result;

typedef struct lba_engine lba_engine;

/* Optimizer::LocalBundleAdjustment(KeyFrame*, bool* pbStopFlag, Map*) (Optimizer.h:112,
 * Optimizer.cc:646-1049) minus the map walk / write-back, which stay in the caller's
 * adapter: two Levenberg-Marquardt runs (5 iterations with Huber kernels, then 10 without
 * the outliers, optimization_algorithm_levenberg.cpp:61-164) with the Schur complement onto
 * the poses (block_solver.hpp:354-486) on the GPU. `stop` is pbStopFlag itself (a C++ bool, read
 * as one byte; NULL = none), with the reference's semantics: checked before optimising
 * (Optimizer.cc:902-904) and between the phases (:913-917) on the host, and inside each
 * optimize() where g2o checks SparseOptimizer::terminate() -- after every rejected LM trial
 * (optimization_algorithm_levenberg.cpp:149) and before every iteration (sparse_optimizer.cpp:376)
 * -- by the device itself: while the call runs, the host copies *stop into a page-locked,
 * device-mapped word that the LM decision kernel reads with a system-scope load, so a flag raised
 * by another thread mid-call ends the optimisation after the trial in flight. With a non-NULL
 * `stop` the call polls its stream instead of blocking in hipStreamSynchronize: a short spin, then
 * sched_yield() between queries (sleeps past 2 ms), so the core goes to any thread that wants it. */
int lba_create(lba_engine **out);
void lba_destroy(lba_engine *e);
int lba_solve(lba_engine *e, const lba_problem *p, lba_result *r, const volatile uint8_t *stop);
/* Test hook (no reference counterpart): every later lba_solve on `e` behaves as if pbStopFlag were
 * raised the moment trial `trial` (1-based; 0 = before the first iteration) of optimize() call
 * `phase` (1 = optimize(5), 2 = optimize(10)) has completed, and stayed raised. phase 0 removes
 * the hook. The CPU oracle has the same hook (lba_oracle_solve_hook), so a stop at any (phase,
 * trial) is parity-tested deterministically. phase 3: a live raise at a deterministic point -- once
 * the call has read back its trial-th chunk of LM trials (trial >= 1; no effect when `stop` is NULL),
 * the flag the device sees reads as raised for the rest of the call, through the same mirrored word
 * as another thread setting mbAbortBA would (the caller's flag itself is never written). */
int lba_set_stop_hook(lba_engine *e, int phase, int trial);
/* Test options (no reference counterpart; the defaults are the product's):
 *   LBA_OPT_FUSE_FINISH  1 (default): the Schur finish and the Cholesky of a window of <= 21 free
 *                        poses in one launch with an in-launch hand-off; 0: two launches. Both give
 *                        bit-identical results (tests/test_lba_gpu.py).
 *   LBA_OPT_SPIN_LIMIT   the in-launch hand-off wait's poll bound; < 0: the default (~1 s); 0: every
 *                        wait times out (fault injection). A timed-out wait ends the optimisation and
 *                        lba_solve returns ORBX_EDEVICE.
 *   LBA_OPT_STREAM_PRIORITY  the engine's stream recreated at the device's lowest (0) or highest (1,
 *                        the default) stream priority (LocalBA beside a saturating extraction stream,
 *                        DESIGN §5). */
#define LBA_OPT_FUSE_FINISH 1
#define LBA_OPT_SPIN_LIMIT 2
#define LBA_OPT_STREAM_PRIORITY 3
int lba_set_test_option(lba_engine *e, int option, long long value);
/* Per-kernel hipEvent timing of lba_solve's trial chain on the engine stream (bench.py localba
 * roofline); same semantics as orbx_profile / orbx_profile_read. */
int lba_profile(lba_engine *e, int enable);
int lba_profile_read(lba_engine *e, int idx, char *name, int name_cap, double *total_ms, int *launches);

/* -------- library / measurement -------- */
const char *orbslam2_amd_version(void);
int orbslam2_amd_device_count(void);
/* hipSetDevice for the calling thread (engines bind the current device at create). */
int orbslam2_amd_set_device(int device);
/* hipDeviceSynchronize on this library's HIP runtime. */
int orbslam2_amd_device_sync(void);
/* Per-kernel hipEvent timing on the launch stream (bench roofline). enable != 0 clears
 * and starts recording; orbx_profile_read aggregates record idx (0..) by kernel name and
 * returns ORBX_ESTATE past the last name. No reference counterpart (the reference only
 * times whole frames, stereo_kitti.cc:96-102). */
int orbx_profile(orbx_engine *e, int enable);
int orbx_profile_read(orbx_engine *e, int idx, char *name, int name_cap, double *total_ms,
                      int *launches);

#ifdef __cplusplus
}
#endif
#endif
