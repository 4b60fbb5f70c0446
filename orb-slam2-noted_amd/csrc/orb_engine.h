// Host-side engine state shared by the extractor, stereo and matcher translation units.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <string>
#include <vector>

#include "orbslam2_amd.h"

#define ORBX_MAXL 16
#define ORBX_TMAX 66          // max FAST cell ROI side (hCell + 6, wCell + 6)
#define ORBX_QT_THREADS 256   // quadtree workgroup

namespace orbamd {

// One FAST cell of ComputeKeyPointsOctTree's grid (ORBextractor.cc:1084-1153): the ROI
// [r0, r0+rh) x [c0, c0+rw) of level `level`, and the cell offset (j*wCell, i*hCell) that
// is added to every keypoint (:1141-1146).
struct CellDesc {
    int16_t level, r0, c0, rh, rw, offx, offy, pad;
};

// Per-launch geometry, passed by value to every extraction kernel.
struct ExtractGeom {
    int nlevels, W, H, nimg;
    int lw[ORBX_MAXL], lh[ORBX_MAXL];
    long long pyr_off[ORBX_MAXL];   // level >= 1 offset inside an image's pyramid block
    long long blur_off[ORBX_MAXL];  // offset inside an image's blurred block (all levels)
    int bp[ORBX_MAXL];              // blurred / strength-map row pitch (lw rounded up to 16)
    long long pyr_stride, blur_stride;
    int in_pitch;
    long long in_stride;
    int cell_base[ORBX_MAXL + 1];
    int cell_cap, ncell_total;
    int N[ORBX_MAXL], nIni[ORBX_MAXL];
    float hX[ORBX_MAXL];
    int maxBX[ORBX_MAXL], maxBY[ORBX_MAXL];
    int out_cap[ORBX_MAXL], out_base[ORBX_MAXL + 1];
    long long qt_off[ORBX_MAXL + 1];  // global fallback key scratch (u32) per level
    int node_cap;                      // max live nodes over levels (quadtree)
    int node_pow2;                     // next pow2 >= node_cap
    long long qt_node_stride;          // u32 words of global node scratch per (image, level)
    int qt_nodes_in_lds;
    int qt_kl;                         // LDS key capacity (candidates) of the quadtree workgroup
    float scale[ORBX_MAXL];
    int scaled_patch[ORBX_MAXL];
    int ini_th, min_th, resize_mode;
    int rz_col_off[ORBX_MAXL], rz_row_off[ORBX_MAXL], rz_simd_end[ORBX_MAXL];
    int blur_tiles_x[ORBX_MAXL], blur_tiles_y[ORBX_MAXL], blur_tile_base[ORBX_MAXL + 1];
    int nms_sm_words, nms_wave_words, nms_mask_off;  // per-wavefront LDS of the cell NMS kernel (u32 words)
};

struct DevBuf {
    void *p = nullptr;
    size_t bytes = 0;
    void release();
    int ensure(size_t n);  // grow-only
    template <class T> T *as() const { return (T *)p; }
};

}  // namespace orbamd

struct orbx_engine {
    orbx_params p{};
    int device = 0;
    hipStream_t stream = nullptr;
    // extractor tables (ORBextractor.cc:471-579)
    float scale[ORBX_MAXL]{}, inv_scale[ORBX_MAXL]{}, sigma2[ORBX_MAXL]{}, inv_sigma2[ORBX_MAXL]{};
    int nfeat[ORBX_MAXL]{};
    int umax[16]{};
    int rz_rows[ORBX_MAXL]{};   // source rows per resize tile, per level
    int8_t pattern[1024]{};
    // geometry for the reserved image size
    int W = 0, H = 0, max_images = 0;
    orbamd::ExtractGeom g{};
    std::vector<orbamd::CellDesc> cells;
    // device buffers
    orbamd::DevBuf d_mmap, d_cells, d_rz, d_rzr, d_pattern, d_in, d_pyr, d_blur, d_cell_cnt, d_cell_keys,
        d_qt, d_qt_nodes, d_sel, d_sel_cnt, d_kps, d_desc, d_cnt;
    // stereo
    orbamd::DevBuf d_st_sorted, d_st_res, d_st_u, d_st_depth, d_st_dist, d_st_rows;
    // last extraction (device pointers of level-0 input)
    const uint8_t *last_in = nullptr;
    const uint8_t *pending_in = nullptr;   // phase-1 batch awaiting phase 2
    int pending_n = 0;
    int last_pitch = 0;
    long long last_stride = 0;
    int last_n = 0;
    std::string err;
    // per-kernel hipEvent profiling (bench.py roofline), recorded on the launch stream
    bool prof = false;
    struct ProfRec { const char *name; hipEvent_t a, b; };
    std::vector<ProfRec> prof_recs;
    std::vector<hipEvent_t> ev_pool;
    size_t ev_used = 0;
};

namespace orbamd {
// profiling helpers: prof_begin records a start event (returns a handle), prof_end the
// matching stop event; both are no-ops when profiling is off.
int prof_begin(orbx_engine *e, hipStream_t s);
void prof_end(orbx_engine *e, hipStream_t s, int h, const char *name);
int engine_reserve(orbx_engine *e, int w, int h, int max_images);
int engine_extract_device(orbx_engine *e, const uint8_t *d_imgs, int n, int pitch,
                          long long stride, hipStream_t s, int phase);
}  // namespace orbamd
