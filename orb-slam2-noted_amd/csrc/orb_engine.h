// Host-side engine state shared by the extractor, stereo and matcher translation units.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <cstdlib>
#include <string>
#include <vector>

#include "orbslam2_amd.h"

#define ORBX_MAXL 16
#define ORBX_TMAX 66          // max FAST cell ROI side (hCell + 6, wCell + 6)
#define ORBX_QT_THREADS 256   // quadtree workgroup

namespace orbamd {

// Marginal-cost experiments (tools/skip_exp.py): ORBX_EXP_TWICE = bit mask of idempotent kernels
// launched twice per batch (1 resize chain, 2 quadtree, 4 describe, 8 stereo_match_left); the
// step time difference against 0 is that kernel's marginal cost inside the pipeline. 0 (unset)
// in every product run.
// Experiment knobs (tools/gpu_*.sh) are read from the environment only by `make variant`
// builds (-DORBX_EXPERIMENTS=1, a build id of their own): the product library ignores them, so a
// stray variable cannot change its results or its speed.
#ifndef ORBX_EXPERIMENTS
#define ORBX_EXPERIMENTS 0
#endif
inline int orbx_knob(const char *name, int dflt) {
#if ORBX_EXPERIMENTS
    const char *ev = std::getenv(name);
    return ev ? std::atoi(ev) : dflt;
#else
    (void)name;
    return dflt;
#endif
}

// Memory-layout knobs of the quadtree (ORBX_QT_LDS_KB, ORBX_QT_NODES_LDS) stay readable in the
// product: every layout gives the same results (tests/test_extract_gpu.py::
// test_extract_quadtree_layouts runs each one against the oracle), only the speed differs.
inline int orbx_layout_knob(const char *name, int dflt) {
    const char *ev = std::getenv(name);
    return ev ? std::atoi(ev) : dflt;
}

inline int exp_twice() {
    static const int v = orbx_knob("ORBX_EXP_TWICE", 0);
    return v;
}

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
    int bp[ORBX_MAXL];              // pyramid row pitch of levels >= 1 (lw rounded up to 16)
    int bbp[ORBX_MAXL];             // blurred-level row pitch (lw rounded up to ORBX_BLUR_ALIGN)
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
    float inv_scale[ORBX_MAXL];        // mvInvScaleFactors = 1.0f / mvScaleFactor (ORBextractor.cc:503)
    int scaled_patch[ORBX_MAXL];
    int ini_th, min_th, resize_mode, blur_mode;
    int rz_col_off[ORBX_MAXL], rz_row_off[ORBX_MAXL], rz_simd_end[ORBX_MAXL];
    int blur_tiles_x[ORBX_MAXL], blur_tiles_y[ORBX_MAXL], blur_tile_base[ORBX_MAXL + 1];
    unsigned blur_tx_rcp[ORBX_MAXL];   // ceil(2^31 / blur_tiles_x): tile row = umulhi(2 t, rcp) on the SALU
    // FAST cell grid per level (ORBextractor.cc:1084-1118): cell sides, the cells kept by the
    // row / column bounds, and ceil(2^20 / side) for the pixel -> cell division
    int hcell[ORBX_MAXL], wcell[ORBX_MAXL], ncell_rows[ORBX_MAXL], ncell_cols[ORBX_MAXL];
    int hcell_mag[ORBX_MAXL], wcell_mag[ORBX_MAXL];
};

struct DevBuf {
    void *p = nullptr;
    size_t bytes = 0;
    void release();
    int ensure(size_t n);  // grow-only
    template <class T> T *as() const { return (T *)p; }
};

// Completion tracking of the single-call and fetch paths. Every producer records the
// engine's `done` event on the stream it launched on; a fetch makes the engine's own stream
// wait for that event and copies on that stream, then waits for that stream only. Nothing
// here touches the legacy null stream or synchronises the device, so engines driven from
// different host threads -- the left / right extractor threads of Frame.cc:144-153, the
// LocalMapping thread running LocalBA (LocalMapping.cc:116-118) -- never wait for each other.
struct HostCopy {
    hipStream_t st;
    hipError_t err = hipSuccess;
    HostCopy(hipStream_t s, hipEvent_t producer) : st(s) {
        if (producer) err = hipStreamWaitEvent(st, producer, 0);
    }
    void d2h(void *dst, const void *src, size_t bytes) {
        if (err == hipSuccess && dst && src && bytes) err = hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost, st);
    }
    void h2d(void *dst, const void *src, size_t bytes) {
        if (err == hipSuccess && dst && src && bytes) err = hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, st);
    }
    // waits for the copies (and the producer) on this stream only
    int finish() {
        if (err == hipSuccess) err = hipStreamSynchronize(st);
        return err == hipSuccess ? ORBX_OK : ORBX_EDEVICE;
    }
};

// one device -> host copy on `st`, complete on return (fetch paths; `st` is the engine's own
// stream, already ordered after the producer)
inline hipError_t d2h_sync(void *dst, const void *src, size_t bytes, hipStream_t st) {
    const hipError_t r = hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost, st);
    return r == hipSuccess ? hipStreamSynchronize(st) : r;
}

// Grow-only page-locked host buffer: the single-frame paths stage host images and results
// through it so every transfer is one DMA (pageable 2-D copies split into a copy per row).
struct PinnedBuf {
    void *p = nullptr;
    size_t bytes = 0;
    void release() {
        if (p) (void)hipHostFree(p);
        p = nullptr;
        bytes = 0;
    }
    int ensure(size_t n) {
        if (n <= bytes && p) return 0;
        release();
        if (hipHostMalloc(&p, n ? n : 16, hipHostMallocDefault) != hipSuccess) { p = nullptr; return ORBX_EDEVICE; }
        bytes = n ? n : 16;
        return 0;
    }
    template <class T> T *as(size_t byte_off = 0) const { return (T *)((char *)p + byte_off); }
};

inline hipEvent_t make_done_event() {
    hipEvent_t ev = nullptr;
    if (hipEventCreateWithFlags(&ev, hipEventDisableTiming) != hipSuccess) return nullptr;
    return ev;
}

}  // namespace orbamd

struct orbf_state;   // per-engine Frame buffers (orb_frame.hip)

struct orbx_engine {
    orbx_params p{};
    int device = 0;
    hipStream_t stream = nullptr;
    hipEvent_t fb_gate = nullptr;   // pipeline: fast_blur_kernel waits for this event (not the resize)
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
    orbamd::DevBuf d_rz, d_rzr, d_pattern, d_in, d_pyr, d_blur, d_cell_cnt, d_cell_keys,
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
    long long gen = 0;            // extraction generation (bumped by every phase-2 launch)
    int pending_w = 0, pending_h = 0, pending_pitch = 0;
    long long pending_stride = 0;
    int st_pairs = 0;             // pairs of the last stereo run (orbm_stereo_fetch bound)
    hipEvent_t done = nullptr;    // recorded after the last launch of every producer
    hipStream_t done_stream = nullptr;   // stream `done` was last recorded on
    orbamd::PinnedBuf h_stage;    // single-frame host staging (input image, results)
    orbf_state *fs = nullptr;     // Frame / SearchForInitialization buffers, owned
    std::string err;
    // per-kernel hipEvent profiling (bench.py roofline), recorded on the launch stream
    bool prof = false;
    struct ProfRec { const char *name; hipEvent_t a, b; int launches; };   // launches: kernels inside the span
    std::vector<ProfRec> prof_recs;
    std::vector<hipEvent_t> ev_pool;
    size_t ev_used = 0;
};

// ORBmatcher(float nnratio, bool checkOri) (ORBmatcher.h:57): the two members plus a private
// stream and grow-only device buffers for the host-pointer matcher entries.
struct orbm_matcher {
    float nnratio = 0.6f;
    int check_ori = 1;
    int device = 0;
    hipStream_t stream = nullptr;
    hipEvent_t done = nullptr;
    hipStream_t done_stream = nullptr;
    orbamd::DevBuf q, db, off, idx, out;                                    // Hamming scans
    orbamd::DevBuf kun, desc, cnt, keys, nkeys, cstart, prev, m12, nmatch, list, lcnt;   // SearchForInitialization
};

namespace orbamd {
// profiling helpers: prof_begin records a start event (returns a handle), prof_end the
// matching stop event; both are no-ops when profiling is off.
int prof_begin(orbx_engine *e, hipStream_t s);
void prof_end(orbx_engine *e, hipStream_t s, int h, const char *name, int launches = 1);
int engine_reserve(orbx_engine *e, int w, int h, int max_images);
int engine_extract_device(orbx_engine *e, const uint8_t *d_imgs, int n, int pitch,
                          long long stride, hipStream_t s, int phase);
void frame_state_free(orbx_engine *e);   // orb_frame.hip

// A producer launching on `s` first orders itself after the engine's previous producer when
// that one ran on another stream (buffers are reused across calls), and records `done` after
// its own last launch. E: any engine with `done` / `done_stream` members.
template <class E> inline hipError_t order_after_done(E *e, hipStream_t s) {
    if (e->done_stream && e->done_stream != s) return hipStreamWaitEvent(s, e->done, 0);
    return hipSuccess;
}
template <class E> inline hipError_t mark_done(E *e, hipStream_t s) {
    e->done_stream = s;
    return hipEventRecord(e->done, s);
}
}  // namespace orbamd
