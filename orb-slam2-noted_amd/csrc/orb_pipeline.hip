// Stereo batch pipeline: k extraction engines, one HIP stream each, that split a batch of
// stereo pairs into k chunks and run every chunk as
//   phase 1 (pyramid + FAST strength map + blur: the VALU-bound half of ORBextractor::operator())
//   phase 2 (cell NMS, DistributeOctTree, IC_Angle + rBRIEF: latency-bound)
//   Frame::ComputeStereoMatches (latency-bound)
// with the chunks' fast_blur launches in turn (chunk j's waits for chunk j-1's, across batches
// too), so one chunk's VALU-bound kernel overlaps the others' latency-bound ones (resize
// chains, quadtree, describe, stereo). The work and
// the results are the same as one engine over the whole batch (each chunk is an independent
// ORBextractor pair; Frame.cc:144-153 runs the left / right extractors on two threads).
// Measured on MI355X, 1241x376 pairs, bench.py C2 leg: one engine x 256 pairs 48.7k stereo
// frames/s, 2 x 128 52.1k, 3 x 128 54.9k, 4 x 128 52.1k (tools/pipeline_exp.py: one engine x 384
// 49.1k, 2 x 192 51.8k, 4 x 64 49.5k). Batches are not separated by a barrier: the next batch's
// chunks start while the previous batch's last chunks finish.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdlib>
#include <vector>

#include "orbslam2_amd.h"
#include "orb_engine.h"
#include "build_id.h"   // ORBX_SRC_HASH (Makefile, tools/src_hash.py)

static void orbx_engine_fb_gate(orbx_engine *e, hipEvent_t ev) { e->fb_gate = ev; }

struct orbx_pipeline {
    std::vector<orbx_engine *> eng;
    std::vector<hipEvent_t> ev_p1;    // end of each engine's phase 1 (orders the next chunk's)
    std::vector<hipEvent_t> ev_done;  // end of each engine's chunk (orbx_pipeline_join)
    hipEvent_t ev_in = nullptr;       // caller stream at entry
    std::vector<int> first, count;    // chunk of the last batch per engine (pairs)
    int last_p1 = -1;                 // engine whose phase 1 was enqueued last
    int device = 0;
    // host-in / host-out mode (orbx_pipeline_stereo_batch_host): two device input slots fed by an
    // H2D stream, outputs drained by a D2H stream, both overlapped with the engines
    hipStream_t h2d = nullptr, d2h = nullptr;
    void *slot_buf[2] = {nullptr, nullptr};
    size_t slot_bytes = 0;
    int next_slot = 0;
    int slot_pairs[2] = {0, 0};          // chunk layout of the last batch uploaded into each slot:
    size_t slot_stride[2] = {0, 0};      // pair count and image stride (they fix every chunk's byte range)
    std::vector<hipEvent_t> ev_h2d[2];   // chunk j of slot s uploaded
    std::vector<hipEvent_t> ev_free[2];  // engine j finished reading slot s (stereo done)
    std::vector<bool> free_rec[2];
    std::vector<hipEvent_t> ev_d2h;      // engine j's outputs of the last host batch copied out
    std::vector<bool> d2h_rec;
};

static int pipeline_fail(orbx_pipeline *pl, int rc) {
    orbx_pipeline_destroy(pl);
    return rc;
}

// One batch over the engines. Device-input mode (slot < 0): every chunk starts after the work
// queued on `caller`. Host mode (slot >= 0): chunk j starts when its upload into `slot` has landed,
// its phase 2 waits until the previous host batch's outputs of engine j have been copied out, and
// after its stereo pass the D2H stream copies the chunk's outputs into `out`.
static int pipeline_run(orbx_pipeline *pl, const uint8_t *d_imgs, int n_pairs, int w, int h, int pitch,
                        size_t image_stride, float mbf, float mb, hipStream_t caller, const orbx_stereo_host_out *out,
                        int slot) {
    if (!pl || !d_imgs || n_pairs <= 0 || pitch < w) return ORBX_EINVAL;
    if (hipSetDevice(pl->device) != hipSuccess) return ORBX_EDEVICE;
    const int k = (int)pl->eng.size();
    const bool host = slot >= 0;
    if (!host && hipEventRecord(pl->ev_in, caller) != hipSuccess) return ORBX_EDEVICE;
    for (int j = 0; j < k; j++) {
        pl->first[j] = (int)((long long)n_pairs * j / k);
        pl->count[j] = (int)((long long)n_pairs * (j + 1) / k) - pl->first[j];
    }
    for (int j = 0; j < k; j++) {
        if (pl->count[j] == 0) continue;
        orbx_engine *e = pl->eng[j];
        const hipStream_t s = (hipStream_t)orbx_stream(e);
        if (hipStreamWaitEvent(s, host ? pl->ev_h2d[slot][j] : pl->ev_in, 0) != hipSuccess) return ORBX_EDEVICE;
        // only the VALU-bound fast_blur launches run in turn: the engine's resize chain starts as
        // soon as its input is there and overlaps the previous engine's fast_blur, and its
        // fast_blur then starts the moment that one ends (measured against ordering the whole
        // phase 1: 71.2-71.8k vs 68.1-69.6k stereo frames/s, and no pipeline phase that leaves
        // describe without a fast_blur to overlap)
        const bool gate = pl->last_p1 >= 0 && pl->last_p1 != j;
        const uint8_t *src = d_imgs + (size_t)2 * pl->first[j] * image_stride;
        const int n_img = 2 * pl->count[j];
        orbx_engine_fb_gate(e, gate ? pl->ev_p1[pl->last_p1] : nullptr);
        int rc = orbx_extract_batch_device_phase(e, src, n_img, w, h, pitch, image_stride, s, 1);
        orbx_engine_fb_gate(e, nullptr);
        if (rc) return rc;
        if (hipEventRecord(pl->ev_p1[j], s) != hipSuccess) return ORBX_EDEVICE;
        pl->last_p1 = j;
        // phase 2 overwrites the engine's keypoint / descriptor / stereo buffers: whatever mode this
        // batch is in, they may still be draining to the host from an earlier host-mode batch
        if (j < (int)pl->d2h_rec.size() && pl->d2h_rec[j] && hipStreamWaitEvent(s, pl->ev_d2h[j], 0) != hipSuccess) return ORBX_EDEVICE;
        rc = orbx_extract_batch_device_phase(e, src, n_img, w, h, pitch, image_stride, s, 2);
        if (rc) return rc;
        rc = orbm_stereo_match_batch_device(e, pl->count[j], mbf, mb, s);
        if (rc) return rc;
        if (hipEventRecord(pl->ev_done[j], s) != hipSuccess) return ORBX_EDEVICE;
        if (!host) continue;
        if (hipEventRecord(pl->ev_free[slot][j], s) != hipSuccess) return ORBX_EDEVICE;
        pl->free_rec[slot][j] = true;
        const int *d_cnt = nullptr;
        const orbx_kp *d_kps = nullptr;
        const uint8_t *d_desc = nullptr;
        const float *d_u = nullptr, *d_z = nullptr;
        int cap = 0;
        if (orbx_batch_results(e, &d_cnt, &d_kps, &d_desc, &cap) || orbm_stereo_results(e, &d_u, &d_z))
            return ORBX_ESTATE;
        const size_t i0 = 2 * (size_t)pl->first[j], p0 = (size_t)pl->first[j], C = (size_t)cap;
        const size_t ni = (size_t)n_img, npr = (size_t)pl->count[j];
        if (hipStreamWaitEvent(pl->d2h, pl->ev_done[j], 0) != hipSuccess ||
            hipMemcpyAsync(out->counts + i0, d_cnt, 4 * ni, hipMemcpyDeviceToHost, pl->d2h) != hipSuccess ||
            hipMemcpyAsync(out->kps + i0 * C, d_kps, sizeof(orbx_kp) * ni * C, hipMemcpyDeviceToHost, pl->d2h) != hipSuccess ||
            hipMemcpyAsync(out->desc + 32 * i0 * C, d_desc, 32 * ni * C, hipMemcpyDeviceToHost, pl->d2h) != hipSuccess ||
            hipMemcpyAsync(out->u_right + p0 * C, d_u, 4 * npr * C, hipMemcpyDeviceToHost, pl->d2h) != hipSuccess ||
            hipMemcpyAsync(out->depth + p0 * C, d_z, 4 * npr * C, hipMemcpyDeviceToHost, pl->d2h) != hipSuccess ||
            hipEventRecord(pl->ev_d2h[j], pl->d2h) != hipSuccess)
            return ORBX_EDEVICE;
        pl->d2h_rec[j] = true;
    }
    return ORBX_OK;
}

extern "C" {

// the hash of the library's sources (tools/src_hash.py); a build with other compile settings than
// the product's (EXTRA flags, `make variant` defines) carries a suffix naming them, so counters
// measured on it never pass for the product's (bench.py load_pmc_doc, tools/stamp.py)
#ifndef ORBX_BUILD_SUFFIX
#define ORBX_BUILD_SUFFIX ""
#endif
const char *orbx_build_id(void) { return ORBX_SRC_HASH ORBX_BUILD_SUFFIX; }

int orbx_pipeline_create(const orbx_params *p, int n_engines, orbx_pipeline **out) {
    if (!p || !out) return ORBX_EINVAL;
    *out = nullptr;
    if (p->struct_size != sizeof(orbx_params)) return ORBX_EINVAL;
    if (n_engines <= 0) n_engines = 3;
    if (n_engines > 16) return ORBX_EINVAL;
    orbx_pipeline *pl = new orbx_pipeline();
    if (hipGetDevice(&pl->device) != hipSuccess) return pipeline_fail(pl, ORBX_EDEVICE);
    for (int i = 0; i < n_engines; i++) {
        orbx_engine *e = nullptr;
        const int rc = orbx_create(p, &e);
        if (rc) return pipeline_fail(pl, rc);
        pl->eng.push_back(e);
        hipEvent_t a, b;
        if (hipEventCreateWithFlags(&a, hipEventDisableTiming) != hipSuccess) return pipeline_fail(pl, ORBX_EDEVICE);
        pl->ev_p1.push_back(a);
        if (hipEventCreateWithFlags(&b, hipEventDisableTiming) != hipSuccess) return pipeline_fail(pl, ORBX_EDEVICE);
        pl->ev_done.push_back(b);
    }
    if (hipEventCreateWithFlags(&pl->ev_in, hipEventDisableTiming) != hipSuccess) return pipeline_fail(pl, ORBX_EDEVICE);
    pl->first.assign(n_engines, 0);
    pl->count.assign(n_engines, 0);
    *out = pl;
    return ORBX_OK;
}

void orbx_pipeline_destroy(orbx_pipeline *pl) {
    if (!pl) return;
    (void)hipSetDevice(pl->device);
    for (orbx_engine *e : pl->eng) orbx_destroy(e);   // synchronises the engine's stream
    for (hipEvent_t ev : pl->ev_p1) (void)hipEventDestroy(ev);
    for (hipEvent_t ev : pl->ev_done) (void)hipEventDestroy(ev);
    if (pl->ev_in) (void)hipEventDestroy(pl->ev_in);
    if (pl->h2d) (void)hipStreamSynchronize(pl->h2d);
    if (pl->d2h) (void)hipStreamSynchronize(pl->d2h);
    for (int sl = 0; sl < 2; sl++) {
        for (hipEvent_t ev : pl->ev_h2d[sl]) (void)hipEventDestroy(ev);
        for (hipEvent_t ev : pl->ev_free[sl]) (void)hipEventDestroy(ev);
        if (pl->slot_buf[sl]) (void)hipFree(pl->slot_buf[sl]);
    }
    for (hipEvent_t ev : pl->ev_d2h) (void)hipEventDestroy(ev);
    if (pl->h2d) (void)hipStreamDestroy(pl->h2d);
    if (pl->d2h) (void)hipStreamDestroy(pl->d2h);
    delete pl;
}

int orbx_pipeline_engines(orbx_pipeline *pl) { return pl ? (int)pl->eng.size() : 0; }

int orbx_pipeline_reserve(orbx_pipeline *pl, int w, int h, int max_pairs) {
    if (!pl || max_pairs <= 0) return ORBX_EINVAL;
    const int k = (int)pl->eng.size();
    const int per = (max_pairs + k - 1) / k;
    for (orbx_engine *e : pl->eng) {
        const int rc = orbx_reserve(e, w, h, 2 * per);
        if (rc) return rc;
    }
    return ORBX_OK;
}

int orbx_pipeline_stereo_batch(orbx_pipeline *pl, const uint8_t *d_imgs, int n_pairs, int w, int h,
                               int pitch, size_t image_stride, float mbf, float mb, void *stream) {
    return pipeline_run(pl, d_imgs, n_pairs, w, h, pitch, image_stride, mbf, mb, (hipStream_t)stream, nullptr, -1);
}

int orbx_pipeline_capacity(orbx_pipeline *pl, int *cap) {
    if (!pl || !cap || pl->eng.empty()) return ORBX_EINVAL;
    return orbx_capacity(pl->eng[0], cap);
}

// Host images in, host keypoints / descriptors / stereo out (the ORBextractor::operator() /
// Frame boundary takes and returns host data, ORBextractor.h:107). The batch is uploaded chunk by
// chunk on an H2D stream into one of two device slots (the upload of batch k+1 overlaps the
// engines' work on batch k), each engine starts when its chunk has arrived, and its outputs are
// copied out on a D2H stream as soon as its stereo pass ends. Returns once everything is enqueued;
// orbx_pipeline_wait blocks until the outputs are in host memory. h_imgs and the output arrays
// should be pinned (orbx_host_alloc) for the copies to overlap; they must stay valid until the wait.
int orbx_pipeline_stereo_batch_host(orbx_pipeline *pl, const uint8_t *h_imgs, int n_pairs, int w, int h,
                                    int pitch, size_t image_stride, float mbf, float mb,
                                    const orbx_stereo_host_out *out) {
    if (!pl || !h_imgs || !out || n_pairs <= 0 || w <= 0 || h <= 0 || pitch < w) return ORBX_EINVAL;
    if (image_stride < (size_t)pitch * (size_t)(h - 1) + (size_t)w) return ORBX_EINVAL;
    if (!out->counts || !out->kps || !out->desc || !out->u_right || !out->depth) return ORBX_EINVAL;
    if (hipSetDevice(pl->device) != hipSuccess) return ORBX_EDEVICE;
    const int k = (int)pl->eng.size();
    if (!pl->h2d) {
        if (hipStreamCreateWithFlags(&pl->h2d, hipStreamNonBlocking) != hipSuccess ||
            hipStreamCreateWithFlags(&pl->d2h, hipStreamNonBlocking) != hipSuccess)
            return ORBX_EDEVICE;
        for (int sl = 0; sl < 2; sl++) {
            pl->ev_h2d[sl].assign(k, nullptr);
            pl->ev_free[sl].assign(k, nullptr);
            pl->free_rec[sl].assign(k, false);
            for (int j = 0; j < k; j++)
                if (hipEventCreateWithFlags(&pl->ev_h2d[sl][j], hipEventDisableTiming) != hipSuccess ||
                    hipEventCreateWithFlags(&pl->ev_free[sl][j], hipEventDisableTiming) != hipSuccess)
                    return ORBX_EDEVICE;
        }
        pl->ev_d2h.assign(k, nullptr);
        pl->d2h_rec.assign(k, false);
        for (int j = 0; j < k; j++)
            if (hipEventCreateWithFlags(&pl->ev_d2h[j], hipEventDisableTiming) != hipSuccess) return ORBX_EDEVICE;
    }
    // device slot: the batch in the caller's layout (no readable tail needed, orbslam2_amd.h)
    const size_t need = 2 * (size_t)n_pairs * image_stride;
    if (need > pl->slot_bytes) {
        for (int sl = 0; sl < 2; sl++) {   // slots may still be read by earlier batches
            for (int j = 0; j < k; j++)
                if (pl->free_rec[sl][j] && hipEventSynchronize(pl->ev_free[sl][j]) != hipSuccess) return ORBX_EDEVICE;
            if (pl->slot_buf[sl]) (void)hipFree(pl->slot_buf[sl]);
            pl->slot_buf[sl] = nullptr;
        }
        pl->slot_bytes = 0;
        for (int sl = 0; sl < 2; sl++)
            if (hipMalloc(&pl->slot_buf[sl], need) != hipSuccess) return ORBX_EDEVICE;
        pl->slot_bytes = need;
    }
    const int sl = pl->next_slot;
    pl->next_slot ^= 1;
    uint8_t *dev = (uint8_t *)pl->slot_buf[sl];
    // Chunk j's upload overwrites the range engine j read in this slot's previous batch. With the
    // same pair count and image stride the chunk byte ranges coincide and waiting for engines 0..j
    // suffices (the waits pile up on the H2D stream); with a different count or stride chunk j can
    // cover an old range of any engine, so the first upload waits for every engine's last read of
    // the slot.
    if (pl->slot_pairs[sl] != n_pairs || pl->slot_stride[sl] != image_stride) {
        for (int j = 0; j < k; j++)
            if (pl->free_rec[sl][j] && hipStreamWaitEvent(pl->h2d, pl->ev_free[sl][j], 0) != hipSuccess)
                return ORBX_EDEVICE;
        pl->slot_pairs[sl] = n_pairs;
        pl->slot_stride[sl] = image_stride;
    }
    for (int j = 0; j < k; j++) {
        const int first = (int)((long long)n_pairs * j / k), cnt = (int)((long long)n_pairs * (j + 1) / k) - first;
        if (pl->free_rec[sl][j] && hipStreamWaitEvent(pl->h2d, pl->ev_free[sl][j], 0) != hipSuccess) return ORBX_EDEVICE;
        if (cnt > 0) {
            const size_t off = 2 * (size_t)first * image_stride, bytes = 2 * (size_t)cnt * image_stride;
            if (hipMemcpyAsync(dev + off, h_imgs + off, bytes, hipMemcpyHostToDevice, pl->h2d) != hipSuccess)
                return ORBX_EDEVICE;
        }
        if (hipEventRecord(pl->ev_h2d[sl][j], pl->h2d) != hipSuccess) return ORBX_EDEVICE;
    }
    return pipeline_run(pl, dev, n_pairs, w, h, pitch, image_stride, mbf, mb, nullptr, out, sl);
}

int orbx_pipeline_wait(orbx_pipeline *pl) {
    if (!pl) return ORBX_EINVAL;
    for (size_t j = 0; j < pl->ev_d2h.size(); j++)
        if (pl->d2h_rec[j] && hipEventSynchronize(pl->ev_d2h[j]) != hipSuccess) return ORBX_EDEVICE;
    return ORBX_OK;
}

int orbx_host_alloc(size_t bytes, void **p) {
    if (!p) return ORBX_EINVAL;
    *p = nullptr;
    return hipHostMalloc(p, bytes ? bytes : 1, hipHostMallocDefault) == hipSuccess ? ORBX_OK : ORBX_EDEVICE;
}

int orbx_host_free(void *p) {
    if (!p) return ORBX_OK;
    return hipHostFree(p) == hipSuccess ? ORBX_OK : ORBX_EDEVICE;
}

// The caller's stream is not made to wait here: that would turn every batch into a barrier and
// stop one batch's chunks from overlapping the next batch's (the measured gain comes from that
// overlap); orbx_pipeline_join orders consumers explicitly.
int orbx_pipeline_join(orbx_pipeline *pl, void *stream) {
    if (!pl) return ORBX_EINVAL;
    for (size_t j = 0; j < pl->eng.size(); j++)
        if (pl->count[j] > 0 && hipStreamWaitEvent((hipStream_t)stream, pl->ev_done[j], 0) != hipSuccess)
            return ORBX_EDEVICE;
    return ORBX_OK;
}

int orbx_pipeline_chunk(orbx_pipeline *pl, int i, orbx_engine **e, int *first_pair, int *n_pairs) {
    if (!pl || i < 0 || i >= (int)pl->eng.size()) return ORBX_EINVAL;
    if (e) *e = pl->eng[i];
    if (first_pair) *first_pair = pl->first[i];
    if (n_pairs) *n_pairs = pl->count[i];
    return ORBX_OK;
}

}  // extern "C"
