// Stereo batch pipeline: k extraction engines, one HIP stream each, that split a batch of
// stereo pairs into k chunks and run every chunk as
//   phase 1 (pyramid + FAST strength map + blur: the VALU-bound half of ORBextractor::operator())
//   phase 2 (cell NMS, DistributeOctTree, IC_Angle + rBRIEF: latency-bound)
//   Frame::ComputeStereoMatches (latency-bound)
// with the chunks' phase 1 in turn (chunk j's phase 1 waits for chunk j-1's, across batches
// too), so one chunk's VALU-bound phase overlaps the others' latency-bound phases. The work and
// the results are the same as one engine over the whole batch (each chunk is an independent
// ORBextractor pair; Frame.cc:144-153 runs the left / right extractors on two threads).
// Measured on MI355X, 1241x376 pairs, bench.py C2 leg: one engine x 256 pairs 48.7k stereo
// frames/s, 2 x 128 52.1k, 3 x 128 54.9k, 4 x 128 52.1k (tools/pipeline_exp.py: one engine x 384
// 49.1k, 2 x 192 51.8k, 4 x 64 49.5k). Batches are not separated by a barrier: the next batch's
// chunks start while the previous batch's last chunks finish.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <vector>

#include "orbslam2_amd.h"

struct orbx_pipeline {
    std::vector<orbx_engine *> eng;
    std::vector<hipEvent_t> ev_p1;    // end of each engine's phase 1 (orders the next chunk's)
    std::vector<hipEvent_t> ev_done;  // end of each engine's chunk (orbx_pipeline_join)
    hipEvent_t ev_in = nullptr;       // caller stream at entry
    std::vector<int> first, count;    // chunk of the last batch per engine (pairs)
    int last_p1 = -1;                 // engine whose phase 1 was enqueued last
    int device = 0;
};

static int pipeline_fail(orbx_pipeline *pl, int rc) {
    orbx_pipeline_destroy(pl);
    return rc;
}

extern "C" {

int orbx_pipeline_create(const orbx_params *p, int n_engines, orbx_pipeline **out) {
    if (!p || !out) return ORBX_EINVAL;
    *out = nullptr;
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
    if (!pl || !d_imgs || n_pairs <= 0 || pitch < w) return ORBX_EINVAL;
    if (hipSetDevice(pl->device) != hipSuccess) return ORBX_EDEVICE;
    const int k = (int)pl->eng.size();
    const hipStream_t caller = (hipStream_t)stream;
    if (hipEventRecord(pl->ev_in, caller) != hipSuccess) return ORBX_EDEVICE;
    for (int j = 0; j < k; j++) {
        pl->first[j] = (int)((long long)n_pairs * j / k);
        pl->count[j] = (int)((long long)n_pairs * (j + 1) / k) - pl->first[j];
    }
    for (int j = 0; j < k; j++) {
        if (pl->count[j] == 0) continue;
        orbx_engine *e = pl->eng[j];
        const hipStream_t s = (hipStream_t)orbx_stream(e);
        if (hipStreamWaitEvent(s, pl->ev_in, 0) != hipSuccess) return ORBX_EDEVICE;
        if (pl->last_p1 >= 0 && pl->last_p1 != j && hipStreamWaitEvent(s, pl->ev_p1[pl->last_p1], 0) != hipSuccess)
            return ORBX_EDEVICE;
        const uint8_t *src = d_imgs + (size_t)2 * pl->first[j] * image_stride;
        const int n_img = 2 * pl->count[j];
        int rc = orbx_extract_batch_device_phase(e, src, n_img, w, h, pitch, image_stride, s, 1);
        if (rc) return rc;
        if (hipEventRecord(pl->ev_p1[j], s) != hipSuccess) return ORBX_EDEVICE;
        pl->last_p1 = j;
        rc = orbx_extract_batch_device_phase(e, src, n_img, w, h, pitch, image_stride, s, 2);
        if (rc) return rc;
        rc = orbm_stereo_match_batch_device(e, pl->count[j], mbf, mb, s);
        if (rc) return rc;
        if (hipEventRecord(pl->ev_done[j], s) != hipSuccess) return ORBX_EDEVICE;
    }
    return ORBX_OK;
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
