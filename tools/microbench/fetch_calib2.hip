// FETCH_SIZE / WRITE_SIZE calibration, round 4: replicas of the load patterns of the extraction
// kernels other than fast_blur (fetch_calib.hip has the streams and fast_blur's tiles), each on a
// 1 GiB buffer (past the 256 MiB Infinity Cache) with a placement in which every requested byte is
// fetched once (no reuse between workgroups), so that counter / requested bytes is the counter's
// tally rule for that pattern:
//   rd_resize      resize_level_kernel's horizontal pass: 32 lanes per source row, one aligned
//                  12-byte window (buffer_load_dwordx3) per lane covering its 4 outputs' sources
//                  (the windows of neighbouring lanes overlap), 128 x 32 output tiles at scale 1.2
//   wr_resize      its vertical pass: one dword per lane, 32 lanes per output row
//   rd_describe    describe2_kernel: per keypoint the IC_Angle rows (31 x 32 B as 16-B loads, two
//                  lanes a row) from one level and the 37 x 40-B BRIEF patch (dword loads) from the
//                  blurred level (the other half of the buffer); keypoints 48 x 40 px apart
//   rd_cells       quadtree_kernel's cell gather: a thread reads its cell's kept keys as 16-B loads
//                  (20 keys of a 64-key slot row)
//   rd_stereo      stereo_match_staged: the right descriptors a band indexes (32 B gathered at
//                  random record indices, two lanes each), 16-B band records read in runs, and per
//                  matched keypoint the 11-row SAD windows (12 B left, 20 B right per row)
// Build on the CPU, run once per counter (tools/fetch_calib2.sh):
//   hipcc -O3 --offload-arch=gfx950 -o fetch_calib2 fetch_calib2.hip
// The program prints, per kernel, the bytes its loads / stores request and the distinct bytes.
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>

constexpr long long kBytes = 1LL << 30;

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const void *p) {
    return __builtin_amdgcn_make_buffer_rsrc((void *)p, 0, 0x7fffffff, 0x00020000);
}

// resize: image i at img + i * w * h (pitch w), level-1 tiles of 128 x 32 outputs
__global__ __launch_bounds__(256) void rd_resize(const uint8_t *img, int w, int h, int dw, int dh, int nimg,
                                                 uint32_t *sink) {
    const int tiles_x = (dw + 127) / 128, tiles_y = (dh + 31) / 32;
    const int t = blockIdx.x, b = t / (tiles_x * tiles_y), r = t % (tiles_x * tiles_y);
    if (b >= nimg) return;
    const int x0 = (r % tiles_x) * 128, y0 = (r / tiles_x) * 32, y1 = min(y0 + 32, dh);
    const float sc = (float)w / dw;
    const int sr0 = max(0, (int)floorf((y0 + 0.5f) * sc - 0.5f));
    const int sr1 = min(h - 1, (int)floorf((y1 - 1 + 0.5f) * sc - 0.5f) + 1);
    const int cg = threadIdx.x & 31;
    const int sxa = min(max(0, (int)floorf((x0 + 4 * cg + 0.5f) * sc - 0.5f)), w - 9);
    const uint8_t *src = img + (long long)b * w * h;
    const uint32_t s0 = (uint32_t)((uintptr_t)src & 3);
    const auto rs = rsrc(src - s0);
    uint32_t acc = 0;
    for (int j = sr0 + (threadIdx.x >> 5); j <= sr1; j += 8) {
        const uint32_t a = (uint32_t)j * (uint32_t)w + (uint32_t)sxa + s0;
        const auto v = __builtin_amdgcn_raw_buffer_load_b96(rs, (int)(a & ~3u), 0, 0);
        acc ^= v[0] ^ v[1] ^ v[2];
    }
    if (acc == 0x12345678u) sink[0] = acc;
}

__global__ __launch_bounds__(256) void wr_resize(uint8_t *img, int dw, int bp, int dh, int nimg) {
    const int tiles_x = (dw + 127) / 128, tiles_y = (dh + 31) / 32;
    const int t = blockIdx.x, b = t / (tiles_x * tiles_y), r = t % (tiles_x * tiles_y);
    if (b >= nimg) return;
    const int x0 = (r % tiles_x) * 128, y0 = (r / tiles_x) * 32, y1 = min(y0 + 32, dh);
    const int cg = threadIdx.x & 31, dx0 = x0 + 4 * cg;
    if (dx0 + 3 >= dw) return;
    const auto rd = rsrc(img + (long long)b * bp * dh);
    for (int dy = y0 + (threadIdx.x >> 5); dy < y1; dy += 8)
        __builtin_amdgcn_raw_buffer_store_b32((uint32_t)(dx0 ^ dy), rd, (int)((uint32_t)dy * bp + dx0), 0, 0);
}

// describe: keypoint k of image b at (24 + 48 (k % kx), 24 + 40 (k / kx)); one wave per keypoint
__global__ __launch_bounds__(256) void rd_describe(const uint8_t *lev, const uint8_t *blur, int w, int h, int kx, int ky,
                                                   int nimg, uint32_t *sink) {
    const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const long long kp = (long long)blockIdx.x * 4 + wv;
    const int per = kx * ky, b = (int)(kp / per), k = (int)(kp % per);
    if (b >= nimg) return;
    const int cx = 24 + 48 * (k % kx), cy = 24 + 40 * (k / kx);
    uint32_t acc = 0;
    {   // IC_Angle: rows cy-15 .. cy+15, 32 B from cx-16 as two 16-B loads
        const auto rs = rsrc(lev + (long long)b * w * h);
        if (lane < 62) {
            const int row = cy - 15 + (lane >> 1);
            const auto q = __builtin_amdgcn_raw_buffer_load_b128(rs, row * w + cx - 16 + 16 * (lane & 1), 0, 0);
            acc ^= q[0] ^ q[1] ^ q[2] ^ q[3];
        }
    }
    {   // BRIEF patch: rows cy-18 .. cy+18, 40 B from cx-20 as dwords (10 lanes a row)
        const auto rs = rsrc(blur + (long long)b * w * h);
        for (int e = lane; e < 370; e += 64) {
            const int row = cy - 18 + e / 10, dw = e % 10;
            acc ^= __builtin_amdgcn_raw_buffer_load_b32(rs, row * w + cx - 20 + 4 * dw, 0, 0);
        }
    }
    if (acc == 0x12345678u) sink[0] = acc;
}

// quadtree cells: cell c = a 64-key slot row (256 B); a thread reads its cell's 20 kept keys
__global__ __launch_bounds__(256) void rd_cells(const uint32_t *cells, long long ncell, uint32_t *sink) {
    const long long c = (long long)blockIdx.x * 256 + threadIdx.x;
    if (c >= ncell) return;
    const uint4 *row = (const uint4 *)(cells + c * 64);
    uint32_t acc = 0;
#pragma unroll
    for (int q = 0; q < 5; q++) {
        const uint4 v = row[q];
        acc ^= v.x ^ v.y ^ v.z ^ v.w;
    }
    if (acc == 0x12345678u) sink[0] = acc;
}

__device__ __forceinline__ uint32_t hash32(uint32_t x) {
    x ^= x >> 16; x *= 0x7feb352du; x ^= x >> 15; x *= 0x846ca68bu; x ^= x >> 16;
    return x;
}

// stereo: wave = one staged band group: 32 records (16 B, a contiguous run), the 32 descriptors
// they index (32 B at a random record index, two lanes each), then 8 matched keypoints' SAD
// windows (11 rows: 12 B left, 20 B right) at random positions
__global__ __launch_bounds__(256) void rd_stereo(const uint8_t *base, long long nrec, long long nwin_img, int w, int h,
                                                 uint32_t *sink) {
    const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const long long g = (long long)blockIdx.x * 4 + wv;
    uint32_t acc = 0;
    const uint8_t *recs = base, *desc = base + (kBytes / 4), *imgs = base + (kBytes / 2);
    if (lane < 32) {   // records
        const uint4 v = ((const uint4 *)recs)[(g * 32 + lane) % (kBytes / 4 / 16)];
        acc ^= v.x ^ v.w;
    }
    {   // descriptors: record index -> 32 B
        const long long idx = hash32((uint32_t)(g * 32 + (lane >> 1))) % (uint32_t)nrec;
        const uint4 v = ((const uint4 *)(desc + idx * 32))[lane & 1];
        acc ^= v.y ^ v.z;
    }
    {   // SAD windows: lane = (keypoint kk = lane / 8 of 8, row) over 11 rows in two passes
        for (int e = lane; e < 88; e += 64) {
            const int kk = e / 11, row = e % 11;
            const uint32_t hsh = hash32((uint32_t)(g * 8 + kk) ^ 0x9e3779b9u);
            const long long img = hsh % (uint32_t)nwin_img;
            const int x = 20 + (int)((hsh >> 8) % (uint32_t)(w - 60)), y = 20 + (int)((hsh >> 20) % (uint32_t)(h - 40));
            const uint8_t *L = imgs + img * 2LL * w * h, *R = L + (long long)w * h;
            const auto rl = rsrc(L), rr = rsrc(R);
            const auto a = __builtin_amdgcn_raw_buffer_load_b96(rl, ((y + row) * w + x) & ~3, 0, 0);
            const auto q = __builtin_amdgcn_raw_buffer_load_b128(rr, ((y + row) * w + x - 40) & ~3, 0, 0);
            const uint32_t q5 = __builtin_amdgcn_raw_buffer_load_b32(rr, (((y + row) * w + x - 40) & ~3) + 16, 0, 0);
            acc ^= a[0] ^ a[2] ^ q[1] ^ q[3] ^ q5;
        }
    }
    if (acc == 0x12345678u) sink[0] = acc;
}

int main() {
    uint8_t *buf;
    uint32_t *sink;
    if (hipMalloc(&buf, kBytes) != hipSuccess || hipMalloc(&sink, 64) != hipSuccess) return 1;
    (void)hipMemset(buf, 1, kBytes);
    (void)hipDeviceSynchronize();
    const int w = 1241, h = 376, dw = 1034, dh = 313, bp = 1040;
    // resize read: source images fill the buffer
    const int nimg = (int)(kBytes / ((long long)w * h));
    const int tpi = ((dw + 127) / 128) * ((dh + 31) / 32);
    rd_resize<<<nimg * tpi, 256>>>(buf, w, h, dw, dh, nimg, sink);
    long long rz_req = 0;
    {
        const float sc = (float)w / dw;
        for (int ty = 0; ty < (dh + 31) / 32; ty++) {
            const int y0 = ty * 32, y1 = y0 + 32 < dh ? y0 + 32 : dh;
            int sr0 = (int)floorf((y0 + 0.5f) * sc - 0.5f); if (sr0 < 0) sr0 = 0;
            int sr1 = (int)floorf((y1 - 1 + 0.5f) * sc - 0.5f) + 1; if (sr1 > h - 1) sr1 = h - 1;
            rz_req += (long long)((dw + 127) / 128) * 32 * (sr1 - sr0 + 1) * 12;
        }
        rz_req *= nimg;
    }
    const int nimg_w = (int)(kBytes / ((long long)bp * dh));
    wr_resize<<<nimg_w * tpi, 256>>>(buf, dw, bp, dh, nimg_w);
    long long wr_req = 0;
    for (int ty = 0; ty < (dh + 31) / 32; ty++)
        for (int cg = 0; cg < 32 * ((dw + 127) / 128); cg++) {
            const int dx0 = 4 * cg;
            if (dx0 + 3 < dw) wr_req += 4LL * ((ty * 32 + 32 < dh ? 32 : dh - ty * 32));
        }
    wr_req *= nimg_w;
    // describe: two halves (levels / blurred levels), keypoints on a 48 x 40 grid
    const int kx = (w - 48) / 48 + 1, ky = (h - 48) / 40 + 1;
    const int nimg_d = (int)((kBytes / 2) / ((long long)w * h));
    const long long nkp = (long long)nimg_d * kx * ky;
    rd_describe<<<(unsigned)((nkp + 3) / 4), 256>>>(buf, buf + kBytes / 2, w, h, kx, ky, nimg_d, sink);
    const long long ds_req = nkp * (31 * 32 + 370 * 4);
    // cells
    const long long ncell = kBytes / 256;
    rd_cells<<<(unsigned)((ncell + 255) / 256), 256>>>((const uint32_t *)buf, ncell, sink);
    const long long qt_req = ncell * 80;
    // stereo: records in the first quarter, descriptors in the second, image pairs in the second half
    const long long nrec = (kBytes / 4) / 32, nwin_img = (kBytes / 2) / (2LL * w * h);
    const long long ngrp = 1LL << 19;   // 16.7 M records: every record run read once
    rd_stereo<<<(unsigned)(ngrp / 4), 256>>>(buf, nrec, nwin_img, w, h, sink);
    const long long st_req = ngrp * (32 * 16 + 32 * 32 + 88 * (12 + 16 + 4));
    if (hipDeviceSynchronize() != hipSuccess) return 2;
    printf("{\"rd_resize\": {\"requested\": %lld, \"distinct\": %lld}, \"wr_resize\": {\"requested\": %lld, \"distinct\": %lld}, "
           "\"rd_describe\": {\"requested\": %lld, \"distinct\": %lld}, \"rd_cells\": {\"requested\": %lld, \"distinct\": %lld}, "
           "\"rd_stereo\": {\"requested\": %lld, \"distinct\": %lld}}\n",
           rz_req, (long long)nimg * w * h, wr_req, wr_req, ds_req, ds_req, qt_req, qt_req, st_req, st_req);
    return 0;
}
