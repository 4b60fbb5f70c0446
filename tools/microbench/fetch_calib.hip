// Calibration of rocprofv3 FETCH_SIZE / WRITE_SIZE on gfx950 for the access widths the
// extraction kernels use (MI355X_MICROARCH.md §HBM calibrates only 16-B-per-lane streams).
// Every kernel touches a known number of distinct bytes of a 1 GiB buffer (far past the 256 MiB
// Infinity Cache, so each line comes from HBM once); run once per counter:
//   hipcc -O3 --offload-arch=gfx950 -o fetch_calib fetch_calib.hip
//   rocprofv3 --kernel-trace --pmc FETCH_SIZE -d out_f -o run --output-format csv -- ./fetch_calib
//   rocprofv3 --kernel-trace --pmc WRITE_SIZE -d out_w -o run --output-format csv -- ./fetch_calib
// and divide the counter (KB x 1024) by the bytes this program prints per kernel
// (tools/microbench/fetch_calib.py does both).
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>

constexpr long long kBytes = 1LL << 30;

// contiguous lanes, W bytes per lane per load, grid-stride over the buffer
template <int W>
__global__ __launch_bounds__(256) void rd_stream(const uint8_t *p, long long n, uint32_t *sink) {
    uint32_t acc = 0;
    const long long stride = (long long)gridDim.x * 256 * W;
    for (long long o = ((long long)blockIdx.x * 256 + threadIdx.x) * W; o + W <= n; o += stride) {
        if constexpr (W == 4) acc ^= *(const uint32_t *)(p + o);
        if constexpr (W == 8) { const uint2 v = *(const uint2 *)(p + o); acc ^= v.x ^ v.y; }
        if constexpr (W == 16) { const uint4 v = *(const uint4 *)(p + o); acc ^= v.x ^ v.y ^ v.z ^ v.w; }
    }
    if (acc == 0x12345678u) sink[0] = acc;
}

// fast_blur_kernel's staging pattern: an image of pitch 1241 read as 128 x 16 tiles, each tile
// reading rows y0-4 .. y0+19 and columns x0-4 .. x0+131 as 17 unaligned 8-byte pairs per row
// (tiles clipped to the image; the halo re-reads are what the counter is asked about)
__global__ __launch_bounds__(256) void rd_tiles(const uint8_t *img, int w, int h, int nimg, uint32_t *sink) {
    const int tiles_x = (w + 127) / 128, tiles_y = (h + 15) / 16;
    const int t = blockIdx.x, b = t / (tiles_x * tiles_y), r = t % (tiles_x * tiles_y);
    if (b >= nimg) return;
    const int x0 = (r % tiles_x) * 128, y0 = (r / tiles_x) * 16;
    const uint8_t *src = img + (long long)b * w * h;
    uint32_t acc = 0;
    if (threadIdx.x < 255) {
        const int rr0 = threadIdx.x / 17, jj = threadIdx.x % 17;
        for (int rr = rr0; rr < 24; rr += 15) {
            const int yy = min(max(y0 - 4 + rr, 0), h - 1);
            const int xs = min(max(x0 - 4 + 8 * jj, 0), w - 8);
            uint2 v;
            __builtin_memcpy(&v, src + (long long)yy * w + xs, 8);
            acc ^= v.x ^ v.y;
        }
    }
    if (acc == 0x12345678u) sink[0] = acc;
}

template <int W>
__global__ __launch_bounds__(256) void wr_stream(uint8_t *p, long long n) {
    const long long stride = (long long)gridDim.x * 256 * W;
    for (long long o = ((long long)blockIdx.x * 256 + threadIdx.x) * W; o + W <= n; o += stride) {
        if constexpr (W == 4) *(uint32_t *)(p + o) = (uint32_t)o;
        if constexpr (W == 16) *(uint4 *)(p + o) = make_uint4((uint32_t)o, 1u, 2u, 3u);
    }
}

// fast_blur_mfma's output pattern: per 16-column block a wave stores 16 rows x 16 bytes (lane:
// row n = lane & 15, 4 bytes at column 4 (lane >> 4)), an image of pitch bp = 1248
__global__ __launch_bounds__(256) void wr_tiles(uint8_t *img, int w, int bp, int h, int nimg) {
    const int tiles_x = (w + 127) / 128, tiles_y = (h + 15) / 16;
    const int t = blockIdx.x, b = t / (tiles_x * tiles_y), r = t % (tiles_x * tiles_y);
    if (b >= nimg) return;
    const int x0 = (r % tiles_x) * 128, y0 = (r / tiles_x) * 16;
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    uint8_t *dst = img + (long long)b * bp * h;
    for (int xb = 2 * wv; xb < 2 * wv + 2; xb++) {
        const int y = y0 + (lane & 15), x = x0 + 16 * xb + 4 * (lane >> 4);
        if (y < h && x + 3 < bp) *(uint32_t *)(dst + (long long)y * bp + x) = (uint32_t)(x ^ y);
    }
}

int main() {
    uint8_t *buf;
    uint32_t *sink;
    if (hipMalloc(&buf, kBytes) != hipSuccess || hipMalloc(&sink, 64) != hipSuccess) return 1;
    (void)hipMemset(buf, 1, kBytes);
    (void)hipDeviceSynchronize();
    const int grid = 256 * 16;
    rd_stream<4><<<grid, 256>>>(buf, kBytes, sink);
    rd_stream<8><<<grid, 256>>>(buf, kBytes, sink);
    rd_stream<16><<<grid, 256>>>(buf, kBytes, sink);
    // tiles: 1241 x 376 images, as many as fit in the buffer
    const int w = 1241, h = 376, bp = 1248;
    const int nimg = (int)(kBytes / ((long long)bp * h));
    const int tpi = ((w + 127) / 128) * ((h + 15) / 16);
    rd_tiles<<<nimg * tpi, 256>>>(buf, w, h, nimg, sink);
    wr_stream<4><<<grid, 256>>>(buf, kBytes);
    wr_stream<16><<<grid, 256>>>(buf, kBytes);
    wr_tiles<<<nimg * tpi, 256>>>(buf, w, bp, h, nimg);
    if (hipDeviceSynchronize() != hipSuccess) return 2;
    // distinct bytes each kernel touches
    printf("{\"rd_stream<4>\": %lld, \"rd_stream<8>\": %lld, \"rd_stream<16>\": %lld, \"rd_tiles\": %lld, "
           "\"wr_stream<4>\": %lld, \"wr_stream<16>\": %lld, \"wr_tiles\": %lld}\n",
           kBytes, kBytes, kBytes, (long long)nimg * w * h, kBytes, kBytes, (long long)nimg * bp * h);
    return 0;
}
