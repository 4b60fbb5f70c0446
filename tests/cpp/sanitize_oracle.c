/* Host AddressSanitizer / UndefinedBehaviorSanitizer run of the CPU oracle (SURVEY.md §5
 * "Race detection / sanitizers"; test infrastructure, built by tests/test_sanitize_cpu.py with
 * -fsanitize=address,undefined). Exercises every oracle entry the parity tests lean on, on
 * deterministic synthetic inputs, including the edge shapes: ORBextractor on a textured
 * 640x480 and a 1241x376 stereo pair, a flat image (no keypoints), ComputeStereoMatches,
 * undistortion + RGB-D depth, the Frame grid + SearchForInitialization (consecutive calls with
 * vbPrevMatched carried), the Hamming scan, and LocalBA / PoseOptimization on a problem file
 * written by the test (same layout as host_api_test lba).
 *   sanitize_oracle [lba_problem.bin]
 * Exit 0 and "sanitize ok" on success; any sanitizer finding aborts with a report. */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "../../oracle/lba_oracle.h"
#include "../../oracle/orb_oracle.h"

static uint32_t rng_state = 12345u;
static uint32_t rnd(void) {
    rng_state = rng_state * 1664525u + 1013904223u;
    return rng_state >> 8;
}

/* smooth gradient + random rectangles + noise: plenty of FAST corners */
static void textured(uint8_t *img, int w, int h, uint32_t seed, int shift) {
    rng_state = seed;
    for (int y = 0; y < h; y++)
        for (int x = 0; x < w; x++) img[y * w + x] = (uint8_t)(64 + ((x + shift) * 3 + y * 2) % 96);
    for (int r = 0; r < 260; r++) {
        const int rw = 6 + (int)(rnd() % 40), rh = 6 + (int)(rnd() % 40);
        const int x0 = (int)(rnd() % (unsigned)(w - rw)), y0 = (int)(rnd() % (unsigned)(h - rh));
        const uint8_t v = (uint8_t)(rnd() & 255);
        for (int y = y0; y < y0 + rh; y++)
            for (int x = x0; x < x0 + rw; x++) {
                const int xs = x + shift;
                if (xs >= 0 && xs < w) img[y * w + xs] = v;
            }
    }
    for (int i = 0; i < w * h; i++) {
        const int v = img[i] + (int)(rnd() % 9) - 4;
        img[i] = (uint8_t)(v < 0 ? 0 : v > 255 ? 255 : v);
    }
}

static void *xmalloc(size_t n) {
    void *p = malloc(n ? n : 1);
    if (!p) { fprintf(stderr, "oom\n"); exit(3); }
    return p;
}

static int extract(orc_extractor *ex, const uint8_t *img, int w, int h, orc_kp **kps, uint8_t **desc) {
    const int cap = 2 * ex->nfeatures + 512;
    *kps = (orc_kp *)xmalloc(sizeof(orc_kp) * cap);
    *desc = (uint8_t *)xmalloc(32 * (size_t)cap);
    const int n = orc_extract(ex, img, w, h, w, *kps, *desc, cap);
    if (n < 0) { fprintf(stderr, "orc_extract cap\n"); exit(4); }
    return n;
}

static int run_lba(const char *path) {
    FILE *f = fopen(path, "rb");
    if (!f) return 0;
    fseek(f, 0, SEEK_END);
    const long sz = ftell(f);
    fseek(f, 0, SEEK_SET);
    uint8_t *b = (uint8_t *)xmalloc((size_t)sz);
    if (fread(b, 1, (size_t)sz, f) != (size_t)sz) { fclose(f); return -1; }
    fclose(f);
    const int32_t *hdr = (const int32_t *)b;
    const int np = hdr[0], nq = hdr[1], ne = hdr[2];
    const uint8_t *p = b + 12;
    lba_problem g;
    memset(&g, 0, sizeof g);
    g.n_poses = np; g.n_points = nq; g.n_edges = ne;
    g.pose_id = (const int32_t *)p; p += 4 * np;
    g.pose_fixed = p; p += np; p += (4 - (np % 4)) % 4;
    g.pose_Tcw = (const float *)p; p += 4 * 16 * np;
    g.pose_cam = (const float *)p; p += 4 * 5 * np;
    g.point_id = (const int32_t *)p; p += 4 * nq;
    g.point_Xw = (const float *)p; p += 4 * 3 * nq;
    g.edge_point = (const int32_t *)p; p += 4 * ne;
    g.edge_pose = (const int32_t *)p; p += 4 * ne;
    g.edge_obs = (const float *)p; p += 4 * 3 * ne;
    g.edge_inv_sigma2 = (const float *)p;
    lba_result r;
    memset(&r, 0, sizeof r);
    r.pose_Tcw = (float *)xmalloc(4 * 16 * (size_t)np);
    r.point_Xw = (float *)xmalloc(4 * 3 * (size_t)nq);
    r.edge_erase = (uint8_t *)xmalloc((size_t)ne);
    volatile uint8_t stop = 0;
    const int rc = lba_oracle_solve(&g, &r, &stop);
    /* PoseOptimization on the first free keyframe's observations */
    int k = 0;
    while (k < np && g.pose_fixed[k]) k++;
    int nobs = 0;
    for (int e = 0; e < ne; e++) nobs += g.edge_pose[e] == k;
    float *Xw = (float *)xmalloc(12 * (size_t)(nobs + 1)), *obs = (float *)xmalloc(12 * (size_t)(nobs + 1));
    float *isg = (float *)xmalloc(4 * (size_t)(nobs + 1));
    int m = 0;
    for (int e = 0; e < ne && k < np; e++) {
        if (g.edge_pose[e] != k) continue;
        memcpy(Xw + 3 * m, g.point_Xw + 3 * g.edge_point[e], 12);
        memcpy(obs + 3 * m, g.edge_obs + 3 * e, 12);
        isg[m] = g.edge_inv_sigma2[e];
        m++;
    }
    orbp_frame pf;
    memset(&pf, 0, sizeof pf);
    pf.n = m;
    if (k < np) {
        memcpy(pf.Tcw, g.pose_Tcw + 16 * k, 64);
        pf.fx = g.pose_cam[5 * k]; pf.fy = g.pose_cam[5 * k + 1]; pf.cx = g.pose_cam[5 * k + 2];
        pf.cy = g.pose_cam[5 * k + 3]; pf.bf = g.pose_cam[5 * k + 4];
    }
    pf.Xw = Xw; pf.obs = obs; pf.inv_sigma2 = isg;
    orbp_result pr;
    memset(&pr, 0, sizeof pr);
    pr.outlier = (uint8_t *)xmalloc((size_t)(m + 1));
    const int prc = pose_oracle_optimize(&pf, &pr);
    printf("lba rc=%d iterations=%d/%d pose rc=%d inliers=%d\n", rc, r.iterations[0], r.iterations[1], prc, pr.n_inliers);
    free(pr.outlier); free(Xw); free(obs); free(isg);
    free(r.pose_Tcw); free(r.point_Xw); free(r.edge_erase); free(b);
    return 1;
}

int main(int argc, char **argv) {
    /* C1: mono 640x480, 1000 features; then a flat image (no keypoints) with the same extractor */
    const int W1 = 640, H1 = 480;
    uint8_t *img = (uint8_t *)xmalloc((size_t)W1 * H1);
    textured(img, W1, H1, 1u, 0);
    orc_extractor ex1;
    orc_extractor_init(&ex1, 1000, 1.2f, 8, 20, 7);
    orc_kp *k1; uint8_t *d1;
    const int n1 = extract(&ex1, img, W1, H1, &k1, &d1);
    memset(img, 128, (size_t)W1 * H1);
    orc_kp *kf; uint8_t *df;
    const int nflat = extract(&ex1, img, W1, H1, &kf, &df);
    /* second frame shifted by 2 px: Frame grid + SearchForInitialization, three chained calls */
    textured(img, W1, H1, 1u, 2);
    orc_kp *k2; uint8_t *d2;
    const int n2 = extract(&ex1, img, W1, H1, &k2, &d2);
    const float K[4] = {517.306408f, 516.469215f, 318.643040f, 255.313989f};
    const float D[5] = {0.262383f, -0.953104f, -0.005358f, 0.002628f, 1.163314f};
    float minX, maxX, minY, maxY;
    orc_image_bounds(W1, H1, K, D, &minX, &maxX, &minY, &maxY);
    float *xy = (float *)xmalloc(8 * (size_t)(n1 > n2 ? n1 : n2) + 8), *xyu = (float *)xmalloc(8 * (size_t)(n1 > n2 ? n1 : n2) + 8);
    for (int i = 0; i < n1; i++) { xy[2 * i] = k1[i].x; xy[2 * i + 1] = k1[i].y; }
    orc_undistort_points(xy, xyu, n1, K, D);
    for (int i = 0; i < n1; i++) { k1[i].x = xyu[2 * i]; k1[i].y = xyu[2 * i + 1]; }
    for (int i = 0; i < n2; i++) { xy[2 * i] = k2[i].x; xy[2 * i + 1] = k2[i].y; }
    orc_undistort_points(xy, xyu, n2, K, D);
    for (int i = 0; i < n2; i++) { k2[i].x = xyu[2 * i]; k2[i].y = xyu[2 * i + 1]; }
    float *depth = (float *)xmalloc(4 * (size_t)W1 * H1), *uR = (float *)xmalloc(4 * (size_t)n2 + 4), *dep = (float *)xmalloc(4 * (size_t)n2 + 4);
    for (int i = 0; i < W1 * H1; i++) depth[i] = (i % 17 == 0) ? 0.0f : 0.5f + (float)(i % 4000) * 1e-3f;
    orc_stereo_from_rgbd(k2, k2, n2, depth, W1, 40.0f, uR, dep);
    orc_frame_grid G1, G2;
    orc_grid_build(&G1, k1, d1, n1, minX, maxX, minY, maxY);
    orc_grid_build(&G2, k2, d2, n2, minX, maxX, minY, maxY);
    float *prev = (float *)xmalloc(8 * (size_t)n1 + 8);
    int *m12 = (int *)xmalloc(4 * (size_t)n1 + 4);
    for (int i = 0; i < n1; i++) { prev[2 * i] = k1[i].x; prev[2 * i + 1] = k1[i].y; }
    int nm = 0;
    for (int c = 0; c < 3; c++) nm += orc_search_for_initialization(&G1, &G2, prev, m12, 100, 0.9f, 1);
    /* Hamming scan: F1 descriptors against F2's */
    int *bi = (int *)xmalloc(4 * (size_t)n1 + 4), *bd = (int *)xmalloc(4 * (size_t)n1 + 4), *sd = (int *)xmalloc(4 * (size_t)n1 + 4);
    orc_hamming_best2(d1, n1, d2, n2, bi, bd, sd);
    /* C2: stereo 1241x376, 2000 features, ComputeStereoMatches */
    const int W2 = 1241, H2 = 376;
    uint8_t *L = (uint8_t *)xmalloc((size_t)W2 * H2), *R = (uint8_t *)xmalloc((size_t)W2 * H2);
    textured(L, W2, H2, 7u, 0);
    textured(R, W2, H2, 7u, -20);
    orc_extractor exL, exR;
    orc_extractor_init(&exL, 2000, 1.2f, 8, 20, 7);
    orc_extractor_init(&exR, 2000, 1.2f, 8, 20, 7);
    orc_kp *kL, *kR; uint8_t *dL, *dR;
    const int nL = extract(&exL, L, W2, H2, &kL, &dL), nR = extract(&exR, R, W2, H2, &kR, &dR);
    float *u = (float *)xmalloc(4 * (size_t)nL + 4), *z = (float *)xmalloc(4 * (size_t)nL + 4);
    orc_stereo_matches(&exL, &exR, kL, dL, nL, kR, dR, nR, 386.1448f, 386.1448f / 718.856f, u, z);
    int ns = 0;
    for (int i = 0; i < nL; i++) ns += u[i] >= 0;
    printf("mono %d flat %d frame2 %d init %d stereo %d/%d matches %d\n", n1, nflat, n2, nm, nL, nR, ns);
    const int lba = argc > 1 ? run_lba(argv[1]) : 0;
    if (lba < 0) return 5;
    orc_grid_free(&G1); orc_grid_free(&G2);
    orc_extractor_free(&ex1); orc_extractor_free(&exL); orc_extractor_free(&exR);
    free(img); free(k1); free(d1); free(kf); free(df); free(k2); free(d2); free(xy); free(xyu);
    free(depth); free(uR); free(dep); free(prev); free(m12); free(bi); free(bd); free(sd);
    free(L); free(R); free(kL); free(kR); free(dL); free(dR); free(u); free(z);
    if (n1 < 100 || nflat != 0 || nL < 100 || ns < 10) { fprintf(stderr, "implausible oracle output\n"); return 6; }
    printf("sanitize ok\n");
    return 0;
}
