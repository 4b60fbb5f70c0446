/*
 * ORACLE — TEST INFRASTRUCTURE ONLY (see orb_oracle.h). Never linked into the product.
 *
 * C restatement of DBoW2's vocabulary transform as ORB-SLAM2 uses it for
 * Frame::ComputeBoW (src/Frame.cc:704-719):
 *   TemplatedVocabulary::loadFromTextFile   Thirdparty/DBoW2/DBoW2/TemplatedVocabulary.h:1385-1460
 *   TemplatedVocabulary::transform(features, BowVector&, FeatureVector&, levelsup)   :1125-1209
 *   TemplatedVocabulary::transform(feature, word_id, weight, nid, levelsup)          :1226-1286
 *   FORB::distance                          Thirdparty/DBoW2/DBoW2/FORB.cpp:81-101
 *   BowVector::addWeight / addIfNotExist / normalize   BowVector.cpp:40-95
 *   FeatureVector::addFeature               FeatureVector.cpp
 *   ScoringObject::mustNormalize            ScoringObject.h:69-84 (L1, L2, ChiSquare, KL,
 *                                           Bhattacharyya normalise; DotProduct does not)
 * BowVector / FeatureVector (std::map) become arrays sorted by key. Two deliberate
 * deviations, both undefined behaviour in the reference: a trailing empty line of the text
 * file is skipped (the reference's while(!eof()) loop would append a garbage node), and a
 * feature whose descent reaches a leaf above the FeatureVector level gets node 0 (the
 * reference leaves `nid` uninitialised).
 */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "bow_oracle.h"
#include "orb_oracle.h"

void orc_vocab_free(orc_vocab *v) {
    free(v->child_start); free(v->children); free(v->desc); free(v->weight); free(v->word_id);
    memset(v, 0, sizeof(*v));
}

int orc_vocab_build(orc_vocab *v, int k, int L, int scoring, int weighting, int n_nodes, const int32_t *parent,
                    const uint8_t *is_leaf, const uint8_t *desc, const double *weight) {
    memset(v, 0, sizeof(*v));
    if (n_nodes < 1 || scoring < 0 || scoring > 5 || weighting < 0 || weighting > 3) return -1;
    v->k = k; v->L = L; v->scoring = scoring; v->weighting = weighting; v->n_nodes = n_nodes;
    v->child_start = (int *)calloc((size_t)n_nodes + 1, sizeof(int));
    v->children = (int *)malloc(sizeof(int) * ((size_t)n_nodes + 1));
    v->desc = (uint8_t *)malloc(32 * (size_t)n_nodes);
    v->weight = (double *)malloc(sizeof(double) * (size_t)n_nodes);
    v->word_id = (int *)malloc(sizeof(int) * (size_t)n_nodes);
    for (int i = 1; i < n_nodes; i++) {
        if (parent[i] < 0 || parent[i] >= i) { orc_vocab_free(v); return -1; }   /* parents precede */
        v->child_start[parent[i] + 1]++;
    }
    for (int i = 0; i < n_nodes; i++) v->child_start[i + 1] += v->child_start[i];
    int *fill = (int *)calloc((size_t)n_nodes + 1, sizeof(int));
    for (int i = 1; i < n_nodes; i++) v->children[v->child_start[parent[i]] + fill[parent[i]]++] = i;  /* push_back order */
    free(fill);
    memcpy(v->desc, desc, 32 * (size_t)n_nodes);
    int nw = 0;
    for (int i = 0; i < n_nodes; i++) {
        v->weight[i] = i == 0 ? 0.0 : weight[i];
        v->word_id[i] = (i > 0 && is_leaf[i]) ? nw++ : 0;
    }
    v->n_words = nw;
    return 0;
}

int orc_vocab_load_text(orc_vocab *v, const char *path) {
    FILE *f = fopen(path, "r");
    if (!f) return -1;
    int k, L, n1, n2;
    char line[4096];
    if (!fgets(line, sizeof line, f) || sscanf(line, "%d %d %d %d", &k, &L, &n1, &n2) != 4 || k < 0 || k > 20 ||
        L < 1 || L > 10 || n1 < 0 || n1 > 5 || n2 < 0 || n2 > 3) {
        fclose(f);
        return -1;
    }
    int cap = 1024, n = 1;
    int32_t *par = (int32_t *)malloc(sizeof(int32_t) * cap);
    uint8_t *leaf = (uint8_t *)malloc(cap), *desc = (uint8_t *)malloc(32 * (size_t)cap);
    double *w = (double *)malloc(sizeof(double) * cap);
    par[0] = -1; leaf[0] = 0; memset(desc, 0, 32); w[0] = 0;
    while (fgets(line, sizeof line, f)) {
        char *p = line;
        while (*p == ' ' || *p == '\t') p++;
        if (*p == '\n' || *p == '\r' || *p == 0) continue;
        if (n == cap) {
            cap *= 2;
            par = (int32_t *)realloc(par, sizeof(int32_t) * cap);
            leaf = (uint8_t *)realloc(leaf, cap);
            desc = (uint8_t *)realloc(desc, 32 * (size_t)cap);
            w = (double *)realloc(w, sizeof(double) * cap);
        }
        char *end;
        par[n] = (int32_t)strtol(p, &end, 10); p = end;
        leaf[n] = strtol(p, &end, 10) > 0; p = end;
        for (int j = 0; j < 32; j++) { desc[32 * (size_t)n + j] = (uint8_t)strtol(p, &end, 10); p = end; }
        w[n] = strtod(p, &end);
        n++;
    }
    fclose(f);
    const int rc = orc_vocab_build(v, k, L, n1, n2, n, par, leaf, desc, w);
    free(par); free(leaf); free(desc); free(w);
    return rc;
}

/* transform(feature, word_id, weight, nid, levelsup) */
static void descend(const orc_vocab *v, const uint8_t *f, int levelsup, int *word, double *w, int *nid) {
    const int nid_level = v->L - levelsup;
    *nid = 0;
    int final_id = 0, level = 0;
    do {
        ++level;
        const int a = v->child_start[final_id], b = v->child_start[final_id + 1];
        final_id = v->children[a];
        double best_d = orc_descriptor_distance(f, v->desc + 32 * (size_t)final_id);
        for (int c = a + 1; c < b; c++) {
            const int id = v->children[c];
            const double d = orc_descriptor_distance(f, v->desc + 32 * (size_t)id);
            if (d < best_d) { best_d = d; final_id = id; }
        }
        if (level == nid_level) *nid = final_id;
    } while (v->child_start[final_id + 1] > v->child_start[final_id]);   /* !isLeaf() */
    *word = v->word_id[final_id];
    *w = v->weight[final_id];
}

static int cmp_u64(const void *a, const void *b) {
    const uint64_t x = *(const uint64_t *)a, y = *(const uint64_t *)b;
    return x < y ? -1 : (x > y ? 1 : 0);
}

int orc_bow_transform(const orc_vocab *v, const uint8_t *desc, int n, int levelsup, uint32_t *words, double *values,
                      int *n_words, uint32_t *fv_nodes, int *fv_start, int *fv_features, int *n_fv) {
    *n_words = 0;
    *n_fv = 0;
    fv_start[0] = 0;
    if (v->n_words == 0 || n <= 0) return 0;                     /* empty() */
    int *wd = (int *)malloc(sizeof(int) * (size_t)n), *nd = (int *)malloc(sizeof(int) * (size_t)n);
    double *wt = (double *)malloc(sizeof(double) * (size_t)n);
    uint64_t *kw = (uint64_t *)malloc(sizeof(uint64_t) * (size_t)n), *kn = (uint64_t *)malloc(sizeof(uint64_t) * (size_t)n);
    int m = 0;
    for (int i = 0; i < n; i++) {
        descend(v, desc + 32 * (size_t)i, levelsup, &wd[i], &wt[i], &nd[i]);
        if (wt[i] > 0) {                                         /* not stopped */
            kw[m] = ((uint64_t)(uint32_t)wd[i] << 32) | (uint32_t)i;
            kn[m] = ((uint64_t)(uint32_t)nd[i] << 32) | (uint32_t)i;
            m++;
        }
    }
    /* BowVector: std::map<WordId, WordValue>, features added in index order */
    qsort(kw, m, sizeof(uint64_t), cmp_u64);
    const int tf = v->weighting == 0 || v->weighting == 1;
    int nw = 0;
    for (int j = 0; j < m;) {
        const uint32_t word = (uint32_t)(kw[j] >> 32);
        double acc = wt[(uint32_t)kw[j]];
        int e = j + 1;
        for (; e < m && (uint32_t)(kw[e] >> 32) == word; e++)
            if (tf) acc += wt[(uint32_t)kw[e]];                  /* addWeight; addIfNotExist keeps the first */
        words[nw] = word;
        values[nw] = acc;
        nw++;
        j = e;
    }
    const int must = v->scoring != 5;                            /* DotProduct: no normalisation */
    const int l2 = v->scoring == 1;
    if (tf && nw > 0 && !must) {
        const double ndv = nw;
        for (int j = 0; j < nw; j++) values[j] /= ndv;
    }
    if (must) {                                                  /* BowVector::normalize */
        double norm = 0.0;
        if (!l2) for (int j = 0; j < nw; j++) norm += fabs(values[j]);
        else { for (int j = 0; j < nw; j++) norm += values[j] * values[j]; norm = sqrt(norm); }
        if (norm > 0.0)
            for (int j = 0; j < nw; j++) values[j] /= norm;
    }
    *n_words = nw;
    /* FeatureVector: std::map<NodeId, std::vector<unsigned int>> */
    qsort(kn, m, sizeof(uint64_t), cmp_u64);
    int nf = 0;
    for (int j = 0; j < m; j++) {
        const uint32_t node = (uint32_t)(kn[j] >> 32);
        if (nf == 0 || fv_nodes[nf - 1] != node) { fv_nodes[nf] = node; fv_start[nf] = j; nf++; }
        fv_features[j] = (int)(uint32_t)kn[j];
    }
    fv_start[nf] = m;
    *n_fv = nf;
    free(wd); free(nd); free(wt); free(kw); free(kn);
    return 0;
}
