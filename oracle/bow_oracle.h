/*
 * ORACLE — TEST INFRASTRUCTURE ONLY. CPU restatement of DBoW2's vocabulary transform used
 * by Frame::ComputeBoW (see bow_oracle.c).
 */
#ifndef BOW_ORACLE_H
#define BOW_ORACLE_H
#include <stdint.h>
#ifdef __cplusplus
extern "C" {
#endif
typedef struct {
    int k, L, scoring, weighting, n_nodes, n_words;
    int *child_start;    /* [n_nodes + 1] CSR over children in push_back order */
    int *children;       /* [n_nodes] */
    uint8_t *desc;       /* [n_nodes][32] */
    double *weight;      /* [n_nodes] */
    int *word_id;        /* [n_nodes] */
} orc_vocab;
int orc_vocab_build(orc_vocab *v, int k, int L, int scoring, int weighting, int n_nodes, const int32_t *parent,
                    const uint8_t *is_leaf, const uint8_t *desc, const double *weight);
int orc_vocab_load_text(orc_vocab *v, const char *path);
void orc_vocab_free(orc_vocab *v);
int orc_bow_transform(const orc_vocab *v, const uint8_t *desc, int n, int levelsup, uint32_t *words, double *values,
                      int *n_words, uint32_t *fv_nodes, int *fv_start, int *fv_features, int *n_fv);
#ifdef __cplusplus
}
#endif
#endif
