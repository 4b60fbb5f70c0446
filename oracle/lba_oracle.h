/*
 * ORACLE — TEST INFRASTRUCTURE ONLY. CPU restatement of Optimizer::LocalBundleAdjustment's
 * g2o optimisation (see lba_oracle.c). Uses the lba_problem / lba_result POD types of the
 * C-ABI header (types only; nothing of the product library is linked).
 */
#ifndef LBA_ORACLE_H
#define LBA_ORACLE_H
#include "../include/orbslam2_amd.h"
#ifdef __cplusplus
extern "C" {
#endif
int lba_oracle_solve(const lba_problem *p, lba_result *r, const volatile uint8_t *stop);
#ifdef __cplusplus
}
#endif
#endif
