/*
 * ORACLE PIN — validates the oracle's glibc logf restatement (track_oracle.c orc_logf,
 * used by MapPoint::PredictScale through std::log(float)) against the live libm over EVERY
 * positive float (normal and subnormal) plus +inf. Exit status 1 on any mismatch.
 */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>
#include "../track_oracle.h"
int main(void) {
    long n = 0, bad = 0;
    for (uint64_t u = 1; u <= 0x7f800000u; ++u) {
        const uint32_t v = (uint32_t)u;
        float x;
        memcpy(&x, &v, 4);
        volatile float a = logf(x);
        const float b = orc_logf(x);
        if (memcmp((const void *)&a, &b, 4)) {
            if (bad < 5) printf("mismatch x=%a libm=%a oracle=%a\n", x, a, b);
            bad++;
        }
        n++;
    }
    printf("{\"inputs\": %ld, \"logf_mismatch\": %ld}\n", n, bad);
    return bad ? 1 : 0;
}
