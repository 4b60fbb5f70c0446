/*
 * ORACLE PIN — validates the oracle's glibc sinf/cosf restatement (orb_oracle.c orc_cosf /
 * orc_sinf) against the live libm over EVERY float angle that computeOrbDescriptor can
 * produce: deg in [0,360] (fastAtan2 output range) times factorPI (ORBextractor.cc:156-158).
 * Prints mismatch counts; exit status 1 on any mismatch.
 */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>
#include "../orb_oracle.h"
int main(void) {
    const float factorPI = (float)(3.1415926535897932384626433832795 / 180.f);
    long nc = 0, ns = 0, n = 0;
    uint32_t hi; float h = 360.0f; memcpy(&hi, &h, 4);
    for (uint32_t u = 0; u <= hi; ++u) {
        float deg; memcpy(&deg, &u, 4);
        float ang = deg * factorPI;
        volatile float a = cosf(ang), b = sinf(ang);
        float a2 = orc_cosf(ang), b2 = orc_sinf(ang);
        n++;
        if (memcmp((const void *)&a, &a2, 4)) nc++;
        if (memcmp((const void *)&b, &b2, 4)) ns++;
    }
    printf("{\"angles\": %ld, \"cos_mismatch\": %ld, \"sin_mismatch\": %ld}\n", n, nc, ns);
    return (nc || ns) ? 1 : 0;
}
