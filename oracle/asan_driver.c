/*
 * asan_driver.c — TEST INFRASTRUCTURE: exercises the CPU restatement under
 * -fsanitize=address,undefined (make -C oracle sanitize; tests/test_sanitizers.py).
 * A small seeded trajectory in both modes: map building from an empty map, re-observation of
 * saved landmarks (matches), unmatched lines, an empty scan, lines beyond the capacity (the
 * capacity status bit) and the reset (Robot.cpp:893-904). Exit 0 when faithful == fast to 1e-9.
 */
#include <math.h>
#include <stdio.h>
#include <stdlib.h>

#include "ekf_oracle.h"

static unsigned long long lcg = 88172645463325252ull;
static double urand(void)
{
    lcg ^= lcg << 13;
    lcg ^= lcg >> 7;
    lcg ^= lcg << 17;
    return (double)(lcg >> 11) * (1.0 / 9007199254740992.0);
}

int main(void)
{
    const int N = 24;
    oracle_robot* a = oracle_create(N, 0, 0, 0, ORACLE_FAITHFUL, ORACLE_R_INTENDED);
    oracle_robot* b = oracle_create(N, 0, 0, 0, ORACLE_FAST, ORACLE_R_INTENDED);
    if (!a || !b) return 2;
    const int n = oracle_n(a);
    double worst = 0.0;
    for (int k = 0; k < 30; k++) {
        oracle_line ln[40];
        int L = (k == 7) ? 0 : (k == 11 ? 40 : 3 + (int)(urand() * 4));
        double pose[3];
        oracle_pose(a, pose);
        const double* y = oracle_y(a);
        const int s = oracle_saved(a);
        for (int i = 0; i < L; i++) {
            if (i < 2 && s > 0) {   /* re-observe a saved landmark */
                const int j = (int)(urand() * s);
                const double al = y[3 + 2 * j], r = y[4 + 2 * j];
                ln[i].alpha = al - pose[2];
                ln[i].r = r - (pose[0] * cos(al) + pose[1] * sin(al));
            } else {
                ln[i].alpha = -3.0 + 6.0 * urand();
                ln[i].r = 0.5 + 5.0 * urand();
            }
            ln[i].R[0] = 1e-3;
            ln[i].R[1] = ln[i].R[2] = 0.0;
            ln[i].R[3] = 2e-3;
        }
        const double enc[3] = {pose[0] + 0.01, pose[1] - 0.004, pose[2] + 0.003};
        int ma[40], mb[40];
        oracle_localize(a, ln, L, enc, ma);
        oracle_localize(b, ln, L, enc, mb);
        for (int i = 0; i < L; i++)
            if (ma[i] != mb[i]) return 3;
        const double* Pa = oracle_P(a);
        const double* Pb = oracle_P(b);
        for (int e = 0; e < n * n; e++) {
            const double d = fabs(Pa[e] - Pb[e]);
            if (d > worst) worst = d;
        }
    }
    oracle_destroy(a);
    oracle_destroy(b);
    printf("max |P_faithful - P_fast| = %.3g\n", worst);
    return worst <= 1e-9 ? 0 : 4;
}
