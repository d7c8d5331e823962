// tools/experiments/filter_check.c -- CPU replay of the fp32 filter search of
// search_filter.patch (round 3, measured slower and not kept) against the exact BFMatcher
// rule of hpe_device.hpp (same fp32 operations, -ffp-contract=off, explicit fmaf): for
// every (particle, cloud point) pair it reports how often the filter is not unique (the
// exact path runs) and counts wrong answers (must be 0 at any KE; KE scales the error bound
// E = KE u (Q + S2), the product uses 64).  Input: the binary file written by a few lines
// of numpy (int P, int N, P x 144 doubles of sphere centres, N x 3 doubles of cloud).
// Build: gcc -O2 -ffp-contract=off -o filter_check filter_check.c -lm
// Run:   ./filter_check data.bin [centre sphere index = 20] [KE = 64]
// Measured on three bench frames (100k-383k pairs): 0.12-0.16 % non-unique at KE = 64,
// 0 wrong at KE = 64 ... 0.
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <stdint.h>
static float hi_sqrt_class(float m) {
    float s = (float)sqrt((double)m);
    uint32_t b; memcpy(&b, &s, 4); b += 1; float sn; memcpy(&sn, &b, 4);
    double mid = 0.5 * ((double)s + (double)sn), mid2 = mid * mid;
    float h = (float)mid2;
    if ((double)h >= mid2) { memcpy(&b, &h, 4); b -= 1; memcpy(&h, &b, 4); }
    return h;
}
static int exact(const float *q, const float S[3][48]) {
    float d2[48], m = INFINITY;
    for (int j = 0; j < 48; ++j) {
        float t0 = q[0] - S[0][j], t1 = q[1] - S[1][j], t2 = q[2] - S[2][j];
        float a = t0 * t0; float b = t1 * t1; float c = t2 * t2;
        d2[j] = (a + b) + c;
        m = fminf(m, d2[j]);
    }
    float hi = hi_sqrt_class(m);
    for (int j = 0; j < 48; ++j) if (d2[j] <= hi) return j;
    return 48;
}
// returns -1 if not unique
static double KE = 64.0;
static int filt(const float *q, const float S[3][48], int cidx) {
    const float u = 5.9604645e-08f;  // 2^-24
    float c0 = S[0][cidx], c1 = S[1][cidx], c2 = S[2][cidx];
    float a0[48], a1[48], a2[48], ss[48], S2 = 0;
    for (int j = 0; j < 48; ++j) {
        float s0 = S[0][j] - c0, s1 = S[1][j] - c1, s2 = S[2][j] - c2;
        a0[j] = -2.f * s0; a1[j] = -2.f * s1; a2[j] = -2.f * s2;
        ss[j] = fmaf(s2, s2, fmaf(s1, s1, s0 * s0));
        S2 = fmaxf(S2, ss[j]);
    }
    float q0 = q[0] - c0, q1 = q[1] - c1, q2 = q[2] - c2;
    float Q = fmaf(q2, q2, fmaf(q1, q1, q0 * q0));
    float dm = INFINITY, dp[48];
    for (int j = 0; j < 48; ++j) {
        dp[j] = fmaf(q0, a0[j], fmaf(q1, a1[j], fmaf(q2, a2[j], ss[j])));
        dm = fminf(dm, dp[j]);
    }
    float E = (float)KE * u * (Q + S2);
    float thr = ((dm + Q) + 2.f * E) * (1.f + 3.8146973e-06f) + 2.f * E - Q;  // (1+2^-18)
    thr = thr + 0.f;
    int first = -1, last = -1;
    for (int j = 0; j < 48; ++j) {
        float t = thr - dp[j];
        if (!signbit(t)) { if (first < 0) first = j; last = j; }
    }
    if (first >= 0 && first == last) return first;
    return -1;
}
int main(int argc, char **argv) {
    // input: binary file: int P, int N; then P x 144 doubles (S, 48x3 row-major, y/z negated); N x 3 doubles cloud
    FILE *f = fopen(argv[1], "rb");
    int cidx = argc > 2 ? atoi(argv[2]) : 20;
    if (argc > 3) KE = atof(argv[3]);
    int P, N; fread(&P, 4, 1, f); fread(&N, 4, 1, f);
    double *Sd = malloc(sizeof(double) * 144 * P), *cl = malloc(sizeof(double) * 3 * N);
    fread(Sd, 8, 144 * P, f); fread(cl, 8, 3 * N, f);
    long tot = 0, nonu = 0, wrong = 0;
    for (int p = 0; p < P; ++p) {
        float S[3][48];
        for (int j = 0; j < 48; ++j) for (int r = 0; r < 3; ++r) S[r][j] = (float)Sd[p * 144 + j * 3 + r];
        for (int i = 0; i < N; ++i) {
            float q[3] = {(float)cl[3 * i], (float)cl[3 * i + 1], (float)cl[3 * i + 2]};
            int e = exact(q, S), g = filt(q, S, cidx);
            tot++;
            if (g < 0) nonu++;
            else if (g != e) wrong++;
        }
    }
    printf("items %ld non-unique %.4f%% wrong %ld\n", tot, 100.0 * nonu / tot, wrong);
    return 0;
}
