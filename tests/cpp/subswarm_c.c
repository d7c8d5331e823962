/* The library's subswarm exchange from plain C through include/hpe.h only (INTEGRATION.md
 * "Several GPUs"): the test_full loop over host frames (hpe_preprocess_depth + hpe_set_frame
 * + hpe_track_frame, testmodel.cpp:117-139) run plain, then on a one-rank communicator
 * (hpe_subswarm_unique_id + hpe_subswarm_init, world 1: every frame's pose and cost must be
 * bit-identical), then with the exchange in its direct-launch form (hpe_subswarm_enable 2).
 * argv: hand dir (hgeo.dat, rad.dat in mm), poses file (n lines of 26), n.  Prints
 * "subswarm_c ok ..." on success. */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "hpe.h"

#define CHECK(x)                                                                       \
    do {                                                                               \
        int rc_ = (x);                                                                 \
        if (rc_ != HPE_OK) {                                                           \
            fprintf(stderr, "%s failed (%d): %s\n", #x, rc_, hpe_last_error(ctx));     \
            return 1;                                                                  \
        }                                                                              \
    } while (0)

enum { NPIX = 240 * 320, MAXF = 16 };
static double depth_cm[NPIX], cloud[NPIX * 3];
static float dt[NPIX], raw[MAXF][NPIX];

static int read_vals(const char *path, double *v, int n) {
    FILE *f = fopen(path, "r");
    if (!f) return 0;
    int k = 0;
    while (k < n && fscanf(f, "%lf", &v[k]) == 1) ++k;
    fclose(f);
    return k == n;
}

static int track(hpe_ctx *ctx, int n, const double x0[26], double out[][27]) {
    double x[26];
    memcpy(x, x0, sizeof(x));
    for (int f = 0; f < n; ++f) {
        int32_t npts = 0;
        double scale = 0, dtmax = 0, K[9];
        CHECK(hpe_preprocess_depth(raw[f], 1, 1, 241.42, depth_cm, dt, cloud, &npts, &scale,
                                   &dtmax, K));
        hpe_frame fr = {depth_cm, dt, cloud, npts, scale, dtmax, {0}};
        memcpy(fr.K, K, sizeof(K));
        CHECK(hpe_set_frame(ctx, &fr));
        double cost = 0;
        CHECK(hpe_track_frame(ctx, 64, 1, x, &cost));  /* refine, pso_evolve, cal_cost */
        memcpy(out[f], x, sizeof(x));
        out[f][26] = cost;
    }
    return 0;
}

int main(int argc, char **argv) {
    hpe_ctx *ctx = NULL;
    if (argc < 4) return 2;
    const int n = atoi(argv[3]);
    if (n < 1 || n > MAXF) return 2;
    char path[4096];
    hpe_hand_params hp;
    memset(&hp, 0, sizeof(hp));
    snprintf(path, sizeof(path), "%s/hgeo.dat", argv[1]);
    if (!read_vals(path, hp.geo_cm, 20)) return 3;
    snprintf(path, sizeof(path), "%s/rad.dat", argv[1]);
    if (!read_vals(path, hp.radii_cm, 48)) return 3;
    for (int k = 0; k < 20; ++k) hp.geo_cm[k] /= 10.0;
    for (int k = 0; k < 48; ++k) hp.radii_cm[k] /= 10.0;
    const double cmc[5] = {150, 107.5, 89.8, 76.5, 59.6}, spc[5] = {-1.86, -1.86, 0, 1.91, 3.84};
    memcpy(hp.cmc_deg, cmc, sizeof(cmc));
    memcpy(hp.spacing_cm, spc, sizeof(spc));
    for (int k = 0; k < 4; ++k) {
        hp.tb_spheres[k] = 2;
        hp.fg_spheres[k] = k == 0 ? 4 : 2;
    }
    if (hpe_create(&ctx, 0, &hp) != HPE_OK) return 4;
    static double poses[MAXF][26];
    if (!read_vals(argv[2], &poses[0][0], 26 * n)) return 3;
    for (int f = 0; f < n; ++f) CHECK(hpe_render_depth(ctx, poses[f], 241.42, raw[f]));
    double ub[26], lb[26], sd[26];  /* testmodel.cpp:74-98 */
    for (int k = 0; k < 26; ++k) {
        if (k < 3) { ub[k] = 180; lb[k] = -180; sd[k] = 9; }
        else if (k < 6) { ub[k] = 100; lb[k] = -100; sd[k] = 7; }
        else {
            const int j = (k - 6) % 4;
            const double u[4] = {15, 90, 110, 90}, l[4] = {-15, 0, 0, 0};
            ub[k] = u[j]; lb[k] = l[j]; sd[k] = 9;
        }
    }
    CHECK(hpe_set_pso_params(ctx, ub, lb, sd, 0.7298, 1.49618, 1.49618, 11, 1e-8, 1e-8));
    static double plain[MAXF][27], xch[MAXF][27], direct[MAXF][27];
    if (track(ctx, n, poses[0], plain)) return 1;
    unsigned char id[HPE_SUBSWARM_ID_BYTES];
    CHECK(hpe_subswarm_unique_id(id));
    CHECK(hpe_subswarm_init(ctx, id, 1, 0));
    if (track(ctx, n, poses[0], xch)) return 1;
    CHECK(hpe_subswarm_enable(ctx, 2));
    if (track(ctx, n, poses[0], direct)) return 1;
    int32_t nr = -1, rk = -1, ver = 0, ig = -1;
    CHECK(hpe_subswarm_info(ctx, &nr, &rk, &ver, &ig, NULL));
    CHECK(hpe_subswarm_fini(ctx));
    if (memcmp(plain, xch, sizeof(double) * 27 * n) || memcmp(plain, direct, sizeof(double) * 27 * n)) {
        fprintf(stderr, "exchange runs differ from the plain loop\n");
        return 5;
    }
    printf("subswarm_c ok frames=%d nranks=%d rank=%d rccl=%d in_graphs=%d cost=%.17g\n", n, nr,
           rk, ver, ig, plain[n - 1][26]);
    hpe_destroy(ctx);
    return 0;
}
