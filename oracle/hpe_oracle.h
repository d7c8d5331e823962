/*
 * oracle/hpe_oracle.h -- CPU restatement of hjurong/hand-pose-estimation's
 * PSO / costfunc / handmodel hot path.
 *
 * TEST INFRASTRUCTURE ONLY.  Nothing in the product (hand-pose-estimation_amd/,
 * include/) links, loads or calls this code.  It is used by tests/ as the
 * parity checker, by __graft_entry__.smoke() as the checker, and by bench.py's
 * cpu_baseline leg (kind "port").
 *
 * PARITY STATUS: "parity unpinned" in the strict sense.  The reference ships no
 * tests, no golden vectors and no fixtures other than misc/hgeo.dat and
 * misc/rad.dat, and it cannot be compiled here (Armadillo, OpenCV, GLUT absent;
 * see DESIGN.md).  This restatement is pinned by (i) analytic known-answer
 * tests built on the reference's own data files (bone lengths, sphere
 * placement, per-branch depth penalties, constraint quirks, a hand-computed
 * PSO step), and (ii) agreement with an independent numpy restatement
 * (oracle/oracle_np.py) whose outputs are committed as tests/golden fixtures.
 *
 * Every function cites the reference file:line it restates.  Floating point
 * follows the reference's evaluation order (left-to-right sums, no FMA
 * contraction: build with -ffp-contract=off).
 */
#ifndef HPE_ORACLE_H
#define HPE_ORACLE_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define ORA_NS 48   /* spheres      handmodel.cpp:282-286 */
#define ORA_DOF 26  /* pose dims    handmodel.cpp:123-149 */
#define ORA_H 240   /* depth rows   observedmodel.cpp:308 */
#define ORA_W 320   /* depth cols */

typedef struct {
    double geo[20];     /* segment lengths, cm (misc/hgeo.dat / 10) */
    double radii[48];   /* sphere radii, cm  (misc/rad.dat / 10)   */
    double cmc[5];      /* CMC angles, degrees (testmodel.cpp:37)   */
    float spacing[5];   /* digit spacing, stored as float (fingermodel.h:43) */
    double F[5][16];    /* T01 (fingers) / Trf (thumb), row-major 4x4 */
    double T10[5][16];  /* palm-base transform, row-major 4x4 */
} ora_hand;

typedef struct {
    int n;               /* cloud points */
    const double *cloud; /* n x 3 row-major, (X, -Y, -Z) cm */
    const double *depth; /* 240 x 320 row-major, cm */
    const float *dt;     /* 240 x 320 row-major, pixels */
    double dtmax;        /* max of dt (costfunc.cpp:298) */
    double scale;        /* cm per pixel (observedmodel.cpp:202) */
    double K[9];         /* camera matrix row-major */
} ora_obs;

void ora_hand_init(ora_hand *h, const double geo_cm[20], const double radii_cm[48],
                   const double cmc_deg[5], const double spacing[5]);
void ora_build_hand_model(const ora_hand *h, const double th[26], double S[144],
                          double joints[63]);
void ora_correspondences(const ora_obs *o, const double S[144], int32_t *match);
double ora_align(const ora_hand *h, const ora_obs *o, const double S[144],
                 const int32_t *match);
double ora_depth_penalty(const ora_hand *h, const ora_obs *o, double S[144]);
double ora_collision(const ora_hand *h, const double S[144]);
double ora_cal_cost(const ora_hand *h, const ora_obs *o, const double th[26]);
double ora_cal_cost2(const ora_hand *h, const ora_obs *o, const double th[26],
                     int32_t *match, int compute_corr, double terms[3]);
void ora_eval_costs(const ora_hand *h, const ora_obs *o, const double *thetas, int P,
                    int with_collision, double *cost, int nthreads);

/* counter-based draws (the reference's Armadillo stream is toolchain dependent,
 * SURVEY.md §8c; the build defines its stream as Philox4x32-10) */
void ora_philox4x32_10(const uint32_t ctr[4], const uint32_t key[2], uint32_t out[4]);
double ora_u01(uint64_t seed, uint32_t stream, uint32_t gen, uint32_t idx, uint32_t k);
void ora_normals(uint64_t seed, int P, double *out);

typedef struct {
    double *gbest_trace;  /* [G]   gbest cost after each generation, or NULL */
    double *fmin_trace;   /* [G]   min pbest cost after each generation, or NULL */
    int *count_trace;     /* [G]   stagnation counter after each generation, or NULL */
    int *topo_trace;      /* [G]   generation whose links were in use, or NULL */
    double *pcost0;       /* [P]   initial costs, or NULL */
} ora_pso_trace;

int ora_pso_evolve(const ora_hand *h, const ora_obs *o, const double x0[26], int P,
                   int maxiter, const double lb[26], const double ub[26],
                   const double stdv[26], uint64_t seed, double bestp[26],
                   double *bestcost, ora_pso_trace *trace, int nthreads);

/* the opt-in per-generation exchange of R subswarms (hpe_set_exchange), TEST mirror of a
 * non-reference extension: bestp R x 26, bestcost R */
int ora_pso_evolve_xch(const ora_hand *h, const ora_obs *o, const double x0[26], int P,
                       int maxiter, const double lb[26], const double ub[26],
                       const double stdv[26], const uint64_t *seeds, int R, int every,
                       double *bestp, double *bestcost, int nthreads);

int ora_refine_init_pose(const ora_hand *h, const ora_obs *o, double x0[26]);
/* The same with test instrumentation: rigid != 0 runs the mirror of the GPU's hand-frame
 * refine (NOT the reference's operation order; hpe_oracle.c); margins[0..cap) receives
 * every decision's relative margin, *ndec their number; the decisions numbered
 * flips[0..nflips) have their outcome inverted (near-tie replay). */
int ora_refine_ex(const ora_hand *h, const ora_obs *o, double x0[26], int rigid,
                  const int *flips, int nflips, double *margins, int cap, int *ndec);
/* spheres of theta by the hand-frame mirror, centres q built from x0's digits */
void ora_rigid_spheres(const ora_hand *h, const double x0[26], const double th[26],
                       double S[144]);
/* test instrumentation: smallest relative decision margin of the last refine */
double ora_refine_last_margin(void);
/* diagnostic: log every Goldstein search's decisions into buf (see hpe_oracle.c) */
void ora_set_gold_log(uint64_t *buf, int cap);
int ora_gold_log_count(void);

int ora_pso_optimise(const ora_hand *h, const ora_obs *o, const double x0[26], int P,
                     int maxiter, const double lb[26], const double ub[26],
                     const double stdv[26], double w, double c1, double c2, uint64_t seed,
                     double bestp[26], double *bestcost, double *gbest_trace, int nthreads);

/* gnd_truth_err, costfunc.cpp:476-507: gnd is an Armadillo-layout (column-major)
 * n_frames x 63 matrix in mm; hand_joints the 21 x 3 row-major cm joints of
 * ora_build_hand_model (handmodel.cpp:291-296). */
double ora_gnd_truth_err(const double hand_joints[63], const double *gnd, int n_frames,
                         int frame);

void ora_dist_transform(const double *depth_cm, float *dt_out);
int ora_preprocess(const float *depth_mm, int to_cm, int downsample, double focal,
                   double *depth_cm_out, float *dt_out, double *cloud_out,
                   int *n_out, double *scale_out, double *dtmax_out, double K_out[9]);

#ifdef __cplusplus
}
#endif
#endif
