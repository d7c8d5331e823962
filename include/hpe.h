/*
 * include/hpe.h -- C ABI of the MI355X-native PSO / costfunc / handmodel hot path.
 *
 * Drop-in boundary for hjurong/hand-pose-estimation (reference paths below are
 * /root/reference/src file:line).  Plain pointers and sizes only; no exceptions
 * or C++ types cross it.  Every entry point returns 0 on success and a negative
 * HPE_E* code on failure; hpe_last_error(ctx) returns the message.
 *
 * Conventions (matching the reference):
 *   - theta: 26 doubles per particle, degrees for angles, cm for position
 *     (handmodel.cpp:123-149); a batch is column-major 26 x P (PSO.cpp:67), i.e.
 *     particle-contiguous, exactly Armadillo's mat::memptr() layout.
 *   - sphere centres: 48 x 3 per particle, row-major here ([sphere][xyz]),
 *     with y and z negated (handmodel.cpp:288).
 *   - depth: 240 x 320 row-major ([v][u]); cm after preprocessing.
 *   - cloud: N x 3 row-major (X, -Y, -Z) cm (observedmodel.cpp:157-161).
 *   - match ids: int32 sphere index per cloud point (uvec matchId, costfunc.h:27).
 *
 * Ownership: the caller owns every host buffer; they are copied in/out and not
 * retained after return.  The context owns all device memory and one HIP stream.
 * Threading: one context per host thread per device; multi-GPU = one context per
 * device.
 */
#ifndef HPE_H
#define HPE_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define HPE_ABI_VERSION 1

#define HPE_OK 0
#define HPE_E_ARG -1      /* bad argument (null pointer, size out of range) */
#define HPE_E_HIP -2      /* HIP runtime error */
#define HPE_E_STATE -3    /* call order (e.g. no frame set, no PSO params) */
#define HPE_E_NOMEM -4    /* allocation failed */
#define HPE_E_NODEVICE -5 /* no gfx950 device visible */

typedef struct hpe_ctx hpe_ctx;

/* Hand geometry.  Replaces handmodel(h_geo, h_spacing, tb_spheres, fg_spheres,
 * h_CMC, sphR) (handmodel.h:9-10, handmodel.cpp:10-27).  Sphere counts must be
 * tb {2,2,2,2}, fg {4,2,2,2}: the reference hard-codes 8 + 4x10 rows
 * (handmodel.cpp:272-286). */
typedef struct {
    double geo_cm[20];    /* misc/hgeo.dat / 10, thumb first (handmodel.cpp:107-121) */
    double radii_cm[48];  /* misc/rad.dat / 10 (testmodel.cpp:49) */
    double cmc_deg[5];    /* testmodel.cpp:37 */
    double spacing_cm[5]; /* testmodel.cpp:36; narrowed to float like fingermodel.h:43 */
    int32_t tb_spheres[4];
    int32_t fg_spheres[4];
} hpe_hand_params;

/* Observation of one frame, already preprocessed (observedmodel getters,
 * observedmodel.h:51-63 / observedmodel.cpp:383-409). */
typedef struct {
    const double *depth_cm; /* 240*320 */
    const float *dt;        /* 240*320 distance transform of the background, px */
    const double *cloud;    /* n*3 */
    int32_t n;
    double scale;           /* cm per pixel (get_img_scale) */
    double dtmax;           /* max(dt) (costfunc.cpp:298) */
    double K[9];            /* camera matrix row-major (get_camera_mat) */
} hpe_frame;

int hpe_abi_version(void);
const char *hpe_last_error(const hpe_ctx *ctx);

/* Context: device buffers, the hand constants and one stream on `device`. */
int hpe_create(hpe_ctx **out, int device, const hpe_hand_params *hand);
int hpe_destroy(hpe_ctx *ctx);
/* hipStream_t of the context (for callers that order their own work after ours). */
void *hpe_stream(hpe_ctx *ctx);
int hpe_sync(hpe_ctx *ctx);

/* observedmodel::init_observation / next_frame preprocessing on the host
 * (observedmodel.cpp:110-219, 272-369): depth .bin (float mm, 240x320 row-major)
 * -> depth cm, cloud (optionally down-sampled to 250), scale, distance transform.
 * cloud_out capacity: 76800*3 doubles. */
int hpe_preprocess_depth(const float *depth_mm, int to_cm, int downsample, double focal,
                         double *depth_cm_out, float *dt_out, double *cloud_out,
                         int32_t *n_out, double *scale_out, double *dtmax_out,
                         double K_out[9]);

/* Frame residency.  `slot` in [0, 4096): a frame stored once stays in HBM; select
 * makes it the observation every following call uses (next_frame equivalent,
 * observedmodel.cpp:420-430).  hpe_set_frame = store into slot 0 + select 0. */
int hpe_store_frame(hpe_ctx *ctx, int slot, const hpe_frame *frame);
int hpe_select_frame(hpe_ctx *ctx, int slot);
int hpe_set_frame(hpe_ctx *ctx, const hpe_frame *frame);

/* observedmodel::next_frame on the GPU (observedmodel.cpp:110-219, 272-369): the raw
 * depth .bin (float mm, 240x320 row-major, host memory) is copied through a pinned
 * buffer and preprocessed by one workgroup on the context's preprocessing stream --
 * depth cm, cloud (down-sampled to 250 points when `downsample`), cm-per-pixel scale,
 * 5x5 chamfer distance transform and its max -- straight into frame slot `slot`.
 * Asynchronous: the call returns once the host buffer is copied; hpe_select_frame(slot)
 * orders the tracking stream after it, so frame f+1 is prepared while frame f is tracked.
 * Cloud, depth, DT, its max and the scale equal hpe_preprocess_depth bit for bit. */
int hpe_prepare_frame(hpe_ctx *ctx, int slot, const float *depth_mm, int to_cm, int downsample,
                      double focal);

/* Copies a stored or prepared frame back to the host (tests, debugging); synchronises.
 * cloud: n*3 doubles (capacity 76800*3); any output may be NULL. */
int hpe_frame_readback(hpe_ctx *ctx, int slot, double *depth_cm, float *dt, double *cloud,
                       int32_t *n_out, double *scale_out, double *dtmax_out);

/* handmodel::build_hand_model for a batch (handmodel.cpp:259-298).
 * theta: 26*P; S_out: P*48*3; joints_out (optional, may be NULL): P*21*3
 * (hand_joints, handmodel.cpp:291-296). */
int hpe_build_spheres(hpe_ctx *ctx, const double *theta, int P, double *S_out,
                      double *joints_out);

/* costfunc::cal_cost for a batch (costfunc.cpp:89-127; with_collision != 0 gives
 * cal_cost2(theta, matchId, true) of costfunc.cpp:31-86).  Replaces the OpenMP
 * particle loops of PSO.cpp:748-763 and :848-861.
 * match_out (optional): P*n int32 correspondences (compute_correspondences). */
int hpe_eval_costs(hpe_ctx *ctx, const double *theta, int P, int with_collision,
                   double *cost_out, int32_t *match_out);

/* costfunc::cal_cost2(theta, matchId, compute_corr, debug) (costfunc.cpp:31-86).
 * match_inout: n int32; written when compute_corr != 0, read otherwise.
 * terms_out (optional): {align, depth, collision}. */
int hpe_cal_cost2(hpe_ctx *ctx, const double theta[26], int32_t *match_inout,
                  int compute_corr, double *cost_out, double terms_out[3]);

/* The cost terms for caller-supplied sphere centres: costfunc::compute_correspondences
 * (costfunc.cpp:306-343), align_models (:346-377), depth_penalty (:227-304) and
 * self_collision_penalty (:130-197), which take a sphere matrix rather than a theta.
 * S: P*48*3 (row-major per particle, y/z negated as build_hand_model returns them).
 * match_inout: P*n int32, written when compute_corr != 0, read otherwise.
 * terms_out: P*3 {align, depth, collision}. */
int hpe_eval_spheres(hpe_ctx *ctx, const double *S, int P, int compute_corr,
                     int32_t *match_inout, double *terms_out);

/* PSO::set_pso_params (PSO.cpp:38-54).  pso_evolve uses the SPSO-2011 constants
 * (PSO.cpp:772-774); pso_optimise uses omega/phip/phig; minstep/minfunc are kept for
 * API parity (no caller reads them). */
int hpe_set_pso_params(hpe_ctx *ctx, const double ub[26], const double lb[26],
                       const double stdv[26], double omega, double phip, double phig,
                       int maxiter, double minstep, double minfunc);
/* The reference reseeds with 1000 on every pso_evolve (PSO.cpp:722). */
int hpe_set_seed(hpe_ctx *ctx, uint64_t seed);

/* PSO::pso_evolve(optfunc, x0, num_p, bestp) (PSO.cpp:717-886).
 * bestcost_out (optional) = gbest cost (pbest cost of the gbest generation). */
int hpe_pso_evolve(hpe_ctx *ctx, const double x0[26], int num_p, double bestp[26],
                   double *bestcost_out);

/* Multi-GPU subswarms, the per-frame best of N after the caller's all-gather
 * of every rank's 27-double state: d_state <- the row of d_gathered (world x 27 device
 * doubles, {bestp, cost} per rank) with the smallest cost -- NaN never wins, ties go to the
 * lowest rank (hpe/dist.py pick_best) -- as one launch on hpe_stream(ctx).  world 1..64.
 * Replaces the reference's shared gbest across its OpenMP loop (PSO.cpp:848-861). */
int hpe_pick_best(hpe_ctx *ctx, const double *d_gathered, int world, double *d_state);

/* Multi-GPU subswarms with the per-frame exchange inside the library (SURVEY.md §8e;
 * BASELINE config 5).  One process per GPU, one context each, seed 1000 + rank
 * (hpe_set_seed).  Rank 0 calls hpe_subswarm_unique_id and hands the 128 bytes to the other
 * ranks (any channel, e.g. a torch.distributed broadcast); then every rank calls
 * hpe_subswarm_init with them -- collective, RCCL's ncclCommInitRank on this context's device.
 * From then on every tracked frame of the context (hpe_track_frame[_dev],
 * hpe_track_pipelined, hpe_track_sequence_dev, hpe_track_raw_sequence_dev) ends with an
 * all-gather of every rank's {bestp, cost} (27 doubles, RCCL over xGMI) and the pick of
 * hpe_pick_best, on hpe_stream(ctx): d_state (and the frame's d_hist row) holds the best of
 * all subswarms, which every rank tracks the next frame from (testmodel.cpp:138).  The
 * exchange is captured into the tracking graphs with the frames, so N ranks run the N = 1
 * loop.  Every rank must issue the same tracking calls in the same order.  nranks = 1 is
 * allowed (the all-gather is in place: RCCL moves nothing).  hpe_subswarm_enable(ctx, 0)
 * suspends the exchange (the communicator stays), 1 resumes it, 2 resumes it with every
 * tracking call launching directly instead of through graphs -- the form the library falls
 * back to by itself (noted once on stderr) if a capture holding the collective fails.
 * hpe_subswarm_fini destroys the communicator (hpe_destroy does too).  hpe_subswarm_info:
 * world size, rank, the RCCL version (ncclGetVersion), whether the exchange runs inside
 * captured graphs (in_graphs) and, if gathered_out != NULL, a synchronous copy of the
 * gather buffer, nranks x 27 doubles (row r = rank r's last frame result; NaN before the
 * first).  RCCL is opened at run time (librccl.so.1): without it hpe_subswarm_unique_id /
 * _init return HPE_E_STATE and nothing else changes.  Any output pointer may be NULL. */
#define HPE_SUBSWARM_ID_BYTES 128
int hpe_subswarm_unique_id(unsigned char id_out[HPE_SUBSWARM_ID_BYTES]);
int hpe_subswarm_init(hpe_ctx *ctx, const unsigned char id[HPE_SUBSWARM_ID_BYTES], int nranks,
                      int rank);
int hpe_subswarm_enable(hpe_ctx *ctx, int on);
int hpe_subswarm_fini(hpe_ctx *ctx);
int hpe_subswarm_info(hpe_ctx *ctx, int32_t *nranks, int32_t *rank, int32_t *version,
                      int32_t *in_graphs, double *gathered_out);

/* Opt-in per-generation exchange between subswarms (ICP-PSO style; NOT the reference's
 * algorithm, whose gbest never enters the velocity, PSO.cpp:824-832).  every > 0: after
 * every `every`-th generation g < maxiter-1 of each pso_evolve of this context (standalone
 * or inside a tracking call) the library writes this subswarm's best pbest {pose[26], cost}
 * into d_ext (27 doubles of caller-owned device memory), then calls
 * fn(user, d_ext, g), which must enqueue on hpe_stream(ctx) the collective that replaces
 * d_ext by the best over all subswarms (lowest cost, ties to the lowest rank) and return
 * 0.  From generation g + 1 on, d_ext is an extra informant candidate of every particle:
 * it replaces the particle's informant when its cost is strictly lower (PSO.cpp:807-832 with
 * one more candidate, ranked after the local ones).  Tracking calls run without graph
 * replay while it is on.  every = 0 turns it off (fn, user, d_ext ignored). */
typedef int (*hpe_exchange_fn)(void *user, double *d_ext, int generation);
int hpe_set_exchange(hpe_ctx *ctx, int every, double *d_ext, hpe_exchange_fn fn, void *user);

/* Per-generation trace of the last pso_evolve (debug / parity):
 * gbest cost, stagnation count, topology generation; arrays of maxiter-1. */
int hpe_pso_trace(hpe_ctx *ctx, double *gbest, int32_t *count, int32_t *topo, int n);

/* PSO::pso_optimise(optfunc, x0, num_p, bestp) (PSO.cpp:539-712): global-best PSO with
 * omega/phip/phig whose particles first take 10 single-coordinate Goldstein steps every
 * generation.  maxiter-1 generations.  Draws: Philox streams 5..8 under hpe_set_seed's
 * seed (the reference draws from an unseeded Armadillo stream).  bestcost_out optional;
 * gbest_trace optional, trace_len <= maxiter-1 gbest costs, one per generation. */
int hpe_pso_optimise(hpe_ctx *ctx, const double x0[26], int num_p, double bestp[26],
                     double *bestcost_out, double *gbest_trace, int trace_len);

/* PSO::refine_init_pose(x0, optfunc) (PSO.cpp:216-266).  evals_out optional. */
int hpe_refine_init_pose(hpe_ctx *ctx, double x0[26], int32_t *evals_out);

/* Sphere placement inside refine_init_pose (every refine of this context, including the
 * tracking loops).  exact = 0 (default): the hand-frame form -- refine moves theta0..5
 * only (PSO.cpp:225-227), so each evaluation places S = Rg(theta0..2) q + u from centres q
 * built once per call, and the self-collision penalty is a constant of the call; spheres
 * within 1e-12 cm and costs within 1e-13 relative of the reference's DH chain
 * (DESIGN.md §2).  exact = 1: the reference's chain on every evaluation (bit-identical
 * FK).  The environment variable HPE_REFINE_EXACT=1 sets the default at hpe_create.
 * Cached tracking graphs are rebuilt on change. */
int hpe_set_refine_exact(hpe_ctx *ctx, int exact);
int hpe_get_refine_exact(const hpe_ctx *ctx);

/* One tracked frame of test_full (testmodel.cpp:124-138) on the selected frame:
 * [refine_init_pose] -> pso_evolve -> cost = cal_cost(bestp) -> x0 = bestp.
 * x0_inout: 26 doubles (host).  cost_out optional. */
int hpe_track_frame(hpe_ctx *ctx, int num_p, int refine, double x0_inout[26],
                    double *cost_out);

/* Same, device-resident: d_state is a device pointer to 27 doubles
 * {x0[26], cost}; read as x0, overwritten with {bestp, cost}.  Asynchronous on
 * hpe_stream(ctx): no host synchronisation. */
int hpe_track_frame_dev(hpe_ctx *ctx, int num_p, int refine, double *d_state);

/* Offline tracking of a recorded sequence: test_full's loop (testmodel.cpp:117-139) over
 * frames already resident in HBM, slots first_slot .. first_slot+n-1 (hpe_store_frame /
 * hpe_prepare_frame), each tracked exactly like hpe_track_frame_dev on its own slot and
 * d_state carried from frame to frame.  Frames are captured frames_per_graph at a time
 * into one graph (0: HPE_SEQ_CHUNK), so the graph-to-graph gap is paid once per chunk;
 * the chunk graphs read each frame's descriptor and history row through a device cursor
 * (k_seq_begin starts it, each frame's final kernel advances it), so a captured chunk
 * serves every chunk of the same shape (frames, kernel forms, d_state, d_hist) wherever
 * its slots lie.  d_hist (device, optional): n x 27 doubles,
 * frame f's {bestp, cost}.  Asynchronous on hpe_stream(ctx); the last frame is the
 * selected one afterwards, and a later hpe_prepare_frame waits for the sequence. */
#define HPE_SEQ_CHUNK 8
#define HPE_SEQ_MAX_CHUNK 32
int hpe_track_sequence_dev(hpe_ctx *ctx, int num_p, int refine, double *d_state,
                           int first_slot, int n, int frames_per_graph, double *d_hist);

/* Pipelined tracking: test_full's loop (testmodel.cpp:117-139) with next_frame
 * (observedmodel.cpp:420-430) of frame f+1 running INSIDE frame f's refine launch, on CUs
 * the single-workgroup refine leaves idle: one stream, one replayed graph per frame.
 * hpe_pipeline_begin prepares the first raw depth frame (float mm, 240x320, host).
 * hpe_track_pipelined tracks the current frame exactly like hpe_track_frame_dev
 * (d_state: 27 device doubles {x0 -> bestp, cost}) and, if next_depth_mm != NULL, copies
 * it (host) and prepares it as the next current frame; NULL ends the sequence. */
int hpe_pipeline_begin(hpe_ctx *ctx, const float *depth_mm, int to_cm, int downsample,
                       double focal);
int hpe_track_pipelined(hpe_ctx *ctx, int num_p, int refine, double *d_state,
                        const float *next_depth_mm);

/* Resident raw sequence: test_full's loop (testmodel.cpp:117-139) over n raw depth frames
 * already in HBM -- d_raw_mm: device, n x 240x320 float mm, frame after frame -- with
 * next_frame (observedmodel.cpp:420-430) of frame f+1 inside frame f's refine launch, as
 * hpe_track_pipelined does, and frames_per_graph frames (0: HPE_SEQ_CHUNK) captured into one
 * graph, so the graph-to-graph gap is paid once per chunk.  The preparation reads its raw
 * frame through a device row cursor that each frame's final kernel advances: a captured
 * chunk serves every chunk of the same shape.  Frame 0 is prepared first, on the same
 * stream.  d_state: 27 device doubles {x0 -> bestp, cost} carried from frame to frame;
 * d_hist (device, optional): n x 27 doubles, frame f's {bestp, cost}.  Asynchronous on
 * hpe_stream(ctx); ends a pipelined sequence in progress. */
int hpe_track_raw_sequence_dev(hpe_ctx *ctx, int num_p, int refine, double *d_state,
                               const float *d_raw_mm, int n, int to_cm, int downsample,
                               double focal, int frames_per_graph, double *d_hist);

/* Kernel timing with HIP events on the context stream (bench instrumentation).
 * While enabled, every dispatch of the profiled kernels is launched through
 * hipExtLaunchKernel with a start/stop event pair (dispatch-packet timestamps: the
 * kernel's own execution interval, as rocprofv3 --kernel-trace reports it).
 * hpe_profile_read_kernel synchronises and returns the launch count and total/min/max
 * device milliseconds of one kernel since the last enable; hpe_profile_read is
 * hpe_profile_read_kernel(HPE_PROF_PSO_GEN). */
#define HPE_PROF_PSO_GEN 0   /* k_pso_gen: one fused PSO generation */
#define HPE_PROF_REFINE 1    /* k_refine: refine_init_pose (+ fused next-frame preparation) */
#define HPE_PROF_PSO_INIT 2  /* k_pso_init */
#define HPE_PROF_PSO_FINAL 3 /* k_pso_final */
#define HPE_PROF_PREP 4      /* k_preprocess (hpe_prepare_frame, preprocessing stream) */
#define HPE_PROF_OPT_DESCENT 5 /* k_opt_descent: pso_optimise descent phase */
#define HPE_PROF_OPT_MOVE 6    /* k_opt_move: pso_optimise velocity / cost phase */
#define HPE_PROF_SWARM_BEST 7 /* k_swarm_best: a subswarm's best for the per-generation exchange */
#define HPE_PROF_EXCHANGE 8   /* the per-frame subswarm exchange (RCCL all-gather + k_pick_best) */
#define HPE_PROF_KERNELS 9
int hpe_profile_enable(hpe_ctx *ctx, int on);
int hpe_profile_read(hpe_ctx *ctx, int32_t *launches, double *total_ms, double *min_ms,
                     double *max_ms);
int hpe_profile_read_kernel(hpe_ctx *ctx, int kernel, int32_t *launches, double *total_ms,
                            double *min_ms, double *max_ms);
/* Evaluations done by refine_init_pose launches (cal_cost2 calls, PSO.cpp:216-266) since
 * the context was created or last reset (bench instrumentation: the algorithmic work of
 * the k_refine launches).  Synchronises; reset != 0 zeroes the count after reading. */
int hpe_refine_eval_count(hpe_ctx *ctx, uint64_t *total, int reset);

/* Number of graphs this context has captured (tracking graphs are captured once per shape
 * and replayed; tests check that a replay captured nothing). */
int hpe_graph_captures(const hpe_ctx *ctx, uint64_t *n);

/* Diagnostic build only (libhpe_stamps.so): per-phase shader-clock cycle sums
 * [0..31] and lap counts [32..63] of block 0, reset on read.  Returns 1 in the
 * stamps build, 0 in the product build (all zeros). */
int hpe_debug_stamps(unsigned long long *out64);

/* Synthetic 240x320 depth (float mm, zero background) of the 48-sphere model at
 * pose theta: front-most ray/sphere hit per pixel centre under K(focal).  Bench /
 * test input generator (no MSRA data on the box). */
int hpe_render_depth(hpe_ctx *ctx, const double theta[26], double focal, float *depth_mm_out);

#ifdef __cplusplus
}
#endif
#endif
