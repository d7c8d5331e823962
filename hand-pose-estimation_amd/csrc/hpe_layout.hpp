// hpe_layout.hpp -- plain-C++ data layout shared by the HIP kernels and the host
// code (no HIP types): sizes, per-context hand constants, frame descriptor, swarm.
#pragma once
#include <stdint.h>

#define HPE_NT 512
#define HPE_NW (HPE_NT / 64)
#define HPE_NS 48
#define HPE_MAX_SLOTS 4096  // resident frames per context
#define HPE_DOF 26
#define HPE_IMG_H 240
#define HPE_IMG_W 320

// Philox4x32-10 streams (counter = {k/2, particle, generation, stream}): pso_evolve uses
// 1..4, pso_optimise 5..8.
enum { ST_NORMAL = 1, ST_RP = 2, ST_RG = 3, ST_LINK = 4, ST_OPT_PERM = 5, ST_OPT_RP = 6,
       ST_OPT_RG = 7, ST_OPT_NORMAL = 8 };

// Hand constants, one copy per context in HBM (read with scalar loads).
struct DevHand {
    double Fc[5], Fs[5], FLc[5], FLs[5];  // T01 / Trf: cos, sin, L*cos, L*sin
    double T10x[5], T10y[5];              // translation of T10
    double L[5][4];                       // segment lengths (cm)
    double twc[5], tws[5];                // twist of the 2nd DH factor (thumb pCMC; fingers 1, 0)
    double radii[HPE_NS];
    // sphere s = wa[s] * joint[a] + wb[s] * joint[a+1] of digit dg[s] (buildSpheres)
    double wa[HPE_NS], wb[HPE_NS];
    int32_t dg[HPE_NS], ja[HPE_NS];
};

// One preprocessed frame (device pointers).  Kept in HBM (one per slot + the selected
// one); kernels take a pointer to the selected descriptor so their arguments never change
// from frame to frame and a tracked frame replays as one hipGraph.
struct DevObs {
    const double *cx, *cy, *cz;  // SoA cloud, n points (X, -Y, -Z) cm
    const double *depth;         // 240 x 320 cm
    const float *dt;             // 240 x 320 px
    int n;
    double lambda;               // (double)48 / n   (costfunc.cpp:372)
    double scale, dtmax;
    double K[9];
};

static_assert(sizeof(DevObs) % 8 == 0, "DevObs is copied as 8-byte words");

struct Sig {  // swarm scalars carried across generation kernels
    double gcost;
    int count;
    int topo;
};

// PSO swarm state.  Positions and pbest costs keep one slot per generation (history:
// the gbest position is resolved once, in the final kernel).  Informant data travels
// by PUSH: at the end of generation g every particle writes {tag g, pbest cost, pbest
// row} into the inbox slots of the particles it informs under both possible
// topologies of generation g+1 (rebuilt at g+1, or kept), so generation g+1 reads all
// it needs from its own inbox in one round trip.
#define IB_FIELDS 28  // tag, pbest cost, pbest position[26]
// doubles between consecutive inbox rows in HBM: 28 packs the rows (a 224-B row straddles
// 128-B lines); 32 starts every row on a line (two lines per row)
#ifndef IB_STRIDE
#define IB_STRIDE 28
#endif
#define GMIN_SHARDS 32  // atomicMin cells per generation
#define GMIN_STRIDE 16  // u64 per cell: one 128-B line each
struct DevSwarm {
    double *xh;               // (G+1) x P x 26   particle positions per generation
    double *pch;              // (G+1) x P        pbest costs per generation
    double *pb;               // P x 26           pbest positions (own particle only)
    double *v;                // P x 26           velocities (own particle only)
    double *inbox;            // 2 x 2 x P x K x IB_STRIDE  [g&1][kept, rebuilt][receiver][slot]
    double *ibtc;             // 2 x 2 x P x K x {tag, cost}  (wave form: compact informant costs)
    unsigned long long *gmin; // (G+1) x GMIN_SHARDS cells (128-B apart): min pbest cost bits
                              // per generation, particle i lowering shard i % GMIN_SHARDS
    Sig *sig;                 // G+1              gbest cost / count / topology per generation
    const double *normals;    // P x 26
    const int *outl;          // (G+1) x P x 3 x 2  (receiver, slot) of each link per topology
    const double *bounds;     // lb[26], ub[26], std[26]
    double *gpos;             // 26               gbest position (final)
    double *trace_g;          // [G]
    int *trace_count, *trace_topo;
    // opt-in per-generation exchange (hpe_set_exchange; NOT the reference's algorithm):
    // {pose[26], cost} of the best pbest over all subswarms at the last exchange, an extra
    // informant candidate of every particle; nullptr: off (the reference's swarm)
    double *ext;
    uint64_t seed;
    int P, G, K;
};

// Valid inbox slots per receiver for ONE generation g of the workgroup form, passed in the
// kernel arguments (read with the other argument words, no dependent round trip).  Slots
// of a topology are filled from 0 (hpe::make_links), so receiver i reads only
// k1[i] = in-degree of i under topology g (rebuilt variant) and k0[i] = the largest
// in-degree of i under any topology 1..g-1 (kept variant), instead of K (the maximum over
// all receivers and topologies) in both.  Swarms above KIN_MAX receivers read K.
#define KIN_MAX 1024
struct InboxCounts {
    uint8_t k0[KIN_MAX];
    uint8_t k1[KIN_MAX];
};


// pso_optimise state (PSO.cpp:539-712): global-best PSO whose particles first take ten
// single-coordinate Goldstein steps each generation.  The gbest position is needed by the
// velocity update inside the generation, so it is resolved at the end of every phase by
// the last workgroup to arrive (gbest[26] = cost, gbest[27] = count).
struct DevOpt {
    double *x, *v, *pb;       // P x 26
    double *pc;               // P  pbest costs
    double *gbest;            // 28: position, cost, count
    double *trace;            // [G] gbest cost after each generation
    int32_t *match;           // P x n_cap correspondences (clouds too large for LDS)
    unsigned *ctr;            // sharded arrival counters (arrive_last_sharded)
    const double *normals;    // P x 26 (stream ST_OPT_NORMAL)
    const double *bounds;     // lb[26], ub[26], std[26]
    uint64_t seed;
    int P, G, n_cap;
    double w, c1, c2;
};

// Multi-workgroup refine (clouds too large for one CU): workgroup 0 runs refine_init_pose
// and publishes each batch of evaluations as a job; Q helper workgroups each own a fixed
// slice of the cloud (and of matchId) and return per-node partial alignment sums.
#define MW_MAX_Q 64
#define MW_MAX_NODES 8
#define MW_DONE_SHARDS 8  // completion counters (MW_MAX_Q a multiple of it)
#define MW_CTR_WORDS (32 * (MW_DONE_SHARDS + 2))
enum { MW_JOB_CORR = 1, MW_JOB_FROZEN = 2, MW_JOB_EXIT = 3 };
struct MwJob {
    int type, nnodes, pad[2];
    double th[MW_MAX_NODES][32];
};
// The subswarm exchange's pick folded into the next frame's refine launch (hpe_subswarm_init,
// inside a sequence chunk): x0 <- the best row of the all-gathered states instead of a
// k_pick_best launch between the frames.  gath == nullptr: x0 is d_state as usual.
struct DevPick {
    const double *gath;  // [world][27] {bestp, cost} per rank
    double *hist;        // the sequence's history (row *cur - 1 gets the picked state), or null
    const int *cur;      // the row cursor
    int world;
};

struct DevMw {
    MwJob *job;
    double *part;    // [MW_MAX_Q][MW_MAX_NODES] partial alignment sums
    unsigned *ctr;   // [0] job sequence; [32 (1 + s)] helper completions of shard s
                     // (helper h -> shard h % MW_DONE_SHARDS); [32 (1 + MW_DONE_SHARDS)] exits
    int *err;        // set when a wait times out (the launch then ends early)
    int *err_host;   // the same flag in pinned host memory (system-scope store): the next
                     // tracking call sees it without a synchronisation
    int Q;
    int spin;        // polls per wait before it counts as timed out (MW_SPIN_MAX; tests)
};
