// hpe_layout.hpp -- plain-C++ data layout shared by the HIP kernels and the host
// code (no HIP types): sizes, per-context hand constants, frame descriptor, swarm.
#pragma once
#include <stdint.h>

#define HPE_NT 512
#define HPE_NW (HPE_NT / 64)
#define HPE_NS 48
#define HPE_DOF 26
#define HPE_IMG_H 240
#define HPE_IMG_W 320

// Hand constants, one copy per context in HBM (read with scalar loads).
struct DevHand {
    double Fc[5], Fs[5], FLc[5], FLs[5];  // T01 / Trf: cos, sin, L*cos, L*sin
    double T10x[5], T10y[5];              // translation of T10
    double L[5][4];                       // segment lengths (cm)
    double twc[5], tws[5];                // twist of the 2nd DH factor (thumb pCMC; fingers 1, 0)
    double radii[HPE_NS];
};

// One preprocessed frame (device pointers), passed by value as a kernel argument.
struct DevObs {
    const double *cx, *cy, *cz;  // SoA cloud, n points (X, -Y, -Z) cm
    const double *depth;         // 240 x 320 cm
    const float *dt;             // 240 x 320 px
    int n;
    double lambda;               // (double)48 / n   (costfunc.cpp:372)
    double scale, dtmax;
    double K[9];
};

struct Sig {  // swarm scalars carried across generation kernels
    double gcost;
    int count;
    int topo;
};

// PSO swarm state; ping-pong slots [g & 1] for everything another workgroup reads.
struct DevSwarm {
    double *x[2], *pb[2], *pc[2];
    double *v;
    double *gpos;
    Sig *sig;                 // [2]
    const double *normals;    // P x 26
    const int *in_off;        // (G+1) x (P+1): incoming-link CSR per topology generation
    const int *in_src;        // (G+1) x 3P
    const double *bounds;     // lb[26], ub[26], std[26], x0[26]
    double *trace_g;          // [G]
    int *trace_count, *trace_topo;
    uint64_t seed;
    int P, G;
};

