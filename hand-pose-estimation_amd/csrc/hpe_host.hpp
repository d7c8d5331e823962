// hpe_host.hpp -- host-side helpers of the product library (see hpe_host.cpp).
#pragma once
#include <stdint.h>

#include <algorithm>
#include <vector>

#include "../../include/hpe.h"

#include "hpe_layout.hpp"

namespace hpe {
void build_dev_hand(const hpe_hand_params &p, DevHand &h);
int preprocess_depth(const float *depth_mm, int to_cm, int downsample, double focal,
                     double *depth_cm, float *dt, double *cloud, int32_t *n_out,
                     double *scale_out, double *dtmax_out, double K[9]);
double host_u01(uint64_t seed, uint32_t stream, uint32_t gen, uint32_t idx, uint32_t k);
void make_normals(uint64_t seed, int P, double *out, uint32_t stream = ST_NORMAL);
// links of every topology 1..G; indeg (optional): (G+1) x P in-degree per topology
int make_links(uint64_t seed, int P, int G, std::vector<int> &outl,
               std::vector<int> *indeg = nullptr);
}  // namespace hpe
