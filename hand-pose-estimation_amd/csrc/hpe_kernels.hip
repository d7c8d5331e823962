// hpe_kernels.hip -- gfx950 kernels of the PSO / costfunc / handmodel hot path.
//
//   k_build       handmodel::build_hand_model for a batch        (handmodel.cpp:259-298)
//   k_eval<MODE>  costfunc::cal_cost / cal_cost2 for a batch     (costfunc.cpp:31-127)
//   k_pso_init    generate_particles + initial evaluation        (PSO.cpp:56-74, 745-763)
//   k_pso_gen     one fused generation: gbest/count/topology of the previous
//                 generation, informant, velocity/position/clamp, evaluation,
//                 pbest update                                    (PSO.cpp:778-879)
//   k_pso_final   last gbest update, bestp                       (PSO.cpp:864-882)
//   k_refine      refine_init_pose as one persistent workgroup    (PSO.cpp:183-266, 438-480)
//   k_render      synthetic depth frames (bench/test input)
//
// One workgroup of HPE_NT threads per particle; see hpe_device.hpp for the block-level
// pieces and DESIGN.md for layout, rooflines and the parity argument.
#include "hpe_device.hpp"

// ------------------------------------------------------------------ batch kernels
__global__ __launch_bounds__(HPE_NT) void k_build(const double *__restrict__ theta, int P,
                                                  const DevHand *__restrict__ H,
                                                  double *__restrict__ S_out,
                                                  double *__restrict__ J_out) {
    __shared__ Smem sm;
    const int i = blockIdx.x, t = threadIdx.x;
    if (t < HPE_DOF) sm.th[t] = theta[(size_t)i * HPE_DOF + t];
    __syncthreads();
    fk_block(sm, H);
    if (t < 3 * HPE_NS) S_out[(size_t)i * 3 * HPE_NS + t] = (&sm.S[0][0])[t];
    if (J_out && t < 63) {  // hand_joints rows: wrist, index..little joints 1-4, thumb 1-4
        double v;
        if (t < 3) v = sm.th[3 + t];
        else {
            const int row = t / 3, c = t % 3, k = (row - 1) / 4, jr = 1 + (row - 1) % 4;
            const int d = (k < 4) ? k + 1 : 0;
            v = sm.J[d][jr][c];
        }
        J_out[(size_t)i * 63 + t] = v;
    }
}

template <int MODE>
__global__ __launch_bounds__(HPE_NT) void k_eval(const double *__restrict__ theta, int P,
                                                 DevObs o, const DevHand *__restrict__ H,
                                                 double *__restrict__ cost,
                                                 int32_t *__restrict__ match,
                                                 double *__restrict__ terms) {
    __shared__ Smem sm;
    const int i = blockIdx.x, t = threadIdx.x;
    if (t < HPE_DOF) sm.th[t] = theta[(size_t)i * HPE_DOF + t];
    __syncthreads();
    int32_t *m = match ? match + (size_t)i * o.n : nullptr;
    const double c = eval_block<MODE>(sm, o, H, m);
    if (t == 0) {
        cost[i] = c;
        if (terms) {
            terms[3 * i + 0] = sm.dscal[0];
            terms[3 * i + 1] = sm.dscal[1];
            terms[3 * i + 2] = sm.dscal[2];
        }
    }
}

// ------------------------------------------------------------------ PSO
// Lexicographic (value, index) minimum; NaN counts as +inf (Armadillo min(index)
// starts from +inf and keeps the first strictly smaller element).
struct VI {
    double v;
    int i;
};
__device__ __forceinline__ bool vi_less(VI a, VI b) {
    return a.v < b.v || (a.v == b.v && a.i < b.i);
}
__device__ __forceinline__ double nan_inf(double v) { return (v != v) ? __builtin_inf() : v; }

__device__ VI block_argmin(Smem &sm, VI mine) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        VI other;
        other.v = __shfl_xor(mine.v, o);
        other.i = __shfl_xor(mine.i, o);
        if (vi_less(other, mine)) mine = other;
    }
    const int w = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 0) {
        sm.red[w][0] = mine.v;
        sm.iscal[w] = mine.i;
    }
    __syncthreads();
    VI best = {sm.red[0][0], sm.iscal[0]};
#pragma unroll
    for (int k = 1; k < HPE_NW; ++k) {
        VI c = {sm.red[k][0], sm.iscal[k]};
        if (vi_less(c, best)) best = c;
    }
    __syncthreads();
    return best;
}

// End-of-generation update (PSO.cpp:864-879) for the generation whose pbest costs are
// pc (g_prev >= 1), or the initial gbest (PSO.cpp:755-760) when g_prev == 0.
// Returns the new Sig; *improved / *fid say whether gbest_pos <- x[fid].
__device__ Sig gbest_update(Smem &sm, const DevSwarm &sw, const double *__restrict__ pc,
                            double *__restrict__ pcs_lds, int g_prev, Sig prev,
                            bool *improved, int *fid) {
    VI mine = {__builtin_inf(), 0};
    for (int k = threadIdx.x; k < sw.P; k += HPE_NT) {
        const double v = pc[k];
        if (pcs_lds) pcs_lds[k] = v;
        const double vv = nan_inf(v);
        if (vv < mine.v) {
            mine.v = vv;
            mine.i = k;
        }
    }
    const VI b = block_argmin(sm, mine);
    Sig s;
    if (g_prev == 0) {
        *improved = b.v < 1e100;
        s.gcost = *improved ? b.v : 1e100;
        s.count = 100;  // PSO.cpp:768
        s.topo = -1;
    } else {
        *improved = b.v < prev.gcost;
        s.gcost = *improved ? b.v : prev.gcost;
        s.count = *improved ? 0 : prev.count + 1;
        s.topo = prev.topo;
    }
    *fid = b.i;
    return s;
}

__global__ __launch_bounds__(HPE_NT) void k_pso_init(DevSwarm sw, const double *__restrict__ x0,
                                                     DevObs o, const DevHand *__restrict__ H) {
    __shared__ Smem sm;
    const int i = blockIdx.x, t = threadIdx.x;
    const double *sd = sw.bounds + 2 * HPE_DOF;
    if (t < HPE_DOF) {  // particles = x0 + randn % std (PSO.cpp:67-72)
        const size_t e = (size_t)i * HPE_DOF + t;
        const double x = x0[t] + sw.normals[e] * sd[t];
        sm.th[t] = x;
        sw.x[0][e] = x;
        sw.pb[0][e] = x;
        sw.v[e] = 0.0;
    }
    __syncthreads();
    const double c = eval_block<EV_COST>(sm, o, H, nullptr);
    if (t == 0) sw.pc[0][i] = c;
}

__global__ __launch_bounds__(HPE_NT) void k_pso_gen(DevSwarm sw, DevObs o,
                                                    const DevHand *__restrict__ H, int g,
                                                    double W1, double C1, double C2) {
    extern __shared__ double pcs[];  // pbest costs of generation g-1, P doubles
    __shared__ Smem sm;
    const int i = blockIdx.x, t = threadIdx.x;
    const int cur = g & 1, prv = cur ^ 1;
    const double *__restrict__ pcp = sw.pc[prv];
    // 1. gbest / count of the previous generation, topology of this one (PSO.cpp:790)
    const Sig prev = (g >= 2) ? sw.sig[prv] : Sig{1e100, 100, -1};
    bool improved;
    int fid;
    Sig s = gbest_update(sm, sw, pcp, pcs, g - 1, prev, &improved, &fid);
    if (s.count > 0) s.topo = g;
    if (i == 0) {
        if (improved && t < HPE_DOF) sw.gpos[t] = sw.x[prv][(size_t)fid * HPE_DOF + t];
        if (t == 0) {
            sw.sig[cur] = s;
            if (g >= 2 && sw.trace_g) {
                sw.trace_g[g - 2] = s.gcost;
                sw.trace_count[g - 2] = s.count;
                sw.trace_topo[g - 2] = prev.topo;
            }
        }
    }
    // 2. informant: first argmin of pbest cost over {i} U incoming links (PSO.cpp:810-812)
    if (t == 0) {
        const int *off = sw.in_off + (size_t)s.topo * (sw.P + 1);
        const int *src = sw.in_src + (size_t)s.topo * 3 * sw.P;
        VI best = {nan_inf(pcs[i]), i};
        for (int e = off[i]; e < off[i + 1]; ++e) {
            const int q = src[e];
            const VI c = {nan_inf(pcs[q]), q};
            if (vi_less(c, best)) best = c;
        }
        sm.iscal[0] = best.i;
    }
    __syncthreads();
    const int inf = sm.iscal[0];
    // 3. velocity, position, check_constraints (PSO.cpp:824-842, 358-377)
    const double *lb = sw.bounds, *ub = sw.bounds + HPE_DOF;
    if (t < HPE_DOF) {
        const size_t e = (size_t)i * HPE_DOF + t;
        const double xo = sw.x[prv][e], vo = sw.v[e], pbi = sw.pb[prv][e];
        const double rp = philox_u01(sw.seed, ST_RP, g, i, t);
        double vn;
        if (inf == i) {
            vn = W1 * vo + (C1 * rp) * (pbi - xo);
        } else {
            const double rg = philox_u01(sw.seed, ST_RG, g, i, t);
            const double pbn = sw.pb[prv][(size_t)inf * HPE_DOF + t];
            vn = (W1 * vo + (C1 * rp) * (pbi - xo)) + (C2 * rg) * (pbn - xo);
        }
        double xn = xo + vn;
        const double xr = xn;
        if (xr < lb[t]) { xn = lb[t]; vn = 0.; }
        if (xr > ub[t]) { xn = lb[t]; vn = 0.; }  // above max -> MIN (PSO.cpp:372)
        sw.v[e] = vn;
        sw.x[cur][e] = xn;
        sm.th[t] = xn;
    }
    __syncthreads();
    // 4. evaluation and pbest (PSO.cpp:848-861)
    const double fx = eval_block<EV_COST>(sm, o, H, nullptr);
    const bool better = fx < pcs[i];
    if (t < HPE_DOF) {
        const size_t e = (size_t)i * HPE_DOF + t;
        sw.pb[cur][e] = better ? sm.th[t] : sw.pb[prv][e];
    }
    if (t == 0) sw.pc[cur][i] = better ? fx : pcs[i];
}

__global__ __launch_bounds__(HPE_NT) void k_pso_final(DevSwarm sw, double *__restrict__ out) {
    __shared__ Smem sm;
    const int t = threadIdx.x, G = sw.G, slot = G & 1;
    const Sig prev = (G >= 1) ? sw.sig[slot] : Sig{1e100, 100, -1};
    bool improved;
    int fid;
    const Sig s = gbest_update(sm, sw, sw.pc[slot], nullptr, G, prev, &improved, &fid);
    __syncthreads();
    if (improved && t < HPE_DOF) sw.gpos[t] = sw.x[slot][(size_t)fid * HPE_DOF + t];
    if (t == 0 && G >= 1 && sw.trace_g) {
        sw.trace_g[G - 1] = s.gcost;
        sw.trace_count[G - 1] = s.count;
        sw.trace_topo[G - 1] = prev.topo;
    }
    __syncthreads();
    if (t < HPE_DOF) out[t] = sw.gpos[t];  // bestp = gbest_pos (PSO.cpp:882)
    if (t == 0) out[HPE_DOF] = s.gcost;
}

// ------------------------------------------------------------------ refine
// refine_init_pose (PSO.cpp:216-266) with cal_grad (:183-214) and goldstein (:438-480),
// all in one workgroup: every thread evaluates the same scalar control flow from LDS.
struct RefineSmem {
    double x0[32], g[32], p[32];
};

__device__ __forceinline__ double acc2(const double *x, int n) {  // arrayops::accumulate
    double a1 = 0, a2 = 0;
    int i, j;
    for (i = 0, j = 1; j < n; i += 2, j += 2) {
        a1 += x[i];
        a2 += x[j];
    }
    if (i < n) a1 += x[i];
    return a1 + a2;
}

__global__ __launch_bounds__(HPE_NT) void k_refine(double *__restrict__ x0g, DevObs o,
                                                   const DevHand *__restrict__ H,
                                                   int32_t *__restrict__ match,
                                                   int *__restrict__ evals_out) {
    __shared__ Smem sm;
    __shared__ RefineSmem rs;
    const int t = threadIdx.x;
    if (t < HPE_DOF) rs.x0[t] = x0g[t];
    __syncthreads();
    int evals = 0;
    for (int blk = 0; blk < 2; ++blk) {
        const int lo = 3 * blk, hi = 3 * blk + 2;
        double tol = 1;
        int cnt = 0, iter = 0;
        while (tol > 1e-6 && iter < 15 && cnt < 1) {
            if (t < HPE_DOF) sm.th[t] = rs.x0[t];
            __syncthreads();
            const double fk = eval_block<EV_COST2_CORR>(sm, o, H, match);
            ++evals;
            __syncthreads();  // match[] visible to the whole block
            for (int d = lo; d <= hi; ++d) {
                const double e = 1e-5;
                if (t < HPE_DOF) sm.th[t] = rs.x0[t] + ((t == d) ? e : 0.0);
                __syncthreads();
                const double fp = eval_block<EV_COST2_FROZEN>(sm, o, H, match);
                if (t < HPE_DOF) sm.th[t] = (t == d) ? rs.x0[t] - e : rs.x0[t];
                __syncthreads();
                const double fm = eval_block<EV_COST2_FROZEN>(sm, o, H, match);
                evals += 2;
                if (t == 0) rs.g[d] = (fp - fm) / (2 * e);
            }
            if (t < HPE_DOF && (t < lo || t > hi)) rs.g[t] = 0;
            __syncthreads();
            if (t < HPE_DOF) rs.p[t] = -1 * rs.g[t];
            __syncthreads();
            // direct_dot_arma: two interleaved accumulators
            double v1 = 0, v2 = 0;
            for (int a = 0, b = 1; b < HPE_DOF; a += 2, b += 2) {
                v1 += rs.g[a] * rs.p[a];
                v2 += rs.g[b] * rs.p[b];
            }
            const double gp = v1 + v2;
            double A = 0, B = 1e100, alpha = 0.5, tk = 0;
            for (int it = 0; it < 30; ++it) {
                if (t < HPE_DOF) sm.th[t] = rs.x0[t] + alpha * rs.p[t];
                __syncthreads();
                const double f1 = eval_block<EV_COST2_FROZEN>(sm, o, H, match);
                ++evals;
                const double armijo = fk + 0.25 * alpha * gp;
                const double gold = fk + (1 - 0.25) * alpha * gp;
                if (f1 <= armijo) {
                    if (f1 >= gold) {
                        tk = alpha;
                        break;
                    }
                    A = alpha;
                    const double up = 2 * alpha, mid = 0.5 * (alpha + B);
                    alpha = (mid < up) ? mid : up;
                } else {
                    B = alpha;
                    alpha = 0.5 * (A + alpha);
                }
            }
            if (tk == 0) cnt += 1;
            __syncthreads();
            if (t < HPE_DOF) rs.x0[t] = rs.x0[t] - tk * rs.g[t];
            double g2[HPE_DOF];
            for (int d = 0; d < HPE_DOF; ++d) g2[d] = rs.g[d] * rs.g[d];
            tol = sqrt(acc2(g2, HPE_DOF));
            iter += 1;
            __syncthreads();
        }
    }
    if (t < HPE_DOF) x0g[t] = rs.x0[t];
    if (t == 0 && evals_out) *evals_out = evals;
}

// ------------------------------------------------------------------ synthetic frames
__global__ void k_render(const double *__restrict__ S, const DevHand *__restrict__ H,
                         double focal, float *__restrict__ out) {
    __shared__ double C[HPE_NS][4];
    const int t = threadIdx.x;
    if (t < HPE_NS) {  // back to the camera frame (un-negate y, z)
        C[t][0] = S[3 * t];
        C[t][1] = -S[3 * t + 1];
        C[t][2] = -S[3 * t + 2];
        C[t][3] = H->radii[t];
    }
    __syncthreads();
    const int pix = blockIdx.x * blockDim.x + t;
    if (pix >= HPE_IMG_H * HPE_IMG_W) return;
    const int r = pix / HPE_IMG_W, c = pix % HPE_IMG_W;
    const double dx = (c - 160.0) / focal, dy = (r - 120.0) / focal;
    const double dd = dx * dx + dy * dy + 1.0;
    double best = __builtin_inf();
    for (int j = 0; j < HPE_NS; ++j) {
        const double b = dx * C[j][0] + dy * C[j][1] + C[j][2];
        const double cc = (C[j][0] * C[j][0] + C[j][1] * C[j][1] + C[j][2] * C[j][2]) -
                          C[j][3] * C[j][3];
        const double disc = b * b - dd * cc;
        if (disc >= 0) {
            const double tt = (b - sqrt(disc)) / dd;
            if (tt > 0 && tt < best) best = tt;
        }
    }
    out[pix] = (best < __builtin_inf()) ? (float)(best * 10.0) : 0.0f;
}

#include "hpe_api.inc"
