// hpe_optimise.hpp -- pso_optimise (PSO.cpp:539-712) on the device.
// Included by hpe_kernels.hip after k_refine: it reuses RefineSm and gold_tree.
//
// One generation is two launches over P workgroups (one particle each):
//   k_opt_descent  ten single-coordinate descent steps per particle (:592-639): f_k,
//                  cal_gradient on coordinate permu(m) (:380-405, two waves), the
//                  speculated Goldstein tree, the step and the pbest update;
//                  check_constraints; then gbest <- particles.col(argmin pcost) (:643-650)
//   k_opt_move     the global-best velocity / position update with w, c1, c2 (:652-677),
//                  cal_cost (:679-689), pbest, then gbest / count (:692-704)
// The gbest update at the end of each phase is done by the last workgroup to arrive
// (release / acquire at agent scope, hpe_prep.hpp:prep_arrive_last), so no extra launch.
//
// Evaluations that the serial code repeats on identical inputs are reused, bitwise:
//   * f_k of step m >= 1 is cal_cost2(theta, matchId, false) of the theta and matchId
//     the previous step ended with -- the value that step's f_k update computed;
//   * the post-step cal_cost2 of a step m >= 1 equals the accepted Goldstein trial
//     (theta + tk * (-g) == theta - tk * g in IEEE arithmetic, same frozen matchId), or
//     f_k when tk = 0; at m = 0 it re-matches (cal_corr), unless tk = 0 left theta as is.
#pragma once

#define OPT_GRADITER 10  // graditer (PSO.cpp:575)

// Arma Col::min(index) over pcost by one workgroup; with (fmin < gbest cost) the gbest
// takes particles.col(fmin_id).  count_mode: count = 0 on improvement, += 1 otherwise
// (:700-703; the descent phase only resets it, :647).  g > 0 records the trace.
__device__ void opt_update_gbest(const DevOpt &op, Smem &sm, bool count_mode, int g,
                                 bool init) {
    const int t = threadIdx.x;
    VI mine = {__builtin_inf(), t < op.P ? t : 0x7fffffff};
    for (int p = t; p < op.P; p += HPE_NT) {
        const double c = op.pc[p];
        if (c < mine.v) {  // NaN never wins: Armadillo's scan starts from +inf
            mine.v = c;
            mine.i = p;
        }
    }
    const VI best = block_argmin(sm, mine);
    const double gc = init ? 1e100 : op.gbest[26];
    const double cnt = init ? 0.0 : op.gbest[27];
    const bool imp = best.v < gc;
    __syncthreads();
    if (t < HPE_DOF) {
        if (imp) op.gbest[t] = op.x[(size_t)best.i * HPE_DOF + t];
        else if (init) op.gbest[t] = 0.0;  // gbest_pos = zeros (:548)
    }
    if (t == 0) {
        const double nc = imp ? best.v : gc;
        op.gbest[26] = nc;
        op.gbest[27] = imp ? 0.0 : (count_mode ? cnt + 1.0 : cnt);
        if (g > 0) op.trace[g - 1] = nc;
    }
}

// generate_particles(particles, x0, num_p, false) and the initial costs (:553-569).
__global__ __launch_bounds__(HPE_NT) void k_opt_init(DevOpt op, const double *__restrict__ x0,
                                                     const DevObs *__restrict__ og,
                                                     const DevHand *__restrict__ Hg) {
    const DevObs o = *og;
    __shared__ Smem sm;
    __shared__ int flag;
    const int i = blockIdx.x, t = threadIdx.x;
    stage_hand<HPE_NT>(sm.hand, Hg);
    const DevHand *__restrict__ H = &sm.hand;
    const double *sd = op.bounds + 2 * HPE_DOF;
    if (t < HPE_DOF) {
        const size_t e = (size_t)i * HPE_DOF + t;
        const double x = x0[t] + op.normals[e] * sd[t];
        sm.fk.th[t] = x;
        op.x[e] = x;
        op.pb[e] = x;
        op.v[e] = 0.0;
    }
    const CloudGlobal cv = obs_cloud(o);
    const Pt pre = load_pt(cv, t);
    __syncthreads();
    const double c = eval_block<EV_COST, HPE_NT>(sm, o, cv, H, nullptr, pre);
    if (t == 0) op.pc[i] = c;
    if (arrive_last_sharded(op.ctr, (unsigned)op.P, &flag)) opt_update_gbest(op, sm, false, 0, true);
}

// Descent phase of generation g (iter = g + 1).  Cloud (+ matchId) staged in LDS when
// the frame has at most RF_STAGE_MAX points, as in k_refine.
template <bool STAGED>
__global__ __launch_bounds__(RF_NT) void k_opt_descent(DevOpt op, const DevObs *__restrict__ og,
                                                       const DevHand *__restrict__ Hg, int g) {
    extern __shared__ __align__(16) unsigned char dyn[];
    const DevObs o = *og;
    __shared__ RefineSm rs;
    __shared__ DevHand hs;
    __shared__ double pbrow[32];
    __shared__ int sel_s[OPT_GRADITER];
    __shared__ int flag;
    const int i = blockIdx.x, t = threadIdx.x, w = t >> 6, l = t & 63;
    stage_hand<RF_NT>(hs, Hg);
    const DevHand *__restrict__ H = &hs;
    using CV = std::conditional_t<STAGED, CloudView, CloudGlobal>;
    CV cv;
    int32_t *match = op.match + (size_t)i * op.n_cap;
    if (STAGED) {
        double *cx = (double *)dyn, *cy = cx + o.n, *cz = cy + o.n;
        for (int p = t; p < o.n; p += RF_NT) {
            cx[p] = gp(o.cx)[p];
            cy[p] = gp(o.cy)[p];
            cz[p] = gp(o.cz)[p];
        }
        if constexpr (STAGED) cv = CV{cx, cy, cz, o.n};
        match = (int32_t *)(cz + o.n);
    }
    if constexpr (!STAGED) cv = obs_cloud(o);
    const size_t e = (size_t)i * HPE_DOF + t;
    double vel = 0.0;
    if (t < HPE_DOF) {
        rs.x0[t] = op.x[e];
        vel = op.v[e];
    }
    if (t < OPT_GRADITER) {  // permu = randi(graditer, [0, 25])
        const double u = philox_u01(op.seed, ST_OPT_PERM, g, i, t);
        const int s = (int)floor(u * HPE_DOF);
        sel_s[t] = s > HPE_DOF - 1 ? HPE_DOF - 1 : s;
    }
    double pci = op.pc[i];
    bool improved = false;
    __syncthreads();
    const double e5 = 1e-5;  // cal_gradient eps (PSO.cpp:384)
    double fk = 0;
    int evals = 0;
    StampClock sc;
    sc.start();
    for (int m = 0; m < OPT_GRADITER; ++m) {
        if (m == 0) {  // f_k = cal_cost2(ctheta, matchId, true)
            if (t < HPE_DOF) rs.base.th[t] = rs.x0[t];
            __syncthreads();
            if (w == 0) fk_wave<true>(rs.base, H);
            __syncthreads();
            const DepthG dg = depth_issue_w0(rs.base, o, H);
            double al = search_align<RF_NT, true>(rs.base, cv, H, match, load_pt(cv, t));
            double co = (t < 144) ? collide_term(rs.base, t, H) : 0.0;
            double dep = depth_finish(dg, o, t < HPE_NS);
            fk = block_sum1<RF_NT>(rs.red, (al * o.lambda + dep) + co);
            sc.lap(26);
        }
        const int sel = sel_s[m];
        if (w < 2) {  // cal_gradient: theta +/- eps on coordinate sel, frozen matchId
            if (l < HPE_DOF) rs.w[w].th[l] = (l == sel) ? (w ? rs.x0[l] - e5 : rs.x0[l] + e5) : rs.x0[l];
            wave_sync();
            const double f = eval_wave_frozen<true>(rs.w[w], o, cv, H, match);
            if (l == 0) rs.f[w] = f;
        }
        __syncthreads();
        const double gs = (rs.f[0] - rs.f[1]) / (2 * e5);
        // g is gs on coordinate sel, 0 elsewhere, p = -1 * g; dot(g, p) by two accumulators
        // (op_dot::direct_dot_arma) has the one nonzero term, exactly
        const double gl = (t == sel) ? gs : 0.0;
        const double pl = -1 * ((l == sel) ? gs : 0.0);  // p = -1 * g, this thread's lane
        const double gp = gs * (-1 * gs);
        __syncthreads();  // rs.f is the Goldstein nodes' next
        sc.lap(27);
        double facc = fk;
        const double tk = gold_tree<false, GOLD_OPT8>(rs, o, cv, H, match, fk, gp, pl, 0.0, evals, &facc);
        sc.start();
        if (t < HPE_DOF) rs.x0[t] = rs.x0[t] - tk * gl;
        __syncthreads();
        double f2 = fk;  // tk == 0: theta unchanged, same matchId -> same cost
        if (tk != 0) {
            if (m == 0) {  // cal_cost2(ctheta, matchId, true): rs.base holds the new spheres
                const DepthG dg = depth_issue_w0(rs.base, o, H);
                double al = search_align<RF_NT, true>(rs.base, cv, H, match, load_pt(cv, t));
                double co = (t < 144) ? collide_term(rs.base, t, H) : 0.0;
                double dep = depth_finish(dg, o, t < HPE_NS);
                f2 = block_sum1<RF_NT>(rs.red, (al * o.lambda + dep) + co);
            } else {
                f2 = facc;
            }
        }
        if (f2 < pci) {  // pcost / pbest_pos (:627-632)
            pci = f2;
            improved = true;
            if (t < HPE_DOF) pbrow[t] = rs.x0[t];
        }
        fk = f2;
        sc.lap(28);
    }
    if (t < HPE_DOF) {  // check_constraints(ctheta, cveloc): above max -> MIN (:372)
        const double *lb = op.bounds, *ub = op.bounds + HPE_DOF;
        const double xo = rs.x0[t];
        double xn = xo;
        if (xo < lb[t]) { xn = lb[t]; vel = 0.; }
        if (xo > ub[t]) { xn = lb[t]; vel = 0.; }
        op.x[e] = xn;
        op.v[e] = vel;
        if (improved) op.pb[e] = pbrow[t];
    }
    if (t == 0) op.pc[i] = pci;
    // last workgroup: gbest <- particles.col(argmin pcost) if better (:643-650)
    Smem &sm = *reinterpret_cast<Smem *>(&rs);  // the refine workspace is dead here
    static_assert(sizeof(Smem) <= sizeof(RefineSm), "Smem overlay");
    if (arrive_last_sharded(op.ctr, (unsigned)op.P, &flag)) opt_update_gbest(op, sm, false, 0, false);
}

// Velocity / position / cost phase of generation g.
__global__ __launch_bounds__(HPE_NT) void k_opt_move(DevOpt op, const DevObs *__restrict__ og,
                                                     const DevHand *__restrict__ Hg, int g) {
    const DevObs o = *og;
    __shared__ Smem sm;
    __shared__ int flag;
    const int i = blockIdx.x, t = threadIdx.x;
    stage_hand<HPE_NT>(sm.hand, Hg);
    const DevHand *__restrict__ H = &sm.hand;
    const size_t e = (size_t)i * HPE_DOF + t;
    double xn = 0;
    if (t < HPE_DOF) {
        const double xo = op.x[e], vo = op.v[e], pbi = op.pb[e], gb = op.gbest[t];
        const double rp = philox_u01(op.seed, ST_OPT_RP, g, i, t);
        const double rg = philox_u01(op.seed, ST_OPT_RG, g, i, t);
        double vn = (op.w * vo + (op.c1 * rp) * (pbi - xo)) + (op.c2 * rg) * (gb - xo);
        xn = xo + vn;
        const double xr = xn;
        const double *lb = op.bounds, *ub = op.bounds + HPE_DOF;
        if (xr < lb[t]) { xn = lb[t]; vn = 0.; }
        if (xr > ub[t]) { xn = lb[t]; vn = 0.; }
        op.v[e] = vn;
        op.x[e] = xn;
        sm.fk.th[t] = xn;
    }
    const CloudGlobal cv = obs_cloud(o);
    const Pt pre = load_pt(cv, t);
    __syncthreads();
    const double fx = eval_block<EV_COST, HPE_NT>(sm, o, cv, H, nullptr, pre);
    const double pci = op.pc[i];
    if (fx < pci) {  // :682-686
        if (t < HPE_DOF) op.pb[e] = xn;
        if (t == 0) op.pc[i] = fx;
    }
    if (arrive_last_sharded(op.ctr, (unsigned)op.P, &flag)) opt_update_gbest(op, sm, true, g, false);
}
