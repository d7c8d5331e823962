// hpe_team.hpp -- the team refine (round 5): refine_init_pose (PSO.cpp:216-266, cal_grad
// :183-214, goldstein :438-480) on a cloud of at most FP_MAX points by one LEADER workgroup
// and TM_NH HELPER workgroups placed on its XCD (blocks 8, 16, ...: blocks b and b + 8 are
// dealt to the same XCD; for speed only, never for correctness).  Included at the end of
// the refine section of hpe_kernels.hip.
//
// Why.  The single-workgroup refine (k_refine) is one dependent chain on one CU of 256: per
// iteration a head (cal_cost2 with new correspondences, then cal_grad's six frozen points)
// and a Goldstein search of speculated 8-node rounds.  The decision logs of the bench
// sequence (tools/gold_shapes.py) say where the time goes: 85 % of searches accept, most in
// the first round, and the eight likeliest accepted trial points ("DDDDA" 28 %, "UA" 12 %,
// "UUA" 10 %, "A" 8 %, ...) cover 87 % of them; the other 15 % run all 30 trials and fail,
// and those 30-trial searches are most of the Goldstein rounds of a frame.
//   * Heads.  At every search the leader publishes a job; helper h < TM_NHH evaluates the
//     NEXT iteration's head at the h-th likeliest accepted point (its alpha is a function of
//     the decision path alone).  When the search accepts there, the leader takes that head's
//     f_k, gradient and correspondences instead of computing them: the head runs beside the
//     search instead of after it.
//   * Trees.  Helper TM_NHH + k evaluates chunk k (8 nodes, one per wave) of a complete tree
//     of the job's next trials (heap order, TM_TREE_N nodes, 7+ levels) from the job's
//     bracket state.  The leader still runs its own 8-node round (k_refine's shapes); when
//     its walk leaves that shape it goes on through the helpers' nodes, and only past the
//     tree does it publish a continuation job and start another round there.
// Exactness.  A helper's evaluation is the leader's own operation sequence on the same
// inputs (the same device functions, thread layout and sum order: team_head, the node of
// tm_round), so a value the leader takes from a helper is bit-identical to the one it would
// have computed, and the leader applies the serial rules to every decision.  Which helper
// results arrive in time changes the timing only.  A helper marks a job's task taken (its
// claim granule) before it starts it; the leader waits only for claimed work, so missing or
// late helpers cost speed, never results.  A bounded wait that times out (a claimed result
// that never arrives) ends the refine with a NaN pose and the error flag, as the
// multi-workgroup form does.
// Hand-offs: 8-byte {tag = launch epoch, 32-bit value} granules stored and loaded with
// agent-scope relaxed atomics (write-through, sc1): a granule is valid when its tag is this
// launch's epoch, so no flags, fences or per-launch clearing (MI355X_MICROARCH.md
// handoff-1to1; cdna_hip_programming.md Guideline 16 R2).  The epoch advances when the last
// member of a launch leaves.
#pragma once

typedef unsigned long long tm_u64;
typedef __attribute__((address_space(1))) tm_u64 tm_g64;
typedef __attribute__((address_space(1))) unsigned tm_g32;

__device__ __forceinline__ void tm_put(tm_u64 *g, unsigned tag, unsigned v) {
    __hip_atomic_store((tm_g64 *)g, ((tm_u64)tag << 32) | v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ tm_u64 tm_get(const tm_u64 *g) {
    return __hip_atomic_load((tm_g64 *)g, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ bool tm_ok(tm_u64 g, unsigned tag) { return (unsigned)(g >> 32) == tag; }
__device__ __forceinline__ double tm_dbl(tm_u64 lo, tm_u64 hi) {
    return __longlong_as_double((long long)(((hi & 0xffffffffull) << 32) | (lo & 0xffffffffull)));
}
__device__ __forceinline__ unsigned tm_half(double v, int hi) {
    const tm_u64 b = (tm_u64)__double_as_longlong(v);
    return hi ? (unsigned)(b >> 32) : (unsigned)b;
}
// the double whose halves are granules g, g + 1 of a wave's load (lane k holds granule k)
__device__ __forceinline__ double tm_lane_dbl(tm_u64 v, int g) {
    return tm_dbl((tm_u64)__shfl((long long)v, g), (tm_u64)__shfl((long long)v, g + 1));
}
__device__ __forceinline__ unsigned tm_pack(const FrozenPts &fp) {
    return (unsigned)fp.id[0] | ((unsigned)fp.id[1] << 8) | ((unsigned)fp.id[2] << 16) |
           ((unsigned)fp.id[3] << 24);
}
__device__ __forceinline__ void tm_unpack(FrozenPts &fp, unsigned v) {
#pragma unroll
    for (int k = 0; k < 4; ++k) fp.id[k] = (int)((v >> (8 * k)) & 0xffu);
}
__device__ __forceinline__ tm_u64 *tm_job(const DevTeam &tm, int j) { return tm.job + (size_t)j * TM_JOB_G; }
__device__ __forceinline__ tm_u64 *tm_claim(const DevTeam &tm, int j, int h) { return tm.claim + (size_t)j * 32 + h; }
__device__ __forceinline__ tm_u64 *tm_headr(const DevTeam &tm, int j, int c) {
    return tm.head + ((size_t)j * TM_NHH + c) * TM_HEAD_G;
}
__device__ __forceinline__ tm_u64 *tm_tree(const DevTeam &tm, int j, int n) {
    return tm.tree + ((size_t)j * TM_TREE_N + n) * 2;
}

// The likeliest accepted trial points of a search (heap index from the search's start:
// node n's decisions are the bits of n + 1 after its leading one, 0 down, 1 up), by their
// share of the oracle's decision logs over three 40-frame bench sequences:
// "DDDDA" .279, "UA" .120, "UUA" .105, "A" .084, "UUUA" .054, "DDDA" .045, "DDDDDA" .036,
// "UUDA" .018 (tools/gold_shapes.py decision_logs).
__device__ __forceinline__ int tm_cand(int c) {
    constexpr int C[TM_NHH] = {15, 2, 6, 0, 14, 7, 31, 13};
    return C[c];
}
__device__ __forceinline__ int tm_cand_of(int hn) {
    int c = -1;
#pragma unroll
    for (int k = TM_NHH - 1; k >= 0; --k)
        if (tm_cand(k) == hn) c = k;
    return c;
}

// The bracket state at heap node n of a tree rooted at (a, b, al): n's decisions replayed
// with the serial rules' updates (gold_up / gold_down), the same operations as the walk.
__device__ __forceinline__ void tm_node_state(int n, double &a, double &b, double &al) {
    const unsigned m = (unsigned)n + 1u;
    const int len = 31 - __builtin_clz(m);
    for (int k = len - 1; k >= 0; --k) {
        if ((m >> k) & 1u) gold_up(a, b, al);
        else gold_down(a, b, al);
    }
}

// The head of a refine iteration (k_refine's single-workgroup small-cloud path): f_k =
// cal_cost2(x0, matchId, true) on the spheres in rs.base, the correspondence search storing
// matchId and the lane's frozen points fp, then cal_grad's six frozen evaluations at
// x0 +/- e on dims lo..lo+2 (waves 0..5; gmode: hand-frame rotation, or translation with
// rs.rg.P).  GRAD_ONLY: fp already holds x0's correspondences and fk_in is its f_k (block 2
// after a failed block-1 search: the same x0, the same spheres, so the same search).
// Returns f_k; rs.fg[0..5] the gradient costs.  Ends with a workgroup barrier.
template <class CV>
__device__ double team_head(RefineSm &rs, const DevObs &o, const CV &cv, const DevHand *__restrict__ H,
                            int32_t *__restrict__ match, FrozenPts &fp, int lo, int gmode,
                            const double *md2_l, bool grad_only, double fk_in) {
    const int t = threadIdx.x, w = t >> 6, l = t & 63;
    const double e = 1e-5;  // cal_grad step (PSO.cpp:195)
    FrozenHead hd{};
    auto head = [&]() {
        if (w < 6) {
            const int d = lo + (w >> 1);
            const double xl = rs.x0[l < HPE_DOF ? l : 0];
            const double thl = (l == d) ? ((w & 1) ? xl - e : xl + e) : xl;
            if (l < HPE_DOF) rs.w[w].th[l] = thl;
            wave_sync();
            hd = gmode ? rigid_head<RG_TRANS>(rs.w[w], o, H, rs.rg, thl)
                       : rigid_head<RG_ROT>(rs.w[w], o, H, rs.rg, thl);
        }
    };
    double fk = fk_in;
    if (!grad_only) {
        const DepthG dgc = depth_issue_w0(rs.base, o, H);
        const bool young = w >= HPE_SETPRIO_FROM;  // as in eval_block
        if (young) __builtin_amdgcn_s_setprio(1);
        // one search item on every wave (HPE_RF_SPREAD's hand-frame layout)
        const double al = search_align<RF_NT, true>(rs.base, cv, H, match, load_pt(cv, 64 * w + l),
                                                    64 * w + l, BT_GENS, 64, 1);
        if (young) __builtin_amdgcn_s_setprio(0);
        const double co = 0.0;
        const double dep = depth_finish(dgc, o, t < HPE_NS);
        const double tot = wave_sum((al * o.lambda + dep) + co);  // as block_sum1
        if (l == 0) rs.red[w][0] = tot;
        head();
        __syncthreads();  // matchId complete, the corr partial sums in red
        REF_TS(rs.ts_n, 2);
        load_frozen_pts(fp, cv, match, l);
        fk = 0;
#pragma unroll
        for (int k = 0; k < RF_NW; ++k) fk += rs.red[k][0];
        fk = fk + rs.rg.C;
    } else {
        head();
    }
    if (w < 6) {
        const double f = frozen_tail<true>(rs.w[w], o, cv, H, match, hd, &fp, md2_l) + rs.rg.C;
        if (l == 0) rs.fg[w] = f;
    }
    __syncthreads();
    return fk;
}

// Team state in LDS (every member).
struct __align__(16) TeamSm {
    double tcost[TM_TREE_N];    // leader: the current job's tree costs
    tm_u64 tval[2];             // ... their valid bits
    unsigned claims;            // ... the job's claimed tasks (bit h: helper h)
    double hv[4];               // a head: f_k, g0, g1, g2
    unsigned hfp[64];           // a head's / a job's packed correspondences per lane
    int hstate;                 // head fetch: 0 not claimed, 1 valid, 2 timed out
    int fail;                   // a bounded wait timed out
    // helper: the job in hand
    double jp[3], jA, jB, jal;
    int jtype, jblk, jnxt, jnhead, jit, jmine, jidx;
    double pang[3];             // the rotation rs.rg.P was formed for (helper)
    int pvalid;
};

__device__ __forceinline__ void tm_fail(const DevTeam &tm) {
    __hip_atomic_store(tm.err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (tm.err_host) __hip_atomic_store(tm.err_host, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// ------------------------------------------------------------------------------ leader
struct TmLead {
    DevTeam tm;
    unsigned E;   // this launch's epoch (granule tag)
    int j;        // next job slot
    bool on;      // still publishing (j < TM_MAXJ - 1)
};
// A job the leader's next round publishes (wave 7, between its node's gathers and their use:
// the stores then never hold up a wait of that wave).
struct TmPub {
    bool on;
    int type, nxt, nhead, it;
    double A, B, al;
};

// Job tl.j's granules (wave 7 only): meta, x0[0..5], the direction p on dims lo..lo+2 (pl:
// component l of p in lane l), f_k, g'p, the bracket state, every lane's correspondences.
__device__ __forceinline__ void tm_publish(const TmLead &tl, const RefineSm &rs, const TmPub &pb, int blk,
                                           double fk, double gp, double pl, int lo, const FrozenPts &fp) {
    const int l = threadIdx.x & 63;
    tm_u64 *job = tm_job(tl.tm, tl.j);
    const int pk = (l >= 13 && l <= 18) ? (l - 13) >> 1 : 0;
    const double pv = __shfl(pl, lo + pk);  // every lane takes part (clamped index)
    unsigned v = 0;
    const int h = (l + 1) & 1;  // granules 1, 3, ... hold low halves
    if (l == 0)
        v = (unsigned)pb.type | ((unsigned)blk << 2) | ((unsigned)pb.nxt << 3) | ((unsigned)pb.nhead << 5) |
            ((unsigned)pb.it << 9);
    else if (l <= 12) v = tm_half(rs.x0[(l - 1) >> 1], h);
    else if (l <= 18) v = tm_half(pv, h);
    else if (l <= 20) v = tm_half(fk, h);
    else if (l <= 22) v = tm_half(gp, h);
    else if (l <= 24) v = tm_half(pb.A, h);
    else if (l <= 26) v = tm_half(pb.B, h);
    else if (l <= 28) v = tm_half(pb.al, h);
    if (l < 32) tm_put(job + l, tl.E, v);
    tm_put(job + 32 + l, tl.E, tm_pack(fp));
}

// Wave 0 reads job j's tree costs and claims into LDS; the caller synchronises.
__device__ __forceinline__ void tm_sweep_tree(TeamSm &ts, const TmLead &tl, int j) {
    const int l = threadIdx.x & 63;
    const tm_u64 a0 = tm_get(tm_tree(tl.tm, j, l)), a1 = tm_get(tm_tree(tl.tm, j, l) + 1);
    const tm_u64 b0 = tm_get(tm_tree(tl.tm, j, l + 64)), b1 = tm_get(tm_tree(tl.tm, j, l + 64) + 1);
    const tm_u64 cl = tm_get(tm_claim(tl.tm, j, l & 31));
    const bool va = tm_ok(a0, tl.E) && tm_ok(a1, tl.E), vb = tm_ok(b0, tl.E) && tm_ok(b1, tl.E);
    ts.tcost[l] = tm_dbl(a0, a1);
    ts.tcost[l + 64] = tm_dbl(b0, b1);
    const tm_u64 ma = __ballot(va), mb = __ballot(vb), mc = __ballot(tm_ok(cl, tl.E) && l < 32);
    if (l == 0) {
        ts.tval[0] = ma;
        ts.tval[1] = mb;
        ts.claims = (unsigned)mc;
    }
}

// One speculated round of the leader's search: waves w < nn evaluate the shape's nodes
// from the bracket state (A, B, alpha) into rs.f (k_refine's eval_nodes, hand-frame small
// cloud); wave 7 publishes pb's job meanwhile.  Ends with a workgroup barrier.
template <class CV>
__device__ __forceinline__ void tm_round(RefineSm &rs, const TmLead &tl, const GoldShape &sh, double A,
                                         double B, double alpha, const DevObs &o, const CV &cv,
                                         const DevHand *__restrict__ H, double pl, const FrozenPts &fp,
                                         int blk, const double *md2_l, const TmPub &pb, double fk,
                                         double gp) {
    const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
    const int nn = sh.n;
    if (w < nn) {
        const int nbw = (int)((sh.nb >> (8 * w)) & 0xff), len = nbw >> 5, bits = nbw & 31;
        double ga = A, gb = B, gal = alpha;
        for (int k = 0; k < len; ++k) {
            if ((bits >> k) & 1) gold_up(ga, gb, gal);
            else gold_down(ga, gb, gal);
        }
        const double thl = rs.x0[l < HPE_DOF ? l : 0] + gal * pl;
        if (l < HPE_DOF) rs.w[w].th[l] = thl;
        wave_sync();
        const FrozenHead hd = blk ? rigid_head<RG_TRANS>(rs.w[w], o, H, rs.rg, thl)
                                  : rigid_head<RG_ROT>(rs.w[w], o, H, rs.rg, thl);
        if (pb.on && w == 7) tm_publish(tl, rs, pb, blk, fk, gp, pl, 3 * blk, fp);
        const double f = frozen_tail<true>(rs.w[w], o, cv, H, nullptr, hd, &fp, md2_l) + rs.rg.C;
        if (l == 0) rs.f[w] = f;
    } else if (pb.on && w == 7) {
        tm_publish(tl, rs, pb, blk, fk, gp, pl, 3 * blk, fp);
    }
    REF_TS(rs.ts_n, 9);
    __syncthreads();
    REF_TS(rs.ts_n, 8);
}

// The Goldstein search (PSO.cpp:438-480) of the team leader: k_refine's speculated rounds
// (shape policy POL), walked on through the helpers' tree of the round's job; x0 -= tk * g
// applied at the end (gl: component threadIdx.x of g).  pb: the search's job (pb.on false:
// none).  acc_hn: the accepted node's heap index from the search's start (-1: accepted in a
// continuation, or no acceptance).
template <int POL, class CV>
__device__ double tm_gold(RefineSm &rs, TeamSm &ts, TmLead &tl, const DevObs &o, const CV &cv,
                          const DevHand *__restrict__ H, double fk, double gp, double pl,
                          double gl, int &evals, const FrozenPts &fp, int blk,
                          const double *md2_l, TmPub pb, int &acc_hn, bool &base_valid) {
    const int t = threadIdx.x;
    double A = 0, B = 1e100, alpha = 0.5, tk = 0;
    int it = 0, ctx = 0;
    bool done = false;
    int jcur = pb.on ? tl.j : -1;  // the job whose tree the round's walk may use
    bool in_search = true;         // ... and it is the search's own job
    acc_hn = -1;
    while (!done) {
        const GoldShape sh = gold_shape<POL>(ctx);
        tm_round(rs, tl, sh, A, B, alpha, o, cv, H, pl, fp, blk, md2_l, pb, fk, gp);
        if (pb.on) {
            ++tl.j;
            tl.on = tl.j < TM_MAXJ - 1;
            pb.on = false;
        }
        // the serial rules on the round's own nodes (k_refine's walk), tracking the heap index
        int node = 0, hj = 0, accepted = -1;
#pragma unroll
        for (int lev = 0; lev < 6; ++lev) {  // the deepest shape path is 6 nodes
            if (node >= 15 || done) break;
            if (it >= 30) {
                done = true;
                tk = 0;
                break;
            }
            ++it;
            const double f1 = rs.f[node];
            const double armijo = fk + 0.25 * alpha * gp;
            const double gold = fk + (1 - 0.25) * alpha * gp;
            if (f1 <= armijo) {
                if (f1 >= gold) {
                    tk = alpha;
                    done = true;
                    accepted = node;
                } else {
                    gold_up(A, B, alpha);
                    node = (int)((sh.up >> (4 * node)) & 15u);
                    hj = 2 * hj + 2;
                    ctx = 2;
                }
            } else {
                gold_down(A, B, alpha);
                node = (int)((sh.dn >> (4 * node)) & 15u);
                hj = 2 * hj + 1;
                ctx = 1;
            }
        }
        if (done && accepted >= 0 && in_search) acc_hn = hj;
        // then on through the helpers' tree of this round's job, as far as it is claimed
        if (!done && jcur >= 0 && hj < TM_TREE_N) {
            int spins = 0;
            bool swept = false;
            for (;;) {
                if (it >= 30) {
                    done = true;
                    tk = 0;
                    break;
                }
                if (!swept || !((ts.tval[hj >> 6] >> (hj & 63)) & 1ull)) {
                    if (swept && !((ts.claims >> (TM_NHH + (hj >> 3))) & 1u)) break;  // nobody took it
                    if (swept && ++spins > tl.tm.spin) {
                        if (t == 0) tm_fail(tl.tm);
                        ts.fail = 1;
                        done = true;
                        tk = __builtin_nan("");
                        break;
                    }
                    if (swept) __builtin_amdgcn_s_sleep(1);
                    if (t < 64) tm_sweep_tree(ts, tl, jcur);
                    __syncthreads();
                    swept = true;
                    continue;
                }
                const double f1 = ts.tcost[hj];
                ++it;
                const double armijo = fk + 0.25 * alpha * gp;
                const double gold = fk + (1 - 0.25) * alpha * gp;
                if (f1 <= armijo) {
                    if (f1 >= gold) {
                        tk = alpha;
                        done = true;
                        if (in_search) acc_hn = hj;
                        break;
                    }
                    gold_up(A, B, alpha);
                    hj = 2 * hj + 2;
                    ctx = 2;
                } else {
                    gold_down(A, B, alpha);
                    hj = 2 * hj + 1;
                    ctx = 1;
                }
                if (hj >= TM_TREE_N) break;
            }
        }
        if (!done && it >= 30) done = true;  // tk stays 0
        if (done && t < HPE_DOF) rs.x0[t] = rs.x0[t] - tk * gl;  // PSO.cpp:256
        if (done && accepted >= 0) {  // the accepted node's spheres: the next f_k's, if needed
            for (int q = t; q < (int)(offsetof(FkSm, J) / 8); q += RF_NT)
                ((double *)&rs.base)[q] = ((const double *)&rs.w[accepted])[q];
        }
        if (done) base_valid = (tk == 0) ? base_valid : accepted >= 0;
        __syncthreads();
        REF_TS(rs.ts_n, 4);
        if (!done) {  // another round from here, publishing a job for the tree below it
            in_search = false;
            jcur = -1;
            if (tl.on) {
                pb = TmPub{true, TM_JOB_CONT, 0, 0, it, A, B, alpha};
                jcur = tl.j;
            }
        }
    }
    evals += it;
    return tk;
}

// Wave 0 polls head candidate c of job js until it is valid or found unclaimed; the result
// goes to LDS (ts.hstate 0 not claimed, 1 valid, 2 timed out).  The caller synchronises.
__device__ __forceinline__ void tm_poll_head(TeamSm &ts, const TmLead &tl, int js, int c) {
    const int l = threadIdx.x & 63;
    const tm_u64 *hd = tm_headr(tl.tm, js, c);
    int st = 2;
    tm_u64 g0 = 0, g1 = 0;
    for (int s = 0; s <= tl.tm.spin; ++s) {
        const tm_u64 cl = tm_get(tm_claim(tl.tm, js, c));
        g0 = tm_get(hd + (l & 7));
        g1 = tm_get(hd + 8 + l);
        if (!tm_ok(cl, tl.E)) {
            st = 0;
            break;
        }
        if (__all(tm_ok(g0, tl.E) && tm_ok(g1, tl.E))) {
            st = 1;
            break;
        }
        __builtin_amdgcn_s_sleep(1);
    }
    const int sv = l & 3;  // scalar sv's halves: granules 2 sv, 2 sv + 1
    const double v = tm_lane_dbl(g0, 2 * sv);
    if (l < 4) ts.hv[l] = v;
    ts.hfp[l] = (unsigned)g1;
    if (l == 0) ts.hstate = st;
}

// The hand-frame centres q (x0's digits at theta0 = -180, theta1..5 = 0) and the call's
// self-collision constant C, by wave 0 (as k_refine); the caller synchronises.
__device__ __forceinline__ void rigid_setup(RefineSm &rs, const DevHand *__restrict__ H) {
    const int t = threadIdx.x, l = t & 63;
    if (t >= 64) return;
    const double xl = rs.x0[l < HPE_DOF ? l : 0];
    const double thq = (l == 0) ? -180.0 : (l < 6) ? 0.0 : xl;
    if (l < HPE_DOF) rs.w[0].th[l] = thq;
    wave_sync();
    SphXYZ own;
    fk_wave<true>(rs.w[0], H, &own, &thq);
    if (l < HPE_NS) {
        rs.rg.q[l][0] = own.x;
        rs.rg.q[l][1] = own.y * -1;
        rs.rg.q[l][2] = own.z * -1;
    }
    CollPair cp[3];
#pragma unroll
    for (int k = 0; k < 3; ++k) cp[k] = collide_load(rs.w[0], k < 2 ? l + 64 * k : ((l < 16) ? l + 128 : l), H);
    double co = 0.0;
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        const double v = collide_value(cp[k], sqrt(collide_d2(cp[k])));
        co += (k < 2 || l < 16) ? v : 0.0;
    }
    co = wave_sum(co);
    if (l == 0) rs.rg.C = co;
}

// refine_init_pose (PSO.cpp:216-266) by the team leader: k_refine's hand-frame small-cloud
// path, every search published to the helpers and the next head taken from a helper when
// the search accepts at a point one of them evaluated.
template <class CV>
__device__ void tm_leader(RefineSm &rs, TeamSm &ts, TmLead &tl, const DevObs &o, const CV &cv,
                          const DevHand *__restrict__ H, int32_t *__restrict__ match,
                          const double *md2_l, int &evals) {
    const int t = threadIdx.x, w = t >> 6, l = t & 63;
    const double e = 1e-5;  // cal_grad step (PSO.cpp:195)
    FrozenPts fpts;
    fpts.id[0] = fpts.id[1] = fpts.id[2] = fpts.id[3] = 0;
    bool base_valid = false, have_head = false, failed_blk = false;
    double fk_h = 0, g0_h = 0, g1_h = 0, g2_h = 0, fk_last = 0;
    for (int blk = 0; blk < 2 && !ts.fail; ++blk) {
        const int lo = 3 * blk;  // start_idx (PSO.cpp:226-227); end_idx = lo + 2
        if (blk == 1) {  // P = Rg q of the block's fixed rotation (translation steps only)
            if (w == 0) rigid_wave<RG_STORE_P>(rs.w[0], rs.rg, rs.x0[l < HPE_DOF ? l : 0], nullptr, rs.rg.P);
            __syncthreads();
        }
        // block 2 after a failed block-1 search: x0 and its spheres are unchanged, so
        // cal_cost2(x0, matchId, true) repeats the last one exactly (f_k, matchId)
        bool grad_only = blk == 1 && failed_blk && !have_head;
        double tol = 1;
        int cnt = 0, iter = 0;
        while (tol > 1e-6 && iter < 15 && cnt < 1) {
            double fk, g0, g1, g2;
            REF_TS(rs.ts_n, 1);
            if (have_head) {  // a helper's head at this x0 (bit-identical to team_head's)
                fk = fk_h;
                g0 = g0_h;
                g1 = g1_h;
                g2 = g2_h;
                have_head = false;
                REF_TS(rs.ts_n, 2);
            } else {
                if (!base_valid && !grad_only) {
                    if (t < HPE_DOF) rs.base.th[t] = rs.x0[t];
                    __syncthreads();
                    if (w == 0) {
                        const double thl = rs.x0[l < HPE_DOF ? l : 0];
                        if (blk) rigid_wave<RG_TRANS>(rs.base, rs.rg, thl);
                        else rigid_wave<RG_ROT>(rs.base, rs.rg, thl);
                    }
                    __syncthreads();
                    base_valid = true;
                }
                if (grad_only) REF_TS(rs.ts_n, 2);
                fk = team_head(rs, o, cv, H, match, fpts, lo, blk, md2_l, grad_only, fk_last);
                g0 = (rs.fg[0] - rs.fg[1]) / (2 * e);
                g1 = (rs.fg[2] - rs.fg[3]) / (2 * e);
                g2 = (rs.fg[4] - rs.fg[5]) / (2 * e);
            }
            grad_only = false;
            fk_last = fk;
            evals += 7;
            REF_TS(rs.ts_n, 3);
            // cal_grad (PSO.cpp:197-212) and the dot products, as k_refine
            const int dl = l - lo;
            const double gl = (dl == 0) ? g0 : (dl == 1) ? g1 : (dl == 2) ? g2 : 0.0;
            const double pl = -1 * gl;
            const double q0 = g0 * (-1 * g0), q1 = g1 * (-1 * g1), q2 = g2 * (-1 * g2);
            const double s0 = g0 * g0, s1 = g1 * g1, s2 = g2 * g2;
            const double gp = (blk == 0) ? (q0 + q2) + q1 : q1 + (q0 + q2);
            const double tol_n = sqrt((blk == 0) ? (s0 + s2) + s1 : s1 + (s0 + s2));
            // the head an accepted point of this search leads to: the same block's next
            // iteration (1), block 2's first (2), or none (0: the refine ends)
            const int nxt = (iter + 1 < 15 && tol_n > 1e-6) ? 1 : (blk == 0 ? 2 : 0);
            const int js = tl.on ? tl.j : -1;
            const TmPub pb{tl.on, TM_JOB_SEARCH, nxt, nxt ? TM_NHH : 0, 0, 0.0, 1e100, 0.5};
            int acc_hn = -1;
            const double tk = tm_gold<HPE_GOLD_POLICY>(rs, ts, tl, o, cv, H, fk, gp, pl, gl, evals, fpts, blk,
                                                       md2_l, pb, acc_hn, base_valid);
            if (ts.fail) break;
            if (tk == 0) cnt += 1;
            tol = tol_n;
            iter += 1;
            failed_blk = tk == 0;
            // the next head from the helper that evaluated the accepted point, if one did
            const int c = (tk != 0 && nxt && js >= 0 && acc_hn >= 0) ? tm_cand_of(acc_hn) : -1;
            if (c >= 0) {
                if (w == 0) tm_poll_head(ts, tl, js, c);
                __syncthreads();
                if (ts.hstate == 2) {
                    if (t == 0) tm_fail(tl.tm);
                    ts.fail = 1;
                    break;
                }
                if (ts.hstate == 1) {
                    have_head = true;
                    fk_h = ts.hv[0];
                    g0_h = ts.hv[1];
                    g1_h = ts.hv[2];
                    g2_h = ts.hv[3];
                    tm_unpack(fpts, ts.hfp[l]);
                }
            }
            REF_TS(rs.ts_n, 5);
        }
    }
}

// ------------------------------------------------------------------------------ helper
// Serve jobs until the leader's EXIT: helper h < TM_NHH takes the head at candidate h of
// every search job (with head tasks), helper TM_NHH + k chunk k of every job's tree; each
// evaluated with the leader's operations and published.
template <class CV>
__device__ void tm_helper(RefineSm &rs, TeamSm &ts, const DevTeam &tm, unsigned E, int h,
                          const DevObs &o, const CV &cv, const DevHand *__restrict__ H,
                          int32_t *__restrict__ match, const double *md2_l) {
    const int t = threadIdx.x, w = t >> 6, l = t & 63;
    const double e = 1e-5;
    int jn = 0;
    if (t == 0) ts.pvalid = 0;
    for (;;) {
        __syncthreads();  // the previous task's reads of the job are done
        // ---- job jn in one round trip (its granules, and the metas of the newer slots: a
        // helper that fell behind moves to the newest job) (wave 0)
        if (w == 0) {
            int found = -1;
            tm_u64 ga = 0, gb = 0;
            for (int s = 0;; ++s) {
                const int jm = jn + 1 + l < TM_MAXJ ? jn + 1 + l : TM_MAXJ - 1;
                ga = tm_get(tm_job(tm, jn) + (l & 31));
                gb = tm_get(tm_job(tm, jn) + 32 + l);
                const tm_u64 gm = tm_get(tm_job(tm, jm));
                const tm_u64 newer = __ballot(tm_ok(gm, E) && jn + 1 + l < TM_MAXJ);
                if (newer) {
                    jn = jn + 1 + (63 - __builtin_clzll(newer));
                    continue;
                }
                const tm_u64 g0 = (tm_u64)__shfl((long long)ga, 0);  // EXIT: its meta alone
                if (__all(tm_ok(ga, E) && tm_ok(gb, E)) ||
                    (tm_ok(g0, E) && ((unsigned)g0 & 3u) == (unsigned)TM_JOB_EXIT)) {
                    found = jn;
                    break;
                }
                if (s >= tm.spin) break;  // the leader never published: leave
                __builtin_amdgcn_s_sleep(1);
            }
            const unsigned meta = (unsigned)__shfl((long long)ga, 0);
            const int type = found < 0 ? TM_JOB_EXIT : (int)(meta & 3u);
            const int nhead = (int)((meta >> 5) & 15u);
            const bool mine = type != TM_JOB_EXIT && (h < TM_NHH ? (type == TM_JOB_SEARCH && h < nhead) : true);
            const double x6 = tm_lane_dbl(ga, 1 + 2 * (l < 6 ? l : 0));
            const double p3 = tm_lane_dbl(ga, 13 + 2 * (l < 3 ? l : 0));
            const double jA = tm_lane_dbl(ga, 23), jB = tm_lane_dbl(ga, 25), jal = tm_lane_dbl(ga, 27);
            if (mine) {
                if (l < 6) rs.x0[l] = x6;
                if (l < 3) ts.jp[l] = p3;
                ts.hfp[l] = (unsigned)gb;
                if (l == 0) {
                    ts.jA = jA;
                    ts.jB = jB;
                    ts.jal = jal;
                    ts.jblk = (int)((meta >> 2) & 1u);
                    ts.jnxt = (int)((meta >> 3) & 3u);
                    ts.jit = (int)((meta >> 9) & 31u);
                    tm_put(tm_claim(tm, found, h), E, 1u);  // taken: the leader may wait for it
                }
            }
            if (l == 0) {
                ts.jtype = type;
                ts.jmine = mine ? 1 : 0;
                ts.jidx = found;
            }
        }
        __syncthreads();
        const int type = ts.jtype, js = ts.jidx;
        if (type == TM_JOB_EXIT) return;
        jn = js + 1;
        if (!ts.jmine) continue;
        const int blk = ts.jblk, lo = 3 * blk;
        // component l of the job's direction p = -1 * g (zero outside the block: -0.0)
        const double pl = (l >= lo && l < lo + 3) ? ts.jp[l - lo] : -1 * 0.0;
        FrozenPts fp;
        tm_unpack(fp, ts.hfp[l]);
        // block 2: P = Rg q of the block's rotation (the job's x0[0..2]), formed once per block
        auto same = [](double a, double b) { return __double_as_longlong(a) == __double_as_longlong(b); };
        if (blk == 1 && !(ts.pvalid && same(ts.pang[0], rs.x0[0]) && same(ts.pang[1], rs.x0[1]) &&
                          same(ts.pang[2], rs.x0[2]))) {
            if (w == 0) rigid_wave<RG_STORE_P>(rs.w[0], rs.rg, rs.x0[l < HPE_DOF ? l : 0], nullptr, rs.rg.P);
            if (t < 3) ts.pang[t] = rs.x0[t];
            if (t == 0) ts.pvalid = 1;
            __syncthreads();
        }
        if (h >= TM_NHH) {
            // ---- tree chunk k: wave w evaluates heap node 8 k + w of the job's tree
            const int n = 8 * (h - TM_NHH) + w;
            const int depth = 31 - __builtin_clz((unsigned)n + 1u);
            if (ts.jit + depth < 30) {  // (a trial the search never reaches is skipped)
                double a = ts.jA, b = ts.jB, al = ts.jal;
                tm_node_state(n, a, b, al);
                const double thl = rs.x0[l < HPE_DOF ? l : 0] + al * pl;
                if (l < HPE_DOF) rs.w[w].th[l] = thl;
                wave_sync();
                const FrozenHead hd = blk ? rigid_head<RG_TRANS>(rs.w[w], o, H, rs.rg, thl)
                                          : rigid_head<RG_ROT>(rs.w[w], o, H, rs.rg, thl);
                const double f = frozen_tail<true>(rs.w[w], o, cv, H, nullptr, hd, &fp, md2_l) + rs.rg.C;
                if (l < 2) tm_put(tm_tree(tm, js, n) + l, E, tm_half(f, l));
            }
            continue;
        }
        // ---- head task: candidate h's point, then the next iteration's head there
        const int nxt = ts.jnxt;  // 1: the same block, 2: block 2's first iteration
        double a = 0, b = 1e100, al = 0.5;
        tm_node_state(tm_cand(h), a, b, al);
        const double thc = rs.x0[l < HPE_DOF ? l : 0] + al * pl;
        __syncthreads();  // every wave has read the job's x0
        if (t < HPE_DOF) rs.x0[t] = thc;  // the leader's x0 - tk * g, bit for bit
        if (w == 0) {
            // the candidate node's spheres as the leader's round evaluated them
            if (blk) rigid_wave<RG_TRANS>(rs.base, rs.rg, thc);
            else rigid_wave<RG_ROT>(rs.base, rs.rg, thc);
        }
        if (nxt == 2 && w == 1) rigid_wave<RG_STORE_P>(rs.w[1], rs.rg, thc, nullptr, rs.rg.P);  // block 2 starts
        if (nxt == 2 && t < 3) ts.pang[t] = thc;
        if (nxt == 2 && t == 0) ts.pvalid = 1;
        __syncthreads();
        const int lo2 = nxt == 2 ? 3 : lo, gm2 = nxt == 2 ? 1 : blk;
        FrozenPts fp2;
        const double fk2 = team_head(rs, o, cv, H, match, fp2, lo2, gm2, md2_l, false, 0.0);
        if (w == 0) {
            const double g0 = (rs.fg[0] - rs.fg[1]) / (2 * e), g1 = (rs.fg[2] - rs.fg[3]) / (2 * e),
                         g2 = (rs.fg[4] - rs.fg[5]) / (2 * e);
            tm_u64 *hd = tm_headr(tm, js, h);
            const double sv = (l < 2) ? fk2 : (l < 4) ? g0 : (l < 6) ? g1 : g2;
            if (l < 8) tm_put(hd + l, E, tm_half(sv, l & 1));
            tm_put(hd + 8 + l, E, tm_pack(fp2));
        }
    }
}

// ------------------------------------------------------------------------------ kernel
// Grid 1 + 8 tm.nh (tm.nh = 0: 1 + PREP_WG).  Block 0 leads; block 8 (h + 1) is helper h on
// the leader's XCD; the first PREP_WG other blocks prepare the next frame (pa, as k_refine's
// extra workgroups), the rest leave at once.  Clouds of at most FP_MAX points, hand-frame
// form (refine_launch chooses it).
__global__ __launch_bounds__(RF_NT) void k_refine_team(double *__restrict__ x0g, const DevObs *__restrict__ og,
                                                      const DevHand *__restrict__ Hg,
                                                      int *__restrict__ evals_out, int do_refine,
                                                      PrepArgs pa, DevTeam tm) {
    extern __shared__ __align__(16) unsigned char dyn[];  // staged cloud + matchId / prep
    const int b = blockIdx.x, nh = tm.nh;
    const bool helper = b > 0 && (b & 7) == 0 && (b >> 3) <= nh;
    if (b > 0 && !helper) {
        const int p = (b - 1) - min((b - 1) >> 3, nh);
        if (pa.ctr && p < PREP_WG) prep_workgroup(pa, p, dyn);
        return;
    }
    if (!do_refine) return;
    const DevObs o = *og;  // the selected frame (device-resident: graph-stable args)
    __shared__ RefineSm rs;
    __shared__ DevHand hs;
    __shared__ TeamSm ts;
    const int t = threadIdx.x;
    const unsigned E = nh ? __hip_atomic_load((tm_g32 *)tm.ctl, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0u;
    stage_hand<RF_NT>(hs, Hg);
    const DevHand *__restrict__ H = &hs;
    double *cx = (double *)dyn, *cy = cx + o.n, *cz = cy + o.n;
    for (int p = t; p < o.n; p += RF_NT) {
        cx[p] = gp(o.cx)[p];
        cy[p] = gp(o.cy)[p];
        cz[p] = gp(o.cz)[p];
    }
    const CloudView cv{cx, cy, cz, o.n};
    int32_t *match = (int32_t *)(cz + o.n);
    if (t < HPE_DOF) rs.x0[t] = x0g[t];
    if (t == 0) {
        rs.ts_n = 0;
        ts.fail = 0;
    }
    REF_TS(rs.ts_n, 0);
    __syncthreads();
    rigid_setup(rs, H);
    __syncthreads();
    // the lane's sphere's off-image depth value, the same for every evaluation of the call
    const double md2_l = depth_off_sq(o, H->radii[(t & 63) < HPE_NS ? (t & 63) : HPE_NS - 1]);
    if (helper) {
        tm_helper(rs, ts, tm, E, (b >> 3) - 1, o, cv, H, match, &md2_l);
    } else {
        TmLead tl{tm, E, 0, nh > 0};
        int evals = 0;
        tm_leader(rs, ts, tl, o, cv, H, match, &md2_l, evals);
        if (nh && t == 0) tm_put(tm_job(tm, tl.j), E, (unsigned)TM_JOB_EXIT);  // (slot <= TM_MAXJ - 1)
        REF_TS(rs.ts_n, 7);
        // a timed-out hand-off leaves no defined result: the pose becomes NaN
        if (t < HPE_DOF) x0g[t] = ts.fail ? __builtin_nan("") : rs.x0[t];
        if (t == 0 && evals_out) {
            *evals_out = evals;
            atomicAdd((unsigned long long *)(evals_out + 2), (unsigned long long)evals);  // running total
        }
    }
    if (nh) {  // the last member out advances the epoch for the next launch
        __syncthreads();
        if (t == 0) {
            const unsigned n = atomicAdd(&tm.ctl[32], 1u);
            if (n == (unsigned)nh) {
                __hip_atomic_store(&tm.ctl[32], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                __hip_atomic_store(&tm.ctl[0], E + 1u == 0u ? 1u : E + 1u, __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_AGENT);
            }
        }
    }
}
