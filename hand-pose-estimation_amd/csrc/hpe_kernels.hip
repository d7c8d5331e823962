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
#include <vector>

#include "hpe_device.hpp"
#include "hpe_prep.hpp"
#include "../../include/hpe.h"

// ------------------------------------------------------------------ batch kernels
__global__ __launch_bounds__(HPE_NT) void k_build(const double *__restrict__ theta, int P,
                                                  const DevHand *__restrict__ Hg,
                                                  double *__restrict__ S_out,
                                                  double *__restrict__ J_out) {
    __shared__ Smem sm;
    const int i = blockIdx.x, t = threadIdx.x;
    stage_hand<HPE_NT>(sm.hand, Hg);
    const DevHand *__restrict__ H = &sm.hand;
    if (t < HPE_DOF) sm.fk.th[t] = theta[(size_t)i * HPE_DOF + t];
    __syncthreads();
    if (t < 64) fk_wave(sm.fk, H);
    __syncthreads();
    if (t < 3 * HPE_NS) S_out[(size_t)i * 3 * HPE_NS + t] = (&sm.fk.S[0][0])[t];
    if (J_out && t < 63) {  // hand_joints rows: wrist, index..little joints 1-4, thumb 1-4
        double v;
        if (t < 3) v = sm.fk.th[3 + t];
        else {
            const int row = t / 3, c = t % 3, k = (row - 1) / 4, jr = 1 + (row - 1) % 4;
            const int d = (k < 4) ? k + 1 : 0;
            v = sm.fk.J[d][jr][c];
        }
        J_out[(size_t)i * 63 + t] = v;
    }
}

template <int MODE>
__global__ __launch_bounds__(HPE_NT) void k_eval(const double *__restrict__ theta, int P,
                                                 const DevObs *__restrict__ og, const DevHand *__restrict__ Hg,
                                                 double *__restrict__ cost,
                                                 int32_t *__restrict__ match,
                                                 double *__restrict__ terms) {
    const DevObs o = *og;  // the selected frame (device-resident: graph-stable args)
    __shared__ Smem sm;
    const int i = blockIdx.x, t = threadIdx.x;
    stage_hand<HPE_NT>(sm.hand, Hg);
    const DevHand *__restrict__ H = &sm.hand;
    if (t < HPE_DOF) sm.fk.th[t] = theta[(size_t)i * HPE_DOF + t];
    const CloudGlobal cv = obs_cloud(o);
    const Pt pre = load_pt(cv, t);
    __syncthreads();
    int32_t *m = match ? match + (size_t)i * o.n : nullptr;
    const double c = eval_block<MODE, HPE_NT>(sm, o, cv, H, m, pre);
    if (t == 0) {
        cost[i] = c;
        if (terms) {
            terms[3 * i + 0] = sm.dscal[0];
            terms[3 * i + 1] = sm.dscal[1];
            terms[3 * i + 2] = sm.dscal[2];
        }
    }
}

// Cost terms for caller-supplied sphere centres (costfunc::align_models, depth_penalty,
// self_collision_penalty and compute_correspondences take a sphere matrix, not a theta:
// costfunc.cpp:130-377).  S: P x 48 x 3 row-major, y/z already negated.
template <int MODE>
__global__ __launch_bounds__(HPE_NT) void k_eval_spheres(const double *__restrict__ S, int P,
                                                         const DevObs *__restrict__ og, const DevHand *__restrict__ Hg,
                                                         int32_t *__restrict__ match,
                                                         double *__restrict__ terms) {
    const DevObs o = *og;  // the selected frame (device-resident: graph-stable args)
    __shared__ Smem sm;
    const int i = blockIdx.x, t = threadIdx.x;
    stage_hand<HPE_NT>(sm.hand, Hg);
    const DevHand *__restrict__ H = &sm.hand;
    if (t < 3 * HPE_NS) {
        const int s = t / 3, r = t - 3 * s;
        const double v = S[(size_t)i * 3 * HPE_NS + t];
        sm.fk.S[s][r] = v;
        sm.fk.Sp[r][s] = (float)v;
    }
    const CloudGlobal cv = obs_cloud(o);
    const Pt pre = load_pt(cv, t);
    __syncthreads();
    eval_block<MODE, HPE_NT, false>(sm, o, cv, H, match + (size_t)i * o.n, pre);
    if (t == 0) {
        terms[3 * i + 0] = sm.dscal[0];
        terms[3 * i + 1] = sm.dscal[1];
        terms[3 * i + 2] = sm.dscal[2];
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
    int wi, unused;
    wave_argmin_lex(nan_inf(mine.v), mine.i, 0, wi, unused);
    mine.v = nan_inf(mine.v);
    {
        // the winner's value: every lane holding idx wi has the minimum
        const unsigned long long b = __ballot(mine.i == wi);
        mine.v = readlane_f64(mine.v, (int)__ffsll((long long)b) - 1);
        mine.i = wi;
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

#define IB_KMAX 24  // max informant in-degree handled (host checks K <= IB_KMAX)

__device__ __forceinline__ double bits_to_f64(unsigned long long b) { return __longlong_as_double((long long)b); }
__device__ __forceinline__ unsigned long long f64_to_bits(double v) {
    return (unsigned long long)__double_as_longlong(v);
}
// The generation's minimum pbest cost (the gmin the next generation's topology decision
// and k_pso_final read), sharded: particle i lowers cell i % GMIN_SHARDS.  All 256 blocks
// of a launch hitting ONE address serialise their atomics at the memory side for ~2 us of
// every generation; 32 cells on separate 128-B lines take 8 each.  Costs are >= 0 (or
// NaN), so u64 order is value order, and the min over the shards is order-free.
__device__ __forceinline__ unsigned long long *gmin_cell(const DevSwarm &sw, int g, int s) {
    return sw.gmin + ((size_t)g * GMIN_SHARDS + s) * GMIN_STRIDE;
}
__device__ __forceinline__ void gmin_lower(const DevSwarm &sw, int g, int i, double c) {
    atomicMin(gmin_cell(sw, g, i % GMIN_SHARDS), f64_to_bits(c));
}
// min over generation g's shards by one whole wave, in every lane; NaN if none was written.
// gmin_load issues lane l's cell (unconditional), gmin_reduce folds the wave.
__device__ __forceinline__ unsigned long long gmin_load(const DevSwarm &sw, int g) {
    const int l = threadIdx.x & 63;
    return *gmin_cell(sw, g, l < GMIN_SHARDS ? l : 0);
}
__device__ __forceinline__ double gmin_reduce(unsigned long long cell) {
    const int l = threadIdx.x & 63;
    double m = (l < GMIN_SHARDS) ? bits_to_f64(cell) : __builtin_nan("");
    m = fmin(m, dpp_f64<0xB1>(m));
    m = fmin(m, dpp_f64<0x4E>(m));
    m = fmin(m, dpp_f64<0x141>(m));
    m = fmin(m, dpp_f64<0x140>(m));
    return fmin(fmin(readlane_f64(m, 0), readlane_f64(m, 16)),
                fmin(readlane_f64(m, 32), readlane_f64(m, 48)));
}
__device__ __forceinline__ double gmin_read(const DevSwarm &sw, int g) {
    return gmin_reduce(gmin_load(sw, g));
}

__device__ __forceinline__ size_t ib_index(const DevSwarm &sw, int par, int var, int r, int slot) {
    return ((((size_t)par * 2 + var) * sw.P + r) * sw.K + slot) * IB_STRIDE;
}

// Push {tag = (g, topology, s), pbest cost, pbest row} of particle s after generation g
// into the inboxes of its receivers under the topology of generation g+1 (var 1) and
// under the kept topology topo_g (var 0).  Lane q in [0, 168): destination q / 28, field
// q % 28; (r, slot) = this lane's link, prefetched by the caller (r < 0: no push).
__device__ __forceinline__ void push_inbox(const DevSwarm &sw, int g, int s, int q, int r, int slot,
                                           int tt, double pc, const double *row) {
    if (r < 0) return;
    const int dst = q / IB_FIELDS, fld = q - IB_FIELDS * dst, var = dst < 3 ? 1 : 0;
    // the tag makes a slot valid only for the exact (g, topology) the reader expects,
    // whatever an earlier call left behind
    const double val = (fld == 0) ? __longlong_as_double(((long long)g << 48) | ((long long)tt << 32) | s)
                       : (fld == 1) ? pc : row[fld - 2];
    sw.inbox[ib_index(sw, g & 1, var, r, slot) + fld] = val;
}

// Link of lane q of the pushing waves for topology tt: {receiver, slot} as one 8-byte
// load.  Loaded unconditionally (a lane with nothing to push reads entry 0 and is marked
// !ok), so no branch merge makes the wave wait for it before its use at the push.
struct Link {
    long long raw;
    bool ok;
};
__device__ __forceinline__ Link load_link(const DevSwarm &sw, int g, int s, int q, int tt,
                                          bool want = true) {
    Link L;
    L.ok = want && g < sw.G && q >= 0 && q < 6 * IB_FIELDS && tt >= 1;
    const size_t k = L.ok ? ((size_t)tt * sw.P + s) * 3 + (q / IB_FIELDS) % 3 : 0;
    L.raw = ((const long long *)sw.outl)[k];
    return L;
}
__device__ __forceinline__ void push_inbox(const DevSwarm &sw, int g, int s, int q, const Link &L,
                                           int tt, double pc, const double *row) {
    push_inbox(sw, g, s, q, L.ok ? (int)(L.raw & 0xffffffff) : -1, (int)(L.raw >> 32), tt, pc, row);
}

// generate_particles + the initial evaluation (PSO.cpp:56-74, 748-763).
template <int NT, bool FILT = false>
__device__ __forceinline__ void pso_init_body(const DevSwarm &sw, const double *__restrict__ x0,
                                              const DevObs *__restrict__ og,
                                              const DevHand *__restrict__ Hg) {
    const DevObs o = *og;  // the selected frame (device-resident: graph-stable args)
    __shared__ Smem sm;
    const int t = threadIdx.x;
    const int i = (int)blockIdx.x;
    const double hw = hand_word<NT>(Hg);
    const DevHand *__restrict__ H = &sm.hand;
    const double *sd = sw.bounds + 2 * HPE_DOF;
    // pushing lanes: waves 1..3 (q = t - 64), topology 1 = rebuilt for gen 1
    const int q = t - 64;
    const Link lk = load_link(sw, 0, i, q, 1, q < 3 * IB_FIELDS);
    const CloudGlobal cv = obs_cloud(o);
    const Pt pre = load_pt(cv, t);
    if (t < HPE_DOF) {  // particles = x0 + randn % std (PSO.cpp:67-72)
        const size_t e = (size_t)i * HPE_DOF + t;
        const double x = x0[t] + sw.normals[e] * sd[t];
        sm.fk.th[t] = x;
        sw.xh[e] = x;
        sw.pb[e] = x;
        sw.v[e] = 0.0;
    }
    if (sw.ext && i == 0 && t == 0) sw.ext[HPE_DOF] = __builtin_inf();  // no candidate yet
    hand_put<NT>(sm.hand, hw);
    __syncthreads();
    const double c = eval_block<EV_COST, NT, true, FILT>(sm, o, cv, H, nullptr, pre, BT_GENS, nullptr, true);
    if (t == 0) {  // PSO.cpp:748-763; pbest costs are >= 0, so their bits order like values
        sw.pch[i] = c;
        gmin_lower(sw, 0, i, c);
    }
    push_inbox(sw, 0, i, q, lk, 1, c, sm.fk.th);
}

template <bool FILT>
__global__ __launch_bounds__(HPE_NT) void k_pso_init(DevSwarm sw, const double *__restrict__ x0,
                                                     const DevObs *__restrict__ og, const DevHand *__restrict__ Hg) {
    pso_init_body<HPE_NT, FILT>(sw, x0, og, Hg);
}

// One fused generation g >= 1 (PSO.cpp:781-879).  Wave 0 carries the serial part: every
// load of the generation at once (own state, draws, sig[g-1] / gmin[g-1], both inboxes),
// the topology decision, the informant, the velocity step and FK, with wave-level syncs
// only.  Waves 1..3 prefetch the push links meanwhile; then all 8 waves search.
// XCH: the opt-in per-generation exchange (sw.ext) is compiled in (k_pso_gen_x and the
// XCH forms); the default kernels carry none of it.  ROW16: every inbox holds at most 15
// slots (sw.K <= 15, the host's choice of instantiation): the informant argmin runs on one
// 16-lane DPP row.  (A run-time K test left one body for both cases: the compiler no longer
// duplicated the kernel per case, and the generation ran 0.15 us slower.)
template <int NT, bool XCH = false, bool ROW16 = true, bool FILT = false>
__device__ __forceinline__ void pso_gen_body(const DevSwarm &sw, const DevObs *__restrict__ og,
                                             const DevHand *__restrict__ Hg, int g, double W1,
                                             double C1, double C2, const InboxCounts &kin) {
    static_assert(NT >= 256 && NT % 64 == 0, "waves 1..3 push, wave 0 carries the particle");
    BLK_TS(g, 0);
    // every argument word round 1 needs, loaded at entry as one batch: left alone the
    // compiler fetched g and the gmin / sig / link / bounds pointers in a second scalar
    // round trip behind the first one's wait, ahead of every global load of the round
    // (a non-volatile asm: it touches no memory, so later loads keep their scalar form)
    int z0 = 0;
    asm("" : "+s"(z0) : "s"(g), "s"(sw.gmin), "s"(sw.sig), "s"(sw.outl), "s"(sw.bounds),
        "s"(sw.xh), "s"(sw.pch), "s"(sw.pb), "s"(sw.v), "s"(sw.inbox), "s"(sw.P), "s"(sw.K),
        "s"(og), "s"(Hg));
    StampClock sc;
    sc.begin();
    const DevObs o = *og;  // the selected frame (device-resident: graph-stable args)
    __shared__ Smem sm;
    __shared__ double ib[2][IB_KMAX][IB_FIELDS];
    const int P = sw.P, K = sw.K;
    const int i = (int)blockIdx.x + z0, t = threadIdx.x;
    // valid slots of this receiver's kept (0) / rebuilt (1) inbox: only these are read
    // (read at blockIdx.x, clamped, unconditionally: the address depends on no loaded
    // argument, so these loads leave with the argument loads instead of after them)
    const int kb = (int)blockIdx.x & (KIN_MAX - 1);
    const int k0r = kin.k0[kb], k1r = kin.k1[kb];
    const int k0 = (P <= KIN_MAX) ? k0r : K, k1 = (P <= KIN_MAX) ? k1r : K;
    // Round 1: every load of the generation is issued before any value is used (one
    // memory round trip): hand words, first cloud point, push links, inbox payload rows
    // (waves 1..7); own state, own pbest cost, inbox tags / costs, gmin cells, sig (wave 0).
    // staged into LDS before the first barrier (after the argument batch: issued ahead of
    // it, this load made the compiler wait for the first argument words alone)
    const double hw = hand_word<NT>((const DevHand *)((const char *)Hg + z0));
    const DevHand *__restrict__ H = &sm.hand;
    sc.lap(4);
    const CloudGlobal cv = obs_cloud(o);
    const size_t e = (size_t)i * HPE_DOF + t;
    const int q = t - 64;  // pushing lanes (waves 1..3): var-1 links now, var-0 after the decision
    const Link lk1 = load_link(sw, g, i, q, g + 1, q < 3 * IB_FIELDS);
    double pbi = 0, xo = 0, vo = 0, rp = 0, rg = 0;  // own state (lanes t < 26 of wave 0)
    double lbt = 0, ubt = 0;                          // bounds of dimension t
    int inf = 0, islot = -1, var = 0;
    double exr = 0.0;       // per-generation exchange (sw.ext): the candidate's row, lane t
    bool use_ext = false;   // ... and whether it beats this particle's informant
    if (t >= 64) {
        // ---- waves 1..7: both informant inboxes (payload rows) into LDS
        // the k0 valid kept slots, then the k1 valid rebuilt ones
        const double *src = sw.inbox + ib_index(sw, (g - 1) & 1, 0, i, 0);
        const size_t var_stride = (size_t)P * K * IB_STRIDE;
        const int n = (k0 + k1) * IB_FIELDS, u0 = t - 64;
        constexpr int NL = (2 * IB_KMAX * IB_FIELDS + NT - 65) / (NT - 64);  // loads per lane
        double a[NL];
#pragma unroll
        for (int k = 0; k < NL; ++k) {  // unconditional (clamped) loads: no early wait
            const int u = min(u0 + k * (NT - 64), max(n - 1, 0));
            const int vr = u >= k0 * IB_FIELDS ? 1 : 0;
            const int uv = u - vr * k0 * IB_FIELDS;  // field uv % 28 of row uv / 28
            const int off = (IB_STRIDE == IB_FIELDS) ? uv : (uv / IB_FIELDS) * IB_STRIDE + uv % IB_FIELDS;
            a[k] = src[vr * var_stride + off];
        }
        if (t < 64 + 2 * HPE_DOF) {  // wave 1 draws rp, rg while the loads are in flight
            const int j = t - 64, d = j < HPE_DOF ? j : j - HPE_DOF;
            sm.draws[j] = philox_u01(sw.seed, j < HPE_DOF ? ST_RP : ST_RG, g, i, d);
        }
#pragma unroll
        for (int k = 0; k < NL; ++k) {
            const int u = u0 + k * (NT - 64);
            if (u < n) (&ib[0][0][0])[(u >= k0 * IB_FIELDS ? IB_KMAX * IB_FIELDS - k0 * IB_FIELDS : 0) + u] = a[k];
        }
    } else {
        // ---- wave 0, round 1: own state, gbest bookkeeping, inbox tags / costs
        const size_t ec = (size_t)i * HPE_DOF + (t < HPE_DOF ? t : HPE_DOF - 1);
        xo = sw.xh[(size_t)(g - 1) * P * HPE_DOF + ec];
        vo = sw.v[ec];
        pbi = sw.pb[ec];
        lbt = sw.bounds[ec - (size_t)i * HPE_DOF];
        ubt = sw.bounds[ec - (size_t)i * HPE_DOF + HPE_DOF];
        const double pci = sw.pch[(size_t)(g - 1) * P + i];  // own pbest cost (uniform)
        double tg[2], tc[2];
#pragma unroll
        for (int vr = 0; vr < 2; ++vr) {
            const int kv = vr ? k1 : k0;
            const double *sl = sw.inbox + ib_index(sw, (g - 1) & 1, vr, i, min(t, max(kv - 1, 0)));
            tg[vr] = sl[0];
            tc[vr] = sl[1];
        }
        const unsigned long long gcell = gmin_load(sw, g - 1);
        const Sig pv = sw.sig[g > 1 ? g - 1 : 0];
        if (XCH) exr = sw.ext[t <= HPE_DOF ? t : HPE_DOF];
        const double fmin = gmin_reduce(gcell);  // NaN when no value was written
        // informant = first argmin of pbest cost over {i} U incoming (PSO.cpp:810-812),
        // under BOTH variants while the gmin reduction is in flight (independent chains):
        // rebuilt = topology g, kept = the topology of g-1 (pv.topo); the decision below
        // only selects.  Candidates in lanes 0..k-1, self in lane 15 (K <= 15: one 16-lane
        // row) or 63.
        const int self_lane = ROW16 ? 15 : 63;
        int infv[2], islv[2];
        double infc[2];
#pragma unroll
        for (int vr = 0; vr < 2; ++vr) {
            const long long tag = __double_as_longlong(tg[vr]);
            const int tt = vr ? g : pv.topo;
            const bool ok = t < (vr ? k1 : k0) && (tag >> 32) == (((long long)(g - 1) << 16) | tt);
            const bool self = t == self_lane;  // L = eye
            double v = ok ? tc[vr] : (self ? pci : __builtin_inf());
            const int idx = ok ? (int)(tag & 0xffffffff) : (self ? i : 0x7fffffff);
            if (v != v) v = __builtin_inf();
            if (ROW16) row0_argmin_lex(v, idx, ok ? t : -1, infv[vr], islv[vr], XCH ? &infc[vr] : nullptr);
            else wave_argmin_lex(v, idx, ok ? t : -1, infv[vr], islv[vr], XCH ? &infc[vr] : nullptr);
        }
        BLK_TS(g, 6);
        // end-of-generation update of g-1 (PSO.cpp:864-877) / initial gbest (:755-760),
        // computed redundantly by every lane (uniform values)
        Sig sg;
        if (g == 1) {
            sg.gcost = fmin < 1e100 ? fmin : 1e100;
            sg.count = 100;  // PSO.cpp:768
            sg.topo = -1;
        } else {
            const bool imp = fmin < pv.gcost;
            sg.gcost = imp ? fmin : pv.gcost;
            sg.count = imp ? 0 : pv.count + 1;
            sg.topo = pv.topo;
        }
        if (sg.count > 0) sg.topo = g;  // topology rebuilt when count > 0 (PSO.cpp:790)
        if (i == 0 && t == 0) sw.sig[g] = sg;
        if (t == 0) {
            sm.iscal[0] = sg.topo;
            sm.dscal[4] = pci;
        }
        // var 1 iff topology g is in use; otherwise (count == 0, g >= 2) it is pv.topo
        var = (sg.topo == g) ? 1 : 0;
        sc.lap(0);
        inf = var ? infv[1] : infv[0];
        islot = var ? islv[1] : islv[0];
        // the exchanged candidate (index "P": after every local one) wins only strictly
        if (XCH) use_ext = readlane_f64(exr, HPE_DOF) < (var ? infc[1] : infc[0]);
        if (t < HPE_DOF) sm.pbr[t] = pbi;  // for the pushing waves, if x does not improve
        BLK_TS(g, 7);
        sc.lap(1);
    }
    hand_put<NT>(sm.hand, hw);
    // this thread's first cloud point, used after FK: issued behind round 1's loads, which
    // the informant choice and the row staging wait for in issue order
    const Pt pre = load_pt(cv, t);
    BLK_TS(g, 1);
    __syncthreads();  // informant rows and draws in LDS
    SphXYZ own0{0.0, 0.0, 0.0};  // wave 0: the centres FK leaves in registers
    BLK_TS(g, 2);
    if (t < 64) {
        double thl = 0.0;  // x of this lane's dimension, handed to FK's trig in a register
        // ---- velocity, position, check_constraints (PSO.cpp:824-842, 358-377)
        if (t < HPE_DOF) {
            rp = sm.draws[t];
            rg = sm.draws[HPE_DOF + t];
            double vn;
            if (inf == i && !use_ext) {
                vn = W1 * vo + (C1 * rp) * (pbi - xo);
            } else {
                const double pbn = use_ext ? exr : ib[var][islot][2 + t];
                vn = (W1 * vo + (C1 * rp) * (pbi - xo)) + (C2 * rg) * (pbn - xo);
            }
            double xn = xo + vn;
            const double xr = xn;
            if (xr < lbt) { xn = lbt; vn = 0.; }
            if (xr > ubt) { xn = lbt; vn = 0.; }  // above max -> MIN (PSO.cpp:372)
            sw.v[e] = vn;
            sw.xh[(size_t)g * P * HPE_DOF + e] = xn;
            sm.fk.th[t] = xn;
            thl = xn;
        }
        wave_sync();
        BLK_TS(g, 10);
        sc.lap(2);
        fk_wave(sm.fk, H, &own0, &thl);
    }
    __syncthreads();  // spheres, topology and own pbest cost published
    BLK_TS(g, 3);
    const int topo = sm.iscal[0];
    const double pci = sm.dscal[4];
    const Link lk0 = load_link(sw, g, i, q, topo, q >= 3 * IB_FIELDS);
    // ---- evaluation and pbest (PSO.cpp:848-861)
    const double fx = eval_block<EV_COST, NT, false, FILT>(sm, o, cv, H, nullptr, pre, g, &own0, true);
    BLK_TS(g, 4);
    sc.start();
    const bool better = fx < pci;
    const double pn = better ? fx : pci;
    if (t < HPE_DOF) sw.pb[e] = better ? sm.fk.th[t] : pbi;
    if (t == 0) {
        sw.pch[(size_t)g * P + i] = pn;
        gmin_lower(sw, g, i, pn);
    }
    // the pushed pbest row: this generation's x (in LDS since the velocity step) or the
    // entry pbest (staged before the first barrier); `better` is block-uniform, so no
    // barrier waits for wave 0 here
    push_inbox(sw, g, i, q, q < 3 * IB_FIELDS ? lk1 : lk0, q < 3 * IB_FIELDS ? g + 1 : topo, pn,
               better ? sm.fk.th : sm.pbr);
    BLK_TS(g, 5);
    sc.lap(3);
    sc.span(5);
}

template <bool ROW16, bool FILT>
__global__ __launch_bounds__(HPE_NT) void k_pso_gen(DevSwarm sw, const DevObs *__restrict__ og,
                                                    const DevHand *__restrict__ Hg, int g,
                                                    double W1, double C1, double C2,
                                                    InboxCounts kin) {
    pso_gen_body<HPE_NT, false, ROW16, FILT>(sw, og, Hg, g, W1, C1, C2, kin);
}
template <bool ROW16, bool FILT>
__global__ __launch_bounds__(HPE_NT) void k_pso_gen_x(DevSwarm sw, const DevObs *__restrict__ og,
                                                      const DevHand *__restrict__ Hg, int g,
                                                      double W1, double C1, double C2,
                                                      InboxCounts kin) {
    pso_gen_body<HPE_NT, true, ROW16, FILT>(sw, og, Hg, g, W1, C1, C2, kin);
}

// ---------------------------------------------------------------- wave-per-particle form
// For swarms much larger than the CU count (BASELINE configs 4 and 5) one workgroup per
// particle leaves the SIMDs idle during the single-wave FK and reductions; here each wave
// carries one particle end to end (same arithmetic and draws, per-wave syncs only) and
// PW_WPB particles share a workgroup, so the CU interleaves many particles' latency
// chains.  The informant's pbest row is read from the inbox after the choice.
#define PW_WPB 4
#define PW_NT (64 * PW_WPB)

__device__ __forceinline__ void push_lane_links(const DevSwarm &sw, int g, int i, int l, int tt0,
                                                int tt1, Link (&lk)[3]) {
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        const int q = l + 64 * k;
        const int tt = (q < 3 * IB_FIELDS) ? tt0 : tt1;
        lk[k] = load_link(sw, g, i, q, tt);
    }
}

// The wave form's pushes: {tag, cost} as ONE 16-B entry of the compact array ibtc
// [g&1][var][receiver][slot] (the receiver reads its K entries of a variant as one
// contiguous run, 2 lines, instead of the first 16 B of K rows, K lines), the pbest row into
// fields 2..27 of the inbox row (read only for the chosen informant).
__device__ __forceinline__ size_t ibtc_index(const DevSwarm &sw, int par, int var, int r, int slot) {
    return (((size_t)par * 2 + var) * sw.P + r) * sw.K + slot;
}
__device__ __forceinline__ void push_inbox_w(const DevSwarm &sw, int g, int s, int q, const Link &L,
                                             int tt, double pc, const double *row) {
    const int r = L.ok ? (int)(L.raw & 0xffffffff) : -1, slot = (int)(L.raw >> 32);
    if (r < 0) return;
    const int dst = q / IB_FIELDS, fld = q - IB_FIELDS * dst, var = dst < 3 ? 1 : 0;
    if (fld == 0) {
        typedef double d2v __attribute__((ext_vector_type(2)));
        const d2v e = {__longlong_as_double(((long long)g << 48) | ((long long)tt << 32) | s), pc};
        *(d2v *)(sw.ibtc + 2 * ibtc_index(sw, g & 1, var, r, slot)) = e;
    } else if (fld >= 2) {
        sw.inbox[ib_index(sw, g & 1, var, r, slot) + fld] = row[fld - 2];
    }
}

template <int WPP, bool COOP>
__global__ __launch_bounds__(PW_NT) void k_pso_init_w(DevSwarm sw, const double *__restrict__ x0,
                                                      const DevObs *__restrict__ og,
                                                      const DevHand *__restrict__ Hg) {
    const DevObs o = *og;
    __shared__ DevHand hs;
    __shared__ FkSm fks[PW_WPB];
    __shared__ FiltSm fls[PW_WPB];
    __shared__ double xpart[PW_WPB];
    const int t = threadIdx.x, w = t >> 6, l = t & 63, sub = w % WPP;
    const int i = blockIdx.x * (PW_WPB / WPP) + w / WPP, P = sw.P;
    const bool valid = i < P;
    const int ic = valid ? i : P - 1;
    const double hw = hand_word<PW_NT>(Hg);
    const DevHand *__restrict__ H = &hs;
    FkSm &f = fks[w];
    Link lk[3];
    push_lane_links(sw, 0, ic, l, 1, -1, lk);
    const CloudGlobal cv = obs_cloud(o);
    const Pt pre = load_pt1(cv, l + 64 * sub);
    const double *sd = sw.bounds + 2 * HPE_DOF;
    if (sw.ext && blockIdx.x == 0 && t == 0) sw.ext[HPE_DOF] = __builtin_inf();  // no candidate yet
    if (l < HPE_DOF) {  // particles = x0 + randn % std (PSO.cpp:67-72)
        const size_t e = (size_t)ic * HPE_DOF + l;
        const double x = x0[l] + sw.normals[e] * sd[l];
        f.th[l] = x;
        if (valid && sub == 0) {
            sw.xh[e] = x;
            sw.pb[e] = x;
            sw.v[e] = 0.0;
        }
    }
    hand_put<PW_NT>(hs, hw);
    __syncthreads();  // hand staged
    const double c = eval_wave_cost<WPP, COOP, PW_WPB>(fks, fls[w], o, cv, H, pre, sub, xpart);
    if (!valid || sub != 0) return;
    if (l == 0) {
        sw.pch[i] = c;
        gmin_lower(sw, 0, i, c);
    }
#pragma unroll
    for (int k = 0; k < 3; ++k) push_inbox_w(sw, 0, i, l + 64 * k, lk[k], 1, c, f.th);
}

// one (four) waves per particle: four waves per SIMD, so every workgroup of a 4096 (1024) swarm is
// resident (the register count sits at the 128 boundary)
template <bool XCH, bool ROW16, int WPP, bool COOP>
__global__ __launch_bounds__(PW_NT, WPP == 2 ? 2 : 4) void k_pso_gen_w(DevSwarm sw, const DevObs *__restrict__ og,
                                                     const DevHand *__restrict__ Hg, int g,
                                                     double W1, double C1, double C2) {
    // every argument word loaded at entry in one batch (see k_pso_gen)
    int z0 = 0;
    asm("" : "+s"(z0) : "s"(g), "s"(sw.gmin), "s"(sw.sig), "s"(sw.outl), "s"(sw.bounds),
        "s"(sw.xh), "s"(sw.pch), "s"(sw.pb), "s"(sw.v), "s"(sw.inbox), "s"(sw.ibtc),
        "s"(sw.P), "s"(sw.K));
    const DevObs o = *og;
    WAVE_TS2(g, 0);
    __shared__ DevHand hs;
    __shared__ FkSm fks[PW_WPB];
    __shared__ FiltSm fls[PW_WPB];
    __shared__ double xpart[PW_WPB];
    const int t = threadIdx.x + z0, w = t >> 6, l = t & 63, sub = w % WPP;
    const int i = blockIdx.x * (PW_WPB / WPP) + w / WPP, P = sw.P, K = sw.K;
    const bool valid = i < P;
    const int ic = valid ? i : P - 1;
    const double hw = hand_word<PW_NT>(Hg);  // staged into LDS before the block barrier
    const DevHand *__restrict__ H = &hs;
    FkSm &f = fks[w];
    // a helper wave (WPP > 1, cooperative FK): its particle's FK and state are the first
    // wave's, so it only stages its share of the hand, takes part in the FK and searches its
    // share of the cloud (the same barriers as the first wave's path).  At two waves per
    // particle the second wave then pushes the particle's pbest while the first writes it,
    // the push links loaded under the evaluation from the topology the first wave leaves in
    // LDS with the entry pbest row and cost (1,024 p: 11.0 -> 10.7 us per generation)
    constexpr bool hpush = COOP && WPP == 2;
    __shared__ double hrow[hpush ? PW_WPB : 1][HPE_DOF];
    __shared__ double hpc[hpush ? PW_WPB : 1];
    __shared__ int htopo[hpush ? PW_WPB : 1];
    if (COOP && WPP > 1 && __builtin_amdgcn_readfirstlane(sub) != 0) {
        const CloudGlobal cv = obs_cloud(o);
        const Pt pre = load_pt1(cv, l + 64 * sub);
        hand_put<PW_NT>(hs, hw);
        __syncthreads();
        Link lk[3];
        const int w0 = w - sub, tp = hpush ? htopo[hpush ? w0 : 0] : 0;
        if (hpush && sub == 1) push_lane_links(sw, g, ic, l, g + 1, tp, lk);
        const double fx = eval_wave_cost<WPP, COOP, PW_WPB>(fks, fls[w], o, cv, H, pre, sub, xpart, g);
        if constexpr (hpush) {
            if (!valid || sub != 1) return;
            const double pci = hpc[w0];
            const bool better = fx < pci;
            const double pn = better ? fx : pci;
            const double *row = better ? fks[w0].th : hrow[w0];
#pragma unroll
            for (int k = 0; k < 3; ++k) {
                const int q = l + 64 * k;
                push_inbox_w(sw, g, i, q, lk[k], q < 3 * IB_FIELDS ? g + 1 : tp, pn, row);
            }
        }
        return;
    }
    // ---- round 1: every load of the generation, all independent and unconditional (the
    // push links follow once the topology is known)
    const CloudGlobal cv = obs_cloud(o);
    const size_t e = (size_t)ic * HPE_DOF + l;
    const size_t ec = (size_t)ic * HPE_DOF + (l < HPE_DOF ? l : HPE_DOF - 1);
    const double xo = sw.xh[(size_t)(g - 1) * P * HPE_DOF + ec];
    const double vo = sw.v[ec];
    const double pbi = sw.pb[ec];
    const double lbt = sw.bounds[ec - (size_t)ic * HPE_DOF];
    const double ubt = sw.bounds[ec - (size_t)ic * HPE_DOF + HPE_DOF];
    const double pci = sw.pch[(size_t)(g - 1) * P + ic];
    double tg[2], tc[2];
#pragma unroll
    for (int vr = 0; vr < 2; ++vr) {  // {tag, cost} of slot l: one 16-B load, contiguous run
        typedef double d2v __attribute__((ext_vector_type(2)));
        const d2v e = *(const d2v *)(sw.ibtc + 2 * ibtc_index(sw, (g - 1) & 1, vr, ic, l < K ? l : K - 1));
        tg[vr] = e.x;
        tc[vr] = e.y;
    }
    const unsigned long long gcell = gmin_load(sw, g - 1);
    const Sig pv = sw.sig[g > 1 ? g - 1 : 0];
    const double exr = XCH ? sw.ext[l <= HPE_DOF ? l : HPE_DOF] : 0.0;  // exchange (sw.ext)
    // the draws while the loads are in flight
    // one Philox pass for both draws: lanes 0..25 draw rp of dimension l, lanes 26..51 rg of
    // dimension l - 26, which one shuffle brings to lane l - 26
    const int dl = l < HPE_DOF ? l : (l < 2 * HPE_DOF ? l - HPE_DOF : 0);
    const double rd = philox_u01(sw.seed, l < HPE_DOF ? ST_RP : ST_RG, g, ic, dl);
    const double rp = rd;
    const double rg = __shfl(rd, l + HPE_DOF);
    const double fmin = gmin_reduce(gcell);
    // ---- end-of-generation update of g-1 (PSO.cpp:864-877), uniform
    Sig sg;
    if (g == 1) {
        sg.gcost = fmin < 1e100 ? fmin : 1e100;
        sg.count = 100;
        sg.topo = -1;
    } else {
        const bool imp = fmin < pv.gcost;
        sg.gcost = imp ? fmin : pv.gcost;
        sg.count = imp ? 0 : pv.count + 1;
        sg.topo = pv.topo;
    }
    if (sg.count > 0) sg.topo = g;
    if (i == 0 && l == 0 && sub == 0) sw.sig[g] = sg;
    const int topo = sg.topo, var = (topo == g) ? 1 : 0;
    // ---- informant (PSO.cpp:810-812)
    const int self_lane = ROW16 ? 15 : 63;  // one 16-lane row when K <= 15
    double v = __builtin_inf();
    int idx = 0x7fffffff, slot = -1;
    if (l < K) {
        const long long tag = __double_as_longlong(var ? tg[1] : tg[0]);
        if ((tag >> 32) == (((long long)(g - 1) << 16) | topo)) {
            v = var ? tc[1] : tc[0];
            idx = (int)(tag & 0xffffffff);
            slot = l;
        }
    } else if (l == self_lane) {
        v = pci;
        idx = ic;
    }
    if (v != v) v = __builtin_inf();
    int inf, islot;
    double infc = 0.0;
    if (ROW16) row0_argmin_lex(v, idx, slot, inf, islot, XCH ? &infc : nullptr);
    else wave_argmin_lex(v, idx, slot, inf, islot, XCH ? &infc : nullptr);
    const bool use_ext = XCH && readlane_f64(exr, HPE_DOF) < infc;  // strictly better
    WAVE_TS2(g, 1);
    // the lane's first cloud point, used after FK: issued behind round 1's loads, which the
    // informant choice waits for in issue order
    const Pt pre = load_pt1(cv, l + 64 * sub);
    // ---- velocity, position, check_constraints (PSO.cpp:824-842, 358-377)
    if (l < HPE_DOF) {
        double vn;
        if (inf == ic && !use_ext) {
            vn = W1 * vo + (C1 * rp) * (pbi - xo);
        } else {
            const double pbn = use_ext ? exr : sw.inbox[ib_index(sw, (g - 1) & 1, var, ic, islot) + 2 + l];
            vn = (W1 * vo + (C1 * rp) * (pbi - xo)) + (C2 * rg) * (pbn - xo);
        }
        double xn = xo + vn;
        const double xr = xn;
        if (xr < lbt) { xn = lbt; vn = 0.; }
        if (xr > ubt) { xn = lbt; vn = 0.; }  // above max -> MIN (PSO.cpp:372)
        if (valid && sub == 0) {
            sw.v[e] = vn;
            sw.xh[(size_t)g * P * HPE_DOF + e] = xn;
        }
        f.th[l] = xn;
    }
    // the push links, loaded before the evaluation so their round trip hides under it (121 ->
    // 127 VGPRs: still four waves per SIMD)
    Link lk[3];
    if (!hpush) push_lane_links(sw, g, ic, l, g + 1, topo, lk);
    if constexpr (hpush) {  // for the pushing helper
        if (l < HPE_DOF) hrow[w][l] = pbi;
        if (l == 0) {
            hpc[w] = pci;
            htopo[w] = topo;
        }
    }
    hand_put<PW_NT>(hs, hw);
    WAVE_TS2(g, 2);
    __syncthreads();  // hand staged (the only block-wide sync)
    WAVE_TS2(g, 3);
    // ---- evaluation and pbest (PSO.cpp:848-861)
    const double fx = eval_wave_cost<WPP, COOP, PW_WPB>(fks, fls[w], o, cv, H, pre, sub, xpart, g);
    WAVE_TS2(g, 8);
    if (!valid || sub != 0) return;
    const bool better = fx < pci;
    const double pn = better ? fx : pci;
    if (l < HPE_DOF) {
        const double row = better ? f.th[l] : pbi;
        sw.pb[e] = row;
        if (!hpush) f.th[l] = row;
    }
    if (l == 0) {
        sw.pch[(size_t)g * P + i] = pn;
        gmin_lower(sw, g, i, pn);
    }
    if (hpush) return;  // the second wave pushes
    wave_sync();
    WAVE_TS2(g, 9);
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        const int q = l + 64 * k;
        push_inbox_w(sw, g, i, q, lk[k], q < 3 * IB_FIELDS ? g + 1 : topo, pn, f.th);
    }
    WAVE_TS2(g, 10);
}

// The opt-in per-generation exchange (hpe_set_exchange): this subswarm's best after
// generation g -- {pbest row, pbest cost} of the first argmin of the generation's pbest
// costs (NaN as +inf, as the informant choice) -- into sw.ext, which the caller's
// collective then replaces by the best over all subswarms.  One workgroup.
__global__ __launch_bounds__(HPE_NT) void k_swarm_best(DevSwarm sw, int g) {
    __shared__ Smem sm;
    const int t = threadIdx.x, P = sw.P;
    VI mine = {__builtin_inf(), 0};
    for (int k = t; k < P; k += HPE_NT) {
        const double v = nan_inf(sw.pch[(size_t)g * P + k]);
        if (v < mine.v) {
            mine.v = v;
            mine.i = k;
        }
    }
    const VI b = block_argmin(sm, mine);
    if (t < HPE_DOF) sw.ext[t] = sw.pb[(size_t)b.i * HPE_DOF + t];
    if (t == HPE_DOF) sw.ext[HPE_DOF] = sw.pch[(size_t)g * P + b.i];
}

// Multi-GPU subswarms, the per-frame best of N (hpe_pick_best): state <- the
// row of gathered (world x 27: {bestp, cost} per rank) with the smallest cost, in one launch
// on the tracker stream right after the all-gather.  Exactly hpe/dist.py pick_best
// (torch.nan_to_num(cost, nan=inf) then the first argmin): NaN -> +inf, +inf -> the largest
// finite double, -inf -> the lowest; ties go to the lowest rank.  One wave, world <= 64.
// Inside a sequence (hist, cur: the library's own exchange, hpe_subswarm_init) the frame's
// history row gets the picked state too: row *cur - 1 of the row cursor, which the frame's
// final kernel has already advanced.
// The rule as a wave argmin (lane l = rank l; every lane gets the winner): the lexicographic
// minimum of (sanitised cost, rank) -- rows past world carry (+inf, rank >= world), so they
// lose to every real row, an all-NaN world included.
__device__ __forceinline__ int pick_best_row(const double *__restrict__ gathered, int world, int l) {
    double v = (l < world) ? gathered[(size_t)l * (HPE_DOF + 1) + HPE_DOF] : __builtin_inf();
    if (l < world) {
        if (v != v) v = __builtin_inf();
        else if (v == __builtin_inf()) v = 1.7976931348623157e308;
        else if (v == -__builtin_inf()) v = -1.7976931348623157e308;
    }
    int i = l;
#pragma unroll
    for (int m = 1; m < 64; m <<= 1) {
        const double ov = __shfl_xor(v, m);
        const int oi = __shfl_xor(i, m);
        if (ov < v || (ov == v && oi < i)) {
            v = ov;
            i = oi;
        }
    }
    return __builtin_amdgcn_readfirstlane(i);
}
// state <- the picked row; inside a sequence the frame's history row too (row *cur - 1).
__device__ __forceinline__ double pick_apply(const double *__restrict__ gathered, int w, int l,
                                             double *__restrict__ state, double *__restrict__ hist,
                                             const int *__restrict__ cur) {
    const double x = l <= HPE_DOF ? gathered[(size_t)w * (HPE_DOF + 1) + l] : 0.0;
    if (l <= HPE_DOF) state[l] = x;
    if (hist && cur && l <= HPE_DOF) hist[(size_t)(HPE_DOF + 1) * (cur[0] - 1) + l] = x;
    return x;
}
__global__ __launch_bounds__(64) void k_pick_best(const double *__restrict__ gathered, int world,
                                                  double *__restrict__ state,
                                                  double *__restrict__ hist = nullptr,
                                                  const int *__restrict__ cur = nullptr) {
    const int l = threadIdx.x;
    pick_apply(gathered, pick_best_row(gathered, world, l), l, state, hist, cur);
}

// u64 wave helpers of k_pso_final's replay: lane l - 1's value (lane 0: fill), the
// inclusive prefix minimum over lanes 0..l (DPP row_shr 1/2/4/8, row_bcast 15/31; lanes
// without a source keep the identity, all ones), a lane's value in every lane.
template <int CTRL, int ROWMASK = 0xf>
__device__ __forceinline__ unsigned long long dpp_min_src_u64(unsigned long long v) {
    const unsigned lo = (unsigned)__builtin_amdgcn_update_dpp(-1, (int)(unsigned)v, CTRL, ROWMASK, 0xf, false);
    const unsigned hi = (unsigned)__builtin_amdgcn_update_dpp(-1, (int)(unsigned)(v >> 32), CTRL, ROWMASK, 0xf, false);
    return ((unsigned long long)hi << 32) | lo;
}
__device__ __forceinline__ unsigned long long wave_prefix_min_u64(unsigned long long v) {
    v = min(v, dpp_min_src_u64<0x111>(v));        // row_shr:1
    v = min(v, dpp_min_src_u64<0x112>(v));        // row_shr:2
    v = min(v, dpp_min_src_u64<0x114>(v));        // row_shr:4
    v = min(v, dpp_min_src_u64<0x118>(v));        // row_shr:8
    v = min(v, dpp_min_src_u64<0x142, 0xa>(v));   // row_bcast:15
    v = min(v, dpp_min_src_u64<0x143, 0xc>(v));   // row_bcast:31
    return v;
}
__device__ __forceinline__ unsigned long long from_left_u64(unsigned long long v, unsigned long long fill) {
    const unsigned lo = (unsigned)__builtin_amdgcn_update_dpp((int)(unsigned)fill, (int)(unsigned)v, 0x138, 0xf, 0xf, false);
    const unsigned hi = (unsigned)__builtin_amdgcn_update_dpp((int)(unsigned)(fill >> 32), (int)(unsigned)(v >> 32), 0x138, 0xf, 0xf, false);
    return ((unsigned long long)hi << 32) | lo;  // wave_shr:1
}
__device__ __forceinline__ unsigned long long readlane_u64(unsigned long long v, int lane) {
    const unsigned lo = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)v, lane);
    const unsigned hi = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)(v >> 32), lane);
    return ((unsigned long long)hi << 32) | lo;
}

// Last end-of-generation update and bestp = gbest_pos (PSO.cpp:864-882).  Replays the
// gbest / count sequence from gmin[], finds the last improving generation g* and takes
// particles.col(first argmin pcost) of that generation; resets gmin[] for the next call.
// TAIL (a tracked frame, testmodel.cpp:130-132): out[26] = cal_cost(bestp), and the
// frame descriptor used is copied to obs_out (the API's "selected frame").  When some
// generation improved, bestp = particles.col(argmin pcost) of the last improving
// generation g*, and that particle's pbest cost was set AT g* (an older value could not
// undercut the previous gbest), i.e. it IS cal_cost(bestp) computed by the same
// eval_block on the same theta: the gbest cost is kept, bit for bit (same_eval: the
// generations used the workgroup form).  Otherwise (nothing beat 1e100, bestp = zeros)
// the block evaluates it.
template <bool TAIL = false, bool FILT = false>
__global__ __launch_bounds__(HPE_NT) void k_pso_final(DevSwarm sw, double *__restrict__ out,
                                                      const DevObs *og = nullptr,
                                                      const DevHand *__restrict__ Hg = nullptr,
                                                      DevObs *__restrict__ obs_out = nullptr,
                                                      int same_eval = 0,
                                                      unsigned long long *__restrict__ seq_dev = nullptr,
                                                      unsigned long long *done_host = nullptr,
                                                      double *__restrict__ hist = nullptr,
                                                      const int *__restrict__ fail = nullptr,
                                                      const DevObs *__restrict__ seq_table = nullptr,
                                                      DevObs *seq_obs = nullptr,  // aliases og
                                                      int *__restrict__ seq_cur = nullptr) {
    constexpr int CH = 2048;  // generations staged per pass
    // offline sequences (hpe_track_sequence_dev): the frame's history row and slot come
    // from the device cursor {slot, row}, and the next frame's descriptor is staged into the
    // descriptor every kernel of the chunk graph reads -- the graph is independent of the
    // slot range it tracks
    int seq_slot = 0;
    if (TAIL && seq_cur) {
        seq_slot = seq_cur[0];
        if (hist) hist += (size_t)(HPE_DOF + 1) * seq_cur[1];
    }
    // a timed-out multi-workgroup refine (DevMw::err, set until the host has reported it):
    // this frame's result is undefined, so bestp and cost become NaN
    const int failed = __builtin_amdgcn_readfirstlane(
        (TAIL && fail) ? __hip_atomic_load(fail, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0);
    __shared__ Smem sm;
    __shared__ double gm[CH];
    __shared__ int tp[CH];
    const int t = threadIdx.x, G = sw.G, P = sw.P;
    if (TAIL && seq_dev && t == HPE_NT - 64) {
        // pipelined tracking: this frame's refine launch (and the preparation of the next
        // frame inside it, which read a pinned host buffer) has completed; publish the
        // frame's sequence number to the host, which polls it before reusing that buffer.
        // Relaxed: the kernel boundary already retired those reads, and no store of this
        // kernel needs publishing with it.  Wave 7, idle until the first barrier, takes the
        // counter's load round trip instead of wave 0, which reads the gmin history.
        const unsigned long long n = *seq_dev + 1;
        *seq_dev = n;
        __hip_atomic_store(done_host, n, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
    if (TAIL) stage_hand<HPE_NT>(sm.hand, Hg);
    // this frame's descriptor, read before the tail stages the next frame's into it (og IS
    // seq_obs in sequence mode).  (A round-5 form staged the next descriptor after
    // the tail's own evaluation, behind a barrier, and returned early before it on `failed`
    // (a per-lane atomic load) and `same_eval && last >= 0` (`last` read from LDS): exits the
    // compiler could not prove uniform, ahead of barriers -- undefined behaviour in the HIP
    // barrier model, not a proven compiler bug.  On the box its same-eval frames came out
    // with a re-evaluated cost (3.3e-7 relative off).  The cause was not isolated further;
    // every such exit is now made provably uniform (readfirstlane).)
    DevObs o_early{};
    if (TAIL) o_early = *og;
    // the frame descriptor handed back at the end, loaded now (off the final chain)
    const unsigned long long obs_word =
        (TAIL && obs_out && t < (int)(sizeof(DevObs) / 8)) ? ((const unsigned long long *)og)[t] : 0ull;
    double bp = 0.0;  // gbest_pos = zeros<vec> (PSO.cpp:739) if nothing beat 1e100
    double gcost = 1e100;
    int last = -1, count = 100;
    if (G <= 63) {
        // G + 1 <= 64 generations: the replay as scans over wave 0's lanes (lane k =
        // generation k), not a serial loop.  Costs are >= 0 or NaN, so their u64 bits
        // order like their values and NaN bits (never written, or all NaN) sort above
        // every cost: a u64 minimum is fmin, and "fm < gcost" is a u64 compare.
        if (t < 64) {
            unsigned long long key = ~0ull;
            if (t <= G) {
                double m = __builtin_nan("");
                for (int c = 0; c < GMIN_SHARDS; ++c) m = fmin(m, bits_to_f64(*gmin_cell(sw, t, c)));
                key = f64_to_bits(m);
            }
            const int topo = (t >= 1 && t <= G) ? sw.sig[t].topo : -1;
            const unsigned long long cap = f64_to_bits(1e100);  // gbest starts at 1e100
            const unsigned long long incl = wave_prefix_min_u64(key);
            const unsigned long long excl = min(from_left_u64(incl, ~0ull), cap);
            const bool imp = t >= 1 && t <= G && key < excl;  // PSO.cpp:864-872
            const unsigned long long mask = __ballot(imp);
            const int last0 = (readlane_u64(key, 0) < cap) ? 0 : -1;  // generation 0 (:755-760)
            last = mask ? 63 - __builtin_clzll(mask) : last0;
            if (t >= 1 && t <= G && sw.trace_g) {
                // count after generation t: 0 at an improvement, +1 otherwise, from 100
                const unsigned long long upto = mask & ((2ull << t) - 1);
                const int L = upto ? 63 - __builtin_clzll(upto) : 0;
                sw.trace_g[t - 1] = bits_to_f64(min(incl, cap));
                sw.trace_count[t - 1] = L >= 1 ? t - L : 100 + t;
                sw.trace_topo[t - 1] = topo;
            }
            if (t == 0) {
                sm.iscal[2] = last;
                sm.dscal[5] = bits_to_f64(min(readlane_u64(incl, G), cap));
            }
        }
    }
    for (int base = 0; G > 63 && base <= G; base += CH) {
        // all loads of the pass at once, then a serial replay from LDS by thread 0
        for (int k = t; k < CH && base + k <= G; k += HPE_NT) {
            double m = __builtin_nan("");  // all-ones (never written) is a NaN too
            for (int c = 0; c < GMIN_SHARDS; ++c)
                m = fmin(m, bits_to_f64(*gmin_cell(sw, base + k, c)));
            gm[k] = m;
            tp[k] = (base + k >= 1) ? sw.sig[base + k].topo : -1;
        }
        __syncthreads();
        if (t == 0) {
            const int n = (G - base + 1) < CH ? (G - base + 1) : CH;
            for (int k = 0; k < n; ++k) {
                const int g = base + k;
                const double fm = gm[k];
                if (g == 0) {
                    if (fm < gcost) {
                        gcost = fm;
                        last = 0;
                    }
                    continue;
                }
                if (fm < gcost) {
                    gcost = fm;
                    count = 0;
                    last = g;
                } else {
                    count += 1;
                }
                if (sw.trace_g) {
                    sw.trace_g[g - 1] = gcost;
                    sw.trace_count[g - 1] = count;
                    sw.trace_topo[g - 1] = tp[k];
                }
            }
        }
        __syncthreads();
    }
    if (G > 63 && t == 0) {
        sm.iscal[2] = last;
        sm.dscal[5] = gcost;
    }
    __syncthreads();
    last = __builtin_amdgcn_readfirstlane(sm.iscal[2]);  // decides the exit below (§7)
    gcost = sm.dscal[5];
    if (last >= 0 && P <= HPE_NT) {
        // one particle per thread: its pbest cost and its position row of generation
        // `last` in one round trip; the winner's thread writes bestp
        const int k = t < P ? t : P - 1;
        const double *row = sw.xh + ((size_t)last * P + k) * HPE_DOF;
        double r[HPE_DOF];
#pragma unroll
        for (int d = 0; d < HPE_DOF; ++d) r[d] = row[d];
        VI mine = {t < P ? nan_inf(sw.pch[(size_t)last * P + k]) : __builtin_inf(), t < P ? t : 0};
        const VI b = block_argmin(sm, mine);
        if (t == b.i) {
#pragma unroll
            for (int d = 0; d < HPE_DOF; ++d) {
                out[d] = r[d];
                sw.gpos[d] = r[d];
                if (hist) hist[d] = r[d];
            }
        }
        if (TAIL && !same_eval) {  // the tail below evaluates cal_cost(bestp)
            if (t == b.i) {
#pragma unroll
                for (int d = 0; d < HPE_DOF; ++d) sm.pbr[d] = r[d];
            }
            __syncthreads();
            if (t < HPE_DOF) bp = sm.pbr[t];
        }
    } else {
        if (last >= 0) {
            const double *pc = sw.pch + (size_t)last * P;
            VI mine = {__builtin_inf(), 0};
            for (int k = t; k < P; k += HPE_NT) {
                const double v = nan_inf(pc[k]);
                if (v < mine.v) {
                    mine.v = v;
                    mine.i = k;
                }
            }
            const VI b = block_argmin(sm, mine);
            if (t < HPE_DOF) bp = sw.xh[((size_t)last * P + b.i) * HPE_DOF + t];
        }
        // bestp stays in each thread's register: no barrier and no re-read of `out`
        if (t < HPE_DOF) {
            out[t] = bp;
            sw.gpos[t] = bp;
            if (hist) hist[t] = bp;
        }
    }
    if (t == 0) {
        out[HPE_DOF] = gcost;
        if (hist) hist[HPE_DOF] = gcost;
    }
    for (int c = t; c < (G + 1) * GMIN_SHARDS; c += HPE_NT) sw.gmin[(size_t)c * GMIN_STRIDE] = ~0ull;
    if (TAIL) {
        if (obs_out && t < (int)(sizeof(DevObs) / 8)) ((unsigned long long *)obs_out)[t] = obs_word;
        if (seq_cur) {
            const int nx = seq_slot + 1 < HPE_MAX_SLOTS ? seq_slot + 1 : seq_slot;
            if (seq_table && t < (int)(sizeof(DevObs) / 8))
                ((unsigned long long *)seq_obs)[t] = ((const unsigned long long *)(seq_table + nx))[t];
            if (t == 0) {
                seq_cur[0] = seq_slot + 1;
                seq_cur[1] = seq_cur[1] + 1;
            }
        }
        if (failed) {
            if (t <= HPE_DOF) {
                out[t] = __builtin_nan("");
                if (hist) hist[t] = __builtin_nan("");
            }
            return;
        }
        if (same_eval && last >= 0) return;  // out[26] = gcost = cal_cost(bestp)
        const DevObs o = o_early;
        if (t < HPE_DOF) sm.fk.th[t] = bp;
        const CloudGlobal cv = obs_cloud(o);
        const Pt pre = load_pt(cv, t);
        __syncthreads();
        const double c = eval_block<EV_COST, HPE_NT, true, FILT>(sm, o, cv, &sm.hand, nullptr, pre);
        if (t == 0) {
            out[HPE_DOF] = c;
            if (hist) hist[HPE_DOF] = c;
        }
    }
}

// Start of an offline sequence (hpe_track_sequence_dev): the first frame's descriptor into
// the chunk graphs' descriptor, the cursor to {first slot, history row 0}.
__global__ void k_seq_begin(const DevObs *__restrict__ table, int first, DevObs *__restrict__ cur_obs,
                            int *__restrict__ cur) {
    const int t = threadIdx.x;
    if (t < (int)(sizeof(DevObs) / 8))
        ((unsigned long long *)cur_obs)[t] = ((const unsigned long long *)(table + first))[t];
    if (t == 0) {
        cur[0] = first;
        cur[1] = 0;
    }
}

// ------------------------------------------------------------------ refine
// refine_init_pose (PSO.cpp:216-266) with cal_grad (:183-214) and goldstein (:438-480)
// as ONE persistent workgroup of RF_NT threads.  Each iteration:
//   * f_k = cal_cost2(x0, matchId, true): FK by wave 0, search by all RF_NT threads;
//   * the 6 central differences run concurrently, one wave each (frozen matchId);
//   * the Goldstein bracket search is evaluated SPECULATIVELY: each wave evaluates one node
//     of a small tree of the search's next decisions (gold_tree, shapes below), then every
//     thread walks the tree with the serial algorithm's exact rules.  Identical arithmetic
//     on identical alphas: the result, the step tk and the evaluation count equal the
//     serial ones.
// Control flow is uniform: every thread evaluates the same scalar decisions from LDS.
#ifndef RF_NT
#define RF_NT 512
#endif
#define RF_NW (RF_NT / 64)
static_assert(RF_NW >= 8, "the speculation shapes use up to 8 waves");
#define RF_STAGE_MAX 2048  // clouds up to this size are staged in LDS with their matchId

struct __align__(16) RefineSm {
    FkSm w[RF_NW];
    FkSm base;  // spheres of the current x0
    double red[16][4];
    double x0[32];
    double f[RF_NW];
    double fg[RF_NW];  // the gradient points' costs (k_refine, single-workgroup form)
    FkX X;  // rotation-only joint terms of x0 (refine block 2: translation steps)
    RigidSm rg;  // hand-frame centres, block 2's rotated centres, collision (rigid refine)
    unsigned ts_n;  // diagnostic build: refine timeline entries written
};

// Goldstein bracket update (PSO.cpp:459-474), shared by the speculating waves and the walk.
__device__ __forceinline__ void gold_up(double &a, double b, double &alpha) {
    a = alpha;
    const double up = 2 * alpha, mid = 0.5 * (alpha + b);
    alpha = (mid < up) ? mid : up;  // std::min(t*alpha, 0.5*(alpha+b))
}
__device__ __forceinline__ void gold_down(double a, double &b, double &alpha) {
    b = alpha;
    alpha = 0.5 * (a + alpha);
}

// The hand-frame form's correspondence search takes one item on every wave (round 4: the
// chain form's spread balanced the SIMDs against the gradient heads' DH chains).
#ifndef HPE_RF_SPREAD
#define HPE_RF_SPREAD 1
#endif

// ---------------------------------------------------------------- multi-workgroup refine
// For clouds larger than RF_STAGE_MAX one CU is throughput-bound (every Goldstein round is
// seven frozen alignments of the whole cloud), so the refine launch adds Q helper
// workgroups.  Workgroup 0 keeps the whole serial algorithm; each batch of evaluations
// (the correspondence eval of x0, the gradient pairs, a Goldstein round) is published as
// a job.  Helper h owns cloud slice h (and its matchId, written by the correspondence
// job and read back by the same workgroup), computes the nodes' FK itself and returns one
// partial alignment sum per node.  Workgroup 0 computes depth + collision meanwhile and
// sums the partials in helper order (deterministic).  Hand-off per the G16 recipe:
// stores drained, barrier, agent release, counter; one-lane agent acquire, barrier.
// Every wait is bounded (~2 s): on a timeout the launch ends early with *err set.
#define MW_SPIN_MAX (1 << 21)
static_assert(MW_MAX_Q % MW_DONE_SHARDS == 0, "helpers split evenly over the shards");

__device__ __forceinline__ bool mw_wait_geq(unsigned *p, unsigned v, int spin) {
    for (int i = 0; i < spin; ++i) {
        if (__hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >= v) {
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
            return true;
        }
        __builtin_amdgcn_s_sleep(2);
    }
    return false;
}

// A hand-off timed out: flag it on the device (hpe_sync) and in pinned host memory (the
// next tracking call), both plain stores of 1.
__device__ __forceinline__ void mw_fail(const DevMw &mw) {
    __hip_atomic_store(mw.err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (mw.err_host) __hip_atomic_store(mw.err_host, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

struct MwLeader {
    DevMw mw;
    unsigned k;   // jobs published so far
    bool failed;  // a wait timed out: stop issuing work
};

// Workgroup 0: publish the next job (CORR: theta = rs.x0; FROZEN: rs.w[0..nn).th).
__device__ void mw_publish(MwLeader &ml, RefineSm &rs, int type, int nn) {
    const int t = threadIdx.x, w = t >> 6, l = t & 63;
    if (type == MW_JOB_CORR) {
        if (t < HPE_DOF) ml.mw.job->th[0][t] = rs.x0[t];
    } else if (type == MW_JOB_FROZEN) {
        if (w < nn && l < HPE_DOF) ml.mw.job->th[w][l] = rs.w[w].th[l];
    }
    if (t == 0) {
        ml.mw.job->type = type;
        ml.mw.job->nnodes = nn;
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    ml.k += 1;
    if (t == 0) {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
        __hip_atomic_store(&ml.mw.ctr[0], ml.k, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
}

// Workgroup 0: wait until every helper has returned job ml.k (each completion shard has
// counted Q / MW_DONE_SHARDS helpers per job).
__device__ void mw_collect(MwLeader &ml, int *flag) {
    if (threadIdx.x == 0) {
        bool ok = !ml.failed;
        const unsigned want = ml.k * (unsigned)(ml.mw.Q / MW_DONE_SHARDS);
        for (int s = 0; s < MW_DONE_SHARDS && ok; ++s)
            ok = mw_wait_geq(&ml.mw.ctr[32 * (1 + s)], want, ml.mw.spin);
        if (!ok) mw_fail(ml.mw);
        *flag = ok ? 1 : 0;
    }
    __syncthreads();
    if (!__builtin_amdgcn_readfirstlane(*flag)) ml.failed = true;  // decides exits (§7)
}

// Node w's alignment sum: the Q partials folded by one wave in a fixed order.
__device__ __forceinline__ double mw_sum(const MwLeader &ml, int w) {
    const int l = threadIdx.x & 63;
    const double v = (l < ml.mw.Q) ? ml.mw.part[l * MW_MAX_NODES + w] : 0.0;
    return wave_sum(v);
}

// rs.f[w] = cal_cost2(rs.w[w].th, matchId, false) for w < nn; each wave has written its
// own rs.w[w].th.  Ends with a workgroup barrier.
// RIGID: the nodes' spheres by rigid_wave (rblk 0: rotation block, 1: translation block),
// the collision the constant rs.rg.C.
template <bool MW, bool RIGID = false, class CV>
__device__ __forceinline__ void eval_nodes(RefineSm &rs, int nn, const DevObs &o, const CV &cv,
                                           const DevHand *__restrict__ H,
                                           const int32_t *__restrict__ match, FkX *Xt,
                                           MwLeader *ml, int *flag, const double *thr = nullptr,
                                           const FrozenPts *fp = nullptr, int rblk = 0,
                                           const double *md2p = nullptr) {
    const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
    if (!MW) {
        if (w < nn) {
            wave_sync();
            double f;
            if (RIGID) {
                const FrozenHead hd = rblk ? rigid_head<RG_TRANS>(rs.w[w], o, H, rs.rg, *thr)
                                           : rigid_head<RG_ROT>(rs.w[w], o, H, rs.rg, *thr);
                f = frozen_tail<true>(rs.w[w], o, cv, H, match, hd, fp, md2p) + rs.rg.C;
            } else {
                f = eval_wave_frozen<true>(rs.w[w], o, cv, H, match, Xt, thr, fp);
            }
            if (l == 0) rs.f[w] = f;
        }
        REF_TS(rs.ts_n, 9);  // wave 0's node done
        __syncthreads();
        REF_TS(rs.ts_n, 8);  // every node done
        return;
    }
    mw_publish(*ml, rs, MW_JOB_FROZEN, nn);
    double dep = 0.0, co = 0.0;
    if (w < nn) {  // depth + collision here while the helpers align
        if (RIGID) {
            const double thl = rs.w[w].th[l < HPE_DOF ? l : 0];
            if (rblk) rigid_wave<RG_TRANS>(rs.w[w], rs.rg, thl);
            else rigid_wave<RG_ROT>(rs.w[w], rs.rg, thl);
            dep = (l < HPE_NS) ? depth_term(rs.w[w], l, o, H) : 0.0;
            dep = wave_sum(dep);
        } else {
            if (Xt) fk_wave_t<FK_TRANSLATE>(rs.w[w], H, Xt);
            else fk_wave(rs.w[w], H);
            dep = (l < HPE_NS) ? depth_term(rs.w[w], l, o, H) : 0.0;
            co = collide_term(rs.w[w], l, H) + collide_term(rs.w[w], l + 64, H) +
                 ((l < 16) ? collide_term(rs.w[w], l + 128, H) : 0.0);
            wave_sum2(dep, co);
        }
    }
    mw_collect(*ml, flag);
    if (w < nn) {
        const double al = mw_sum(*ml, w);
        const double f = RIGID ? (al * o.lambda + dep) + rs.rg.C : (al * o.lambda + dep) + co;
        const double fr = ml->failed ? __builtin_nan("") : f;
        if (l == 0) rs.f[w] = fr;
    }
    __syncthreads();
}

// f_k = cal_cost2(x0, matchId, true) with the spheres of x0 in rs.base.
template <bool MW, bool RIGID = false, class CV>
__device__ __forceinline__ double eval_corr(RefineSm &rs, const DevObs &o, const CV &cv,
                                            const DevHand *__restrict__ H, int32_t *__restrict__ match,
                                            MwLeader *ml, int *flag) {
    const int t = threadIdx.x;
    if (MW) mw_publish(*ml, rs, MW_JOB_CORR, 1);
    const DepthG dg = depth_issue_w0(rs.base, o, H);
    const bool young = (t >> 6) >= HPE_SETPRIO_FROM;  // as in eval_block
    if (young) __builtin_amdgcn_s_setprio(1);
    double al = MW ? 0.0 : search_align<RF_NT, true>(rs.base, cv, H, match, load_pt(cv, t));
    if (young) __builtin_amdgcn_s_setprio(0);
    double co = (!RIGID && t < 144) ? collide_term(rs.base, t, H) : 0.0;
    double dep = depth_finish(dg, o, t < HPE_NS);
    block_sum3<RF_NT>(rs.red, al, dep, co);  // also publishes matchId to the block
    if (MW) {
        mw_collect(*ml, flag);
        al = mw_sum(*ml, 0);
        if (ml->failed) return __builtin_nan("");
    }
    if (RIGID) return (al * o.lambda + dep) + rs.rg.C;
    return (al * o.lambda + dep) + co;
}

// Helper workgroup h of a multi-workgroup refine launch: serve jobs until EXIT.
template <bool RIGID>
__device__ void mw_helper(const DevMw &mw, int h, const DevObs *__restrict__ og,
                          const DevHand *__restrict__ Hg, int32_t *__restrict__ match_g) {
    __shared__ FkSm nodes[MW_MAX_NODES];
    __shared__ RigidSm hq;  // RIGID: hand-frame centres, built from the first job's digits
    bool have_q = false;
    __shared__ DevHand hs;
    __shared__ double red[16][4];
    __shared__ int sh[2];
    const DevObs o = *og;
    const int t = threadIdx.x, w = t >> 6, l = t & 63;
    stage_hand<RF_NT>(hs, Hg);
    const DevHand *__restrict__ H = &hs;
    const int Q = mw.Q, per = (o.n + Q - 1) / Q;
    const int s0 = min(h * per, o.n), s1 = min(s0 + per, o.n);
    const CloudGlobal cs{gp(o.cx) + s0, gp(o.cy) + s0, gp(o.cz) + s0, s1 - s0};
    int32_t *ms = match_g + s0;
    __syncthreads();
    for (unsigned k = 1;; ++k) {
        if (t == 0) {
            int type = -1, nn = 0;
            if (mw_wait_geq(&mw.ctr[0], k, mw.spin)) {
                type = mw.job->type;
                nn = mw.job->nnodes;
            } else {
                mw_fail(mw);
            }
            sh[0] = type;
            sh[1] = nn;
        }
        __syncthreads();
        // uniform to the compiler: they decide the exit and the barriers below (§7)
        const int type = __builtin_amdgcn_readfirstlane(sh[0]), nn = __builtin_amdgcn_readfirstlane(sh[1]);
        if (type != MW_JOB_CORR && type != MW_JOB_FROZEN) {
            // the last helper out resets the counters for the next launch
            if (type == MW_JOB_EXIT && t == 0 &&
                atomicAdd(&mw.ctr[32 * (1 + MW_DONE_SHARDS)], 1u) == (unsigned)Q - 1) {
                for (int c = 0; c < MW_CTR_WORDS; c += 32) mw.ctr[c] = 0u;
            }
            return;
        }
        if (type == MW_JOB_CORR) {  // search + alignment over the slice, matchId stored
            const double th0 = mw.job->th[0][t < HPE_DOF ? t : 0];
            if (RIGID && !have_q) {  // the digits are fixed for the whole refine launch
                if (t < HPE_DOF) nodes[0].th[t] = (t == 0) ? -180.0 : (t < 6) ? 0.0 : th0;
                __syncthreads();
                if (w == 0) {
                    SphXYZ own;
                    fk_wave(nodes[0], H, &own);
                    if (l < HPE_NS) {
                        hq.q[l][0] = own.x;
                        hq.q[l][1] = own.y * -1;
                        hq.q[l][2] = own.z * -1;
                    }
                }
                have_q = true;
                __syncthreads();
            }
            if (t < HPE_DOF) nodes[0].th[t] = th0;
            __syncthreads();
            if (w == 0) {
                if (RIGID) rigid_wave<RG_ROT>(nodes[0], hq, th0);
                else fk_wave(nodes[0], H);
            }
            __syncthreads();
            double al = search_align<RF_NT, true>(nodes[0], cs, H, ms, load_pt(cs, t));
            double z1 = 0.0, z2 = 0.0;
            block_sum3<RF_NT>(red, al, z1, z2);
            if (t == 0) mw.part[h * MW_MAX_NODES] = al;
        } else if (w < nn) {  // one node per wave, frozen matchId of the slice
            const double thl = mw.job->th[w][l < HPE_DOF ? l : 0];
            if (l < HPE_DOF) nodes[w].th[l] = thl;
            wave_sync();
            if (RIGID) rigid_wave<RG_ROT>(nodes[w], hq, thl);  // (Rg q) + u == P + u
            else fk_wave(nodes[w], H);
            const double al = wave_sum(align_frozen(nodes[w], cs, H, ms, l, 64));
            if (l == 0) mw.part[h * MW_MAX_NODES + w] = al;
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        if (t == 0) {
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
            atomicAdd(&mw.ctr[32 * (1 + h % MW_DONE_SHARDS)], 1u);
        }
    }
}

// Speculation shapes of the Goldstein search.  A round evaluates the nodes of a small
// tree of decision prefixes, relative to the bracket state (a, b, alpha) at the round's
// start: node j lies len decisions below it, decision k = bit k of bits (1 = "up": Armijo
// holds but Goldstein fails, PSO.cpp:461-466; 0 = "down": Armijo fails, :468-471), packed
// as byte j of nb = len << 5 | bits; nibble j of dn / up is node j's child (15: outside the
// shape, the round ends there).  Node 0 is the current alpha.  The shape depends on the
// previous round's last decision (context 0 = a search's first round, 1 = "down", 2 =
// "up"): the decision logs of the bench sequence (the oracle's refine over three 40-frame
// trajectories) are mostly runs -- "DDDDA" alone is ~27 % of the searches -- so deep runs
// are speculated where they are likely.  Rounds over those 1,297 searches: balanced depth 3
// (7 nodes, rounds 1-2) 3,807; the 8-node shapes 3,175; the 7-node shapes 3,361; the 4-node
// shapes 4,553 (one node per SIMD).  The tables are compile-time constants selected by the
// context (no memory read on the walk).  Identical arithmetic on identical alphas in every
// shape: the walk replays the serial rules, so the result, tk and the evaluation count
// equal the serial ones.
struct GoldShape {
    int n;
    unsigned long long nb;
    unsigned dn, up;
};
#define GOLD_BALANCED 0
#define GOLD_8 1
#define GOLD_4 2
#define GOLD_OPT8 3  // pso_optimise's descent (tools/gold_shapes.py optimise)
#define GOLD_MIX 4   // GOLD_8 after a search's start and a "down", GOLD_4 after an "up"
#ifndef HPE_GOLD_POLICY
#define HPE_GOLD_POLICY GOLD_MIX  // refine_init_pose
#endif
template <int POL>
__device__ __forceinline__ GoldShape gold_shape(int ctx) {
    constexpr GoldShape T[15] = {
    // GOLD_BALANCED
    {7, 0x0043414240212000ull, 0xfffff531u, 0xfffff642u},  // first: '' 'D' 'U' 'DD' 'DU' 'UD' 'UU'
    {7, 0x0043414240212000ull, 0xfffff531u, 0xfffff642u},  // D: '' 'D' 'U' 'DD' 'DU' 'UD' 'UU'
    {7, 0x0043414240212000ull, 0xfffff531u, 0xfffff642u},  // U: '' 'D' 'U' 'DD' 'DU' 'UD' 'UU'
    // GOLD_8
    {8, 0xa080604340212000ull, 0xf76f5f31u, 0xfffff4f2u},  // first: '' 'D' 'U' 'DD' 'UU' 'DDD' 'DDDD' 'DDDDD'
    {8, 0x6043414240212000ull, 0xffff7531u, 0xfffff642u},  // D: '' 'D' 'U' 'DD' 'DU' 'UD' 'UU' 'DDD'
    {8, 0x6243414240212000ull, 0xfff7f531u, 0xfffff642u},  // U: '' 'D' 'U' 'DD' 'DU' 'UD' 'UU' 'DUD'
    // GOLD_4
    {4, 0x0000000043212000ull, 0xfffffff1u, 0xfffff3f2u},  // first: '' 'D' 'U' 'UU'
    {4, 0x0000000060402000ull, 0xfffff321u, 0xffffffffu},  // D: '' 'D' 'DD' 'DDD'
    {4, 0x0000000040212000ull, 0xffffff31u, 0xfffffff2u},  // U: '' 'D' 'U' 'DD'
    // GOLD_OPT8
    {8, 0xbf8f674340212000ull, 0xffffff31u, 0xf765f4f2u},  // first: '' 'D' 'U' 'DD' 'UU' 'UUU' 'UUUU' 'UUUUU'
    {8, 0x6043414240212000ull, 0xffff7531u, 0xfffff642u},  // D: '' 'D' 'U' 'DD' 'DU' 'UD' 'UU' 'DDD'
    {8, 0x6743414240212000ull, 0xfffff531u, 0xf7fff642u},  // U: '' 'D' 'U' 'DD' 'DU' 'UD' 'UU' 'UUU'
    // GOLD_MIX (4 nodes, one wave per SIMD, run a round in ~0.71 of an 8-node one)
    {8, 0xa080604340212000ull, 0xf76f5f31u, 0xfffff4f2u},  // first: '' 'D' 'U' 'DD' 'UU' 'DDD' 'DDDD' 'DDDDD'
    {8, 0x6043414240212000ull, 0xffff7531u, 0xfffff642u},  // D: '' 'D' 'U' 'DD' 'DU' 'UD' 'UU' 'DDD'
    {4, 0x0000000040212000ull, 0xffffff31u, 0xfffffff2u},  // U: '' 'D' 'U' 'DD'
    };
    return ctx == 0 ? T[3 * POL] : ctx == 1 ? T[3 * POL + 1] : T[3 * POL + 2];
}

// goldstein(x, g, matchId, f_k, optfunc, tk, 30) (PSO.cpp:438-480) along p from rs.x0
// with frozen correspondences, speculated per round with shape policy POL (above): wave w
// evaluates node w, then every thread walks the nodes with the serial algorithm's rules.
// pl: component (threadIdx.x & 63) of the direction p, in every thread.  Returns tk (0
// after 30 rejected trials); the accepted node's spheres are copied into rs.base and its
// cost to *f_acc.  UPD: the search also applies x0 = x0 - tk * g (PSO.cpp:256; gl =
// component threadIdx.x of g) before its last barrier.  evals grows by the serial count.
template <bool MW = false, int POL = GOLD_BALANCED, bool UPD = false, bool RIGID = false, class CV>
__device__ __forceinline__ double gold_tree(RefineSm &rs, const DevObs &o, const CV &cv,
                                            const DevHand *__restrict__ H,
                                            const int32_t *__restrict__ match, double fk,
                                            double gp, double pl, double gl, int &evals,
                                            double *f_acc, FkX *Xt = nullptr,
                                            MwLeader *ml = nullptr, int *flag = nullptr,
                                            const FrozenPts *fp = nullptr, int rblk = 0,
                                            const double *md2p = nullptr) {
    const int t = threadIdx.x, w = t >> 6, l = t & 63;
    StampClock sc;
    sc.start();
    double A = 0, B = 1e100, alpha = 0.5, tk = 0;
    int it = 0, accepted = -1, ctx = 0;
    bool done = false;
    [[maybe_unused]] unsigned long long path = 0;  // diagnostic build: decision bits (1 = up)
    while (!done) {
        const GoldShape sh = gold_shape<POL>(ctx);
        const int nn = sh.n;
        double thl = 0.0;  // theta[l] of this wave's node (FK's trig reads it in a register)
        if (w < nn) {
            const int nbw = (int)((sh.nb >> (8 * w)) & 0xff), len = nbw >> 5, bits = nbw & 31;
            double ga = A, gb = B, gal = alpha;
            for (int k = 0; k < len; ++k) {
                if ((bits >> k) & 1) gold_up(ga, gb, gal);
                else gold_down(ga, gb, gal);
            }
            thl = rs.x0[l < HPE_DOF ? l : 0] + gal * pl;
            if (l < HPE_DOF) rs.w[w].th[l] = thl;
        }
        eval_nodes<MW, RIGID>(rs, nn, o, cv, H, match, Xt, ml, flag, &thl, fp, rblk, md2p);
        if (MW && ml->failed) break;  // the launch is ending early (DevMw::err)
        // the serial rules walked level by level on the nodes' costs
        int node = 0;
        accepted = -1;
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
                    ctx = 2;
                }
            } else {
                gold_down(A, B, alpha);
                node = (int)((sh.dn >> (4 * node)) & 15u);
                ctx = 1;
            }
        }
        if (!done && it >= 30) done = true;  // tk stays 0
        // the round's outcome decides the next round's barriers: provably uniform (every lane
        // walked the same LDS costs)
        done = __builtin_amdgcn_readfirstlane(done ? 1 : 0) != 0;
        ctx = __builtin_amdgcn_readfirstlane(ctx);
        // x0 is read only before eval_nodes' barrier in a round
        if (UPD && done && t < HPE_DOF) rs.x0[t] = rs.x0[t] - tk * gl;
        if (done && accepted >= 0) {  // keep the accepted node's spheres for the next f_k
            for (int q = t; q < (int)(offsetof(FkSm, J) / 8); q += RF_NT)
                ((double *)&rs.base)[q] = ((const double *)&rs.w[accepted])[q];
            if (f_acc) *f_acc = rs.f[accepted];
        }
        __syncthreads();
        REF_TS(rs.ts_n, 4);
        sc.lap(19);  // one speculated round
    }
    evals += it;
    if (HPE_STAMPS && blockIdx.x == 0 && t == 0) {  // decision statistics (diagnostic build)
        hpe_stamps[9] += (tk != 0) ? 1 : 0;
        hpe_stamps[30] += (unsigned long long)it;
        hpe_stamps[32 + 9] += 1;
    }
#if HPE_STAMPS
    if (t == 0) {  // every search of every block: {path bits, trials << 32, accepted << 40}
        const unsigned long long k = atomicAdd(&hpe_gold_log[0], 1ull);
        if (k < HPE_GOLD_LOG)
            hpe_gold_log[1 + k] = path | ((unsigned long long)it << 32) |
                                  ((unsigned long long)(tk != 0) << 40);
    }
#endif
    return tk;
}

// Grid 1 or 1 + PREP_WG: workgroup 0 refines the selected frame (do_refine != 0); the
// others, when present, prepare the NEXT frame meanwhile (hpe_prep.hpp) on
// CUs this single-workgroup refine leaves idle -- one launch, one stream, no cross-queue
// dependencies in the frame loop.
// MW (clouds > RF_STAGE_MAX): workgroups 1..mw.Q are the helpers of the multi-workgroup
// form above; the preparation workgroups follow them.
// RIGID: the hand-frame refine (rigid_wave, hpe_device.hpp): every evaluation of the call
// places its spheres as Rg q + u from centres q built once from x0's digit angles, the
// collision a constant of the call; HPE_REFINE_EXACT=1 selects the reference's chain.
template <bool STAGED, bool MW = false, bool RIGID = false>
__global__ __launch_bounds__(RF_NT) void k_refine(double *__restrict__ x0g, const DevObs *__restrict__ og,
                                                  const DevHand *__restrict__ Hg,
                                                  int32_t *__restrict__ match_g,
                                                  int *__restrict__ evals_out, int do_refine,
                                                  PrepArgs pa, DevMw mw, DevPick pk) {
    extern __shared__ __align__(16) unsigned char dyn[];  // staged cloud + matchId / prep
    const int nhelp = MW ? mw.Q : 0;
    if (MW && blockIdx.x >= 1 && (int)blockIdx.x <= nhelp) {
        if (do_refine) mw_helper<RIGID>(mw, blockIdx.x - 1, og, Hg, match_g);
        return;
    }
    if (blockIdx.x >= 1) {
        const unsigned long long t0 = HPE_STAMPS ? __builtin_amdgcn_s_memtime() : 0;
        prep_workgroup(pa, blockIdx.x - 1 - nhelp, dyn);
        if (HPE_STAMPS && threadIdx.x == 0) {  // diagnostic build: prep workgroup spans
            const int k = ((int)blockIdx.x - 1 - nhelp < PREP_BANDS) ? 24 : 25;
            atomicAdd(&hpe_stamps[k], __builtin_amdgcn_s_memtime() - t0);
            atomicAdd(&hpe_stamps[32 + k], 1ull);
        }
        return;
    }
    if (!do_refine) return;
    const DevObs o = *og;  // the selected frame (device-resident: graph-stable args)
    __shared__ RefineSm rs;
    __shared__ DevHand hs;  // hand constants in LDS: keeps them out of the loop's registers
    const int t = threadIdx.x, w = t >> 6, l = t & 63;
    stage_hand<RF_NT>(hs, Hg);
    const DevHand *__restrict__ H = &hs;
    using CV = std::conditional_t<STAGED, CloudView, CloudGlobal>;
    CV cv;
    int32_t *match = match_g;
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
    if (pk.gath) {
        // the previous frame's subswarm exchange: x0 = the best all-gathered state (k_pick_best's
        // rule), also stored to d_state and the previous frame's history row
        if (w == 0) {
            const double x = pick_apply(pk.gath, pick_best_row(pk.gath, pk.world, l), l, x0g,
                                        pk.hist, pk.cur);
            if (l < HPE_DOF) rs.x0[l] = x;
        }
    } else if (t < HPE_DOF) {
        rs.x0[t] = x0g[t];
    }
    if (t == 0) rs.ts_n = 0;
    REF_TS(rs.ts_n, 0);
    __shared__ int mwflag;
    MwLeader ml{mw, 0u, false};
    __syncthreads();
    if (RIGID) {
        // hand-frame centres q (x0's digits, theta0 = -180, theta1..5 = 0: Tgb = I, u = 0)
        // and the call's constant self-collision penalty
        if (w == 0) {
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
        __syncthreads();
    }
    StampClock sc;
    sc.start();
    int evals = 0;
    bool base_valid = false;
    const double e = 1e-5;  // cal_grad step (PSO.cpp:195)
    // clouds of at most FP_MAX points: each lane keeps its frozen points in registers
    const bool small = !MW && STAGED && o.n >= 1 && o.n <= FP_MAX;  // (N = 0: no point to clamp to)
    FrozenPts fpts;
    // the lane's sphere (lane l, clamped) off-image depth value, the same for every
    // evaluation of the call (depth_finish's md * md, computed once)
    const double md2_l = depth_off_sq(o, H->radii[l < HPE_NS ? l : HPE_NS - 1]);
    for (int blk = 0; blk < 2; ++blk) {
        const int lo = 3 * blk;  // start_idx (PSO.cpp:226-227); end_idx = lo + 2
        // Block 2 moves only the global position u = x0[3..5]: every FK of the block is
        // the stored rotation terms of x0 plus u (FK_TRANSLATE, bit-identical).
        FkX *Xt = nullptr;
        if (RIGID && blk == 1) {  // P = Rg q of the block's fixed rotation
            if (w == 0) rigid_wave<RG_STORE_P>(rs.w[0], rs.rg, rs.x0[l < HPE_DOF ? l : 0], nullptr, rs.rg.P);
            __syncthreads();
        } else if (blk == 1) {
            if (w == 0) {
                if (l < HPE_DOF) rs.w[0].th[l] = rs.x0[l];
                wave_sync();
                fk_wave_t<FK_STORE_X, true>(rs.w[0], H, &rs.X);
            }
            __syncthreads();
            Xt = &rs.X;
        }
        double tol = 1;
        int cnt = 0, iter = 0;
        while (tol > 1e-6 && iter < 15 && cnt < 1 && !(MW && ml.failed)) {
            // f_k = cal_cost2(x0, matchId, true).  The spheres of x0 are already in rs.base
            // when x0 is the accepted Goldstein point of the previous iteration
            // (x0 + tk*p == x0 - tk*g bitwise) or an unchanged x0.
            if (!base_valid) {
                if (t < HPE_DOF) rs.base.th[t] = rs.x0[t];
                __syncthreads();
                if (w == 0) {
                    if (RIGID) {
                        const double thl = rs.x0[l < HPE_DOF ? l : 0];
                        if (blk) rigid_wave<RG_TRANS>(rs.base, rs.rg, thl);
                        else rigid_wave<RG_ROT>(rs.base, rs.rg, thl);
                    } else if (Xt) {
                        fk_wave_t<FK_TRANSLATE>(rs.base, H, Xt);
                    } else {
                        fk_wave<true>(rs.base, H);
                    }
                }
                __syncthreads();
            }
            REF_TS(rs.ts_n, 1);
            double fk;
            if (MW) {
                fk = eval_corr<MW, RIGID>(rs, o, cv, H, match, &ml, &mwflag);
                REF_TS(rs.ts_n, 2);
                // cal_grad: x0 +/- e along the 3 block dims, one wave per evaluation
                if (w < 6) {
                    const int d = lo + (w >> 1);
                    if (l < HPE_DOF)
                        rs.w[w].th[l] = (l == d) ? ((w & 1) ? rs.x0[l] - e : rs.x0[l] + e) : rs.x0[l];
                }
                eval_nodes<MW, RIGID>(rs, 6, o, cv, H, match, Xt, &ml, &mwflag, nullptr, nullptr, blk);
            } else {
                // f_k = cal_cost2(x0, matchId, true) and cal_grad's six frozen evaluations
                // (x0 +/- e along the 3 block dims, one wave each) with one barrier between
                // them: the search stores matchId, and while the slowest search waves and the
                // corr sums finish, waves 0..5 already run the parts of their gradient point
                // that need no matchId (FK, depth gathers, collision)
                FrozenHead hd{};
                auto head = [&]() {
                    if (w < 6) {
                        const int d = lo + (w >> 1);
                        const double xl = rs.x0[l < HPE_DOF ? l : 0];
                        const double thl = (l == d) ? ((w & 1) ? xl - e : xl + e) : xl;
                        if (l < HPE_DOF) rs.w[w].th[l] = thl;
                        wave_sync();
                        if (RIGID) hd = blk ? rigid_head<RG_TRANS>(rs.w[w], o, H, rs.rg, thl)
                                            : rigid_head<RG_ROT>(rs.w[w], o, H, rs.rg, thl);
                        else hd = frozen_head<true>(rs.w[w], o, H, Xt, &thl);
                    }
                };
                const DepthG dgc = depth_issue_w0(rs.base, o, H);
                const bool young = w >= HPE_SETPRIO_FROM;  // as in eval_block
                if (young) __builtin_amdgcn_s_setprio(1);
                // (n <= 256) the items go where the SIMDs have room.  Chain form: waves 0..5
                // also run a gradient point's head below (FK), two of them on SIMDs 0 and 1
                // each, one on SIMDs 2 and 3; so waves 4, 5 search nothing and waves 6, 7 two
                // items.  Hand-frame form (HPE_RF_SPREAD): the heads are short (no DH chain),
                // so every wave takes one item and no wave searches twice.
                double al;
                if (small) {
                    const bool spread = RIGID && HPE_RF_SPREAD;
                    const int f0 = (w < 4 || spread) ? 64 * w : (w >= 6) ? 256 + 128 * (w - 6) : 0;
                    const int cnt = (w < 4 || spread) ? 1 : (w >= 6) ? 2 : 0;
                    al = search_align<RF_NT, true>(rs.base, cv, H, match, load_pt(cv, f0 + l),
                                                   f0 + l, BT_GENS, 64, cnt);
                } else {
                    al = search_align<RF_NT, true>(rs.base, cv, H, match, load_pt(cv, t));
                }
                if (young) __builtin_amdgcn_s_setprio(0);
                double co = (!RIGID && t < 144) ? collide_term(rs.base, t, H) : 0.0;
                const double dep = depth_finish(dgc, o, t < HPE_NS);
                const double tot = wave_sum((al * o.lambda + dep) + co);  // as block_sum1
                if (l == 0) rs.red[w][0] = tot;
                head();
                __syncthreads();  // matchId complete, the corr partial sums in red
                if (small) load_frozen_pts(fpts, cv, match, l);
                fk = 0;
#pragma unroll
                for (int k = 0; k < RF_NW; ++k) fk += rs.red[k][0];
                if (RIGID) fk = fk + rs.rg.C;
                REF_TS(rs.ts_n, 2);
                if (w < 6) {
                    double f = RIGID ? frozen_tail<true>(rs.w[w], o, cv, H, match, hd,
                                                         small ? &fpts : nullptr, &md2_l)
                                     : frozen_tail(rs.w[w], o, cv, H, match, hd, small ? &fpts : nullptr);
                    if (RIGID) f = f + rs.rg.C;
                    if (l == 0) rs.fg[w] = f;
                }
                __syncthreads();
            }
            ++evals;
            sc.lap(20);
            evals += 6;
            // cal_grad (PSO.cpp:197-212): g on the block dims, p = -1 * g, computed by every
            // thread for its lane -- no barrier: fg is rewritten only by the next iteration's
            // gradient points (the multi-workgroup form's rs.f by this search's first round,
            // hence its barrier)
            const double *fg = MW ? rs.f : rs.fg;
            const double g0 = (fg[0] - fg[1]) / (2 * e), g1 = (fg[2] - fg[3]) / (2 * e),
                         g2 = (fg[4] - fg[5]) / (2 * e);
            const int dl = l - lo;
            const double gl = (dl == 0) ? g0 : (dl == 1) ? g1 : (dl == 2) ? g2 : 0.0;
            const double pl = -1 * gl;
            if (MW) __syncthreads();
            REF_TS(rs.ts_n, 3);
            sc.lap(21);
            // g'p by op_dot::direct_dot_arma (two accumulators: even / odd indices).  g is
            // zero outside the block, and a zero term leaves an accumulator unchanged
            // (x + -0 = x; the empty sums stay zero), so the sums reduce to the block's
            // terms in the same order: block 0 (dims 0..2) v1 = g0 p0 + g2 p2, v2 = g1 p1;
            // block 1 (dims 3..5) v1 = g4 p4, v2 = g3 p3 + g5 p5.  Same for |g|^2 (tol).
            const double q0 = g0 * (-1 * g0), q1 = g1 * (-1 * g1), q2 = g2 * (-1 * g2);
            const double s0 = g0 * g0, s1 = g1 * g1, s2 = g2 * g2;
            const double gp = (blk == 0) ? (q0 + q2) + q1 : q1 + (q0 + q2);
            // goldstein(x0, grad, matchId, f_k, optfunc, tk, 30)
            // goldstein(x0, grad, matchId, f_k, optfunc, tk, 30), then x0 = x0 - tk*grad
            const double tk = gold_tree<MW, HPE_GOLD_POLICY, true, RIGID>(
                rs, o, cv, H, match, fk, gp, pl, gl, evals, nullptr, Xt, &ml, &mwflag,
                small ? &fpts : nullptr, blk, &md2_l);
            sc.lap(22);
            if (tk == 0) cnt += 1;
            // tol = sqrt(sum(grad % grad)): arrayops::accumulate (two accumulators)
            tol = uniform_f64(sqrt((blk == 0) ? (s0 + s2) + s1 : s1 + (s0 + s2)));
            iter += 1;
            // gold_tree's last barrier published x0 and the accepted node's spheres
            base_valid = true;  // accepted node copied, or tk == 0 and x0 unchanged
            REF_TS(rs.ts_n, 5);
            sc.lap(23);
        }
    }
    if (MW) mw_publish(ml, rs, MW_JOB_EXIT, 0);
    REF_TS(rs.ts_n, 7);
    // a timed-out multi-workgroup refine has no defined result: the pose becomes NaN, so
    // this frame's PSO (and its cost) is NaN and never wins an exchange
    if (t < HPE_DOF) x0g[t] = (MW && ml.failed) ? __builtin_nan("") : rs.x0[t];
    if (t == 0 && evals_out) {
        *evals_out = evals;
        atomicAdd((unsigned long long *)(evals_out + 2), (unsigned long long)evals);  // running total
    }
}

#include "hpe_optimise.hpp"

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

#if HPE_STAMPS
// Diagnostic build only: per-block k_pso_gen stamps, then cleared (not part of include/hpe.h).
extern "C" int hpe_debug_blk_ts(unsigned long long *out) {
    if (!out) return HPE_E_ARG;
    const size_t nb = sizeof(unsigned long long) * BT_GENS * BT_BLK * BT_PTS;
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(hpe_blk_ts), nb, 0, hipMemcpyDeviceToHost) != hipSuccess)
        return HPE_E_HIP;
    std::vector<unsigned long long> z(BT_GENS * BT_BLK * BT_PTS, 0ull);
    if (hipMemcpyToSymbol(HIP_SYMBOL(hpe_blk_ts), z.data(), nb, 0, hipMemcpyHostToDevice) != hipSuccess)
        return HPE_E_HIP;
    return HPE_OK;
}
// Diagnostic build only: the refine timeline of the last frame, then cleared.
extern "C" int hpe_debug_ref_ts(unsigned long long *out) {
    if (!out) return HPE_E_ARG;
    const size_t nb = sizeof(unsigned long long) * RT_LOG;
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(hpe_ref_ts), nb, 0, hipMemcpyDeviceToHost) != hipSuccess)
        return HPE_E_HIP;
    std::vector<unsigned long long> z(RT_LOG, 0ull);
    if (hipMemcpyToSymbol(HIP_SYMBOL(hpe_ref_ts), z.data(), nb, 0, hipMemcpyHostToDevice) != hipSuccess)
        return HPE_E_HIP;
    return HPE_OK;
}
// Diagnostic build only: the Goldstein decision log (not part of include/hpe.h).
extern "C" int hpe_debug_gold_log(unsigned long long *out, int n) {
    if (!out || n < 1) return HPE_E_ARG;
    if (n > HPE_GOLD_LOG + 1) n = HPE_GOLD_LOG + 1;
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(hpe_gold_log), sizeof(unsigned long long) * n, 0,
                            hipMemcpyDeviceToHost) != hipSuccess)
        return HPE_E_HIP;
    const unsigned long long z = 0;
    if (hipMemcpyToSymbol(HIP_SYMBOL(hpe_gold_log), &z, sizeof(z), 0, hipMemcpyHostToDevice) != hipSuccess)
        return HPE_E_HIP;
    return HPE_OK;
}
#endif

extern "C" int hpe_debug_stamps(unsigned long long *out64) {
    if (!out64) return HPE_E_ARG;
    if (hipMemcpyFromSymbol(out64, HIP_SYMBOL(hpe_stamps), sizeof(unsigned long long) * 64, 0,
                            hipMemcpyDeviceToHost) != hipSuccess)
        return HPE_E_HIP;
    unsigned long long z[64] = {0};
    if (hipMemcpyToSymbol(HIP_SYMBOL(hpe_stamps), z, sizeof(z), 0, hipMemcpyHostToDevice) != hipSuccess)
        return HPE_E_HIP;
    return HPE_STAMPS;
}

#include "hpe_api.inc"
