// hpe_host.cpp -- host-side pieces of the product library (no GPU calls):
//   * per-hand constant transforms (fingermodel.cpp:106-132, thumbmodel.cpp:112-138)
//   * observation preprocessing (observedmodel.cpp:110-219, 272-369)
//   * the PSO draw tables: Philox4x32-10 normals and informant-link CSR
// Built with -ffp-contract=off like the device code.
#include "hpe_host.hpp"

#include <cmath>
#include <cstring>
#include <vector>

namespace hpe {

static const double kPi = 3.141592653589793115997963468544185161590576171875;  // acos(-1)
static double d2r(double a) { return a / 180.0 * kPi; }

void build_dev_hand(const hpe_hand_params &p, DevHand &h) {
    std::memset(&h, 0, sizeof(h));
    for (int d = 0; d < 5; ++d) {
        const double L0 = p.geo_cm[4 * d];
        const float sp = (float)p.spacing_cm[d];  // float member, fingermodel.h:43
        const double n = d2r(p.cmc_deg[d]);
        h.Fc[d] = std::cos(n);
        h.Fs[d] = std::sin(n);
        h.FLc[d] = L0 * std::cos(n);
        h.FLs[d] = L0 * std::sin(n);
        const float sp2 = sp * sp;  // float product
        const double a = std::sqrt(L0 * L0 + (double)sp2 - 2 * L0 * sp * std::cos(n));
        const double beta = std::asin(std::sin(n) * sp / a);
        if (d == 0) {
            h.T10x[d] = -a * std::cos(beta);
            h.T10y[d] = -a * std::sin(beta);
            const double pc = n + kPi;  // thumbmodel.cpp:149
            h.twc[d] = std::cos(pc);
            h.tws[d] = std::sin(pc);
        } else {
            h.T10x[d] = -L0 * std::sin(n) * std::cos(beta);
            h.T10y[d] = -L0 * std::sin(n) * std::sin(beta);
            h.twc[d] = 1.0;
            h.tws[d] = 0.0;
        }
        for (int k = 0; k < 4; ++k) h.L[d][k] = p.geo_cm[4 * d + k];
    }
    for (int i = 0; i < HPE_NS; ++i) h.radii[i] = p.radii_cm[i];
    // sphere placement (fingermodel.cpp:223-265, thumbmodel.cpp:242-272):
    // (1. - t*j) * joint1 + (t*j) * joint2, weights computed exactly as there
    int s = 0;
    for (int d = 0; d < 5; ++d) {
        const int ns[4] = {d == 0 ? 2 : 4, 2, 2, 2};
        for (int seg = 0; seg < 4; ++seg) {
            const bool first = (seg == 0 && d != 0);
            const double t = first ? 1. / (ns[0] - 1) : 1. / ns[seg];
            const int j0 = first ? 0 : 1, j1 = first ? ns[0] : ns[seg] + 1;
            for (int j = j0; j < j1; ++j, ++s) {
                h.wa[s] = 1. - t * j;
                h.wb[s] = t * j;
                h.dg[s] = d;
                h.ja[s] = seg;
            }
        }
    }
}

// ---------------------------------------------------------------- preprocessing
// OpenCV 3.0 distanceTransform_5x5 (CV_DIST_L2, mask 5) on the inverted map:
// 16.16 fixed point, metrics {1, 1.4f, 2.1969f}; border = INT_MAX >> 2.
static void chamfer_dt(const double *depth_cm, float *dt) {
    const unsigned HV = 65536u, DG = 91750u, LG = 143976u, INIT = 0x7FFFFFFFu >> 2;
    const int W = HPE_IMG_W, H = HPE_IMG_H, B = 2, ST = W + 2 * B;
    std::vector<unsigned> buf((size_t)ST * (H + 2 * B), INIT);
    auto at = [&](int r, int c) -> unsigned & { return buf[(size_t)(r + B) * ST + c + B]; };
    for (int r = 0; r < H; ++r)
        for (int c = 0; c < W; ++c) {
            if (depth_cm[r * W + c] != 0) {
                at(r, c) = 0;
                continue;
            }
            unsigned m = at(r - 2, c - 1) + LG;
            m = std::min(m, at(r - 2, c + 1) + LG);
            m = std::min(m, at(r - 1, c - 2) + LG);
            m = std::min(m, at(r - 1, c - 1) + DG);
            m = std::min(m, at(r - 1, c) + HV);
            m = std::min(m, at(r - 1, c + 1) + DG);
            m = std::min(m, at(r - 1, c + 2) + LG);
            m = std::min(m, at(r, c - 1) + HV);
            at(r, c) = m;
        }
    const float sc = 1.f / 65536;
    for (int r = H - 1; r >= 0; --r)
        for (int c = W - 1; c >= 0; --c) {
            unsigned m = at(r, c);
            if (m > HV) {
                m = std::min(m, at(r + 2, c + 1) + LG);
                m = std::min(m, at(r + 2, c - 1) + LG);
                m = std::min(m, at(r + 1, c + 2) + LG);
                m = std::min(m, at(r + 1, c + 1) + DG);
                m = std::min(m, at(r + 1, c) + HV);
                m = std::min(m, at(r + 1, c - 1) + DG);
                m = std::min(m, at(r + 1, c - 2) + LG);
                m = std::min(m, at(r, c + 1) + HV);
                at(r, c) = m;
            }
            dt[r * W + c] = (float)m * sc;
        }
}

int preprocess_depth(const float *depth_mm, int to_cm, int downsample, double focal,
                     double *depth_cm, float *dt, double *cloud, int32_t *n_out,
                     double *scale_out, double *dtmax_out, double K[9]) {
    const int W = HPE_IMG_W, H = HPE_IMG_H;
    // init_observation(imW=240, imH=320): img_center = (imH/2, imW/2) = (160, 120)
    const double c0 = 320 / 2., c1 = 240 / 2.;
    const double Kv[9] = {focal, 0.0, c0, 0.0, focal, c1, 0.0, 0.0, 1.0};
    std::memcpy(K, Kv, sizeof(Kv));
    for (int i = 0; i < W * H; ++i) depth_cm[i] = to_cm ? (double)depth_mm[i] / 10. : depth_mm[i];
    int n = 0, ncm = 0;
    double acc[2] = {0, 0};
    for (int r = 0; r < H; ++r) {
        for (int c = 0; c < W; ++c) {
            const double Z = depth_cm[r * W + c];
            if (Z == 0) continue;
            const double X = ((c - c0) * Z) / focal;
            const double Y = ((r - c1) * Z) / focal;
            cloud[3 * n + 0] = X;
            cloud[3 * n + 1] = Y * -1;
            cloud[3 * n + 2] = Z * -1;
            ++n;
            // cm-per-pixel from the projection of (X,Y,Z) and (X+2,Y,Z) (:171-202)
            const double w = (Kv[6] * X + Kv[7] * Y) + Kv[8] * Z;
            const double u = (Kv[0] * X + Kv[1] * Y) + Kv[2] * Z;
            const double v = (Kv[3] * X + Kv[4] * Y) + Kv[5] * Z;
            const double Xe = X + 2.0;
            const double we = (Kv[6] * Xe + Kv[7] * Y) + Kv[8] * Z;
            const double ue = (Kv[0] * Xe + Kv[1] * Y) + Kv[2] * Z;
            const double ve = (Kv[3] * Xe + Kv[4] * Y) + Kv[5] * Z;
            const double du = std::floor(ue / we) - std::floor(u / w);
            const double dv = std::floor(ve / we) - std::floor(v / w);
            const double dn = std::sqrt(du * du + dv * dv);
            if (dn != 0) {
                acc[ncm & 1] += 2.0 / dn;  // arma::mean -> accumulate (2 accumulators)
                ++ncm;
            }
        }
    }
    *scale_out = ncm ? (acc[0] + acc[1]) / ncm : std::nan("");
    if (downsample) {  // :204-217
        const int ns = 250, f = n / ns;
        std::vector<double> tmp(3 * ns, 0.0);
        for (int k = 0; k < ns && n > 0; ++k)
            for (int q = 0; q < 3; ++q) tmp[3 * k + q] = cloud[3 * (k * f) + q];
        std::memcpy(cloud, tmp.data(), sizeof(double) * 3 * ns);
        n = ns;
    }
    *n_out = n;
    chamfer_dt(depth_cm, dt);
    float mx = dt[0];
    for (int i = 1; i < W * H; ++i) mx = dt[i] > mx ? dt[i] : mx;
    *dtmax_out = mx;
    return 0;
}

// ---------------------------------------------------------------- draws
static void philox(uint32_t c[4], uint32_t k0, uint32_t k1) {
    for (int r = 0; r < 10; ++r) {
        if (r) {
            k0 += 0x9E3779B9u;
            k1 += 0xBB67AE85u;
        }
        const uint64_t p0 = (uint64_t)0xD2511F53u * c[0], p1 = (uint64_t)0xCD9E8D57u * c[2];
        const uint32_t n0 = (uint32_t)(p1 >> 32) ^ c[1] ^ k0, n1 = (uint32_t)p1;
        const uint32_t n2 = (uint32_t)(p0 >> 32) ^ c[3] ^ k1, n3 = (uint32_t)p0;
        c[0] = n0; c[1] = n1; c[2] = n2; c[3] = n3;
    }
}

double host_u01(uint64_t seed, uint32_t stream, uint32_t gen, uint32_t idx, uint32_t k) {
    uint32_t c[4] = {k >> 1, idx, gen, stream};
    philox(c, (uint32_t)seed, (uint32_t)(seed >> 32));
    const uint32_t a = (k & 1) ? c[2] : c[0], b = (k & 1) ? c[3] : c[1];
    return (double)((((uint64_t)a) << 21) | (b >> 11)) * 0x1.0p-53;
}

void make_normals(uint64_t seed, int P, double *out, uint32_t stream) {
    for (int i = 0; i < P; ++i)
        for (int q = 0; q < HPE_DOF / 2; ++q) {
            const double u1 = host_u01(seed, stream, 0, i, 2 * q);
            const double u2 = host_u01(seed, stream, 0, i, 2 * q + 1);
            const double r = std::sqrt(-2.0 * std::log(1.0 - u1));
            const double t = 6.283185307179586231995926937088370323181152343750 * u2;
            out[HPE_DOF * i + 2 * q] = r * std::cos(t);
            out[HPE_DOF * i + 2 * q + 1] = r * std::sin(t);
        }
}

// Topology of generation t (PSO.cpp:790-803): each particle s links to
// r = floor(u*(P-1) + 0.5) for 3 draws; receiver r's informants are {r} U {s -> r}.
// outl[t][s][k] = (r, slot of s in r's ascending source list); K = max in-degree.
int make_links(uint64_t seed, int P, int G, std::vector<int> &outl, std::vector<int> *indeg) {
    outl.assign((size_t)(G + 1) * P * 6, -1);
    if (indeg) indeg->assign((size_t)(G + 1) * P, 0);
    std::vector<int> fill(P);
    int K = 1;
    for (int t = 1; t <= G; ++t) {
        std::fill(fill.begin(), fill.end(), 0);
        for (int s = 0; s < P; ++s)  // ascending s: slots follow the reference's find() order
            for (int k = 0; k < 3; ++k) {
                const double u = host_u01(seed, ST_LINK, t, s, k);
                const int r = (int)std::floor(u * (P - 1) + 0.5);
                int *o = &outl[(((size_t)t * P + s) * 3 + k) * 2];
                o[0] = r;
                o[1] = fill[r]++;
                K = std::max(K, fill[r]);
            }
        if (indeg) std::copy(fill.begin(), fill.end(), indeg->begin() + (size_t)t * P);
    }
    return K;
}

}  // namespace hpe
