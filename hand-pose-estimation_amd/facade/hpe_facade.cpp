// hpe_facade.cpp -- the reference's handmodel / observedmodel / costfunc / PSO classes
// over the C ABI (include/hpe.h).  Host glue only: every evaluation runs in libhpe.so's
// gfx950 kernels.  Reference semantics are cited per method (/root/reference/src).
#include "hpe_facade.hpp"

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <iostream>
#include <stdexcept>

namespace {

void check(hpe_ctx *c, int rc, const char *what) {
    if (rc == HPE_OK) return;
    std::string msg = std::string("hpe: ") + what + " failed (" + std::to_string(rc) + ")";
    if (c) msg += std::string(": ") + hpe_last_error(c);
    throw std::runtime_error(msg);
}

int device_index() {
    const char *e = std::getenv("HPE_DEVICE");
    return e ? std::atoi(e) : 0;
}

template <typename V>
void copy_in(V &dst, const V &src, arma::uword n, const char *const *msg) {
    if (src.n_elem != n) {  // handmodel.cpp:150-208: print, zero-fill, carry on
        dst.zeros(n);
        for (const char *const *m = msg; *m; ++m) std::cout << *m;
        std::cout << std::endl;
    } else {
        dst = src;
    }
}

// arma 48 x 3 (column-major) <-> the ABI's row-major [sphere][xyz]
void spheres_to_rows(const arma::mat &S, double *out) {
    if (S.n_rows != 48 || S.n_cols != 3) throw std::invalid_argument("spheres must be 48 x 3");
    for (int s = 0; s < 48; ++s)
        for (int r = 0; r < 3; ++r) out[3 * s + r] = S(s, r);
}

}  // namespace

// ------------------------------------------------------------------ handmodel
handmodel::handmodel(arma::vec h_geo, arma::vec h_spacing, arma::vec tb_spheres,
                     arma::vec fg_spheres, arma::vec h_CMC, arma::vec sphR) {
    // handmodel.cpp:10-27
    set_hand_CMC(h_CMC);
    set_hand_geo(h_geo);
    set_spacing(h_spacing);
    set_num_spheres(tb_spheres, fg_spheres);
    set_hand_rad(sphR);
    init_hand();
    hand_joints.zeros(21, 3);
}

handmodel::~handmodel() {
    if (ctx_) hpe_destroy(ctx_);
}

void handmodel::init_hand() { dirty_ = true; }
handmodel &handmodel::update_hand() {
    dirty_ = true;
    return *this;
}
handmodel &handmodel::build_spheres() { return *this; }

void handmodel::set_hand_CMC(arma::vec &h_CMC) {
    static const char *const m[] = {"hand_CMC contains the CMC-angels for each finger/thumb",
                                    "==> must be of size (5, 1)\n",
                                    "call set_hand_CMC() to re-initialise", nullptr};
    copy_in(hand_CMC, h_CMC, 5, m);
    dirty_ = true;
}

void handmodel::set_hand_geo(arma::vec &h_geo) {
    static const char *const m[] = {
        "hand_geo contains the geometry of each finger/thumb; ",
        "each instance has four segments ==> 20 params are needed ",
        "call set_hand_geo() to re-initialise", nullptr};
    copy_in(hand_geo, h_geo, 20, m);
    dirty_ = true;
}

void handmodel::set_spacing(arma::vec &h_spacing) {
    static const char *const m[] = {
        "h_spacing Specifies the distance between neighbouring base joints; ",
        "must be of shape (5,1)\n", "call set_spacing() to re-initialise", nullptr};
    copy_in(spacing, h_spacing, 5, m);
    dirty_ = true;
}

void handmodel::set_num_spheres(arma::vec &tb_spheres, arma::vec &fg_spheres) {
    tb_num_spheres = tb_spheres;
    fg_num_spheres = fg_spheres;
    dirty_ = true;
}

void handmodel::set_hand_rad(arma::vec &rad) {
    spheres_radii = rad;
    dirty_ = true;
}

hpe_ctx *handmodel::context() {
    if (ctx_ && !dirty_) return ctx_;
    if (ctx_) {
        hpe_destroy(ctx_);
        ctx_ = nullptr;
    }
    // the reference hard-codes 8 + 4 x 10 sphere rows (handmodel.cpp:272-286)
    const double tb[4] = {2, 2, 2, 2}, fg[4] = {4, 2, 2, 2};
    if (tb_num_spheres.n_elem != 4 || fg_num_spheres.n_elem != 4)
        throw std::invalid_argument("sphere counts must be tb {2,2,2,2}, fg {4,2,2,2}");
    for (int k = 0; k < 4; ++k)
        if (tb_num_spheres(k) != tb[k] || fg_num_spheres(k) != fg[k])
            throw std::invalid_argument("sphere counts must be tb {2,2,2,2}, fg {4,2,2,2}");
    if (spheres_radii.n_elem != 48) throw std::invalid_argument("sphR must hold 48 radii");
    hpe_hand_params p;
    std::memset(&p, 0, sizeof(p));
    for (int k = 0; k < 20; ++k) p.geo_cm[k] = hand_geo(k);
    for (int k = 0; k < 48; ++k) p.radii_cm[k] = spheres_radii(k);
    for (int k = 0; k < 5; ++k) {
        p.cmc_deg[k] = hand_CMC(k);
        p.spacing_cm[k] = spacing(k);
    }
    for (int k = 0; k < 4; ++k) {
        p.tb_spheres[k] = (int32_t)tb[k];
        p.fg_spheres[k] = (int32_t)fg[k];
    }
    check(nullptr, hpe_create(&ctx_, device_index(), &p), "hpe_create");
    dirty_ = false;
    bound_obs_ = nullptr;
    return ctx_;
}

void handmodel::build_hand_model(arma::vec &h_theta, arma::mat &sphere_centres) {
    // handmodel.cpp:259-298
    if (h_theta.n_elem != 26) throw std::invalid_argument("theta must have 26 elements");
    hpe_ctx *c = context();
    double S[48 * 3], J[21 * 3];
    check(c, hpe_build_spheres(c, h_theta.memptr(), 1, S, J), "hpe_build_spheres");
    sphere_centres.set_size(48, 3);
    for (int s = 0; s < 48; ++s)
        for (int r = 0; r < 3; ++r) sphere_centres(s, r) = S[3 * s + r];
    hand_joints.set_size(21, 3);
    for (int j = 0; j < 21; ++j)
        for (int r = 0; r < 3; ++r) hand_joints(j, r) = J[3 * j + r];
}

void handmodel::build_hand_model_batch(arma::mat &thetas, arma::mat &spheres) {
    if (thetas.n_rows != 26 || thetas.n_cols < 1) throw std::invalid_argument("thetas: 26 x P");
    hpe_ctx *c = context();
    spheres.set_size(48 * 3, thetas.n_cols);
    check(c, hpe_build_spheres(c, thetas.memptr(), (int)thetas.n_cols, spheres.memptr(), nullptr),
          "hpe_build_spheres");
}

// ------------------------------------------------------------------ observedmodel
observedmodel::observedmodel() {
    // observedmodel.cpp:24-38 defaults
    path = "../handModelling/Release_2014_5_28/Subject1/";
    filename = "000001_depth.bin";
    img_center.zeros(2);
    img_center(0) = 160;
    img_center(1) = 120;
    camera_calibration.zeros(3, 3);
}

void observedmodel::init_observation(std::string dpath, std::string dfname, bool mm_to_cm,
                                     int imW, int imH, double foclen, bool down) {
    // observedmodel.cpp:41-63
    if (imW != 240 || imH != 320)
        throw std::invalid_argument("observedmodel: only 240 x 320 frames are supported");
    path = dpath;
    filename = dfname;
    to_cm = mm_to_cm;
    imgW = imW;
    imgH = imH;
    focal_len = foclen;
    downsample = down;
    img_center(0) = imH / 2.;
    img_center(1) = imW / 2.;
    load_data();
    get_observed();
}

void observedmodel::set_img_center(arma::vec ncenter) { img_center = ncenter; }

void observedmodel::load_data() {
    // observedmodel.cpp:272-310: headerless float32 (mm), 320 x 240 column-major = 240 x 320
    // row-major after the transpose the reference applies
    const std::string full = path + filename;
    std::ifstream fin(full.c_str(), std::ios::in | std::ios::binary);
    if (!fin.is_open()) {
        std::cerr << "error: open file for input failed!" << std::endl;
        std::abort();
    }
    raw_mm_.assign(240 * 320, 0.f);
    fin.read(reinterpret_cast<char *>(raw_mm_.data()), sizeof(float) * raw_mm_.size());
}

void observedmodel::set_depth_mm(const float *depth_mm) {
    raw_mm_.assign(depth_mm, depth_mm + 240 * 320);
    get_observed();
}

void observedmodel::get_observed() {
    // observedmodel.cpp:66-75: cloud (+ scale, down-sample) and distance transform
    if (img_center.n_elem != 2 || img_center(0) != 160 || img_center(1) != 120)
        throw std::invalid_argument("observedmodel: image centre must be (160, 120)");
    if (raw_mm_.size() != 240 * 320) throw std::logic_error("observedmodel: no depth loaded");
    depth_cm_.assign(240 * 320, 0.0);
    dt_.assign(240 * 320, 0.f);
    cloud_.assign(240 * 320 * 3, 0.0);
    int32_t n = 0;
    double K[9];
    check(nullptr,
          hpe_preprocess_depth(raw_mm_.data(), to_cm ? 1 : 0, downsample ? 1 : 0, focal_len,
                               depth_cm_.data(), dt_.data(), cloud_.data(), &n, &scale, &dtmax_, K),
          "hpe_preprocess_depth");
    n_ = n;
    cloud_.resize((size_t)3 * n);
    depthmap.set_size(240, 320);
    disttran.set_size(240, 320);
    for (int r = 0; r < 240; ++r)
        for (int c = 0; c < 320; ++c) {
            depthmap(r, c) = depth_cm_[r * 320 + c];
            disttran(r, c) = dt_[r * 320 + c];
        }
    pointcld.set_size(n, 3);
    for (int i = 0; i < n; ++i)
        for (int q = 0; q < 3; ++q) pointcld(i, q) = cloud_[3 * i + q];
    camera_calibration.set_size(3, 3);
    for (int r = 0; r < 3; ++r)
        for (int c = 0; c < 3; ++c) camera_calibration(r, c) = K[3 * r + c];
    ++version_;
}

hpe_frame observedmodel::frame() const {
    hpe_frame f;
    f.depth_cm = depth_cm_.data();
    f.dt = dt_.data();
    f.cloud = cloud_.data();
    f.n = n_;
    f.scale = scale;
    f.dtmax = dtmax_;
    for (int r = 0; r < 3; ++r)
        for (int c = 0; c < 3; ++c) f.K[3 * r + c] = camera_calibration(r, c);
    return f;
}

observedmodel &observedmodel::next_frame(std::string next) {
    // observedmodel.cpp:420-430
    set_filename(next);
    load_data();
    get_observed();
    return *this;
}

void observedmodel::depth_to_ptncloud(arma::mat &ptncloud) { ptncloud = pointcld; }

void observedmodel::downsample_ptncloud(arma::uvec &rows_id) {
    // observedmodel.cpp:204-217: rows k * floor(N / 250), k < 250
    const arma::uword ns = 250, f = pointcld.n_rows / ns;
    rows_id.zeros(ns);
    arma::mat out(ns, 3);
    for (arma::uword k = 0; k < ns; ++k) {
        rows_id(k) = k * f;
        for (int q = 0; q < 3; ++q) out(k, q) = pointcld.n_rows ? pointcld(k * f, q) : 0.0;
    }
    pointcld = out;
}

void observedmodel::invert_depthmap(arma::mat &depthmp, bool) {
    // observedmodel.cpp:313-337: zeros -> 255, non-zeros -> 0
    for (arma::uword i = 0; i < depthmp.n_elem; ++i) depthmp(i) = depthmp(i) == 0 ? 255.0 : 0.0;
}

void observedmodel::dist_transform(arma::mat &dist_trans) { dist_trans = disttran; }

void observedmodel::show_depthmap() {
    std::cout << "observedmodel::show_depthmap: display is out of scope (DESIGN.md)" << std::endl;
}
void observedmodel::visualise_ptncloud() {
    std::cout << "observedmodel::visualise_ptncloud: display is out of scope (DESIGN.md)"
              << std::endl;
}

// ------------------------------------------------------------------ costfunc
costfunc::costfunc(handmodel *handM, observedmodel *observed) : hand(handM), observation(observed) {}

hpe_ctx *costfunc::sync() {
    hpe_ctx *c = hand->context();
    if (hand->bound_obs_ != observation || hand->bound_ver_ != observation->version()) {
        const hpe_frame f = observation->frame();
        check(c, hpe_set_frame(c, &f), "hpe_set_frame");
        hand->bound_obs_ = observation;
        hand->bound_ver_ = observation->version();
    }
    return c;
}

double costfunc::cal_cost(arma::vec &theta) {
    // costfunc.cpp:89-127
    if (theta.n_elem != 26) throw std::invalid_argument("theta must have 26 elements");
    hpe_ctx *c = sync();
    double cost = 0;
    check(c, hpe_eval_costs(c, theta.memptr(), 1, 0, &cost, nullptr), "hpe_eval_costs");
    return cost;
}

void costfunc::cal_cost_batch(arma::mat &thetas, arma::vec &costs, bool with_collision) {
    if (thetas.n_rows != 26 || thetas.n_cols < 1) throw std::invalid_argument("thetas: 26 x P");
    hpe_ctx *c = sync();
    costs.zeros(thetas.n_cols);
    check(c, hpe_eval_costs(c, thetas.memptr(), (int)thetas.n_cols, with_collision ? 1 : 0,
                            costs.memptr(), nullptr),
          "hpe_eval_costs");
}

double costfunc::cal_cost2(arma::vec &theta, arma::uvec &matchId, bool compute_corr, bool debug) {
    // costfunc.cpp:31-86
    if (theta.n_elem != 26) throw std::invalid_argument("theta must have 26 elements");
    hpe_ctx *c = sync();
    const int n = observation->frame().n;
    std::vector<int32_t> m((size_t)(n > 0 ? n : 1), 0);
    if (!compute_corr) {
        if ((int)matchId.n_elem != n) throw std::invalid_argument("matchId size != cloud size");
        for (int i = 0; i < n; ++i) m[i] = (int32_t)matchId(i);
    }
    double cost = 0, terms[3];
    check(c, hpe_cal_cost2(c, theta.memptr(), m.data(), compute_corr ? 1 : 0, &cost, terms),
          "hpe_cal_cost2");
    if (compute_corr) {
        matchId.zeros(n);
        for (int i = 0; i < n; ++i) matchId(i) = (arma::uword)m[i];
    }
    if (debug) {
        std::cout << terms[0] << std::endl;
        std::cout << terms[1] << std::endl;
        std::cout << terms[2] << "\n" << std::endl;
    }
    return cost;
}

// term 0 align, 1 depth, 2 collision (3: correspondences only) for a caller-supplied
// sphere matrix
double costfunc::sphere_term(arma::mat &spheres, arma::uvec *matchId, int term) {
    hpe_ctx *c = sync();
    const int n = observation->frame().n;
    double S[48 * 3], terms[3];
    spheres_to_rows(spheres, S);
    std::vector<int32_t> m((size_t)(n > 0 ? n : 1), 0);
    const bool corr = (matchId == nullptr) || (term != 0);
    if (!corr) {
        if ((int)matchId->n_elem != n) throw std::invalid_argument("matchId size != cloud size");
        for (int i = 0; i < n; ++i) m[i] = (int32_t)(*matchId)(i);
    }
    check(c, hpe_eval_spheres(c, S, 1, corr ? 1 : 0, m.data(), terms), "hpe_eval_spheres");
    if (matchId && term != 0) {
        matchId->zeros(n);
        for (int i = 0; i < n; ++i) (*matchId)(i) = (arma::uword)m[i];
    }
    return term < 3 ? terms[term] : 0.0;
}

void costfunc::compute_correspondences(arma::mat &ptns, arma::mat &sphM, arma::uvec &matchId) {
    // costfunc.cpp:306-343 (the device evaluates the observation's own cloud)
    if (ptns.n_rows != observation->get_ptncloud()->n_rows)
        throw std::invalid_argument("compute_correspondences: cloud is not the observation's");
    sphere_term(sphM, &matchId, 3);
    matchIdx = matchId;
}

double costfunc::align_models(arma::vec &spheresR, arma::mat &spheresM, arma::mat &ptncloud,
                              arma::uvec &matchId) {
    // costfunc.cpp:346-377 (the hand's radii, the observation's cloud)
    if (spheresR.n_elem != 48 || ptncloud.n_rows != observation->get_ptncloud()->n_rows)
        throw std::invalid_argument("align_models: radii / cloud are not the model's");
    return sphere_term(spheresM, &matchId, 0);
}

double costfunc::depth_penalty(arma::mat &, arma::mat &, arma::mat &spheres, arma::mat &, double) {
    // costfunc.cpp:227-304 on the observation's K / depth / DT / scale; like the
    // reference it leaves `spheres` with y and z un-negated (:249)
    const double v = sphere_term(spheres, nullptr, 1);
    for (int s = 0; s < 48; ++s) {
        spheres(s, 1) *= -1;
        spheres(s, 2) *= -1;
    }
    return v;
}

double costfunc::self_collision_penalty(arma::mat &spheresM, arma::vec &) {
    // costfunc.cpp:130-197 (the hand's radii)
    return sphere_term(spheresM, nullptr, 2);
}

double costfunc::gnd_truth_err(arma::mat &gnd_truth, int frame) {
    // costfunc.cpp:476-507 on the host joints of the last build_hand_model (evaluation only)
    if (gnd_truth.n_cols != 63 || frame < 0 || (arma::uword)frame >= gnd_truth.n_rows)
        throw std::invalid_argument("gnd_truth: frames x 63");
    const arma::mat &hj = hand->hand_joints;
    double d[6];
    const int sel[6] = {0, 4, 8, 12, 16, 20};
    for (int q = 0; q < 6; ++q) {
        const int j = sel[q];
        double e[3];
        for (int r = 0; r < 3; ++r) {
            double v = hj(j, r) * 10.0;  // back to mm
            if (r > 0) v *= -1;          // hand_joints.cols(1,2) *= -1
            e[r] = gnd_truth(frame, 3 * j + r) - v;
        }
        d[q] = std::sqrt((e[0] * e[0] + e[1] * e[1]) + e[2] * e[2]);
    }
    // sum(): arrayops::accumulate, two alternating accumulators
    return ((d[0] + d[2]) + d[4]) + ((d[1] + d[3]) + d[5]);
}

// ------------------------------------------------------------------ PSO
PSO::PSO() : w(0.7298), c1(1.49618), c2(1.49618), minstep(1e-6), minfunc(1e-6), maxiter(100) {
    // PSO.cpp:16-36
}

void PSO::set_pso_params(arma::vec &upperbound, arma::vec &lowerbound, arma::vec &std,
                         double &omega, double &phip, double &phig, int &maxIter,
                         double &minStep, double &minFunc) {
    // PSO.cpp:38-54
    if (upperbound.n_elem != 26 || lowerbound.n_elem != 26 || std.n_elem != 26)
        throw std::invalid_argument("bounds / std must have 26 elements");
    theta_max = upperbound;
    theta_min = lowerbound;
    theta_std = std;
    w = omega;
    c1 = phip;
    c2 = phig;
    maxiter = maxIter;
    minstep = minStep;
    minfunc = minFunc;
    have_params_ = true;
}

// The reference copies rows 0..12 and the three later fingers' MCP1 / MCP2 / PIP in
// place, and writes each DIP as (2./3) * PIP with the product rounded once (PSO.cpp:169-177).
// Out-of-range rows throw as Armadillo's bounds check does (std::logic_error).
void PSO::dim_restore(arma::vec &theta_in, arma::vec &theta_out) {
    if (theta_in.n_elem < 22 || theta_out.n_elem < 26)
        throw std::logic_error("Mat::rows(): indices out of bounds or incorrectly used");
    for (int k = 0; k <= 12; ++k) theta_out(k) = theta_in(k);  // g_rot, g_pos, thumb, index
    theta_out(13) = 2. / 3 * theta_in(12);
    for (int f = 0; f < 3; ++f) {  // middle, ring, little: rows 14-16, 18-20, 22-24
        const int o = 14 + 4 * f, i = 13 + 3 * f;
        for (int k = 0; k < 3; ++k) theta_out(o + k) = theta_in(i + k);
        theta_out(o + 3) = 2. / 3 * theta_in(i + 2);
    }
}

void PSO::push(hpe_ctx *c) {
    if (!have_params_) throw std::logic_error("PSO: call set_pso_params first");
    check(c, hpe_set_pso_params(c, theta_max.memptr(), theta_min.memptr(), theta_std.memptr(), w,
                                c1, c2, maxiter, minstep, minfunc),
          "hpe_set_pso_params");
    check(c, hpe_set_seed(c, seed), "hpe_set_seed");
}

void PSO::refine_init_pose(arma::vec &x0, costfunc &optfunc) {
    // PSO.cpp:216-266
    if (x0.n_elem != 26) throw std::invalid_argument("x0 must have 26 elements");
    hpe_ctx *c = optfunc.sync();
    int32_t ev = 0;
    check(c, hpe_refine_init_pose(c, x0.memptr(), &ev), "hpe_refine_init_pose");
    refine_evals_ = ev;
}

int PSO::pso_evolve(costfunc &optfunc, arma::vec &x0, int num_particles, arma::vec &bestp) {
    // PSO.cpp:717-886
    if (x0.n_elem != 26) throw std::invalid_argument("x0 must have 26 elements");
    hpe_ctx *c = optfunc.sync();
    push(c);
    bestp.zeros(26);
    check(c, hpe_pso_evolve(c, x0.memptr(), num_particles, bestp.memptr(), &gbest_cost_),
          "hpe_pso_evolve");
    return 1;
}

int PSO::pso_optimise(costfunc &optfunc, arma::vec &x0, int num_p, arma::vec &bestp) {
    // PSO.cpp:539-712
    if (x0.n_elem != 26) throw std::invalid_argument("x0 must have 26 elements");
    hpe_ctx *c = optfunc.sync();
    push(c);
    bestp.zeros(26);
    check(c, hpe_pso_optimise(c, x0.memptr(), num_p, bestp.memptr(), &gbest_cost_, nullptr, 0),
          "hpe_pso_optimise");
    return 1;
}

double PSO::track_frame(costfunc &optfunc, arma::vec &x0, int num_particles, bool refine) {
    if (x0.n_elem != 26) throw std::invalid_argument("x0 must have 26 elements");
    hpe_ctx *c = optfunc.sync();
    push(c);
    double cost = 0;
    check(c, hpe_track_frame(c, num_particles, refine ? 1 : 0, x0.memptr(), &cost),
          "hpe_track_frame");
    return cost;
}
