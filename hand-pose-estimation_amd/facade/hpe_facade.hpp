// hpe_facade.hpp -- host C++ façade with the reference's class and method names
// (handmodel, observedmodel, costfunc, PSO) over the C ABI of include/hpe.h.
//
// A caller of the reference replaces #include "PSO.h" / "costfunc.h" / "handmodel.h" /
// "observedmodel.h" with this header and links libhpe_facade.so + libhpe.so; the call
// sites of test_full (testmodel.cpp:27-146) compile unchanged.  Everything is passed by
// non-const reference as in the reference; pso_evolve returns 1 (PSO.cpp:884).
//
// Every cost evaluation, FK, PSO generation and refine step runs on the GPU (gfx950
// kernels in libhpe.so).  There is no CPU fallback: a device or HIP error throws
// std::runtime_error carrying hpe_last_error().  Bad vector sizes print the reference's
// message and zero-fill (handmodel.cpp:150-208); an unreadable .bin aborts
// (observedmodel.cpp:290-293).
//
// Device selection: environment variable HPE_DEVICE (default 0); one context per
// handmodel, created on first use.
#pragma once

#if !defined(HPE_FACADE_LITE) && defined(__has_include)
#if __has_include(<armadillo>)
#include <armadillo>
#define HPE_FACADE_ARMADILLO 1
#endif
#endif
#ifndef HPE_FACADE_ARMADILLO
#include "arma_lite.hpp"
#endif

#include <string>
#include <vector>

#include "../../include/hpe.h"

class observedmodel;

// handmodel.h:9-32
class handmodel {
public:
    handmodel(arma::vec h_geo, arma::vec h_spacing, arma::vec tb_spheres, arma::vec fg_spheres,
              arma::vec h_CMC, arma::vec sphR);
    ~handmodel();
    handmodel(const handmodel &) = delete;
    handmodel &operator=(const handmodel &) = delete;

    void init_hand();
    void set_hand_CMC(arma::vec &h_CMC);
    void set_hand_geo(arma::vec &h_geo);
    void set_spacing(arma::vec &h_spacing);
    void set_hand_rad(arma::vec &rad);
    void set_num_spheres(arma::vec &tb_spheres, arma::vec &fg_spheres);
    // 48 x 3 sphere centres (y, z negated) and hand_joints (21 x 3) of one theta
    void build_hand_model(arma::vec &h_theta, arma::mat &sphere_centres);
    arma::vec get_hand_geo() const { return hand_geo; }
    arma::vec get_hand_CMC() const { return hand_CMC; }
    arma::vec get_spacing() const { return spacing; }
    arma::vec get_tb_num_spheres() const { return tb_num_spheres; }
    arma::vec get_fg_num_spheres() const { return fg_num_spheres; }
    arma::vec get_spheres_radii() const { return spheres_radii; }
    arma::vec *get_radii() { return &spheres_radii; }
    handmodel &update_hand();
    handmodel &build_spheres();
    arma::mat hand_joints;

    // --- extensions
    // thetas 26 x P (one particle per column) -> S (48*3) x P, column p = row-major 48 x 3
    void build_hand_model_batch(arma::mat &thetas, arma::mat &spheres);
    hpe_ctx *context();  // the device context (created / rebuilt on demand)

private:
    friend class costfunc;
    arma::vec hand_geo, spacing, hand_CMC, tb_num_spheres, fg_num_spheres, spheres_radii;
    hpe_ctx *ctx_ = nullptr;
    bool dirty_ = true;
    const observedmodel *bound_obs_ = nullptr;  // frame resident in ctx_
    unsigned long long bound_ver_ = 0;
};

// observedmodel.h:10-63 (GUI members show_depthmap / visualise_ptncloud are out of scope)
class observedmodel {
public:
    observedmodel();
    void init_observation(std::string dpath, std::string dfname, bool mm_to_cm, int imW,
                          int imH, double foclen, bool downsample);
    void get_observed();
    void show_depthmap();
    void visualise_ptncloud();
    void depth_to_ptncloud(arma::mat &ptncloud);
    void load_data();
    void downsample_ptncloud(arma::uvec &rows_id);
    void set_focal_len(double nfocal) { focal_len = nfocal; }
    void set_img_center(arma::vec ncenter);
    void set_filename(std::string name) { filename = name; }
    void set_path(std::string newdir) { path = newdir; }
    void set_mm_to_cm(bool mm_to_cm) { to_cm = mm_to_cm; }
    arma::mat *get_camera_mat() { return &camera_calibration; }
    arma::mat *get_depthmap() { return &depthmap; }
    arma::mat *get_ptncloud() { return &pointcld; }
    arma::mat *get_disttran() { return &disttran; }
    arma::mat get_cam_mat() const { return camera_calibration; }
    arma::mat get_depth() const { return depthmap; }
    arma::vec get_img_center() const { return img_center; }
    double get_img_scale() const { return scale; }
    double get_focal_len() const { return focal_len; }
    int get_imgH() const { return imgH; }
    int get_imgW() const { return imgW; }
    observedmodel &next_frame(std::string next);
    void invert_depthmap(arma::mat &depthmp, bool display = false);
    void dist_transform(arma::mat &dist_trans);

    // --- extensions
    void set_depth_mm(const float *depth_mm);  // in-memory frame (synthetic input)
    unsigned long long version() const { return version_; }
    hpe_frame frame() const;  // row-major views for the C ABI

private:
    std::string path, filename;
    arma::mat depthmap, pointcld, disttran, camera_calibration;
    arma::vec img_center;
    int imgW = 240, imgH = 320;
    bool to_cm = true, downsample = false;
    double focal_len = 241.42, scale = 0, dtmax_ = 0;
    std::vector<float> raw_mm_, dt_;
    std::vector<double> depth_cm_, cloud_;
    int n_ = 0;
    unsigned long long version_ = 0;
};

// costfunc.h:25-41
class costfunc {
public:
    costfunc(handmodel *handM, observedmodel *observed);
    double cal_cost(arma::vec &theta);
    double cal_cost2(arma::vec &theta, arma::uvec &matchId, bool compute_corr, bool debug = false);
    double align_models(arma::vec &spheresR, arma::mat &spheresM, arma::mat &ptncloud,
                        arma::uvec &matchId);
    double depth_penalty(arma::mat &cam_mat, arma::mat &depthmp, arma::mat &spheres,
                         arma::mat &disttrans, double scale);
    double self_collision_penalty(arma::mat &spheresM, arma::vec &spheresR);
    void compute_correspondences(arma::mat &ptns, arma::mat &sphM, arma::uvec &matchId);
    arma::uvec get_matchIdx() const { return matchIdx; }
    // costfunc.cpp:476-507: wrist + five finger tips error (mm) of the hand_joints left by
    // the last build_hand_model against row `frame` of gnd_truth (frames x 63, joint j at
    // columns 3j..3j+2)
    double gnd_truth_err(arma::mat &gnd_truth, int frame);

    // --- extensions: the OpenMP particle loops of PSO.cpp:748,848 as one launch
    void cal_cost_batch(arma::mat &thetas, arma::vec &costs, bool with_collision = false);
    hpe_ctx *sync();  // context with this cost function's observation resident

private:
    double sphere_term(arma::mat &spheres, arma::uvec *matchId, int term);
    handmodel *hand;
    observedmodel *observation;
    arma::uvec matchIdx;
};

// PSO.h:15-72 (the pso_solve variant is listed in DESIGN.md §8)
class PSO {
public:
    PSO();
    void refine_init_pose(arma::vec &x0, costfunc &optfunc);
    int pso_evolve(costfunc &optfunc, arma::vec &x0, int num_particles, arma::vec &bestp);
    // PSO.cpp:539-712: descent + global-best PSO (omega / phip / phig); the reference
    // marks it "merely used for testing gradient descent + pso"
    int pso_optimise(costfunc &optfunc, arma::vec &x0, int num_p, arma::vec &bestp);
    void set_pso_params(arma::vec &upperbound, arma::vec &lowerbound, arma::vec &std,
                        double &omega, double &phip, double &phig, int &maxiter,
                        double &minstep, double &minfunc);
    // PSO.cpp:160-180: 22 -> 26 DOF, each finger's DIP = 2/3 of its PIP (host arithmetic;
    // theta_out must already hold 26 elements, as the reference's .rows() assignments need)
    void dim_restore(arma::vec &theta_in, arma::vec &theta_out);

    // --- extensions
    // testmodel.cpp:126-138 in one device-resident call; x0 <- bestp; returns the cost
    double track_frame(costfunc &optfunc, arma::vec &x0, int num_particles, bool refine = true);
    void set_seed(unsigned long long s) { seed = s; }
    double last_gbest_cost() const { return gbest_cost_; }
    int last_refine_evals() const { return refine_evals_; }

private:
    void push(hpe_ctx *c);
    arma::vec theta_min, theta_max, theta_std;
    double w, c1, c2, minstep, minfunc;
    int maxiter;
    unsigned long long seed = 1000;  // arma_rng::set_seed(1000) (PSO.cpp:722)
    bool have_params_ = false;
    double gbest_cost_ = 0;
    int refine_evals_ = 0;
};
