// Drives the façade methods once on the GPU (tests/test_gpu_facade.py compares the
// printed values with the Python mirror).  argv: hand dir, frames dir.
#include <cstdio>
#include <fstream>
#include <string>

#include "hpe_facade.hpp"

static arma::vec load(const std::string &f, int n) {
    std::ifstream in(f);
    arma::vec v(n);
    for (int i = 0; i < n; ++i) in >> v(i);
    return v;
}

int main(int argc, char **argv) {
    if (argc < 3) return 2;
    arma::vec geo = load(std::string(argv[1]) + "/hgeo.dat", 20);
    arma::vec rad = load(std::string(argv[1]) + "/rad.dat", 48);
    for (int k = 0; k < 20; ++k) geo(k) /= 10.;
    for (int k = 0; k < 48; ++k) rad(k) /= 10.;
    arma::vec tb{2, 2, 2, 2}, fg{4, 2, 2, 2}, spc{-1.86, -1.86, 0, 1.91, 3.84},
        cmc{150, 107.5, 89.8, 76.5, 59.6};
    handmodel hand(geo, spc, tb, fg, cmc, rad);
    observedmodel obs;
    obs.init_observation(argv[2], "000000_depth.bin", true, 240, 320, 241.42, true);
    costfunc cf(&hand, &obs);
    const double x0[26] = {0, -10, -40, 0, 3, 32, 6, 9, 8, 9, 3, 9, 9,
                           6, 1,   9,   8, 7, 4, 8,  7, 6, 2, 7, 7, 7};
    arma::vec th(26);
    for (int k = 0; k < 26; ++k) th(k) = x0[k] + 1.5;
    arma::uvec m;
    std::printf("cal_cost=%.17g\n", cf.cal_cost(th));
    std::printf("cal_cost2=%.17g\n", cf.cal_cost2(th, m, true));
    arma::mat S;
    hand.build_hand_model(th, S);
    std::printf("S0x=%.17g S47z=%.17g\n", S(0, 0), S(47, 2));
    std::printf("align=%.17g\n", cf.align_models(rad, S, *obs.get_ptncloud(), m));
    std::printf("collision=%.17g\n", cf.self_collision_penalty(S, rad));
    arma::mat K = obs.get_cam_mat(), D = obs.get_depth(), T;
    obs.dist_transform(T);
    std::printf("depth=%.17g\n", cf.depth_penalty(K, D, S, T, obs.get_img_scale()));
    unsigned long long s = 0;
    for (arma::uword i = 0; i < m.n_elem; ++i) s += m(i);
    std::printf("m_sum=%llu\n", s);
    // gnd_truth_err (costfunc.cpp:476-507) of GPU-FK hand_joints: argv[3] holds a
    // frames x 63 ground-truth matrix (mm, one frame per line), argv[4] one pose per line;
    // the pose of line f is built and scored against row f
    if (argc >= 5) {
        std::ifstream gin(argv[3]), pin(argv[4]);
        int nf = 0;
        gin >> nf;
        arma::mat gt(nf, 63);
        for (int f = 0; f < nf; ++f)
            for (int k = 0; k < 63; ++k) gin >> gt(f, k);
        for (int f = 0; f < nf; ++f) {
            arma::vec p(26);
            for (int k = 0; k < 26; ++k) pin >> p(k);
            arma::mat Sf;
            hand.build_hand_model(p, Sf);
            std::printf("gte%d=%.17g\n", f, cf.gnd_truth_err(gt, f));
        }
    }
    return 0;
}
