// hpe_track -- the reference's tracking driver (test_full, testmodel.cpp:27-146) written
// against the façade, so the same call sequence runs on the GPU:
//   handmodel(hgeo/10, spacing, counts, CMC, rad/10); observedmodel.init_observation;
//   per frame: next_frame -> refine_init_pose -> pso_evolve -> cal_cost(bestp) -> x0 = bestp
// and prints "frameNNNNNN-cost: <cost>" in the reference's scientific / precision-15 format
// (testmodel.cpp:133-134, 289-290).
//
// usage: hpe_track --hand DIR (hgeo.dat, rad.dat raw ascii, mm) --frames DIR
//                  [--n 10] [--first 0] [--particles 32] [--maxiter 200] [--refine 1]
//                  [--fused 0] [--full-cloud 0] [--pose-out FILE]
// --fused 1 runs each frame as one device-resident PSO::track_frame call instead of the
// three reference calls (same results; no host round trips inside the frame).
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <iomanip>
#include <iostream>
#include <sstream>
#include <string>

#include "hpe_facade.hpp"

static arma::vec load_ascii(const std::string &file, arma::uword n) {
    std::ifstream in(file);
    if (!in.is_open()) {
        std::cerr << "error: cannot open " << file << std::endl;
        std::exit(2);
    }
    arma::vec v(n);
    for (arma::uword i = 0; i < n; ++i)
        if (!(in >> v(i))) {
            std::cerr << "error: " << file << " holds fewer than " << n << " values" << std::endl;
            std::exit(2);
        }
    return v;
}

int main(int argc, char **argv) {
    std::string hand_dir, frames_dir, pose_out;
    int nframes = 10, first = 0, num_p = 32, maxiter = 200, refine = 1, fused = 0, full = 0;
    for (int a = 1; a + 1 < argc; a += 2) {
        const std::string k = argv[a], v = argv[a + 1];
        if (k == "--hand") hand_dir = v;
        else if (k == "--frames") frames_dir = v;
        else if (k == "--n") nframes = std::atoi(v.c_str());
        else if (k == "--first") first = std::atoi(v.c_str());
        else if (k == "--particles") num_p = std::atoi(v.c_str());
        else if (k == "--maxiter") maxiter = std::atoi(v.c_str());
        else if (k == "--refine") refine = std::atoi(v.c_str());
        else if (k == "--fused") fused = std::atoi(v.c_str());
        else if (k == "--full-cloud") full = std::atoi(v.c_str());
        else if (k == "--pose-out") pose_out = v;
        else {
            std::cerr << "unknown option " << k << std::endl;
            return 2;
        }
    }
    if (hand_dir.empty() || frames_dir.empty()) {
        std::cerr << "usage: hpe_track --hand DIR --frames DIR [options]" << std::endl;
        return 2;
    }
    if (frames_dir.back() != '/') frames_dir += '/';
    std::cout.precision(15);
    std::cout << std::scientific;
    try {
        // testmodel.cpp:33-52
        arma::vec x0(26), tbnum(4), fgnum(4), spc(5), hcmc(5);
        tbnum << 2 << 2 << 2 << 2 << arma::endr;
        fgnum << 4 << 2 << 2 << 2 << arma::endr;
        spc << -1.86 << -1.86 << 0 << 1.91 << 3.84 << arma::endr;
        hcmc << 150 << 107.5 << 89.8 << 76.5 << 59.6 << arma::endr;
        const double x0v[26] = {0, -10, -40, 0, 3, 32, 6, 9, 8, 9, 3, 9, 9,
                                6, 1,   9,   8, 7, 4, 8,  7, 6, 2, 7, 7, 7};
        for (int k = 0; k < 26; ++k) x0(k) = x0v[k];
        arma::vec hgeo = load_ascii(hand_dir + "/hgeo.dat", 20);
        arma::vec hrad = load_ascii(hand_dir + "/rad.dat", 48);
        for (int k = 0; k < 20; ++k) hgeo(k) = hgeo(k) / 10.;
        for (int k = 0; k < 48; ++k) hrad(k) = hrad(k) / 10.;
        handmodel hand(hgeo, spc, tbnum, fgnum, hcmc, hrad);

        observedmodel observation;
        std::ostringstream f0;
        f0 << std::setw(6) << std::setfill('0') << first << "_depth.bin";
        observation.init_observation(frames_dir, f0.str(), true, 240, 320, 241.42, full == 0);
        costfunc optfunc(&hand, &observation);

        // testmodel.cpp:74-111
        arma::vec ub(26), lb(26), sd(26);
        const double tu[4] = {15, 90, 110, 90}, tl[4] = {-15, 0, 0, 0};
        for (int k = 0; k < 26; ++k) {
            ub(k) = k < 3 ? 180 : k < 6 ? 100 : tu[(k - 6) % 4];
            lb(k) = k < 3 ? -180 : k < 6 ? -100 : tl[(k - 6) % 4];
            sd(k) = (k >= 3 && k < 6) ? 7.0 : 9.0;
        }
        double w = 0.7298, c1 = 1.49618, c2 = 1.49618, minstep = 1e-8, minfunc = 1e-8;
        PSO optimiser;
        optimiser.set_pso_params(ub, lb, sd, w, c1, c2, maxiter, minstep, minfunc);

        std::ofstream poses;
        if (!pose_out.empty()) {
            poses.open(pose_out);
            poses.precision(17);
        }
        const auto t0 = std::chrono::steady_clock::now();
        for (int frame = first; frame < first + nframes; ++frame) {
            std::ostringstream ss;
            ss << std::setw(6) << std::setfill('0') << frame;
            observation.next_frame(ss.str() + "_depth.bin");
            double c;
            if (fused) {
                c = optimiser.track_frame(optfunc, x0, num_p, refine != 0);
            } else {
                if (refine) optimiser.refine_init_pose(x0, optfunc);
                arma::vec bestp(26);
                optimiser.pso_evolve(optfunc, x0, num_p, bestp);
                c = optfunc.cal_cost(bestp);
                x0 = bestp;
            }
            std::cout << "frame" << ss.str() << "-cost: " << c << std::endl;
            if (poses.is_open()) {
                for (int k = 0; k < 26; ++k) poses << x0(k) << (k < 25 ? ' ' : '\n');
            }
        }
        const double s =
            std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
        std::cout.unsetf(std::ios::floatfield);
        std::cout.precision(6);
        std::cout << "frames " << nframes << " wall " << s << " s  tracked_fps " << nframes / s
                  << std::endl;
    } catch (const std::exception &e) {
        std::cerr << e.what() << std::endl;
        return 1;
    }
    return 0;
}
