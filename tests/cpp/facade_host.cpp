// Host-only façade checks (no GPU call): arma_lite semantics, the reference's size-error
// behaviour (print + zero-fill, handmodel.cpp:150-208) and the .bin abort
// (observedmodel.cpp:290-293, when argv[1] == "abort").
#include <cstdio>
#include <cstring>
#include <stdexcept>

#include "hpe_facade.hpp"

int main(int argc, char **argv) {
    if (argc > 1 && std::strcmp(argv[1], "abort") == 0) {
        observedmodel o;
        o.init_observation("/nonexistent/", "000000_depth.bin", true, 240, 320, 241.42, true);
        return 0;  // not reached
    }
    arma::vec x(5);
    x << 1 << 2 << 3 << 4 << 5 << arma::endr;
    arma::mat M(2, 3);
    for (int i = 0; i < 6; ++i) M(i) = i;
    int ok = (x(4) == 5) && (M(1, 2) == 5) && (M.memptr()[3] == 3) && (M.n_elem == 6);
    arma::vec bad(3), spc{-1.86, -1.86, 0, 1.91, 3.84}, cmc{150, 107.5, 89.8, 76.5, 59.6};
    arma::vec tb{2, 2, 2, 2}, fg{4, 2, 2, 2}, rad(48);
    handmodel h(bad, spc, tb, fg, cmc, rad);  // 3 != 20 geometry values
    arma::vec g = h.get_hand_geo();
    ok = ok && g.n_elem == 20;
    for (int i = 0; i < 20; ++i) ok = ok && g(i) == 0.0;
    ok = ok && h.get_spacing()(4) == 3.84 && h.get_radii()->n_elem == 48;
    // PSO::dim_restore (PSO.cpp:160-180): 22 -> 26 with DIP = 2/3 PIP, hand-written values
    {
        PSO pso;
        arma::vec in(22), out(26);
        for (int i = 0; i < 22; ++i) in(i) = 1.5 * i - 7.25;
        pso.dim_restore(in, out);
        const int src[26] = {0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, -12,
                             13, 14, 15, -15, 16, 17, 18, -18, 19, 20, 21, -21};
        for (int k = 0; k < 26; ++k) {
            const double want = src[k] >= 0 ? in(src[k]) : 2. / 3 * in(-src[k]);
            ok = ok && out(k) == want;
        }
        ok = ok && out(13) == 2. / 3 * 10.75 && out(25) == 2. / 3 * 24.25;
        arma::vec small(20);
        bool threw = false;
        try {
            pso.dim_restore(small, out);
        } catch (const std::logic_error &) {
            threw = true;
        }
        ok = ok && threw;
        if (!ok) std::printf("dim_restore mismatch\n");
    }
    std::printf("facade_host %s\n", ok ? "ok" : "FAILED");
    return ok ? 0 : 1;
}
