"""Diagnostic: phase-skeleton builds of the wave-form generation (k_pso_gen_w) for SQ
instruction attribution.  Each variant is the product source with ONE
phase compiled out (results invalid), built into hand-pose-estimation_amd/libhpe_skel_<v>.so
for tools/skel/run_sq.sh (HPE_LIB_VARIANT).  The product source is not modified.
Usage: python tools/skel/build_variants.py [variant ...]"""
import shutil
import subprocess
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[2]
PKG = ROOT / "hand-pose-estimation_amd"
EDITS = {
    "base": [],
    # FK: the spheres stay whatever the workspace held (no sincos, no chain)
    "nofk": [("hpe_device.hpp", "    SphXYZ own;\n    fk_wave(f, H, &own);\n    const DepthG dg = depth_issue_at(own, l, o, H);",
              "    SphXYZ own{0.0, 0.0, 0.0};\n    const DepthG dg = depth_issue_at(own, l, o, H);")],
    # the correspondence search + alignment
    "nosearch": [("hpe_device.hpp", "    double al = search_align_lane(f, cv, H, pre);",
                  "    double al = 0.0;")],
    # the fp64 alignment residual inside the search (the match is still found)
    "noalign": [("hpe_device.hpp", "        const double e = sqrt((dx * dx + dy * dy) + dz * dz) - r.cr;\n        acc += e * e;\n        q = qn;",
                 "        acc += dx + (dy + dz);\n        q = qn;")],
    # the informant's pbest row (a dependent global load in the wave form)
    "norow": [("hpe_kernels.hip", "            const double pbn = use_ext ? exr : sw.inbox[ib_index(sw, (g - 1) & 1, var, ic, islot) + 2 + l];",
               "            const double pbn = use_ext ? exr : xo + 1e-3 * islot;")],
    # the workgroup form's depth term (wave 0's projection, gathers and finish)
    "blknodepth": [("hpe_device.hpp", "    if (t < 64 && with_depth) dg = (FK || own_w0) ? depth_issue_at(own, t, o, H) : depth_issue(sm.fk, t, o, H);",
                    "    if (false) dg = depth_issue(sm.fk, t, o, H);")],
    # the workgroup form's correspondence search (cal_cost at N <= 256)
    "blknosearch": [("hpe_device.hpp", "    else al = search_align<NT, false>(sm.fk, cv, H, nullptr, pre, -1, g_ts);",
                     "    else al = 0.0;")],
    # mutation check of the filter tie test: the filter's estimate accepted without its bound
    # (no exact fallback; results wrong on near ties)
    "nofallback": [("hpe_device.hpp", "        if ((v2 - v1 > E * 2.0f + M) && (E < 0.5f)) {\n            const int ic = (int)(m.m & 63u);",
                    "        if (true) {\n            const int ic = (int)(m.m & 63u);"),
                   ("hpe_device.hpp", "    if ((v2 - v1 > E * 2.0f + M) && (E < 0.5f)) {\n        const int ic = (int)(r.m & 63u);",
                    "    if (true) {\n        const int ic = (int)(r.m & 63u);")],
    # the wave form with eight waves per workgroup (same residency: two workgroups per CU)
    "wpb8": [("hpe_kernels.hip", "#define PW_WPB 4", "#define PW_WPB 8"),
             ("hpe_kernels.hip", "__launch_bounds__(PW_NT, WPP == 2 ? 2 : 4)", "__launch_bounds__(PW_NT, WPP == 2 ? 1 : 2)")],
    # every depth / DT gather at pixel 0 (the gathers' latency and traffic)
    "nogather": [("hpe_device.hpp", "    const int pix = d.in ? (int)dy * HPE_IMG_W + (int)dx : 0;\n",
                  "    const int pix = 0;\n")],
    # the workgroup form's inbox payload rows (waves 1..7's round-1 loads)
    "blknorow": [("hpe_kernels.hip", "            a[k] = src[vr * var_stride + off];",
                  "            a[k] = (double)(vr + off);")],
    # both (the rows' own traffic, with the gathers' taken out)
    "blknorow_nogather": [("hpe_kernels.hip", "            a[k] = src[vr * var_stride + off];",
                           "            a[k] = (double)(vr + off);"),
                          ("hpe_device.hpp", "    const int pix = d.in ? (int)dy * HPE_IMG_W + (int)dx : 0;\n",
                           "    const int pix = 0;\n")],
    # the rp / rg draws of the wave form
    "nophilox": [("hpe_kernels.hip", "    const double rd = philox_u01(sw.seed, l < HPE_DOF ? ST_RP : ST_RG, g, ic, dl);",
                  "    const double rd = 0.25 + dl * 1e-3;")],
}


def build(v):
    d = Path(f"/tmp/skel_{v}")
    if d.exists():
        shutil.rmtree(d)
    (d / "hand-pose-estimation_amd").mkdir(parents=True)
    shutil.copytree(PKG / "csrc", d / "hand-pose-estimation_amd" / "csrc")
    shutil.copytree(ROOT / "include", d / "include")
    for f, old, new in EDITS[v]:
        p = d / "hand-pose-estimation_amd" / "csrc" / f
        s = p.read_text()
        assert s.count(old) == 1, (v, f, old[:60])
        p.write_text(s.replace(old, new))
    out = PKG / f"libhpe_skel_{v}.so"
    cmd = ["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "-fPIC", "-ffp-contract=off", "-fno-slp-vectorize",
           "--offload-arch=gfx950", "-shared", "-o", str(out), "csrc/hpe_kernels.hip", "csrc/hpe_host.cpp"]
    subprocess.run(cmd, cwd=d / "hand-pose-estimation_amd", check=True)
    print(v, out)


if __name__ == "__main__":
    vs = sys.argv[1:] or list(EDITS)
    procs = []
    for v in vs:
        build(v)
