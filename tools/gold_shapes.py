"""Diagnostic: fit the Goldstein speculation shapes of gold_tree (hpe_kernels.hip) from the
C oracle's decision logs (ora_set_gold_log): the oracle tracks synthetic bench sequences
(refine_init_pose + pso_evolve per frame, testmodel.cpp:124-138) or runs pso_optimise, every
Goldstein search (PSO.cpp:438-480) is logged as its decision string ("DDDDA": four Armijo
failures then acceptance), and for a node budget K a shape per context (the previous round's
last decision: a search's first round, "down", "up") is fitted by coordinate descent over
all prefix-closed node sets of size K, minimising the speculated rounds.  Prints the round
counts of each budget, the cross-validation over the sequences and the packed table entries
gold_shape() takes, then the per-context choice of 4 or 8 nodes by expected round time
(GOLD_MIX).  CPU only.

Usage: python tools/gold_shapes.py [refine|optimise] [frames] [seeds...]
"""
import ctypes as C
import itertools
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT / "oracle"), str(ROOT / "tests"), str(ROOT / "hand-pose-estimation_amd")]
import hand_data  # noqa: E402
import oracle_c  # noqa: E402
import oracle_np  # noqa: E402
from hpe import synth  # noqa: E402

CTX = ("", "D", "U")


def decision_logs(mode, frames, seed):
    o = oracle_c.load(build=False)
    o.lib.ora_set_gold_log.argtypes = [C.POINTER(C.c_uint64), C.c_int]
    o.lib.ora_gold_log_count.restype = C.c_int
    cap = 1 << 20
    buf = np.zeros(cap, dtype=np.uint64)
    o.lib.ora_set_gold_log(buf.ctypes.data_as(C.POINTER(C.c_uint64)), cap)
    geo, rad = hand_data.geometry_cm()
    h, nh = o.hand(geo, rad), oracle_np.Hand(geo, rad)
    ub, lb, sd = oracle_np.reference_bounds()
    poses = synth.trajectory(frames, seed, revert=0.02)  # the bench sequence's model
    x = poses[0].copy()
    for f in range(frames):
        obs = o.preprocess(oracle_np.render_depth_mm(nh, poses[f]))
        if mode == "refine":
            x, _ = o.refine(h, obs, x)
            x, _, _ = o.pso_evolve(h, obs, x, 256, 31, lb, ub, sd, seed=1000)
        else:
            x, _, _ = o.pso_optimise(h, obs, x, 32, 6, lb, ub, sd, 0.7298, 1.49618, 1.49618,
                                     seed=1000)
    n = min(o.lib.ora_gold_log_count(), cap)
    o.lib.ora_set_gold_log(C.POINTER(C.c_uint64)(), 0)
    out = []
    for v in buf[:n].tolist():
        trials, acc = (v >> 32) & 0xff, (v >> 40) & 1
        dec = "".join("U" if (v >> k) & 1 else "D" for k in range(trials - (1 if acc else 0)))
        out.append(dec + ("A" if acc else "X"))
    return out


def rounds(policy, s):
    dec = s[:-1]
    n = len(s) if s[-1] == "A" else len(dec)  # trials
    pos = r = 0
    while pos < n:
        T = policy["" if pos == 0 else dec[pos - 1]]
        r += 1
        start = pos
        while pos < n and dec[start:pos] in T:
            pos += 1
    return r


def rounds_time(policy, nodes, s, t4=0.71):
    dec = s[:-1]
    n = len(s) if s[-1] == "A" else len(dec)
    pos, t = 0, 0.0
    while pos < n:
        c = "" if pos == 0 else dec[pos - 1]
        T = policy[c]
        t += t4 if nodes[c] <= 4 else 1.0
        start = pos
        while pos < n and dec[start:pos] in T:
            pos += 1
    return t


def total(policy, logs):
    return sum(rounds(policy, s) for s in logs)


def prefix_closed(k, maxdepth=6):  # nodes up to 5 decisions deep: gold_shape's 5 bits
    res = set()

    def grow(S):
        if len(S) == k:
            res.add(frozenset(S))
            return
        for s in list(S):
            for c in "DU":
                t = s + c
                if t not in S and len(t) < maxdepth:
                    grow(S | {t})
    grow(frozenset({""}))
    return list(res)


def fit(k, logs):
    sets = prefix_closed(k)
    pol = {c: sets[0] for c in CTX}
    cur = total(pol, logs)
    for _ in range(5):
        for c in CTX:
            for T in sets:
                q = dict(pol)
                q[c] = T
                v = total(q, logs)
                if v < cur:
                    cur, pol = v, q
    return pol, cur


def packed(pol):
    rows = []
    for c in CTX:
        nodes = sorted(pol[c], key=lambda x: (len(x), x))
        idx = {s: i for i, s in enumerate(nodes)}
        nb = dn = up = 0
        for i, s in enumerate(nodes):
            assert len(s) <= 5
            nb |= ((len(s) << 5) | sum(1 << k for k, ch in enumerate(s) if ch == "U")) << (8 * i)
        for i in range(8):
            s = nodes[i] if i < len(nodes) else None
            dn |= (idx.get(s + "D", 15) if s is not None else 15) << (4 * i)
            up |= (idx.get(s + "U", 15) if s is not None else 15) << (4 * i)
        rows.append(f"{{{len(nodes)}, 0x{nb:016x}ull, 0x{dn:08x}u, 0x{up:08x}u}},  // "
                    f"{c or 'first'}: " + " ".join(f"'{x}'" for x in nodes))
    return rows


def main():
    mode = sys.argv[1] if len(sys.argv) > 1 else "refine"
    frames = int(sys.argv[2]) if len(sys.argv) > 2 else 40
    seeds = [int(a) for a in sys.argv[3:]] or [0, 1, 2]
    logs = {s: decision_logs(mode, frames, s) for s in seeds}
    allg = [x for v in logs.values() for x in v]
    trials = sum(len(s) if s[-1] == "A" else len(s) - 1 for s in allg)
    print(f"{mode}: {len(allg)} searches, {trials} trials")
    import collections
    for s, c in collections.Counter(allg).most_common(8):
        print(f"   {c:6d} {s}")
    bal = frozenset("".join(p) for k in range(3) for p in itertools.product("DU", repeat=k))
    print("balanced depth 3 (7 nodes):", total({c: bal for c in CTX}, allg))
    fitted = {}
    for k in (4, 7, 8):
        pol, cur = fit(k, allg)
        fitted[k] = pol
        xv = {s: total(pol, v) for s, v in logs.items()}
        print(f"{k} nodes: {cur} rounds, per sequence {xv}")
        for r in packed(pol):
            print("    " + r)
    # round TIME: a round of <= 4 nodes runs one wave per SIMD, ~0.71 of an 8-node round
    # (measured: two node waves on a SIMD take ~1.4x one); per context, 4 or 8 nodes
    best = None
    for choice in itertools.product((4, 8), repeat=3):
        pol = {c: fitted[k][c] for c, k in zip(CTX, choice)}
        t = sum(rounds_time(pol, {c: k for c, k in zip(CTX, choice)}, s) for s in allg)
        print(f"time-weighted, nodes per context {dict(zip(('first', 'D', 'U'), choice))}: {t:.1f}")
        best = min(best or (t, choice), (t, choice))
    print("best:", best)


if __name__ == "__main__":
    main()
