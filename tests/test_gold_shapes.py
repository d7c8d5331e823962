"""The Goldstein speculation tables of k_refine / k_opt_descent (gold_shape in
csrc/hpe_kernels.hip) against the serial search they speculate (PSO.cpp:438-480).

A round evaluates the nodes of a shape -- decision prefixes relative to the bracket state at
the round's start -- and the walk then replays the serial rules from node 0 along the dn /
up pointers.  The speculation is exact only if every shape is prefix-closed, its pointers
name exactly its children, node 0 is the round's own alpha, and a path fits the walk's six
levels.  These checks read the packed words from the kernel source and replay random and
exhaustive decision strings through them with the kernel's walk, comparing the trial
sequence (alphas bit for bit, the evaluation count, tk) with the serial goldstein.  CPU only.
"""
import itertools
import random
import re

import pytest

import hand_data

SRC = hand_data.ROOT / "hand-pose-estimation_amd" / "csrc" / "hpe_kernels.hip"
POLICIES = ("GOLD_BALANCED", "GOLD_8", "GOLD_4", "GOLD_OPT8", "GOLD_MIX")


def _tables():
    src = SRC.read_text()
    body = src[src.index("__device__ __forceinline__ GoldShape gold_shape(int ctx)"):]
    body = body[:body.index("};")]
    rows = re.findall(r"\{(\d+), 0x([0-9a-f]+)ull, 0x([0-9a-f]+)u, 0x([0-9a-f]+)u\}", body)
    return [(int(n), int(nb, 16), int(dn, 16), int(up, 16)) for n, nb, dn, up in rows]


def _decode(row):
    n, nb, dn, up = row
    paths = []
    for j in range(n):
        b = (nb >> (8 * j)) & 0xff
        ln, bits = b >> 5, b & 31
        paths.append("".join("U" if (bits >> k) & 1 else "D" for k in range(ln)))
    kids = [((dn >> (4 * j)) & 15, (up >> (4 * j)) & 15) for j in range(8)]
    return paths, kids


def test_table_has_every_policy_and_context():
    rows = _tables()
    assert len(rows) == 3 * len(POLICIES)
    src = SRC.read_text()
    for k, name in enumerate(POLICIES):
        assert re.search(rf"#define {name} {k}\b", src), name


@pytest.mark.parametrize("row", range(3 * len(POLICIES)))
def test_shape_is_prefix_closed_with_exact_pointers(row):
    paths, kids = _decode(_tables()[row])
    n = len(paths)
    assert 1 <= n <= 8  # one node per wave of the 8-wave workgroup
    assert paths[0] == ""  # node 0 = the round's current alpha
    assert len(set(paths)) == n
    idx = {p: j for j, p in enumerate(paths)}
    for j, p in enumerate(paths):
        assert len(p) <= 5  # 5 decision bits per packed byte
        if p:
            assert p[:-1] in idx, p  # prefix-closed
        for c, child in zip("DU", kids[j]):
            if p + c in idx:
                assert child == idx[p + c], (p, c)
            else:
                assert child == 15, (p, c)  # outside the shape: the round ends there
    for j in range(n, 8):
        assert kids[j] == (15, 15)


# ---- the serial search and the kernel's speculated form, on decision strings ----------
def gold_up(a, b, alpha):
    a = alpha
    up, mid = 2 * alpha, 0.5 * (alpha + b)
    return a, b, (mid if mid < up else up)


def gold_down(a, b, alpha):
    return a, alpha, 0.5 * (a + alpha)


def serial(decide):
    """goldstein with trial outcomes from decide(trial, alpha) in {'D', 'U', 'A'}."""
    A, B, alpha, trials = 0.0, 1e100, 0.5, []
    for it in range(30):
        d = decide(it, alpha)
        trials.append(alpha)
        if d == "A":
            return alpha, trials
        A, B, alpha = (gold_up if d == "U" else gold_down)(A, B, alpha)
    return 0.0, trials


def speculated(decide, policy_rows):
    """gold_tree's rounds: nodes replayed from the round's start state, then the walk."""
    A, B, alpha, ctx, it, evaluated, rounds = 0.0, 1e100, 0.5, 0, 0, [], 0
    while True:
        paths, kids = _decode(policy_rows[ctx])
        node_alpha = []
        for p in paths:
            a, b, al = A, B, alpha
            for c in p:
                a, b, al = (gold_up if c == "U" else gold_down)(a, b, al)
            node_alpha.append(al)
        rounds += 1
        node = 0
        for _ in range(6):  # the kernel's unrolled walk
            if node >= 15:
                break
            if it >= 30:
                return 0.0, evaluated, rounds
            it += 1
            assert node_alpha[node] == alpha  # the node IS the serial trial, bit for bit
            evaluated.append(node_alpha[node])
            d = decide(it - 1, alpha)
            if d == "A":
                return alpha, evaluated, rounds
            if d == "U":
                A, B, alpha = gold_up(A, B, alpha)
                node, ctx = kids[node][1], 2
            else:
                A, B, alpha = gold_down(A, B, alpha)
                node, ctx = kids[node][0], 1
        if it >= 30:
            return 0.0, evaluated, rounds


def _check(decisions, rows):
    def decide(k, alpha):
        return decisions[k] if k < len(decisions) else "D"
    tk, trials = serial(decide)
    tk2, ev, rounds = speculated(decide, rows)
    assert tk2 == tk and ev == trials, decisions
    return rounds


@pytest.mark.parametrize("pol", range(len(POLICIES)))
def test_walk_replays_serial_search_exhaustive(pol):
    rows = _tables()[3 * pol: 3 * pol + 3]
    for n in range(0, 9):  # every decision string up to 8 trials, then acceptance
        for s in itertools.product("DU", repeat=n):
            _check("".join(s) + "A", rows)


@pytest.mark.parametrize("pol", range(len(POLICIES)))
def test_walk_replays_serial_search_random(pol):
    rows = _tables()[3 * pol: 3 * pol + 3]
    rng = random.Random(1000 + pol)
    for _ in range(3000):
        n = rng.randrange(0, 34)  # beyond 30: the search fails (tk = 0)
        s = "".join(rng.choice("DDDU") for _ in range(n))
        _check(s + ("A" if rng.random() < 0.8 else ""), rows)


def test_runs_need_fewer_rounds_with_context_shapes():
    rows = _tables()
    bal, g8 = rows[0:3], rows[3:6]
    # the commonest refine strings: context shapes never need more
    for s in ("DDDDA", "UA", "UUA", "UUUA", "A", "DDDDDDDDA"):
        assert _check(s, g8) <= _check(s, bal), s
