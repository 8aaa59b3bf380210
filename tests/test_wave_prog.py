"""The stage programs of the wave-per-check pairing kernel (k_wave.hip), executed by the exact
emulator of tools/gen_wave_prog.py, against the oracle's pairing (oracle/bls12_381.py).

This pins the programs -- formulas, scheduling, slot reuse, gating of inactive pairs and the
table-line plumbing -- without a GPU; tests/test_gpu_wave.py then checks the kernel that runs them.
"""
import os
import random
import sys

import pytest

from oracle import bls12_381 as C

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))
import gen_wave_prog as W  # noqa: E402


@pytest.fixture(scope="module")
def progs():
    return W.build()


def wbasis(f12):
    (c0, c1) = f12
    out = []
    for i in range(3):
        out.append(tuple(x % C.P for x in c0[i]))
        out.append(tuple(x % C.P for x in c1[i]))
    return [out[0], out[1], out[2], out[3], out[4], out[5]]


def tower_to_w(f12):
    c0, c1 = f12
    return [tuple(v % C.P for v in c0[0]), tuple(v % C.P for v in c1[0]), tuple(v % C.P for v in c0[1]),
            tuple(v % C.P for v in c1[1]), tuple(v % C.P for v in c0[2]), tuple(v % C.P for v in c1[2])]


def cube(f):
    return C.f12_mul(C.f12_mul(f, f), f)


ONE_W = [(1, 0)] + [(0, 0)] * 5


def test_committed_include_is_current(progs, tmp_path):
    p = tmp_path / "wave_prog.inc"
    W.emit(progs, str(p))
    with open(os.path.join(ROOT, "hbbft_amd", "csrc", "wave_prog.inc")) as f:
        assert f.read() == p.read_text(), "regenerate with python tools/gen_wave_prog.py"


def test_program_shape(progs):
    for m, v in progs["variants"].items():
        assert v["nstages_miller"] <= 215 and v["nstages_fe"] <= 80, m
        assert progs["nslots"] <= 136


TWO_SIDED = [m for m in W.MODES if m != "W1J"]  # W1J: one pair per wave (test_single_pair_homogeneous_walk)


@pytest.mark.parametrize("mode", TWO_SIDED)
def test_single_pairing_value(progs, mode):
    rnd = random.Random(7 + W.MODES.index(mode))
    Pp = C.g1_mul(C.G1_GEN, rnd.randrange(1, C.R))
    Q = C.g2_mul(C.G2_GEN, rnd.randrange(1, C.R))
    got = W.emulate(progs["variants"][mode], [(Pp, Q, False), (None, Q, False)], conj=True)
    assert got == tower_to_w(cube(C.pairing(Pp, Q)))


@pytest.mark.parametrize("mode", TWO_SIDED)
def test_pairing_equality(progs, mode):
    rnd = random.Random(11 + W.MODES.index(mode))
    a, b = rnd.randrange(1, C.R), rnd.randrange(1, C.R)
    # e(a g1, b g2) == e(g1, ab g2): the verifier's product with P2 negated is 1
    P1, Q1 = C.g1_mul(C.G1_GEN, a), C.g2_mul(C.G2_GEN, b)
    Q2 = C.g2_mul(C.G2_GEN, a * b % C.R)
    v = progs["variants"][mode]
    assert W.emulate(v, [(P1, Q1, False), ("GEN", Q2, True)]) == ONE_W
    Q2bad = C.g2_mul(C.G2_GEN, (a * b + 1) % C.R)
    assert W.emulate(v, [(P1, Q1, False), ("GEN", Q2bad, True)]) != ONE_W


def test_inactive_pairs(progs):
    rnd = random.Random(3)
    Pp = C.g1_mul(C.G1_GEN, rnd.randrange(1, C.R))
    Q = C.g2_mul(C.G2_GEN, rnd.randrange(1, C.R))
    v = progs["variants"]["WT"]
    # both pairs at infinity -> the value is 1; one pair inactive -> the other pair's value
    assert W.emulate(v, [(None, Q, False), (Pp, None, False)]) == ONE_W
    got = W.emulate(v, [(None, Q, False), (Pp, Q, False)], conj=True)
    assert got == tower_to_w(cube(C.pairing(Pp, Q)))


def test_split_master_check(progs):
    """The split master check of hbh_combine_verify_g2: partial Miller values of pairs (lambda_k g1,
    sigma_k) and (-mpk, H), two pairs per wave (miller-only mode), multiplied by the MULF program and
    one final exponentiation -- 1 exactly when the product of the pairings is 1."""
    rnd = random.Random(5)
    a = [rnd.randrange(1, C.R) for _ in range(3)]
    b = [rnd.randrange(1, C.R) for _ in range(3)]
    c = sum(x * y for x, y in zip(a, b)) % C.R
    v = progs["variants"]["WW"]
    P = [C.g1_mul(C.G1_GEN, x) for x in a]
    Q = [C.g2_mul(C.G2_GEN, y) for y in b]
    for cc, want in ((c, True), ((c + 1) % C.R, False)):
        mpk = C.g1_mul(C.G1_GEN, cc)
        fs = [W.emulate_miller(v, [(P[0], Q[0], False), (P[1], Q[1], False)]),
              W.emulate_miller(v, [(P[2], Q[2], False), (mpk, C.G2_GEN, True)])]
        assert (W.emulate_prod_fe(v, fs) == ONE_W) == want
    # an inactive padding pair (P = O) contributes 1
    mpk = C.g1_mul(C.G1_GEN, a[0] * b[0] % C.R)
    f = W.emulate_miller(v, [(P[0], Q[0], False), (None, Q[1], False)])
    g = W.emulate_miller(v, [(mpk, C.G2_GEN, True), (None, Q[2], False)])
    assert W.emulate_prod_fe(v, [f, g]) == ONE_W


def test_split_master_check_jacobian_p(progs):
    """Mode WWJ (the split master check's lambda_k g1 straight from the device tree, no inversion):
    P = (X, Y, Z) Jacobian; the Miller value differs from the affine one by an Fp factor, the final
    exponentiation's output does not."""
    rnd = random.Random(9)
    a = [rnd.randrange(1, C.R) for _ in range(3)]
    b = [rnd.randrange(1, C.R) for _ in range(3)]
    c = sum(x * y for x, y in zip(a, b)) % C.R
    vj, v = progs["variants"]["WWJ"], progs["variants"]["WW"]

    def jac(pt):
        z = rnd.randrange(1, C.P)
        return ("JAC", (pt[0] * z * z % C.P, pt[1] * z * z * z % C.P, z))

    P = [C.g1_mul(C.G1_GEN, x) for x in a]
    Q = [C.g2_mul(C.G2_GEN, y) for y in b]
    mpk = C.g1_mul(C.G1_GEN, c)
    negmpk = (mpk[0], (-mpk[1]) % C.P)
    fs = [W.emulate_miller(vj, [(jac(P[0]), Q[0], False), (jac(P[1]), Q[1], False)]),
          W.emulate_miller(vj, [(jac(P[2]), Q[2], False), (("JAC", (negmpk[0], negmpk[1], 1)), C.G2_GEN, False)])]
    assert W.emulate_prod_fe(v, fs) == ONE_W
    # a Jacobian P at infinity (Z = 0) is an inactive pair; the same value as the affine program
    f = W.emulate_miller(vj, [(jac(P[0]), Q[0], False), (("JAC", (1, 1, 0)), Q[1], False)])
    g = W.emulate_miller(v, [(P[0], Q[0], False), (None, Q[1], False)])
    assert W.emulate_prod_fe(v, [f]) == W.emulate_prod_fe(v, [g])


def test_single_pair_homogeneous_walk(progs):
    """Mode W1J (one pair per wave, homogeneous-projective walk, Jacobian P): after the final
    exponentiation the same value as the two-pair Jacobian walk with the second pair inactive, and the
    split master check's product over one-pair waves is 1 exactly for a valid relation."""
    rnd = random.Random(13)
    v1, v = progs["variants"]["W1J"], progs["variants"]["WW"]
    assert v1["nstages_miller"] <= 150

    def jac(pt):
        z = rnd.randrange(1, C.P)
        return ("JAC", (pt[0] * z * z % C.P, pt[1] * z * z * z % C.P, z))

    a, b = rnd.randrange(1, C.R), rnd.randrange(1, C.R)
    Pp, Q = C.g1_mul(C.G1_GEN, a), C.g2_mul(C.G2_GEN, b)
    got = W.emulate_prod_fe(v, [W.emulate_miller(v1, [(jac(Pp), Q, False)])])
    want = W.emulate_prod_fe(v, [W.emulate_miller(v, [(Pp, Q, False), (None, Q, False)])])
    assert got == want
    assert W.emulate_prod_fe(v, [W.emulate_miller(v1, [(("JAC", (1, 1, 0)), Q, False)])]) == ONE_W
    # e(a g1, b g2) e(-(ab) g1, g2) == 1 over two one-pair waves; off by one -> != 1
    for k, want1 in ((a * b % C.R, True), ((a * b + 1) % C.R, False)):
        m = C.g1_mul(C.G1_GEN, k)
        fs = [W.emulate_miller(v1, [(jac(Pp), Q, False)]),
              W.emulate_miller(v1, [(jac((m[0], (-m[1]) % C.P)), C.G2_GEN, False)])]
        assert (W.emulate_prod_fe(v, fs) == ONE_W) == want1


# ---------------------------------------------------------------- the 64-pair set (k_wave64, round 6)
@pytest.fixture(scope="module")
def progs64():
    return W.build(64)


def test_committed_include64_is_current(progs64, tmp_path):
    p = tmp_path / "wave_prog64.inc"
    W.emit(progs64, str(p), ns="hbw64")
    with open(os.path.join(ROOT, "hbbft_amd", "csrc", "wave_prog64.inc")) as f:
        assert f.read() == p.read_text(), "regenerate with python tools/gen_wave_prog.py"


def test_program_shape64(progs, progs64):
    """Combined lines (op_mul_ll beside f^2, one op_mul_fl per step) and the homogeneous walk: two
    stages per step where the 32-pair walking programs take three."""
    for m, v in progs64["variants"].items():
        assert v["nstages_miller"] <= 150 and v["nstages_fe"] == progs["variants"][m]["nstages_fe"], m
        assert max(st.npairs for st in v["stages_miller"]) <= 64
    assert progs["variants"]["TT"]["nstages_miller"] <= 140  # the 32-pair TT takes the combined lines too
    assert progs64["nslots"] <= 170


@pytest.mark.parametrize("mode", W.MODES64)
def test_single_pairing_value64(progs64, mode):
    rnd = random.Random(17 + W.MODES64.index(mode))
    Pp = C.g1_mul(C.G1_GEN, rnd.randrange(1, C.R))
    Q = C.g2_mul(C.G2_GEN, rnd.randrange(1, C.R))
    got = W.emulate(progs64["variants"][mode], [(Pp, Q, False), (None, Q, False)], conj=True)
    assert got == tower_to_w(cube(C.pairing(Pp, Q)))


@pytest.mark.parametrize("mode", W.MODES64)
def test_pairing_equality64(progs64, mode):
    rnd = random.Random(21 + W.MODES64.index(mode))
    a, b = rnd.randrange(1, C.R), rnd.randrange(1, C.R)
    P1, Q1 = C.g1_mul(C.G1_GEN, a), C.g2_mul(C.G2_GEN, b)
    Q2 = C.g2_mul(C.G2_GEN, a * b % C.R)
    v = progs64["variants"][mode]
    assert W.emulate(v, [(P1, Q1, False), ("GEN", Q2, True)]) == ONE_W
    Q2bad = C.g2_mul(C.G2_GEN, (a * b + 1) % C.R)
    assert W.emulate(v, [(P1, Q1, False), ("GEN", Q2bad, True)]) != ONE_W


@pytest.mark.parametrize("mode", ["WT", "TW"])
def test_inactive_pairs64(progs64, mode):
    rnd = random.Random(23)
    Pp = C.g1_mul(C.G1_GEN, rnd.randrange(1, C.R))
    Q = C.g2_mul(C.G2_GEN, rnd.randrange(1, C.R))
    v = progs64["variants"][mode]
    assert W.emulate(v, [(None, Q, False), (Pp, None, False)]) == ONE_W
    got = W.emulate(v, [(None, Q, False), (Pp, Q, False)], conj=True)
    assert got == tower_to_w(cube(C.pairing(Pp, Q)))
    got = W.emulate(v, [(Pp, Q, False), (None, Q, False)], conj=True)
    assert got == tower_to_w(cube(C.pairing(Pp, Q)))
