"""The endomorphism subgroup criteria the device decoder uses (hbbft_amd/csrc/k_wire.hip, round 6),
checked on the CPU with the oracle's arithmetic against the definition r * P == O:
  G1: P in G1 <=> phi(P) == [-x^2] P, phi(x, y) = (beta x, y)
  G2: P in G2 <=> psi(P) == [x] P
on subgroup points (equality holds), on random on-curve points and on points of every prime order
dividing the cofactors h1 / h2 (equality fails).  A non-subgroup point passes the criterion only
if its cofactor part does, and that part is a sum of prime-power-order components, so the torsion
points of each prime power are the cases that matter."""
import random

from oracle import bls12_381 as C
from tests import subgroup_points as S

BETA = 0x5F19672FDF76CE51BA69C6076A0F77EADDB3A93BE6F89688DE17D813620A00022E01FFFFFFFEFFFE
PSI_C1 = C.f2_inv(C.f2_pow((1, 1), (C.P - 1) // 3))
PSI_C2 = C.f2_inv(C.f2_pow((1, 1), (C.P - 1) // 2))


def phi(pt):
    return None if pt is None else (BETA * pt[0] % C.P, pt[1])


def psi(pt):
    if pt is None:
        return None
    return (C.f2_mul(C.f2_conj(pt[0]), PSI_C1), C.f2_mul(C.f2_conj(pt[1]), PSI_C2))


def g1_criterion(pt):
    return phi(pt) == C.g1_neg(C.g1_mul(pt, C.X_ABS ** 2)) if pt is not None else True


def g2_criterion(pt):
    return psi(pt) == C.g2_neg(C.g2_mul(pt, C.X_ABS)) if pt is not None else True


def test_g1_criterion_equals_r_mul():
    for label, pt in S.sample(False, 40, seed=601):
        assert C.g1_on_curve(pt)
        want = C.g1_mul(pt, C.R) is None
        assert g1_criterion(pt) == want, label
        assert want == (label == "subgroup"), label


def test_g2_criterion_equals_r_mul():
    for label, pt in S.sample(True, 12, seed=602):
        assert C.g2_on_curve(pt)
        want = C.g2_mul(pt, C.R) is None
        assert g2_criterion(pt) == want, label
        assert want == (label == "subgroup"), label


def test_criteria_determinants():
    """Why the criteria are exact on the whole curve: on the l-power torsion (l != r) the map
    phi + [x^2] has determinant N(-x^2 - phi) = x^4 - x^2 + 1 = r (phi^2 + phi + 1 = 0), and
    psi - [x] has x^2 - t x + p = p - x = h1 r (psi^2 - t psi + p = 0, t = x + 1): both are units
    mod every prime of the cofactors, so neither map has a non-zero kernel off the r-torsion."""
    x = -C.X_ABS
    assert x ** 4 - x ** 2 + 1 == C.R
    assert x * x - (x + 1) * x + C.P == C.H1 * C.R
    for l, _ in S.H1_FACTORS:
        assert C.R % l != 0
    for l, _ in S.h2_factors():
        assert (C.H1 * C.R) % l != 0
