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


def g2_criterion_on_isomorph(pt):
    """The decoder's two-role form (k_g2_decompress, session 2 of round 6): with rhs = x^3 + b = y^2
    the isomorphism iota(X, Y) = (y^2 X, y^3 Y) sends P to P' = (rhs x, rhs^2) -- known from x alone, so
    [|x|] P' runs beside the square root -- and psi(P) to (C1 rhs conj(x), C2 rhs N(y)), N(y) = y conj(y)
    in Fp (the same for both roots).  iota commutes with [k] (the a = 0 formulas never read b), so
    psi(P) == -[|x|] P  <=>  [|x|] P' == (C1 rhs conj(x), -C2 rhs N(y))."""
    if pt is None:
        return True
    x, y = pt
    rhs = C.f2_add(C.f2_mul(C.f2_sqr(x), x), C.B2)
    assert not C.f2_is_zero(rhs)  # #E'(Fp2) = h2 r is odd: no point has y = 0
    Pp = (C.f2_mul(rhs, x), C.f2_sqr(rhs))
    J = (C.F2_ONE, C.F2_ONE, C.F2_ZERO)
    for bit in bin(C.X_ABS)[2:]:
        J = C._j2_dbl(J)
        if bit == "1":
            J = C._j2_add_aff(J, Pp)
    norm = (y[0] * y[0] + y[1] * y[1]) % C.P
    want = (C.f2_mul(C.f2_mul(rhs, C.f2_conj(x)), PSI_C1), C.f2_neg(C.f2_muls(C.f2_mul(rhs, PSI_C2), norm)))
    return C._j2_to_aff(J) == want


def test_g2_criterion_on_isomorph_equals_r_mul():
    for label, pt in S.sample(True, 12, seed=603):
        want = C.g2_mul(pt, C.R) is None
        assert g2_criterion_on_isomorph(pt) == want, label
        neg = C.g2_neg(pt)
        assert g2_criterion_on_isomorph(neg) == want, label


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
