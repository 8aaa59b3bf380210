"""Test points for the device decoder's subgroup tests (k_wire.hip, round 6): random on-curve
points of E(Fp) / E'(Fp2) (almost never in the prime-order subgroups) and points of every prime
order dividing the cofactors h1 (G1) and h2 (G2), alone and plus a subgroup point.  Built with the
oracle (test infrastructure)."""
import random

from oracle import bls12_381 as C

# h1 = 3 * 11^2 * 10177^2 * 859267^2 * 52437899^2
H1_FACTORS = [(3, 1), (11, 2), (10177, 2), (859267, 2), (52437899, 2)]
# h2 = 13^2 * 23^2 * 2713 * 11953 * 262069 * q (q a 448-bit prime)
_H2_SMALL = [(13, 2), (23, 2), (2713, 1), (11953, 1), (262069, 1)]


def h2_factors():
    q = C.H2
    for l, e in _H2_SMALL:
        q //= l ** e
    assert pow(3, q - 1, q) == 1 and q.bit_length() == 448
    return _H2_SMALL + [(q, 1)]


def _prod(fs):
    n = 1
    for l, e in fs:
        n *= l ** e
    return n


assert _prod(H1_FACTORS) == C.H1


def random_g1_on_curve(rng):
    while True:
        x = rng.randrange(C.P)
        y = C.fp_sqrt((x * x * x + C.B1) % C.P)
        if y is not None:
            return (x, y if rng.random() < 0.5 else (C.P - y) % C.P)


def random_g2_on_curve(rng):
    while True:
        x = (rng.randrange(C.P), rng.randrange(C.P))
        y = C.f2_sqrt(C.f2_add(C.f2_mul(C.f2_sqr(x), x), C.B2))
        if y is not None:
            return (x, y if rng.random() < 0.5 else C.f2_neg(y))


def torsion_points(g2, rng):
    """[(label, point)]: for each prime power l^e dividing the cofactor, [N / l^k] Q (k = 1..e) for
    a random on-curve Q (order dividing l^k, not 1; skipped when every try gives O, i.e. the l-part
    of the group is not cyclic of order l^e), the same plus a random subgroup point, and [r] Q (the
    whole cofactor part)."""
    mul, add = (C.g2_mul, C.g2_add) if g2 else (C.g1_mul, C.g1_add)
    rand = random_g2_on_curve if g2 else random_g1_on_curve
    gen = C.G2_GEN if g2 else C.G1_GEN
    fs = h2_factors() if g2 else H1_FACTORS
    n = (C.H2 if g2 else C.H1) * C.R
    out = []
    for l, e in fs:
        for k in range(1, e + 1):
            for _ in range(8):   # no point of order l^k when that part of the group is not cyclic
                t = mul(rand(rng), n // l ** k)
                if t is not None:
                    break
            if t is None:
                continue
            out.append(("order|%d^%d" % (l, k), t))
            out.append(("order|%d^%d + G" % (l, k), add(t, mul(gen, rng.randrange(1, C.R)))))
    for _ in range(2):
        out.append(("cofactor part", mul(rand(rng), C.R)))
    return out


def sample(g2, n_random, seed):
    """Points to decode: n_random random on-curve points, the torsion points, and subgroup points."""
    rng = random.Random(seed)
    rand = random_g2_on_curve if g2 else random_g1_on_curve
    pts = [("random", rand(rng)) for _ in range(n_random)]
    pts += torsion_points(g2, rng)
    mul, gen = (C.g2_mul, C.G2_GEN) if g2 else (C.g1_mul, C.G1_GEN)
    pts += [("subgroup", mul(gen, rng.randrange(1, C.R))) for _ in range(16)]
    return pts
