"""Integer models of k_wave's round-6 reductions (hbbft_amd/csrc/k_wave.hpp), checked on random inputs at
the bounds the stage programs allow (tools/gen_wave_prog.py check_bounds: per component at most 8 positive
and 8 negative coefficient units on normalised slot values):
* assemble(): plain + xi-twisted sums joined on unnormalised limbs, ONE carry pass with the quotient from
  the top limb -> normalised limbs, value congruent, in (-p/256, p + p/256);
* fp_carry1(): one parallel carry step keeps the value and gives limbs in [-8, 2^28 + 8);
* fp_red_3k(): reduce(3 t + k a) with the parallel carry -> limbs in [-32, 2^28 + 32), value congruent
  and within fp_red_mk's range.
These are restatements of the device code for its bounds, not the parity evidence (the GPU tests are)."""
import random

P = 0x1A0111EA397FE69A4B1BA7B6434BACD764774B84F38512BF6730D2A0F6B0F6241EABFFFEB153FFFFB9FEFFFFFFFFAAAB
M = (1 << 28) - 1
PL = [(P >> (28 * i)) & M for i in range(14)]
QINV = (1 << 396) // P


def val(limbs):
    return sum(x << (28 * i) for i, x in enumerate(limbs))


def norm_limbs(v):
    limbs = [(v >> (28 * i)) & M for i in range(13)]
    limbs.append(v >> (28 * 13))
    assert val(limbs) == v
    return limbs


def one_pass(u):
    q = (u[13] * QINV) >> 32
    acc, r = 0, [0] * 14
    for i in range(13):
        acc += u[i] - q * PL[i]
        r[i] = acc & M
        acc >>= 28
    r[13] = acc + u[13] - q * PL[13]
    return r


def carry1(a):
    c = [a[i] >> 28 for i in range(13)]
    r = [a[i] & M for i in range(13)] + [a[13]]
    for i in range(1, 14):
        r[i] += c[i - 1]
    return r


def red_3k(t, a, k):
    top = t[13] * 3 + k * a[13]
    q = (top * QINV) >> 32
    v = [t[i] * 3 + k * a[i] - q * PL[i] for i in range(13)] + [top - q * PL[13]]
    r = [v[0] & M] + [(v[i] & M) + (v[i - 1] >> 28) for i in range(1, 13)] + [v[13] + (v[12] >> 28)]
    return r


def test_assembly_one_pass():
    assert QINV == 40323  # sfp.hpp
    rng = random.Random(6)
    lo = hi = 0.0
    for _ in range(4000):
        def slot():
            return norm_limbs(rng.randrange(-P, 2 * P))

        def coefs(nterms, budget):  # check_bounds: positive and negative units each <= budget
            out, pos, neg = [], budget, budget
            for _ in range(nterms):
                c = rng.randint(-min(8, neg), min(7, pos))
                pos, neg = (pos - c, neg) if c > 0 else (pos, neg + c)
                out.append(c)
            return out
        twisted = rng.random() < 0.5
        nt = rng.randint(1, 3) if twisted else 0
        ap = [0] * 14
        for c in coefs(rng.randint(1, 7 - nt), 6 if twisted else 8):
            v = slot()
            ap = [ap[i] + c * v[i] for i in range(14)]
        u = ap
        if twisted:
            t0, t1 = [0] * 14, [0] * 14
            for c in coefs(nt, 8):
                v0, v1 = slot(), slot()
                t0 = [t0[i] + c * v0[i] for i in range(14)]
                t1 = [t1[i] + c * v1[i] for i in range(14)]
            assert all(abs(x) < 1 << 31 for x in t0 + t1)  # the device's int32 twisted limbs
            h = rng.randint(0, 1)
            own, part = (t0, t1) if h == 0 else (t1, t0)
            u = [ap[i] + own[i] + (part[i] if h else -part[i]) for i in range(14)]
        assert all(abs(x) < 1 << 33 for x in u)
        r = one_pass(u)
        assert all(0 <= r[i] <= M for i in range(13))
        assert (val(r) - val(u)) % P == 0
        lo, hi = min(lo, val(r) / P), max(hi, val(r) / P)
    assert -1 / 256 < lo and hi < 1 + 1 / 256


def test_parallel_carries():
    rng = random.Random(7)
    for _ in range(4000):
        a = [rng.randrange(-(1 << 29) + 1, 1 << 29) for _ in range(14)]
        r = carry1(a)
        assert val(r) == val(a)
        assert all(-8 <= x < M + 1 + 8 for x in r[:13])
        # reduce(3 T + k L): T a lazy Granger-Scott combination (|limb| < 2^30), L a run value
        t = [rng.randrange(-(1 << 30) + 1, 1 << 30) for _ in range(13)] + [rng.randrange(-(1 << 21), 1 << 21)]
        L = carry1(norm_limbs(rng.randrange(-P, 2 * P)))
        k = rng.choice((-2, 2))
        r = red_3k(t, L, k)
        assert (val(r) - 3 * val(t) - k * val(L)) % P == 0
        assert all(-32 <= x < M + 1 + 32 for x in r[:13])
        assert -P < val(r) < 2 * P
