"""CPU restatement (ORACLE) of the BLS12-381 arithmetic behind hbbft's threshold crypto.

TEST INFRASTRUCTURE ONLY.  Nothing in the product path (``hbbft_amd``) may import this
module; only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg
use it, and only as the checker.

What it restates
----------------
hbbft (``/root/reference``) does no curve arithmetic itself: every call on the hot path goes
to the external crates ``threshold_crypto = "0.3.0"`` (``Cargo.toml:37``) -> ``pairing`` 0.14
-> ``ff`` 0.4, which are *not* vendored in the reference (no ``Cargo.lock``).
This module therefore restates the published BLS12-381 definition and the ``pairing`` 0.14
conventions recalled in SURVEY.md Appendix A/B:

* Fp / Fr prime fields, tower Fp2 = Fp[u]/(u^2+1), Fp6 = Fp2[v]/(v^3-(u+1)),
  Fp12 = Fp6[w]/(w^2-v)  (SURVEY Appendix A).
* G1: y^2 = x^3 + 4 over Fp; G2: y^2 = x^3 + 4(u+1) over Fp2 (D-type sextic twist).
* Optimal-ate pairing, Miller loop over |x| = 0xd201000000010000, conjugation for x < 0,
  final exponentiation (p^12-1)/r.  Call sites: ``src/threshold_sign.rs:223,264``,
  ``src/threshold_decrypt.rs:142,227``.
* Canonical encodings (compressed / uncompressed, zcash flag bits) - SURVEY Appendix B.1.

Parity status
-------------
Pinned: SHA3-256 (``hashlib``), ChaCha20 (RFC 7539 / rand_chacha zero-key vectors, see
``tests/test_oracle.py``), the standard compressed encodings of the G1/G2 generators,
curve/subgroup/bilinearity identities.  The ``threshold_crypto`` host conventions
(hash_g2's RNG-to-point mapping, XOR stream, parity) are *restated from SURVEY Appendix B*
and remain "parity unpinned" against the real crate (no Rust toolchain and no crate
sources in this container; the reference's tests carry no known-answer vectors,
SURVEY §8c).

Representation: plain Python ints; Fp2 = (c0, c1); Fp6 = (a0, a1, a2) of Fp2;
Fp12 = (g0, g1) of Fp6.  Points: ``None`` is the point at infinity, otherwise affine
``(x, y)``.  Pure-Python: for small cases only (a pairing takes ~0.1-0.3 s).
"""

# ----------------------------------------------------------------------------- constants
P = 0x1A0111EA397FE69A4B1BA7B6434BACD764774B84F38512BF6730D2A0F6B0F6241EABFFFEB153FFFFB9FEFFFFFFFFAAAB
R = 0x73EDA753299D7D483339D80809A1D80553BDA402FFFE5BFEFFFFFFFF00000001
X_ABS = 0xD201000000010000          # |x|, x = -0xd201000000010000
X_IS_NEG = True
H1 = 0x396C8C005555E1568C00AAAB0000AAAB
H2 = 0x5D543A95414E7F1091D50792876A202CD91DE4547085ABAA68A205B2E5A7DDFA628F1CB4D9E82EF21537E293A6691AE1616EC6E786F0C70CF1C38E31C7238E5

G1_GEN = (
    0x17F1D3A73197D7942695638C4FA9AC0FC3688C4F9774B905A14E3A3F171BAC586C55E83FF97A1AEFFB3AF00ADB22C6BB,
    0x08B3F481E3AAA0F1A09E30ED741D8AE4FCF5E095D5D00AF600DB18CB2C04B3EDD03CC744A2888AE40CAA232946C5E7E1,
)
G2_GEN = (
    (0x024AA2B2F08F0A91260805272DC51051C6E47AD4FA403B02B4510B647AE3D1770BAC0326A805BBEFD48056C8C121BDB8,
     0x13E02B6052719F607DACD3A088274F65596BD0D09920B61AB5DA61BBDC7F5049334CF11213945D57E5AC7D055D042B7E),
    (0x0CE5D527727D6E118CC9CDC6DA2E351AADFD9BAA8CBDD3A76D429A695160D12C923AC9CC3BACA289E193548608B82801,
     0x0606C4A02EA734CC32ACD2B02BC28B99CB3E287E85A763AF267492AB572E99AB3F370D275CEC1DA1AAA9075FF05F79BE),
)

# ----------------------------------------------------------------------------- Fp
def fp_inv(a):
    return pow(a, P - 2, P)


def fp_sqrt(a):
    """Square root in Fp (p = 3 mod 4) or None."""
    a %= P
    s = pow(a, (P + 1) // 4, P)
    return s if s * s % P == a else None


# ----------------------------------------------------------------------------- Fp2
F2_ZERO = (0, 0)
F2_ONE = (1, 0)


def f2_add(a, b):
    return ((a[0] + b[0]) % P, (a[1] + b[1]) % P)


def f2_sub(a, b):
    return ((a[0] - b[0]) % P, (a[1] - b[1]) % P)


def f2_neg(a):
    return ((-a[0]) % P, (-a[1]) % P)


def f2_mul(a, b):
    a0, a1 = a
    b0, b1 = b
    return ((a0 * b0 - a1 * b1) % P, (a0 * b1 + a1 * b0) % P)


def f2_sqr(a):
    return f2_mul(a, a)


def f2_muls(a, s):
    return (a[0] * s % P, a[1] * s % P)


def f2_conj(a):
    return (a[0], (-a[1]) % P)


def f2_inv(a):
    t = fp_inv((a[0] * a[0] + a[1] * a[1]) % P)
    return (a[0] * t % P, (-a[1]) * t % P)


def f2_mul_xi(a):
    """Multiply by xi = u + 1."""
    return ((a[0] - a[1]) % P, (a[0] + a[1]) % P)


def f2_pow(a, e):
    r = F2_ONE
    b = a
    while e:
        if e & 1:
            r = f2_mul(r, b)
        b = f2_sqr(b)
        e >>= 1
    return r


def f2_is_zero(a):
    return a[0] == 0 and a[1] == 0


def f2_sqrt(a):
    """Square root in Fp2 or None (p = 3 mod 4 algorithm; any root - callers pick the sign)."""
    if f2_is_zero(a):
        return F2_ZERO
    a1 = f2_pow(a, (P - 3) // 4)
    alpha = f2_mul(f2_sqr(a1), a)
    a0 = f2_mul(f2_pow(alpha, P), alpha)
    if a0 == (P - 1, 0):
        return None
    x0 = f2_mul(a1, a)
    if alpha == (P - 1, 0):
        res = f2_mul(x0, (0, 1))
    else:
        b = f2_pow(f2_add(F2_ONE, alpha), (P - 1) // 2)
        res = f2_mul(b, x0)
    return res if f2_sqr(res) == a else None


def f2_gt(a, b):
    """pairing 0.14 ``Ord for Fq2``: compare c1 first, then c0 (canonical integers)."""
    if a[1] != b[1]:
        return a[1] > b[1]
    return a[0] > b[0]


# ----------------------------------------------------------------------------- Fp6
F6_ZERO = (F2_ZERO, F2_ZERO, F2_ZERO)
F6_ONE = (F2_ONE, F2_ZERO, F2_ZERO)


def f6_add(a, b):
    return (f2_add(a[0], b[0]), f2_add(a[1], b[1]), f2_add(a[2], b[2]))


def f6_sub(a, b):
    return (f2_sub(a[0], b[0]), f2_sub(a[1], b[1]), f2_sub(a[2], b[2]))


def f6_neg(a):
    return (f2_neg(a[0]), f2_neg(a[1]), f2_neg(a[2]))


def f6_mul(a, b):
    a0, a1, a2 = a
    b0, b1, b2 = b
    t0 = f2_mul(a0, b0)
    t1 = f2_mul(a1, b1)
    t2 = f2_mul(a2, b2)
    c0 = f2_add(t0, f2_mul_xi(f2_add(f2_mul(a1, b2), f2_mul(a2, b1))))
    c1 = f2_add(f2_add(f2_mul(a0, b1), f2_mul(a1, b0)), f2_mul_xi(t2))
    c2 = f2_add(f2_add(f2_mul(a0, b2), f2_mul(a2, b0)), t1)
    return (c0, c1, c2)


def f6_mul_v(a):
    """Multiply by v (v^3 = xi)."""
    return (f2_mul_xi(a[2]), a[0], a[1])


def f6_inv(a):
    a0, a1, a2 = a
    c0 = f2_sub(f2_sqr(a0), f2_mul_xi(f2_mul(a1, a2)))
    c1 = f2_sub(f2_mul_xi(f2_sqr(a2)), f2_mul(a0, a1))
    c2 = f2_sub(f2_sqr(a1), f2_mul(a0, a2))
    t = f2_add(f2_mul(a0, c0), f2_mul_xi(f2_add(f2_mul(a2, c1), f2_mul(a1, c2))))
    ti = f2_inv(t)
    return (f2_mul(c0, ti), f2_mul(c1, ti), f2_mul(c2, ti))


# ----------------------------------------------------------------------------- Fp12
F12_ONE = (F6_ONE, F6_ZERO)


def f12_mul(a, b):
    a0, a1 = a
    b0, b1 = b
    t0 = f6_mul(a0, b0)
    t1 = f6_mul(a1, b1)
    c1 = f6_sub(f6_sub(f6_mul(f6_add(a0, a1), f6_add(b0, b1)), t0), t1)
    c0 = f6_add(t0, f6_mul_v(t1))
    return (c0, c1)


def f12_sqr(a):
    return f12_mul(a, a)


def f12_conj(a):
    return (a[0], f6_neg(a[1]))


def f12_inv(a):
    a0, a1 = a
    t = f6_sub(f6_mul(a0, a0), f6_mul_v(f6_mul(a1, a1)))
    ti = f6_inv(t)
    return (f6_mul(a0, ti), f6_neg(f6_mul(a1, ti)))


def f12_pow(a, e):
    r = F12_ONE
    b = a
    while e:
        if e & 1:
            r = f12_mul(r, b)
        b = f12_sqr(b)
        e >>= 1
    return r


def f12_frob(a, k=1):
    """a^(p^k) by plain exponentiation (oracle: slow but obviously correct)."""
    return f12_pow(a, P ** k)


# ----------------------------------------------------------------------------- curves (affine)
B1 = 4
B2 = (4, 4)  # 4(u+1)


def g1_on_curve(pt):
    if pt is None:
        return True
    x, y = pt
    return (y * y - x * x * x - B1) % P == 0


def g2_on_curve(pt):
    if pt is None:
        return True
    x, y = pt
    return f2_sub(f2_sqr(y), f2_add(f2_mul(f2_sqr(x), x), B2)) == F2_ZERO


def g1_neg(pt):
    return None if pt is None else (pt[0], (-pt[1]) % P)


def g2_neg(pt):
    return None if pt is None else (pt[0], f2_neg(pt[1]))


def g1_add(a, b):
    if a is None:
        return b
    if b is None:
        return a
    x1, y1 = a
    x2, y2 = b
    if x1 == x2:
        if (y1 + y2) % P == 0:
            return None
        lam = 3 * x1 * x1 * fp_inv(2 * y1) % P
    else:
        lam = (y2 - y1) * fp_inv(x2 - x1) % P
    x3 = (lam * lam - x1 - x2) % P
    return (x3, (lam * (x1 - x3) - y1) % P)


def g2_add(a, b):
    if a is None:
        return b
    if b is None:
        return a
    x1, y1 = a
    x2, y2 = b
    if x1 == x2:
        if f2_is_zero(f2_add(y1, y2)):
            return None
        lam = f2_mul(f2_muls(f2_sqr(x1), 3), f2_inv(f2_muls(y1, 2)))
    else:
        lam = f2_mul(f2_sub(y2, y1), f2_inv(f2_sub(x2, x1)))
    x3 = f2_sub(f2_sub(f2_sqr(lam), x1), x2)
    return (x3, f2_sub(f2_mul(lam, f2_sub(x1, x3)), y1))


# Jacobian helpers for faster scalar multiplication (internal to the oracle).
def _j1_dbl(X, Y, Z):
    if Z == 0:
        return (1, 1, 0)
    A = X * X % P
    Bv = Y * Y % P
    C = Bv * Bv % P
    D = 2 * ((X + Bv) ** 2 - A - C) % P
    E = 3 * A % P
    F = E * E % P
    X3 = (F - 2 * D) % P
    Y3 = (E * (D - X3) - 8 * C) % P
    Z3 = 2 * Y * Z % P
    return (X3, Y3, Z3)


def _j1_add_aff(J, Q):
    X1, Y1, Z1 = J
    if Q is None:
        return J
    if Z1 == 0:
        return (Q[0], Q[1], 1)
    x2, y2 = Q
    Z1Z1 = Z1 * Z1 % P
    U2 = x2 * Z1Z1 % P
    S2 = y2 * Z1 * Z1Z1 % P
    H = (U2 - X1) % P
    rr = (S2 - Y1) % P
    if H == 0:
        if rr == 0:
            return _j1_dbl(X1, Y1, Z1)
        return (1, 1, 0)
    HH = H * H % P
    HHH = H * HH % P
    V = X1 * HH % P
    X3 = (rr * rr - HHH - 2 * V) % P
    Y3 = (rr * (V - X3) - Y1 * HHH) % P
    Z3 = Z1 * H % P
    return (X3, Y3, Z3)


def _j1_to_aff(J):
    X, Y, Z = J
    if Z == 0:
        return None
    zi = fp_inv(Z)
    zi2 = zi * zi % P
    return (X * zi2 % P, Y * zi2 * zi % P)


def g1_mul(pt, k):
    """Scalar multiplication (k any non-negative int; the group result is canonical)."""
    if pt is None or k == 0:
        return None
    J = (1, 1, 0)
    for bit in bin(k)[2:]:
        J = _j1_dbl(*J)
        if bit == "1":
            J = _j1_add_aff(J, pt)
    return _j1_to_aff(J)


def _j2_dbl(J):
    X, Y, Z = J
    if f2_is_zero(Z):
        return J
    A = f2_sqr(X)
    Bv = f2_sqr(Y)
    C = f2_sqr(Bv)
    D = f2_muls(f2_sub(f2_sub(f2_sqr(f2_add(X, Bv)), A), C), 2)
    E = f2_muls(A, 3)
    F = f2_sqr(E)
    X3 = f2_sub(F, f2_muls(D, 2))
    Y3 = f2_sub(f2_mul(E, f2_sub(D, X3)), f2_muls(C, 8))
    Z3 = f2_muls(f2_mul(Y, Z), 2)
    return (X3, Y3, Z3)


def _j2_add_aff(J, Q):
    X1, Y1, Z1 = J
    if Q is None:
        return J
    if f2_is_zero(Z1):
        return (Q[0], Q[1], F2_ONE)
    x2, y2 = Q
    Z1Z1 = f2_sqr(Z1)
    U2 = f2_mul(x2, Z1Z1)
    S2 = f2_mul(f2_mul(y2, Z1), Z1Z1)
    H = f2_sub(U2, X1)
    rr = f2_sub(S2, Y1)
    if f2_is_zero(H):
        if f2_is_zero(rr):
            return _j2_dbl(J)
        return (F2_ONE, F2_ONE, F2_ZERO)
    HH = f2_sqr(H)
    HHH = f2_mul(H, HH)
    V = f2_mul(X1, HH)
    X3 = f2_sub(f2_sub(f2_sqr(rr), HHH), f2_muls(V, 2))
    Y3 = f2_sub(f2_mul(rr, f2_sub(V, X3)), f2_mul(Y1, HHH))
    Z3 = f2_mul(Z1, H)
    return (X3, Y3, Z3)


def _j2_to_aff(J):
    X, Y, Z = J
    if f2_is_zero(Z):
        return None
    zi = f2_inv(Z)
    zi2 = f2_sqr(zi)
    return (f2_mul(X, zi2), f2_mul(f2_mul(Y, zi2), zi))


def g2_mul(pt, k):
    if pt is None or k == 0:
        return None
    J = (F2_ONE, F2_ONE, F2_ZERO)
    for bit in bin(k)[2:]:
        J = _j2_dbl(J)
        if bit == "1":
            J = _j2_add_aff(J, pt)
    return _j2_to_aff(J)


def g1_in_subgroup(pt):
    return g1_on_curve(pt) and g1_mul(pt, R) is None


def g2_in_subgroup(pt):
    return g2_on_curve(pt) and g2_mul(pt, R) is None


# ----------------------------------------------------------------------------- pairing
def _line(lam, xT, yT, Pp):
    """Line through psi(T) with E'-slope lam evaluated at P, scaled by w^3 (an Fp4 factor the
    final exponentiation removes): l = (lam*xT - yT) - lam*xP * w^2 + yP * w^3.
    Non-zero slots: c0.c0, c0.c1, c1.c1 (the '014' sparse form of pairing 0.14)."""
    xP, yP = Pp
    c00 = f2_sub(f2_mul(lam, xT), yT)
    c01 = f2_neg(f2_muls(lam, xP))
    c11 = (yP % P, 0)
    return ((c00, c01, F2_ZERO), (F2_ZERO, c11, F2_ZERO))


def miller_loop(pairs):
    """Product of Miller functions f_{|x|,Q}(P) over (P in G1, Q in G2) pairs; pairs with a
    point at infinity contribute 1 (pairing 0.14 skips them). Conjugated for x < 0."""
    pairs = [(p_, q_) for (p_, q_) in pairs if p_ is not None and q_ is not None]
    f = F12_ONE
    Ts = [q for (_, q) in pairs]
    bits = bin(X_ABS)[3:]  # skip the leading 1
    for bit in bits:
        f = f12_sqr(f)
        for k, (Pp, Q) in enumerate(pairs):
            xT, yT = Ts[k]
            lam = f2_mul(f2_muls(f2_sqr(xT), 3), f2_inv(f2_muls(yT, 2)))
            f = f12_mul(f, _line(lam, xT, yT, Pp))
            Ts[k] = g2_add(Ts[k], Ts[k])
        if bit == "1":
            for k, (Pp, Q) in enumerate(pairs):
                xT, yT = Ts[k]
                xQ, yQ = Q
                lam = f2_mul(f2_sub(yQ, yT), f2_inv(f2_sub(xQ, xT)))
                f = f12_mul(f, _line(lam, xT, yT, Pp))
                Ts[k] = g2_add(Ts[k], Q)
    if X_IS_NEG:
        f = f12_conj(f)
    return f


HARD_EXP = (P ** 4 - P ** 2 + 1) // R


def final_exponentiation(f):
    """f^((p^12-1)/r) = easy part (p^6-1)(p^2+1) then hard part (p^4-p^2+1)/r."""
    f1 = f12_mul(f12_conj(f), f12_inv(f))      # f^(p^6-1)
    f2 = f12_mul(f12_frob(f1, 2), f1)          # ^(p^2+1)
    return f12_pow(f2, HARD_EXP)


def pairing(Pp, Q):
    if Pp is None or Q is None:
        return F12_ONE
    return final_exponentiation(miller_loop([(Pp, Q)]))


def pairing_product_is_one(pairs):
    """prod e(P_i, Q_i) == 1 via one multi-Miller loop + one final exponentiation."""
    return final_exponentiation(miller_loop(pairs)) == F12_ONE


# ----------------------------------------------------------------------------- encodings
def fp_to_be(a):
    return a.to_bytes(48, "big")


def g1_compress(pt):
    if pt is None:
        return bytes([0xC0]) + bytes(47)
    x, y = pt
    out = bytearray(fp_to_be(x))
    if y > (P - y) % P:
        out[0] |= 0x20
    out[0] |= 0x80
    return bytes(out)


def g1_uncompressed(pt):
    if pt is None:
        return bytes([0x40]) + bytes(95)
    return fp_to_be(pt[0]) + fp_to_be(pt[1])


def g2_compress(pt):
    if pt is None:
        return bytes([0xC0]) + bytes(95)
    x, y = pt
    out = bytearray(fp_to_be(x[1]) + fp_to_be(x[0]))
    if f2_gt(y, f2_neg(y)):
        out[0] |= 0x20
    out[0] |= 0x80
    return bytes(out)


def g2_uncompressed(pt):
    if pt is None:
        return bytes([0x40]) + bytes(191)
    x, y = pt
    return fp_to_be(x[1]) + fp_to_be(x[0]) + fp_to_be(y[1]) + fp_to_be(y[0])


class DecodeError(ValueError):
    pass


def g1_decompress(b, in_subgroup=None):
    """pairing 0.14 ``G1Compressed::into_affine``: flags, on-curve and subgroup checks.
    ``in_subgroup``: the r * P == O test to use (default the pure-Python one; tests pass the C
    oracle's scalar multiplication for large samples)."""
    if len(b) != 48:
        raise DecodeError("length")
    if not (b[0] & 0x80):
        raise DecodeError("not compressed")
    if b[0] & 0x40:
        if (b[0] & 0x3F) or any(b[1:]):
            raise DecodeError("bad infinity")
        return None
    greatest = bool(b[0] & 0x20)
    x = int.from_bytes(bytes([b[0] & 0x1F]) + b[1:], "big")
    if x >= P:
        raise DecodeError("x not in field")
    y = fp_sqrt((x * x * x + B1) % P)
    if y is None:
        raise DecodeError("not on curve")
    ny = (P - y) % P
    if (y > ny) != greatest:
        y = ny
    pt = (x, y)
    if not (in_subgroup or g1_in_subgroup)(pt):
        raise DecodeError("not in subgroup")
    return pt


def g2_decompress(b, in_subgroup=None):
    if len(b) != 96:
        raise DecodeError("length")
    if not (b[0] & 0x80):
        raise DecodeError("not compressed")
    if b[0] & 0x40:
        if (b[0] & 0x3F) or any(b[1:]):
            raise DecodeError("bad infinity")
        return None
    greatest = bool(b[0] & 0x20)
    x1 = int.from_bytes(bytes([b[0] & 0x1F]) + b[1:48], "big")
    x0 = int.from_bytes(b[48:96], "big")
    if x0 >= P or x1 >= P:
        raise DecodeError("x not in field")
    x = (x0, x1)
    y = f2_sqrt(f2_add(f2_mul(f2_sqr(x), x), B2))
    if y is None:
        raise DecodeError("not on curve")
    ny = f2_neg(y)
    if f2_gt(y, ny) != greatest:
        y = ny
    pt = (x, y)
    if not (in_subgroup or g2_in_subgroup)(pt):
        raise DecodeError("not in subgroup")
    return pt


# ----------------------------------------------------------------------------- Fr
def fr_inv(a):
    return pow(a, R - 2, R)
