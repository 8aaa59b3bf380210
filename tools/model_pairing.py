"""Python model of the exact algorithm the HIP kernels run (Jacobian Miller steps with
scaled lines, '014' sparse products, Granger-Scott cyclotomic squaring, the x-chain hard part).

Dev tool: checked against the oracle's textbook pairing so formula errors are caught on the CPU
before they are translated into HIP.  Not part of the product; run: python tools/model_pairing.py
"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from oracle import bls12_381 as C  # noqa: E402

P = C.P
add, sub, mul, sqr, neg = C.f2_add, C.f2_sub, C.f2_mul, C.f2_sqr, C.f2_neg


def dbl2(a):
    return add(a, a)


# ---------------------------------------------------------------- Miller steps (Jacobian)
def dbl_step(T, xP, yP):
    X, Y, Z = T
    A = sqr(X)
    B = sqr(Y)
    Cc = sqr(B)
    D = dbl2(sub(sub(sqr(add(X, B)), A), Cc))
    E = add(dbl2(A), A)
    F = sqr(E)
    X3 = sub(F, dbl2(D))
    Y3 = sub(mul(E, sub(D, X3)), dbl2(dbl2(dbl2(Cc))))
    ZZ = sqr(Z)
    Z3 = sub(sub(sqr(add(Y, Z)), B), ZZ)          # 2YZ
    c0 = sub(mul(E, X), dbl2(B))                   # 3X^3 - 2Y^2
    EZZ = mul(E, ZZ)
    c1 = neg(C.f2_muls(EZZ, xP))                   # -3X^2 Z^2 xP
    c4 = C.f2_muls(mul(Z3, ZZ), yP)                # 2YZ^3 yP
    return (X3, Y3, Z3), (c0, c1, c4)


def add_step(T, Q, xP, yP):
    X1, Y1, Z1 = T
    xQ, yQ = Q
    Z1Z1 = sqr(Z1)
    U2 = mul(xQ, Z1Z1)
    S2 = mul(mul(yQ, Z1), Z1Z1)
    H = sub(U2, X1)
    r = sub(S2, Y1)
    HH = sqr(H)
    HHH = mul(H, HH)
    V = mul(X1, HH)
    X3 = sub(sub(sqr(r), HHH), dbl2(V))
    Y3 = sub(mul(r, sub(V, X3)), mul(Y1, HHH))
    Z3 = mul(Z1, H)
    c0 = sub(mul(r, xQ), mul(yQ, Z3))
    c1 = neg(C.f2_muls(r, xP))
    c4 = C.f2_muls(Z3, yP)
    return (X3, Y3, Z3), (c0, c1, c4)


def line_to_f12(c):
    c0, c1, c4 = c
    return ((c0, c1, C.F2_ZERO), (C.F2_ZERO, c4, C.F2_ZERO))


def f6_mul_01(x, a, b):
    """x * (a + b v)."""
    x0, x1, x2 = x
    t0 = mul(x0, a)
    t1 = mul(x1, b)
    c0 = add(t0, C.f2_mul_xi(mul(x2, b)))
    c1 = sub(sub(mul(add(x0, x1), add(a, b)), t0), t1)
    c2 = add(t1, mul(x2, a))
    return (c0, c1, c2)


def f6_mul_1(x, b):
    """x * (b v)."""
    x0, x1, x2 = x
    return (C.f2_mul_xi(mul(x2, b)), mul(x0, b), mul(x1, b))


def f12_mul_014(f, c):
    c0, c1, c4 = c
    f0, f1 = f
    t0 = f6_mul_01(f0, c0, c1)
    t1 = f6_mul_1(f1, c4)
    s = f6_mul_01(C.f6_add(f0, f1), c0, add(c1, c4))
    r1 = C.f6_sub(C.f6_sub(s, t0), t1)
    r0 = C.f6_add(t0, C.f6_mul_v(t1))
    return (r0, r1)


def f12_sqr(f):
    f0, f1 = f
    t = C.f6_mul(f0, f1)
    a = C.f6_mul(C.f6_add(f0, f1), C.f6_add(f0, C.f6_mul_v(f1)))
    c0 = C.f6_sub(C.f6_sub(a, t), C.f6_mul_v(t))
    return (c0, C.f6_add(t, t))


def miller(pairs):
    f = C.F12_ONE
    Ts = [(q[0], q[1], C.F2_ONE) for (_, q) in pairs]
    bits = bin(C.X_ABS)[3:]
    for bit in bits:
        f = f12_sqr(f)
        for k, (p_, q_) in enumerate(pairs):
            Ts[k], l = dbl_step(Ts[k], p_[0], p_[1])
            f = f12_mul_014(f, l)
        if bit == "1":
            for k, (p_, q_) in enumerate(pairs):
                Ts[k], l = add_step(Ts[k], q_, p_[0], p_[1])
                f = f12_mul_014(f, l)
    return f  # not conjugated: conjugation does not change "FE(f) == 1"


# ---------------------------------------------------------------- final exponentiation
def gamma(k, e):
    return C.f2_pow((1, 1), k * (P ** e - 1) // 6)


def coeffs(f):
    (a0, a2, a4), (a1, a3, a5) = f
    return [a0, a1, a2, a3, a4, a5]


def from_coeffs(a):
    return ((a[0], a[2], a[4]), (a[1], a[3], a[5]))


def frob(f, e):
    a = coeffs(f)
    out = []
    for k in range(6):
        ak = a[k] if e % 2 == 0 else C.f2_conj(a[k])
        out.append(mul(ak, gamma(k, e)))
    return from_coeffs(out)


def fp4_sqr(x0, x1):
    """(x0 + x1 t)^2 with t^2 = xi."""
    s0 = sqr(x0)
    s1 = sqr(x1)
    return add(s0, C.f2_mul_xi(s1)), sub(sub(sqr(add(x0, x1)), s0), s1)


def cyclo_sqr(f):
    a = coeffs(f)
    # A = a0 + a3 t, B = a1 + a4 t, C = a2 + a5 t  (t = w^3)
    A0, A1 = fp4_sqr(a[0], a[3])
    B0, B1 = fp4_sqr(a[1], a[4])
    C0, C1 = fp4_sqr(a[2], a[5])
    three = lambda z: add(dbl2(z), z)  # noqa: E731
    # A' = 3A^2 - 2 conj(A)
    n0 = sub(three(A0), dbl2(a[0]))
    n3 = add(three(A1), dbl2(a[3]))
    # B' = 3 t C^2 + 2 conj(B);  t*C^2 = xi*C1 + C0 t
    n1 = add(three(C.f2_mul_xi(C1)), dbl2(a[1]))
    n4 = sub(three(C0), dbl2(a[4]))
    # C' = 3 B^2 - 2 conj(C)
    n2 = sub(three(B0), dbl2(a[2]))
    n5 = add(three(B1), dbl2(a[5]))
    return from_coeffs([n0, n1, n2, n3, n4, n5])


def cyc_exp_abs(f, e):
    r = f
    for bit in bin(e)[3:]:
        r = cyclo_sqr(r)
        if bit == "1":
            r = C.f12_mul(r, f)
    return r


def exp_x(f):            # f^x, x < 0
    return C.f12_conj(cyc_exp_abs(f, C.X_ABS))


def exp_x_minus_1(f):    # f^(x-1) = conj(f^(|x|+1))
    return C.f12_conj(cyc_exp_abs(f, C.X_ABS + 1))


def final_exp_x3(f):
    f1 = C.f12_mul(C.f12_conj(f), C.f12_inv(f))
    f2 = C.f12_mul(frob(f1, 2), f1)
    a = exp_x_minus_1(exp_x_minus_1(f2))
    b = C.f12_mul(exp_x(a), frob(a, 1))
    c = C.f12_mul(C.f12_mul(exp_x(exp_x(b)), frob(b, 2)), C.f12_conj(b))
    return C.f12_mul(c, C.f12_mul(cyclo_sqr(f2), f2))


if __name__ == "__main__":
    g1, g2 = C.G1_GEN, C.G2_GEN
    P1 = C.g1_mul(g1, 5)
    Q1 = C.g2_mul(g2, 7)
    f_model = miller([(P1, Q1)])
    # frobenius check
    assert frob(f_model, 1) == C.f12_frob(f_model, 1)
    assert frob(f_model, 2) == C.f12_frob(f_model, 2)
    # cyclotomic squaring check on an element of the cyclotomic subgroup
    z = C.f12_mul(C.f12_conj(f_model), C.f12_inv(f_model))
    z = C.f12_mul(C.f12_frob(z, 2), z)
    assert cyclo_sqr(z) == C.f12_sqr(z)
    e_oracle = C.pairing(P1, Q1)
    e_model = final_exp_x3(C.f12_conj(f_model))
    assert e_model == C.f12_pow(e_oracle, 3), "model pairing != oracle^3"
    # product check: e(5g1, 7g2) * e(-35 g1, g2) == 1
    f = miller([(P1, Q1), (C.g1_neg(C.g1_mul(g1, 35)), g2)])
    assert final_exp_x3(f) == C.F12_ONE
    f = miller([(P1, Q1), (C.g1_neg(C.g1_mul(g1, 36)), g2)])
    assert final_exp_x3(f) != C.F12_ONE
    print("model OK")
