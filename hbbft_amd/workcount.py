"""Algorithmic work of the hot-path units, in Fp multiplications, derived from the kernels' own
formulas (csrc/pfp.hpp, k_pair.hip, curve.hpp).  Used by bench.py for the roofline's 'achieved'
figure.  Fp2 mul = 3 Fp-mul (Karatsuba), Fp2 sqr = 2 (complex), Fp2 x Fp = 2.

Pricing: one Fp multiplication = 300 32x32->64 multiply-adds (12-limb CIOS
Montgomery: 144 product + 156 reduction); an Fp squaring = 222 (78 product + 144 reduction).
True Fp squarings occur in the Fp inversion (380 of them) and in the G1 curve formulas
(dbl-2009-l 2M+5S, madd-2007-bl 7M+4S, add-2007-bl 11M+5S); Fp2/Fp12 squarings are products.
"""
X_ABS = 0xD201000000010000
NBITS = X_ABS.bit_length() - 1          # 63 doubling steps
NADD = bin(X_ABS).count("1") - 1        # 5 addition steps
F2M, F2S, F2F = 3, 2, 2

F6_MUL = 6 * F2M                         # 18
F12_SQR = 2 * F6_MUL                     # 36 (complex squaring)
F12_MUL = 3 * F6_MUL                     # 54
F12_MUL_014 = 2 * 5 * F2M + 3 * F2M      # 39
LINE_EVAL = 2 * F2F                      # c1*xP, c4*yP
CYCLO_SQR = 9 * F2S                      # 18 (Granger-Scott)
FROB1 = 5 * F2M
FROB2 = 5 * F2F

DBL_STEP = 7 * F2S + 4 * F2M             # 26
ADD_STEP = 3 * F2S + 10 * F2M            # 36
G2_WALK = NBITS * DBL_STEP + NADD * ADD_STEP

MILLER_2PAIR = NBITS * (F12_SQR + 2 * (F12_MUL_014 + LINE_EVAL)) + NADD * 2 * (F12_MUL_014 + LINE_EVAL)

# The final exponentiation's one Fp inversion (of a public norm) is T. Pornin's binary GCD
# (words.hpp words_inv_vartime): 25 rounds of 31 divsteps on 64-bit approximations; per round the
# 2x2 update of (a, b) (2 x 12 limbs x 2 MADs each) and of the Bezout pair (u, v) with its
# Montgomery division by 2^31 (2 x (24 + 12) MADs) = 120 MADs -> 3,000 MADs = 10 Fp products.
# (Round 2 priced Fermat's a^(p-2): 380 squarings + 190 products.)
BINGCD_ROUNDS = (2 * 381 - 1 + 30) // 31
BINGCD_MADS = BINGCD_ROUNDS * 120
FP_INV = BINGCD_MADS // 300
F2_INV = 2 + FP_INV + 2
F6_INV = 3 * (F2S + F2M) + 3 * F2M + F2_INV + 3 * F2M
F12_INV = 2 * F6_MUL + F6_INV + 2 * F6_MUL
EASY = F12_INV + F12_MUL + FROB2 + F12_MUL


def _exp(e):
    return NBITS * CYCLO_SQR + (bin(e).count("1") - 1) * F12_MUL


HARD = 2 * _exp(X_ABS + 1) + 3 * _exp(X_ABS) + FROB1 + FROB2 + 5 * F12_MUL + CYCLO_SQR
FINAL_EXP = EASY + HARD

# per check: multi-Miller loop over (pk_i, H) and (-g1, sig_i), the G2 walk over sig_i (H's walk
# is shared by the 64 shares of a document), one final exponentiation
FP_MULS_PER_CHECK = MILLER_2PAIR + G2_WALK + FINAL_EXP

# The reference's work for the same verdict (SURVEY §8(d) "reference work"): threshold_crypto's
# verify_g2 computes e(pk_i, H) and e(g1, sig_i) as two separate pairings (pairing 0.14: each its own
# G2Prepared walk, single-pair Miller loop and final exponentiation), then compares them.
MILLER_1PAIR = NBITS * (F12_SQR + F12_MUL_014 + LINE_EVAL) + NADD * (F12_MUL_014 + LINE_EVAL)
REFERENCE_CHECK = 2 * (MILLER_1PAIR + G2_WALK + FINAL_EXP)

if __name__ == "__main__":
    print("miller", MILLER_2PAIR, "g2 walk", G2_WALK, "final exp", FINAL_EXP, "(easy", EASY, "hard", HARD,
          ") total", FP_MULS_PER_CHECK)


# ---------------------------------------------------------------------------- MAD pricing
MAD_PER_FPMUL = 300
MAD_PER_FPSQR = 222
FP_INV_SQR = 0                        # binary-GCD inverse: no Fp squarings (Fermat had 380)


def mads(fpmul, fpsqr=0):
    """32x32->64 multiply-adds of fpmul products (of which fpsqr are squarings)."""
    return (fpmul - fpsqr) * MAD_PER_FPMUL + fpsqr * MAD_PER_FPSQR


# per-unit algorithmic work of each kernel: (Fp ops, of which Fp squarings)
PAIR_CHECK_WALK = (MILLER_2PAIR + G2_WALK + FINAL_EXP, FP_INV_SQR)   # k_pair_verify, one side walked
PAIR_CHECK_TABLE = (MILLER_2PAIR + FINAL_EXP, FP_INV_SQR)            # k_pair_verify, both sides tabled
PAIR_PREP_DOC = (G2_WALK, 0)                                         # k_oct_prep (k_pair_prep), per G2 point
REFERENCE_CHECK_OPS = (REFERENCE_CHECK, FP_INV_SQR)                  # two separate pairings

G1_DBL = (7, 5)
G1_MADD = (11, 4)
G1_ADD = (16, 5)


def _add(*ops):
    return (sum(o[0] for o in ops), sum(o[1] for o in ops))


def _scale(op, k):
    return (op[0] * k, op[1] * k)


def g1_mul_small(k):
    """jac_mul_small(P, k): double-and-add from the top bit with full Jacobian additions."""
    if k <= 1:
        return (0, 0)
    return _add(_scale(G1_DBL, k.bit_length() - 1), _scale(G1_ADD, bin(k).count("1") - 1))


def bivar_ack(t, y, val_windows=32):
    """k_bivar_check for one ack: Horner over the t+1 row points with the small y, then g1 * val
    from the fixed-base comb table (one mixed addition per nonzero byte of val: 32 windows) and a
    cross-multiplied compare."""
    horner = _scale(_add(g1_mul_small(y), G1_MADD), t + 1)
    return _add(horner, _scale(G1_MADD, val_windows), (4, 2))


def bivar_row_fd(t, ymin, ymax, nacks, val_windows=16):
    """The finite-difference Ack check of one row (k_bivar_fd_seed / _run / _check): the difference
    table at y0 (0 when ymin <= t + 1, as the engine's plan_fd seeds) by the seed levels -- per level
    m < t and k = 1 .. t - m one product k (D_k + D_{k-1}) for y0 = 0, else (y0 + k) D_k + k D_{k-1},
    and per level one mixed addition of R_m --, t additions per further y (ymax - y0 steps), and per
    ack g1 * val from the 16-bit comb (one mixed addition per nonzero 16-bit window) and the compare."""
    y0 = 0 if ymin <= t + 1 else ymin
    parts = [_scale(G1_MADD, t + 1)]
    for m in range(t - 1, -1, -1):
        for k in range(1, t - m + 1):
            if y0 == 0:
                parts.append(_add(G1_ADD, g1_mul_small(k)))
            else:
                parts.append(_add(G1_ADD, g1_mul_small(y0 + k), g1_mul_small(k)))
    steps = _scale(G1_ADD, t * (ymax - y0))
    acks = _scale(_add(_scale(G1_MADD, val_windows), (4, 2)), nacks)
    return _add(*parts, steps, acks)


# ---------------------------------------------------------------------------- wire decoding (round 6)
# k_g1_decompress / k_g2_decompress per valid point (csrc/k_wire.hip).  The square root's one
# exponent (p-3)/4 is tools/gen_sqrt_chain.py's width-4 sliding-window chain: a^2 + 375 squarings
# and 7 table + 78 window products.
SQRT_CHAIN = (376 + 85, 376)
G2_DBL = (2 * F2M + 5 * F2S, 0)          # dbl-2009-l over Fp2 (Fp2 squarings are Fp products)
G2_MADD = (7 * F2M + 4 * F2S, 0)         # madd-2007-bl over Fp2
# G1: to Montgomery, x^3 + 4, y = rhs * rhs^((p-3)/4) and its check, canonical y; subgroup by
# phi(P') == [-x^2] P' on the isomorphic point P' = (rhs x, rhs^2) (2 products): [|x|] twice (63
# doublings + 5 mixed / 5 general additions), beta x and the Jacobian-affine compare.  (One chain over
# x^2 -- 127 doublings + 16 mixed additions -- spills less but measured slower: 2.09 vs 1.96 ms.)
WIRE_G1_DECODE = _add((1, 0), (2, 1), SQRT_CHAIN, (2, 1), (1, 0), (2, 1),
                      _scale(G1_DBL, 2 * NBITS), _scale(G1_MADD, NADD), _scale(G1_ADD, NADD), (5, 1))
# G2: to Montgomery, x^3 + b, the norm-method root (norm, two chains, s, t, t w, a1 w / 2, t w^2,
# the y^2 check), the sign's canonical compare; subgroup by psi(P) == [x] P: [|x|] (63 doublings +
# 5 mixed additions), psi and the compare
WIRE_G2_DECODE = _add((2, 0), (F2S + F2M, 0), (2, 2), _scale(SQRT_CHAIN, 2), (1, 0), (1, 1), (1, 0),
                      (1, 0), (2, 0), (1, 0), (F2S, 0), (6, 0),
                      _scale(G2_DBL, NBITS), _scale(G2_MADD, NADD), (2 + F2M, 0), (F2S + 3 * F2M, 0))
