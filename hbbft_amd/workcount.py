"""Algorithmic work of one share check, in Fp multiplications, derived from the kernel's own
formulas (csrc/tower.hpp, pairing.hpp, kernels.hpp).  Used by bench.py for the roofline's
'achieved' figure.  Fp2 mul = 3 Fp-mul (Karatsuba), Fp2 sqr = 2,
Fp2 x Fp = 2; an Fp squaring counts as one Fp-mul.
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

FP_INV = 380 + bin(0x1A0111EA397FE69A4B1BA7B6434BACD764774B84F38512BF6730D2A0F6B0F6241EABFFFEB153FFFFB9FEFFFFFFFFAAA9).count("1") - 1
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

if __name__ == "__main__":
    print("miller", MILLER_2PAIR, "g2 walk", G2_WALK, "final exp", FINAL_EXP, "(easy", EASY, "hard", HARD,
          ") total", FP_MULS_PER_CHECK)
