#!/usr/bin/env python3
"""Stage programs for the wave-per-check pairing kernel (hbbft_amd/csrc/k_wave.hip).

Why: a single pairing check (the master check of combine_and_verify_sig, src/threshold_sign.rs:264,
and the small per-message batches of the protocol flows) is a serial chain.  The lane-pair kernel
gives one check two lanes; here one check gets a whole wave -- 32 lane pairs -- and every Fp12 /
curve operation is cut into independent Fp2 products that run side by side, one per lane pair.

The kernel is a small interpreter.  A program is a list of STAGES; every stage is
  1. product phase: lane pair j forms X = +-(S[a] +- S[b]) and Y = +-(S[c] +- S[d]) from LDS slots
     and computes one Fp2 product X*Y (kind M1), a sum of two (M2, one reduction) or a square (SQ),
     written to slot PROD+j;
  2. assembly phase: lane pair o writes slot dst_o = sum c * V + xi * sum c' * V' over products and
     slots (small integer c, optional Fp2 conjugation per term), optionally gated by "side active".
Stages are separated by barriers.  This script builds the programs (Miller loop for each
WALK / TABLE side combination and the shared final exponentiation), list-schedules the operations
into stages under the 32-pair / 32-output / 7-term limits, checks every limb bound the kernel
relies on, and writes hbbft_amd/csrc/wave_prog.inc.  `emulate()` executes a program with exact
field arithmetic and is what tests/test_wave_prog.py checks against the oracle's pairing.

Formulas are those of pfp.hpp / k_pair.hip (pairing 0.14's line functions and final_exp chain):
the Fp12 element is kept in the w-basis f = sum f_k w^k, w^6 = xi = 1 + u (f_{2i} = c0_i,
f_{2i+1} = c1_i of the tower).
"""
import os
import sys

P = 0x1A0111EA397FE69A4B1BA7B6434BACD764774B84F38512BF6730D2A0F6B0F6241EABFFFEB153FFFFB9FEFFFFFFFFAAAB
X_ABS = 0xD201000000010000
NPAIRS = 32
MAXJ = 7
COEF_LIMIT = 8  # per accumulator: sum of positive / of negative coefficients (int32 limbs, 28-bit)

KIND = {"M1": 0, "M2": 1, "SQ": 2, "NONE": 3}
SPECIAL_INV = 1
SPECIAL_CYC = 2  # a run of cyclotomic squarings kept in registers (k_wave.hip cyc_run)

# fixed slot map shared with the kernel prologue
CONSTS = (["ZERO", "ONE"] + ["F1_%d" % k for k in range(6)] + ["F2_%d" % k for k in range(6)] + ["G1X", "G1Y", "G1NY"]
          + ["K12XI"])  # 12 xi = 3 b' (the homogeneous walk of mode W1J)
SIDE_FIELDS = ["XP", "YP", "QX", "QY", "TX", "TY", "TZ", "ZP"]  # ZP: Z^3 of a Jacobian P (mode WWJ)
MULF_G = ["S0_" + f for f in SIDE_FIELDS[:6]]


class Prod:
    """One Fp2 product term: X = sx * (S[a] + sb * S[b]), Y = sy * (S[c] + sd * S[d]), where sx / sy
    are -1 (neg), or a conjugation (conj)."""

    def __init__(self, a, c, b=None, sb=0, d=None, sd=0, negx=False, conjx=False, negy=False, conjy=False):
        self.a, self.b, self.sb, self.c, self.d, self.sd = a, b, sb, c, d, sd
        self.negx, self.conjx, self.negy, self.conjy = negx, conjx, negy, conjy


class Out:
    """dst = sum(plain terms) + xi * sum(twisted terms); term = (src, coef, conj) with src a slot name
    or ('P', j) = product j of the operation.  gate: None / 0 / 1 (side index): when that side is
    inactive the kernel writes `default` ('ONE' or 'ZERO') instead."""

    def __init__(self, dst, plain=(), tw=(), gate=None, default="ZERO"):
        self.dst, self.plain, self.tw, self.gate, self.default = dst, list(plain), list(tw), gate, default


class Op:
    def __init__(self, kind, prods=(), outs=(), special=None, tload=None, name=""):
        self.kind = kind          # M1 M2 SQ NONE INV TLOAD
        self.prods = list(prods)  # list of lists of Prod (K terms per lane pair)
        self.outs = list(outs)
        self.special = special    # ('INV', src, dst)
        self.tload = tload        # (side, step, first dst slot name of 3 consecutive)
        self.name = name
        self.stage = None

    def reads_prod(self):
        r = set()
        for pl in self.prods:
            for t in pl:
                for s in (t.a, t.b, t.c, t.d):
                    if s is not None:
                        r.add(s)
        if self.special:
            if self.special[0] == "CYC":
                r |= set(self.special[1])
            else:
                r.add(self.special[1])
        return r

    def reads_asm(self):
        r = set()
        for o in self.outs:
            for (src, _, _) in o.plain + o.tw:
                if not isinstance(src, tuple):
                    r.add(src)
            r.add(o.default)
        return r

    def writes(self):
        w = {o.dst for o in self.outs}
        if self.special:
            if self.special[0] == "CYC":
                w |= set(self.special[2])
            else:
                w.add(self.special[2])
        if self.tload:
            w |= set(self.tload[3])
        return w

    def j12(self):
        return (max([len(o.plain) for o in self.outs] or [0]), max([len(o.tw) for o in self.outs] or [0]))


# ------------------------------------------------------------------------------- operations
def P_(j):
    return ("P", j)


def op_sqr12(dst, src, conj_src=False):
    """dst = src^2 (or conj(src)^2): 21 products f_i f_j, i <= j."""
    prods, idx = [], {}
    for i in range(6):
        for j in range(i, 6):
            idx[(i, j)] = len(prods)
            prods.append([Prod(src[i], src[j])])
    outs = []
    for k in range(6):
        plain, tw = [], []
        for (i, j), q in sorted(idx.items()):
            s = i + j
            if s % 6 != k:
                continue
            c = 1 if i == j else 2
            if conj_src and (i + j) % 2 == 1:
                c = -c
            (tw if s >= 6 else plain).append((P_(q), c, 0))
        outs.append(Out(dst[k], plain, tw))
    return Op("M1", prods, outs, name="sqr12")


def op_mul12(dst, a, b, nega_odd=False, negb_odd=False, conj_out=False, m1=False):
    """dst = a * b (with a / b conjugated in Fp12 when nega_odd / negb_odd, dst conjugated when
    conj_out): 36 products, two per lane pair (M2) -- or one per lane pair (M1) in the 64-pair
    programs, where the 36 fit one stage."""
    if m1:
        prods, terms = [], {k: ([], []) for k in range(6)}
        for i in range(6):
            for j in range(6):
                sgn = (-1 if (nega_odd and i % 2) else 1) * (-1 if (negb_odd and j % 2) else 1)
                k = (i + j) % 6
                c = sgn * (-1 if (conj_out and k % 2) else 1)
                terms[k][1 if i + j >= 6 else 0].append((P_(len(prods)), c, 0))
                prods.append([Prod(a[i], b[j])])
        return Op("M1", prods, [Out(dst[k], *terms[k]) for k in range(6)], name="mul12m1")
    groups = {}
    for i in range(6):
        for j in range(6):
            s = i + j
            sign = (-1 if (nega_odd and i % 2) else 1) * (-1 if (negb_odd and j % 2) else 1)
            groups.setdefault((s % 6, s >= 6, sign), []).append((i, j))
    prods, outs_terms = [], {k: ([], []) for k in range(6)}
    for (k, tw, sign), lst in sorted(groups.items()):
        for q in range(0, len(lst), 2):
            chunk = lst[q:q + 2]
            terms = [Prod(a[i], b[j]) for (i, j) in chunk]
            if len(terms) == 1:
                terms.append(Prod("ZERO", "ZERO"))
            c = sign * (-1 if (conj_out and k % 2) else 1)
            outs_terms[k][1 if tw else 0].append((P_(len(prods)), c, 0))
            prods.append(terms)
    outs = [Out(dst[k], outs_terms[k][0], outs_terms[k][1]) for k in range(6)]
    return Op("M2", prods, outs, name="mul12")


def op_mul_line(dst, f, l, gate_free=True):
    """dst = f * (l0 + l1 w^2 + l2 w^3) (the 014-sparse line of pairing 0.14): 18 products."""
    prods, terms = [], {k: ([], []) for k in range(6)}
    for k in range(6):
        for (lc, sh) in ((l[0], 0), (l[1], 2), (l[2], 3)):
            o = k + sh
            terms[o % 6][1 if o >= 6 else 0].append((P_(len(prods)), 1, 0))
            prods.append([Prod(f[k], lc)])
    return Op("M1", prods, [Out(dst[k], *terms[k]) for k in range(6)], name="mulline")


def op_mul_fp6(dst, f, t):
    """dst = f * (t0 + t1 w^2 + t2 w^4) (an Fp6 element in the w-basis): 18 products."""
    prods, terms = [], {k: ([], []) for k in range(6)}
    for k in range(6):
        for j in range(3):
            o = k + 2 * j
            terms[o % 6][1 if o >= 6 else 0].append((P_(len(prods)), 1, 0))
            prods.append([Prod(f[k], t[j])])
    return Op("M1", prods, [Out(dst[k], *terms[k]) for k in range(6)], name="mulfp6")


def op_mul_ll(dst, a, b):
    """dst = a * b for two 014-sparse lines (positions 0, 2, 3 of the w-basis): 9 products; the
    result lives at positions 0, 2, 3, 4, 5 (w^6 = xi folds a3 b3 into position 0).  dst: 9 slots --
    the five positions and xi times positions 2, 3, 4, 5, so that op_mul_fl's wrapped terms are plain
    terms (an output of mixed plain / twisted terms would need 9 assembly terms per stage)."""
    prods = [[Prod(a[0], b[0])], [Prod(a[2], b[2])], [Prod(a[0], b[1])], [Prod(a[1], b[0])], [Prod(a[0], b[2])],
             [Prod(a[2], b[0])], [Prod(a[1], b[1])], [Prod(a[1], b[2])], [Prod(a[2], b[1])]]
    pos = {0: [P_(0)], 2: [P_(2), P_(3)], 3: [P_(4), P_(5)], 4: [P_(6)], 5: [P_(7), P_(8)]}
    outs = [Out(dst[0], [(P_(0), 1, 0)], [(P_(1), 1, 0)])]
    for k, sh in enumerate(LL_POS[1:]):
        outs.append(Out(dst[1 + k], [(q, 1, 0) for q in pos[sh]]))
        outs.append(Out(dst[5 + k], [], [(q, 1, 0) for q in pos[sh]]))
    return Op("M1", prods, outs, name="mulll")


LL_POS = (0, 2, 3, 4, 5)


def op_mul_fl(dst, f, ll):
    """dst = f * ll, ll a product of two lines (op_mul_ll's 9 slots: positions 0, 2, 3, 4, 5, then
    xi times positions 2, 3, 4, 5): 30 products, five plain terms per output."""
    prods, terms = [], {k: [] for k in range(6)}
    for k in range(6):
        for q, sh in enumerate(LL_POS):
            o = k + sh
            slot = ll[q] if o < 6 else ll[4 + q]
            terms[o % 6].append((P_(len(prods)), 1, 0))
            prods.append([Prod(f[k], slot)])
    return Op("M1", prods, [Out(dst[k], terms[k]) for k in range(6)], name="mulfl")


def op_cyclo(dst, f, conj_out=False):
    """Granger-Scott cyclotomic squaring (pfp.hpp h12_cyclo_sqr) on the Fp4 pairs (f0, f3),
    (f1, f4), (f2, f5): nine Fp2 squarings (SQ)."""
    prods = []

    def sq(x, y=None):
        prods.append([Prod(x, x, b=y, sb=1 if y else 0, d=y, sd=1 if y else 0)])
        return P_(len(prods) - 1)

    s0, s3, s03 = sq(f[0]), sq(f[3]), sq(f[0], f[3])
    s1, s4, s14 = sq(f[1]), sq(f[4]), sq(f[1], f[4])
    s2, s5, s25 = sq(f[2]), sq(f[5]), sq(f[2], f[5])
    spec = {
        0: ([(s0, 3), (f[0], -2)], [(s3, 3)]),
        3: ([(s03, 3), (s0, -3), (s3, -3), (f[3], 2)], []),
        2: ([(s1, 3), (f[2], -2)], [(s4, 3)]),
        5: ([(s14, 3), (s1, -3), (s4, -3), (f[5], 2)], []),
        1: ([(f[1], 2)], [(s25, 3), (s2, -3), (s5, -3)]),
        4: ([(s2, 3), (f[4], -2)], [(s5, 3)]),
    }
    outs = []
    for k in range(6):
        sg = -1 if (conj_out and k % 2) else 1
        pl, tw = spec[k]
        outs.append(Out(dst[k], [(s, c * sg, 0) for (s, c) in pl], [(s, c * sg, 0) for (s, c) in tw]))
    return Op("SQ", prods, outs, name="cyclo")


def op_cycrun(dst, f, count, conj_out=False):
    """`count` Granger-Scott cyclotomic squarings of f (op_cyclo's formulas) in ONE stage: k_wave's
    cyc_run keeps the three Fp4 squarings in registers of three lane rows and exchanges values by DPP
    and lane shuffles -- no LDS round trip or barrier per squaring.  dst conjugated when conj_out."""
    assert 1 <= count <= 255
    return Op("CYC", special=("CYC", list(f), list(dst), count, bool(conj_out)), name="cycrun")


def op_frob1(dst, f):
    prods = [[Prod(f[k], "F1_%d" % k, conjx=True)] for k in range(6)]
    return Op("M1", prods, [Out(dst[k], [(P_(k), 1, 0)]) for k in range(6)], name="frob1")


def op_frob2(dst, f):
    prods = [[Prod(f[k], "F2_%d" % k)] for k in range(6)]
    return Op("M1", prods, [Out(dst[k], [(P_(k), 1, 0)]) for k in range(6)], name="frob2")


def op_copy(dst, src, conj_out=False):
    return Op("NONE", [], [Out(dst[k], [(src[k], -1 if (conj_out and k % 2) else 1, 0)]) for k in range(6)],
              name="copy")


# ------------------------------------------------------------------------------- programs
class Builder:
    def __init__(self, name, cyc_runs=True, m1=False):
        self.name = name
        self.m1 = m1  # 64-pair programs: Fp12 products as 36 one-product pairs (M1) instead of 18 M2
        self.cyc_runs = cyc_runs  # final exponentiation squarings as CYC runs (False: one SQ stage each)
        self.slots = {}
        for c in CONSTS:
            self.slot(c)
        self.F = ["F%d" % k for k in range(6)]
        for name in self.F:
            self.slot(name)
        for s in range(2):
            for fld in SIDE_FIELDS:
                self.slot("S%d_%s" % (s, fld))
        for j in range(NPAIRS):
            self.slot("PROD%d" % j)
        self.ops = []

    def slot(self, name):
        if name not in self.slots:
            self.slots[name] = len(self.slots)
        return self.slots[name]

    def mul12(self, *a, **k):
        return op_mul12(*a, m1=self.m1, **k)

    def group(self, name, n=6):
        return [name + str(k) for k in range(n)]

    def add(self, op):
        if op.tload:
            for s in op.tload[3]:  # the kernel writes a table line into 3 consecutive slots
                self.slot(s)
        for s in sorted(op.reads_prod() | op.reads_asm() | op.writes()):
            self.slot(s)
        self.ops.append(op)
        return op

    # ---- Miller loop (k_pair.hip k_pair_verify): sides = ('W' | 'T', 'W' | 'T')
    def miller(self, modes):
        """modes[side] = 'W' (walk Q in the program) or 'T' (table lines); modes of length 3 ending in
        'J' (WWJ): both P given in Jacobian form (X, Y, Z): the kernel stores XP = X Z, YP = Y and
        ZP = Z^3, and every line's c0 is multiplied by ZP -- the line scaled by Z^3 (an Fp factor the
        final exponentiation removes), so P needs no inversion (the split master check's lambda_k g1)."""
        jac = len(modes) == 3 and modes[2] == "J"
        steps = []
        for b in range(62, -1, -1):
            steps.append("D")
            if (X_ABS >> b) & 1:
                steps.append("A")
        assert len(steps) == 68

        def S(side, fld):
            return "S%d_%s" % (side, fld)

        def L(side, s):
            return ["L%d_%d_%d" % (side, s % 2, c) for c in range(3)]

        def walk(side, s):
            T = lambda n: "W%d_%s" % (side, n)
            TX, TY, TZ, XP, YP, QX, QY = (S(side, f) for f in ("TX", "TY", "TZ", "XP", "YP", "QX", "QY"))
            l = L(side, s)
            if modes[side] == "T":
                raw = ["R%d_%d_%d" % (side, s % 2, c) for c in range(3)]
                self.add(Op("TLOAD", tload=(side, s, raw[0], raw), name="tload"))
                self.add(Op("M1", [[Prod(raw[1], XP)], [Prod(raw[2], YP)]],
                            [Out(l[0], [(raw[0], 1, 0)], gate=side, default="ONE"),
                             Out(l[1], [(P_(0), 1, 0)], gate=side), Out(l[2], [(P_(1), 1, 0)], gate=side)],
                            name="tbl"))
                return
            if steps[s] == "D":
                # h_dbl_step with D = 4 X B (= 2((X+B)^2 - A - C)), levels of independent products
                self.add(Op("M1", [[Prod(TX, TX)], [Prod(TY, TY)], [Prod(TZ, TZ)],
                                   [Prod(TY, TY, b=TZ, sb=1, d=TZ, sd=1)]],
                            [Out(T("E"), [(P_(0), 3, 0)]), Out(T("B"), [(P_(1), 1, 0)]),
                             Out(T("ZZ"), [(P_(2), 1, 0)]),
                             Out(TZ, [(P_(3), 1, 0), (P_(1), -1, 0), (P_(2), -1, 0)])], name="dbl1"))
                l0 = T("L0R") if jac else l[0]
                self.add(Op("M1", [[Prod(T("B"), T("B"))], [Prod(TX, T("B"))], [Prod(T("E"), T("E"))],
                                   [Prod(T("E"), TX)], [Prod(T("E"), T("ZZ"))], [Prod(TZ, T("ZZ"))]],
                            [Out(T("C"), [(P_(0), 1, 0)]), Out(T("D"), [(P_(1), 4, 0)]),
                             Out(TX, [(P_(2), 1, 0), (P_(1), -8, 0)]),
                             Out(l0, [(P_(3), 1, 0), (T("B"), -2, 0)], **({} if jac else dict(gate=side, default="ONE"))),
                             Out(T("LC1"), [(P_(4), -1, 0)]), Out(T("LC4"), [(P_(5), 1, 0)])], name="dbl2"))
                prods = [[Prod(T("E"), T("D"), d=TX, sd=-1)], [Prod(T("LC1"), XP)], [Prod(T("LC4"), YP)]]
                outs = [Out(TY, [(P_(0), 1, 0), (T("C"), -8, 0)]),
                        Out(l[1], [(P_(1), 1, 0)], gate=side), Out(l[2], [(P_(2), 1, 0)], gate=side)]
                if jac:
                    prods.append([Prod(l0, S(side, "ZP"))])
                    outs.append(Out(l[0], [(P_(3), 1, 0)], gate=side, default="ONE"))
                self.add(Op("M1", prods, outs, name="dbl3"))
            else:
                # h_add_step (mixed addition with the affine Q)
                self.add(Op("M1", [[Prod(TZ, TZ)], [Prod(QY, TZ)]],
                            [Out(T("Z1Z1"), [(P_(0), 1, 0)]), Out(T("YQZ"), [(P_(1), 1, 0)])], name="add1"))
                self.add(Op("M1", [[Prod(QX, T("Z1Z1"))], [Prod(T("YQZ"), T("Z1Z1"))]],
                            [Out(T("H"), [(P_(0), 1, 0), (TX, -1, 0)]), Out(T("R"), [(P_(1), 1, 0), (TY, -1, 0)])],
                            name="add2"))
                self.add(Op("M1", [[Prod(T("H"), T("H"))], [Prod(T("R"), T("R"))], [Prod(TZ, T("H"))],
                                   [Prod(T("R"), QX)]],
                            [Out(T("HH"), [(P_(0), 1, 0)]), Out(T("RR"), [(P_(1), 1, 0)]), Out(TZ, [(P_(2), 1, 0)]),
                             Out(T("RXQ"), [(P_(3), 1, 0)])], name="add3"))
                l0 = T("L0R") if jac else l[0]
                self.add(Op("M1", [[Prod(T("H"), T("HH"))], [Prod(TX, T("HH"))], [Prod(QY, TZ)],
                                   [Prod(T("R"), XP)], [Prod(TZ, YP)]],
                            [Out(T("HHH"), [(P_(0), 1, 0)]), Out(T("V"), [(P_(1), 1, 0)]),
                             Out(TX, [(T("RR"), 1, 0), (P_(0), -1, 0), (P_(1), -2, 0)]),
                             Out(l0, [(T("RXQ"), 1, 0), (P_(2), -1, 0)], **({} if jac else dict(gate=side, default="ONE"))),
                             Out(l[1], [(P_(3), -1, 0)], gate=side), Out(l[2], [(P_(4), 1, 0)], gate=side)],
                            name="add4"))
                prods = [[Prod(T("R"), T("V"), d=TX, sd=-1)], [Prod(TY, T("HHH"))]]
                outs = [Out(TY, [(P_(0), 1, 0), (P_(1), -1, 0)])]
                if jac:
                    prods.append([Prod(l0, S(side, "ZP"))])
                    outs.append(Out(l[0], [(P_(2), 1, 0)], gate=side, default="ONE"))
                self.add(Op("M1", prods, outs, name="add5"))

        for side in (0, 1):
            walk(side, 0)
        for s, typ in enumerate(steps):
            if s + 1 < len(steps):
                for side in (0, 1):
                    walk(side, s + 1)
            if typ == "D" and s > 0:
                self.add(op_sqr12(self.F, self.F))
            for side in (0, 1):
                self.add(op_mul_line(self.F, self.F, L(side, s)))

    # ---- Miller loop of ONE pair (mode W1J: the split master check, one pair per wave)
    def miller1(self):
        """Side 0 only, WALK, Jacobian P (XP = X Z, YP = Y, ZP = Z^3 as in WWJ).  T is kept in
        HOMOGENEOUS projective coordinates (x = X/Z, y = Y/Z) with Zk = 12 xi Z = 3 b' Z carried along,
        so a doubling is two product levels instead of three (Costello-Lange-Naehrig / Aranha et al.
        2011 formulas for a = 0, scaled by -4 to clear the halves):
          X3 = -2 XY (B - 3 E), Y3 = 12 E^2 - (B + 3 E)^2, Z3 = -8 B YZ, Zk3 = -8 B (Y Zk)
          (B = Y^2, E = Z Zk = 3 b' Z^2), line (c0, c1, c4) = (B - E, -3 X^2, 2 YZ);
        a mixed addition is four levels (theta = Y - yQ Z, lambda = X - xQ Z; line (theta xQ - lambda
        yQ, -theta, lambda)).  These lines are pairing 0.14's times Fp2 factors, which the final
        exponentiation removes, and with one pair the f update (square, then one sparse line) is two
        stages per step like the walk: ~145 stages instead of 211."""
        steps = []
        for b in range(62, -1, -1):
            steps.append("D")
            if (X_ABS >> b) & 1:
                steps.append("A")
        XP, YP, ZP, QX, QY, TX, TY, TZ = ("S0_" + f for f in ("XP", "YP", "ZP", "QX", "QY", "TX", "TY", "TZ"))
        ZK = "W0_ZK"
        T = lambda n: "W0_" + n
        L = lambda s: ["L0_%d_%d" % (s % 2, c) for c in range(3)]
        self.add(Op("NONE", [], [Out(ZK, [("K12XI", 1, 0)])], name="zk0"))  # Z = 1

        def walk(s):
            l = L(s)
            if steps[s] == "D":
                self.add(Op("M1", [[Prod(TX, TX)], [Prod(TY, TY)], [Prod(TZ, ZK)], [Prod(TX, TY)], [Prod(TY, TZ)],
                                   [Prod(TY, ZK)]],
                            [Out(T("LC1"), [(P_(0), -3, 0)]), Out(T("B"), [(P_(1), 1, 0)]),
                             Out(T("BFM"), [(P_(1), 1, 0), (P_(2), -3, 0)]), Out(T("BFP"), [(P_(1), 1, 0), (P_(2), 3, 0)]),
                             Out(T("E2"), [(P_(2), 2, 0)]), Out(T("E6"), [(P_(2), 6, 0)]), Out(T("XY"), [(P_(3), 1, 0)]),
                             Out(T("YZ"), [(P_(4), 1, 0)]), Out(T("LC4"), [(P_(4), 2, 0)]), Out(T("YZK"), [(P_(5), 1, 0)]),
                             Out(T("L0R"), [(P_(1), 1, 0), (P_(2), -1, 0)])], name="hdbl1"))
                self.add(Op("M1", [[Prod(T("XY"), T("BFM"))], [Prod(T("BFP"), T("BFP"))], [Prod(T("E2"), T("E6"))],
                                   [Prod(T("B"), T("YZ"))], [Prod(T("B"), T("YZK"))], [Prod(T("LC1"), XP)],
                                   [Prod(T("LC4"), YP)], [Prod(T("L0R"), ZP)]],
                            [Out(TX, [(P_(0), -2, 0)]), Out(TY, [(P_(2), 1, 0), (P_(1), -1, 0)]),
                             Out(TZ, [(P_(3), -8, 0)]), Out(ZK, [(P_(4), -8, 0)]),
                             Out(l[1], [(P_(5), 1, 0)], gate=0), Out(l[2], [(P_(6), 1, 0)], gate=0),
                             Out(l[0], [(P_(7), 1, 0)], gate=0, default="ONE")], name="hdbl2"))
            else:
                self.add(Op("M1", [[Prod(QY, TZ)], [Prod(QX, TZ)]],
                            [Out(T("TH"), [(TY, 1, 0), (P_(0), -1, 0)]), Out(T("LA"), [(TX, 1, 0), (P_(1), -1, 0)])],
                            name="hadd1"))
                self.add(Op("M1", [[Prod(T("TH"), T("TH"))], [Prod(T("LA"), T("LA"))], [Prod(T("TH"), QX)],
                                   [Prod(T("LA"), QY)], [Prod(T("TH"), XP)], [Prod(T("LA"), YP)]],
                            [Out(T("C"), [(P_(0), 1, 0)]), Out(T("D"), [(P_(1), 1, 0)]),
                             Out(T("L0R"), [(P_(2), 1, 0), (P_(3), -1, 0)]),
                             Out(l[1], [(P_(4), -1, 0)], gate=0), Out(l[2], [(P_(5), 1, 0)], gate=0)], name="hadd2"))
                self.add(Op("M1", [[Prod(T("LA"), T("D"))], [Prod(TZ, T("C"))], [Prod(TX, T("D"))], [Prod(T("L0R"), ZP)]],
                            [Out(T("E"), [(P_(0), 1, 0)]), Out(T("G"), [(P_(2), 1, 0)]),
                             Out(T("H"), [(P_(0), 1, 0), (P_(1), 1, 0), (P_(2), -2, 0)]),
                             Out(l[0], [(P_(3), 1, 0)], gate=0, default="ONE")], name="hadd3"))
                self.add(Op("M1", [[Prod(T("LA"), T("H"))], [Prod(T("TH"), T("G"), d=T("H"), sd=-1)], [Prod(TY, T("E"))],
                                   [Prod(TZ, T("E"))], [Prod(ZK, T("E"))]],
                            [Out(TX, [(P_(0), 1, 0)]), Out(TY, [(P_(1), 1, 0), (P_(2), -1, 0)]),
                             Out(TZ, [(P_(3), 1, 0)]), Out(ZK, [(P_(4), 1, 0)])], name="hadd4"))

        walk(0)
        for s, typ in enumerate(steps):
            if s + 1 < len(steps):
                walk(s + 1)
            if typ == "D" and s > 0:
                self.add(op_sqr12(self.F, self.F))
            self.add(op_mul_line(self.F, self.F, L(s)))

    # ---- Miller loop with combined lines (the 64-pair programs of k_wave64)
    def miller_c(self, modes):
        """Two pairs, 64 lane pairs per check.  Per step the two lines are multiplied together first
        (op_mul_ll, 9 products, beside f^2's 21) and f takes their product in one 30-product stage
        (op_mul_fl): f costs two stages per step where multiplying the lines in one by one costs three.
        A WALK side keeps T in homogeneous projective coordinates with Zk = 12 xi Z (miller1's
        formulas: a doubling is two product levels instead of three) and affine P, so its line needs no
        Z^3 scaling; a TABLE side reads the k_oct_prep lines as in miller().  The lines are pairing
        0.14's up to Fp2 factors, which the final exponentiation removes."""
        steps = []
        for b in range(62, -1, -1):
            steps.append("D")
            if (X_ABS >> b) & 1:
                steps.append("A")
        assert len(steps) == 68

        def S(side, fld):
            return "S%d_%s" % (side, fld)

        def L(side, s):
            return ["L%d_%d_%d" % (side, s % 2, c) for c in range(3)]

        for side in (0, 1):
            if modes[side] == "W":
                self.add(Op("NONE", [], [Out("W%d_ZK" % side, [("K12XI", 1, 0)])], name="zk0"))

        def walk(side, s):
            T = lambda n: "W%d_%s" % (side, n)
            TX, TY, TZ, XP, YP, QX, QY = (S(side, f) for f in ("TX", "TY", "TZ", "XP", "YP", "QX", "QY"))
            ZK = T("ZK")
            l = L(side, s)
            if modes[side] == "T":
                raw = ["R%d_%d_%d" % (side, s % 2, c) for c in range(3)]
                self.add(Op("TLOAD", tload=(side, s, raw[0], raw), name="tload"))
                self.add(Op("M1", [[Prod(raw[1], XP)], [Prod(raw[2], YP)]],
                            [Out(l[0], [(raw[0], 1, 0)], gate=side, default="ONE"),
                             Out(l[1], [(P_(0), 1, 0)], gate=side), Out(l[2], [(P_(1), 1, 0)], gate=side)],
                            name="tbl"))
                return
            if steps[s] == "D":
                self.add(Op("M1", [[Prod(TX, TX)], [Prod(TY, TY)], [Prod(TZ, ZK)], [Prod(TX, TY)], [Prod(TY, TZ)],
                                   [Prod(TY, ZK)]],
                            [Out(T("LC1"), [(P_(0), -3, 0)]), Out(T("B"), [(P_(1), 1, 0)]),
                             Out(T("BFM"), [(P_(1), 1, 0), (P_(2), -3, 0)]), Out(T("BFP"), [(P_(1), 1, 0), (P_(2), 3, 0)]),
                             Out(T("E2"), [(P_(2), 2, 0)]), Out(T("E6"), [(P_(2), 6, 0)]), Out(T("XY"), [(P_(3), 1, 0)]),
                             Out(T("YZ"), [(P_(4), 1, 0)]), Out(T("LC4"), [(P_(4), 2, 0)]), Out(T("YZK"), [(P_(5), 1, 0)]),
                             Out(l[0], [(P_(1), 1, 0), (P_(2), -1, 0)], gate=side, default="ONE")], name="hdbl1"))
                self.add(Op("M1", [[Prod(T("XY"), T("BFM"))], [Prod(T("BFP"), T("BFP"))], [Prod(T("E2"), T("E6"))],
                                   [Prod(T("B"), T("YZ"))], [Prod(T("B"), T("YZK"))], [Prod(T("LC1"), XP)],
                                   [Prod(T("LC4"), YP)]],
                            [Out(TX, [(P_(0), -2, 0)]), Out(TY, [(P_(2), 1, 0), (P_(1), -1, 0)]),
                             Out(TZ, [(P_(3), -8, 0)]), Out(ZK, [(P_(4), -8, 0)]),
                             Out(l[1], [(P_(5), 1, 0)], gate=side), Out(l[2], [(P_(6), 1, 0)], gate=side)],
                            name="hdbl2"))
            else:
                self.add(Op("M1", [[Prod(QY, TZ)], [Prod(QX, TZ)]],
                            [Out(T("TH"), [(TY, 1, 0), (P_(0), -1, 0)]), Out(T("LA"), [(TX, 1, 0), (P_(1), -1, 0)])],
                            name="hadd1"))
                self.add(Op("M1", [[Prod(T("TH"), T("TH"))], [Prod(T("LA"), T("LA"))], [Prod(T("TH"), QX)],
                                   [Prod(T("LA"), QY)], [Prod(T("TH"), XP)], [Prod(T("LA"), YP)]],
                            [Out(T("C"), [(P_(0), 1, 0)]), Out(T("D"), [(P_(1), 1, 0)]),
                             Out(l[0], [(P_(2), 1, 0), (P_(3), -1, 0)], gate=side, default="ONE"),
                             Out(l[1], [(P_(4), -1, 0)], gate=side), Out(l[2], [(P_(5), 1, 0)], gate=side)],
                            name="hadd2"))
                self.add(Op("M1", [[Prod(T("LA"), T("D"))], [Prod(TZ, T("C"))], [Prod(TX, T("D"))]],
                            [Out(T("E"), [(P_(0), 1, 0)]), Out(T("G"), [(P_(2), 1, 0)]),
                             Out(T("H"), [(P_(0), 1, 0), (P_(1), 1, 0), (P_(2), -2, 0)])], name="hadd3"))
                self.add(Op("M1", [[Prod(T("LA"), T("H"))], [Prod(T("TH"), T("G"), d=T("H"), sd=-1)], [Prod(TY, T("E"))],
                                   [Prod(TZ, T("E"))], [Prod(ZK, T("E"))]],
                            [Out(TX, [(P_(0), 1, 0)]), Out(TY, [(P_(1), 1, 0), (P_(2), -1, 0)]),
                             Out(TZ, [(P_(3), 1, 0)]), Out(ZK, [(P_(4), 1, 0)])], name="hadd4"))

        LL = ["LL%d" % k for k in LL_POS] + ["XLL%d" % k for k in LL_POS[1:]]
        for side in (0, 1):
            walk(side, 0)
        for s, typ in enumerate(steps):
            if s + 1 < len(steps):
                for side in (0, 1):
                    walk(side, s + 1)
            if typ == "D" and s > 0:
                self.add(op_sqr12(self.F, self.F))
            self.add(op_mul_ll(LL, L(0, s), L(1, s)))
            self.add(op_mul_fl(self.F, self.F, LL))

    # ---- final exponentiation (k_pair.hip h_final_exp, the chain of pairing.hpp final_exp_x3)
    def final_exp(self):
        F = self.F
        G, T, A, B, X1, X2, FR, R = (self.group(n) for n in ("G", "T", "A", "B", "X1", "X2", "FR", "RS"))
        t = self.group("IT", 3)
        c = self.group("IC", 3)
        ti = self.group("ITI", 3)
        f0, f1, f2, f3, f4, f5 = F
        # f1 = conj(f)^2 / (f conj(f)); f conj(f) = c0^2 - v c1^2 is in Fp6
        self.add(op_sqr12(R, F, conj_src=True))
        prods = [[Prod(a, b)] for (a, b) in ((f0, f0), (f2, f4), (f3, f3), (f1, f5), (f0, f2), (f4, f4), (f1, f1),
                                             (f3, f5), (f2, f2), (f0, f4), (f1, f3), (f5, f5))]
        self.add(Op("M1", prods, [
            Out(t[0], [(P_(0), 1, 0)], [(P_(1), 2, 0), (P_(2), -1, 0), (P_(3), -2, 0)]),
            Out(t[1], [(P_(4), 2, 0), (P_(6), -1, 0)], [(P_(5), 1, 0), (P_(7), -2, 0)]),
            Out(t[2], [(P_(8), 1, 0), (P_(9), 2, 0), (P_(10), -2, 0)], [(P_(11), -1, 0)])], name="inv1"))
        self.add(Op("M1", [[Prod(t[0], t[0])], [Prod(t[1], t[2])], [Prod(t[2], t[2])], [Prod(t[0], t[1])],
                           [Prod(t[1], t[1])], [Prod(t[0], t[2])]], [
            Out(c[0], [(P_(0), 1, 0)], [(P_(1), -1, 0)]),
            Out(c[1], [(P_(3), -1, 0)], [(P_(2), 1, 0)]),
            Out(c[2], [(P_(4), 1, 0), (P_(5), -1, 0)])], name="inv2"))
        self.add(Op("M1", [[Prod(t[0], c[0])], [Prod(t[2], c[1])], [Prod(t[1], c[2])]],
                    [Out("IN", [(P_(0), 1, 0)], [(P_(1), 1, 0), (P_(2), 1, 0)])], name="inv3"))
        self.add(Op("INV", special=("INV", "IN", "INI"), name="inv4"))
        self.add(Op("M1", [[Prod(c[k], "INI")] for k in range(3)], [Out(ti[k], [(P_(k), 1, 0)]) for k in range(3)],
                    name="inv5"))
        self.add(op_mul_fp6(X1, R, ti))                 # f1 = f^(p^6 - 1)
        self.add(op_frob2(X2, X1))
        self.add(self.mul12(G, X2, X1))                   # g = f1^(p^2 + 1)

        def exp(dst, base, plus1, conj_out):
            e = X_ABS + (1 if plus1 else 0)
            src, run = base, 0
            for k in range(62, -1, -1):
                run += 1
                bit = (e >> k) & 1
                if bit or k == 0:  # a run of squarings ends at each set bit (and at the end)
                    if self.cyc_runs:
                        self.add(op_cycrun(dst, src, run, conj_out=conj_out and k == 0 and not bit))
                    else:
                        for q in range(run):
                            last = q == run - 1 and k == 0 and not bit
                            self.add(op_cyclo(dst, src if q == 0 else dst, conj_out=conj_out and last))
                    src, run = dst, 0
                if bit:
                    self.add(self.mul12(dst, dst, base, conj_out=conj_out and k == 0))

        if self.cyc_runs:
            self.add(op_cycrun(X1, G, 1))               # cyclo(g) g, needed for w
        else:
            self.add(op_cyclo(X1, G))
        self.add(self.mul12(X1, X1, G))
        exp(T, G, True, True)                           # t = g^(x-1)
        exp(A, T, True, True)                           # a = t^(x-1)
        exp(T, A, False, True)                          # t = a^x
        self.add(op_frob1(FR, A))
        self.add(self.mul12(B, T, FR))                    # b = a^x frob1(a)
        self.add(op_frob2(X2, B))
        self.add(self.mul12(X2, X2, B, negb_odd=True))    # frob2(b) conj(b)
        self.add(self.mul12(X1, X2, X1))                  # w
        exp(T, B, False, True)                          # b^x
        exp(A, T, False, True)                          # c = (b^x)^x
        self.add(self.mul12(self.group("E"), A, X1))      # e = c w
        return self.group("E")

    # ---- F <- F * G: the product of partial Miller values (the split master check of
    # hbh_combine_verify_g2); G is loaded into side 0's first six slots, free once no Miller runs
    def mulf(self):
        self.add(op_mul12(self.F, self.F, MULF_G))


# ------------------------------------------------------------------------------- scheduler
class Stage:
    def __init__(self):
        self.ops = []
        self.kind = None
        self.npairs = 0
        self.nouts = 0
        self.j1 = 0
        self.j2 = 0
        self.tload = {}
        self.special = None


def op_ok_in(op, st):
    if op.kind == "TLOAD":
        return op.tload[0] not in st.tload and st.special is None
    if op.kind in ("INV", "CYC"):
        return not st.ops
    if st.special is not None:
        return False
    if op.kind in ("M1", "M2", "SQ"):
        if st.kind not in (None, "NONE"):
            if op.kind == "SQ" and st.kind != "SQ":
                return False
            if op.kind != "SQ" and st.kind == "SQ":
                return False
            if op.kind == "M2" and st.kind == "M1":
                return False
        if st.npairs + len(op.prods) > NPAIRS:
            return False
    if st.nouts + len(op.outs) > NPAIRS:
        return False
    j1, j2 = op.j12()
    if max(st.j1, j1) + max(st.j2, j2) > MAXJ:
        return False
    return True


def schedule(ops):
    stages = []
    last_w, last_rp, last_ra = {}, {}, {}
    for op in ops:
        lb = 0
        for s in op.reads_prod() | op.reads_asm():
            if s in last_w:
                lb = max(lb, last_w[s] + 1)
        for s in op.writes():
            lb = max(lb, last_rp.get(s, -1), last_ra.get(s, -2) + 1, last_w.get(s, -2) + 1)
        t = lb
        while t < len(stages) and not op_ok_in(op, stages[t]):
            t += 1
        while t >= len(stages):
            stages.append(Stage())
        st = stages[t]
        op.stage = t
        op.pair0 = st.npairs
        op.out0 = st.nouts
        st.ops.append(op)
        if op.kind == "TLOAD":
            st.tload[op.tload[0]] = op
        elif op.kind in ("INV", "CYC"):
            st.special = op
            st.kind = "NONE"
        else:
            if op.kind in ("M1", "M2", "SQ"):
                if st.kind in (None, "NONE"):
                    st.kind = op.kind
                st.npairs += len(op.prods)
            elif st.kind is None:
                st.kind = "NONE"
            st.nouts += len(op.outs)
            j1, j2 = op.j12()
            st.j1, st.j2 = max(st.j1, j1), max(st.j2, j2)
        for s in op.reads_prod():
            last_rp[s] = max(last_rp.get(s, -1), t)
        for s in op.reads_asm():
            last_ra[s] = max(last_ra.get(s, -1), t)
        for s in op.writes():
            last_w[s] = max(last_w.get(s, -1), t)
    for st in stages:
        if st.kind is None:
            st.kind = "NONE"
    return stages


def check_bounds(op):
    """int32 limb accumulators: per lane component, positive and negative coefficient sums <= 8, and
    <= 6 for the plain terms of an output with twisted terms (the kernel adds the normalised twisted
    sum and its partner component, up to 2 x 2^28 per limb, before the final carry pass)."""
    for o in op.outs:
        for terms in (o.plain, o.tw):
            limit = COEF_LIMIT - 2 if (terms is o.plain and o.tw) else COEF_LIMIT
            for h in (0, 1):
                pos = neg = 0
                for (_, c, cj) in terms:
                    ce = -c if (cj and h) else c
                    if ce > 0:
                        pos += ce
                    else:
                        neg -= ce
                assert pos <= limit and neg <= limit, (op.name, o.dst, terms)
                for (_, c, _) in terms:
                    assert -8 <= c <= 7, (op.name, c)


# ------------------------------------------------------------------------------- encoding
def encode(b, stages):
    """Headers (4 u32 per stage), product descriptors (u64 per lane pair and term) and assembly
    descriptors (8 u16 per output), deduplicated by content."""
    S = b.slots
    assert len(S) <= 256, len(S)
    hdrs, pdesc, adesc = [], [], []
    pcache, acache = {}, {}

    def sgn(v):
        return {0: 0, 1: 1, -1: 2}[v]

    for st in stages:
        K = 2 if st.kind == "M2" else 1
        pblock, ablock = [], []
        flags_xsum = flags_ysum = flags_neg = flags_conj = 0
        for op in st.ops:
            if op.kind in ("M1", "M2", "SQ"):
                for pl in op.prods:
                    terms = list(pl) + [Prod("ZERO", "ZERO")] * (K - len(pl))
                    assert len(terms) == K
                    for t in terms:
                        a, bb = S[t.a], S[t.b] if t.b else S["ZERO"]
                        c, d = S[t.c], S[t.d] if t.d else S["ZERO"]
                        w = a | (bb << 8) | (c << 16) | (d << 24)
                        w |= sgn(t.sb) << 32 | sgn(t.sd) << 34
                        w |= (int(t.negx) << 36) | (int(t.conjx) << 37) | (int(t.negy) << 38) | (int(t.conjy) << 39)
                        flags_xsum |= int(t.sb != 0)
                        flags_ysum |= int(t.sd != 0)
                        flags_neg |= int(t.negx or t.negy)
                        flags_conj |= int(t.conjx or t.conjy)
                        pblock.append(w)
            for o in op.outs:
                check_bounds(op)
                gate = 0 if o.gate is None else 1 + o.gate
                ws = [S[o.dst] | (gate << 8) | ((1 if o.default == "ONE" else 0) << 10)]

                def term(tm):
                    src, c, cj = tm
                    if isinstance(src, tuple):
                        idx = S["PROD%d" % (op.pair0 + src[1])]
                    else:
                        idx = S[src]
                    return idx | ((c & 0xF) << 8) | (int(bool(cj)) << 12)

                pl = [term(t) for t in o.plain] + [S["ZERO"]] * (st.j1 - len(o.plain))
                tw = [term(t) for t in o.tw] + [S["ZERO"]] * (st.j2 - len(o.tw))
                ws += pl + tw
                ws += [0] * (8 - len(ws))
                assert len(ws) == 8
                ablock.extend(ws)
        key = tuple(pblock)
        if key not in pcache:
            pcache[key] = len(pdesc)
            pdesc.extend(pblock)
        akey = tuple(ablock)
        if akey not in acache:
            acache[akey] = len(adesc) // 8
            adesc.extend(ablock)
        h0 = KIND[st.kind] | (st.j1 << 2) | (st.j2 << 5) | (flags_xsum << 8) | (flags_ysum << 9) | (flags_neg << 10)
        h0 |= (flags_conj << 11)
        h3 = 0
        if st.special is not None and st.special.special[0] == "CYC":
            _, src, dst, count, conj = st.special.special
            w0 = sum(S[n] << (8 * k) for k, n in enumerate(src))
            w1 = sum(S[n] << (8 * k) for k, n in enumerate(dst)) | (count << 48) | (int(conj) << 56)
            key = (w0, w1)
            if key not in pcache:
                pcache[key] = len(pdesc)
                pdesc.extend([w0, w1])
            h0 |= SPECIAL_CYC << 12
        elif st.special is not None:
            h0 |= SPECIAL_INV << 12
            h3 = S[st.special.special[1]] | (S[st.special.special[2]] << 8)
        else:
            for side, op in st.tload.items():
                raw = op.tload[3]
                assert [S[r] for r in raw] == [S[raw[0]] + k for k in range(3)]
                h3 |= (1 | (op.tload[1] << 1) | (S[raw[0]] << 8)) << (16 * side)
        assert st.npairs < 128 and st.nouts < 128
        h0 |= (st.npairs << 16) | (st.nouts << 23)
        hdrs.extend([h0, pcache[key], acache[akey], h3])
    return hdrs, pdesc, adesc


# ------------------------------------------------------------------------------- emulator
def f2add(a, b):
    return ((a[0] + b[0]) % P, (a[1] + b[1]) % P)


def f2mul(a, b):
    return ((a[0] * b[0] - a[1] * b[1]) % P, (a[0] * b[1] + a[1] * b[0]) % P)


def f2scale(a, c):
    return ((a[0] * c) % P, (a[1] * c) % P)


def f2conj(a):
    return (a[0], (-a[1]) % P)


def f2xi(a):
    return ((a[0] - a[1]) % P, (a[0] + a[1]) % P)


def cyclo_w(f):
    """Granger-Scott cyclotomic squaring on the w-basis (op_cyclo's formulas)."""
    sq = lambda x: f2mul(x, x)
    s0, s3, s03 = sq(f[0]), sq(f[3]), sq(f2add(f[0], f[3]))
    s1, s4, s14 = sq(f[1]), sq(f[4]), sq(f2add(f[1], f[4]))
    s2, s5, s25 = sq(f[2]), sq(f[5]), sq(f2add(f[2], f[5]))
    lin = lambda a, b, c: f2add(f2scale(a, 3), f2scale(b, c))
    u = lambda sab, sa, sb: f2add(sab, f2scale(f2add(sa, sb), -1))
    return [lin(f2add(s0, f2xi(s3)), f[0], -2), f2add(f2scale(f[1], 2), f2scale(f2xi(u(s25, s2, s5)), 3)),
            lin(f2add(s1, f2xi(s4)), f[2], -2), lin(u(s03, s0, s3), f[3], 2),
            lin(f2add(s2, f2xi(s5)), f[4], -2), lin(u(s14, s1, s4), f[5], 2)]


def f2pow(a, e):
    r = (1, 0)
    while e:
        if e & 1:
            r = f2mul(r, a)
        a = f2mul(a, a)
        e >>= 1
    return r


def f2inv(a):
    n = (a[0] * a[0] + a[1] * a[1]) % P
    ni = pow(n, P - 2, P)
    return ((a[0] * ni) % P, (-a[1] * ni) % P)


def const_values():
    xi = (1, 1)
    v = {"ZERO": (0, 0), "ONE": (1, 0)}
    for k in range(6):
        v["F1_%d" % k] = f2pow(xi, k * (P - 1) // 6)
        v["F2_%d" % k] = f2pow(xi, k * (P * P - 1) // 6)
    g1x = 0x17F1D3A73197D7942695638C4FA9AC0FC3688C4F9774B905A14E3A3F171BAC586C55E83FF97A1AEFFB3AF00ADB22C6BB
    g1y = 0x08B3F481E3AAA0F1A09E30ED741D8AE4FCF5E095D5D00AF600DB18CB2C04B3EDD03CC744A2888AE40CAA232946C5E7E1
    v["G1X"], v["G1Y"], v["G1NY"] = (g1x, 0), (g1y, 0), ((-g1y) % P, 0)
    v["K12XI"] = (12, 12)
    return v


def raw_lines(Q):
    """Raw (c0, c1, c4) lines of the lane-pair walk (pfp.hpp h_dbl_step / h_add_step) from Q, as
    k_pair_prep stores them; Q = None walks from (1, 1) like the kernel."""
    xq, yq = Q if Q is not None else ((1, 0), (1, 0))
    X, Y, Z = xq, yq, (1, 0)
    out = []
    for b in range(62, -1, -1):
        for add in range(2 if (X_ABS >> b) & 1 else 1):
            if not add:
                A, Bv, ZZ = f2mul(X, X), f2mul(Y, Y), f2mul(Z, Z)
                C = f2mul(Bv, Bv)
                XB2 = f2mul(f2add(X, Bv), f2add(X, Bv))
                D = f2scale(f2add(f2add(XB2, f2scale(A, -1)), f2scale(C, -1)), 2)
                E = f2scale(A, 3)
                c0 = f2add(f2mul(E, X), f2scale(Bv, -2))
                c1 = f2scale(f2mul(E, ZZ), -1)
                YZ = f2add(Y, Z)
                Z3 = f2add(f2add(f2mul(YZ, YZ), f2scale(Bv, -1)), f2scale(ZZ, -1))
                c4 = f2mul(Z3, ZZ)
                F = f2mul(E, E)
                X3 = f2add(F, f2scale(D, -2))
                Y = f2add(f2mul(E, f2add(D, f2scale(X3, -1))), f2scale(C, -8))
                X, Z = X3, Z3
            else:
                Z1Z1 = f2mul(Z, Z)
                U2 = f2mul(xq, Z1Z1)
                S2 = f2mul(f2mul(yq, Z), Z1Z1)
                H = f2add(U2, f2scale(X, -1))
                r = f2add(S2, f2scale(Y, -1))
                HH = f2mul(H, H)
                HHH = f2mul(H, HH)
                V = f2mul(X, HH)
                X3 = f2add(f2add(f2mul(r, r), f2scale(HHH, -1)), f2scale(V, -2))
                Y3 = f2add(f2mul(r, f2add(V, f2scale(X3, -1))), f2scale(f2mul(Y, HHH), -1))
                Z3 = f2mul(Z, H)
                c0 = f2add(f2mul(r, xq), f2scale(f2mul(yq, Z3), -1))
                c1 = f2scale(r, -1)
                c4 = Z3
                X, Y, Z = X3, Y3, Z3
            out.append((c0, c1, c4))
    assert len(out) == 68
    return out


PROD_BASE = Builder("fixed").slots["PROD0"]  # fixed slots: the same index in every program


def _setup(prog, sides):
    """LDS image, pair activity and table lines of one check before its Miller program."""
    S = prog["slots"]
    mem = [(0, 0)] * 256
    for k, v in const_values().items():
        mem[S[k]] = v
    mem[S["F0"]] = (1, 0)
    act = []
    tables = []
    for k, (Pk, Qk, neg) in enumerate(sides):
        zp = 1
        if isinstance(Pk, tuple) and Pk and Pk[0] == "JAC":  # Jacobian (X, Y, Z): XP = X Z, YP = Y, ZP = Z^3
            X, Y, Z = Pk[1]
            xp, yp, zp, pinf = X * Z % P, Y, pow(Z, 3, P), Z % P == 0
        elif Pk == "GEN":
            xp, yp = const_values()["G1X"][0], const_values()["G1Y"][0]
            pinf = False
        elif Pk is None:
            xp, yp, pinf = 0, 0, True
        else:
            (xp, yp), pinf = Pk, False
        if neg:
            yp = (-yp) % P
        mem[S["S%d_XP" % k]] = (xp, 0)
        mem[S["S%d_YP" % k]] = (yp, 0)
        mem[S["S%d_ZP" % k]] = (zp, 0)
        xq, yq = Qk if Qk is not None else ((1, 0), (1, 0))
        mem[S["S%d_QX" % k]] = xq
        mem[S["S%d_QY" % k]] = yq
        mem[S["S%d_TX" % k]] = xq
        mem[S["S%d_TY" % k]] = yq
        mem[S["S%d_TZ" % k]] = (1, 0)
        act.append(not pinf and Qk is not None)
        tables.append(raw_lines(Qk))
    return mem, act, tables


def _run(mem, act, tables, hdrs, pdesc, adesc, names=None):
    """Execute the stages of one program on the LDS image `mem` (exact Fp2 arithmetic)."""
    for st in range(len(hdrs) // 4):
        h0, po, ao, h3 = hdrs[4 * st:4 * st + 4]
        kind, j1, j2 = h0 & 3, (h0 >> 2) & 7, (h0 >> 5) & 7
        special = (h0 >> 12) & 0xF
        npairs, nouts = (h0 >> 16) & 127, (h0 >> 23) & 127
        K = 2 if kind == 1 else 1
        new = {}
        if special == SPECIAL_CYC:
            w0, w1 = pdesc[po], pdesc[po + 1]
            f = [mem[(w0 >> (8 * k)) & 0xFF] for k in range(6)]
            for _ in range((w1 >> 48) & 0xFF):
                f = cyclo_w(f)
            if (w1 >> 56) & 1:
                f = [f[k] if k % 2 == 0 else f2scale(f[k], -1) for k in range(6)]
            for k in range(6):
                mem[(w1 >> (8 * k)) & 0xFF] = f[k]
            continue
        if special == SPECIAL_INV:
            new[(h3 >> 8) & 0xFF] = f2inv(mem[h3 & 0xFF])
        prod = {}
        for j in range(npairs):
            acc = (0, 0)
            for t in range(K):
                w = pdesc[po + j * K + t]

                def operand(base, other, sc, negb, conjb):
                    v = mem[base]
                    s = {0: 0, 1: 1, 2: -1}[sc]
                    if s:
                        v = f2add(v, f2scale(mem[other], s))
                    if negb:
                        v = f2scale(v, -1)
                    if conjb:
                        v = f2conj(v)
                    return v

                X = operand(w & 0xFF, (w >> 8) & 0xFF, (w >> 32) & 3, (w >> 36) & 1, (w >> 37) & 1)
                Y = operand((w >> 16) & 0xFF, (w >> 24) & 0xFF, (w >> 34) & 3, (w >> 38) & 1, (w >> 39) & 1)
                acc = f2add(acc, f2mul(X, X) if kind == 2 else f2mul(X, Y))
            prod[PROD_BASE + j] = acc
        view = lambda i: prod[i] if i in prod else mem[i]
        for o in range(nouts):
            ws = adesc[(ao + o) * 8:(ao + o) * 8 + 8]
            dst, gate, defone = ws[0] & 0xFF, (ws[0] >> 8) & 3, (ws[0] >> 10) & 1
            accp, acct = (0, 0), (0, 0)
            for t in range(j1 + j2):
                tm = ws[1 + t]
                src, c, cj = tm & 0xFF, (tm >> 8) & 0xF, (tm >> 12) & 1
                c = c - 16 if c >= 8 else c
                v = view(src)
                if cj:
                    v = f2conj(v)
                if t < j1:
                    accp = f2add(accp, f2scale(v, c))
                else:
                    acct = f2add(acct, f2scale(v, c))
            val = f2add(accp, f2xi(acct))
            if gate and not act[gate - 1]:
                val = (1, 0) if defone else (0, 0)
            assert dst not in new, (st, dst)
            new[dst] = val
        for side in (0, 1):
            e = (h3 >> (16 * side)) & 0xFFFF
            if e & 1 and special == 0:
                step, base = (e >> 1) & 0x7F, e >> 8
                for c in range(3):
                    new[base + c] = tables[side][step][c]
        for k, v in new.items():
            mem[k] = v


def emulate(prog, sides, conj=False):
    """Run `prog` (dict from build()) for one check.  sides[k] = (Pk, Qk, negate): Pk affine G1
    (x, y) or None or 'GEN'; Qk affine G2 ((x0, x1), (y0, y1)) or None.  Returns f as 6 Fp2 (w-basis)
    after the program, conjugated when `conj`."""
    mem, act, tables = _setup(prog, sides)
    _run(mem, act, tables, *prog["miller"])
    _run(mem, act, tables, *prog["fe"])
    f = [mem[prog["slots_fe"]["E%d" % k]] for k in range(6)]
    if conj:
        f = [f[k] if k % 2 == 0 else f2scale(f[k], -1) for k in range(6)]
    return f


def emulate_miller(prog, sides):
    """The Miller program alone (k_wave's miller-only mode): f as 6 Fp2 (w-basis)."""
    mem, act, tables = _setup(prog, sides)
    _run(mem, act, tables, *prog["miller"])
    return [mem[prog["slots"]["F%d" % k]] for k in range(6)]


def emulate_prod_fe(prog, fs):
    """k_wave's product mode: F = fs[0] * fs[1] * ... (one MULF program per factor), then the final
    exponentiation; returns e (w-basis)."""
    S = prog["slots"]
    mem = [(0, 0)] * 256
    for k, v in const_values().items():
        mem[S[k]] = v
    for k in range(6):
        mem[S["F%d" % k]] = fs[0][k]
    for f in fs[1:]:
        for k in range(6):
            mem[S[MULF_G[k]]] = f[k]
        _run(mem, [True, True], [None, None], *prog["mulf"])
    _run(mem, [True, True], [None, None], *prog["fe"])
    return [mem[prog["slots_fe"]["E%d" % k]] for k in range(6)]


# ------------------------------------------------------------------------------- build / emit
MODES = ["WW", "WT", "TW", "TT", "WWJ", "W1J"]


def allocate(b, stages):
    """Physical LDS slots by live range: the fixed slots (constants, F, the two sides, PROD) keep
    their indices; every other name (a TLOAD triple as one block of 3) gets the lowest free index
    whose previous occupant was last read in an earlier stage than this name's first write."""
    fixed = Builder("fixed").slots
    first, last = {}, {}
    for t, st in enumerate(stages):
        for op in st.ops:
            for n in op.reads_prod() | op.reads_asm():
                last[n] = max(last.get(n, -1), t)
            for n in op.writes():
                first[n] = min(first.get(n, 1 << 30), t)
                last[n] = max(last.get(n, -1), t)
    units, seen = [], set(fixed)
    for st in stages:
        for op in st.ops:
            if op.tload and op.tload[3][0] not in seen:
                units.append(list(op.tload[3]))
                seen |= set(op.tload[3])
    for n in b.slots:
        if n not in seen:
            units.append([n])
            seen.add(n)
    span = []
    for u in units:
        s0 = min(first.get(n, last.get(n, 0)) for n in u)
        e0 = max(last.get(n, s0) for n in u)
        span.append((s0, e0, u))
    span.sort(key=lambda x: (x[0], x[2][0]))
    busy = {}
    mapping = dict(fixed)
    base0 = len(fixed)
    for (s0, e0, u) in span:
        k = base0
        while any(busy.get(k + j, -1) >= s0 for j in range(len(u))):
            k += 1
        for j, n in enumerate(u):
            mapping[n] = k + j
            busy[k + j] = e0
    assert max(mapping.values()) < 256
    return mapping


MODES64 = ["WW", "WT", "TW", "TT"]  # the 64-pair set (k_wave64): plain two-pair checks only
COMBINED32 = ("TT",)                # 32-pair modes whose Miller program uses the combined lines


def build(npairs=32):
    """One program per WALK/TABLE combination for the Miller part and one final exponentiation,
    each scheduled into stages and then given physical LDS slots by live range (allocate).
    npairs = 32: k_wave's set (one wave per check); mode TT takes the combined-line Miller program
    (miller_c: 138 stages instead of 200 -- two tabled sides fit 32 pairs), the walking modes keep
    miller() (the homogeneous walk's levels beside f^2 and the line product need more than 32).
    npairs = 64: k_wave64's set (two waves per check), every mode on miller_c (149 stages for a
    walked side instead of 210-211); the final exponentiation is the 32-pair one (its Fp12 products
    stay M2: one-product pairs would need more than 7 assembly terms per output)."""
    global NPAIRS
    saved, NPAIRS = NPAIRS, 32
    try:
        out = {"variants": {}, "npairs": npairs}
        fe = Builder("fe")
        fe.final_exp()
        fe_stages = schedule(fe.ops)
        mf = Builder("mulf")
        mf.mulf()
        mf_stages = schedule(mf.ops)
        NPAIRS = npairs
        fe.slots = allocate(fe, fe_stages)
        fe_enc = encode(fe, fe_stages)
        nslots = max(fe.slots.values()) + 1
        for m in (MODES if npairs == 32 else MODES64):
            b = Builder(m)
            if m == "W1J":
                b.miller1()
            elif npairs == 64 or m in COMBINED32:
                b.miller_c(tuple(m))
            else:
                b.miller(tuple(m))
            st = schedule(b.ops)
            b.slots = allocate(b, st)
            nslots = max(nslots, max(b.slots.values()) + 1)
            out["variants"][m] = {"miller": encode(b, st), "fe": fe_enc, "slots": b.slots, "slots_fe": fe.slots,
                                  "nstages_miller": len(st), "nstages_fe": len(fe_stages),
                                  "stages_miller": st, "stages_fe": fe_stages}
        mf.slots = allocate(mf, mf_stages)
        mf_enc = encode(mf, mf_stages)
        for v in out["variants"].values():
            v["mulf"] = mf_enc
        out["mulf"] = mf_enc
        out["nstages_mulf"] = len(mf_stages)
        out["nslots"] = nslots
        out["slots"] = fe.slots
        return out
    finally:
        NPAIRS = saved


def emit(out, path, ns="hbw"):
    slots = out["slots"]
    modes = MODES if out["npairs"] == 32 else MODES64
    lines = ["// Generated by tools/gen_wave_prog.py -- do not edit.  Stage programs of the wave-per-check",
             "// pairing kernel (k_wave.hip; %d lane pairs per check): 4 u32 header per stage, u64 product" % out["npairs"],
             "// descriptors, 8 x u16 assembly descriptors (formats in tools/gen_wave_prog.py).",
             "#pragma once", "#include <stdint.h>", "namespace %s {" % ns,
             "constexpr int WP_NPAIRS = %d;" % out["npairs"],
             "constexpr int WP_NSLOTS = %d;" % out["nslots"],
             "constexpr int WP_F = %d;" % slots["F0"],
             "constexpr int WP_E = %d;" % slots["E0"],
             "constexpr int WP_PROD = %d;" % slots["PROD0"],
             "constexpr int WP_SIDE0 = %d;  // XP YP QX QY TX TY TZ" % slots["S0_XP"],
             "constexpr int WP_SIDE1 = %d;" % slots["S1_XP"]]
    for i, c in enumerate(CONSTS):
        assert slots[c] == i
    hdr_all, pd_all, ad_all = [], [], []
    info = []
    fe = out["variants"]["WW"]["fe"]

    def append(enc):
        h, p, a = enc
        h0 = len(hdr_all) // 4
        po, ao = len(pd_all), len(ad_all) // 8
        for k in range(0, len(h), 4):
            hdr_all.extend([h[k], h[k + 1] + po, h[k + 2] + ao, h[k + 3]])
        pd_all.extend(p)
        ad_all.extend(a)
        return h0, len(h) // 4

    fe_off, fe_n = append(fe)
    mf_off, mf_n = append(out["mulf"])
    for m in modes:
        mo, mn = append(out["variants"][m]["miller"])
        info.append((mo, mn))
    lines.append("constexpr int WP_FE_OFF = %d, WP_FE_N = %d;" % (fe_off, fe_n))
    lines.append("// F <- F * G with G in side 0's slots XP YP QX QY TX TY (product of partial Miller values)")
    lines.append("constexpr int WP_MULF_OFF = %d, WP_MULF_N = %d;" % (mf_off, mf_n))
    lines.append("// Miller programs: WALK/TABLE for side 0 and side 1 -> index (side0 is TABLE) * 2 + (side1 is TABLE);")
    if out["npairs"] == 32:
        lines.append("// index 4: both sides WALK with Jacobian P (XP = X Z, YP = Y, ZP = Z^3); 5: side 0 only, the same")
        lines.append("// Jacobian P, homogeneous walk (one pair per wave)")
    lines.append("constexpr int WP_NMODES = %d;" % len(modes))
    lines.append("constexpr int WP_MILLER_OFF[%d] = {%s};" % (len(modes), ", ".join(str(i[0]) for i in info)))
    lines.append("constexpr int WP_MILLER_N[%d] = {%s};" % (len(modes), ", ".join(str(i[1]) for i in info)))

    def arr(name, typ, vals, per):
        lines.append("__device__ __attribute__((aligned(16))) const %s %s[%d] = {" % (typ, name, len(vals)))
        for k in range(0, len(vals), per):
            lines.append("  " + ", ".join(("0x%x" % v) + ("ull" if typ == "uint64_t" else "u") for v in vals[k:k + per]) + ",")
        lines.append("};")

    arr("WP_HDR", "uint32_t", hdr_all, 8)
    arr("WP_PDESC", "uint64_t", pd_all, 6)
    arr("WP_ADESC", "uint16_t", ad_all, 16)
    lines.append("}  // namespace %s" % ns)
    with open(path, "w") as f:
        f.write("\n".join(lines) + "\n")


def stats(out):
    cost = {"M1": 1.0, "M2": 1.67, "SQ": 0.67, "NONE": 0.2}
    for m, v in out["variants"].items():
        c = sum(cost[s.kind] for s in v["stages_miller"]) + sum(cost[s.kind] for s in v["stages_fe"])
        print("%d pairs %s: %d Miller stages + %d final-exp stages, %.0f M1-equivalents, %d slots" % (
            out["npairs"], m, v["nstages_miller"], v["nstages_fe"], c, out["nslots"]))


if __name__ == "__main__":
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    o = build()
    stats(o)
    emit(o, os.path.join(root, "hbbft_amd", "csrc", "wave_prog.inc"))
    o64 = build(64)
    stats(o64)
    emit(o64, os.path.join(root, "hbbft_amd", "csrc", "wave_prog64.inc"), ns="hbw64")
