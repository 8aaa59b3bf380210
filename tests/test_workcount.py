"""The algorithmic work counts behind the bench lines' rooflines (hbbft_amd/workcount.py), on the CPU:
the finite-difference Ack check (round 5) against Horner at configs[3]'s shape, and the seed's two
forms (y0 = 0: one small product per entry; a later y0: two)."""
from hbbft_amd import workcount as W


def per_ack(op, n):
    return (op[0] / n, op[1] / n)


def test_fd_ack_cheaper_than_horner_at_configs3():
    t, n = 33, 100
    fd = per_ack(W.bivar_row_fd(t, 1, n, n), n)
    horner = [W.bivar_ack(t, y) for y in range(1, n + 1)]
    h = (sum(o[0] for o in horner) / n, sum(o[1] for o in horner) / n)
    assert fd[0] < h[0] / 2.5          # 1,016 vs 3,064 Fp products per ack
    assert 1000 < fd[0] < 1030


def test_fd_seed_forms():
    t = 5
    z = W.bivar_row_fd(t, 1, 40, 40, val_windows=0)        # ymin <= t + 1: seeded at y0 = 0
    late = W.bivar_row_fd(t, 41, 80, 40, val_windows=0)    # seeded at y0 = 41: (y0 + k) and k products
    steps_z = W._scale(W.G1_ADD, t * 40)
    steps_late = W._scale(W.G1_ADD, t * 39)
    assert late[0] - steps_late[0] > z[0] - steps_z[0]     # the two-product seed costs more


def test_fd_degree_zero():
    # t = 0: the table is R_0 itself (one mixed addition), no steps' additions (t per step), the acks' combs
    op = W.bivar_row_fd(0, 1, 10, 10, val_windows=16)
    assert op == W._add(W.G1_MADD, W._scale(W._add(W._scale(W.G1_MADD, 16), (4, 2)), 10))
