"""Device-resident commitment sets (hbh_commit_set_*, include/hbbft_hip.h): a SyncKeyGen instance's
BivarCommitments uploaded once and checked by index (ProposalState::commit,
src/sync_key_gen.rs:254-262, rows :496, Acks :542).

* the set's rows and Ack verdicts equal the stateless hbh_bivar_row / hbh_bivar_ack_check on the
  same commitments, across two appends and with rows cached by an earlier call;
* configs[3] at network scale: all 100 nodes' acks (10^6 checks over 100 Parts of degree 33, 1/97
  tampered) in one call equal the construction, and a sample equals the C oracle's
  BivarCommitment::evaluate == g1 * val (oracle/c/bls_cpu.c)."""
import random

import numpy as np
import pytest

from oracle import bls12_381 as C
from oracle import cbls
from hbbft_amd._lib import ACK_AUTO, ACK_LANE, ACK_LANE_HORNER, ACK_QUAD, HbhError
from hbbft_amd.engine import g1_abi_from_uncompressed as g1a

pytestmark = pytest.mark.gpu
R = C.R
G1 = g1a(C.g1_uncompressed(C.G1_GEN))


def cp(i, j):
    return j * (j + 1) // 2 + i if i <= j else i * (i + 1) // 2 + j


def f_eval(c, t, x, y):
    return sum(c[cp(i, j)] * pow(x, i, R) * pow(y, j, R) for i in range(t + 1) for j in range(t + 1)) % R


def test_commit_set_matches_stateless(engine):
    rng = random.Random(61)
    t, nparts = 4, 7
    npos = (t + 1) * (t + 2) // 2
    coefs = [[rng.randrange(R) for _ in range(npos)] for _ in range(nparts)]
    flat = engine.g1_mul_gen([c for cs in coefs for c in cs])
    commits = [flat[p * npos:(p + 1) * npos] for p in range(nparts)]
    cs = engine.commit_set(t)
    assert cs.add(commits[:3]) == 0 and cs.add(commits[3:]) == 3 and cs.size() == (nparts, 0)
    rp = [rng.randrange(nparts) for _ in range(20)]
    rx = [rng.randrange(1, 50) for _ in range(20)]
    assert cs.rows(rp, rx) == engine.bivar_row(t, commits, rp, rx)
    acks = [(rng.randrange(nparts), rng.randrange(1, 9), rng.randrange(1, 60)) for _ in range(300)]
    vals = [f_eval(coefs[p], t, x, y) for p, x, y in acks]
    bad = set(range(0, len(acks), 7))
    vals = [(v + 1) % R if a in bad else v for a, v in enumerate(vals)]
    args = ([a[0] for a in acks], [a[1] for a in acks], [a[2] for a in acks], vals)
    want = bytes(0 if a in bad else 1 for a in range(len(acks)))
    assert engine.bivar_ack_check(t, commits, *args) == want
    packed = np.frombuffer(b"".join(v.to_bytes(32, "little") for v in vals), dtype=np.uint8).reshape(-1, 32)
    try:
        for impl in (ACK_QUAD, ACK_LANE):  # lane quads on Jacobian rows, one lane on affine rows
            engine.set_ack_impl(impl)
            assert cs.ack_check(*args) == want, impl
            nrows = cs.size()[1]
            assert 0 < nrows <= 2 * nparts * 8
            assert cs.ack_check(*args) == want and cs.size()[1] == nrows  # rows served from the cache
            assert cs.ack_check(np.array(args[0]), np.array(args[1]), np.array(args[2]), packed) == want
    finally:
        engine.set_ack_impl(ACK_AUTO)
    with pytest.raises(HbhError):
        cs.ack_check([nparts], [1], [1], [0])
    with pytest.raises(ValueError):
        cs.add([commits[0][:-1]])
    cs.close()


def test_config3_network_acks(engine):
    """configs[3] network-wide: 10^6 Ack checks (every node x of 100 checks the acks of all 100
    senders for all 100 Parts) in one call against resident commitments."""
    import bench
    n_nodes, t = 100, 33
    commits, pidx, xs, ys, vals, expected = bench.dkg_workload(engine, 100, n_nodes, t, range(1, n_nodes + 1))
    assert len(expected) == n_nodes ** 3
    cs = engine.commit_set(t)
    cs.add(commits)
    got = cs.ack_check(pidx, xs, ys, vals)   # AUTO: one lane per ack at this size
    assert cs.size() == (n_nodes, n_nodes * n_nodes)
    assert got == expected
    try:
        engine.set_ack_impl(ACK_QUAD)
        assert cs.ack_check(pidx[:200000], xs[:200000], ys[:200000], vals[:200000]) == expected[:200000]
    finally:
        engine.set_ack_impl(ACK_AUTO)
    rng = random.Random(62)
    sample = sorted(rng.sample(range(len(expected)), 20)) + [0, 97, len(expected) - 1]
    for a in sample:
        lhs = cbls.bivar_evaluate(t, commits[int(pidx[a])], int(xs[a]), int(ys[a]))
        rhs = cbls.g1_mul(G1, int.from_bytes(bytes(vals[a]), "little"))
        assert (lhs == rhs) == bool(got[a]), a
    cs.close()


@pytest.mark.parametrize("t", [33, 5, 1])
def test_ack_finite_differences_match_horner(engine, t):
    """Round 5: the one-lane Ack path checks the acks of a row whose y form a dense run by finite
    differences (hbl::bivar_fd: the forward-difference table at y0 seeded from the row -- y0 = 0, or
    the run's first y when it starts beyond t + 1 -- then t G1 additions per further y).  Rows of every
    shape -- a node's full run y = 1..100, runs with gaps, a run starting at 50 (the general seed),
    duplicated y, a run of exactly 2 (t + 1) acks, a longer run, sparse rows and a heavily duplicated
    short run (enough acks, too short a span for the seed's two tables: Horner at t = 33) -- with 1/11
    tampered values: FD verdicts == Horner-only == lane quads == the construction, plus C-oracle
    samples (BivarCommitment::evaluate == g1 * val, sync_key_gen.rs:542)."""
    from hbbft_amd import hoststage
    rng = random.Random(700 + t)
    T1 = t + 1
    npos = T1 * (t + 2) // 2
    nparts = 6
    coefs = [[rng.randrange(R) for _ in range(npos)] for _ in range(nparts)]
    flat = engine.g1_mul_gen([c for cs in coefs for c in cs])
    commits = [flat[p * npos:(p + 1) * npos] for p in range(nparts)]
    runs = [(0, 1, list(range(1, 101))),
            (0, 2, [y for y in range(1, 101) if y % 5]),
            (1, 1, list(range(50, 150))),
            (1, 2, [y for y in range(1, 71) for _ in range(2)]),
            (2, 1, sorted(rng.sample(range(1, 1000), 30))),
            (3, 1, list(range(1, 2 * T1 + 1))),
            (4, 7, list(range(1, 201))),
            (5, 3, list(range(1, T1 + 2))),
            (5, 5, [y for y in range(1, T1 + 8) for _ in range(3)])]
    acks = [(p, x, y) for p, x, ys in runs for y in ys]
    rng.shuffle(acks)
    # vals: row(x) of part p is the polynomial in y with coefficients sum_i c(i, j) x^i
    rowpoly = {}
    for p, x, _ in runs:
        ev = hoststage.fr_poly_eval([[coefs[p][cp(i, j)] for i in range(T1)] for j in range(T1)], [x])
        rowpoly[(p, x)] = [ev[j][0] for j in range(T1)]
    keys = sorted(rowpoly)
    ys_all = sorted({y for _, _, y in acks})
    table = dict(zip(keys, hoststage.fr_poly_eval([rowpoly[k] for k in keys], ys_all)))
    yi = {y: k for k, y in enumerate(ys_all)}
    vals = [table[(p, x)][yi[y]] for p, x, y in acks]
    bad = set(range(3, len(acks), 11))
    vals = [(v + 1) % R if a in bad else v for a, v in enumerate(vals)]
    want = bytes(0 if a in bad else 1 for a in range(len(acks)))
    args = ([a[0] for a in acks], [a[1] for a in acks], [a[2] for a in acks], vals)
    cs = engine.commit_set(t)
    cs.add(commits)
    got = {}
    try:
        for impl in (ACK_LANE, ACK_LANE_HORNER, ACK_QUAD, ACK_LANE):
            engine.set_ack_impl(impl)
            got[impl] = cs.ack_check(*args)
            assert got[impl] == want, impl
    finally:
        engine.set_ack_impl(ACK_AUTO)
    for a in sorted(rng.sample(range(len(acks)), 6)) + sorted(bad)[:2]:
        p, x, y = acks[a]
        lhs = cbls.bivar_evaluate(t, commits[p], x, y)
        rhs = cbls.g1_mul(G1, vals[a])
        assert (lhs == rhs) == bool(want[a]), a
    cs.close()


def test_commit_set_outlives_engine():
    """a set closed after its engine must not touch the freed engine.  hbh_engine_destroy
    frees the set's device memory and detaches it; later calls on the set fail loudly, and closing it
    (explicitly or from __del__) is safe."""
    from hbbft_amd.engine import Engine

    eng = Engine(0)
    rng = random.Random(62)
    t = 2
    npos = (t + 1) * (t + 2) // 2
    coefs = [rng.randrange(R) for _ in range(npos)]
    cs = eng.commit_set(t)
    cs.add([eng.g1_mul_gen(coefs)])
    assert cs.size() == (1, 0)
    before = cs.ack_check([0], [1], [2], [f_eval(coefs, t, 1, 2)])
    assert before == b"\x01"
    eng.close()
    with pytest.raises(HbhError):
        cs.ack_check([0], [1], [2], [f_eval(coefs, t, 1, 2)])
    with pytest.raises(HbhError):
        cs.add([[G1] * npos])
    cs.close()
    cs.close()
    # and the other order on a fresh engine: set first, then engine
    eng2 = Engine(0)
    cs2 = eng2.commit_set(t)
    cs2.add([eng2.g1_mul_gen(coefs)])
    cs2.close()
    eng2.close()
