"""DynamicHoneyBadger's validator-change votes (hbbft_amd/dynamic_honey_badger.py VoteCounter,
mirroring src/dynamic_honey_badger/votes.rs).

* the reference's own unit tests (votes.rs:225-296, test_pending_votes / test_committed_votes)
  restated: obsolescence by vote number, InvalidVoteSignature against the sender of a pending vote,
  InvalidCommittedVote against the proposer, committed votes hiding older pending ones, the f + 1
  winner;
* a random batch (16 voters, several proposers, forged signatures, wrong eras, stale and repeated
  vote numbers, unknown voters) applied through ONE engine call equals the vote-by-vote
  application with the C oracle's PublicKey::verify (oracle/c/bls_cpu.c).

The CPU variants run the host logic on an engine stand-in backed by the C oracle; the ``gpu``
variants run the same checks through hbh_verify_sig_shares."""
import random

import pytest

from hbbft_amd import hoststage
from hbbft_amd.dynamic_honey_badger import (SignedVote, Vote, VoteCounter, encryption_schedule, node_change,
                                            vote_bytes)
from hbbft_amd.protocol import Fault
from hbbft_amd.sync_key_gen import G1_GEN, R_ORDER
from oracle import cbls


class OracleEngine:
    """verify_signatures through the C oracle, one scalar check per item (test stand-in)."""

    def __init__(self):
        self.calls = 0

    def verify_signatures(self, pks, sigs, hashes):
        self.calls += 1
        return bytes(int(cbls.verify_g2(p, s, h)) for p, s, h in zip(pks, sigs, hashes))


@pytest.fixture(params=["cpu", pytest.param("gpu", marks=pytest.mark.gpu)])
def eng(request):
    if request.param == "cpu":
        return OracleEngine()
    return request.getfixturevalue("engine")


def setup(eng, node_num, era, seed=5):
    """votes.rs:206-222: one counter per node; sv[i][j] = node i's vote (number j) for making j the
    only validator, signed in order j = 0, 1, ..."""
    rng = random.Random(seed)
    sks = [rng.randrange(1, R_ORDER) for _ in range(node_num)]
    pks = dict(enumerate(hoststage.g1_mul([G1_GEN] * node_num, sks)))
    f = (node_num - 1) // 3
    counters = [VoteCounter(eng, era, i, sks[i], pks, f) for i in range(node_num)]
    sv = [[c.sign_vote_for(node_change({j: pks[j]})) for j in range(node_num)] for c in counters]
    return counters, sv, sks, pks


def forge(sv, other):
    """SignedVote { sig: other.sig, ..sv }"""
    return SignedVote(sv.vote, sv.voter, other.sig)


def test_pending_votes(eng):
    counters, sv, _, _ = setup(eng, 4, 5)
    ct = counters[0]
    assert ct.add_pending_vote(1, sv[1][2]) == []
    assert ct.add_pending_vote(2, sv[2][1]) == []
    assert ct.add_pending_vote(1, forge(sv[3][1], sv[2][1])) == [Fault(1, "InvalidVoteSignature")]
    assert ct.pending_votes() == [sv[0][3], sv[1][2], sv[2][1]]
    assert ct.add_pending_vote(3, sv[1][1]) == []   # older: ignored
    assert ct.add_pending_vote(1, sv[2][2]) == []   # newer: replaces
    assert ct.pending_votes() == [sv[0][3], sv[1][2], sv[2][2]]
    ct.add_committed_votes(1, [sv[1][3], sv[2][1], sv[0][3]])
    assert ct.pending_votes() == [sv[2][2]]


def test_committed_votes(eng):
    counters, sv, _, pks = setup(eng, 4, 5)
    ct = counters[0]
    faults = ct.add_committed_votes(1, [sv[1][1], forge(sv[3][1], sv[2][1])])
    assert faults == [Fault(1, "InvalidCommittedVote")]
    assert ct.calls == 1 and ct.checks == 2          # both signatures in one engine call
    assert ct.compute_winner() is None
    assert ct.add_committed_vote(1, sv[2][1]) == []
    assert ct.compute_winner() == node_change({1: pks[1]})
    # a vote of another era is InvalidCommittedVote without a signature check
    other = VoteCounter(eng, 6, 0, 1, pks, 1)
    checks = other.checks
    assert other.add_committed_vote(2, sv[1][1]) == [Fault(2, "InvalidCommittedVote")]
    assert other.checks == checks


def test_vote_bytes_layout():
    pk = hoststage.g1_mul([G1_GEN], [7])[0]
    (b,) = vote_bytes([Vote(node_change({3: pk}), 5, 2)])
    comp = hoststage.g1_compress([pk])[0]
    assert b == (b"\0\0\0\0" + (1).to_bytes(8, "little") + (3).to_bytes(8, "little")
                 + (48).to_bytes(8, "little") + comp + (5).to_bytes(8, "little") + (2).to_bytes(8, "little"))
    (b,) = vote_bytes([Vote(encryption_schedule("TickTock", 2, 3), 1, 0)])
    assert b == bytes([1, 0, 0, 0, 3, 0, 0, 0, 2, 0, 0, 0, 3, 0, 0, 0]) + bytes([1] + [0] * 7) + bytes(8)
    with pytest.raises(ValueError):
        encryption_schedule("EveryNthEpoch")


def scalar_apply(era, pks, committed, flat, f):
    """votes.rs:117-135 vote by vote with the oracle's verify (the checker)."""
    faults = []
    for pid, sv in flat:
        c = committed.get(sv.voter)
        if c is not None and c.num >= sv.vote.num:
            continue
        pk = pks.get(sv.voter)
        ok = (sv.vote.era == era and pk is not None
              and cbls.verify_g2(pk, sv.sig, hoststage.hash_g2(vote_bytes([sv.vote]))[0]))
        if not ok:
            faults.append(Fault(pid, "InvalidCommittedVote"))
            continue
        committed[sv.voter] = sv.vote
    return faults


def test_random_committed_batch(eng):
    n, era = 16, 9
    counters, _, sks, pks = setup(eng, n, era, seed=11)
    rng = random.Random(12)
    changes = [node_change({j: pks[j]}) for j in range(3)] + [encryption_schedule("EveryNthEpoch", 4)]
    votes = []
    for voter in range(n):
        for num in range(rng.randrange(1, 4)):
            v = Vote(rng.choice(changes), era if rng.random() > 0.1 else era - 1, num)
            votes.append((voter, v))
    hs = hoststage.hash_g2(vote_bytes([v for _, v in votes]))
    sigs = hoststage.g2_mul(hs, [sks[voter] for voter, _ in votes])
    svs = [SignedVote(v, voter, s) for (voter, v), s in zip(votes, sigs)]
    for k in range(0, len(svs), 5):                 # forged
        svs[k] = forge(svs[k], svs[(k + 1) % len(svs)])
    svs.append(SignedVote(Vote(changes[0], era, 7), 99, sigs[0]))  # unknown voter
    rng.shuffle(svs)
    svs += svs[:6]                                   # replays of committed numbers
    contributions = [(p, svs[p::5]) for p in range(5)]
    ct = counters[0]
    faults = ct.add_committed_batch(contributions)
    assert ct.calls == 1 and ct.checks <= len(svs)  # the whole batch in one engine call
    want_committed = {}
    want = scalar_apply(era, pks, want_committed, [(p, sv) for p, b in contributions for sv in b], ct.num_faulty)
    assert faults == want and len(want) > 0
    assert ct.committed == want_committed
    assert ct.compute_winner() == _winner(want_committed, ct.num_faulty)


def _winner(committed, f):
    counts = {}
    for _, v in sorted(committed.items()):
        counts[v.change] = counts.get(v.change, 0) + 1
        if counts[v.change] > f:
            return v.change
    return None
