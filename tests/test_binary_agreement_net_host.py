"""The whole Binary Agreement (hbbft_amd/binary_agreement.py BinaryAgreement: SBV broadcast, Conf
round, Term, coin schedule, future-epoch queue) in a virtual network on the CPU, with a stand-in
engine for the coin's crypto (every share valid, one fixed combined signature): the properties of
the reference's tests/binary_agreement.rs -- agreement, termination, validity -- under random
message reordering, and the reordering (man-in-the-middle) attack of tests/binary_agreement_mitm.rs.
The same tests with real threshold signatures on the GPU: tests/test_gpu_ba_network.py."""
import random

import pytest

from hbbft_amd.binary_agreement import BOTH, FALSE, NONE, TRUE, BinaryAgreement, SbvBroadcast, bs_iter
from hbbft_amd.protocol import BatchVerifier, NetworkInfo

from . import ba_mitm
from .virtual_net import ReorderingAdversary, VirtualNet

SIG = bytes([7]) * 192


class FakeEngine:
    def verify_sig_shares(self, pks, sigs, hashes, doc_idx):
        return bytes(1 for _ in sigs)

    def combine_verify_g2(self, t, idx, shares, mpk, hs):
        return [SIG] * len(idx), [0] * len(idx), [1] * len(idx)


def fake_netinfo(n):
    pks = {i: bytes([i + 1]) * 96 for i in range(n)}
    t = (n - 1) // 3
    return lambda i: NetworkInfo(i, range(n), t, bytes(96), pks, sign_g2=lambda H, i=i: bytes([i]) * 192)


def run_network(n, faulty, inp, seed, make_netinfo, verifier):
    """binary_agreement.rs:79-104: every node gets input (random when inp is None), messages are
    delivered in random order until every node terminated; returns the outputs."""
    rng = random.Random(seed)
    net = VirtualNet(range(n), faulty, lambda nid, f: BinaryAgreement(make_netinfo(nid), verifier,
                                                                      BinaryAgreement.session_bytes(0)),
                     adversary=ReorderingAdversary(), message_limit=10000 * n)
    for nid in range(n):
        net.send_input(nid, inp if inp is not None else rng.random() < 0.5)
    while not all(nd.algorithm.terminated() for nd in net.nodes.values()):
        net.crank_expect(rng)
    outs = [nd.outputs for nd in net.nodes.values()]
    assert all(len(o) == 1 for o in outs)
    assert len({o[0] for o in outs}) == 1  # agreement
    if inp is not None:
        assert outs[0] == [inp]            # validity
    return net


def test_boolset_iteration_order():
    assert list(bs_iter(BOTH)) == [True, False] and list(bs_iter(NONE)) == []
    assert list(bs_iter(TRUE)) == [True] and list(bs_iter(FALSE)) == [False]


def test_sbv_broadcast_counts():
    """f + 1 BVal(b) -> our BVal(b); 2 f + 1 -> bin_values, first entry -> Aux(b); N - f Aux with
    values in bin_values -> output (sbv_broadcast.rs:114-170); duplicates are faults."""
    ni = fake_netinfo(4)(0)  # f = 1
    s = SbvBroadcast(ni)
    assert s.handle_bval(1, True).messages == []
    st = s.handle_bval(2, True)                    # f + 1 = 2: echo BVal(true) (and handle it: 3 = 2f+1)
    assert ("all", ("BVal", True)) in st.messages and ("all", ("Aux", True)) in st.messages
    assert s.bin_values == TRUE
    assert [f.kind for f in s.handle_bval(1, True).fault_log] == ["DuplicateBVal"]
    assert s.handle_aux(1, True).output == []
    out = s.handle_aux(2, True)                    # our Aux + 2 = 3 = N - f
    assert out.output == [TRUE]
    assert [f.kind for f in s.handle_aux(2, True).fault_log] == ["DuplicateAux"]


@pytest.mark.parametrize("n,faulty,inp,seed", [(1, 0, None, 1), (2, 0, True, 2), (4, 1, None, 3), (4, 1, False, 4),
                                                (7, 2, None, 5), (7, 2, True, 6), (10, 3, None, 7), (13, 4, None, 8)])
def test_binary_agreement_reordering(n, faulty, inp, seed):
    run_network(n, faulty, inp, seed, fake_netinfo(n), BatchVerifier(FakeEngine()))


def test_term_expedites_and_future_queue():
    """A Term(b) counts as BVal, Aux and Conf for every later epoch and f + 1 of them decide at once
    (binary_agreement.rs:337-351); messages of a future epoch wait in the queue and are replayed
    (:245-267, :489-521); a second Conf / Term of one sender for a future epoch is a fault."""
    ni = fake_netinfo(4)(0)
    ba = BinaryAgreement(ni, BatchVerifier(FakeEngine()), BinaryAgreement.session_bytes(0))
    ba.propose(True)
    assert ba.handle_message(1, (3, ("Conf", TRUE))).fault_log == []
    assert [f.kind for f in ba.handle_message(1, (3, ("Conf", FALSE))).fault_log] == ["MultipleConf"]
    assert [f.kind for f in ba.handle_message(2, (1, ("Term", True))).fault_log] == []
    assert [f.kind for f in ba.handle_message(2, (1, ("Term", True))).fault_log] == ["MultipleTerm"]
    assert [f.kind for f in ba.handle_message(1, (2000, ("BVal", True))).fault_log] == ["AgreementEpoch"]
    st = ba.handle_message(3, (0, ("Term", False)))   # one Term(false): counted as BVal/Aux/Conf
    assert st.output == [] and ba.decision is None
    st = ba.handle_message(1, (0, ("Term", False)))   # f + 1 = 2 Term(false): decide false
    assert st.output == [False] and ba.decision is False
    assert ("all", (1, ("Term", False))) in st.messages
    assert ba.handle_message(2, (0, ("BVal", True))).messages == []  # terminated: ignored


@pytest.mark.parametrize("seed", [11, 12, 13])
def test_reordering_attack_fake_coin(seed):
    """binary_agreement_mitm.rs with the stand-in coin: every correct node terminates with the same
    output within the reference's 10,000 cranks."""
    net = ba_mitm.reordering_attack(fake_netinfo(ba_mitm.NUM_NODES), BatchVerifier(FakeEngine()),
                                    random.Random(seed))
    outs = [net.nodes[i].outputs for i in range(1, ba_mitm.NUM_NODES)]
    assert all(len(o) == 1 for o in outs) and len({o[0] for o in outs}) == 1


class RandomFaultyAdversary(ReorderingAdversary):
    """Faulty nodes ignore the protocol: every message to one of them is answered with a random
    Binary Agreement message (BVal / Aux / Conf / Term with a random value, for the current or a
    nearby epoch) to a random correct node; deliveries are reordered at random.  Correct nodes must
    still agree, terminate, keep validity among the correct inputs, and blame only faulty nodes."""

    def __init__(self, rng):
        self.rng = rng

    def tamper(self, net, msg, rng):
        from hbbft_amd.protocol import Step
        from hbbft_amd.binary_agreement import BOTH, FALSE, TRUE
        from .virtual_net import NetMessage
        r = self.rng
        epoch = max(0, msg.payload[0] + r.choice((-1, 0, 0, 1)))
        kind = r.choice(("BVal", "Aux", "Conf", "Term"))
        val = r.choice((FALSE, TRUE, BOTH)) if kind == "Conf" else r.random() < 0.5
        good = [n for n, nd in net.nodes.items() if not nd.faulty]
        net.inject_message(False, NetMessage(msg.to, (epoch, (kind, val)), r.choice(good)))
        return Step()


@pytest.mark.parametrize("n,faulty,inp,seed", [(4, 1, True, 41), (7, 2, False, 42), (7, 2, None, 43),
                                                (10, 3, None, 44)])
def test_binary_agreement_random_faulty_nodes(n, faulty, inp, seed):
    """tests/binary_agreement.rs's properties with faulty nodes that send random BA messages: the
    correct nodes decide one value, the correct nodes' common input when they share one, and every
    fault a correct node records names a faulty node (VirtualNet raises otherwise)."""
    rng = random.Random(seed)
    net = VirtualNet(range(n), faulty, lambda nid, f: BinaryAgreement(fake_netinfo(n)(nid), BatchVerifier(FakeEngine()),
                                                                      BinaryAgreement.session_bytes(0)),
                     adversary=RandomFaultyAdversary(random.Random(seed + 1)), message_limit=10000 * n)
    correct = [nid for nid, nd in net.nodes.items() if not nd.faulty]
    for nid in correct:
        net.send_input(nid, inp if inp is not None else rng.random() < 0.5)
    # faulty nodes start the noise with one message each
    for nid, nd in net.nodes.items():
        if nd.faulty:
            net.inject_message(False, ba_mitm.NetMessage(nid, (0, ("BVal", True)), correct[0]))
    while not all(net.nodes[i].algorithm.terminated() for i in correct):
        net.crank_expect(rng)
    outs = [net.nodes[i].outputs for i in correct]
    assert all(len(o) == 1 for o in outs) and len({o[0] for o in outs}) == 1
    if inp is not None:
        assert outs[0] == [inp]
    assert all(f.node_id < faulty for i in correct for f in net.nodes[i].faults)
