"""The reordering (man-in-the-middle) adversary of the reference's tests/binary_agreement_mitm.rs
(test infrastructure): one faulty node F and groups A0, A1, B of NODES_PER_GROUP nodes; the adversary
schedules BVal / Aux / Coin deliveries stage by stage (amiller/HoneyBadgerBFT issue 59) and, in the
epochs with a threshold coin, predicts the coin from its own ThresholdSign over the shares that reach
F -- the attack the Conf round defeats."""
from hbbft_amd.binary_agreement import BinaryAgreement
from hbbft_amd.protocol import ProtocolError, Step, ThresholdSign, signature_parity

from .virtual_net import NetMessage

NODES_PER_GROUP = 2
NUM_NODES = NODES_PER_GROUP * 3 + 1
A0, A1, B, F = 0, 1, 2, 3


class Stage:
    def __init__(self, src, dst, ty, contents, count):
        self.src, self.dst, self.ty, self.contents, self.count = src, dst, ty, contents, count


G = NODES_PER_GROUP
# ("A", v): a_estimated ^ v; ("C", v): coin ^ v (binary_agreement_mitm.rs:68-73, 90-220)
STAGES = [
    Stage([F], [A0], "BVal", ("A", True), G),
    Stage([F], [A1], "BVal", ("A", False), G),
    Stage([B], [A0, A1], "BVal", None, G * (G * 2)),
    Stage([A0], [A0], "BVal", None, G * (G - 1)),
    Stage([A1], [A1], "BVal", None, G * (G - 1)),
    Stage([A0], [A1], "BVal", ("A", False), G * G),
    Stage([A0, A1], [A0, A1], "BVal", None, (G * 2) * (G * 2 - 1)),
    Stage([A0, A1], [A0, A1], "Aux", None, (G * 2) * (G * 2 - 1)),
    Stage([F], [A0, A1], "BVal", ("A", False), G * 2),
    Stage([F], [A0, A1], "BVal", ("A", True), G * 2),
    Stage([F], [A0, A1], "Aux", ("A", False), G * 2),
    Stage([A0, A1], [F], "Coin", None, G * 2),
    Stage([A0, A1, F], [B], "BVal", ("C", True), (G * 2 + 1) * G),
    Stage([A0, A1, B, F], [B], "Aux", ("C", True), (G + 1) * G + G * (G - 1)),
]


def type_and_content(content):  # :57-66
    kind, v = content
    if kind in ("BVal", "Aux"):
        return kind, v
    if kind == "Coin":
        return "Coin", None
    return None


def group(nid):
    return F if nid == 0 else (nid - 1) // G


class AbaCommonCoinAdversary:
    """binary_agreement_mitm.rs:226-437.  netinfo_box[0]: node 0's NetworkInfo (set when the network
    is built); verifier: the BatchVerifier the adversary's coin checks shares with."""

    def __init__(self, netinfo_box, verifier, rng, epoch=0, a_estimated=False):
        self.netinfo_box, self.verifier = netinfo_box, verifier
        self.stage = self.stage_progress = 0
        self.sent_stage_messages = False
        self.epoch, self.a_estimated = epoch, a_estimated
        self.coin_value, self.coin = None, None
        if epoch % 3 == 0:
            self.coin_value = True
        elif epoch % 3 == 1:
            self.coin_value = False
        else:
            ni = netinfo_box[0]
            self.coin = ThresholdSign(ni, verifier)
            self.coin.set_document(bytes([0]) + epoch.to_bytes(8, "little"))  # bincode((0u8, epoch))
            self.coin.handle_input()

    def eval_state_bool(self, sb):
        kind, v = sb
        if kind == "A":
            return self.a_estimated ^ v
        assert self.coin_value is not None, "state relied upon the coin value before it was known"
        return self.coin_value ^ v

    def inject_stage_messages(self, net):  # :298-332
        if self.sent_stage_messages:
            return
        self.sent_stage_messages = True
        if self.stage >= len(STAGES):
            return
        st = STAGES[self.stage]
        if F not in st.src:
            return
        assert st.contents is not None and st.ty != "Coin"
        msg = (self.epoch, (st.ty, self.eval_state_bool(st.contents)))
        for dg in st.dst:
            if dg == F:
                continue
            for i in range(G):
                net.inject_message(True, NetMessage(0, msg, 1 + G * dg + i))

    def on_stage_progress_update(self):  # :335-349
        while self.stage < len(STAGES):
            st = STAGES[self.stage]
            if not ((st.ty == "Coin" and self.coin_value is not None) or self.stage_progress >= st.count):
                return
            self.stage += 1
            self.stage_progress = 0
            self.sent_stage_messages = False

    def stage_matches_msg(self, m):  # :351-377
        if self.stage >= len(STAGES):
            return False
        st = STAGES[self.stage]
        tc = type_and_content(m.payload[1])
        if tc is None:
            return False
        ty, content = tc
        ok = True
        if st.contents is not None and content is not None:
            ok = self.eval_state_bool(st.contents) == content
        return group(m.frm) in st.src and group(m.to) in st.dst and st.ty == ty and ok

    def pre_crank(self, net, rng):  # :381-413
        while True:
            self.inject_stage_messages(net)
            net.sort_messages_by_key(lambda m: (m.payload[0], 0 if self.stage_matches_msg(m) else 1))
            if not net.messages:
                return
            front = net.messages[0]
            if front.payload[0] == self.epoch and self.stage_matches_msg(front):
                self.stage_progress += 1
                self.on_stage_progress_update()
            if front.payload[0] <= self.epoch:
                return
            assert self.coin_value is not None, "coin value not known at the end of the epoch"
            self.__init__(self.netinfo_box, self.verifier, rng, front.payload[0], self.coin_value)

    def tamper(self, net, msg, rng):  # :415-436
        kind, v = msg.payload[1]
        if kind == "Coin" and self.coin is not None:
            try:
                step = self.coin.handle_message(msg.frm, v)
            except ProtocolError:
                step = None
            if step is not None and step.output:
                self.coin_value, self.coin = signature_parity(step.output[0]), None
        return Step()


def reordering_attack(make_netinfo, verifier, rng, crank_limit=10000):
    """do_reordering_attack (:447-495): node 0 is F, nodes 1..2G (group A) propose false, the rest
    (group B) true; returns the network after every correct node terminated."""
    from .virtual_net import VirtualNet
    box = [None]

    def make(nid, faulty):
        ni = make_netinfo(nid)
        if nid == 0:
            box[0] = ni
        return BinaryAgreement(ni, verifier, BinaryAgreement.session_bytes(0))

    net = VirtualNet(range(NUM_NODES), 1, make, crank_limit=crank_limit)
    net.adversary = AbaCommonCoinAdversary(box, verifier, rng)
    for nid in range(NUM_NODES):
        if nid == 0:
            continue
        net.send_input(nid, nid >= 1 + G * 2)
    while not all(net.nodes[i].algorithm.terminated() for i in range(1, NUM_NODES)):
        net.crank_expect(rng)
    return net
