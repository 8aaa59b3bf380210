"""BinaryAgreement's epoch / coin machinery (hbbft_amd/binary_agreement.py) on the CPU with a
stand-in engine (no GPU): the fixed coins of epochs 0 and 1, the decision rule, the future-epoch
queue with its AgreementEpoch faults and its replay in one drain, expiry of past-epoch messages
(src/binary_agreement/binary_agreement.rs:100-105, 245-266, 411-448, 489-519)."""
from hbbft_amd.binary_agreement import BinaryAgreementCoin
from hbbft_amd.protocol import BatchVerifier, NetworkInfo

SIG = bytes(range(192))  # the stand-in combined signature


class FakeEngine:
    """verdict = first byte of the share is even; combines return SIG (parity of SIG: see below)."""

    def __init__(self):
        self.calls = []

    def verify_sig_shares(self, pks, sigs, hashes, doc_idx):
        self.calls.append(len(pks))
        return bytes(int(s[0] % 2 == 0) for s in sigs)

    def combine_verify_g2(self, t, idx, shares, mpk, hs):
        return [SIG] * len(idx), [0] * len(idx), [1] * len(idx)


def make(max_future=1000, our=0):
    pks = {i: bytes([i + 1]) * 96 for i in range(4)}
    ni = NetworkInfo(our, range(4), 1, bytes(96), pks, sign_g2=lambda H: bytes([100]) * 192)
    eng = FakeEngine()
    return BinaryAgreementCoin(ni, BatchVerifier(eng), (5, 6, 2), max_future_epochs=max_future), eng


def share(b):
    return bytes([b]) * 192


def test_fixed_coins_and_decision():
    ba, _ = make()
    assert (ba.epoch, ba.coin_decided, ba.coin_value) == (0, True, True)
    step = ba.sbv_output({False, True})          # both values: the estimate is the coin (True)
    assert step.output == [] and ba.epoch == 1 and ba.estimated is True
    assert (ba.coin_decided, ba.coin_value) == (True, False)
    step = ba.sbv_output({False})                # definite False == coin of epoch 1: decide
    assert step.output == [False] and ba.decision is False
    assert ba.handle_message(1, 1, share(2)).fault_log == []  # decided: messages are ignored


def test_future_queue_faults_and_replay():
    ba, eng = make(max_future=3)
    assert [f.kind for f in ba.handle_message(1, 4, share(2)).fault_log] == ["AgreementEpoch"]  # > 0 + 3
    assert ba.handle_message(1, 2, share(2)).fault_log == []           # queued for epoch 2
    assert [f.kind for f in ba.handle_message(1, 2, share(4)).fault_log] == ["AgreementEpoch"]  # second Coin
    assert ba.handle_message(2, 2, share(3)).fault_log == []           # queued (an invalid share)
    assert ba.handle_message(3, 2, share(6)).fault_log == []
    assert ba.queued == 3 and eng.calls == []                          # nothing verified yet
    ba.sbv_output({False, True})                                       # -> epoch 1 (estimate True)
    step = ba.sbv_output({True})                                       # coin False != True -> epoch 2
    assert ba.epoch == 2
    # the three queued shares were replayed through ONE drain; sender 2's share is invalid
    assert eng.calls == [3]
    assert [(f.node_id, f.kind) for f in step.fault_log] == [(2, "CoinFault:UnverifiedSignatureShareSender")]
    # t = 1: two valid shares (senders 1 and 3) combine -> the coin is the parity of SIG
    assert ba.coin_decided and 2 in ba.coins
    assert ba.handle_message(1, 1, share(2)).fault_log == []           # a past epoch's Coin expires


def test_conf_round_signs_and_broadcasts():
    ba, eng = make()
    ba.sbv_output({False, True})
    ba.sbv_output({False, True})                 # epoch 2: threshold coin in progress
    assert ba.epoch == 2 and not ba.coin_decided
    assert ba.sbv_output({True}).output == []    # Conf round started; coin not decided yet
    step = ba.conf_round_complete()              # our share is signed and broadcast
    assert step.messages == [("all", (2, bytes([100]) * 192))]
    assert ba.conf_round_complete().messages == []  # only once (had_input)
