"""The coin path of Binary Agreement (src/binary_agreement/binary_agreement.rs) over the GPU verifier.

BinaryAgreement needs threshold cryptography in one place: the common coin of every epoch with
``epoch % 3 == 2`` is a ThresholdSign over ``bincode((session_id, epoch))`` whose signature parity
is the coin value (:395-405, :437-448).  This mirror keeps the reference's epoch machinery around
that coin -- the epoch counter, the per-epoch coin state, the incoming queue that holds messages of
future epochs and replays them when the epoch advances (:245-266, :489-519), the ``AgreementEpoch``
faults (too far in the future :250-251, a second coin share of one sender for one future epoch
:100-105), the decision rule (:411-432) -- and runs every coin share check through the
``BatchVerifier`` (hbbft_amd.protocol), i.e. batched on the GPU.

Two forms.  ``BinaryAgreementCoin`` is the coin path alone, driven by the HoneyBadger epoch flows
(honey_badger.py): the outcome of an epoch's SBV broadcast and Conf round (``sbv_output``,
``conf_round_complete``) is handed in by the driver at the points where handle_sbvb_step (:301-324)
and try_finish_conf_round (:469-480) act on it.  ``BinaryAgreement`` (round 5) is the whole
instance -- SbvBroadcast (sbv_broadcast.rs: BVal / Aux counting, bin_values), the Conf round, Term
messages with expedited termination, the coin schedule and the future-epoch queue of every message
kind -- for networks of instances (tests/test_binary_agreement_net_host.py, test_gpu_ba_network.py:
the reference's tests/binary_agreement.rs and the reordering attack of binary_agreement_mitm.rs).
"""
import struct

from .protocol import Deferred, Fault, ProtocolError, Step, ThresholdSign, signature_parity

__all__ = ["BinaryAgreement", "BinaryAgreementCoin", "SbvBroadcast", "MAX_FUTURE_EPOCHS", "coin_document"]


def coin_document(hb_id, hb_epoch, proposer_idx, ba_epoch):
    """bincode of ((BaSessionId{subset_id: EpochId{hb_id, epoch}, proposer_idx}), ba_epoch): the
    ThresholdSign document of a BA coin (binary_agreement.rs:442; subset.rs:182-185)."""
    return struct.pack("<QQIQ", hb_id, hb_epoch, proposer_idx, ba_epoch)

MAX_FUTURE_EPOCHS = 1000  # BinaryAgreement::new (binary_agreement.rs:214)
REPLAY_SLACK = 4          # replayed coin shares verified beyond the t + 1 a coin needs


class BinaryAgreementCoin:
    """One BinaryAgreement instance's epochs and coins.

    session: (hb_id, hb_epoch, proposer_idx) -- BaSessionId{subset_id: EpochId{hb_id, hb_epoch},
    proposer_idx} (subset.rs:182-185).  Messages are ``(epoch, share)`` -- MessageContent::Coin
    with its epoch; Step messages are ``("all", (epoch, share))``; faults of the coin's
    ThresholdSign are wrapped as ``CoinFault:<kind>`` (Step::extend_with(.., FaultKind::CoinFault,
    ..), :397-400)."""

    def __init__(self, netinfo, verifier, session, max_future_epochs=MAX_FUTURE_EPOCHS):
        self.netinfo, self.verifier = netinfo, verifier
        self.session = tuple(session)
        self.max_future_epochs = max_future_epochs
        self.epoch = 0
        self.decision = None
        self.estimated = None
        self.conf_values = None
        self.incoming = {}   # epoch -> {sender: share}: the incoming_queue of future epochs
        self.queued = 0      # messages that went through the future-epoch queue
        self.coins = {}      # epoch -> coin value (threshold coins only)
        self.signatures = {} # epoch -> combined coin signature
        self.pending = None  # a deferred coin combine (BatchVerifier recording mode): resolve_pending
        self.coin_decided, self.coin_value, self.ts = self._coin_state()

    # ------------------------------------------------------------ coin state (:437-448)
    def coin_document(self, epoch=None):
        hb_id, hb_epoch, proposer = self.session
        return coin_document(hb_id, hb_epoch, proposer, self.epoch if epoch is None else epoch)

    def _coin_state(self):
        if self.epoch % 3 == 0:
            return True, True, None
        if self.epoch % 3 == 1:
            return True, False, None
        ts = ThresholdSign(self.netinfo, self.verifier)
        try:
            ts.set_document(self.coin_document())
        except ProtocolError as e:  # Error::InvokeCoin
            raise ProtocolError("InvokeCoin", e.kind)
        return False, None, ts

    # ------------------------------------------------------------ messages (:245-266)
    def handle_fast(self, sender, epoch, share):
        """The outcomes most coin messages have, without building Steps: True when handle_message's
        result would be an empty Step and its state change is done here -- ignored (decided, an
        expired epoch, a coin already decided or pending), a future epoch's first share from this
        sender stored in the incoming queue, or a current-epoch share stored by
        ThresholdSign.store_cached.  False: nothing changed (a fault, the share that completes the
        coin, an uncached verdict, or the verifier's shortcuts off) -- call handle_message."""
        if not self.verifier.shortcuts:
            return False
        be = self.epoch
        if self.decision is not None or epoch < be:
            return True
        if epoch > be:
            if epoch > be + self.max_future_epochs or type(share) is not bytes:
                return False
            q = self.incoming.get(epoch)
            if q is None:
                q = self.incoming[epoch] = {}
            elif sender in q:
                return False
            q[sender] = share
            self.queued += 1
            return True
        if self.coin_decided or self.pending is not None:
            return True
        return self.ts.store_cached(sender, share)

    def handle_message(self, sender, epoch, share):
        if self.handle_fast(sender, epoch, share):
            return Step()
        if self.decision is not None or epoch < self.epoch:  # Coin messages can expire
            return Step()
        if epoch > self.epoch + self.max_future_epochs:
            return Step.fault(sender, "AgreementEpoch")
        if epoch > self.epoch:
            q = self.incoming.setdefault(epoch, {})
            if sender in q:  # ReceivedMessages::insert: a second Coin for this epoch
                return Step.fault(sender, "AgreementEpoch")
            q[sender] = bytes(share)
            self.queued += 1
            return Step()
        return self._handle_coin(sender, share)

    def _handle_coin(self, sender, share):  # :355-363
        # a pending (deferred) coin's ThresholdSign has terminated: it ignores further shares
        if self.coin_decided or self.pending is not None:
            return Step()
        try:
            ts_step = self.ts.handle_message(sender, share)
        except ProtocolError as e:  # Error::HandleThresholdSign
            raise ProtocolError("HandleThresholdSign", e.kind)
        return self._on_coin_step(ts_step)

    def _on_coin_step(self, ts_step):  # :394-405
        epoch = self.epoch
        step = Step(fault_log=[Fault(f.node_id, "CoinFault:" + f.kind) for f in ts_step.fault_log],
                    messages=[(target, (epoch, share)) for target, share in ts_step.messages])
        if ts_step.output and not self.coin_decided:
            sig = ts_step.output[0]
            self.signatures[epoch] = sig
            if isinstance(sig, Deferred):  # combined in the driver's next batch: resolve_pending
                self.pending = sig
                return step
            self.coin_decided, self.coin_value = True, signature_parity(sig)
            self.coins[epoch] = self.coin_value
            step.extend(self.try_update_epoch())
        return step

    def resolve_pending(self):
        """The driver flushed the deferred combines (BatchVerifier.flush_combines): the coin of the
        current epoch becomes the signature's parity and the epoch may advance (its queued shares are
        replayed).  A failed combine is the reference's Err from the call that completed the coin
        (threshold_sign.rs:249-270 through Error::HandleThresholdSign)."""
        d, self.pending = self.pending, None
        if d is None:
            return Step()
        if not d.ok:
            kind = "VerificationFailed" if d.result[1] == 0 else "CombineAndVerifySigCrypto"
            raise ProtocolError("HandleThresholdSign", kind)
        self.signatures[self.epoch] = d.result[0]
        self.coin_decided, self.coin_value = True, signature_parity(d.result[0])
        self.coins[self.epoch] = self.coin_value
        return self.try_update_epoch()

    # ------------------------------------------------------------ SBV broadcast / Conf round outcomes
    def sbv_output(self, values):
        """The epoch's SBV broadcast output its aux values (handle_sbvb_step, :301-324): with a
        decided coin (epochs 0 and 1 mod 3, or a threshold coin already combined from the others'
        shares) they become the Conf values at once and the epoch may advance; otherwise the Conf
        round starts (send_conf, :366-380, sets the Conf values)."""
        if self.decision is not None or self.conf_values is not None:
            return Step()
        self.conf_values = frozenset(values)
        return self.try_update_epoch() if self.coin_decided else Step()

    def conf_round_complete(self):
        """N - f Conf messages arrived (try_finish_conf_round, :469-480): the coin is invoked --
        our share is signed and broadcast -- unless it already decided."""
        if self.decision is not None or self.conf_values is None or self.coin_decided:
            return Step()
        try:
            ts_step = self.ts.sign()
        except ProtocolError as e:  # Error::InvokeCoin
            raise ProtocolError("InvokeCoin", e.kind)
        return self._on_coin_step(ts_step).extend(self.try_update_epoch())

    def try_update_epoch(self):  # :411-432
        if self.decision is not None or not self.coin_decided or self.conf_values is None:
            return Step()
        coin = self.coin_value
        definite = next(iter(self.conf_values)) if len(self.conf_values) == 1 else None
        if definite == coin:
            return self.decide(coin)
        return self.update_epoch(coin if definite is None else definite)

    def decide(self, b):  # :450-466 (the Term message is BA's, not the coin's: not modelled)
        if self.decision is not None:
            return Step()
        self.decision = b
        return Step(output=[b])

    def update_epoch(self, b):  # :489-519
        self.conf_values = None
        self.epoch += 1
        self.coin_decided, self.coin_value, self.ts = self._coin_state()
        self.estimated = b
        step = Step()
        replay = sorted(self.incoming.pop(self.epoch, {}).items())  # BTreeMap<sender, ..> order
        if replay and not self.coin_decided:
            # the replayed shares' checks in one drain (the reference verifies them one by one as
            # handle_message_content reaches them; verdicts are pure, so the Steps are the same) --
            # only as many as the coin can use: t + 1 + REPLAY_SLACK counting those a driver
            # already pre-verified; a later share the coin still reads is verified on its own
            # the coin reads the replay in sender order until t + 1 valid shares: verify that
            # prefix (cached verdicts count; unknown ones are assumed valid) plus a small slack
            need, have, queued = self.netinfo.num_faulty() + 1 + REPLAY_SLACK, 0, False
            for sender, share in replay:
                if have >= need:
                    break
                pk = self.netinfo.public_key_share(sender)
                if pk is None:
                    continue
                v = self.verifier.cached_sig(pk, self.ts.doc_hash, share)
                if v is None:
                    self.verifier.queue_sig(pk, self.ts.doc_hash, share)
                    queued = True
                have += 0 if v is False else 1
            if queued:
                self.verifier.drain()
        for sender, share in replay:
            if not self.coin_decided and self.pending is None and self.ts.store_cached(sender, share):
                continue
            step.extend(self._handle_coin(sender, share))
            if self.decision is not None:
                return step
            if self.coin_decided or self.pending is not None:
                break  # every later _handle_coin of this replay is an empty Step (:355-363)
        return step


# ================================================================== the whole protocol
# BoolSet (src/binary_agreement/bool_set.rs): a 2-bit set, iterated true first
NONE, FALSE, TRUE, BOTH = 0, 1, 2, 3


def bs_of(b):
    return TRUE if b else FALSE


def bs_iter(s):
    if s & TRUE:
        yield True
    if s & FALSE:
        yield False


def bs_definite(s):
    return True if s == TRUE else False if s == FALSE else None


class SbvBroadcast:
    """Synchronized Binary Value Broadcast (src/binary_agreement/sbv_broadcast.rs): the BVal / Aux
    steps of an epoch.  Steps carry ``("all", ("BVal" | "Aux", b))`` messages and at most one output,
    the BoolSet of aux values (:159-170)."""

    def __init__(self, netinfo):
        self.netinfo = netinfo
        self.bin_values = NONE
        self.received_bval = {False: set(), True: set()}
        self.sent_bval = NONE
        self.received_aux = {False: set(), True: set()}
        self.terminated = False

    def clear(self, init):  # :81-87 -- init: the Term senders by value (received_term)
        self.bin_values = NONE
        self.received_bval = {b: set(init[b]) for b in (False, True)}
        self.sent_bval = NONE
        self.received_aux = {b: set(init[b]) for b in (False, True)}
        self.terminated = False

    def handle_message(self, sender, msg):
        kind, b = msg
        return self.handle_bval(sender, b) if kind == "BVal" else self.handle_aux(sender, b)

    def send_bval(self, b):  # :102-108
        if self.sent_bval & bs_of(b):
            return Step()
        self.sent_bval |= bs_of(b)
        return self._send(("BVal", b))

    def handle_bval(self, sender, b):  # :114-139
        rb = self.received_bval[b]
        if sender in rb:
            return Step.fault(sender, "DuplicateBVal")
        rb.add(sender)
        count = len(rb)
        step = Step()
        f = self.netinfo.num_faulty()
        if count == 2 * f + 1:
            self.bin_values |= bs_of(b)
            if self.bin_values != BOTH:
                step.extend(self._send(("Aux", b)))  # first entry: send Aux(b)
            else:
                step.extend(self.try_output())
        if count == f + 1:
            step.extend(self.send_bval(b))
        return step

    def _send(self, msg):  # :142-149
        if not self.netinfo.is_validator():
            return self.try_output()
        step = Step(messages=[("all", msg)])
        return step.join(self.handle_message(self.netinfo.our_id, msg))

    def handle_aux(self, sender, b):  # :152-157
        ra = self.received_aux[b]
        if sender in ra:
            return Step.fault(sender, "DuplicateAux")
        ra.add(sender)
        return self.try_output()

    def try_output(self):  # :160-170
        if self.terminated or self.bin_values == NONE:
            return Step()
        count, vals = 0, NONE
        for b in bs_iter(self.bin_values):  # count_aux (:178-188)
            if self.received_aux[b]:
                vals |= bs_of(b)
                count += len(self.received_aux[b])
        if count < len(self.netinfo._ids) - self.netinfo.num_faulty():  # num_correct
            return Step()
        self.terminated = True
        return Step(output=[vals])


class _Received:
    """ReceivedMessages (binary_agreement.rs:44-138): one sender's messages for a future epoch."""
    __slots__ = ("bval", "aux", "conf", "term", "coin")

    def __init__(self):
        self.bval, self.aux, self.conf, self.term, self.coin = NONE, NONE, None, None, None

    def insert(self, content):  # :72-109 -> fault kind or None
        kind, v = content
        if kind == "BVal":
            if self.bval & bs_of(v):
                return "DuplicateBVal"
            self.bval |= bs_of(v)
        elif kind == "Aux":
            if self.aux & bs_of(v):
                return "DuplicateAux"
            self.aux |= bs_of(v)
        elif kind == "Conf":
            if self.conf is not None:
                return "MultipleConf"
            self.conf = v
        elif kind == "Term":
            if self.term is not None:
                return "MultipleTerm"
            self.term = v
        else:
            if self.coin is not None:
                return "AgreementEpoch"
            self.coin = v
        return None

    def messages(self):  # :112-137
        out = [("BVal", b) for b in bs_iter(self.bval)] + [("Aux", b) for b in bs_iter(self.aux)]
        if self.conf is not None:
            out.append(("Conf", self.conf))
        if self.term is not None:
            out.append(("Term", self.term))
        if self.coin is not None:
            out.append(("Coin", self.coin))
        return out


class BinaryAgreement:
    """The whole BinaryAgreement instance (src/binary_agreement/binary_agreement.rs): SBV broadcast,
    Conf round, Term messages, the coin schedule true, false, ThresholdSign, ... and the future-epoch
    queue -- with every coin share check through the BatchVerifier (GPU).  Messages are
    ``(epoch, content)``; content ``("BVal" | "Aux", bool)``, ``("Conf", BoolSet)``, ``("Term", bool)``
    or ``("Coin", share)``; Steps carry ``("all", (epoch, content))``; coin faults are
    ``CoinFault:<kind>``.  session: the bytes bincode writes for the session id (the coin document is
    session || epoch as u64 LE, :442); ``session_bytes(sid)`` for a u8 id as in the reference's
    tests."""

    def __init__(self, netinfo, verifier, session, max_future_epochs=MAX_FUTURE_EPOCHS):
        self.netinfo, self.verifier = netinfo, verifier
        self.session = bytes(session)
        self.epoch = 0
        self.max_future_epochs = max_future_epochs
        self.sbv = SbvBroadcast(netinfo)
        self.received_conf = {}
        self.received_term = {False: set(), True: set()}
        self.estimated = None
        self.decision = None
        self.incoming = {}      # epoch -> {sender: _Received}
        self.conf_values = None
        self.coin_value, self.ts = True, None  # CoinState::Decided(true)
        self.coins = {}         # epoch -> threshold coin value (the epochs 2 mod 3 this instance ran)

    @staticmethod
    def session_bytes(sid):
        return struct.pack("<B", sid)

    def coin_document(self, epoch=None):
        return self.session + struct.pack("<Q", self.epoch if epoch is None else epoch)

    def terminated(self):
        return self.decision is not None

    def handle_input(self, b):
        return self.propose(b)

    def can_propose(self):  # :271-273
        return self.epoch == 0 and self.estimated is None

    def propose(self, b):  # :232-240
        if not self.can_propose():
            return Step()
        self.estimated = b
        return self._sbvb_step(self.sbv.send_bval(b))

    def handle_message(self, sender, msg):  # :245-267
        epoch, content = msg
        if self.decision is not None or (epoch < self.epoch and content[0] != "Term"):
            return Step()
        if epoch > self.epoch + self.max_future_epochs:
            return Step.fault(sender, "AgreementEpoch")
        if epoch > self.epoch:
            rec = self.incoming.setdefault(epoch, {}).setdefault(sender, _Received())
            kind = rec.insert(content)
            return Step() if kind is None else Step.fault(sender, kind)
        return self._content(sender, content)

    def _content(self, sender, content):  # :276-287
        kind, v = content
        if kind in ("BVal", "Aux"):
            return self._sbvb_step(self.sbv.handle_message(sender, content))
        if kind == "Conf":
            return self._handle_conf(sender, v)
        if kind == "Term":
            return self._handle_term(sender, v)
        return self._handle_coin(sender, v)

    def _sbvb_step(self, sbvb):  # :301-325
        epoch = self.epoch
        step = Step(fault_log=sbvb.fault_log, messages=[(t, (epoch, m)) for t, m in sbvb.messages])
        if self.conf_values is not None:
            return step  # the Conf round has already started
        if sbvb.output:
            aux_vals = sbvb.output[0]
            if self.ts is None:  # CoinState::Decided
                self.conf_values = aux_vals
                step.extend(self._try_update_epoch())
            else:
                step.extend(self._send_conf(aux_vals))
        return step

    def _handle_conf(self, sender, v):  # :329-332
        self.received_conf[sender] = v
        return self._try_finish_conf_round()

    def _handle_term(self, sender, b):  # :337-351
        self.received_term[b].add(sender)
        if self.decision is not None:
            return Step()
        if len(self.received_term[b]) > self.netinfo.num_faulty():
            return self._decide(b)
        sbvb = self.sbv.handle_bval(sender, b)
        sbvb.extend(self.sbv.handle_aux(sender, b))
        step = self._sbvb_step(sbvb)
        return step.join(self._handle_conf(sender, bs_of(b)))

    def _handle_coin(self, sender, share):  # :355-363
        if self.ts is None:
            return Step()
        try:
            ts_step = self.ts.handle_message(sender, share)
        except ProtocolError as e:
            raise ProtocolError("HandleThresholdSign", e.kind)
        return self._on_coin_step(ts_step)

    def _send_conf(self, values):  # :366-380
        if self.conf_values is not None:
            return Step()
        self.conf_values = values
        if not self.netinfo.is_validator():
            return self._try_finish_conf_round()
        return self._send(("Conf", values))

    def _send(self, content):  # :383-392
        if not self.netinfo.is_validator():
            return Step()
        step = Step(messages=[("all", (self.epoch, content))])
        return step.join(self._content(self.netinfo.our_id, content))

    def _on_coin_step(self, ts_step):  # :395-406
        epoch = self.epoch
        step = Step(fault_log=[Fault(f.node_id, "CoinFault:" + f.kind) for f in ts_step.fault_log],
                    messages=[(t, (epoch, ("Coin", s))) for t, s in ts_step.messages])
        if ts_step.output:
            if isinstance(ts_step.output[0], Deferred):  #  BinaryAgreementCoin resolves these
                raise ProtocolError("BinaryAgreement needs a non-recording verifier: its coin's combined "
                                    "signature is deferred (use BinaryAgreementCoin with resolve_pending)")
            self.coin_value, self.ts = signature_parity(ts_step.output[0]), None
            self.coins[epoch] = self.coin_value
            step.extend(self._try_update_epoch())
        return step

    def _try_update_epoch(self):  # :414-433
        if self.decision is not None or self.ts is not None or self.conf_values is None:
            return Step()
        coin, definite = self.coin_value, bs_definite(self.conf_values)
        if definite == coin:
            return self._decide(coin)
        return self._update_epoch(coin if definite is None else definite)

    def _coin_state(self):  # :437-448
        if self.epoch % 3 == 0:
            return True, None
        if self.epoch % 3 == 1:
            return False, None
        ts = ThresholdSign(self.netinfo, self.verifier)
        try:
            ts.set_document(self.coin_document())
        except ProtocolError as e:
            raise ProtocolError("InvokeCoin", e.kind)
        return None, ts

    def _decide(self, b):  # :451-466
        if self.decision is not None:
            return Step()
        self.decision = b
        step = Step(output=[b])
        if self.netinfo.is_validator():
            step.messages.append(("all", (self.epoch + 1, ("Term", b))))
        return step

    def _try_finish_conf_round(self):  # :469-480
        if self.conf_values is None:
            return Step()
        bv = self.sbv.bin_values
        if sum(1 for v in self.received_conf.values() if v & bv == v) < len(self.netinfo._ids) - self.netinfo.num_faulty():
            return Step()
        if self.ts is None:
            return Step()
        try:
            ts_step = self.ts.sign()
        except ProtocolError as e:
            raise ProtocolError("InvokeCoin", e.kind)
        return self._on_coin_step(ts_step).join(self._try_update_epoch())

    def _update_epoch(self, b):  # :489-521
        self.sbv.clear(self.received_term)
        self.received_conf = {}
        for v in (False, True):  # BoolMultimap iteration: false's ids, then true's (a later insert wins)
            for nid in sorted(self.received_term[v]):
                self.received_conf[nid] = bs_of(v)
        self.conf_values = None
        self.epoch += 1
        self.coin_value, self.ts = self._coin_state()
        self.estimated = b
        step = self._sbvb_step(self.sbv.send_bval(b))
        for sender, rec in sorted(self.incoming.pop(self.epoch, {}).items()):
            for m in rec.messages():
                step.extend(self._content(sender, m))
                if self.decision is not None:
                    return step
        return step
