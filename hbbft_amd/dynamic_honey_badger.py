"""DynamicHoneyBadger's signed key-generation messages over the GPU verifier.

DynamicHoneyBadger runs SyncKeyGen inside Honey Badger batches: every Part / Ack a node produces is
signed with the node's secret key and committed as a ``SignedKeyGenMsg(era, node_id, msg, sig)``
(src/dynamic_honey_badger/mod.rs:210, ``send_transaction`` dynamic_honey_badger.rs:481-491).  When a
batch is output, every committed key-gen message is checked -- era, then
``PublicKey::verify(sig, bincode(msg))`` against the sender's current key or its candidate key
(:335-347, ``verify_signature`` :514-526) -- and handed to SyncKeyGen (``handle_part`` :433-458,
``handle_ack`` :460-478).

This mirror keeps that order and those faults and moves the crypto off the per-message path: the
messages of a batch are serialised and hashed (``hash_g2``) in one threaded host-stage call, every
signature check of the batch (current and candidate key) runs in ONE ``hbh_verify_sig_shares`` call,
and consecutive Parts / Acks go to SyncKeyGen's batched ``handle_parts`` / ``handle_acks`` (device-
resident commitments).  Votes (votes.rs) and the rest of DHB are out of scope.
"""
import struct

from . import hoststage
from .protocol import Fault, Step
from .sync_key_gen import Ack, Part

__all__ = ["KeyGenMessage", "SignedKeyGenMsg", "DhbKeyGen", "key_gen_msg_bytes"]


def key_gen_msg_bytes(msg):
    """bincode(KeyGenMessage): enum Part(Part) = 0 | Ack(Ack) = 1 as a u32 LE variant index, then the
    payload (hbbft_amd.wire encodings of Part / Ack)."""
    if isinstance(msg, Part):
        return struct.pack("<I", 0) + msg.to_bytes()
    if isinstance(msg, Ack):
        return struct.pack("<I", 1) + msg.to_bytes()
    raise TypeError(type(msg))


KeyGenMessage = (Part, Ack)


class SignedKeyGenMsg:
    """SignedKeyGenMsg(era, node_id, KeyGenMessage, Signature) (mod.rs:210)."""
    __slots__ = ("era", "node_id", "msg", "sig")

    def __init__(self, era, node_id, msg, sig):
        self.era, self.node_id, self.msg, self.sig = era, node_id, msg, bytes(sig)


class DhbKeyGen:
    """The key-generation state of one DynamicHoneyBadger node.

    engine: the GPU engine; era: the current era; our_id; secret_key: the node's secret key (Fr int,
    signs on the host stage); public_keys: {node_id: G1} current validators' keys (NetworkInfo);
    key_gen: the ongoing SyncKeyGen (None: no key generation); candidate_keys: its public keys
    (KeyGenState::public_keys, the validator set being generated; None when no key generation)."""

    def __init__(self, engine, era, our_id, secret_key, public_keys, key_gen=None, candidate_keys=None,
                 is_validator=True, threads=0):
        self.engine, self.era, self.our_id = engine, era, our_id
        self.secret_key = secret_key
        self.public_keys = dict(public_keys)
        self.key_gen = key_gen
        self.candidate_keys = dict(candidate_keys or {})
        self.is_validator = is_validator
        self.threads = threads
        self.key_gen_msg_buffer = []
        self.checks = 0
        self.calls = 0

    # ------------------------------------------------------------ send_transaction (:481-491)
    def send_transaction(self, kg_msg):
        """Sign ``kg_msg`` (SecretKey::sign = hash_g2(bincode(msg)) * sk, host stage) and broadcast
        it; a validator also buffers it for its next contribution."""
        return self.send_transactions([kg_msg])

    def send_transactions(self, kg_msgs):
        if not kg_msgs:
            return Step()
        hs = hoststage.hash_g2([key_gen_msg_bytes(m) for m in kg_msgs], threads=self.threads)
        sigs = hoststage.g2_mul(hs, [self.secret_key] * len(hs), threads=self.threads)
        step = Step()
        for m, sig in zip(kg_msgs, sigs):
            if self.is_validator:
                self.key_gen_msg_buffer.append(SignedKeyGenMsg(self.era, self.our_id, m, sig))
            step.messages.append(("all", ("KeyGen", self.era, m, sig)))
        return step

    # ------------------------------------------------------------ committed batch (:323-347)
    def verify_signatures(self, items):
        """verify_signature (:514-526) for [(node_id, sig, kg_msg)]: valid under the current key OR
        the candidate key -- every check of the list in one engine call."""
        hs = hoststage.hash_g2([key_gen_msg_bytes(m) for _, _, m in items], threads=self.threads) if items else []
        pks, sigs, hidx, owner = [], [], [], []
        for k, ((nid, sig, _), h) in enumerate(zip(items, hs)):
            seen = set()
            for keys in (self.public_keys, self.candidate_keys if self.key_gen is not None else {}):
                pk = keys.get(nid)
                if pk is not None and bytes(pk) not in seen:  # the same key twice: one check
                    seen.add(bytes(pk))
                    pks.append(pk)
                    sigs.append(sig)
                    hidx.append(k)
                    owner.append(k)
        ok = [False] * len(items)
        if pks:
            v = self.engine.verify_sig_shares(pks, sigs, hs, hidx)
            self.calls += 1
            self.checks += len(pks)
            for k, good in zip(owner, v):
                ok[k] = ok[k] or bool(good)
        return ok

    def handle_committed(self, contributions, rng=None):
        """The key-gen messages of an output batch: [(proposer_id, [SignedKeyGenMsg])] in the
        batch's contribution order.  Returns the Step: faults (InvalidKeyGenMessageEra /
        InvalidKeyGenMessageSignature against the PROPOSER, SyncKeyGenPart(..) / SyncKeyGenAck(..)
        / UnexpectedKeyGen* against the signer) and the signed Acks our valid Parts produce."""
        flat = [(pid, skm) for pid, msgs in contributions for skm in msgs]
        for pid, msgs in contributions:  # key_gen_msg_buffer.retain(|skgm| !committed.contains(skgm))
            committed = {(m.era, m.node_id, key_gen_msg_bytes(m.msg), m.sig) for m in msgs}
            self.key_gen_msg_buffer = [m for m in self.key_gen_msg_buffer
                                       if (m.era, m.node_id, key_gen_msg_bytes(m.msg), m.sig) not in committed]
        in_era = [(pid, skm) for pid, skm in flat if skm.era == self.era]
        sig_ok = dict(zip((id(s) for _, s in in_era),
                          self.verify_signatures([(s.node_id, s.sig, s.msg) for _, s in in_era])))
        step = Step()
        run = []  # consecutive verified messages of one kind, handled in one SyncKeyGen call

        def flush():
            if run:
                step.extend(self._handle_run(run, rng))
                run.clear()

        for pid, skm in flat:
            if skm.era != self.era:
                flush()
                step.fault_log.append(Fault(pid, "InvalidKeyGenMessageEra"))
            elif not sig_ok[id(skm)]:
                flush()
                step.fault_log.append(Fault(pid, "InvalidKeyGenMessageSignature"))
            else:
                if run and type(run[0].msg) is not type(skm.msg):
                    flush()
                run.append(skm)
        flush()
        return step

    def _handle_run(self, run, rng):
        if self.key_gen is None:  # no key generation ongoing (:444-447, :465-468)
            kind = "UnexpectedKeyGenPart" if isinstance(run[0].msg, Part) else "UnexpectedKeyGenAck"
            return Step(fault_log=[Fault(m.node_id, kind) for m in run])
        step = Step()
        if isinstance(run[0].msg, Part):
            outs = self.key_gen.handle_parts([(m.node_id, m.msg) for m in run], rng)
            acks = []
            for m, o in zip(run, outs):
                if o.fault is not None:
                    step.fault_log.append(Fault(m.node_id, "SyncKeyGenPart(%s)" % o.fault))
                elif o.ack is not None:
                    acks.append(o.ack)
            step.extend(self.send_transactions(acks))
        else:
            outs = self.key_gen.handle_acks([(m.node_id, m.msg) for m in run])
            for m, o in zip(run, outs):
                if o.fault is not None:
                    step.fault_log.append(Fault(m.node_id, "SyncKeyGenAck(%s)" % o.fault))
        return step
