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
resident commitments).

``VoteCounter`` mirrors the validator-change votes (src/dynamic_honey_badger/votes.rs): pending and
committed votes, each checked ``PublicKey::verify(sig, bincode(vote))`` under the voter's key
(``validate`` :152-158); a batch of votes is serialised and hashed in one host call and every
signature it needs goes to ONE engine call, then the votes are applied in order with the
reference's obsolescence rules.  The rest of DHB (era switches, the Honey Badger wrapper) is out of
scope.
"""
import struct

from . import hoststage
from .protocol import Fault, Step
from .sync_key_gen import Ack, Part

__all__ = ["KeyGenMessage", "SignedKeyGenMsg", "DhbKeyGen", "key_gen_msg_bytes", "node_change",
           "encryption_schedule", "Vote", "SignedVote", "VoteCounter", "vote_bytes"]


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
        # The reference (:333-347) runs, per contribution in batch order, key_gen_msg_buffer.retain(|m|
        # !committed_i.contains(m)) and then handles that contribution's messages -- which may buffer new
        # signed Acks (send_transaction).  Messages already buffered are removed by every retain either
        # way, so the retains are applied to them up front; a message buffered while handling
        # contribution i is filtered by the retains of the contributions AFTER i only (``later[i]``).
        # The signature checks and SyncKeyGen calls stay batched across contributions.
        flat = [(ci, pid, skm) for ci, (pid, msgs) in enumerate(contributions) for skm in msgs]
        keyed = [{_skm_key(m) for m in msgs} for _, msgs in contributions]
        later = [set() for _ in contributions]
        acc = set()
        for ci in range(len(contributions) - 1, -1, -1):
            later[ci] = acc
            acc = acc | keyed[ci]
        self.key_gen_msg_buffer = [m for m in self.key_gen_msg_buffer if _skm_key(m) not in acc]
        in_era = [skm for _, _, skm in flat if skm.era == self.era]
        sig_ok = dict(zip((id(s) for s in in_era), self.verify_signatures([(s.node_id, s.sig, s.msg) for s in in_era])))
        step = Step()
        run = []  # consecutive verified messages of one kind, handled in one SyncKeyGen call: (ci, skm)

        def flush():
            if run:
                step.extend(self._handle_run(run, rng, later))
                run.clear()

        for ci, pid, skm in flat:
            if skm.era != self.era:
                flush()
                step.fault_log.append(Fault(pid, "InvalidKeyGenMessageEra"))
            elif not sig_ok[id(skm)]:
                flush()
                step.fault_log.append(Fault(pid, "InvalidKeyGenMessageSignature"))
            else:
                if run and type(run[0][1].msg) is not type(skm.msg):
                    flush()
                run.append((ci, skm))
        flush()
        return step

    def _handle_run(self, run, rng, later):
        if self.key_gen is None:  # no key generation ongoing (:444-447, :465-468)
            kind = "UnexpectedKeyGenPart" if isinstance(run[0][1].msg, Part) else "UnexpectedKeyGenAck"
            return Step(fault_log=[Fault(m.node_id, kind) for _, m in run])
        step = Step()
        if isinstance(run[0][1].msg, Part):
            outs = self.key_gen.handle_parts([(m.node_id, m.msg) for _, m in run], rng)
            acks, acis = [], []
            for (ci, m), o in zip(run, outs):
                if o.fault is not None:
                    step.fault_log.append(Fault(m.node_id, "SyncKeyGenPart(%s)" % o.fault))
                elif o.ack is not None:
                    acks.append(o.ack)
                    acis.append(ci)
            first = len(self.key_gen_msg_buffer)
            step.extend(self.send_transactions(acks))
            if self.is_validator and acks:  # the later contributions' retains on the Acks just buffered
                fresh = self.key_gen_msg_buffer[first:]
                self.key_gen_msg_buffer[first:] = [m for m, ci in zip(fresh, acis) if _skm_key(m) not in later[ci]]
        else:
            outs = self.key_gen.handle_acks([(m.node_id, m.msg) for _, m in run])
            for (_, m), o in zip(run, outs):
                if o.fault is not None:
                    step.fault_log.append(Fault(m.node_id, "SyncKeyGenAck(%s)" % o.fault))
        return step


def _skm_key(m):
    """Equality of SignedKeyGenMsg (era, node_id, message, signature), as the reference's retain uses."""
    return (m.era, m.node_id, key_gen_msg_bytes(m.msg), bytes(m.sig))


# ================================================================ votes (src/dynamic_honey_badger/votes.rs)
_SCHEDULES = {"Always": 0, "Never": 1, "EveryNthEpoch": 2, "TickTock": 3}


def node_change(keys):
    """Change::NodeChange(BTreeMap<N, PublicKey>) (change.rs:14): {node_id (int): ABI G1 key}."""
    return ("NodeChange", tuple(sorted((int(k), bytes(v)) for k, v in keys.items())))


def encryption_schedule(kind, *args):
    """Change::EncryptionSchedule(EncryptionSchedule) (change.rs:17, honey_badger.rs:201-210)."""
    if kind not in _SCHEDULES or len(args) != {0: 0, 1: 0, 2: 1, 3: 2}[_SCHEDULES[kind]]:
        raise ValueError((kind, args))
    return ("EncryptionSchedule", (kind,) + tuple(int(a) for a in args))


class Vote(tuple):
    """Vote { change, era: u64, num: u64 } (votes.rs:163-170)."""
    __slots__ = ()

    def __new__(cls, change, era, num):
        return tuple.__new__(cls, (change, int(era), int(num)))

    change = property(lambda s: s[0])
    era = property(lambda s: s[1])
    num = property(lambda s: s[2])


class SignedVote:
    """SignedVote { vote, voter, sig } (votes.rs:174-178)."""
    __slots__ = ("vote", "voter", "sig")

    def __init__(self, vote, voter, sig):
        self.vote, self.voter, self.sig = vote, voter, bytes(sig)

    def era(self):
        return self.vote.era

    def __eq__(self, o):
        return isinstance(o, SignedVote) and (self.vote, self.voter, self.sig) == (o.vote, o.voter, o.sig)

    def __hash__(self):
        return hash((self.vote, self.voter, self.sig))

    def __repr__(self):
        return "SignedVote(voter=%r, era=%d, num=%d)" % (self.voter, self.vote.era, self.vote.num)


def vote_bytes(votes):
    """bincode(Vote) per vote: the Change enum as a u32 variant index and its payload (NodeChange:
    u64 count, then per entry the u64 node id and the key as u64 48 + compressed G1 -- the wire.py
    encoding; EncryptionSchedule: u32 variant and its u32 fields), then era and num as u64 LE.  All
    keys of the batch are compressed in one host call.  Restated from serde's derive rules; no
    pinned vectors exist."""
    keys = [pk for v in votes if v.change[0] == "NodeChange" for _, pk in v.change[1]]
    comp = iter(hoststage.g1_compress(keys) if keys else [])
    out = []
    for v in votes:
        kind, body = v.change
        if kind == "NodeChange":
            b = struct.pack("<IQ", 0, len(body)) + b"".join(
                struct.pack("<QQ", nid, 48) + next(comp) for nid, _ in body)
        else:
            b = struct.pack("<II", 1, _SCHEDULES[body[0]]) + b"".join(struct.pack("<I", a) for a in body[1:])
        out.append(b + struct.pack("<QQ", v.era, v.num))
    return out


class VoteCounter:
    """VoteCounter (votes.rs:17-31): the pending and committed validator-change votes of one era.

    engine: the GPU engine; era; our_id; secret_key (Fr int, signs on the host stage); public_keys:
    {node_id: ABI G1} (NetworkInfo::public_key); num_faulty: f.  ``calls`` / ``checks`` count the
    engine calls and the signatures they verified."""

    def __init__(self, engine, era, our_id, secret_key, public_keys, num_faulty, threads=0):
        self.engine, self.era, self.our_id = engine, era, our_id
        self.secret_key = secret_key
        self.public_keys = dict(public_keys)
        self.num_faulty = num_faulty
        self.threads = threads
        self.pending = {}    # voter -> SignedVote
        self.committed = {}  # voter -> Vote
        self.calls = 0
        self.checks = 0

    def sign_vote_for(self, change):
        """sign_vote_for (:47-63): the next vote number of our pending vote, signed, replacing it."""
        prev = self.pending.get(self.our_id)
        vote = Vote(change, self.era, 0 if prev is None else prev.vote.num + 1)
        h = hoststage.hash_g2(vote_bytes([vote]), threads=self.threads)
        sig = hoststage.g2_mul(h, [self.secret_key], threads=self.threads)[0]
        self.pending[self.our_id] = SignedVote(vote, self.our_id, sig)
        return self.pending[self.our_id]

    def validate(self, signed_votes):
        """validate (:152-158) for a list of SignedVotes in one engine call; no key: False."""
        ok = [False] * len(signed_votes)
        idx = [k for k, sv in enumerate(signed_votes) if sv.voter in self.public_keys]
        if idx:
            hs = hoststage.hash_g2(vote_bytes([signed_votes[k].vote for k in idx]), threads=self.threads)
            v = self.engine.verify_signatures([self.public_keys[signed_votes[k].voter] for k in idx],
                                              [signed_votes[k].sig for k in idx], hs)
            self.calls += 1
            self.checks += len(idx)
            for k, good in zip(idx, v):
                ok[k] = bool(good)
        return ok

    def _verdicts(self, items, need):
        """Signature verdicts for the items ``need`` selects against the state BEFORE the batch: a
        vote obsolete then stays obsolete (vote numbers only grow), so one engine call covers every
        signature the in-order application can reach."""
        sel = [k for k, sv in enumerate(items) if need(sv)]
        got = self.validate([items[k] for k in sel])
        return dict(zip(sel, got))

    # ---------------------------------------------------------------- pending (:66-90)
    def add_pending_votes(self, items):
        """add_pending_vote for [(sender_id, SignedVote)] in order; faults InvalidVoteSignature
        against the sender."""
        svs = [sv for _, sv in items]
        pend = self.pending

        def need(sv):
            p = pend.get(sv.voter)
            return sv.vote.era == self.era and (p is None or p.vote.num < sv.vote.num)

        ok = self._verdicts(svs, need)
        faults = []
        for k, (sender, sv) in enumerate(items):
            p = self.pending.get(sv.voter)
            if sv.vote.era != self.era or (p is not None and p.vote.num >= sv.vote.num):
                continue  # obsolete or already present
            if not ok[k]:
                faults.append(Fault(sender, "InvalidVoteSignature"))
                continue
            self.pending[sv.voter] = sv
        return faults

    def add_pending_vote(self, sender_id, signed_vote):
        return self.add_pending_votes([(sender_id, signed_vote)])

    def pending_votes(self):
        """pending_votes (:93-99): pending votes newer than their voter's committed vote, in voter
        order (BTreeMap)."""
        return [sv for voter, sv in sorted(self.pending.items())
                if voter not in self.committed or self.committed[voter].num < sv.vote.num]

    # ---------------------------------------------------------------- committed (:103-135)
    def add_committed_batch(self, contributions):
        """add_committed_votes for every proposer of an output batch, [(proposer_id, [SignedVote])]
        in contribution order, with ONE engine call; faults InvalidCommittedVote against the
        proposer."""
        flat = [(pid, sv) for pid, svs in contributions for sv in svs]
        com = self.committed

        def need(sv):
            c = com.get(sv.voter)
            return (c is None or c.num < sv.vote.num) and sv.vote.era == self.era

        ok = self._verdicts([sv for _, sv in flat], need)
        faults = []
        for k, (pid, sv) in enumerate(flat):
            c = self.committed.get(sv.voter)
            if c is not None and c.num >= sv.vote.num:
                continue  # obsolete or already present
            if sv.vote.era != self.era or not ok[k]:
                faults.append(Fault(pid, "InvalidCommittedVote"))
                continue
            self.committed[sv.voter] = sv.vote
        return faults

    def add_committed_votes(self, proposer_id, signed_votes):
        return self.add_committed_batch([(proposer_id, list(signed_votes))])

    def add_committed_vote(self, proposer_id, signed_vote):
        return self.add_committed_batch([(proposer_id, [signed_vote])])

    def compute_winner(self):
        """compute_winner (:138-150): the first change, in voter order, to reach f + 1 votes."""
        counts = {}
        for _, vote in sorted(self.committed.items()):
            counts[vote.change] = counts.get(vote.change, 0) + 1
            if counts[vote.change] > self.num_faulty:
                return vote.change
        return None
