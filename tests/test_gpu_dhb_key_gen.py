"""DynamicHoneyBadger's signed key-generation messages (hbbft_amd/dynamic_honey_badger.py) through
the GPU path: every node signs its SyncKeyGen Part and the Acks it produces (send_transaction,
src/dynamic_honey_badger/dynamic_honey_badger.rs:481-491); committed batches are checked as
:323-347 does -- era, then PublicKey::verify against the current or the candidate key (:514-526),
all signature checks of a batch in one engine call -- and handed to SyncKeyGen.  All nodes generate
the same key set; a forged signature and a wrong era are blamed on the proposer that committed
them; a joining candidate's messages verify under its candidate key only."""
import random

import pytest

from hbbft_amd import hoststage
from hbbft_amd.dynamic_honey_badger import DhbKeyGen, SignedKeyGenMsg, key_gen_msg_bytes
from hbbft_amd.sync_key_gen import G1_GEN, G2_GEN, R_ORDER, SyncKeyGen

pytestmark = pytest.mark.gpu


def test_dhb_key_gen_signed_messages(engine):
    rng = random.Random(77)
    n, t, era = 4, 1, 7
    sks = [rng.randrange(1, R_ORDER) for _ in range(n)]
    pub = dict(enumerate(hoststage.g1_mul([G1_GEN] * n, sks)))
    current = {i: pub[i] for i in range(n - 1)}  # node 3 is a joining candidate: no current key
    dhbs, parts = [], []
    for i in range(n):
        kg, part = SyncKeyGen.new(i, sks[i], pub, t, engine, rng=rng)
        dhbs.append(DhbKeyGen(engine, era, i, sks[i], current, key_gen=kg, candidate_keys=pub))
        parts.append(part)
    for i in range(n):
        step = dhbs[i].send_transaction(parts[i])
        assert step.messages[0][1][:2] == ("KeyGen", era)
    contributions = [(i, list(dhbs[i].key_gen_msg_buffer)) for i in range(n)]
    # proposer 1 also commits node 0's Part under a forged signature, proposer 2 a wrong-era copy
    forged = SignedKeyGenMsg(era, 0, parts[0], hoststage.g2_mul([G2_GEN], [12345])[0])
    stale = SignedKeyGenMsg(era - 1, 2, parts[2], contributions[2][1][0].sig)
    contributions[1] = (1, contributions[1][1] + [forged])
    contributions[2] = (2, [stale] + contributions[2][1])
    for d in dhbs:
        step = d.handle_committed(contributions, rng)
        assert [(f.node_id, f.kind) for f in step.fault_log] == [(1, "InvalidKeyGenMessageSignature"),
                                                                   (2, "InvalidKeyGenMessageEra")]
        assert len(step.messages) == n  # one signed Ack per valid Part
        assert d.calls == 1             # every signature check of the batch in one engine call
    # the committed messages left the buffers; the Acks are the next batch
    contributions = [(i, list(dhbs[i].key_gen_msg_buffer)) for i in range(n)]
    assert all(len(m) == n for _, m in contributions)
    for d in dhbs:
        assert d.handle_committed(contributions, rng).fault_log == []
        assert d.key_gen.is_ready()
    pks0, _ = dhbs[0].key_gen.generate()
    for d in dhbs:
        assert d.key_gen.generate()[0] == pks0
    # a message of the candidate signed with another key is rejected
    bad = SignedKeyGenMsg(era, 3, parts[3], hoststage.g2_mul(hoststage.hash_g2([key_gen_msg_bytes(parts[3])]), [sks[0]])[0])
    assert dhbs[0].verify_signatures([(bad.node_id, bad.sig, bad.msg)]) == [False]
    # no key generation ongoing: Parts are UnexpectedKeyGenPart faults of their signer
    idle = DhbKeyGen(engine, era, 0, sks[0], pub)
    step = idle.handle_committed([(0, [contributions[0][1][0]])])
    assert [(f.node_id, f.kind) for f in step.fault_log] == [(0, "UnexpectedKeyGenAck")]


def test_dhb_retain_runs_per_contribution(engine):
    """key_gen_msg_buffer.retain runs per contribution in batch order, BEFORE that contribution's
    messages are handled (src/dynamic_honey_badger/dynamic_honey_badger.rs:333-347): a signed Ack our
    node buffers while handling contribution i is removed by the retain of a LATER contribution that
    commits the same message, and survives one committed EARLIER.  Two replicas of node 0
    with identical seeds produce identical Acks; the second sees its own future Acks committed."""
    rng = random.Random(78)
    n, t, era = 4, 1, 3
    sks = [rng.randrange(1, R_ORDER) for _ in range(n)]
    pub = dict(enumerate(hoststage.g1_mul([G1_GEN] * n, sks)))
    parts = [SyncKeyGen.new(i, sks[i], pub, t, engine, rng=rng)[1] for i in range(1, n)]

    def replica():
        kg, part0 = SyncKeyGen.new(0, sks[0], pub, t, engine, rng=random.Random(5))
        return DhbKeyGen(engine, era, 0, sks[0], pub, key_gen=kg), part0

    def signed(i, msg):
        return SignedKeyGenMsg(era, i, msg, hoststage.g2_mul(hoststage.hash_g2([key_gen_msg_bytes(msg)]), [sks[i]])[0])

    a, part0 = replica()
    allparts = [part0] + parts
    contributions = [(i, [signed(i, allparts[i])]) for i in range(n)]
    a.handle_committed(contributions, random.Random(6))
    acks = list(a.key_gen_msg_buffer)
    assert len(acks) == n and all(m.node_id == 0 for m in acks)
    b, _ = replica()
    later = [(i, list(m)) for i, m in contributions]
    later[3][1].append(acks[1])      # the Ack for contribution 1's Part, committed by contribution 3
    later[0][1].append(acks[2])      # the Ack for contribution 2's Part, committed BEFORE it exists
    b.handle_committed(later, random.Random(6))
    keys = [(m.node_id, key_gen_msg_bytes(m.msg), bytes(m.sig)) for m in b.key_gen_msg_buffer]
    want = [(m.node_id, key_gen_msg_bytes(m.msg), bytes(m.sig)) for m in (acks[0], acks[2], acks[3])]
    assert keys == want
