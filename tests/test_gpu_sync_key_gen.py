"""SyncKeyGen flow through the GPU engine, ported from the reference's tests/sync_key_gen.rs:10-103:
node counts {1, 2, 3, 4, 8, 15} with threshold max_faulty(n); only the first t+1 Parts are
handled; Acks come from 2t+1 nodes; not ready before / ready after; every node generates the same
PublicKeySet; every secret share signs a message whose share verifies against
public_key_share(idx); the combination of t+1 shares verifies against the master key.  Plus the
fault paths of handle_part_or_fault / handle_ack_or_fault (sync_key_gen.rs:481-547)."""
import random

import pytest

from hbbft_amd import hoststage
from hbbft_amd.sync_key_gen import G1_GEN, R_ORDER, Ack, Ciphertext, Part, SyncKeyGen

pytestmark = pytest.mark.gpu
MSG = b"Help I'm trapped in a unit test factory"


def make_nodes(engine, n, t, rng):
    sks = [rng.randrange(1, R_ORDER) for _ in range(n)]
    pks = hoststage.g1_mul([G1_GEN] * n, sks)
    pub = {i: pks[i] for i in range(n)}
    nodes, props = [], []
    for i in range(n):
        kg, part = SyncKeyGen.new(i, sks[i], pub, t, engine, rng=rng)
        nodes.append(kg)
        props.append(part)
    return nodes, props


def test_generator_constant(engine):
    from hbbft_amd.engine import g1_abi_from_uncompressed
    g1_unc = bytes.fromhex(
        "17f1d3a73197d7942695638c4fa9ac0fc3688c4f9774b905a14e3a3f171bac586c55e83ff97a1aeffb3af00adb22c6bb"
        "08b3f481e3aaa0f1a09e30ed741d8ae4fcf5e095d5d00af600db18cb2c04b3edd03cc744a2888ae40caa232946c5e7e1")
    assert G1_GEN == g1_abi_from_uncompressed(g1_unc)


@pytest.mark.parametrize("node_num", [1, 2, 3, 4, 8, 15])
def test_sync_key_gen(engine, node_num):
    t = (node_num - 1) // 3  # util::max_faulty
    rng = random.Random(1000 + node_num)
    nodes, props = make_nodes(engine, node_num, t, rng)
    # the first t+1 proposals; Acks of nodes 0..2t are kept, in (proposal, node) order
    acks = [[] for _ in range(t + 1)]
    for sender in range(t + 1):
        for node_id, node in enumerate(nodes):
            out = node.handle_parts([(sender, props[sender])], rng)[0]
            assert out.valid and out.ack is not None, out.fault
            if node_id <= 2 * t:
                acks[sender].append((node_id, out.ack))
    # Acks of all proposals but the last: t complete parts, not ready; then the rest: ready
    first = [a for s in range(t) for a in acks[s]]
    last = acks[t]
    for node in nodes:
        assert not node.is_ready()
        assert all(o.valid for o in node.handle_acks(first))
        assert not node.is_ready()
        assert all(o.valid for o in node.handle_acks(last))
        assert node.is_ready()
    pks0, _ = nodes[0].generate()
    h = hoststage.hash_g2([MSG])[0]
    sigs = []
    for idx, node in enumerate(nodes):
        pks, sk = node.generate()
        assert sk is not None
        assert pks == pks0
        share_pk = pks.public_key_shares(engine, [idx])[0]
        assert hoststage.g1_mul([G1_GEN], [sk])[0] == share_pk
        sig = hoststage.g2_mul([h], [sk])[0]
        assert engine.verify_sig_shares([share_pk], [sig], [h], [0]) == b"\x01"
        sigs.append(sig)
    out, st, v = engine.combine_verify_g2(t, [list(range(t + 1))], [sigs[: t + 1]], pks0.public_key(), [h])
    assert st == [0] and v == b"\x01"


def test_sync_key_gen_faults(engine):
    """PartFault / AckFault paths (sync_key_gen.rs:481-547, 551-588)."""
    n, t = 4, 1
    rng = random.Random(77)
    nodes, props = make_nodes(engine, n, t, rng)
    node = nodes[1]
    # RowCount
    short = Part(props[0].degree, props[0].commit, props[0].rows[:-1])
    assert node.handle_part(0, short, rng).fault == "RowCount"
    # valid, then the same Part again (Valid(None)), then a different one (MultipleParts)
    out = node.handle_part(0, props[0], rng)
    assert out.valid and out.ack is not None
    again = node.handle_part(0, props[0], rng)
    assert again.valid and again.ack is None
    assert node.handle_part(0, props[2], rng).fault == "MultipleParts"
    # RowCommitment: sender 2's rows under sender 3's commitment
    swapped = Part(props[3].degree, props[3].commit, props[2].rows)
    assert node.handle_part(3, swapped, rng).fault == "RowCommitment"
    # DecryptRow: a tampered ciphertext for our row fails Ciphertext::verify
    rows = list(props[2].rows)
    c = rows[1]
    rows[1] = Ciphertext(c.u, c.v, props[2].rows[0].w)
    assert node.handle_part(2, Part(props[2].degree, props[2].commit, rows), rng).fault == "DecryptRow"
    # Acks: good one from node 0 for part 0; ValueCount; MissingPart; duplicate; ValueCommitment
    good = nodes[0].handle_part(0, props[0], rng).ack
    assert node.handle_ack(0, Ack(0, good.values[:-1])).fault == "ValueCount"
    assert node.handle_ack(0, Ack(1, good.values)).fault == "MissingPart"  # no Part from node 1 handled
    bad = nodes[2].handle_part(0, props[0], rng).ack  # node 2's values, claimed by node 3
    outs = node.handle_acks([(0, good), (0, good), (3, bad)])
    assert outs[0].valid and outs[1].valid and outs[2].fault == "ValueCommitment"
    assert node.parts[0].acks == {0, 3} and list(node.parts[0].values) == [1]


def test_multiple_parts_after_ack(engine):
    """ProposalState's derived PartialEq covers values and acks (sync_key_gen.rs:254-262, 489-493):
    an identical Part re-sent after an Ack for that proposer is MultipleParts, not Valid(None)."""
    n, t = 4, 1
    rng = random.Random(78)
    nodes, props = make_nodes(engine, n, t, rng)
    node = nodes[1]
    assert node.handle_part(0, props[0], rng).ack is not None
    again = node.handle_part(0, props[0], rng)
    assert again.valid and again.ack is None          # no Ack yet: the same Part is ignored
    ack = nodes[2].handle_part(0, props[0], rng).ack
    assert node.handle_ack(2, ack).valid
    assert node.handle_part(0, props[0], rng).fault == "MultipleParts"
    # an observer records acks too (without values): the same rule holds for it
    obs, _ = SyncKeyGen.new(99, 5, nodes[0].pub_keys, t, engine, rng=rng)
    assert obs.handle_part(0, props[0], rng).valid
    assert obs.handle_ack(2, ack).valid
    assert obs.handle_part(0, props[0], rng).fault == "MultipleParts"


def _ack_with_payload(kg, ack, our_idx, payload, rng):
    """``ack`` with the value encrypted to node ``our_idx`` replaced by ``payload``."""
    from hbbft_amd.sync_key_gen import _encrypt_batch
    vals = list(ack.values)
    vals[our_idx] = _encrypt_batch([kg.pub_keys[our_idx]], [payload], rng)[0]
    return Ack(ack.proposer_idx, vals)


def test_ack_value_faults(engine):
    """AckFault::DecryptValue / DeserializeValue (sync_key_gen.rs:535-541): a tampered ciphertext
    fails Ciphertext::verify; a payload that is not a bincode FieldWrap<Fr> (too short, or >= r)
    does not deserialise.  bincode 1.x ignores trailing bytes, so a 33-byte payload whose first
    32 bytes are the right value is Valid.  The sender's ack is recorded in every case (:527)."""
    from hbbft_amd.sync_key_gen import _decrypt_batch
    n, t = 4, 1
    rng = random.Random(79)
    nodes, props = make_nodes(engine, n, t, rng)
    node = nodes[1]
    acks = {j: nodes[j].handle_part(0, props[0], rng).ack for j in range(n)}  # node 1 handles part 0 too
    # DecryptValue: our value's W swapped for another ciphertext's
    vals = list(acks[0].values)
    vals[1] = Ciphertext(vals[1].u, vals[1].v, vals[0].w)
    assert node.handle_ack(0, Ack(0, vals)).fault == "DecryptValue"
    # DeserializeValue: 31 bytes; a value >= r
    out = node.handle_ack(2, _ack_with_payload(nodes[2], acks[2], 1, b"\x01" * 31, rng))
    assert out.fault == "DeserializeValue"
    out = node.handle_ack(3, _ack_with_payload(nodes[3], acks[3], 1, (R_ORDER + 5).to_bytes(32, "little"), rng))
    assert out.fault == "DeserializeValue"
    assert node.parts[0].acks == {0, 2, 3} and node.parts[0].values == {}
    # 33 bytes = the right value + one trailing byte: Valid
    v1 = _decrypt_batch(engine, node.sec_key, [acks[1].values[1]])[0]
    assert len(v1) == 32
    out = node.handle_ack(1, _ack_with_payload(nodes[1], acks[1], 1, v1 + b"\x07", rng))
    assert out.valid and list(node.parts[0].values) == [2]


def test_part_row_faults(engine):
    """PartFault::DeserializeRow (sync_key_gen.rs:507) for a row payload that is not a bincode Poly
    (truncated, or a coefficient >= r); a well-formed row with the wrong coefficient count
    deserialises and fails the commitment comparison (RowCommitment, :508-510)."""
    from hbbft_amd.sync_key_gen import _encrypt_batch, ser_row
    n, t = 4, 1
    rng = random.Random(80)
    nodes, props = make_nodes(engine, n, t, rng)
    node = nodes[1]
    pk1 = node.pub_keys[1]

    def with_row(part, payload):
        rows = list(part.rows)
        rows[1] = _encrypt_batch([pk1], [payload], rng)[0]
        return Part(part.degree, part.commit, rows)

    good_row = [3] * (t + 1)
    assert node.handle_part(0, with_row(props[0], ser_row(good_row)[:-1]), rng).fault == "DeserializeRow"
    assert node.handle_part(2, with_row(props[2], ser_row([R_ORDER] + [1] * t)), rng).fault == "DeserializeRow"
    assert node.handle_part(3, with_row(props[3], ser_row([1] * (t + 2))), rng).fault == "RowCommitment"
    # each was recorded (the state is inserted before the row is checked): a re-send is Valid(None)
    assert set(node.parts) == {0, 2, 3}


def test_mixed_degree_parts(engine):
    """Parts of another degree are valid in the reference (row / evaluate run at the part's own
    degree); a batch mixing degrees runs one engine call per degree and equals one-by-one handling;
    generate() adds row(0) commitments of different lengths (Commitment's AddAssign resizes)."""
    n, t = 4, 1
    rng = random.Random(81)
    sks = [rng.randrange(1, R_ORDER) for _ in range(n)]
    pub = dict(enumerate(hoststage.g1_mul([G1_GEN] * n, sks)))
    nodes, props = [], []
    for i in range(n):
        kg, part = SyncKeyGen.new(i, sks[i], pub, t + (i == 2), engine, rng=rng)  # node 2 proposes degree 2
        kg.threshold = t
        nodes.append(kg)
        props.append(part)
    assert props[2].degree == t + 1 and len(props[2].commit) == 6
    outs = nodes[0].handle_parts([(p, props[p]) for p in range(n)], rng)
    assert all(o.valid and o.ack is not None for o in outs)
    acks = [[] for _ in range(n)]
    for j, kg in enumerate(nodes):
        for p in range(n):
            o = kg.handle_part(p, props[p], rng) if j else None
            if j:
                assert o.valid and o.ack is not None
                acks[p].append((j, o.ack))
    acks_all = [a for p in range(n) for a in acks[p]] + [(0, o.ack) for o in outs]
    res = nodes[0].handle_acks(acks_all)
    assert all(r.valid for r in res)
    assert all(nodes[0].parts[p].is_complete(t) for p in range(n))
    pks, sk = nodes[0].generate()
    assert len(pks.commit) == t + 2  # degree-2 part's row(0) extends the key's commitment


def _pt1(b):
    return None if b == bytes(96) else (int.from_bytes(b[:48], "little"), int.from_bytes(b[48:], "little"))


def _pt2(b):
    if b == bytes(192):
        return None
    w = [int.from_bytes(b[48 * k:48 * (k + 1)], "little") for k in range(4)]
    return ((w[0], w[1]), (w[2], w[3]))


def test_encrypt_decrypt_batches_match_oracle(engine):
    """encrypt_with_rng on fixed nonces (hbh_encrypt: comb U = g1 r, GLV pk r, W = [KCOF r] Q_bp) and
    SecretKey::decrypt over a batch (_decrypt_batch: host hash_g1_g2, engine Ciphertext::verify,
    host GLV U sk + XOR) against oracle/tc.py (src/sync_key_gen.rs:346-357, 386-390, 503-506, 535-538):
    byte-identical (U, V, W) for 32-byte Ack values and 1,096-byte Part rows (the two |V| branches of
    hash_g1_g2) plus 0 / 64 / 65-byte edge messages; plaintexts recovered; tampered U, V or W -> None,
    as the oracle's Ciphertext::verify rejects them."""
    from oracle import tc
    from hbbft_amd.sync_key_gen import _decrypt_batch, ser_row, ser_val
    rng = random.Random(77)
    sk = rng.randrange(1, R_ORDER)
    pk = hoststage.g1_mul([G1_GEN], [sk])[0]
    msgs = ([ser_val(rng.randrange(R_ORDER)) for _ in range(5)]
            + [ser_row([rng.randrange(R_ORDER) for _ in range(34)]) for _ in range(3)] + [b"", bytes(64), bytes(65)])
    nonces = [rng.randrange(1, R_ORDER) for _ in msgs]
    got = hoststage.encrypt([pk], msgs, nonces, threads=4)
    for (u, v, w), m, r in zip(got, msgs, nonces):
        eu, ev, ew = tc.encrypt(_pt1(pk), m, r)
        assert (_pt1(u), v, _pt2(w)) == (eu, ev, ew)
    cts = [Ciphertext(u, v, w) for u, v, w in got]
    # tampered copies: V byte flipped, W of another ciphertext, U of another ciphertext
    bad = [Ciphertext(cts[0].u, bytes([cts[0].v[0] ^ 1]) + cts[0].v[1:], cts[0].w),
           Ciphertext(cts[6].u, cts[6].v, cts[1].w),
           Ciphertext(cts[2].u, cts[7].v, cts[7].w)]
    for c in bad:
        assert not tc.ciphertext_verify((_pt1(c.u), c.v, _pt2(c.w)))
    # the Q-form check (hash_g1_g2_bp + e(G1K, W) == e(U, Q)) gives Ciphertext::verify's verdicts
    us, vs, ws = [c.u for c in cts + bad], [c.v for c in cts + bad], [c.w for c in cts + bad]
    want = bytes([1] * len(cts) + [0] * len(bad))
    assert engine.verify_ciphertexts(us, ws, hoststage.hash_g1_g2(us, vs)) == want
    assert engine.verify_ciphertexts_bp(us, ws, hoststage.hash_g1_g2_bp(us, vs)) == want
    plain = _decrypt_batch(engine, sk, cts + bad, threads=4)
    assert plain[:len(msgs)] == msgs
    assert plain[len(msgs):] == [None] * len(bad)
