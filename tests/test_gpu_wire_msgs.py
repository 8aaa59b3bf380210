"""Batched bincode decoding on the GPU (hbbft_amd.wire) and the drivers fed raw
message bytes: the engine's decoding equals the oracle's on valid, infinity, off-curve and
non-subgroup encodings; a HoneyBadger epoch replayed from bincode bytes equals the same epoch
from ABI points, and damaged messages / contributions are faulted (DeserializeMessage /
DeserializeCiphertext, epoch_state.rs:377-381); a SyncKeyGen run fed Part / Ack bytes equals the
object-fed run (sync_key_gen.rs:481-547)."""
import random
import struct

import pytest

from oracle import bls12_381 as C
from hbbft_amd import hoststage, wire
from hbbft_amd.honey_badger import EpochTrace, NetworkKeys, run_epoch
from hbbft_amd.sync_key_gen import G1_GEN, R_ORDER, SyncKeyGen

from tests.test_wire_msgs import OracleDecompressor

pytestmark = pytest.mark.gpu


def _encs(rng):
    """Valid, infinity, off-curve and on-curve non-subgroup compressed G1 / G2 encodings."""
    g1 = [C.g1_compress(C.g1_mul(C.G1_GEN, rng.randrange(1, C.R))) for _ in range(6)] + [C.g1_compress(None)]
    g2 = [C.g2_compress(C.g2_mul(C.G2_GEN, rng.randrange(1, C.R))) for _ in range(3)] + [C.g2_compress(None)]
    for dec, lst, size in ((C.g1_decompress, g1, 48), (C.g2_decompress, g2, 96)):
        kinds = set()
        while len(kinds) < 2:
            b = bytearray(rng.randrange(C.P).to_bytes(size, "big") if size == 48 else
                          rng.randrange(C.P).to_bytes(48, "big") + rng.randrange(C.P).to_bytes(48, "big"))
            b[0] |= 0x80
            try:
                dec(bytes(b))
            except C.DecodeError as e:
                k = "curve" if "curve" in str(e) else ("subgroup" if "subgroup" in str(e) else None)
                if k and k not in kinds:
                    kinds.add(k)
                    lst.append(bytes(b))
    return g1, g2


def test_share_message_decoding_matches_oracle(engine):
    rng = random.Random(11)
    g1, g2 = _encs(rng)
    m1 = [struct.pack("<Q", 48) + e for e in g1] + [b"\x01"]
    m2 = [struct.pack("<Q", 96) + e for e in g2] + [struct.pack("<Q", 96) + g2[0][:50]]
    ora = OracleDecompressor()
    got1, got2 = wire.decode_dec_share_msgs(engine, m1), wire.decode_sig_share_msgs(engine, m2)
    assert got1 == wire.decode_dec_share_msgs(ora, m1)
    assert got2 == wire.decode_sig_share_msgs(ora, m2)
    assert sum(x is None for x in got1) == 3 and sum(x is None for x in got2) == 3


@pytest.mark.parametrize("pipelined", [False, True])
def test_epoch_from_raw_bytes(engine, pipelined):
    n, t = 7, 2
    rng = random.Random(900)
    keys = NetworkKeys(engine, n, t, rng)
    trace = EpochTrace.generate(engine, keys, rng, hb_epoch=3, bad_every=9, proposal_bytes=90)
    ref = run_epoch(engine, keys, trace, window=5, pipelined=pipelined)
    trace.serialize()
    raw = run_epoch(engine, keys, trace, window=5, pipelined=pipelined, raw=True)
    assert (raw.plaintexts, raw.coins, raw.signatures) == (ref.plaintexts, ref.coins, ref.signatures)
    key = lambda r: sorted((k, p, f.node_id, f.kind) for k, p, f in r.faults)
    assert key(raw) == key(ref)
    # damaged bytes: one coin share, one decryption share, one whole contribution
    coin_p = sorted(trace.coin_docs)[0]
    corrupt = [("coin", coin_p, 3), ("dec", 1, 4), ("ct", 5)]
    trace.serialize(corrupt=corrupt)
    bad = run_epoch(engine, keys, trace, window=5, pipelined=pipelined, raw=True)
    kinds = {(k, p, f.node_id, f.kind) for k, p, f in bad.faults}
    assert ("coin", coin_p, 3, "DeserializeMessage") in kinds
    assert ("dec", 1, 4, "DeserializeMessage") in kinds
    assert ("dec", 5, 5, "DeserializeCiphertext") in kinds
    assert 5 not in bad.plaintexts and {p: v for p, v in ref.plaintexts.items() if p != 5} == bad.plaintexts
    assert bad.coins == ref.coins


def test_sync_key_gen_from_raw_bytes(engine):
    n, t = 4, 1
    rng = random.Random(901)
    sks = [rng.randrange(1, R_ORDER) for _ in range(n)]
    pub = dict(enumerate(hoststage.g1_mul([G1_GEN] * n, sks)))
    nodes, props = [], []
    for i in range(n):
        kg, part = SyncKeyGen.new(i, sks[i], pub, t, engine, rng=rng)
        nodes.append(kg)
        props.append(part)
    twins = [SyncKeyGen(i, sks[i], pub, t, engine) for i in range(n)]   # fed bytes
    acks = []
    for p in range(n):
        for j in range(n):
            o = nodes[j].handle_parts([(p, props[p])], rng)[0]
            ob = twins[j].handle_part_msgs([(p, props[p].to_bytes())], rng)[0]
            assert o.valid and ob.valid and o.ack is not None and ob.ack is not None
            acks.append((j, o.ack))
    # a damaged Part message: DeserializeMessage, state untouched
    damaged = props[0].to_bytes()[:-7]
    assert twins[1].handle_part_msgs([(0, damaged)], rng)[0].fault == "DeserializeMessage"
    for kg, tw in zip(nodes, twins):
        r1 = kg.handle_acks(acks)
        r2 = tw.handle_ack_msgs([(s, a.to_bytes()) for s, a in acks])
        assert [o.fault for o in r1] == [o.fault for o in r2] and all(o.valid for o in r1)
    for kg, tw in zip(nodes, twins):
        assert kg.generate() == tw.generate()


def test_ba_epoch_from_raw_bytes(engine):
    """BA-driven coins fed bincode coin-share messages (round 6: the raw epoch line): each window
    is decoded in one engine call before it is queued; outputs equal the point-fed epoch's, and a
    truncated coin-share message is a DeserializeMessage fault of its sender that changes no
    decision or coin."""
    n, t = 7, 2
    rng = random.Random(902)
    keys = NetworkKeys(engine, n, t, rng)
    trace = EpochTrace.generate(engine, keys, rng, hb_epoch=5, bad_every=9, proposal_bytes=70)
    trace.with_ba(engine, rng, extra=0.3, bad_every=11)
    ref = run_epoch(engine, keys, trace, window=16)
    trace.serialize()
    raw = run_epoch(engine, keys, trace, window=16, raw=True)
    assert (raw.plaintexts, raw.coins, raw.signatures) == (ref.plaintexts, ref.coins, ref.signatures)
    assert (raw.ba_decisions, raw.ba_coins) == (ref.ba_decisions, ref.ba_coins)
    key = lambda r: sorted((k, p, f.node_id, f.kind) for k, p, f in r.faults)
    assert key(raw) == key(ref)
    m = next(k for k in trace.ba.msgs if ("coin", k[0], k[2]) not in (trace.bad | trace.ba.bad) and k[2] != 0)
    trace.serialize(corrupt=[("ba",) + tuple(m)])
    bad = run_epoch(engine, keys, trace, window=16, raw=True)
    assert ("coin", m[0], m[2], "DeserializeMessage") in {(k, p, f.node_id, f.kind) for k, p, f in bad.faults}
    assert (bad.ba_decisions, bad.ba_coins, bad.plaintexts) == (ref.ba_decisions, ref.ba_coins, ref.plaintexts)
