"""ThresholdSign / ThresholdDecrypt message flows (hbbft_amd/protocol.py, the host mirror of
src/threshold_sign.rs and src/threshold_decrypt.rs) running on the GPU engine, in the style of the
reference's tests/threshold_sign.rs: a simulated network of N nodes with f silent or lying nodes;
every correct node and an observer output the same value; no correct node is ever blamed; shares
are verified in batches through the verdict cache."""
import random

import pytest

from oracle import bls12_381 as C
from oracle import cbls, tc
from hbbft_amd.engine import g1_abi_from_uncompressed as g1a, g2_abi_from_uncompressed as g2a
from hbbft_amd.protocol import (BatchVerifier, Ciphertext, NetworkInfo, ProtocolError, Step, ThresholdDecrypt,
                                ThresholdSign, xor_with_hash)

pytestmark = pytest.mark.gpu
G1 = g1a(C.g1_uncompressed(C.G1_GEN))
G2 = g2a(C.g2_uncompressed(C.G2_GEN))


def keyset(rng, n, t):
    coeffs = [rng.randrange(1, C.R) for _ in range(t + 1)]
    sks = {i: tc.poly_eval(coeffs, i + 1) for i in range(n)}
    pks = {i: cbls.g1_mul(G1, sks[i]) for i in range(n)}
    return coeffs, sks, pks, cbls.g1_mul(G1, coeffs[0])


class Net:
    """In-process network: messages are (sender, target, payload), delivered in seeded random order."""

    def __init__(self, rng):
        self.rng, self.queue = rng, []

    def dispatch(self, sender, step, ids):
        for target, payload in step.messages:
            assert target == "all"
            for i in ids:
                if i != sender:
                    self.queue.append((sender, i, payload))


def run_sign(engine, n, f, seed, liars=(), window=1):
    rng = random.Random(seed)
    coeffs, sks, pks, mpk = keyset(rng, n, f)
    h = cbls.g2_mul(G2, rng.randrange(1, C.R))
    ids = list(range(n))
    silent = set(range(n - f, n)) - set(liars)
    nodes = {}
    for i in ids + ["observer"]:
        sk = sks.get(i)
        ni = NetworkInfo(i, ids, f, mpk, pks, sign_g2=(lambda H, sk=sk: cbls.g2_mul(H, sk)) if sk else None)
        nodes[i] = ThresholdSign(ni, BatchVerifier(engine))
    net = Net(rng)
    outputs, faults = {}, []
    for i in rng.sample(ids, len(ids)):  # documents arrive at different times
        if i in silent:
            continue
        nodes[i].set_document_hash(h)
        if i in liars:  # a lying node broadcasts a share of the wrong document
            net.queue += [(i, j, cbls.g2_mul(G2, 12345)) for j in ids + ["observer"] if j != i]
            continue
        step = nodes[i].handle_input()
        net.dispatch(i, step, ids + ["observer"])
        outputs.setdefault(i, []).extend(step.output)
        faults += [(i, flt) for flt in step.fault_log]
    nodes["observer"].set_document_hash(h)
    while net.queue:
        # a window of deliveries: every receiver pre-verifies the shares in it in one drain
        batch = [net.queue.pop(rng.randrange(len(net.queue))) for _ in range(min(window, len(net.queue)))]
        batch = [(s_, t_, p_) for s_, t_, p_ in batch if t_ not in silent and t_ not in liars]
        for sender, target, payload in batch:
            if nodes[target].doc_hash is not None and sender in pks:
                nodes[target].verifier.queue_sig(pks[sender], nodes[target].doc_hash, payload)
        for target in {t_ for _, t_, _ in batch}:
            nodes[target].verifier.drain()
        for sender, target, payload in batch:
            step = nodes[target].handle_message(sender, payload)
            net.dispatch(target, step, ids + ["observer"])
            outputs.setdefault(target, []).extend(step.output)
            faults += [(target, flt) for flt in step.fault_log]
    step = nodes["observer"].handle_input()
    outputs.setdefault("observer", []).extend(step.output)
    return outputs, faults, cbls.g2_mul(h, coeffs[0]), silent, nodes


@pytest.mark.parametrize("n,f,seed", [(4, 1, 1), (10, 3, 2), (13, 4, 3)])
def test_threshold_sign_silent_faulty(engine, n, f, seed):
    outputs, faults, want, silent, _ = run_sign(engine, n, f, seed)
    correct = [i for i in range(n) if i not in silent]
    for i in correct + ["observer"]:
        assert outputs[i] == [want], i  # exactly one output, the combined signature
    assert faults == []


def test_threshold_sign_lying_nodes_are_blamed(engine):
    n, f = 10, 3
    liars = (8, 9)
    outputs, faults, want, silent, nodes = run_sign(engine, n, f, 11, liars=liars, window=24)
    for i in range(n):
        if i not in silent and i not in liars:
            assert outputs[i] == [want]
    assert faults and all(flt.node_id in liars and flt.kind == "UnverifiedSignatureShareSender" for _, flt in faults)
    # verdicts went through the batched verifier (windowed drains): fewer engine calls than checks
    honest = [i for i in range(n) if i not in silent and i not in liars]
    calls = sum(nodes[i].verifier.calls for i in honest)
    checks = sum(nodes[i].verifier.checks for i in honest)
    assert 0 < calls < checks
    assert max(nodes[i].verifier.max_batch for i in honest) > 1


def test_threshold_sign_errors_and_postponed_verification(engine):
    rng = random.Random(5)
    coeffs, sks, pks, mpk = keyset(rng, 4, 1)
    h = cbls.g2_mul(G2, 77)
    ni = NetworkInfo(0, range(4), 1, mpk, pks, sign_g2=lambda H: cbls.g2_mul(H, sks[0]))
    ts = ThresholdSign(ni, BatchVerifier(engine))
    with pytest.raises(ProtocolError) as e:
        ts.sign()
    assert e.value.kind == "DocumentHashIsNone"
    with pytest.raises(ProtocolError) as e:
        ts.handle_message(99, cbls.g2_mul(h, 1))
    assert e.value.kind == "UnknownSender"
    # a bad share before the document is stored unverified and blamed at sign() (:165)
    assert ts.handle_message(2, cbls.g2_mul(G2, 5)).fault_log == []
    ts.set_document_hash(h)
    step = ts.sign()
    assert [flt.node_id for flt in step.fault_log] == [2]
    assert ts.verifier.calls >= 1
    with pytest.raises(ProtocolError):
        ts.set_document_hash(h)
    # the share of node 1 completes the signature
    step = ts.handle_message(1, cbls.g2_mul(h, sks[1]))
    assert step.output == [cbls.g2_mul(h, coeffs[0])]
    assert ts.terminated and ts.handle_message(3, b"\0" * 192).fault_log == []  # no blame after termination


def test_threshold_decrypt_flow(engine):
    rng = random.Random(21)
    n, f = 7, 2
    coeffs, sks, pks, mpk = keyset(rng, n, f)
    msg = bytes(rng.randrange(256) for _ in range(100))
    mpk_pt = (int.from_bytes(mpk[:48], "little"), int.from_bytes(mpk[48:], "little"))
    u, v, w = tc.encrypt(mpk_pt, msg, rng.randrange(1, C.R))
    huv = tc.hash_g1_g2(u, v)
    ct = Ciphertext(g1a(C.g1_uncompressed(u)), v, g2a(C.g2_uncompressed(w)), g2a(C.g2_uncompressed(huv)))
    nodes = {i: ThresholdDecrypt(NetworkInfo(i, range(n), f, mpk, pks,
                                             decrypt_share=lambda U, sk=sks[i]: cbls.g1_mul(U, sk)),
                                 BatchVerifier(engine)) for i in range(n)}
    # node 0 receives shares (one forged) before it has the ciphertext: verified later in one batch
    early = {j: cbls.g1_mul(ct.u, sks[j]) for j in (1, 2, 3)}
    early[3] = cbls.g1_mul(G1, 999)
    for j, s in early.items():
        assert nodes[0].handle_message(j, s).fault_log == []
    nodes[0].set_ciphertext(ct)
    step = nodes[0].handle_input()
    assert [flt.node_id for flt in step.fault_log] == [3]
    assert step.output == [msg]
    # Ciphertext::verify, the three early shares in one drain, the interpolation
    assert nodes[0].verifier.calls == 3 and nodes[0].verifier.max_batch == 3
    # duplicate share -> MultipleDecryptionShares; invalid ciphertext -> InvalidCiphertext
    nodes[1].set_ciphertext(ct)
    assert nodes[1].handle_message(2, cbls.g1_mul(ct.u, sks[2])).fault_log == []
    dup = nodes[1].handle_message(2, cbls.g1_mul(ct.u, sks[2]))
    assert [flt.kind for flt in dup.fault_log] == ["MultipleDecryptionShares"]
    bad = Ciphertext(ct.u, ct.v, cbls.g2_mul(G2, 3), ct.huv)
    with pytest.raises(ProtocolError) as e:
        nodes[2].set_ciphertext(bad)
    assert e.value.kind == "InvalidCiphertext"
    assert xor_with_hash(cbls.g1_mul(G1, 5), b"abc") == tc.xor_with_hash(C.g1_mul(C.G1_GEN, 5), b"abc")


def test_threshold_sign_document_and_coin(engine):
    """set_document(doc) hashes on the host stage (hbh_hash_g2, threshold_sign.rs:147-153); the
    combined signature is msk * hash_g2(doc) and its parity is the BA coin (binary_agreement.rs:402)."""
    from hbbft_amd import hoststage
    from hbbft_amd.protocol import signature_parity
    rng = random.Random(31)
    n, f = 4, 1
    coeffs, sks, pks, mpk = keyset(rng, n, f)
    doc = (7).to_bytes(8, "little") + (2).to_bytes(8, "little") + (3).to_bytes(4, "little") + (2).to_bytes(8, "little")
    nodes = {i: ThresholdSign(NetworkInfo(i, range(n), f, mpk, pks,
                                          sign_g2=lambda H, sk=sks[i]: hoststage.g2_mul([H], [sk])[0]),
                              BatchVerifier(engine)) for i in range(n)}
    for node in nodes.values():
        node.set_document(doc)
    steps = {i: nodes[i].handle_input() for i in range(n)}
    shares = {i: steps[i].messages[0][1] for i in range(n)}
    out = None
    for j in (1, 2):
        st = nodes[0].handle_message(j, shares[j])
        out = st.output or out
    h = g2a(C.g2_uncompressed(tc.hash_g2(doc)))
    assert nodes[0].doc_hash == h
    want = cbls.g2_mul(h, coeffs[0])
    assert out == [want]
    assert signature_parity(want) == tc.signature_parity(C.g2_mul(tc.hash_g2(doc), coeffs[0]))
    assert nodes[0].verifier.cached() == 0  # released at termination


def test_threshold_decrypt_raw_ciphertext(engine):
    """Ciphertexts from encrypt_with_rng on the host stage; H_uv computed by set_ciphertext's
    Ciphertext (hash_g1_g2 on the host); plaintext recovered byte for byte."""
    from hbbft_amd import hoststage
    rng = random.Random(41)
    n, f = 4, 1
    coeffs, sks, pks, mpk = keyset(rng, n, f)
    msg = bytes(rng.randrange(256) for _ in range(90))
    u, v, w = hoststage.encrypt([mpk], [msg], [rng.randrange(1, C.R)])[0]
    nodes = {i: ThresholdDecrypt(NetworkInfo(i, range(n), f, mpk, pks,
                                             decrypt_share=lambda U, sk=sks[i]: hoststage.g1_mul([U], [sk])[0]),
                                 BatchVerifier(engine)) for i in range(n)}
    ct = Ciphertext(u, v, w)
    for node in nodes.values():
        node.set_ciphertext(ct)
    steps = {i: nodes[i].handle_input() for i in range(n)}
    got = None
    for j in (1, 2):
        st = nodes[0].handle_message(j, steps[j].messages[0][1])
        got = st.output or got
    assert got == [msg]
