"""BatchVerifier's drain bookkeeping on the CPU with a stand-in engine (no GPU): the synchronous
drain and the pipelined drain_async/commit cache the same verdicts, every queued check reaches
the engine once, and verdicts of an instance released while its drain was in flight are dropped
(hbbft_amd/protocol.py; the windowed driver is hbbft_amd/honey_badger._deliver)."""
import threading

from hbbft_amd.protocol import BatchVerifier


class FakeEngine:
    """verdict = first byte of the share is even; records the thread of every call."""

    def __init__(self):
        self.calls = []

    def verify_sig_shares(self, pks, sigs, hashes, doc_idx):
        self.calls.append(("sig", len(pks), threading.current_thread().name))
        return bytes(int(s[0] % 2 == 0) for s in sigs)

    def verify_dec_shares(self, shares, pks, huv, w, ct_idx):
        self.calls.append(("dec", len(shares), threading.current_thread().name))
        return bytes(int(s[0] % 2 == 0) for s in shares)

    def verify_ciphertexts(self, u, w, huv):
        self.calls.append(("ct", len(u), threading.current_thread().name))
        return bytes(1 for _ in u)


def _fill(ver, docs=3, per=5):
    items = []
    for d in range(docs):
        h = bytes([d]) * 8
        for j in range(per):
            pk, sh = bytes([j]) * 4, bytes([d * per + j]) * 4
            ver.queue_sig(pk, h, sh)
            items.append((pk, h, sh))
    return items


def test_sync_and_async_drains_cache_the_same_verdicts():
    e1, e2 = FakeEngine(), FakeEngine()
    v1, v2 = BatchVerifier(e1), BatchVerifier(e2)
    items = _fill(v1)
    _fill(v2)
    v1.drain()
    v2.commit(v2.drain_async())
    for pk, h, sh in items:
        assert v1.sig_valid(pk, h, sh) == v2.sig_valid(pk, h, sh) == (sh[0] % 2 == 0)
    assert [c[:2] for c in e1.calls] == [c[:2] for c in e2.calls] == [("sig", 15)]
    assert e2.calls[0][2].startswith("hbh-drain")
    assert v2.checks == 15 and v2.calls == 1


def test_release_during_async_drain_drops_verdicts():
    eng = FakeEngine()
    ver = BatchVerifier(eng)
    _fill(ver, docs=2)
    pending = ver.drain_async()
    ver.release_doc(bytes([0]) * 8)      # instance 0 terminates while its drain is in flight
    ver.commit(pending)
    assert bytes([0]) * 8 not in ver._sig and bytes([1]) * 8 in ver._sig
    assert ver.cached() == 5
    assert not ver._released            # nothing in flight any more: the release set is empty


def test_duplicates_are_checked_once():
    eng = FakeEngine()
    ver = BatchVerifier(eng)
    _fill(ver, docs=1)
    _fill(ver, docs=1)
    ver.commit(ver.drain_async())
    _fill(ver, docs=1)                   # already cached: nothing queued
    ver.drain()
    assert [c[:2] for c in eng.calls] == [("sig", 5)]


def test_shared_instance_key_survives_one_release():
    """Two running instances with the same key (a copied ciphertext, a repeated document): the
    first one's termination must not drop verdicts the second still reads, and a synchronous
    miss after the last release still returns its verdict (no KeyError)."""
    eng = FakeEngine()
    ver = BatchVerifier(eng)
    h = bytes([7]) * 8
    ver.open_doc(h)
    ver.open_doc(h)
    ver.queue_sig(b"pk", h, b"\x02sh")
    pending = ver.drain_async()
    ver.release_doc(h)                   # instance A terminates while the drain is in flight
    ver.commit(pending)
    assert ver.sig_valid(b"pk", h, b"\x02sh") is True   # instance B: still cached
    assert len(eng.calls) == 1
    assert ver.sig_valid(b"pk2", h, b"\x03sh") is False  # B's miss: verified and cached
    ver.release_doc(h)                   # B terminates: dropped
    assert ver.cached() == 0
    assert ver.sig_valid(b"pk3", h, b"\x04sh") is True   # a stray miss after release: no KeyError
    assert ver.cached() == 0


class FlowEngine(FakeEngine):
    """FakeEngine plus a combine that always succeeds."""

    def combine_verify_g2(self, t, idx, shares, master_pk, hashes):
        return [b"S" * 192 for _ in idx], [0] * len(idx), b"\x01" * len(idx)


def test_two_threshold_sign_instances_same_document():
    """Two ThresholdSign instances on one document and one BatchVerifier: both terminate with
    the reference's outputs and faults, whichever terminates first."""
    from hbbft_amd.protocol import NetworkInfo, ThresholdSign
    ver = BatchVerifier(FlowEngine())
    n, t = 4, 1
    pks = {i: bytes([i]) * 96 for i in range(n)}
    ni = NetworkInfo(0, range(n), t, b"M" * 96, pks)       # observer: no secret key
    a, b = ThresholdSign(ni, ver), ThresholdSign(ni, ver)
    h = bytes([9]) * 192
    a.set_document_hash(h)
    b.set_document_hash(h)
    for inst in (a, b):
        inst.handle_input()
        for j in range(n):
            ver.queue_sig(pks[j], h, bytes([2 * j]) * 192)
    ver.drain()
    sa = a.handle_message(1, bytes([2]) * 192)
    sa.extend(a.handle_message(2, bytes([4]) * 192))
    assert a.terminated and sa.output == [b"S" * 192]
    # b reads verdicts cached before a's release, then one that was never queued (a miss)
    sb = b.handle_message(3, bytes([6]) * 192)
    sb.extend(b.handle_message(2, bytes([5]) * 192))   # odd first byte: invalid -> fault
    sb.extend(b.handle_message(1, bytes([2]) * 192))
    assert b.terminated and sb.output == [b"S" * 192]
    assert [f.kind for f in sb.fault_log] == ["UnverifiedSignatureShareSender"]
    assert ver.cached() == 0


def test_verdict_store_groups_per_instance_and_serves_a_sync_miss():
    """Round 4's verdict store: dec and ct checks land under their ciphertext key, sig checks under
    their document; a synchronous miss drains once and returns its own verdict."""
    eng = FakeEngine()
    ver = BatchVerifier(eng)
    huv, w = b"H" * 192, b"W" * 192
    ver.queue_dec(b"pk1", b"\x02s", huv, w)
    ver.queue_dec(b"pk2", b"\x03s", huv, w)
    ver.drain()
    assert ver._dec[(huv, w)] == {(b"pk1", b"\x02s"): True, (b"pk2", b"\x03s"): False}
    assert ver.dec_valid(b"pk1", b"\x02s", huv, w) is True and len(eng.calls) == 1
    assert ver.dec_valid(b"pk3", b"\x05s", huv, w) is False and len(eng.calls) == 2   # miss: one drain
    assert ver.sig_valid(bytearray(b"pk"), bytearray(b"D" * 8), bytearray(b"\x04s")) is True  # non-bytes keys
    assert ver._sig[b"D" * 8] == {(b"pk", b"\x04s"): True}
    assert ver.lookups == 3 and ver.checks == 4


def test_add_doc_hashes_feeds_the_hash_cache():
    """Prefetched document hashes (honey_badger.prefetch_coins) are served without hashing."""
    ver = BatchVerifier(FakeEngine())
    ver.add_doc_hashes({b"doc": b"H" * 192})
    assert ver.doc_hash_of(b"doc") == b"H" * 192
    assert ver.hash_doc(b"doc") == b"H" * 192     # set_document takes it out of the cache
    assert b"doc" not in ver._docs


def test_engine_wait_is_accounted():
    """wait_s counts the time the calling thread spent in engine calls (the epoch line's
    host / GPU split), async_s the worker's."""
    import time as _t

    class Slow(FakeEngine):
        def verify_sig_shares(self, *a):
            _t.sleep(0.02)
            return super().verify_sig_shares(*a)

    ver = BatchVerifier(Slow())
    _fill(ver, docs=1)
    ver.drain()
    assert ver.wait_s >= 0.015
    _fill(ver, docs=2)
    w0 = ver.wait_s
    ver.commit(ver.drain_async())
    assert ver.async_s >= 0.015 and ver.wait_s >= w0


def test_speculative_g1_combines_serve_deferred_decryptions():
    """BatchVerifier._spec_g1 (round 5, honey_badger._dec_preverify): a deferred G1 combine tagged with a
    ciphertext key whose point was combined early takes that point without an engine call; untagged
    ones, keys without a point, and a set with a repeated index go to the engine."""
    from hbbft_amd.protocol import Deferred

    class G1Engine(FakeEngine):
        def interpolate_g1(self, t, idx, pts):
            self.calls.append(("g1", len(idx), threading.current_thread().name))
            return [b"engine" + bytes(len(i)) for i in idx], [0] * len(idx)

    eng = G1Engine()
    ver = BatchVerifier(eng)
    ver.recording = True
    ver.add_speculative_g1({(b"huv1", b"w1"): b"spec-point"})
    d1, _ = ver.interpolate_g1(1, [0, 1], [b"a", b"b"])
    d1.tag = (b"huv1", b"w1")
    d2, _ = ver.interpolate_g1(1, [2, 3], [b"c", b"d"])
    d2.tag = (b"huv2", b"w2")                      # no speculative point for this ciphertext
    d3, _ = ver.interpolate_g1(1, [4, 4], [b"e", b"e"])
    d3.tag = (b"huv1", b"w1")                      # repeated index: the engine decides (DuplicateEntry)
    d4, _ = ver.interpolate_g1(1, [5, 6], [b"f", b"g"])  # untagged
    assert all(isinstance(d, Deferred) for d in (d1, d2, d3, d4))
    ver.flush_combines()
    assert d1.result == (b"spec-point", 0)
    assert d2.result[0].startswith(b"engine") and d3.result[0].startswith(b"engine")
    assert d4.result[0].startswith(b"engine")
    assert [c[:2] for c in eng.calls] == [("g1", 3)]
