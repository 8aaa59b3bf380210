"""Host-side mirror of hbbft's ThresholdSign and ThresholdDecrypt message flows over the GPU engine.

Reference: ``src/threshold_sign.rs`` and ``src/threshold_decrypt.rs`` (the ``ConsensusProtocol``
instances of SURVEY.md §3.1/§3.2).  Same method names, argument meaning, error and fault
behaviour; the only change is *where the crypto runs*: every share check goes through a
``BatchVerifier`` -- the verdict cache / batch drain of SURVEY §8f f1 -- which verifies all
shares queued at the reference's own deferred-verification points (``remove_invalid_shares``)
or by a driver's pre-verification window in ONE C-ABI call, and combines run through
``hbh_interpolate_g2/g1``.  Verdicts are a pure function of (public key, hash point, share), so
caching them cannot change which ``Step`` a fault lands in.

What stays on the host, as in the reference and the north star: hashing to G2 (the caller passes
the document hash point / ``hash_g1_g2(U, V)``), secret-key operations (``sign_g2``,
``decrypt_share_no_verify``: ``NetworkInfo`` holds callables), and the XOR stream of
``PublicKeySet::decrypt`` (``xor_with_hash`` below: SHA3-256 + ChaCha20).
"""
import hashlib
import struct

from ._lib import G1_BYTES, G2_BYTES

P_FIELD = 0x1A0111EA397FE69A4B1BA7B6434BACD764774B84F38512BF6730D2A0F6B0F6241EABFFFEB153FFFFB9FEFFFFFFFFAAAB


# ------------------------------------------------------------------ Step / faults (src/traits.rs:64-74)
class Fault:
    def __init__(self, node_id, kind):
        self.node_id, self.kind = node_id, kind

    def __eq__(self, o):
        return isinstance(o, Fault) and (self.node_id, self.kind) == (o.node_id, o.kind)

    def __repr__(self):
        return "Fault(%r, %s)" % (self.node_id, self.kind)


class Step:
    """``Step { output, fault_log, messages }``; messages are (target, payload), target "all"."""

    def __init__(self, output=None, fault_log=None, messages=None):
        self.output = list(output or [])
        self.fault_log = list(fault_log or [])
        self.messages = list(messages or [])

    @staticmethod
    def fault(node_id, kind):
        return Step(fault_log=[Fault(node_id, kind)])

    def extend(self, other):
        self.output += other.output
        self.fault_log += other.fault_log
        self.messages += other.messages
        return self

    join = extend

    def with_output(self, out):
        self.output.append(out)
        return self


class ProtocolError(Exception):
    """The reference's ``Error`` enums (``threshold_sign::Error``, ``threshold_decrypt::Error``)."""

    def __init__(self, kind, detail=None):
        super().__init__(kind if detail is None else "%s(%s)" % (kind, detail))
        self.kind, self.detail = kind, detail


# ------------------------------------------------------------------ keys (src/network_info.rs)
class NetworkInfo:
    """Node ids, the public key set and this node's secret-key operations.

    pk_shares: {node_id: G1 ABI bytes}; master_pk: G1 ABI bytes; t: threshold (num_faulty);
    sign_g2(H) / decrypt_share(U): this node's secret operations (None for an observer)."""

    def __init__(self, our_id, node_ids, t, master_pk, pk_shares, sign_g2=None, decrypt_share=None):
        self.our_id = our_id
        self._ids = sorted(node_ids)
        self._index = {n: i for i, n in enumerate(self._ids)}
        self.t = t
        self.master_pk = master_pk
        self.pk_shares = dict(pk_shares)
        self.sign_g2 = sign_g2
        self.decrypt_share = decrypt_share

    def node_index(self, node_id):
        return self._index.get(node_id)

    def num_faulty(self):
        return self.t

    def public_key_share(self, node_id):
        return self.pk_shares.get(node_id)

    def is_validator(self):
        return self.sign_g2 is not None


# ------------------------------------------------------------------ verdict cache / batch drain
class BatchVerifier:
    """Pure, order-independent verdict cache.  ``queue_*`` records checks; ``drain`` verifies every
    queued check in one engine call per kind; ``*_valid`` returns a cached verdict (or verifies a
    single miss immediately).  ``calls`` counts engine calls (the batching evidence in tests)."""

    def __init__(self, engine):
        self.eng = engine
        self._sig, self._dec = {}, {}
        self._qsig, self._qdec = [], []
        self.calls = 0

    # ThresholdSign: PublicKeyShare::verify_g2(share, H)  (src/threshold_sign.rs:223)
    def queue_sig(self, pk, h, share):
        key = (bytes(pk), bytes(h), bytes(share))
        if key not in self._sig:
            self._qsig.append(key)

    def sig_valid(self, pk, h, share):
        key = (bytes(pk), bytes(h), bytes(share))
        if key not in self._sig:
            self._qsig.append(key)
            self.drain()
        return self._sig[key]

    # ThresholdDecrypt: PublicKeyShare::verify_decryption_share(share, ct)  (src/threshold_decrypt.rs:227)
    def queue_dec(self, pk, share, huv, w):
        key = (bytes(pk), bytes(share), bytes(huv), bytes(w))
        if key not in self._dec:
            self._qdec.append(key)

    def dec_valid(self, pk, share, huv, w):
        key = (bytes(pk), bytes(share), bytes(huv), bytes(w))
        if key not in self._dec:
            self._qdec.append(key)
            self.drain()
        return self._dec[key]

    def drain(self):
        if self._qsig:
            keys = list(dict.fromkeys(self._qsig))
            self._qsig = []
            hs = list(dict.fromkeys(k[1] for k in keys))
            hidx = {h: i for i, h in enumerate(hs)}
            v = self.eng.verify_sig_shares([k[0] for k in keys], [k[2] for k in keys], hs, [hidx[k[1]] for k in keys])
            self.calls += 1
            for k, ok in zip(keys, v):
                self._sig[k] = bool(ok)
        if self._qdec:
            keys = list(dict.fromkeys(self._qdec))
            self._qdec = []
            cts = list(dict.fromkeys((k[2], k[3]) for k in keys))
            cidx = {c: i for i, c in enumerate(cts)}
            v = self.eng.verify_dec_shares([k[1] for k in keys], [k[0] for k in keys], [c[0] for c in cts],
                                           [c[1] for c in cts], [cidx[(k[2], k[3])] for k in keys])
            self.calls += 1
            for k, ok in zip(keys, v):
                self._dec[k] = bool(ok)


# ------------------------------------------------------------------ ThresholdSign (src/threshold_sign.rs)
class ThresholdSign:
    def __init__(self, netinfo, verifier):
        self.netinfo = netinfo
        self.verifier = verifier
        self.doc_hash = None
        self.received_shares = {}  # node_id -> (idx, share); BTreeMap order = sorted ids
        self.had_input = False
        self.terminated = False

    def set_document_hash(self, h):
        """``set_document`` (:147) with ``hash_g2(doc)`` computed by the caller (host hashing)."""
        if self.doc_hash is not None:
            raise ProtocolError("MultipleMessagesToSign")
        self.doc_hash = bytes(h)

    def handle_input(self):
        return self.sign()

    def sign(self):  # :157-178
        if self.had_input:
            return Step()
        if self.doc_hash is None:
            raise ProtocolError("DocumentHashIsNone")
        self.had_input = True
        step = Step()
        step.fault_log += self.remove_invalid_shares()
        if not self.netinfo.is_validator():
            return step.join(self.try_output())
        share = self.netinfo.sign_g2(self.doc_hash)
        step.messages.append(("all", share))
        return step.extend(self.handle_message(self.netinfo.our_id, share))

    def handle_message(self, sender_id, share):  # :181-197
        if self.terminated:
            return Step()
        idx = self.netinfo.node_index(sender_id)
        if idx is None:
            raise ProtocolError("UnknownSender")
        if not self.is_share_valid(sender_id, share):
            return Step.fault(sender_id, "UnverifiedSignatureShareSender")
        self.received_shares[sender_id] = (idx, bytes(share))
        return self.try_output()

    def remove_invalid_shares(self):  # :200-213 -- the natural batch point: one drain
        for sid, (_, share) in self.received_shares.items():
            pk = self.netinfo.public_key_share(sid)
            if self.doc_hash is not None and pk is not None:
                self.verifier.queue_sig(pk, self.doc_hash, share)
        self.verifier.drain()
        faulty = [sid for sid, (_, share) in sorted(self.received_shares.items())
                  if not self.is_share_valid(sid, share)]
        for sid in faulty:
            del self.received_shares[sid]
        return [Fault(sid, "UnverifiedSignatureShareSender") for sid in faulty]

    def is_share_valid(self, sender_id, share):  # :216-225
        if self.doc_hash is None:
            return True
        pk = self.netinfo.public_key_share(sender_id)
        if pk is None:
            return False
        return self.verifier.sig_valid(pk, self.doc_hash, share)

    def try_output(self):  # :227-247
        if self.doc_hash is None:
            return Step()
        if not self.terminated and len(self.received_shares) > self.netinfo.num_faulty():
            sig = self.combine_and_verify_sig()
            self.terminated = True
            step = self.sign()
            return step.with_output(sig)
        return Step()

    def combine_and_verify_sig(self):  # :249-270
        t = self.netinfo.num_faulty()
        items = [self.received_shares[k] for k in sorted(self.received_shares)][: t + 1]
        out, st, v = self.verifier.eng.combine_verify_g2(t, [[i for i, _ in items]], [[s for _, s in items]],
                                                         self.netinfo.master_pk, [self.doc_hash])
        if st[0] != 0:
            raise ProtocolError("CombineAndVerifySigCrypto", "DuplicateEntry")
        if not v[0]:
            raise ProtocolError("VerificationFailed")
        return out[0]


# ------------------------------------------------------------------ ThresholdDecrypt (src/threshold_decrypt.rs)
def _chacha_block(key_words, counter):
    def rotl(v, c):
        return ((v << c) & 0xFFFFFFFF) | (v >> (32 - c))
    s = [0x61707865, 0x3320646E, 0x79622D32, 0x6B206574] + list(key_words) + [counter & 0xFFFFFFFF, counter >> 32, 0, 0]
    x = list(s)
    for _ in range(10):
        for a, b, c, d in ((0, 4, 8, 12), (1, 5, 9, 13), (2, 6, 10, 14), (3, 7, 11, 15),
                           (0, 5, 10, 15), (1, 6, 11, 12), (2, 7, 8, 13), (3, 4, 9, 14)):
            x[a] = (x[a] + x[b]) & 0xFFFFFFFF
            x[d] = rotl(x[d] ^ x[a], 16)
            x[c] = (x[c] + x[d]) & 0xFFFFFFFF
            x[b] = rotl(x[b] ^ x[c], 12)
            x[a] = (x[a] + x[b]) & 0xFFFFFFFF
            x[d] = rotl(x[d] ^ x[a], 8)
            x[c] = (x[c] + x[d]) & 0xFFFFFFFF
            x[b] = rotl(x[b] ^ x[c], 7)
    return [(x[i] + s[i]) & 0xFFFFFFFF for i in range(16)]


def g1_compress_abi(p):
    """ABI G1 bytes -> the 48-byte compressed encoding (zcash flags)."""
    p = bytes(p)
    if not any(p):
        return bytes([0xC0]) + bytes(47)
    x = int.from_bytes(p[:48], "little")
    y = int.from_bytes(p[48:], "little")
    out = bytearray(x.to_bytes(48, "big"))
    out[0] |= 0x80 | (0x20 if y > (P_FIELD - y) % P_FIELD else 0)
    return bytes(out)


def xor_with_hash(g1_abi, data):
    """threshold_crypto ``xor_with_hash(g, V)``: V xor the low bytes of successive ChaCha20 words
    keyed by SHA3-256(compress(g)).  Host-side, as in the reference."""
    key = struct.unpack("<8I", hashlib.sha3_256(g1_compress_abi(g1_abi)).digest())
    out, block, words, ctr = bytearray(), [], 0, 0
    for b in bytes(data):
        if words == len(block):
            block, words, ctr = _chacha_block(key, ctr), 0, ctr + 1
        out.append(b ^ (block[words] & 0xFF))
        words += 1
    return bytes(out)


class Ciphertext:
    """(U in G1, V bytes, W in G2) plus H_uv = hash_g1_g2(U, V), hashed once on the host."""

    def __init__(self, u, v, w, huv):
        self.u, self.v, self.w, self.huv = bytes(u), bytes(v), bytes(w), bytes(huv)


class ThresholdDecrypt:
    def __init__(self, netinfo, verifier):
        self.netinfo = netinfo
        self.verifier = verifier
        self.ciphertext = None
        self.shares = {}
        self.had_input = False
        self.terminated = False

    def set_ciphertext(self, ct):  # :138-147
        if self.ciphertext is not None:
            raise ProtocolError("MultipleInputs")
        if not self.verifier.eng.verify_ciphertexts([ct.u], [ct.w], [ct.huv])[0]:
            raise ProtocolError("InvalidCiphertext")
        self.ciphertext = ct

    def handle_input(self):
        return self.start_decryption()

    def start_decryption(self):  # :151-170
        if self.had_input:
            return Step()
        if self.ciphertext is None:
            raise ProtocolError("CiphertextIsNone")
        self.had_input = True
        step = Step()
        step.fault_log += self.remove_invalid_shares()
        if self.netinfo.decrypt_share is None:
            return step.join(self.try_output())
        share = self.netinfo.decrypt_share(self.ciphertext.u)
        our = self.netinfo.our_id
        self.shares[our] = (self.netinfo.node_index(our), bytes(share))  # own share: not verified (:167)
        step.messages.append(("all", share))
        return step.join(self.try_output())

    def handle_message(self, sender_id, share):  # :182-201
        if self.terminated:
            return Step()
        idx = self.netinfo.node_index(sender_id)
        if idx is None:
            raise ProtocolError("UnknownSender")
        if not self.is_share_valid(sender_id, share):
            return Step.fault(sender_id, "UnverifiedDecryptionShareSender")
        dup = sender_id in self.shares
        self.shares[sender_id] = (idx, bytes(share))
        if dup:
            return Step.fault(sender_id, "MultipleDecryptionShares")
        return self.try_output()

    def remove_invalid_shares(self):  # :204-217 -- one drain for every share received early
        ct = self.ciphertext
        for sid, (_, share) in self.shares.items():
            pk = self.netinfo.public_key_share(sid)
            if ct is not None and pk is not None:
                self.verifier.queue_dec(pk, share, ct.huv, ct.w)
        self.verifier.drain()
        faulty = [sid for sid, (_, share) in sorted(self.shares.items()) if not self.is_share_valid(sid, share)]
        for sid in faulty:
            del self.shares[sid]
        return [Fault(sid, "UnverifiedDecryptionShareSender") for sid in faulty]

    def is_share_valid(self, sender_id, share):  # :220-229
        ct = self.ciphertext
        if ct is None:
            return True
        pk = self.netinfo.public_key_share(sender_id)
        if pk is None:
            return False
        return self.verifier.dec_valid(pk, share, ct.huv, ct.w)

    def try_output(self):  # :232-252
        if self.terminated or len(self.shares) <= self.netinfo.num_faulty():
            return Step()
        if self.ciphertext is None:
            return Step()
        self.terminated = True
        step = self.start_decryption()
        t = self.netinfo.num_faulty()
        items = [self.shares[k] for k in sorted(self.shares)][: t + 1]
        out, st = self.verifier.eng.interpolate_g1(t, [[i for i, _ in items]], [[s for _, s in items]])
        if st[0] != 0:
            raise ProtocolError("Decryption", "DuplicateEntry")
        return step.with_output(xor_with_hash(out[0], self.ciphertext.v))


__all__ = ["Fault", "Step", "ProtocolError", "NetworkInfo", "BatchVerifier", "ThresholdSign",
           "ThresholdDecrypt", "Ciphertext", "xor_with_hash", "g1_compress_abi", "G1_BYTES", "G2_BYTES"]
