"""Batched bincode message decoding for the crypto messages on the hot path.

A node receives its threshold-crypto inputs as bincode bytes (bincode 1.x, hbbft's
``Cargo.toml:24``):

  threshold_sign::Message(SignatureShare)        src/threshold_sign.rs:73
  threshold_decrypt::Message(DecryptionShare)    src/threshold_decrypt.rs:65
  Ciphertext (a Subset contribution)             src/honey_badger/epoch_state.rs:377-381
  Part(BivarCommitment, Vec<Ciphertext>)         src/sync_key_gen.rs:225
  Ack(u64, Vec<Ciphertext>)                      src/sync_key_gen.rs:242

This module turns a WINDOW of such messages into ABI points with one host framing pass and one
batched GPU decompression per group (``hbh_g1_decompress`` / ``hbh_g2_decompress``: on-curve and
subgroup checks, the contract of threshold_crypto's ``into_affine``), instead of one
deserialisation per message.  A message that does not decode yields ``None`` -- the reference's
``bincode::deserialize`` error (``FaultKind::DeserializeCiphertext`` for a contribution,
epoch_state.rs:377-381; a transport-level drop for the others).

Encoding (threshold_crypto 0.3 ``serde_impl``, restated; no pinned vectors exist):
a group element is serialised through ``into_compressed().as_ref()`` as a byte sequence, i.e. a
u64 LE length (48 for G1, 96 for G2) followed by the zcash compressed encoding; ``Vec<T>`` is a
u64 LE count followed by the elements; ``Vec<u8>`` a u64 LE length and the bytes; a newtype
(``Message(share)``) is its field; ``usize`` / ``u64`` are 8 bytes LE.  bincode 1.x's
``deserialize`` reads what the type needs and ignores trailing bytes.
"""
import struct

from . import hoststage
from ._lib import G1_BYTES, G2_BYTES

G1C, G2C = 48, 96  # compressed sizes


class _Reader:
    __slots__ = ("b", "o")

    def __init__(self, b):
        self.b, self.o = b, 0

    def u64(self):
        if self.o + 8 > len(self.b):
            raise ValueError("truncated")
        v = struct.unpack_from("<Q", self.b, self.o)[0]
        self.o += 8
        return v

    def take(self, n):
        if n > len(self.b) - self.o:
            raise ValueError("truncated")
        v = self.b[self.o:self.o + n]
        self.o += n
        return v

    def point(self, size):
        if self.u64() != size:
            raise ValueError("group element length")
        return self.take(size)


def _u64(v):
    return struct.pack("<Q", v)


# ---------------------------------------------------------------- encoders (host stage compression)
def encode_sig_share_msgs(sigs):
    """bincode(threshold_sign::Message(SignatureShare)) per ABI G2 point."""
    return [_u64(G2C) + c for c in hoststage.g2_compress(list(sigs))] if sigs else []


def encode_dec_share_msgs(shares):
    """bincode(threshold_decrypt::Message(DecryptionShare)) per ABI G1 point."""
    return [_u64(G1C) + c for c in hoststage.g1_compress(list(shares))] if shares else []


def _ct_bytes(u_c, v, w_c):
    return _u64(G1C) + u_c + _u64(len(v)) + bytes(v) + _u64(G2C) + w_c


def encode_ciphertexts(cts):
    """bincode(Ciphertext(U, V, W)) per (u, v, w) of ABI points and bytes."""
    cts = list(cts)
    if not cts:
        return []
    us = hoststage.g1_compress([c[0] for c in cts])
    ws = hoststage.g2_compress([c[2] for c in cts])
    return [_ct_bytes(u, c[1], w) for u, c, w in zip(us, cts, ws)]


def encode_part(degree, commit, rows):
    """bincode(Part(BivarCommitment{degree, commit}, rows)); rows: [(u, v, w)]."""
    cs = hoststage.g1_compress(list(commit)) if commit else []
    out = [_u64(degree), _u64(len(cs))] + [_u64(G1C) + c for c in cs] + [_u64(len(rows))]
    return b"".join(out) + b"".join(encode_ciphertexts(rows))


def encode_ack(proposer_idx, values):
    """bincode(Ack(proposer_idx, values)); values: [(u, v, w)]."""
    return _u64(proposer_idx) + _u64(len(values)) + b"".join(encode_ciphertexts(values))


# ---------------------------------------------------------------- batched decoding
class _Batch:
    """Compressed points gathered from a window of messages; one GPU call per group."""

    def __init__(self):
        self.g1, self.g2 = [], []

    def add_g1(self, enc):
        self.g1.append(bytes(enc))
        return len(self.g1) - 1

    def add_g2(self, enc):
        self.g2.append(bytes(enc))
        return len(self.g2) - 1

    def run(self, engine):
        self.p1, self.ok1 = engine.g1_decompress(self.g1) if self.g1 else ([], b"")
        self.p2, self.ok2 = engine.g2_decompress(self.g2) if self.g2 else ([], b"")

    def get1(self, k):
        return self.p1[k] if self.ok1[k] else None

    def get2(self, k):
        return self.p2[k] if self.ok2[k] else None


def _decode_points(engine, msgs, size, g2):
    b = _Batch()
    slot = []
    for m in msgs:
        try:
            r = _Reader(bytes(m))
            slot.append(b.add_g2(r.point(size)) if g2 else b.add_g1(r.point(size)))
        except ValueError:
            slot.append(None)
    b.run(engine)
    get = b.get2 if g2 else b.get1
    return [None if k is None else get(k) for k in slot]


def decode_sig_share_msgs(engine, msgs):
    """SignatureShare ABI G2 point per message, or None where bincode would fail (framing, a
    non-canonical or off-curve / non-subgroup point)."""
    return _decode_points(engine, msgs, G2C, True)


def decode_dec_share_msgs(engine, msgs):
    """DecryptionShare ABI G1 point per message, or None."""
    return _decode_points(engine, msgs, G1C, False)


def _read_ct(r, b):
    u = b.add_g1(r.point(G1C))
    v = bytes(r.take(r.u64()))
    w = b.add_g2(r.point(G2C))
    return (u, v, w)


def _ct_out(b, ct):
    u, v, w = ct
    pu, pw = b.get1(u), b.get2(w)
    return None if pu is None or pw is None else (pu, v, pw)


def decode_ciphertexts(engine, blobs):
    """(U, V, W) ABI tuple per serialised Ciphertext, or None (FaultKind::DeserializeCiphertext,
    epoch_state.rs:377-381)."""
    b = _Batch()
    plan = []
    for m in blobs:
        try:
            plan.append(_read_ct(_Reader(bytes(m)), b))
        except ValueError:
            plan.append(None)
    b.run(engine)
    return [None if c is None else _ct_out(b, c) for c in plan]


def decode_parts(engine, blobs):
    """(degree, commit, rows) per serialised Part, or None.  The commitment must hold
    (degree+1)(degree+2)/2 points (what BivarPoly::commitment builds; the batched engine calls
    index by it) and every point must decode."""
    b = _Batch()
    plan = []
    for m in blobs:
        try:
            r = _Reader(bytes(m))
            degree = r.u64()
            n = r.u64()
            if degree > 1 << 16 or n != (degree + 1) * (degree + 2) // 2:
                raise ValueError("commitment length")
            commit = [b.add_g1(r.point(G1C)) for _ in range(n)]
            rows = [_read_ct(r, b) for _ in range(r.u64())]
            plan.append((degree, commit, rows))
        except ValueError:
            plan.append(None)
    b.run(engine)
    out = []
    for p in plan:
        if p is None:
            out.append(None)
            continue
        degree, commit, rows = p
        pts = [b.get1(k) for k in commit]
        cts = [_ct_out(b, c) for c in rows]
        out.append(None if any(x is None for x in pts) or any(c is None for c in cts) else (degree, pts, cts))
    return out


def decode_acks(engine, blobs):
    """(proposer_idx, values) per serialised Ack, or None."""
    b = _Batch()
    plan = []
    for m in blobs:
        try:
            r = _Reader(bytes(m))
            proposer = r.u64()
            plan.append((proposer, [_read_ct(r, b) for _ in range(r.u64())]))
        except ValueError:
            plan.append(None)
    b.run(engine)
    out = []
    for p in plan:
        if p is None:
            out.append(None)
            continue
        cts = [_ct_out(b, c) for c in p[1]]
        out.append(None if any(c is None for c in cts) else (p[0], cts))
    return out


__all__ = ["encode_sig_share_msgs", "encode_dec_share_msgs", "encode_ciphertexts", "encode_part", "encode_ack",
           "decode_sig_share_msgs", "decode_dec_share_msgs", "decode_ciphertexts", "decode_parts", "decode_acks",
           "G1_BYTES", "G2_BYTES"]
