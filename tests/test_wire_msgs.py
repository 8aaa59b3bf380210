"""bincode message framing of hbbft_amd.wire on the CPU.  Encodings are built by
the product host stage (hoststage compression) and checked byte for byte against the oracle's
compressed encodings plus the bincode framing; decoding runs the framing parser with a stand-in
decompressor backed by the oracle (the GPU decompression itself is covered by
tests/test_gpu_wire_msgs.py and tests/test_gpu_curve.py).  Vectors: parity unpinned (no bincode
vectors exist in the reference)."""
import random
import struct

from oracle import bls12_381 as C
from hbbft_amd import wire
from hbbft_amd.engine import g1_abi_from_uncompressed as g1a, g2_abi_from_uncompressed as g2a


class OracleDecompressor:
    """engine.g1_decompress / g2_decompress semantics (points, ok bytes) from the oracle."""

    @staticmethod
    def _dec(fn, unc, conv, size, encs):
        pts, ok = [], []
        for e in encs:
            try:
                p = fn(e)
                pts.append(bytes(size) if p is None else conv(unc(p)))
                ok.append(1)
            except C.DecodeError:
                pts.append(bytes(size))
                ok.append(0)
        return pts, bytes(ok)

    def g1_decompress(self, encs):
        return self._dec(C.g1_decompress, C.g1_uncompressed, g1a, 96, encs)

    def g2_decompress(self, encs):
        return self._dec(C.g2_decompress, C.g2_uncompressed, g2a, 192, encs)


def _pts(rng, n):
    p1 = [C.g1_mul(C.G1_GEN, rng.randrange(1, C.R)) for _ in range(n)] + [None]
    p2 = [C.g2_mul(C.G2_GEN, rng.randrange(1, C.R)) for _ in range(2)] + [None]
    return p1, p2


def test_share_messages_framing_and_round_trip():
    rng = random.Random(5)
    p1, p2 = _pts(rng, 3)
    a1 = [bytes(96) if p is None else g1a(C.g1_uncompressed(p)) for p in p1]
    a2 = [bytes(192) if p is None else g2a(C.g2_uncompressed(p)) for p in p2]
    m1 = wire.encode_dec_share_msgs(a1)
    m2 = wire.encode_sig_share_msgs(a2)
    assert m1 == [struct.pack("<Q", 48) + C.g1_compress(p) for p in p1]
    assert m2 == [struct.pack("<Q", 96) + C.g2_compress(p) for p in p2]
    eng = OracleDecompressor()
    assert wire.decode_dec_share_msgs(eng, m1) == a1
    assert wire.decode_sig_share_msgs(eng, m2) == a2
    # framing errors: truncated, wrong length prefix, empty; trailing bytes are ignored (bincode 1.x)
    bad = [m2[0][:-1], struct.pack("<Q", 95) + m2[0][8:], b"", m2[0] + b"\x00\x01"]
    assert wire.decode_sig_share_msgs(eng, bad) == [None, None, None, a2[0]]
    # a G1 message where a G2 one is expected, and a point that is not on the curve
    off = bytearray(m1[0])
    off[-1] ^= 1
    got = wire.decode_dec_share_msgs(eng, [bytes(off)])
    want = None
    try:
        want = g1a(C.g1_uncompressed(C.g1_decompress(bytes(off[8:]))))
    except C.DecodeError:
        pass
    assert got == [want]
    assert wire.decode_sig_share_msgs(eng, [m1[0]]) == [None]


def test_ciphertext_part_ack_round_trip():
    rng = random.Random(6)
    p1, p2 = _pts(rng, 7)
    u = [g1a(C.g1_uncompressed(p)) for p in p1[:3]]
    w = [g2a(C.g2_uncompressed(p)) for p in p2[:2]] + [bytes(192)]
    cts = [(u[0], b"", w[0]), (u[1], bytes(range(70)), w[1]), (u[2], b"\x05" * 3, w[2])]
    eng = OracleDecompressor()
    blobs = wire.encode_ciphertexts(cts)
    assert blobs[1] == (struct.pack("<Q", 48) + C.g1_compress(p1[1]) + struct.pack("<Q", 70) + bytes(range(70))
                        + struct.pack("<Q", 96) + C.g2_compress(p2[1]))
    assert wire.decode_ciphertexts(eng, blobs) == cts
    assert wire.decode_ciphertexts(eng, [blobs[1][:60], blobs[0][:-3]]) == [None, None]
    # Part: degree 1 -> 3 commitment points; Ack
    commit = [g1a(C.g1_uncompressed(p)) for p in p1[3:6]]
    part = wire.encode_part(1, commit, cts)
    assert wire.decode_parts(eng, [part]) == [(1, commit, cts)]
    short = wire.encode_part(1, commit[:2], cts)                 # 2 points for degree 1
    assert wire.decode_parts(eng, [short, part[:-1]]) == [None, None]
    ack = wire.encode_ack(4, cts[:2])
    assert wire.decode_acks(eng, [ack, ack[:20]]) == [(4, cts[:2]), None]
