"""Host-side pieces of the protocol mirror (no GPU): the XOR stream of PublicKeySet::decrypt and
the compressed G1 encoding it hashes, against the oracle; Step/fault plumbing."""
from oracle import bls12_381 as C
from oracle import tc
from hbbft_amd.engine import g1_abi_from_uncompressed as g1a
from hbbft_amd.protocol import Fault, Step, g1_compress_abi, xor_with_hash


def test_compress_and_xor_stream_match_oracle():
    for k in (1, 5, 12345, C.R - 1):
        p = C.g1_mul(C.G1_GEN, k)
        assert g1_compress_abi(g1a(C.g1_uncompressed(p))) == C.g1_compress(p)
        for n in (0, 1, 63, 64, 65, 200):  # across ChaCha block boundaries
            data = bytes((i * 7) & 0xFF for i in range(n))
            assert xor_with_hash(g1a(C.g1_uncompressed(p)), data) == tc.xor_with_hash(p, data)
    assert g1_compress_abi(bytes(96)) == C.g1_compress(None)


def test_step_join():
    a = Step.fault(3, "UnverifiedSignatureShareSender")
    b = Step(output=["sig"], messages=[("all", b"x")])
    a.join(b)
    assert a.output == ["sig"] and a.messages == [("all", b"x")]
    assert a.fault_log == [Fault(3, "UnverifiedSignatureShareSender")]
