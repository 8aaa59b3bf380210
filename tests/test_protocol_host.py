"""Host-side pieces of the protocol mirror (no GPU): the XOR stream of PublicKeySet::decrypt and
the compressed G1 encoding it hashes, against the oracle; Step/fault plumbing."""
from oracle import bls12_381 as C
from oracle import tc
from hbbft_amd.engine import g1_abi_from_uncompressed as g1a
from hbbft_amd.protocol import Fault, Step, g1_compress_abi, xor_with_hash
import hbbft_amd.sync_key_gen as skg
import pytest


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


def test_uncompressed_flag_and_field_checks():
    """g1/g2_abi_from_uncompressed reject what pairing 0.14's into_affine_unchecked rejects."""
    import pytest
    from hbbft_amd.engine import P_FIELD, g1_abi_from_uncompressed, g2_abi_from_uncompressed
    from oracle import bls12_381 as C
    g1 = C.g1_uncompressed(C.G1_GEN)
    g2 = C.g2_uncompressed(C.G2_GEN)
    assert g1_abi_from_uncompressed(g1)[:48] == C.G1_GEN[0].to_bytes(48, "little")
    assert g1_abi_from_uncompressed(bytes([0x40]) + bytes(95)) == bytes(96)
    assert g2_abi_from_uncompressed(bytes([0x40]) + bytes(191)) == bytes(192)
    for bad in (bytes([g1[0] | 0x80]) + g1[1:], bytes([g1[0] | 0x20]) + g1[1:], bytes([0x40]) + bytes(94) + b"\x01",
                P_FIELD.to_bytes(48, "big") + g1[48:], b"\x00" * 95):
        with pytest.raises(ValueError):
            g1_abi_from_uncompressed(bad)
    with pytest.raises(ValueError):
        g2_abi_from_uncompressed(g2[:96] + P_FIELD.to_bytes(48, "big") + g2[144:])


def test_malformed_commitment_rejected():
    """A BivarCommitment whose point count does not match its degree cannot be built (it would
    misalign every other part of a batched engine call)."""
    with pytest.raises(ValueError):
        skg.Part(2, [bytes(96)] * 5, [])
    with pytest.raises(ValueError):
        skg.Part(1, [bytes(96)] * 4, [])
