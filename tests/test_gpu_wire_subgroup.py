"""Device point decoding (k_g1_decompress / k_g2_decompress, round 6: norm-method square root,
endomorphism subgroup tests) against the oracle's decoding with the definition r * P == O
(pairing 0.14 into_affine): 1,000 random on-curve points per group (both y signs;
almost all outside the subgroup), points of every prime order dividing the cofactors (alone and
plus a subgroup point), the cofactor parts [r] Q, and subgroup points.  Accept / reject and the
decoded bytes must be identical; the same through the _dev entry points."""
import numpy as np
import pytest
import torch

from oracle import bls12_381 as C
from oracle import cbls
from hbbft_amd.engine import g1_abi_from_uncompressed as g1a, g2_abi_from_uncompressed as g2a
from tests import subgroup_points as S

pytestmark = pytest.mark.gpu


def c_in_g1(pt):
    return cbls.g1_mul(g1a(C.g1_uncompressed(pt)), C.R) == bytes(96)


def c_in_g2(pt):
    return cbls.g2_mul(g2a(C.g2_uncompressed(pt)), C.R) == bytes(192)


def oracle_decode(g2, encs):
    dec = C.g2_decompress if g2 else C.g1_decompress
    chk = c_in_g2 if g2 else c_in_g1
    unc, abi, size = (C.g2_uncompressed, g2a, 192) if g2 else (C.g1_uncompressed, g1a, 96)
    pts, ok = [], []
    for e in encs:
        try:
            pt = dec(e, in_subgroup=chk)
            pts.append(bytes(size) if pt is None else abi(unc(pt)))
            ok.append(1)
        except C.DecodeError:
            pts.append(bytes(size))
            ok.append(0)
    return pts, ok


@pytest.mark.parametrize("g2", [False, True], ids=["G1", "G2"])
def test_decode_subgroup_matches_r_mul(engine, g2):
    sample = S.sample(g2, 1000, seed=700 + g2)
    comp = C.g2_compress if g2 else C.g1_compress
    encs = [comp(pt) for _, pt in sample]
    want_pts, want_ok = oracle_decode(g2, encs)
    got_pts, got_ok = (engine.g2_decompress if g2 else engine.g1_decompress)(encs)
    labels = [lab for lab, _ in sample]
    bad = [labels[i] for i in range(len(encs)) if got_ok[i] != want_ok[i]]
    assert not bad, bad[:10]
    assert got_pts == want_pts
    # the oracle itself: exactly the subgroup points decode
    assert want_ok == [int(lab == "subgroup") for lab in labels]
    assert sum(lab.startswith("order|") for lab in labels) >= (8 if g2 else 10)


@pytest.mark.parametrize("g2", [False, True], ids=["G1", "G2"])
def test_decode_subgroup_dev_entry(engine, g2):
    """The device-resident entry point (encodings already in HBM) gives the same verdicts."""
    sample = S.sample(g2, 64, seed=710 + g2)
    comp = C.g2_compress if g2 else C.g1_compress
    encs = [comp(pt) for _, pt in sample]
    want_pts, want_ok = oracle_decode(g2, encs)
    size, n = (96, 192) if g2 else (48, 96)
    d_in = torch.from_numpy(np.frombuffer(b"".join(encs), dtype=np.uint8).copy()).to("cuda:0")
    d_out = torch.zeros(len(encs) * n, dtype=torch.uint8, device="cuda:0")
    d_ok = torch.zeros(len(encs), dtype=torch.uint8, device="cuda:0")
    (engine.g2_decompress_dev if g2 else engine.g1_decompress_dev)(None, len(encs), d_in.data_ptr(), d_out.data_ptr(),
                                                                   d_ok.data_ptr())
    torch.cuda.synchronize()
    assert list(d_ok.cpu().numpy()) == want_ok
    got = d_out.cpu().numpy().tobytes()
    assert [got[i * n:(i + 1) * n] for i in range(len(encs))] == want_pts
