"""Device-resident entry points (hbh_*_dev): inputs and outputs in HBM (torch tensors), launched on
a caller stream; byte-identical to the host-pointer calls on the same data, including the error
statuses (duplicate index, 0xffffffff index) and rejected encodings."""
import random

import numpy as np
import pytest
import torch

from oracle import bls12_381 as C
from hbbft_amd.engine import g1_abi_from_uncompressed as g1a, g2_abi_from_uncompressed as g2a

pytestmark = pytest.mark.gpu
R = C.R
G1 = g1a(C.g1_uncompressed(C.G1_GEN))
G2 = g2a(C.g2_uncompressed(C.G2_GEN))


def dev(b, dtype=torch.uint8):
    a = np.frombuffer(bytes(b), dtype=np.uint8).copy()
    t = torch.from_numpy(a).to("cuda:0")
    return t if dtype == torch.uint8 else t.view(dtype)


@pytest.mark.parametrize("g2", [False, True], ids=["g1", "g2"])
def test_interpolate_dev(engine, g2):
    rng = random.Random(5 + g2)
    t, ncomb = 3, 6
    size = 192 if g2 else 96
    base = G2 if g2 else G1
    pts = (engine.g2_mul if g2 else engine.g1_mul)([base] * (ncomb * (t + 1)),
                                                    [rng.randrange(1, R) for _ in range(ncomb * (t + 1))])
    idx = [rng.sample(range(20), t + 1) for _ in range(ncomb)]
    idx[2][1] = idx[2][0]            # duplicate -> HBH_ERR_DUPLICATE_ENTRY
    want_out, want_st = (engine.interpolate_g2 if g2 else engine.interpolate_g1)(t, idx, pts)
    d_idx = dev(np.array([i for row in idx for i in row], dtype=np.uint32).tobytes(), torch.int32)
    d_pts = dev(b"".join(pts))
    d_out = torch.zeros(ncomb * size, dtype=torch.uint8, device="cuda:0")
    d_st = torch.full((ncomb,), -1, dtype=torch.int32, device="cuda:0")
    s = torch.cuda.Stream()
    fn = engine.interpolate_g2_dev if g2 else engine.interpolate_g1_dev
    fn(s.cuda_stream, ncomb, t, d_idx.data_ptr(), d_pts.data_ptr(), d_out.data_ptr(), d_st.data_ptr())
    torch.cuda.synchronize()
    assert d_st.cpu().tolist() == want_st and want_st[2] == 5
    out = bytes(d_out.cpu().numpy())
    for c in range(ncomb):
        if want_st[c] == 0:
            assert out[c * size:(c + 1) * size] == want_out[c]
    # an index of 0xffffffff -> status HBH_ERR_ARG for that combine only
    bad = np.array([i for row in idx for i in row], dtype=np.uint32)
    bad[0] = 0xFFFFFFFF
    d_idx2 = dev(bad.tobytes(), torch.int32)
    fn(None, ncomb, t, d_idx2.data_ptr(), d_pts.data_ptr(), d_out.data_ptr(), d_st.data_ptr())
    torch.cuda.synchronize()
    st = d_st.cpu().tolist()
    assert st[0] == 1 and st[1:] == want_st[1:]


@pytest.mark.parametrize("g2", [False, True], ids=["g1", "g2"])
def test_decompress_dev(engine, g2):
    rng = random.Random(8)
    base = C.G2_GEN if g2 else C.G1_GEN
    mul = C.g2_mul if g2 else C.g1_mul
    comp = C.g2_compress if g2 else C.g1_compress
    encs = [comp(mul(base, rng.randrange(1, R))) for _ in range(5)] + [comp(None)]
    e = bytearray(encs[0])
    e[0] &= 0x7F                      # not compressed -> reject
    encs.append(bytes(e))
    e = bytearray(encs[1])
    e[-1] ^= 1                        # probably off-curve -> reject
    encs.append(bytes(e))
    want_pts, want_ok = (engine.g2_decompress if g2 else engine.g1_decompress)(encs)
    n, esz, psz = len(encs), (96 if g2 else 48), (192 if g2 else 96)
    d_in = dev(b"".join(encs))
    d_out = torch.zeros(n * psz, dtype=torch.uint8, device="cuda:0")
    d_ok = torch.zeros(n, dtype=torch.uint8, device="cuda:0")
    (engine.g2_decompress_dev if g2 else engine.g1_decompress_dev)(None, n, d_in.data_ptr(), d_out.data_ptr(),
                                                                   d_ok.data_ptr())
    torch.cuda.synchronize()
    assert bytes(d_ok.cpu().numpy()) == want_ok
    assert bytes(d_out.cpu().numpy()) == b"".join(want_pts)
    assert want_ok[:6] == b"\x01" * 6 and want_ok[6] == 0


def test_bivar_ack_check_dev(engine):
    rng = random.Random(12)
    t, nparts = 2, 3
    npos = (t + 1) * (t + 2) // 2
    coefs = [rng.randrange(1, R) for _ in range(nparts * npos)]
    flat = engine.g1_mul([G1] * (nparts * npos), coefs)
    parts = [flat[p * npos:(p + 1) * npos] for p in range(nparts)]
    acks = [(p, x, y) for p in range(nparts) for x in (2, 7) for y in range(1, 5)]

    def cp(i, j):
        return j * (j + 1) // 2 + i if i <= j else i * (i + 1) // 2 + j

    def value(p, x, y):  # BivarPoly::evaluate with the symmetric coefficient layout
        return sum(coefs[p * npos + cp(i, j)] * pow(x, i, R) * pow(y, j, R)
                   for i in range(t + 1) for j in range(t + 1)) % R

    vals = [value(*a) if k % 3 else rng.randrange(0, R) for k, a in enumerate(acks)]
    want = engine.bivar_ack_check(t, parts, [a[0] for a in acks], [a[1] for a in acks], [a[2] for a in acks], vals)
    rows = list(dict.fromkeys((p, x) for p, x, _ in acks))
    row_of = [rows.index((p, x)) for p, x, _ in acks]
    u32 = lambda v: dev(np.array(v, dtype=np.uint32).tobytes(), torch.int32)  # noqa: E731
    d_commits = dev(b"".join(flat))
    d_vals = dev(b"".join(v.to_bytes(32, "little") for v in vals))
    d_v = torch.zeros(len(acks), dtype=torch.uint8, device="cuda:0")
    rp, rx, ro, ys = u32([r[0] for r in rows]), u32([r[1] for r in rows]), u32(row_of), u32([a[2] for a in acks])
    engine.bivar_ack_check_dev(None, len(acks), t, d_commits.data_ptr(), len(rows), rp.data_ptr(), rx.data_ptr(),
                               ro.data_ptr(), ys.data_ptr(), d_vals.data_ptr(), d_v.data_ptr())
    torch.cuda.synchronize()
    assert bytes(d_v.cpu().numpy()) == want
    assert want == bytes(1 if k % 3 else 0 for k in range(len(acks)))


def test_g1_mul_gen_fixed_base(engine):
    """hbh_g1_mul_gen (comb table of g1) equals hbh_g1_mul(g1, k) and the C oracle, edge scalars
    included (0 -> infinity, r - 1, r, 2^256 - 1, single-window values)."""
    from oracle import cbls
    rng = random.Random(77)
    ks = [0, 1, 2, 255, 256, 1 << 248, R - 1, R, R + 5, (1 << 256) - 1] + [rng.randrange(0, 1 << 256) for _ in range(500)]
    got = engine.g1_mul_gen(ks)
    assert got == engine.g1_mul([G1] * len(ks), ks)
    assert got[0] == bytes(96) and got[R and 7] == bytes(96)
    for k, g in list(zip(ks, got))[:12]:
        assert g == cbls.g1_mul(G1, k % R)


def _sign_batch(engine, rng, ndocs, per_doc):
    from oracle import tc
    coeffs = [rng.randrange(1, R) for _ in range(3)]
    sks = [tc.poly_eval(coeffs, i + 1) for i in range(per_doc)]
    pks = engine.g1_mul([G1] * per_doc, sks)
    hs = engine.g2_mul([G2] * ndocs, [rng.randrange(1, R) for _ in range(ndocs)])
    n = ndocs * per_doc
    bad = set(rng.sample(range(n), n // 7))
    sigs = engine.g2_mul([hs[i // per_doc] for i in range(n)],
                         [rng.randrange(1, R) if i in bad else sks[i % per_doc] for i in range(n)])
    want = bytes(0 if i in bad else 1 for i in range(n))
    return ([pks[i % per_doc] for i in range(n)], sigs, hs, [i // per_doc for i in range(n)], want)


@pytest.mark.parametrize("impl", [4, 5, 8], ids=["pair", "wave", "wave2"])
def test_dev_calls_on_two_streams(engine, impl):
    """Two hbh_verify_pairing_eq_dev calls queued back-to-back on two different streams:
    the second call's line tables must not overwrite the first call's while its kernels still read
    them -- the engine orders calls with its completion event.  Both verdict arrays are exact."""
    from hbbft_amd._lib import IMPL_AUTO
    rng = random.Random(2024)
    batches = [_sign_batch(engine, rng, 64, 32), _sign_batch(engine, rng, 48, 32)]
    engine.set_pairing_impl(impl)
    try:
        streams = [torch.cuda.Stream(), torch.cuda.Stream()]
        keep, outs = [], []
        torch.cuda.synchronize()
        for (pks, sigs, hs, di, want), s in zip(batches, streams):
            d_pk, d_sg, d_h = dev(b"".join(pks)), dev(b"".join(sigs)), dev(b"".join(hs))
            d_di = dev(np.array(di, dtype=np.uint32).tobytes(), torch.int32)
            d_v = torch.zeros(len(want), dtype=torch.uint8, device="cuda:0")
            engine.verify_pairing_eq_dev(s.cuda_stream, len(want), d_pk.data_ptr(), d_h.data_ptr(), len(hs),
                                         d_di.data_ptr(), None, d_sg.data_ptr(), len(want), None, d_v.data_ptr())
            keep += [d_pk, d_sg, d_h, d_di]
            outs.append((d_v, want))
        torch.cuda.synchronize()
        for d_v, want in outs:
            assert bytes(d_v.cpu().numpy()) == want
    finally:
        engine.set_pairing_impl(IMPL_AUTO)


@pytest.mark.parametrize("impl", [4, 5, 6, 7, 8], ids=["pair", "wave", "quad", "oct", "wave2"])
def test_dev_index_out_of_range_rejects(engine, impl):
    """HBH_IMPL_PAIR, HBH_IMPL_WAVE, HBH_IMPL_QUAD, HBH_IMPL_OCT and HBH_IMPL_WAVE2 validate device index arrays in-kernel: an index >= its table
    size gives verdict 0 for that item only (never a read past the table)."""
    from hbbft_amd._lib import IMPL_AUTO
    rng = random.Random(9)
    pks, sigs, hs, di, want = _sign_batch(engine, rng, 8, 16)
    di = list(di)
    di[5] = 8          # == table size
    di[77] = 1 << 30   # far out of range
    engine.set_pairing_impl(impl)
    try:
        d_pk, d_sg, d_h = dev(b"".join(pks)), dev(b"".join(sigs)), dev(b"".join(hs))
        d_di = dev(np.array(di, dtype=np.uint32).tobytes(), torch.int32)
        d_v = torch.full((len(want),), 7, dtype=torch.uint8, device="cuda:0")
        engine.verify_pairing_eq_dev(None, len(want), d_pk.data_ptr(), d_h.data_ptr(), len(hs), d_di.data_ptr(),
                                     None, d_sg.data_ptr(), len(want), None, d_v.data_ptr())
        torch.cuda.synchronize()
        got = bytes(d_v.cpu().numpy())
    finally:
        engine.set_pairing_impl(IMPL_AUTO)
    exp = bytearray(want)
    exp[5] = exp[77] = 0
    assert got == bytes(exp)
