"""Host stage of the path over the C ABI (include/hbbft_hip.h "host stage"): what the north star
keeps on the CPU -- hashing to G2, the XOR stream, the coin parity, point compression and the
secret-key scalar multiplications -- batched and multithreaded in C++ (csrc/host_hash.cpp).
No GPU is needed for any of these.  Points use the ABI format (affine, little-endian canonical;
infinity = all zero bytes), scalars are Python ints < 2^256."""
import ctypes

import numpy as np

from . import _lib
from ._lib import G1_BYTES, G2_BYTES, check_host


def _concat(items):
    items = [bytes(x) for x in items]
    offs = np.zeros(len(items) + 1, dtype=np.uint64)
    if items:
        offs[1:] = np.cumsum([len(x) for x in items], dtype=np.uint64)
    data = b"".join(items)
    return data, offs


def _buf(b):
    cb = (ctypes.c_uint8 * max(len(b), 1)).from_buffer_copy(bytes(b) or b"\0")
    return cb, ctypes.cast(cb, ctypes.c_void_p)


def _out(n):
    o = (ctypes.c_uint8 * max(n, 1))()
    return o, ctypes.cast(o, ctypes.c_void_p)


def _split(raw, size, n):
    return [raw[i * size:(i + 1) * size] for i in range(n)]


def hash_g2(msgs, threads=0):
    """threshold_crypto hash_g2 per message (src/threshold_sign.rs:151) -> ABI G2 points."""
    l = _lib.lib()
    data, offs = _concat(msgs)
    n = len(msgs)
    keep, pd = _buf(data)
    o, po = _out(n * G2_BYTES)
    check_host(l.hbh_hash_g2(n, pd, offs.ctypes.data_as(ctypes.c_void_p), po, int(threads)))
    return _split(bytes(o), G2_BYTES, n)


def hash_g1_g2(us, vs, threads=0):
    """hash_g1_g2(U, V) per ciphertext (H_uv of src/threshold_decrypt.rs:142,227)."""
    l = _lib.lib()
    n = len(us)
    if len(vs) != n:
        raise ValueError("us / vs length mismatch")
    data, offs = _concat(vs)
    ku, pu = _buf(b"".join(bytes(u) for u in us))
    kd, pd = _buf(data)
    o, po = _out(n * G2_BYTES)
    check_host(l.hbh_hash_g1_g2(n, pu, pd, offs.ctypes.data_as(ctypes.c_void_p), po, int(threads)))
    return _split(bytes(o), G2_BYTES, n)


def hash_g1_g2_bp(us, vs, threads=0):
    """Q_i with hash_g1_g2(U_i, V_i) = [KCOF] Q_i (hbh_hash_g1_g2_bp): Ciphertext::verify is then
    e(hash_bp_g1(), W) == e(U, Q) (hbh_verify_pairing_eq), one G2 scalar multiplication less per
    ciphertext than hash_g1_g2."""
    l = _lib.lib()
    n = len(us)
    if len(vs) != n:
        raise ValueError("us / vs length mismatch")
    data, offs = _concat(vs)
    ku, pu = _buf(b"".join(bytes(u) for u in us))
    kd, pd = _buf(data)
    o, po = _out(n * G2_BYTES)
    check_host(l.hbh_hash_g1_g2_bp(n, pu, pd, offs.ctypes.data_as(ctypes.c_void_p), po, int(threads)))
    return _split(bytes(o), G2_BYTES, n)


_BP_G1 = None


def hash_bp_g1():
    """G1K = [KCOF^-1 mod r] g1, the P1 of the Q-form Ciphertext::verify (hbh_hash_bp_g1)."""
    global _BP_G1
    if _BP_G1 is None:
        o, po = _out(G1_BYTES)
        check_host(_lib.lib().hbh_hash_bp_g1(po))
        _BP_G1 = bytes(o)
    return _BP_G1


def xor_with_hash(gs, datas, threads=0):
    """V xor stream(g) per item (PublicKeySet::decrypt's last step, SecretKey::decrypt)."""
    l = _lib.lib()
    n = len(gs)
    data, offs = _concat(datas)
    kg, pg = _buf(b"".join(bytes(g) for g in gs))
    kd, pd = _buf(data)
    o, po = _out(len(data))
    check_host(l.hbh_xor_with_hash(n, pg, pd, offs.ctypes.data_as(ctypes.c_void_p), po, int(threads)))
    raw = bytes(o)[:len(data)]
    return [raw[int(offs[i]):int(offs[i + 1])] for i in range(n)]


def host_threads():
    """Workers the host stage uses for threads=0: the CPUs this process may use (affinity,
    cgroup cpu.max quota, HBH_HOST_THREADS / OMP_NUM_THREADS; hbh_host_threads)."""
    n = ctypes.c_int()
    check_host(_lib.lib().hbh_host_threads(ctypes.byref(n)))
    return n.value


def signature_parity(sigs):
    """Signature::parity per G2 point (the BA coin value, binary_agreement.rs:402)."""
    l = _lib.lib()
    n = len(sigs)
    ks, ps = _buf(b"".join(bytes(s) for s in sigs))
    o, po = _out(n)
    check_host(l.hbh_signature_parity(n, ps, po))
    return [bool(b) for b in bytes(o)[:n]]


def g1_compress(pts):
    l = _lib.lib()
    n = len(pts)
    k, p = _buf(b"".join(bytes(x) for x in pts))
    o, po = _out(n * 48)
    check_host(l.hbh_g1_compress(n, p, po))
    return _split(bytes(o), 48, n)


def g2_compress(pts):
    l = _lib.lib()
    n = len(pts)
    k, p = _buf(b"".join(bytes(x) for x in pts))
    o, po = _out(n * 96)
    check_host(l.hbh_g2_compress(n, p, po))
    return _split(bytes(o), 96, n)


def _mul(fn, size, pts, scalars, threads):
    n = len(pts)
    if len(scalars) != n:
        raise ValueError("points / scalars length mismatch")
    kp, pp = _buf(b"".join(bytes(x) for x in pts))
    ks, ps = _buf(b"".join(int(k).to_bytes(32, "little") for k in scalars))
    o, po = _out(n * size)
    check_host(fn(n, pp, ps, po, int(threads)))
    return _split(bytes(o), size, n)


def g1_mul(pts, scalars, threads=0):
    """Secret-scalar G1 multiplication on the host (decrypt_share_no_verify, SecretKey::decrypt)."""
    return _mul(_lib.lib().hbh_host_g1_mul, G1_BYTES, pts, scalars, threads)


def g2_mul(pts, scalars, threads=0):
    """Secret-scalar G2 multiplication on the host (SecretKeyShare::sign_g2)."""
    return _mul(_lib.lib().hbh_host_g2_mul, G2_BYTES, pts, scalars, threads)


def g1_add(a, b):
    """a[i] + b[i] for public G1 points."""
    l = _lib.lib()
    n = len(a)
    if len(b) != n:
        raise ValueError("length mismatch")
    ka, pa = _buf(b"".join(bytes(x) for x in a))
    kb, pb = _buf(b"".join(bytes(x) for x in b))
    o, po = _out(n * G1_BYTES)
    check_host(l.hbh_host_g1_add(n, pa, pb, po))
    return _split(bytes(o), G1_BYTES, n)


def encrypt(pks, msgs, nonces, threads=0):
    """PublicKey::encrypt_with_rng per message with caller-drawn nonces: [(U, V, W)].  pks: one
    key for all messages, or one per message."""
    l = _lib.lib()
    n = len(msgs)
    if len(nonces) != n:
        raise ValueError("msgs / nonces length mismatch")
    per_item = len(pks) != 1
    if per_item and len(pks) != n:
        raise ValueError("pks must hold one key or one per message")
    data, offs = _concat(msgs)
    kk, pk = _buf(b"".join(bytes(x) for x in pks))
    kd, pd = _buf(data)
    kn, pn = _buf(b"".join(int(r).to_bytes(32, "little") for r in nonces))
    ou, pu = _out(n * G1_BYTES)
    ov, pv = _out(len(data))
    ow, pw = _out(n * G2_BYTES)
    check_host(l.hbh_encrypt(n, pk, 1 if per_item else 0, pd, offs.ctypes.data_as(ctypes.c_void_p), pn, pu, pv, pw,
                             int(threads)))
    raw_v = bytes(ov)[:len(data)]
    us, ws = _split(bytes(ou), G1_BYTES, n), _split(bytes(ow), G2_BYTES, n)
    return [(us[i], raw_v[int(offs[i]):int(offs[i + 1])], ws[i]) for i in range(n)]


def fr_poly_eval(polys, xs, threads=0):
    """Poly::evaluate over Fr (hbh_fr_poly_eval): [[poly(x) for x in xs] for poly in polys]; every
    polynomial is a coefficient list (constant term first) of one common length, coefficients < r."""
    npoly = len(polys)
    if npoly == 0 or not xs:
        return [[] for _ in polys]
    ncoef = len(polys[0])
    if any(len(c) != ncoef for c in polys):
        raise ValueError("polynomials of different lengths")
    kc, pc = _buf(b"".join(int(c).to_bytes(32, "little") for poly in polys for c in poly))
    xa = np.asarray([int(x) for x in xs], dtype=np.uint64)
    o, po = _out(npoly * len(xa) * 32)
    check_host(_lib.lib().hbh_fr_poly_eval(npoly, ncoef, pc, len(xa), xa.ctypes.data_as(ctypes.c_void_p), po,
                                           int(threads)))
    raw = bytes(o)
    m = len(xa)
    return [[int.from_bytes(raw[32 * (q * m + k):32 * (q * m + k + 1)], "little") for k in range(m)]
            for q in range(npoly)]
