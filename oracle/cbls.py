"""ctypes binding of the C oracle (oracle/c/bls_cpu.c -> oracle/build/libbls_cpu.so).

TEST INFRASTRUCTURE ONLY: imported by tests/ and by bench.py's cpu_baseline leg, never by the
product path.  Same point/scalar formats as include/hbbft_hip.h.
"""
import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "build", "libbls_cpu.so")
_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError("oracle/build/libbls_cpu.so not built (make -C oracle)")
        l = ctypes.CDLL(LIB_PATH)
        P, I, SZ, U64 = ctypes.c_char_p, ctypes.c_int, ctypes.c_size_t, ctypes.c_uint64
        vp = ctypes.c_void_p
        l.bls_verify_g2.argtypes = [P, P, P]
        l.bls_verify_g2.restype = I
        l.bls_pairing_eq.argtypes = [P, P, P, P]
        l.bls_pairing_eq.restype = I
        l.bls_pairing.argtypes = [P, P, vp]
        l.bls_g1_mul.argtypes = [P, P, vp]
        l.bls_g2_mul.argtypes = [P, P, vp]
        l.bls_g2_clear_cofactor.argtypes = [P, vp]
        l.bls_g1_add.argtypes = [P, P, vp]
        l.bls_combine_g2.argtypes = [I, I, vp, P, vp]
        l.bls_combine_g2.restype = I
        l.bls_combine_g1.argtypes = [I, I, vp, P, vp]
        l.bls_combine_g1.restype = I
        l.bls_bivar_evaluate.argtypes = [I, P, U64, U64, vp]
        l.bls_bivar_row.argtypes = [I, P, U64, vp]
        l.bls_verify_g2_batch.argtypes = [SZ, vp, vp, vp, vp, vp, I]
        _lib = l
    return _lib


def _out(n):
    return ctypes.create_string_buffer(n)


def k32(k):
    return int(k).to_bytes(32, "little")


def g1_mul(p96, k):
    o = _out(96)
    lib().bls_g1_mul(bytes(p96), k32(k), o)
    return o.raw


def g2_mul(q192, k):
    o = _out(192)
    lib().bls_g2_mul(bytes(q192), k32(k), o)
    return o.raw


def g2_clear_cofactor(q192):
    o = _out(192)
    lib().bls_g2_clear_cofactor(bytes(q192), o)
    return o.raw


def g1_add(a, b):
    o = _out(96)
    lib().bls_g1_add(bytes(a), bytes(b), o)
    return o.raw


def verify_g2(pk96, sig192, h192):
    return bool(lib().bls_verify_g2(bytes(pk96), bytes(sig192), bytes(h192)))


def pairing_eq(p1, q1, p2, q2):
    return bool(lib().bls_pairing_eq(bytes(p1), bytes(q1), bytes(p2), bytes(q2)))


def pairing(p96, q192):
    o = _out(576)
    lib().bls_pairing(bytes(p96), bytes(q192), o)
    return o.raw


def _idx(idx):
    a = (ctypes.c_uint64 * max(len(idx), 1))(*idx)
    return a


def combine_g2(t, idx, pts):
    o = _out(192)
    rc = lib().bls_combine_g2(t, len(idx), _idx(idx), b"".join(bytes(p) for p in pts), o)
    return rc, o.raw


def combine_g1(t, idx, pts):
    o = _out(96)
    rc = lib().bls_combine_g1(t, len(idx), _idx(idx), b"".join(bytes(p) for p in pts), o)
    return rc, o.raw


def bivar_evaluate(t, commit, x, y):
    o = _out(96)
    lib().bls_bivar_evaluate(t, b"".join(bytes(c) for c in commit), x, y, o)
    return o.raw


def bivar_row(t, commit, x):
    o = _out(96 * (t + 1))
    lib().bls_bivar_row(t, b"".join(bytes(c) for c in commit), x, o)
    return [o.raw[96 * i:96 * (i + 1)] for i in range(t + 1)]


def verify_g2_batch(pks, sigs, hashes, doc_idx, threads=1):
    import numpy as np
    n = len(pks) // 96
    v = np.zeros(n, dtype=np.uint8)
    di = None if doc_idx is None else np.ascontiguousarray(doc_idx, dtype=np.uint32)
    pk = np.frombuffer(bytes(pks), dtype=np.uint8)
    sg = np.frombuffer(bytes(sigs), dtype=np.uint8)
    hs = np.frombuffer(bytes(hashes), dtype=np.uint8)
    lib().bls_verify_g2_batch(n, pk.ctypes.data, sg.ctypes.data, hs.ctypes.data,
                              None if di is None else di.ctypes.data, v.ctypes.data, threads)
    return v
