"""ctypes binding of the C ABI in include/hbbft_hip.h (libhbbft_hip.so, built in-tree).

Loading fails loudly when the shared library is missing: there is no CPU fallback anywhere in
the product path.
"""
import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
# HBBFT_HIP_LIB overrides the in-tree library (A/B builds of the same sources)
LIB_PATH = os.environ.get("HBBFT_HIP_LIB") or os.path.join(_HERE, "libhbbft_hip.so")

G1_BYTES = 96
G2_BYTES = 192
FR_BYTES = 32

# (name, restype, argtypes) for every symbol declared in include/hbbft_hip.h
_c = ctypes
_P = _c.c_void_p
_SZ = _c.c_size_t
_I = _c.c_int
SIGNATURES = [
    ("hbh_engine_create", _I, [_I, _c.POINTER(_P)]),
    ("hbh_engine_destroy", _I, [_P]),
    ("hbh_last_error", _c.c_char_p, []),
    ("hbh_device_count", _I, [_c.POINTER(_I)]),
    ("hbh_verify_pairing_eq", _I, [_P, _SZ, _P, _P, _SZ, _P, _P, _P, _SZ, _P, _P]),
    ("hbh_verify_sig_shares", _I, [_P, _SZ, _P, _P, _P, _SZ, _P, _P]),
    ("hbh_verify_dec_shares", _I, [_P, _SZ, _P, _P, _P, _P, _SZ, _P, _P]),
    ("hbh_verify_ciphertexts", _I, [_P, _SZ, _P, _P, _P, _P]),
    ("hbh_verify_pairing_eq_dev", _I, [_P, _P, _SZ, _P, _P, _SZ, _P, _P, _P, _SZ, _P, _P]),
    ("hbh_dbg_pairing", _I, [_P, _SZ, _P, _P, _P]),
    ("hbh_interpolate_g2", _I, [_P, _SZ, _I, _P, _P, _P, _P]),
    ("hbh_interpolate_g1", _I, [_P, _SZ, _I, _P, _P, _P, _P]),
    ("hbh_combine_verify_g2", _I, [_P, _SZ, _I, _P, _P, _P, _P, _P, _P, _P]),
    ("hbh_g1_mul", _I, [_P, _SZ, _P, _P, _P]),
    ("hbh_g2_mul", _I, [_P, _SZ, _P, _P, _P]),
    ("hbh_g1_mul_gen", _I, [_P, _SZ, _P, _P]),
    ("hbh_bivar_row", _I, [_P, _SZ, _I, _SZ, _P, _P, _P, _P]),
    ("hbh_g1_decompress", _I, [_P, _SZ, _P, _P, _P]),
    ("hbh_g2_decompress", _I, [_P, _SZ, _P, _P, _P]),
    ("hbh_commitment_eval", _I, [_P, _SZ, _I, _SZ, _P, _P, _P, _P]),
    ("hbh_bivar_ack_check", _I, [_P, _SZ, _I, _SZ, _P, _P, _P, _P, _P, _P]),
    ("hbh_commit_set_create", _I, [_P, _I, _c.POINTER(_P)]),
    ("hbh_commit_set_destroy", _I, [_P]),
    ("hbh_commit_set_add", _I, [_P, _SZ, _P, _c.POINTER(_SZ)]),
    ("hbh_commit_set_size", _I, [_P, _c.POINTER(_SZ), _c.POINTER(_SZ)]),
    ("hbh_bivar_row_set", _I, [_P, _SZ, _P, _P, _P]),
    ("hbh_bivar_ack_check_set", _I, [_P, _SZ, _P, _P, _P, _P, _P]),
    ("hbh_engine_set_pairing_impl", _I, [_P, _I]),
    ("hbh_engine_set_ack_impl", _I, [_P, _I]),
    ("hbh_engine_set_profiling", _I, [_P, _I]),
    ("hbh_engine_stage_time", _I, [_P, _I, _c.POINTER(_c.c_double), _c.POINTER(_I)]),
    # device-resident variants
    ("hbh_interpolate_g1_dev", _I, [_P, _P, _SZ, _I, _P, _P, _P, _P]),
    ("hbh_interpolate_g2_dev", _I, [_P, _P, _SZ, _I, _P, _P, _P, _P]),
    ("hbh_g1_decompress_dev", _I, [_P, _P, _SZ, _P, _P, _P]),
    ("hbh_g2_decompress_dev", _I, [_P, _P, _SZ, _P, _P, _P]),
    ("hbh_bivar_ack_check_dev", _I, [_P, _P, _SZ, _I, _P, _SZ, _P, _P, _P, _P, _P, _P]),
    # engine pool (multi-device fan-out)
    ("hbh_pool_create", _I, [_P, _I, _c.POINTER(_P)]),
    ("hbh_pool_destroy", _I, [_P]),
    ("hbh_pool_shards", _I, [_P, _c.POINTER(_I)]),
    ("hbh_pool_engine", _I, [_P, _I, _c.POINTER(_P)]),
    ("hbh_pool_set_pairing_impl", _I, [_P, _I]),
    ("hbh_pool_verify_sig_shares", _I, [_P, _SZ, _P, _P, _P, _SZ, _P, _P]),
    ("hbh_pool_verify_dec_shares", _I, [_P, _SZ, _P, _P, _P, _P, _SZ, _P, _P]),
    ("hbh_pool_combine_verify_g2", _I, [_P, _SZ, _I, _P, _P, _P, _P, _P, _P, _P]),
    ("hbh_pool_interpolate_g1", _I, [_P, _SZ, _I, _P, _P, _P, _P]),
    ("hbh_pool_bivar_ack_check", _I, [_P, _SZ, _I, _SZ, _P, _P, _P, _P, _P, _P]),
    # host stage (no engine, no GPU)
    ("hbh_host_last_error", _c.c_char_p, []),
    ("hbh_host_threads", _I, [_c.POINTER(_I)]),
    ("hbh_hash_g2", _I, [_SZ, _P, _P, _P, _I]),
    ("hbh_hash_g1_g2", _I, [_SZ, _P, _P, _P, _P, _I]),
    ("hbh_xor_with_hash", _I, [_SZ, _P, _P, _P, _P, _I]),
    ("hbh_signature_parity", _I, [_SZ, _P, _P]),
    ("hbh_g1_compress", _I, [_SZ, _P, _P]),
    ("hbh_g2_compress", _I, [_SZ, _P, _P]),
    ("hbh_host_g1_mul", _I, [_SZ, _P, _P, _P, _I]),
    ("hbh_host_g2_mul", _I, [_SZ, _P, _P, _P, _I]),
    ("hbh_host_g1_add", _I, [_SZ, _P, _P, _P]),
    ("hbh_encrypt", _I, [_SZ, _P, _I, _P, _P, _P, _P, _P, _P, _I]),
    ("hbh_fr_poly_eval", _I, [_SZ, _SZ, _P, _SZ, _P, _P, _I]),
    ("hbh_hash_g1_g2_bp", _I, [_SZ, _P, _P, _P, _P, _I]),
    ("hbh_hash_bp_g1", _I, [_P]),
]
STAGE_PREPARE, STAGE_PAIRING, STAGE_CURVE = 0, 1, 2
IMPL_AUTO, IMPL_PAIR, IMPL_WAVE, IMPL_QUAD, IMPL_OCT, IMPL_WAVE2 = 3, 4, 5, 6, 7, 8   # HBH_IMPL_* (0, 1, 2 = retired THREAD, LANE_COOP, THREAD_SIGNED)
ACK_AUTO, ACK_QUAD, ACK_LANE, ACK_LANE_HORNER = 0, 1, 2, 3  # HBH_ACK_*

_lib = None


class HbhError(RuntimeError):
    pass


def lib():
    """Load libhbbft_hip.so (raises if absent - no fallback)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise HbhError("libhbbft_hip.so not built (run __graft_entry__.build() or `make -C hbbft_amd`)")
        l = ctypes.CDLL(LIB_PATH)
        for name, res, args in SIGNATURES:
            f = getattr(l, name)
            f.restype = res
            f.argtypes = args
        _lib = l
    return _lib


def check(rc):
    if rc != 0:
        raise HbhError("hbbft_hip error %d: %s" % (rc, lib().hbh_last_error().decode()))


def check_host(rc):
    if rc != 0:
        raise HbhError("hbbft_hip host stage error %d: %s" % (rc, lib().hbh_host_last_error().decode()))


def buf(b):
    """bytes-like -> (ctypes buffer, pointer) kept alive by the caller."""
    if b is None:
        return None, None
    if isinstance(b, (bytes, bytearray, memoryview)):
        cb = (ctypes.c_uint8 * len(b)).from_buffer_copy(bytes(b))
        return cb, ctypes.cast(cb, ctypes.c_void_p)
    raise TypeError(type(b))
