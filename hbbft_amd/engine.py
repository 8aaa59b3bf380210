"""Host-side handle on one GPU's batch engine (C ABI in include/hbbft_hip.h).

Inputs are in the ABI point format (affine, canonical little-endian; infinity = all-zero); the
``wire`` helpers convert from the reference's uncompressed wire encoding (pairing 0.14
``into_uncompressed``: big-endian, G2 as x.c1 || x.c0 || y.c1 || y.c0, 0x40 flag = infinity).
"""
import ctypes

import numpy as np

from . import _lib
from ._lib import G1_BYTES, G2_BYTES, buf, check


def _u32(idx, n):
    if idx is None:
        return None, None
    a = np.ascontiguousarray(np.asarray(idx, dtype=np.uint32))
    if a.shape != (n,):
        raise ValueError("index array must have shape (n,)")
    return a, a.ctypes.data_as(ctypes.c_void_p)


def _fr_buf(vals, n):
    """(owner, pointer) of n 32-byte LE scalars: ints, or already packed (bytes / uint8 array of
    n * 32) -- a 10^6-ack call then skips the per-value packing."""
    if isinstance(vals, np.ndarray):
        a = np.ascontiguousarray(vals, dtype=np.uint8).reshape(-1)
    elif isinstance(vals, (bytes, bytearray)):
        a = np.frombuffer(bytes(vals), dtype=np.uint8)
    else:
        a = np.frombuffer(b"".join(int(v).to_bytes(32, "little") for v in vals), dtype=np.uint8)
    if a.size != 32 * n:
        raise ValueError("expected %d 32-byte scalars" % n)
    return a, a.ctypes.data_as(ctypes.c_void_p)


def _check_bivar(t, commits, part_idx):
    """Every BivarCommitment of a degree-t call holds (t+1)(t+2)/2 points, and every request names
    one of them: the kernels stride through the joined buffer by that count."""
    ncoef = (t + 1) * (t + 2) // 2
    for k, c in enumerate(commits):
        if len(c) != ncoef:
            raise ValueError("commitment %d has %d points, degree %d needs %d" % (k, len(c), t, ncoef))
    if any(not 0 <= int(i) < len(commits) for i in part_idx):
        raise ValueError("commitment index out of range")


def _join(points, size):
    if isinstance(points, (bytes, bytearray)):
        b = bytes(points)
    else:
        try:  # bytes-like items (bytes, bytearray, memoryview, uint8 arrays) join directly
            b = b"".join(points)
        except TypeError:
            b = b"".join(bytes(p) for p in points)
    if len(b) % size:
        raise ValueError("point buffer length %d is not a multiple of %d" % (len(b), size))
    return b


class Engine:
    """One engine per GPU (one process per GPU for multi-GPU runs)."""

    def __init__(self, device=0):
        self._l = _lib.lib()
        h = ctypes.c_void_p()
        check(self._l.hbh_engine_create(int(device), ctypes.byref(h)))
        self._h = h
        self.device = device

    def close(self):
        if getattr(self, "_h", None):
            self._l.hbh_engine_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    @property
    def handle(self):
        return self._h

    # ------------------------------------------------------------ pairing-equality checks
    def verify_pairing_eq(self, p1, q1_table, q1_idx, p2, q2_table, q2_idx):
        """verdict[i] = e(p1[i], q1[q1_idx[i]]) == e(p2[i], q2[q2_idx[i]])."""
        p1b, p2b = _join(p1, G1_BYTES), _join(p2, G1_BYTES)
        q1b, q2b = _join(q1_table, G2_BYTES), _join(q2_table, G2_BYTES)
        n = len(p1b) // G1_BYTES
        if len(p2b) // G1_BYTES != n:
            raise ValueError("p1/p2 length mismatch")
        nq1, nq2 = len(q1b) // G2_BYTES, len(q2b) // G2_BYTES
        i1, pi1 = _u32(q1_idx, n)
        i2, pi2 = _u32(q2_idx, n)
        out = (ctypes.c_uint8 * max(n, 1))()
        keep = [buf(x) for x in (p1b, q1b, p2b, q2b)]
        check(self._l.hbh_verify_pairing_eq(self._h, n, keep[0][1], keep[1][1], nq1, pi1,
                                            keep[2][1], keep[3][1], nq2, pi2, ctypes.cast(out, ctypes.c_void_p)))
        return bytes(out)[:n]

    def verify_sig_shares(self, pks, sigs, hashes, doc_idx):
        """PublicKeyShare::verify_g2 batch (src/threshold_sign.rs:216-225)."""
        pkb, sgb, hb = _join(pks, G1_BYTES), _join(sigs, G2_BYTES), _join(hashes, G2_BYTES)
        n = len(pkb) // G1_BYTES
        if len(sgb) // G2_BYTES != n:
            raise ValueError("pks/sigs length mismatch")
        di, pdi = _u32(doc_idx, n)
        out = (ctypes.c_uint8 * max(n, 1))()
        keep = [buf(x) for x in (pkb, sgb, hb)]
        check(self._l.hbh_verify_sig_shares(self._h, n, keep[0][1], keep[1][1], keep[2][1], len(hb) // G2_BYTES,
                                            pdi, ctypes.cast(out, ctypes.c_void_p)))
        return bytes(out)[:n]

    def verify_signatures(self, pks, sigs, hashes):
        """PublicKey::verify(sig, msg) batch with H = hash_g2(msg) hashed on the host: DHB signed
        votes (src/dynamic_honey_badger/votes.rs:153-158) and key-gen messages
        (src/dynamic_honey_badger/dynamic_honey_badger.rs:514-526).  Same pairing-equality check as
        verify_sig_shares, one hash per item."""
        n = len(_join(pks, G1_BYTES)) // G1_BYTES
        return self.verify_sig_shares(pks, sigs, hashes, list(range(n)))

    def verify_dec_shares(self, shares, pks, huv, w, ct_idx):
        """PublicKeyShare::verify_decryption_share batch (src/threshold_decrypt.rs:220-229)."""
        sb, pkb = _join(shares, G1_BYTES), _join(pks, G1_BYTES)
        hb, wb = _join(huv, G2_BYTES), _join(w, G2_BYTES)
        n = len(sb) // G1_BYTES
        ci, pci = _u32(ct_idx, n)
        out = (ctypes.c_uint8 * max(n, 1))()
        keep = [buf(x) for x in (sb, pkb, hb, wb)]
        check(self._l.hbh_verify_dec_shares(self._h, n, keep[0][1], keep[1][1], keep[2][1], keep[3][1],
                                            len(hb) // G2_BYTES, pci, ctypes.cast(out, ctypes.c_void_p)))
        return bytes(out)[:n]

    def verify_ciphertexts(self, u, w, huv):
        """Ciphertext::verify batch (src/threshold_decrypt.rs:142)."""
        ub, wb, hb = _join(u, G1_BYTES), _join(w, G2_BYTES), _join(huv, G2_BYTES)
        n = len(ub) // G1_BYTES
        out = (ctypes.c_uint8 * max(n, 1))()
        keep = [buf(x) for x in (ub, wb, hb)]
        check(self._l.hbh_verify_ciphertexts(self._h, n, keep[0][1], keep[1][1], keep[2][1],
                                             ctypes.cast(out, ctypes.c_void_p)))
        return bytes(out)[:n]

    def verify_ciphertexts_bp(self, u, w, qbp):
        """Ciphertext::verify batch from hoststage.hash_g1_g2_bp points: e(G1K, W) == e(U, Q), the
        reference's e(g1, W) == e(U, [KCOF] Q) by bilinearity (include/hbbft_hip.h hbh_hash_g1_g2_bp)."""
        from . import hoststage
        n = len(u)
        if not n:
            return b""
        return self.verify_pairing_eq([hoststage.hash_bp_g1()] * n, w, None, u, qbp, None)

    def verify_pairing_eq_dev(self, stream, n, d_p1, d_q1, nq1, d_i1, d_p2, d_q2, nq2, d_i2, d_v):
        """Device-pointer variant (ints are raw device addresses, e.g. torch ``data_ptr()``);
        d_p1 / d_p2 = None means the G1 generator for every item."""
        vp = ctypes.c_void_p
        check(self._l.hbh_verify_pairing_eq_dev(self._h, vp(stream) if stream else None, n,
                                                vp(d_p1) if d_p1 else None, vp(d_q1), nq1,
                                                vp(d_i1) if d_i1 else None, vp(d_p2) if d_p2 else None, vp(d_q2), nq2,
                                                vp(d_i2) if d_i2 else None, vp(d_v)))

    # ------------------------------------------------------------ combine / scalar mult / DKG
    def _interp(self, fn, size, t, idx, pts):
        """idx: [[node index] * (t+1)] per combine; pts: matching point bytes (flat or nested)."""
        ncomb = len(idx)
        flat_idx = [int(i) for row in idx for i in row]
        if any(len(row) != t + 1 for row in idx):
            raise ValueError("each combine needs exactly t+1 samples")
        pb = _join([p for row in pts for p in row] if ncomb and isinstance(pts[0], (list, tuple)) else pts, size)
        if len(pb) != ncomb * (t + 1) * size:
            raise ValueError("point count mismatch")
        ia, pia = _u32(flat_idx, len(flat_idx))
        out = (ctypes.c_uint8 * max(ncomb * size, 1))()
        st = (ctypes.c_int * max(ncomb, 1))()
        keep = buf(pb)
        check(fn(self._h, ncomb, t, pia, keep[1], ctypes.cast(out, ctypes.c_void_p), ctypes.cast(st, ctypes.c_void_p)))
        raw = bytes(out)
        return [raw[c * size:(c + 1) * size] for c in range(ncomb)], list(st)[:ncomb]

    def interpolate_g2(self, t, idx, pts):
        """PublicKeySet::combine_signatures batch (src/threshold_sign.rs:249-259): (points, status)."""
        return self._interp(self._l.hbh_interpolate_g2, G2_BYTES, t, idx, pts)

    def combine_verify_g2(self, t, idx, pts, master_pk, hashes):
        """ThresholdSign::combine_and_verify_sig batch (src/threshold_sign.rs:249-270): one device
        pass of combine_signatures + PublicKey::verify_g2 per document.  Returns
        (signatures, statuses, verdicts); hashes[c] is H of document c."""
        ncomb = len(idx)
        if any(len(row) != t + 1 for row in idx):
            raise ValueError("each combine needs exactly t+1 samples")
        pb = _join([p for row in pts for p in row] if ncomb and isinstance(pts[0], (list, tuple)) else pts, G2_BYTES)
        hb = _join(hashes, G2_BYTES)
        if len(pb) != ncomb * (t + 1) * G2_BYTES or len(hb) != ncomb * G2_BYTES or len(bytes(master_pk)) != G1_BYTES:
            raise ValueError("point count mismatch")
        ia, pia = _u32([int(i) for row in idx for i in row], ncomb * (t + 1))
        out = (ctypes.c_uint8 * max(ncomb * G2_BYTES, 1))()
        st = (ctypes.c_int * max(ncomb, 1))()
        v = (ctypes.c_uint8 * max(ncomb, 1))()
        keep = [buf(x) for x in (pb, bytes(master_pk), hb)]
        check(self._l.hbh_combine_verify_g2(self._h, ncomb, t, pia, keep[0][1], keep[1][1], keep[2][1],
                                            ctypes.cast(out, ctypes.c_void_p), ctypes.cast(st, ctypes.c_void_p),
                                            ctypes.cast(v, ctypes.c_void_p)))
        raw = bytes(out)
        return ([raw[c * G2_BYTES:(c + 1) * G2_BYTES] for c in range(ncomb)], list(st)[:ncomb],
                bytes(v)[:ncomb])

    def interpolate_g1(self, t, idx, pts):
        """G1 interpolation of PublicKeySet::decrypt (src/threshold_decrypt.rs:242-250)."""
        return self._interp(self._l.hbh_interpolate_g1, G1_BYTES, t, idx, pts)

    def _mul(self, fn, size, pts, scalars):
        pb = _join(pts, size)
        n = len(pb) // size
        sb = b"".join(int(k).to_bytes(32, "little") for k in scalars)
        if len(sb) != 32 * n:
            raise ValueError("scalar count mismatch")
        out = (ctypes.c_uint8 * max(n * size, 1))()
        keep = [buf(pb), buf(sb)]
        check(fn(self._h, n, keep[0][1], keep[1][1], ctypes.cast(out, ctypes.c_void_p)))
        raw = bytes(out)
        return [raw[i * size:(i + 1) * size] for i in range(n)]

    def g1_mul(self, pts, scalars):
        return self._mul(self._l.hbh_g1_mul, G1_BYTES, pts, scalars)

    def g2_mul(self, pts, scalars):
        return self._mul(self._l.hbh_g2_mul, G2_BYTES, pts, scalars)

    def g1_mul_gen(self, scalars):
        """g1 * k for each scalar from the fixed-base comb table (hbh_g1_mul_gen)."""
        sb = b"".join(int(k).to_bytes(32, "little") for k in scalars)
        n = len(scalars)
        out = (ctypes.c_uint8 * max(n * G1_BYTES, 1))()
        keep = buf(sb)
        check(self._l.hbh_g1_mul_gen(self._h, n, keep[1], ctypes.cast(out, ctypes.c_void_p)))
        raw = bytes(out)
        return [raw[i * G1_BYTES:(i + 1) * G1_BYTES] for i in range(n)]

    def bivar_row(self, t, commits, part_idx, xs):
        """BivarCommitment::row(x) (src/sync_key_gen.rs:496) for each (part, x)."""
        _check_bivar(t, commits, part_idx)
        cb = _join([c for part in commits for c in part], G1_BYTES)
        nrow = len(part_idx)
        pa, ppa = _u32(part_idx, nrow)
        xa, pxa = _u32(xs, nrow)
        out = (ctypes.c_uint8 * max(nrow * (t + 1) * G1_BYTES, 1))()
        keep = buf(cb)
        check(self._l.hbh_bivar_row(self._h, nrow, t, len(commits), keep[1], ppa, pxa, ctypes.cast(out, ctypes.c_void_p)))
        raw = bytes(out)
        return [[raw[(r * (t + 1) + i) * G1_BYTES:(r * (t + 1) + i + 1) * G1_BYTES] for i in range(t + 1)]
                for r in range(nrow)]

    def _decompress(self, fn, enc_size, pt_size, encodings):
        b = _join(encodings, enc_size)
        n = len(b) // enc_size
        out = (ctypes.c_uint8 * max(n * pt_size, 1))()
        ok = (ctypes.c_uint8 * max(n, 1))()
        keep = buf(b)
        check(fn(self._h, n, keep[1], ctypes.cast(out, ctypes.c_void_p), ctypes.cast(ok, ctypes.c_void_p)))
        raw = bytes(out)
        return [raw[i * pt_size:(i + 1) * pt_size] for i in range(n)], bytes(ok)[:n]

    def g1_decompress(self, encodings):
        """pairing 0.14 G1Compressed::into_affine per 48-byte encoding: (ABI points, ok bytes)."""
        return self._decompress(self._l.hbh_g1_decompress, 48, G1_BYTES, encodings)

    def g2_decompress(self, encodings):
        """pairing 0.14 G2Compressed::into_affine per 96-byte encoding: (ABI points, ok bytes)."""
        return self._decompress(self._l.hbh_g2_decompress, 96, G2_BYTES, encodings)

    def commitment_eval(self, t, commits, commit_idx, xs):
        """Commitment::evaluate(x) per (commitment, x) request; public_key_share(i) = evaluate(i + 1)
        as NetworkInfo::new precomputes it (src/network_info.rs:59-62)."""
        if any(len(c) != t + 1 for c in commits):
            raise ValueError("each commitment needs t+1 points")
        cb = _join([p for c in commits for p in c], G1_BYTES)
        n = len(xs)
        ca, pca = _u32(commit_idx, n)
        xa, pxa = _u32(xs, n)
        out = (ctypes.c_uint8 * max(n * G1_BYTES, 1))()
        keep = buf(cb)
        check(self._l.hbh_commitment_eval(self._h, n, t, len(commits), keep[1], pca, pxa,
                                          ctypes.cast(out, ctypes.c_void_p)))
        raw = bytes(out)
        return [raw[r * G1_BYTES:(r + 1) * G1_BYTES] for r in range(n)]

    def bivar_ack_check(self, t, commits, part_idx, xs, ys, vals):
        """BivarCommitment::evaluate(x, y) == g1 * val (src/sync_key_gen.rs:542) per ack."""
        _check_bivar(t, commits, part_idx)
        cb = _join([c for part in commits for c in part], G1_BYTES)
        n = len(part_idx)
        pa, ppa = _u32(part_idx, n)
        xa, pxa = _u32(xs, n)
        ya, pya = _u32(ys, n)
        vb = b"".join(int(v).to_bytes(32, "little") for v in vals)
        out = (ctypes.c_uint8 * max(n, 1))()
        keep = [buf(cb), buf(vb)]
        check(self._l.hbh_bivar_ack_check(self._h, n, t, len(commits), keep[0][1], ppa, pxa, pya, keep[1][1],
                                          ctypes.cast(out, ctypes.c_void_p)))
        return bytes(out)[:n]

    # ------------------------------------------------------------ device-resident variants
    # ints are raw device addresses (e.g. torch ``data_ptr()``); stream None = engine stream
    def interpolate_g1_dev(self, stream, ncomb, t, d_idx, d_pts, d_out, d_status):
        vp = ctypes.c_void_p
        check(self._l.hbh_interpolate_g1_dev(self._h, vp(stream) if stream else None, ncomb, t, vp(d_idx), vp(d_pts),
                                             vp(d_out), vp(d_status)))

    def interpolate_g2_dev(self, stream, ncomb, t, d_idx, d_pts, d_out, d_status):
        vp = ctypes.c_void_p
        check(self._l.hbh_interpolate_g2_dev(self._h, vp(stream) if stream else None, ncomb, t, vp(d_idx), vp(d_pts),
                                             vp(d_out), vp(d_status)))

    def g1_decompress_dev(self, stream, n, d_in, d_out, d_ok):
        vp = ctypes.c_void_p
        check(self._l.hbh_g1_decompress_dev(self._h, vp(stream) if stream else None, n, vp(d_in), vp(d_out), vp(d_ok)))

    def g2_decompress_dev(self, stream, n, d_in, d_out, d_ok):
        vp = ctypes.c_void_p
        check(self._l.hbh_g2_decompress_dev(self._h, vp(stream) if stream else None, n, vp(d_in), vp(d_out), vp(d_ok)))

    def commit_set(self, t):
        """An empty device-resident set of degree-t BivarCommitments (hbh_commit_set_create)."""
        return CommitSet(self, t)

    def bivar_ack_check_dev(self, stream, nack, t, d_commits, nrow, d_row_part, d_row_x, d_row_of, d_ys, d_vals,
                            d_verdicts):
        vp = ctypes.c_void_p
        check(self._l.hbh_bivar_ack_check_dev(self._h, vp(stream) if stream else None, nack, t, vp(d_commits), nrow,
                                              vp(d_row_part), vp(d_row_x), vp(d_row_of), vp(d_ys), vp(d_vals),
                                              vp(d_verdicts)))

    def set_pairing_impl(self, impl):
        """HBH_IMPL_*: 3 = auto (default: wave up to HBH_AUTO_WAVE_MAX checks, lane octo up to
        HBH_AUTO_OCT_MAX, lane quad up to HBH_AUTO_QUAD_MAX, lane pair above),
        4 = lane pair (two lanes per check, fused), 5 = wave (one 64-lane wave per check: the latency
        kernel), 6 = lane quad (four lanes per check: mid-size batches), 7 = lane octo (eight lanes per
        check).  0, 1, 2 are retired
        implementations (HBH_ERR_ARG)."""
        check(self._l.hbh_engine_set_pairing_impl(self._h, int(impl)))

    def set_ack_impl(self, impl):
        """HBH_ACK_*: 0 = auto (default), 1 = lane quads, 2 = one lane per ack (finite differences for
        dense y runs), 3 = one lane per ack, Horner only (commitment sets)."""
        check(self._l.hbh_engine_set_ack_impl(self._h, int(impl)))

    # ------------------------------------------------------------ profiling
    def set_profiling(self, on):
        check(self._l.hbh_engine_set_profiling(self._h, 1 if on else 0))

    def stage_time(self, stage):
        """(total device ms, launches) of a stage since set_profiling."""
        ms = ctypes.c_double()
        nl = ctypes.c_int()
        check(self._l.hbh_engine_stage_time(self._h, int(stage), ctypes.byref(ms), ctypes.byref(nl)))
        return ms.value, nl.value

    def dbg_pairing(self, p, q):
        """e(p[i], q[i])^3 as 12 canonical Fp coefficients (LE, 48 B each) per item."""
        pb, qb = _join(p, G1_BYTES), _join(q, G2_BYTES)
        n = len(pb) // G1_BYTES
        out = (ctypes.c_uint8 * max(n * 576, 1))()
        keep = [buf(x) for x in (pb, qb)]
        check(self._l.hbh_dbg_pairing(self._h, n, keep[0][1], keep[1][1], ctypes.cast(out, ctypes.c_void_p)))
        raw = bytes(out)[: n * 576]
        return [raw[i * 576:(i + 1) * 576] for i in range(n)]


# ------------------------------------------------------------------ wire-format helpers
P_FIELD = 0x1A0111EA397FE69A4B1BA7B6434BACD764774B84F38512BF6730D2A0F6B0F6241EABFFFEB153FFFFB9FEFFFFFFFFAAAB


def _check_uncompressed(b, size):
    """The flag and field checks of pairing 0.14's into_affine_unchecked for the uncompressed
    encoding: no compression flag (0x80), no sort flag (0x20), an infinity flag (0x40) only with
    every other bit zero, every coordinate < p.  Returns True for the point at infinity.  (On-curve
    and subgroup membership are not checked here: the engine's decompress kernels check on-curve,
    and the subgroup contract is documented in include/hbbft_hip.h.)"""
    b = bytes(b)
    if len(b) != size:
        raise ValueError("uncompressed point must be %d bytes" % size)
    if b[0] & 0x80:
        raise ValueError("unexpected compression mode")
    if b[0] & 0x20:
        raise ValueError("unexpected information (sort flag)")
    if b[0] & 0x40:
        if b[0] != 0x40 or any(b[1:]):
            raise ValueError("unexpected information (infinity with coordinates)")
        return True
    for o in range(0, size, 48):
        if int.from_bytes(b[o:o + 48], "big") >= P_FIELD:
            raise ValueError("coordinate not in field")
    return False


def g1_abi_from_uncompressed(b):
    """pairing 0.14 G1Uncompressed (96 B, BE, 0x40 = infinity) -> ABI bytes."""
    b = bytes(b)
    if _check_uncompressed(b, 96):
        return bytes(96)
    return b[0:48][::-1] + b[48:96][::-1]


class CommitSet:
    """Device-resident BivarCommitments of one degree (hbh_commit_set_*): a SyncKeyGen instance
    uploads each Part's commitment once (ProposalState::commit, src/sync_key_gen.rs:254-262) and
    checks rows (:496) and Acks (:542) against it by index; rows row(x) stay cached in HBM."""

    def __init__(self, engine, t):
        self._eng, self._l, self.t = engine, engine._l, int(t)
        h = ctypes.c_void_p()
        check(self._l.hbh_commit_set_create(engine._h, self.t, ctypes.byref(h)))
        self._h = h

    def add(self, commits):
        """Append commitments ((t+1)(t+2)/2 ABI G1 points each); returns the first one's index."""
        commits = list(commits)
        _check_bivar(self.t, commits, [])
        first = ctypes.c_size_t()
        if not commits:
            check(self._l.hbh_commit_set_add(self._h, 0, None, ctypes.byref(first)))
            return first.value
        keep = buf(_join([c for part in commits for c in part], G1_BYTES))
        check(self._l.hbh_commit_set_add(self._h, len(commits), keep[1], ctypes.byref(first)))
        return first.value

    def size(self):
        """(commitments held, rows cached)."""
        a, b = ctypes.c_size_t(), ctypes.c_size_t()
        check(self._l.hbh_commit_set_size(self._h, ctypes.byref(a), ctypes.byref(b)))
        return a.value, b.value

    def rows(self, part_idx, xs):
        """BivarCommitment::row(x) per (set index, x), affine: as Engine.bivar_row."""
        t, nrow = self.t, len(part_idx)
        if nrow == 0:
            return []
        pa, ppa = _u32(part_idx, nrow)
        xa, pxa = _u32(xs, nrow)
        out = (ctypes.c_uint8 * (nrow * (t + 1) * G1_BYTES))()
        check(self._l.hbh_bivar_row_set(self._h, nrow, ppa, pxa, ctypes.cast(out, ctypes.c_void_p)))
        raw = bytes(out)
        return [[raw[(r * (t + 1) + i) * G1_BYTES:(r * (t + 1) + i + 1) * G1_BYTES] for i in range(t + 1)]
                for r in range(nrow)]

    def ack_check(self, part_idx, xs, ys, vals):
        """BivarCommitment::evaluate(x, y) == g1 * val per ack (set index, x, y, val): as
        Engine.bivar_ack_check, without re-uploading the commitments."""
        n = len(part_idx)
        if n == 0:
            return b""
        pa, ppa = _u32(part_idx, n)
        xa, pxa = _u32(xs, n)
        ya, pya = _u32(ys, n)
        vb = _fr_buf(vals, n)
        out = (ctypes.c_uint8 * n)()
        check(self._l.hbh_bivar_ack_check_set(self._h, n, ppa, pxa, pya, vb[1], ctypes.cast(out, ctypes.c_void_p)))
        return bytes(out)

    def close(self):
        if getattr(self, "_h", None):
            self._l.hbh_commit_set_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def g2_abi_from_uncompressed(b):
    """pairing 0.14 G2Uncompressed (192 B: x.c1 x.c0 y.c1 y.c0, BE) -> ABI (x.c0 x.c1 y.c0 y.c1, LE)."""
    b = bytes(b)
    if _check_uncompressed(b, 192):
        return bytes(192)
    return b[48:96][::-1] + b[0:48][::-1] + b[144:192][::-1] + b[96:144][::-1]


def g1_uncompressed_from_abi(b):
    b = bytes(b)
    if not any(b):
        return bytes([0x40]) + bytes(95)
    return b[0:48][::-1] + b[48:96][::-1]


def g2_uncompressed_from_abi(b):
    b = bytes(b)
    if not any(b):
        return bytes([0x40]) + bytes(191)
    return b[48:96][::-1] + b[0:48][::-1] + b[144:192][::-1] + b[96:144][::-1]


class _PoolCalls:
    """Routes Engine's ``hbh_<op>`` calls to the pool's ``hbh_pool_<op>`` entry points."""

    def __init__(self, lib):
        self._lib = lib

    def __getattr__(self, name):
        return getattr(self._lib, name.replace("hbh_engine_", "hbh_", 1).replace("hbh_", "hbh_pool_", 1))


class Pool(Engine):
    """Multi-device fan-out (hbh_pool_*): one engine per shard, the batch split by instance,
    one host thread per shard, outputs gathered in order.  ``devices`` lists each shard's device
    (repeat a device for several shards on it).  Offers the batched calls of Engine that have a
    pool entry point: verify_sig_shares, verify_signatures, verify_dec_shares, combine_verify_g2,
    interpolate_g1, bivar_ack_check, set_pairing_impl."""

    POOLED = {"verify_sig_shares", "verify_signatures", "verify_dec_shares", "combine_verify_g2",
              "interpolate_g1", "bivar_ack_check", "set_pairing_impl", "close", "shards", "handle", "device",
              "shard_engine"}

    def __init__(self, devices):
        lib = _lib.lib()
        devs = (ctypes.c_int * len(devices))(*[int(d) for d in devices])
        h = ctypes.c_void_p()
        check(lib.hbh_pool_create(devs, len(devices), ctypes.byref(h)))
        self._raw = lib
        self._l = _PoolCalls(lib)
        self._h = h
        self.device = list(devices)

    def close(self):
        if getattr(self, "_h", None):
            self._raw.hbh_pool_destroy(self._h)
            self._h = None

    def shard_engine(self, s):
        """Borrowed Engine view of shard s (owned by the pool; for profiling counters)."""
        h = ctypes.c_void_p()
        check(self._raw.hbh_pool_engine(self._h, int(s), ctypes.byref(h)))
        e = Engine.__new__(Engine)
        e._l, e._h, e.device = self._raw, h, self.device[s]
        e.close = lambda: None
        return e

    @property
    def shards(self):
        n = ctypes.c_int()
        check(self._raw.hbh_pool_shards(self._h, ctypes.byref(n)))
        return n.value

    def __getattribute__(self, name):
        if not name.startswith("_") and name not in Pool.POOLED and hasattr(Engine, name):
            raise AttributeError("Pool has no pooled entry point for %s" % name)
        return object.__getattribute__(self, name)
