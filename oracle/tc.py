"""CPU restatement (ORACLE) of the ``threshold_crypto`` 0.3 operations hbbft calls on its hot path.

TEST INFRASTRUCTURE ONLY (see ``oracle/bls12_381.py`` header).  The crate is not vendored in
``/root/reference``; every function below restates the convention recorded in
SURVEY.md Appendix B and cites the hbbft call site it serves.  Byte-level conventions of the
real crate (hash_g2 RNG mapping, XOR stream, parity) are "parity unpinned" - see DESIGN.md.
"""
import hashlib
import struct

from . import bls12_381 as C

P, R = C.P, C.R


# ----------------------------------------------------------------------------- SHA3 / ChaCha20
def sha3_256(data):
    """tiny-keccak 1.4 ``sha3_256`` = FIPS-202 SHA3-256 (``Cargo.toml:38``)."""
    return hashlib.sha3_256(bytes(data)).digest()


def _rotl(v, c):
    return ((v << c) & 0xFFFFFFFF) | (v >> (32 - c))


def chacha20_block(key_words, counter, nonce_words=(0, 0)):
    """One ChaCha20 block (20 rounds), rand_chacha 0.1 layout: constants, 8 key words (LE),
    64-bit block counter in words 12-13, 64-bit nonce (zero) in words 14-15."""
    s = [0x61707865, 0x3320646E, 0x79622D32, 0x6B206574] + list(key_words) + [
        counter & 0xFFFFFFFF, (counter >> 32) & 0xFFFFFFFF, nonce_words[0], nonce_words[1]]
    x = list(s)

    def qr(a, b, c, d):
        x[a] = (x[a] + x[b]) & 0xFFFFFFFF; x[d] = _rotl(x[d] ^ x[a], 16)
        x[c] = (x[c] + x[d]) & 0xFFFFFFFF; x[b] = _rotl(x[b] ^ x[c], 12)
        x[a] = (x[a] + x[b]) & 0xFFFFFFFF; x[d] = _rotl(x[d] ^ x[a], 8)
        x[c] = (x[c] + x[d]) & 0xFFFFFFFF; x[b] = _rotl(x[b] ^ x[c], 7)

    for _ in range(10):
        qr(0, 4, 8, 12); qr(1, 5, 9, 13); qr(2, 6, 10, 14); qr(3, 7, 11, 15)
        qr(0, 5, 10, 15); qr(1, 6, 11, 12); qr(2, 7, 8, 13); qr(3, 4, 9, 14)
    return [(x[i] + s[i]) & 0xFFFFFFFF for i in range(16)]


class ChaChaRng:
    """``ChaChaRng::from_seed(seed)`` consumed through rand 0.4 / rand_core ``BlockRng``
    (SURVEY Appendix B.3): ``next_u32`` = next key-stream word, ``next_u64`` = two consecutive
    words, low word first - i.e. a flat little-endian word stream."""

    def __init__(self, seed32):
        assert len(seed32) == 32
        self.key = list(struct.unpack("<8I", bytes(seed32)))
        self.counter = 0
        self.buf = []
        self.idx = 0

    def next_u32(self):
        if self.idx >= len(self.buf):
            self.buf = chacha20_block(self.key, self.counter)
            self.counter += 1
            self.idx = 0
        w = self.buf[self.idx]
        self.idx += 1
        return w

    def next_u64(self):
        lo = self.next_u32()
        hi = self.next_u32()
        return (hi << 32) | lo

    def gen_fq(self):
        """ff 0.4 ``Fq::rand``: 6 x next_u64 little-endian limbs, clear top 3 bits, retry if
        >= p, and the limbs are the *Montgomery* representation (value = limbs / 2^384)."""
        rinv = pow(1 << 384, P - 2, P)
        while True:
            limbs = [self.next_u64() for _ in range(6)]
            limbs[5] &= 0xFFFFFFFFFFFFFFFF >> 3
            v = sum(l << (64 * i) for i, l in enumerate(limbs))
            if v < P:
                return v * rinv % P

    def gen_bool(self):
        """rand 0.4 ``bool``: ``gen::<u8>() & 1 == 1`` with ``u8`` = ``next_u32() as u8``."""
        return (self.next_u32() & 0xFF) & 1 == 1


# ----------------------------------------------------------------------------- hash to G2
def g2_rand(rng):
    """pairing 0.14 ``G2::rand``: x = Fq2{c0: rand, c1: rand}; greatest = rand bool;
    if x^3 + b is a square: y chosen by ``(y < -y) ^ greatest``; P = h2 * (x, y);
    return P if P != O."""
    while True:
        c0 = rng.gen_fq()
        c1 = rng.gen_fq()
        x = (c0, c1)
        greatest = rng.gen_bool()
        rhs = C.f2_add(C.f2_mul(C.f2_sqr(x), x), C.B2)
        y = C.f2_sqrt(rhs)
        if y is None:
            continue
        negy = C.f2_neg(y)
        y_lt = C.f2_gt(negy, y)
        if not (y_lt ^ greatest):
            y = negy
        pt = C.g2_mul((x, y), C.H2)
        if pt is not None:
            return pt


def hash_g2(msg):
    """threshold_crypto ``hash_g2`` - called by ``ThresholdSign::set_document``
    (``src/threshold_sign.rs:151``)."""
    return g2_rand(ChaChaRng(sha3_256(msg)))


def hash_g1_g2(g1pt, msg):
    """``hash_g1_g2(U, V)``: V if |V| <= 64 else sha3(V), then compress(U)."""
    msg = bytes(msg)
    m = sha3_256(msg) if len(msg) > 64 else msg
    return hash_g2(m + C.g1_compress(g1pt))


def xor_with_hash(g1pt, data):
    """``xor_with_hash(g, V)``: V xor low byte of successive next_u32."""
    rng = ChaChaRng(sha3_256(C.g1_compress(g1pt)))
    return bytes((b ^ (rng.next_u32() & 0xFF)) for b in bytes(data))


def signature_parity(g2pt):
    """``Signature::parity`` (used as the coin, ``src/binary_agreement/binary_agreement.rs:402``):
    parity of the popcount of the XOR-fold of the 192-byte uncompressed encoding."""
    x = 0
    for b in C.g2_uncompressed(g2pt):
        x ^= b
    return bin(x).count("1") % 2 == 1


# ----------------------------------------------------------------------------- polynomials
def poly_eval(coeffs, x):
    r = 0
    for c in reversed(coeffs):
        r = (r * x + c) % R
    return r


def commit_eval_g1(commit, x):
    """``Commitment::evaluate`` (Horner over G1): used by ``PublicKeySet::public_key_share``
    (``src/network_info.rs:59-62``)."""
    acc = None
    for c in reversed(commit):
        acc = C.g1_add(C.g1_mul(acc, x % R) if acc is not None else None, c)
    return acc


def lagrange_coeffs_at_zero(xs):
    """lambda_k(0) = prod_{m != k} x_m / (x_m - x_k) over Fr."""
    out = []
    for k, xk in enumerate(xs):
        num, den = 1, 1
        for m, xm in enumerate(xs):
            if m == k:
                continue
            num = num * xm % R
            den = den * (xm - xk) % R
        out.append(num * pow(den, R - 2, R) % R)
    return out


class NotEnoughShares(Exception):
    pass


def interpolate(t, items, add, mul):
    """threshold_crypto ``interpolate``: first t+1 items, x_k = idx_k + 1, result sum lambda_k P_k;
    ``NotEnoughShares`` if fewer; t == 0 returns the single sample."""
    samples = list(items)[: t + 1]
    if len(samples) <= t:
        raise NotEnoughShares()
    if t == 0:
        return samples[0][1]
    xs = [(i + 1) % R for (i, _) in samples]
    lams = lagrange_coeffs_at_zero(xs)
    acc = None
    for lam, (_, pt) in zip(lams, samples):
        acc = add(acc, mul(pt, lam))
    return acc


def combine_signatures(t, shares):
    """``PublicKeySet::combine_signatures`` (``src/threshold_sign.rs:249-259``). shares: [(idx, G2)]."""
    return interpolate(t, shares, C.g2_add, C.g2_mul)


def combine_decryption(t, shares, ct):
    """``PublicKeySet::decrypt`` (``src/threshold_decrypt.rs:242-250``)."""
    g = interpolate(t, shares, C.g1_add, C.g1_mul)
    return xor_with_hash(g, ct[1])


# ----------------------------------------------------------------------------- keys / checks
class KeySet:
    """``SecretKeySet::random`` + ``public_keys`` (``src/network_info.rs:174-215``) from given Fr
    coefficients (the reference draws them from an RNG; tests fix them by seed)."""

    def __init__(self, coeffs):
        self.coeffs = [c % R for c in coeffs]
        self.t = len(coeffs) - 1
        self.commit = [C.g1_mul(C.G1_GEN, c) for c in self.coeffs]

    def sk_share(self, i):
        return poly_eval(self.coeffs, i + 1)

    def pk_share(self, i):
        return C.g1_mul(C.G1_GEN, self.sk_share(i))

    def master_pk(self):
        return self.commit[0]


def verify_g2(pk, sig, h):
    """``PublicKeyShare::verify_g2`` / ``PublicKey::verify_g2``: e(pk, H) == e(g1, sig)
    (``src/threshold_sign.rs:223,264``)."""
    return C.pairing_product_is_one([(pk, h), (C.g1_neg(C.G1_GEN), sig)])


def encrypt(pk, msg, r):
    """``PublicKey::encrypt_with_rng`` (Appendix B.8) with the Fr nonce r given."""
    u = C.g1_mul(C.G1_GEN, r)
    v = xor_with_hash(C.g1_mul(pk, r), msg)
    w = C.g2_mul(hash_g1_g2(u, v), r)
    return (u, v, w)


def ciphertext_verify(ct):
    """``Ciphertext::verify``: e(g1, W) == e(U, hash_g1_g2(U, V)) (``src/threshold_decrypt.rs:142``)."""
    u, v, w = ct
    h = hash_g1_g2(u, v)
    return C.pairing_product_is_one([(C.G1_GEN, w), (C.g1_neg(u), h)])


def decrypt_share(sk_i, ct):
    """``SecretKeyShare::decrypt_share_no_verify``: D_i = U * sk_i (``threshold_decrypt.rs:161``)."""
    return C.g1_mul(ct[0], sk_i)


def verify_decryption_share(pk_i, share, ct, h_uv=None):
    """``PublicKeyShare::verify_decryption_share``: e(D_i, H_uv) == e(pk_i, W) (``threshold_decrypt.rs:227``)."""
    u, v, w = ct
    h = hash_g1_g2(u, v) if h_uv is None else h_uv
    return C.pairing_product_is_one([(share, h), (C.g1_neg(pk_i), w)])


# ----------------------------------------------------------------------------- SyncKeyGen
def coeff_pos(i, j):
    """threshold_crypto ``coeff_pos``: symmetric index j(j+1)/2 + i for i <= j."""
    if j < i:
        i, j = j, i
    return j * (j + 1) // 2 + i


class BivarPoly:
    def __init__(self, degree, coeffs):
        assert len(coeffs) == (degree + 1) * (degree + 2) // 2
        self.degree = degree
        self.coeffs = [c % R for c in coeffs]

    def evaluate(self, x, y):
        s = 0
        for i in range(self.degree + 1):
            for j in range(self.degree + 1):
                s = (s + self.coeffs[coeff_pos(i, j)] * pow(x, i, R) * pow(y, j, R)) % R
        return s

    def row(self, x):
        return [sum(self.coeffs[coeff_pos(i, j)] * pow(x, j, R) for j in range(self.degree + 1)) % R
                for i in range(self.degree + 1)]

    def commitment(self):
        return [C.g1_mul(C.G1_GEN, c) for c in self.coeffs]


def bivar_commit_row(degree, commit, x):
    """``BivarCommitment::row`` (``src/sync_key_gen.rs:496``)."""
    out = []
    for i in range(degree + 1):
        acc = None
        for j in range(degree + 1):
            acc = C.g1_add(acc, C.g1_mul(commit[coeff_pos(i, j)], pow(x, j, R)))
        out.append(acc)
    return out


def bivar_commit_evaluate(degree, commit, x, y):
    """``BivarCommitment::evaluate`` (``src/sync_key_gen.rs:542``)."""
    acc = None
    for i in range(degree + 1):
        for j in range(degree + 1):
            acc = C.g1_add(acc, C.g1_mul(commit[coeff_pos(i, j)], pow(x, i, R) * pow(y, j, R) % R))
    return acc


def poly_commitment(coeffs):
    """``Poly::commitment`` (``src/sync_key_gen.rs:508``)."""
    return [C.g1_mul(C.G1_GEN, c % R) for c in coeffs]
