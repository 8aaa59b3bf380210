"""Host-side mirror of hbbft's SyncKeyGen (``src/sync_key_gen.rs``) over the GPU engine.

Same message types (``Part``, ``Ack``), outcomes (``PartOutcome`` / ``AckOutcome``), fault names
(``PartFault`` / ``AckFault``, ``sync_key_gen.rs:551-588``) and state rules (``ProposalState``,
``is_complete``, ``is_ready``, ``generate``) as the reference.  Where the crypto runs:

  GPU (engine, public data)   BivarCommitment::row (hbh_bivar_row), Poly::commitment (hbh_g1_mul_gen of
                              g1), BivarPoly::commitment, Ciphertext::verify (hbh_verify_ciphertexts),
                              BivarCommitment::evaluate == g1 * val (hbh_bivar_ack_check)
  host (secrets, hashing)     SecretKey::decrypt's U * sk and XOR stream, encrypt_with_rng,
                              hash_g1_g2 (hbbft_amd.hoststage, csrc/host_hash.cpp); Fr arithmetic

``handle_parts`` / ``handle_acks`` take a list of messages and return exactly the outcomes that
calling ``handle_part`` / ``handle_ack`` on each in order would: every check is a pure function of
(commitment, ciphertext), so all of them are verified in one engine call per kind first (the DKG
ack stream drain of SURVEY §8f f1), then the reference's sequential state logic is applied.

Serialisation of the encrypted payloads (threshold_crypto's serde of Poly / FieldWrap<Fr> through
bincode): a row is a u64 LE coefficient count followed by 32-byte LE canonical Fr values; a value
is one 32-byte LE Fr.  Parity with the real crate's bytes is unpinned; the payloads
never leave the key generation, so only the node set has to agree on them.
"""
import random

from . import hoststage, wire
from ._lib import G1_BYTES

R_ORDER = 0x73EDA753299D7D483339D80809A1D80553BDA402FFFE5BFEFFFFFFFF00000001
G1_GEN = bytes.fromhex(
    "bbc622db0af03afbef1a7af93fe8556c58ac1b173f3a4ea105b974974f8c68c30faca94f8c63952694d79731a7d3f117"
    "e1e7c5462923aa0ce48a88a244c73cd0edb3042ccb18db00f60ad0d595e0f5fce48a1d74ed309ea0f1a0aae381f4b308")
G2_GEN = bytes.fromhex(
    "b8bd21c1c85680d4efbb05a82603ac0b77d1e37a640b51b4023b40fad47ae4c65110c52d27050826910a8ff0b2a24a02"
    "7e2b045d057dace5575d941312f14c3349507fdcbb61dab51ab62099d0d06b59654f2788a0d3ac7d609f7152602be013"
    "0128b808865493e189a2ac3bccc93a922cd16051699a426da7d3bd8caa9bfdad1a352edac6cdc98c116e7d7227d5e50c"
    "be795ff05f07a9aaa11dec5c270d373fab992e57ab927426af63a7857e283ecb998bc22bb0d2ac32cc34a72ea0c40606")


# ------------------------------------------------------------------ Fr helpers (host, secret data)
def poly_eval(coeffs, x):
    r = 0
    for c in reversed(coeffs):
        r = (r * x + c) % R_ORDER
    return r


def coeff_pos(i, j):
    """threshold_crypto coeff_pos: symmetric index j(j+1)/2 + i for i <= j."""
    if j < i:
        i, j = j, i
    return j * (j + 1) // 2 + i


def interpolate_at_zero(samples):
    """Poly::interpolate(samples).evaluate(0) over Fr; samples: [(x, y)] with distinct x."""
    acc = 0
    for k, (xk, yk) in enumerate(samples):
        num, den = 1, 1
        for m, (xm, _) in enumerate(samples):
            if m != k:
                num = num * xm % R_ORDER
                den = den * (xm - xk) % R_ORDER
        acc = (acc + yk * num * pow(den, R_ORDER - 2, R_ORDER)) % R_ORDER
    return acc


def ncoef(degree):
    """Points of a degree-d BivarCommitment: (d+1)(d+2)/2 (coeff_pos(d, d) + 1)."""
    return (degree + 1) * (degree + 2) // 2


def ser_row(coeffs):
    return len(coeffs).to_bytes(8, "little") + b"".join(c.to_bytes(32, "little") for c in coeffs)


def de_row(b):
    """bincode::deserialize::<Poly> (sync_key_gen.rs:507): a u64 LE coefficient count, then that many
    32-byte LE canonical Fr.  bincode 1.x's ``deserialize`` reads what the type needs and ignores
    trailing bytes; a short buffer or a non-canonical Fr is an error (None).  Any count
    deserialises: a row of the wrong length is caught by the commitment comparison (RowCommitment),
    as in the reference."""
    if len(b) < 8:
        return None
    n = int.from_bytes(b[:8], "little")
    if len(b) < 8 + 32 * n:
        return None
    out = [int.from_bytes(b[8 + 32 * k:40 + 32 * k], "little") for k in range(n)]
    return out if all(c < R_ORDER for c in out) else None


def ser_val(v):
    return v.to_bytes(32, "little")


def de_val(b):
    """bincode::deserialize::<FieldWrap<Fr>> (sync_key_gen.rs:539-541): 32 bytes LE, canonical;
    trailing bytes are ignored (bincode 1.x), fewer than 32 bytes or a value >= r is an error."""
    if len(b) < 32:
        return None
    v = int.from_bytes(b[:32], "little")
    return v if v < R_ORDER else None


# ------------------------------------------------------------------ messages / outcomes
class Ciphertext:
    def __init__(self, u, v, w):
        self.u, self.v, self.w = bytes(u), bytes(v), bytes(w)

    def __eq__(self, o):
        return isinstance(o, Ciphertext) and (self.u, self.v, self.w) == (o.u, o.v, o.w)

    def __hash__(self):
        return hash((self.u, self.v, self.w))


class Part:
    """Part(BivarCommitment, Vec<Ciphertext>) (sync_key_gen.rs:225).

    A BivarCommitment of degree d holds exactly ncoef(d) points (threshold_crypto builds it that
    way; a message that carries another count does not decode, see wire.decode_part), so a Part
    with an inconsistent count cannot be constructed: the batched engine calls rely on it."""

    def __init__(self, degree, commit, rows):
        self.degree, self.commit, self.rows = int(degree), [bytes(c) for c in commit], list(rows)
        if self.degree < 0 or len(self.commit) != ncoef(self.degree):
            raise ValueError("BivarCommitment of degree %d needs %d points, got %d"
                             % (self.degree, ncoef(max(self.degree, 0)), len(self.commit)))

    def __eq__(self, o):
        return isinstance(o, Part) and (self.degree, self.commit, self.rows) == (o.degree, o.commit, o.rows)

    def to_bytes(self):
        """bincode(Part) (hbbft_amd.wire)."""
        return wire.encode_part(self.degree, self.commit, [(c.u, c.v, c.w) for c in self.rows])


class Ack:
    """Ack(u64 proposer index, Vec<Ciphertext>) (sync_key_gen.rs:242)."""

    def __init__(self, proposer_idx, values):
        self.proposer_idx, self.values = proposer_idx, list(values)

    def to_bytes(self):
        """bincode(Ack) (hbbft_amd.wire)."""
        return wire.encode_ack(self.proposer_idx, [(c.u, c.v, c.w) for c in self.values])


class PartOutcome:
    def __init__(self, ack=None, fault=None):
        self.ack, self.fault = ack, fault

    @property
    def valid(self):
        return self.fault is None


class AckOutcome:
    def __init__(self, fault=None):
        self.fault = fault

    @property
    def valid(self):
        return self.fault is None


class SyncKeyGenError(Exception):
    """sync_key_gen::Error (UnknownSender, ...)."""


class ProposalState:
    def __init__(self, degree, commit):
        self.degree, self.commit = degree, list(commit)
        self.values = {}   # sender index + 1 -> Fr
        self.acks = set()  # sender indices
        self.set_idx = None  # index of the commitment in the instance's device-resident set

    def equals_new(self, part):
        """``*state == ProposalState::new(commit)`` (sync_key_gen.rs:489): the derived PartialEq
        compares the commitment AND the recorded values and acks, so once any Ack was handled for
        this proposer even an identical Part is ``MultipleParts``."""
        return (part.degree == self.degree and part.commit == self.commit
                and not self.values and not self.acks)

    def is_complete(self, threshold):
        return len(self.acks) > 2 * threshold


class PublicKeySet:
    """PublicKeySet{commit: Commitment} -- the generated key (threshold = degree)."""

    def __init__(self, commit):
        self.commit = [bytes(c) for c in commit]

    def threshold(self):
        return len(self.commit) - 1

    def public_key(self):
        return self.commit[0]

    def public_key_shares(self, engine, indices):
        """PublicKeySet::public_key_share(i) = commit.evaluate(i + 1) (hbh_commitment_eval)."""
        t = self.threshold()
        return engine.commitment_eval(t, [self.commit], [0] * len(indices), [i + 1 for i in indices])

    def __eq__(self, o):
        return isinstance(o, PublicKeySet) and self.commit == o.commit


# ------------------------------------------------------------------ crypto batches
def _decrypt_batch(engine, sec_key, cts, threads=0):
    """SecretKey::decrypt for a list of ciphertexts: None where Ciphertext::verify fails
    (sync_key_gen.rs:503-506, 535-538)."""
    if not cts:
        return []
    # Ciphertext::verify in its Q form (hbh_hash_g1_g2_bp): the same verdicts without the final
    # G2 scalar multiplication of each hash
    qbp = hoststage.hash_g1_g2_bp([c.u for c in cts], [c.v for c in cts], threads)
    ok = engine.verify_ciphertexts_bp([c.u for c in cts], [c.w for c in cts], qbp)
    good = [k for k, v in enumerate(ok) if v]
    out = [None] * len(cts)
    if good:
        gs = hoststage.g1_mul([cts[k].u for k in good], [sec_key] * len(good), threads)
        pts = hoststage.xor_with_hash(gs, [cts[k].v for k in good], threads)
        for k, p in zip(good, pts):
            out[k] = p
    return out


def _encrypt_batch(pks, payloads, rng, threads=0):
    """PublicKey::encrypt_with_rng per (pk, payload); nonces drawn from the caller's rng."""
    nonces = [rng.randrange(1, R_ORDER) for _ in payloads]
    return [Ciphertext(u, v, w) for (u, v, w) in hoststage.encrypt(pks, payloads, nonces, threads)]


# ------------------------------------------------------------------ SyncKeyGen
class SyncKeyGen:
    def __init__(self, our_id, sec_key, pub_keys, threshold, engine, threads=0):
        """sec_key: this node's encryption secret key (Fr int); pub_keys: {node_id: G1 ABI}."""
        self.our_id = our_id
        self.sec_key = sec_key
        self.pub_keys = dict(sorted(pub_keys.items()))
        ids = list(self.pub_keys)
        self.our_idx = ids.index(our_id) if our_id in self.pub_keys else None
        self.threshold = threshold
        self.parts = {}
        self.engine = engine
        self.threads = threads
        self._sets = {}  # degree -> CommitSet: every Part's commitment uploaded to HBM once

    def _commit_set(self, degree):
        cs = self._sets.get(degree)
        if cs is None:
            cs = self._sets[degree] = self.engine.commit_set(degree)
        return cs

    @classmethod
    def new(cls, our_id, sec_key, pub_keys, threshold, engine, rng=None, threads=0):
        """SyncKeyGen::new (sync_key_gen.rs:323-357): the instance and our Part (None for an
        observer).  BivarPoly::random(threshold), commitment on the GPU, one encrypted row per
        node on the host."""
        rng = rng or random.SystemRandom()
        kg = cls(our_id, sec_key, pub_keys, threshold, engine, threads)
        if kg.our_idx is None:
            return kg, None
        t = threshold
        ncoef = (t + 1) * (t + 2) // 2
        coeffs = [rng.randrange(0, R_ORDER) for _ in range(ncoef)]
        commit = engine.g1_mul_gen(coeffs)
        # row(x)_a = sum_b c(a, b) x^b for every node x (BivarPoly::row, sync_key_gen.rs:349-352):
        # t+1 polynomials in x evaluated at the N node indices on the host stage
        xs = [i + 1 for i in range(len(kg.pub_keys))]
        ev = hoststage.fr_poly_eval([[coeffs[coeff_pos(a, b)] for b in range(t + 1)] for a in range(t + 1)], xs,
                                    threads)
        rows = [[ev[a][i] for a in range(t + 1)] for i in range(len(xs))]
        cts = _encrypt_batch(list(kg.pub_keys.values()), [ser_row(r) for r in rows], rng, threads)
        return kg, Part(t, commit, cts)

    def public_keys(self):
        return self.pub_keys

    def node_index(self, node_id):
        return list(self.pub_keys).index(node_id) if node_id in self.pub_keys else None

    def num_nodes(self):
        return len(self.pub_keys)

    def count_complete(self):
        return sum(1 for p in self.parts.values() if p.is_complete(self.threshold))

    def is_node_ready(self, proposer_id):
        idx = self.node_index(proposer_id)
        return idx is not None and idx in self.parts and self.parts[idx].is_complete(self.threshold)

    def is_ready(self):
        return self.count_complete() > self.threshold

    # -------------------------------------------------------------- Part (sync_key_gen.rs:372-392, 481-512)
    def handle_part(self, sender_id, part, rng=None):
        return self.handle_parts([(sender_id, part)], rng)[0]

    def handle_parts(self, items, rng=None):
        rng = rng or random.SystemRandom()
        n = len(self.pub_keys)
        # 1. sequential state pass: which parts are new, what each outcome depends on
        plan = []
        seen = {}
        for sender_id, part in items:
            sidx = self.node_index(sender_id)
            if sidx is None:
                raise SyncKeyGenError("UnknownSender")
            if len(part.rows) != n:
                plan.append(("fault", "RowCount"))
                continue
            state = self.parts.get(sidx) or seen.get(sidx)
            if state is not None:
                plan.append(("fault", "MultipleParts") if not state.equals_new(part) else ("none", None))
                continue
            st = ProposalState(part.degree, part.commit)
            seen[sidx] = st
            plan.append(("new", (sidx, part, st)))
        new = [p[1] for p in plan if p[0] == "new"]
        # 2. crypto in batches: our commitment rows, our decrypted rows, the rows' commitments.
        #    Parts may carry any degree (the reference accepts them); one engine call per degree.
        rows_ok = {}
        if new and self.our_idx is not None:
            x = self.our_idx + 1
            commit_rows = [None] * len(new)
            for d, js in _by_degree(range(len(new)), lambda j: new[j][1].degree).items():
                # the commitments go to the device-resident set once; rows and later Ack checks
                # name them by index
                cs = self._commit_set(d)
                first = cs.add([new[j][1].commit for j in js])
                for k, j in enumerate(js):
                    new[j][2].set_idx = first + k
                got = cs.rows([first + k for k in range(len(js))], [x] * len(js))
                for j, r in zip(js, got):
                    commit_rows[j] = r
            plain = _decrypt_batch(self.engine, self.sec_key, [p.rows[self.our_idx] for _, p, _ in new], self.threads)
            polys = [de_row(b) if b is not None else None for b in plain]
            # Poly::commitment() only where the lengths agree: a row of another length can never
            # equal the commitment row (Commitment's derived PartialEq compares the vectors)
            match = [j for j in range(len(new)) if polys[j] is not None and len(polys[j]) == len(commit_rows[j])]
            flat = [c for j in match for c in polys[j]]
            comm = self.engine.g1_mul_gen(flat) if flat else []
            row_comm, k = {}, 0
            for j in match:
                row_comm[j] = comm[k:k + len(polys[j])]
                k += len(polys[j])
            for j, (sidx, part, st) in enumerate(new):
                if plain[j] is None:
                    rows_ok[sidx] = ("fault", "DecryptRow")
                elif polys[j] is None:
                    rows_ok[sidx] = ("fault", "DeserializeRow")
                elif row_comm.get(j) == commit_rows[j]:
                    rows_ok[sidx] = ("row", polys[j])
                else:
                    rows_ok[sidx] = ("fault", "RowCommitment")
        # 3. apply in order; encrypt the Acks of valid rows in one host batch
        outs, ack_jobs = [], []
        for kind, val in plan:
            if kind == "fault":
                outs.append(PartOutcome(fault=val))
            elif kind == "none":
                outs.append(PartOutcome())
            else:
                sidx, part, st = val
                self.parts[sidx] = st
                if self.our_idx is None:
                    outs.append(PartOutcome())
                    continue
                r = rows_ok[sidx]
                if r[0] == "fault":
                    outs.append(PartOutcome(fault=r[1]))
                else:
                    outs.append(PartOutcome())
                    ack_jobs.append((len(outs) - 1, sidx, r[1]))
        if ack_jobs:
            pks = list(self.pub_keys.values())
            vals = _eval_rows([row for _, _, row in ack_jobs], [i + 1 for i in range(n)], self.threads)
            payloads = [ser_val(v) for vs in vals for v in vs]
            cts = _encrypt_batch([pk for _ in ack_jobs for pk in pks], payloads, rng, self.threads)
            for j, (o, sidx, _) in enumerate(ack_jobs):
                outs[o].ack = Ack(sidx, cts[j * n:(j + 1) * n])
        return outs

    def handle_part_msgs(self, items, rng=None):
        """handle_parts over received bincode bytes: [(sender_id, bytes)].  The window's Parts are
        decoded in one batch (hbbft_amd.wire: one GPU decompression for every commitment point and
        ciphertext); a message that does not decode gets PartOutcome(fault="DeserializeMessage")
        -- the reference's transport would drop it before handle_part -- and the others the
        outcomes handle_parts gives them, in order."""
        dec = wire.decode_parts(self.engine, [b for _, b in items])
        good = [(sid, Part(d[0], d[1], [Ciphertext(*c) for c in d[2]])) for (sid, _), d in zip(items, dec)
                if d is not None]
        outs = iter(self.handle_parts(good, rng))
        return [next(outs) if d is not None else PartOutcome(fault="DeserializeMessage") for d in dec]

    # -------------------------------------------------------------- Ack (sync_key_gen.rs:398-404, 515-547)
    def handle_ack(self, sender_id, ack):
        return self.handle_acks([(sender_id, ack)])[0]

    def handle_ack_msgs(self, items):
        """handle_acks over received bincode bytes (see handle_part_msgs)."""
        dec = wire.decode_acks(self.engine, [b for _, b in items])
        good = [(sid, Ack(d[0], [Ciphertext(*c) for c in d[1]])) for (sid, _), d in zip(items, dec) if d is not None]
        outs = iter(self.handle_acks(good))
        return [next(outs) if d is not None else AckOutcome(fault="DeserializeMessage") for d in dec]

    def handle_acks(self, items):
        n = len(self.pub_keys)
        plan = []
        pending = {}  # proposer -> senders acked within this batch
        for sender_id, ack in items:
            sidx = self.node_index(sender_id)
            if sidx is None:
                raise SyncKeyGenError("UnknownSender")
            if len(ack.values) != n:
                plan.append(("fault", "ValueCount"))
                continue
            part = self.parts.get(ack.proposer_idx)
            if part is None:
                plan.append(("fault", "MissingPart"))
                continue
            acked = pending.setdefault(ack.proposer_idx, set(part.acks))
            if sidx in acked:
                plan.append(("none", None))
                continue
            acked.add(sidx)
            plan.append(("new", (sidx, ack, part)))
        new = [p[1] for p in plan if p[0] == "new"]
        verdict = {}
        if new and self.our_idx is not None:
            plain = _decrypt_batch(self.engine, self.sec_key, [a.values[self.our_idx] for _, a, _ in new], self.threads)
            vals = [de_val(b) if b is not None else None for b in plain]
            chk = [j for j, v in enumerate(vals) if v is not None]
            okmap = {}
            # one check per commitment degree against the device-resident commitments (uploaded
            # once by handle_parts); only indices and values travel
            for d, js in _by_degree(chk, lambda j: new[j][2].degree).items():
                ok = self._commit_set(d).ack_check([new[j][2].set_idx for j in js], [self.our_idx + 1] * len(js),
                                                   [new[j][0] + 1 for j in js], [vals[j] for j in js])
                okmap.update(zip(js, ok))
            for j in range(len(new)):
                if plain[j] is None:
                    verdict[j] = ("fault", "DecryptValue")
                elif vals[j] is None:
                    verdict[j] = ("fault", "DeserializeValue")
                elif not okmap[j]:
                    verdict[j] = ("fault", "ValueCommitment")
                else:
                    verdict[j] = ("val", vals[j])
        outs, j = [], 0
        for kind, val in plan:
            if kind == "fault":
                outs.append(AckOutcome(val))
            elif kind == "none":
                outs.append(AckOutcome())
            else:
                sidx, ack, part = val
                part.acks.add(sidx)  # valid or not, the sender has acked
                if self.our_idx is None:
                    outs.append(AckOutcome())
                else:
                    v = verdict[j]
                    if v[0] == "fault":
                        outs.append(AckOutcome(v[1]))
                    else:
                        part.values[sidx + 1] = v[1]
                        outs.append(AckOutcome())
                j += 1
        return outs

    # -------------------------------------------------------------- generate (sync_key_gen.rs:444-462)
    def generate(self):
        """(PublicKeySet, secret key share or None) (sync_key_gen.rs:444-462): pk_commit starts as
        Poly::zero().commitment() (empty) and ``+= part.commit.row(0)`` for every complete part --
        Commitment's AddAssign resizes to the longer operand and removes trailing zero points --;
        our share = sum over those parts of the interpolation at 0 of the first t+1 values."""
        t = self.threshold
        complete = [self.parts[k] for k in sorted(self.parts) if self.parts[k].is_complete(t)]
        zero = bytes(G1_BYTES)
        commit = []
        sk = 0 if self.our_idx is not None else None
        for part in complete:
            row0 = [part.commit[coeff_pos(i, 0)] for i in range(part.degree + 1)]  # row(0)_i = C(i, 0)
            m = max(len(commit), len(row0))
            commit = hoststage.g1_add(commit + [zero] * (m - len(commit)), row0 + [zero] * (m - len(row0)))
            while commit and commit[-1] == zero:
                commit.pop()
            if sk is not None:
                samples = sorted(part.values.items())[: t + 1]
                sk = (sk + interpolate_at_zero(samples)) % R_ORDER
        return PublicKeySet(commit), sk


def _eval_rows(rows, xs, threads=0):
    """[[Poly::evaluate(row, x) for x in xs] for row in rows] on the host stage (hbh_fr_poly_eval),
    one call per row length (Parts of different degrees give rows of different lengths)."""
    out = [None] * len(rows)
    for ln, js in _by_degree(range(len(rows)), lambda j: len(rows[j])).items():
        for j, v in zip(js, hoststage.fr_poly_eval([rows[j] for j in js], xs, threads)):
            out[j] = v
    return out


def _by_degree(items, degree):
    """Group items by commitment degree (order kept within a group)."""
    groups = {}
    for it in items:
        groups.setdefault(degree(it), []).append(it)
    return groups


__all__ = ["SyncKeyGen", "Part", "Ack", "PartOutcome", "AckOutcome", "PublicKeySet", "Ciphertext",
           "SyncKeyGenError", "interpolate_at_zero"]
