"""HoneyBadger epoch crypto trace (BASELINE.json configs[4]).

What one node of a HoneyBadger network does with threshold cryptography in one epoch, replayed
through the mirrored message flows (hbbft_amd/protocol.py) with windowed BatchVerifier drains:

* Binary Agreement coins (src/binary_agreement/binary_agreement.rs:437-448): a BA instance whose
  epoch is 2 (mod 3) runs a ThresholdSign on ``bincode((BaSessionId{EpochId{hb_id, epoch},
  proposer_idx}, ba_epoch))`` (28 bytes, subset.rs:182-185, epoch_state.rs:401-404) and takes the
  signature's parity as the coin (:395-405).  ``coins`` of the N BA instances reach such an epoch
  (0 on the all-agree path, where epoch 0's fixed coin decides; N when every instance needs one
  threshold coin).
* Threshold decryption (src/honey_badger/epoch_state.rs:376-395): the N accepted contributions are
  ciphertexts (encrypt_with_rng of the proposer's batch); each goes through set_ciphertext
  (Ciphertext::verify), our own decryption share and the other nodes' shares, then
  combine_decryption_shares and the plaintext.

Messages are delivered in seeded random order, ``window`` at a time.  Before a window is delivered
the node queues the checks its messages will need (for instances that have not terminated) and
drains them: one engine call per kind per window, instead of one pairing check per message (the
reference's per-message verify).  Combines are deferred within the epoch and run in one batch
(BatchVerifier deferred mode); Steps and outputs are identical to per-message processing.

The CPU comparison is the reference-equivalent work: the checks the flows actually consumed
(``BatchVerifier.lookups``: shares that arrived before their instance terminated) plus the
combines, timed on the C restatement by bench.py (oracle use stays in bench/tests).
"""
import concurrent.futures
import os
import random
import struct
import sys
import time

from . import hoststage
from . import wire
from .binary_agreement import BinaryAgreementCoin, coin_document
from .protocol import BatchVerifier, Ciphertext, Deferred, Fault, NetworkInfo, ProtocolError, Step, \
    ThresholdDecrypt, ThresholdSign, signature_parity
from .sync_key_gen import G1_GEN, G2_GEN, R_ORDER

__all__ = ["NetworkKeys", "EpochTrace", "coin_document", "run_epoch", "EpochResult"]




def _poly_eval(coeffs, x):
    r = 0
    for c in reversed(coeffs):
        r = (r * x + c) % R_ORDER
    return r


class NetworkKeys:
    """A synthetic dealer's key set (SecretKeySet::random of degree t): secret shares sk_i =
    p(i+1), public-key shares g1*sk_i, master key g1*p(0).  Generated with the engine's scalar
    multiplication (test data, not the measured path)."""

    def __init__(self, engine, n, t, rng):
        self.n, self.t = n, t
        self.coeffs = [rng.randrange(1, R_ORDER) for _ in range(t + 1)]
        self.sks = [_poly_eval(self.coeffs, i + 1) for i in range(n)]
        pts = engine.g1_mul([G1_GEN] * (n + 1), self.sks + [self.coeffs[0]])
        self.pks = {i: pts[i] for i in range(n)}
        self.master_pk = pts[n]

    @property
    def msk(self):
        return self.coeffs[0]


class EpochTrace:
    """Every crypto message node ``our`` receives in one HoneyBadger epoch."""

    def __init__(self, keys, hb_epoch, proposals, cts, coin_docs, coin_shares, dec_shares, coin_msgs, dec_msgs):
        self.keys, self.hb_epoch = keys, hb_epoch
        self.proposals = proposals      # proposer -> plaintext contribution
        self.cts = cts                  # proposer -> (u, v, w) (encrypt_with_rng output)
        self.coin_docs = coin_docs      # proposer -> 28-byte coin document (BA instances with a coin)
        self.coin_shares = coin_shares  # (proposer, node) -> signature share
        self.dec_shares = dec_shares    # (proposer, node) -> decryption share
        self.coin_msgs = coin_msgs      # [(proposer, sender)] in delivery order
        self.dec_msgs = dec_msgs        # [(proposer, sender)] in delivery order
        self.bad = set()                # (kind, proposer, sender) of forged shares

    @classmethod
    def generate(cls, engine, keys, rng, hb_epoch=0, coins=None, proposal_bytes=256, bad_every=64, hb_id=0,
                 our=0, n_adv=0, adversary="silent", inject=0.1):
        """Node ``our``'s view of one epoch.  ``bad_every``: every bad_every-th share of an honest
        sender is forged (None: none).  ``n_adv`` nodes (ids n - n_adv .. n - 1, as the reference's
        TestNetwork numbers them) are adversarial: they propose nothing and send no correct share;
        ``adversary`` says what they send instead (tests/honey_badger.rs):
          "silent"       nothing (SilentAdversary);
          "faulty_share" FaultyShareAdversary (:26-115): every adversarial node broadcasts, for
                         every proposer, its (correct) decryption share of a FAKE ciphertext --
                         encrypt(b"X marks the spot") to the master key;
          "random"       RandomAdversary (:236-245, tests/network/mod.rs:237-350): about
                         ``inject`` x (honest messages) messages injected from random adversarial
                         senders, each a random coin (G2) or decryption (G1) share -- random valid
                         subgroup points, rand::random()'s Message -- for a random instance."""
        n = keys.n
        adv = set(range(n - n_adv, n))
        assert our not in adv
        good = [p for p in range(n) if p not in adv]
        coins = n if coins is None else coins
        proposals = {p: bytes(rng.randrange(256) for _ in range(proposal_bytes)) for p in good}
        enc = hoststage.encrypt([keys.master_pk], [proposals[p] for p in good],
                                [rng.randrange(1, R_ORDER) for _ in good])
        cts = dict(zip(good, enc))
        coin_docs = {p: coin_document(hb_id, hb_epoch, p, 2) for p in rng.sample(range(n), coins)}
        hashes = dict(zip(coin_docs, hoststage.hash_g2([coin_docs[p] for p in coin_docs]))) if coins else {}
        others = [j for j in good if j != our]
        bad = set()

        def forged(p, j, k):
            return bad_every is not None and (p * n + j) % bad_every == k

        # decryption shares D_{p,j} = U_p * sk_j (a few forged: U_p * random)
        keys_d, bases, scal = [], [], []
        for p in good:
            for j in others:
                fk = forged(p, j, 1)
                keys_d.append((p, j))
                bases.append(cts[p][0])
                scal.append(rng.randrange(1, R_ORDER) if fk else keys.sks[j])
                if fk:
                    bad.add(("dec", p, j))
        if adversary == "faulty_share" and adv:
            fake_u = hoststage.encrypt([keys.master_pk], [b"X marks the spot"], [rng.randrange(1, R_ORDER)])[0][0]
            for a in sorted(adv):
                for p in good:  # (shares for proposers without a contribution reach no instance)
                    keys_d.append((p, a))
                    bases.append(fake_u)
                    scal.append(keys.sks[a])
                    bad.add(("dec", p, a))
        dec_shares = dict(zip(keys_d, engine.g1_mul(bases, scal))) if keys_d else {}
        keys_s, bases, scal = [], [], []
        for p in coin_docs:
            for j in others:
                fk = forged(p, j, 2)
                keys_s.append((p, j))
                bases.append(hashes[p])
                scal.append(rng.randrange(1, R_ORDER) if fk else keys.sks[j])
                if fk:
                    bad.add(("coin", p, j))
        coin_shares = dict(zip(keys_s, engine.g2_mul(bases, scal))) if keys_s else {}
        if adversary == "random" and adv:
            slots = [("coin", p, a) for p in coin_docs for a in adv] + [("dec", p, a) for p in cts for a in adv]
            k = min(len(slots), max(1, int(inject * (len(keys_d) + len(keys_s)))))
            picks = rng.sample(slots, k)
            g1_keys = [(p, a) for kind, p, a in picks if kind == "dec"]
            g2_keys = [(p, a) for kind, p, a in picks if kind == "coin"]
            if g1_keys:
                dec_shares.update(zip(g1_keys, engine.g1_mul([G1_GEN] * len(g1_keys),
                                                             [rng.randrange(1, R_ORDER) for _ in g1_keys])))
            if g2_keys:
                coin_shares.update(zip(g2_keys, engine.g2_mul([G2_GEN] * len(g2_keys),
                                                              [rng.randrange(1, R_ORDER) for _ in g2_keys])))
            keys_d += g1_keys
            keys_s += g2_keys
            bad.update(picks)
        coin_msgs = list(keys_s)
        rng.shuffle(coin_msgs)
        dec_msgs = list(keys_d)
        rng.shuffle(dec_msgs)
        tr = cls(keys, hb_epoch, proposals, cts, coin_docs, coin_shares, dec_shares, coin_msgs, dec_msgs)
        tr.bad = bad
        tr.hashes = hashes
        tr.adv = adv
        return tr


def _serialize(trace, corrupt=()):
    """Attach the bincode bytes node ``our`` receives (hbbft_amd.wire): raw_coin / raw_dec per
    (proposer, sender) share message, raw_cts per contribution.  ``corrupt``: keys
    ("coin" | "dec", p, j) or ("ct", p) whose bytes are damaged (test use)."""
    ck = sorted(trace.coin_shares)
    dk = sorted(trace.dec_shares)
    trace.raw_coin = dict(zip(ck, wire.encode_sig_share_msgs([trace.coin_shares[k] for k in ck])))
    trace.raw_dec = dict(zip(dk, wire.encode_dec_share_msgs([trace.dec_shares[k] for k in dk])))
    ps = sorted(trace.cts)
    trace.raw_cts = dict(zip(ps, wire.encode_ciphertexts([trace.cts[p] for p in ps])))
    if getattr(trace, "ba", None) is not None:  # BA coin shares, keyed (p, e, j)
        bk = sorted(trace.ba.shares)
        trace.raw_ba = dict(zip(bk, wire.encode_sig_share_msgs([trace.ba.shares[k] for k in bk])))
    for c in corrupt:
        if c[0] == "ba":
            trace.raw_ba[c[1:]] = trace.raw_ba[c[1:]][:-1]              # truncated
        elif c[0] == "ct":
            b = trace.raw_cts[c[1]]
            trace.raw_cts[c[1]] = b[:8] + bytes([b[8] ^ 0x01]) + b[9:]  # a compressed x that is not on the curve
        else:
            d = trace.raw_coin if c[0] == "coin" else trace.raw_dec
            d[(c[1], c[2])] = d[(c[1], c[2])][:-1]                      # truncated
    return trace


EpochTrace.serialize = _serialize

BOTH = frozenset((False, True))
_EMPTY = Step()  # the Step of a message to a terminated instance: read by the drivers, never extended


class BaTrace:
    """The Binary Agreement side of an epoch for node ``our``: per BA instance (proposer p) the
    aux values its SBV broadcast outputs in each epoch (``sched[p][e]``), the coin documents and the
    other nodes' coin shares of every threshold-coin epoch on the instance's path (``docs[(p, e)]``,
    ``shares[(p, e, j)]``), the share messages in delivery order (``msgs``: (p, e, j)) and, per
    (p, e), the message positions after which our SBV output and our Conf round complete
    (``release``).  Shares of an epoch our instance has not reached go through its future-epoch
    queue (binary_agreement.rs:245-266)."""

    def __init__(self):
        self.sched, self.docs, self.shares, self.msgs, self.release = {}, {}, {}, [], {}
        self.decision, self.coins, self.bad = {}, {}, set()


def _with_ba(trace, engine, rng, extra=0.0, bad_every=None, spread=0.5):
    """Drive the epoch's coins through Binary Agreement (hbbft_amd.binary_agreement): every
    proposer with a coin runs a BA instance whose epochs 0 and 1 end with both values (estimate =
    the fixed coins true, false) and whose epoch 2 flips the threshold coin of trace.coin_docs[p];
    with probability ``extra`` the instance disagrees with that coin and runs on to epoch 5's
    threshold coin (epochs 3, 4: both values; epoch 5: decides).  ``spread``: the fraction of the
    message stream over which our SBV / Conf outcomes are released (the rest of the time our
    instance lags the network, so early shares wait in its future-epoch queue)."""
    keys = trace.keys
    n, our = keys.n, 0
    adv = getattr(trace, "adv", set())
    others = [j for j in range(n) if j != our and j not in adv]
    ba = BaTrace()
    ps = sorted(trace.coin_docs)
    h2 = [trace.hashes[p] for p in ps]
    c2 = dict(zip(ps, hoststage.signature_parity(engine.g2_mul(h2, [keys.msk] * len(h2))))) if ps else {}
    longer = [p for p in ps if rng.random() < extra]
    docs5 = {p: coin_document(0, trace.hb_epoch, p, 5) for p in longer}
    h5 = dict(zip(longer, hoststage.hash_g2([docs5[p] for p in longer]))) if longer else {}
    c5 = dict(zip(longer, hoststage.signature_parity(engine.g2_mul([h5[p] for p in longer],
                                                                       [keys.msk] * len(longer))))) if longer else {}
    sh_keys, bases, scal = [], [], []
    for p in ps:
        ba.docs[(p, 2)] = trace.coin_docs[p]
        if p in longer:
            ba.sched[p] = [BOTH, BOTH, frozenset([not c2[p]]), BOTH, BOTH, frozenset([c5[p]])]
            ba.decision[p], ba.coins[p] = c5[p], {2: c2[p], 5: c5[p]}
            ba.docs[(p, 5)] = docs5[p]
            for j in others:
                forged = bad_every is not None and (p * n + j) % bad_every == 3
                sh_keys.append((p, 5, j))
                bases.append(h5[p])
                scal.append(rng.randrange(1, R_ORDER) if forged else keys.sks[j])
                if forged:
                    ba.bad.add(("coin", p, j))
        else:
            ba.sched[p] = [BOTH, BOTH, frozenset([c2[p]])]
            ba.decision[p], ba.coins[p] = c2[p], {2: c2[p]}
        for j in others:
            if (p, j) in trace.coin_shares:
                ba.shares[(p, 2, j)] = trace.coin_shares[(p, j)]
    if sh_keys:
        ba.shares.update(zip(sh_keys, engine.g2_mul(bases, scal)))
    ba.msgs = list(ba.shares)
    rng.shuffle(ba.msgs)
    span = max(1, int(spread * len(ba.msgs)))
    for p in ps:
        for e in range(len(ba.sched[p])):
            a = rng.randrange(span)
            ba.release[(p, e)] = (a, a + rng.randrange(max(1, span // 4)))
    ba.bad |= {b for b in trace.bad if b[0] == "coin" and b[1] in ps}
    ba.hashes = {(p, 2): trace.hashes[p] for p in ps}
    ba.hashes.update({(p, 5): h5[p] for p in longer})
    trace.ba = ba
    return trace


EpochTrace.with_ba = _with_ba


class EpochResult:
    def __init__(self):
        self.coins = {}        # proposer -> bool (signature parity)
        self.signatures = {}   # proposer -> combined signature (ABI G2)
        self.plaintexts = {}   # proposer -> bytes
        self.faults = []       # (instance kind, proposer, Fault)
        self.errors = []       # (instance kind, proposer, ProtocolError): the reference's Err results
        self.timing = {}       # phase -> seconds
        self.engine_calls = 0
        self.checks_gpu = 0    # checks drained through the engine (incl. post-termination window tail)
        self.checks_consumed = 0  # verdicts the flows used (the reference's per-message checks)
        self.combines = 0
        self.wait = {}          # phase -> seconds the flows spent blocked on engine calls
        self.overlap = {}       # pipelined drains: host handling beside a drain in flight, worker engine time
        self.ba_decisions = {}  # proposer -> BA decision (BA-driven coins)
        self.ba_coins = {}      # proposer -> {BA epoch: threshold coin}
        self.ba_queued = 0      # coin shares that waited in a BA future-epoch queue


def _deliver(verifier, msgs, window, instance, queue, handle, res, kind, pipelined=True, limit=None, decode=None):
    """Deliver msgs in windows: queue the checks of messages whose instance is still running,
    drain once, then hand every message to its instance.

    pipelined: window k's drain runs on the GPU (drain_async) while the host hands window k - 1's
    messages to their instances; window k's checks are queued before window k - 1 is handled, so
    an instance that terminates in window k - 1 may have a few checks drained that it never reads
    (the verdicts, steps and faults are those of the serial order: verdicts are pure).

    limit: pre-verify at most this many shares per instance (threshold + slack); a share the
    instance still reads after that is a cache miss, verified on its own (BatchVerifier.*_valid)
    -- same verdicts, fewer checks drained for instances that terminate early.

    decode: raw-message mode -- decode(batch) turns a window's message bytes into share points in
    one batched call (hbbft_amd.wire) before the window is queued; a message that does not decode
    is dropped and logged as a ``DeserializeMessage`` fault of its sender."""
    def hand(batch):
        for p, j in batch:
            try:
                step = handle(p, j)
            except ProtocolError as e:  # the reference's Err from handle_message (immediate combines)
                res.errors.append((kind, p, e))
                continue
            if step.fault_log:
                res.faults += [(kind, p, f) for f in step.fault_log]
            if step.output:
                yield p, step.output[0]

    yield from _windows(verifier, msgs, window, instance, queue, hand, pipelined, limit, {}, decode, res, kind)


def _windows(verifier, msgs, window, instance, queue, hand, pipelined, limit, queued, decode=None, res=None,
             kind=None):
    prev = None
    for w0 in range(0, len(msgs), window):
        batch = msgs[w0:w0 + window]
        if decode is not None:
            bad = decode(batch)
            if bad:
                res.faults += [(kind, p, Fault(j, "DeserializeMessage")) for p, j in batch if (p, j) in bad]
                batch = [m for m in batch if m not in bad]
        for p, j in batch:
            if not instance[p].terminated:
                c = queued.get(p, 0)
                if limit is None or c < limit:
                    queue(p, j)
                    queued[p] = c + 1
        if not pipelined:
            verifier.drain()
            yield from hand(batch)
            continue
        pending = verifier.drain_async()
        if prev is not None:
            t0 = time.perf_counter()
            yield from hand(prev)
            if res is not None:
                res.overlap["hand_s"] = res.overlap.get("hand_s", 0.0) + time.perf_counter() - t0
        verifier.commit(pending)
        prev = batch
    if prev is not None:
        yield from hand(prev)


def run_epoch(engine, keys, trace, window=6144, our=0, threads=0, pipelined=False, slack=4, switch_interval=2e-4,
              defer=True, raw=False, ba=None, coin_prefetch=None, preverify=True, preverify_at="start",
              after_prep=None, fast_paths=True):
    """Replay ``trace`` as node ``our``; returns an EpochResult.  ``window`` = messages per drain;
    ``pipelined`` overlaps each window's GPU drain with the host handling of the previous window;
    ``slack``: shares pre-verified per instance beyond the t + 1 it needs (None: every share).
    ``switch_interval``: the interpreter's thread switch interval while the epoch runs pipelined
    (the drain thread needs the GIL around its engine call; at the default 5 ms it waits that long
    for the flows to yield, twice per drain); restored on return.  None leaves it alone.
    ``defer``: combines run in one batch at the end of the epoch (False: one engine call each,
    when the instance asks; the reference's order, used to check the deferred path).
    ``raw``: the node receives bincode bytes (``trace.serialize()``): contributions are decoded in
    one batch (DeserializeCiphertext faults, epoch_state.rs:377-381) and every window of share
    messages in one batch before it is queued (hbbft_amd.wire).
    ``preverify``: the contributions' ciphertext checks and the first t + 1 + slack decryption shares
    of each are checked on a second engine while the coin phase runs (_dec_preverify), started with
    the epoch (``preverify_at="start"``, round 5 default) or after the coin phase's first drain
    (``"first_drain"``, round 4's).  Round 5's host decryption prep finishes in well under a millisecond,
    so a pre-verification started at the first drain lands its GPU work on the coin phase's combines
    and local engine calls (coin resolve + local 11 + 4 -> 21 ms); started with the epoch it is done
    before they need the GPU: 19.7-19.9 -> 25.2-27.2 epochs/s (profiles/r05/c15_epoch_schedule.txt).
    ``after_prep``: called (from a host-pool thread) once this epoch's host decryption prep is done --
    a driver starts lower-priority host work there (the next epoch's coin prefetch) so that it does
    not share the host threads with the prep.
    ``ba``: the coins come from Binary Agreement instances (``trace.with_ba``; default: when the
    trace has a BA side) -- hbbft_amd.binary_agreement's epochs, fixed coins and future-epoch queue,
    our SBV / Conf outcomes released along the message stream, coin combines deferred per window.
    ``fast_paths``: the instances' cached-verdict transitions (ThresholdSign / ThresholdDecrypt
    ``store_cached``, BinaryAgreementCoin ``handle_fast``); False sends every message through the full
    ``handle_message`` path (tests/test_gpu_honey_badger.py compares the two)."""
    if ba is None:
        ba = getattr(trace, "ba", None) is not None
    old = sys.getswitchinterval()
    if pipelined and switch_interval:
        sys.setswitchinterval(switch_interval)
    try:
        return _run_epoch(engine, keys, trace, window, our, threads, pipelined, slack, defer, raw, ba, coin_prefetch,
                          preverify, preverify_at, after_prep, fast_paths)
    finally:
        sys.setswitchinterval(old)


def _decoder(engine, raw_msgs, out, fn):
    """decode(batch) for _deliver: fills out[(p, j)], returns the keys that did not decode."""
    def decode(batch):
        pts = fn(engine, [raw_msgs[m] for m in batch])
        bad = set()
        for m, pt in zip(batch, pts):
            if pt is None:
                bad.add(m)
            else:
                out[m] = pt
        return bad
    return decode


_HOST = None  # workers for host-stage crypto that overlaps the flows (ctypes calls release the GIL)
_COMBINE_ENGINES = {}  # id(engine) -> (engine, a second engine on its device for pipelined combines)


def combine_engine(engine):
    """The second engine (own stream and lock) that a pipelined epoch's combines run on, so a BA
    window's coin combines proceed while the next window's drain holds the first engine."""
    key = id(engine)
    if key not in _COMBINE_ENGINES:
        _COMBINE_ENGINES[key] = (engine, type(engine)(engine.device))
    return _COMBINE_ENGINES[key][1]


def _host_pool():
    global _HOST
    if _HOST is None:
        # two: an epoch's own decryption prep never waits behind the next epoch's coin prefetch
        _HOST = concurrent.futures.ThreadPoolExecutor(max_workers=2, thread_name_prefix="hbh-host")
    return _HOST


def _decrypt_prep(cts, sk, threads):
    """The host work of a contribution that depends only on its ciphertext bytes: H_uv =
    hash_g1_g2(U, V) (Ciphertext::verify's and every share check's hash) and our own decryption
    share U * sk (threshold_decrypt.rs:164).  RBC delivers a contribution before the BA instances and
    the Subset decide (src/honey_badger/epoch_state.rs: decryption starts at the Subset output), so
    this runs on a host thread from the start of the epoch, beside the coin phase; the threshold
    decryption itself still starts at the Subset output."""
    ps = sorted(cts)
    if not ps:
        return {}, {}
    huv = hoststage.hash_g1_g2([cts[p][0] for p in ps], [cts[p][1] for p in ps], threads=threads)
    own = hoststage.g1_mul([cts[p][0] for p in ps], [sk] * len(ps), threads=threads)
    return dict(zip(ps, huv)), dict(zip(ps, own))


def prefetch_coins(keys, hb_epoch, proposers, our=0, ba_epochs=(2,), hb_id=0, threads=0):
    """Start hashing the threshold-coin documents of a LATER HoneyBadger epoch and signing our
    shares on them, on the host-stage thread, while the current epoch runs.  A coin document is
    bincode((hb_id, hb_epoch, proposer), ba_epoch) (binary_agreement.rs:442; subset.rs:182-185), so
    the next epoch's first threshold coins (BA epoch 2 of every proposer's instance) are known before
    that epoch starts; the reference hashes and signs each when its Conf round completes
    (threshold_sign.rs:151, 176) -- same values, computed earlier.  Returns a future of
    {document: (hash_g2(document), our share)} for run_epoch(..., coin_prefetch=)."""
    docs = [coin_document(hb_id, hb_epoch, p, e) for p in proposers for e in ba_epochs]
    sk = keys.sks[our]
    bg = threads if threads else max(1, hoststage.host_threads() - 2)

    def job():
        if not docs:
            return {}
        hs = hoststage.hash_g2(docs, threads=bg)
        sigs = hoststage.g2_mul(hs, [sk] * len(hs), threads=bg)
        return {d: (h, g) for d, h, g in zip(docs, hs, sigs)}
    return _host_pool().submit(job)


_DEC_POOL = None  # one worker: speculative decryption-share pre-verification on the second engine


def _dec_preverify(engine2, keys, trace, prep, limit):
    """Ciphertext::verify of every contribution and PublicKeyShare::verify_decryption_share of the
    first ``limit`` shares (in arrival order) of each, on the second engine (own stream) while the
    coin phase runs: a node holds the RBC-delivered ciphertexts and the decryption shares that
    arrive for them before the Subset output starts the ThresholdDecrypt instances (they wait in the
    instance until set_ciphertext / remove_invalid_shares, threshold_decrypt.rs:138-147, 204-217).
    Verdicts are pure, so checking them early changes no Step; the decrypt phase finds them in the
    cache and queues only the rest.  Returns the engine results for BatchVerifier._store (main
    thread)."""
    t0 = time.perf_counter()
    huv_of, _ = prep.result()
    t_prep = time.perf_counter() - t0
    pre = BatchVerifier(engine2)
    for p in sorted(trace.cts):
        if p in huv_of:
            u, v, w = trace.cts[p]
            pre.queue_ct(Ciphertext(u, v, w, huv_of[p]))
    cnt = {}
    for p, j in trace.dec_msgs:
        if p not in huv_of:
            continue
        c = cnt.get(p, 0)
        if limit is not None and c >= limit:
            continue
        cnt[p] = c + 1
        pre.queue_dec(keys.pks[j], trace.dec_shares[(p, j)], huv_of[p], trace.cts[p][2])
    t0 = time.perf_counter()
    out = _one_call(engine2, pre._take_jobs())
    # speculative decryption combines on the same engine: per valid ciphertext, the first t + 1 shares
    # (arrival order: the order they were queued) whose verdicts are valid.  Any t + 1 valid shares of
    # a ciphertext interpolate to U * msk, so the deferred G1 combine of its ThresholdDecrypt
    # (threshold_decrypt.rs:242-250) takes this point unchanged (BatchVerifier._spec_g1) and leaves
    # the decrypt phase's critical path (HBH_EPOCH_SPEC_G1=0: off)
    spec = {}
    if os.environ.get("HBH_EPOCH_SPEC_G1", "1") != "0":
        by = {kind: (ks, v) for kind, ks, v in out}
        cks, cv = by.get("ct", ((), b""))
        dks, dv = by.get("dec", ((), b""))
        valid_ct = {(k[2], k[1]) for k, ok in zip(cks, cv) if ok}
        pk_idx = {pk: j for j, pk in keys.pks.items()}
        t = keys.t
        sel = {}
        for k, ok in zip(dks, dv):  # k = (pk, share, H_uv, W)
            if not ok:
                continue
            c = (k[2], k[3])
            if c not in valid_ct:
                continue
            got = sel.get(c)
            if got is None:
                got = sel[c] = {}
            elif len(got) > t:
                continue
            j = pk_idx.get(k[0])
            if j is not None and j not in got:
                got[j] = k[1]
        cs = [c for c in sel if len(sel[c]) == t + 1]
        if cs:
            idx = [sorted(sel[c]) for c in cs]
            pts, st = engine2.interpolate_g1(t, idx, [[sel[c][j] for j in ix] for c, ix in zip(cs, idx)])
            spec = {c: pt for c, pt, s_ in zip(cs, pts, st) if s_ == 0}
    return (out, spec), t_prep, time.perf_counter() - t0


def _one_call(engine2, jobs):
    """The pre-verification's ciphertext and decryption-share checks in ONE engine call: Ciphertext::verify
    e(U, H_uv) == e(g1, W) has the shape of a share check e(share, H_uv) == e(pk, W) with share = U and
    pk = g1, so the ciphertexts ride along as extra rows of verify_dec_shares over the same (H_uv, W)
    table (the same pairing equation as hbh_verify_ciphertexts, sides swapped).  Returns the
    BatchVerifier._store results of both kinds."""
    by = {kind: (keys, args) for kind, keys, args in jobs}
    if set(by) != {"ct", "dec"}:
        return BatchVerifier(engine2)._run_jobs(jobs)
    ckeys, _ = by["ct"]
    dkeys, (shares, pks, huvt, wt, cidx) = by["dec"]
    shares, pks, huvt, wt, cidx = list(shares), list(pks), list(huvt), list(wt), list(cidx)
    ctab = {c: i for i, c in enumerate(zip(huvt, wt))}
    for u, w, h in ckeys:  # ct keys: (U, W, H_uv)
        c = ctab.get((h, w))
        if c is None:
            c = ctab[(h, w)] = len(huvt)
            huvt.append(h)
            wt.append(w)
        shares.append(u)
        pks.append(G1_GEN)
        cidx.append(c)
    v = engine2.verify_dec_shares(shares, pks, huvt, wt, cidx)
    nd = len(dkeys)
    return [("dec", dkeys, v[:nd]), ("ct", ckeys, v[nd:])]


def _run_epoch(engine, keys, trace, window, our, threads, pipelined, slack, defer, raw, ba, coin_prefetch=None,
               preverify=True, preverify_at="start", after_prep=None, fast_paths=True):
    limit = None if slack is None else keys.t + 1 + slack
    res = EpochResult()
    # the background host work leaves two of the host threads to the flows and the drain worker
    bg = threads if threads else max(1, hoststage.host_threads() - 2)
    prep = None if raw else _host_pool().submit(_decrypt_prep, trace.cts, keys.sks[our], bg)
    if after_prep is not None:
        if prep is None:
            after_prep()
        else:
            prep.add_done_callback(lambda _f: after_prep())
    ver = BatchVerifier(engine, combine_engine(engine) if pipelined and hasattr(engine, "device") else None)
    ver.recording = defer                  # combines of the epoch run in one batch at the end
    ver.shortcuts = fast_paths
    pre_box = []  # the pre-verification future, once started

    def start_preverify():
        # after the coin phase's first drain: the checks then share the GPU with the flows' host work
        # (handling that window), not with the drain itself
        global _DEC_POOL
        if pre_box or not preverify or prep is None or not hasattr(engine, "device"):
            return
        if _DEC_POOL is None:
            _DEC_POOL = concurrent.futures.ThreadPoolExecutor(max_workers=1, thread_name_prefix="hbh-pre")
        pre_box.append(_DEC_POOL.submit(_dec_preverify, combine_engine(engine), keys, trace, prep, limit))
    if preverify_at == "start":
        start_preverify()
    sk = keys.sks[our]
    n = keys.n
    t_all = time.perf_counter()

    # --- Binary Agreement coins: ThresholdSign per BA instance that reaches a coin epoch
    t0 = time.perf_counter()
    if ba:
        coin_out = _ba_coins(engine, keys, trace, ver, window, our, threads, limit, res, pipelined, coin_prefetch,
                             start_preverify, raw)
        coin_sh, dec_sh = ({}, {}) if raw else (trace.coin_shares, trace.dec_shares)
        handed = {}
        ni_sign = None
        ts = {}
        res.timing["coin_verify"] = time.perf_counter() - t0
        res.wait["coin"] = ver.wait_s
    else:
        coin_out, handed, ni_sign, ts, coin_sh, dec_sh = _coins(engine, keys, trace, ver, window, our, threads,
                                                               pipelined, limit, res, raw, sk, n, t0)
    start_preverify()  # (no-op when already started; the synthetic coin phase starts it here)
    return _decrypt_and_output(engine, keys, trace, ver, window, our, threads, pipelined, limit, res, raw, sk, n,
                               t_all, coin_out, handed, ni_sign, ts, coin_sh, dec_sh, prep,
                               pre_box[0] if pre_box else None)


def _ba_coins(engine, keys, trace, ver, window, our, threads, limit, res, pipelined=False, coin_prefetch=None,
              after_first_drain=None, raw=False):
    """The BA-driven coin phase: one BinaryAgreementCoin per proposer with a coin (trace.ba).
    Messages (p, e, j) come in windows; before a window's drain, every share of a running or
    FUTURE epoch of its instance is queued (coin documents are hashed when first seen; a future
    epoch's verdicts wait in the cache for the ThresholdSign its replay opens); between windows our
    SBV / Conf outcomes whose release position has passed are fired, and the window's coin combines
    run as one deferred batch whose results resume the BA state machines (which may replay queued
    shares and complete further coins: repeated until no combine is pending).  Returns
    {p: signature of the instance's first threshold coin}, as the synthetic phase does.
    ``raw``: the coin-share messages arrive as bincode bytes (trace.raw_ba); each window is decoded
    in one batched engine call before it is queued, and a message that does not decode is dropped
    as a ``DeserializeMessage`` fault of its sender (as _windows does)."""
    ba = trace.ba
    bsh = {} if raw else ba.shares  # the coin shares the flows read (decoded per window when raw)
    sk = keys.sks[our]
    hb_id = 0
    own_sig = {}
    ni = NetworkInfo(our, range(keys.n), keys.t, keys.master_pk, keys.pks, sign_g2=lambda H: own_sig[bytes(H)])
    # our own shares: one batched host signing for every coin document on the instances' paths
    # (the reference signs each when its Conf round completes; the share is the same)
    t0 = time.perf_counter()
    pe = sorted(ba.docs)
    ready = coin_prefetch.result() if coin_prefetch is not None else {}  # (hash, our share) per document
    ver.add_doc_hashes({bytes(ba.docs[k]): ready[bytes(ba.docs[k])][0] for k in pe if bytes(ba.docs[k]) in ready})
    ver.hash_docs([ba.docs[k] for k in pe])  # one threaded host-stage call for the documents not prefetched
    hs = [ver.doc_hash_of(ba.docs[k]) for k in pe]
    hmap = dict(zip(pe, hs))
    res.timing["coin_hash"] = time.perf_counter() - t0
    t0 = time.perf_counter()
    todo = [h for k, h in zip(pe, hs) if bytes(ba.docs[k]) not in ready]
    for h, sgn in zip(todo, hoststage.g2_mul(todo, [sk] * len(todo), threads=threads) if todo else []):
        own_sig[bytes(h)] = sgn
    for k, h in zip(pe, hs):
        d = bytes(ba.docs[k])
        if d in ready:
            own_sig[bytes(h)] = ready[d][1]
        ver.queue_sig(keys.pks[our], h, own_sig[bytes(h)])
    res.timing["coin_own_shares"] = time.perf_counter() - t0
    bas = {p: BinaryAgreementCoin(ni, ver, (hb_id, trace.hb_epoch, p)) for p in sorted(ba.sched)}
    fired = set()
    queued_n = {}

    def record(p, step):
        if step.fault_log:
            res.faults += [("coin", p, f) for f in step.fault_log]
        if step.output:
            res.ba_decisions[p] = step.output[-1]

    def local_events(pos):
        progressed = True
        while progressed:
            progressed = False
            for p, b in bas.items():
                if b.decision is not None or b.pending is not None:
                    continue
                e = b.epoch
                rel = ba.release.get((p, e))
                if rel is None or e >= len(ba.sched[p]):
                    continue
                try:
                    if b.conf_values is None and pos >= rel[0]:
                        record(p, b.sbv_output(ba.sched[p][e]))
                        progressed = True
                    elif (b.conf_values is not None and not b.coin_decided and pos >= rel[1]
                          and (p, e) not in fired):
                        fired.add((p, e))
                        record(p, b.conf_round_complete())
                        progressed = True
                except ProtocolError as err:
                    res.errors.append(("coin", p, err))

    def resolve():
        while any(b.pending is not None for b in bas.values()):
            ver.flush_combines()  # failures surface in resolve_pending as the reference's Err
            for p, b in bas.items():
                if b.pending is not None:
                    try:
                        record(p, b.resolve_pending())
                    except ProtocolError as err:
                        res.errors.append(("coin", p, err))

    sig_cache = ver._sig

    pks = keys.pks

    def queue_window(batch):
        shares, qsig = bsh, ver._qsig  # (a drain replaces ver._qsig; none runs in here)
        for m in batch:
            p, e, j = m
            b = bas[p]
            if b.decision is None and e >= b.epoch and (b.epoch < e or not b.coin_decided):
                # a current epoch's shares are read in arrival order: the first t + 1 + slack; a
                # future epoch's are replayed in sender order (binary_agreement.rs:507-519), so
                # all of them are pre-verified
                pe = (p, e)
                c = queued_n.get(pe, 0)
                if limit is None or c < limit or e > b.epoch:
                    pk, h, sh = pks[j], hmap[pe], shares[m]
                    if type(pk) is bytes and type(h) is bytes and type(sh) is bytes:  # queue_sig inlined
                        if (pk, sh) not in sig_cache.get(h, ()):
                            qsig.append((pk, h, sh))
                    else:
                        ver.queue_sig(pk, h, sh)
                    queued_n[pe] = c + 1

    def hand_window(batch, end):
        shares, fast = bsh, ver.shortcuts
        t_msgs = time.perf_counter()
        for m in batch:
            p, e, j = m
            b = bas[p]
            # a message handle_message would ignore without a state change (decided instance, expired
            # epoch, coin decided or pending: :245-252, _handle_coin) is skipped here -- most of an
            # epoch's messages once its coins are done; the common transitions (future share queued,
            # cached valid share stored) are BinaryAgreementCoin.handle_fast's, the rest handle_message's
            if fast:
                be = b.epoch
                if b.decision is not None or e < be or (e == be and (b.coin_decided or b.pending is not None)):
                    continue
            if b.handle_fast(j, e, shares[m]):
                continue
            try:
                step = b.handle_message(j, e, shares[m])
            except ProtocolError as err:
                res.errors.append(("coin", p, err))
                continue
            if step.fault_log or step.output:
                record(p, step)
        t1 = time.perf_counter()
        tm = res.timing
        tm["coin_messages"] = tm.get("coin_messages", 0.0) + t1 - t_msgs
        resolve()
        t2 = time.perf_counter()
        local_events(end)
        t3 = time.perf_counter()
        resolve()
        t4 = time.perf_counter()
        tm["coin_resolve"] = tm.get("coin_resolve", 0.0) + (t2 - t1) + (t4 - t3)
        tm["coin_local"] = tm.get("coin_local", 0.0) + t3 - t2

    local_events(0)
    resolve()
    msgs = ba.msgs
    # pipelined (as _deliver): window k's checks are queued from the state before window k - 1 is
    # handled and drained on the GPU while the host handles window k - 1 -- a few checks of instances
    # that decide in window k - 1 may be drained unread; verdicts are pure, the Steps are the serial ones
    prev = None
    for w0 in range(0, len(msgs), window):
        batch = msgs[w0:w0 + window]
        t_q = time.perf_counter()
        if raw:
            pts = wire.decode_sig_share_msgs(engine, [trace.raw_ba[m] for m in batch])
            good = []
            for m, pt in zip(batch, pts):
                if pt is None:
                    res.faults.append(("coin", m[0], Fault(m[2], "DeserializeMessage")))
                else:
                    bsh[m] = pt
                    good.append(m)
            batch = good
            res.timing["coin_decode"] = res.timing.get("coin_decode", 0.0) + time.perf_counter() - t_q
        queue_window(batch)
        res.timing["coin_queue"] = res.timing.get("coin_queue", 0.0) + time.perf_counter() - t_q
        if not pipelined:
            ver.drain()
            if after_first_drain is not None:
                after_first_drain()
            hand_window(batch, w0 + len(batch))
            continue
        pending = ver.drain_async()
        if prev is not None:
            t0 = time.perf_counter()
            hand_window(*prev)
            res.overlap["hand_s"] = res.overlap.get("hand_s", 0.0) + time.perf_counter() - t0
        ver.commit(pending)
        prev = (batch, w0 + len(batch))
    if prev is not None:
        hand_window(*prev)
    local_events(len(msgs) + 1)
    resolve()
    out = {}
    for p, b in bas.items():
        res.ba_coins[p] = dict(b.coins)
        res.ba_queued += b.queued
        if 2 in b.signatures:
            out[p] = b.signatures[2]
    return out


def _coins(engine, keys, trace, ver, window, our, threads, pipelined, limit, res, raw, sk, n, t0):
    """The synthetic coin phase: one ThresholdSign per coin document (BA epoch 2), shares in windows."""
    ver.hash_docs([trace.coin_docs[p] for p in trace.coin_docs])
    own_sig = {}
    ni_sign = NetworkInfo(our, range(n), keys.t, keys.master_pk, keys.pks,
                          sign_g2=lambda H: own_sig[bytes(H)])
    ts = {p: ThresholdSign(ni_sign, ver) for p in trace.coin_docs}
    for p, inst in ts.items():
        inst.set_document(trace.coin_docs[p])
    hs = [ts[p].doc_hash for p in ts]
    for h, s in zip(hs, hoststage.g2_mul(hs, [sk] * len(hs), threads=threads) if hs else []):
        own_sig[bytes(h)] = s
        ver.queue_sig(keys.pks[our], h, s)  # sign() handles our own share as a message (:176)
    res.timing["coin_setup"] = time.perf_counter() - t0
    t0 = time.perf_counter()
    coin_out = {}
    for p, inst in ts.items():
        step = _input(inst, "coin", p, res)
        res.faults += [("coin", p, f) for f in step.fault_log]
        if step.output:
            coin_out[p] = step.output[0]
    handed = {}  # (kind, proposer) -> senders handed to the instance, in order (for a replay)
    coin_sh = {} if raw else trace.coin_shares
    dec_sh = {} if raw else trace.dec_shares

    handed_coin = {p: handed.setdefault(("coin", p), []) for p in ts}

    def hand_coin(p, j):
        handed_coin[p].append(j)
        inst = ts[p]
        if inst.terminated:
            return _EMPTY
        return inst.handle_message(j, coin_sh[(p, j)])

    for p, out in _deliver(ver, trace.coin_msgs, window, ts,
                           lambda p, j: ver.queue_sig(keys.pks[j], ts[p].doc_hash, coin_sh[(p, j)]),
                           hand_coin, res, "coin", pipelined, limit,
                           _decoder(engine, trace.raw_coin, coin_sh, wire.decode_sig_share_msgs) if raw else None):
        coin_out[p] = out
    res.timing["coin_verify"] = time.perf_counter() - t0
    res.wait["coin"] = ver.wait_s
    return coin_out, handed, ni_sign, ts, coin_sh, dec_sh


def _decrypt_and_output(engine, keys, trace, ver, window, our, threads, pipelined, limit, res, raw, sk, n, t_all,
                        coin_out, handed, ni_sign, ts, coin_sh, dec_sh, prep=None, dec_pre=None):
    # --- Subset output: the N ciphertexts into ThresholdDecrypt
    t0 = time.perf_counter()
    ps = sorted(trace.cts)
    if raw:  # the Subset outputs are serialised Ciphertexts: one batched decode
        got = dict(zip(ps, wire.decode_ciphertexts(engine, [trace.raw_cts[p] for p in ps])))
        res.faults += [("dec", p, Fault(p, "DeserializeCiphertext")) for p in ps if got[p] is None]
        ps = [p for p in ps if got[p] is not None]
    else:
        got = trace.cts
    if prep is not None:  # hashed and our shares computed beside the coin phase (_decrypt_prep)
        huv_of, own_of = prep.result()
        huv = [huv_of[p] for p in ps]
        own_dec = {p: own_of[p] for p in ps}
    else:
        huv = hoststage.hash_g1_g2([got[p][0] for p in ps], [got[p][1] for p in ps], threads=threads) if ps else []
        own_dec = dict(zip(ps, hoststage.g1_mul([got[p][0] for p in ps], [sk] * len(ps), threads=threads)))
    cts = {p: Ciphertext(got[p][0], got[p][1], got[p][2], h) for p, h in zip(ps, huv)}
    by_u = {cts[p].u: own_dec[p] for p in ps}
    ni_dec = NetworkInfo(our, range(n), keys.t, keys.master_pk, keys.pks, decrypt_share=lambda U: by_u[bytes(U)])
    td = {p: ThresholdDecrypt(ni_dec, ver) for p in ps}
    if dec_pre is not None:  # the verdicts checked beside the coin phase (_dec_preverify) into the cache
        t1 = time.perf_counter()
        (pre, spec), t_prep, t_eng = dec_pre.result()
        res.timing["decrypt_pre_prep"], res.timing["decrypt_pre_engine"] = t_prep, t_eng
        t2 = time.perf_counter()
        ver.wait_s += t2 - t1
        res.timing["decrypt_pre_wait"] = t2 - t1
        ver._store(pre)
        ver.add_speculative_g1(spec)
        res.timing["decrypt_pre_store"] = time.perf_counter() - t2
    for p in ps:
        ver.queue_ct(cts[p])  # (our own decryption share is not verified, threshold_decrypt.rs:167)
    t1 = time.perf_counter()
    ver.drain()
    res.timing["decrypt_drain"] = time.perf_counter() - t1
    res.timing["decrypt_setup"] = time.perf_counter() - t0
    t0 = time.perf_counter()
    dec_out = {}
    for p in list(ps):
        try:
            td[p].set_ciphertext(cts[p])
        except ProtocolError as e:  # HoneyBadger faults the proposer (epoch_state.rs:388-391)
            if e.kind != "InvalidCiphertext":
                raise
            res.faults.append(("dec", p, Fault(p, "InvalidCiphertext")))
            del td[p]
            ps.remove(p)
            continue
        step = _input(td[p], "dec", p, res)
        res.faults += [("dec", p, f) for f in step.fault_log]
        if step.output:
            dec_out[p] = step.output[0]

    handed_dec = {p: handed.setdefault(("dec", p), []) for p in td}

    dec_cache = ver._dec

    def hand_dec(p, j):
        handed_dec[p].append(j)
        inst = td[p]
        if inst.terminated:  # handle_message of a terminated instance is an empty Step (:183-185)
            return _EMPTY
        share = dec_sh[(p, j)]
        # the outcome most shares have (ThresholdDecrypt.store_cached), else the full path
        if inst.store_cached(j, share):
            return _EMPTY
        return inst.handle_message(j, share)

    dec_msgs = [m for m in trace.dec_msgs if m[0] in td]  # (shares of a faulted contribution: no instance)
    pks = keys.pks
    ct_key = {p: (cts[p].huv, cts[p].w) for p in td}

    def queue_dec(p, j):
        # most shares were pre-verified (_dec_preverify): a cached verdict queues nothing
        pk, sh, c = pks[j], dec_sh[(p, j)], ct_key[p]
        if type(pk) is bytes and type(sh) is bytes:
            d = dec_cache.get(c)
            if d is not None and (pk, sh) in d:
                return
        ver.queue_dec(pk, sh, c[0], c[1])

    for p, out in _deliver(ver, dec_msgs, window, td, queue_dec,
                           hand_dec, res, "dec", pipelined, limit,
                           _decoder(engine, trace.raw_dec, dec_sh, wire.decode_dec_share_msgs) if raw else None):
        dec_out[p] = out
    res.timing["decrypt_verify"] = time.perf_counter() - t0
    res.wait["decrypt"] = ver.wait_s - res.wait.get("coin", 0.0)

    # --- deferred combines: one G2 combine+verify batch, one G1 interpolation batch
    t0 = time.perf_counter()
    failed = {id(d) for d in ver.flush_combines()}
    res.timing["combine"] = time.perf_counter() - t0
    res.wait["combine"] = ver.wait_s - res.wait.get("coin", 0.0) - res.wait["decrypt"]
    t0 = time.perf_counter()
    # A failed deferred combine: the reference returned Err from the call that triggered it (and a
    # ThresholdSign stayed open), so that instance is replayed with immediate combines; its Steps
    # (outputs, faults, errors) replace the optimistic ones.
    for kind, outs in (("coin", coin_out), ("dec", dec_out)):
        for p in [p for p, d in outs.items() if isinstance(d, Deferred) and id(d) in failed]:
            del outs[p]
            res.faults = [f for f in res.faults if f[:2] != (kind, p)]
            out = _replay(engine, kind, p, ni_sign if kind == "coin" else ni_dec,
                          ts[p].doc_hash if kind == "coin" else cts[p], handed.get((kind, p), []),
                          coin_sh if kind == "coin" else dec_sh, res)
            if out is not None:
                outs[p] = out
    sigs = {p: (d.result[0] if isinstance(d, Deferred) else d) for p, d in coin_out.items()}
    order = sorted(sigs)
    res.signatures = sigs
    res.coins = dict(zip(order, hoststage.signature_parity([sigs[p] for p in order]))) if order else {}
    order = sorted(dec_out)
    direct = {p: dec_out[p] for p in order if not isinstance(dec_out[p], Deferred)}
    order = [p for p in order if p not in direct]
    gs = [dec_out[p].result[0] for p in order]
    res.plaintexts = dict(zip(order, hoststage.xor_with_hash(gs, [dec_out[p].data for p in order],
                                                              threads=threads))) if order else {}
    res.plaintexts.update(direct)
    res.timing["output"] = time.perf_counter() - t0
    res.timing["epoch"] = time.perf_counter() - t_all
    res.engine_calls, res.checks_gpu, res.checks_consumed = ver.calls, ver.checks, ver.lookups
    if pipelined:
        res.overlap["worker_engine_s"] = ver.async_s
    res.combines = len(coin_out) + len(dec_out)
    return res


def _input(inst, kind, p, res):
    """inst.handle_input(); the reference's Err is recorded (an empty Step is returned)."""
    try:
        return inst.handle_input()
    except ProtocolError as e:
        res.errors.append((kind, p, e))
        return Step()


def _replay(engine, kind, p, netinfo, doc_or_ct, senders, shares, res):
    """Re-run one instance with immediate combines (a fresh, non-recording verifier): its input,
    then every message it was handed, in order.  An Err of the reference is recorded in
    ``res.errors`` and handling continues, as a caller of the reference's handle_message would.
    Returns the instance's output (signature / plaintext) or None."""
    ver = BatchVerifier(engine)
    inst = ThresholdSign(netinfo, ver) if kind == "coin" else ThresholdDecrypt(netinfo, ver)
    output = None

    def run(call):
        nonlocal output
        try:
            step = call()
        except ProtocolError as e:
            res.errors.append((kind, p, e))
            return
        res.faults += [(kind, p, f) for f in step.fault_log]
        if step.output and output is None:
            output = step.output[0]

    if kind == "coin":
        inst.set_document_hash(doc_or_ct)
    else:
        inst.set_ciphertext(doc_or_ct)
    run(inst.handle_input)
    for j in senders:
        run(lambda: inst.handle_message(j, shares[(p, j)]))
    return output
