"""Host-side mirror of hbbft's ThresholdSign and ThresholdDecrypt message flows over the GPU engine.

Reference: ``src/threshold_sign.rs`` and ``src/threshold_decrypt.rs`` (the ``ConsensusProtocol``
instances of SURVEY.md §3.1/§3.2).  Same method names, argument meaning, error and fault
behaviour; the only change is *where the crypto runs*: every share check goes through a
``BatchVerifier`` -- the verdict cache / batch drain of SURVEY §8f f1 -- which verifies all
shares queued at the reference's own deferred-verification points (``remove_invalid_shares``)
or by a driver's pre-verification window in ONE C-ABI call, and combines run through
``hbh_interpolate_g2/g1``.  Verdicts are a pure function of (public key, hash point, share), so
caching them cannot change which ``Step`` a fault lands in.

What stays on the host, as in the reference and the north star: hashing to G2 (``set_document``
-> ``hash_g2``; ``set_ciphertext`` -> ``hash_g1_g2(U, V)``), secret-key operations (``sign_g2``,
``decrypt_share_no_verify``: ``NetworkInfo`` holds callables) and the XOR stream of
``PublicKeySet::decrypt`` -- all through the product host stage (``hbbft_amd.hoststage``, C++).
"""
import concurrent.futures
import time

from . import hoststage
from ._lib import G1_BYTES, G2_BYTES



# ------------------------------------------------------------------ Step / faults (src/traits.rs:64-74)
class Fault:
    def __init__(self, node_id, kind):
        self.node_id, self.kind = node_id, kind

    def __eq__(self, o):
        return isinstance(o, Fault) and (self.node_id, self.kind) == (o.node_id, o.kind)

    def __repr__(self):
        return "Fault(%r, %s)" % (self.node_id, self.kind)


class Step:
    """``Step { output, fault_log, messages }``; messages are (target, payload), target "all"."""
    __slots__ = ("output", "fault_log", "messages")

    def __init__(self, output=None, fault_log=None, messages=None):
        # the flows create ~30,000 Steps per epoch: no copies of the caller's lists (callers pass
        # fresh lists) and no per-instance dict
        self.output = [] if output is None else output
        self.fault_log = [] if fault_log is None else fault_log
        self.messages = [] if messages is None else messages

    @staticmethod
    def fault(node_id, kind):
        return Step(fault_log=[Fault(node_id, kind)])

    def extend(self, other):
        self.output += other.output
        self.fault_log += other.fault_log
        self.messages += other.messages
        return self

    join = extend

    def with_output(self, out):
        self.output.append(out)
        return self


class ProtocolError(Exception):
    """The reference's ``Error`` enums (``threshold_sign::Error``, ``threshold_decrypt::Error``)."""

    def __init__(self, kind, detail=None):
        super().__init__(kind if detail is None else "%s(%s)" % (kind, detail))
        self.kind, self.detail = kind, detail


# ------------------------------------------------------------------ keys (src/network_info.rs)
class NetworkInfo:
    """Node ids, the public key set and this node's secret-key operations.

    pk_shares: {node_id: G1 ABI bytes}; master_pk: G1 ABI bytes; t: num_faulty (the share-count
    gate of try_output); threshold: the PublicKeySet's polynomial degree, which sets how many shares
    are interpolated (combine_signatures / decrypt take threshold + 1; defaults to t as in
    NetworkInfo::generate_map, src/network_info.rs:174-215); sign_g2(H) / decrypt_share(U): this
    node's secret operations (None for an observer)."""

    def __init__(self, our_id, node_ids, t, master_pk, pk_shares, sign_g2=None, decrypt_share=None, threshold=None):
        self.our_id = our_id
        self._ids = sorted(node_ids)
        self._index = {n: i for i, n in enumerate(self._ids)}
        self.t = t
        self.threshold = t if threshold is None else threshold
        self.master_pk = master_pk
        self.pk_shares = dict(pk_shares)
        self.sign_g2 = sign_g2
        self.decrypt_share = decrypt_share

    def node_index(self, node_id):
        return self._index.get(node_id)

    def num_faulty(self):
        return self.t

    def pk_set_threshold(self):
        return self.threshold

    def public_key_share(self, node_id):
        return self.pk_shares.get(node_id)

    def is_validator(self):
        return self.sign_g2 is not None


# ------------------------------------------------------------------ verdict cache / batch drain
class Deferred:
    """A combine recorded by a BatchVerifier in deferred mode; ``flush_combines`` fills ``result``
    ((signature, status, verdict) for G2, (point, status) for G1).  ``data`` carries the
    ciphertext's V for a deferred decryption (the plaintext is xor_with_hash(result[0], data)).

    ``ok`` says whether the combine succeeded.  A deferred combine lets its instance terminate
    optimistically; when it failed, the reference would have returned ``Err`` from the call that
    triggered it and (ThresholdSign) stayed open, so the driver replays that instance's inputs with
    immediate combines (honey_badger.run_epoch) -- the Steps and errors are then the reference's."""
    __slots__ = ("key", "result", "data", "tag")

    def __init__(self, key, data=None):
        self.key, self.result, self.data, self.tag = key, None, data, None

    @property
    def ok(self):
        if self.result is None:
            raise RuntimeError("deferred combine not flushed")
        return self.result[1] == 0 and (len(self.result) == 2 or self.result[2])


class BatchVerifier:
    """Pure, order-independent verdict cache.  ``queue_*`` records checks; ``drain`` verifies every
    queued check in one engine call per kind; ``*_valid`` returns a cached verdict (or verifies a
    single miss immediately).  ``calls`` counts engine calls (the batching evidence in tests)."""

    def __init__(self, engine, combine_engine=None):
        self.eng = engine
        # combines on their own engine (stream) when given: a flow that combines while a
        # drain_async is in flight then does not wait for the drain's engine call
        self.ceng = combine_engine if combine_engine is not None else engine
        self._sig, self._dec, self._ct = {}, {}, {}
        self._qsig, self._qdec, self._qct = [], [], []
        self.calls = 0
        self.checks = 0
        self.max_batch = 0
        self.recording = False  # deferred mode: combines return Deferred, run later in one batch
        self.lookups = 0        # verdicts the flows consumed (the checks the reference performs)
        # the instances' store_cached / handle_fast transitions (one copy each, inside ThresholdSign,
        # ThresholdDecrypt and BinaryAgreementCoin); False routes every message through the full
        # handle_message path (run_epoch(fast_paths=False): the equivalence tests)
        self.shortcuts = True
        self._docs = {}
        self._rec_g2, self._rec_g1 = [], []
        # speculative G1 combines (honey_badger._dec_preverify): ciphertext key (H_uv, W) -> U * msk from
        # t + 1 shares whose verdicts are valid; any t + 1 valid decryption shares of one ciphertext
        # interpolate to that same point, so a deferred combine of the ciphertext takes it unchanged
        self._spec_g1 = {}
        self._released = set()  # instances released since the last drain was stored
        self._open = {}         # instance key -> number of running instances that use it
        self._inflight = 0      # drain_async calls not yet committed
        self.wait_s = 0.0       # time the calling thread spent blocked on engine calls (drains, combines)
        self.async_s = 0.0      # drain_async: time of the engine calls on the worker thread

    # -------------------------------------------------------------- host hashing
    def hash_docs(self, docs):
        """hash_g2 of many documents in one threaded host-stage call (cached for set_document)."""
        docs = [bytes(d) for d in docs if bytes(d) not in self._docs]
        for d, h in zip(docs, hoststage.hash_g2(docs) if docs else []):
            self._docs[d] = h

    def add_doc_hashes(self, hashes):
        """Documents hashed elsewhere ({document: hash_g2(document)}, e.g. prefetched by
        honey_badger.prefetch_coins) into the hash_docs cache."""
        for d, h in hashes.items():
            self._docs.setdefault(bytes(d), h)

    def hash_doc(self, doc):
        doc = bytes(doc)
        h = self._docs.pop(doc, None)
        return h if h is not None else hoststage.hash_g2([doc])[0]

    def doc_hash_of(self, doc):
        """hash_g2(doc) from the hash_docs cache (kept for a later set_document), or hashed now."""
        doc = bytes(doc)
        h = self._docs.get(doc)
        if h is None:
            h = self._docs[doc] = hoststage.hash_g2([doc])[0]
        return h

    # -------------------------------------------------------------- combines
    def combine_verify_g2(self, t, idx, shares, master_pk, h):
        """combine_and_verify_sig's crypto (src/threshold_sign.rs:249-270): (signature, status,
        verdict) from the cache, or one engine call.  While recording, the request is noted and a
        valid placeholder is returned (the state machine does not depend on the signature)."""
        key = (t, tuple(idx), tuple(bytes(s) for s in shares), bytes(master_pk), bytes(h))
        if self.recording:
            d = Deferred(key)
            self._rec_g2.append(d)
            return d, 0, True
        t0 = time.perf_counter()
        out, st, v = self.ceng.combine_verify_g2(t, [list(idx)], [list(shares)], master_pk, [h])
        self.wait_s += time.perf_counter() - t0
        self.calls += 1
        return out[0], st[0], bool(v[0])

    def interpolate_g1(self, t, idx, shares):
        """PublicKeySet::decrypt's interpolation (src/threshold_decrypt.rs:242-250): (point, status)."""
        key = (t, tuple(idx), tuple(bytes(s) for s in shares))
        if self.recording:
            d = Deferred(key)
            self._rec_g1.append(d)
            return d, 0
        t0 = time.perf_counter()
        out, st = self.ceng.interpolate_g1(t, [list(idx)], [list(shares)])
        self.wait_s += time.perf_counter() - t0
        self.calls += 1
        return out[0], st[0]

    def flush_combines(self):
        """Run every deferred combine: one engine call per (t, master key) for G2 and per t for G1;
        fills each Deferred's result; returns the Deferreds whose combine failed."""
        t0 = time.perf_counter()
        groups = {}
        for d in self._rec_g2:
            groups.setdefault((d.key[0], d.key[3]), []).append(d)
        for (t, mpk), ds in groups.items():
            out, st, v = self.ceng.combine_verify_g2(t, [list(d.key[1]) for d in ds], [list(d.key[2]) for d in ds],
                                                    mpk, [d.key[4] for d in ds])
            self.calls += 1
            for d, o, s_, vv in zip(ds, out, st, v):
                d.result = (o, s_, bool(vv))
        groups = {}
        for d in self._rec_g1:
            pt = self._spec_g1.get(d.tag) if d.tag is not None else None
            if pt is not None and len(set(d.key[1])) == len(d.key[1]):  # (a repeated index: compute)
                d.result = (pt, 0)
                continue
            groups.setdefault(d.key[0], []).append(d)
        for t, ds in groups.items():
            out, st = self.ceng.interpolate_g1(t, [list(d.key[1]) for d in ds], [list(d.key[2]) for d in ds])
            self.calls += 1
            for d, o, s_ in zip(ds, out, st):
                d.result = (o, s_)
        self.wait_s += time.perf_counter() - t0
        failed = [d for d in self._rec_g2 + self._rec_g1 if not d.ok]
        self._rec_g2, self._rec_g1 = [], []
        return failed

    def add_speculative_g1(self, points):
        """{(H_uv, W): G1 point} combined early from verified decryption shares (see _spec_g1)."""
        self._spec_g1.update(points)

    # Instances are reference-counted by their key (document hash; (H_uv, W) for a ciphertext):
    # two running instances may share one (a Byzantine proposer can copy another's ciphertext, two
    # BA instances could sign the same document), and a release drops the cached verdicts only
    # when the last of them terminates.
    def open_doc(self, h):
        self._open_key(bytes(h))

    def open_ct(self, huv, w):
        self._open_key((bytes(huv), bytes(w)))

    def _open_key(self, key):
        self._open[key] = self._open.get(key, 0) + 1
        self._released.discard(key)

    def _close_key(self, key):
        """True when the last running instance of ``key`` is gone."""
        n = self._open.get(key, 0) - 1
        if n > 0:
            self._open[key] = n
            return False
        self._open.pop(key, None)
        self._released.add(key)
        return True

    def release_doc(self, h):
        """A ThresholdSign instance (document hash h) terminated: drop the cached verdicts if no
        other running instance signs the same document."""
        if self._close_key(bytes(h)):
            self._sig.pop(bytes(h), None)

    def release_ct(self, huv, w):
        """A ThresholdDecrypt instance terminated (or its ciphertext was rejected): drop the cached
        verdicts if no other running instance holds the same ciphertext."""
        key = (bytes(huv), bytes(w))
        if self._close_key(key):
            self._dec.pop(key, None)
            self._ct.pop(key, None)

    def cached(self):
        return (sum(len(d) for d in self._sig.values()) + sum(len(d) for d in self._dec.values())
                + sum(len(d) for d in self._ct.values()))

    # Verdicts are kept per instance (document hash / ciphertext) so that a terminated instance's
    # entries are released in O(1).
    # ThresholdSign: PublicKeyShare::verify_g2(share, H)  (src/threshold_sign.rs:223)
    def queue_sig(self, pk, h, share):
        if type(h) is not bytes:
            h = bytes(h)
        if type(pk) is not bytes:
            pk = bytes(pk)
        if type(share) is not bytes:
            share = bytes(share)
        if (pk, share) not in self._sig.get(h, ()):
            self._qsig.append((pk, h, share))

    def cached_sig(self, pk, h, share):
        """The cached verdict of a share check, or None (no engine call)."""
        return self._sig.get(bytes(h), {}).get((bytes(pk), bytes(share)))

    def sig_valid(self, pk, h, share):
        self.lookups += 1
        if type(h) is not bytes:
            h = bytes(h)
        k = (pk if type(pk) is bytes else bytes(pk), share if type(share) is bytes else bytes(share))
        d = self._sig.get(h)
        v = d.get(k) if d is not None else None
        if v is None:
            self._qsig.append((k[0], h, k[1]))
            v = self._drain(("sig", h, k))
        return v

    # ThresholdDecrypt: PublicKeyShare::verify_decryption_share(share, ct)  (src/threshold_decrypt.rs:227)
    def queue_dec(self, pk, share, huv, w):
        if type(pk) is not bytes:
            pk = bytes(pk)
        if type(share) is not bytes:
            share = bytes(share)
        c = (huv if type(huv) is bytes else bytes(huv), w if type(w) is bytes else bytes(w))
        if (pk, share) not in self._dec.get(c, ()):
            self._qdec.append((pk, share) + c)

    def dec_valid(self, pk, share, huv, w):
        self.lookups += 1
        c = (huv if type(huv) is bytes else bytes(huv), w if type(w) is bytes else bytes(w))
        k = (pk if type(pk) is bytes else bytes(pk), share if type(share) is bytes else bytes(share))
        d = self._dec.get(c)
        v = d.get(k) if d is not None else None
        if v is None:
            self._qdec.append(k + c)
            v = self._drain(("dec", c, k))
        return v

    # Ciphertext::verify  (src/threshold_decrypt.rs:142)
    def queue_ct(self, ct):
        c, u = (bytes(ct.huv), bytes(ct.w)), bytes(ct.u)
        if u not in self._ct.get(c, ()):
            self._qct.append((u, c[1], c[0]))

    def ct_valid(self, ct):
        self.lookups += 1
        c, u = (bytes(ct.huv), bytes(ct.w)), bytes(ct.u)
        v = self._ct.get(c, {}).get(u)
        if v is None:
            self._qct.append((u, c[1], c[0]))
            v = self._drain(("ct", c, u))
        return v

    def drain(self):
        """Verify everything queued: one engine call per kind."""
        self._drain(None)

    def _drain(self, want):
        jobs = self._take_jobs()
        if not jobs:
            if not self._inflight:
                self._released.clear()
            return None
        t0 = time.perf_counter()
        res = self._run_jobs(jobs)
        self.wait_s += time.perf_counter() - t0
        return self._store(res, want)

    def drain_async(self):
        """Start verifying everything queued on a worker thread (one engine call per kind, the
        calls release the GIL) and return a handle for ``commit``.  Meanwhile the flows may handle
        messages whose verdicts are already cached: a windowed driver overlaps the GPU drain of
        window k with the host handling of window k - 1 (honey_badger._deliver)."""
        global _POOL
        jobs = self._take_jobs()
        self._inflight += 1
        if _POOL is None:
            _POOL = concurrent.futures.ThreadPoolExecutor(max_workers=1, thread_name_prefix="hbh-drain")
        return _POOL.submit(self._run_jobs_timed, jobs)

    def _run_jobs_timed(self, jobs):
        t0 = time.perf_counter()
        try:
            return self._run_jobs(jobs)
        finally:
            self.async_s += time.perf_counter() - t0

    def commit(self, pending):
        """Wait for a ``drain_async`` and cache its verdicts."""
        t0 = time.perf_counter()
        try:
            res = pending.result()
        finally:
            self.wait_s += time.perf_counter() - t0
            self._inflight -= 1
        self._store(res)

    def _take_jobs(self):
        """Snapshot the queues as engine-call arguments (main thread)."""
        jobs = []
        if self._qct:
            keys = list(dict.fromkeys(self._qct))
            self._qct = []
            jobs.append(("ct", keys, ([k[0] for k in keys], [k[1] for k in keys], [k[2] for k in keys])))
        if self._qsig:
            keys = list(dict.fromkeys(self._qsig))
            self._qsig = []
            hs = list(dict.fromkeys(k[1] for k in keys))
            hidx = {h: i for i, h in enumerate(hs)}
            jobs.append(("sig", keys, ([k[0] for k in keys], [k[2] for k in keys], hs, [hidx[k[1]] for k in keys])))
        if self._qdec:
            keys = list(dict.fromkeys(self._qdec))
            self._qdec = []
            cts = list(dict.fromkeys((k[2], k[3]) for k in keys))
            cidx = {c: i for i, c in enumerate(cts)}
            jobs.append(("dec", keys, ([k[1] for k in keys], [k[0] for k in keys], [c[0] for c in cts],
                                       [c[1] for c in cts], [cidx[(k[2], k[3])] for k in keys])))
        return jobs

    def _run_jobs(self, jobs):
        """The engine calls of a snapshot (any thread): [(kind, keys, verdict bytes)]."""
        fn = {"ct": "verify_ciphertexts", "sig": "verify_sig_shares", "dec": "verify_dec_shares"}
        return [(kind, keys, getattr(self.eng, fn[kind])(*args)) for kind, keys, args in jobs]

    def _store(self, results, want=None):
        """Cache verdicts (main thread).  Verdicts of instances whose last running instance
        terminated while the drain was in flight are not cached, so a terminated instance leaves
        nothing behind.  want = (kind, instance key, item key): that verdict is returned (a
        synchronous *_valid reads its verdict from here even when no running instance keeps it)."""
        rel = self._released
        got = None
        for kind, keys, v in results:
            self._count(len(keys))
            if kind == "sig":
                cache = self._sig
                for k, ok in zip(keys, v):
                    h = k[1]
                    d = cache.get(h)
                    if d is None:  # an existing entry is never a released instance's (release pops it)
                        if h in rel:
                            continue
                        d = cache[h] = {}
                    d[(k[0], k[2])] = ok == 1
            elif kind == "dec":
                cache = self._dec
                for k, ok in zip(keys, v):
                    c = (k[2], k[3])
                    d = cache.get(c)
                    if d is None:
                        if c in rel:
                            continue
                        d = cache[c] = {}
                    d[(k[0], k[1])] = ok == 1
            else:
                cache = self._ct
                for k, ok in zip(keys, v):
                    c = (k[2], k[1])
                    d = cache.get(c)
                    if d is None:
                        if c in rel:
                            continue
                        d = cache[c] = {}
                    d[k[0]] = ok == 1
            if want is not None and want[0] == kind:
                for k, ok in zip(keys, v):
                    if self._item(kind, k) == want[1:]:
                        got = ok == 1
                        break
        # nothing queued after the last release can name the released instance (the drivers
        # queue only for running instances), so the set only has to outlive the drains in flight
        if not self._inflight:
            self._released.clear()
        return got

    @staticmethod
    def _item(kind, k):
        """(instance key, item key) of a queued check."""
        if kind == "sig":
            return k[1], (k[0], k[2])
        if kind == "dec":
            return (k[2], k[3]), (k[0], k[1])
        return (k[2], k[1]), k[0]

    def _count(self, n):
        self.calls += 1
        self.checks += n
        self.max_batch = max(self.max_batch, n)


_POOL = None  # one worker thread for drain_async (engine calls are serialised per engine anyway)


# ------------------------------------------------------------------ ThresholdSign (src/threshold_sign.rs)
class ThresholdSign:
    def __init__(self, netinfo, verifier):
        self.netinfo = netinfo
        self.verifier = verifier
        self.doc_hash = None
        self.received_shares = {}  # node_id -> (idx, share); BTreeMap order = sorted ids
        self.unverified = False    # a share was stored before the document was set (not checked)
        self.had_input = False
        self.terminated = False

    def set_document(self, doc):
        """``set_document`` (:147-153): H = hash_g2(doc) on the host (hbh_hash_g2)."""
        if self.doc_hash is not None:
            raise ProtocolError("MultipleMessagesToSign")
        self.doc_hash = self.verifier.hash_doc(doc)
        self.verifier.open_doc(self.doc_hash)

    def set_document_hash(self, h):
        """``set_document`` with H already computed, e.g. by a driver that hashes the documents of
        many instances in one hbh_hash_g2 batch."""
        if self.doc_hash is not None:
            raise ProtocolError("MultipleMessagesToSign")
        self.doc_hash = bytes(h)
        self.verifier.open_doc(self.doc_hash)

    def handle_input(self):
        return self.sign()

    def sign(self):  # :157-178
        if self.had_input:
            return Step()
        if self.doc_hash is None:
            raise ProtocolError("DocumentHashIsNone")
        self.had_input = True
        step = Step()
        step.fault_log += self.remove_invalid_shares()
        if not self.netinfo.is_validator():
            return step.join(self.try_output())
        share = self.netinfo.sign_g2(self.doc_hash)
        step.messages.append(("all", share))
        return step.extend(self.handle_message(self.netinfo.our_id, share))

    def store_cached(self, sender_id, share):
        """handle_message's most common transition without building its Step (:181-197): the document
        is set, the sender is new, the verifier already holds a VALID verdict for the share, and
        storing it leaves the instance at <= t shares -- the share is stored, True is returned, and
        handle_message's result would have been an empty Step.  Otherwise (or with the verifier's
        shortcuts off) nothing changes and False is returned: handle_message decides."""
        rs, h, ver = self.received_shares, self.doc_hash, self.verifier
        if self.terminated or h is None or sender_id in rs or type(share) is not bytes or not ver.shortcuts:
            return False
        ni = self.netinfo
        if len(rs) >= ni.t:
            return False
        d = ver._sig.get(h)
        pk = ni.pk_shares.get(sender_id)
        if d is None or type(pk) is not bytes or d.get((pk, share)) is not True:
            return False
        idx = ni._index.get(sender_id)
        if idx is None:
            return False
        ver.lookups += 1  # the verdict consumed, as sig_valid counts it
        rs[sender_id] = (idx, share)
        return True

    def handle_message(self, sender_id, share):  # :181-197
        if self.terminated or self.store_cached(sender_id, share):
            return Step()
        ni = self.netinfo
        idx = ni._index.get(sender_id)  # node_index
        if idx is None:
            raise ProtocolError("UnknownSender")
        # is_share_valid (:216-225), inlined on this per-message path
        if self.doc_hash is not None:
            pk = ni.pk_shares.get(sender_id)
            if pk is None or not self.verifier.sig_valid(pk, self.doc_hash, share):
                return Step.fault(sender_id, "UnverifiedSignatureShareSender")
        self.received_shares[sender_id] = (idx, share if type(share) is bytes else bytes(share))
        if self.doc_hash is None:
            self.unverified = True
        if self.doc_hash is None or len(self.received_shares) <= ni.t:  # try_output's gate (:227-247)
            return Step()
        return self.try_output()

    def remove_invalid_shares(self):  # :200-213 -- the natural batch point: one drain
        if self.doc_hash is not None and not self.unverified:
            # every stored share passed is_share_valid when it arrived with the document set, and
            # verdicts are pure: nothing to remove
            return []
        for sid, (_, share) in self.received_shares.items():
            pk = self.netinfo.public_key_share(sid)
            if self.doc_hash is not None and pk is not None:
                self.verifier.queue_sig(pk, self.doc_hash, share)
        self.verifier.drain()
        faulty = [sid for sid, (_, share) in sorted(self.received_shares.items())
                  if not self.is_share_valid(sid, share)]
        for sid in faulty:
            del self.received_shares[sid]
        if self.doc_hash is not None:
            self.unverified = False
        return [Fault(sid, "UnverifiedSignatureShareSender") for sid in faulty]

    def is_share_valid(self, sender_id, share):  # :216-225
        if self.doc_hash is None:
            return True
        pk = self.netinfo.public_key_share(sender_id)
        if pk is None:
            return False
        return self.verifier.sig_valid(pk, self.doc_hash, share)

    def try_output(self):  # :227-247
        if self.doc_hash is None:
            return Step()
        if not self.terminated and len(self.received_shares) > self.netinfo.num_faulty():
            sig = self.combine_and_verify_sig()
            self.terminated = True
            step = self.sign()
            self.verifier.release_doc(self.doc_hash)
            return step.with_output(sig)
        return Step()

    def combine_and_verify_sig(self):  # :249-270
        t = self.netinfo.pk_set_threshold()
        items = [self.received_shares[k] for k in sorted(self.received_shares)][: t + 1]
        sig, st, ok = self.verifier.combine_verify_g2(t, [i for i, _ in items], [s for _, s in items],
                                                      self.netinfo.master_pk, self.doc_hash)
        if st != 0:
            raise ProtocolError("CombineAndVerifySigCrypto", "DuplicateEntry")
        if not ok:
            raise ProtocolError("VerificationFailed")
        return sig


# ------------------------------------------------------------------ ThresholdDecrypt (src/threshold_decrypt.rs)
def g1_compress_abi(p):
    """ABI G1 bytes -> the 48-byte compressed encoding (hbh_g1_compress)."""
    return hoststage.g1_compress([bytes(p)])[0]


def xor_with_hash(g1_abi, data):
    """threshold_crypto ``xor_with_hash(g, V)`` on the host stage (hbh_xor_with_hash)."""
    return hoststage.xor_with_hash([bytes(g1_abi)], [bytes(data)])[0]


def signature_parity(sig):
    """``Signature::parity`` -- the coin value of Binary Agreement (binary_agreement.rs:402)."""
    return hoststage.signature_parity([bytes(sig)])[0]


class Ciphertext:
    """(U in G1, V bytes, W in G2) plus H_uv = hash_g1_g2(U, V), hashed once on the host (the
    reference rehashes it in every check; the value is the same)."""

    def __init__(self, u, v, w, huv=None):
        self.u, self.v, self.w = bytes(u), bytes(v), bytes(w)
        self.huv = bytes(huv) if huv is not None else hoststage.hash_g1_g2([self.u], [self.v])[0]


class ThresholdDecrypt:
    def __init__(self, netinfo, verifier):
        self.netinfo = netinfo
        self.verifier = verifier
        self.ciphertext = None
        self.shares = {}
        self.had_input = False
        self.terminated = False

    def set_ciphertext(self, ct):  # :138-147
        if self.ciphertext is not None:
            raise ProtocolError("MultipleInputs")
        self.verifier.open_ct(ct.huv, ct.w)
        if not self.verifier.ct_valid(ct):
            self.verifier.release_ct(ct.huv, ct.w)
            raise ProtocolError("InvalidCiphertext")
        self.ciphertext = ct

    def handle_input(self):
        return self.start_decryption()

    def start_decryption(self):  # :151-170
        if self.had_input:
            return Step()
        if self.ciphertext is None:
            raise ProtocolError("CiphertextIsNone")
        self.had_input = True
        step = Step()
        step.fault_log += self.remove_invalid_shares()
        if self.netinfo.decrypt_share is None:
            return step.join(self.try_output())
        share = self.netinfo.decrypt_share(self.ciphertext.u)
        our = self.netinfo.our_id
        self.shares[our] = (self.netinfo.node_index(our), bytes(share))  # own share: not verified (:167)
        step.messages.append(("all", share))
        return step.join(self.try_output())

    def store_cached(self, sender_id, share):
        """handle_message's most common transition without building its Step (:182-201): the
        ciphertext is set, the sender is new (no MultipleDecryptionShares), the verifier already holds
        a VALID verdict for the share, and storing it leaves the instance at <= t shares -- stored,
        True returned (handle_message would return an empty Step).  Otherwise (or with the verifier's
        shortcuts off) nothing changes and False is returned: handle_message decides."""
        sh, ct, ver = self.shares, self.ciphertext, self.verifier
        if self.terminated or ct is None or sender_id in sh or type(share) is not bytes or not ver.shortcuts:
            return False
        ni = self.netinfo
        if len(sh) >= ni.t:
            return False
        d = ver._dec.get((ct.huv, ct.w))
        pk = ni.pk_shares.get(sender_id)
        if d is None or type(pk) is not bytes or d.get((pk, share)) is not True:
            return False
        idx = ni._index.get(sender_id)
        if idx is None:
            return False
        ver.lookups += 1  # the verdict consumed, as dec_valid counts it
        sh[sender_id] = (idx, share)
        return True

    def handle_message(self, sender_id, share):  # :182-201
        if self.terminated or self.store_cached(sender_id, share):
            return Step()
        ni = self.netinfo
        idx = ni._index.get(sender_id)  # node_index
        if idx is None:
            raise ProtocolError("UnknownSender")
        ct = self.ciphertext
        if ct is not None:  # is_share_valid (:220-229), inlined on this per-message path
            pk = ni.pk_shares.get(sender_id)
            if pk is None or not self.verifier.dec_valid(pk, share, ct.huv, ct.w):
                return Step.fault(sender_id, "UnverifiedDecryptionShareSender")
        dup = sender_id in self.shares
        self.shares[sender_id] = (idx, share if type(share) is bytes else bytes(share))
        if dup:
            return Step.fault(sender_id, "MultipleDecryptionShares")
        if len(self.shares) <= ni.t:  # try_output's gate (:232-252)
            return Step()
        return self.try_output()

    def remove_invalid_shares(self):  # :204-217 -- one drain for every share received early
        ct = self.ciphertext
        for sid, (_, share) in self.shares.items():
            pk = self.netinfo.public_key_share(sid)
            if ct is not None and pk is not None:
                self.verifier.queue_dec(pk, share, ct.huv, ct.w)
        self.verifier.drain()
        faulty = [sid for sid, (_, share) in sorted(self.shares.items()) if not self.is_share_valid(sid, share)]
        for sid in faulty:
            del self.shares[sid]
        return [Fault(sid, "UnverifiedDecryptionShareSender") for sid in faulty]

    def is_share_valid(self, sender_id, share):  # :220-229
        ct = self.ciphertext
        if ct is None:
            return True
        pk = self.netinfo.public_key_share(sender_id)
        if pk is None:
            return False
        return self.verifier.dec_valid(pk, share, ct.huv, ct.w)

    def try_output(self):  # :232-252
        if self.terminated or len(self.shares) <= self.netinfo.num_faulty():
            return Step()
        if self.ciphertext is None:
            return Step()
        self.terminated = True
        step = self.start_decryption()
        self.verifier.release_ct(self.ciphertext.huv, self.ciphertext.w)
        t = self.netinfo.pk_set_threshold()
        items = [self.shares[k] for k in sorted(self.shares)][: t + 1]
        g, st = self.verifier.interpolate_g1(t, [i for i, _ in items], [s for _, s in items])
        if st != 0:
            raise ProtocolError("Decryption", "DuplicateEntry")
        if isinstance(g, Deferred):
            g.data = self.ciphertext.v
            g.tag = (self.ciphertext.huv, self.ciphertext.w)
            return step.with_output(g)
        return step.with_output(xor_with_hash(g, self.ciphertext.v))


__all__ = ["Fault", "Step", "ProtocolError", "NetworkInfo", "BatchVerifier", "ThresholdSign",
           "ThresholdDecrypt", "Ciphertext", "xor_with_hash", "g1_compress_abi", "signature_parity", "G1_BYTES",
           "G2_BYTES"]
