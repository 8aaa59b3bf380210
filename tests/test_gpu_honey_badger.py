"""HoneyBadger epoch crypto trace (BASELINE configs[4]) through the mirrored flows on the GPU
engine: every decrypted contribution equals the proposal byte for byte, every coin signature is
msk * hash_g2(coin document) (C oracle) with the oracle's parity, only forged shares are blamed,
and the windowed drains give the same result as per-message verification (window = 1).
References: examples/simulation.rs:164-177, 296-316; src/honey_badger/epoch_state.rs:376-395;
src/binary_agreement/binary_agreement.rs:245-264, 395-405, 437-448."""
import random

import pytest

from oracle import cbls, tc
from hbbft_amd.honey_badger import EpochTrace, NetworkKeys, coin_document, run_epoch

pytestmark = pytest.mark.gpu


def parity_oracle(sig):
    x0, x1, y0, y1 = (int.from_bytes(sig[o:o + 48], "little") for o in (0, 48, 96, 144))
    return tc.signature_parity(((x0, x1), (y0, y1)))


def check(trace, res, keys):
    assert res.plaintexts == trace.proposals
    assert sorted(res.coins) == sorted(trace.coin_docs)
    for p, sig in res.signatures.items():
        assert sig == cbls.g2_mul(trace.hashes[p], keys.msk)
        assert res.coins[p] == parity_oracle(sig)
    for kind, p, flt in res.faults:
        assert (kind, p, flt.node_id) in trace.bad
        assert flt.kind == ("UnverifiedSignatureShareSender" if kind == "coin" else "UnverifiedDecryptionShareSender")


def test_coin_document_layout():
    d = coin_document(7, 3, 2, 5)
    assert len(d) == 28 and d[:8] == (7).to_bytes(8, "little") and d[16:20] == (2).to_bytes(4, "little")


@pytest.mark.parametrize("n", [4, 7])
def test_epoch_small_and_window_equivalence(engine, n):
    t = (n - 1) // 3
    rng = random.Random(300 + n)
    keys = NetworkKeys(engine, n, t, rng)
    trace = EpochTrace.generate(engine, keys, rng, hb_epoch=1, bad_every=5, proposal_bytes=100)
    big = run_epoch(engine, keys, trace, window=1 << 20)
    check(trace, big, keys)
    one = run_epoch(engine, keys, trace, window=1, pipelined=False, preverify=False)
    check(trace, one, keys)
    assert (one.plaintexts, one.coins, one.signatures) == (big.plaintexts, big.coins, big.signatures)
    assert [(k, p, f.node_id, f.kind) for k, p, f in one.faults] == [(k, p, f.node_id, f.kind) for k, p, f in big.faults]
    # per-message verification checks exactly what the flows consume; the big window batches
    assert one.checks_gpu == one.checks_consumed
    # decryption shares pre-verified beside the coin phase: same steps, at most t + 1 + slack extra
    # checks per instance, and the consumed checks are the per-message run's
    pre = run_epoch(engine, keys, trace, window=1, pipelined=False, preverify=True)
    check(trace, pre, keys)
    assert (pre.plaintexts, pre.coins, pre.signatures) == (big.plaintexts, big.coins, big.signatures)
    assert [(k, p, f.node_id, f.kind) for k, p, f in pre.faults] == [(k, p, f.node_id, f.kind) for k, p, f in big.faults]
    assert pre.checks_consumed == one.checks_consumed and pre.checks_gpu >= one.checks_gpu
    assert big.engine_calls < one.engine_calls
    # pipelined small windows (drain k on the GPU while window k - 1 is handled): same steps
    for w in (1, 3):
        pip = run_epoch(engine, keys, trace, window=w, pipelined=True)
        check(trace, pip, keys)
        assert (pip.plaintexts, pip.coins, pip.signatures) == (big.plaintexts, big.coins, big.signatures)
        assert [(k, p, f.node_id, f.kind) for k, p, f in pip.faults] == [(k, p, f.node_id, f.kind) for k, p, f in big.faults]
        assert pip.checks_gpu >= pip.checks_consumed


def test_epoch_n100_f33(engine):
    """configs[4] at full size: N=100, f=33, every BA instance flips one threshold coin."""
    rng = random.Random(100)
    keys = NetworkKeys(engine, 100, 33, rng)
    trace = EpochTrace.generate(engine, keys, rng, hb_epoch=0, proposal_bytes=1000)
    res = run_epoch(engine, keys, trace, window=4096)
    check(trace, res, keys)
    assert len(res.plaintexts) == 100 and len(res.coins) == 100
    assert res.engine_calls <= 16
    ser = run_epoch(engine, keys, trace, window=4096, pipelined=False)
    assert (ser.plaintexts, ser.coins, ser.signatures) == (res.plaintexts, res.coins, res.signatures)
    assert [(k, p, f.node_id) for k, p, f in ser.faults] == [(k, p, f.node_id) for k, p, f in res.faults]
    print("epoch N=100: %.3f s, %d engine calls, %d checks drained, %d consumed, timing %s" % (
        res.timing["epoch"], res.engine_calls, res.checks_gpu, res.checks_consumed,
        {k: round(v, 4) for k, v in res.timing.items()}))


def test_failed_deferred_combine_is_replayed(engine):
    """A combine that fails (here: the signing NetworkInfo's master key does not match the key
    shares, so every combined signature fails PublicKey::verify) must surface as the reference's
    Err(VerificationFailed) in the owning instance, which stays open (threshold_sign.rs:227-270),
    not as an output.  The deferred epoch equals the immediate-combine epoch (defer=False)."""
    n, t = 4, 1
    rng = random.Random(404)
    keys = NetworkKeys(engine, n, t, rng)
    trace = EpochTrace.generate(engine, keys, rng, hb_epoch=2, bad_every=5, proposal_bytes=80)
    keys.master_pk = keys.pks[1]  # wrong master key: coins cannot verify; decryption is unaffected
    dfr = run_epoch(engine, keys, trace, window=1 << 20)
    imm = run_epoch(engine, keys, trace, window=1 << 20, defer=False)
    assert dfr.coins == {} and dfr.signatures == {}
    assert dfr.plaintexts == trace.proposals
    assert {p for k, p, e in dfr.errors} == set(trace.coin_docs)
    assert all(k == "coin" and e.kind == "VerificationFailed" for k, p, e in dfr.errors)
    key = lambda r: (sorted((k, p, e.kind) for k, p, e in r.errors),
                     sorted((k, p, f.node_id, f.kind) for k, p, f in r.faults))
    assert key(dfr) == key(imm)
    assert (imm.plaintexts, imm.coins) == (dfr.plaintexts, dfr.coins)


def max_faulty(n):  # src/util.rs:22-25
    return (n - 1) // 3


@pytest.mark.parametrize("adversary", ["silent", "faulty_share", "random"])
def test_epoch_adversaries_different_sizes(engine, adversary):
    """tests/honey_badger.rs:191-245 through the GPU verifier: network sizes 1, 2, 3, 5 and one of
    6..9 with max_faulty(size) adversarial nodes that propose nothing and send no correct share --
    SilentAdversary, FaultyShareAdversary (every adversarial node broadcasts, for every proposer,
    its decryption share of a fake ciphertext) and RandomAdversary (random coin / decryption shares
    injected from adversarial senders).  Every contribution decrypts to its proposal, every coin is
    msk * H with the oracle's parity, only adversarial senders are ever blamed, and the windowed
    pipelined epoch equals per-message handling (window 1)."""
    rng = random.Random({"silent": 71, "faulty_share": 72, "random": 73}[adversary])
    sizes = [1, 2, 3, 5, rng.randrange(6, 10)]
    blamed_total = 0
    for size in sizes:
        f = max_faulty(size)
        keys = NetworkKeys(engine, size, f, rng)
        trace = EpochTrace.generate(engine, keys, rng, hb_epoch=len(sizes), bad_every=None, proposal_bytes=40,
                                    n_adv=f, adversary=adversary, inject=0.5)
        res = run_epoch(engine, keys, trace, window=5)
        check(trace, res, keys)
        assert sorted(res.plaintexts) == list(range(size - f))
        assert all(flt.node_id >= size - f for _, _, flt in res.faults), (size, res.faults)
        assert res.errors == []
        one = run_epoch(engine, keys, trace, window=1, pipelined=False)
        assert (one.plaintexts, one.coins, one.signatures) == (res.plaintexts, res.coins, res.signatures)
        assert sorted((k, p, x.node_id) for k, p, x in one.faults) == sorted((k, p, x.node_id) for k, p, x in res.faults)
        blamed_total += len(res.faults)
    if adversary == "silent":
        assert blamed_total == 0
    else:
        assert blamed_total > 0


def test_epoch_random_adversary_raw_bytes(engine):
    """RandomAdversary on the wire (tests/honey_badger.rs:235-245): the node receives bincode bytes;
    injected messages are random shares or bytes that do not decode (truncated, or a compressed x
    off the curve).  Undecodable messages are DeserializeMessage faults of their (adversarial)
    senders, decodable forged shares UnverifiedDecryptionShareSender / UnverifiedSignatureShareSender;
    outputs equal the proposals and the oracle's coins."""
    rng = random.Random(745)
    n, f = 7, 2
    keys = NetworkKeys(engine, n, f, rng)
    trace = EpochTrace.generate(engine, keys, rng, hb_epoch=3, bad_every=None, proposal_bytes=64, n_adv=f,
                                adversary="random", inject=0.5)
    injected = sorted(trace.bad)
    garbage = injected[::3]
    trace.serialize(corrupt=garbage)
    res = run_epoch(engine, keys, trace, window=6, raw=True)
    assert res.plaintexts == trace.proposals
    for p, sig in res.signatures.items():
        assert sig == cbls.g2_mul(trace.hashes[p], keys.msk)
        assert res.coins[p] == parity_oracle(sig)
    kinds = {"coin": "UnverifiedSignatureShareSender", "dec": "UnverifiedDecryptionShareSender"}
    assert res.faults
    for kind, p, flt in res.faults:
        assert (kind, p, flt.node_id) in trace.bad and flt.node_id >= n - f
        want = "DeserializeMessage" if (kind, p, flt.node_id) in garbage else kinds[kind]
        assert flt.kind == want, (kind, p, flt)
    # every undecodable message is blamed whether or not its instance is still running
    assert {(k, p, x.node_id) for k, p, x in res.faults if x.kind == "DeserializeMessage"} == set(garbage)


@pytest.mark.parametrize("n,extra", [(7, 0.5), (13, 0.3)])
def test_epoch_coins_through_binary_agreement(engine, n, extra):
    """The epoch's coins from Binary Agreement instances (hbbft_amd/binary_agreement.py) instead of a
    synthetic coin set: epochs 0 and 1 end on both values, epoch 2 flips the threshold coin and
    decides -- or, for a share of the instances, disagrees and runs on to epoch 5's coin.  Coin
    shares of epochs the instance has not reached wait in its future-epoch queue
    (binary_agreement.rs:245-266) and are replayed when it gets there (:489-519); coin combines are
    deferred per window and resume the BA state machines.  Decisions and threshold coins equal the
    schedule's (coins from msk * hash_g2(coin document), oracle parity); plaintexts equal the
    proposals; only forged shares are blamed; window 1 unpipelined gives the same result."""
    t = (n - 1) // 3
    rng = random.Random(800 + n)
    keys = NetworkKeys(engine, n, t, rng)
    trace = EpochTrace.generate(engine, keys, rng, hb_epoch=4, bad_every=9, proposal_bytes=60)
    trace.with_ba(engine, rng, extra=extra, bad_every=9)
    ba = trace.ba
    assert any(len(s) > 3 for s in ba.sched.values())  # some instances need a second threshold coin
    res = run_epoch(engine, keys, trace, window=16)
    assert res.errors == []
    assert res.plaintexts == trace.proposals
    assert res.ba_decisions == ba.decision
    assert res.ba_coins == ba.coins
    assert res.ba_queued > 0
    for p, sig in res.signatures.items():
        assert sig == cbls.g2_mul(trace.hashes[p], keys.msk)
        assert res.coins[p] == parity_oracle(sig) == ba.coins[p][2]
    for kind, p, flt in res.faults:
        assert (kind, p, flt.node_id) in (trace.bad | ba.bad), (kind, p, flt)
    one = run_epoch(engine, keys, trace, window=1, pipelined=False)
    assert (one.ba_decisions, one.ba_coins, one.plaintexts) == (res.ba_decisions, res.ba_coins, res.plaintexts)


def test_preverify_one_call_matches_separate_calls(engine):
    """honey_badger._one_call: the ciphertext checks ride as extra rows of the decryption-share call
    (e(U, H) == e(g1, W) in share-check form); the verdicts equal verify_ciphertexts' and
    verify_dec_shares' separate calls, incl. a ciphertext with another contribution's W, one with
    another contribution's U, and forged shares."""
    from hbbft_amd import hoststage
    from hbbft_amd.honey_badger import _one_call
    from hbbft_amd.protocol import BatchVerifier, Ciphertext
    rng = random.Random(77)
    keys = NetworkKeys(engine, 7, 2, rng)
    trace = EpochTrace.generate(engine, keys, rng, hb_epoch=1, bad_every=3, proposal_bytes=64)
    ps = sorted(trace.cts)
    cts = {p: list(trace.cts[p]) for p in ps}
    cts[ps[0]][2] = cts[ps[1]][2]               # W of another contribution
    cts[ps[2]][0] = cts[ps[3]][0]               # U of another contribution
    huv = hoststage.hash_g1_g2([cts[p][0] for p in ps], [cts[p][1] for p in ps])
    pre = BatchVerifier(engine)
    for p, h in zip(ps, huv):
        pre.queue_ct(Ciphertext(cts[p][0], cts[p][1], cts[p][2], h))
    for p, j in trace.dec_msgs:
        c = ps.index(p)
        pre.queue_dec(keys.pks[j], trace.dec_shares[(p, j)], huv[c], cts[p][2])
    jobs = pre._take_jobs()
    merged = {kind: (keys_, v) for kind, keys_, v in _one_call(engine, jobs)}
    separate = {kind: (keys_, v) for kind, keys_, v in BatchVerifier(engine)._run_jobs(jobs)}
    assert merged == separate
    assert 0 < sum(separate["ct"][1]) < len(ps) and 0 < sum(separate["dec"][1]) < len(separate["dec"][0])


def _outcome(r):
    """Everything an epoch's Steps determine, faults and errors in order."""
    return (r.ba_decisions, r.ba_coins, r.coins, r.signatures, r.plaintexts,
            [(k, p, f.node_id, f.kind) for k, p, f in r.faults], [(k, p, e.kind, e.detail) for k, p, e in r.errors])


@pytest.mark.parametrize("adversary", ["random", "faulty_share"])
def test_epoch_fast_paths_equal_full_path_n100(engine, adversary):
    """configs[4] at N=100, f=33 with BA coins and the Random / FaultyShare adversaries of
    tests/honey_badger.rs:26-245: the cached-verdict transitions (ThresholdSign / ThresholdDecrypt
    .store_cached, BinaryAgreementCoin.handle_fast; threshold_sign.rs:181-197, threshold_decrypt.rs:
    182-201, binary_agreement.rs:245-264) give the same decisions, coins, signatures, plaintexts,
    faults (in order) and errors as every message through handle_message (fast_paths=False)."""
    rng = random.Random({"random": 5100, "faulty_share": 5101}[adversary])
    keys = NetworkKeys(engine, 100, 33, rng)
    trace = EpochTrace.generate(engine, keys, rng, hb_epoch=1, bad_every=41, proposal_bytes=200, n_adv=33,
                                adversary=adversary, inject=0.3)
    trace.with_ba(engine, rng, extra=0.2, bad_every=43)
    fast = run_epoch(engine, keys, trace)
    full = run_epoch(engine, keys, trace, fast_paths=False)
    assert _outcome(fast) == _outcome(full)
    assert fast.plaintexts == trace.proposals and fast.errors == []
    assert fast.ba_decisions == trace.ba.decision and fast.ba_coins == trace.ba.coins
    assert fast.faults and all(f.node_id in trace.adv or (k, p, f.node_id) in (trace.bad | trace.ba.bad)
                               for k, p, f in fast.faults)


@pytest.mark.parametrize("n", [7, 13])
def test_ba_epoch_pipelined_and_prefetch_equal_serial(engine, n):
    """the pipelined BA coin phase (windows 1 and 3) and the prefetched coin documents
    (prefetch_coins: hashes and our shares computed before the epoch) give the serial run's Steps
    at the same window: decisions, coins, plaintexts and the full fault list (kind, proposer,
    sender, fault kind) in order; fast paths off gives them too."""
    from hbbft_amd.honey_badger import prefetch_coins
    t = (n - 1) // 3
    rng = random.Random(900 + n)
    keys = NetworkKeys(engine, n, t, rng)
    trace = EpochTrace.generate(engine, keys, rng, hb_epoch=4, bad_every=7, proposal_bytes=48)
    trace.with_ba(engine, rng, extra=0.4, bad_every=7)
    for w in (1, 3):
        serial = run_epoch(engine, keys, trace, window=w, pipelined=False)
        assert serial.ba_decisions == trace.ba.decision and serial.plaintexts == trace.proposals
        pip = run_epoch(engine, keys, trace, window=w, pipelined=True)
        pre = run_epoch(engine, keys, trace, window=w, pipelined=True,
                        coin_prefetch=prefetch_coins(keys, trace.hb_epoch, range(n)))
        full = run_epoch(engine, keys, trace, window=w, pipelined=False, fast_paths=False)
        assert _outcome(pip) == _outcome(serial)
        assert _outcome(pre) == _outcome(serial)
        assert _outcome(full) == _outcome(serial)


@pytest.mark.parametrize("adversary", ["random", "faulty_share"])
def test_speculative_g1_combines_equal_off(engine, monkeypatch, adversary):
    """the speculative decryption combines of the pre-verification (HBH_EPOCH_SPEC_G1,
    on by default) change no outcome -- the same decisions, coins, signatures, plaintexts, faults in
    order and errors with them off, under an adversary forging decryption and coin shares."""
    rng = random.Random({"random": 5200, "faulty_share": 5201}[adversary])
    keys = NetworkKeys(engine, 16, 5, rng)
    trace = EpochTrace.generate(engine, keys, rng, hb_epoch=2, bad_every=7, proposal_bytes=90, n_adv=5,
                                adversary=adversary, inject=0.3)
    trace.with_ba(engine, rng, extra=0.3, bad_every=9)
    monkeypatch.setenv("HBH_EPOCH_SPEC_G1", "1")
    on = run_epoch(engine, keys, trace, window=64)
    monkeypatch.setenv("HBH_EPOCH_SPEC_G1", "0")
    off = run_epoch(engine, keys, trace, window=64)
    assert _outcome(on) == _outcome(off)
    assert on.plaintexts == trace.proposals and on.errors == []
