"""Port of the reference's tests/threshold_sign.rs:67-127 through the GPU path: networks of random
sizes with silent faulty nodes (SilentAdversary, MessageScheduler::Random / ::First), many samples
per size, each a ThresholdSign::new_with_document(nonce) run to termination; every good node and
the observer output the same signature (:17-44), and its parity -- the Binary Agreement coin --
is split between both values as check_coin_distribution (:51-65) demands.

The networks of all samples advance in lockstep (one delivery per network per tick) so that the
share checks of one tick run in ONE BatchVerifier drain on the GPU; each network is still the
reference's TestNetwork (tests/network/mod.rs:534-564): the scheduler picks a non-idle good node,
that node handles the first message of its queue, its messages are dispatched to the good nodes
and the observer, and the observer handles its whole queue right after each dispatch.  Messages to
silent nodes are dropped.  The reference draws from thread_rng; this port from a seeded
random.Random (recorded per test), so a failure reproduces."""
import collections
import math
import random

import pytest

from hbbft_amd import hoststage
from hbbft_amd.honey_badger import NetworkKeys
from hbbft_amd.protocol import BatchVerifier, NetworkInfo, ThresholdSign, signature_parity

pytestmark = pytest.mark.gpu

GOOD_SAMPLE_SET = 400.0


def max_faulty(n):  # src/util.rs:22-25
    assert n > 0
    return (n - 1) // 3


def check_coin_distribution(num_samples, count_true, count_false):  # tests/threshold_sign.rs:51-65
    expected_share = 0.4
    max_gain = math.log2(GOOD_SAMPLE_SET)
    gain = min(math.log2(num_samples), max_gain)
    step = expected_share / max_gain
    min_throws = int(num_samples * gain * step)
    assert count_true > min_throws, (count_true, count_false, min_throws)
    assert count_false > min_throws, (count_true, count_false, min_throws)


class SimNet:
    """One TestNetwork<SilentAdversary, ThresholdSign>: good nodes 0..g-1, silent nodes g..n-1,
    an observer.  Shares are checked through the shared BatchVerifier."""

    def __init__(self, engine, verifier, keys, n_good, n_adv, doc, scheduler, rng):
        self.rng, self.scheduler, self.ver = rng, scheduler, verifier
        ids = list(range(n_good + n_adv))
        self.good = list(range(n_good))
        self.keys = keys
        self.nodes = {}
        for i in self.good:
            ni = NetworkInfo(i, ids, keys.t, keys.master_pk, keys.pks,
                             sign_g2=lambda H, sk=keys.sks[i]: hoststage.g2_mul([H], [sk])[0])
            self.nodes[i] = ThresholdSign(ni, verifier)
        self.observer = ThresholdSign(NetworkInfo("observer", ids, keys.t, keys.master_pk, keys.pks), verifier)
        for node in list(self.nodes.values()) + [self.observer]:
            node.set_document(doc)  # new_with_document(netinfo, nonce): hash_g2 on the host
        self.queues = {i: collections.deque() for i in self.good}
        self.obs_queue = collections.deque()
        self.outputs = {i: [] for i in self.good}
        self.obs_outputs = []
        self.faults = []

    # TestNetwork::dispatch_messages: Target::All reaches every good node but the sender, and the observer
    def dispatch(self, sender, step):
        for target, payload in step.messages:
            assert target == "all"
            for i in self.good:
                if i != sender:
                    self.queues[i].append((sender, payload))
            self.obs_queue.append((sender, payload))

    def record(self, who, step):
        (self.obs_outputs if who == "observer" else self.outputs[who]).extend(step.output)
        self.faults += [(who, f) for f in step.fault_log]

    def input_all(self):
        for i in self.good:
            step = self.nodes[i].handle_input()
            self.record(i, step)
            self.dispatch(i, step)
        step = self.observer.handle_input()
        self.record("observer", step)

    def done(self):
        return all(self.nodes[i].terminated for i in self.good)

    def pick(self):  # MessageScheduler::pick_node (tests/network/mod.rs:111-131)
        busy = [i for i in self.good if self.queues[i]]
        if self.scheduler == "first" and self.rng.random() >= 0.1:
            return busy[0]
        return self.rng.choice(busy)

    def queue_check(self, target, sender, share):
        inst = self.nodes[target] if target != "observer" else self.observer
        if not inst.terminated and sender in self.keys.pks:
            self.ver.queue_sig(self.keys.pks[sender], inst.doc_hash, share)


def observer_round(ver, nets):
    """The observer handles its whole queue (observer_handle_messages, mod.rs:508-515), its checks
    drained in one batch for all networks."""
    for net in nets:
        for sender, share in net.obs_queue:
            net.queue_check("observer", sender, share)
    ver.drain()
    for net in nets:
        while net.obs_queue:
            sender, share = net.obs_queue.popleft()
            net.record("observer", net.observer.handle_message(sender, share))


def run_lockstep(engine, nets):
    """Advance every network one delivery per tick; two drains per tick (the picked messages, then
    the observer's queue after the dispatch)."""
    ver = nets[0].ver
    for net in nets:
        net.input_all()
    observer_round(ver, nets)
    live = [n for n in nets if not n.done()]
    ticks = 0
    while live:
        ticks += 1
        picked = []
        for net in live:
            i = net.pick()
            sender, share = net.queues[i].popleft()
            net.queue_check(i, sender, share)
            picked.append((net, i, sender, share))
        ver.drain()
        for net, i, sender, share in picked:
            step = net.nodes[i].handle_message(sender, share)
            net.record(i, step)
            net.dispatch(i, step)
        observer_round(ver, live)
        live = [n for n in live if not n.done()]
        assert ticks < 10_000
    return ticks


def different_sizes(engine, scheduler, num_samples, seed):
    """test_threshold_sign_different_sizes (:67-115)."""
    rng = random.Random(seed)
    last, sizes = 1, [1]
    for _ in range(int(math.log2(GOOD_SAMPLE_SET) - math.log2(num_samples))):
        last += rng.randrange(3, 7)  # gen_range(3, 7)
        sizes.append(last)
    ver = BatchVerifier(engine)
    for size in sizes:
        n_adv = max_faulty(size)
        n_good = size - n_adv
        unique_id = rng.getrandbits(64)
        nets = []
        for i in range(num_samples):
            keys = NetworkKeys(engine, size, n_adv, rng)  # NetworkInfo::generate_map: a fresh key set
            nonce = ("My very unique nonce %x:%d" % (unique_id, i)).encode()
            nets.append(SimNet(engine, ver, keys, n_good, n_adv, nonce, scheduler, random.Random(rng.getrandbits(64))))
        run_lockstep(engine, nets)
        count_true = count_false = 0
        hs = [net.observer.doc_hash for net in nets]
        want = engine.g2_mul(hs, [net.keys.msk for net in nets])
        for net, w in zip(nets, want):
            # test_threshold_sign (:17-44): one output per good node, all equal, the observer's too
            outs = [net.outputs[i] for i in net.good]
            assert all(o == [w] for o in outs), size
            assert net.obs_outputs == [w]
            assert net.faults == []  # silent nodes send nothing: nobody is blamed
            if signature_parity(w):
                count_true += 1
            else:
                count_false += 1
        check_coin_distribution(num_samples, count_true, count_false)
    assert ver.cached() == 0  # every instance terminated and released its verdicts
    return sizes


def test_threshold_sign_random_silent_200_samples(engine):
    sizes = different_sizes(engine, "random", 200, seed=20200)
    assert len(sizes) == 2


def test_threshold_sign_first_silent_50_samples(engine):
    sizes = different_sizes(engine, "first", 50, seed=5050)
    assert len(sizes) == 4
