"""The whole Binary Agreement over real threshold coins on the GPU (hbbft_amd/binary_agreement.py
BinaryAgreement; coin shares checked and combined by the engine through the BatchVerifier): ports of
the reference's tests/binary_agreement.rs (agreement, termination, validity under random message
reordering, networks of 1-16 nodes) and tests/binary_agreement_mitm.rs (the reordering attack with
an adversary that predicts the coin from its own ThresholdSign over the shares reaching its node).
Coin values are checked against msk * hash_g2(bincode((0u8, epoch))) (engine scalar multiplication)."""
import random

import pytest

from hbbft_amd import hoststage
from hbbft_amd.binary_agreement import BinaryAgreement
from hbbft_amd.honey_badger import NetworkKeys
from hbbft_amd.protocol import BatchVerifier, NetworkInfo

from . import ba_mitm
from .test_binary_agreement_net_host import run_network

pytestmark = pytest.mark.gpu


def real_netinfo(engine, n, seed):
    keys = NetworkKeys(engine, n, (n - 1) // 3, random.Random(seed))

    def make(i):
        return NetworkInfo(i, range(n), keys.t, keys.master_pk, keys.pks,
                           sign_g2=lambda H, sk=keys.sks[i]: hoststage.g2_mul([H], [sk])[0])
    return keys, make


def check_coins(engine, keys, net):
    """every threshold coin a node used is parity(msk * hash_g2(bincode((0u8, epoch))))"""
    seen = 0
    for nd in net.nodes.values():
        for e, coin in nd.algorithm.coins.items():
            h = hoststage.hash_g2([nd.algorithm.coin_document(e)])[0]
            assert coin == hoststage.signature_parity(engine.g2_mul([h], [keys.msk]))[0], (nd.id, e)
            seen += 1
    return seen


@pytest.mark.parametrize("n,faulty,inp,seed", [(1, 0, None, 21), (4, 1, None, 22), (7, 2, True, 23),
                                                (10, 3, None, 24), (16, 5, None, 25)])
def test_binary_agreement_network(engine, n, faulty, inp, seed):
    keys, make = real_netinfo(engine, n, seed)
    ver = BatchVerifier(engine)
    net = run_network(n, faulty, inp, seed, make, ver)
    check_coins(engine, keys, net)


@pytest.mark.parametrize("seed", [31, 32])
def test_reordering_attack(engine, seed):
    """binary_agreement_mitm.rs:447-495: with the Conf round the attack cannot stall the network --
    every correct node terminates with the same output within 10,000 cranks, and the adversary's
    coin predictions equal the real coins."""
    keys, make = real_netinfo(engine, ba_mitm.NUM_NODES, seed)
    ver = BatchVerifier(engine)
    net = ba_mitm.reordering_attack(make, ver, random.Random(seed))
    outs = [net.nodes[i].outputs for i in range(1, ba_mitm.NUM_NODES)]
    assert all(len(o) == 1 for o in outs) and len({o[0] for o in outs}) == 1
    adv = net.adversary
    if adv.epoch % 3 == 2 and adv.coin_value is not None:
        h = hoststage.hash_g2([bytes([0]) + adv.epoch.to_bytes(8, "little")])[0]
        assert adv.coin_value == hoststage.signature_parity(engine.g2_mul([h], [keys.msk]))[0]
    assert ver.calls > 0
