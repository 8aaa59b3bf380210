"""A virtual network for protocol tests (test infrastructure), restating the reference's
tests/net/mod.rs + tests/net/adversary.rs: nodes keyed by id, the first ``num_faulty`` marked faulty,
one FIFO message queue; before every crank the adversary may reorder / inject (pre_crank), the front
message is delivered -- to the algorithm of a correct receiver, to the adversary's ``tamper`` for a
faulty one -- and the resulting Step's broadcasts are expanded into one message per other node
(process_step, mod.rs:218-286), with a correct node blaming a correct node an error."""
import collections


class NetMessage:
    __slots__ = ("frm", "payload", "to")

    def __init__(self, frm, payload, to):
        self.frm, self.payload, self.to = frm, payload, to

    def __repr__(self):
        return "%r->%r %r" % (self.frm, self.to, self.payload)


class Node:
    def __init__(self, nid, algorithm, faulty):
        self.id, self.algorithm, self.faulty = nid, algorithm, faulty
        self.outputs = []
        self.faults = []


class CrankError(Exception):
    pass


class VirtualNet:
    def __init__(self, node_ids, num_faulty, make_algorithm, adversary=None, crank_limit=None, message_limit=None):
        ids = sorted(node_ids)
        assert num_faulty * 3 < len(ids), "f must satisfy 3f < total nodes"
        self.nodes = {nid: Node(nid, make_algorithm(nid, k < num_faulty), k < num_faulty) for k, nid in enumerate(ids)}
        self.messages = collections.deque()
        self.adversary = adversary if adversary is not None else NullAdversary()
        self.crank_limit, self.message_limit = crank_limit, message_limit
        self.crank_count = self.message_count = 0

    # mod.rs:218-286
    def process_step(self, stepped, step):
        node = self.nodes[stepped]
        for target, msg in step.messages:
            tos = [to for to in self.nodes if to != stepped] if target == "all" else [target]
            for to in tos:
                if not node.faulty:
                    self.message_count += 1
                self.messages.append(NetMessage(stepped, msg, to))
        node.outputs.extend(step.output)
        node.faults.extend(step.fault_log)
        if not node.faulty:
            for flt in step.fault_log:
                other = self.nodes.get(flt.node_id)
                if other is not None and not other.faulty:
                    raise CrankError("correct node %r blamed correct node %r: %s" % (stepped, flt.node_id, flt.kind))

    def send_input(self, nid, value):  # mod.rs:854-869
        step = self.nodes[nid].algorithm.handle_input(value)
        self.process_step(nid, step)
        return step

    def dispatch_message(self, msg):  # mod.rs:823-843
        return self.nodes[msg.to].algorithm.handle_message(msg.frm, msg.payload)

    def inject_message(self, front, msg):  # adversary.rs:173-194
        assert self.nodes[msg.frm].faulty, "injected messages must come from a faulty node"
        assert msg.to in self.nodes
        if front:
            self.messages.appendleft(msg)
        else:
            self.messages.append(msg)

    def sort_messages_by_key(self, key):  # mod.rs:707-722 (stable)
        self.messages = collections.deque(sorted(self.messages, key=key))

    def crank(self, rng):  # mod.rs:893-981
        if self.crank_limit is not None and self.crank_count >= self.crank_limit:
            raise CrankError("crank limit %d exceeded" % self.crank_limit)
        if self.message_limit is not None and self.message_count >= self.message_limit:
            raise CrankError("message limit %d exceeded" % self.message_limit)
        self.adversary.pre_crank(self, rng)
        if not self.messages:
            return None
        msg = self.messages.popleft()
        if self.nodes[msg.to].faulty:
            step = self.adversary.tamper(self, msg, rng)
        else:
            step = self.dispatch_message(msg)
        self.process_step(msg.to, step)
        self.crank_count += 1
        return msg.to, step

    def crank_expect(self, rng):
        r = self.crank(rng)
        if r is None:
            raise CrankError("crank: network queue empty")
        return r


class NullAdversary:  # adversary.rs:363-384
    def pre_crank(self, net, rng):
        pass

    def tamper(self, net, msg, rng):
        return net.dispatch_message(msg)


class ReorderingAdversary(NullAdversary):  # adversary.rs:416-443
    """Swaps the front message with a random one before every crank."""

    def pre_crank(self, net, rng):
        n = len(net.messages)
        if n > 0:
            j = rng.randrange(n)
            net.messages[0], net.messages[j] = net.messages[j], net.messages[0]
