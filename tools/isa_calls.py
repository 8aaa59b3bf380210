#!/usr/bin/env python3
"""Per-call-site view of one kernel: for each s_swappc (product call) the callee and the
instructions between it and the previous call by category (spills = scratch).  usage:
isa_calls.py <code object> <kernel substring> [start_off end_off]"""
import collections
import re
import sys

sys.path.insert(0, __import__("os").path.dirname(__file__))
import isa_report as R  # noqa: E402

funcs = R.parse(R.disasm(sys.argv[1]))
for name, (base, ins) in funcs.items():
    if sys.argv[2] not in name:
        continue
    lo = int(sys.argv[3], 16) if len(sys.argv) > 3 else 0
    hi = int(sys.argv[4], 16) if len(sys.argv) > 4 else 1 << 40
    seg = collections.Counter()
    for a, op, l in ins:
        if not lo <= a - base <= hi:
            continue
        seg[R.cat(op)] += 1
        if op == "s_swappc_b64":
            print("+%#x  glue %4d  %s" % (a - base, sum(seg.values()) - 1, dict(seg)))
            seg = collections.Counter()
    print("tail", dict(seg))
    break
