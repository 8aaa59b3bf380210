#!/usr/bin/env python3
"""Static ISA report of a gfx950 code object: per kernel / function, and per loop (backward branch),
instruction counts by category (MAD, other VALU, moves, DPP, scratch, LDS, calls).

usage: tools/isa_report.py <file.o | file.co | file.elf> [kernel-substring]
Used to drive register-pressure work on k_pair.hip without a GPU (scratch instructions inside the
hot loops = spills that reach HBM)."""
import collections
import os
import re
import subprocess
import sys
import tempfile

LLVM = "/opt/rocm/lib/llvm/bin"


def disasm(path):
    with tempfile.TemporaryDirectory() as d:
        elf = os.path.join(d, "dev.elf")
        r = subprocess.run([f"{LLVM}/clang-offload-bundler", "--unbundle", "--type=o", f"--input={path}",
                            "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--output={elf}"], capture_output=True)
        if r.returncode != 0 or not os.path.exists(elf) or os.path.getsize(elf) == 0:
            # new-driver objects and shared libraries keep the bundle in the .hip_fatbin section
            fb = os.path.join(d, "fatbin")
            subprocess.run([f"{LLVM}/llvm-objcopy", f"--dump-section=.hip_fatbin={fb}", path, os.path.join(d, "x")],
                           capture_output=True)
            if os.path.exists(fb):
                r = subprocess.run([f"{LLVM}/clang-offload-bundler", "--unbundle", "--type=o", f"--input={fb}",
                                    "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--output={elf}"],
                                   capture_output=True)
        src = elf if r.returncode == 0 and os.path.exists(elf) and os.path.getsize(elf) > 0 else path
        out = subprocess.run([f"{LLVM}/llvm-objdump", "-d", "--no-show-raw-insn", src], capture_output=True, text=True)
        return out.stdout.split("\n")


def parse(lines):
    funcs = collections.OrderedDict()
    cur = None
    for l in lines:
        m = re.match(r"^([0-9a-f]+) <(.*)>:", l)
        if m:
            cur = m.group(2)
            funcs[cur] = (int(m.group(1), 16), [])
            continue
        m = re.search(r"//\s*([0-9A-F]+):", l)
        if cur and m:
            s = re.sub(r"\s*//.*", "", l).strip()
            op = s.split()[0] if s else ""
            funcs[cur][1].append((int(m.group(1), 16), op, l))
    return funcs


def cat(op):
    if "mad_" in op and "64" in op:
        return "mad"
    if op.startswith("scratch") or op.startswith("buffer"):
        return "scratch"
    if op.startswith("global"):
        return "global"
    if op.startswith("ds_"):
        return "lds"
    if op == "s_swappc_b64":
        return "call"
    if op in ("v_mov_b32_e32", "v_mov_b64_e32"):
        return "mov"
    if "dpp" in op:
        return "dpp"
    if "accvgpr" in op:
        return "agpr"
    if op.startswith("s_"):
        return "salu"
    return "valu"


def summary(ins):
    c = collections.Counter(cat(op) for _, op, _ in ins)
    return len(ins), dict(sorted(c.items()))


def loops(base, ins):
    out = []
    for a, op, s in ins:
        if op.startswith("s_cbranch") or op == "s_branch":
            m = re.search(r"\+0x([0-9a-f]+)>", s)
            if m:
                t = base + int(m.group(1), 16)
                if t < a:
                    out.append((t, a))
    return out


def main():
    path = sys.argv[1]
    filt = sys.argv[2] if len(sys.argv) > 2 else ""
    funcs = parse(disasm(path))
    for name, (base, ins) in funcs.items():
        if filt and filt not in name:
            continue
        n, c = summary(ins)
        print(f"{name[:90]}  {n} {c}")
        for t, a in loops(base, ins):
            body = [x for x in ins if t <= x[0] <= a]
            if len(body) < 200:
                continue
            n, c = summary(body)
            print(f"    loop +{t - base:#x}..+{a - base:#x} ({(a - t) / 1024:.1f} KB): {n} {c}")


if __name__ == "__main__":
    main()


def loop_head(path, kernel, loop_start):
    """Instructions of a loop from its start to the first conditional branch (the unconditional hot
    part, e.g. the squaring of a square-and-multiply loop)."""
    funcs = parse(disasm(path))
    for name, (base, ins) in funcs.items():
        if kernel in name:
            body = []
            for a, op, l in ins:
                if a - base < loop_start:
                    continue
                body.append((a, op, l))
                if op.startswith("s_cbranch"):
                    break
            return summary(body)
