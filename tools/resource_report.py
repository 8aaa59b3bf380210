#!/usr/bin/env python3
"""Register / scratch / LDS report of every kernel in the built gfx950 objects (hbbft_amd/build/*.o),
from the code objects' metadata notes -- the same numbers as `make resource`
(-Rpass-analysis=kernel-resource-usage) without recompiling (k_pair / k_quad take ~10 minutes each).

usage: tools/resource_report.py [build dir]  -> one line per kernel: VGPR, AGPR, VGPR spills,
scratch bytes per lane, static LDS, waves per SIMD the registers allow (512 per SIMD lane on gfx950;
the VGPR column is the unified allocation, AGPRs included)."""
import glob
import os
import re
import subprocess
import sys
import tempfile

LLVM = "/opt/rocm/lib/llvm/bin"
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def code_object(obj, d):
    fb, elf = os.path.join(d, "fatbin"), os.path.join(d, "dev.elf")
    subprocess.run([f"{LLVM}/llvm-objcopy", f"--dump-section=.hip_fatbin={fb}", obj, os.path.join(d, "x")],
                   capture_output=True)
    if not os.path.exists(fb):
        return None
    r = subprocess.run([f"{LLVM}/clang-offload-bundler", "--unbundle", "--type=o", f"--input={fb}",
                        "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--output={elf}"], capture_output=True)
    return elf if r.returncode == 0 else None


def kernels(elf):
    notes = subprocess.run([f"{LLVM}/llvm-readelf", "--notes", elf], capture_output=True, text=True).stdout
    out, cur = [], None
    for line in notes.split("\n"):
        m = re.match(r"\s*-?\s*\.(\w+):\s+(.*)", line)
        if not m:
            continue
        k, v = m.group(1), m.group(2).strip()
        if k == "args":
            continue
        if line.lstrip().startswith("- .") and k in ("agpr_count",):
            cur = {}
            out.append(cur)
        if cur is not None:
            cur[k] = v
    return [k for k in out if "name" in k and not k["name"].endswith(".kd")]


def demangle(names):
    tool = f"{LLVM}/llvm-cxxfilt" if os.path.exists(f"{LLVM}/llvm-cxxfilt") else "c++filt"
    r = subprocess.run([tool], input="\n".join(names), capture_output=True, text=True)
    return r.stdout.split("\n")


def main():
    bdir = sys.argv[1] if len(sys.argv) > 1 else os.path.join(ROOT, "hbbft_amd", "build")
    rows = []
    for obj in sorted(glob.glob(os.path.join(bdir, "k_*.o"))):
        with tempfile.TemporaryDirectory() as d:
            elf = code_object(obj, d)
            if not elf:
                continue
            for k in kernels(elf):
                rows.append((os.path.basename(obj), k))
    names = demangle([k["name"] for _, k in rows])
    print("%-12s %-62s %5s %5s %6s %8s %6s %5s" % ("object", "kernel", "VGPR", "AGPR", "spill", "scratch", "LDS", "w/SIMD"))
    for (obj, k), nm in zip(rows, names):
        v, a = int(k.get("vgpr_count", 0)), int(k.get("agpr_count", 0))
        # gfx950 metadata: vgpr_count is the unified allocation (architectural + accumulation)
        waves = min(8, 512 // max(v, 1)) if v else 8
        print("%-12s %-62s %5d %5d %6s %8s %6s %5d" % (obj, nm[:62], v, a, k.get("vgpr_spill_count", "0"),
                                                     k.get("private_segment_fixed_size", "0"),
                                                     k.get("group_segment_fixed_size", "0"), waves))


if __name__ == "__main__":
    main()
