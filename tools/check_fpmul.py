"""Check the CHECK lines printed by ubench_fpmul against big-int arithmetic."""
import sys
P = 0x1A0111EA397FE69A4B1BA7B6434BACD764774B84F38512BF6730D2A0F6B0F6241EABFFFEB153FFFFB9FEFFFFFFFFAAAB
inp = [int(l, 16) for l in open("gpurun_out/fpmul_in.txt")]
ok = True
for line in open(sys.argv[1]):
    if not line.startswith("CHECK"):
        continue
    parts = line.split()
    if parts[2] != "ILP1":
        continue  # ILP>1 rows print the XOR of independent chains (keeps every chain live)
    name, limbs = parts[1], [int(x, 16) for x in parts[3:]]
    w, nl = (28, 14) if name in ("fips28", "os28") else (32, 12)
    a = sum(inp[j * 64 + 0] << (w * j) for j in range(nl))
    b = sum(inp[(nl + j) * 64 + 0] << (w * j) for j in range(nl))
    rinv = pow(1 << (w * nl), P - 2, P)
    for _ in range(1000):
        a = a * b * rinv % P
    got = sum(l << (w * j) for j, l in enumerate(limbs))
    good = got % P == a
    ok &= good
    print(name, "OK" if good else "MISMATCH", "(lazy <2p)" if got >= P else "")
sys.exit(0 if ok else 1)
