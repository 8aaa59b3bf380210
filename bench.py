"""Benchmark of the hot path on MI355X: batched ThresholdSign share verification
(PublicKeyShare::verify_g2, reference src/threshold_sign.rs:216-225) at N=64 f=21, plus the
combine latency of combine_and_verify_sig (src/threshold_sign.rs:249-270).

One step = one batch of 65,536 share checks (1,024 documents x 64 shares, BASELINE.json
configs[1]) resident in HBM -> verdict bytes in HBM, through the C ABI
(hbh_verify_pairing_eq_dev).  Multi-GPU: one process per GPU, every rank verifies its own batch
(shards by batch index, no collective on the data path; weak scaling).

Inputs are synthetic and seeded: a degree-21 master polynomial, public-key shares g1 * sk_i,
1,024 document points H_m = g2 * r_m (uniform in G2 like hash_g2's output; hashing stays on the
host in the reference flow and is not part of the path), shares sigma_{m,i} = sk_i * H_m, and one
share per document replaced by a random G2 point (1/64 invalid).  Keys and shares are generated
on the GPU with the engine's own scalar-multiplication kernels; verdicts are checked against the
construction.

Prints ONE JSON line on rank 0.
"""
import argparse
import hashlib
import json
import os
import random
import statistics
import sys
import threading
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

N_NODES, F_FAULTY = 64, 21
T = F_FAULTY
NDOCS = 1024
METRIC = "verified BLS sig shares/sec (whole node) + combine latency, N=64 f=21"
R_ORDER = 0x73EDA753299D7D483339D80809A1D80553BDA402FFFE5BFEFFFFFFFF00000001
# Roofline denominator: measured v_mad_u64_u32 throughput on one MI355X
# (tools/ubench_v2.hip, profiles/r02/ubench_v2_mad.txt: 8 independent chains per wave), by waves
# per SIMD; the theoretical half-rate figure is reported beside it.
ACK_LANE_MIN = 65536                            # HBH_ACK_LANE_MIN (include/hbbft_hip.h)
MAD_PEAK_MEASURED = 38.12                       # T MAD/s at 8 waves/SIMD
MAD_CEILING_BY_WAVES = {1: 17.48, 2: 33.64, 4: 35.20, 8: 38.12}
MAD_PEAK_THEORETICAL = 256 * 4 * 32 * 2.4e9 / 2 / 1e12   # 256 CU x 4 SIMD32 x 2.4 GHz, half rate = 39.32
IMPLS = {"auto": 3, "pair": 4, "wave": 5, "quad": 6, "oct": 7, "wave2": 8}   # HBH_IMPL_* (include/hbbft_hip.h)
PAIR_SIGN = "hbs::k_pair_verify<false, true, 2>"
PAIR_DECRYPT = "hbs::k_pair_verify<false, false, 0>"
KERNEL_NAMES = {"pair": PAIR_SIGN,
                "wave": "hbs::k_wave (one wave per check)",
                "wave2": "hbs64::k_wave (two waves per check)",
                "quad": "hbs::k_quad_verify<false, true, 2>",
                "oct": "hbs::k_oct_verify<false, true, 2>",
                "auto": PAIR_SIGN,
                "decrypt": PAIR_DECRYPT}
G1_UNC = bytes.fromhex(
    "17f1d3a73197d7942695638c4fa9ac0fc3688c4f9774b905a14e3a3f171bac586c55e83ff97a1aeffb3af00adb22c6bb"
    "08b3f481e3aaa0f1a09e30ed741d8ae4fcf5e095d5d00af600db18cb2c04b3edd03cc744a2888ae40caa232946c5e7e1")
G2_UNC = bytes.fromhex(
    "13e02b6052719f607dacd3a088274f65596bd0d09920b61ab5da61bbdc7f5049334cf11213945d57e5ac7d055d042b7e"
    "024aa2b2f08f0a91260805272dc51051c6e47ad4fa403b02b4510b647ae3d1770bac0326a805bbefd48056c8c121bdb8"
    "0606c4a02ea734cc32acd2b02bc28b99cb3e287e85a763af267492ab572e99ab3f370d275cec1da1aaa9075ff05f79be"
    "0ce5d527727d6e118cc9cdc6da2e351aadfd9baa8cbdd3a76d429a695160d12c923ac9cc3baca289e193548608b82801")


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def dist_backend():
    """gloo on host tensors by default: the ranks exchange only a barrier, the max step time and
    per-rank reports, and the design has no device collective (north star: RCCL is
    deliberately unused), so a multi-GPU record carries no RCCL traffic.  HBH_DIST_BACKEND=nccl
    selects RCCL for the same few host values (moved to the device); HBH_REHEARSE=1 (or the legacy
    HBH_DIST_BACKEND=gloo) rehearses N ranks on fewer GPUs (ranks share devices round-robin)."""
    return os.environ.get("HBH_DIST_BACKEND", "gloo")


def rehearsal():
    """N ranks on fewer devices than N (tests/test_bench_launch.py): explicit opt-in only."""
    return os.environ.get("HBH_REHEARSE") == "1" or os.environ.get("HBH_DIST_BACKEND") == "gloo"


def _free_port():
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def pool_devices(n):
    """Devices of the --launcher pool shards: 0..n-1, or HBH_POOL_DEVICES (e.g. "0,0" runs two
    shards on device 0, the one-GPU rehearsal of the pool path)."""
    env = os.environ.get("HBH_POOL_DEVICES")
    devs = [int(x) for x in env.split(",") if x.strip()] if env else list(range(n))
    if len(devs) != n:
        raise SystemExit("bench.py: HBH_POOL_DEVICES lists %d devices, --gpus %d" % (len(devs), n))
    return devs


def launch(args):
    """Honour --gpus N.  Returns None when this process should run the benchmark itself, else the
    exit code to leave with:
      * under torchrun (WORLD_SIZE set): WORLD_SIZE must equal --gpus and, on RCCL, that many
        devices must be visible;
      * --gpus N > 1 without WORLD_SIZE, --launcher ranks (default): spawn N ranks with
        torch.distributed.run as a CHILD process (this process has not touched the GPU) and return
        its exit code;
      * --launcher pool: one process drives the in-ABI engine pool over N devices;
    fewer visible devices than asked for is an error (exit 2), never a silent 1-GPU run."""
    visible = torch.cuda.device_count()
    # rehearsal (HBH_REHEARSE=1 or HBH_DIST_BACKEND=gloo explicitly): N ranks share the visible device(s)
    need = 1 if rehearsal() else args.gpus
    env = os.environ.get("WORLD_SIZE")
    if env is not None:
        if int(env) != args.gpus:
            log("bench.py: WORLD_SIZE=%s but --gpus %d" % (env, args.gpus))
            return 2
        if visible < need:
            log("bench.py: %d ranks need %d devices, %d visible" % (args.gpus, need, visible))
            return 2
        return None
    if args.gpus < 1:
        return 2
    if args.launcher == "pool":
        devs = pool_devices(args.gpus)
        if visible < 1 or max(devs) >= visible:
            log("bench.py: pool devices %s, %d visible" % (devs, visible))
            return 2
        return None
    if visible < need:
        log("bench.py: --gpus %d but %d devices visible" % (args.gpus, visible))
        return 2
    if args.gpus == 1:
        return None
    import subprocess
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=%d" % args.gpus,
           "--master-addr=127.0.0.1", "--master-port=%d" % _free_port(), os.path.abspath(__file__)] + sys.argv[1:]
    log("bench.py: spawning %d ranks: %s" % (args.gpus, " ".join(cmd)))
    return subprocess.call(cmd)


def gather_per_rank(value, world):
    """Every rank's value on every rank (reporting only: per-rank kernel times)."""
    if world == 1:
        return [value]
    out = [None] * world
    dist.all_gather_object(out, value)
    return out


def rank_device(local):
    return local % max(1, torch.cuda.device_count())


def allreduce_max(value, dev):
    t = torch.tensor([value], dtype=torch.float64)
    if dist_backend() == "nccl":
        t = t.to(dev)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def poly_eval(coeffs, x):
    r = 0
    for c in reversed(coeffs):
        r = (r * x + c) % R_ORDER
    return r


class Workload:
    """Seeded ThresholdSign instance set, generated on the GPU (engine scalar multiplication)."""

    def __init__(self, eng, batch, seed):
        from hbbft_amd.engine import g1_abi_from_uncompressed as g1a, g2_abi_from_uncompressed as g2a
        rng = random.Random(seed)
        self.g1, self.g2 = g1a(G1_UNC), g2a(G2_UNC)
        self.coeffs = [rng.randrange(1, R_ORDER) for _ in range(T + 1)]
        self.sk = [poly_eval(self.coeffs, i + 1) for i in range(N_NODES)]
        self.pks = eng.g1_mul([self.g1] * N_NODES, self.sk)
        self.master_pk = eng.g1_mul([self.g1], [self.coeffs[0]])[0]
        ndocs = max(1, batch // N_NODES)
        self.hashes = eng.g2_mul([self.g2] * ndocs, [rng.randrange(1, R_ORDER) for _ in range(ndocs)])
        doc_idx = np.arange(batch, dtype=np.int64) // N_NODES
        node = np.arange(batch, dtype=np.int64) % N_NODES
        bad = {m * N_NODES + (m * 37) % N_NODES for m in range(ndocs)}
        bases, scal = [], []
        for i in range(batch):
            if i in bad:
                bases.append(self.g2)
                scal.append(rng.randrange(1, R_ORDER))
            else:
                bases.append(self.hashes[doc_idx[i]])
                scal.append(self.sk[node[i]])
        t0 = time.time()
        self.sigs = eng.g2_mul(bases, scal)
        log("generated %d shares on the GPU in %.2f s" % (batch, time.time() - t0))
        self.expected = np.array([0 if i in bad else 1 for i in range(batch)], dtype=np.uint8)
        self.doc_idx = doc_idx.astype(np.int32)
        self.node = node
        self.pk_batch = b"".join(self.pks[j] for j in node)
        self.sig_batch = b"".join(self.sigs)
        self.hash_table = b"".join(self.hashes)


def timed_steps(step, streams, steps, world, dev):
    """Time `steps` calls of step(k) (k-th call on streams[k % len]) with HIP events: start on
    stream 0 (the others wait for it), end on stream 0 after waiting for the others; barrier +
    synchronize on both sides; max over ranks.  Returns ms per step."""
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ev0.record(streams[0])
    for st in streams[1:]:
        st.wait_event(ev0)
    for k in range(steps):
        step(k)
    for st in streams[1:]:
        e = torch.cuda.Event()
        e.record(st)
        streams[0].wait_event(e)
    ev1.record(streams[0])
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    ms = ev0.elapsed_time(ev1)
    return (allreduce_max(ms, dev) if world > 1 else ms) / steps


def roofline_entry(kernel, launches, avg_ms, units, op, unit_name, waves_per_simd=None, source=None):
    """One kernel's roofline: achieved = units per launch x algorithmic MADs per unit (workcount,
    300 per Fp-mul, 222 per Fp-sqr) / average launch time (HIP events on the engine's stream)."""
    from hbbft_amd import workcount
    mad = workcount.mads(*op)
    achieved = units * mad / (avg_ms / 1e3) / 1e12 if avg_ms > 0 else 0.0
    e = {"kernel": kernel, "launches": launches, "avg_launch_ms": avg_ms, "units_per_launch": units,
         "unit": unit_name, "fp_ops_per_unit": op[0], "fp_sqr_per_unit": op[1], "mad_per_unit": mad,
         "achieved": achieved, "peak": MAD_PEAK_MEASURED, "frac": achieved / MAD_PEAK_MEASURED,
         "peak_theoretical": MAD_PEAK_THEORETICAL}
    e.update(traffic_fields(kernel, source))
    if waves_per_simd:
        if waves_per_simd < 1:  # below one wave per SIMD on average: the 1-wave ceiling scaled by occupancy
            ceil = MAD_CEILING_BY_WAVES[1] * waves_per_simd
        else:  # the measured ceiling of the largest measured occupancy not above it
            ceil = MAD_CEILING_BY_WAVES[max(k for k in MAD_CEILING_BY_WAVES if k <= waves_per_simd)]
        e["waves_per_simd"] = waves_per_simd
        e["occupancy_ceiling"] = ceil
        e["frac_of_occupancy_ceiling"] = achieved / ceil
    return e


def reference_work(main_k, workcount):
    """SURVEY §8(d)'s "reference work" beside the algorithmic roofline: the same verdicts as the
    reference computes them (two separate pairings per check, workcount.REFERENCE_CHECK), priced
    per unit at 300 MADs per Fp product, over the same measured launch time.  A throughput
    equivalent, not a roofline: it counts work this kernel does not do."""
    mad = workcount.mads(*workcount.REFERENCE_CHECK_OPS)
    ach = main_k["units_per_launch"] * mad / (main_k["avg_launch_ms"] / 1e3) / 1e12 if main_k["avg_launch_ms"] else 0
    return {"fp_ops_per_check": workcount.REFERENCE_CHECK, "mad_per_check": mad, "equivalent_T_mad_s": ach,
            "equivalent_frac_of_peak": ach / MAD_PEAK_MEASURED,
            "note": "two pairings per check as threshold_crypto's verify does (2 x (single-pair Miller + G2 walk + "
                    "final exp)); the kernel's own count is roofline.mad_per_unit"}


def pair_waves_per_simd(checks, lanes=2):
    """Waves per SIMD of the lane-pair kernel k_pair_verify (two lanes per check), the lane-quad
    kernel k_quad_verify (lanes=4) or the lane-octo kernel k_oct_verify (lanes=8): 64-lane waves,
    1,024 SIMDs."""
    w = checks * lanes / 64 / 1024
    return 2 if w >= 2 else (1 if w >= 1 else round(w, 3))


def cpu_info():
    """(nproc, affinity CPUs, threads the CPU baseline uses).  The thread count is the host stage's
    own detection (hbh_host_threads: affinity mask, cgroup cpu.max quota, HBH_HOST_THREADS /
    OMP_NUM_THREADS -- 16 on the GPU box, one GPU's share of the host)."""
    from hbbft_amd import hoststage
    ncpu = os.cpu_count() or 1
    aff = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else ncpu
    return ncpu, aff, max(1, hoststage.host_threads())


def timed_pool(fn, items, threads):
    """Run fn over items on `threads` host threads (the C oracle releases the GIL); seconds."""
    from concurrent.futures import ThreadPoolExecutor
    t0 = time.perf_counter()
    if threads == 1:
        out = [fn(x) for x in items]
    else:
        with ThreadPoolExecutor(threads) as ex:
            out = list(ex.map(fn, items))
    return time.perf_counter() - t0, out


def _ensure_oracle():
    from oracle import cbls
    if not os.path.exists(cbls.LIB_PATH):
        import subprocess
        subprocess.check_call(["make", "-s", "-C", os.path.join(ROOT, "oracle")])
    return cbls


def cpu_baseline(w, budget_s=12.0):
    """Reference-equivalent CPU path (oracle/c/bls_cpu.c: pairing 0.14 algorithms, two pairings per
    check) on a bounded sample of the same workload, one thread and all host threads."""
    cbls = _ensure_oracle()
    n1 = 200
    pk, sg = w.pk_batch[:96 * n1], w.sig_batch[:192 * n1]
    t0 = time.perf_counter()
    v = cbls.verify_g2_batch(pk, sg, w.hash_table, w.doc_idx[:n1], threads=1)
    st = time.perf_counter() - t0
    assert (v == w.expected[:n1]).all(), "CPU baseline verdicts disagree"
    ncpu, aff, threads = cpu_info()
    n2 = int(min(len(w.expected), max(threads * 8, (budget_s / (st / n1)) * threads * 0.5)))
    t0 = time.perf_counter()
    v = cbls.verify_g2_batch(w.pk_batch[:96 * n2], w.sig_batch[:192 * n2], w.hash_table, w.doc_idx[:n2],
                             threads=threads)
    mt = time.perf_counter() - t0
    assert (v == w.expected[:n2]).all(), "CPU baseline verdicts disagree"
    # combine latency on the CPU: interpolate 22 G2 shares + master verify_g2
    idx = [k for k in range(N_NODES) if w.expected[k]][: T + 1]
    pts = [w.sigs[k] for k in idx]
    t0 = time.perf_counter()
    rc, sig = cbls.combine_g2(T, idx, pts)
    ok = cbls.verify_g2(w.master_pk, sig, w.hashes[0])
    comb_ms = (time.perf_counter() - t0) * 1e3
    assert rc == 0 and ok
    return {"value": n2 / mt, "unit": "shares/s", "cores": threads, "kind": "port",
            "sample": "%d verify_g2 checks of the same batch on %d threads (and %d on 1 thread: %.1f shares/s); "
                      "C restatement of pairing 0.14 (two pairings per check)" % (n2, threads, n1, n1 / st),
            "single_thread_value": n1 / st, "combine_latency_ms": comb_ms,
            "nproc": ncpu, "affinity": aff,
            "cores_note": "measured on %d threads = the CPUs this process may use (hbh_host_threads: affinity, "
                          "cgroup quota, OMP_NUM_THREADS); nproc %d counts the whole machine" % (threads, ncpu)}


def traffic_fields(kernel, source=None):
    """roofline "traffic" (HBM bytes per launch, or None) and "traffic_source" (profile file, its
    commit, whether it measured the library loaded now).  kernel: a name, or names joined by " + "
    (summed); source: the bench workload whose profile to prefer (kernels shared between workloads)."""
    d = pmc_traffic(kernel.split(" + "), source)
    return {"traffic": d["hbm_bytes_per_launch"] if d else None, "traffic_source": d}


def pmc_traffic(kernels, source=None):
    """HBM bytes per launch of `kernels` (summed) from the latest committed rocprofv3 --pmc passes
    (FETCH_SIZE x2 gfx950 correction + WRITE_SIZE; profiles/<round>/pmc_traffic.json), with the file
    it came from and whether those passes ran the library this process loaded (sha256 of the .so the
    profile recorded vs the loaded one); None when no committed profile covers every kernel."""
    import glob
    import hashlib
    from hbbft_amd import _lib
    try:
        loaded = hashlib.sha256(open(_lib.LIB_PATH, "rb").read()).hexdigest()
    except OSError:
        loaded = None
    for fn in sorted(glob.glob(os.path.join(ROOT, "profiles", "r*", "pmc_traffic.json")), reverse=True):
        with open(fn) as f:
            d = json.load(f)
        table = d.get("by_source", {}).get(source) if source else None
        if not table or not all(k in table for k in kernels):
            table = d.get("kernels", {})
        if all(k in table for k in kernels):
            return {"hbm_bytes_per_launch": sum(table[k].get("hbm_bytes_per_launch") or 0 for k in kernels),
                    "profile": os.path.relpath(fn, ROOT), "profile_commit": d.get("git_commit"),
                    "matches_loaded_lib": (d.get("lib_sha256") == loaded) if d.get("lib_sha256") else None}
    return None


def combine_latency(eng, w, reps=7):
    """combine_and_verify_sig for one document: interpolate the first t+1 valid shares (G2 MSM
    with Lagrange coefficients) + verify the result against the master key; host-to-host wall
    time through the C ABI (median of reps).  Also the batched rate (one combine per document)."""
    idx = [k for k in range(N_NODES) if w.expected[k]][: T + 1]
    pts = [w.sigs[k] for k in idx]
    times = []
    for _ in range(reps):
        t0 = time.perf_counter()
        out, st, v = eng.combine_verify_g2(T, [idx], [pts], w.master_pk, [w.hashes[0]])
        times.append((time.perf_counter() - t0) * 1e3)
        assert st == [0] and v == b"\x01", "combined signature does not verify"
    ndocs = len(w.hashes)
    allidx, allpts = [], []
    for m in range(ndocs):
        ids = [k for k in range(N_NODES) if w.expected[m * N_NODES + k]][: T + 1]
        allidx.append(ids)
        allpts.append([w.sigs[m * N_NODES + k] for k in ids])
    from hbbft_amd._lib import STAGE_CURVE
    eng.set_profiling(True)
    t0 = time.perf_counter()
    out, st = eng.interpolate_g2(T, allidx, allpts)
    bt = time.perf_counter() - t0
    dev_ms = eng.stage_time(STAGE_CURVE)[0]
    eng.set_profiling(False)
    assert all(s == 0 for s in st)
    v = eng.verify_sig_shares([w.master_pk] * ndocs, out, w.hashes, list(range(ndocs)))
    assert all(v), "a batched combined signature does not verify"
    return statistics.median(times), ndocs / bt, ndocs / (dev_ms / 1e3)


P_FIELD = int("1a0111ea397fe69a4b1ba7b6434bacd764774b84f38512bf6730d2a0f6b0f6241eabfffeb153ffffb9feffffffffaaab", 16)


def g2_compress_abi(b):
    """ABI G2 point -> the reference's 96-byte compressed wire encoding (pairing 0.14 G2Compressed:
    x.c1 || x.c0 big-endian, 0x80 compressed, 0x40 infinity, 0x20 larger y in Fq2 order c1, c0)."""
    if not any(b):
        return bytes([0xC0]) + bytes(95)
    x0, x1, y0, y1 = (int.from_bytes(b[o:o + 48], "little") for o in (0, 48, 96, 144))
    n0, n1 = (P_FIELD - y0) % P_FIELD, (P_FIELD - y1) % P_FIELD
    greatest = y1 > n1 if y1 != n1 else y0 > n0
    e = bytearray(x1.to_bytes(48, "big") + x0.to_bytes(48, "big"))
    e[0] |= 0x80 | (0x20 if greatest else 0)
    return bytes(e)


def g1_compress_abi(b):
    """ABI G1 point -> 48-byte compressed wire encoding (pairing 0.14 G1Compressed)."""
    if not any(b):
        return bytes([0xC0]) + bytes(47)
    x, y = (int.from_bytes(b[o:o + 48], "little") for o in (0, 48))
    e = bytearray(x.to_bytes(48, "big"))
    e[0] |= 0x80 | (0x20 if y > (P_FIELD - y) % P_FIELD else 0)
    return bytes(e)


def decode_rate(eng, w, n):
    """Wire decoding of the batch's n signature shares (G2) and n public-key-share encodings (G1)
    (SURVEY §8f f2): hbh_g2_decompress rate host-to-host (PCIe + host flag parsing included) and
    device-only, and the device-only G1 rate; decoded bytes must equal the generated points."""
    from hbbft_amd._lib import STAGE_CURVE
    sig = w.sig_batch[:n * 192]
    encs = b"".join(g2_compress_abi(sig[i * 192:(i + 1) * 192]) for i in range(n))
    eng.g2_decompress(encs[:96 * 64])  # warm-up
    eng.set_profiling(True)
    t0 = time.perf_counter()
    pts, ok = eng.g2_decompress(encs)
    host_s = time.perf_counter() - t0
    dev_ms = eng.stage_time(STAGE_CURVE)[0]
    eng.set_profiling(False)
    assert all(ok) and b"".join(pts) == sig, "G2 decoding differs from the generated shares"
    pk = w.pk_batch[:n * 96]
    pk_enc = {}
    encs1 = b"".join(pk_enc.setdefault(pk[i * 96:(i + 1) * 96], g1_compress_abi(pk[i * 96:(i + 1) * 96]))
                     for i in range(n))
    eng.g1_decompress(encs1[:48 * 64])  # warm-up (the first launch of a kernel loads its code object)
    eng.set_profiling(True)
    pts1, ok1 = eng.g1_decompress(encs1)
    dev1_ms = eng.stage_time(STAGE_CURVE)[0]
    eng.set_profiling(False)
    assert all(ok1) and b"".join(pts1) == pk, "G1 decoding differs from the generated keys"
    return {"g2_decode_per_s": n / host_s, "g2_decode_per_s_device": n / (dev_ms / 1e3),
            "g2_decode_ms_device": dev_ms, "g1_decode_per_s_device": n / (dev1_ms / 1e3),
            "g1_decode_ms_device": dev1_ms, "decode_points": n}


def from_wire(eng, w, n, streams, steps, warmup, world, dev, d_pk, d_hs, d_di, to_dev):
    """The whole node from wire bytes: each step takes the batch's n signature
    shares as the 96-byte compressed encodings a node receives (threshold_sign::Message,
    src/threshold_sign.rs:73; the Message's bincode framing is host work, wire.py) already in HBM,
    decodes them on the device (k_wire_parse + k_g2_decompress: flags, square root, subgroup test,
    hbh_g2_decompress_dev) and verifies them (verify_pairing_eq_dev), consecutive batches on
    alternating streams as the device-resident line.  A share that fails to decode is a
    DeserializeMessage fault in the reference, never a verdict; every encoding here decodes and
    the decoded bytes and verdicts are checked after the timed steps."""
    from hbbft_amd import workcount
    from hbbft_amd._lib import STAGE_CURVE, STAGE_PAIRING
    sig = w.sig_batch[:n * 192]
    encs = b"".join(g2_compress_abi(sig[i * 192:(i + 1) * 192]) for i in range(n))
    d_enc = to_dev(encs)
    d_sg = [torch.empty(n * 192, dtype=torch.uint8, device=dev) for _ in streams]
    d_ok = [torch.zeros(n, dtype=torch.uint8, device=dev) for _ in streams]
    d_v = [torch.zeros(n, dtype=torch.uint8, device=dev) for _ in streams]
    nh = len(w.hashes)

    def step(k=0):
        j = k % len(streams)
        cs = streams[j].cuda_stream
        eng.g2_decompress_dev(cs, n, d_enc.data_ptr(), d_sg[j].data_ptr(), d_ok[j].data_ptr())
        eng.verify_pairing_eq_dev(cs, n, d_pk.data_ptr(), d_hs.data_ptr(), nh, d_di.data_ptr(), None,
                                  d_sg[j].data_ptr(), n, None, d_v[j].data_ptr())

    def outputs_ok(nbuf=None):
        return all(bool(d_ok[j].cpu().numpy().all()) and bool((d_v[j].cpu().numpy() == w.expected).all())
                   and d_sg[j].cpu().numpy().tobytes() == sig for j in range(len(streams))[:nbuf])

    for k in range(len(streams)):
        step(k)
    torch.cuda.synchronize(dev)
    ok = outputs_ok()
    for k in range(warmup):
        step(k)
    torch.cuda.synchronize(dev)
    for j in range(len(streams)):
        d_ok[j].zero_()
        d_v[j].zero_()
        d_sg[j].zero_()
    ms = timed_steps(step, streams, steps, world, dev)
    ok = ok and outputs_ok(min(steps, len(streams)))
    eng.set_profiling(True)
    for _ in range(3):
        step(0)
    torch.cuda.synchronize(dev)
    dec_ms, dec_n = eng.stage_time(STAGE_CURVE)
    pair_ms, pair_n = eng.stage_time(STAGE_PAIRING)
    eng.set_profiling(False)
    dec_avg = dec_ms / max(dec_n, 1)
    return {"value": n * world / (ms / 1e3), "unit": "shares/s", "ms_per_step": ms, "steps": steps,
            "outputs_ok": ok, "decode_ms_isolated": dec_avg, "verify_ms_isolated": pair_ms / max(pair_n, 1),
            "kernels": [roofline_entry("hb::k_g2_decompress", dec_n, dec_avg, n, workcount.WIRE_G2_DECODE,
                                       "compressed G2 point (flags, sqrt, subgroup)",
                                       n / 64 / 1024, source="sign")],
            "input": "%d compressed 96-byte signature shares in HBM per step (%d documents)" % (n, nh)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--batch", type=int, default=NDOCS * N_NODES)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-combine", action="store_true")
    ap.add_argument("--no-wire", action="store_true",
                    help="sign workload: skip the whole-node-from-wire-bytes line (decode + verify per step)")
    ap.add_argument("--from-wire", action="store_true",
                    help="sign workload: the line's value is the whole node from wire bytes (compressed shares "
                         "decoded on the device inside every timed step) instead of device-resident points")
    ap.add_argument("--no-node-round", action="store_true",
                    help="dkg workload: skip the one-node SyncKeyGen round (node_round)")
    ap.add_argument("--streams", type=int, default=2, help="sign workload: streams the consecutive batches alternate on")
    ap.add_argument("--impl", choices=["pair", "wave", "quad", "oct", "auto", "wave2"], default="auto",
                    help="pairing implementation (hbh_engine_set_pairing_impl)")
    ap.add_argument("--profile-epoch", default=None, metavar="FILE",
                    help="epoch workload: cProfile the timed epochs (main thread), pstats text to FILE")
    ap.add_argument("--prefetch-after-prep", action="store_true",
                    help="epoch workload: start the next epoch's coin prefetch once this epoch's decryption prep "
                         "is done (round 4's order) instead of with the epoch (round 5 default, c16)")
    ap.add_argument("--preverify-at", choices=["first_drain", "start"], default="start",
                    help="epoch workload: when the decryption-share pre-verification starts")
    ap.add_argument("--window", type=int, default=6144,
                    help="epoch workload: messages per verifier drain (6,144: 5 engine calls per epoch, 18.3-21.6 "
                         "epochs/s; 8,192: 18.5-19.4; 4,096: 8 calls, 15.9-18.9; profiles/r04/c27_*, c28_*)")
    ap.add_argument("--epoch-coins", choices=["ba", "synthetic"], default="ba",
                    help="epoch workload: coins from Binary Agreement instances or one ThresholdSign each")
    ap.add_argument("--ack-impl", choices=["auto", "quad", "lane", "horner"], default="auto",
                    help="dkg workload: Ack-check kernel (hbh_engine_set_ack_impl)")
    ap.add_argument("--dkg-nodes", type=int, default=0,
                    help="dkg workload, network scope: checking nodes (0 = all 100; 10,000 acks each)")
    ap.add_argument("--dkg-scope", choices=["network", "node"], default="network",
                    help="dkg workload: the whole network's 10^6 ack checks split over the ranks, or one node's "
                         "10,000 per rank")
    ap.add_argument("--pipeline", action="store_true",
                    help="epoch workload: drain window k on a worker thread while the flows handle window k - 1 "
                         "(measured slower than serial drains on MI355X, profiles/r04/c6_epoch_ab.txt)")
    ap.add_argument("--raw", action="store_true",
                    help="epoch workload: the node receives bincode bytes (contributions, coin-share and "
                         "decryption-share messages), decoded on the device per window inside the timed epoch")
    ap.add_argument("--no-preverify", action="store_true",
                    help="epoch workload: no decryption-share pre-verification beside the coin phase")
    ap.add_argument("--no-prefetch", action="store_true",
                    help="epoch workload: no next-epoch coin prefetch (hash and sign every coin document in "
                         "its own epoch)")
    ap.add_argument("--launcher", choices=["ranks", "pool"], default="ranks",
                    help="--gpus N > 1 without torchrun: spawn N ranks (one process per GPU, default) or drive "
                         "the in-ABI engine pool (hbh_pool_*) over N devices from this process")
    ap.add_argument("--workload", choices=["sign", "decrypt", "dkg", "epoch"], default="sign",
                    help="sign = BASELINE configs[1] (default, the headline metric); decrypt = configs[2] "
                         "(64k decryption-share checks + G1 combines, strong-scaled over ranks); dkg = configs[3] "
                         "(SyncKeyGen N=100 t=33 ack checks of one node); epoch = configs[4] (HoneyBadger N=100 f=33 "
                         "epoch crypto of one node)")
    args = ap.parse_args()
    rc = launch(args)
    if rc is not None:
        sys.exit(rc)
    if args.launcher == "pool" and "WORLD_SIZE" not in os.environ:
        return run_pool(args)
    if args.workload != "sign":
        return run_other(args)

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        dist.init_process_group(dist_backend())
    local = rank_device(local)
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)

    from hbbft_amd import workcount
    from hbbft_amd._lib import STAGE_PAIRING, STAGE_PREPARE
    from hbbft_amd.engine import Engine
    eng = Engine(local)
    eng.set_pairing_impl(IMPLS[args.impl])
    n = args.batch
    w = Workload(eng, n, seed=20261016 + rank)

    def to_dev(b):
        return torch.from_numpy(np.frombuffer(b, dtype=np.uint8).copy()).to(dev)

    d_pk = to_dev(w.pk_batch)
    d_sg = to_dev(w.sig_batch)
    d_hs = to_dev(w.hash_table)
    d_di = torch.from_numpy(w.doc_idx.copy()).to(dev)
    nh = len(w.hashes)
    # Consecutive batches alternate between two streams (--streams 2): the engine gives each in-flight
    # call its own table slot, so one batch's prepare and first waves fill the SIMDs the previous
    # batch's last waves leave idle.  Verdict buffers are per stream.
    streams = [torch.cuda.Stream(dev) for _ in range(max(1, args.streams))]
    d_vs = [torch.zeros(n, dtype=torch.uint8, device=dev) for _ in streams]
    torch.cuda.synchronize(dev)

    def step(k=0):
        eng.verify_pairing_eq_dev(streams[k % len(streams)].cuda_stream, n, d_pk.data_ptr(), d_hs.data_ptr(), nh,
                                  d_di.data_ptr(), None, d_sg.data_ptr(), n, None,
                                  d_vs[k % len(streams)].data_ptr())   # P2 = g1 (flag)

    def verdicts_ok(nbuf=None):
        return all(bool((d.cpu().numpy() == w.expected).all()) for d in d_vs[:nbuf])

    for k in range(len(streams)):
        step(k)
    torch.cuda.synchronize(dev)
    ok = verdicts_ok()
    if not ok:
        raise SystemExit("verdict mismatch against the construction")
    for k in range(args.warmup):
        step(k)
    torch.cuda.synchronize(dev)
    for d in d_vs:      # the timed steps must write every verdict again
        d.zero_()
    ms_step = timed_steps(step, streams, args.steps, world, dev)
    value = n * world / (ms_step / 1e3)
    ok = ok and verdicts_ok(min(args.steps, len(streams)))
    # roofline: isolated launches on one stream (no overlap), HIP events around each launch
    eng.set_profiling(True)
    for _ in range(max(2, min(args.steps, 5))):
        step(0)
    torch.cuda.synchronize(dev)
    pair_ms, pair_n = eng.stage_time(STAGE_PAIRING)
    prep_ms, prep_n = eng.stage_time(STAGE_PREPARE)
    eng.set_profiling(False)
    ok = ok and verdicts_ok()
    per_rank = gather_per_rank({"rank": rank, "device": local, "kernel_ms": pair_ms / max(pair_n, 1),
                                "ms_per_step": ms_step, "verdicts_ok": ok}, world)
    ok = all(r["verdicts_ok"] for r in per_rank)
    wire = None
    if args.from_wire or not args.no_wire:
        wire = from_wire(eng, w, n, streams, max(2, args.steps if args.from_wire else min(args.steps, 5)),
                         args.warmup, world, dev, d_pk, d_hs, d_di, to_dev)
        ok = ok and wire["outputs_ok"]

    if rank == 0:
        kern_ms = pair_ms / max(pair_n, 1)
        main_k = roofline_entry(KERNEL_NAMES[args.impl], pair_n, kern_ms, n, workcount.PAIR_CHECK_WALK, "share check",
                                pair_waves_per_simd(n, {"quad": 4, "oct": 8}.get(args.impl, 2))
                                if args.impl in ("pair", "auto", "quad", "oct") else None)
        kernels = [main_k]
        if prep_n:
            kernels.append(roofline_entry("hbs::k_oct_prep" if args.impl in ("pair", "auto", "quad", "oct") else "hb::k_g2_prepare",
                                          prep_n, prep_ms / prep_n, nh, workcount.PAIR_PREP_DOC, "document (G2 walk)",
                                          nh * 8 / 64 / 1024))  # one lane octo per point
        out = {
            "metric": METRIC, "value": value, "unit": "shares/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": ms_step,
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "u32 limbs (Fp, 14x28-bit)",
            "data": "synthetic, seeded (degree-21 key, 1024 document points, 1/64 invalid shares; generated on GPU)",
            "config": {"workload": "ThresholdSign share verification, BASELINE configs[1]", "batch_per_gpu": n,
                       "streams": len(streams),
                       "documents_per_gpu": nh, "n_nodes": N_NODES, "f": F_FAULTY, "pairing_impl": args.impl,
                       "parallelism": "shard-by-batch x%d" % world},
            "verdicts_ok": ok, "per_rank": per_rank, "reference_work": reference_work(main_k, workcount),
            "roofline": dict(main_k, bound="valu-int", unit="T MAD/s (v_mad_u64_u32 32x32->64)",
                             **traffic_fields(KERNEL_NAMES[args.impl], "sign"), kernels=kernels,
                             note="achieved = checks x algorithmic MADs per check (workcount.PAIR_CHECK_WALK: "
                                  "2-pair Miller + sigma G2 walk + final exp; 300 MAD/Fp-mul, 222/Fp-sqr) / "
                                  "average launch time of isolated single-stream launches (the throughput value alternates two "
                                  "streams); peak = measured MAD rate at 8 waves/SIMD"),
        }
        if wire is not None:
            out["whole_node_from_wire"] = wire
            if args.from_wire:
                out["value"], out["ms_per_step"] = wire["value"], wire["ms_per_step"]
                out["roofline"]["kernels"] = out["roofline"]["kernels"] + wire["kernels"]
                out["config"]["workload"] += ", from compressed wire bytes (decode + verify per step)"
        if not args.no_combine:
            lat, rate, dev_rate = combine_latency(eng, w)
            out["combine_latency_ms"] = lat
            out["combines_per_s_batched"] = rate          # host-to-host, 1,024 combines in one call
            out["combines_per_s_batched_device"] = dev_rate  # k_interp_endo time only
            out.update(decode_rate(eng, w, n))  # hbh_g2/g1_decompress: host-to-host and kernel-only rates
        if not args.no_cpu_baseline and world == 1:
            out["cpu_baseline"] = cpu_baseline(w)
        print(json.dumps(out), flush=True)
    eng.close()
    if world > 1:
        dist.destroy_process_group()


# ---------------------------------------------------------------------------------------- other configs
def _dist_env():
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1 and not dist.is_initialized():
        dist.init_process_group(dist_backend())
    local = rank_device(local)
    torch.cuda.set_device(local)
    return world, rank, local


def _max_over_ranks(ms, world, dev):
    return allreduce_max(ms, dev) if world > 1 else float(ms)


def run_decrypt(args, eng, world, rank, dev):
    """configs[2]: 65,536 decryption-share checks e(D_i, H_uv) == e(pk_i, W) over 1,024 ciphertexts
    (src/threshold_decrypt.rs:227) + one G1 interpolation per ciphertext (:249); the whole batch is
    fixed and split over the ranks by ciphertext (hbbft_amd/shard.py) -> strong scaling."""
    from hbbft_amd.engine import g1_abi_from_uncompressed as g1a, g2_abi_from_uncompressed as g2a
    from hbbft_amd.shard import shard_by_instance
    rng = random.Random(4242)
    g1, g2 = g1a(G1_UNC), g2a(G2_UNC)
    ncts, total = NDOCS, NDOCS * N_NODES
    inst = np.arange(total) // N_NODES
    lo, hi = shard_by_instance(total, inst, rank, world)
    clo, chi = int(inst[lo]) if hi > lo else 0, int(inst[hi - 1]) + 1 if hi > lo else 0
    coeffs = [rng.randrange(1, R_ORDER) for _ in range(T + 1)]
    sk = [poly_eval(coeffs, i + 1) for i in range(N_NODES)]
    pks = eng.g1_mul([g1] * N_NODES, sk)
    rs = [rng.randrange(1, R_ORDER) for _ in range(ncts)]
    hs = [rng.randrange(1, R_ORDER) for _ in range(ncts)]
    mine = list(range(clo, chi))
    us = eng.g1_mul([g1] * len(mine), [rs[c] for c in mine])                        # U = g1 r
    huv = eng.g2_mul([g2] * len(mine), [hs[c] for c in mine])                       # H_uv (synthetic hash)
    ws = eng.g2_mul([g2] * len(mine), [hs[c] * rs[c] % R_ORDER for c in mine])      # W = H_uv r
    bad = {c * N_NODES + (c * 29) % N_NODES for c in mine}
    items = list(range(lo, hi))
    shares = eng.g1_mul([us[inst[i] - clo] for i in items],
                        [(rng.randrange(1, R_ORDER) if i in bad else sk[i % N_NODES]) for i in items])
    expected = np.array([0 if i in bad else 1 for i in items], dtype=np.uint8)
    n = len(items)
    to_dev = lambda b: torch.from_numpy(np.frombuffer(b, dtype=np.uint8).copy()).to(dev)  # noqa: E731
    d_d = to_dev(b"".join(shares))
    d_pk = to_dev(b"".join(pks[i % N_NODES] for i in items))
    d_h = to_dev(b"".join(huv))
    d_w = to_dev(b"".join(ws))
    d_ci = torch.from_numpy((inst[lo:hi] - clo).astype(np.int32)).to(dev)
    streams = [torch.cuda.Stream(dev) for _ in range(max(1, args.streams))]
    d_vs = [torch.zeros(max(n, 1), dtype=torch.uint8, device=dev) for _ in streams]
    torch.cuda.synchronize(dev)

    def step(k=0):
        eng.verify_pairing_eq_dev(streams[k % len(streams)].cuda_stream, n, d_d.data_ptr(), d_h.data_ptr(), len(mine),
                                  d_ci.data_ptr(), d_pk.data_ptr(), d_w.data_ptr(), len(mine), d_ci.data_ptr(),
                                  d_vs[k % len(streams)].data_ptr())

    def verdicts_ok(nbuf=None):
        return all(bool((d.cpu().numpy()[:n] == expected).all()) for d in d_vs[:nbuf])

    for k in range(len(streams)):
        step(k)
    torch.cuda.synchronize(dev)
    ok = verdicts_ok()
    for k in range(args.warmup):
        step(k)
    torch.cuda.synchronize(dev)
    for d in d_vs:      # the timed steps must write every verdict again
        d.zero_()
    ms_step = timed_steps(step, streams, args.steps, world, dev)
    ok = ok and verdicts_ok(min(args.steps, len(streams)))
    from hbbft_amd._lib import STAGE_PAIRING, STAGE_PREPARE
    eng.set_profiling(True)   # roofline: isolated single-stream launches
    for _ in range(max(2, min(args.steps, 5))):
        step(0)
    torch.cuda.synchronize(dev)
    pair_ms, pair_n = eng.stage_time(STAGE_PAIRING)
    prep_ms, prep_n = eng.stage_time(STAGE_PREPARE)
    eng.set_profiling(False)
    ok = ok and verdicts_ok()
    # combines: first t+1 valid shares per ciphertext -> g = U * msk
    cidx, cpts = [], []
    for j, c in enumerate(mine):
        ids = [k for k in range(N_NODES) if expected[(c - clo) * N_NODES + k]][: T + 1]
        cidx.append(ids)
        cpts.append([shares[(c - clo) * N_NODES + k] for k in ids])
    from hbbft_amd._lib import STAGE_CURVE
    from hbbft_amd import workcount
    eng.interpolate_g1(T, cidx[:8], cpts[:8])  # warm-up
    eng.set_profiling(True)
    t0 = time.perf_counter()
    out, st = eng.interpolate_g1(T, cidx, cpts)
    comb_s = time.perf_counter() - t0
    comb_dev_ms, _ = eng.stage_time(STAGE_CURVE)
    eng.set_profiling(False)
    want = eng.g1_mul(us, [coeffs[0]] * len(mine))
    ok = ok and out == want and all(x == 0 for x in st)
    per_rank = gather_per_rank({"rank": rank, "checks": n, "ciphertexts": len(mine), "first_check": lo,
                                "kernel_ms": pair_ms / max(pair_n, 1), "ms_per_step": ms_step, "ok": ok}, world)
    ok = all(r["ok"] for r in per_rank)
    # the gathered outputs (verdicts of the last step, combined G1 points), in rank order = batch order:
    # their digests equal the one-rank run's when the shards are right (tests/test_bench_launch.py)
    blobs = gather_per_rank((d_vs[0].cpu().numpy()[:n].tobytes(), b"".join(out)), world)
    if rank == 0:
        main_k = roofline_entry(KERNEL_NAMES["decrypt"], pair_n, pair_ms / max(pair_n, 1), n,
                                workcount.PAIR_CHECK_TABLE, "decryption-share check", pair_waves_per_simd(n))
        kernels = [main_k]
        if prep_n:
            kernels.append(roofline_entry("hbs::k_oct_prep", prep_n, prep_ms / prep_n, 2 * len(mine),
                                          workcount.PAIR_PREP_DOC, "G2 point (H_uv, W) walk",
                                          2 * len(mine) * 8 / 64 / 1024))  # one lane octo per point
        line = {
            "metric": "verified decryption shares/sec (whole node), N=64 f=21", "value": total / (ms_step / 1e3),
            "unit": "shares/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup, "ms_per_step": ms_step,
            "higher_is_better": True, "scaling": "strong", "vs_baseline": None, "dtype": "u32 limbs (Fp, 14x28-bit)",
            "data": "synthetic, seeded (H_uv synthetic in G2; 1/64 invalid shares)",
            "config": {"workload": "ThresholdDecrypt, BASELINE configs[2]", "total_checks": total, "streams": len(streams),
                       "ciphertexts": ncts, "parallelism": "shard-by-ciphertext x%d" % world},
            "verdicts_ok": ok, "combines_ok": out == want, "per_rank": per_rank,
            "verdicts_sha256": hashlib.sha256(b"".join(b[0] for b in blobs)).hexdigest(),
            "combines_sha256": hashlib.sha256(b"".join(b[1] for b in blobs)).hexdigest(),
            "reference_work": reference_work(main_k, workcount),
            "combines_per_s_rank0": len(mine) / comb_s,                 # host-to-host, one call
            "combines_per_s_rank0_device": len(mine) / (comb_dev_ms / 1e3),
            "roofline": dict(main_k, bound="valu-int", unit="T MAD/s (v_mad_u64_u32 32x32->64)",
                             **traffic_fields(KERNEL_NAMES["decrypt"], "decrypt"), kernels=kernels,
                             note="both G2 sides (H_uv, W) are per-ciphertext line tables: per check = 2-pair "
                                  "Miller + final exp (workcount.PAIR_CHECK_TABLE)"),
        }
        if not args.no_cpu_baseline and world == 1:
            line["cpu_baseline"] = cpu_baseline_decrypt(shares, pks, huv, ws, us, inst, expected, cidx, cpts,
                                                        coeffs[0])
        print(json.dumps(line), flush=True)


def cpu_baseline_decrypt(shares, pks, huv, ws, us, inst, expected, cidx, cpts, msk, per_thread=8):
    """verify_decryption_share (e(D_i, H_uv) == e(pk_i, W), two pairings, C restatement) on a
    bounded sample, 1 thread and the CPU share; plus one combine_decryption_shares interpolation."""
    cbls = _ensure_oracle()
    ncpu, aff, threads = cpu_info()
    n_nodes = N_NODES

    def check(i):
        c = int(inst[i])
        return cbls.pairing_eq(shares[i], huv[c], pks[i % n_nodes], ws[c])

    n1 = 24
    st, v = timed_pool(check, list(range(n1)), 1)
    assert v == [bool(x) for x in expected[:n1]], "CPU decrypt verdicts disagree"
    n2 = threads * per_thread
    mt, v = timed_pool(check, list(range(n2)), threads)
    assert v == [bool(x) for x in expected[:n2]], "CPU decrypt verdicts disagree"
    t0 = time.perf_counter()
    rc, g = cbls.combine_g1(T, cidx[0], cpts[0])
    comb_ms = (time.perf_counter() - t0) * 1e3
    assert rc == 0 and g == cbls.g1_mul(us[0], msk)
    return {"value": n2 / mt, "unit": "shares/s", "cores": threads, "kind": "port",
            "sample": "%d decryption-share checks on %d threads (%d on 1 thread: %.1f shares/s); C restatement of "
                      "pairing 0.14, two pairings per check" % (n2, threads, n1, n1 / st),
            "single_thread_value": n1 / st, "combine_g1_ms": comb_ms, "nproc": ncpu, "affinity": aff}


def dkg_workload(eng, seed, n_nodes, t, nodes, tamper_every=97):
    """SyncKeyGen acks of configs[3]: n_nodes random degree-t bivariate polynomials (the Parts) and,
    for every checking node x in ``nodes`` (1-based), the acks (proposer p, sender y) of all
    n_nodes x n_nodes pairs with val = f_p(x, y) -- every value a node decrypts from an Ack
    (src/sync_key_gen.rs:515-547) -- 1/tamper_every of them tampered.  Values come from one
    object-array matrix product per Part (rows = X C, vals = rows Y^T mod r).
    Returns (commits, pidx, xs, ys, vals as n x 32 uint8 LE, expected verdict bytes)."""
    rng = random.Random(seed)
    npos = (t + 1) * (t + 2) // 2

    def cp(i, j):
        return j * (j + 1) // 2 + i if i <= j else i * (i + 1) // 2 + j

    coefs = [[rng.randrange(1, R_ORDER) for _ in range(npos)] for _ in range(n_nodes)]
    commits = eng.g1_mul_gen([c for cs in coefs for c in cs])
    commits = [commits[p * npos:(p + 1) * npos] for p in range(n_nodes)]
    nodes = list(nodes)
    X = np.array([[pow(x, i) for i in range(t + 1)] for x in nodes], dtype=object)
    Y = np.array([[pow(y, j) for y in range(1, n_nodes + 1)] for j in range(t + 1)], dtype=object)
    vals = []   # per node x, per part p: n_nodes values
    for p in range(n_nodes):
        C = np.array([[coefs[p][cp(i, j)] for j in range(t + 1)] for i in range(t + 1)], dtype=object)
        vals.append(((X @ C) % R_ORDER) @ Y % R_ORDER)     # [x][y]
    nx, n = len(nodes), len(nodes) * n_nodes * n_nodes
    pidx = np.repeat(np.tile(np.arange(n_nodes, dtype=np.uint32), nx), n_nodes)
    xs = np.repeat(np.array(nodes, dtype=np.uint32), n_nodes * n_nodes)
    ys = np.tile(np.arange(1, n_nodes + 1, dtype=np.uint32), nx * n_nodes)
    flat = [int(vals[p][k][y]) for k in range(nx) for p in range(n_nodes) for y in range(n_nodes)]
    # tampered: every tamper_every-th ack of the WHOLE network's order (x, p, y), so a node's acks
    # are the same whichever ranks check it (the rank split of tests/test_bench_launch.py)
    nn = n_nodes * n_nodes
    bad = {k * nn + a for k, x in enumerate(nodes) for a in range((-(x - 1) * nn) % tamper_every, nn, tamper_every)}
    for a in bad:
        flat[a] = (flat[a] + 1) % R_ORDER
    vb = np.frombuffer(b"".join(v.to_bytes(32, "little") for v in flat), dtype=np.uint8).reshape(n, 32)
    expected = bytes(0 if a in bad else 1 for a in range(n))
    return commits, pidx, xs, ys, vb, expected


def run_dkg(args, eng, world, rank, dev):
    """configs[3]: SyncKeyGen N=100 t=33 Ack checks (BivarCommitment::evaluate == g1*val,
    src/sync_key_gen.rs:542) over 100 Parts with 595-point commitments, held in a device-resident
    commitment set (uploaded once, as a SyncKeyGen instance keeps them).
    --dkg-scope network (default): the whole network's 10^6 checks -- all 100 nodes' 10,000 acks --
      split by checking node over the ranks (strong scaling: the total is fixed);
    --dkg-scope node: one node's 10,000 acks per rank (weak scaling: every rank plays one node)."""
    n_nodes, t = 100, 33
    npos = (t + 1) * (t + 2) // 2
    network = args.dkg_scope == "network"
    if network:
        nodes = [x for x in range(1, (args.dkg_nodes or n_nodes) + 1) if (x - 1) % world == rank]
    else:
        nodes = [rank + 1]
    eng.set_ack_impl({"auto": 0, "quad": 1, "lane": 2, "horner": 3}[args.ack_impl])
    t0 = time.perf_counter()
    commits, pidx, xs, ys, vals, expected = dkg_workload(eng, 100, n_nodes, t, nodes)
    gen_s = time.perf_counter() - t0
    cs = eng.commit_set(t)
    cs.add(commits)
    v = cs.ack_check(pidx, xs, ys, vals)            # warm-up: builds the rows row(x) once
    ok = v == expected
    if world > 1:
        dist.barrier()
    from hbbft_amd._lib import STAGE_CURVE
    from hbbft_amd import workcount
    times = []
    nsteps = max(1, args.steps // 2)
    eng.set_profiling(True)
    for _ in range(nsteps):
        t0 = time.perf_counter()
        v = cs.ack_check(pidx, xs, ys, vals)
        times.append((time.perf_counter() - t0) * 1e3)
        ok = ok and v == expected
    dev_ms, dev_n = eng.stage_time(STAGE_CURVE)
    eng.set_profiling(False)
    dev_ms /= max(dev_n, 1)
    nack = len(vals)
    # row build (once per (part, x), cached in the set) timed separately on a fresh set
    cs2 = eng.commit_set(t)
    cs2.add(commits)
    eng.set_profiling(True)
    cs2.ack_check(pidx[:1], xs[:1], ys[:1], vals[:1])
    row_ms, _ = eng.stage_time(STAGE_CURVE)
    eng.set_profiling(False)
    cs2.close()
    # BivarPoly::commitment (src/sync_key_gen.rs:346-357): the 595-point commitment of one Part, and
    # of all 100 Parts in one call, on the fixed-base comb table (hbh_g1_mul_gen); host-to-host
    crng = random.Random(7)
    commit_ms = {}
    for k in (1, n_nodes):
        sc = [crng.randrange(R_ORDER) for _ in range(k * npos)]
        eng.g1_mul_gen(sc[:8])
        ts_ = []
        for _ in range(5):
            t0 = time.perf_counter()
            eng.g1_mul_gen(sc)
            ts_.append((time.perf_counter() - t0) * 1e3)
        commit_ms[k] = statistics.median(ts_)
    enc = dkg_encrypt_cost(eng, n_nodes, t)
    node_round = dkg_node_round(eng, n_nodes, t) if rank == 0 and not args.no_node_round else None
    ms = _max_over_ranks(dev_ms, world, dev)
    host_ms = _max_over_ranks(statistics.median(times), world, dev)
    per_rank = gather_per_rank({"rank": rank, "device_ms": dev_ms, "host_ms": statistics.median(times), "ok": ok,
                                "acks": nack, "nodes": len(nodes), "node_list": nodes}, world)
    ok = all(r["ok"] for r in per_rank)
    total = sum(r["acks"] for r in per_rank)
    # verdicts per checking node, gathered: the digest over nodes in order equals the one-rank run's
    xa = np.asarray(xs)
    vb = np.frombuffer(bytes(v), dtype=np.uint8)
    by_node = {}
    for part in gather_per_rank({int(x): vb[xa == x].tobytes() for x in nodes}, world):
        by_node.update(part)
    if rank == 0:
        lane = args.ack_impl in ("lane", "horner") or (args.ack_impl == "auto" and nack >= ACK_LANE_MIN)
        fd = lane and args.ack_impl != "horner"
        if fd:   # every row (part, x) holds the acks of all senders y = 1..N: one dense run
            row = workcount.bivar_row_fd(t, 1, n_nodes, n_nodes)
            op = (row[0] / n_nodes, row[1] / n_nodes)
        else:
            ops = [workcount.bivar_ack(t, y) for y in range(1, n_nodes + 1)]
            op = (sum(o[0] for o in ops) / n_nodes, sum(o[1] for o in ops) / n_nodes)
        kname = ("hb::k_bivar_fd_seed + hb::k_bivar_fd_run + hb::k_bivar_fd_check" if fd else
                 "hb::k_bivar_check" if lane else "hbs::k_bivar_check_quad")
        waves = (1 if lane else 4) * nack / 64 / 1024
        main_k = roofline_entry(kname, dev_n, dev_ms, nack, op, "ack check", waves)
        line = {
            "metric": "SyncKeyGen ack checks/sec (%s), N=100 t=33" % ("whole network" if network else "whole node set"),
            "value": total / (ms / 1e3), "unit": "acks/s", "n_gpus": world, "steps": nsteps, "warmup": 1,
            "ms_per_step": ms, "higher_is_better": True, "scaling": "strong" if network else "weak",
            "vs_baseline": None, "dtype": "u32 limbs (Fp, 14x28-bit)",
            "data": "synthetic, seeded (100 random degree-33 bivariate polynomials; 1/97 tampered values)",
            "config": {"workload": "SyncKeyGen ack checks, BASELINE configs[3]", "scope": args.dkg_scope,
                       "total_acks": total, "acks_per_rank": nack, "checking_nodes_per_rank": len(nodes),
                       "parts": n_nodes, "commitment_points": npos,
                       "parallelism": ("checking nodes split over %d ranks" if network else "one node per rank x%d")
                       % world,
                       "timing": "device time of the ack-check kernel (HIP events) with the commitments and rows "
                                 "resident in HBM (commitment set); host_to_host_ms: the whole call incl. the "
                                 "upload of indices and values"},
            "host_to_host_ms": host_ms, "row_build_ms": row_ms, "rows": len(nodes) * n_nodes,
            "encrypt": enc,
            "node_round": node_round,
            "bivar_commitment_ms": {"1 part (595 points)": commit_ms[1], "100 parts (59,500 points)": commit_ms[n_nodes],
                                    "note": "BivarPoly::commitment on the comb table (hbh_g1_mul_gen), host-to-host"},
            "data_gen_s": round(gen_s, 2), "verdicts_ok": ok, "per_rank": per_rank,
            "verdicts_sha256": hashlib.sha256(b"".join(by_node[x] for x in sorted(by_node))).hexdigest(),
            "roofline": dict(main_k, bound="valu-int", unit="T MAD/s (v_mad_u64_u32 32x32->64)",
                             note="%s; %.1f waves per SIMD launched" % (
                                 "finite differences over each row's dense y run (Horner at t + 1 points, t "
                                 "additions per further y; per-ack work = the row's work / its acks)" if fd else
                                 "one lane per ack on affine rows" if lane else "four lanes per ack (lane quads)",
                                 waves)),
            "ack_impl": kname,
        }
        if not args.no_cpu_baseline and world == 1:
            line["cpu_baseline"] = cpu_baseline_dkg(t, commits, pidx, xs, ys, vals, expected, eng)
        print(json.dumps(line), flush=True)
    cs.close()


def dkg_encrypt_cost(eng, n_nodes, t, reps=3):
    """The DKG's generation side: PublicKey::encrypt_with_rng of one Part's N rows
    (src/sync_key_gen.rs:346-357: bincode Poly of t+1 Fr, 1,096 B) and of one Ack's N values (:386-390:
    32-byte Fr) on the host stage (hbh_encrypt: U = g1 r, V = msg ^ hash(pk r), W = hash_g1_g2(U, V) r),
    host-to-host, median of reps.  A node encrypts one Part and one Ack per Part it accepts:
    N + N^2 encryptions per DKG (10,100 at N = 100)."""
    from hbbft_amd import hoststage
    from hbbft_amd.sync_key_gen import ser_row
    rng = random.Random(11)
    g1 = g1a_abi()
    pks = eng.g1_mul([g1] * n_nodes, [rng.randrange(1, R_ORDER) for _ in range(n_nodes)])
    rows = [ser_row([rng.randrange(R_ORDER) for _ in range(t + 1)]) for _ in range(n_nodes)]
    vals = [rng.randrange(R_ORDER).to_bytes(32, "little") for _ in range(n_nodes)]
    threads = hoststage.host_threads()
    out = {}
    for name, msgs in (("part_rows_ms", rows), ("ack_values_ms", vals)):
        ts_ = []
        for _ in range(reps):
            nonces = [rng.randrange(1, R_ORDER) for _ in msgs]
            t0 = time.perf_counter()
            hoststage.encrypt(pks, msgs, nonces, threads=threads)
            ts_.append((time.perf_counter() - t0) * 1e3)
        out[name] = statistics.median(ts_)
    out["per_node_dkg_ms"] = out["part_rows_ms"] + n_nodes * out["ack_values_ms"]
    out["encryptions_per_node"] = n_nodes + n_nodes * n_nodes
    out["host_threads"] = threads
    out["note"] = ("host stage, %d threads; one Part = %d row encryptions, one Ack = %d value encryptions; "
                   "per_node_dkg_ms = one Part + %d Acks" % (threads, n_nodes, n_nodes, n_nodes))
    return out


def dkg_node_round(eng, n_nodes, t, seed=5):
    """One node's whole SyncKeyGen round through hbbft_amd.sync_key_gen (src/sync_key_gen.rs): generate
    our Part (SyncKeyGen::new: BivarPoly::random, its commitment, N row encryptions, :323-357), handle
    the N Parts (decrypt our row of each, Poly::commitment == row(x), one Ack of N value encryptions per
    valid Part, :372-392, 481-512) and the N^2 Acks (decrypt our value of each, evaluate == g1 val,
    :398-404, 515-547) -- every SecretKey::decrypt, encrypt_with_rng, hash and check a node runs.
    Setup (untimed): the other nodes' Parts and Acks; in each only the ciphertext addressed to our node
    is real (the others are a copy of it: our node reads only its own, checks only the count).
    Returns the timings and whether every outcome is fault-free."""
    from hbbft_amd import hoststage
    from hbbft_amd.sync_key_gen import SyncKeyGen, Part, Ack, Ciphertext, coeff_pos, ser_row, ser_val
    rng = random.Random(seed)
    g1 = g1a_abi()
    sks = [rng.randrange(1, R_ORDER) for _ in range(n_nodes)]
    pks = dict(enumerate(eng.g1_mul([g1] * n_nodes, sks)))
    our = 0
    ox = our + 1
    npos = (t + 1) * (t + 2) // 2
    coefs = [[rng.randrange(R_ORDER) for _ in range(npos)] for _ in range(n_nodes)]
    flat = eng.g1_mul_gen([c for cs in coefs for c in cs])
    commits = [flat[p * npos:(p + 1) * npos] for p in range(n_nodes)]
    ys = list(range(1, n_nodes + 1))
    # our row of part p: row_p(ox)_a = sum_b c_p(a, b) ox^b; the values acks carry for us: f_p(y, ox)
    our_rows = [[poly_eval([coefs[p][coeff_pos(a, b)] for b in range(t + 1)], ox) for a in range(t + 1)]
                for p in range(n_nodes)]
    our_vals = hoststage.fr_poly_eval(our_rows, ys)
    threads = hoststage.host_threads()
    row_cts = hoststage.encrypt([pks[our]], [ser_row(r) for r in our_rows],
                                [rng.randrange(1, R_ORDER) for _ in range(n_nodes)], threads)
    val_cts = hoststage.encrypt([pks[our]], [ser_val(v) for vs in our_vals for v in vs],
                                [rng.randrange(1, R_ORDER) for _ in range(n_nodes * n_nodes)], threads)
    parts = [(p, Part(t, commits[p], [Ciphertext(*row_cts[p])] * n_nodes)) for p in range(n_nodes)]
    acks = [(y - 1, Ack(p, [Ciphertext(*val_cts[p * n_nodes + y - 1])] * n_nodes))
            for p in range(n_nodes) for y in ys]
    out = {}
    # one untimed Part first: the process's one-time lazy set-up (host comb tables, engine tables,
    # kernel modules) is not part of a node's round
    SyncKeyGen.new(our, sks[our], pks, t, eng, rng=random.Random(seed + 3), threads=threads)
    t0 = time.perf_counter()
    _, own_part = SyncKeyGen.new(our, sks[our], pks, t, eng, rng=random.Random(seed + 1), threads=threads)
    out["generate_part_ms"] = (time.perf_counter() - t0) * 1e3
    kg = SyncKeyGen(our, sks[our], pks, t, eng, threads=threads)
    t0 = time.perf_counter()
    p_out = kg.handle_parts(parts, rng=random.Random(seed + 2))
    out["handle_parts_ms"] = (time.perf_counter() - t0) * 1e3
    t0 = time.perf_counter()
    a_out = kg.handle_acks(acks)
    out["handle_acks_ms"] = (time.perf_counter() - t0) * 1e3
    out["node_round_ms"] = out["generate_part_ms"] + out["handle_parts_ms"] + out["handle_acks_ms"]
    ok = (own_part is not None and len(own_part.rows) == n_nodes
          and all(o.valid and o.ack is not None and len(o.ack.values) == n_nodes for o in p_out)
          and all(o.valid for o in a_out) and kg.is_ready())
    out.update({"outcomes_ok": ok, "host_threads": threads, "encryptions": n_nodes + n_nodes * n_nodes,
                "decryptions": n_nodes + n_nodes * n_nodes, "parts": n_nodes, "acks": n_nodes * n_nodes,
                "note": "one node's SyncKeyGen round through hbbft_amd.sync_key_gen, host-to-host: host stage "
                        "(hash_g1_g2, encrypt_with_rng, U*sk, Fr Horner) on %d threads, engine calls "
                        "(Ciphertext::verify, Poly::commitment, ack checks) on the GPU" % threads})
    return out


def g1a_abi():
    from hbbft_amd.engine import g1_abi_from_uncompressed as g1a
    return g1a(G1_UNC)


def cpu_baseline_dkg(t, parts, pidx, xs, ys, vals, expected, eng, per_thread=16):
    """The reference's ack check (BivarCommitment::evaluate(x, y) == g1 * val, sync_key_gen.rs:542,
    C restatement: 595-term evaluation + one scalar multiplication) on a bounded sample."""
    from hbbft_amd.engine import g1_abi_from_uncompressed as g1a
    cbls = _ensure_oracle()
    ncpu, aff, threads = cpu_info()
    g1 = g1a(G1_UNC)

    def check(a):
        lhs = cbls.bivar_evaluate(t, parts[int(pidx[a])], int(xs[a]), int(ys[a]))
        return lhs == cbls.g1_mul(g1, int.from_bytes(bytes(vals[a]), "little"))

    n1 = 8
    st, v = timed_pool(check, list(range(n1)), 1)
    assert v == [bool(expected[a]) for a in range(n1)], "CPU ack verdicts disagree"
    n2 = threads * per_thread
    mt, v = timed_pool(check, list(range(n2)), threads)
    assert v == [bool(expected[a]) for a in range(n2)], "CPU ack verdicts disagree"
    return {"value": n2 / mt, "unit": "acks/s", "cores": threads, "kind": "port",
            "sample": "%d ack checks on %d threads (%d on 1 thread: %.1f acks/s); C restatement of "
                      "BivarCommitment::evaluate + G1 scalar multiplication" % (n2, threads, n1, n1 / st),
            "single_thread_value": n1 / st, "nproc": ncpu, "affinity": aff}


def run_epoch_bench(args, eng, world, rank, dev):
    """configs[4]: the threshold-crypto work of one node in a HoneyBadger epoch at N=100, f=33
    (hbbft_amd/honey_badger.py): 100 BA threshold coins + 100 ThresholdDecrypt instances through
    the mirrored flows with windowed drains and batched combines.  One step = one epoch (a fresh
    trace each); every rank plays its own node (weak scaling, no collective)."""
    from hbbft_amd import workcount
    from hbbft_amd._lib import STAGE_CURVE, STAGE_PAIRING, STAGE_PREPARE
    from hbbft_amd.honey_badger import EpochTrace, NetworkKeys, prefetch_coins, run_epoch
    rng = random.Random(5000 + rank)
    n, f = 100, 33
    keys = NetworkKeys(eng, n, f, rng)
    t0 = time.time()
    # one trace beyond the timed epochs: the last timed epoch prefetches its coin documents
    traces = [EpochTrace.generate(eng, keys, rng, hb_epoch=e, proposal_bytes=1000)
              for e in range(args.warmup + args.steps + 1)]
    if args.epoch_coins == "ba":  # coins from Binary Agreement instances (future-epoch queue, per-window combines)
        for tr in traces:
            tr.with_ba(eng, rng, extra=0.0)
    if args.raw:  # the bincode bytes the node receives (hbbft_amd.wire); decoding is inside the timed epochs
        for tr in traces:
            tr.serialize()
    log("generated %d epoch traces in %.1f s" % (len(traces), time.time() - t0))
    ok = True
    # each epoch starts the next one's coin prefetch (honey_badger.prefetch_coins: hash_g2 and our
    # share of the next epoch's BA coin documents, on the host-stage thread); the timed region
    # waits for the prefetch the last timed epoch started, so every timed epoch carries one
    pf_on = args.epoch_coins == "ba" and not args.no_prefetch

    def prefetch(k):
        return prefetch_coins(keys, traces[k].hb_epoch, range(n)) if pf_on else None

    pf = prefetch(0)

    def epoch_with_prefetch(k, tr, pf):
        # the next epoch's coin prefetch starts once this epoch's decryption prep has the host threads
        # to itself (after_prep) with --prefetch-after-prep; by default with the epoch (round 5: the prep
        # takes well under a millisecond, and the early prefetch measured 25.6-27.0 vs 22.4-23.9 epochs/s, c16)
        box, ev = [], threading.Event()

        def start_next():
            box.append(prefetch(k + 1))
            ev.set()

        if not args.prefetch_after_prep:
            start_next()
        r = run_epoch(eng, keys, tr, window=args.window, pipelined=args.pipeline, coin_prefetch=pf, raw=args.raw,
                      preverify=not args.no_preverify, preverify_at=args.preverify_at,
                      after_prep=start_next if args.prefetch_after_prep else None)
        ev.wait()  # (the prep's done-callback may still be running on its pool thread)
        return r, box[0]

    for k, tr in enumerate(traces[:args.warmup]):
        r, pf = epoch_with_prefetch(k, tr, pf)
        ok = ok and r.plaintexts == tr.proposals
    if world > 1:
        dist.barrier()
    results = []
    eng.set_profiling(True)
    # the second engine (decryption-share pre-verification beside the coin phase; pipelined
    # combines): its kernels count as GPU time too
    from hbbft_amd.honey_badger import combine_engine
    ceng = combine_engine(eng)
    ceng.set_profiling(True)
    prof = None
    if args.profile_epoch:
        import cProfile
        prof = cProfile.Profile()
        prof.enable()
    t0 = time.perf_counter()
    for k in range(args.warmup, len(traces) - 1):
        r, pf = epoch_with_prefetch(k, traces[k], pf)
        results.append(r)
    if pf is not None:
        pf.result()
    wall = time.perf_counter() - t0
    if prof is not None:
        import pstats
        prof.disable()
        with open(args.profile_epoch, "w") as fh:
            pstats.Stats(prof, stream=fh).sort_stats("tottime").print_stats(45)
    pair_ms, pair_n = eng.stage_time(STAGE_PAIRING)
    stage_ms = {name: eng.stage_time(st)[0] + (ceng.stage_time(st)[0] if ceng else 0.0) for name, st in
                (("line_tables", STAGE_PREPARE), ("pairing", STAGE_PAIRING), ("curve", STAGE_CURVE))}
    eng.set_profiling(False)
    if ceng:
        ceng.set_profiling(False)
    for tr, r in zip(traces[args.warmup:-1], results):
        ok = ok and r.plaintexts == tr.proposals and len(r.coins) == len(tr.coin_docs)
        if args.epoch_coins == "ba":
            ok = ok and r.ba_decisions == tr.ba.decision and r.ba_coins == tr.ba.coins
    ms = _max_over_ranks(wall * 1e3 / args.steps, world, dev)
    if rank == 0:
        drained = sum(r.checks_gpu for r in results)
        consumed = sum(r.checks_consumed for r in results) / len(results)
        phases = {k: sum(r.timing[k] for r in results) / len(results) * 1e3 for k in results[0].timing}
        waits = {k: sum(r.wait.get(k, 0.0) for r in results) / len(results) * 1e3 for k in results[0].wait}
        kern = {k: v / len(results) for k, v in stage_ms.items()}
        # host time = the epoch minus the time the flows sat blocked on engine calls (GPU kernels,
        # copies and the engine's own host work); the kernels' own time is the event-timed stages
        host_gpu = {"epoch_ms": phases["epoch"], "blocked_on_engine_ms": sum(waits.values()),
                    "host_ms": phases["epoch"] - sum(waits.values()), "gpu_kernel_ms": sum(kern.values()),
                    "blocked_by_phase_ms": waits, "gpu_kernel_by_stage_ms": kern}
        host_gpu["host_over_gpu"] = host_gpu["host_ms"] / max(host_gpu["gpu_kernel_ms"], 1e-9)
        if args.pipeline:
            host_gpu["pipelined_ms"] = {k: sum(r.overlap.get(k, 0.0) for r in results) / len(results) * 1e3
                                        for k in ("hand_s", "worker_engine_s")}
        # AUTO sends drains of <= HBH_AUTO_WAVE_MAX (4,096) checks to the wave kernel, <= 8,192 to the
        # lane-octo kernel and larger ones to the lane quad; the stage time is all of them
        main_k = roofline_entry("hbs::k_wave + hbs::k_oct_verify (AUTO by drain size)", pair_n,
                                pair_ms / max(pair_n, 1), drained / max(pair_n, 1),
                                workcount.PAIR_CHECK_WALK, "share / ciphertext check")
        line = {
            "metric": "HoneyBadger epochs/sec, one node's threshold crypto, N=100 f=33", "value": world * 1e3 / ms,
            "unit": "epochs/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup, "ms_per_step": ms,
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "u32 limbs (Fp, 14x28-bit)",
            "data": "synthetic, seeded (dealer key set, 1,000-byte contributions, 100 coin documents per epoch, "
                    "1/64 forged shares); messages in random order",
            "config": {"workload": "HoneyBadger epoch crypto trace, BASELINE configs[4]", "n_nodes": n, "f": f,
                       "coins_per_epoch": len(traces[0].coin_docs), "window": args.window,
                       "coins_from": ("BinaryAgreementCoin instances (epochs 0-2, coin shares through the future-epoch "
                                      "queue, combines deferred per window)" if args.epoch_coins == "ba"
                                      else "synthetic: one ThresholdSign per BA instance at epoch 2"),
                       "pipelined_drains": args.pipeline,
                       "from_wire_bytes": args.raw,
                       "coin_prefetch": pf_on, "coin_prefetch_start": "after_prep" if args.prefetch_after_prep else "epoch",
                       "dec_preverify": not args.no_preverify and not args.raw, "dec_preverify_at": args.preverify_at,
                       "parallelism": "one node per rank x%d" % world,
                       "timing": "host wall time of run_epoch (flows + host stage + engine calls)"},
            "outputs_ok": ok, "phase_ms": phases, "host_vs_gpu": host_gpu,
            "engine_calls_per_epoch": sum(r.engine_calls for r in results) / len(results),
            "checks_drained_per_epoch": drained / len(results), "checks_consumed_per_epoch": consumed,
            #  checks verified on the GPU that no instance read: shares pre-verified
            # for instances that terminated first (the reference never verifies those,
            # threshold_sign.rs:182-184, threshold_decrypt.rs:183-185) -- latency hiding, priced at the
            # drains' average kernel time per check
            "checks_unconsumed_per_epoch": drained / len(results) - consumed,
            "unconsumed_gpu_ms_per_epoch_est": (kern.get("pairing", 0.0) + kern.get("line_tables", 0.0))
            * max(0.0, 1.0 - consumed * len(results) / max(drained, 1)),
            "roofline": dict(main_k, bound="valu-int", unit="T MAD/s (v_mad_u64_u32 32x32->64)", traffic=None,
                             traffic_note="the drains mix kernels at varying sizes; their per-launch HBM is in "
                                          "profiles/r04/pmc_traffic.json (by_source wave4k: k_wave 4,096 checks, "
                                          "oct8k: k_oct_verify 8,192 checks, quad16k: k_quad_verify 16,384 checks)",
                             note="drains of different sizes (a few thousand checks, 100 ciphertexts, 100 master "
                                  "verifies) run below one wave per SIMD: latency-bound; no single occupancy ceiling"),
        }
        if not args.no_cpu_baseline and world == 1:
            # the last timed epoch's trace (traces[-1] only feeds the last prefetch)
            line["cpu_baseline"] = cpu_baseline_epoch(eng, keys, traces[args.warmup + len(results) - 1], results[-1])
        print(json.dumps(line), flush=True)


def cpu_baseline_epoch(eng, keys, tr, res, sample=12):
    """The same epoch on the reference-equivalent CPU path: one pairing check (C restatement) per
    verdict the flows consumed (the reference verifies each share as it arrives, on the node's one
    thread), one G2 combine + master verify per coin and one G1 interpolation per ciphertext;
    per-item costs timed on a bounded sample and multiplied by this epoch's counts."""
    cbls = _ensure_oracle()
    ncpu, aff, threads = cpu_info()
    t = keys.t
    coin = sorted(tr.coin_docs)[0]
    h = tr.hashes[coin]
    items = [(j, tr.coin_shares[(coin, j)]) for j in range(1, keys.n)][:sample]
    t0 = time.perf_counter()
    for j, sgm in items:
        cbls.verify_g2(keys.pks[j], sgm, h)
    per_check = (time.perf_counter() - t0) / len(items)
    ids = [j for j in range(1, keys.n) if ("coin", coin, j) not in tr.bad][:t + 1]
    t0 = time.perf_counter()
    rc, sig = cbls.combine_g2(t, ids, [tr.coin_shares[(coin, j)] for j in ids])
    ok = cbls.verify_g2(keys.master_pk, sig, h)
    comb_g2 = time.perf_counter() - t0
    assert rc == 0 and ok and sig == res.signatures[coin], "CPU coin combine differs"
    p = 0
    ids = [j for j in range(1, keys.n) if ("dec", p, j) not in tr.bad][:t + 1]
    t0 = time.perf_counter()
    rc, g = cbls.combine_g1(t, ids, [tr.dec_shares[(p, j)] for j in ids])
    comb_g1 = time.perf_counter() - t0
    assert rc == 0 and g == cbls.g1_mul(tr.cts[p][0], keys.msk), "CPU decryption combine differs"
    ncoin, nct = len(res.coins), len(res.plaintexts)
    epoch_s = res.checks_consumed * per_check + ncoin * comb_g2 + nct * comb_g1
    return {"value": 1.0 / epoch_s, "unit": "epochs/s", "cores": 1, "kind": "port",
            "sample": "%d verify_g2 checks, 1 G2 combine+verify, 1 G1 combine timed on one thread, scaled to the "
                      "epoch's %d consumed checks, %d coins, %d decryptions (a HoneyBadger node handles its "
                      "messages on one thread)" % (len(items), res.checks_consumed, ncoin, nct),
            "epoch_ms": epoch_s * 1e3, "per_check_ms": per_check * 1e3, "combine_g2_ms": comb_g2 * 1e3,
            "combine_g1_ms": comb_g1 * 1e3, "nproc": ncpu, "affinity": aff}


def run_pool(args):
    """--launcher pool: ONE process drives the in-ABI engine pool (hbh_pool_*, csrc/pool.cpp) over
    --gpus N shards (devices 0..N-1, or HBH_POOL_DEVICES).  Weak scaling like the ranks path: the
    batch is N x --batch checks over N x the documents (each shard's slice = one configs[1] batch),
    split by instance inside the pool, one host thread and stream per shard, verdicts gathered in
    order.  The pool's entry points take HOST buffers, so a step here is host-to-host (the PCIe
    upload of 288 B per check and the verdict download included); the per-shard kernel times are
    the engines' HIP-event times.  Workloads: sign, decrypt (1,024 x N ciphertexts)."""
    import ctypes
    from hbbft_amd import workcount
    from hbbft_amd._lib import STAGE_PAIRING, buf, check
    from hbbft_amd.engine import Engine, Pool
    if args.workload not in ("sign", "decrypt"):
        raise SystemExit("bench.py: --launcher pool runs the sign and decrypt workloads")
    devs = pool_devices(args.gpus)
    nsh = len(devs)
    gen = Engine(devs[0])
    n = args.batch
    w = Workload(gen, n, seed=20261016)
    nh = len(w.hashes)
    total = n * nsh
    di = np.ascontiguousarray(np.concatenate([w.doc_idx + s * nh for s in range(nsh)]).astype(np.uint32))
    expected = np.tile(w.expected, nsh)
    if args.workload == "sign":
        ins = [w.pk_batch * nsh, w.sig_batch * nsh, w.hash_table * nsh]
        fn_name, kernel, op, unit_name = ("hbh_verify_sig_shares", KERNEL_NAMES["pair"], workcount.PAIR_CHECK_WALK,
                                          "share check")
    else:
        # decryption shares with the sign batch's layout: D_i = U_c * sk_i, H_uv / W per ciphertext
        rng = random.Random(4243)
        rs = [rng.randrange(1, R_ORDER) for _ in range(nh)]
        us = gen.g1_mul([w.g1] * nh, rs)
        ws = gen.g2_mul(w.hashes, rs)                                              # W = H_uv r
        bad = np.nonzero(w.expected == 0)[0]
        dsh = gen.g1_mul([us[w.doc_idx[i]] for i in range(n)],
                         [rng.randrange(1, R_ORDER) if i in set(bad) else w.sk[w.node[i]] for i in range(n)])
        ins = [b"".join(dsh) * nsh, w.pk_batch * nsh, w.hash_table * nsh, b"".join(ws) * nsh]
        fn_name, kernel, op, unit_name = ("hbh_verify_dec_shares", KERNEL_NAMES["decrypt"],
                                          workcount.PAIR_CHECK_TABLE, "decryption-share check")
    gen.close()
    pool = Pool(devs)
    pool.set_pairing_impl(IMPLS[args.impl])
    keep = [buf(b) for b in ins]
    out = (ctypes.c_uint8 * total)()
    pout = ctypes.cast(out, ctypes.c_void_p)
    pdi = di.ctypes.data_as(ctypes.c_void_p)
    fn = getattr(pool._l, fn_name)

    def step():
        ptrs = [k[1] for k in keep]
        if args.workload == "sign":
            check(fn(pool._h, total, ptrs[0], ptrs[1], ptrs[2], nh * nsh, pdi, pout))
        else:
            check(fn(pool._h, total, ptrs[0], ptrs[1], ptrs[2], ptrs[3], nh * nsh, pdi, pout))

    def verdicts_ok():
        return bool((np.frombuffer(bytes(out), dtype=np.uint8) == expected).all())

    step()
    ok = verdicts_ok()
    for _ in range(args.warmup):
        step()
    ctypes.memset(out, 0, total)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    ms_step = (time.perf_counter() - t0) * 1e3 / args.steps
    ok = ok and verdicts_ok()
    engines = [pool.shard_engine(s) for s in range(nsh)]
    for e in engines:
        e.set_profiling(True)
    step()
    per_shard = []
    for s, e in enumerate(engines):
        ms, nl = e.stage_time(STAGE_PAIRING)
        per_shard.append({"shard": s, "device": devs[s], "kernel_ms": ms / max(nl, 1), "launches": nl})
        e.set_profiling(False)
    ok = ok and verdicts_ok()
    kern = max(p["kernel_ms"] for p in per_shard)
    main_k = roofline_entry(kernel, 1, kern, n, op, unit_name, pair_waves_per_simd(n))
    metric = METRIC if args.workload == "sign" else "verified decryption shares/sec (whole node), N=64 f=21"
    line = {
        "metric": metric, "value": total / (ms_step / 1e3), "unit": "shares/s", "n_gpus": len(set(devs)),
        "shards": nsh, "steps": args.steps, "warmup": args.warmup, "ms_per_step": ms_step,
        "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "u32 limbs (Fp, 14x28-bit)",
        "data": "synthetic, seeded (one configs[1] batch per shard; 1/64 invalid)",
        "config": {"workload": "%s through the engine pool, BASELINE configs[1]/[2]" % args.workload,
                   "batch_per_shard": n, "documents_per_shard": nh, "devices": devs,
                   "parallelism": "engine pool, shard-by-instance x%d" % nsh,
                   "timing": "host-to-host pool calls (PCIe upload + verdict gather included)"},
        "verdicts_ok": ok, "per_shard": per_shard,
        "roofline": dict(main_k, bound="valu-int", unit="T MAD/s (v_mad_u64_u32 32x32->64)",
                         note="slowest shard's kernel time (HIP events on the shard's stream)"),
    }
    print(json.dumps(line), flush=True)
    pool.close()


def run_other(args):
    world, rank, local = _dist_env()
    dev = torch.device("cuda", local)
    from hbbft_amd.engine import Engine
    eng = Engine(local)
    if args.workload == "decrypt":
        run_decrypt(args, eng, world, rank, dev)
    elif args.workload == "epoch":
        run_epoch_bench(args, eng, world, rank, dev)
    else:
        run_dkg(args, eng, world, rank, dev)
    eng.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
