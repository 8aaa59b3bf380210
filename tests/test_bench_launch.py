"""bench.py honours --gpus N: never a silent one-GPU run.

CPU: too few visible devices, a WORLD_SIZE that disagrees with --gpus and a pool over absent
devices all exit non-zero before any GPU work.  GPU (one MI355X): the pool path with two shards
on device 0 and the spawned-ranks path with two ranks rehearsed on device 0 (gloo) both report
their shards / ranks and exact verdicts."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(ROOT, "bench.py")


def _run(args, env_extra, timeout=120):
    env = dict(os.environ)
    env.update(env_extra)
    return subprocess.run([sys.executable, BENCH] + args, env=env, capture_output=True, text=True, timeout=timeout)


def test_too_few_devices_exits_nonzero():
    r = _run(["--gpus", "2", "--steps", "1", "--warmup", "0"], {"HIP_VISIBLE_DEVICES": "", "CUDA_VISIBLE_DEVICES": ""})
    assert r.returncode != 0 and "devices visible" in r.stderr
    assert not r.stdout.strip()


def test_world_size_must_match_gpus():
    r = _run(["--gpus", "2", "--steps", "1"], {"WORLD_SIZE": "4", "RANK": "0", "LOCAL_RANK": "0"})
    assert r.returncode == 2 and "WORLD_SIZE=4" in r.stderr


def test_pool_over_absent_devices_exits_nonzero():
    r = _run(["--gpus", "2", "--launcher", "pool"], {"HIP_VISIBLE_DEVICES": "", "CUDA_VISIBLE_DEVICES": ""})
    assert r.returncode == 2


def _json_line(out):
    lines = [l for l in out.splitlines() if l.startswith("{")]
    assert len(lines) == 1, out
    return json.loads(lines[0])


@pytest.mark.gpu
def test_pool_bench_two_shards_on_device0():
    r = _run(["--gpus", "2", "--launcher", "pool", "--batch", "4096", "--steps", "2", "--warmup", "1"],
             {"HBH_POOL_DEVICES": "0,0"}, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    d = _json_line(r.stdout)
    assert d["verdicts_ok"] is True
    assert d["shards"] == 2 and d["n_gpus"] == 1 and len(d["per_shard"]) == 2
    assert all(p["launches"] >= 1 and p["kernel_ms"] > 0 for p in d["per_shard"])


@pytest.mark.gpu
def test_spawned_ranks_rehearsed_on_device0():
    r = _run(["--gpus", "2", "--batch", "4096", "--steps", "2", "--warmup", "1", "--no-combine",
              "--no-cpu-baseline"], {"HBH_DIST_BACKEND": "gloo"}, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    d = _json_line(r.stdout)
    assert d["n_gpus"] == 2 and d["verdicts_ok"] is True and len(d["per_rank"]) == 2


def _strong_pair(workload, extra, timeout=600):
    """The same strong-scaled workload on one rank and on two ranks rehearsed on device 0 (gloo):
    (one-rank line, two-rank line)."""
    base = ["--workload", workload, "--steps", "2", "--warmup", "1", "--no-cpu-baseline"] + extra
    r1 = _run(base + ["--gpus", "1"], {}, timeout=timeout)
    assert r1.returncode == 0, r1.stderr[-3000:]
    r2 = _run(base + ["--gpus", "2"], {"HBH_DIST_BACKEND": "gloo"}, timeout=timeout)
    assert r2.returncode == 0, r2.stderr[-3000:]
    return _json_line(r1.stdout), _json_line(r2.stdout)


@pytest.mark.gpu
def test_decrypt_two_ranks_match_one_rank():
    """configs[2] split by ciphertext over two ranks (src/threshold_decrypt.rs:220-250):
    the per-rank checks sum to the batch, and the gathered verdicts and G1 combines are byte-identical
    to the one-rank run (digests over the rank-ordered concatenation)."""
    d1, d2 = _strong_pair("decrypt", [])
    assert d1["n_gpus"] == 1 and d2["n_gpus"] == 2
    assert d1["verdicts_ok"] is True and d2["verdicts_ok"] is True
    total = d1["config"]["total_checks"]
    assert d2["config"]["total_checks"] == total
    assert len(d2["per_rank"]) == 2 and sum(r["checks"] for r in d2["per_rank"]) == total
    assert sum(r["ciphertexts"] for r in d2["per_rank"]) == d1["config"]["ciphertexts"]
    assert d2["per_rank"][1]["first_check"] == d2["per_rank"][0]["checks"]  # contiguous ranges in order
    assert d2["verdicts_sha256"] == d1["verdicts_sha256"]
    assert d2["combines_sha256"] == d1["combines_sha256"]


@pytest.mark.gpu
def test_dkg_two_ranks_match_one_rank():
    """configs[3] network scope split by checking node over two ranks (src/sync_key_gen.rs:515-547):
    the per-rank acks sum to the total, every node is checked exactly once, and the gathered
    verdicts (per node, in node order) equal the one-rank run's."""
    d1, d2 = _strong_pair("dkg", ["--dkg-nodes", "6", "--no-node-round"])
    assert d1["n_gpus"] == 1 and d2["n_gpus"] == 2
    assert d1["verdicts_ok"] is True and d2["verdicts_ok"] is True
    assert d2["config"]["total_acks"] == d1["config"]["total_acks"] == 6 * 100 * 100
    assert sum(r["acks"] for r in d2["per_rank"]) == d1["config"]["total_acks"]
    nodes = sorted(x for r in d2["per_rank"] for x in r["node_list"])
    assert nodes == list(range(1, 7))
    assert d2["verdicts_sha256"] == d1["verdicts_sha256"]


@pytest.mark.gpu
def test_pool_decrypt_two_shards_on_device0():
    r = _run(["--gpus", "2", "--launcher", "pool", "--workload", "decrypt", "--batch", "4096", "--steps", "2",
              "--warmup", "1"], {"HBH_POOL_DEVICES": "0,0"}, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    d = _json_line(r.stdout)
    assert d["verdicts_ok"] is True and d["shards"] == 2 and len(d["per_shard"]) == 2
