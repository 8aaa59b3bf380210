"""The C-ABI boundary driven from C alone (examples/threshold_flow.c): the ThresholdSign scenario of
tests/threshold_sign.rs (N = 10, f = 3: shares verified, a forged share rejected, the first t + 1
valid shares combined and checked against the master key, byte-equal to msk * H, DuplicateEntry)
and a ThresholdDecrypt round (Ciphertext::verify incl. a tampered W, decryption-share checks with
one garbage share, interpolation, plaintext) -- no Python between the caller and
libhbbft_hip.so.  The CPU test compiles and links it; the gpu test runs it."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "examples", "threshold_flow.c")
LIBDIR = os.path.join(ROOT, "hbbft_amd")


def build(tmp_path):
    exe = str(tmp_path / "threshold_flow")
    subprocess.run(["gcc", "-O2", "-Wall", "-Werror", "-I", os.path.join(ROOT, "include"), SRC, "-L", LIBDIR,
                    "-lhbbft_hip", "-Wl,-rpath," + LIBDIR, "-o", exe], check=True, timeout=120)
    return exe


def test_c_harness_builds(tmp_path):
    if not os.path.exists(os.path.join(LIBDIR, "libhbbft_hip.so")):
        pytest.skip("libhbbft_hip.so not built")
    assert os.path.exists(build(tmp_path))


@pytest.mark.gpu
@pytest.mark.parametrize("seed", ["7", "20260501"])
def test_c_harness_runs(tmp_path, seed):
    exe = build(tmp_path)
    r = subprocess.run([exe, seed], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    assert r.stdout.strip().endswith("threshold_flow OK"), r.stdout
