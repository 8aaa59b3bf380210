"""The device inversion's two forms agree (CPU: hbbft_amd/csrc/words.hpp compiled with g++): the wave
kernel's batched, lazily reduced variable-time inverse (round 6) against the per-divstep form that the
divergent callers keep, and y * y^-1 == 1 on a sample, over the BLS12-381 base and scalar fields."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.skipif(shutil.which("g++") is None, reason="needs g++")
def test_batched_inverse_matches_per_divstep(tmp_path):
    exe = str(tmp_path / "words_inv_check")
    subprocess.check_call(["g++", "-O2", "-std=c++17", "-I", os.path.join(ROOT, "hbbft_amd", "csrc"), "-o", exe,
                           os.path.join(ROOT, "tests", "csrc", "words_inv_check.cpp")])
    out = subprocess.run([exe], capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stdout + out.stderr
    assert "p: 0 bad, r: 0 bad" in out.stdout
