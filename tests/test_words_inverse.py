"""The variable-time inverse of hbbft_amd/csrc/words.hpp (Pornin's batched binary GCD, used by the
combine's affine conversion and the wave kernel's final exponentiation) compiled for the host and
checked on 40,000 random inputs mod p and mod r, the edge values 1, 2, m - 1, 2^k and 0 -> 0."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.skipif(shutil.which("g++") is None, reason="needs g++")
def test_words_inv_vartime(tmp_path):
    exe = tmp_path / "words_inv_test"
    subprocess.check_call(["g++", "-O2", "-std=c++17", "-I", os.path.join(ROOT, "hbbft_amd", "csrc"), "-o", str(exe),
                           os.path.join(ROOT, "tests", "native", "words_inv_test.cpp")])
    out = subprocess.run([str(exe)], capture_output=True, text=True, timeout=120)
    assert out.returncode == 0, out.stdout + out.stderr
    assert "bad: p 0, r 0" in out.stdout
