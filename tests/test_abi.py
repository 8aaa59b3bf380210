"""The C-ABI library loads and exports every symbol include/hbbft_hip.h declares (CPU-only: no
compute call is made without a GPU)."""
import ctypes
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "hbbft_hip.h")


def declared_symbols():
    text = open(HEADER).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(hbh_[a-z0-9_]+)\s*\(", text)))


def test_header_declares_entry_points():
    syms = declared_symbols()
    for must in ("hbh_engine_create", "hbh_verify_sig_shares", "hbh_verify_dec_shares", "hbh_verify_ciphertexts"):
        assert must in syms


def test_library_exports_every_declared_symbol():
    from hbbft_amd import _lib
    if not os.path.exists(_lib.LIB_PATH):
        pytest.skip("libhbbft_hip.so not built")
    so = ctypes.CDLL(_lib.LIB_PATH)
    missing = [s for s in declared_symbols() if not hasattr(so, s)]
    assert not missing, missing
    bound = {name for name, _, _ in _lib.SIGNATURES}
    assert set(declared_symbols()) == bound, set(declared_symbols()) ^ bound


def test_no_cpu_fallback_when_library_missing(monkeypatch, tmp_path):
    from hbbft_amd import _lib
    monkeypatch.setattr(_lib, "LIB_PATH", str(tmp_path / "absent.so"))
    monkeypatch.setattr(_lib, "_lib", None)
    with pytest.raises(_lib.HbhError):
        _lib.lib()
