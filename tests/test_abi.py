"""CPU: the C-ABI library builds/loads and exports every symbol include/fgv.h declares."""
import ctypes
import os
import re

from fabric_amd import _lib

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_symbols():
    txt = open(os.path.join(ROOT, "include", "fgv.h")).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"\b(fgv_[a-z0-9_]+)\s*\(", txt)))


def test_every_declared_symbol_is_exported():
    L = _lib.load()
    syms = declared_symbols()
    assert len(syms) >= 7
    missing = [s for s in syms if not hasattr(L, s)]
    assert not missing, missing
    assert set(_lib.EXPORTED) <= set(syms)


def test_strerror_without_gpu():
    L = _lib.load()
    assert L.fgv_strerror(0) == b"ok"
    assert L.fgv_strerror(-2) == b"HIP device error"


def test_no_oracle_in_product():
    """The product library must not link the oracle or OpenSSL-based verification."""
    import subprocess
    out = subprocess.run(["ldd", _lib.LIB_PATH], capture_output=True, text=True).stdout
    assert "oracle" not in out
    nm = subprocess.run(["nm", "-D", _lib.LIB_PATH], capture_output=True, text=True).stdout
    assert "oracle_" not in nm and "ECDSA_do_verify" not in nm
