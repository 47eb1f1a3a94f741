"""CPU-side checks of the drop-in boundary: the C-ABI library builds, loads, and exports every
symbol include/rnnt_mi355x.h declares (no compute calls: there is no GPU here)."""
import os

import pytest

from rnnt_amd import _lib


def test_library_built_in_tree():
    assert os.path.exists(_lib.LIB_PATH), "run `make -C rnnt-inference_amd/csrc` (or __graft_entry__.build())"


def test_exports_every_header_symbol():
    names = _lib.header_functions()
    assert "rnnt_engine_create" in names and "rnnt_op_lstm_int8" in names
    lib = _lib.lib()
    missing = [n for n in names if not hasattr(lib, n)]
    assert not missing, missing
    assert set(_lib._SIGS) == set(names), "python binding out of sync with the header"


def test_abi_version_and_error_path():
    lib = _lib.lib()
    assert lib.rnnt_abi_version() == 8
    rc = lib.rnnt_engine_create(None, 0, None, None)
    assert rc == _lib.RNNT_EINVAL
    assert b"null" in lib.rnnt_last_error()


def test_no_cpu_fallback(monkeypatch, tmp_path):
    """The product path fails loudly when the HIP library is missing."""
    monkeypatch.setattr(_lib, "LIB_PATH", str(tmp_path / "missing.so"))
    monkeypatch.setattr(_lib, "_lib", None)
    with pytest.raises(RuntimeError, match="no CPU fallback"):
        _lib.lib()
