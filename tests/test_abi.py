"""CPU: the C-ABI library builds/loads and exports every symbol include/alert_engine.h declares
(no compute calls here: there is no GPU in the build container)."""
import ctypes
import re

import pytest

from conftest import ROOT


def declared_symbols():
    txt = (ROOT / "include" / "alert_engine.h").read_text()
    return sorted(set(re.findall(r"^\s*(?:int|const char \*)\s*(ae_\w+)\s*\(", txt, re.M)))


def test_header_declares_the_boundary():
    syms = declared_symbols()
    for s in ("ae_create", "ae_score", "ae_splice", "ae_mlm_topk", "ae_topk", "ae_cosine_rank",
              "ae_encode", "ae_last_error"):
        assert s in syms


def test_library_exports_every_declared_symbol():
    from apmc_amd import LIB_PATH
    from apmc_amd.engine import EXPORTS
    if not LIB_PATH.exists():
        pytest.fail(f"{LIB_PATH} not built (run make / __graft_entry__.build())")
    import torch  # noqa: F401  (bind to torch's HIP runtime, as the product does)
    lib = ctypes.CDLL(str(LIB_PATH))
    for s in declared_symbols():
        assert hasattr(lib, s), s
    assert set(declared_symbols()) == set(EXPORTS)
    lib.ae_version.restype = ctypes.c_char_p
    assert b"gfx950" in lib.ae_version()


def test_library_has_gfx950_code_object():
    from apmc_amd import LIB_PATH
    data = LIB_PATH.read_bytes()
    assert b"gfx950" in data


def test_libraries_built_from_this_tree():
    """Both libraries embed the hash of the sources they were built from (buildinfo.py); the
    loaders refuse a library left over from other sources, so the tests and the bench can only
    run binaries built from exactly this tree."""
    from apmc_amd import HOSTLIB_PATH, LIB_PATH
    from apmc_amd.buildinfo import source_hash
    import torch  # noqa: F401
    eng = ctypes.CDLL(str(LIB_PATH))
    eng.ae_source_hash.restype = ctypes.c_char_p
    assert eng.ae_source_hash().decode() == source_hash("engine")
    host = ctypes.CDLL(str(HOSTLIB_PATH))
    host.ah_source_hash.restype = ctypes.c_char_p
    assert host.ah_source_hash().decode() == source_hash("host")
