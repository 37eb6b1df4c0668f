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


def _dynamic_symbols(path):
    import subprocess
    out = subprocess.run(["nm", "-D", "--defined-only", str(path)], capture_output=True, text=True,
                         check=True).stdout
    return {line.split()[-1] for line in out.splitlines() if line.strip()}


def test_product_library_has_no_experiment_entry_points():
    """The product library exports the engine and the launchers it runs, nothing else: the
    timing / A-B entry points (ae_bench_*: kernel variants and DIAG builds whose results are
    wrong on purpose) and the engine's AE_* knobs live only in the tools library built from the
    same sources with -DAE_TOOLS."""
    from apmc_amd import LIB_PATH, TOOLS_LIB_PATH
    prod = _dynamic_symbols(LIB_PATH)
    assert not [s for s in prod if s.startswith("ae_bench")], sorted(prod)
    assert b"AE_ATTN_VARIANT" not in LIB_PATH.read_bytes()
    assert b"AE_SPLIT_STREAMS" not in LIB_PATH.read_bytes()
    tools = _dynamic_symbols(TOOLS_LIB_PATH)
    for s in ("ae_bench_gemm_packed", "ae_bench_attention_pp", "ae_bench_attention_x3",
              "ae_bench_gemm_packed_res_stats", "ae_bench_gemm_packed_fold"):
        assert s in tools, s
    assert set(declared_symbols()) <= tools


def test_streams_config_validated():
    """ae_config.streams (AE_STREAMS_TWO / AE_STREAMS_ONE) is checked before any device call."""
    from apmc_amd.engine import AE_HEAD, AE_PREC, AeConfig
    lib = _lib()
    c = AeConfig(layers=12, hidden=768, heads=12, ffn=3072, vocab=50265, max_pos=514,
                 type_vocab=1, num_labels=1, head_kind=AE_HEAD["sigmoid1"],
                 precision=AE_PREC["f32x3"], pad_id=1, with_mlm=0, ln_eps=1e-5, streams=2)
    out = ctypes.c_void_p()
    assert lib.ae_create(ctypes.byref(c), None, 0, 0, ctypes.byref(out)) == -22
    assert "streams" in _err(lib)


def test_library_has_gfx950_code_object():
    from apmc_amd import LIB_PATH
    data = LIB_PATH.read_bytes()
    assert b"gfx950" in data


def test_libraries_built_from_this_tree():
    """Both libraries embed the hash of the sources they were built from (buildinfo.py); the
    loaders refuse a library left over from other sources, so the tests and the bench can only
    run binaries built from exactly this tree."""
    from apmc_amd import HOSTLIB_PATH, LIB_PATH, TOOLS_LIB_PATH
    from apmc_amd.buildinfo import source_hash
    import torch  # noqa: F401
    for path in (LIB_PATH, TOOLS_LIB_PATH):
        eng = ctypes.CDLL(str(path))
        eng.ae_source_hash.restype = ctypes.c_char_p
        assert eng.ae_source_hash().decode() == source_hash("engine"), path
    host = ctypes.CDLL(str(HOSTLIB_PATH))
    host.ah_source_hash.restype = ctypes.c_char_p
    assert host.ah_source_hash().decode() == source_hash("host")


def _lib():
    from apmc_amd.engine import load_library
    return load_library()


def _err(lib):
    lib.ae_last_error.restype = ctypes.c_char_p
    return lib.ae_last_error().decode()


def test_argument_errors_before_any_device_call():
    """Every entry point validates its arguments before the first HIP call and reports
    AE_EINVAL (-22) with a message in ae_last_error() — the error contract include/alert_engine.h
    states; these calls never reach the device, so they run here without a GPU."""
    from apmc_amd.engine import AE_HEAD, AE_PREC, AeConfig
    lib = _lib()
    EINVAL = -22
    buf = (ctypes.c_int32 * 64)()
    fbuf = (ctypes.c_float * 64)()
    p = ctypes.cast(buf, ctypes.c_void_p)
    fp = ctypes.cast(fbuf, ctypes.c_void_p)

    def cfg(**kw):
        c = dict(layers=12, hidden=768, heads=12, ffn=3072, vocab=50265, max_pos=514, type_vocab=1,
                 num_labels=1, head_kind=AE_HEAD["sigmoid1"], precision=AE_PREC["f32x3"], pad_id=1,
                 with_mlm=0, ln_eps=1e-5)
        c.update(kw)
        return AeConfig(**c)

    out = ctypes.c_void_p()
    for bad, msg in ((dict(hidden=1024), "hidden=768"), (dict(heads=16), "hidden=768"),
                     (dict(ffn=3000), "ffn"), (dict(layers=0), "ffn/layers"),
                     (dict(num_labels=0), "num_labels"), (dict(num_labels=2), "sigmoid head"),
                     (dict(head_kind=AE_HEAD["pair2"]), "pair head"),
                     (dict(precision=7), "precision")):
        c = cfg(**bad)
        assert lib.ae_create(ctypes.byref(c), None, 0, 0, ctypes.byref(out)) == EINVAL, bad
        assert msg in _err(lib), (bad, _err(lib))
    c = cfg()
    assert lib.ae_create(None, None, 0, 0, ctypes.byref(out)) == EINVAL
    assert lib.ae_create(ctypes.byref(c), None, 3, 0, ctypes.byref(out)) == EINVAL
    assert "null argument" in _err(lib)
    # scoring / encoding on a null engine, null inputs, bad shapes
    assert lib.ae_score(None, p, p, None, None, 4, 512, fp, None) == EINVAL
    assert "null engine" in _err(lib)
    assert lib.ae_score_graph(None, p, p, None, None, 4, 640, fp, None) == EINVAL
    assert "pos and mask_bits" in _err(lib)
    assert lib.ae_encode_ex(None, p, p, 4, 512, 0, 0, 1, fp, None) == EINVAL
    assert lib.ae_encode_rows(None, p, p, 4, 512, 0, p, 1, fp, None) == EINVAL
    assert "null engine" in _err(lib)
    assert lib.ae_set_profiling(None, 0, 1) == EINVAL
    # standalone kernels: shapes checked before launch
    assert lib.ae_topk(fp, 1, 10, 0, fp, p, None) == EINVAL and "bad shape" in _err(lib)
    assert lib.ae_topk(fp, 1, 10, 11, fp, p, None) == EINVAL
    assert lib.ae_topk(fp, 1, 1000, 257, fp, p, None) == EINVAL
    assert lib.ae_topk(None, 1, 10, 5, fp, p, None) == EINVAL and "null" in _err(lib)
    assert lib.ae_splice(p, p, p, p, 4, 1, 0, 2, 1, p, p, None) == EINVAL
    assert lib.ae_splice(p, None, p, p, 4, 512, 0, 2, 1, p, p, None) == EINVAL
    assert lib.ae_graph_mask(p, p, p, p, 2, 100, 4, p, None) == EINVAL  # L % 32
    assert lib.ae_graph_mask(p, p, p, p, 2, 2048, 4, p, None) == EINVAL  # L > 1024
    assert lib.ae_graph_mask(p, p, p, p, 2, 640, 0, p, None) == EINVAL  # e_cap < 1
    assert lib.ae_cosine_rank(fp, fp, 4, 0, 768, ctypes.c_float(1e-8), fp, None) == EINVAL


def test_engine_refuses_to_run_without_a_gpu():
    """The product path fails loudly when there is no device: no CPU fallback."""
    import torch
    if torch.cuda.is_available():
        pytest.skip("a GPU is present")
    from apmc_amd.engine import Engine
    with pytest.raises(RuntimeError, match="no CPU fallback"):
        Engine({}, head="sigmoid1", num_labels=1, precision="f32x3")
