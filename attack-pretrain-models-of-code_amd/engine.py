"""ctypes binding of the C-ABI in include/alert_engine.h (lib/libalert_engine.so).

There is no CPU or PyTorch fallback: if the HIP library is missing or fails to load, every entry
point raises.  Device buffers are torch tensors (torch is the allocator / stream provider); the
engine owns its weights and workspaces in HBM.
"""
from __future__ import annotations

import ctypes
import os

import numpy as np

from . import LIB_PATH, TOOLS_LIB_PATH
from .weights import CODEBERT, RobertaShape

AE_HEAD = {"sigmoid1": 0, "softmaxN": 1, "pair2": 2, "none": 3}
AE_PREC = {"fp32": 0, "bf16": 1, "f32x3": 2}
AE_KIND = {"gemm_ffn1": 0, "gemm_any": 1, "attention": 2}


class AeConfig(ctypes.Structure):
    _fields_ = [("layers", ctypes.c_int32), ("hidden", ctypes.c_int32), ("heads", ctypes.c_int32),
                ("ffn", ctypes.c_int32), ("vocab", ctypes.c_int32), ("max_pos", ctypes.c_int32),
                ("type_vocab", ctypes.c_int32), ("num_labels", ctypes.c_int32),
                ("head_kind", ctypes.c_int32), ("precision", ctypes.c_int32),
                ("pad_id", ctypes.c_int32), ("with_mlm", ctypes.c_int32),
                ("ln_eps", ctypes.c_float), ("streams", ctypes.c_int32)]


AE_STREAMS = {"two": 0, "one": 1}


class AeWeightView(ctypes.Structure):
    _fields_ = [("name", ctypes.c_char_p), ("data", ctypes.c_void_p), ("numel", ctypes.c_int64)]


# every symbol include/alert_engine.h declares (checked by tests/test_abi.py)
EXPORTS = ("ae_create", "ae_destroy", "ae_score", "ae_score_graph", "ae_graph_mask", "ae_encode",
           "ae_encode_ex", "ae_encode_rows", "ae_mlm_topk",
           "ae_mlm_nll", "ae_splice",
           "ae_topk", "ae_cosine_rank", "ae_set_profiling", "ae_kernel_time", "ae_last_error",
           "ae_version", "ae_source_hash")

_LIBS: dict[str, ctypes.CDLL] = {}


def load_library(path: str | os.PathLike | None = None, tools: bool = False) -> ctypes.CDLL:
    """Load (once) the engine library: the product library lib/libalert_engine.so, or with
    tools=True the tools library lib/libalert_engine_tools.so (the same sources built with
    -DAE_TOOLS: the product plus the timing / A-B entry points ae_bench_* and the engine's AE_*
    knobs).  torch must be imported first so that the library binds to the HIP runtime torch
    already loaded (one runtime per process: shared streams and pointers)."""
    key = str(path) if path else ("tools" if tools else "product")
    if key in _LIBS:
        return _LIBS[key]
    import torch  # noqa: F401  (HIP runtime first)

    p = str(path or (TOOLS_LIB_PATH if tools else LIB_PATH))
    if not os.path.exists(p):
        raise RuntimeError(f"HIP engine library not built: {p} is missing (run `make` or "
                           f"__graft_entry__.build()); there is no CPU fallback")
    lib = ctypes.CDLL(p)
    if path is None:
        from .buildinfo import source_hash

        lib.ae_source_hash.restype = ctypes.c_char_p
        built, here = lib.ae_source_hash().decode(), source_hash("engine")
        if built != here:
            raise RuntimeError(f"{p} was built from other sources (hash {built}, this tree "
                               f"{here}): rebuild it (`make` or __graft_entry__.build())")
    vp, i32, i64 = ctypes.c_void_p, ctypes.c_int32, ctypes.c_int64
    lib.ae_create.argtypes = [ctypes.POINTER(AeConfig), ctypes.POINTER(AeWeightView), i32, i32,
                              ctypes.POINTER(vp)]
    lib.ae_destroy.argtypes = [vp]
    lib.ae_score.argtypes = [vp, vp, vp, vp, vp, i32, i32, vp, vp]
    lib.ae_score_graph.argtypes = [vp, vp, vp, vp, vp, i32, i32, vp, vp]
    lib.ae_graph_mask.argtypes = [vp, vp, vp, vp, i32, i32, i32, vp, vp]
    lib.ae_encode.argtypes = [vp, vp, vp, i32, i32, vp, vp]
    lib.ae_encode_ex.argtypes = [vp, vp, vp, i32, i32, i32, i32, i32, vp, vp]
    if path is None or hasattr(lib, "ae_encode_rows"):  # an older library at an explicit path
        lib.ae_encode_rows.argtypes = [vp, vp, vp, i32, i32, i32, vp, i32, vp, vp]  # (same-box A/B)
    lib.ae_mlm_topk.argtypes = [vp, vp, i32, i32, vp, vp, vp]
    lib.ae_mlm_nll.argtypes = [vp, vp, i32, i32, vp, vp]
    lib.ae_splice.argtypes = [vp, vp, vp, vp, i32, i32, i32, i32, i32, vp, vp, vp]
    lib.ae_topk.argtypes = [vp, i32, i32, i32, vp, vp, vp]
    lib.ae_cosine_rank.argtypes = [vp, vp, i32, i32, i32, ctypes.c_float, vp, vp]
    lib.ae_set_profiling.argtypes = [vp, i32, i32]
    lib.ae_kernel_time.argtypes = [vp, ctypes.POINTER(ctypes.c_double), ctypes.POINTER(i64),
                                   ctypes.POINTER(ctypes.c_double)]
    lib.ae_last_error.restype = ctypes.c_char_p
    lib.ae_version.restype = ctypes.c_char_p
    for name in EXPORTS:
        if name not in ("ae_last_error", "ae_version", "ae_source_hash") and \
                (path is None or hasattr(lib, name)):
            getattr(lib, name).restype = ctypes.c_int
    _LIBS[key] = lib
    return lib


def _check(rc: int, what: str, lib: ctypes.CDLL | None = None):
    if rc != 0:
        lib = lib if lib is not None else _LIBS.get("product")
        msg = lib.ae_last_error().decode(errors="replace") if lib is not None else ""
        raise RuntimeError(f"{what} failed ({rc}): {msg}")


def _ptr(t) -> ctypes.c_void_p:
    return ctypes.c_void_p(t.data_ptr()) if t is not None else ctypes.c_void_p(None)


def _stream(stream=None):
    import torch

    s = stream if stream is not None else torch.cuda.current_stream()
    return ctypes.c_void_p(s.cuda_stream)


class Engine:
    """One RoBERTa victim (or MLM) resident on one GPU."""

    def __init__(self, state_dict: dict[str, np.ndarray], head: str = "sigmoid1",
                 num_labels: int = 1, precision: str = "fp32", device: int = 0,
                 with_mlm: bool = False, shape: RobertaShape = CODEBERT, streams: str = "two",
                 tools: bool = False):
        """streams: "two" (default: the split-precision encoder as two half-batch HIP streams)
        or "one" (every kernel on the caller's stream).  tools=True builds the engine from the
        tools library (lib/libalert_engine_tools.so, the same sources with -DAE_TOOLS), whose
        engine also reads the A/B knobs AE_ATTN_VARIANT, AE_SPLIT_STREAMS / _PARTS / _LAG,
        AE_CLS_ABSORB at creation (tools/engine_ab.py, alternative-form
        parity tests); the product library reads no environment."""
        import torch

        self.lib = load_library(tools=tools)
        if not torch.cuda.is_available():
            raise RuntimeError("apmc_amd.Engine needs a ROCm GPU (torch.cuda.is_available() is "
                               "False); there is no CPU fallback")
        self.device = device
        self.head = head
        self.num_labels = num_labels
        self.shape = shape
        self.pad_id = shape.pad_id
        cfg = AeConfig(shape.layers, shape.hidden, shape.heads, shape.ffn, shape.vocab,
                       shape.max_pos, shape.type_vocab, num_labels, AE_HEAD[head],
                       AE_PREC[precision], shape.pad_id, int(with_mlm), shape.ln_eps,
                       AE_STREAMS[streams])
        keep = []
        views = (AeWeightView * len(state_dict))()
        for i, (k, v) in enumerate(state_dict.items()):
            a = np.ascontiguousarray(v, dtype=np.float32)
            keep.append(a)
            views[i] = AeWeightView(k.encode(), a.ctypes.data, a.size)
        handle = ctypes.c_void_p()
        torch.cuda.set_device(device)
        _check(self.lib.ae_create(ctypes.byref(cfg), views, len(state_dict), device,
                                  ctypes.byref(handle)), "ae_create", self.lib)
        self.handle = handle
        self.out_cols = 1 if head == "sigmoid1" else num_labels

    def close(self):
        if getattr(self, "handle", None):
            self.lib.ae_destroy(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # ------------------------------------------------------------------------------------------
    def score(self, ids, lens: np.ndarray, pos=None, mask_bits=None, out=None, stream=None):
        """ids: device int32 [n, L]; lens: host int32 [n] (non-pad counts).  Returns device
        float32 [n_out, C] (asynchronous on `stream`)."""
        import torch

        n, L = ids.shape
        assert ids.dtype == torch.int32 and ids.is_cuda and ids.is_contiguous()
        lens = np.ascontiguousarray(lens, dtype=np.int32)
        assert lens.shape == (n,)
        n_out = n // 2 if self.head == "pair2" else n
        if out is None:
            out = torch.empty((n_out, self.out_cols), dtype=torch.float32, device=ids.device)
        _check(self.lib.ae_score(self.handle, _ptr(ids), ctypes.c_void_p(lens.ctypes.data),
                                 _ptr(pos), _ptr(mask_bits), n, L, _ptr(out), _stream(stream)),
               "ae_score", self.lib)
        return out

    def score_graph(self, ids, lens: np.ndarray, pos, mask_bits, out=None, stream=None):
        """GraphCodeBERT forward (data-flow node averaging + explicit positions + data-flow mask).
        ids/pos: device int32 [n, L]; mask_bits: device int32/uint32 [n, L, L/32]; lens: host
        int32 [n] leading columns that take part, pads included (normally L)."""
        import torch

        n, L = ids.shape
        assert ids.dtype == torch.int32 and ids.is_cuda and ids.is_contiguous()
        assert pos.shape == (n, L) and pos.dtype == torch.int32 and pos.is_contiguous()
        assert L % 32 == 0 and mask_bits.shape == (n, L, L // 32) and mask_bits.is_contiguous()
        assert mask_bits.element_size() == 4
        lens = np.ascontiguousarray(lens, dtype=np.int32)
        assert lens.shape == (n,)
        n_out = n // 2 if self.head == "pair2" else n
        if out is None:
            out = torch.empty((n_out, self.out_cols), dtype=torch.float32, device=ids.device)
        _check(self.lib.ae_score_graph(self.handle, _ptr(ids), ctypes.c_void_p(lens.ctypes.data),
                                       _ptr(pos), _ptr(mask_bits), n, L, _ptr(out),
                                       _stream(stream)), "ae_score_graph", self.lib)
        return out

    def graph_mask(self, ids, meta, spans, edges, out=None, stream=None):
        """Device-built bit mask [n, L, L/32] (ae_graph_mask) from the compact features of
        Tokenizer.gcb_features (all device int32: ids / spans [n, L], meta [n, 4], edges
        [n, e_cap])."""
        import torch

        n, L = ids.shape
        for t in (ids, meta, spans, edges):
            assert t.dtype == torch.int32 and t.is_cuda and t.is_contiguous()
        assert meta.shape == (n, 4) and spans.shape == (n, L) and edges.shape[0] == n
        if out is None:
            out = torch.empty((n, L, L // 32), dtype=torch.int32, device=ids.device)
        _check(self.lib.ae_graph_mask(_ptr(ids), _ptr(meta), _ptr(spans), _ptr(edges), n, L,
                                      edges.shape[1], _ptr(out), _stream(stream)),
               "ae_graph_mask", self.lib)
        return out

    def encode(self, ids, lens: np.ndarray, attend_pad: bool = False, row0: int = 0,
               nrows: int | None = None, stream=None):
        """Hidden states [n, nrows, hidden] of rows [row0, row0+nrows) (default all L rows).
        attend_pad: the model is called without attention_mask (every id of the first lens[i]
        is attended, pad included)."""
        import torch

        n, L = ids.shape
        assert ids.dtype == torch.int32 and ids.is_cuda and ids.is_contiguous()
        nrows = L - row0 if nrows is None else nrows
        lens = np.ascontiguousarray(lens, dtype=np.int32)
        out = torch.zeros((n, nrows, self.shape.hidden), dtype=torch.float32, device=ids.device)
        _check(self.lib.ae_encode_ex(self.handle, _ptr(ids), ctypes.c_void_p(lens.ctypes.data),
                                     n, L, 1 if attend_pad else 0, row0, nrows, _ptr(out),
                                     _stream(stream)), "ae_encode_ex", self.lib)
        return out

    def encode_rows(self, ids, lens: np.ndarray, row0: np.ndarray, nrows: int,
                    attend_pad: bool = False, stream=None):
        """Hidden states [n, nrows, hidden] of rows [row0[i], row0[i]+nrows) of sequence i
        (ae_encode_rows: the last layer runs for those rows only).  Rows past lens[i] stay 0."""
        import torch

        n, L = ids.shape
        assert ids.dtype == torch.int32 and ids.is_cuda and ids.is_contiguous()
        lens = np.ascontiguousarray(lens, dtype=np.int32)
        row0 = np.ascontiguousarray(row0, dtype=np.int32)
        assert lens.shape == (n,) and row0.shape == (n,)
        out = torch.zeros((n, nrows, self.shape.hidden), dtype=torch.float32, device=ids.device)
        _check(self.lib.ae_encode_rows(self.handle, _ptr(ids), ctypes.c_void_p(lens.ctypes.data),
                                       n, L, 1 if attend_pad else 0,
                                       ctypes.c_void_p(row0.ctypes.data), nrows, _ptr(out),
                                       _stream(stream)), "ae_encode_rows", self.lib)
        return out

    def mlm_nll(self, ids, stream=None):
        """Per-token MLM cross entropy of full rows ids [n, L] (no attention_mask)."""
        import torch

        n, L = ids.shape
        assert ids.dtype == torch.int32 and ids.is_cuda and ids.is_contiguous()
        out = torch.empty((n, L), dtype=torch.float32, device=ids.device)
        _check(self.lib.ae_mlm_nll(self.handle, _ptr(ids), n, L, _ptr(out), _stream(stream)),
               "ae_mlm_nll", self.lib)
        return out

    def mlm_topk(self, ids, k: int, stream=None):
        import torch

        (L,) = ids.shape
        scores = torch.empty((L, k), dtype=torch.float32, device=ids.device)
        idx = torch.empty((L, k), dtype=torch.int32, device=ids.device)
        _check(self.lib.ae_mlm_topk(self.handle, _ptr(ids), L, k, _ptr(scores), _ptr(idx),
                                    _stream(stream)), "ae_mlm_topk", self.lib)
        return scores, idx

    def set_profiling(self, kind: str, enabled: bool = True):
        _check(self.lib.ae_set_profiling(self.handle, AE_KIND[kind], int(enabled)),
               "ae_set_profiling", self.lib)

    def kernel_time(self):
        ms, cnt, fl = ctypes.c_double(), ctypes.c_int64(), ctypes.c_double()
        _check(self.lib.ae_kernel_time(self.handle, ctypes.byref(ms), ctypes.byref(cnt),
                                       ctypes.byref(fl)), "ae_kernel_time", self.lib)
        return ms.value, cnt.value, fl.value


# ---------------------------------------------------------------------------------------------
# engine-free device ops
def splice(word_tok, word_off, mut_words, mut_off, n_mut: int, L: int, cls_id=0, sep_id=2,
           pad_id=1, stream=None):
    import torch

    lib = load_library()
    dev = word_tok.device
    ids = torch.empty((n_mut, L), dtype=torch.int32, device=dev)
    lens = torch.empty((n_mut,), dtype=torch.int32, device=dev)
    _check(lib.ae_splice(_ptr(word_tok), _ptr(word_off), _ptr(mut_words), _ptr(mut_off), n_mut, L,
                         cls_id, sep_id, pad_id, _ptr(ids), _ptr(lens), _stream(stream)),
           "ae_splice")
    return ids, lens


def topk(x, k: int, stream=None):
    import torch

    rows, cols = x.shape
    vals = torch.empty((rows, k), dtype=torch.float32, device=x.device)
    idx = torch.empty((rows, k), dtype=torch.int32, device=x.device)
    _check(load_library().ae_topk(_ptr(x), rows, cols, k, _ptr(vals), _ptr(idx), _stream(stream)),
           "ae_topk")
    return vals, idx


def cosine_rank(ref, cand, eps: float = 1e-6, stream=None):
    import torch

    n, span, hidden = cand.shape
    sims = torch.empty((n,), dtype=torch.float32, device=cand.device)
    _check(load_library().ae_cosine_rank(_ptr(ref), _ptr(cand), n, span, hidden,
                                         ctypes.c_float(eps), _ptr(sims), _stream(stream)),
           "ae_cosine_rank")
    return sims
