"""GPU unit tests of individual kernels called through their extern "C" launchers in
lib/libalert_engine.so (not part of the public C-ABI; the engine tests cover them end to end).

Packed-plane GEMM (gemm_planes.hip): C = A·W^T over packed bf16 planes must equal the float64 sum
of the split products A_hi·W_hi + A_hi·W_lo + A_lo·W_hi (f32 accumulation: |Δ| ≤ 1e-5·Σ|a||w|), for
ragged M, both tile widths, the ping-pong 256 x 256 and 256 x 192 kernels, both plane counts and every
epilogue."""
import ctypes

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _lib():
    from apmc_amd.engine import load_library
    lib = load_library(tools=True)  # the ae_bench_* entry points live in the tools library
    vp, i32 = ctypes.c_void_p, ctypes.c_int32
    lib.ae_launch_gemm_packed.argtypes = [vp] * 6 + [i32] * 5 + [vp]
    lib.ae_launch_gemm_packed.restype = ctypes.c_int
    lib.ae_bench_gemm_packed.argtypes = [vp] * 6 + [i32] * 7 + [vp]
    lib.ae_bench_gemm_packed.restype = ctypes.c_int
    return lib


def _split(x):
    """f32 tensor -> (hi, lo) bf16 planes."""
    hi = x.to(torch.bfloat16)
    lo = (x - hi.float()).to(torch.bfloat16)
    return hi, lo


def _pack(hi, lo, np_):
    """[R, K] planes -> packed [R, np*K] (np = 2: K/32 blocks of [hi 32 | lo 32])."""
    if np_ == 1:
        return hi.contiguous()
    R, K = hi.shape
    return torch.stack([hi.reshape(R, K // 32, 32), lo.reshape(R, K // 32, 32)], 2).reshape(R, 2 * K)


def _unpack(p, np_, N):
    R = p.shape[0]
    if np_ == 1:
        return p.double()
    b = p.reshape(R, N // 32, 2, 32).double()
    return (b[:, :, 0] + b[:, :, 1]).reshape(R, N)


def _p(t):
    return ctypes.c_void_p(t.data_ptr()) if t is not None else ctypes.c_void_p(None)


@pytest.mark.parametrize("M,N,K,np_,epi,bn", [
    (64, 2304, 768, 2, 0, ""),
    # ping-pong 256 x 256 kernel (tile code 512): ragged M / N, one- and two-K-tile loops
    (300, 256, 128, 2, 0, "512"),
    (512, 768, 768, 2, 2, "512"),
    (257, 512, 192, 2, 1, "512"),
    (1000, 384, 64, 1, 3, "512"),
    (700, 256, 256, 1, 1, "512"),
    (64, 2304, 768, 2, 3, "512"),
    (600, 3072, 768, 2, 1, "512"),
    # the same kernel on a persistent grid (one workgroup per CU looping over > 256 tiles)
    (8192, 2304, 256, 2, 0, "512p"),
    (8200, 3072, 128, 2, 1, "512p"),
    (2000, 768, 192, 1, 2, "512p"),
    # ping-pong 256 x 192 kernel (f32 epilogues): ragged M / N, short and long K
    (300, 768, 128, 2, 0, "192"),
    (512, 768, 768, 2, 2, "192"),
    (1000, 384, 64, 1, 3, "192"),
    (64, 768, 3072, 2, 2, "192"),
    (257, 192, 192, 1, 0, "192"),
    (700, 576, 256, 2, 2, "192"),
    # its packed-plane epilogue (N % 192 == 0, ragged M; a tools-library variant of the QKV GEMM)
    (300, 2304, 768, 2, 4, "192"),
    (1000, 576, 256, 1, 4, "192"),
    (4100, 2304, 128, 2, 4, "192"),
])
def test_gemm_packed_matches_split_products(gpu, M, N, K, np_, epi, bn):
    lib = _lib()
    g = torch.Generator().manual_seed(M + N + K)
    A = torch.randn(M, K, generator=g) * 0.7
    W = torch.randn(N, K, generator=g) * 0.05
    bias = torch.randn(N, generator=g)
    R = torch.randn(M, N, generator=g)
    Ah, Al = _split(A)
    Wh, Wl = _split(W)
    ref = Ah.double() @ Wh.double().T
    if np_ == 2:
        ref = ref + Ah.double() @ Wl.double().T + Al.double() @ Wh.double().T
    ref = ref + bias.double()
    scale = A.abs().double() @ W.abs().double().T
    if epi == 1:
        ref = torch.nn.functional.gelu(ref)
    elif epi == 2:
        ref = ref + R.double()
    elif epi == 3:
        ref = torch.tanh(ref)
    dA = _pack(Ah, Al, np_).cuda()
    dW = _pack(Wh, Wl, np_).cuda()
    db, dR = bias.cuda(), R.cuda()
    C = torch.full((M, N), float("nan"), device="cuda")
    Cp = torch.zeros((M, np_ * N), dtype=torch.bfloat16, device="cuda")
    st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    if bn:  # explicit tile width through the experiment entry point (production kernel, diag 0;
        # "512p": diag 9, the persistent grid)
        rc = lib.ae_bench_gemm_packed(_p(dA), _p(dW), _p(db), _p(dR), _p(C), _p(Cp), M, N, K, epi,
                                      np_, int(bn.rstrip("p")), 9 if bn.endswith("p") else 0, st)
    else:
        rc = lib.ae_launch_gemm_packed(_p(dA), _p(dW), _p(db), _p(dR), _p(C), _p(Cp), M, N, K,
                                       epi, np_, st)
    assert rc == 0
    torch.cuda.synchronize()
    if epi in (1, 4):
        got = _unpack(Cp.cpu(), np_, N)
        # the packed planes hold the GELU / biased output to ~2^-17 relative (np 2) / 2^-9 (np 1)
        rel = 2e-5 if np_ == 2 else 5e-3
        tol = 1e-5 * scale + rel * ref.abs() + 1e-6
    else:
        got = C.double().cpu()
        tol = 1e-5 * scale + 1e-6
    assert torch.isfinite(got).all()
    err = (got - ref).abs()
    assert (err <= tol).all(), float((err - tol).max())


def test_gemm_packed_gelu_propagates_nan(gpu):
    """The FFN1 GELU epilogue (gelu_exp2_pairs) passes a NaN pre-activation through as NaN and
    an infinite one as non-finite — never as a finite value (an upstream overflow must not turn
    into finite scores; its max(x, 0) is the IEEE maximum, not maxnum).  Every other element
    keeps the float64 tolerance of test_gemm_packed_matches_split_products."""
    lib = _lib()
    M, N, K, np_ = 300, 512, 128, 2
    g = torch.Generator().manual_seed(11)
    A = torch.randn(M, K, generator=g) * 0.7
    W = torch.randn(N, K, generator=g) * 0.05
    bias = torch.randn(N, generator=g)
    A[5, 17] = float("nan")  # row 5: every pre-activation NaN
    bias[7] = float("inf")  # column 7: +inf pre-activations
    Ah, Al = _split(A)
    Wh, Wl = _split(W)
    ref = Ah.double() @ Wh.double().T + Ah.double() @ Wl.double().T + Al.double() @ Wh.double().T
    ref = torch.nn.functional.gelu(ref + bias.double())
    scale = A.abs().double().nan_to_num(0) @ W.abs().double().T
    C = torch.full((M, N), float("nan"), device="cuda")
    Cp = torch.zeros((M, np_ * N), dtype=torch.bfloat16, device="cuda")
    st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    assert lib.ae_bench_gemm_packed(_p(_pack(Ah, Al, np_).cuda()), _p(_pack(Wh, Wl, np_).cuda()),
                                    _p(bias.cuda()), _p(None), _p(C), _p(Cp), M, N, K, 1, np_,
                                    512, 0, st) == 0
    torch.cuda.synchronize()
    planes = Cp.cpu().reshape(M, N // 32, 2, 32).double()
    hi = planes[:, :, 0].reshape(M, N)
    got = _unpack(Cp.cpu(), np_, N)
    assert torch.isnan(hi[5]).all() and torch.isnan(got[5]).all()
    assert not torch.isfinite(hi[:, 7]).any() and not torch.isfinite(got[:, 7]).any()
    keep = torch.ones(M, N, dtype=torch.bool)
    keep[5], keep[:, 7] = False, False
    err = (got - ref).abs()[keep]
    tol = (1e-5 * scale + 2e-5 * ref.abs() + 1e-6)[keep]
    assert (err <= tol).all(), float((err - tol).max())


def _attn_ref(qkv, cu, n, mask=None, L=0, q_rows=None):
    """float64 attention per (sequence, head): softmax(Q·K^T/8 (+ finfo.min where the bit-packed
    mask excludes a key)) · V over each sequence's keys; [T, 768]."""
    H, heads, D = 768, 12, 64
    outs = []
    for s in range(n):
        a, b = int(cu[s]), int(cu[s + 1])
        x = qkv[a:b].double()
        q = x[:, :H].view(-1, heads, D).transpose(0, 1)
        k = x[:, H:2 * H].view(-1, heads, D).transpose(0, 1)
        v = x[:, 2 * H:].view(-1, heads, D).transpose(0, 1)
        sc = q @ k.transpose(1, 2) / 8.0
        if mask is not None:
            words = mask[s].view(L, L // 32)[: b - a]
            bits = ((words.unsqueeze(-1) >> torch.arange(32)) & 1).reshape(b - a, L)[:, : b - a]
            sc = sc + (bits == 0).double() * torch.finfo(torch.float32).min
        o = (torch.softmax(sc, dim=-1) @ v).transpose(0, 1).reshape(b - a, H)
        outs.append(o)
    return torch.cat(outs)


@pytest.mark.parametrize("variant", [0, 1, 2, 3])
@pytest.mark.parametrize("case", ["ragged", "mask", "cls", "planes"])
def test_attention_x3_variants_match_f64(gpu, variant, case):
    """attn_x3_kernel (every variant bit: transposed-read V, exp2 + rescale skip) against a float64
    reference: ragged lengths (1..300, one tile boundary each side), the GraphCodeBERT bit mask
    (incl. a fully-masked query row -> uniform over the keys, HF's finfo.min semantics), the
    CLS-only query launch of the last layer and the packed-plane context output."""
    lib = _lib()
    vp, i32 = ctypes.c_void_p, ctypes.c_int32
    lib.ae_bench_attention_x3.argtypes = [vp] * 5 + [i32] * 3 + [vp, i32, i32, i32, vp]
    lib.ae_bench_attention_x3.restype = ctypes.c_int
    g = torch.Generator().manual_seed(7 + variant)
    lens = [1, 31, 32, 33, 129, 300, 64] if case != "mask" else [40, 97, 128]
    n = len(lens)
    cu = torch.zeros(n + 1, dtype=torch.int32)
    cu[1:] = torch.cumsum(torch.tensor(lens), 0)
    T = int(cu[-1])
    qkv = torch.randn(T, 3 * 768, generator=g)
    L, mask, dmask = 0, None, None
    if case == "mask":
        L = 128
        dense = (torch.rand(n, L, L, generator=g) < 0.6)
        dense[:, :, 0] = True
        dense[1, 5, :] = False  # a query row that excludes every key
        words = (dense.view(n, L, L // 32, 32).long() << torch.arange(32)).sum(-1)
        mask = words
        dmask = (words - (words >= 2 ** 31).long() * 2 ** 32).to(torch.int32).cuda()
    ref = _attn_ref(qkv, cu, n, mask, L)
    dq, dcu = qkv.cuda(), cu.cuda()
    out = torch.full((T, 768), float("nan"), device="cuda")
    op = torch.zeros((T, 2 * 768), dtype=torch.bfloat16, device="cuda") if case == "planes" else None
    one = torch.ones(1, dtype=torch.int32, device="cuda") if case == "cls" else None
    st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    rc = lib.ae_bench_attention_x3(_p(dq), _p(out), _p(op), _p(dcu), _p(one),
                                   1 if case == "cls" else max(lens), n, 12, _p(dmask), L, 3,
                                   variant, st)
    assert rc == 0
    torch.cuda.synchronize()
    # split-bf16 products carry ~2^-16 relative error: ~1e-4 on these scores; layout errors are O(1)
    if case == "planes":
        got = _unpack(op.cpu(), 2, 768)
        tol = 2e-4 + 2e-5 * ref.abs()
    else:
        got = out.double().cpu()
        tol = 2e-4
    if case == "cls":
        rows = cu[:-1].long()
        got, ref = got[rows], ref[rows]
    assert torch.isfinite(got).all()
    err = (got - ref).abs()
    assert (err <= tol).all(), float(err.max())


def _qkv_planes(qkv, np_):
    """f32 qkv [T, 2304] -> the QKV GEMM's packed-plane output with Q pre-scaled by log2(e)/8
    (what the engine feeds attention_pp: gemm_planes PK_EPI_BIAS_PACKED over scaled Wq, bq)."""
    x = qkv.clone()
    x[:, :768] *= 0.18033688011112042
    hi, lo = _split(x)
    return _pack(hi, lo, np_)


@pytest.mark.parametrize("variant", [6, 66, 67, 72, 74, 80, 81, 86])
@pytest.mark.parametrize("np_", [2, 1])
@pytest.mark.parametrize("case", ["ragged", "mask", "cls", "planes", "grow"])
def test_attention_pp_matches_f64(gpu, np_, case, variant):
    """attn_pp_kernel (packed-plane Q/K/V moved by LDS-DMA, swizzled K/V images, transposed V
    reads) against the float64 reference, for both plane counts (np 1 = bf16 mode: stated
    tolerance 2e-2), every loop (6: 3-slot rings + deferred rescale, its mask launches on the
    software-pipelined PIPE 4; 66: 6 with saddr DMA and a permlane row max; 67 (production): 66
    with a tree row max) and
    the ragged / mask / CLS-only / packed-output launches.  "grow": spike keys whose scores
    rise along the sequence, so every row max jumps past the deferred-rescale threshold (2^8)
    several times — the rare branch of variant 6."""
    lib = _lib()
    vp, i32 = ctypes.c_void_p, ctypes.c_int32
    lib.ae_bench_attention_pp.argtypes = [vp] * 5 + [i32] * 3 + [vp, i32, i32, i32, vp]
    lib.ae_bench_attention_pp.restype = ctypes.c_int
    g = torch.Generator().manual_seed(11 + np_)
    lens = {"mask": [40, 97, 128], "grow": [300, 517, 64]}.get(case, [1, 31, 32, 33, 129, 300, 64])
    n = len(lens)
    cu = torch.zeros(n + 1, dtype=torch.int32)
    cu[1:] = torch.cumsum(torch.tensor(lens), 0)
    T = int(cu[-1])
    qkv = torch.randn(T, 3 * 768, generator=g)
    if case == "grow":
        # every query ~ the all-ones direction; keys at 40, 100, 200, 400 of a sequence are c x ones,
        # so a row's max jumps 0.5 -> 6 -> 13 -> 20 -> 27 (natural units; > 8 in log2 each time)
        qkv *= 0.25
        qkv[:, :768] += 1.0
        start = 0
        for x in lens:
            for p_, c in ((40, 0.75), (100, 1.625), (200, 2.5), (400, 3.375)):
                if p_ < x:
                    qkv[start + p_, 768:1536] = c
            start += x
    L, mask, dmask = 0, None, None
    if case == "mask":
        L = 128
        dense = (torch.rand(n, L, L, generator=g) < 0.6)
        dense[:, :, 0] = True
        dense[1, 5, :] = False  # a query row that excludes every key
        words = (dense.view(n, L, L // 32, 32).long() << torch.arange(32)).sum(-1)
        mask = words
        dmask = (words - (words >= 2 ** 31).long() * 2 ** 32).to(torch.int32).cuda()
    ref = _attn_ref(qkv, cu, n, mask, L)
    dq, dcu = _qkv_planes(qkv, np_).cuda(), cu.cuda()
    out = torch.full((T, 768), float("nan"), device="cuda")
    op = torch.zeros((T, np_ * 768), dtype=torch.bfloat16, device="cuda") if case == "planes" else None
    one = torch.ones(1, dtype=torch.int32, device="cuda") if case == "cls" else None
    st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    rc = lib.ae_bench_attention_pp(_p(dq), _p(out), _p(op), _p(dcu), _p(one),
                                   1 if case == "cls" else max(lens), n, 12, _p(dmask), L, np_,
                                   variant, st)
    assert rc == 0
    torch.cuda.synchronize()
    if case == "planes":
        got = _unpack(op.cpu(), np_, 768)
    else:
        got = out.double().cpu()
    if case == "cls":
        rows = cu[:-1].long()
        got, ref = got[rows], ref[rows]
    tol = (2e-4 + 2e-5 * ref.abs()) if np_ == 2 else (2e-2 + 2e-2 * ref.abs())
    assert torch.isfinite(got).all()
    err = (got - ref).abs()
    assert (err <= tol).all(), float(err.max())


@pytest.mark.parametrize("case", ["ragged", "grow"])
def test_attention_pp_restructured_loops_bit_identical(gpu, case):
    """Variants 66 (saddr DMA with clamped offsets in the last tile, permlane row max, three
    workgroups per CU) and 67 (production: 66 with a tree row max) restructure PIPE 6 without
    changing its arithmetic: their packed-plane context must equal PIPE 6's bit for bit."""
    lib = _lib()
    vp, i32 = ctypes.c_void_p, ctypes.c_int32
    lib.ae_bench_attention_pp.argtypes = [vp] * 5 + [i32] * 3 + [vp, i32, i32, i32, vp]
    lib.ae_bench_attention_pp.restype = ctypes.c_int
    g = torch.Generator().manual_seed(5)
    lens = [1, 31, 32, 33, 129, 300, 512, 64] if case == "ragged" else [300, 517, 64]
    n = len(lens)
    cu = torch.zeros(n + 1, dtype=torch.int32)
    cu[1:] = torch.cumsum(torch.tensor(lens), 0)
    T = int(cu[-1])
    qkv = torch.randn(T, 3 * 768, generator=g)
    if case == "grow":  # row maxes jump past the deferred-rescale threshold several times
        qkv *= 0.25
        qkv[:, :768] += 1.0
        start = 0
        for x in lens:
            for p_, c in ((40, 0.75), (100, 1.625), (200, 2.5), (400, 3.375)):
                if p_ < x:
                    qkv[start + p_, 768:1536] = c
            start += x
    dq, dcu = _qkv_planes(qkv, 2).cuda(), cu.cuda()
    st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    outs = {}
    for v in (6, 66, 67, 72, 80, 81, 86):
        op = torch.zeros((T, 2 * 768), dtype=torch.int16, device="cuda")
        assert lib.ae_bench_attention_pp(_p(dq), None, _p(op), _p(dcu), None, max(lens), n, 12,
                                         None, 0, 2, v, st) == 0
        outs[v] = op
    torch.cuda.synchronize()
    assert torch.equal(outs[66], outs[6])
    assert torch.equal(outs[67], outs[6])
    assert torch.equal(outs[72], outs[6])  # exp / split and the next S MFMAs hand-interleaved
    assert torch.equal(outs[80], outs[6])  # two 32-query blocks per wave, 256-query workgroups
    assert torch.equal(outs[81], outs[6])  # the same with 3-slot K / V rings
    assert torch.equal(outs[86], outs[6])  # 81 with the K fragments read once for both blocks


def test_attention_pp_masked_fast_path_bit_identical(gpu):
    """Variant 74: a masked launch's full tile whose mask words are all ones for every query of
    the wave takes the unmasked tree max (no per-key select) — GraphCodeBERT's code rows over code
    keys.  The scores are the same, so the context must equal variant 66's (the production masked
    loop) bit for bit, on a GraphCodeBERT-shaped mask (dense code block, sparse node rows, a node
    row with no key at all) and ragged lengths."""
    lib = _lib()
    vp, i32 = ctypes.c_void_p, ctypes.c_int32
    lib.ae_bench_attention_pp.argtypes = [vp] * 5 + [i32] * 3 + [vp, i32, i32, i32, vp]
    lib.ae_bench_attention_pp.restype = ctypes.c_int
    g = torch.Generator().manual_seed(21)
    L = 320
    lens = [320, 250, 97, 33]
    n = len(lens)
    cu = torch.zeros(n + 1, dtype=torch.int32)
    cu[1:] = torch.cumsum(torch.tensor(lens), 0)
    T = int(cu[-1])
    dense = torch.zeros(n, L, L, dtype=torch.bool)
    for i, ln in enumerate(lens):
        ncode = max(1, ln - ln // 5)
        dense[i, :ncode, :ncode] = True
        for q in range(ncode, ln - 1):  # node rows: a few code keys and one node key
            a = int(torch.randint(0, ncode, (1,), generator=g))
            dense[i, q, a:a + 3] = True
            dense[i, q, ncode + int(torch.randint(0, ln - ncode, (1,), generator=g))] = True
    words = (dense.view(n, L, L // 32, 32).long() << torch.arange(32)).sum(-1)
    dmask = (words - (words >= 2 ** 31).long() * 2 ** 32).to(torch.int32).cuda()
    qkv = torch.randn(T, 3 * 768, generator=g)
    dq, dcu = _qkv_planes(qkv, 2).cuda(), cu.cuda()
    st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    outs = {}
    for v in (66, 74):
        op = torch.zeros((T, 2 * 768), dtype=torch.int16, device="cuda")
        assert lib.ae_bench_attention_pp(_p(dq), None, _p(op), _p(dcu), None, max(lens), n, 12,
                                         _p(dmask), L, 2, v, st) == 0
        outs[v] = op
    torch.cuda.synchronize()
    assert torch.equal(outs[74], outs[66])


def _fold_lib():
    lib = _lib()
    vp, i32, f32 = ctypes.c_void_p, ctypes.c_int32, ctypes.c_float
    lib.ae_launch_gemm_packed_fold.argtypes = [vp] * 5 + [f32, vp] + [i32] * 5 + [vp, vp]
    lib.ae_launch_gemm_packed_fold.restype = ctypes.c_int
    lib.ae_launch_gemm_packed_res_stats.argtypes = [vp] * 7 + [f32] + [vp] * 3 + [i32] * 4 + \
        [vp, vp]
    lib.ae_launch_gemm_packed_res_stats.restype = ctypes.c_int
    lib.ae_bench_gemm_packed_fold.argtypes = [vp] * 5 + [f32, vp] + [i32] * 5 + [vp, i32, i32, vp]
    lib.ae_bench_gemm_packed_fold.restype = ctypes.c_int
    return lib


def _split_prod(A, W, np_):
    """float64 of the split products a_hi·w_hi (+ a_hi·w_lo + a_lo·w_hi)."""
    Ah, Al = _split(A)
    Wh, Wl = _split(W)
    y = Ah.double() @ Wh.double().T
    if np_ == 2:
        y = y + Ah.double() @ Wl.double().T + Al.double() @ Wh.double().T
    return y


def _tile_stats(v):
    """[M, 768] -> the [M][4] RowStat words of the kernels: (mean, M2) of each 192-column tile."""
    t = v.double().reshape(v.shape[0], 4, 192)
    mean = t.mean(2)
    m2 = ((t - mean[:, :, None]) ** 2).sum(2)
    rs = torch.stack([mean.float(), m2.float()], 2).contiguous()  # [M, 4, 2] f32
    return rs.view(torch.int64).reshape(-1)


def _ln64(v, gamma, beta, eps=1e-5):
    v = v.double()
    mu = v.mean(1, keepdim=True)
    var = ((v - mu) ** 2).mean(1, keepdim=True)
    return (v - mu) / torch.sqrt(var + eps) * gamma.double() + beta.double(), var


@pytest.mark.parametrize("variant", [0, 1, 2])
@pytest.mark.parametrize("M,K,np_,shift", [(300, 768, 2, 0), (4097, 768, 2, 1), (37, 3072, 2, 1),
                                            (1000, 768, 1, 0), (1000, 768, 1, 1), (200, 64, 1, 1),
                                            (300, 64, 2, 0)])
def test_gemm_packed_res_stats_matches_f64(gpu, M, K, np_, shift, variant):
    """ae_launch_gemm_packed_res_stats (256 x 192 kernel): v = A·W^T + bias + r as f32 and packed
    planes plus the (mean, M2) of every row over its 4 192-column tiles, first with a plain
    residual (PK_EPI_RES_STATS: layer 0), then with the residual the previous pre-LayerNorm rows
    normalised on the fly from the statistics the first launch wrote (PK_EPI_RES_STATS_LN).
    Both in place (R = C), as the engine runs them; against float64 of the split products.  With
    shift, the planes hold v - kappa (the plane shift; kappa = bias + beta, as the engine passes)
    while f32 v and its statistics stay those of v.  variants 1 / 2: the two-per-CU 128 x 192 kernel
    (gemm_p2_kernel, tools library; 2 = its fragment reads pipelined against the MFMAs); K = 64
    its one- (np 1) and two-K-tile (np 2) paths."""
    lib = _fold_lib()
    lib.ae_bench_gemm_packed_res_stats.argtypes = [ctypes.c_void_p] * 7 + [ctypes.c_float] + \
        [ctypes.c_void_p] * 3 + [ctypes.c_int32] * 4 + [ctypes.c_void_p, ctypes.c_int32,
                                                         ctypes.c_int32, ctypes.c_void_p]
    lib.ae_bench_gemm_packed_res_stats.restype = ctypes.c_int
    N = 768
    g = torch.Generator().manual_seed(7 * M + K)
    st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    gamma = 1.0 + 0.1 * torch.randn(N, generator=g)
    beta = 0.1 * torch.randn(N, generator=g)
    dg, dbeta = gamma.cuda(), beta.cuda()
    s1 = torch.zeros(M * 4, dtype=torch.int64, device="cuda")
    s2 = torch.zeros(M * 4, dtype=torch.int64, device="cuda")
    R0 = torch.randn(M, N, generator=g) * 2.0 + 0.5
    v = R0.cuda()
    prev = None
    for it, (rst, out_st) in enumerate(((None, s1), (s1, s2))):
        A = torch.randn(M, K, generator=g) * 0.7
        W = torch.randn(N, K, generator=g) * 0.05
        bias = torch.randn(N, generator=g) * 0.5
        dA, dW, db = _pack(*_split(A), np_).cuda(), _pack(*_split(W), np_).cuda(), bias.cuda()
        vp = torch.zeros((M, np_ * N), dtype=torch.bfloat16, device="cuda")
        if rst is None:
            r = R0.double()
        else:
            r, _ = _ln64(prev, gamma, beta)
        kap = (bias + (beta if rst is not None else 0.5)) if shift else None
        rc = lib.ae_bench_gemm_packed_res_stats(
            _p(dA), _p(dW), _p(db), _p(v), _p(rst), _p(dg if rst is not None else None),
            _p(dbeta if rst is not None else None), 1e-5, _p(v), _p(vp), _p(out_st), M, N, K,
            np_, _p(kap.cuda() if shift else None), variant, 0, st)
        assert rc == 0
        torch.cuda.synchronize()
        ref = _split_prod(A, W, np_) + bias.double() + r
        scale = (A.abs().double() @ W.abs().double().T).amax(1, keepdim=True)
        got = v.double().cpu()
        # the on-the-fly LayerNorm reads f32 tile statistics: ~1e-6 relative on the residual
        tol = 1e-5 * scale + 1e-6 + (2e-6 * (r.abs() + 1.0) if rst is not None else 0.0)
        assert torch.isfinite(got).all()
        assert ((got - ref).abs() <= tol).all(), (it, float(((got - ref).abs() - tol).max()))
        planes = _unpack(vp.cpu(), np_, N)
        rel = 2e-5 if np_ == 2 else 5e-3
        want = got - kap.double() if shift else got
        assert ((planes - want).abs() <= rel * want.abs() + 1e-7).all(), it
        # the tile statistics of the f32 output, against float64 of the same values
        ws = out_st.cpu().view(torch.float32).reshape(M, 4, 2).double()
        t = got.reshape(M, 4, 192)
        mean = t.mean(2)
        m2 = ((t - mean[:, :, None]) ** 2).sum(2)
        assert ((ws[:, :, 0] - mean).abs() <= 1e-6 * (t.abs().amax(2) + 1)).all(), it
        assert ((ws[:, :, 1] - m2).abs() <= 1e-5 * m2 + 1e-6).all(), it
        prev = got


@pytest.mark.parametrize("variant", [0, 1])
@pytest.mark.parametrize("M,N,np_,gelu,shift", [
    (300, 2304, 2, 0, 0), (4100, 3072, 2, 1, 0), (37, 3072, 2, 1, 0), (1000, 2304, 1, 0, 0),
    (600, 3072, 1, 1, 0), (300, 2304, 2, 0, 1), (4100, 3072, 2, 1, 1), (600, 3072, 1, 1, 1)])
def test_gemm_packed_fold_matches_f64(gpu, M, N, np_, gelu, shift, variant):
    """ae_launch_gemm_packed_fold (256 x 256 kernel, PK_EPI_BIAS_FOLD / PK_EPI_GELU_FOLD): the
    QKV / FFN1 GEMM over PRE-LayerNorm rows v with the LayerNorm folded in,
        y = rstd · (v·W'^T - mean · s) + bias',  W' = W·diag(gamma), s = rowsums(W'),
        bias' = bias + W·beta                                    (GELU'd for FFN1)
    must equal LayerNorm(v)·W^T + bias in float64 — rows with a mean offset and varied scale, so
    the mean · s cancellation is exercised.  Packed-plane output.  With shift (the plane shift):
    v carries per-column constants kappa (|kappa| ~ 3, outlier columns at 30-40), the A planes
    hold v - kappa and the accumulators start at kc = kappa·W'^T — the split error then scales
    with |v - kappa|, which the tolerance states.  Variant 1: the two-per-CU 128 x 192 kernel
    (tools library, ae_bench_gemm_packed_fold; kc added in its epilogue)."""
    lib = _fold_lib()
    K = 768
    g = torch.Generator().manual_seed(3 * M + N + gelu)
    st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    v = torch.randn(M, K, generator=g) * (0.5 + 2.0 * torch.rand(M, 1, generator=g)) + \
        3.0 * torch.randn(M, 1, generator=g)
    kap = 3.0 * torch.randn(K, generator=g)
    kap[[77, 300, 588]] = torch.tensor([30.0, -40.0, 35.0])
    if shift:
        v = v + kap
    gamma = 1.0 + 0.1 * torch.randn(K, generator=g)
    beta = 0.1 * torch.randn(K, generator=g)
    W = torch.randn(N, K, generator=g) * 0.05
    bias = torch.randn(N, generator=g) * 0.5
    Wf = W * gamma  # W·diag(gamma) in f32, as ae_create folds it
    Wh, Wl = _split(Wf)
    s = (Wh.double() + (Wl.double() if np_ == 2 else 0.0)).sum(1).float()
    bf = (bias.double() + W.double() @ beta.double()).float()
    dv = _pack(*_split(v - kap if shift else v), np_).cuda()
    dW = _pack(Wh, Wl, np_).cuda()
    ds, dbf = s.cuda(), bf.cuda()
    held = Wh.double() + (Wl.double() if np_ == 2 else 0.0)
    dkc = (held @ kap.double()).float().cuda() if shift else None
    dst = _tile_stats(v).cuda()
    out = torch.zeros((M, np_ * N), dtype=torch.bfloat16, device="cuda")
    if variant == 0:
        rc = lib.ae_launch_gemm_packed_fold(_p(dv), _p(dW), _p(dbf), _p(ds), _p(dst), 1e-5,
                                            _p(out), M, N, K, gelu, np_, _p(dkc), st)
    else:
        rc = lib.ae_bench_gemm_packed_fold(_p(dv), _p(dW), _p(dbf), _p(ds), _p(dst), 1e-5,
                                           _p(out), M, N, K, gelu, np_, _p(dkc), variant, 0, st)
    assert rc == 0
    torch.cuda.synchronize()
    x, var = _ln64(v, gamma, beta)
    ref = x @ W.double().T + bias.double()
    if gelu:
        ref = 0.5 * ref * (1.0 + torch.erf(ref / np.sqrt(2.0)))
    got = _unpack(out.cpu(), np_, N)
    # the split products' error on the planes' rows (v, or v - kappa under the plane shift), times
    # rstd: |v| includes the mean offset
    va = (v - kap if shift else v).abs().double()
    scale = (va @ Wf.abs().double().T) / torch.sqrt(var + 1e-5)
    rel = 1e-5 if np_ == 2 else 8e-3
    tol = rel * scale + (2e-5 if np_ == 2 else 1e-2) * ref.abs() + 2e-6
    assert torch.isfinite(got).all()
    assert ((got - ref).abs() <= tol).all(), float(((got - ref).abs() - tol).max())
