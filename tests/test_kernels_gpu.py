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
    # its packed-plane epilogue (the QKV GEMM, AE_QKV192): N % 192 == 0, ragged M
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


@pytest.mark.parametrize("variant", [6, 66, 67, 72])
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
    for v in (6, 66, 67, 72):
        op = torch.zeros((T, 2 * 768), dtype=torch.int16, device="cuda")
        assert lib.ae_bench_attention_pp(_p(dq), None, _p(op), _p(dcu), None, max(lens), n, 12,
                                         None, 0, 2, v, st) == 0
        outs[v] = op
    torch.cuda.synchronize()
    assert torch.equal(outs[66], outs[6])
    assert torch.equal(outs[67], outs[6])
    assert torch.equal(outs[72], outs[6])  # exp / split and the next S MFMAs hand-interleaved


@pytest.mark.parametrize("M,K,np_", [(300, 768, 2), (512, 3072, 2), (1000, 768, 1), (37, 768, 2),
                                     (4097, 768, 2)])
def test_gemm_packed_ln_matches_f64(gpu, M, K, np_):
    """ae_launch_gemm_packed_ln (256 x 192 kernel, PK_EPI_RES_LN): x = LayerNorm(A·W^T + bias + x)
    over 768-wide rows whose 4 column tiles live in 4 workgroups that exchange row statistics.
    Against float64 of the split products; the residual aliases the output (in place, as the
    engine runs it); three launches in a row reuse the self-resetting row-block counters (a
    counter left non-zero would make a later launch read stale statistics or time out)."""
    lib = _lib()
    vp, i32 = ctypes.c_void_p, ctypes.c_int32
    lib.ae_launch_gemm_packed_ln.argtypes = [vp] * 6 + [i32] * 4 + [vp, vp, ctypes.c_float] + \
        [vp] * 4
    lib.ae_launch_gemm_packed_ln.restype = ctypes.c_int
    N = 768
    g = torch.Generator().manual_seed(M + K)
    W = torch.randn(N, K, generator=g) * 0.05
    bias = torch.randn(N, generator=g) * 0.5
    gamma = 1.0 + 0.1 * torch.randn(N, generator=g)
    beta = 0.1 * torch.randn(N, generator=g)
    Wh, Wl = _split(W)
    dW = _pack(Wh, Wl, np_).cuda()
    # device copies held by name: a temporary's memory is recycled before the launch reads it
    db, dg, dbeta = bias.cuda(), gamma.cuda(), beta.cuda()
    blocks = (M + 255) // 256
    stats = torch.zeros(blocks * 256 * 4, dtype=torch.int64, device="cuda")
    ctr = torch.zeros(2 * blocks, dtype=torch.int32, device="cuda")
    err = torch.zeros(4, dtype=torch.int32, device="cuda")
    st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    for it in range(3):
        A = torch.randn(M, K, generator=g) * 0.7
        X = torch.randn(M, N, generator=g) * 2.0 + 0.5
        Ah, Al = _split(A)
        y = Ah.double() @ Wh.double().T
        if np_ == 2:
            y = y + Ah.double() @ Wl.double().T + Al.double() @ Wh.double().T
        y = y + bias.double() + X.double()
        mu = y.mean(1, keepdim=True)
        var = ((y - mu) ** 2).mean(1, keepdim=True)
        ref = (y - mu) / torch.sqrt(var + 1e-5) * gamma.double() + beta.double()
        scale = (A.abs().double() @ W.abs().double().T).amax(1, keepdim=True)
        dA = _pack(Ah, Al, np_).cuda()
        x = X.cuda()
        xp = torch.zeros((M, np_ * N), dtype=torch.bfloat16, device="cuda")
        rc = lib.ae_launch_gemm_packed_ln(_p(dA), _p(dW), _p(db), _p(x), _p(x), _p(xp),
                                          M, N, K, np_, _p(dg), _p(dbeta), 1e-5,
                                          _p(stats), _p(ctr), _p(err), st)
        assert rc == 0
        torch.cuda.synchronize()
        assert int(err[0]) == 0 and int(ctr.abs().sum()) == 0, it
        got = x.double().cpu()
        # LN amplifies the GEMM's f32-accumulation error by rstd * gamma
        tol = (1e-5 * scale + 1e-6) * 1.2 / torch.sqrt(var + 1e-5) + 2e-6
        assert torch.isfinite(got).all()
        assert ((got - ref).abs() <= tol).all(), (it, float(((got - ref).abs() - tol).max()))
        planes = _unpack(xp.cpu(), np_, N)
        rel = 2e-5 if np_ == 2 else 5e-3
        assert ((planes - got).abs() <= rel * got.abs() + 1e-7).all(), it
