"""GPU parity: the HIP engine (through the C-ABI) against the oracle and the golden vectors.

Tolerances (BASELINE.json north_star): class probabilities within 1e-4 in fp32 mode; integer work
(splice ids, top-k ids, query counts) bit-exact.
"""
import numpy as np
import pytest
import torch

from conftest import golden, synthetic_sd
from oracle import roberta_cpu as ora

pytestmark = pytest.mark.gpu

PROB_TOL = 1e-4


def _engine(seed, head, num_labels=1, with_mlm=False, precision="fp32"):
    from apmc_amd.engine import Engine
    cache = _engine.__dict__.setdefault("cache", {})
    key = (seed, head, num_labels, with_mlm, precision)
    if key not in cache:
        cache[key] = Engine(synthetic_sd(seed, head, num_labels, with_mlm), head=head,
                            num_labels=num_labels, with_mlm=with_mlm, precision=precision)
    return cache[key]


def _score(eng, ids):
    ids = np.ascontiguousarray(ids, dtype=np.int32)
    lens = (ids != 1).sum(1).astype(np.int32)
    out = eng.score(torch.from_numpy(ids).cuda(), lens)
    torch.cuda.synchronize()
    return out.cpu().numpy()


def _rand_ids(rng, n, L, lens):
    ids = np.full((n, L), 1, dtype=np.int32)
    for i, ln in enumerate(lens):
        ids[i, 0] = 0
        ids[i, 1:ln - 1] = rng.integers(4, 50264, size=ln - 2)
        ids[i, ln - 1] = 2
    return ids


def test_devign_matches_golden(gpu):
    g = golden()
    p = _score(_engine(0, "sigmoid1"), g["devign_ids"])
    np.testing.assert_allclose(p, g["devign_probs"], atol=PROB_TOL, rtol=0)


def test_authorship_matches_golden(gpu):
    g = golden()
    p = _score(_engine(1, "softmaxN", 66), g["aa_ids"])
    np.testing.assert_allclose(p, g["aa_probs"], atol=PROB_TOL, rtol=0)


def test_clone_pair_matches_golden(gpu):
    g = golden()
    p = _score(_engine(2, "pair2", 2), g["clone_ids"])
    np.testing.assert_allclose(p, g["clone_probs"], atol=PROB_TOL, rtol=0)


@pytest.mark.parametrize("precision", ["fp32", "f32x3"])
@pytest.mark.parametrize("seed,head,num_labels,key", [(0, "sigmoid1", 1, "devign"),
                                                      (1, "softmaxN", 66, "aa"),
                                                      (2, "pair2", 2, "clone")])
def test_heads_match_golden_at_block_512(gpu, precision, seed, head, num_labels, key):
    """The headline config's length pinned to transformers directly (not only through the oracle):
    rows of 512, 510, 300, 129 tokens, one with literal <pad> ids inside, for every head
    (tests/golden/make_golden_encoder_512.py; ref CodeXGLUE/Defect-detection/code/model.py:24-34,
    gi_attack.py:129-131)."""
    from conftest import golden512
    g = golden512()
    p = _score(_engine(seed, head, num_labels, precision=precision), g[f"{key}_ids"])
    np.testing.assert_allclose(p, g[f"{key}_probs"], atol=PROB_TOL, rtol=0)


@pytest.mark.parametrize("L,lens", [(128, [128, 1 + 2, 77, 31, 128, 64, 100, 2, 33, 97]),
                                    (512, [512, 300, 511, 129])])
def test_varlen_batch_matches_oracle(gpu, L, lens):
    rng = np.random.default_rng(L)
    ids = _rand_ids(rng, len(lens), L, lens)
    sd = synthetic_sd(0, "sigmoid1")
    ref = ora.score(sd, ids, "sigmoid1")
    p = _score(_engine(0, "sigmoid1"), ids)
    np.testing.assert_allclose(p, ref, atol=PROB_TOL, rtol=0)


def test_encode_hidden_matches_oracle(gpu):
    rng = np.random.default_rng(7)
    lens = [96, 40, 65]
    ids = _rand_ids(rng, 3, 96, lens)
    sd = synthetic_sd(0, "sigmoid1")
    ref = ora.encoder_forward(sd, ids).numpy()
    eng = _engine(0, "sigmoid1")
    h = eng.encode(torch.from_numpy(ids).cuda(), np.array(lens, np.int32))
    torch.cuda.synchronize()
    h = h.cpu().numpy()
    for i, ln in enumerate(lens):
        np.testing.assert_allclose(h[i, :ln], ref[i, :ln], atol=5e-4, rtol=0)


def test_rows_are_batch_invariant_bitwise(gpu):
    rng = np.random.default_rng(11)
    ids = _rand_ids(rng, 6, 160, [160, 20, 90, 160, 5, 129])
    eng = _engine(0, "sigmoid1")
    full = _score(eng, ids)
    for i in range(6):
        one = _score(eng, ids[i:i + 1])
        assert one[0, 0] == full[i, 0]


def test_mlm_topk_matches_golden(gpu):
    g = golden()
    eng = _engine(3, "none", 1, True)
    sc, ix = eng.mlm_topk(torch.from_numpy(g["mlm_ids"][0]).cuda(), 60)
    torch.cuda.synchronize()
    np.testing.assert_allclose(sc.cpu().numpy(), g["mlm_top_scores"], atol=1e-3, rtol=0)
    # ids exact wherever the golden order is decided by more than twice the measured score error:
    # a position is exempt only when its golden score is within 2·max|score - golden| of a
    # neighbour's (a near-tie that error may reorder); the last position is exempt (the 61st
    # golden score is unknown)
    gs, gi, got = g["mlm_top_scores"], g["mlm_top_ids"], ix.cpu().numpy()
    eps = 2.0 * float(np.abs(sc.cpu().numpy() - gs).max()) + 1e-7
    prev = np.concatenate([np.full((gs.shape[0], 1), np.inf), gs[:, :-1]], 1)
    nxt = np.concatenate([gs[:, 1:], np.full((gs.shape[0], 1), -np.inf)], 1)
    clear = (np.abs(prev - gs) > eps) & (np.abs(gs - nxt) > eps)
    clear[:, -1] = False
    assert clear.mean() > 0.8, (clear.mean(), eps)
    assert (got[clear] == gi[clear]).all(), np.argwhere((got != gi) & clear)[:5]


def test_topk_kernel_exact_with_ties(gpu):
    from apmc_amd.engine import topk
    rng = np.random.default_rng(3)
    x = rng.standard_normal((37, 50265)).astype(np.float32)
    x[5, 100:200] = 9.0          # 100-way tie above everything else: take the 60 lowest indices
    x[6, :] = 0.0                # all equal
    x[7, 3] = -np.inf
    vals, idx = topk(torch.from_numpy(x).cuda(), 60)
    torch.cuda.synchronize()
    vals, idx = vals.cpu().numpy(), idx.cpu().numpy()
    for r in range(x.shape[0]):
        order = np.lexsort((np.arange(x.shape[1]), -x[r]))[:60]
        assert (idx[r] == order).all(), r
        assert (vals[r] == x[r, order]).all(), r


def test_splice_kernel_bit_exact(gpu):
    from apmc_amd.engine import splice
    rng = np.random.default_rng(9)
    n_words = 50
    wlens = rng.integers(1, 6, n_words)
    word_off = np.concatenate([[0], np.cumsum(wlens)]).astype(np.int32)
    word_tok = rng.integers(4, 50000, word_off[-1]).astype(np.int32)
    muts = [rng.integers(0, n_words, rng.integers(0, 400)).astype(np.int32) for _ in range(23)]
    mut_off = np.concatenate([[0], np.cumsum([len(m) for m in muts])]).astype(np.int32)
    mut_words = np.concatenate(muts).astype(np.int32)
    L = 128
    ids, lens = splice(torch.from_numpy(word_tok).cuda(), torch.from_numpy(word_off).cuda(),
                       torch.from_numpy(mut_words).cuda(), torch.from_numpy(mut_off).cuda(),
                       len(muts), L)
    torch.cuda.synchronize()
    ids, lens = ids.cpu().numpy(), lens.cpu().numpy()
    for m, ws in enumerate(muts):
        toks = [t for w in ws for t in word_tok[word_off[w]:word_off[w + 1]]][:L - 2]
        ref = [0] + toks + [2] + [1] * (L - 2 - len(toks))
        assert ids[m].tolist() == ref
        assert lens[m] == len(toks) + 2


def test_cosine_rank_matches_torch(gpu):
    from apmc_amd.engine import cosine_rank
    rng = np.random.default_rng(4)
    ref = rng.standard_normal((3, 768)).astype(np.float32)
    cand = rng.standard_normal((60, 3, 768)).astype(np.float32)
    sims = cosine_rank(torch.from_numpy(ref).cuda(), torch.from_numpy(cand).cuda())
    torch.cuda.synchronize()
    cos = torch.nn.CosineSimilarity(dim=1, eps=1e-6)
    exp = [float(sum(cos(torch.from_numpy(ref), torch.from_numpy(cand[i]))) / 3) for i in range(60)]
    np.testing.assert_allclose(sims.cpu().numpy(), exp, atol=1e-5)


def test_model_get_results_contract(gpu):
    from apmc_amd.model import Model
    g = golden()
    m = Model(_engine(0, "sigmoid1"))
    ds = [(torch.from_numpy(r.astype(np.int64)), torch.tensor(1)) for r in g["devign_ids"]]
    probs, preds = m.get_results(ds, 64)
    assert m.query == len(ds)
    probs2, _ = m.get_results([ds[0]], 64)
    assert m.query == len(ds) + 1
    assert len(probs) == len(ds) and all(len(p) == 2 for p in probs)
    p1 = np.array([p[1] for p in probs])
    np.testing.assert_allclose(p1, g["devign_probs"][:, 0], atol=PROB_TOL)
    assert preds == [int(v > 0.5) for v in p1]
    assert isinstance(probs[0][1], np.float32)
    assert probs2[0][1] == probs[0][1]


# split-bf16 ("f32x3") must stay inside the fp32 parity tolerance; plain bf16 is the stated
# bf16 tolerance (2e-2 on probabilities, measured ~1e-2 max in CPU emulation)
@pytest.mark.parametrize("precision,tol", [("f32x3", PROB_TOL), ("bf16", 2e-2)])
def test_split_precision_modes(gpu, precision, tol):
    rng = np.random.default_rng(21)
    lens = [512, 300, 129, 77, 512, 5, 256, 400]
    ids = _rand_ids(rng, len(lens), 512, lens)
    sd = synthetic_sd(0, "sigmoid1")
    ref = ora.score(sd, ids, "sigmoid1")
    p = _score(_engine(0, "sigmoid1", precision=precision), ids)
    np.testing.assert_allclose(p, ref, atol=tol, rtol=0)


def test_split_precision_other_heads(gpu):
    g = golden()
    p = _score(_engine(1, "softmaxN", 66, precision="f32x3"), g["aa_ids"])
    np.testing.assert_allclose(p, g["aa_probs"], atol=PROB_TOL, rtol=0)
    p = _score(_engine(2, "pair2", 2, precision="f32x3"), g["clone_ids"])
    np.testing.assert_allclose(p, g["clone_probs"], atol=PROB_TOL, rtol=0)


def _pack_mask(m):
    """bool [n, L, L] -> uint32 [n, L, L/32] (bit k%32 of word k/32 = query may attend key k)."""
    n, L, _ = m.shape
    bits = m.reshape(n, L, L // 32, 32).astype(np.uint64)
    w = (bits << np.arange(32, dtype=np.uint64)).sum(-1)
    return w.astype(np.uint32)


@pytest.mark.parametrize("precision,tol", [("fp32", PROB_TOL), ("f32x3", PROB_TOL)])
def test_dataflow_mask_and_explicit_positions(gpu, precision, tol):
    """GraphCodeBERT path (GraphCodeBERT/Defect-detection/code/model.py:24-45): explicit position
    ids and a [L, L] attention mask (bit-packed), pads only at the tail."""
    rng = np.random.default_rng(17)
    L, lens = 96, [96, 70, 33]
    ids = _rand_ids(rng, len(lens), L, lens)
    pos = np.ones((len(lens), L), dtype=np.int32)
    m = np.zeros((len(lens), L, L), dtype=bool)
    for i, ln in enumerate(lens):
        n_code = ln - ln // 4                       # code tokens then "DFG nodes"
        pos[i, :n_code] = np.arange(2, n_code + 2)
        pos[i, n_code:ln] = 0
        ids[i, n_code:ln - 1] = 3                   # nodes carry <unk>
        blk = rng.random((ln, ln)) < 0.3
        blk[np.arange(ln), np.arange(ln)] = True
        blk[:n_code, :n_code] = True
        blk[0, :] = True
        m[i, :ln, :ln] = blk
    sd = synthetic_sd(0, "sigmoid1")
    ref = ora.score(sd, ids, "sigmoid1", pos=pos, attn_mask=m)
    eng = _engine(0, "sigmoid1", precision=precision)
    lens_np = np.array(lens, np.int32)
    out = eng.score(torch.from_numpy(ids).cuda(), lens_np, pos=torch.from_numpy(pos).cuda(),
                    mask_bits=torch.from_numpy(_pack_mask(m)).cuda())
    torch.cuda.synchronize()
    np.testing.assert_allclose(out.cpu().numpy(), ref, atol=tol, rtol=0)


@pytest.mark.parametrize("precision", ["fp32", "f32x3"])
@pytest.mark.parametrize("head,num_labels", [("sigmoid1", 1), ("pair2", 2)])
def test_scores_batch_invariant_across_split_k(gpu, precision, head, num_labels):
    """A row's probabilities do not depend on how many rows share the launch: 8 rows take the
    segmented split-K form of the last layer's CLS GEMMs and the classifier head (grids of < 128
    tiles), 3000 rows the unsplit form; both sum the same K segments in the same order, so the
    8 rows' scores must be bit-identical (the batched attack drivers rely on this)."""
    eng = _engine(4, head, num_labels, precision=precision)
    rng = np.random.default_rng(21)
    n, L = 3000, 16
    ids = _rand_ids(rng, n, L, rng.integers(3, L + 1, n))
    big = _score(eng, ids)
    small = _score(eng, ids[:8])  # 8 sequences = 4 pair rows for the pair head
    k = small.shape[0]
    assert np.array_equal(big[:k], small), np.abs(big[:k] - small).max()


@pytest.mark.parametrize("precision", ["f32x3", "bf16"])
@pytest.mark.parametrize("n", [1, 3, 64])
def test_two_stream_encoder_matches_single_stream(gpu, monkeypatch, precision, n):
    """The split-precision engine's default two-stream encoder (two half-batch streams, residual +
    LayerNorm as its own kernel) against the same engine built with AE_SPLIT_STREAMS=0 (one
    stream, fused residual + LayerNorm epilogue): odd and single-row batches, ragged lengths
    across a 256-row tile boundary; the two differ only by LayerNorm rounding."""
    from apmc_amd.engine import Engine
    sd = synthetic_sd(6, "softmaxN", 5)
    engines = {}
    for mode, streams in (("1", "two"), ("0", "one")):  # ae_config.streams
        engines[mode] = Engine(sd, head="softmaxN", num_labels=5, precision=precision,
                               streams=streams)
    rng = np.random.default_rng(30 + n)
    L = 384
    ids = _rand_ids(rng, n, L, rng.integers(3, L + 1, n))
    a, b = _score(engines["1"], ids), _score(engines["0"], ids)
    tol = 1e-4 if precision == "f32x3" else 2e-2
    np.testing.assert_allclose(a, b, atol=tol, rtol=0)
    for e in engines.values():
        e.close()


@pytest.mark.parametrize("precision,tol", [("fp32", 2e-6), ("f32x3", 2e-5), ("bf16", 2e-2)])
def test_cls_absorbed_attention_matches_full_path(gpu, monkeypatch, precision, tol):
    """The last layer's CLS attention with W_k absorbed into the query and W_v applied to the
    p-weighted row sum (cls_attention.hip, the default) against the same engine built with
    AE_CLS_ABSORB=0 (the full-T QKV GEMM and a one-query attention): ragged lengths with
    1..10 chunks of 64 keys and partial 16-key tiles, and the 66-way head; the two differ only
    by summation order (plus the split products of the full path's K / V in split modes)."""
    from apmc_amd.engine import Engine
    sd = synthetic_sd(7, "softmaxN", 66)
    engines = {}
    for mode in ("1", "0"):
        monkeypatch.setenv("AE_CLS_ABSORB", mode)  # a knob of the tools library's engine
        engines[mode] = Engine(sd, head="softmaxN", num_labels=66, precision=precision,
                               tools=mode == "0")
    rng = np.random.default_rng(40)
    L = 640
    lens = np.array([640, 2, 3, 17, 63, 64, 65, 130, 511, 512, 333, 600], np.int32)
    ids = _rand_ids(rng, len(lens), L, lens)
    a, b = _score(engines["1"], ids), _score(engines["0"], ids)
    np.testing.assert_allclose(a, b, atol=tol, rtol=0)
    for e in engines.values():
        e.close()


@pytest.mark.parametrize("precision", ["fp32", "f32x3"])
def test_long_rows_batch_invariant_bitwise(gpu, precision):
    """Rows of 512 tokens (8 key chunks of the CLS attention, the two-stream encoder's parts):
    a row's probability is bit-identical whether it is scored among 200 rows or 5."""
    eng = _engine(4, "sigmoid1", 1, precision=precision)
    rng = np.random.default_rng(22)
    n, L = 200, 512
    ids = _rand_ids(rng, n, L, rng.integers(200, L + 1, n))
    big = _score(eng, ids)
    small = _score(eng, ids[:5])
    assert np.array_equal(big[:5], small), np.abs(big[:5] - small).max()


@pytest.mark.parametrize("precision", ["f32x3", "bf16"])
def test_encoder_forms_bit_identical(gpu, precision):
    """The two-stream encoder (the batch in parts, each on its own stream) and the single-stream
    one (streams="one") run the same per-row arithmetic — both LayerNorms folded into the GEMMs
    that follow them, no LayerNorm pass and no exchange between workgroups — so their scores are
    bit-identical: ragged lengths across 256-row blocks and the parts' boundaries, one row."""
    from apmc_amd.engine import Engine
    sd = synthetic_sd(6, "softmaxN", 5)
    engines = {s: Engine(sd, head="softmaxN", num_labels=5, precision=precision, streams=s)
               for s in ("two", "one")}
    rng = np.random.default_rng(50)
    for n, L in ((64, 384), (5, 300), (1, 77)):
        ids = _rand_ids(rng, n, L, rng.integers(3, L + 1, n))
        a, b = _score(engines["two"], ids), _score(engines["one"], ids)
        assert np.array_equal(a, b), np.abs(a - b).max()
    for e in engines.values():
        e.close()


OUTLIER_DIMS = np.array([77, 300, 588])
OUTLIER_SHIFT = np.array([25.0, -40.0, 30.0], dtype=np.float32)


def _fold_case_sd(case):
    """Synthetic weights for the folded-LayerNorm robustness test (seeded, deterministic).
    base: LayerNorm gains from 0.5..2 (so s = rowsum(W·diag(g)) is far from 0), every encoder /
    head weight row centred (W·1 = 0: a common row offset stays in the residual stream instead of
    swamping the tokens' signal), the classifier out_proj ~ N(0, 0.5) (the standard synthetic
    victim's) so the logits spread by about half a unit across rows (its bias is centred per case
    by the test).  shifted: every LayerNorm bias +4 and the O-projection / FFN2 biases +3, a row
    mean of about 7 against a std of 1-2 at every folded GEMM.  outlier: RoBERTa-style outlier
    features — three hidden dimensions carry LayerNorm shifts of +25 / -40 / +30 (gain 0.05), so
    the residual stream holds |v| of 25-40 there and the rows' variance is dominated by them; the
    other dimensions' gains are doubled to keep their scale after the LayerNorm, and the weights
    that read the residual stream (QKV, FFN1, the head's dense) read the outlier dimensions at
    0.2x, as trained models do (otherwise the constant outliers swamp every query and key and the
    rows' token signal vanishes)."""
    rng = np.random.default_rng(9)
    sd = {k: v.copy() for k, v in synthetic_sd(9, "sigmoid1", out_std=0.5).items()}
    for k in sd:
        if k.endswith("LayerNorm.weight"):
            sd[k] = rng.uniform(0.5, 2.0, sd[k].shape).astype(np.float32)
            if case == "outlier" and not k.startswith("lm_head"):
                sd[k] *= np.float32(2.0)
                sd[k][OUTLIER_DIMS] = 0.05
        elif (k.startswith("encoder.") or k.startswith("classifier.")) and sd[k].ndim == 2:
            sd[k] -= sd[k].mean(1, keepdims=True)
    for k in sd:
        if case == "shifted":
            if k.endswith("LayerNorm.bias") and not k.startswith("lm_head"):
                sd[k] += 4.0
            elif k.startswith("encoder.") and k.endswith("output.dense.bias"):  # O-proj and FFN2
                sd[k] += 3.0
        elif case == "outlier":
            if k.endswith("LayerNorm.bias") and not k.startswith("lm_head"):
                sd[k][OUTLIER_DIMS] += OUTLIER_SHIFT
            if k.endswith(("attention.self.query.weight", "attention.self.key.weight",
                           "attention.self.value.weight", "intermediate.dense.weight")) or \
                    k == "classifier.dense.weight":
                sd[k][:, OUTLIER_DIMS] *= np.float32(0.2)
    return sd


def _host_logits(sd, h):
    """The sequence-classification head (dense -> tanh -> out_proj, model.py:25 via
    RobertaClassificationHead) in float64 on the host, from the CLS rows h[:, 0]."""
    x = h[:, 0, :].astype(np.float64)
    x = np.tanh(x @ sd["classifier.dense.weight"].astype(np.float64).T +
                sd["classifier.dense.bias"].astype(np.float64))
    return (x @ sd["classifier.out_proj.weight"].astype(np.float64).T)[:, 0]


@pytest.mark.parametrize("precision", ["f32x3", "bf16"])
def test_folded_layernorm_robust_to_row_mean_offsets(gpu, precision):
    """The split modes fold each LayerNorm into the next GEMM: it multiplies the PRE-LayerNorm
    rows (split into bf16 planes) and subtracts mean · s in the epilogue, so the planes' rounding
    error scales with |v| instead of |v - mean|.  Three weight sets (_fold_case_sd): base, rows
    shifted to a mean of about 7σ at every folded GEMM, and RoBERTa-style outlier features (three
    dimensions at |v| 20-60).  Against the exact-fp32 mode (which normalises explicitly), per case:
    (i) the head's pre-sigmoid logits, computed in float64 from each mode's CLS rows with the
    out_proj bias centred (a non-saturation guard: logit std across rows >= 0.3) — |Δlogit| <= 4e-4
    in f32x3, which bounds |Δp| by 1e-4 at any logit (bf16, a diagnostic mode: 0.5); (ii) the
    engine's own probabilities at those logits, 1e-4 (bf16: 0.1, see below); (iii) the
    hidden-state error per row against that row's own spread (max_j |Δh_ij| / std_j h_ij over the
    real tokens): with the plane shift (gemm_planes.hip FoldArgs) the offsets and outliers cost
    nothing, so the shifted and outlier cases stay within 1.5x of the base weights' error in f32x3
    (2x in bf16) — without it the shifted case measured 2.7x (profiles/r6b_fold_test_noshift.log).
    The printed numbers are committed in profiles/."""
    from apmc_amd.engine import Engine
    rng = np.random.default_rng(9)
    n, L = 24, 512
    ids = _rand_ids(rng, n, L, rng.integers(40, L + 1, n))
    lens = (ids != 1).sum(1).astype(np.int32)
    dev_ids = torch.from_numpy(ids).cuda()
    real = ids != 1
    # bf16 (hi plane only) is a diagnostic mode: on these amplifying weights (gains up to 2) its
    # probabilities move by ~5e-2 already in the base case (r6c), so its bound here is the base
    # case's own scale, and the claim checked is relative: the offsets add nothing
    logit_tol, prob_tol = (4e-4, PROB_TOL) if precision == "f32x3" else (0.5, 0.1)
    rowrel, res = {}, {}
    for case in ("base", "shifted", "outlier"):
        sd = _fold_case_sd(case)
        e32 = Engine(sd, head="sigmoid1", precision="fp32")
        h32 = e32.encode(dev_ids, lens).cpu().numpy()
        e32.close()
        z = _host_logits(sd, h32)
        sd["classifier.out_proj.bias"] = np.array([-z.mean()], dtype=np.float32)
        e32 = Engine(sd, head="sigmoid1", precision="fp32")
        ex = Engine(sd, head="sigmoid1", precision=precision)
        hx = ex.encode(dev_ids, lens).cpu().numpy()
        z32, zx = _host_logits(sd, h32) - z.mean(), _host_logits(sd, hx) - z.mean()
        p32, px = _score(e32, ids), _score(ex, ids)
        e32.close()
        ex.close()
        # per real row against its own spread (pad rows stay 0 in both: no spread to divide by)
        d = np.abs(hx - h32)[real].max(-1) / h32[real].std(-1)
        rowrel[case] = float(d.max())
        vmax = float(np.abs(h32[real]).max())
        res[case] = (float(z32.std()), float(np.abs(zx - z32).max()),
                     float(np.abs(px - p32).max()), vmax)
        print(f"{precision} {case}: logit std {z32.std():.3f} range [{z32.min():.3f}, "
              f"{z32.max():.3f}], max |dlogit| {np.abs(zx - z32).max():.2e}, max |dp| "
              f"{np.abs(px - p32).max():.2e}, per-row rel {rowrel[case]:.2e}, max |h| {vmax:.1f}")
    for case, (zstd, dz, dp, vmax) in res.items():
        assert zstd >= 0.3, (case, zstd)
        assert dz <= logit_tol and dp <= prob_tol, (case, dz, dp)
        if case == "outlier":
            assert vmax >= 20.0, vmax
    k = 1.5 if precision == "f32x3" else 2.0
    assert rowrel["shifted"] <= k * rowrel["base"] and rowrel["outlier"] <= k * rowrel["base"], \
        rowrel


def test_bench_size_batch_properties(gpu):
    """At the bench's full sizes (config-2 rows of L = 512; the batch-1024 microbenchmark), the
    properties that do not need the oracle to run the whole batch: one 1024-row call equals
    sixteen 64-row calls bit for bit (the two-stream parts, tile rounds and split-K forms change
    with the batch, the arithmetic per row does not), every row of the f32x3 step is within the
    north-star tolerance of the exact-fp32 mode, and the first and last rows match the oracle."""
    rng = np.random.default_rng(0)
    n, L = 1024, 512
    ids = rng.integers(4, 50264, size=(n, L)).astype(np.int32)  # bench.py's id recipe
    ids[:, 0], ids[:, -1] = 0, 2
    eng = _engine(0, "sigmoid1", precision="f32x3")
    big = _score(eng, ids)
    chunks = np.concatenate([_score(eng, ids[i:i + 64]) for i in range(0, n, 64)])
    assert np.array_equal(big, chunks), np.abs(big - chunks).max()
    exact = _score(_engine(0, "sigmoid1", precision="fp32"), ids)
    np.testing.assert_allclose(big, exact, atol=PROB_TOL, rtol=0)
    ref = ora.score(synthetic_sd(0, "sigmoid1"), ids[[0, n - 1]], "sigmoid1")
    np.testing.assert_allclose(big[[0, n - 1]], ref, atol=PROB_TOL, rtol=0)
