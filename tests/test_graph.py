"""GraphCodeBERT path: data-flow featurisation + graph-guided mask (CPU, bit-exact against
oracle/graph_ref.py on the reference's Devign fixture functions) and the node-averaged forward
through ae_score_graph (GPU, probabilities within 1e-4 of the oracle in fp32 / f32x3)."""
import types

import numpy as np
import pytest

from conftest import ROOT, synthetic_sd
from oracle import graph_ref

DEVIGN = ROOT / "data" / "devign" / "test_subs_0_400.jsonl"
PROB_TOL = 1e-4
# GraphCodeBERT Devign attack defaults (GraphCodeBERT/Defect-detection/code/attack.py:460-467)
ARGS = types.SimpleNamespace(code_length=256, data_flow_length=64, block_size=512,
                             eval_batch_size=64)


def _funcs(limit):
    import json
    out = []
    with open(DEVIGN) as f:
        for i, line in enumerate(f):
            if i >= limit:
                break
            js = json.loads(line)
            out.append((js["func"], int(js["target"])))
    return out


@pytest.fixture(scope="module")
def tok():
    from apmc_amd.host import Tokenizer
    return Tokenizer()


def _oracle_features(code, args):
    from apmc_amd.graph import extract_dataflow
    code = " ".join(code.split())
    dfg, _, toks = extract_dataflow(code, "c")
    return graph_ref.convert_code_to_features(dfg, toks, args.code_length, args.data_flow_length)


@pytest.mark.parametrize("code_length,dfl", [(256, 64), (512, 128), (64, 32)])
def test_features_and_mask_match_oracle(tok, code_length, dfl):
    from apmc_amd.graph import convert_code_to_features, graph_mask, pack_mask
    args = types.SimpleNamespace(code_length=code_length, data_flow_length=dfl)
    L = code_length + dfl
    n_nodes = 0
    for code, label in _funcs(60):
        f = convert_code_to_features(code, tok, label, args)
        ids, pos, d2c, d2d = _oracle_features(code, args)
        assert f.input_ids == ids
        assert f.position_idx == pos
        assert [tuple(x) for x in f.dfg_to_code] == [tuple(x) for x in d2c]
        assert f.dfg_to_dfg == d2d
        m = graph_mask(f.input_ids, f.position_idx, f.dfg_to_code, f.dfg_to_dfg)
        np.testing.assert_array_equal(m, graph_ref.graph_mask(ids, pos, d2c, d2d, L))
        bits = pack_mask(m).view(np.uint32)
        for r in (0, 5, L - 1):  # bit layout: bit j of word w = key 32 w + j
            np.testing.assert_array_equal(
                np.array([(bits[r, k // 32] >> (k % 32)) & 1 for k in range(L)], bool), m[r])
        n_nodes += sum(p == 0 for p in pos)
    assert n_nodes > 0


def test_dataset_items_have_reference_shapes(tok):
    from apmc_amd.graph import (CodePairDataset, GraphCodeDataset, GraphPairFeatures,
                                convert_code_to_features)
    fs = [convert_code_to_features(c, tok, y, ARGS) for c, y in _funcs(3)]
    L = ARGS.code_length + ARGS.data_flow_length
    ids, m, pos, lab = GraphCodeDataset(fs)[1]
    assert ids.shape == (L,) and m.shape == (L, L) and pos.shape == (L,) and int(lab) == fs[1].label
    ids, pos, bits = GraphCodeDataset(fs).packed()
    assert ids.shape == (3, L) and bits.shape == (3, L, L // 32)
    item = CodePairDataset([GraphPairFeatures(fs[0], fs[1], 1)])[0]
    assert len(item) == 7 and item[2].shape == (L, L) and item[5].shape == (L, L)


# ---------------------------------------------------------------------------------------- GPU
def _gmodel(task, precision="fp32"):
    from apmc_amd.graph import GraphModel
    cache = _gmodel.__dict__.setdefault("cache", {})
    key = (task, precision)
    if key not in cache:
        head, nl, seed = ("sigmoid1", 1, 0) if task == "devign" else ("pair2", 2, 2)
        cache[key] = GraphModel(synthetic_sd(seed, head, nl), config=nl, args=ARGS, task=task,
                                precision=precision)
    return cache[key]


@pytest.mark.gpu
@pytest.mark.parametrize("precision", ["fp32", "f32x3"])
def test_graph_devign_matches_oracle(gpu, tok, precision):
    from apmc_amd.graph import GraphCodeDataset, convert_code_to_features
    funcs = _funcs(6)
    fs = [convert_code_to_features(c, tok, y, ARGS) for c, y in funcs]
    L = ARGS.code_length + ARGS.data_flow_length
    ids = np.array([f.input_ids for f in fs])
    pos = np.array([f.position_idx for f in fs])
    m = np.stack([graph_ref.graph_mask(f.input_ids, f.position_idx, f.dfg_to_code, f.dfg_to_dfg,
                                       L) for f in fs])
    ref = graph_ref.graph_score(synthetic_sd(0, "sigmoid1"), ids, m, pos, "sigmoid1")
    model = _gmodel("devign", precision)
    q0 = model.query
    probs, preds = model.get_results(GraphCodeDataset(fs, ARGS), 64)
    assert model.query - q0 == len(fs)
    got = np.array([p[1] for p in probs])
    np.testing.assert_allclose(got, ref[:, 0], atol=PROB_TOL, rtol=0)
    assert preds == [1 if p > 0.5 else 0 for p in got]
    # the reference's tuple items (bool masks) take the same path
    ds = GraphCodeDataset(fs, ARGS)
    probs2, _ = model.get_results([ds[i] for i in range(len(ds))], 64)
    np.testing.assert_array_equal(np.array(probs2), np.array(probs))


@pytest.mark.gpu
def test_graph_node_average_matters(gpu, tok):
    """Without node averaging (plain ae_score) the probabilities differ: the averaging runs."""
    import torch
    from apmc_amd.graph import GraphCodeDataset, convert_code_to_features
    fs = [convert_code_to_features(c, tok, y, ARGS) for c, y in _funcs(4)]
    ids, pos, bits = GraphCodeDataset(fs).packed()
    model = _gmodel("devign")
    a = model.score_packed(ids, pos, bits)
    lens = (ids != 1).sum(1).astype(np.int32)
    b = model.engine.score(torch.from_numpy(ids).cuda(), lens, pos=torch.from_numpy(pos).cuda(),
                           mask_bits=torch.from_numpy(bits).cuda()).cpu().numpy()
    assert np.abs(a - b).max() > 1e-6


@pytest.mark.gpu
def test_graph_clone_pairs_match_oracle(gpu, tok):
    from apmc_amd.graph import CodePairDataset, GraphPairFeatures, convert_code_to_features
    fs = [convert_code_to_features(c, tok, y, ARGS) for c, y in _funcs(6)]
    pairs = [GraphPairFeatures(fs[i], fs[i + 1], i % 2) for i in range(0, 6, 2)]
    ds = CodePairDataset(pairs, ARGS)
    ids, pos, bits = ds.packed()
    L = ids.shape[1]
    m = np.stack([graph_ref.graph_mask(f.input_ids, f.position_idx, f.dfg_to_code, f.dfg_to_dfg,
                                       L) for f in fs])
    ref = graph_ref.graph_score(synthetic_sd(2, "pair2", 2), ids, m, pos, "pair2")
    model = _gmodel("clone")
    probs, preds = model.get_results(ds, 64)
    np.testing.assert_allclose(np.asarray(probs), ref, atol=PROB_TOL, rtol=0)
    assert preds == [0 if p[0] > 0.5 else 1 for p in ref]


# ---------------------------------------------------------------- transformers golden at L=640
def _golden():
    return dict(np.load(ROOT / "tests" / "golden" / "graph_golden.npz"))


def _unpack(bits):
    L = bits.shape[-1] * 32
    return np.unpackbits(bits.view(np.uint8), axis=-1, bitorder="little")[..., :L].astype(bool)


def test_golden_graph_features_are_reproduced(tok):
    """The golden's inputs (tests/golden/make_golden_graph.py) are today's features of the same
    fixture functions at L = 640 (code_length 512 + data_flow_length 128)."""
    from apmc_amd.graph import convert_code_to_features, graph_mask, pack_mask
    g = _golden()
    funcs = _funcs(60)
    args = types.SimpleNamespace(code_length=512, data_flow_length=128)
    for row, i in enumerate(g["gcb_pick"]):
        f = convert_code_to_features(funcs[i][0], tok, 0, args)
        assert f.input_ids == g["gcb_ids"][row].tolist()
        assert f.position_idx == g["gcb_pos"][row].tolist()
        m = graph_mask(f.input_ids, f.position_idx, f.dfg_to_code, f.dfg_to_dfg)
        np.testing.assert_array_equal(pack_mask(m), g["gcb_bits"][row])


@pytest.mark.parametrize("name,seed,head,nl", [("devign", 6, "sigmoid1", 1),
                                               ("clone", 7, "pair2", 2)])
def test_oracle_graph_forward_matches_transformers_golden(name, seed, head, nl):
    """oracle/graph_ref.graph_score (node averaging + roberta_cpu with the 3-D mask and explicit
    positions) against transformers' RobertaModel(inputs_embeds, 4-D additive mask, position_ids)
    at L = 640: pins the oracle the GPU graph tests compare the engine with."""
    g = _golden()
    sd = synthetic_sd(seed=seed, head=head, num_labels=nl)
    got = graph_ref.graph_score(sd, g["gcb_ids"], _unpack(g["gcb_bits"]), g["gcb_pos"], head)
    np.testing.assert_allclose(got, g[f"gcb_{name}_probs"], atol=1e-5, rtol=0)


@pytest.mark.gpu
@pytest.mark.parametrize("precision", ["fp32", "f32x3"])
def test_engine_graph_forward_matches_transformers_golden(precision):
    """ae_score_graph at L = 640 against the transformers golden (devign sigmoid and clone pair
    heads), probabilities within 1e-4."""
    from apmc_amd.graph import GraphModel
    g = _golden()
    for name, seed, head, nl, task in [("devign", 6, "sigmoid1", 1, "devign"),
                                       ("clone", 7, "pair2", 2, "clone")]:
        m = GraphModel(synthetic_sd(seed=seed, head=head, num_labels=nl), task=task,
                       precision=precision)
        got = m.score_packed(g["gcb_ids"], g["gcb_pos"], g["gcb_bits"])
        np.testing.assert_allclose(got, g[f"gcb_{name}_probs"], atol=PROB_TOL, rtol=0)


def _task_texts(task, n):
    from apmc_amd.drivers import load_fixture
    path = {"devign": ROOT / "data" / "devign" / "test_subs_0_400.jsonl",
            "clone": ROOT / "data" / "clone" / "test_subs_0_500.jsonl",
            "authorship": ROOT / "data" / "authorship" / "valid_subs.jsonl"}[task]
    codes, _, _ = load_fixture(path, 0, n)
    if task == "clone":
        return [c[2] for c in codes] + [c[3] for c in codes]
    return codes


@pytest.mark.parametrize("task,run_trunc", [("devign", False), ("clone", False), ("clone", True),
                                            ("authorship", False)])
def test_batch_featuriser_matches_python_features(task, run_trunc):
    """ah_gcb_features_batch (C++, worker threads) against graph.py convert_code_to_features on
    fixture texts of every GraphCodeBERT task (language, whitespace rule, data-flow builder, the
    clone run.py truncation): identical ids / positions / node count, and the mask rebuilt from
    the compact spans + edges equals GraphCodeDataset's bool mask."""
    import _apmc  # noqa: F401
    from apmc_amd.drivers import AttackArgs
    from apmc_amd.graph import DFG_GCB_RUN, TASK_FEATURES, convert_code_to_features, \
        graph_mask, graph_mask_from_compact
    from apmc_amd.host import Tokenizer

    tok = Tokenizer()
    args = AttackArgs(code_length=512, data_flow_length=128)
    texts = _task_texts(task, 30)
    lang, normalize, variant = TASK_FEATURES[task]
    if run_trunc:
        variant = DFG_GCB_RUN
    c = tok.gcb_features(texts, lang, variant, normalize, 512, 128, run_trunc=run_trunc, threads=3)
    for i, t in enumerate(texts):
        f = convert_code_to_features(t, tok, 0, args, lang, normalize, variant=variant,
                                     run_trunc=run_trunc)
        assert c["ids"][i].tolist() == f.input_ids, i
        assert c["pos"][i].tolist() == f.position_idx, i
        assert c["meta"][i][2] == len(f.dfg_to_code), i
        m = graph_mask(f.input_ids, f.position_idx, f.dfg_to_code, f.dfg_to_dfg)
        m2 = graph_mask_from_compact(c["ids"][i], c["meta"][i], c["spans"][i], c["edges"][i])
        assert (m == m2).all(), i


def edge_heavy_python():
    """A program whose data-flow graph has far more node-to-node edges than 4 x L at small
    code_length: 60 uses of a name defined in 24 if/elif branches (each use comes from all 24
    definitions)."""
    lines = ["def f(c):", "    if c == 0:", "        v = 0"]
    for i in range(1, 24):
        lines += [f"    elif c == {i}:", f"        v = {i}"]
    return "\n".join(lines + ["    y = " + " + ".join(["v"] * 60), "    return y"])


def test_edge_heavy_query_widens_edge_array():
    """the reference has no edge limit, so a query with more data-flow edges than the
    default edge capacity (4 x L) must not fail the batch: the featuriser retries with a wider
    array, and the compact features still rebuild GraphCodeDataset's exact mask; joining such a
    batch with ordinary ones pads the edge arrays."""
    import _apmc  # noqa: F401
    from apmc_amd.drivers import AttackArgs
    from apmc_amd.graph import TASK_FEATURES, _cat_compact, convert_code_to_features, \
        graph_mask, graph_mask_from_compact
    from apmc_amd.host import Tokenizer

    tok = Tokenizer()
    lang, normalize, variant = TASK_FEATURES["authorship"]
    cl, dfl = 32, 128
    texts = [edge_heavy_python()] + _task_texts("authorship", 3)
    c = tok.gcb_features(texts, lang, variant, normalize, cl, dfl)
    assert c["meta"][0][3] > 4 * (cl + dfl) and c["edges"].shape[1] >= c["meta"][0][3]
    args = AttackArgs(code_length=cl, data_flow_length=dfl)
    for i, t in enumerate(texts):
        f = convert_code_to_features(t, tok, 0, args, lang, normalize, variant=variant)
        assert c["ids"][i].tolist() == f.input_ids, i
        m = graph_mask(f.input_ids, f.position_idx, f.dfg_to_code, f.dfg_to_dfg)
        assert (m == graph_mask_from_compact(c["ids"][i], c["meta"][i], c["spans"][i],
                                             c["edges"][i])).all(), i
    plain = tok.gcb_features(texts[1:], lang, variant, normalize, cl, dfl)
    assert plain["edges"].shape[1] < c["edges"].shape[1]
    joined = _cat_compact([plain, c])
    assert joined["edges"].shape == (len(texts) + 3, c["edges"].shape[1])
    for i in range(3):
        assert (graph_mask_from_compact(joined["ids"][i], joined["meta"][i], joined["spans"][i],
                                        joined["edges"][i]) ==
                graph_mask_from_compact(plain["ids"][i], plain["meta"][i], plain["spans"][i],
                                        plain["edges"][i])).all()


@pytest.mark.gpu
def test_device_graph_mask_matches_host(gpu):
    """ae_graph_mask (rowops.hip) builds exactly pack_mask(graph_mask) of every query, for the
    three tasks' fixture texts (L = 640) and a short L = 96 case."""
    import torch

    import _apmc  # noqa: F401
    from apmc_amd.engine import Engine
    from apmc_amd.graph import TASK_FEATURES, graph_mask_from_compact, pack_mask
    from apmc_amd.host import Tokenizer
    from apmc_amd.weights import RobertaShape, synthetic_state_dict

    tok = Tokenizer()
    shape = RobertaShape(layers=1)
    eng = Engine(synthetic_state_dict(seed=1, shape=shape, head="sigmoid1"), head="sigmoid1",
                 num_labels=1, shape=shape, precision="fp32")
    for task in ("devign", "clone", "authorship"):
        lang, normalize, variant = TASK_FEATURES[task]
        for cl, dfl in ((512, 128), (64, 32), (32, 128)):
            texts = _task_texts(task, 12) + ([edge_heavy_python()] if task == "authorship" else [])
            c = tok.gcb_features(texts, lang, variant, normalize, cl, dfl)
            t = {k: torch.from_numpy(v).cuda() for k, v in c.items()}
            bits = eng.graph_mask(t["ids"], t["meta"], t["spans"], t["edges"]).cpu().numpy()
            for i in range(len(c["ids"])):
                ref = pack_mask(graph_mask_from_compact(c["ids"][i], c["meta"][i], c["spans"][i],
                                                        c["edges"][i]))
                assert (bits[i] == ref).all(), (task, cl, i)
    eng.close()
