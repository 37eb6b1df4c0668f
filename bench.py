"""Benchmark of the victim-query hot path (BASELINE.json metric, config 2 workload shape).

A "step" = one Model.get_results-equivalent pass of the engine over one GA population batch of
synthetic mutants: B (=64, GA eval_batch_size, CodeXGLUE/Defect-detection/README.md:261) sequences
x L=512 tokens (no padding, CLS=0 / SEP=2, interior ids uniform in [4, 50263], seed 0+rank),
scored by the CodeBERT-shaped Devign victim (seeded synthetic weights: no checkpoint offline).
Inputs are resident in HBM before the timed region.  Per-GPU work is fixed (weak scaling): each
rank scores its own batches; there is no data-path collective.  The only collectives are the
barrier around the timed region and the MAX-reduction of the elapsed time.

Prints ONE JSON line (rank 0).  `roofline` is the dominant kernel (the FFN1 GEMM,
[T,768]x[768,3072] + bias + GELU) timed live with HIP events on the launch stream;
`cpu_baseline` is oracle/roberta_cpu.py (PyTorch-CPU fp32 eager restatement) on host cores.
"""
import argparse
import glob
import json
import os
import pathlib
import sys
import time

ROOT = pathlib.Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT))

import numpy as np  # noqa: E402
import torch  # noqa: E402

import _apmc  # noqa: E402,F401

FP32_MFMA_PEAK_TFLOPS = 157.3   # MI355X_MICROARCH.md: f32-input MFMA dense peak (spec)
BF16_MFMA_PEAK_TFLOPS = 2516.6  # dense bf16 (spec, no sparsity)
METRIC = "victim queries/sec + attacked examples/min (node), CodeBERT Devign GA attack"


def flops_per_query(L, C=1):
    per_tok = 2 * (4 * 768 * 768 + 2 * 768 * 3072)
    return 12 * (L * per_tok + 4 * L * L * 768) + 2 * 768 * 768 + 2 * 768 * C


def pmc_traffic_per_launch(precision):
    """HBM bytes per FFN1 launch of this precision's kernel from the committed rocprofv3 PMC
    summary (profiles/*pmc_ffn1.json, newest first), or None."""
    for f in sorted(glob.glob(str(ROOT / "profiles" / "*pmc*ffn1*.json")), reverse=True):
        try:
            d = json.load(open(f))
            if d.get("precision", "fp32") == precision:
                return float(d["hbm_bytes_per_launch"])
        except Exception:
            continue
    return None


def cpu_baseline(L, seconds, threads):
    from apmc_amd.weights import synthetic_state_dict
    from oracle import roberta_cpu as ora

    torch.set_num_threads(threads)
    sd = synthetic_state_dict(seed=0, head="sigmoid1")
    rng = np.random.default_rng(0)
    B = 4
    ids = rng.integers(4, 50264, size=(B, L)).astype(np.int64)
    ids[:, 0], ids[:, -1] = 0, 2
    ora.score(sd, ids[:1, :64], "sigmoid1")  # warm up allocator / threads
    done, t0 = 0, time.perf_counter()
    while True:
        ora.score(sd, ids, "sigmoid1")
        done += B
        el = time.perf_counter() - t0
        if el >= seconds:
            break
    return {"value": done / el, "unit": "victim queries/s", "cores": threads, "kind": "port",
            "sample": f"{done} queries of L={L} (batches of {B}) in {el:.1f} s, "
                      f"oracle/roberta_cpu.py fp32 eager, torch threads={threads}"}


def attack_leg(dev, seconds, rank, world, precision):
    """End-to-end config-2 workload: greedy -> GA attack (gi_attack.py --use_ga) over the
    test_subs_0_400 fixture, examples pulled in order from a shared queue until the time budget is
    spent; victim queries/s and attacked examples/min over the whole job."""
    from apmc_amd.drivers import AttackArgs, load_fixture, run_gi_attack
    from apmc_amd.model import Model
    from apmc_amd.weights import synthetic_state_dict

    codes, subs, labels = load_fixture(ROOT / "data" / "devign" / "test_subs_0_400.jsonl")
    model = Model(synthetic_state_dict(seed=0, head="sigmoid1"), task="devign",
                  precision=precision, device=dev.index)
    args = AttackArgs(block_size=512, eval_batch_size=64, seed=123456, rng="per_example")
    from apmc_amd.dist import DynamicQueue

    # all ranks pull the next example index from one atomic counter in the torch.distributed
    # store (no tensor traffic), until the time budget is spent
    queue = DynamicQueue(len(codes), key="bench_attack_queue",
                         deadline=time.time() + seconds)
    if world > 1:
        import torch.distributed as dist
        dist.barrier()
    out = run_gi_attack(model, codes, subs, labels, args, queue=queue)
    stats = np.array([out["examples"], out["total_cnt"], out["success"], out["queries"],
                      out["wall_s"]], dtype=np.float64)
    if world > 1:
        import torch.distributed as dist
        t = torch.tensor(stats, device=dev)
        g = [torch.zeros_like(t) for _ in range(world)]
        dist.all_gather(g, t)
        allst = torch.stack(g).cpu().numpy()
    else:
        allst = stats[None]
    ex, cnt, suc, q = allst[:, 0].sum(), allst[:, 1].sum(), allst[:, 2].sum(), allst[:, 3].sum()
    wall = allst[:, 4].max()
    ga = sum(r["attack_type"] == "GA" for r in out["records"])
    return {"workload": "CodeBERT Devign greedy->GA attack (gi_attack --use_ga), "
                        "test_subs_0_400.jsonl in order, block 512, eval_batch_size 64",
            "precision": precision,
            "examples": int(ex), "correctly_classified": int(cnt), "successes": int(suc),
            "success_rate": round(suc / cnt, 4) if cnt else None, "victim_queries": int(q),
            "wall_s": round(wall, 2), "victim_queries_per_s": round(q / wall, 2),
            "attacked_examples_per_min": round(60 * ex / wall, 3),
            "rank0_ga_runs": int(ga), "rng": "random.seed(123456 + index) per example",
            "sharding": "dynamic queue (torch.distributed store counter)"}


def mhm_leg(dev, n_examples, seq_examples, rank, world, precision):
    """Config-5 baseline workload: MHM-NS (mhm_attack.py, n_candi 30, max_iter 100, threshold 1)
    over test_subs_0_400 with the CodeBERT Devign victim.  Batched: the first `n_examples` fixture
    examples (strided over ranks) with every chain in flight at once (`mcmc_batched`); sequential:
    the reference loop (one ≤31-candidate batch per query round) over the first `seq_examples`
    of them, for the comparison (rank 0, N=1 only)."""
    from apmc_amd.drivers import AttackArgs, load_fixture, run_mhm_attack
    from apmc_amd.model import Model
    from apmc_amd.weights import synthetic_state_dict

    codes, subs, labels = load_fixture(ROOT / "data" / "devign" / "test_subs_0_400.jsonl")
    model = Model(synthetic_state_dict(seed=0, head="sigmoid1"), task="devign",
                  precision=precision, device=dev.index)
    args = AttackArgs(block_size=512, eval_batch_size=64, seed=123456)
    mine = list(range(rank, n_examples, world))
    if world > 1:
        import torch.distributed as dist
        dist.barrier()
    out = run_mhm_attack(model, codes, subs, labels, args, indices=mine, max_iter=100,
                         prob_threshold=1, max_inflight=len(mine))
    st = np.array([out["examples"], out["total_cnt"], out["success"], out["queries"],
                   out["wall_s"]], dtype=np.float64)
    if world > 1:
        import torch.distributed as dist
        t = torch.tensor(st, device=dev)
        g = [torch.zeros_like(t) for _ in range(world)]
        dist.all_gather(g, t)
        allst = torch.stack(g).cpu().numpy()
    else:
        allst = st[None]
    ex, cnt, suc, q = allst[:, :4].sum(0)
    wall = allst[:, 4].max()
    res = {"workload": "MHM-NS (mhm_attack.py: n_candi 30, max_iter 100) CodeBERT Devign victim, "
                       f"test_subs_0_400 examples [0, {n_examples}), block 512",
           "precision": precision, "examples": int(ex), "correctly_classified": int(cnt),
           "successes": int(suc), "victim_queries": int(q), "wall_s": round(wall, 2),
           "victim_queries_per_s": round(q / wall, 2),
           "attacked_examples_per_min": round(60 * ex / wall, 3),
           "mode": "cross-example batched chains (mcmc_batched), random.Random(123456 + index)"}
    if rank == 0 and world == 1 and seq_examples > 0:
        seq = run_mhm_attack(model, codes, subs, labels, args, indices=mine[:seq_examples],
                             max_iter=100, prob_threshold=1, max_inflight=1)
        res["sequential"] = {"examples": seq["examples"], "victim_queries": seq["queries"],
                             "wall_s": round(seq["wall_s"], 2),
                             "victim_queries_per_s": round(seq["queries"] / seq["wall_s"], 2)}
        res["batched_speedup"] = round(res["victim_queries_per_s"]
                                       / res["sequential"]["victim_queries_per_s"], 2)
    return res


def subs_leg(dev, seconds, rank, world, precision):
    """Config-3 workload: masked-LM substitute generation (get_substitutes.py) over the Devign
    fixture functions in order (12-layer codebert-shaped MLM, synthetic weights), items pulled
    from a shared queue until the time budget is spent."""
    from apmc_amd.dist import DynamicQueue
    from apmc_amd.engine import Engine
    from apmc_amd.host import Tokenizer
    from apmc_amd.substitutes import SubstituteGenerator
    from apmc_amd.weights import synthetic_state_dict

    eng = Engine(synthetic_state_dict(seed=0, head="none", with_mlm=True), head="none",
                 with_mlm=True, precision=precision, device=dev.index)
    gen = SubstituteGenerator(eng, Tokenizer(), block_size=512)
    codes = [json.loads(line)["func"] for line in
             open(ROOT / "data" / "devign" / "test_subs_0_400.jsonl")]
    gen.generate(codes[0])  # warm-up (workspaces, logits buffer)
    gen.stats = {k: 0 for k in gen.stats}
    queue = DynamicQueue(len(codes), key="bench_subs_queue", deadline=time.time() + seconds)
    if world > 1:
        import torch.distributed as dist
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    while True:
        i = queue()
        if i is None:
            break
        gen.generate(codes[i])
    torch.cuda.synchronize(dev)
    wall = time.perf_counter() - t0
    st = gen.stats
    v = np.array([st["examples"], st["occurrences"], st["encoded_seqs"], st["encoded_tokens"],
                  st["encoder_flop"], wall], dtype=np.float64)
    if world > 1:
        import torch.distributed as dist
        t = torch.tensor(v, device=dev)
        g = [torch.zeros_like(t) for _ in range(world)]
        dist.all_gather(g, t)
        allv = torch.stack(g).cpu().numpy()
    else:
        allv = v[None]
    tot = allv[:, :5].sum(0)
    wall = allv[:, 5].max()
    eng.close()
    return {"workload": "CodeBERT masked-LM substitute generation (get_substitutes.py: top-60, "
                        "60 re-encodes per identifier occurrence, cosine top-30, BPE perplexity), "
                        "test_subs_0_400 functions in order, block 512",
            "precision": precision, "items": int(tot[0]), "occurrences": int(tot[1]),
            "reencoded_sequences": int(tot[2]), "wall_s": round(wall, 2),
            "items_per_min": round(60 * tot[0] / wall, 2),
            "reencoded_sequences_per_s": round(tot[2] / wall, 1),
            "encoder_tflops": round(tot[4] / wall / 1e12, 2)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--seq", type=int, default=512)
    ap.add_argument("--precision", default="f32x3", choices=["fp32", "f32x3", "bf16"])
    ap.add_argument("--cpu-seconds", type=float, default=15.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--subs-seconds", type=float, default=30.0,
                    help="time budget of the substitute-generation leg (config 3; 0 disables)")
    ap.add_argument("--attack-seconds", type=float, default=90.0,
                    help="time budget of the end-to-end GA attack leg over test_subs_0_400 "
                         "(0 disables)")
    ap.add_argument("--mhm-examples", type=int, default=32,
                    help="examples of the batched MHM-NS leg (config 5 baseline; 0 disables)")
    ap.add_argument("--mhm-seq-examples", type=int, default=4,
                    help="examples of the sequential MHM-NS comparison run")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    if world > 1:
        import torch.distributed as dist
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device(f"cuda:{local}"))
    else:
        torch.cuda.set_device(0)
    dev = torch.device(f"cuda:{local if world > 1 else 0}")

    from apmc_amd.engine import Engine
    from apmc_amd.weights import synthetic_state_dict

    eng = Engine(synthetic_state_dict(seed=0, head="sigmoid1"), head="sigmoid1", num_labels=1,
                 precision=args.precision, device=dev.index)
    B, L = args.batch, args.seq
    rng = np.random.default_rng(0 + rank)
    ids = rng.integers(4, 50264, size=(B, L)).astype(np.int32)
    ids[:, 0], ids[:, -1] = 0, 2
    lens = np.full((B,), L, dtype=np.int32)
    ids_dev = torch.from_numpy(ids).to(dev)
    out = torch.empty((B, 1), dtype=torch.float32, device=dev)
    stream = torch.cuda.current_stream(dev)

    for _ in range(args.warmup):
        eng.score(ids_dev, lens, out=out)
    torch.cuda.synchronize(dev)
    eng.kernel_time()  # drop anything recorded so far
    eng.set_profiling("gemm_ffn1", True)

    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        eng.score(ids_dev, lens, out=out, stream=stream)
    torch.cuda.synchronize(dev)
    if dist is not None:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    eng.set_profiling("gemm_ffn1", False)
    k_ms, k_n, k_flop = eng.kernel_time()

    if dist is not None:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
        kt = torch.tensor([k_ms, float(k_n), k_flop], dtype=torch.float64, device=dev)
        dist.all_reduce(kt, op=dist.ReduceOp.SUM)
        k_ms, k_n, k_flop = float(kt[0]), int(kt[1]), float(kt[2])

    probs = out.cpu().numpy()[:, 0]
    total_q = world * args.steps * B
    value = total_q / elapsed
    per_launch_s = (k_ms / 1e3) / max(k_n, 1)
    achieved = (k_flop / max(k_n, 1)) / per_launch_s / 1e12 if k_n else None
    # roofline peak of the arithmetic the GEMMs run: f32 MFMA; bf16 MFMA; split-bf16 issues
    # 3 bf16 MFMAs per product, so its ceiling in algorithmic FLOP/s is the bf16 peak / 3
    peak = {"fp32": FP32_MFMA_PEAK_TFLOPS, "bf16": BF16_MFMA_PEAK_TFLOPS,
            "f32x3": BF16_MFMA_PEAK_TFLOPS / 3}[args.precision]
    parity = None
    if args.precision != "fp32" and rank == 0:
        # the split / bf16 numbers are only meaningful with their parity on this very batch
        ref_eng = Engine(synthetic_state_dict(seed=0, head="sigmoid1"), head="sigmoid1",
                         num_labels=1, precision="fp32", device=dev.index)
        ref = ref_eng.score(ids_dev, lens).cpu().numpy()[:, 0]
        ref_eng.close()
        parity = float(np.abs(out.cpu().numpy()[:, 0] - ref).max())
    res = {
        "metric": METRIC,
        "value": round(value, 3),
        "unit": "victim queries/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(1e3 * elapsed / args.steps, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": {"fp32": "fp32", "f32x3": "f32x3 (fp32 operands as bf16 hi+lo, 3 bf16 MFMAs "
                                           "per product, f32 accumulate; |dp| vs fp32 <= 1e-4)",
                  "bf16": "bf16 (f32 accumulate / residual)"}[args.precision],
        "precision_mode": args.precision,
        "max_abs_dprob_vs_fp32_mode": parity,
        "data": "synthetic (seeded RoBERTa-base weights; uniform token ids; no checkpoint offline)",
        "config": {"workload": "CodeBERT Devign victim scoring of one GA mutant population per "
                               "step (config 2 shape: eval_batch_size 64 x block 512)",
                   "global_batch": B * world, "seq_len": L, "parallelism": f"dp{world} (example shards)"},
        "roofline": {
            "bound": "mfma",
            "kernel": {"fp32": "gemm_f32_nt_kernel<EPI_BIAS_GELU>",
                       "f32x3": "gemm_pk_kernel<256, 2, EPI_GELU_PACKED>",
                       "bf16": "gemm_pk_kernel<256, 1, EPI_GELU_PACKED>"}[args.precision]
                      + " (FFN1 [T,768]x[768,3072])",
            "achieved": round(achieved, 3) if achieved else None,
            "peak": peak,
            "unit": "TFLOP/s",
            "frac": round(achieved / peak, 4) if achieved else None,
            "traffic": pmc_traffic_per_launch(args.precision),
            "launches": k_n,
            "avg_launch_us": round(per_launch_s * 1e6, 2),
            "flop_per_launch": (k_flop / k_n) if k_n else None,
        },
        "whole_step_tflops": round(flops_per_query(L) * total_q / elapsed / 1e12, 3),
        "whole_step_frac_of_peak": round(flops_per_query(L) * total_q / elapsed / 1e12 / world / peak, 4),
        "probs_checksum": float(np.round(probs.astype(np.float64).sum(), 6)),
    }
    if args.attack_seconds > 0:
        res["attack"] = attack_leg(dev, args.attack_seconds, rank, world, args.precision)
    if args.subs_seconds > 0:
        res["substitutes"] = subs_leg(dev, args.subs_seconds, rank, world, args.precision)
    if args.mhm_examples > 0:
        res["mhm"] = mhm_leg(dev, args.mhm_examples, args.mhm_seq_examples, rank, world,
                             args.precision)
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        threads = int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or min(16, os.cpu_count() or 1)
        res["cpu_baseline"] = cpu_baseline(L, args.cpu_seconds, threads)
        res["speedup_vs_cpu"] = round(value / res["cpu_baseline"]["value"], 2)
    if rank == 0:
        print(json.dumps(res), flush=True)
    eng.close()
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
