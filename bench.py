"""Benchmark of the victim-query hot path (BASELINE.json metric, config 2 workload shape).

A "step" = one Model.get_results-equivalent pass of the engine over one GA population batch of
synthetic mutants: B (=64, GA eval_batch_size, CodeXGLUE/Defect-detection/README.md:261) sequences
x L=512 tokens (no padding, CLS=0 / SEP=2, interior ids uniform in [4, 50263], seed 0+rank),
scored by the CodeBERT-shaped Devign victim (seeded synthetic weights: no checkpoint offline).
Inputs are resident in HBM before the timed region.  Per-GPU work is fixed (weak scaling): each
rank scores its own batches; there is no data-path collective.  The only collectives are the
barrier around the timed region and the MAX-reduction of the elapsed time.

`--gpus N` (N > 1) without torchrun's environment re-launches this script as N ranks through
`python -m torch.distributed.run` (a child process started before anything touches the GPU);
under torchrun (WORLD_SIZE set) every rank checks WORLD_SIZE == N and that RCCL sees N ranks.

Prints ONE JSON line (rank 0).  The engine runs the encoder as two half-batch streams (its
default); `roofline` is the dominant kernel (the FFN1 GEMM, [T,768]x[768,3072] + bias + GELU)
timed with HIP events on its launch stream (events created before the timed steps) in a
single-stream pass over the same batch right after the timed region, so that no other kernel
shares the CUs during a measured launch; `cpu_baseline` is oracle/roberta_cpu.py (PyTorch-CPU fp32 eager
restatement of the reference's scoring) on the host cores this job may use.  Sub-objects: the
exact-fp32 mode of the same step (`fp32_mode`), the bf16 mode as a bound diagnostic
(`bf16_mode`: one bf16 MFMA per product instead of three), the end-to-end config-2 GA attack over all of
test_subs_0_400 (`attack`), config 1 (greedy, 16 functions) on GPU and CPU (`config1`), masked-LM
substitute generation (`substitutes`), the MHM-NS baseline (`mhm`) and config 5 (`authorship`:
CodeBERT GA vs MHM-NS, GraphCodeBERT GA).
"""
import argparse
import glob
import json
import os
import pathlib
import random
import subprocess
import sys
import time

ROOT = pathlib.Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT))

FP32_MFMA_PEAK_TFLOPS = 157.3   # MI355X_MICROARCH.md: f32-input MFMA dense peak (spec)
BF16_MFMA_PEAK_TFLOPS = 2516.6  # dense bf16 (spec, no sparsity)
METRIC = "victim queries/sec + attacked examples/min (node), CodeBERT Devign GA attack"
FIXTURE = ROOT / "data" / "devign" / "test_subs_0_400.jsonl"
AA_FIXTURE = ROOT / "data" / "authorship" / "valid_subs.jsonl"
CLONE_FIXTURE = ROOT / "data" / "clone" / "test_subs_0_500.jsonl"
# attack-sensitive synthetic victim (the attack parity tests' weights): a larger classifier
# out_proj spreads probabilities so that substitutions can flip predictions
VICTIM_SEED, VICTIM_OUT_STD = 5, 8.0
COLL_DEV = None  # device of the collectives' tensors (main sets it: the rank's GPU, or host for gloo)


def parse_args():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--seq", type=int, default=512)
    ap.add_argument("--precision", default="f32x3", choices=["fp32", "f32x3", "bf16"])
    ap.add_argument("--cpu-seconds", type=float, default=12.0,
                    help="CPU scoring microbenchmark budget (cpu_baseline)")
    ap.add_argument("--cpu-e2e-seconds", type=float, default=60.0,
                    help="cap (s) of the CPU config-1 greedy attack (config1.cpu); all 16 "
                         "functions take ~9 min on 16 threads (tools/config1_cpu_full.py ran "
                         "them once on the GPU box's host: profiles/r4_config1_cpu_full.json, "
                         "compared as config1.cpu_full_run)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--attack-examples", type=int, default=400,
                    help="examples of test_subs_0_400 in the config-2 GA attack leg (0 disables)")
    ap.add_argument("--attack-deadline", type=float, default=420.0,
                    help="safety cap (s) of the attack leg; hitting it is reported")
    ap.add_argument("--attack-inflight", type=int, default=64,
                    help="examples whose attacks share each device batch")
    ap.add_argument("--subs-seconds", type=float, default=20.0,
                    help="time budget of the substitute-generation leg (config 3; 0 disables)")
    ap.add_argument("--mhm-examples", type=int, default=32,
                    help="examples of the batched MHM-NS leg (config 5 baseline; 0 disables)")
    ap.add_argument("--mhm-seq-examples", type=int, default=4,
                    help="examples of the sequential MHM-NS comparison run")
    ap.add_argument("--aa-examples", type=int, default=132,
                    help="authorship programs of the config-5 leg (GA vs MHM-NS; 0 disables)")
    ap.add_argument("--aa-gcb-examples", type=int, default=132,
                    help="of them, attacked by GA and MHM-NS on the GraphCodeBERT victim too (0 "
                         "disables; all 132 take ~80 s)")
    ap.add_argument("--clone-examples", type=int, default=32,
                    help="config-4 leg: GraphCodeBERT BigCloneBench pairs attacked (0 = skip; all "
                         "500 take ~9 min: profiles/r6a_config4_full_500.jsonl)")
    ap.add_argument("--no-config1", action="store_true", help="skip the config-1 leg")
    ap.add_argument("--no-microbench", action="store_true",
                    help="skip the SURVEY §8(d) microbenchmarks (batch 1024, varlen, GCB 640)")
    ap.add_argument("--no-fp32-mode", action="store_true")
    return ap.parse_args()


def log(msg):
    """Progress on stderr (the JSON line alone goes to stdout): a long default run keeps writing."""
    print(f"[bench {time.strftime('%H:%M:%S')}] {msg}", file=sys.stderr, flush=True)


class heartbeat:
    """`with heartbeat("leg"):` logs every `every` s while a long leg runs (a full-fixture config-4
    leg runs ~10 min with no other output, and a silent GPU command reads as hung)."""

    def __init__(self, what, every=45.0):
        import threading
        self.what, self.every, self.stop = what, every, threading.Event()
        self.thread = threading.Thread(target=self._run, daemon=True)

    def _run(self):
        t0 = time.time()
        while not self.stop.wait(self.every):
            log(f"{self.what}: running, {time.time() - t0:.0f} s")

    def __enter__(self):
        self.thread.start()
        return self

    def __exit__(self, *exc):
        self.stop.set()
        self.thread.join()
        return False


def rank_thread_budget(ranks, env=None):
    """Host threads of one rank when `ranks` ranks share this host: the CPUs of this process's
    affinity divided by the ranks, 1..16 (the featurisers' cap, host.gcb_threads), unless the
    user set APMC_HOST_THREADS.  Every rank runs the host side of its attacks (mutant builder,
    tokenizer, GCB featuriser threads) and its torch CPU ops on this many threads, so N ranks
    never oversubscribe the host (torch.distributed.run alone would leave each rank at
    OMP_NUM_THREADS=1 and the featurisers at the whole affinity each)."""
    env = os.environ if env is None else env
    if env.get("APMC_HOST_THREADS"):
        return max(1, int(env["APMC_HOST_THREADS"]))
    try:
        cpus = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        cpus = os.cpu_count() or 1
    return max(1, min(16, cpus // max(1, ranks)))


def relaunch_env(gpus, env=None):
    """Environment of the N ranks relaunch_as_ranks starts: the dmabuf IPC mode RCCL needs on
    this pool and each rank's host thread budget (rank_thread_budget) as OMP_NUM_THREADS and
    APMC_HOST_THREADS."""
    env = dict(os.environ if env is None else env)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    t = rank_thread_budget(gpus, env)
    env["OMP_NUM_THREADS"] = str(t)
    env["APMC_HOST_THREADS"] = str(t)
    return env


def relaunch_as_ranks(args):
    """--gpus N outside torchrun: run N ranks via torch.distributed.run as a child process
    (started before this process touches the GPU) and exit with its status."""
    port = 29000 + (os.getpid() % 2000)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
           f"--nproc-per-node={args.gpus}", "--master-addr", "127.0.0.1",
           f"--master-port={port}", str(pathlib.Path(__file__).resolve())] + sys.argv[1:]
    return subprocess.call(cmd, env=relaunch_env(args.gpus))


def executed_flops_per_query(L, C=1):
    """FLOP the engine executes per query of L tokens: 11 full layers, then the last layer for
    the CLS row only (engine.hip run_encoder, cls_attention.hip): its query, u = W_k^T q per head,
    scores and the p-weighted row sum over the L layer-input rows, W_v of that sum, the O
    projection and the FFN — no K / V projection of the L rows — then the head."""
    H, F, NH, D = 768, 3072, 12, 64
    per_tok = 2 * (4 * H * H + 2 * H * F)
    full = 11 * (L * per_tok + 4 * L * L * H)
    last = 2 * H * H + 2 * NH * D * H + 4 * L * H * NH + 2 * NH * H * D + 2 * H * H + 4 * H * F
    return full + last + 2 * H * H + 2 * H * C


def flops_per_query(L, C=1):
    """SURVEY §8(d) algorithmic F(L) (12 full layers)."""
    per_tok = 2 * (4 * 768 * 768 + 2 * 768 * 3072)
    return 12 * (L * per_tok + 4 * L * L * 768) + 2 * 768 * 768 + 2 * 768 * C


def pmc_traffic_per_launch(precision):
    """HBM bytes per FFN1 launch of this precision's kernel from the committed rocprofv3 PMC
    summary (profiles/*pmc*ffn1*.json, newest round first), or None."""
    import re

    def order(f):  # r<round><letters>_...: r3z < r3aa < r3ap (round, then run letters)
        m = re.match(r"r(\d+)([a-z]*)_", pathlib.Path(f).name)
        return (int(m.group(1)), len(m.group(2)), m.group(2)) if m else (-1, 0, "")
    for f in sorted(glob.glob(str(ROOT / "profiles" / "*pmc*ffn1*.json")), key=order,
                    reverse=True):
        try:
            d = json.load(open(f))
            if d.get("precision", "fp32") == precision:
                return float(d["hbm_bytes_per_launch"])
        except Exception:
            continue
    return None


def host_cores():
    """CPU threads for the CPU reference path: one per PHYSICAL core this process may run on
    (its sched affinity mapped through sysfs topology, so SMT siblings count once).  Returns
    (threads, facts) — facts states the affinity, the physical cores behind it and the host's
    physical cores, so the line says exactly what was used."""
    aff = sorted(os.sched_getaffinity(0))

    def core_of(c):
        base = f"/sys/devices/system/cpu/cpu{c}/topology/"
        try:
            return (open(base + "physical_package_id").read().strip(),
                    open(base + "core_id").read().strip())
        except OSError:
            return ("?", str(c))
    mine = {core_of(c) for c in aff}
    host = set()
    for d in glob.glob("/sys/devices/system/cpu/cpu[0-9]*"):
        host.add(core_of(int(d.rsplit("cpu", 1)[1])))
    threads = max(1, len(mine))
    return threads, {"affinity_cpus": len(aff), "physical_cores_in_affinity": len(mine),
                     "host_physical_cores": len(host) or None,
                     "job_share_threads": int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or None}


# ------------------------------------------------------------------------------------------ legs
def single_stream_engine(sd, precision, dev):
    """An engine with the encoder on one stream (ae_config.streams = AE_STREAMS_ONE): the kernels
    a profiled pass times then run with nothing beside them."""
    from apmc_amd.engine import Engine

    return Engine(sd, head="sigmoid1", num_labels=1, precision=precision, device=dev.index,
                  streams="one")


def attention_summary(a_ms, a_n, steps, B, L, peak, where):
    """Attention of the 11 full-length layers (4·L²·64 FLOP per (sequence, head): S = QKᵀ and
    PV) over the time of every attention launch of the step, the CLS-only last layer's included
    (conservative)."""
    if not a_n:
        return None
    per_layer_flop = 4.0 * L * L * 64 * 12 * B
    attn_ms = a_ms / steps
    tf = 11 * per_layer_flop / attn_ms / 1e9
    return {"ms_per_step": round(attn_ms, 4), "launches_per_step": a_n // steps,
            "full_layer_algorithmic_gflop": round(per_layer_flop / 1e9, 2),
            "algorithmic_tflops": round(tf, 2), "frac_of_peak": round(tf / peak, 4),
            "timing": "HIP events on the launch stream around every attention launch (11 full "
                      "layers + the CLS-only last layer), " + where}


def time_steps(eng, ids_dev, lens, out, steps, warmup, dev, dist, profile, kind="gemm_ffn1"):
    import torch

    stream = torch.cuda.current_stream(dev)
    for _ in range(warmup):
        eng.score(ids_dev, lens, out=out, stream=stream)
    torch.cuda.synchronize(dev)
    if profile:
        eng.kernel_time()  # drop anything recorded so far
        eng.set_profiling(kind, True)  # events are created here, before the timed region
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(steps):
        eng.score(ids_dev, lens, out=out, stream=stream)
    torch.cuda.synchronize(dev)
    if dist is not None:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    kt = None
    if profile:
        eng.set_profiling(kind, False)
        kt = eng.kernel_time()
    return elapsed, kt


def cpu_baseline(L, seconds, threads, impl="oracle"):
    """The reference's CPU path on the scoring step over [64, L] batches — the DataLoader batch of
    model.py:40 — on `threads` torch threads; whole batches until `seconds` have passed.
    impl "oracle": oracle/roberta_cpu.py (PyTorch-CPU fp32 eager restatement of Model.get_results'
    forward); "hf": the installed transformers RobertaForSequenceClassification (the library the
    reference's Model.forward calls, model.py:25), built from a local config (eager attention,
    fp32) with the same synthetic weights, called as the reference does:
    sigmoid(model(ids, attention_mask=ids.ne(1))[0])."""
    import numpy as np
    import torch

    from apmc_amd.weights import synthetic_state_dict

    torch.set_num_threads(threads)
    sd = synthetic_state_dict(seed=0, head="sigmoid1")
    rng = np.random.default_rng(0)
    B = 64
    ids = rng.integers(4, 50264, size=(B, L)).astype(np.int64)
    ids[:, 0], ids[:, -1] = 0, 2
    if impl == "hf":
        from apmc_amd.weights import to_hf_state_dict
        from transformers import RobertaConfig, RobertaForSequenceClassification

        c = RobertaConfig(vocab_size=50265, hidden_size=768, num_hidden_layers=12,
                          num_attention_heads=12, intermediate_size=3072,
                          max_position_embeddings=514, type_vocab_size=1, pad_token_id=1,
                          bos_token_id=0, eos_token_id=2, layer_norm_eps=1e-5, num_labels=1,
                          hidden_act="gelu", hidden_dropout_prob=0.0,
                          attention_probs_dropout_prob=0.0)
        c._attn_implementation = "eager"
        m = RobertaForSequenceClassification(c).eval()
        m.load_state_dict(to_hf_state_dict(sd, "seqcls"), strict=False)

        @torch.no_grad()
        def run(x):
            t = torch.from_numpy(x)
            return torch.sigmoid(m(t, attention_mask=t.ne(1))[0]).numpy()
    else:
        from oracle import roberta_cpu as ora

        def run(x):
            return ora.score(sd, x, "sigmoid1")
    run(ids[:2, :64])  # warm up allocator / threads
    done, t0 = 0, time.perf_counter()
    while True:
        run(ids)
        done += B
        el = time.perf_counter() - t0
        log(f"CPU baseline ({impl}): {done} queries in {el:.1f} s ({threads} threads)")
        if el >= seconds:
            break
    return done / el, f"{done} queries of L={L} (batches of {B}, model.py:40) in {el:.1f} s"


def cpu_victim(threads):
    """The CPU reference path of config 1: oracle/roberta_cpu.py (PyTorch-CPU fp32 eager, the
    reference's padded [n, 512] batches with the key-padding mask) behind the request API."""
    import numpy as np
    import torch

    from apmc_amd.model import HostIdsVictim
    from apmc_amd.weights import synthetic_state_dict
    from oracle import roberta_cpu as ora

    torch.set_num_threads(threads)
    sd = synthetic_state_dict(seed=VICTIM_SEED, head="sigmoid1", out_std=VICTIM_OUT_STD)

    state = {"deadline": None, "scored": 0, "t0": time.time()}

    def score(ids):
        out = []
        for s in range(0, ids.shape[0], 64):  # model.py:40 DataLoader batch_size = eval_batch_size
            if state["deadline"] is not None and time.time() > state["deadline"]:
                raise TimeoutError  # bounded sample: stop at the next batch past the budget
            out.append(ora.score(sd, ids[s:s + 64], "sigmoid1"))
            state["scored"] += out[-1].shape[0]
            el = time.time() - state["t0"]
            log(f"config-1 CPU: {state['scored']} queries in {el:.0f} s "
                f"({state['scored'] / el:.2f} q/s, {threads} threads)")
        return np.concatenate(out)

    v = HostIdsVictim(score)
    v.state = state
    return v


def greedy_run(model, codes, subs, labels, indices):
    """Config 1: gi_attack.py without --use_ga (greedy only), sequential reference loop.  A
    victim with a `state` dict (the CPU path) may stop the loop at its deadline; queries are then
    the rows it actually scored."""
    from apmc_amd.drivers import AttackArgs, run_gi_attack

    args = AttackArgs(block_size=512, eval_batch_size=64, use_ga=False, seed=123456,
                      rng="per_example")
    q0 = model.query
    done = []
    t0 = time.time()
    try:
        run_gi_attack(model, codes, subs, labels, args, indices=indices, log=done.append)
    except TimeoutError:
        pass
    wall = time.time() - t0
    st = getattr(model, "state", None)
    return dict(examples=len(done), queries=st["scored"] if st else model.query - q0, wall_s=wall,
                successes=sum(r["is_success"] == 1 for r in done), records=done)


def config1_leg(dev, precision, threads, cpu_seconds):
    """Config 1 (BASELINE configs[0]): greedy attack on the first 16 test_subs_0_400 functions at
    block 512 — on the GPU engine end to end, and on the CPU reference path (host featurisation +
    oracle scoring) over a bounded prefix of the same loop."""
    from apmc_amd.drivers import load_fixture
    from apmc_amd.model import Model
    from apmc_amd.weights import synthetic_state_dict

    codes, subs, labels = load_fixture(FIXTURE, 0, 16)
    model = Model(synthetic_state_dict(seed=VICTIM_SEED, head="sigmoid1", out_std=VICTIM_OUT_STD),
                  task="devign", precision=precision, device=dev.index)
    g = greedy_run(model, codes, subs, labels, list(range(16)))
    model.engine.close()
    res = {"workload": "CodeBERT Devign greedy attack (gi_attack.py without --use_ga), "
                       "test_subs_0_400 functions [0, 16), block 512, eval_batch_size 64",
           "gpu": {"precision": precision, "examples": g["examples"], "queries": g["queries"],
                   "successes": g["successes"], "wall_s": round(g["wall_s"], 2),
                   "victim_queries_per_s": round(g["queries"] / g["wall_s"], 1)}}
    full = sorted(glob.glob(str(ROOT / "profiles" / "*config1_cpu_full*.json")))
    if full:
        # the CPU path run to completion outside the bench (tools/config1_cpu_full.py): its
        # per-function outcome / query count / adversarial-code hash against this GPU run's
        from tools.config1_cpu_full import record_key
        rec = json.load(open(full[-1]))
        mine = [record_key(r) for r in g["records"]]
        res["cpu_full_run"] = {k: rec[k] for k in ("kind", "cores", "host", "cpu_count",
                                                   "examples_completed", "complete", "queries",
                                                   "successes", "wall_s", "victim_queries_per_s")
                               if k in rec}
        res["cpu_full_run"]["record"] = "profiles/" + pathlib.Path(full[-1]).name
        res["cpu_full_run"]["same_outcome_as_gpu"] = sum(a == b for a, b in zip(mine, rec["records"]))
    if cpu_seconds > 0:
        import torch
        host_threads = torch.get_num_threads()
        cv = cpu_victim(threads)
        cv.state["deadline"] = time.time() + cpu_seconds
        cv.state["t0"] = time.time()
        c = greedy_run(cv, codes, subs, labels, list(range(16)))
        res["cpu"] = {"kind": "port", "cores": threads, "examples_completed": c["examples"],
                      "complete": c["examples"] == 16,
                      "queries": c["queries"], "wall_s": round(c["wall_s"], 2),
                      "victim_queries_per_s": round(c["queries"] / c["wall_s"], 3),
                      "sample": f"the same greedy loop (host featurisation + oracle/roberta_cpu.py "
                                f"fp32 eager scoring of padded 512-id rows in batches of 64, "
                                f"torch threads={threads}, one per physical core of the "
                                f"process's affinity), all 16 functions unless the "
                                f"{cpu_seconds:.0f} s cap stops it at the first batch past it"}
        key = lambda r: (r["is_success"], r["queries"], r.get("adv_code"))  # noqa: E731
        res["cpu"]["same_outcome_as_gpu"] = sum(key(a) == key(b) for a, b in
                                                zip(g["records"], c["records"]))
        torch.set_num_threads(host_threads)
        res["gpu_vs_cpu_queries_per_s"] = round(res["gpu"]["victim_queries_per_s"]
                                                / max(res["cpu"]["victim_queries_per_s"], 1e-9), 1)
    return res


def attack_leg(dev, n_examples, deadline_s, inflight, rank, world, precision):
    """End-to-end config-2 workload: greedy -> GA attack (gi_attack.py --use_ga) over the first
    `n_examples` of test_subs_0_400, block 512, eval_batch_size 64, with cross-example batching;
    ranks pull examples from one shared queue (dist.run_sharded_gi_batched)."""
    from apmc_amd.dist import run_sharded_gi_batched
    from apmc_amd.drivers import AttackArgs, load_fixture
    from apmc_amd.model import Model
    from apmc_amd.weights import synthetic_state_dict

    codes, subs, labels = load_fixture(FIXTURE, 0, n_examples)
    model = Model(synthetic_state_dict(seed=VICTIM_SEED, head="sigmoid1", out_std=VICTIM_OUT_STD),
                  task="devign", precision=precision, device=dev.index)
    args = AttackArgs(block_size=512, eval_batch_size=64, seed=123456, rng="per_example")
    _, t = run_sharded_gi_batched(model, codes, subs, labels, args, max_inflight=inflight,
                                  device=dev, deadline=time.time() + deadline_s,
                                  key="bench_attack_queue")
    tokens = model.tokens
    model.engine.close()
    wall = t["wall_s"]
    return {"workload": "CodeBERT Devign greedy->GA attack (gi_attack --use_ga), "
                        f"test_subs_0_400.jsonl examples [0, {n_examples}), block 512, "
                        "eval_batch_size 64, attack-sensitive synthetic victim "
                        f"(seed {VICTIM_SEED}, out_proj std {VICTIM_OUT_STD})",
            "precision": precision,
            "examples": t["examples"], "complete": t["examples"] == n_examples,
            "correctly_classified": t["total_cnt"], "successes": t["success"],
            "success_rate": round(t["success_rate"], 4) if t["total_cnt"] else None,
            "ga_runs": t["ga_runs"], "ga_successes": t["ga_successes"],
            "victim_queries": t["queries"], "wall_s": round(wall, 2),
            "victim_queries_per_s": round(t["queries"] / wall, 2),
            "attacked_examples_per_min": round(60 * t["examples"] / wall, 3),
            # scored non-pad tokens (this rank's victim): the device-side work rate, comparable
            # with the microbench varlen leg's tokens / s
            "tokens_scored": tokens,
            "tokens_per_s": round(tokens / wall, 1) if tokens else None,
            "mean_tokens_per_query": round(tokens / t["queries"], 1) if t["queries"] else None,
            "per_rank": t["per_rank"],
            "rng": "random.Random(123456 + index) per example",
            "batching": f"cross-example: up to {inflight} examples' requests per device batch",
            "sharding": "dynamic queue (torch.distributed store counter)"}


def mhm_leg(dev, n_examples, seq_examples, rank, world, precision):
    """Config-5 baseline workload: MHM-NS (mhm_attack.py, n_candi 30, max_iter 100, threshold 1)
    over test_subs_0_400 with the CodeBERT Devign victim.  Batched: the first `n_examples` fixture
    examples pulled from one queue shared by the ranks (dist.run_sharded_mhm), every chain a
    rank holds in flight at once; sequential: the reference loop (one <=31-candidate batch per
    query round) over the first `seq_examples` of them, for the comparison (rank 0, N=1 only)."""
    from apmc_amd.dist import run_sharded_mhm
    from apmc_amd.drivers import AttackArgs, load_fixture, run_mhm_attack
    from apmc_amd.model import Model
    from apmc_amd.weights import synthetic_state_dict

    codes, subs, labels = load_fixture(FIXTURE)
    model = Model(synthetic_state_dict(seed=VICTIM_SEED, head="sigmoid1", out_std=VICTIM_OUT_STD),
                  task="devign", precision=precision, device=dev.index)
    args = AttackArgs(block_size=512, eval_batch_size=64, seed=123456)
    _, t = run_sharded_mhm(model, codes, subs, labels, args, max_iter=100, prob_threshold=1,
                           max_inflight=64, device=dev, n=n_examples, key="bench_mhm_queue")
    wall = t["wall_s"]
    res = {"workload": "MHM-NS (mhm_attack.py: n_candi 30, max_iter 100) CodeBERT Devign victim, "
                       f"test_subs_0_400 examples [0, {n_examples}), block 512",
           "precision": precision, "examples": t["examples"],
           "correctly_classified": t["total_cnt"], "successes": t["success"],
           "success_rate": round(t["success_rate"], 4) if t["total_cnt"] else None,
           "victim_queries": t["queries"], "wall_s": round(wall, 2),
           "victim_queries_per_s": round(t["queries"] / wall, 2),
           "attacked_examples_per_min": round(60 * t["examples"] / wall, 3),
           "per_rank": t["per_rank"],
           "mode": "cross-example batched chains (up to 64 per device batch), "
                   "random.Random(123456 + index), dynamic queue"}
    if rank == 0 and world == 1 and seq_examples > 0:
        seq = run_mhm_attack(model, codes, subs, labels, args, indices=range(seq_examples),
                             max_iter=100, prob_threshold=1, max_inflight=1)
        res["sequential"] = {"examples": seq["examples"], "victim_queries": seq["queries"],
                             "wall_s": round(seq["wall_s"], 2),
                             "victim_queries_per_s": round(seq["queries"] / seq["wall_s"], 2)}
        res["batched_speedup"] = round(res["victim_queries_per_s"]
                                       / res["sequential"]["victim_queries_per_s"], 2)
    model.engine.close()
    return res


def _summary(t):
    wall = t["wall_s"]
    return {"examples": t["examples"], "attacked": t["total_cnt"], "successes": t["success"],
            "success_rate": round(t["success_rate"], 4) if t["total_cnt"] else None,
            "victim_queries": t["queries"], "wall_s": round(wall, 2),
            "victim_queries_per_s": round(t["queries"] / wall, 1) if wall else None,
            "attacked_examples_per_min": round(60 * t["examples"] / wall, 2) if wall else None,
            "per_rank": t["per_rank"]}


def aa_leg(dev, n_examples, n_gcb, rank, world, precision):
    """Config 5 (Authorship-Attribution, 66 classes): the ALERT greedy->GA attack
    (CodeXGLUE/Authorship-Attribution/code/attack.py: block 512, eval_batch_size 32) against the
    MHM-NS sampling baseline (mhm.py: n_candi 30, max_iter 100, eval_batch_size 64) on the same
    CodeBERT victim and programs of valid_subs.jsonl, then the GraphCodeBERT victim's GA and
    MHM-NS (GraphCodeBERT/Authorship-Attribution gi_attack.py / mhm_attack.py, code_length 512 +
    data_flow_length 128) on the first n_gcb programs.  Synthetic victims (seed 5, out_proj std 8) do not know the authors, so each
    program's label is the victim's own prediction (every program is attacked).  Each half pulls
    its programs from one queue shared by the ranks."""
    from apmc_amd.dist import run_sharded_gi_batched, run_sharded_mhm
    from apmc_amd.drivers import AttackArgs, _example, load_fixture
    from apmc_amd.graph import GraphModel
    from apmc_amd.host import Tokenizer
    from apmc_amd.model import Model
    from apmc_amd.weights import synthetic_state_dict

    codes, subs, _ = load_fixture(AA_FIXTURE, 0, n_examples)
    tok = Tokenizer()
    sd = synthetic_state_dict(seed=VICTIM_SEED, head="softmaxN", num_labels=66,
                              out_std=VICTIM_OUT_STD)
    model = Model(sd, task="authorship", precision=precision, device=dev.index)
    labels = [int(p) for p in model.get_results(
        [_example(tok, c, 0, 512, "authorship") for c in codes])[1]]
    res = {"workload": f"Authorship-Attribution valid_subs.jsonl programs [0, {len(codes)}), "
                       "66-way CodeBERT victim (synthetic, labels = its own predictions)",
           "precision": precision}
    args = AttackArgs(block_size=512, eval_batch_size=32, seed=123456, rng="per_example",
                      task="authorship")
    _, t = run_sharded_gi_batched(model, codes, subs, labels, args, max_inflight=64, device=dev,
                                  key="bench_aa_ga_queue")
    res["ga"] = dict(_summary(t), mode="greedy -> GA (attack.py), cross-example batched")
    log("authorship leg: MHM-NS")
    margs = AttackArgs(block_size=512, eval_batch_size=64, seed=123456, task="authorship")
    _, t = run_sharded_mhm(model, codes, subs, labels, margs, max_iter=100, prob_threshold=1,
                           max_inflight=128, device=dev, key="bench_aa_mhm_queue")
    res["mhm"] = dict(_summary(t), mode="MHM-NS (mhm.py), cross-example batched chains")
    model.engine.close()
    if n_gcb > 0:
        log("authorship leg: GraphCodeBERT GA")
        gargs = AttackArgs(block_size=512, eval_batch_size=32, seed=123456, rng="per_example",
                           task="gcb_authorship", code_length=512, data_flow_length=128)
        gmodel = GraphModel(sd, task="authorship", args=gargs, precision=precision,
                            device=dev.index)
        gcodes, gsubs = codes[:n_gcb], subs[:n_gcb]
        glabels = [int(gmodel.get_results([_example(tok, c, 0, 512, "gcb_authorship", gargs)])[1][0])
                   for c in gcodes]
        _, t = run_sharded_gi_batched(gmodel, gcodes, gsubs, glabels, gargs, max_inflight=64,
                                      device=dev, key="bench_aa_gcb_queue")
        res["gcb_ga"] = dict(_summary(t),
                             mode="GraphCodeBERT victim, greedy -> GA (GraphAuthorshipAttacker), "
                                  f"programs [0, {len(gcodes)}), L = 640 with the data-flow mask")
        log("authorship leg: GraphCodeBERT MHM-NS")
        margs = AttackArgs(block_size=512, eval_batch_size=64, seed=123456, task="gcb_authorship",
                           code_length=512, data_flow_length=128)
        _, t = run_sharded_mhm(gmodel, gcodes, gsubs, glabels, margs, max_iter=100,
                               prob_threshold=1, max_inflight=128, device=dev,
                               key="bench_aa_gcb_mhm_queue")
        res["gcb_mhm"] = dict(_summary(t),
                              mode="GraphCodeBERT victim, MHM-NS (GraphAuthorshipMHM_Attacker, "
                                   "mhm_attack.py: n_candi 30, max_iter 100, threshold 1), "
                                   f"programs [0, {len(gcodes)}), cross-example batched chains")
        gmodel.engine.close()
    return res


def clone_leg(dev, n_examples, rank, world, precision):
    """Config 4: the GraphCodeBERT BigCloneBench pair attack (GraphCodeBERT/clonedetection/code/
    attack.py with README's --code_length 512 --data_flow_length 128 --eval_batch_size 32):
    greedy -> GA on code1 of each pair, both codes through the graph forward at L = 640 with the
    data-flow mask, the pair head over [code1 | code2] CLS rows.  Synthetic victim (seed 5,
    out_proj std 8); labels are its own predictions, so every pair is attacked."""
    from apmc_amd.dist import run_sharded_gi_batched
    from apmc_amd.drivers import AttackArgs, _example, load_fixture
    from apmc_amd.graph import GraphModel
    from apmc_amd.host import Tokenizer
    from apmc_amd.weights import synthetic_state_dict

    codes, subs, _ = load_fixture(CLONE_FIXTURE, 0, n_examples)
    tok = Tokenizer()
    sd = synthetic_state_dict(seed=VICTIM_SEED, head="pair2", num_labels=2, out_std=VICTIM_OUT_STD)
    gargs = AttackArgs(block_size=512, eval_batch_size=32, seed=123456, rng="per_example",
                       task="gcb_clone", code_length=512, data_flow_length=128)
    gmodel = GraphModel(sd, task="clone", args=gargs, precision=precision, device=dev.index)
    labels = [int(gmodel.get_results([_example(tok, c, 0, 512, "gcb_clone", gargs)])[1][0])
              for c in codes]
    _, t = run_sharded_gi_batched(gmodel, codes, subs, labels, gargs, max_inflight=64,
                                  device=dev, key="bench_clone_gcb_queue")
    gmodel.engine.close()
    out = _summary(t)
    out["sequences_per_s"] = round(2 * t["queries"] / t["wall_s"], 1) if t["wall_s"] else None
    return dict({"workload": f"GraphCodeBERT BigCloneBench pairs test_subs_0_500.jsonl "
                             f"[0, {len(codes)}), greedy -> GA on code1, code_length 512 + "
                             "data_flow_length 128 per code, pair head (synthetic victim, "
                             "labels = its own predictions)",
                 "precision": precision}, **out,
                batching="cross-example: up to 64 pairs' requests per device batch")


def subs_leg(dev, seconds, rank, world, precision):
    """Config-3 workload: masked-LM substitute generation (get_substitutes.py) over the Devign
    fixture functions in order (12-layer codebert-shaped MLM, synthetic weights), items pulled
    from a shared queue until the time budget is spent."""
    import numpy as np
    import torch

    from apmc_amd.dist import DynamicQueue, call_key
    from apmc_amd.engine import Engine
    from apmc_amd.host import Tokenizer
    from apmc_amd.substitutes import SubstituteGenerator
    from apmc_amd.weights import synthetic_state_dict

    eng = Engine(synthetic_state_dict(seed=0, head="none", with_mlm=True), head="none",
                 with_mlm=True, precision=precision, device=dev.index)
    gen = SubstituteGenerator(eng, Tokenizer(), block_size=512)
    codes = [json.loads(line)["func"] for line in open(FIXTURE)]
    gen.generate(codes[0])  # warm-up (workspaces, logits buffer)
    gen.stats = {k: 0 for k in gen.stats}
    queue = DynamicQueue(len(codes), key=call_key("bench_subs_queue"),
                         deadline=time.time() + seconds)
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
        t = torch.tensor(v, device=COLL_DEV)
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


def devign_lengths():
    """Sub-word lengths (CLS + tokens[:510] + SEP) of the 2,732 Devign test functions of the seven
    fixture files — the varlen mix of SURVEY §8(d) is resampled from this distribution."""
    from apmc_amd.host import Tokenizer

    tok = Tokenizer()
    codes = []
    for f in sorted(glob.glob(str(ROOT / "data" / "devign" / "test_subs_*.jsonl"))):
        codes += [json.loads(line)["func"] for line in open(f)]
    _, lens = tok.featurize(codes, 512)
    return lens


def synthetic_gcb_batch(B, code_len=512, nodes=128, seed=0):
    """SURVEY §8(d) GraphCodeBERT step input: L = code_len + nodes = 640 with every position used
    (CLS + 510 code tokens + SEP, then `nodes` data-flow nodes, id <unk> at position 0), each node
    spanning 1-3 code tokens and with 1-2 edges to other nodes (seed 0); the reference's mask
    (utils.py:540-576, graph.graph_mask) bit-packed."""
    import numpy as np

    from apmc_amd.graph import graph_mask, pack_mask

    rng = np.random.default_rng(seed)
    L = code_len + nodes
    ids = np.empty((B, L), np.int32)
    pos = np.empty((B, L), np.int32)
    bits = np.empty((B, L, L // 32), np.int32)
    for b in range(B):
        ids[b, 0], ids[b, code_len - 1] = 0, 2
        ids[b, 1:code_len - 1] = rng.integers(4, 50264, code_len - 2)
        ids[b, code_len:] = 3
        pos[b, :code_len] = np.arange(2, code_len + 2)
        pos[b, code_len:] = 0
        starts = rng.integers(1, code_len - 4, nodes)
        d2c = [(int(s), int(s + rng.integers(1, 4))) for s in starts]
        d2d = [sorted({int(x) for x in rng.integers(0, nodes, rng.integers(1, 3))})
               for _ in range(nodes)]
        bits[b] = pack_mask(graph_mask(ids[b], pos[b], d2c, d2d, L))
    return ids, pos, bits


def microbench_leg(dev, precision, steps, warmup, world):
    """SURVEY §8(d)'s scoring microbenchmarks beside the headline shape, on the same synthetic
    victim and precision: batch 1024 x 512 (several examples' populations in flight), the
    Devign varlen mix (B = 64, lengths resampled from the fixture distribution, pads skipped),
    and the GraphCodeBERT step (B = 64 x L = 640 with the data-flow mask, node averaging,
    explicit positions).  Each: HIP-event-free wall time of `steps` batches bracketed by device
    syncs, victim queries/s, algorithmic TFLOP/s of F(L) per row and its fraction
    of the arithmetic's ceiling."""
    import numpy as np
    import torch

    from apmc_amd.engine import Engine
    from apmc_amd.weights import synthetic_state_dict

    peak = {"fp32": FP32_MFMA_PEAK_TFLOPS, "bf16": BF16_MFMA_PEAK_TFLOPS,
            "f32x3": BF16_MFMA_PEAK_TFLOPS / 3}[precision]
    sd = synthetic_state_dict(seed=0, head="sigmoid1")
    eng = Engine(sd, head="sigmoid1", num_labels=1, precision=precision, device=dev.index)
    out = {}

    def timed(fn, n_steps, kind=None, on=None):
        on = on or eng
        for _ in range(warmup):
            fn()
        torch.cuda.synchronize(dev)
        if kind:
            on.kernel_time()
            on.set_profiling(kind, True)
        t0 = time.perf_counter()
        for _ in range(n_steps):
            fn()
        torch.cuda.synchronize(dev)
        el = time.perf_counter() - t0
        kt = None
        if kind:
            on.set_profiling(kind, False)
            kt = on.kernel_time()
        return el, kt

    def summary(rows_flop, rows, el, n_steps, what):
        tf = rows_flop * n_steps / el / 1e12
        return {"workload": what, "steps": n_steps, "ms_per_step": round(1e3 * el / n_steps, 3),
                "victim_queries_per_s": round(rows * n_steps / el, 1),
                "algorithmic_tflops": round(tf, 2), "frac_of_peak": round(tf / peak, 4),
                "peak_tflops": peak}

    rng = np.random.default_rng(0)
    # (1) batch 1024 x 512
    B, L = 1024, 512
    ids = rng.integers(4, 50264, size=(B, L)).astype(np.int32)
    ids[:, 0], ids[:, -1] = 0, 2
    ids_d = torch.from_numpy(ids).to(dev)
    lens = np.full((B,), L, np.int32)
    o = torch.empty((B, 1), dtype=torch.float32, device=dev)
    n1 = max(3, steps // 4)
    el, _ = timed(lambda: eng.score(ids_d, lens, out=o), n1)
    out["batch1024"] = summary(flops_per_query(L) * B, B, el, n1,
                               "B = 1024 x L = 512 uniform ids (16 GA populations in flight)")
    log(f"microbench batch 1024: {out['batch1024']['victim_queries_per_s']} q/s")
    # (2) Devign varlen mix: 8 batches of 64 resampled lengths, cycled
    dl = devign_lengths()
    batches = []
    for _ in range(8):
        ln = rng.choice(dl, 64).astype(np.int32)
        x = np.full((64, 512), 1, np.int32)
        for i, n in enumerate(ln):
            x[i, 0], x[i, n - 1] = 0, 2
            x[i, 1:n - 1] = rng.integers(4, 50264, n - 2)
        batches.append((torch.from_numpy(x).to(dev), ln))
    ov = torch.empty((64, 1), dtype=torch.float32, device=dev)
    it = iter(range(1 << 30))
    el, _ = timed(lambda: eng.score(*batches[next(it) % 8], out=ov), steps)
    flop = np.mean([sum(flops_per_query(int(n)) for n in ln) for _, ln in batches])
    tok = np.mean([int(ln.sum()) for _, ln in batches])
    out["varlen"] = dict(summary(flop, 64, el, steps,
                                 "B = 64, lengths resampled (seed 0) from the 2,732 Devign test "
                                 "functions' sub-word lengths (truncated at 512), pads skipped"),
                         mean_tokens_per_row=round(tok / 64, 1),
                         fixture_median_len=int(np.median(dl)),
                         fixture_frac_over_400=round(float((dl > 400).mean()), 3))
    log(f"microbench varlen: {out['varlen']['victim_queries_per_s']} q/s")
    # (3) GraphCodeBERT L = 640 with the data-flow mask
    gi, gp, gb = synthetic_gcb_batch(64)
    gi_d, gp_d, gb_d = (torch.from_numpy(a).to(dev) for a in (gi, gp, gb))
    glens = np.full((64,), 640, np.int32)
    el, _ = timed(lambda: eng.score_graph(gi_d, glens, gp_d, gb_d, out=ov), steps)
    res = summary(flops_per_query(640) * 64, 64, el, steps,
                  "GraphCodeBERT step: B = 64 x L = 640 (512 code + 128 data-flow nodes, 1-3 code "
                  "tokens and 1-2 edges per node, seed 0), bit-packed mask, node averaging")
    # the masked attention kernels timed where nothing runs beside them (in the two-stream engine
    # a launch's events also span the other half's kernels sharing the CUs)
    eng_s = single_stream_engine(sd, precision, dev)
    ov_s = torch.empty_like(ov)
    _, (a_ms, a_n, _) = timed(lambda: eng_s.score_graph(gi_d, glens, gp_d, gb_d, out=ov_s), steps,
                              kind="attention", on=eng_s)
    eng_s.close()
    att = attention_summary(a_ms, a_n, steps, 64, 640, peak,
                            f"single-stream engine, the same batch, {steps} steps")
    if att:
        res["attention"] = att
    out["gcb640"] = res
    log(f"microbench gcb640: {res['victim_queries_per_s']} q/s")
    eng.close()
    return out


# ------------------------------------------------------------------------------------------ main
def main():
    args = parse_args()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(relaunch_as_ranks(args))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"bench.py: WORLD_SIZE={world} but --gpus {args.gpus}")

    import numpy as np
    import torch

    import _apmc  # noqa: F401

    # APMC_BENCH_REHEARSE=1: rehearsal of the N-rank path on a one-GPU box — every rank on cuda:0,
    # collectives over gloo (host tensors); the numbers of such a run are not a measurement
    rehearse = os.environ.get("APMC_BENCH_REHEARSE") == "1"
    dist = None
    if world > 1:
        import torch.distributed as dist
        gpu = 0 if rehearse else local
        torch.cuda.set_device(gpu)
        if rehearse:
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=torch.device(f"cuda:{gpu}"))
        seen = torch.ones(1, device="cpu" if rehearse else f"cuda:{gpu}")
        dist.all_reduce(seen)
        if int(seen.item()) != args.gpus:
            raise SystemExit(f"all-reduce saw {int(seen.item())} ranks, expected {args.gpus}")
    else:
        gpu = 0
        torch.cuda.set_device(0)
    dev = torch.device(f"cuda:{gpu}")
    if world > 1:  # the rank's share of the host (relaunch_env; torchrun alone gives 1 thread)
        torch.set_num_threads(rank_thread_budget(world))
    global COLL_DEV
    COLL_DEV = torch.device("cpu") if rehearse else dev  # where collective tensors live

    from apmc_amd.engine import Engine
    from apmc_amd.weights import synthetic_state_dict

    sd = synthetic_state_dict(seed=0, head="sigmoid1")
    eng = Engine(sd, head="sigmoid1", num_labels=1, precision=args.precision, device=dev.index)
    B, L = args.batch, args.seq
    rng = np.random.default_rng(0 + rank)
    ids = rng.integers(4, 50264, size=(B, L)).astype(np.int32)
    ids[:, 0], ids[:, -1] = 0, 2
    lens = np.full((B,), L, dtype=np.int32)
    ids_dev = torch.from_numpy(ids).to(dev)
    out = torch.empty((B, 1), dtype=torch.float32, device=dev)

    # the headline: the production engine with no instrumentation in the timed steps
    elapsed, _ = time_steps(eng, ids_dev, lens, out, args.steps, args.warmup, dev, dist,
                            profile=False)
    # FFN1 launch times inside the two-stream engine (context only), on separate steps
    _, (s_ms, s_n, s_flop) = time_steps(eng, ids_dev, lens, out, max(5, args.steps // 2), 1,
                                        dev, dist, profile=True)
    # the roofline kernel on its own: the production engine runs the encoder as two half-batch
    # streams (engine.hip run_encoder), so its FFN1 launches share the CUs with the other half's
    # kernels; FFN1 is timed (HIP events on its launch stream) on a single-stream engine over the
    # same batch, where nothing else runs beside it
    eng1 = single_stream_engine(sd, args.precision, dev)
    out1 = torch.empty_like(out)
    n1 = max(5, args.steps // 2)
    el1, (k_ms, k_n, k_flop) = time_steps(eng1, ids_dev, lens, out1, n1, args.warmup, dev, dist,
                                          profile=True)
    # the attention kernels of the same single-stream steps (11 full layers + the CLS-only last
    # layer), HIP events on their launch stream
    _, (at_ms, at_n, _) = time_steps(eng1, ids_dev, lens, out1, n1, args.warmup, dev, dist,
                                     profile=True, kind="attention")
    eng1.close()
    if dist is not None:
        t = torch.tensor([at_ms], dtype=torch.float64, device=COLL_DEV)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        at_ms = float(t.item())
    if dist is not None:
        t = torch.tensor([elapsed, el1], dtype=torch.float64, device=COLL_DEV)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed, el1 = float(t[0]), float(t[1])
        kt = torch.tensor([k_ms, float(k_n), k_flop, s_ms, float(s_n)], dtype=torch.float64,
                          device=COLL_DEV)
        dist.all_reduce(kt, op=dist.ReduceOp.SUM)
        k_ms, k_n, k_flop, s_ms, s_n = float(kt[0]), int(kt[1]), float(kt[2]), float(kt[3]), int(kt[4])

    probs = out.cpu().numpy()[:, 0]
    total_q = world * args.steps * B
    value = total_q / elapsed
    per_launch_s = (k_ms / 1e3) / max(k_n, 1)
    achieved = (k_flop / max(k_n, 1)) / per_launch_s / 1e12 if k_n else None
    # roofline peak of the arithmetic the GEMMs run: f32 MFMA; bf16 MFMA; split-bf16 issues
    # 3 bf16 MFMAs per product, so its ceiling in algorithmic FLOP/s is the bf16 peak / 3
    peak = {"fp32": FP32_MFMA_PEAK_TFLOPS, "bf16": BF16_MFMA_PEAK_TFLOPS,
            "f32x3": BF16_MFMA_PEAK_TFLOPS / 3}[args.precision]
    attention = attention_summary(at_ms, at_n, n1, B, L, peak,
                                  f"single-stream engine, the same batch, {n1} steps")
    fp32_mode = bf16_mode = None
    if args.precision != "fp32" and not args.no_fp32_mode:
        # the exact-fp32 mode of the same step, and the split / bf16 parity on this very batch
        ref_eng = Engine(sd, head="sigmoid1", num_labels=1, precision="fp32", device=dev.index)
        ref_out = torch.empty_like(out)
        el32, _ = time_steps(ref_eng, ids_dev, lens, ref_out, max(3, args.steps // 2),
                             args.warmup, dev, dist, profile=False)
        if dist is not None:
            t = torch.tensor([el32], dtype=torch.float64, device=COLL_DEV)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            el32 = float(t.item())
        n32 = max(3, args.steps // 2)
        fp32_mode = {"value": round(world * n32 * B / el32, 3), "unit": "victim queries/s",
                     "steps": n32, "ms_per_step": round(1e3 * el32 / n32, 4),
                     "max_abs_dprob_vs_this_mode": float(np.abs(ref_out.cpu().numpy()[:, 0]
                                                                - probs).max())}
        ref_eng.close()
        if args.precision == "f32x3":
            # bound diagnostic: the same step with one bf16 MFMA per product (hi planes only) —
            # what the split products cost; not a parity mode (stated tolerance 2e-2)
            b_eng = Engine(sd, head="sigmoid1", num_labels=1, precision="bf16", device=dev.index)
            b_out = torch.empty_like(out)
            el16, _ = time_steps(b_eng, ids_dev, lens, b_out, n32, args.warmup, dev, dist,
                                 profile=False)
            if dist is not None:
                t = torch.tensor([el16], dtype=torch.float64, device=COLL_DEV)
                dist.all_reduce(t, op=dist.ReduceOp.MAX)
                el16 = float(t.item())
            bf16_mode = {
                "value": round(world * n32 * B / el16, 3), "unit": "victim queries/s", "steps": n32,
                "ms_per_step": round(1e3 * el16 / n32, 4),
                "max_abs_dprob_vs_fp32_mode": float(np.abs(ref_out.cpu().numpy()[:, 0]
                                                           - b_out.cpu().numpy()[:, 0]).max()),
                "note": "diagnostic only: 1 bf16 MFMA per product instead of 3"}
            b_eng.close()
    executed = executed_flops_per_query(L) * total_q / elapsed / 1e12
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
        "max_abs_dprob_vs_fp32_mode": fp32_mode["max_abs_dprob_vs_this_mode"] if fp32_mode else None,
        "data": "synthetic (seeded RoBERTa-base weights; uniform token ids; no checkpoint offline)",
        "config": {"workload": "CodeBERT Devign victim scoring of one GA mutant population per "
                               "step (config 2 shape: eval_batch_size 64 x block 512)",
                   "global_batch": B * world, "seq_len": L,
                   "parallelism": f"dp{world} (example shards)"},
        "roofline": {
            "bound": "mfma",
            "kernel": {"fp32": "gemm_f32_nt_kernel<EPI_BIAS_GELU>",
                       "f32x3": "gemm_pp_kernel<2, PK_EPI_GELU_FOLD>",
                       "bf16": "gemm_pp_kernel<1, PK_EPI_GELU_FOLD>"}[args.precision]
                      + " (FFN1 [T,768]x[768,3072])",
            "achieved": round(achieved, 3) if achieved else None,
            "peak": peak,
            "unit": "TFLOP/s",
            "frac": round(achieved / peak, 4) if achieved else None,
            "traffic": pmc_traffic_per_launch(args.precision),
            "launches": k_n,
            "avg_launch_us": round(per_launch_s * 1e6, 2),
            "flop_per_launch": (k_flop / k_n) if k_n else None,
            "measured_on": f"single-stream engine (AE_STREAMS_ONE), the same batch, {n1} steps "
                           f"({round(1e3 * el1 / n1, 3)} ms per step); in the headline's "
                           "two-stream engine each FFN1 launch covers half the tokens and shares "
                           "the CUs with the other half's kernels",
            "two_stream_avg_launch_us": round(1e3 * s_ms / max(s_n, 1), 2) if s_n else None,
        },
        "attention": attention,
        "whole_step_executed_tflops": round(executed, 3),
        "whole_step_frac_of_peak": round(executed / world / peak, 4),
        "probs_checksum": float(np.round(probs.astype(np.float64).sum(), 6)),
    }
    if fp32_mode:
        res["fp32_mode"] = fp32_mode
    if bf16_mode:
        res["bf16_mode"] = bf16_mode
    eng.close()
    threads, cpu_facts = host_cores()
    log(f"scoring step: {value:.1f} q/s")
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        # the CPU reference path on this host, at the job's CPU share and at one thread per
        # physical core of the affinity (on a shared 8-GPU host the latter can be SLOWER: the
        # other jobs' load); the best point is the baseline, every point is reported
        sweep = sorted({t for t in (cpu_facts.get("job_share_threads"), threads // 2, threads)
                        if t})
        import torch as _torch
        host_threads = _torch.get_num_threads()  # the GPU legs' host work keeps its own setting
        points = []
        for t in sweep:
            log(f"CPU baseline ({t} threads)")
            v, sample = cpu_baseline(L, args.cpu_seconds, t)
            points.append({"cores": t, "value": round(v, 4), "sample": sample,
                           "path": "oracle/roberta_cpu.py fp32 eager"})
        try:  # the transformers forward the reference itself calls, at every point of the sweep
            for t in sweep:
                log(f"CPU baseline, transformers ({t} threads)")
                v, sample = cpu_baseline(L, args.cpu_seconds, t, impl="hf")
                points.append({"cores": t, "value": round(v, 4), "sample": sample,
                               "path": "transformers RobertaForSequenceClassification eager fp32"})
        except ImportError as e:
            log(f"transformers not importable: {e}")
        best = max(points, key=lambda q: q["value"])
        threads = best["cores"]
        _torch.set_num_threads(host_threads)
        res["cpu_baseline"] = {"value": best["value"], "unit": "victim queries/s",
                               "cores": best["cores"], "kind": "port",
                               "sample": best["sample"] + f", {best['path']}, torch "
                                                          f"threads={best['cores']} (the fastest "
                                                          "point of the sweep)",
                               "thread_sweep": points, **cpu_facts}
        res["speedup_vs_cpu"] = round(value / best["value"], 2)
    if not args.no_microbench:
        log("microbenchmarks (batch 1024, varlen, GCB 640)")
        res["microbench"] = microbench_leg(dev, args.precision, args.steps, args.warmup, world)
    if args.attack_examples > 0:
        log("config-2 attack leg")
        with heartbeat("config-2 attack leg"):
            res["attack"] = attack_leg(dev, args.attack_examples, args.attack_deadline,
                                       args.attack_inflight, rank, world, args.precision)
    if rank == 0 and world == 1 and not args.no_config1:
        log("config-1 leg")
        res["config1"] = config1_leg(dev, args.precision, threads,
                                     0 if args.no_cpu_baseline else args.cpu_e2e_seconds)
    if args.subs_seconds > 0:
        log("substitutes leg")
        res["substitutes"] = subs_leg(dev, args.subs_seconds, rank, world, args.precision)
    if args.aa_examples > 0:
        log("authorship leg")
        with heartbeat("authorship leg"):
            res["authorship"] = aa_leg(dev, args.aa_examples, args.aa_gcb_examples, rank, world,
                                       args.precision)
    if args.clone_examples > 0:
        log("config-4 leg (GraphCodeBERT clone)")
        with heartbeat("config-4 leg"):
            res["clone_gcb"] = clone_leg(dev, args.clone_examples, rank, world, args.precision)
    if args.mhm_examples > 0:
        log("MHM-NS leg")
        with heartbeat("MHM-NS leg"):
            res["mhm"] = mhm_leg(dev, args.mhm_examples, args.mhm_seq_examples, rank, world,
                                 args.precision)
    if rank == 0:
        print(json.dumps(res), flush=True)
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
