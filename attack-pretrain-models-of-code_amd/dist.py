"""Multi-GPU execution of the attack drivers: one process per GPU, examples sharded dynamically.

The reference scales by launching one OS process per GPU over static 400-example chunks
(CodeXGLUE/Defect-detection/code/run.sh:1-106).  Per-example query counts are extremely skewed
(a greedy success costs a handful of queries, a full GA thousands), so static chunks leave GPUs
idle; here every rank pulls the next example index from one atomic counter in the
torch.distributed store (TCPStore.add — no tensor traffic on the data path).  At the end the
per-rank statistics [examples, correct, successes, queries, wall_ns] are all-gathered (RCCL over
xGMI with backend "nccl", gloo in CPU tests) and the records are merged by example index, so the
CSV and every per-example outcome are those of a 1-GPU run when the per-example RNG is used
(`AttackArgs.rng = "per_example"`: random.seed(seed + index) before each example).
"""
from __future__ import annotations

import os
import time

import numpy as np


def init_from_env(backend: str = "nccl"):
    """Initialise torch.distributed from torchrun's RANK / WORLD_SIZE / MASTER_* (127.0.0.1)."""
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world <= 1 or dist.is_initialized():
        return dist if dist.is_initialized() else None
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if backend == "nccl":
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device(f"cuda:{local}"))
    else:
        dist.init_process_group(backend)
    return dist


class DynamicQueue:
    """Work queue over example indices [0, n) shared by all ranks (atomic store counter)."""

    def __init__(self, n: int, key: str = "apmc_attack_queue", store=None, order=None,
                 deadline: float | None = None):
        import torch.distributed as dist

        self.n = n
        self.order = list(order) if order is not None else None
        self.deadline = deadline
        if store is None and dist.is_available() and dist.is_initialized():
            store = dist.distributed_c10d._get_default_store()
        self.store = store
        self.key = key
        self.local = 0

    def __call__(self):
        if self.deadline is not None and time.time() > self.deadline:
            return None
        if self.store is None:
            i = self.local
            self.local += 1
        else:
            i = int(self.store.add(self.key, 1)) - 1
        if i >= self.n:
            return None
        return self.order[i] if self.order is not None else i


_CALLS = {}


def call_key(prefix: str) -> str:
    """A store key unique to this collective call: every rank makes the same sequence of sharded
    calls, so a per-prefix call counter gives all ranks the same fresh key (a TCPStore counter
    lives as long as the process group; reusing one would hand every rank None at once)."""
    n = _CALLS.get(prefix, 0)
    _CALLS[prefix] = n + 1
    return f"{prefix}_{n}"


def gather_stats(stats, device=None):
    """All-gather one float64 vector per rank -> [world, len] numpy array.  With the nccl (RCCL)
    backend the vector travels from this rank's current GPU."""
    import torch
    import torch.distributed as dist

    v = np.asarray(stats, dtype=np.float64)
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
        return v[None]
    if dist.get_backend() != "nccl":
        device = torch.device("cpu")  # gloo: host tensors
    elif device is None:
        device = torch.device("cuda", torch.cuda.current_device())
    t = torch.tensor(v, dtype=torch.float64, device=device)
    out = [torch.zeros_like(t) for _ in range(dist.get_world_size())]
    dist.all_gather(out, t)
    return torch.stack(out).cpu().numpy()


def merge_records(records):
    """All-gather the per-rank record lists and return them merged by example index."""
    import torch.distributed as dist

    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
        return sorted(records, key=lambda r: r["index"])
    parts = [None] * dist.get_world_size()
    dist.all_gather_object(parts, records)
    merged = [r for p in parts for r in p]
    return sorted(merged, key=lambda r: r["index"])


def run_sharded_gi_attack(model, codes, subs, labels, args, device=None, tok=None):
    """run_gi_attack over all ranks with a dynamic queue; returns (merged records, totals).
    Across ranks the examples are taken in scheduling order, so the per-example RNG
    (args.rng == "per_example") is required for records identical to a 1-GPU run."""
    import torch.distributed as dist

    from .drivers import run_gi_attack

    world = dist.get_world_size() if dist.is_available() and dist.is_initialized() else 1
    if world > 1 and args.rng != "per_example":
        raise ValueError("run_sharded_gi_attack with world > 1 needs AttackArgs.rng='per_example' "
                         "(one global random stream would depend on which rank took an example)")
    q = DynamicQueue(len(codes), key=call_key("apmc_attack_queue"))
    rank = dist.get_rank() if world > 1 else 0
    t0 = time.time()
    out = run_gi_attack(model, codes, subs, labels, _rank_csv(args, rank, world), queue=q, tok=tok)
    wall = time.time() - t0
    st = gather_stats([out["examples"], out["total_cnt"], out["success"], out["queries"], wall],
                      device=device)
    recs = merge_records(out["records"])
    merge_csv_shards(dist, rank, world, getattr(args, "csv_store_path", None))
    tot = dict(examples=int(st[:, 0].sum()), total_cnt=int(st[:, 1].sum()),
               success=int(st[:, 2].sum()), queries=int(st[:, 3].sum()),
               wall_s=float(st[:, 4].max()), per_rank=st.tolist())
    tot["success_rate"] = tot["success"] / tot["total_cnt"] if tot["total_cnt"] else 0.0
    return recs, tot


def _rank_world():
    import torch.distributed as dist

    on = dist.is_available() and dist.is_initialized()
    return (dist, dist.get_rank(), dist.get_world_size()) if on else (None, 0, 1)


def _job_totals(st, names, nsum):
    """Sum the first `nsum` gathered columns over ranks, max the rest (wall clocks); keep every
    rank's row so the tail of a skewed queue stays visible."""
    tot = {n: (float(st[:, i].sum()) if i < nsum else float(st[:, i].max()))
           for i, n in enumerate(names)}
    for n in names[:nsum]:
        tot[n] = int(round(tot[n]))
    tot["per_rank"] = [{n: (int(round(v)) if i < nsum else round(float(v), 3))
                        for i, (n, v) in enumerate(zip(names, row))} for row in st]
    return tot


def _inflight(max_inflight, n, world):
    """Examples a rank keeps in flight: on one rank all it may; on several, at most half an even
    share of the queue, so the other half is handed out as ranks free up (per-example cost is
    skewed; the ranks fill their first batches at the same instant after the barrier, and an
    uncapped fill would hand the whole queue out statically).  No floor: one GA example or two
    MHM-NS chains already fill most of a 64-row device batch, while a floor of 8 left ranks idle
    on short queues (32 MHM-NS examples over 8 ranks went to 4 of them)."""
    if world <= 1:
        return max_inflight
    return max(1, min(max_inflight, -(-n // (2 * world))))


GI_STATS = ["examples", "total_cnt", "success", "queries", "ga_runs", "ga_successes", "wall_s"]
MHM_STATS = ["examples", "total_cnt", "success", "queries", "errors", "wall_s"]


def _rank_csv(args, rank, world):
    """args with this rank's Recorder shard `<csv_store_path>.rank<r>` (world > 1): ranks never
    open the one CSV together (Recorder truncates it, utils.py:654)."""
    import dataclasses

    if world <= 1 or not getattr(args, "csv_store_path", None):
        return args
    return dataclasses.replace(args, csv_store_path=f"{args.csv_store_path}.rank{rank}")


def merge_csv_shards(dist, rank, world, path):
    """Rank 0 merges the ranks' Recorder shards into `path`, rows in example-index order (the
    1-GPU file), and removes the shards."""
    import csv

    if world <= 1 or not path:
        return
    dist.barrier()
    if rank == 0:
        header, rows = None, []
        for r in range(world):
            shard = f"{path}.rank{r}"
            if not os.path.exists(shard):  # a rank that never opened its Recorder
                continue
            with open(shard, newline="") as f:
                rd = csv.reader(f)
                head = next(rd, None)
                if head is not None:
                    header = head
                    rows.extend(rd)
            os.remove(shard)
        if header is None:
            from .utils import Recorder
            header = Recorder.HEADER
        rows.sort(key=lambda row: int(row[0]))
        with open(path, "w", newline="") as f:
            w = csv.writer(f)
            w.writerow(header)
            w.writerows(rows)
    dist.barrier()


def run_sharded_gi_batched(model, codes, subs, labels, args, max_inflight=64, device=None,
                           deadline: float | None = None, key: str = "apmc_gi_batched_queue"):
    """run_gi_attack_batched (cross-example batched greedy -> GA) over all ranks: one dynamic
    example queue, each rank batching the examples it pulled; statistics all-gathered, records
    merged by index.  Per-example RNG (random.Random(seed + index)) makes every record equal the
    1-GPU run whichever rank took the example.  Returns (merged records, job totals)."""
    from .drivers import run_gi_attack_batched

    dist, rank, world = _rank_world()
    q = DynamicQueue(len(codes), key=call_key(key), deadline=deadline)
    if dist is not None:
        dist.barrier()
    out = run_gi_attack_batched(model, codes, subs, labels, _rank_csv(args, rank, world), queue=q,
                                max_inflight=_inflight(max_inflight, len(codes), world))
    recs = out["records"]
    ga = [r for r in recs if r["attack_type"] == "GA"]
    st = gather_stats([out["examples"], out["total_cnt"], out["success"], out["queries"],
                       len(ga), sum(r["is_success"] == 1 for r in ga), out["wall_s"]],
                      device=device)
    tot = _job_totals(st, GI_STATS, 6)
    tot["success_rate"] = tot["success"] / tot["total_cnt"] if tot["total_cnt"] else 0.0
    merge_csv_shards(dist, rank, world, getattr(args, "csv_store_path", None))
    return merge_records(recs), tot


def run_sharded_mhm(model, codes, subs, labels, args, n_candi=30, max_iter=None, prob_threshold=1,
                    original=False, max_inflight=64, device=None, n: int | None = None,
                    key: str = "apmc_mhm_queue"):
    """run_mhm_attack (cross-example batched MHM-NS chains) over all ranks with one dynamic
    queue over examples [0, n) — per-example MCMC cost is as skewed as GA's (a success after one
    round vs 100 rounds of 31 candidates).  max_iter None = the task driver's own count
    (drivers.MHM_MAX_ITER).  Returns (merged records, job totals)."""
    from .drivers import run_mhm_attack

    dist, rank, world = _rank_world()
    n_ex = len(codes) if n is None else n
    q = DynamicQueue(n_ex, key=call_key(key))
    if dist is not None:
        dist.barrier()
    out = run_mhm_attack(model, codes, subs, labels, _rank_csv(args, rank, world), n_candi=n_candi,
                         max_iter=max_iter, prob_threshold=prob_threshold, original=original,
                         max_inflight=_inflight(max_inflight, n_ex, world), queue=q)
    st = gather_stats([out["examples"], out["total_cnt"], out["success"], out["queries"],
                       out["errors"], out["wall_s"]], device=device)
    tot = _job_totals(st, MHM_STATS, 5)
    tot["success_rate"] = tot["success"] / tot["total_cnt"] if tot["total_cnt"] else 0.0
    merge_csv_shards(dist, rank, world, getattr(args, "csv_store_path", None))
    return merge_records(out["records"]), tot


def run_sharded_substitutes(gen, in_path, out_path, start=0, end=None, device=None,
                            deadline: float | None = None, log=None):
    """get_substitutes.py over all ranks (examples across ranks, jsonl merged by
    index): every rank pulls item indices from the shared queue and writes its shard
    `<out_path>.rank<r>`; rank 0 merges the shards into `out_path` in input order.  Returns the
    job totals (all-gathered).  log(idx, item): called after each item this rank finishes."""
    import torch.distributed as dist

    from .substitutes import generate_file, merge_shards

    on = dist.is_available() and dist.is_initialized()
    rank, world = (dist.get_rank(), dist.get_world_size()) if on else (0, 1)
    n_items = 0
    with open(in_path) as f:
        for i, _ in enumerate(f):
            if i >= start and (end is None or i < end):
                n_items += 1
    q = DynamicQueue(n_items, key=call_key("apmc_subs_queue"), deadline=deadline)
    shard = f"{out_path}.rank{rank}"
    t0 = time.time()
    out = generate_file(gen, in_path, shard, start, end, queue=q, log=log)
    wall = time.time() - t0
    st = gather_stats([out["items"], out["occurrences"], out["encoded_seqs"],
                       out["encoded_tokens"], wall], device=device)
    if on:
        dist.barrier()
    if rank == 0:
        merge_shards([f"{out_path}.rank{r}" for r in range(world)], out_path)
        for r in range(world):
            os.remove(f"{out_path}.rank{r}")
    if on:
        dist.barrier()
    return dict(items=int(st[:, 0].sum()), occurrences=int(st[:, 1].sum()),
                encoded_seqs=int(st[:, 2].sum()), encoded_tokens=int(st[:, 3].sum()),
                wall_s=float(st[:, 4].max()), per_rank=st.tolist())
