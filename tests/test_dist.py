"""CPU multi-process (gloo, world_size 2): the sharded attack driver — dynamic example queue over
the torch.distributed store, all-gather of statistics, records merged by index — reproduces the
single-process run exactly.  The victim here is a deterministic numpy stand-in that scores the
real featurised ids (built by the C++ host library), so only the scoring arithmetic is faked;
queue, featurisation, attack logic and merging are the product code."""
import os
import pathlib
import sys

import numpy as np
import pytest
import torch.multiprocessing as mp

ROOT = pathlib.Path(__file__).resolve().parents[1]
FIXTURE = ROOT / "data" / "devign" / "test_subs_0_400.jsonl"
N_EX = 10


def FakeVictim():
    """Devign-format victim over ids: p = sigmoid(<ids, w> / scale) (deterministic numpy
    stand-in for the engine behind the product's request API, apmc_amd.model.HostIdsVictim)."""
    sys.path.insert(0, str(ROOT))
    import _apmc  # noqa: F401
    from apmc_amd.model import HostIdsVictim

    w = np.random.default_rng(0).standard_normal(50265).astype(np.float64)

    def score(ids):
        ids = np.asarray(ids)
        z = np.where(ids != 1, w[ids], 0.0).sum(1) / 8.0
        return (1.0 / (1.0 + np.exp(-z))).astype(np.float32)[:, None]

    return HostIdsVictim(score)


def _worker(rank, world, port, outdir):
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), MASTER_ADDR="127.0.0.1",
                      MASTER_PORT=str(port), LOCAL_RANK=str(rank))
    sys.path.insert(0, str(ROOT))
    import _apmc  # noqa: F401
    from apmc_amd.dist import init_from_env, run_sharded_gi_attack
    from apmc_amd.drivers import AttackArgs, load_fixture
    import torch.distributed as dist

    init_from_env("gloo")
    codes, subs, labels = load_fixture(FIXTURE, 0, N_EX)
    args = AttackArgs(block_size=128, eval_batch_size=8, rng="per_example")
    recs, tot = run_sharded_gi_attack(FakeVictim(), codes, subs, labels, args)
    # a second sharded call in the same process group (run.sh runs several chunks) must get a
    # fresh queue, not the drained counter of the first call
    recs2, tot2 = run_sharded_gi_attack(FakeVictim(), codes, subs, labels, args)
    try:  # the global RNG stream would depend on which rank took an example: refused
        run_sharded_gi_attack(FakeVictim(), codes, subs, labels,
                              AttackArgs(block_size=128, eval_batch_size=8, rng="global"))
        refused = False
    except ValueError:
        refused = True
    if rank == 0:
        import json
        (pathlib.Path(outdir) / "dist.json").write_text(json.dumps(
            {"recs": recs, "tot": tot, "recs2": recs2, "tot2": tot2, "refused": refused}))
    dist.barrier()
    dist.destroy_process_group()


def test_two_ranks_match_single_process(tmp_path):
    sys.path.insert(0, str(ROOT))
    import json
    import random
    import _apmc  # noqa: F401
    from apmc_amd.drivers import AttackArgs, load_fixture, run_gi_attack

    port = 29500 + random.Random(os.getpid()).randint(0, 2000)
    mp.spawn(_worker, args=(2, port, str(tmp_path)), nprocs=2, join=True)
    got = json.loads((tmp_path / "dist.json").read_text())

    codes, subs, labels = load_fixture(FIXTURE, 0, N_EX)
    single = run_gi_attack(FakeVictim(), codes, subs, labels,
                           AttackArgs(block_size=128, eval_batch_size=8, rng="per_example"))
    keys = ["index", "is_success", "attack_type", "queries", "adv_code", "replace_info"]
    a = [{k: r[k] for k in keys} for r in got["recs"]]
    b = [{k: r[k] for k in keys} for r in single["records"]]
    assert a == b
    assert [{k: r[k] for k in keys} for r in got["recs2"]] == b
    assert got["tot2"]["examples"] == N_EX and got["refused"]
    assert got["tot"]["examples"] == N_EX
    assert got["tot"]["queries"] == single["queries"]
    # one row per rank, summing to the job (which rank pulled how much is scheduling)
    per_rank = got["tot"]["per_rank"]
    assert len(per_rank) == 2 and sum(r[0] for r in per_rank) == N_EX


class FakeSubsGen:
    """Stands in for SubstituteGenerator (the masked-LM arithmetic needs the GPU): the real host
    identifier extraction, a deterministic substitute rule."""

    def __init__(self):
        self.stats = {"examples": 0, "occurrences": 0, "encoded_seqs": 0, "encoded_tokens": 0}

    def generate(self, func):
        from apmc_amd.attacker import get_identifiers
        from apmc_amd.host import remove_comments
        ids, _ = get_identifiers(remove_comments(func), "c")
        self.stats["examples"] += 1
        self.stats["occurrences"] += len(ids)
        return {i[0]: [i[0] + "_x", "v" + str(len(i[0]))] for i in ids}


def _subs_worker(rank, world, port, outdir):
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), MASTER_ADDR="127.0.0.1",
                      MASTER_PORT=str(port), LOCAL_RANK=str(rank))
    sys.path.insert(0, str(ROOT))
    import _apmc  # noqa: F401
    from apmc_amd.dist import init_from_env, run_sharded_substitutes
    import torch.distributed as dist

    init_from_env("gloo")
    tot = run_sharded_substitutes(FakeSubsGen(), FIXTURE, str(pathlib.Path(outdir) / "subs.jsonl"),
                                  0, N_EX)
    if rank == 0:
        import json
        (pathlib.Path(outdir) / "tot.json").write_text(json.dumps(tot))
    dist.barrier()
    dist.destroy_process_group()


def test_sharded_substitutes_match_single_process(tmp_path):
    """get_substitutes.py sharded over 2 ranks: merged jsonl == single-process output."""
    sys.path.insert(0, str(ROOT))
    import json
    import random
    import _apmc  # noqa: F401
    from apmc_amd.substitutes import generate_file

    port = 31500 + random.Random(os.getpid()).randint(0, 2000)
    mp.spawn(_subs_worker, args=(2, port, str(tmp_path)), nprocs=2, join=True)
    generate_file(FakeSubsGen(), FIXTURE, tmp_path / "single.jsonl", 0, N_EX)
    assert (tmp_path / "subs.jsonl").read_text() == (tmp_path / "single.jsonl").read_text()
    tot = json.loads((tmp_path / "tot.json").read_text())
    assert tot["items"] == N_EX and sum(r[0] for r in tot["per_rank"]) == N_EX
    assert not list(tmp_path.glob("subs.jsonl.rank*"))


def _batched_worker(rank, world, port, outdir):
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), MASTER_ADDR="127.0.0.1",
                      MASTER_PORT=str(port), LOCAL_RANK=str(rank))
    sys.path.insert(0, str(ROOT))
    import _apmc  # noqa: F401
    from apmc_amd.dist import init_from_env, run_sharded_gi_batched, run_sharded_mhm
    from apmc_amd.drivers import AttackArgs, load_fixture
    import torch.distributed as dist

    init_from_env("gloo")
    codes, subs, labels = load_fixture(FIXTURE, 0, N_EX)
    out = pathlib.Path(outdir)
    args = AttackArgs(block_size=128, eval_batch_size=8, rng="per_example",
                      csv_store_path=str(out / "gi.csv"))
    gi, gi_tot = run_sharded_gi_batched(FakeVictim(), codes, subs, labels, args, max_inflight=4)
    margs = AttackArgs(block_size=128, eval_batch_size=8, rng="per_example",
                       csv_store_path=str(out / "mhm.csv"))
    mhm, mhm_tot = run_sharded_mhm(FakeVictim(), codes, subs, labels, margs, max_iter=8,
                                   max_inflight=4)
    if rank == 0:
        import json
        (pathlib.Path(outdir) / "batched.json").write_text(json.dumps(
            {"gi": gi, "gi_tot": gi_tot, "mhm": mhm, "mhm_tot": mhm_tot}))
    dist.barrier()
    dist.destroy_process_group()


def test_two_ranks_batched_drivers_match_single_process(tmp_path):
    """The bench legs' multi-GPU form (dist.run_sharded_gi_batched / run_sharded_mhm: one dynamic
    queue per leg, cross-example batching inside each rank, all-gathered totals with per-rank
    rows, records merged by index) on 2 gloo ranks equals the single-process batched drivers."""
    sys.path.insert(0, str(ROOT))
    import json
    import random
    import _apmc  # noqa: F401
    from apmc_amd.drivers import AttackArgs, load_fixture, run_gi_attack_batched, run_mhm_attack

    port = 33500 + random.Random(os.getpid()).randint(0, 2000)
    mp.spawn(_batched_worker, args=(2, port, str(tmp_path)), nprocs=2, join=True)
    got = json.loads((tmp_path / "batched.json").read_text())

    codes, subs, labels = load_fixture(FIXTURE, 0, N_EX)
    args = AttackArgs(block_size=128, eval_batch_size=8, rng="per_example",
                      csv_store_path=str(tmp_path / "gi_single.csv"))
    gi = run_gi_attack_batched(FakeVictim(), codes, subs, labels, args, max_inflight=4)
    keys = ["index", "is_success", "attack_type", "queries", "adv_code", "replace_info"]
    assert [{k: r[k] for k in keys} for r in got["gi"]] == \
        [{k: r[k] for k in keys} for r in gi["records"]]
    assert got["gi_tot"]["queries"] == gi["queries"] and got["gi_tot"]["examples"] == N_EX
    margs = AttackArgs(block_size=128, eval_batch_size=8, rng="per_example",
                       csv_store_path=str(tmp_path / "mhm_single.csv"))
    mhm = run_mhm_attack(FakeVictim(), codes, subs, labels, margs, max_iter=8, max_inflight=4)
    # each rank wrote its own Recorder shard; rank 0 merged them in index order: the CSVs equal
    # the single-process ones but for the wall-clock column
    import csv

    def rows(name):
        with open(tmp_path / name, newline="") as f:
            return [r[:15] for r in csv.reader(f)]
    assert rows("gi.csv") == rows("gi_single.csv") and len(rows("gi.csv")) == N_EX + 1
    assert rows("mhm.csv") == rows("mhm_single.csv") and len(rows("mhm.csv")) > 1
    assert not list(tmp_path.glob("*.rank*"))
    assert got["mhm"] == mhm["records"]
    assert got["mhm_tot"]["queries"] == mhm["queries"]
    assert {r["is_success"] for r in mhm["records"]} & {1, -1}
    for tot in (got["gi_tot"], got["mhm_tot"]):
        # one row per rank, summing to the job; which rank takes how many examples is scheduling
        # (with this instant victim one rank can drain the queue before the other's first pull)
        assert len(tot["per_rank"]) == 2
        assert sum(r["examples"] for r in tot["per_rank"]) == N_EX


def test_inflight_cap_spreads_short_queues():
    """A rank keeps at most half an even share of the queue in flight (no floor), so a short
    queue reaches every rank: 32 MHM-NS examples over 8 ranks -> 2 in flight each."""
    sys.path.insert(0, str(ROOT))
    import _apmc  # noqa: F401
    from apmc_amd.dist import _inflight

    assert _inflight(64, 32, 8) == 2
    assert _inflight(64, 400, 8) == 25
    assert _inflight(64, 400, 1) == 64
    assert _inflight(64, 3, 8) == 1


def test_relaunch_splits_host_threads_per_rank(tmp_path):
    """bench.py --gpus N relaunches itself as N ranks with each rank's host budget = the host's
    CPUs / N (1..16): torch threads, OMP_NUM_THREADS and the C++ featurisers' worker threads
    (host.gcb_threads) all take it, so N ranks sharing one host do not oversubscribe it.  Runs
    the relaunch's own environment (bench.relaunch_env) under torch.distributed.run, gloo,
    world 2."""
    import json
    import subprocess

    sys.path.insert(0, str(ROOT))
    import bench
    env = bench.relaunch_env(2)
    want = bench.rank_thread_budget(2, {k: v for k, v in env.items() if k != "APMC_HOST_THREADS"})
    assert env["OMP_NUM_THREADS"] == env["APMC_HOST_THREADS"] == str(want)
    cpus = len(os.sched_getaffinity(0))
    assert want == max(1, min(16, cpus // 2))
    out = tmp_path / "threads.json"
    port = 29500 + os.getpid() % 1000
    subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
                    "--nproc-per-node=2", "--master-addr", "127.0.0.1", f"--master-port={port}",
                    str(ROOT / "tests" / "_rank_threads.py"), str(out)],
                   env=env, check=True, timeout=300, capture_output=True)
    parts = json.loads(out.read_text())
    assert sorted(p["rank"] for p in parts) == [0, 1]
    for p in parts:
        assert p["torch"] == want and p["host"] == want and p["omp"] == str(want), p
    # an explicit APMC_HOST_THREADS wins
    assert bench.rank_thread_budget(8, {"APMC_HOST_THREADS": "5"}) == 5


def test_collectives_pick_the_backend_device(monkeypatch):
    """gather_stats all-gathers on the rank's current GPU under nccl (RCCL) and on the host under
    gloo (or an explicit device when given); merge_records uses all_gather_object (which places
    its buffers on the current device under nccl).  Checked against a stand-in torch.distributed
    that records the device of every tensor it is handed."""
    import torch
    import torch.distributed as tdist

    sys.path.insert(0, str(ROOT))
    import _apmc  # noqa: F401
    from apmc_amd import dist as adist

    seen = {}

    def all_gather(out, t):
        seen["device"] = t.device
        for o in out:
            o.copy_(t)

    def all_gather_object(parts, obj):
        seen["object"] = True
        for i in range(len(parts)):
            parts[i] = [dict(r, index=r["index"] + 100 * i) for r in obj]

    for name, val in (("is_available", lambda: True), ("is_initialized", lambda: True),
                      ("get_world_size", lambda: 2), ("all_gather", all_gather),
                      ("all_gather_object", all_gather_object)):
        monkeypatch.setattr(tdist, name, val)
    monkeypatch.setattr(tdist, "get_backend", lambda: "gloo")
    st = adist.gather_stats([1.0, 2.0], device=torch.device("meta"))
    assert seen["device"].type == "cpu" and st.shape == (2, 2)  # gloo: host, whatever is asked
    monkeypatch.setattr(tdist, "get_backend", lambda: "nccl")
    # nccl without an explicit device: the rank's current GPU (a stand-in index here, no GPU)
    monkeypatch.setattr(torch.cuda, "current_device", lambda: 3)
    orig_tensor = torch.tensor

    def tensor(v, dtype=None, device=None):
        seen["asked"] = torch.device(device) if device is not None else None
        return orig_tensor(v, dtype=dtype)  # built on the host: no GPU in this container
    monkeypatch.setattr(torch, "tensor", tensor)
    adist.gather_stats([1.0, 2.0])
    assert seen["asked"] == torch.device("cuda", 3)
    adist.gather_stats([1.0, 2.0], device=torch.device("cuda", 1))
    assert seen["asked"] == torch.device("cuda", 1)
    recs = adist.merge_records([{"index": 2}, {"index": 0}])
    assert seen["object"] and [r["index"] for r in recs] == [0, 2, 100, 102]
