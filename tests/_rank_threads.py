"""Rank body of tests/test_dist.py::test_relaunch_splits_host_threads_per_rank: started by
torch.distributed.run (gloo) under bench.relaunch_env(2); reports each rank's thread budget."""
import json
import os
import pathlib
import sys

ROOT = pathlib.Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

import _apmc  # noqa: E402,F401
import bench  # noqa: E402
from apmc_amd.host import gcb_threads  # noqa: E402

dist.init_process_group("gloo")
world = dist.get_world_size()
torch.set_num_threads(bench.rank_thread_budget(world))  # what bench.main does for world > 1
mine = {"rank": dist.get_rank(), "torch": torch.get_num_threads(), "host": gcb_threads(),
        "omp": os.environ.get("OMP_NUM_THREADS")}
parts = [None] * world
dist.all_gather_object(parts, mine)
if dist.get_rank() == 0:
    pathlib.Path(sys.argv[1]).write_text(json.dumps(parts))
dist.destroy_process_group()
