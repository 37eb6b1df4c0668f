"""Cross-example request batching, shared by the greedy/GA driver and the MHM-NS chains.

Every attack (attack_one_gen, MHM_Attacker._run_gen, ...) is written as a generator that yields
its victim requests (`Payload`, model.py) and receives `(probs, preds)` back — the reference's
`get_results` call sites (CodeXGLUE/Defect-detection/code/attacker.py:32,71,114,196,249,295,410,
640,706) turned inside out.  `run_requests` keeps up to `max_inflight` such generators alive and
answers ALL their pending requests with one device batch per round, so the GPU scores thousands
of rows at a time instead of one population of <= 64.  Rows are scored batch-invariantly, so
every generator sees exactly the answers its sequential run would see.

With a victim that can submit asynchronously (`Model.submit`: pinned uploads, kernels, a pinned
D2H copy, an event) the live generators run as two groups: while one group's batch is on the
device, the host advances the other group's attacks (mutation, featurisation) on its answers.
"""
from __future__ import annotations

import time


def run_requests(model, next_item, start, on_done, max_inflight=64, pipeline=True):
    """Drive request generators to completion.

    next_item() -> the next work key, or None when the source is drained (a list cursor, or a
        dist.DynamicQueue shared by all ranks);
    start(key)  -> a fresh (unprimed) generator for that key;
    on_done(key, value, queries, t_start) is called as each generator returns `value`, with the
        rows its requests carried (Model.query's increments for it) and its start time."""
    groups = 2 if (pipeline and hasattr(model, "submit")) else 1
    cap = max(1, max_inflight // groups)
    live = [[] for _ in range(groups)]   # entries: [key, generator, pending payload, rows, t0]
    pend = [None] * groups
    drained = False

    def refill(group):
        nonlocal drained
        while not drained and len(group) < cap:
            key = next_item()
            if key is None:
                drained = True
                break
            gen = start(key)
            t0 = time.time()
            try:
                group.append([key, gen, next(gen), 0, t0])
            except StopIteration as stop:
                on_done(key, stop.value, 0, t0)

    def advance(group, answers):
        still = []
        for c, ans in zip(group, answers):
            c[3] += c[2].n
            try:
                c[2] = c[1].send(ans)
                still.append(c)
            except StopIteration as stop:
                on_done(c[0], stop.value, c[3], c[4])
        return still

    while True:
        for g in range(groups):
            if pend[g] is not None:
                live[g] = advance(live[g], pend[g].result())
                pend[g] = None
            refill(live[g])
            if live[g]:
                payloads = [c[2] for c in live[g]]
                if groups == 1:
                    live[g] = advance(live[g], model.score_prepared(payloads))
                else:
                    pend[g] = model.submit(payloads)
        if drained and not any(live) and all(x is None for x in pend):
            break


def list_source(items):
    """next_item over a fixed list."""
    it = iter(items)
    return lambda: next(it, None)
