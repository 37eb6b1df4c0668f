"""Drop-in victim `Model` with the reference's query boundary `get_results`.

Mirrors, argument for argument and return value for return value:
  Devign (CodeBERT)     CodeXGLUE/Defect-detection/code/model.py:14-59
  Clone  (CodeBERT)     CodeXGLUE/Clone-detection-BigCloneBench/code/model.py:31-85
  Authorship (CodeBERT) CodeXGLUE/Authorship-Attribution/code/model.py:32-91

`get_results(dataset, batch_size)` adds len(dataset) to `self.query` (the metric's counter,
model.py:38) and returns (probs, pred_labels) in dataset order.  The reference iterates a
DataLoader(batch_size, num_workers=4) and syncs every batch; every row of the encoder is
independent of the other rows of its batch, so the engine scores the whole dataset as one device
batch (split only to bound workspace) with one host->device copy and one device->host copy.
`batch_size` is accepted for signature parity and does not change any result.
"""
from __future__ import annotations

import numpy as np

from .engine import Engine

TASK_HEAD = {"devign": ("sigmoid1", 1), "clone": ("pair2", 2), "authorship": ("softmaxN", 66)}


def _row_ids(item):
    """First element of a dataset item (CodeDataset tuple, InputFeatures, list or tensor)."""
    if hasattr(item, "input_ids"):
        return np.asarray(item.input_ids)
    x = item[0] if isinstance(item, (tuple, list)) and len(item) and not np.isscalar(item[0]) \
        else item
    if hasattr(x, "detach"):
        x = x.detach().cpu().numpy()
    return np.asarray(x)


def stack_ids(dataset) -> np.ndarray:
    rows = [_row_ids(dataset[i]).reshape(-1) for i in range(len(dataset))]
    if not rows:
        return np.zeros((0, 0), dtype=np.int32)
    return np.stack(rows).astype(np.int32, copy=False)


class Payload:
    """A featurised victim request: `ids` (device rows; numpy arrays for graph models), host
    `lens`, `n` = the queries it is charged (rows / 2 for clone pairs).  `extra` carries the graph
    inputs (pos, mask bits) of GraphCodeBERT victims."""

    __slots__ = ("ids", "lens", "n", "extra")

    def __init__(self, ids, lens, n, extra=None):
        self.ids, self.lens, self.n, self.extra = ids, lens, n, extra


def _checked(logits: np.ndarray) -> np.ndarray:
    """The engine turns every output of a call NaN when a row's lens disagreed with its ids
    (ae_score contract); never let that reach an attack decision."""
    if not np.isfinite(logits).all():
        raise RuntimeError("ae_score returned non-finite probabilities: the lens passed for some "
                           "row disagree with its count of non-pad ids")
    return logits


def to_device(a, dev):
    """Host array -> device tensor through pinned memory, non-blocking on the current stream:
    a pageable .to(dev) synchronises the stream, which would stall the host behind the batch
    already running (run_gi_attack_batched overlaps one group's host work with the other's
    device batch).  The caching host allocator keeps the pinned buffer until the copy ran."""
    import torch

    t = a if torch.is_tensor(a) else torch.from_numpy(np.ascontiguousarray(a))
    return t.pin_memory().to(dev, non_blocking=True)


class ScoresReady:
    """A submit() whose answers are already known (no live rows)."""

    def __init__(self, out):
        self.out = out

    def result(self):
        return self.out


class PendingScores:
    """The device scores of one submitted batch: the device-to-host copy is queued (pinned, non-
    blocking) behind the kernels, so the caller can do host work for other examples while the
    GPU runs; result() waits for this batch only and formats it per payload."""

    def __init__(self, dev_logits, payloads, fmt, threshold):
        import torch

        self.dev = dev_logits  # alive until the copy has run
        self.host = torch.empty(dev_logits.shape, dtype=dev_logits.dtype, pin_memory=True)
        self.host.copy_(dev_logits, non_blocking=True)
        self.ev = torch.cuda.Event()
        self.ev.record()
        self.payloads, self.fmt, self.threshold = payloads, fmt, threshold

    def result(self):
        self.ev.synchronize()
        logits = _checked(self.host.numpy())
        out, off = [], 0
        for p in self.payloads:
            out.append(self.fmt(logits[off:off + p.n], self.threshold) if p.n else ([], []))
            off += p.n
        return out


class Model:
    """Victim model.  `encoder` is an `Engine` (or a state dict, from which one is built)."""

    max_rows_per_launch = 2048

    def __init__(self, encoder, config=None, tokenizer=None, args=None, task: str = "devign",
                 precision: str = "fp32", device: int = 0):
        head, num_labels = TASK_HEAD[task]
        if isinstance(config, int):
            num_labels = config
        elif config is not None and hasattr(config, "num_labels") and task == "authorship":
            num_labels = int(config.num_labels)
        if isinstance(encoder, Engine):
            self.engine = encoder
        else:
            self.engine = Engine(encoder, head=head, num_labels=num_labels, precision=precision,
                                 device=device)
        self.task = task
        self.config = config
        self.tokenizer = tokenizer
        self.args = args
        self.query = 0
        self.tokens = 0  # non-pad tokens of every scored row (diagnostics: tokens / s on device)
        self.block_size = getattr(args, "block_size", None)
        # the Authorship-Attribution victim tokenizes raw source (no ' '.join(code.split()))
        self.raw = task == "authorship"

    # the reference calls model.eval()/.to(device) around get_results; keep them as no-ops
    def eval(self):
        return self

    def to(self, *a, **k):
        return self

    # ---- requests -------------------------------------------------------------------------
    # Every victim query goes through prepare*/score_prepared: a request is featurised into a
    # `Payload` (device ids + host lens), and score_prepared scores any number of payloads as
    # ONE device batch and splits the results per payload.  get_results is the one-payload case;
    # the cross-example attack drivers (drivers.run_gi_attack_batched) hand in the pending
    # requests of many attacked examples at once.  Rows are scored batch-invariantly, so the
    # split results equal separate calls bit for bit.
    def prepare(self, dataset) -> "Payload":
        """A get_results dataset (CodeDataset / IdsDataset / [example] list) -> Payload."""
        import torch

        n = len(dataset)
        if hasattr(dataset, "ids") and hasattr(dataset, "lens") and dataset.lens is not None:
            ids, lens = dataset.ids, np.asarray(dataset.lens, dtype=np.int32)
        else:
            ids = stack_ids(dataset) if n else np.zeros((0, self.block_size or 2), np.int32)
            lens = None
        if self.task == "clone" and n:
            # model.py:44 input_ids.view(-1, block_size): each row holds code1 | code2
            bs = self.block_size or ids.shape[1] // 2
            ids = ids.reshape(-1, bs)
            lens = None
        ids = np.ascontiguousarray(ids, dtype=np.int32)
        if lens is None:
            lens = (ids != self.engine.pad_id).sum(axis=1).astype(np.int32)
        dev = to_device(ids, f"cuda:{self.engine.device}")
        return Payload(dev, lens, n)

    def population_rows(self, example, tokenizer, population, mode: int, block_size: int):
        """Device ids [n, block] + host lens of a population of chromosomes of one program.

        The host library reduces every mutant to its word-id sequence (the mutant text is built
        exactly as get_example / get_example_batch would); ae_splice assembles the [n, block]
        ids on the GPU from the example's word table.  Identical ids to featurising the mutant
        texts (tests/test_host.py, tests/test_engine_gpu.py).  A raw-text victim (authorship)
        tokenizes whole mutant texts on the host instead: without the whitespace normalisation
        the token runs are not word-local."""
        import torch

        from .engine import splice
        from .host import MODE_RAW

        n = len(population)
        dev = f"cuda:{self.engine.device}"
        if n == 0:
            return (torch.zeros((0, block_size), dtype=torch.int32, device=dev),
                    np.zeros((0,), np.int32))
        if self.raw:
            ids, lens = example.mutant_ids(tokenizer, population, block_size, mode | MODE_RAW)
            return to_device(ids, dev), lens
        word_tok, word_off, mut_words, mut_off, lens = example.mutant_words(
            tokenizer, population, block_size, mode)
        ids, _ = splice(to_device(word_tok, dev), to_device(word_off, dev),
                        to_device(mut_words, dev), to_device(mut_off, dev),
                        n, block_size, tokenizer.cls_token_id, tokenizer.sep_token_id,
                        tokenizer.pad_token_id)
        return ids, lens

    def prepare_population(self, example, tokenizer, population, mode: int, block_size: int):
        """A population of chromosomes of one program (len(population) queries)."""
        ids, lens = self.population_rows(example, tokenizer, population, mode, block_size)
        return Payload(ids, lens, len(population))

    def prepare_pairs(self, ids1, lens1, ids2_row, len2) -> "Payload":
        """Clone queries (Clone-detection-BigCloneBench/code/model.py:44): row i of ids1 paired
        with the one fixed code2 row, interleaved code1, code2 per pair as the [2n, block] view
        of the reference's [n, 2*block] ids."""
        import torch

        dev = f"cuda:{self.engine.device}"
        a = ids1 if torch.is_tensor(ids1) else torch.from_numpy(np.ascontiguousarray(ids1))
        a = (a if a.is_cuda else to_device(a, dev)).to(dtype=torch.int32)
        n, L = a.shape
        b = to_device(np.ascontiguousarray(ids2_row, dtype=np.int32), dev)
        rows = torch.stack([a, b.expand(n, L)], 1).reshape(2 * n, L).contiguous()
        lens = np.empty((2 * n,), np.int32)
        lens[0::2], lens[1::2] = np.asarray(lens1, np.int32), int(len2)
        return Payload(rows, lens, n)

    def score_prepared(self, payloads, threshold: float = 0.5):
        """Score payloads as one device batch; query += their total queries.  Returns one
        (probs, pred_labels) per payload, each exactly what get_results gives for it alone."""
        return self.submit(payloads, threshold).result()

    def submit(self, payloads, threshold: float = 0.5):
        """score_prepared split in two: queue the device batch now (query += at once), answer
        with .result() later (PendingScores)."""
        import torch

        nq = [p.n for p in payloads]
        self.query += sum(nq)
        self.tokens += int(sum(int(p.lens.sum()) for p in payloads if p.n))
        live = [p for p in payloads if p.n]
        if not live:
            return ScoresReady([([], []) for _ in payloads])
        ids = torch.cat([p.ids for p in live], 0) if len(live) > 1 else live[0].ids
        lens = np.concatenate([p.lens for p in live]) if len(live) > 1 else live[0].lens
        per_row = 2 if self.task == "clone" else 1
        assert sum(nq) * per_row == ids.shape[0]
        return PendingScores(self._score_dev_async(ids, lens), payloads, self._format, threshold)

    def _score_dev_async(self, ids, lens: np.ndarray):
        import torch

        n = ids.shape[0]
        step = self.max_rows_per_launch
        outs = [self.engine.score(ids[s:s + step].contiguous(), lens[s:s + step])
                for s in range(0, n, step)]
        return torch.cat(outs, 0) if len(outs) > 1 else outs[0]

    def _score_dev(self, ids, lens: np.ndarray) -> np.ndarray:
        return _checked(self._score_dev_async(ids, lens).cpu().numpy())

    def get_results(self, dataset, batch_size=None, threshold: float = 0.5):
        """(probs, pred_labels) exactly as the reference's get_results of this task."""
        if len(dataset) == 0:
            return [], []
        return self.score_prepared([self.prepare(dataset)], threshold)[0]

    def dataset_from_texts(self, texts, tokenizer, args, label=0):
        """Mutant texts -> the dataset get_results consumes (convert_code_to_features of every
        text, CodeXGLUE/Defect-detection/code/attacker.py:38-45, batched in the host library)."""
        from .utils import IdsDataset

        ids, lens = tokenizer.featurize(list(texts), args.block_size, raw=self.raw)
        return IdsDataset(ids, lens)

    def get_results_population(self, example, tokenizer, population, mode: int, block_size: int,
                               threshold: float = 0.5):
        """Score a population of chromosomes of one program (len(population) queries)."""
        if len(population) == 0:
            return [], []
        return self.score_prepared([self.prepare_population(example, tokenizer, population, mode,
                                                            block_size)], threshold)[0]

    def _format(self, logits, threshold: float = 0.5):
        return format_results(self.task, logits, threshold)


def format_results(task, logits, threshold: float = 0.5):
    """(probs, pred_labels) of one get_results call from the head outputs [n, C]."""
    if task == "devign":
        # model.py:56-57
        probs = [[1 - prob[0], prob[0]] for prob in logits]
        pred_labels = [1 if label else 0 for label in logits[:, 0] > 0.5]
    elif task == "clone":
        # Clone-detection-BigCloneBench/code/model.py:81-82
        probs = logits
        pred_labels = [0 if first_softmax > threshold else 1 for first_softmax in logits[:, 0]]
    else:
        # Authorship-Attribution/code/model.py:84-89
        probs = logits
        pred_labels = [np.argmax(logit) for logit in logits]
    return probs, pred_labels


class HostIdsVictim:
    """The Model request API (prepare / prepare_population / score_prepared / get_results) over a
    host scoring function `score_fn(ids int32 [n, L]) -> head outputs [n, C]` — for victims that
    are not the engine (the CPU baseline of bench.py, multi-process CPU tests).  Mutant ids come
    from the host featuriser (Example.mutant_ids), the same ids the device splice builds."""

    def __init__(self, score_fn, task: str = "devign", block_size=None, pad_id: int = 1):
        self.score_fn = score_fn
        self.task = task
        self.block_size = block_size
        self.pad_id = pad_id
        self.query = 0

    def prepare(self, dataset) -> Payload:
        n = len(dataset)
        if hasattr(dataset, "ids"):
            ids = dataset.ids
        else:
            ids = stack_ids(dataset)
        if self.task == "clone" and n:
            ids = ids.reshape(-1, self.block_size or ids.shape[1] // 2)
        return Payload(np.ascontiguousarray(ids, dtype=np.int32), None, n)

    def population_rows(self, example, tokenizer, population, mode: int, block_size: int):
        from .host import MODE_RAW

        return example.mutant_ids(tokenizer, population, block_size,
                                  mode | (MODE_RAW if self.task == "authorship" else 0))

    def prepare_population(self, example, tokenizer, population, mode: int, block_size: int):
        ids, lens = self.population_rows(example, tokenizer, population, mode, block_size)
        return Payload(ids, lens, len(population))

    def prepare_pairs(self, ids1, lens1, ids2_row, len2) -> Payload:
        ids1 = np.asarray(ids1, np.int32)
        n, L = ids1.shape
        rows = np.stack([ids1, np.broadcast_to(np.asarray(ids2_row, np.int32), (n, L))], 1)
        return Payload(np.ascontiguousarray(rows.reshape(2 * n, L)), None, n)

    def submit(self, payloads, threshold: float = 0.5):
        """The asynchronous request API of Model, answered at once (host scoring)."""
        return ScoresReady(self.score_prepared(payloads, threshold))

    def score_prepared(self, payloads, threshold: float = 0.5):
        self.query += sum(p.n for p in payloads)
        live = [p for p in payloads if p.n]
        if not live:
            return [([], []) for _ in payloads]
        logits = np.asarray(self.score_fn(np.concatenate([p.ids for p in live])))
        out, off = [], 0
        for p in payloads:
            out.append(format_results(self.task, logits[off:off + p.n], threshold)
                       if p.n else ([], []))
            off += p.n
        return out

    def get_results(self, dataset, batch_size=None, threshold: float = 0.5):
        if len(dataset) == 0:
            return [], []
        return self.score_prepared([self.prepare(dataset)], threshold)[0]

    def dataset_from_texts(self, texts, tokenizer, args, label=0):
        from .utils import IdsDataset

        ids, lens = tokenizer.featurize(list(texts), args.block_size,
                                        raw=self.task == "authorship")
        return IdsDataset(ids, lens)

    def get_results_population(self, example, tokenizer, population, mode: int, block_size: int,
                               threshold: float = 0.5):
        if len(population) == 0:
            return [], []
        return self.score_prepared([self.prepare_population(example, tokenizer, population, mode,
                                                            block_size)], threshold)[0]
