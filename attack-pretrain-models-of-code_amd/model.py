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
        self.block_size = getattr(args, "block_size", None)

    # the reference calls model.eval()/.to(device) around get_results; keep them as no-ops
    def eval(self):
        return self

    def to(self, *a, **k):
        return self

    def _score_ids(self, ids: np.ndarray, lens: np.ndarray | None = None) -> np.ndarray:
        import torch

        pad = self.engine.pad_id
        if self.task == "clone":
            # model.py:44 input_ids.view(-1, block_size): each row holds code1 | code2
            bs = self.block_size or ids.shape[1] // 2
            ids = ids.reshape(-1, bs)
        n = ids.shape[0]
        outs = []
        step = self.max_rows_per_launch
        for s in range(0, n, step):
            chunk = np.ascontiguousarray(ids[s:s + step], dtype=np.int32)
            cl = (chunk != pad).sum(axis=1).astype(np.int32) if lens is None or \
                self.task == "clone" else np.ascontiguousarray(lens[s:s + step], dtype=np.int32)
            dev = torch.from_numpy(chunk).to(f"cuda:{self.engine.device}", non_blocking=False)
            outs.append(self.engine.score(dev, cl))
        return torch.cat(outs, 0).cpu().numpy() if len(outs) > 1 else outs[0].cpu().numpy()

    def get_results(self, dataset, batch_size=None, threshold: float = 0.5):
        """(probs, pred_labels) exactly as the reference's get_results of this task."""
        self.query += len(dataset)
        if len(dataset) == 0:
            return [], []
        if hasattr(dataset, "ids") and hasattr(dataset, "lens"):  # utils.IdsDataset fast path
            logits = self._score_ids(dataset.ids, dataset.lens)
        else:
            logits = self._score_ids(stack_ids(dataset))
        return self._format(logits, threshold)

    def dataset_from_texts(self, texts, tokenizer, args, label=0):
        """Mutant texts -> the dataset get_results consumes (convert_code_to_features of every
        text, CodeXGLUE/Defect-detection/code/attacker.py:38-45, batched in the host library)."""
        from .utils import IdsDataset

        ids, lens = tokenizer.featurize(list(texts), args.block_size)
        return IdsDataset(ids, lens)

    def get_results_population(self, example, tokenizer, population, mode: int, block_size: int,
                               threshold: float = 0.5):
        """Score a population of chromosomes of one program (len(population) queries).

        The host library reduces every mutant to its word-id sequence (the mutant text is built
        exactly as get_example / get_example_batch would); ae_splice assembles the [n, block]
        ids on the GPU from the example's word table; the engine scores them.  Identical ids to
        featurising the mutant texts (tests/test_host.py, tests/test_engine_gpu.py)."""
        import torch

        from .engine import splice

        n = len(population)
        self.query += n
        if n == 0:
            return [], []
        word_tok, word_off, mut_words, mut_off, lens = example.mutant_words(
            tokenizer, population, block_size, mode)
        dev = f"cuda:{self.engine.device}"
        ids, _ = splice(torch.from_numpy(word_tok).to(dev), torch.from_numpy(word_off).to(dev),
                        torch.from_numpy(mut_words).to(dev), torch.from_numpy(mut_off).to(dev),
                        n, block_size, tokenizer.cls_token_id, tokenizer.sep_token_id,
                        tokenizer.pad_token_id)
        logits = self.engine.score(ids, lens).cpu().numpy()
        return self._format(logits, threshold)

    def _format(self, logits, threshold: float = 0.5):
        if self.task == "devign":
            # model.py:56-57
            probs = [[1 - prob[0], prob[0]] for prob in logits]
            pred_labels = [1 if label else 0 for label in logits[:, 0] > 0.5]
        elif self.task == "clone":
            # Clone-detection-BigCloneBench/code/model.py:81-82
            probs = logits
            pred_labels = [0 if first_softmax > threshold else 1 for first_softmax in logits[:, 0]]
        else:
            # Authorship-Attribution/code/model.py:84-89
            probs = logits
            pred_labels = [np.argmax(logit) for logit in logits]
        return probs, pred_labels
