import functools
import pathlib
import sys

import pytest

ROOT = pathlib.Path(__file__).resolve().parents[1]
if str(ROOT) not in sys.path:
    sys.path.insert(0, str(ROOT))
import _apmc  # noqa: E402,F401  (registers the apmc_amd package)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a ROCm GPU (MI355X) and the built HIP engine")
    config.addinivalue_line("markers", "slow: longer CPU test")


@functools.lru_cache(maxsize=None)
def synthetic_sd(seed: int, head: str, num_labels: int = 1, with_mlm: bool = False,
                 out_std: float = 0.5):
    from apmc_amd.weights import synthetic_state_dict
    return synthetic_state_dict(seed=seed, head=head, num_labels=num_labels, with_mlm=with_mlm,
                                out_std=out_std)


@functools.lru_cache(maxsize=None)
def golden():
    import numpy as np
    return dict(np.load(ROOT / "tests" / "golden" / "encoder_golden.npz"))


@pytest.fixture(scope="session")
def gpu():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch.device("cuda:0")


@functools.lru_cache(maxsize=None)
def golden512():
    """transformers goldens at the attacks' block size (tests/golden/make_golden_encoder_512.py)."""
    import numpy as np
    return dict(np.load(ROOT / "tests" / "golden" / "encoder_golden_512.npz"))
