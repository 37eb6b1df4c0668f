"""CPU: the pure-host helpers bench.py builds its line from (no device work here)."""
import json
import os
import sys

import pytest

from conftest import ROOT

sys.path.insert(0, str(ROOT))
import bench  # noqa: E402


def test_attention_summary_counts_the_eleven_full_layers():
    """4·L²·64 FLOP per (sequence, head) for S = QKᵀ and PV, 12 heads, 11 full layers, over the
    time of every attention launch of the step (the CLS-only layer's time included)."""
    B, L, steps, peak = 64, 512, 10, 838.9
    per_layer = 4.0 * L * L * 64 * 12 * B
    ms_total = 18.73  # 1.873 ms per step
    a = bench.attention_summary(ms_total, 12 * steps, steps, B, L, peak, "here")
    assert a["launches_per_step"] == 12
    assert a["full_layer_algorithmic_gflop"] == round(per_layer / 1e9, 2) == 51.54
    tf = 11 * per_layer / (ms_total / steps) / 1e9
    assert a["algorithmic_tflops"] == round(tf, 2)
    assert a["frac_of_peak"] == round(tf / peak, 4)
    assert a["timing"].endswith("here")
    assert bench.attention_summary(0.0, 0, steps, B, L, peak, "here") is None


def test_single_stream_engine_is_a_config_not_the_environment(monkeypatch):
    """The roofline / attention passes build their engine with ae_config.streams = one stream
    (the product library reads no AE_* environment) and leave the environment untouched."""
    import apmc_amd.engine as eng_mod
    seen = []

    class FakeEngine:
        def __init__(self, *a, **kw):
            seen.append(kw)

    monkeypatch.setattr(eng_mod, "Engine", FakeEngine)

    class Dev:
        index = 0

    before = dict(os.environ)
    bench.single_stream_engine({}, "f32x3", Dev())
    assert seen[-1]["streams"] == "one" and not seen[-1].get("tools")
    assert dict(os.environ) == before


def test_pmc_traffic_comes_from_the_newest_round():
    """roofline.traffic: the committed FETCH / WRITE summary of the newest round for the
    precision (r<round><letters>_ ordering: r4z after r4k after r3ap after r3z)."""
    import re

    def order(f):
        m = re.match(r"r(\d+)([a-z]*)_", f.name)
        return (int(m.group(1)), len(m.group(2)), m.group(2))
    split = [f for f in (ROOT / "profiles").glob("r*pmc*ffn1*.json")
             if json.loads(f.read_text()).get("precision") == "f32x3"]
    if not split:
        pytest.skip("no f32x3 PMC summary committed")
    newest = max(split, key=order)
    want = float(json.loads(newest.read_text())["hbm_bytes_per_launch"])
    assert bench.pmc_traffic_per_launch("f32x3") == want
