"""The multi-GPU step's prediction (DESIGN §5 "Predicted N-GPU step") on the CPU: the
committed one-GPU component measurements (profiles/r06_multi_model.json, dev/multi_model.py) and
bench.predict_multi_step, which the N > 1 bench line reports as multi.predicted_ms_per_step."""
import json
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parent.parent
MODEL = ROOT / "profiles" / "r06_multi_model.json"


@pytest.fixture(scope="module")
def bench():
    sys.path.insert(0, str(ROOT))
    import bench as b
    return b


@pytest.fixture(scope="module")
def model():
    return json.loads(MODEL.read_text())


def test_model_has_every_component(model):
    assert model["keys_per_gpu"] == 1 << 30 and model["k_bits"] == 8
    assert model["single_gpu_sort_ms"] > 0 and model["world1_full_protocol_ms"]["ms_plan"] > 0
    for w in ("2", "4", "8"):
        row = model["worlds"][w]
        assert row["partition_ms"] > 0 and row["overlap_partition_ms"] > 0 and row["local_sort_ms"] > 0
        assert row["bytes_per_link"] == (1 << 30) // int(w) * 4
        # distinct keys: one plain splitter per rank boundary (hot-only equal-key buckets)
        assert row["buckets"] == int(w) and row["overlap_buckets"] == 2 * int(w)
    ov = model["overlap"]["plans"]["default"]
    assert ov["alone_ms"] > 0 and ov["contended"]["link_153GBs_wgs8"]["sort_ms"] > ov["alone_ms"]


def test_prediction_by_hand(bench, model):
    """world 8 without halves: plan + 3 all-gather latencies + partition + 512 MiB over one link + local sort."""
    row = model["worlds"]["8"]
    want = (model["world1_full_protocol_ms"]["ms_plan"] + 3 * model["allgather_latency_ms_assumed"]
            + row["partition_ms"] + row["bytes_per_link"] / 153e9 * 1e3 + row["local_sort_ms"])
    assert bench.predict_multi_step(model, 8, 1, 153.0) == pytest.approx(want)
    assert bench.predict_multi_step(model, 1, 1, 153.0) == model["single_gpu_sort_ms"]
    assert bench.predict_multi_step(model, 3, 1, 153.0) is None  # (not measured)


def test_prediction_orders(bench, model):
    """Slower links predict slower steps; the automatic overlap (2 <= N <= 8, rsort.h) predicts faster steps
    at every N it runs at, on both link rates."""
    for w in (2, 4, 8):
        for h in (1, 2):
            assert bench.predict_multi_step(model, w, h, 64.0) > bench.predict_multi_step(model, w, h, 153.0)
        for link in (64.0, 153.0):
            assert bench.predict_multi_step(model, w, 2, link) < bench.predict_multi_step(model, w, 1, link)
    main, detail = bench.multi_prediction(8, 2)
    assert main == pytest.approx(bench.predict_multi_step(model, 8, 2, 153.0), abs=1e-3)
    assert detail["halves"] == 2 and detail["link_64GBs_ms"] > main
