"""tools/rehearsal_check.py: the assertions kept on the N = 8 rehearsal JSONs."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools"))

from rehearsal_check import check  # noqa: E402


def _rec(**over):
    rec = {"n_gpus": 8, "steps": 4, "warmup": 2, "params_finite": True, "staleness_hist": [16, 80],
           "autotune_source": {"local": 0, "claimed": 70, "peer": 490, "file": 0},
           "config": {"ps_mode": "async", "async_fallback": None, "async_xfer": "kernel", "async_xfer_fallback": None,
                      "worker_ranks": list(range(8)), "ps_shards": 2, "staleness_bound": 1}}
    for k, v in over.items():
        if k in rec["config"]:
            rec["config"][k] = v
        else:
            rec[k] = v
    return rec


def test_good_record_passes():
    assert check(_rec(), 8) == []


def test_each_failure_is_named():
    assert any("fell back" in b for b in check(_rec(ps_mode="collective"), 8))
    assert any("transport" in b for b in check(_rec(async_xfer="hipMemcpyAsync"), 8))
    assert any("autotune" in b for b in check(_rec(autotune_source={"local": 3, "claimed": 0, "peer": 0}), 8))
    assert any("histogram total" in b for b in check(_rec(staleness_hist=[16, 79]), 8))
    assert any("beyond the bound" in b for b in check(_rec(staleness_hist=[16, 78, 0, 2]), 8))
    assert any("non-finite" in b for b in check(_rec(params_finite=False), 8))
    assert any("n_gpus" in b for b in check(_rec(), 4))
