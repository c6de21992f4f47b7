"""Class-level multi-GPU path: WaveletAttribution1D/2D/3D(..., dist=True) at world
size 2 (gloo, both ranks on cuda:0) vs the unsharded call, for sample / step sharding (ragged,
IG trapezoid weights, 3D legacy weights, a rank with no samples) and batch sharding (all-reduce MAX
of the batch-global maxima, rows gathered). Run by tests/conftest.py as child processes before
the pytest process touches the GPU; this test reads their report."""
import pytest

pytestmark = pytest.mark.gpu


def test_classes_sharded_world2_match_unsharded(dist_world2):
    assert dist_world2 is not None, "world-2 run not launched (run the GPU suite with -m gpu)"
    assert dist_world2["rc"] == 0 and dist_world2["result"], dist_world2["log"]
    res = dist_world2["result"]
    print(res)
    assert len(res) >= 10
    for name, r in res.items():
        assert "error" not in r, (name, r.get("error"))
        assert r["shape_ok"], name
        # partial sums in another order (fp64 frames, fp32 weighted trapz) and per-rank model batches
        assert r["err"] <= 2e-5, (name, r["err"])
        # parameter .grad: the ranks' increments all-reduced once per call (relative to max |grad|)
        assert r.get("grad_err", 1e9) <= 1e-4, (name, r.get("grad_err"))
