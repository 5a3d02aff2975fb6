"""bench.py's host-side pieces without a GPU: the CPU baseline leg (the oracle on host cores, a tiny
sample here), the algorithmic-bytes model the roofline uses, and the committed PMC traffic lookup."""
import bench
from lsm.perf_model import step_bytes


def test_cpu_baseline_leg_small_sample():
    c = bench.CONFIGS[2]   # filter off: no HJ table needed
    args = bench.make_args(c)
    r = bench.cpu_baseline(args, None, None, ep=4, cores=2, envs_per_worker=1, steps=3)
    assert set(r) == {"value", "unit", "cores", "kind", "sample"}
    assert r["value"] > 0 and r["cores"] == 2 and r["kind"] == "port" and r["unit"] == "agent-steps/s"


def test_step_bytes_model():
    d = step_bytes(8, 2, "double_integrator", True, "reference")
    assert d["hbm_bytes"] == 31753 and d["gather_bytes"] == 5632 and not d["block"]
    d = step_bytes(64, 2, "double_integrator", True, "compact")
    assert d["block"] and d["E"] == 192 and d["hbm_bytes"] == 680897


def test_traffic_lookup_matches_workload():
    assert bench.load_traffic(3, 4096) is None or bench.load_traffic(3, 4096) > 1e8
    assert bench.load_traffic(3, 123) is None   # a different workload never borrows the number
