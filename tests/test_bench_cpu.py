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
    """record (read whole, hot part written) + outputs + HJ gathers (64 B per ordered
    agent pair + 256 B per ego for the 4-D table)."""
    d = step_bytes(8, 2, "double_integrator", True, "reference")
    assert d["gather_bytes"] == 64 * 8 * 7 + 256 * 8 == 5632 and not d["block"]
    assert d["hbm_bytes"] == d["state"] + d["outputs"] + d["gather_bytes"] == 37465   # state incl. actions
    assert step_bytes(8, 2, "double_integrator", False)["gather_bytes"] == 0
    d = step_bytes(64, 2, "double_integrator", True, "compact")
    assert d["block"] and d["E"] == 192 and d["hbm_bytes"] == 955409
    d = step_bytes(16, 2, "airtaxi", True, "reference")
    assert d["gather_bytes"] == 128 * 16 * 15 + 32 * 32 * 16


def test_timed_window_straddles_an_episode_boundary():
    for w, k, epl in ((5, 20, 250), (250, 1000, 250), (0, 1, 350), (3, 7, 10), (100, 2, 250)):
        pre = bench.timed_window(w, k, epl)
        assert pre >= w
        boundaries = [t for t in range(pre, pre + k) if (t + 1) % epl == 0]
        assert boundaries or k < 2, (w, k, epl, pre)


def test_multi_rank_launch_dry_run():
    """bench.py --gpus 2 starts two rank processes itself (no torchrun): each sees WORLD_SIZE=2, owns
    the env block [r * n, (r + 1) * n) and joins the episode-summary collective (gloo here)."""
    import json
    import subprocess
    import sys
    out = subprocess.run([sys.executable, bench.__file__, "--gpus", "2", "--dry-run", "--envs", "8",
                          "--steps", "20", "--warmup", "5"], capture_output=True, text=True, timeout=240)
    assert out.returncode == 0, out.stderr[-2000:]
    line = json.loads([ln for ln in out.stdout.splitlines() if ln.startswith("{")][-1])
    assert line["n_gpus"] == 2 and line["world_size"] == 2
    assert [(r["rank"], r["env_offset"], r["envs"]) for r in line["ranks"]] == [(0, 0, 8), (1, 8, 8)]
    assert line["max_over_ranks"] == 2.0
    # mean over both ranks' 16 envs of arange rows
    assert line["episode_summary"]["travel_time_mean"] == 60.0
    assert line["untimed_steps"] == 240


def test_world_size_must_match_gpus():
    import os
    import subprocess
    import sys
    env = dict(os.environ, WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    out = subprocess.run([sys.executable, bench.__file__, "--gpus", "2", "--dry-run"], capture_output=True,
                         text=True, timeout=120, env=env)
    assert out.returncode != 0 and "WORLD_SIZE" in (out.stderr + out.stdout)


def test_traffic_lookup_matches_workload_and_build():
    import json
    import os
    p = os.path.join(os.path.dirname(bench.__file__), "profiles", "pmc_traffic.json")
    e = json.load(open(p)).get("config3", {})
    bid = e.get("build_id")
    if bid:
        assert bench.load_traffic(3, e["num_envs"], bid) > 1e8
    assert bench.load_traffic(3, 123, bid) is None       # a different workload never borrows the number
    assert bench.load_traffic(3, 4096, "not-this-build") is None   # nor a different library build
