"""GPU: bench.py's single-GPU lines for every named workload (BASELINE.json
configs[1], [3], [4]): one JSON line with the metric, the per-kernel roofline of
both kernels, the end state matched against the oracle's per-round fixture, and
for the workloads whose rounds change along the run (c2, c5) kernel durations
from a second engine replaying the timed rounds, not from events inside them."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _bench(extra):
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--no-cpu-baseline", "--no-drop-in"] + extra,
                       capture_output=True, text=True, timeout=300, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [x for x in r.stdout.splitlines() if x.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    return json.loads(lines[0])


@pytest.mark.parametrize("wl,extra", [("c2", []), ("c5", []), ("c4", ["--steps", "20", "--warmup", "5"])])
def test_bench_workload_line(wl, extra):
    res = _bench(["--workload", wl] + extra)
    assert res["config"]["name"] == wl and res["n_gpus"] == 1 and res["value"] > 0
    assert res["metric"].endswith("; bit-exact")
    assert res["parity"]["match"] is True, res["parity"]
    rf = res["roofline"]
    assert set(rf["per_kernel"]) == {"k_proc", "k_scatter"}
    for k in ("k_proc", "k_scatter"):
        assert rf["per_kernel"][k]["avg_us"] > 0 and 0 < rf["per_kernel"][k]["frac"] < 1
    if wl in ("c2", "c5"):
        assert "replayed" in rf["timing_method"], rf["timing_method"]
        assert rf["timing_rounds"] == res["steps"]
