"""The bench's committed inputs, on the CPU: every workload's PMC profile (the
`roofline.traffic` the bench line quotes, bench.py PMC_JSON) exists under
profiles/, parses, and carries both kernels of a round with the corrected and
the as-counted traffic."""
import importlib.util
import os

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _bench():
    spec = importlib.util.spec_from_file_location("bench_under_test", os.path.join(ROOT, "bench.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def test_pmc_profile_for_every_workload():
    b = _bench()
    for wl in ("c4", "c2", "c5"):
        for kernel in ("k_proc", "k_scatter"):
            traffic, lower, src = b.pmc_traffic(wl, 1_000_000, kernel)
            assert src is not None, (wl, kernel)
            assert src.startswith("profiles/") and os.path.exists(os.path.join(ROOT, src)), src
            # FETCH_SIZE doubled (MI355X_MICROARCH.md) against as counted
            assert 0 < lower < traffic, (wl, kernel, lower, traffic)


def test_pmc_profile_only_for_the_measured_size():
    # configs[3]'s profile is of the 1M-host bench; a resized run quotes none
    assert _bench().pmc_traffic("c4", 125_000) == (None, None, None)
