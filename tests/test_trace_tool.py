"""CPU: the pop-trace writer/diff tool (shadow_amd.trace) and the restated
log stripper, on oracle traces of the survey's probe workload."""
import numpy as np
import pytest

from shadow_amd import phold
from shadow_amd import trace as T
from oracle import oracle as O


def _trace(cfg, mode):
    s = O.Sim(cfg, mode=mode, trace_capacity=1 << 21)
    s.boot()
    if mode == O.MODE_SERIAL:
        s.run_serial()
    else:
        s.run()
    return s.trace()


@pytest.fixture(scope="module")
def probe5():
    cfg = phold.probe_config(n_hosts=300, jump_ms=5, end_time_s=0.5)
    return _trace(cfg, O.MODE_HOST), _trace(cfg, O.MODE_SERIAL)


def test_serial_equals_host_single_at_min_latency_window(probe5):
    # with the window = min latency, serial and host_single traces agree
    host, serial = probe5
    r = T.diff(host, serial)
    assert r["identical"] and r["pops_a"] == r["pops_b"] > 1000


def test_bump_shows_as_first_divergence():
    cfg = phold.probe_config(n_hosts=300, jump_ms=10, end_time_s=0.5)
    r = T.diff(_trace(cfg, O.MODE_HOST), _trace(cfg, O.MODE_SERIAL))
    assert not r["identical"] and r["hosts_differing"] > 0
    d = r["first"][0]
    assert d["a"] is None or d["b"] is None or d["a"] != d["b"]


def test_roundtrip_text_and_npy(tmp_path, probe5):
    host, _ = probe5
    for name in ("t.txt", "t.npy"):
        p = str(tmp_path / name)
        assert T.write(host[::-1], p) == len(host)  # canonical order on write
        back = T.read(p)
        assert np.array_equal(back, T.canonical(host))
    with open(tmp_path / "t.txt") as f:
        assert f.readline().strip() == T.HEADER


def test_diff_reports_swapped_and_missing_pops(probe5):
    host, _ = probe5
    t = T.canonical(host).copy()
    h = int(t["host"][100])
    idx = np.nonzero(t["host"] == h)[0]
    a, b = idx[1], idx[2]
    t[["time", "src", "seq"]][[a, b]] = t[["time", "src", "seq"]][[b, a]]
    r = T.diff(host, t)
    assert r["hosts_differing"] == 1 and r["first"][0]["host"] == h and r["first"][0]["pos"] == 1
    r = T.diff(host, np.delete(T.canonical(host), idx[-1]))
    assert r["hosts_differing"] == 1 and r["first"][0]["b"] is None


def test_cli(tmp_path, probe5):
    host, serial = probe5
    pa, pb = str(tmp_path / "a.txt"), str(tmp_path / "b.npy")
    T.write(host, pa)
    T.write(serial, pb)
    assert T.main(["diff", pa, pb]) == 0
    T.write(np.delete(T.canonical(serial), 0), pb)
    assert T.main(["diff", pa, pb]) == 1
    assert T.main(["bogus"]) == 2


def test_strip_log_matches_reference_rule(tmp_path):
    # strip_log_for_compare.py:20-27: drop column 1 and 0x tokens, "tok " joined
    lines = ["00:00:01.000 [thread-1] 0x7f00aa [message] [host:1.2.3.4] event 0xdead done\n",
             "t2\n", "\n"]
    out = list(T.strip_log(lines))
    assert out == ["[thread-1] [message] [host:1.2.3.4] event done \n", "\n", "\n"]
    src, dst = tmp_path / "in.log", tmp_path / "out.log"
    src.write_text("".join(lines))
    assert T.main(["strip", str(src), str(dst)]) == 0
    assert dst.read_text() == "".join(out)
