"""GPU, two processes: the multi-rank engine path of shadow_amd.dist with real
EngineShards, the way the N > 1 bench runs it (one process per rank, the step
protocol driven by dist.run / run_until_round / finish_round, one all-to-all per
step).  Both ranks share GPU 0, so the exchange goes over gloo through host
memory (RCCL needs one GPU per rank; the RCCL native loop is covered at world 1
in test_gpu_sharded.py).  This replaces the execute barrier and MIN of
scheduler.c:386-398 and master.c:450-480 with the header-carried window.

  configs[3] at 1M hosts, 2 x 500k, against the oracle's per-round fixture
  configs[4] gossip, 100k hosts, the whole run, against its whole-run fixture
  bench.py --gpus 2 --same-device --dist-backend gloo: parity.match true
The first two also run with the blocks stored straight into the peer's
exchange region (sg_xlink), the exchange the N > 1 bench takes by default.
"""
import json
import os
import socket
import subprocess
import sys

import pytest
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
FIX = json.load(open(os.path.join(ROOT, "tests", "golden", "oracle_fixtures.json")))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, kind, xcap, stop_round, q, xlink=False):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    sys.path.insert(0, ROOT)
    import torch
    import torch.distributed as dist
    from shadow_amd import dist as D
    from shadow_amd import phold
    try:
        dist.init_process_group("gloo", rank=rank, world_size=world)
        cfg = phold.c4_config(n_hosts=1_000_000) if kind == "c4" else phold.c5_config()
        sh = D.EngineShard(cfg, rank, world, 0, exchange_cap=xcap)
        sh.boot()
        if xlink:  # every step from here through the xGMI exchange regions (sg_xlink)
            sh.enable_xlink()
        if stop_round:
            D.run_until_round(sh, world, stop_round, check_every=4)
            st = D.finish_round(sh, world)
        else:
            D.run(sh, world, check_every=8)
            st = sh.stats()
        fp = sh.fingerprint()
        sh.close_native()  # collective: raises if an exchange wait timed out
        q.put((rank, None, st, fp))
        dist.barrier()
        dist.destroy_process_group()
    except Exception as exc:  # reported by the parent
        import traceback
        q.put((rank, traceback.format_exc(), None, None))
        raise


def _run(kind, world, xcap, stop_round=0, timeout=240, xlink=False):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_worker, args=(r, world, port, kind, xcap, stop_round, q, xlink))
          for r in range(world)]
    for p in ps:
        p.start()
    try:
        res = [q.get(timeout=timeout) for _ in range(world)]
    finally:
        for p in ps:
            p.join(30)
            if p.is_alive():
                p.kill()
    errs = [r[1] for r in res if r[1]]
    assert not errs, errs[0]
    for p in ps:
        assert p.exitcode == 0
    return sorted(res, key=lambda x: x[0])


@pytest.mark.parametrize("xcap", [None, 8192])
@pytest.mark.parametrize("xlink", [False, True], ids=["gloo", "xgmi"])
def test_c4_1m_two_processes(xcap, xlink):
    """configs[3]: 1M hosts as 2 ranks of 500k; default blocks and 8192-row
    blocks (drain steps); the blocks exchanged over gloo or stored straight
    into the peer's exchange region (sg_xlink: IPC-mapped uncached memory,
    arrival counters, parity buffers); the state at the round boundary after
    round 24 against the oracle's fixture for that round."""
    res = _run("c4", 2, xcap, stop_round=24, xlink=xlink)
    st = [r[2] for r in res]
    r = st[0]["rounds"]
    assert r >= 24 and all(x["rounds"] == r and x["phase"] == 0 for x in st)
    assert all(x["overflow"] == 0 for x in st), [hex(x["overflow"]) for x in st]
    rows = {row[0]: row for row in FIX["c4_1m"]["rounds"]}
    assert sum(x["pops"] for x in st) == rows[r][1]
    assert (sum(x[3] for x in res) & ((1 << 64) - 1)) == rows[r][2]
    for x in st:
        assert (x["window_start"], x["window_end"]) == (rows[r][3], rows[r][4])
    if xcap:
        assert st[0]["exchange_steps"] > r  # drain steps happened


def test_c4_1m_two_processes_xgmi_fenced(monkeypatch):
    """The xGMI exchange with the system-scope release before each arrival, as
    it runs between GPUs (SG_XFENCE=1; ranks on one device default to the
    unfenced arrival): configs[3] at round 24 against the fixture."""
    monkeypatch.setenv("SG_XFENCE", "1")  # the spawned ranks inherit it
    res = _run("c4", 2, None, stop_round=24, xlink=True)
    st = [r[2] for r in res]
    r = st[0]["rounds"]
    rows = {row[0]: row for row in FIX["c4_1m"]["rounds"]}
    assert sum(x["pops"] for x in st) == rows[r][1]
    assert (sum(x[3] for x in res) & ((1 << 64) - 1)) == rows[r][2]


@pytest.mark.parametrize("xlink", [False, True], ids=["gloo", "xgmi"])
def test_c5_gossip_two_processes(xlink):
    res = _run("c5", 2, 8192, xlink=xlink)
    st = [r[2] for r in res]
    fx = FIX["c5"]["stats"]
    assert all(x["overflow"] == 0 for x in st)
    for k in ("pops", "boots", "sends", "drop_reliability", "drop_endtime", "bumped", "same_round"):
        assert sum(x[k] for x in st) == fx[k], k
    for x in st:
        assert x["rounds"] == fx["rounds"] and x["done"]
    assert (sum(x[3] for x in res) & ((1 << 64) - 1)) == FIX["c5"]["fingerprint"]


def _self_launched_bench(n, extra, timeout):
    env = dict(os.environ)
    env.pop("WORLD_SIZE", None)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", str(n), "--same-device",
                        "--dist-backend", "gloo"] + extra,
                       capture_output=True, text=True, timeout=timeout, env=env, cwd=ROOT)
    # rank 0's traceback, not the launcher's summary around it
    tb = "\n".join(x for x in r.stderr.splitlines() if x.startswith("[rank0]"))
    assert r.returncode == 0, (tb or r.stderr[-3000:]) + r.stdout[-2000:]
    lines = [x for x in r.stdout.splitlines() if x.startswith("{")]
    assert len(lines) == 1, r.stdout[-3000:]
    res = json.loads(lines[0])
    assert res["n_gpus"] == n and res["value"] > 0
    assert res["parity"]["match"] is True, res["parity"]
    assert res["metric"].endswith("; bit-exact")
    # the N > 1 line's roofline: every rank's k_proc / k_scatter fraction and
    # the exchange's bytes per step (north_star: a fraction per kernel at N > 1)
    rf = res["roofline"]
    assert rf["bound"] == "hbm" and 0 < rf["frac"] < 1 and rf["kernel"] == "k_proc"
    assert len(rf["per_rank"]) == n
    for pr in rf["per_rank"]:
        for k in ("k_proc", "k_scatter"):
            assert pr[k]["avg_us"] > 0 and pr[k]["alg_bytes_per_launch"] > 0 and 0 < pr[k]["frac"] < 1, (k, pr)
        assert pr["exchange"]["bytes_per_step"] > 0
    assert set(rf["per_kernel"]) == {"k_proc", "k_scatter"}
    return res


@pytest.mark.parametrize("exchange", ["xgmi", "rccl"])
def test_bench_two_ranks_self_launched(exchange):
    """`python bench.py --gpus 2` with no launcher of its own (bench.py starts
    torch.distributed.run), ranks on GPU 0: one JSON line with the two ranks'
    events and parity.match true, the timed steps exchanging blocks by xGMI
    peer stores (sg_xlink) or, with --exchange rccl on a gloo group, by
    gloo's all-to-all."""
    res = _self_launched_bench(2, ["--steps", "20", "--warmup", "10", "--exchange", exchange], 300)
    want = "xGMI" if exchange == "xgmi" else "gloo"
    assert res["config"]["exchange"].startswith(want), res["config"]


@pytest.mark.timeout(600)
def test_bench_eight_ranks_self_launched():
    """The driver's N = 8 command, rehearsed: `bench.py --gpus 8` starting its
    own torch.distributed.run, 8 ranks of 125k hosts of configs[3] (all on GPU
    0, gloo in place of RCCL, which refuses two ranks on one device): the
    parity point matches the oracle's per-round fixture and the line carries
    8 per-rank roofline rows."""
    res = _self_launched_bench(8, ["--steps", "20", "--warmup", "5", "--kernel-rounds", "10"], 600)
    assert res["config"]["n_hosts"] == 1_000_000 and res["config"]["name"] == "c4"
    # the default exchange (auto) took the xGMI link after its self-test
    assert res["config"]["exchange"].startswith("xGMI"), res["config"]


@pytest.mark.timeout(600)
def test_bench_two_ranks_gossip_workload():
    """`bench.py --gpus 2 --workload c5`: configs[4]'s lossy gossip sharded over
    two ranks (its 2/4/8-GPU scaling config is one flag away), checked against
    the per-round fixture of the gossip run."""
    res = _self_launched_bench(2, ["--workload", "c5", "--steps", "30", "--warmup", "100",
                                   "--kernel-rounds", "10"], 600)
    assert res["config"]["name"] == "c5" and res["config"]["n_hosts"] == 100_000
