"""GPU: the metrics row (f)-4 beyond path packet counters — Mode S barrier-idle
timers (scheduler.c:380-389) and Event object counts (object_counter.c:90-230,
the Event type's new/free counts) — against the oracle's counters."""
import numpy as np
import pytest

from oracle import oracle as O
from shadow_amd import phold
from shadow_amd.engine import Engine

pytestmark = pytest.mark.gpu


def test_barrier_timers_account_every_partition():
    cfg = phold.c4_config(n_hosts=200_000, V=64)
    eng = Engine(cfg)
    eng.boot()
    eng.run(5)
    eng.barrier_timers(True)
    eng.run(40)
    t = eng.barrier_times()
    P = eng.geometry()["partitions"]
    busy, idle = t["busy_ns"].astype(np.float64), t["idle_ns"].astype(np.float64)
    assert len(busy) == len(idle) == P
    assert (busy > 0).all()
    # every round one partition is last (no wait); over 40 rounds every
    # partition spends busy + idle = the rounds' k_proc spans, minus its start lag
    span = busy + idle
    assert span.max() - span.min() < 0.25 * span.mean(), (span.min(), span.max())
    assert idle.min() < idle.max()
    eng.barrier_timers(False)
    assert len(eng.barrier_times()["busy_ns"]) == 0


@pytest.mark.parametrize("rounds", [1, 30, None])
def test_event_object_counts_match_oracle(rounds):
    """Event objects created / freed / live (object_counter.c:90-230 for the
    Event type): created = boot events + every event a send or a schedule
    made, freed = executed + dropped at endTime (scheduler.c:343-346); the
    oracle's counters give the same three numbers."""
    cfg = phold.c4_config(n_hosts=2000, V=16, end_time_s=0.5)
    eng = Engine(cfg)
    eng.boot()
    orc = O.Sim(cfg)
    orc.boot()
    if rounds is None:
        eng.run()
        orc.run()
    else:
        eng.run(rounds)
        orc.run(rounds)
    oc = eng.object_counts()
    st = orc.stats()
    # PHOLD: every send that passes the reliability draw makes an Event
    # (worker.c:268-287), also those then dropped at endTime or kept same-round
    assert oc["event_new"] == st["boots"] + st["sends"] - st["drop_reliability"]
    assert oc["event_free"] == st["pops"] + st["drop_endtime"]
    assert oc["event_live"] == st["pending"]
    assert oc["event_new"] - oc["event_free"] == oc["event_live"]
    if rounds is None:
        assert oc["event_live"] == 0
