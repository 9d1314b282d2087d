"""The synthetic workloads bench.py measures (BASELINE.json configs), by name.

  c4  configs[3]: PHOLD, 1M hosts x 16 events, V = 1024 log-normal latency
      (median 30 ms, sigma 0.9, min 1 ms), runahead 1 ms, weights rule, seed 1.
      BASELINE.json's metric is quoted on it; bench.py's default.
  c2  configs[1]: PHOLD, 10k hosts x 16 events on the uniform 50 ms full mesh
      (one vertex, src/test/phold/phold.test.shadow.config.xml:1-26).
  c5  configs[4]: gossip, 100k hosts, fanout 8, 64 messages 5 ms apart, lossy
      log-normal links over 256 vertices (the per-host RNG replay of the drop
      draws); the 2/4/8-GPU scaling config.

Each entry: the config builder, a description for the bench line's
config.workload, the default warmup / timed rounds (a window of the run where
the rounds are busy: gossip floods peak around rounds 100-240), where the
per-kernel durations come from (rounds after the timed region, or the timed
rounds replayed where the rounds change along the run), and the key of its
per-round oracle fixture in tests/golden/oracle_fixtures.json.  "replay": a
second engine replays the timed rounds with HIP events on every launch (events
inside the timed region itself added ~10 us of gaps per round).
"""
from __future__ import annotations

from . import phold

METRIC_C4 = "committed events/sec (whole node), 1M-host PHOLD at 1/2/4/8 MI355X; bit-exact"


def _c4(hosts):
    return phold.c4_config(n_hosts=hosts)


WORKLOADS = {
    "c4": dict(
        build=lambda hosts: _c4(hosts or 1_000_000),
        describe=lambda cfg: (f"PHOLD configs[3]: {cfg['n_hosts']} hosts x 16, V=1024 log-normal latency "
                              "(median 30 ms, sigma 0.9, min 1 ms), runahead 1 ms, weights rule, seed 1"),
        metric=lambda cfg: METRIC_C4,
        warmup=20, steps=200, cpu_warmup=12, kernel_timing="after",
        fixture=lambda cfg: "c4_1m" if cfg["n_hosts"] == 1_000_000 else None),
    "c2": dict(
        build=lambda hosts: phold.c2_config(),
        describe=lambda cfg: (f"PHOLD configs[1]: {cfg['n_hosts']} hosts x 16, uniform 50 ms full mesh "
                              "(one vertex), weights rule, seed 1 (50 ms windows: every event due each round)"),
        metric=lambda cfg: "committed events/sec (whole node), configs[1] 10k-host PHOLD on MI355X; bit-exact",
        warmup=10, steps=150, cpu_warmup=12, kernel_timing="replay",
        fixture=lambda cfg: "c2_rounds"),
    "c5": dict(
        build=lambda hosts: phold.c5_config(),
        describe=lambda cfg: (f"gossip configs[4]: {cfg['n_hosts']} hosts, fanout 8, 64 messages 5 ms apart, "
                              "V=256 log-normal latency (median 40 ms, min 2 ms), edge loss 0.5-5 %, seed 1"),
        metric=lambda cfg: ("committed events/sec (whole node), configs[4] 100k-host lossy gossip on "
                            "MI355X; bit-exact"),
        warmup=100, steps=120, cpu_warmup=100, kernel_timing="replay",
        fixture=lambda cfg: "c5_rounds"),
}


def get(name: str) -> dict:
    if name not in WORKLOADS:
        raise SystemExit(f"unknown workload {name!r}: one of {', '.join(WORKLOADS)}")
    return WORKLOADS[name]
