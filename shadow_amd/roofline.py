"""Algorithmic bytes per kernel launch and the HBM roofline fraction
(DESIGN.md §3), shared by bench.py's one-GPU line and the
N > 1 line of shadow_amd.dist.bench."""
from __future__ import annotations

HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md chip table (spec)

# k_proc: 64 B per committed event (24 B popped record + 24 B new record + 8 B
# delay + 4 B threshold + 4 B index) + 24 B per active host (RNG and sequence state)
ALG_BYTES_PER_EVENT = 64
ALG_BYTES_PER_ACTIVE_HOST = 24
# k_scatter: every record it moves is read once and written once, 16 B each way:
# staged events into the calendar (insert role, due ones routed straight to their
# partition), the new window's calendar events into the host partitions (gather
# role) and, with several shards, received events routed into partitions; the
# rmin and refill roles' few KB are not counted
ALG_BYTES_PER_MOVE = 32


def proc_bytes(pops: int, active_host_rounds: int) -> int:
    return ALG_BYTES_PER_EVENT * pops + ALG_BYTES_PER_ACTIVE_HOST * active_host_rounds


def scatter_bytes(moves: dict) -> int:
    return ALG_BYTES_PER_MOVE * (moves["emitted"] + moves["gathered"] + moves.get("received", 0))


def kernel_line(alg_bytes_per_launch: float, avg_s: float) -> dict:
    """Algorithmic bytes per launch over the average launch time, against HBM peak."""
    ach = alg_bytes_per_launch / avg_s / 1e9 if avg_s > 0 else 0.0
    return {"avg_us": avg_s * 1e6, "alg_bytes_per_launch": alg_bytes_per_launch, "achieved": ach,
            "frac": ach / HBM_PEAK_GBS}
