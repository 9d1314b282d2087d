"""shadow_amd — MI355X-native event-scheduling core for Shadow 1.14.

The hot path (per-host event queues, event_compare order, barrier bump, packet
delivery time / drop resolution, MIN next-event time and runahead windows)
runs as hand-written gfx950 HIP kernels in libshadowgpu.so behind a plain
C-ABI (include/shadowgpu.h).  This package is the thin host-side mirror:

  shadow_amd.phold    PHOLD workload configs built with the reference arithmetic
  shadow_amd.engine   the HBM-resident round engine (one shard)
  shadow_amd.dist     one process per GPU, hosts sharded, RCCL exchange
  shadow_amd.policy   the `gpu` SchedulerPolicy (push/pop/getNextTime) mirror
"""
from . import _lib  # noqa: F401

__all__ = ["_lib"]
