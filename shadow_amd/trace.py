"""Per-host pop traces: the parity artefact of the scheduler.

A committed event is one executed pop (worker.c:165-176); a host's pop
sequence under event_compare order (core/work/event.c:110-153) is what the
north star's "trace diff on identical configs and seeds" compares.  The trace
file holds one line per pop, hosts in index order, each host's pops in pop
order:

    # shadow-amd pop trace v1: host pos time_ns src_host src_event_id
    0 0 0 0 0
    0 1 1000000 17 3
    ...

`strip_log` restates the reference's own log normaliser
(src/tools/strip_log_for_compare.py:20-27: drop the first (timer) column and
every 0x… token) so Shadow logs can be diffed the same way.

CLI:
    python -m shadow_amd.trace diff A B        first divergence per host (exit 1 if any)
    python -m shadow_amd.trace strip IN OUT    the reference log stripper
    python -m shadow_amd.trace convert IN OUT  .npy <-> text
"""
from __future__ import annotations

import sys

import numpy as np

from ._lib import TRACE_DTYPE

HEADER = "# shadow-amd pop trace v1: host pos time_ns src_host src_event_id"


def _fmix64(z: np.ndarray) -> np.ndarray:
    z = z ^ (z >> np.uint64(33))
    z = z * np.uint64(0xFF51AFD7ED558CCD)
    z = z ^ (z >> np.uint64(33))
    z = z * np.uint64(0xC4CEB9FE1A85EC53)
    return z ^ (z >> np.uint64(33))


def state_fingerprint(first_host: int, digest, pops, rng, ev) -> int:
    """Order-independent 64-bit fingerprint of per-host end state (trace digest,
    pop count, rand_r state, srcHostEventID counter) — a checksum of checksums.
    Additive over hosts (mod 2^64), so shards' fingerprints sum to the
    unsharded one; position-sensitive through the host index."""
    n = len(digest)
    if n == 0:
        return 0
    with np.errstate(over="ignore"):
        h = np.arange(first_host, first_host + n, dtype=np.uint64)
        z = _fmix64(np.asarray(digest, np.uint64) + (h + np.uint64(1)) * np.uint64(0x9E3779B97F4A7C15))
        z = _fmix64(z ^ np.asarray(pops, np.uint64))
        z = _fmix64(z ^ np.asarray(rng, np.uint64))
        z = _fmix64(z ^ np.asarray(ev, np.uint64))
        return int(z.sum(dtype=np.uint64))


def canonical(trace: np.ndarray) -> np.ndarray:
    """Hosts in index order, each host's pops in pop order."""
    t = np.asarray(trace)
    if t.dtype != TRACE_DTYPE:
        t = t.astype(TRACE_DTYPE)
    return np.sort(t, order=["host", "pos"], kind="stable")


def write(trace: np.ndarray, path: str) -> int:
    """Write a trace (text, or binary when path ends in .npy); returns the pop count."""
    t = canonical(trace)
    if path.endswith(".npy"):
        np.save(path, t, allow_pickle=False)
        return len(t)
    with open(path, "w") as f:
        f.write(HEADER + "\n")
        cols = np.stack([t["host"].astype(np.uint64), t["pos"], t["time"], t["src"].astype(np.uint64),
                         t["seq"]], axis=1)
        np.savetxt(f, cols, fmt="%d")
    return len(t)


def read(path: str) -> np.ndarray:
    if path.endswith(".npy"):
        return canonical(np.load(path, allow_pickle=False))
    with open(path) as f:
        first = f.readline().rstrip("\n")
        if first != HEADER:
            raise ValueError(f"{path}: not a pop trace (header {first!r})")
        rows = np.loadtxt(f, dtype=np.uint64, ndmin=2)
    out = np.zeros(len(rows), TRACE_DTYPE)
    if len(rows):
        out["host"], out["pos"], out["time"], out["src"], out["seq"] = (rows[:, i] for i in range(5))
    return canonical(out)


def diff(a: np.ndarray, b: np.ndarray, max_report: int = 10) -> dict:
    """Compare two traces host by host.  Returns the pop counts, the number of
    hosts whose sequences differ and, for the first max_report of them, the
    first differing position with both records (None where a side has no pop)."""
    a, b = canonical(a), canonical(b)
    keys = ("time", "src", "seq")
    res = {"pops_a": int(len(a)), "pops_b": int(len(b)), "hosts_differing": 0, "first": []}
    hosts = np.union1d(np.unique(a["host"]), np.unique(b["host"]))
    a0, a1 = np.searchsorted(a["host"], hosts, "left"), np.searchsorted(a["host"], hosts, "right")
    b0, b1 = np.searchsorted(b["host"], hosts, "left"), np.searchsorted(b["host"], hosts, "right")
    for k, h in enumerate(hosts.tolist()):
        sa, sb = a[a0[k]:a1[k]], b[b0[k]:b1[k]]
        n = min(len(sa), len(sb))
        neq = np.zeros(n, bool)
        for f in keys:
            neq |= sa[f][:n] != sb[f][:n]
        if not neq.any() and len(sa) == len(sb):
            continue
        res["hosts_differing"] += 1
        if len(res["first"]) < max_report:
            pos = int(np.argmax(neq)) if neq.any() else n
            rec = lambda s: None if pos >= len(s) else {f: int(s[f][pos]) for f in keys}  # noqa: E731
            res["first"].append({"host": int(h), "pos": pos, "a": rec(sa), "b": rec(sb)})
    res["identical"] = res["hosts_differing"] == 0
    return res


def strip_log(lines):
    """src/tools/strip_log_for_compare.py:20-27: per line, drop the first
    (timer) column and every token starting with 0x; tokens re-joined with a
    trailing space each."""
    for line in lines:
        parts = line.strip().split()[1:]
        yield "".join(p + " " for p in parts if not p.startswith("0x")) + "\n"


def main(argv=None) -> int:
    argv = sys.argv[1:] if argv is None else argv
    if len(argv) == 3 and argv[0] == "diff":
        r = diff(read(argv[1]), read(argv[2]))
        print(f"pops: {r['pops_a']} vs {r['pops_b']}; hosts differing: {r['hosts_differing']}")
        for d in r["first"]:
            print(f"  host {d['host']} pos {d['pos']}: {d['a']} vs {d['b']}")
        return 0 if r["identical"] else 1
    if len(argv) == 3 and argv[0] == "strip":
        n = 0
        with open(argv[1]) as fi, open(argv[2], "w") as fo:
            for out in strip_log(fi):
                fo.write(out)
                n += 1
        print(f"Done! Processed {n} lines.", file=sys.stderr)
        return 0
    if len(argv) == 3 and argv[0] == "convert":
        print(write(read(argv[1]), argv[2]), "pops")
        return 0
    print(__doc__.split("CLI:")[1], file=sys.stderr)
    return 2


if __name__ == "__main__":
    sys.exit(main())
