"""Round time of the 1M-host C4 engine without the bench's parity check (for
experimental variant libraries whose state intentionally differs):
SG_LIB=libshadowgpu_<v>.so python tools/quick_time.py [rounds] (QT_HOSTS: host count)."""
import os
import sys
import time

sys.path.insert(0, ".")
from shadow_amd import phold  # noqa: E402
from shadow_amd.engine import Engine  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 200
eng = Engine(phold.c4_config(n_hosts=int(os.environ.get("QT_HOSTS", 1_000_000))))
eng.boot()
eng.run(20)
eng.set_timing(True, ["process", "insert", "plan"])
eng.enqueue_rounds(50)
eng.sync()
kt = eng.kernel_times()
eng.set_timing(False)
eng.sync()
t = time.perf_counter()
eng.enqueue_rounds(n)
eng.sync()
dt = (time.perf_counter() - t) / n * 1e6
print("us/round %.2f  " % dt + "  ".join("%s %.2f" % (k, ms * 1e3 / c) for k, (ms, c) in kt.items() if c))
