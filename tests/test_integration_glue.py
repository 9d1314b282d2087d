"""CPU: the Shadow-side glue (integration/scheduler_policy_gpu.c) compiles
against the reference's own, unmodified headers — the SchedulerPolicy vtable
of core/scheduler/scheduler_policy.h:31-51, event.h, host.h — and conda GLib,
with implicit declarations as errors.  Skipped where /root/reference is absent
(the GPU box)."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF = "/root/reference/src"
GLIB = ["/opt/conda/include/glib-2.0", "/opt/conda/lib/glib-2.0/include"]


@pytest.mark.skipif(not os.path.isdir(REF) or not all(os.path.isdir(g) for g in GLIB),
                    reason="reference sources or conda GLib headers absent")
@pytest.mark.parametrize("registered", [False, True])
def test_glue_compiles_against_reference_headers(tmp_path, registered):
    src = os.path.join(ROOT, "integration", "scheduler_policy_gpu.c")
    flags = ["-std=gnu99", "-D_GNU_SOURCE", "-Wall", "-Werror=implicit-function-declaration",
             "-Werror=incompatible-pointer-types", "-Werror=int-conversion",
             "-I" + REF, "-I" + os.path.join(ROOT, "include")] + ["-I" + g for g in GLIB]
    if registered:
        # as after the maintainer's enum edit: a header that
        # extends the enum is simulated by defining the value the glue expects
        flags += ["-DSHADOW_HAS_SP_PARALLEL_GPU", "-DSP_PARALLEL_GPU=(SP_PARALLEL_THREAD_PERHOST+1)"]
    r = subprocess.run(["gcc", "-c", src, "-o", str(tmp_path / "glue.o")] + flags,
                       capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    nm = subprocess.run(["nm", str(tmp_path / "glue.o")], capture_output=True, text=True).stdout
    assert " T schedulerpolicygpu_new" in nm
    for sym in ("sg_policy_create", "sg_policy_push", "sg_policy_pop", "sg_policy_next_time",
                "sg_policy_remaining", "sg_policy_thread_hosts", "sg_policy_add_host"):
        assert f" U {sym}" in nm, sym
