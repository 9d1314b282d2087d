"""In-tree build of libshadowgpu.so (gfx950) and of the Shadow-side glue linked
to it (integration/_bin/, only where the reference headers are present).

hipcc cross-compiles for gfx950 without a GPU, so this runs in the CPU
container; the .so files travel to the GPU box with the repository snapshot.
"""
from __future__ import annotations

import os
import subprocess
import sys

PKG = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(PKG)
CSRC = os.path.join(PKG, "csrc")
INC = os.path.join(ROOT, "include")
BUILD = os.path.join(ROOT, "build")
LIB = os.path.join(PKG, "libshadowgpu.so")

HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = "gfx950"

C_FLAGS = ["-O2", "-std=c11", "-fPIC", "-ffp-contract=off", "-fno-fast-math", "-Wall",
           "-Wextra", "-Wno-unused-parameter", "-I" + INC]
HIP_FLAGS = ["--offload-arch=" + ARCH, "-O3", "-fPIC", "-std=c++17", "-ffp-contract=off",
             "-fno-fast-math", "-Wall", "-I" + INC, "-I" + CSRC]

C_SOURCES = ["sg_host.c", "sg_policy.c", "sg_sched.c", "sg_topology.c"]
HIP_SOURCES = ["sg_engine.hip", "sg_policy_dev.hip"]


def _run(cmd, verbose):
    if verbose:
        print(" ".join(cmd), flush=True)
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        sys.stderr.write(r.stdout + r.stderr)
        raise RuntimeError("build step failed: " + " ".join(cmd))
    return r


def _stale(out, srcs):
    if not os.path.exists(out):
        return True
    t = os.path.getmtime(out)
    return any(os.path.getmtime(s) > t for s in srcs)


def build(verbose: bool = False, force: bool = False, variant: str = "", defines=()) -> str:
    """variant / defines: an A/B build (libshadowgpu_<variant>.so, objects in
    build/<variant>/) with extra -D flags; the default build has neither."""
    global BUILD, LIB
    if variant:
        BUILD = os.path.join(ROOT, "build", variant)
        LIB = os.path.join(PKG, f"libshadowgpu_{variant}.so")
    os.makedirs(BUILD, exist_ok=True)
    hdrs = [os.path.join(INC, f) for f in os.listdir(INC) if f.endswith(".h")]
    hdrs += [os.path.join(CSRC, f) for f in os.listdir(CSRC) if f.endswith(".h")]
    objs = []
    for src in C_SOURCES:
        path = os.path.join(CSRC, src)
        if not os.path.exists(path):
            continue
        obj = os.path.join(BUILD, src + ".o")
        if force or _stale(obj, [path] + hdrs):
            _run(["gcc"] + C_FLAGS + ["-c", path, "-o", obj], verbose)
        objs.append(obj)
    for src in HIP_SOURCES:
        path = os.path.join(CSRC, src)
        if not os.path.exists(path):
            continue
        obj = os.path.join(BUILD, src + ".o")
        if force or _stale(obj, [path] + hdrs):
            _run([HIPCC] + HIP_FLAGS + list(defines) + ["-c", path, "-o", obj], verbose)
        objs.append(obj)
    if force or _stale(LIB, objs):
        _run([HIPCC, "--offload-arch=" + ARCH, "-shared", "-o", LIB] + objs + ["-lpthread"],
             verbose)
    return LIB


REF_SRC = "/root/reference/src"
GLIB_INC = ["/opt/conda/include/glib-2.0", "/opt/conda/lib/glib-2.0/include"]
GLIB_LIB = "/opt/conda/lib"
GLUE_BIN = os.path.join(ROOT, "integration", "_bin")
GLUE_VARIANTS = {"relabel": [], "exact": ["-DSHADOW_HAS_EVENT_SRCID"]}


def glue_available() -> bool:
    return os.path.isdir(REF_SRC) and all(os.path.isdir(g) for g in GLIB_INC)


def build_glue(verbose: bool = False, force: bool = False) -> list:
    """integration/scheduler_policy_gpu.c + tests/glue_phold.c, compiled against
    the reference's unmodified headers and linked to the real libshadowgpu.so
    (rpath $ORIGIN/../../shadow_amd) and conda GLib: integration/_bin/
    libsgglue_<variant>.so.  Needs /root/reference, so it runs in the build
    container only; the .so files travel to the GPU box with the tree."""
    if not glue_available():
        return []
    os.makedirs(GLUE_BIN, exist_ok=True)
    srcs = [os.path.join(ROOT, "integration", "scheduler_policy_gpu.c"),
            os.path.join(ROOT, "tests", "glue_phold.c"), os.path.join(INC, "shadowgpu.h"), LIB]
    outs = []
    for name, defs in GLUE_VARIANTS.items():
        out = os.path.join(GLUE_BIN, f"libsgglue_{name}.so")
        if force or _stale(out, srcs):
            _run(["gcc", "-shared", "-fPIC", "-O2", "-std=gnu99", "-D_GNU_SOURCE", "-Wall",
                  "-Werror=implicit-function-declaration", "-I" + REF_SRC, "-I" + INC] +
                 ["-I" + g for g in GLIB_INC] + defs + srcs[:2] +
                 ["-o", out, "-L" + GLIB_LIB, "-Wl,-rpath," + GLIB_LIB, "-lglib-2.0",
                  "-L" + PKG, "-lshadowgpu", "-Wl,-rpath,$ORIGIN/../../shadow_amd", "-lpthread"], verbose)
        outs.append(out)
    return outs


if __name__ == "__main__":
    a = sys.argv[1:]
    v = a[a.index("--variant") + 1] if "--variant" in a else ""
    print(build(verbose=True, force="--force" in a, variant=v, defines=[x for x in a if x.startswith("-D")]))
