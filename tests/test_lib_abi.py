"""CPU: libshadowgpu.so loads, exports every symbol include/shadowgpu.h declares,
and the engine fails loudly (no CPU fallback) when no gfx950 GPU is present."""
import ctypes
import os
import re
import subprocess

import pytest

from shadow_amd import _lib as L
from shadow_amd import phold

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _declared():
    names = set()
    for f in os.listdir(os.path.join(ROOT, "include")):
        if f.endswith(".h"):
            src = open(os.path.join(ROOT, "include", f)).read()
            src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
            names |= set(re.findall(r"\b(sg_[a-z0-9_]+)\s*\((?!\*)", src))
    return names


def test_header_symbols_exported():
    declared = _declared()
    assert len(declared) > 20
    out = subprocess.run(["nm", "-D", "--defined-only", L.LIB_PATH], capture_output=True,
                         text=True, check=True).stdout
    exported = set(re.findall(r" T (sg_[a-z0-9_]+)", out))
    missing = declared - exported
    assert not missing, missing
    # and every declared symbol is named by the Python mirror's export list
    assert declared <= set(L.EXPORTS), declared - set(L.EXPORTS)


def test_abi_version():
    import re
    hdr = open(os.path.join(ROOT, "include", "shadowgpu.h")).read()
    assert L.lib().sg_abi_version() == int(re.search(r"SG_ABI_VERSION (\d+)", hdr).group(1))


def test_engine_without_gpu_fails_loudly():
    try:
        import torch
        if torch.cuda.is_available():
            pytest.skip("GPU present")
    except ImportError:
        pass
    from shadow_amd.engine import Engine
    cfg = phold.tiny_config(n_hosts=8)
    with pytest.raises(L.SgError) as ei:
        Engine(cfg)
    assert ei.value.code == L.SG_ERR_NODEV


def test_invalid_params_rejected():
    from shadow_amd.engine import Engine
    cfg = phold.tiny_config(n_hosts=8)
    cfg["load"] = 0
    with pytest.raises(L.SgError) as ei:
        Engine(cfg)
    assert ei.value.code in (L.SG_ERR_INVAL, L.SG_ERR_NODEV)
