"""Read-only access to the reference implementation as a numerics oracle.

The reference (SuperbTUM/Faster-Distributed-Training) is mounted at /root/reference in
the authoring container only; tests that need it skip elsewhere.  Only its pure-torch
modules are imported (resnet.py, transformer.py, ngd_optimizer.py): they import nothing
beyond torch/math.  No reference file is modified and no bytecode is written there.
"""
from __future__ import annotations

import importlib.util
import os
import sys

import pytest

REF = os.environ.get("FDT_REFERENCE", "/root/reference")


def available(name: str) -> bool:
    return os.path.isfile(os.path.join(REF, name + ".py"))


def load(name: str):
    if not available(name):
        pytest.skip(f"reference {name}.py not present")
    key = f"_fdt_ref_{name}"
    if key in sys.modules:
        return sys.modules[key]
    old = sys.dont_write_bytecode
    sys.dont_write_bytecode = True
    try:
        spec = importlib.util.spec_from_file_location(key, os.path.join(REF, name + ".py"))
        mod = importlib.util.module_from_spec(spec)
        sys.modules[key] = mod
        spec.loader.exec_module(mod)
    finally:
        sys.dont_write_bytecode = old
    return mod
