"""Loader for the in-tree HIP extension ``_fdt_native`` (built by ``build_native.py``).

Policy (MI355X-first, no silent fallbacks):

* On a machine with a GPU, the fast path *requires* the extension: ``native()`` raises
  if it is missing, so a GPU run never quietly degrades to eager PyTorch.
* ``FDT_NATIVE=0`` disables the fast path explicitly (the "w/o tricks" ablation and the
  CPU oracle path); that choice is visible in every benchmark line.
* On CPU-only machines the pure-PyTorch reference implementations are used (they are
  also the numerics oracle for the kernel tests).
"""
from __future__ import annotations

import glob
import importlib.util
import os

import torch

_PKG_DIR = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
_mod = None
_err = None


def _so_path():
    cands = sorted(glob.glob(os.path.join(_PKG_DIR, "_fdt_native*.so")))
    return cands[0] if cands else None


def load():
    """Import the extension (once).  Returns the module or None."""
    global _mod, _err
    if _mod is not None or _err is not None:
        return _mod
    path = _so_path()
    if path is None:
        _err = "extension _fdt_native not built (run `python build_native.py`)"
        return None
    try:
        spec = importlib.util.spec_from_file_location("_fdt_native", path)
        m = importlib.util.module_from_spec(spec)
        spec.loader.exec_module(m)
    except Exception as e:  # pragma: no cover - depends on build state
        _err = f"failed to load {path}: {e}"
        return None
    # provenance: the binary must have been built from the csrc/ next to it
    from ._provenance import source_hash
    want = source_hash(arch=getattr(m, "arch", None))  # (the arch the binary was built for)
    got = m.source_hash() if hasattr(m, "source_hash") else None
    if want is not None and got != want and os.environ.get("FDT_ALLOW_STALE_NATIVE", "0") != "1":
        _err = (f"{path} is stale: built from sources with hash {got}, the tree has {want} "
                f"(run `python build_native.py`)")
        if os.environ.get("FDT_NATIVE") == "1":
            raise RuntimeError(f"FDT_NATIVE=1 but {_err}")
        import warnings
        warnings.warn(f"HIP extension refused: {_err}", RuntimeWarning, stacklevel=2)
        return None
    _mod = m
    if hasattr(m, "set_conv_write_through"):
        # write-through (sc1) streaming outputs of the conv epilogues and the BN / join passes
        # (conv_igemm_impl.h st_out, common.h st8): measured bs128 5.56 -> 5.47 ms, bs1024 neutral
        m.set_conv_write_through(os.environ.get("FDT_CONV_WT", "1") == "1")
    if hasattr(m, "set_ew_unroll"):
        # loads-first streaming form of the join / normalise / fold passes (bn_kernels.hip kEwU)
        m.set_ew_unroll(os.environ.get("FDT_EW_UNROLL", "1") == "1")
    return _mod


def built_from() -> str | None:
    """Hash of the sources the loaded extension was built from (None if not loaded)."""
    m = load()
    return m.source_hash() if m is not None else None


def enabled() -> bool:
    """True when hot ops should run through the HIP kernels."""
    if os.environ.get("FDT_NATIVE", "1") == "0":
        return False
    return torch.cuda.is_available()


def native():
    """The extension module; raises loudly if it is needed but unavailable."""
    m = load()
    if m is None:
        raise RuntimeError(f"HIP fast path requested but {_err}")
    return m


def use_native(t: torch.Tensor) -> bool:
    """Dispatch predicate for one op call: GPU tensor and fast path enabled."""
    return t.is_cuda and enabled()


def stream_ptr(device: torch.device | None = None) -> int:
    """Raw hipStream_t of the current torch stream (kernels are enqueued on it, so
    they order correctly with PyTorch work and are captured by HIP graphs)."""
    idx = torch.cuda.current_device() if device is None else device.index
    return torch._C._cuda_getCurrentRawStream(idx)


def ptr(t: torch.Tensor | None) -> int:
    return 0 if t is None else t.data_ptr()


# ---------------------------------------------------------------- deterministic mode
_DET = False


def set_deterministic(on: bool = True) -> None:
    """Bitwise-repeatable engine steps (``--deterministic``; SURVEY section 5 race detection).

    The ResNet engine's per-channel statistics producers write one slot row per workgroup
    (no wrapping onto shared rows, so no two fp32 atomics meet on an address), the split-K
    conv reducer sums partials in split order, and 1x1 weight gradients go through the
    ordered slab reduction instead of fp32 atomics.  Costs a little time (larger slot
    buffers; see profiles/deterministic_cost.json)."""
    global _DET
    _DET = bool(on)
    m = load()
    if m is not None:
        m.set_deterministic_mode(_DET)


def deterministic() -> bool:
    return _DET
