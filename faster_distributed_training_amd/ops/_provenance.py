"""Build provenance of the in-tree extension: a hash of every native source.

``build_native.py`` links the hash of ``csrc/**`` (sources, headers, target arch) into the
``.so`` (``_fdt_native.source_hash()``); ``_native.load()`` recomputes it from the tree it
runs in and refuses a binary built from other sources, so a stale ``.so`` can never run
silently next to newer kernels.  Pure stdlib: imported by the build script too.
"""
from __future__ import annotations

import glob
import hashlib
import os

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
CSRC = os.path.join(ROOT, "csrc")
EXTS = (".hip", ".cpp", ".h")


def native_sources(csrc: str = CSRC):
    files = [f for f in glob.glob(os.path.join(csrc, "**", "*"), recursive=True) if f.endswith(EXTS)]
    return sorted(files, key=lambda f: os.path.relpath(f, csrc))


def source_hash(arch: str | None = None, csrc: str = CSRC) -> str | None:
    """sha256 over (relative path, content) of every native source plus the target arch;
    None when the sources are not present (an installed copy without csrc/)."""
    files = native_sources(csrc)
    if not files:
        return None
    h = hashlib.sha256()
    h.update((arch or os.environ.get("FDT_OFFLOAD_ARCH", "gfx950")).encode())
    for f in files:
        h.update(os.path.relpath(f, csrc).replace(os.sep, "/").encode() + b"\0")
        with open(f, "rb") as fh:
            h.update(fh.read())
        h.update(b"\0")
    return h.hexdigest()
