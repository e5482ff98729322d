#!/usr/bin/env python3
"""Build the in-tree HIP extension ``faster_distributed_training_amd/_fdt_native*.so``.

Every ``csrc/kernels/*.hip`` and ``csrc/runtime/*.cpp`` (+ ``csrc/bindings.cpp``) is
compiled by ``hipcc --offload-arch=gfx950`` (CDNA4 / MI355X only — no other targets, no
CUDA paths) into an object, in parallel, and linked into one pybind11 module placed in
the package directory (so it ships with the tree to the GPU box; no JIT cache).
Objects are rebuilt only when their source or any header changed.

    python build_native.py            # incremental
    python build_native.py --clean    # from scratch
    python build_native.py --asm      # also keep .s (register / occupancy audit)
"""
from __future__ import annotations

import argparse
import concurrent.futures as cf
import glob
import os
import shutil
import subprocess
import sys
import sysconfig

ROOT = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(ROOT, "csrc")
PKG = os.path.join(ROOT, "faster_distributed_training_amd")
BUILD = os.path.join(ROOT, "build", "native")
ARCH = os.environ.get("FDT_OFFLOAD_ARCH", "gfx950")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")


def _pybind_include():
    import pybind11
    return pybind11.get_include()


def sources():
    srcs = sorted(glob.glob(os.path.join(CSRC, "kernels", "*.hip")))
    srcs += sorted(glob.glob(os.path.join(CSRC, "runtime", "*.cpp")))
    srcs.append(os.path.join(CSRC, "bindings.cpp"))
    return srcs


def headers():
    return glob.glob(os.path.join(CSRC, "**", "*.h"), recursive=True)


def common_flags():
    return [
        "-O3", "-std=c++17", "-fPIC", f"--offload-arch={ARCH}",
        "-I", CSRC, "-I", os.path.join(CSRC, "kernels"),
        "-I", _pybind_include(), "-I", sysconfig.get_paths()["include"],
        "-Wno-unused-result", "-Wno-unused-command-line-argument",
        "-fvisibility=hidden",
    ]


def obj_path(src):
    rel = os.path.relpath(src, CSRC).replace(os.sep, "__")
    return os.path.join(BUILD, rel + ".o")


def needs_build(src, obj, hdr_mtime):
    if not os.path.exists(obj):
        return True
    m = os.path.getmtime(obj)
    return os.path.getmtime(src) > m or hdr_mtime > m


def compile_one(src, obj, asm=False):
    cmd = [HIPCC, *common_flags(), "-c", src, "-o", obj]
    if src.endswith(".cpp"):
        cmd = [HIPCC, *common_flags(), "-x", "hip", "-c", src, "-o", obj]
    if asm:
        cmd += ["-save-temps=obj"]
    r = subprocess.run(cmd, capture_output=True, text=True, cwd=BUILD)
    if r.returncode != 0:
        raise RuntimeError(f"compile failed: {src}\n{' '.join(cmd)}\n{r.stdout}\n{r.stderr}")
    return src


def out_path():
    suffix = sysconfig.get_config_var("EXT_SUFFIX") or ".so"
    return os.path.join(PKG, "_fdt_native" + suffix)


def build(clean=False, jobs=None, asm=False, verbose=True):
    if clean and os.path.isdir(BUILD):
        shutil.rmtree(BUILD)
    os.makedirs(BUILD, exist_ok=True)
    hdr_m = max([os.path.getmtime(h) for h in headers()] + [0])
    srcs = sources()
    todo = [s for s in srcs if asm or needs_build(s, obj_path(s), hdr_m)]
    jobs = jobs or min(8, os.cpu_count() or 4, max(1, len(todo)))
    if todo:
        if verbose:
            print(f"[build_native] compiling {len(todo)} file(s) for {ARCH} with {jobs} job(s)", flush=True)
        with cf.ThreadPoolExecutor(jobs) as ex:
            futs = [ex.submit(compile_one, s, obj_path(s), asm) for s in todo]
            for f in cf.as_completed(futs):
                s = f.result()
                if verbose:
                    print(f"  ok  {os.path.relpath(s, ROOT)}", flush=True)
    out = out_path()
    objs = [obj_path(s) for s in srcs]
    if todo or not os.path.exists(out) or any(os.path.getmtime(o) > os.path.getmtime(out) for o in objs):
        tmp = out + ".tmp"
        cmd = [HIPCC, "-shared", "-fPIC", f"--offload-arch={ARCH}", *objs, "-o", tmp]
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"link failed\n{' '.join(cmd)}\n{r.stdout}\n{r.stderr}")
        os.replace(tmp, out)
        if verbose:
            print(f"[build_native] linked {os.path.relpath(out, ROOT)}", flush=True)
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--clean", action="store_true")
    ap.add_argument("--jobs", type=int, default=None)
    ap.add_argument("--asm", action="store_true")
    a = ap.parse_args()
    try:
        build(a.clean, a.jobs, a.asm)
    except RuntimeError as e:
        print(e, file=sys.stderr)
        sys.exit(1)


if __name__ == "__main__":
    main()
