"""Download / integrity / archive helpers (D3).

Behavioural equivalent of the reference's vendored torchvision helpers
(``torchvision_utils.py``: ``download_url`` :123-171, ``check_integrity`` :86-91,
``calculate_md5`` :71-79, ``download_and_extract_archive`` :424-442, archive type
detection :322-359) in a compact form: http(s)/file URLs with redirects, MD5
verification, tar/tgz/tbz/txz/zip/gz/bz2/xz extraction with path-traversal protection.
Rank-0-only download + barrier is done by the callers (survey Q16).
"""
from __future__ import annotations

import bz2
import gzip
import hashlib
import lzma
import os
import shutil
import tarfile
import urllib.request
import zipfile

USER_AGENT = "faster_distributed_training_amd"


def calculate_md5(fpath: str, chunk_size: int = 1024 * 1024) -> str:
    md5 = hashlib.md5(usedforsecurity=False)
    with open(fpath, "rb") as f:
        for chunk in iter(lambda: f.read(chunk_size), b""):
            md5.update(chunk)
    return md5.hexdigest()


def check_md5(fpath: str, md5: str) -> bool:
    return md5 == calculate_md5(fpath)


def check_integrity(fpath: str, md5: str | None = None) -> bool:
    if not os.path.isfile(fpath):
        return False
    return True if md5 is None else check_md5(fpath, md5)


def _urlretrieve(url: str, fpath: str, chunk_size: int = 1024 * 32, max_redirects: int = 5):
    req = urllib.request.Request(url, headers={"User-Agent": USER_AGENT})
    for _ in range(max_redirects + 1):
        with urllib.request.urlopen(req) as resp:
            final = resp.geturl()
            if final != url and resp.status in (301, 302, 303, 307, 308):
                url = final
                req = urllib.request.Request(url, headers={"User-Agent": USER_AGENT})
                continue
            tmp = fpath + ".part"
            with open(tmp, "wb") as fh:
                for chunk in iter(lambda: resp.read(chunk_size), b""):
                    fh.write(chunk)
            os.replace(tmp, fpath)
            return
    raise RuntimeError(f"too many redirects for {url}")


def download_url(url: str, root: str, filename: str | None = None, md5: str | None = None) -> str:
    root = os.path.expanduser(root)
    filename = filename or os.path.basename(url)
    fpath = os.path.join(root, filename)
    os.makedirs(root, exist_ok=True)
    if check_integrity(fpath, md5):
        return fpath
    _urlretrieve(url, fpath)
    if not check_integrity(fpath, md5):
        raise RuntimeError(f"file not found or corrupted: {fpath}")
    return fpath


def _detect(path: str):
    p = path.lower()
    for suf, kind in ((".tar.gz", "tar"), (".tgz", "tar"), (".tar.bz2", "tar"), (".tbz", "tar"),
                      (".tar.xz", "tar"), (".txz", "tar"), (".tar", "tar"), (".zip", "zip"),
                      (".gz", "gz"), (".bz2", "bz2"), (".xz", "xz")):
        if p.endswith(suf):
            return kind, suf
    raise RuntimeError(f"unknown archive type: {path}")


def _safe_members(tf: tarfile.TarFile, dest: str):
    base = os.path.realpath(dest)
    for m in tf.getmembers():
        target = os.path.realpath(os.path.join(dest, m.name))
        if not (target == base or target.startswith(base + os.sep)) or m.issym() or m.islnk():
            raise RuntimeError(f"unsafe archive member: {m.name}")
        yield m


def extract_archive(from_path: str, to_path: str | None = None, remove_finished: bool = False) -> str:
    to_path = to_path or os.path.dirname(from_path)
    kind, suf = _detect(from_path)
    if kind == "tar":
        with tarfile.open(from_path, "r:*") as tf:
            tf.extractall(to_path, members=list(_safe_members(tf, to_path)))
    elif kind == "zip":
        with zipfile.ZipFile(from_path) as zf:
            for n in zf.namelist():
                t = os.path.realpath(os.path.join(to_path, n))
                if not t.startswith(os.path.realpath(to_path)):
                    raise RuntimeError(f"unsafe archive member: {n}")
            zf.extractall(to_path)
    else:
        opener = {"gz": gzip.open, "bz2": bz2.open, "xz": lzma.open}[kind]
        out = os.path.join(to_path, os.path.basename(from_path)[: -len(suf)])
        with opener(from_path, "rb") as fi, open(out, "wb") as fo:
            shutil.copyfileobj(fi, fo)
    if remove_finished:
        os.remove(from_path)
    return to_path


def download_and_extract_archive(url: str, download_root: str, extract_root: str | None = None,
                                 filename: str | None = None, md5: str | None = None,
                                 remove_finished: bool = False) -> None:
    extract_root = extract_root or download_root
    path = download_url(url, download_root, filename, md5)
    extract_archive(path, extract_root, remove_finished)
