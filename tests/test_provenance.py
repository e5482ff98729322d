"""Build provenance: the extension carries the hash of the csrc/
sources it was built from and the loader refuses a binary built from other sources."""
import os
import shutil

import pytest

from faster_distributed_training_amd.ops import _native, _provenance


def test_source_hash_tracks_every_source(tmp_path):
    src = tmp_path / "csrc"
    shutil.copytree(_provenance.CSRC, src)
    h0 = _provenance.source_hash("gfx950", str(src))
    assert h0 == _provenance.source_hash("gfx950", str(src))
    assert h0 != _provenance.source_hash("gfx942", str(src))  # target arch is part of it
    f = sorted(p for p in _provenance.native_sources(str(src)) if p.endswith(".h"))[0]
    with open(f, "a") as fh:
        fh.write("\n// edit\n")
    assert _provenance.source_hash("gfx950", str(src)) != h0


@pytest.mark.skipif(_native._so_path() is None, reason="extension not built")
def test_loaded_extension_matches_tree():
    m = _native.load()
    assert m is not None, _native._err
    assert _native.built_from() == _provenance.source_hash()


@pytest.mark.skipif(_native._so_path() is None, reason="extension not built")
def test_stale_extension_refused(monkeypatch):
    monkeypatch.setattr(_native, "_mod", None)
    monkeypatch.setattr(_native, "_err", None)
    monkeypatch.setattr(_provenance, "source_hash", lambda *a, **k: "0" * 64)
    monkeypatch.delenv("FDT_ALLOW_STALE_NATIVE", raising=False)
    monkeypatch.delenv("FDT_NATIVE", raising=False)
    with pytest.warns(RuntimeWarning, match="stale"):  # refused loudly, not silently
        assert _native.load() is None and "stale" in _native._err
    with pytest.raises(RuntimeError, match="stale"):
        _native.native()
    # an explicit FDT_NATIVE=1 makes the refusal an error at load time
    monkeypatch.setattr(_native, "_err", None)
    monkeypatch.setenv("FDT_NATIVE", "1")
    with pytest.raises(RuntimeError, match="FDT_NATIVE=1"):
        _native.load()
