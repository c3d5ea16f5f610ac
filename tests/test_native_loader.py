"""The native loader never imports a module built from other sources than the
tree's: a source edit is seen through the content hash
recorded next to the module, and leads to a rebuild -- or, with no compiler,
to a loud error.  The real module is never touched: the build and the import
are stubbed and the hash is taken over a scratch copy of the sources."""
from __future__ import annotations

import os
import shutil

import pytest

from akka_allreduce_amd import _build, _native_loader


@pytest.fixture()
def tree(tmp_path):
    """A scratch copy of csrc/ plus a fake module and its recorded hash."""
    shutil.copytree(_build.CSRC, tmp_path / "csrc")
    ext = tmp_path / "_native.so"
    ext.write_bytes(b"\x7fELF fake")
    with open(_build.hash_path(str(ext)), "w") as f:
        f.write(_build.source_hash(str(tmp_path)) + "\n")
    return tmp_path, str(ext)


def test_hash_tracks_contents_not_timestamps(tree):
    root, ext = tree
    assert _build.stale_reason(ext, str(root)) is None
    src = root / "csrc" / "kernels" / "kernels.hip"
    t = os.path.getmtime(src)
    os.utime(src, (t + 3600, t + 3600))  # a newer timestamp alone changes nothing
    assert _build.stale_reason(ext, str(root)) is None
    src.write_text(src.read_text() + "\n// edited\n")
    os.utime(src, (t - 3600, t - 3600))  # ... and an OLDER timestamp hides no edit
    assert _build.stale_reason(ext, str(root)) == "sources changed since the module was built"
    hdr = root / "csrc" / "engine" / "geometry.h"
    src.write_text(src.read_text().replace("\n// edited\n", ""))
    assert _build.stale_reason(ext, str(root)) is None
    hdr.write_text(hdr.read_text() + "\n")
    assert _build.stale_reason(ext, str(root)) is not None  # headers count


def test_missing_hash_or_module_is_stale(tree):
    root, ext = tree
    os.remove(_build.hash_path(ext))
    assert _build.stale_reason(ext, str(root)) == "no source hash recorded next to the module"
    assert _build.stale_reason(str(root / "absent.so"), str(root)) == "not built"


def test_no_sources_means_nothing_to_compare(tmp_path):
    ext = tmp_path / "_native.so"
    ext.write_bytes(b"x")
    assert _build.source_hash(str(tmp_path)) is None
    assert _build.stale_reason(str(ext), str(tmp_path)) is None


@pytest.fixture()
def fresh_loader(monkeypatch):
    saved = _native_loader._mod
    monkeypatch.setattr(_native_loader, "_mod", None)
    monkeypatch.delenv("AKKA_NATIVE_PATH", raising=False)
    monkeypatch.delenv("AKKA_REBUILD", raising=False)
    imported = []
    monkeypatch.setattr(_native_loader.importlib, "import_module", lambda name: imported.append(name) or "module")
    yield imported
    _native_loader._mod = saved


def test_loader_rebuilds_a_stale_module(fresh_loader, monkeypatch):
    builds = []
    monkeypatch.setattr(_build, "stale_reason", lambda *a, **k: "sources changed since the module was built")
    monkeypatch.setattr(_build, "have_compiler", lambda: True)
    monkeypatch.setattr(_build, "build", lambda *a, **k: builds.append(1))
    assert _native_loader.load() == "module"
    assert builds == [1] and fresh_loader == ["akka_allreduce_amd._native"]


def test_loader_skips_the_build_when_current(fresh_loader, monkeypatch):
    monkeypatch.setattr(_build, "stale_reason", lambda *a, **k: None)
    monkeypatch.setattr(_build, "build", lambda *a, **k: pytest.fail("a current module was rebuilt"))
    assert _native_loader.load() == "module"


def test_loader_fails_loudly_without_a_compiler(fresh_loader, monkeypatch):
    monkeypatch.setattr(_build, "stale_reason", lambda *a, **k: "sources changed since the module was built")
    monkeypatch.setattr(_build, "have_compiler", lambda: False)
    monkeypatch.setattr(_build, "build", lambda *a, **k: pytest.fail("no compiler: must not try to build"))
    with pytest.raises(RuntimeError, match="must be rebuilt"):
        _native_loader.load()
    assert fresh_loader == []


def test_in_tree_module_is_current():
    """The module this checkout ships (and the GPU box loads) matches its sources."""
    assert _build.stale_reason() is None
