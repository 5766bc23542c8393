"""The native build really recompiles: ``build(force=True)`` replaces the in-tree library even
when it is newer than its sources (the driver's ``__graft_entry__.build()`` uses force)."""
import os
import time

from ome_amd import build as b


def test_forced_rebuild_replaces_library(tmp_path, monkeypatch):
    monkeypatch.setattr(b, "LIBDIR", tmp_path / "lib")
    monkeypatch.setattr(b, "OBJDIR", tmp_path / "obj")
    (lib,) = b.build(force=True, verbose=False, only=("omeio",))
    assert lib.exists() and lib.parent == tmp_path / "lib"
    t1 = lib.stat().st_mtime
    os.utime(lib, (t1 + 3600, t1 + 3600))  # newer than every source: a non-forced build keeps it
    (lib2,) = b.build(force=False, verbose=False, only=("omeio",))
    assert lib2.stat().st_mtime == t1 + 3600
    time.sleep(0.01)
    (lib3,) = b.build(force=True, verbose=False, only=("omeio",))
    assert lib3.stat().st_mtime < t1 + 3600, "forced build reused the stale library"
