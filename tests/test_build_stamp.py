"""build.up_to_date(): libkad.so counts as current when its stamp holds the content hash of the sources it was
linked from — not when its modification time happens to be newer (copies and checkouts reset mtimes)."""
import os

from kubeadmiral_amd import build


def test_stamp_decides_over_mtimes(tmp_path, monkeypatch):
    lib = tmp_path / "libkad.so"
    lib.write_bytes(b"\0")
    os.utime(lib, (0, 0))  # older than every source: the mtime rule alone would rebuild
    monkeypatch.setattr(build, "LIB", str(lib))
    monkeypatch.setattr(build, "STAMP", str(lib) + ".sha256")
    assert not build.up_to_date()
    build._write_stamp(build.inputs_hash())
    assert build.up_to_date()
    build._write_stamp("0" * 64)  # a library of other sources, however new its file
    os.utime(lib, None)
    assert not build.up_to_date()


def test_inputs_hash_covers_every_input():
    h = build.inputs_hash()
    assert len(h) == 64 and h == build.inputs_hash()
    names = {os.path.basename(p) for p in build._inputs()}
    assert set(build.SOURCES) <= names and "kad_sched.h" in names
