"""CPU tests of build provenance: libplk.so carries a hash of the sources and flags it was
compiled from (plk_build_info, build_ext.py source_id / flags_id), and the Python mirror
refuses a library whose sources differ from the tree it is loaded from (plonk.check_build,
called by the `plk` fixture, __graft_entry__.smoke() and bench.py)."""
import importlib.util
import shutil
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parent.parent


def _build_ext():
    spec = importlib.util.spec_from_file_location("_be", ROOT / "dusk-plonk_amd" / "build_ext.py")
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return m


def _copy_sources(dst: Path):
    shutil.copytree(ROOT / "dusk-plonk_amd" / "csrc", dst / "dusk-plonk_amd" / "csrc")
    (dst / "include").mkdir()
    shutil.copy(ROOT / "include" / "plk.h", dst / "include" / "plk.h")


def test_library_matches_tree(plk):
    info = plk.check_build()
    be = _build_ext()
    assert info["src"] == be.source_id() and len(info["src"]) == 16
    assert info["flags"] == be.flags_id()
    assert info["variant"] == "default"


def test_edited_source_fails_the_check(plk, tmp_path):
    be = _build_ext()
    _copy_sources(tmp_path)
    assert be.source_id(tmp_path) == be.source_id()  # the hash is path-independent
    f = tmp_path / "dusk-plonk_amd" / "csrc" / "msm_acc.hip"
    f.write_text(f.read_text() + "\n// an edit\n")
    assert be.source_id(tmp_path) != be.source_id()
    with pytest.raises(ImportError, match="other sources"):
        plk.check_build(root=tmp_path)


def test_added_header_changes_the_id(tmp_path):
    be = _build_ext()
    _copy_sources(tmp_path)
    (tmp_path / "dusk-plonk_amd" / "csrc" / "new.hpp").write_text("#pragma once\n")
    assert be.source_id(tmp_path) != be.source_id()


def test_flags_id_ignores_the_tree_path():
    be = _build_ext()
    moved = [f.replace(str(be.ROOT), "/elsewhere/repo") for f in be.CFLAGS]
    assert be.flags_id(be.CFLAGS) == be.flags_id(be.CFLAGS)
    assert be.flags_id(be.CFLAGS + ["-DX=1"]) != be.flags_id(be.CFLAGS)
    # only the tree's own path is normalised: another absolute path is a different build
    assert be.flags_id(moved) != be.flags_id(be.CFLAGS)
