"""The in-tree extension is tied to its sources: ``_C`` carries the content hash of ``csrc/`` and the
loader refuses (or, under ``PVR_AUTOBUILD=1``, rebuilds) a binary built from other sources."""
import shutil

import pytest

from pytorch_vit_paper_replication_amd import _ext, build


def _so():
    so = build.ext_path()
    if not so.exists():
        pytest.skip("extension not built in this tree")
    return so


def test_binary_matches_tree():
    so = _so()
    assert build.embedded_hash(so) == build.source_hash(), "in-tree _C is stale: rebuild it"
    assert _ext.check_source_hash(so, build.CSRC) == build.source_hash()


def test_edited_header_is_refused(tmp_path):
    so = _so()
    csrc = tmp_path / "csrc"
    shutil.copytree(build.CSRC, csrc)
    assert _ext.check_source_hash(so, csrc) == build.source_hash(csrc)
    with open(csrc / "common.h", "a") as f:  # touch a header: one more comment line
        f.write("// edited\n")
    with pytest.raises(_ext.StaleExtensionError):
        _ext.check_source_hash(so, csrc)


def test_loader_refuses_stale_binary(tmp_path, monkeypatch):
    _so()
    csrc = tmp_path / "csrc"
    shutil.copytree(build.CSRC, csrc)
    with open(csrc / "gemm_params.h", "a") as f:
        f.write("// edited\n")
    monkeypatch.setattr(build, "CSRC", csrc)
    monkeypatch.delenv("PVR_AUTOBUILD", raising=False)
    monkeypatch.setattr(_ext, "_TRIED", False)
    monkeypatch.setattr(_ext, "_C", None)
    monkeypatch.setattr(_ext, "_ERR", None)
    assert _ext.load() is None
    assert isinstance(_ext._ERR, _ext.StaleExtensionError)
    with pytest.raises(RuntimeError, match="other sources"):
        _ext.ext()
