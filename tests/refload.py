"""Load the read-only reference implementation (pure-PyTorch source files only) for parity tests."""
import importlib.util
import os

import pytest

REF = "/root/reference"


def ref_module(rel: str, name: str):
    path = os.path.join(REF, rel)
    if not os.path.exists(path):
        pytest.skip(f"reference file {path} not available")
    spec = importlib.util.spec_from_file_location(name, path)
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod
