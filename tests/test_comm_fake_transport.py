"""C++ unit test of the native communicator's mesh all-reduce schedule over a fake in-process
transport (threads + shared buffers standing in for RCCL's grouped p2p), also
under ThreadSanitizer and AddressSanitizer/UBSan (host code only). Needs g++, no GPU."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "tests", "cpp", "test_comm_core.cpp")
INC = os.path.join(ROOT, "pytorch_vit_paper_replication_amd", "csrc")


def _build_and_run(tmp_path, flags, name):
    exe = str(tmp_path / name)
    cmd = ["g++", "-std=c++17", "-pthread", "-I", INC, SRC, "-o", exe] + flags
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    out = subprocess.run([exe], capture_output=True, text=True, timeout=300)
    assert out.returncode == 0 and "ALL OK" in out.stdout, out.stdout[-2000:] + out.stderr[-2000:]
    return out.stdout


@pytest.mark.skipif(shutil.which("g++") is None, reason="needs g++")
def test_mesh_all_reduce_fake_transport(tmp_path):
    print(_build_and_run(tmp_path, ["-O2", "-Wall", "-Werror"], "comm_core"))


@pytest.mark.skipif(shutil.which("g++") is None, reason="needs g++")
@pytest.mark.parametrize("san", ["thread", "address,undefined"])
def test_mesh_all_reduce_fake_transport_sanitized(tmp_path, san):
    env_ok = subprocess.run(["g++", f"-fsanitize={san}", "-x", "c++", "-", "-o", str(tmp_path / "probe")],
                            input="int main(){return 0;}", capture_output=True, text=True)
    if env_ok.returncode != 0:
        pytest.skip(f"-fsanitize={san} unavailable")
    _build_and_run(tmp_path, ["-O1", "-g", f"-fsanitize={san}", "-fno-omit-frame-pointer"], "comm_core_" + san.replace(",", "_"))
