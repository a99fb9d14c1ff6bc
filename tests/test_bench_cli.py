"""bench.py's run description for BASELINE.json configs 1-5 without a GPU: per-GPU batch, metric
string, sequence length and data-parallel settings (the 2/4/8-GPU runs are made by the round driver,
so their plumbing is pinned here as data)."""
import importlib.util
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _bench():
    spec = importlib.util.spec_from_file_location("bench_mod", os.path.join(ROOT, "bench.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def _desc(argv, world):
    bench = _bench()
    old = sys.argv
    try:
        sys.argv = ["bench.py"] + argv
        return bench.describe(bench.parse(), world=world)
    finally:
        sys.argv = old


def test_headline_config_one_and_eight_gpus():
    d = _desc([], 1)
    assert d["per_gpu_batch"] == 256 and d["global_batch"] == 256 and not d["ddp"] and d["parallelism"] == "dp1"
    assert d["metric"] == "images/sec (whole node) ViT-B/16 224px bf16 at 1/2/4/8 MI355X" and d["seq_len"] == 197
    d = _desc(["--gpus", "8"], 8)
    assert d["per_gpu_batch"] == 512 and d["global_batch"] == 4096 and d["ddp"] and d["parallelism"] == "dp8"
    assert d["metric"] == "images/sec (whole node) ViT-B/16 224px bf16 at 1/2/4/8 MI355X"


def test_vit_h14_fp8_eight_gpus():
    d = _desc(["--gpus", "8", "--model", "vit_h14", "--dtype", "fp8"], 8)
    assert d["per_gpu_batch"] == 256 and d["global_batch"] == 2048 and d["ddp"]
    assert d["metric"] == "images/sec (whole node) ViT-H/14 224px fp8" and d["seq_len"] == 257


def test_vit_l16_384_eight_gpus():
    d = _desc(["--gpus", "8", "--model", "vit_l16", "--image-size", "384"], 8)
    assert d["seq_len"] == 577 and d["per_gpu_batch"] == 128 and d["global_batch"] == 1024
    assert d["metric"] == "images/sec (whole node) ViT-L/16 384px bf16"


def test_per_gpu_defaults_fit_hbm():
    """Every data-parallel default per-GPU batch fits one MI355X (288 GB) with >= 10 % margin by the
    fitted peak-memory model; a batch that would not is refused before any allocation."""
    bench = _bench()
    for model, size in (("vit_b16", 224), ("vit_l16", 384), ("vit_h14", 224)):
        b = bench.default_per_gpu_batch(model, 8)
        assert bench.estimate_peak_gb(model, size, b) < 0.9 * 288, (model, b)
    assert bench.estimate_peak_gb("vit_h14", 224, 640) > 0.95 * 288  # refused up front
    assert abs(bench.estimate_peak_gb("vit_b16", 224, 256) - 17.9) < 0.5
    assert abs(bench.estimate_peak_gb("vit_l16", 384, 128) - 63.8) < 0.5
    assert abs(bench.estimate_peak_gb("vit_h14", 224, 256) - 134.2) < 0.5


def test_world1_forced_ddp_and_inference():
    assert _desc(["--force-ddp"], 1)["ddp"]
    d = _desc(["--infer"], 1)
    assert d["metric"] == "inference images/sec (whole node) ViT-B/16 224px bf16"


def _run_bench(argv, timeout=420):
    import subprocess

    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0")
    env.pop("WORLD_SIZE", None)  # the top-level command relaunches itself under torch.distributed.run
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), *argv], cwd=ROOT, env=env,
                       stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True, timeout=timeout)
    assert r.returncode == 0, r.stderr[-3000:]
    return r.stdout


def _json_lines(out):
    import json

    return [json.loads(l) for l in out.splitlines() if l.startswith("{")]


import pytest  # noqa: E402


@pytest.mark.gpu
def test_bench_distributed_branch_two_ranks():
    """The driver's multi-GPU command path end to end with 2 ranks on one GPU: `bench.py --gpus 2`
    relaunches itself under torch.distributed.run (127.0.0.1 rendezvous), both ranks build the model,
    DDP broadcasts rank 0's parameters and all-reduces the bucketed gradients (gloo test transport:
    RCCL needs one GPU per rank), the timed region's MAX over ranks, rank 0 prints exactly ONE JSON
    line, and every rank destroys its process group (clean exit)."""
    out = _run_bench(["--gpus", "2", "--backend", "gloo", "--batch", "16", "--steps", "2", "--warmup", "1"])
    lines = _json_lines(out)
    assert len(lines) == 1, out
    j = lines[0]
    assert j["n_gpus"] == 2 and j["steps"] == 2 and j["warmup"] == 1
    assert j["config"]["global_batch"] == 2 * j["config"]["per_gpu_batch"] == 32
    assert j["config"]["parallelism"] == "dp2" and "gloo" in j["config"]["grad_transport"]
    assert j["metric"] == "images/sec (whole node) ViT-B/16 224px bf16 at 1/2/4/8 MI355X"
    assert j["value"] > 0 and abs(j["value"] - 32 * 2 / (j["ms_per_step"] * 2 / 1000.0)) < 0.02 * j["value"]
