"""bench.py with every bf16 copy written on the fp8 path (A/B of the fp8-only skips in
ops/fused_vit.py: a no-op DGRAD_TAP turns them off). Usage: python scripts/probes/bench_fp8_noskip.py <bench args>"""
import os
import runpy
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import pytorch_vit_paper_replication_amd.ops.fused_vit as f  # noqa: E402

f.DGRAD_TAP = lambda which, t: None
sys.argv = ["bench.py"] + sys.argv[1:]
runpy.run_path("bench.py", run_name="__main__")
