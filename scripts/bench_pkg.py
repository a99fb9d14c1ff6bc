"""Run bench.py against another build of the package (A/B of native code on one box).

usage: python scripts/bench_pkg.py <package root relative to the repo, e.g. ab_old, or .> [bench args]
"""
import os
import runpy
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
pkg_root = ROOT if sys.argv[1] == "." else os.path.join(ROOT, sys.argv[1])
sys.path.insert(0, pkg_root)
sys.argv = [os.path.join(ROOT, "bench.py")] + sys.argv[2:]
import pytorch_vit_paper_replication_amd as _p  # noqa: E402

print(f"[bench_pkg] package from {os.path.dirname(_p.__file__)}", file=sys.stderr, flush=True)
runpy.run_path(sys.argv[0], run_name="__main__")
