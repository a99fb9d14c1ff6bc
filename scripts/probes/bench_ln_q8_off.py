import runpy, sys
sys.path.insert(0, ".")
import pytorch_vit_paper_replication_amd.ops.fused_vit as f
f.LN_BWD_FP8_COPY = False
sys.argv = ["bench.py"] + sys.argv[1:]
runpy.run_path("bench.py", run_name="__main__")
