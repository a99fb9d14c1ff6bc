#!/bin/bash
# Build an A/B copy of the package: scripts/mk_abtree.sh <dir> [hipcc flags...]
# -> <dir>/pytorch_vit_paper_replication_amd with its own _C built from the current sources and the
# given extra hipcc flags (e.g. -DPVR_PP_PRE=0). Select it with PVR_PKG_ROOT=<dir> (bench.py,
# scripts/gemm_ab.py, scripts/attn_ab.py). Runs on the CPU host; the built tree travels with gpurun.
set -e
R="$(cd "$(dirname "$0")/.." && pwd)"
D="$1"; shift
rm -rf "$D"; mkdir -p "$D"
tar -C "$R" --exclude _build --exclude _build_debug --exclude __pycache__ --exclude '*.so' \
  -cf - pytorch_vit_paper_replication_amd | tar -C "$D" -xf -
FLAGS=$(printf "'%s'," "$@")
(cd "$D" && python -c "from pytorch_vit_paper_replication_amd import build; build.build_extension(force=True, extra_flags=($FLAGS))")
rm -rf "$D/pytorch_vit_paper_replication_amd/_build"
ls -la "$D"/pytorch_vit_paper_replication_amd/_C*.so
