#!/bin/bash
# One parameterised driver for the GPU sessions (run on the box: gpurun -- bash scripts/gpu.sh <mode> ...).
# Every GPU step runs under its own timeout; the first failing step ends the session.
#   check [tag]                 pytest -m gpu, smoke, the headline bench twice, then `prof <tag>`
#   tests [pytest args]         pytest -m gpu (or the given test selection)
#   bench <tag> [bench args]    one bench.py run -> gpurun_out/<tag>.log
#   prof <tag> [bench args]     rocprofv3 kernel stats + step timeline of the bench, in-step (side
#                               stream on) and serial (--serial-wgrad) -> gpurun_out/<tag>/
#   roofline [tag]              serial kernel trace + FETCH_SIZE / WRITE_SIZE / MFMA-busy PMC passes
#   kbench [bench_kernels args] per-kernel microbenchmarks (scripts/bench_kernels.py)
#   ddp [tag]                   DDP transports at world 1 vs no DDP (b512), per-step JSONL
#   conv [convergence args]     fused vs fp32-reference training trajectory (scripts/convergence_check.py)
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
MODE="${1:-check}"; shift

run() {  # run <seconds> <log> <cmd...>: log under gpurun_out/, stop the session on failure
  local t=$1 log=$2; shift 2
  mkdir -p "$(dirname "$R/gpurun_out/$log")"
  timeout -k 10 "$t" "$@" > "$R/gpurun_out/$log" 2>&1
  local rc=$?
  echo "[$log] rc=$rc"; tail -n "${TAILN:-3}" "$R/gpurun_out/$log" | cut -c1-250
  if [ $rc -ne 0 ]; then echo "STOP: $log rc=$rc"; exit $rc; fi
}

prof() {
  local tag=$1; shift
  local O="$R/gpurun_out/$tag"; mkdir -p "$O"
  for mode in instep serial; do
    local extra=""; [ $mode = serial ] && extra="--serial-wgrad"
    cd /tmp
    timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/$mode" -o step --output-format csv -- \
      python3 "$R/bench.py" --steps 6 --warmup 3 $extra "$@" > "$O/${mode}_run.log" 2>&1
    local rc=$?; cd "$R"
    if [ $rc -ne 0 ]; then echo "STOP prof $mode rc=$rc"; tail -5 "$O/${mode}_run.log"; exit $rc; fi
    tail -1 "$O/${mode}_run.log" | cut -c1-160
    local S T
    S=$(find "$O/$mode" -name "*kernel_stats.csv" | head -n1)
    T=$(find "$O/$mode" -name "*kernel_trace.csv" | head -n1)
    python scripts/summarize_prof.py "$S" 9 "bench kernel stats ($tag, $mode)" > "$O/kernel_stats_$mode.md" 2>&1
    python scripts/step_timeline.py "$T" > "$O/timeline_$mode.txt" 2>&1
    head -3 "$O/timeline_$mode.txt"; sed -n '5,24p' "$O/kernel_stats_$mode.md" | cut -c1-150
  done
}

case "$MODE" in
  check)
    TAG="${1:-chk}"
    TAILN=2 run 600 "${TAG}_pytest.log" python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread
    TAILN=1 run 180 "${TAG}_smoke.log" python -c "import __graft_entry__ as g; g.smoke()"
    TAILN=1 run 200 "${TAG}_bench1.log" python bench.py --steps 20 --warmup 5
    TAILN=1 run 200 "${TAG}_bench2.log" python bench.py --steps 20 --warmup 5
    prof "$TAG" ;;
  tests)
    TAILN=3 run 900 tests.log python -u -m pytest ${@:-tests -m gpu} -x -v -p no:cacheprovider --timeout 120 --timeout-method thread ;;
  bench)
    TAG="${1:-bench}"; shift
    TAILN=1 run 600 "$TAG.log" python bench.py "$@" ;;
  prof)
    TAG="${1:-prof}"; shift
    prof "$TAG" "$@" ;;
  roofline)
    O="$R/gpurun_out/${1:-roof}"; mkdir -p "$O"; cd /tmp
    timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/trace" -o k --output-format csv -- \
      python3 "$R/bench.py" --steps 3 --warmup 2 --serial-wgrad > "$O/trace.log" 2>&1 || exit $?
    i=0
    for set in "FETCH_SIZE" "WRITE_SIZE" "SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE"; do
      i=$((i+1))
      timeout -s KILL 240 rocprofv3 --kernel-trace --pmc $set -d "$O/pmc$i" -o p --output-format csv -- \
        python3 "$R/bench.py" --steps 1 --warmup 1 --serial-wgrad > "$O/pmc$i.log" 2>&1
      rc=$?; echo "pmc$i ($set) rc=$rc"; [ $rc -eq 0 ] || { tail -5 "$O/pmc$i.log"; exit $rc; }
    done ;;
  kbench)
    TAILN=40 run 600 kbench.log python scripts/bench_kernels.py "$@" ;;
  ddp)
    TAG="${1:-ddp}"; B="python bench.py --steps 30 --warmup 5 --batch 512"
    TAILN=1 run 240 "$TAG/none.log" $B
    TAILN=1 run 240 "$TAG/torch.log" $B --force-ddp --metrics-jsonl "gpurun_out/$TAG/steps_torch.jsonl"
    TAILN=1 run 240 "$TAG/torch_bf16.log" $B --force-ddp --comm-dtype bf16
    TAILN=1 run 240 "$TAG/none2.log" $B ;;
  conv)
    TAILN=2 run 1000 conv.log python -u scripts/convergence_check.py "$@" ;;
  *)
    echo "unknown mode $MODE"; exit 2 ;;
esac
exit 0
