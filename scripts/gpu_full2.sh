#!/bin/bash
# Full -m gpu suite, then every config's bench line (stage times).  Usage: bash scripts/gpu_full2.sh TAG
set -o pipefail
T=${1:-full2}
mkdir -p gpurun_out/$T
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread \
  > gpurun_out/$T/tests.txt 2>&1 || { tail -40 gpurun_out/$T/tests.txt; exit 1; }
tail -1 gpurun_out/$T/tests.txt
bash scripts/gpu_bench_quick.sh $T "C3 C4 AR" || exit 2
