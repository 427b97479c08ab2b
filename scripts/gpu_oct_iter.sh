#!/bin/bash
# Octree iteration: extraction parity tests (drop-in and batch plans), then the drop-in
# latency with its kernel trace and the C2 / C5 bench lines.  Usage: bash scripts/gpu_oct_iter.sh TAG
set -o pipefail
T=${1:-oct}
mkdir -p gpurun_out/$T
timeout -k 10 500 python -u -m pytest tests/test_extract_gpu.py -m gpu -q -x \
  --timeout 240 --timeout-method thread > gpurun_out/$T/tests.txt 2>&1 || { tail -30 gpurun_out/$T/tests.txt; exit 1; }
tail -1 gpurun_out/$T/tests.txt
bash scripts/gpu_dropin.sh $T/dropin || exit 2
bash scripts/gpu_bench_quick.sh $T "C2 C5" || exit 3
