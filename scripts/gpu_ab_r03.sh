#!/bin/bash
# Round-3 A/B of the per-cell FAST kernel (k_fast_cells) against the round-2 tile path
# (ORBX_FAST_LEGACY=1), plus the parity tests that exercise them.  Every GPU step has its own
# time limit and the steps stop at the first failure.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_extract_gpu.py tests/test_pipeline_gpu.py tests/test_projection_gpu.py \
  -m gpu -v --maxfail=3 --timeout 300 --timeout-method thread -k "not topology" > gpurun_out/r03_cells_tests.txt 2>&1 || exit 1
timeout -k 10 200 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-upload > gpurun_out/r03_cells_bench.jsonl 2> gpurun_out/r03_cells_bench.err || exit 2
ORBX_FAST_LEGACY=1 timeout -k 10 200 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-upload > gpurun_out/r03_legacy_bench.jsonl 2>> gpurun_out/r03_cells_bench.err || exit 3
timeout -k 10 200 python bench.py --config C5 --steps 10 --warmup 2 --no-cpu-baseline --no-upload > gpurun_out/r03_cells_bench_c5.jsonl 2>> gpurun_out/r03_cells_bench.err || exit 4
ORBX_FAST_LEGACY=1 timeout -k 10 200 python bench.py --config C5 --steps 10 --warmup 2 --no-cpu-baseline --no-upload > gpurun_out/r03_legacy_bench_c5.jsonl 2>> gpurun_out/r03_cells_bench.err || exit 5
