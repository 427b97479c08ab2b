#!/bin/bash
# One-thread drop-in run under rocprofv3 with kernel, HIP API and memory-copy traces (no
# counters): where a call's wall time goes.  Usage: bash scripts/gpu_dropin_trace.sh TAG
set -e -o pipefail
TAG=${1:-dtr}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --hip-trace --memory-copy-trace --output-format csv -d $O/tr -o run -- \
  python3 $R/bench.py --dropin --threads 1 --dropin-frames 60 --warmup-frames 10 > $O/tr.json 2> $O/tr.err
for k in kernel_trace hip_api_trace memory_copy_trace; do
  f=$(find $O/tr -name "*${k}.csv" | head -1)
  [ -n "$f" ] && cp "$f" $O/$k.csv
done
rm -rf $O/tr
ls -la $O
