#!/bin/bash
# Drop-in path: host-thread and hardware-queue scan, plus kernel traces of the 1- and 8-thread
# runs (per-dispatch CSV: queue, start, end) to separate queue oversubscription from host-side
# serialisation.  Usage (repo root, on the box): bash scripts/gpu_dropin_scan.sh TAG
set -e -o pipefail
TAG=${1:-dscan}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
run() {  # name threads [ENV=V]
  local n=$1 t=$2; shift 2
  env "$@" timeout -k 10 200 python -u bench.py --dropin --threads $t --dropin-frames 300 > $O/$n.json 2> $O/$n.err
  python3 -c "import json,sys; d=json.load(open('$O/$n.json')); x=d['dropin']; print('$n', round(d['value']), x['median_ms'], x['per_call_median_ms'])"
}
run t1 1
run t2 2
run t4 4
run t8 8
run t8_q8 8 GPU_MAX_HW_QUEUES=8
run t8_q16 8 GPU_MAX_HW_QUEUES=16
run t4_q16 4 GPU_MAX_HW_QUEUES=16
cd /tmp && export TMPDIR=/tmp
for t in 1 8; do
  timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $O/tr$t -o run -- \
    python3 $R/bench.py --dropin --threads $t --dropin-frames 150 > $O/tr$t.json 2> $O/tr$t.err
  cp $(find $O/tr$t -name "*kernel_trace.csv") $O/kernel_trace_t$t.csv
  rm -rf $O/tr$t
done
echo done
