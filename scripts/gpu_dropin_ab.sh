#!/bin/bash
# Drop-in A/B: parity tests of the per-call paths, then bench.py --dropin lines (1 / 4 / 8
# threads, and 1 thread with extra environment per item).  Usage:
#   bash scripts/gpu_dropin_ab.sh TAG [name:ENV=V,...]...
set -o pipefail
T=${1:-dab}; shift
O=gpurun_out/$T; mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_extract_gpu.py tests/test_match_gpu.py tests/test_vocab_gpu.py tests/test_threads_gpu.py -m gpu -q -x \
  --timeout 300 --timeout-method thread > $O/tests.txt 2>&1 || { tail -30 $O/tests.txt; exit 1; }
tail -1 $O/tests.txt
run() {  # name threads [ENV=V...]
  local n=$1 t=$2; shift 2
  env "$@" timeout -k 10 200 python -u bench.py --dropin --threads $t --dropin-frames 300 > $O/$n.json 2> $O/$n.err || { tail -5 $O/$n.err; exit 2; }
  python3 -c "import json,sys; d=json.load(open('$O/$n.json')); x=d['dropin']; print('$n', round(d['value']), x['median_ms'], x['per_call_median_ms'])"
}
run t1 1
run t4 4
run t8 8
for item in "$@"; do
  name=${item%%:*}; envs=${item#*:}
  run $name 1 ${envs//,/ }
done
