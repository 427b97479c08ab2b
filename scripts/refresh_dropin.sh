#!/bin/bash
# Drop-in per-frame path evidence (bench.py --dropin at 1 / 4 / 8 host threads, plus a
# rocprofv3 kernel trace of the one-thread run) into gpurun_out/$TAG/ as profiles/ names it:
#   <tag>_dropin_t{1,4,8}.json, <tag>_dropin_shim_t1.json, <tag>_dropin_under_rocprof.json,
#   <tag>_dropin_kernel_stats.csv
# Usage: bash scripts/refresh_dropin.sh r02
set -e -o pipefail
TAG=${1:-r02}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
for T in 1 4 8; do
  timeout -k 10 200 python -u bench.py --dropin --threads $T > $O/${TAG}_dropin_t$T.json 2> $O/dropin_t$T.err
  tail -c 300 $O/${TAG}_dropin_t$T.json
done
# the reference-side shims' per-call marshalling around the same calls (lazy pyramid export,
# std::map FeatureVector -> CSR, MapPoint masks), one thread
timeout -k 10 200 python -u bench.py --dropin --threads 1 --dropin-mode shim > $O/${TAG}_dropin_shim_t1.json 2> $O/dropin_shim_t1.err
tail -c 300 $O/${TAG}_dropin_shim_t1.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace_dropin -o run -- \
  python3 $R/bench.py --dropin --threads 1 > $O/${TAG}_dropin_under_rocprof.json 2> $O/trace_dropin.err
cp $(find $O/trace_dropin -name "*kernel_stats.csv") $O/${TAG}_dropin_kernel_stats.csv
rm -rf $O/trace_dropin
echo done
