#!/bin/bash
# Drop-in A/B: the resident frame cache (default) against the staged per-call copies
# (ORBX_NO_RESIDENT=1), C ABI and shim-shaped, one thread; then the kernel trace of the
# resident C ABI run.  Usage: bash scripts/gpu_dropin_ab.sh TAG
set -o pipefail
T=${1:-dab}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$T
mkdir -p $O
for round in 1 2; do
  for v in res staged; do
    if [ $v = staged ]; then export ORBX_NO_RESIDENT=1; else unset ORBX_NO_RESIDENT; fi
    timeout -k 10 200 python $R/bench.py --dropin --threads 1 --dropin-frames 400 > $O/${v}_d1.$round.json 2> $O/${v}_d1.$round.err || exit 4
    timeout -k 10 200 python $R/bench.py --dropin --dropin-mode shim --threads 1 --dropin-frames 400 > $O/${v}_d1s.$round.json 2> $O/${v}_d1s.$round.err || exit 5
    python - $O $v $round <<'PY'
import json, sys
o, v, r = sys.argv[1:]
for f in ("d1", "d1s"):
    d = json.loads(open("%s/%s_%s.%s.json" % (o, v, f, r)).read())
    print(v, f, round(d["value"]), d["dropin"]["median_ms"], d["dropin"]["per_call_median_ms"])
PY
  done
done
unset ORBX_NO_RESIDENT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- \
  python3 $R/bench.py --dropin --threads 1 --dropin-frames 200 > $O/kt.json 2> $O/kt.err || exit 6
cp $(find $O/trace -name "*kernel_stats.csv" | head -1) $O/kernel_stats.csv
rm -rf $O/trace
python3 - <<PY
import csv
for r in list(csv.DictReader(open("$O/kernel_stats.csv")))[:16]:
    print("%-60s %6s %9.1f" % (r["Name"][:60], r["Calls"], float(r["AverageNs"]) / 1e3))
PY
