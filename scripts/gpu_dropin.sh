#!/bin/bash
# Drop-in latency (C ABI and shim-shaped, one thread) and the per-kernel trace of the C ABI run.
# Usage: bash scripts/gpu_dropin.sh TAG
set -o pipefail
T=${1:-dropin}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$T
mkdir -p $O
timeout -k 10 200 python $R/bench.py --dropin --threads 1 --dropin-frames 400 > $O/d1.json 2> $O/d1.err || exit 4
timeout -k 10 200 python $R/bench.py --dropin --dropin-mode shim --threads 1 --dropin-frames 400 > $O/d1s.json 2> $O/d1s.err || exit 5
python - <<PY
import json
for f in ("d1", "d1s"):
    d = json.loads(open("$O/%s.json" % f).read())
    print(f, d["value"], d["dropin"]["median_ms"], {k: v for k, v in d["dropin"]["per_call_median_ms"].items()})
PY
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
