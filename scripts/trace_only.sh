#!/bin/bash
# rocprofv3 kernel trace + stats of one bench command.  Usage: bash scripts/trace_only.sh TAG "bench args"
set -e -o pipefail
TAG=${1:-trace}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 $R/bench.py --steps 4 --warmup 2 --no-cpu-baseline ${2:-} > $O/bench.jsonl 2> $O/err.txt
python3 - $O/trace/run_kernel_stats.csv <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"])):
    print(f'{r["Name"].split("(")[0][:60]:60s} calls {r["Calls"]:>6s} avg_us {float(r["AverageNs"])/1e3:9.2f}')
PY
