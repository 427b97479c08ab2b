#!/bin/bash
# One rocprofv3 counter pass of the default bench command on the L1 -> L2 request counters
# (per-kernel vector-L1 traffic).  Usage: bash scripts/gpu_tcp_pass.sh TAG [bench args...]
# (ORBX_LIB_DIR / ORBX_ALLOW_CUSTOM_BUILD in the environment select an experiment build)
set -o pipefail
T=${1:-tcp}; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$T
case "${ORBX_LIB_DIR:-}" in ""|/*) ;; *) export ORBX_LIB_DIR=$R/$ORBX_LIB_DIR ;; esac
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 150 rocprofv3 --pmc TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum TCC_HIT_sum TCC_MISS_sum \
  --output-format csv -d $O/p -o run -- python3 $R/bench.py --no-cpu-baseline --no-upload --steps 5 "$@" > $O/b.json 2> $O/p.err || { tail -5 $O/p.err; exit 1; }
cp $(find $O/p -name "*counter_collection.csv") $O/tcp.csv && rm -rf $O/p
python3 - $O/tcp.csv <<'PY'
import csv, sys, collections
agg = collections.defaultdict(float); disp = collections.defaultdict(set)
for r in csv.DictReader(open(sys.argv[1])):
    k = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("orbx::", "")
    agg[(k, r["Counter_Name"])] += float(r["Counter_Value"]); disp[k].add(r["Dispatch_Id"])
for k in sorted(disp):
    n = len(disp[k])
    print("%-40s %5d" % (k[:40], n), " ".join("%s=%.3g" % (c.replace("_sum", ""), agg[(k, c)] / n) for (kk, c) in sorted(agg) if kk == k))
PY
