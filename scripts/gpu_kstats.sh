#!/bin/bash
# Kernel trace stats + one SQ counter pass of a bench command (roofline pass times per kernel).
# Usage: bash scripts/gpu_kstats.sh TAG "bench args"
set -o pipefail
T=${1:-ks}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$T
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- \
  python3 $R/bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-upload ${2:-} > $O/bench.jsonl 2> $O/trace.err || exit 1
cp $(find $O/trace -name "*kernel_stats.csv") $O/kernel_stats.csv
cp $(find $O/trace -name "*kernel_trace.csv") $O/kernel_trace.csv
rm -rf $O/trace
SQ="SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VALU2 SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_INSTS_LDS"
timeout -s KILL 150 rocprofv3 --pmc $SQ --output-format csv -d $O/s -o run -- \
  python3 $R/bench.py --steps 4 --warmup 2 --no-cpu-baseline --no-upload ${2:-} > /dev/null 2> $O/s.err || exit 2
cp $(find $O/s -name "*counter_collection.csv") $O/sq.csv
rm -rf $O/s
python3 $R/scripts/pmc_compact.py $O > /dev/null 2>&1 || true
python3 - <<PY
import csv, collections
rows = list(csv.DictReader(open("$O/kernel_stats.csv")))
for r in rows[:14]:
    print("%-60s %6s %10.1f" % (r["Name"][:60], r["Calls"], float(r["AverageNs"]) / 1e3))
d = collections.defaultdict(dict)
for r in csv.DictReader(open("$O/sq.csv")):
    d[r["Kernel_Name"].split("(")[0][-40:]].setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
for k, cs in d.items():
    a = {c: sum(v) / len(v) for c, v in cs.items()}
    w = max(a.get("SQ_WAVES", 1), 1)
    print("%-40s waves %7d valu/w %7.0f salu/w %6.0f lds/w %6.0f wait%% %4.1f" % (k, w, a.get("SQ_INSTS_VALU", 0) / w,
          a.get("SQ_INSTS_SALU", 0) / w, a.get("SQ_INSTS_LDS", 0) / w, 100 * a.get("SQ_WAIT_ANY", 0) / max(a.get("SQ_WAVE_CYCLES", 1), 1)))
PY
