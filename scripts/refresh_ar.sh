#!/bin/bash
# The AR marker config's evidence alone (PMC passes, bench line, kernel stats), as
# refresh_profiles.sh's main part writes it.  Usage: bash scripts/refresh_ar.sh r03
set -e -o pipefail
TAG=${1:-r03}
SQ="SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VALU2 SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_INSTS_LDS"
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
D=$O/${TAG}_pmc_ar
mkdir -p $D
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $D/f -o run -- \
  python3 $R/bench.py --config AR --no-cpu-baseline --steps 5 > /dev/null 2> $D/f.err
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $D/w -o run -- \
  python3 $R/bench.py --config AR --no-cpu-baseline --steps 5 > /dev/null 2> $D/w.err
timeout -s KILL 120 rocprofv3 --pmc $SQ --output-format csv -d $D/s -o run -- \
  python3 $R/bench.py --config AR --no-cpu-baseline --steps 5 > /dev/null 2> $D/s.err
cp $(find $D/f -name "*counter_collection.csv") $D/fetch_size.csv
cp $(find $D/w -name "*counter_collection.csv") $D/write_size.csv
cp $(find $D/s -name "*counter_collection.csv") $D/sq_counters.csv
rm -rf $D/f $D/w $D/s
python3 $R/scripts/pmc_compact.py $D
cd $R
timeout -k 10 300 python -u bench.py --config AR --pmc-dir $D > $O/${TAG}_bench_ar.jsonl 2> $O/bench_ar.err
cat $O/${TAG}_bench_ar.jsonl
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace_ar -o run -- \
  python3 $R/bench.py --config AR --no-cpu-baseline --pmc-dir $D \
  > $O/${TAG}_bench_ar_under_rocprof.jsonl 2> $O/trace_ar.err
cp $(find $O/trace_ar -name "*kernel_stats.csv") $O/${TAG}_kernel_stats_ar.csv
mkdir -p $O/traces
cp $(find $O/trace_ar -name "*kernel_trace.csv") $O/traces/kernel_trace_ar.csv
rm -rf $O/trace_ar
echo done
