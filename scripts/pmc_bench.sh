#!/bin/bash
# The three rocprofv3 --pmc passes bench.py reads for roofline.traffic and the issue floors
# (FETCH_SIZE, WRITE_SIZE, and the SQ issue counters), each in a run of its own, for one bench
# command; written as <dir>/{fetch_size,write_size,sq_counters}.csv.
# Usage (repo root, on the box): bash scripts/pmc_bench.sh <outdir> [bench args...]
set -e -o pipefail
D=$(cd "$(dirname "$1")" && pwd)/$(basename "$1"); shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
SQ="SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VALU2 SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_INSTS_LDS"
mkdir -p $D
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $D/f -o run -- \
  python3 $R/bench.py --no-cpu-baseline --no-upload --steps 5 "$@" > /dev/null 2> $D/f.err
timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $D/w -o run -- \
  python3 $R/bench.py --no-cpu-baseline --no-upload --steps 5 "$@" > /dev/null 2> $D/w.err
timeout -s KILL 150 rocprofv3 --pmc $SQ --output-format csv -d $D/s -o run -- \
  python3 $R/bench.py --no-cpu-baseline --no-upload --steps 5 "$@" > /dev/null 2> $D/s.err
cp $(find $D/f -name "*counter_collection.csv") $D/fetch_size.csv
cp $(find $D/w -name "*counter_collection.csv") $D/write_size.csv
cp $(find $D/s -name "*counter_collection.csv") $D/sq_counters.csv
rm -rf $D/f $D/w $D/s
