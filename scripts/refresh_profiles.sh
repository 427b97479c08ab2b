#!/bin/bash
# Round-end evidence in one GPU-box session (run from the repo root on the box):
#   GPU parity tests, then for the default bench command (C2) and the AR marker command:
#   separate rocprofv3 --pmc passes (FETCH_SIZE / WRITE_SIZE / SQ counters, one group per pass),
#   the bench line computed against those passes, and rocprofv3 --kernel-trace --stats of the
#   same command.  Everything lands in gpurun_out/$TAG/ with the layout of profiles/:
#     <tag>_gpu_tests.txt, <tag>_bench.jsonl, <tag>_bench_ar.jsonl, <tag>_kernel_stats.csv,
#     <tag>_kernel_stats_ar.csv, <tag>_pmc/{fetch_size,write_size,sq_counters}.csv, <tag>_pmc_ar/...
# With a second argument "configs" it does the same for C3 C4 C5 instead (PMC passes, bench line,
# kernel stats: <tag>_pmc_c3/, <tag>_bench_c3.jsonl, <tag>_kernel_stats_c3.csv, ...), without the
# tests; the two parts fit one gpurun call each.
# PMC passes are compacted to one row per (kernel, counter) (scripts/pmc_compact.py); the
# kernel traces stay under gpurun_out/$TAG/traces (scripts/summarize_profiles.py reads them there).
# Usage: bash scripts/refresh_profiles.sh r05 [configs ["C3 C4"]]
set -e -o pipefail
TAG=${1:-r05}
PART=${2:-main}
CFGS=${3:-C3 C4 C5}
# issue-rate counters (8 SQ counters, one pass): dual-issued VALU quad-cycles and SALU
# instructions give bench.py's issue floors (profiles/valu_calibration.json)
SQ="SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VALU2 SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_INSTS_LDS"
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
cd $R
if [ "$PART" = configs ]; then
  mkdir -p $O
  for C in $CFGS; do
    c=$(echo $C | tr A-Z a-z)
    (cd /tmp && export TMPDIR=/tmp && D=$O/${TAG}_pmc_$c && mkdir -p $D &&
     timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $D/f -o run -- \
       python3 $R/bench.py --config $C --no-cpu-baseline --steps 5 > /dev/null 2> $D/f.err &&
     timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $D/w -o run -- \
       python3 $R/bench.py --config $C --no-cpu-baseline --steps 5 > /dev/null 2> $D/w.err &&
     timeout -s KILL 150 rocprofv3 --pmc $SQ --output-format csv -d $D/s -o run -- \
       python3 $R/bench.py --config $C --no-cpu-baseline --steps 5 > /dev/null 2> $D/s.err &&
     cp $(find $D/f -name "*counter_collection.csv") $D/fetch_size.csv &&
     cp $(find $D/w -name "*counter_collection.csv") $D/write_size.csv &&
     cp $(find $D/s -name "*counter_collection.csv") $D/sq_counters.csv && rm -rf $D/f $D/w $D/s &&
     python3 $R/scripts/pmc_compact.py $D)
    timeout -k 10 300 python -u bench.py --config $C --pmc-dir $O/${TAG}_pmc_$c \
      > $O/${TAG}_bench_$c.jsonl 2> $O/bench_$c.err
    cat $O/${TAG}_bench_$c.jsonl
    (cd /tmp && export TMPDIR=/tmp &&
     timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace_$c -o run -- \
       python3 $R/bench.py --config $C --no-cpu-baseline --pmc-dir $O/${TAG}_pmc_$c \
       > $O/${TAG}_bench_${c}_under_rocprof.jsonl 2> $O/trace_$c.err &&
     cp $(find $O/trace_$c -name "*kernel_stats.csv") $O/${TAG}_kernel_stats_$c.csv &&
     mkdir -p $O/traces && cp $(find $O/trace_$c -name "*kernel_trace.csv") $O/traces/kernel_trace_$c.csv &&
     rm -rf $O/trace_$c)
  done
  echo done
  exit 0
fi
rm -rf $O && mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread \
  > $O/${TAG}_gpu_tests.txt 2>&1
tail -1 $O/${TAG}_gpu_tests.txt
cd /tmp && export TMPDIR=/tmp
pmc() {  # pmc <outdir> <bench args...>
  local D=$1; shift
  mkdir -p $D
  timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $D/f -o run -- \
    python3 $R/bench.py --no-cpu-baseline --steps 5 "$@" > /dev/null 2> $D/f.err
  timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $D/w -o run -- \
    python3 $R/bench.py --no-cpu-baseline --steps 5 "$@" > /dev/null 2> $D/w.err
  timeout -s KILL 120 rocprofv3 --pmc $SQ --output-format csv -d $D/s -o run -- \
    python3 $R/bench.py --no-cpu-baseline --steps 5 "$@" > /dev/null 2> $D/s.err
  cp $(find $D/f -name "*counter_collection.csv") $D/fetch_size.csv
  cp $(find $D/w -name "*counter_collection.csv") $D/write_size.csv
  cp $(find $D/s -name "*counter_collection.csv") $D/sq_counters.csv
  rm -rf $D/f $D/w $D/s
  python3 $R/scripts/pmc_compact.py $D
}
pmc $O/${TAG}_pmc
pmc $O/${TAG}_pmc_ar --config AR
cd $R
timeout -k 10 300 python -u bench.py --pmc-dir $O/${TAG}_pmc > $O/${TAG}_bench.jsonl 2> $O/bench.err
cat $O/${TAG}_bench.jsonl
timeout -k 10 300 python -u bench.py --config AR --pmc-dir $O/${TAG}_pmc_ar \
  > $O/${TAG}_bench_ar.jsonl 2> $O/bench_ar.err
cat $O/${TAG}_bench_ar.jsonl
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- \
  python3 $R/bench.py --no-cpu-baseline --pmc-dir $O/${TAG}_pmc > $O/${TAG}_bench_under_rocprof.jsonl 2> $O/trace.err
cp $(find $O/trace -name "*kernel_stats.csv") $O/${TAG}_kernel_stats.csv
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace_ar -o run -- \
  python3 $R/bench.py --config AR --no-cpu-baseline --pmc-dir $O/${TAG}_pmc_ar \
  > $O/${TAG}_bench_ar_under_rocprof.jsonl 2> $O/trace_ar.err
cp $(find $O/trace_ar -name "*kernel_stats.csv") $O/${TAG}_kernel_stats_ar.csv
mkdir -p $O/traces
cp $(find $O/trace -name "*kernel_trace.csv") $O/traces/kernel_trace.csv
cp $(find $O/trace_ar -name "*kernel_trace.csv") $O/traces/kernel_trace_ar.csv
rm -rf $O/trace $O/trace_ar
echo done
