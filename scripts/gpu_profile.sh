#!/bin/bash
# One GPU-box session: parity tests, the bench line, rocprofv3 kernel stats of the same bench
# command, and separate --pmc passes (FETCH_SIZE, WRITE_SIZE, SQ counters) for roofline.traffic.
# Usage (from the repo root, on the box): bash scripts/gpu_profile.sh TAG
set -e -o pipefail
TAG=${1:-r01}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
timeout -k 10 600 python -m pytest tests -m gpu -x -q > $O/gpu_tests.txt 2>&1
tail -2 $O/gpu_tests.txt
timeout -k 10 300 python bench.py > $O/bench.jsonl 2> $O/bench.err
cat $O/bench.jsonl
BENCH="bench.py ${2:-}"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 $R/$BENCH > $O/bench_under_rocprof.jsonl 2> $O/rocprof_trace.err
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_fetch -o run -- python3 $R/$BENCH > /dev/null 2> $O/pmc_fetch.err
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc_write -o run -- python3 $R/$BENCH > /dev/null 2> $O/pmc_write.err
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_INSTS_LDS SQ_INSTS_SALU --output-format csv -d $O/pmc_sq -o run -- python3 $R/$BENCH > /dev/null 2> $O/pmc_sq.err
find $O -name "*.csv" | sort
echo done
