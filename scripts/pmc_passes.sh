#!/bin/bash
# Stall/LDS/VALU breakdown per kernel: rocprofv3 --pmc passes (one counter group each) of one
# bench command.  Usage (repo root, on the box): bash scripts/pmc_passes.sh TAG "bench args"
set -e -o pipefail
TAG=${1:-pmc}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p $O
BENCH="bench.py --steps 4 --warmup 2 --no-cpu-baseline --no-upload ${2:-}"
cd /tmp && export TMPDIR=/tmp
i=0
for grp in "SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" \
           "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS" \
           "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_SCA SQ_INSTS_VALU" \
           "GRBM_GUI_ACTIVE SQ_BUSY_CYCLES SQ_INSTS_LDS SQ_INSTS_SALU"; do
  i=$((i + 1))
  timeout -k 10 300 rocprofv3 --pmc $grp --output-format csv -d $O/p$i -o run -- python3 $R/$BENCH > /dev/null 2> $O/p$i.err
done
python3 $R/scripts/pmc_table.py $O > $O/table.txt
cat $O/table.txt
