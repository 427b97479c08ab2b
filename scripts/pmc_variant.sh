#!/bin/bash
# SQ / FETCH / WRITE counter passes of one bench command for the default build or an experiment
# build in ar_orbslam2_amd/_lib_exp/<variant>, compacted to one row per (kernel, counter), then
# the bench line computed against them.  Usage: bash scripts/pmc_variant.sh TAG VARIANT CONFIG
set -e -o pipefail
T=$1; V=$2; C=$3
R=${GRAFT_REPO_ROOT:-$(pwd)}
D=$R/gpurun_out/$T/pmc_${V}_$C
mkdir -p $D
if [ "$V" != default ]; then export ORBX_LIB_DIR=$R/ar_orbslam2_amd/_lib_exp/$V ORBX_ALLOW_CUSTOM_BUILD=1; fi
SQ="SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VALU2 SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_INSTS_LDS"
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc $SQ --output-format csv -d $D/s -o run -- \
  python3 $R/bench.py --config $C --no-cpu-baseline --no-upload --steps 5 > /dev/null 2> $D/s.err
cp $(find $D/s -name "*counter_collection.csv") $D/sq_counters.csv
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $D/f -o run -- \
  python3 $R/bench.py --config $C --no-cpu-baseline --no-upload --steps 5 > /dev/null 2> $D/f.err
cp $(find $D/f -name "*counter_collection.csv") $D/fetch_size.csv
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $D/w -o run -- \
  python3 $R/bench.py --config $C --no-cpu-baseline --no-upload --steps 5 > /dev/null 2> $D/w.err
cp $(find $D/w -name "*counter_collection.csv") $D/write_size.csv
rm -rf $D/s $D/f $D/w
python3 $R/scripts/pmc_compact.py $D
cd $R
timeout -k 10 200 python bench.py --config $C --steps 20 --warmup 3 --no-cpu-baseline --no-upload --pmc-dir $D > $D/bench.jsonl 2> $D/bench.err
python3 - $D <<'PY'
import csv, json, sys
D = sys.argv[1]
d = json.loads(open(D + "/bench.jsonl").read())
print("value", round(d["value"]), "dominant", d["roofline"]["kernel"], {k: v for k, v in d["roofline"]["stages_ms_per_step"].items() if v > 0.05})
per = {}
for r in csv.DictReader(open(D + "/sq_counters.csv")):
    k = r["Kernel_Name"].split("(")[0].replace("void orbx::", "")
    per.setdefault(k, {}).setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
for k, cs in sorted(per.items()):
    avg = {c: sum(v) / len(v) for c, v in cs.items()}
    qc = avg.get("SQ_ACTIVE_INST_VALU", 0) - avg.get("SQ_ACTIVE_INST_VALU2", 0)
    floor_us = qc * 4 / 1024 / 2400
    wait = avg.get("SQ_WAIT_ANY", 0) / max(avg.get("SQ_WAVE_CYCLES", 1), 1)
    print(f"  {k[:60]:60s} valu_floor_us {floor_us:8.1f} valu_instr {avg.get('SQ_INSTS_VALU',0):12.0f} lds {avg.get('SQ_INSTS_LDS',0):11.0f} wait {wait:.2f}")
PY
