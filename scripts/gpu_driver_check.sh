#!/bin/bash
# What the driver runs at round end, minus the test suite: smoke(), then the default bench line
# (its PMC fields must bind to profiles/<round>_pmc).  Usage: bash scripts/gpu_driver_check.sh TAG
set -o pipefail
T=${1:-drv}
mkdir -p gpurun_out/$T
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/$T/smoke.txt 2>&1 || { tail -20 gpurun_out/$T/smoke.txt; exit 1; }
tail -1 gpurun_out/$T/smoke.txt
timeout -k 10 600 python bench.py > gpurun_out/$T/bench.json 2> gpurun_out/$T/bench.err || { tail -20 gpurun_out/$T/bench.err; exit 2; }
python - <<PY
import json
d = json.loads(open("gpurun_out/$T/bench.json").read().strip().splitlines()[-1])
r = d["roofline"]
print(d["value"], r["kernel"], r["frac"], r.get("traffic"), r["issue_roofline"].get("frac"), r.get("traffic_note", "")[:120])
PY
