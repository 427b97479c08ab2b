set -e -o pipefail
mkdir -p gpurun_out/v6
for C in C4 C2; do for M in 65536 49152 40960 32768 24576; do
ORBX_PY_MAX_SMEM=$M timeout -k 10 120 python -u bench.py --config $C --no-cpu-baseline --no-upload --steps 10 | python -c "import json,sys; d=json.loads(sys.stdin.read().splitlines()[-1]); print('$C', $M, d['value'], d['roofline']['stages_ms_per_step']['k_pyramid'])" >> gpurun_out/v6/py.txt
done; done
cat gpurun_out/v6/py.txt
