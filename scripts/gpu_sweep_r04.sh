mkdir -p gpurun_out/sweep4
for r in 1 2; do for BS in "512 3" "768 2" "384 4" "1024 3" "256 6" "1536 1"; do set -- $BS
timeout -k 10 150 python -u bench.py --config C2 --batch $1 --streams $2 --steps 20 --no-cpu-baseline --no-upload --no-profile > gpurun_out/sweep4/c2_$1_$2_$r.jsonl 2>/dev/null || exit 1
python -c "import json; d=json.loads(open('gpurun_out/sweep4/c2_$1_$2_$r.jsonl').read().splitlines()[-1]); print('$1 x $2', round(d['value']))"
done; done
