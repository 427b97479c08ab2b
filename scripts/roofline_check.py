"""Cross-check bench.py's roofline kernel duration (HIP events, single-stream roofline pass)
against the rocprofv3 kernel trace of the same command.

The timed region runs several camera streams concurrently, so the trace's overall average for
a kernel includes launches that share the GPU with other streams' kernels; bench.py times the
roofline kernel in a separate pass on stream 0 alone (its last `--roofline-steps` launches).
This prints both the overall trace average and the average over those last launches.

Usage: python3 scripts/roofline_check.py <trace dir | kernel_trace.csv> <bench json line file>
       [roofline_steps]"""
import csv
import json
import sys

trace_dir, bench_file = sys.argv[1], sys.argv[2]
steps = int(sys.argv[3]) if len(sys.argv) > 3 else 5
b = json.loads(open(bench_file).read().strip().splitlines()[-1])
kern = b["roofline"]["kernel"]
import os
path = trace_dir if trace_dir.endswith(".csv") else os.path.join(trace_dir, "run_kernel_trace.csv")
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bench import kernel_instance  # noqa: E402
# the exact instances the bench line's roofline pass launched for the stage
inst = set(b["roofline"].get("kernel_instances") or [])
rows = [r for r in csv.DictReader(open(path)) if kernel_instance(r["Kernel_Name"]) in inst]
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
dur = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in rows]
# the roofline pass's dispatches: every instance of the stage's kernels (k_fast_cells: the pair
# kernel and two cell instances) times its launches per step (k_pyramid: one per pyramid stage)
lps = b["roofline"].get("launches_per_step", 1) or 1
ninst = len({r["Kernel_Name"] for r in rows})
solo = dur[-int(round(steps * lps * ninst)):]
per_launch = sum(solo) / (steps * lps)
print(f"kernel {kern} ({', '.join(sorted(inst))}): {len(dur)} dispatches ({ninst} instance(s), {lps} launch(es) per step)")
print(f"  trace average, all dispatches (timed region with concurrent streams + roofline pass): "
      f"{sum(dur) / len(dur):.2f} us")
print(f"  trace, last {len(solo)} dispatches (roofline pass, stream 0 alone), per launch: "
      f"{per_launch:.2f} us")
print(f"  bench.py roofline avg_launch_us (HIP events, same pass): {b['roofline']['avg_launch_us']} us")
