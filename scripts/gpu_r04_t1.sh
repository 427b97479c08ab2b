set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 1000 python -u -m pytest -x -v -s --timeout 900 --timeout-method thread tests/test_projection_gpu.py tests/test_dropin_gpu.py tests/test_distributed_gpu.py "tests/test_pipeline_gpu.py::test_bench_timed_topology_matches_oracle[C2-argv0]" "tests/test_pipeline_gpu.py::test_bench_timed_topology_matches_oracle[C3-argv1]" "tests/test_pipeline_gpu.py::test_bench_timed_topology_matches_oracle[C4-argv2]" > gpurun_out/r04_t1.log 2>&1
