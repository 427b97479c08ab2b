#!/bin/bash
# Experiment builds of liborbx.so with -D overrides, one directory each under
# ar_orbslam2_amd/_lib_exp/<name>/ (run here, on the CPU; the .so files travel with gpurun).
# Usage: bash scripts/build_variants.sh name1 "-DFOO=1 -DBAR=0" name2 "-DFOO=0" ...
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
while [ $# -ge 2 ]; do
  make -s -j8 -C $R/ar_orbslam2_amd/csrc OUT=$R/ar_orbslam2_amd/_lib_exp/$1 EXTRA="$2" \
    $R/ar_orbslam2_amd/_lib_exp/$1/liborbx.so
  shift 2
done
