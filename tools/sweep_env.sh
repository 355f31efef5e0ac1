#!/bin/bash
# Run parity tests + bench for several settings of an environment knob.
# usage: KNOBS="WGSR_FWD_PPL WGSR_BWD_PPL" VALUES="1 2 4" bash tools/sweep_env.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out
mkdir -p $OUT
for v in ${VALUES}; do
  envs=""
  for k in ${KNOBS}; do envs="$envs $k=$v"; done
  env $envs timeout -k 10 400 python -m pytest tests/test_gpu_raster.py -q -x -p no:cacheprovider \
      -k "${TEST_FILTER:-golden or random or config1}" > $OUT/sweep_tests_$v.log 2>&1; rc=$?
  echo "tests $v rc=$rc" | tee -a $OUT/sweep.log
  case $rc in 124|134|137|139) exit $rc;; esac
  env $envs timeout -k 10 300 python bench.py --no-cpu-baseline ${BENCH_ARGS:-} > $OUT/sweep_bench_$v.json 2> $OUT/sweep_bench_$v.err; rc=$?
  echo "bench $v rc=$rc" | tee -a $OUT/sweep.log
  case $rc in 124|134|137|139) exit $rc;; esac
done
