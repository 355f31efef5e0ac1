#!/bin/bash
# rocprofv3 kernel stats of bench.py per environment setting: ENV_AB="base NAME=VALUE ..."
# ("base" = no extra variable), REPS rounds interleaved, BENCH_ARGS per run
# -> gpurun_out/profenv_<tag>_<rep>/ (+ .json bench line)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
R=$PWD
for rep in $(seq 1 ${REPS:-1}); do
  for e in ${ENV_AB}; do
    tag=$(echo "$e" | sed 's|=.*/|_|; s|\.so$||' | tr '=' '_')  # (a library path: its file name)
    out=$R/gpurun_out/profenv_${tag}${SFX:-}_$rep
    if [ "$e" = base ]; then
      (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out -o run --output-format csv -- python $R/bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-profile --no-knn ${BENCH_ARGS:-} > $out.json 2> $out.err) || exit $?
    else
      (cd /tmp && export "$e" && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out -o run --output-format csv -- python $R/bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-profile --no-knn ${BENCH_ARGS:-} > $out.json 2> $out.err) || exit $?
    fi
  done
done
