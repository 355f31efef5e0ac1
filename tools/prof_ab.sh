#!/bin/bash
# rocprofv3 kernel stats of bench.py per A/B library: AB_LIBS="base name ..."
# (lib/variants/<name>.so), BENCH_ARGS per run -> gpurun_out/profab_<name><SFX>/
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
R=$PWD
for v in ${AB_LIBS}; do
  if [ "$v" = base ]; then lib=$R/wildgs-slam-blackwell_amd/lib/libwgsr.so; else lib=$R/wildgs-slam-blackwell_amd/lib/variants/$v.so; fi
  (cd /tmp && WGSR_LIB=$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/profab_$v${SFX:-} -o run --output-format csv -- python $R/bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-profile --no-knn ${BENCH_ARGS:-} > $R/gpurun_out/profab_$v${SFX:-}.json 2> $R/gpurun_out/profab_$v${SFX:-}.err) || exit $?
done
