#!/bin/bash
# rocprofv3 kernel-trace + stats of a short bench run; summary lands in gpurun_out/prof/
R=${GRAFT_REPO_ROOT:-$(pwd)}
export TMPDIR=/tmp
mkdir -p $R/gpurun_out/prof
cd /tmp && rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof -o bench -- \
  python3 $R/bench.py --steps ${STEPS:-2} --warmup 1 --cpu-baseline off "$@"
