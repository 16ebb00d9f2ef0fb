#!/bin/bash
# Same-box A/B of libfvp builds on the JLN line (tools/bench_jln.py):
#   LIBS="ab_libs/a.so ab_libs/b.so" REPS=3 bash tools/r4_ab_jln.sh
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; export TMPDIR=/tmp; mkdir -p gpurun_out/ab_jln
for r in $(seq 1 ${REPS:-2}); do
  for lib in ${LIBS}; do
    n=$(basename $lib .so)
    FVP_LIB=$PWD/$lib timeout -k 10 200 python3 tools/bench_jln.py --frames ${FRAMES:-32} --steps ${STEPS:-10} \
      > gpurun_out/ab_jln/${n}_$r.json 2> gpurun_out/ab_jln/${n}_$r.err || { tail -20 gpurun_out/ab_jln/${n}_$r.err; exit 1; }
    python3 -c "import json,sys; d=json.loads(open('gpurun_out/ab_jln/${n}_$r.json').read().strip().splitlines()[-1]); print('$n rep$r', d['us_per_proposal'], d['per_frame_calls_us_per_proposal'], d['tap_stream']['achieved_tb_s'], d.get('cache_build'))"
  done
done
