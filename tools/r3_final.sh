#!/bin/bash
# Round-3 end-of-session refresh: full GPU tests, smoke, the default bench line (CPU
# baseline + traffic PMC) and its rocprofv3 kernel stats, then one line per config.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 120 --timeout-method thread > gpurun_out/fin_tests.log 2>&1 || { tail -40 gpurun_out/fin_tests.log; exit 1; }
tail -1 gpurun_out/fin_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/fin_smoke.log 2>&1 || { tail -20 gpurun_out/fin_smoke.log; exit 1; }
echo "smoke ok"
timeout -k 10 600 python bench.py > gpurun_out/fin_bench.json 2> gpurun_out/fin_bench.err || { tail -20 gpurun_out/fin_bench.err; exit 1; }
tail -1 gpurun_out/fin_bench.json | cut -c1-400
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/fin_prof -o run -- python3 bench.py --traffic off --cpu-baseline off > gpurun_out/fin_prof.log 2>&1 || { tail -20 gpurun_out/fin_prof.log; exit 1; }
echo "prof ok"
CPU=on bash tools/bench_all.sh || exit 1
