#!/bin/bash
# Round 4 GPU call K: the -m gpu suite on the tree (eager fast path past the custom-op
# dispatcher, xy plane written directly), smoke, the person probe, JLN A/B (jdxy = xy
# memset + deferred stores, jxyd = the product), C2 / C3 B=8 bench lines.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; export TMPDIR=/tmp; mkdir -p gpurun_out
TAG=r4k WORKLOADS="c2:256 c3:8" bash tools/r3_check.sh || exit 1
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r4k_smoke.log 2>&1 || { tail -20 gpurun_out/r4k_smoke.log; exit 1; }
tail -3 gpurun_out/r4k_smoke.log
timeout -k 10 300 python3 tools/person_probe.py --iters 20 > gpurun_out/r4k_person_probe.jsonl 2>&1 || { tail -20 gpurun_out/r4k_person_probe.jsonl; exit 1; }
cat gpurun_out/r4k_person_probe.jsonl
LIBS="ab_libs/jdxy.so ab_libs/jxyd.so" REPS=3 bash tools/r4_ab_jln.sh || exit 1
echo callK done
