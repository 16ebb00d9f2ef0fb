#!/bin/bash
# Round 4 GPU call M: person probe (incl. half-lane xz atomics), the JLN line with the
# channels-last line, the same on the fly (fine grid projected in the kernel).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; export TMPDIR=/tmp; mkdir -p gpurun_out/r4m
timeout -k 10 300 python3 tools/person_probe.py --iters 20 > gpurun_out/r4m/person_probe.jsonl 2>&1 || { tail -20 gpurun_out/r4m/person_probe.jsonl; exit 1; }
cat gpurun_out/r4m/person_probe.jsonl
for r in 1 2; do
  timeout -k 10 200 python3 tools/bench_jln.py --frames 32 --steps 10 > gpurun_out/r4m/jln_$r.json 2> gpurun_out/r4m/jln_$r.err || { tail -20 gpurun_out/r4m/jln_$r.err; exit 1; }
  timeout -k 10 200 python3 tools/bench_jln.py --frames 32 --steps 10 --on-the-fly > gpurun_out/r4m/jln_otf_$r.json 2> gpurun_out/r4m/jln_otf_$r.err || { tail -20 gpurun_out/r4m/jln_otf_$r.err; exit 1; }
  for t in jln_$r jln_otf_$r; do python3 -c "import json; d=json.loads(open('gpurun_out/r4m/$t.json').read().strip().splitlines()[-1]); print('$t', d['us_per_proposal'], d['channels_last_input_us_per_proposal'], d['per_frame_calls_us_per_proposal'], d['cache_build'])"; done
done
echo callM done
