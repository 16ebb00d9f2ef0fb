set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/nt_tests.log 2>&1 || { echo tests failed; tail -30 gpurun_out/nt_tests.log; exit 1; }
tail -2 gpurun_out/nt_tests.log
timeout -k 10 120 python tools/latency_b1.py > gpurun_out/nt_lat.log 2>&1 && cat gpurun_out/nt_lat.log | tail -3
timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/nt_prof -o run -- python3 tools/latency_b1.py > gpurun_out/nt_prof.log 2>&1
echo prof rc=$?
