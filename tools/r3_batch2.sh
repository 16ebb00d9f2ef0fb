# round 3 GPU batch: CNN bench with graph replay + C5/C4/C2 block-size and band A/B (temporary knobs)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
timeout -k 10 200 python3 tools/bench_cnn.py > gpurun_out/r3_bench_cnn2.json 2> gpurun_out/r3_bench_cnn2.err || exit 1
echo cnn ok
bash tools/r3_ab_c5.sh
