# Mahalanobis refresh (round 5): parity tests, tail latency, kernel stats.
set -o pipefail
mkdir -p gpurun_out/r05m
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u -m pytest tests/test_outliers.py -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/r05m/pytest_outliers.log 2>&1 || { tail -30 gpurun_out/r05m/pytest_outliers.log; exit 1; }
tail -2 gpurun_out/r05m/pytest_outliers.log
timeout -k 10 300 python -u tools/maha_bench.py --p 9 32 64 --requests 2000 --threads 16 --out gpurun_out/r05m/maha.json > gpurun_out/r05m/maha.log 2>&1 || { tail -20 gpurun_out/r05m/maha.log; exit 1; }
tail -3 gpurun_out/r05m/maha.log
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/r05m/prof" -o maha -- python "$GRAFT_REPO_ROOT/tools/maha_bench.py" --p 64 --requests 2000 --threads 1 > "$GRAFT_REPO_ROOT/gpurun_out/r05m/prof.log" 2>&1
rc=$?; tail -3 "$GRAFT_REPO_ROOT/gpurun_out/r05m/prof.log"; exit $rc
