# Server CPU profiles: the single-model headline vs the A/B router graph.
set -o pipefail
O=gpurun_out/${R06_OUT:-r06k}
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python3 bench.py --extras none --cpu-profile $O/single.json > $O/single.log 2>&1 || { tail -30 $O/single.log; exit 1; }
grep '^{' $O/single.log | tail -1 | cut -c1-200
timeout -k 10 300 python3 bench.py --graph abtest --extras none --cpu-profile $O/abtest.json > $O/abtest.log 2>&1 || { tail -30 $O/abtest.log; exit 1; }
grep '^{' $O/abtest.log | tail -1 | cut -c1-200
timeout -k 10 300 python3 bench.py --graph abtest --extras none --cpu-profile $O/abtest_paths.json --cpu-profile-depth 6 > $O/abtest_paths.log 2>&1 || { tail -30 $O/abtest_paths.log; exit 1; }
