# A/B router graph after the engine continuation refactor: abtest + headline,
# plus one CPU profile of the abtest server.
set -o pipefail
O=gpurun_out/${R06_OUT:-r06l}
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
for g in abtest single abtest; do
  if [ $g = single ]; then a=""; else a="--graph $g"; fi
  timeout -k 10 300 python3 bench.py $a --extras none > $O/$g.log 2>&1 || { tail -30 $O/$g.log; exit 1; }
  grep '^{' $O/$g.log | tail -1 | cut -c1-240
done
timeout -k 10 300 python3 bench.py --graph abtest --extras none --cpu-profile $O/abtest.json > $O/abtest_prof.log 2>&1 || { tail -30 $O/abtest_prof.log; exit 1; }
grep '^{' $O/abtest_prof.log | tail -1 | cut -c1-240
