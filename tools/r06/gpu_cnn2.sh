# Ensemble throughput vs the interpreter switch interval (default rule, 5 ms, 0.05 ms).
set -o pipefail
O=gpurun_out/${R06_OUT:-r06n5}
mkdir -p $O
for si in "" 0.005 0.00005; do
  SCA_PY_SWITCH_INTERVAL=$si timeout -k 10 300 python3 -u tools/r06/imagenet_bench.py > $O/ensemble_si$si.log 2>&1 || { tail -40 $O/ensemble_si$si.log; exit 1; }
  grep '^{' $O/ensemble_si$si.log | cut -c1-260
done
