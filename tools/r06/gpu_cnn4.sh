# Ensemble with the transformer in 4 / 8 worker processes.
set -o pipefail
O=gpurun_out/${R06_OUT:-r06n7}
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
for w in 4 8; do
  IMAGENET_TR_WORKERS=$w timeout -k 10 300 python3 -u tools/r06/imagenet_bench.py > $O/ensemble_w$w.log 2>&1 || { tail -40 $O/ensemble_w$w.log; exit 1; }
  grep '^{"graph' $O/ensemble_w$w.log | cut -c1-250
done
