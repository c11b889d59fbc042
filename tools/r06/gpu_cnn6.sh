# MIOpen-tuned CNN graphs, both layouts, both families; then the ensemble.
set -o pipefail
O=gpurun_out/${R06_OUT:-r06n9}
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
CNN_CONFIGS=tuned timeout -k 10 600 python3 -u tools/r06/cnn_bench.py resnet50,densenet169 > $O/tuned.log 2>&1 || { tail -40 $O/tuned.log; exit 1; }
grep '^{' $O/tuned.log | cut -c1-420
IMAGENET_TR_WORKERS=4 timeout -k 10 400 python3 -u tools/r06/imagenet_bench.py > $O/ensemble_w4.log 2>&1 || { tail -40 $O/ensemble_w4.log; exit 1; }
grep '^{' $O/ensemble_w4.log | cut -c1-250
