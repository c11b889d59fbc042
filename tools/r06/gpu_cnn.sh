# ImageNet CNN serving path: kernel-level bench + the ensemble smoke.
set -o pipefail
O=gpurun_out/${R06_OUT:-r06n}
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
[ -n "$SKIP_CNN" ] || timeout -k 10 500 python3 -u tools/r06/cnn_bench.py resnet50 > $O/cnn_resnet.log 2>&1 || { tail -40 $O/cnn_resnet.log; exit 1; }
[ -n "$SKIP_CNN" ] || grep "^{" $O/cnn_resnet.log
[ -n "$SKIP_CNN" ] || timeout -k 10 500 python3 -u tools/r06/cnn_bench.py densenet169 > $O/cnn_densenet.log 2>&1 || { tail -40 $O/cnn_densenet.log; exit 1; }
[ -n "$SKIP_CNN" ] || grep "^{" $O/cnn_densenet.log
timeout -k 10 400 python3 -u tools/r06/imagenet_bench.py > $O/ensemble.log 2>&1 || { tail -40 $O/ensemble.log; exit 1; }
grep '^{' $O/ensemble.log
