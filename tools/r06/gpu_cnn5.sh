# CNN dtype / layout / MIOpen-find A/B (ResNet-50, DenseNet-169).
set -o pipefail
O=gpurun_out/${R06_OUT:-r06n8}
mkdir -p $O
CNN_CONFIGS=layouts timeout -k 10 400 python3 -u tools/r06/cnn_bench.py resnet50,densenet169 > $O/layouts.log 2>&1 || { tail -40 $O/layouts.log; exit 1; }
grep '^{' $O/layouts.log | cut -c1-400
CNN_BENCHMARK=1 timeout -k 10 500 python3 -u tools/r06/cnn_bench.py resnet50 > $O/find.log 2>&1 || { tail -40 $O/find.log; exit 1; }
grep '^{' $O/find.log | cut -c1-400
