# Fused residual add+ReLU (ResNet): op + CNN tests, ResNet-50 bench (serving default).
set -o pipefail
O=gpurun_out/${R06_OUT:-r06y}
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -m gpu tests/test_ops_gpu.py tests/test_cnn.py > $O/pytest.log 2>&1 || { grep -E "FAILED|Error" $O/pytest.log | head; tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
CNN_CONFIGS=default timeout -k 10 400 python3 -u tools/r06/cnn_bench.py resnet50 > $O/resnet.log 2>&1 || { tail -30 $O/resnet.log; exit 1; }
grep '^{' $O/resnet.log | cut -c1-420
