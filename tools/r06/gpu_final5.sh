# Final tree: full GPU suite, smoke(), headline, then the ImageNet ensemble over REST.
set -o pipefail
O=gpurun_out/${R06_OUT:-r06z2}
R06_OUT=${R06_OUT:-r06z2} bash tools/r06/gpu_final4.sh || exit 1
timeout -k 10 700 python3 -u tools/r06/imagenet_rest_bench.py > $O/rest.log 2>&1 || { tail -30 $O/rest.log; exit 1; }
grep '^{' $O/rest.log
