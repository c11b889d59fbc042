set -o pipefail
O=gpurun_out/${R06_OUT:-r06n3}
mkdir -p $O
timeout -k 10 400 python3 -u tools/r06/imagenet_isolate.py > $O/isolate.log 2>&1 || { tail -40 $O/isolate.log; exit 1; }
grep '^{' $O/isolate.log
