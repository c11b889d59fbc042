# rocprofv3 kernel stats of the CNN graphs, one network per run, untuned and tuned.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
O=gpurun_out/${R06_OUT:-r06r}
mkdir -p $O
for arch in resnet50 densenet169; do
  for t in 0 1; do
    CNN_ARCH=$arch CNN_TUNE=$t timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/${arch}_t$t -o run -- python3 tools/r06/cnn_prof.py > $O/${arch}_t$t.log 2>&1 || { tail -30 $O/${arch}_t$t.log; exit 1; }
    find $O -name "*_trace.csv" -delete
    echo "$arch tune=$t done"
  done
done
du -sh $O
