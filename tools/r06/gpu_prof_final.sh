# rocprofv3 kernel stats: headline bench (current tree) and the CNN graphs.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
O=gpurun_out/${R06_OUT:-r06q}
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
SCA_BENCH_CLEAN_EXIT=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/head -o run -- python3 bench.py --extras none --steps 5 --warmup 2 > $O/head.log 2>&1 || { tail -30 $O/head.log; exit 1; }
grep '^{' $O/head.log | tail -1 | cut -c1-300
find $O -name "*_trace.csv" -delete
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/cnn -o run -- python3 tools/r06/cnn_prof.py > $O/cnn.log 2>&1 || { tail -30 $O/cnn.log; exit 1; }
tail -2 $O/cnn.log
find $O -name "*_trace.csv" -delete
du -sh $O
find $O -name "*kernel_stats.csv" | head
