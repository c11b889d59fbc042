# Round-6 close-out #2: full GPU suite, smoke(), headline bench, folded 2- and 4-rank rehearsals.
set -o pipefail
O=gpurun_out/${R06_OUT:-r06o}
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest_gpu.log 2>&1 || { tail -60 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 300 python bench.py > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 1; }
grep '^{' $O/bench.log | tail -1 | cut -c1-700
SCA_BENCH_FOLD_GPUS=1 timeout -k 10 480 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29531 bench.py --gpus 2 --steps 5 --warmup 2 > $O/fold2.log 2>&1 || { tail -30 $O/fold2.log; exit 1; }
grep '^{"metric' $O/fold2.log | tail -1 | cut -c1-400
SCA_BENCH_FOLD_GPUS=1 timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29541 bench.py --gpus 4 --steps 5 --warmup 2 > $O/fold4.log 2>&1 || { tail -30 $O/fold4.log; exit 1; }
grep '^{"metric' $O/fold4.log | tail -1 | cut -c1-400
