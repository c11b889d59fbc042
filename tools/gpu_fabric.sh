#!/usr/bin/env bash
# RCCL fabric rehearsal on a 1-GPU box: 2 ranks sharing GPU 0, then a tree bench.
set -u
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 240 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 \
  --master-port 29533 tools/fabric_probe.py > gpurun_out/fabric1.log 2>&1
echo "fabric world=1 rc=$?"; tail -3 gpurun_out/fabric1.log
timeout -k 10 240 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29534 tools/fabric_probe.py --same-device > gpurun_out/fabric2.log 2>&1
rc=$?
echo "fabric world=2 same-device rc=$rc"; tail -8 gpurun_out/fabric2.log
if [ $rc -eq 124 ] || [ $rc -eq 137 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ]; then exit $rc; fi
timeout -k 10 300 python bench.py --model xgb1000 --step-requests 20000 > gpurun_out/bench_xgb.log 2>&1
echo "bench_xgb rc=$?"; tail -1 gpurun_out/bench_xgb.log | cut -c1-400
