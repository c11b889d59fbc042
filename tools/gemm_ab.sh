#!/usr/bin/env bash
# LDS GEMM kernel medians under a rocprofv3 kernel trace (XCD remap on / off);
# medians per kernel and grid: python tools/trace_medians.py
export TMPDIR=/tmp
mkdir -p gpurun_out
for remap in 1 0; do
  SCA_GEMM_REMAP=$remap timeout -k 10 200 rocprofv3 --kernel-trace -d gpurun_out/ab_remap$remap -o run --output-format csv -- python3 tools/kernel_microbench.py --only dense_prec --iters 20 > gpurun_out/ab_remap$remap.log 2>&1 || exit 1
done
