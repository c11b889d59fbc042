#!/usr/bin/env bash
# Whole-batch MLP 784-512-256-10 @ 8192 rows: our fused fp32 / layer-wise fp32 / bf16
# kernels vs torch eager fp32 (hipBLASLt) with fp32 and with fp64 in/out, kernel trace.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/mlp_vs_torch
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_mlp.py -p no:cacheprovider > $OUT/pytest.log 2>&1 || exit $?
tail -1 $OUT/pytest.log
timeout -k 10 240 rocprofv3 --kernel-trace -d $OUT/trace -o run --output-format csv -- python3 tools/kernel_microbench.py --only mlp_torch,mlp_torch_fp64io,dense_prec --iters 20 > $OUT/microbench.log 2>&1 || exit $?
python3 tools/kernel_medians.py $OUT/trace > $OUT/medians.txt 2>&1 || exit $?
grep "float\|mlp_\|Cijk\|SK3" $OUT/medians.txt | cut -c60-
timeout -k 10 240 python3 tools/kernel_microbench.py --only mlp_torch,mlp_torch_fp64io,dense_prec --iters 50 > $OUT/microbench_notrace.log 2>&1 || exit $?
grep '"case"' $OUT/microbench_notrace.log
