#!/usr/bin/env bash
# fp32 LDS-GEMM check: dense GPU tests (both fp32 MFMA forms), then per-kernel
# medians of the dense microbench (fp32 / bf16 layer-wise, fused fp32, torch
# eager) under a kernel trace, 16x16x4 vs 32x32x2 fp32 MFMA (SCA_GEMM_F32_M32).
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/gemm_fp32
mkdir -p $OUT
for w in 0 1; do
  SCA_GEMM_F32_M32=$w timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_mlp.py -p no:cacheprovider > $OUT/pytest_w$w.log 2>&1 || exit $?
  tail -1 $OUT/pytest_w$w.log
done
for w in 0 1; do
  SCA_GEMM_F32_M32=$w timeout -k 10 240 rocprofv3 --kernel-trace -d $OUT/trace_w$w -o run --output-format csv -- python3 tools/kernel_microbench.py --only dense_prec,mlp_torch --iters 20 > $OUT/microbench_w$w.log 2>&1 || exit $?
  python3 tools/kernel_medians.py $OUT/trace_w$w > $OUT/medians_w$w.txt 2>&1 || exit $?
  grep "float\|mlp_kernel\|Cijk\|softmax\|relu\|clamp" $OUT/medians_w$w.txt
done
