#!/usr/bin/env bash
# fp32 GEMM tile A/B: 128 x 64 vs 64 x 64 tiles (SCA_GEMM_F32_T64 = 0 / 1 / 2)
# -- dense GPU tests under each setting, then kernel-trace medians of the
# dense microbench (MLP 784-512-256-10 @ 8192 rows, VAE) per setting.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/gemm_t64
mkdir -p $OUT
for w in 2 1; do
  SCA_GEMM_F32_T64=$w timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_mlp.py tests/test_gemm.py -p no:cacheprovider > $OUT/pytest_t$w.log 2>&1 || exit $?
  tail -1 $OUT/pytest_t$w.log
done
for w in 0 1 2; do
  SCA_GEMM_F32_T64=$w timeout -k 10 240 rocprofv3 --kernel-trace -d $OUT/trace_t$w -o run --output-format csv -- python3 tools/kernel_microbench.py --only dense_prec,mlp_torch --iters 20 > $OUT/microbench_t$w.log 2>&1 || exit $?
  python3 tools/kernel_medians.py $OUT/trace_t$w > $OUT/medians_t$w.txt 2>&1 || exit $?
  echo "== T64=$w"; grep "float\|mlp_kernel\|Cijk" $OUT/medians_t$w.txt | cut -c1-200
done
