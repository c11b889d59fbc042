#!/usr/bin/env bash
# fp32 MLP first-layer A/B: fp64 rows staged by the GEMM (SCA_MLP_DIRECT_IN=1)
# vs convert pass + fp32 GEMM, x tile choice (SCA_GEMM_F32_T64), kernel-trace medians.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/mlp_ab
mkdir -p $OUT
for cfg in "1 1" "0 1" "0 2" "1 2"; do
  set -- $cfg
  tag=d$1_t$2
  SCA_MLP_DIRECT_IN=$1 SCA_GEMM_F32_T64=$2 timeout -k 10 240 rocprofv3 --kernel-trace -d $OUT/trace_$tag -o run --output-format csv -- python3 tools/kernel_microbench.py --only dense_prec --iters 20 > $OUT/microbench_$tag.log 2>&1 || exit $?
  python3 tools/kernel_medians.py $OUT/trace_$tag > $OUT/medians_$tag.txt 2>&1 || exit $?
  echo "== $tag"; grep "float\|mlp_convert" $OUT/medians_$tag.txt | cut -c1-150; grep "layer_fp32" $OUT/microbench_$tag.log | cut -c1-200
done
