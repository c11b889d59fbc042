export TMPDIR=/tmp
mkdir -p gpurun_out
for cfg in "0 0" "1 0"; do
  set -- $cfg
  SCA_GEMM_REMAP=$1 SCA_GEMM_F64A=$2 timeout -k 10 200 rocprofv3 --kernel-trace -d gpurun_out/ab_$1_$2 -o run --output-format csv -- python3 tools/kernel_microbench.py --only dense_prec --iters 20 > gpurun_out/ab_$1_$2.log 2>&1 || exit 1
done
