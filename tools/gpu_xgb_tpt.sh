set -o pipefail
mkdir -p gpurun_out
for t in 1 2 4; do
  SCA_TREE_WHOLE_TPT=$t timeout -k 10 300 python bench.py --model xgb1000 > gpurun_out/xgb_tpt$t.log 2>&1 || exit 1
  python3 -c "
import json
l=[json.loads(x) for x in open('gpurun_out/xgb_tpt$t.log') if x.startswith('{')][-1]
print('tpt=$t', l['value'], l['p50_ms'], l['p99_ms'], l['config']['mean_rows_per_gpu_batch'], l['config']['gpu_busy_frac_per_slot'])"
done
