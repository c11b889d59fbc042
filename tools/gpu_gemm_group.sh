#!/usr/bin/env bash
# bf16 glds-family GEMMs: tile-group sweep (SCA_GEMM_GROUP_M = 1 row-major,
# 2, 4, 8) after the GEMM tests; TFLOP/s per path vs torch (hipBLASLt).
set -o pipefail
OUT=gpurun_out/gemm_group
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gemm.py -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -5 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
for g in ${GROUPS_M:-1 2 4 8}; do
  SCA_GEMM_GROUP_M=$g GEMM_SHAPES=${GEMM_SHAPES:-4096x4096x4096,8192x8192x8192} timeout -k 10 200 python tools/kernel_microbench.py --only gemm --iters 20 > $OUT/gm$g.jsonl 2>&1 || exit 1
  python3 - $g $OUT/gm$g.jsonl <<'PY'
import json, sys
g, f = sys.argv[1], sys.argv[2]
for l in open(f):
    if l.startswith("{"):
        d = json.loads(l)
        print("gm=%s M=%d" % (g, d["M"]), " ".join("%s=%s" % (k[:-7], d[k]) for k in d if k.endswith("_tflops")))
PY
done
