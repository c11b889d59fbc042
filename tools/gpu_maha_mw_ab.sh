#!/usr/bin/env bash
# Mahalanobis: multi-wave tridiagonalisation A/B (SCA_MAHA_MW_MIN_P) after the
# GPU parity tests; tools/maha_bench.py per setting, interleaved.
set -o pipefail
OUT=gpurun_out/maha_mw
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_outliers.py tests/test_checkpoint.py -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -20 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
for rep in 1 2; do
  for mw in ${VALUES:-99 32 16}; do
    SCA_MAHA_MW_MIN_P=$mw timeout -k 10 240 python tools/maha_bench.py --p ${PS:-20 32 64} --requests 1500 --threads 16 --out $OUT/mw${mw}_r$rep.json > $OUT/mw${mw}_r$rep.log 2>&1 || exit 1
    echo "mw=$mw rep=$rep"; grep '^{' $OUT/mw${mw}_r$rep.log | cut -c1-400
  done
done
