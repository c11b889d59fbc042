set -o pipefail
for p in 9 20 32 64; do timeout -k 5 60 ./tools/micro/jacobi_probe $p || exit 1; done
