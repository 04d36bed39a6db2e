set -eo pipefail
out=gpurun_out/ub; mkdir -p $out
timeout -k 10 120 ./tools/ubench/stores2 > $out/stores2.txt 2>&1
