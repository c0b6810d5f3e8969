set -o pipefail
RESET=kernels P=2 SAMPLES=10000 TAG=_k2c DUMP=2 bash tools/gpu.sh timeline > /dev/null && head -4 gpurun_out/timeline/summary_k2c.txt
P=5 TAG=_p5c DUMP=1 bash tools/gpu.sh timeline > /dev/null && head -4 gpurun_out/timeline/summary_p5c.txt
