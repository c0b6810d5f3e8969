set -o pipefail
export GENTUN_NO_AUTOBUILD=1
mkdir -p gpurun_out/r5/mnist
TAG=mnist TESTS="tests/test_hip_conv_variants.py tests/test_padded_geometry.py tests/test_hip_fp32.py tests/test_hip_kernels.py tests/test_hip_train.py" LIBS= bash tools/r5_exp.sh || exit 1
for spec in "32,32,3 1" "28,28,1 1" "28,28,1 0"; do set -- $spec
  SHAPE=$1 PAD=$2 DTYPE=fp32 RESET=all timeout -k 10 300 python tools/probe_pop.py 5 5 1 1 10000 > gpurun_out/r5/mnist/pop.log 2>&1 || { tail -5 gpurun_out/r5/mnist/pop.log; exit 1; }
  echo "SHAPE=$1 PAD=$2 $(grep '^{' gpurun_out/r5/mnist/pop.log | cut -c1-260)" | tee -a gpurun_out/r5/mnist/pop_summary.txt
done
