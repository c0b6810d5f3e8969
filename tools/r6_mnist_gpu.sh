# Round 6 final tree: MNIST config RR-GA bench (28x28x1, population 20, 8 timed rounds after 2 warm-up) and the
# MNIST + BatchNorm generality bench (4 timed rounds after 1), each under its own limit.
export GENTUN_NO_AUTOBUILD=1
mkdir -p gpurun_out/r6m
( while sleep 50; do date >> gpurun_out/r6m/heartbeat; done ) & HB=$!
trap 'kill $HB 2>/dev/null' EXIT
timeout -k 10 560 python3 -u bench.py --gpus 1 --input-shape 28,28,1 --population 20 --steps 8 --warmup 2 \
  > gpurun_out/r6m/mnist.json 2> gpurun_out/r6m/mnist.err || { tail -3 gpurun_out/r6m/mnist.err; exit 1; }
cut -c1-200 gpurun_out/r6m/mnist.json
timeout -k 10 420 python3 -u bench.py --gpus 1 --steps 4 --warmup 1 --input-shape 28,28,1 --batch-norm \
  > gpurun_out/r6m/mnist_bn.json 2> gpurun_out/r6m/mnist_bn.err || { tail -3 gpurun_out/r6m/mnist_bn.err; exit 1; }
cut -c1-200 gpurun_out/r6m/mnist_bn.json
