export GENTUN_NO_AUTOBUILD=1
timeout -k 10 400 python -u -m pytest -m gpu -x -q --timeout 120 --timeout-method thread tests/test_hip_kernels.py tests/test_hip_fp32.py tests/test_hip_train.py > gpurun_out/adam_tests.log 2>&1 || { tail -30 gpurun_out/adam_tests.log; exit 1; }
tail -1 gpurun_out/adam_tests.log
P=5 TAG=_adamvec DUMP=0 bash tools/gpu.sh timeline || exit 1
SPACE=deep KERNELS=64,128,256 BN=1 WARM=0 bash tools/gpu.sh prof widevec -- python3 tools/probe_pop.py 5 5 1 1 2000
