export GENTUN_NO_AUTOBUILD=1
timeout -k 10 400 python -m pytest tests/test_hip_kernels.py -q -x > gpurun_out/pytest_k.log 2>&1 || { tail -n 40 gpurun_out/pytest_k.log; exit 1; }
tail -n 2 gpurun_out/pytest_k.log
timeout -k 10 200 python tools/bench_kernels.py 50 > gpurun_out/bk_modes.log 2>&1 || exit 1
GENTUN_CONV_MODES=1 GENTUN_CONV_WGS=256 timeout -k 10 200 python tools/bench_kernels.py 50 > gpurun_out/bk_w256.log 2>&1 || exit 1
GENTUN_CONV_MODES=1 GENTUN_CONV_WGS=1024 timeout -k 10 200 python tools/bench_kernels.py 50 > gpurun_out/bk_w1024.log 2>&1 || exit 1
