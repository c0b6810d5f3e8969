export GENTUN_NO_AUTOBUILD=1
GENTUN_TILES=64,128 timeout -k 10 200 python tools/bench_kernels.py 50 > gpurun_out/bk_tiles.log 2>&1 || exit 1
