mkdir -p gpurun_out
export GENTUN_NO_AUTOBUILD=1
timeout -k 10 400 python -m pytest tests/ -q -m gpu -x > gpurun_out/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
timeout -k 10 200 python tools/probe_learning.py --noise 1.2 --epochs 6 --lr 1e-3 > gpurun_out/learn_n12.log 2>&1 || exit 1
timeout -k 10 200 python tools/probe_learning.py --noise 0.6 --epochs 6 --lr 1e-3 > gpurun_out/learn_n06.log 2>&1 || exit 1
timeout -k 10 200 python tools/probe_learning.py --noise 1.2 --epochs 6 --lr 1e-3 --genes S_1=000,S_2=0000000000 > gpurun_out/learn_n12_zero.log 2>&1 || exit 1
timeout -k 10 200 python tools/probe_learning.py --noise 1.2 --epochs 6 --lr 1e-3 --backend torch --samples 3000 > gpurun_out/learn_n12_torch.log 2>&1 || exit 1
tools/gpu_prof.sh hip -- python3 tools/probe_steps.py hip 101-0101110011 1 4000 > gpurun_out/prof_hip.log 2>&1 || exit 1
