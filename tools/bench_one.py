"""Run one kernel of tools/bench_kernels.py shapes repeatedly (for PMC profiles).
usage: python tools/bench_one.py KERNEL SHAPE_INDEX REPS"""
import os, sys
sys.argv = [sys.argv[0]] + sys.argv[1:]
os.environ["GENTUN_BENCH_ONLY"] = sys.argv[1] + ":" + sys.argv[2]
sys.argv = [sys.argv[0], sys.argv[3] if len(sys.argv) > 3 else "20"]
exec(open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "bench_kernels.py")).read())
