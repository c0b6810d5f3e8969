export GENTUN_NO_AUTOBUILD=1
timeout -k 10 300 python3 -u tools/probe_graph.py "1,2,5,10" "1,10,50" "all,kernels" > gpurun_out/probe_graph.log 2>&1 || { tail -5 gpurun_out/probe_graph.log; exit 1; }
cat gpurun_out/probe_graph.log | grep mode
for kw in '{"same_color": true}' '{"same_color": true, "distractors": 3}' '{"same_color": true, "shift": 6}'; do
  timeout -k 10 200 python3 -u tools/probe_spread.py 12 parts "$kw" >> gpurun_out/probe_spread.log 2>&1 || { tail -5 gpurun_out/probe_spread.log; exit 1; }
done
grep summary gpurun_out/probe_spread.log
