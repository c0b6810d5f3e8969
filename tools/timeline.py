"""Timeline analysis of a rocprofv3 kernel trace of population train steps:
per step (step_begin_kernel to the next), wall time vs busy time of the
main-stream chain and of all kernels (union of intervals), and per-kernel
share of the wall time. usage: python tools/timeline.py run_kernel_trace.csv"""
import csv
import sys
from collections import defaultdict

rows = list(csv.DictReader(open(sys.argv[1])))
ks = []
for r in rows:
    name = r.get("Kernel_Name", "?")
    ks.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), name, r.get("Queue_Id", r.get("Stream_Id", "?"))))
ks.sort()
starts = [i for i, k in enumerate(ks) if k[2].startswith("step_begin")]
steps = []
for a, b in zip(starts[5:], starts[6:]):           # skip the first steps (graph warm-up)
    seg = ks[a:b]
    t0, t1 = seg[0][0], ks[b][0]
    # union of busy intervals
    busy, cur_s, cur_e = 0, None, None
    for s, e, _, _ in seg:
        if cur_e is None or s > cur_e:
            if cur_e is not None:
                busy += cur_e - cur_s
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    busy += cur_e - cur_s
    per = defaultdict(int)
    cnt = defaultdict(int)
    for s, e, n, _ in seg:
        per[n.split("(")[0][:60]] += e - s
        cnt[n.split("(")[0][:60]] += 1
    steps.append((t1 - t0, busy, sum(e - s for s, e, _, _ in seg), per, cnt, len(seg)))
if not steps:
    print("no steps found")
    sys.exit(0)
n = len(steps)
wall = sum(s[0] for s in steps) / n
busy = sum(s[1] for s in steps) / n
ksum = sum(s[2] for s in steps) / n
print("steps analysed: {}  wall/step {:.1f} us  busy (union) {:.1f} us ({:.0f}%)  sum of kernel times {:.1f} us "
      "(overlap factor {:.2f})".format(n, wall / 1e3, busy / 1e3, 100 * busy / wall, ksum / 1e3, ksum / busy))
print("launches per step: {:.1f}; gap (wall - busy) per launch: {:.2f} us".format(
    sum(s[5] for s in steps) / n, (wall - busy) / 1e3 / max(1.0, sum(s[5] for s in steps) / n)))
tot, tcnt = defaultdict(int), defaultdict(int)
for s in steps:
    for k, v in s[3].items():
        tot[k] += v
    for k, v in s[4].items():
        tcnt[k] += v
for k, v in sorted(tot.items(), key=lambda kv: -kv[1]):
    print("{:62s} {:8.1f} us/step {:5.1f}% of wall  {:5.1f} calls/step {:7.1f} us/call".format(
        k, v / n / 1e3, 100 * v / n / wall, tcnt[k] / n, v / max(1, tcnt[k]) / 1e3))

# one steady-state step in detail: TIMELINE_DUMP=k prints the k-th analysed step's launches
import os  # noqa: E402
if os.environ.get("TIMELINE_DUMP"):
    k = int(os.environ["TIMELINE_DUMP"])
    a, b = starts[5 + k], starts[6 + k]
    t0 = ks[a][0]
    print("\n# step {} in detail: start / end us relative to step_begin, queue, kernel".format(k))
    for s, e, name, q in ks[a:b]:
        print("{:8.1f} {:8.1f} {:7.1f}  q{:<3s} {}".format((s - t0) / 1e3, (e - t0) / 1e3, (e - s) / 1e3, str(q),
                                                        name.split("(")[0][:70]))
