"""Join the per-kernel means of the PMC passes of ``tools/gpu.sh profstep`` into one table.

usage: python tools/pmc_table.py DIR   (DIR holds kernel_stats.csv and pmc1.txt .. pmc3.txt)

Columns: mean us per call (kernel stats); MFMA% = SQ_VALU_MFMA_BUSY_CYCLES per CU-cycle
(GRBM_GUI_ACTIVE / 8 XCDs x 256 CUs x 4 SIMDs: a busy pipe on every SIMD = 100 %); LDSbc =
SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE; issue-stall = SQ_WAIT_INST_ANY / SQ_WAVE_CYCLES;
L2 hit = TCC_HIT / (TCC_HIT + TCC_MISS); rd / wr MB = TCC_EA0_RDREQ / WRREQ x 64 B (upper bound:
128-B reads tallied at 64 B).
"""
import csv
import os
import re
import sys

root = sys.argv[1]
ncu = int(os.environ.get("NCU", "256"))


def read_pmc(path):
    out = {}
    if not os.path.exists(path):
        return out
    for ln in open(path):
        name = ln[:48].strip()
        out[name] = {k: float(v) for k, v in re.findall(r"(\w+)=([-+0-9.eE]+)", ln[48:])}
    return out


pm = {}
for i in (1, 2, 3):
    for k, v in read_pmc(os.path.join(root, "pmc{}.txt".format(i))).items():
        pm.setdefault(k, {}).update(v)
us = {}
st = os.path.join(root, "kernel_stats.csv")
if os.path.exists(st):
    for r in csv.DictReader(open(st)):
        us[r["Name"][:48].strip()] = float(r["AverageNs"]) / 1000.0
print("{:48s} {:>8s} {:>6s} {:>6s} {:>6s} {:>6s} {:>8s} {:>8s}".format(
    "kernel (per-call mean)", "us", "MFMA%", "LDSbc", "stall", "L2hit", "rd MB", "wr MB"))
for name in sorted(pm, key=lambda n: -us.get(n, 0.0)):
    c = pm[name]
    g = c.get("GRBM_GUI_ACTIVE", 0.0)
    mf = 100.0 * c.get("SQ_VALU_MFMA_BUSY_CYCLES", 0.0) / (g / 8 * ncu * 4) if g else 0.0   # GRBM summed over 8 XCDs
    lds = c.get("SQ_LDS_BANK_CONFLICT", 0.0) / c["SQ_LDS_IDX_ACTIVE"] if c.get("SQ_LDS_IDX_ACTIVE") else 0.0
    stall = c.get("SQ_WAIT_INST_ANY", 0.0) / c["SQ_WAVE_CYCLES"] if c.get("SQ_WAVE_CYCLES") else 0.0
    h, m = c.get("TCC_HIT_sum", 0.0), c.get("TCC_MISS_sum", 0.0)
    print("{:48s} {:8.1f} {:6.1f} {:6.2f} {:6.2f} {:6.2f} {:8.1f} {:8.1f}".format(
        name, us.get(name, 0.0), mf, lds, stall, h / (h + m) if h + m else 0.0,
        c.get("TCC_EA0_RDREQ_sum", 0.0) * 64 / 1e6, c.get("TCC_EA0_WRREQ_sum", 0.0) * 64 / 1e6))
