"""Derived per-kernel metrics from a tools/gpu_prof_head.sh directory
(pmc1.txt / pmc2.txt / pmc3.txt summaries of rocprofv3 --pmc passes).

Normalisation (MI355X_MICROARCH.md §rocprofv3): GRBM_GUI_ACTIVE is summed over
the 8 XCDs; SQ_VALU_MFMA_BUSY_CYCLES is summed over SIMDs (16 cycles per
v_mfma_f32_16x16x32_bf16), so MFMA util = busy / (GRBM/8 * 256 CUs * 4 SIMDs);
gfx950 FETCH requests are tallied at 64 B for 128-B streaming reads, so the
read side is doubled (upper bound).

usage: python tools/pmc_derive.py gpurun_out/prof_head > profiles/...txt
"""
import os
import re
import sys

CLOCK_GHZ = 2.4
root = sys.argv[1]
K = {}
for i in (1, 2, 3):
    path = os.path.join(root, "pmc{}.txt".format(i))
    if not os.path.exists(path):
        continue
    for line in open(path):
        name = line[:48].strip()
        for k, v in re.findall(r"(\w+)=([0-9.e+-]+)", line[48:]):
            K.setdefault(name, {})[k] = float(v)

rows = []
for name, c in K.items():
    g = c.get("GRBM_GUI_ACTIVE", 0) / 8.0
    if g <= 0:
        continue
    us = g / (CLOCK_GHZ * 1e3)
    mfma = c.get("SQ_VALU_MFMA_BUSY_CYCLES", 0) / (g * 256 * 4)
    lds = c.get("SQ_LDS_BANK_CONFLICT", 0) / max(1.0, c.get("SQ_LDS_IDX_ACTIVE", 0))
    rd = 2 * c.get("TCC_EA0_RDREQ_sum", 0) * 64
    wr = c.get("TCC_EA0_WRREQ_sum", 0) * 64
    hbm = (rd + wr) / (us * 1e-6) / 1e12 if us > 0 else 0
    hit = c.get("TCC_HIT_sum", 0) / max(1.0, c.get("TCC_HIT_sum", 0) + c.get("TCC_MISS_sum", 0))
    wait = c.get("SQ_WAIT_INST_ANY", 0) / max(1.0, c.get("SQ_WAVE_CYCLES", 0))
    # v_mfma_f32_16x16x32_bf16: 16 busy cycles, 16384 FLOP -> 1024 FLOP per busy cycle
    tfs = 1024.0 * c.get("SQ_VALU_MFMA_BUSY_CYCLES", 0) / (us * 1e-6) / 1e12 if us > 0 else 0
    rows.append((us, name, mfma, tfs, lds, rd / 1e6, wr / 1e6, hbm, hit, wait))

print("# MFMA TF/s = bf16 matrix-core FLOP rate (1024 FLOP per busy cycle of 16x16x32); an fp32 (split)")
print("# product costs 6 of them, so the fp32-equivalent rate of a split kernel is TF/s / 6. HBM TB/s from")
print("# the L2 fabric requests (read side doubled: gfx950 tallies 128-B reads at 64 B -> an upper bound).")
print("{:48s} {:>8s} {:>6s} {:>8s} {:>6s} {:>8s} {:>8s} {:>7s} {:>6s} {:>6s}".format(
    "kernel (per-call mean)", "us", "MFMA%", "MFMA TF/s", "LDSbc", "rd MB", "wr MB", "TB/s", "L2hit", "wait"))
for us, name, mfma, tfs, lds, rd, wr, hbm, hit, wait in sorted(rows, reverse=True):
    print("{:48s} {:8.1f} {:6.1f} {:8.1f} {:6.2f} {:8.1f} {:8.1f} {:7.2f} {:6.2f} {:6.2f}".format(
        name, us, 100 * mfma, tfs, lds, rd, wr, hbm, hit, wait))
