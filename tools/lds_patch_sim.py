"""LDS bank-conflict model of the shape-specialised conv's patch layout (csrc/hip/conv_fast_impl.h, FastCfg):
LDS cycles of every ds_read_b128 lane group of the MFMA B-operand reads (all k-steps, pixel groups, waves of a
tile) and every ds_write_b128 8-lane group of the staging, for the pixel-major layout (pixel stride NCBP
chunks) and the PAIR layout (chunk pairs side by side, pixel stride 2, pair-plane stride PP2).
Lane groups / banking: /opt/skills/guides/MI355X_MICROARCH.md (LDS table).

usage: python tools/lds_patch_sim.py KH KW NCBI W TH [parts]   (parts: the stage-2 part-major order)
"""
import sys

KH, KW, NCBI, W, TH = (int(v) for v in (sys.argv[1:6] if len(sys.argv) > 5 else (3, 3, 7, 16, 8)))
PARTS = len(sys.argv) > 6 and sys.argv[6] == "parts" or len(sys.argv) <= 5
PH, PW = TH + KH - 1, W + KW - 1
NPIX = PH * PW
NCH = KH * KW * NCBI
NKS = (NCH + 3) // 4
NCBP = NCBI + (0 if NCBI & 1 else 1)


def ent(e):
    if PARTS:
        if e < KH * KW * 4:
            return e >> 2, e & 3
        e1 = e - KH * KW * 4
        kk = e1 // 3
        return kk, 4 + e1 - kk * 3
    return e // NCBI, e % NCBI


RGROUPS = [list(range(0, 4)) + list(range(12, 16)) + list(range(20, 28)),
           list(range(4, 12)) + list(range(16, 20)) + list(range(28, 32))]
RGROUPS += [[l + 32 for l in g] for g in RGROUPS]


def read_cycles(slot):
    tot = 0
    for s in range(NKS):
        for pg in range(TH * W // 16):
            p0 = pg * 16
            for g in RGROUPS:
                cnt = {}
                for l in g:
                    kq, l16 = l >> 4, l & 15
                    e = s * 4 + kq
                    kk, cb = ent(e) if e < NCH else (0, 0)
                    p = p0 + l16
                    pix = (p // W + kk // KW) * PW + p % W + kk % KW
                    c = slot(pix, cb) % 16
                    cnt[c] = cnt.get(c, 0) + 1
                tot += max(cnt.values())
    return tot


def write_cycles(slot):
    NP, tot = NPIX * NCBI, 0
    for j in range((NP + 255) // 256):
        for w0 in range(0, 256, 8):
            cnt = {}
            for t in range(w0, w0 + 8):
                i = t + 256 * j
                if i < NP:
                    c = slot(i // NCBI, i % NCBI) % 8
                    cnt[c] = cnt.get(c, 0) + 1
            if cnt:
                tot += max(cnt.values())
    return tot


ideal = NKS * (TH * W // 16) * 4
print("shape KH={} KW={} NCBI={} W={} TH={} order={}: ideal read cycles {}".format(
    KH, KW, NCBI, W, TH, "parts" if PARTS else "kk-major", ideal))
old = lambda pix, cb: pix * NCBP + cb
print("  pixel-major (stride {}): read {} write {}".format(NCBP, read_cycles(old), write_cycles(old)))
for r in range(8):
    PP2 = 2 * NPIX + (r - 2 * NPIX) % 8
    new = lambda pix, cb, PP2=PP2: (cb >> 1) * PP2 + pix * 2 + (cb & 1)
    print("  pair PP2={} (= {} mod 8): read {} write {}".format(PP2, PP2 % 8, read_cycles(new), write_cycles(new)))
# PAIR with the unpaired last chunk (odd NCBI) at pixel stride 1 in its own plane: the pixel-major LDS size
if NCBI & 1 and NCBI > 1:
    for r in range(8):
        PP2 = 2 * NPIX + (r - 2 * NPIX) % 8
        last = NCBI - 1
        tail = lambda pix, cb, PP2=PP2: (cb >> 1) * PP2 + (pix * 2 + (cb & 1) if cb != last else pix)
        print("  pair+tail1 PP2={} (= {} mod 8): read {} write {}".format(PP2, PP2 % 8, read_cycles(tail),
                                                                           write_cycles(tail)))
