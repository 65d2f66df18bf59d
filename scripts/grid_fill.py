"""Grid fill of the update-block conv launches: workgroups vs 256 CUs x resident workgroups.

    python scripts/grid_fill.py [pytorch_raft_amd/tune_db/conv_gfx950.txt]

For every key of the persisted conv tile table (pytorch_raft_amd/tune_db/) at the chairs
geometry (P = 34,224 pixels: batch 12 at 46 x 62) it prints the chosen tile, the workgroup
count, the workgroups a CU holds at once (LDS: 160 KB per CU; registers: the 4-wave
workgroup's per-lane VGPR + AGPR count from the gfx950 build, hipcc -Rpass-analysis), the
number of dispatch rounds of the chip and the occupancy of the last round (the tail).
"""
import math
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
DB = os.path.join(ROOT, 'pytorch_raft_amd', 'tune_db', 'conv_gfx950.txt')

# kCfgs of conv_igemm.hip: (tm, tn, wvm, bm, bn, stages or 'halo' / 'reg')
CFGS = {
    0: (2, 2, 2, 128, 128, 'reg'), 1: (1, 2, 2, 64, 128, 'reg'), 2: (2, 1, 2, 128, 64, 'reg'),
    3: (1, 1, 2, 64, 64, 'reg'), 4: (1, 1, 4, 128, 32, 'reg'), 5: (4, 2, 2, 256, 128, 'reg'),
    6: (5, 2, 1, 160, 256, 'reg'), 7: (5, 1, 1, 160, 128, 'reg'), 8: (4, 2, 1, 128, 256, 'reg'),
    9: (3, 2, 1, 96, 256, 'reg'),
    10: (2, 2, 2, 128, 128, 2), 11: (1, 2, 2, 64, 128, 2), 12: (2, 1, 2, 128, 64, 2),
    13: (4, 2, 2, 256, 128, 2), 14: (4, 2, 1, 128, 256, 2), 15: (3, 2, 1, 96, 256, 2),
    16: (5, 1, 1, 160, 128, 2), 17: (1, 1, 2, 64, 64, 2), 18: (2, 2, 2, 128, 128, 4),
    19: (1, 2, 2, 64, 128, 3), 20: (5, 1, 1, 160, 128, 4), 21: (2, 1, 2, 128, 64, 4),
    22: (1, 1, 2, 64, 64, 4), 23: (4, 2, 1, 128, 256, 3), 24: (3, 1, 1, 96, 128, 4),
    25: (3, 1, 1, 96, 128, 2), 26: (5, 2, 1, 160, 256, 2), 27: (5, 2, 1, 160, 256, 3),
    28: (9, 1, 1, 288, 128, 2), 29: (3, 3, 2, 192, 192, 2),
    30: (5, 1, 1, 160, 128, 'halo'), 31: (5, 2, 1, 160, 256, 'halo'),
    32: (4, 2, 1, 128, 256, 'halo'), 33: (2, 2, 2, 128, 128, 'halo'),
}
ECLASS = {0: 'bf16 out', 1: 'fp32 / dgrad', 2: 'GRU gates', 3: 'dgrad + gate'}
CUS = 256
LDS_CU = 160 * 1024


def lds_bytes(c):
    tm, tn, wvm, bm, bn, st = c
    if st == 'reg':
        return 2 * (bm + bn) * 128
    if st == 'halo':
        return 2 * (bm + 8) * 144   # A image of a 64-channel chunk (+ halo), B straight to VGPRs
    return st * (bm + bn) * 128


# VGPR + AGPR per lane of the LDS-DMA kernels, gfx950 build (hipcc -Rpass-analysis=
# kernel-resource-usage on conv_glds.hip, bf16 epilogues): (tm, tn) -> registers
MEASURED = {(5, 1): 208, (3, 1): 92, (5, 2): 352, (9, 1): 346}


def regs(c):
    """Registers per lane: measured where known, else the accumulators (16 per 32x32 tile) + one
    K step's fragments + addressing, the floor the compiler needs."""
    tm, tn = c[0], c[1]
    return MEASURED.get((tm, tn), 16 * tm * tn + 16 * (tm + tn) + 40)


def main():
    path = sys.argv[1] if len(sys.argv) > 1 else DB
    rows = []
    for line in open(path):
        line = line.split('#', 1)[0].strip()
        if not line:
            continue
        r = [int(x) for x in line.split()]
        if r[0] != 34224:
            continue
        rows.append(r)
    print('%-34s %-15s %-16s %6s %4s %6s %6s' % ('key (KHxKW cin->cout)', 'epilogue', 'tile (cfg)',
                                                  'WGs', 'occ', 'rounds', 'tail'))
    for r in sorted(rows, key=lambda r: (r[3], r[4], r[5], r[6], r[8])):
        P, H, W, KH, KW, cin, cout, small, ec, cfg, bm, bn, creal = r
        c = CFGS[cfg]
        wgs = math.ceil(P / bm) * math.ceil(cout / bn)
        occ_lds = max(1, LDS_CU // lds_bytes(c))
        occ_reg = max(1, min(8, 512 // ((regs(c) + 7) // 8 * 8)))   # 4-wave WG: 1 wave / SIMD each
        occ = min(occ_lds, occ_reg)
        slots = CUS * occ
        rounds = wgs / slots
        tail = (wgs % slots) / slots if wgs % slots else 1.0
        kind = 'halo' if c[5] == 'halo' else ('reg' if c[5] == 'reg' else 'glds%d' % c[5])
        print('%-34s %-15s %-16s %6d %4d %6.2f %5.0f%%' % (
            '%dx%d %d->%d (real %d)' % (KH, KW, cin, cout, creal), ECLASS.get(ec & 3, ec),
            '%dx%d %s (%d)' % (bm, bn, kind, cfg), wgs, occ, rounds, 100 * tail))


if __name__ == '__main__':
    main()
