#!/usr/bin/env python3
"""Exhaustive search of the k_brick sweep-buffer strides (PY, PZ, KS, WB in
16-byte packs) under the ds_read_b128 / ds_write_b128 lane-group bank model of
MI355X_MICROARCH.md §LDS, for NP packs per point (2: FP64, 1: FP32).
    python scripts/lds_layout_search.py 1
With --lattice: the brick lattice strides (PLx, PLy; 3D Q2, 4x4 cells per
layer, one or two layers) -- the x sweep's ds_read_b128 from the src lattice
and the ds_add_f64 accumulation (4 x 16 contiguous lanes, (a/4) mod 32, as
ds_write_b64) -- in LDS cycles per wave instruction (conflict free: 4 / 4).
    python scripts/lds_layout_search.py --lattice
With --xdpp: the same two searches for the x-line lane map of the brick.h
xline kernels (lane 16 r + 3 s + x; only the y / z sweeps read the buffers,
each lane reads and adds its own lattice node).
    python scripts/lds_layout_search.py --xdpp"""
import itertools
G128=[list(range(0,4))+list(range(12,16))+list(range(20,28)),
      list(range(4,12))+list(range(16,20))+list(range(28,32)),
      list(range(32,36))+list(range(44,48))+list(range(52,60)),
      list(range(36,44))+list(range(48,52))+list(range(60,64))]
lanes=[]
for l in range(64):
    slot,p=divmod(l,27)
    if slot<2: lanes.append((l,slot,(p%3,(p//3)%3,p//9)))
def rd_cost(addrs):  # addrs: lane->pack index (16B units)
    tot=0
    for g in G128:
        banks={}
        for l in g:
            if l in addrs:
                a=addrs[l]
                for i in range(4):
                    banks.setdefault((a*4+i)%64,set()).add(a)
        if banks: tot+=max(len(v) for v in banks.values())
    return tot
def wr_cost(addrs):
    tot=0
    for g0 in range(0,64,8):
        banks={}
        for l in range(g0,g0+8):
            if l in addrs:
                a=addrs[l]
                for i in range(4): banks.setdefault((a*4+i)%32,set()).add(a)
        if banks: tot+=max(len(v) for v in banks.values())
    return max(13,tot)
def cost(PY,PZ,KS,WB,NP):
    st=[1,PY,PZ]
    tot=0; n_rd=0
    for half in (0,1):            # buffer A or B
        for kp in range(NP):
            # reads along each axis, j = 0..2
            for ax in range(3):
                for j in range(3):
                    ad={}
                    for l,slot,pa in lanes:
                        q=pa[0]+PY*pa[1]+PZ*pa[2]
                        ad[l]=slot*WB+half*NP*KS+kp*KS+q-pa[ax]*st[ax]+j*st[ax]
                    tot+=rd_cost(ad); n_rd+=1
            ad={l:slot*WB+half*NP*KS+kp*KS+pa[0]+PY*pa[1]+PZ*pa[2] for l,slot,pa in lanes}
            tot+=wr_cost(ad)
    return tot, n_rd
import sys


def lattice(PLx, PLy, layers=1):
    G64W = [list(range(i, i + 16)) for i in range(0, 64, 16)]

    def grp(groups, addrs, width, nb):
        tot = 0
        for g in groups:
            banks = {}
            for l in g:
                if l in addrs:
                    for i in range(width):
                        banks.setdefault((addrs[l] + i) % nb, set()).add(addrs[l])
            if banks:
                tot += max(len(v) for v in banks.values())
        return tot
    rd = ad = n = na = 0
    for w in range(4):
        for r in range(2 * layers):
            cells = [r * 8 + w * 2 + sl for sl in range(2)]
            org = [(c % 4) * 2 + PLx * ((c // 4) % 4 * 2 + PLy * (c // 16) * 2) for c in cells]
            for jj in range(3):
                rd += grp(G128, {l: 4 * (org[sl] + jj + PLx * pa[1] + PLx * PLy * pa[2])
                                 for l, sl, pa in lanes}, 4, 64)
                n += 1
            ad += grp(G64W, {l: 2 * (org[sl] + pa[0] + PLx * pa[1] + PLx * PLy * pa[2])
                             for l, sl, pa in lanes}, 2, 32)
            na += 1
    return rd / n, ad / na


def xline_lanes():
    xl = []
    for l in range(64):
        row, wl = divmod(l, 16)
        if wl == 15:
            continue
        s, x = divmod(wl, 3)
        G = 5 * row + s
        if G >= 18:
            continue
        slot, line = divmod(G, 9)
        xl.append((l, slot, (x, line % 3, line // 3)))
    return xl


def cost_axes(PY, PZ, KS, WB, NP, lns, axes):
    st = [1, PY, PZ]
    tot = 0
    for half in (0, 1):
        for kp in range(NP):
            for ax in axes:
                for j in range(3):
                    ad = {}
                    for l, slot, pa in lns:
                        q = pa[0] + PY * pa[1] + PZ * pa[2]
                        ad[l] = slot * WB + half * NP * KS + kp * KS + q - pa[ax] * st[ax] + j * st[ax]
                    tot += rd_cost(ad)
            ad = {l: slot * WB + half * NP * KS + kp * KS + pa[0] + PY * pa[1] + PZ * pa[2]
                  for l, slot, pa in lns}
            tot += wr_cost(ad) * 3  # about three reads per write
    return tot


def lattice_own(PLx, PLy, lns):
    G64W = [list(range(i, i + 16)) for i in range(0, 64, 16)]

    def grp(groups, addrs, width, nb):
        tot = 0
        for g in groups:
            banks = {}
            for l in g:
                if l in addrs:
                    for i in range(width):
                        banks.setdefault((addrs[l] + i) % nb, set()).add(addrs[l])
            if banks:
                tot += max(len(v) for v in banks.values())
        return tot
    rd = ad = n = 0
    for w in range(4):
        for r in range(2):
            cells = [r * 8 + w * 2 + sl for sl in range(2)]
            org = [(c % 4) * 2 + PLx * ((c // 4) % 4 * 2) for c in cells]
            a = {l: (org[sl] + pa[0] + PLx * pa[1] + PLx * PLy * pa[2]) for l, sl, pa in lns}
            rd += grp(G128, {l: 4 * v for l, v in a.items()}, 4, 64)
            ad += grp(G64W, {l: 2 * v for l, v in a.items()}, 2, 32)
            n += 1
    return rd / n, ad / n


if sys.argv[1] == "--xdpp":
    xl = xline_lanes()
    for NP in (1, 2):
        best = []
        for PY in range(3, 9):
            for PZ in range(3 * PY, 3 * PY + 24):
                for KS in range(2 + 2 * PY + 2 * PZ + 1, 2 + 2 * PY + 2 * PZ + 12):
                    for WB in range(2 * NP * KS, 2 * NP * KS + 12):
                        best.append((cost_axes(PY, PZ, KS, WB, NP, xl, (1, 2)), PY, PZ, KS, WB))
        best.sort()
        print(f"NP {NP}: (cost, PY, PZ, KS, WB) {best[:4]}")
    res = []
    for PLx in range(9, 17):
        for PLy in range(9, 17):
            rd, ad = lattice_own(PLx, PLy, xl)
            res.append((rd + 4 * ad, rd, ad, PLx, PLy, PLx * PLy * 3))
    res.sort()
    print("lattice (read + 4 adds, read, add, PLx, PLy, positions):", res[:6])
    sys.exit(0)
if sys.argv[1] == "--lattice":
    for layers in (1, 2):
        for PLx, PLy in ((9, 9), (9, 10), (9, 11), (11, 12)):
            print(f"{layers} layer(s) PLx {PLx} PLy {PLy}: positions {PLx * PLy * (2 * layers + 1)}"
                  f", x-sweep read / accumulate cycles {lattice(PLx, PLy, layers)}")
    sys.exit(0)
NP=int(sys.argv[1])
print('current', cost(3,9,27,54,1) if NP==1 else cost(4,13,37,151,2), 'unpadded', cost(3,9,27,2*NP*27,NP))
best=[]
for PY in range(3,9):
    for PZ in range(3*PY, 3*PY+24):
        for KS in range(2+2*PY+2*PZ+1, 2+2*PY+2*PZ+20):
            for WB in range(2*NP*KS, 2*NP*KS+20):
                c,_=cost(PY,PZ,KS,WB,NP)
                best.append((c,PY,PZ,KS,WB))
best.sort(); print(best[:8])
