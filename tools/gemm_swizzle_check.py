"""Offline bank-conflict check of the LDS swizzles used by csrc/kernels/gemm.hip
(ds_read_b128 lane groups and ds_read_b64_tr_b16 32-lane halves; prints the
worst n-way conflict per image, 1 = conflict free)."""
G128 = [list(range(0,4))+list(range(12,16))+list(range(20,28)),
        list(range(4,12))+list(range(16,20))+list(range(28,32)),
        list(range(32,36))+list(range(44,48))+list(range(52,60)),
        list(range(36,44))+list(range(48,52))+list(range(60,64))]
def kmaj(f):
    worst=1
    for r0 in range(0,256,16):
      for ks in range(2):
        addr={}
        for l in range(64):
            row=r0+(l&15); c=ks*4+(l>>4)
            pos=c^f(row)
            addr[l]=row*128+pos*16
        for g in G128:
            slots={}
            for l in g:
                s=(addr[l]//16)%16
                slots.setdefault(s,set()).add(addr[l])
            worst=max(worst,max(len(v) for v in slots.values()))
    return worst
print("kmaj none", kmaj(lambda r:0), "swz", kmaj(lambda r:(r>>1)&7))
def mnmaj(BMN, h):
    rowb=BMN*2; nch=BMN//8
    worst=1
    for ks in range(2):
      for half in range(2):
        for m0 in range(0,BMN,16):
          for sub in range(2):
            banks={}
            for l in range(32*half,32*half+32):
                g=l>>4; i=l&15; q=i>>2; p=i&3
                k=ks*32+8*g+4*sub+q
                m=m0+4*p
                ch=m//8; within=(m%8)*2
                pos=ch ^ h(k)
                assert 0<=pos<nch, (pos,nch)
                a=k*rowb+pos*16+within
                for b in (a//4%64, a//4%64+1):
                    banks.setdefault(b%64,set()).add(a)
            worst=max(worst,max(len(v) for v in banks.values()))
    return worst
print("mn256 none",mnmaj(256,lambda k:0),"swz",mnmaj(256,lambda k:2*((k&3)|(((k>>3)&1)<<2))))
print("mn320 none",mnmaj(320,lambda k:0),"swz",mnmaj(320,lambda k:2*(((k>>1)&1)|(((k>>3)&1)<<1))))



# K-major image with 64-B rows (BK = 32, gemm_pp kernel): chunk pos = c ^ f(row), f from a table
def kmaj64(f):
    worst = 1
    for r0 in range(0, 256, 16):
        addr = {}
        for l in range(64):
            row = r0 + (l & 15); c = l >> 4
            addr[l] = row * 64 + (c ^ f(row)) * 16
        for g in G128:
            slots = {}
            for l in g:
                slots.setdefault((addr[l] // 16) % 16, set()).add(addr[l])
            worst = max(worst, max(len(v) for v in slots.values()))
    return worst


import itertools
best = None
for tab in itertools.product(range(4), repeat=4):
    for sh in (2, 3):
        w = kmaj64(lambda r, tab=tab, sh=sh: tab[(r >> sh) & 3])
        if best is None or w < best[0]:
            best = (w, tab, sh)
print("kmaj64 none", kmaj64(lambda r: 0), "best", best)
