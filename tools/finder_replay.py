"""CPU replay of k_inf_find's filters over one configs[4] pool image (round 5):
per 32 KiB chunk, how far the scan runs before the first real dynamic block
header, how many positions survive the header-field and Kraft filters before
it, and what the full-check rounds cost (longest lane per 64-position round).

    python tools/finder_replay.py
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))
import bench
from deflate_tokens import png_idat
from datago_amd import synth
spec = synth.mixed_spec(5, 8, 256, 2048)
CLO=[16,17,18,0,8,7,9,6,10,5,11,4,12,3,13,2,14,1,15]
def header_full(bits, pos):
    g=lambda o,n: int(sum(int(bits[pos+o+k])<<k for k in range(n)))
    nlen=g(3,5)+257; ndist=g(8,5)+1; ncode=g(13,4)+4
    cl=[0]*19
    for i in range(ncode): cl[CLO[i]]=g(17+3*i,3)
    # canonical code for cl
    cnt=[0]*8
    for l in cl: cnt[l]+=1
    cnt[0]=0
    code=0; first=[0]*8; nxt={}
    codes={}
    c=0
    for L in range(1,8):
        c=(c+cnt[L-1])<<1 if L>1 else 0
        first[L]=c
    nextc=first[:]
    for s in range(19):
        l=cl[s]
        if l: codes[(l,nextc[l])]=s; nextc[l]+=1
    p=pos+17+3*ncode; i=0; total=nlen+ndist; prev=0; kl=kd=0; dn=0; eob=0; it=0
    while i<total:
        it+=1
        cc=0; sym=None
        for L in range(1,8):
            cc=(cc<<1)|int(bits[p+L-1])
            if (L,cc) in codes: sym=codes[(L,cc)]; p+=L; break
        if sym is None: return False,it
        v=sym; rep=1
        if sym==16:
            if i==0: return False,it
            v=prev; rep=3+int(bits[p])+2*int(bits[p+1]); p+=2
        elif sym==17: v=0; rep=3+sum(int(bits[p+k])<<k for k in range(3)); p+=3
        elif sym==18: v=0; rep=11+sum(int(bits[p+k])<<k for k in range(7)); p+=7
        if i+rep>total: return False,it
        nl = 0 if i>=nlen else min(rep, nlen-i); nd=rep-nl
        if v:
            w=1<<(15-v); kl+=nl*w; kd+=nd*w; dn+=nd
            if i<=256<i+nl: eob=1
            if kl>32768 or kd>32768: return False,it
        prev=v; i+=rep
    return (eob and kl==32768 and (kd==32768 or dn==0 or (dn==1 and kd==16384))), it
for i in [1]:
    img, mask = bench.png_pair((5*1_000_003+i, spec[i]))
    z = png_idat(img)
    bits = np.unpackbits(np.frombuffer(z, np.uint8), bitorder='little').astype(np.uint32)
    bits = np.concatenate([bits, np.zeros(4096, np.uint32)])
    N = len(z)*8
    def f(off, n):
        v = np.zeros(N, np.uint32)
        for k in range(n): v |= bits[off+k:off+k+N] << k
        return v
    h = f(0, 17)
    s1 = ((h&7)==4) & (((h>>3)&31)<=29) & (((h>>8)&31)<=29)
    idx = np.nonzero(s1)[0]
    ncode = ((h[idx]>>13)&15)+4
    hist = np.zeros((len(idx), 8), np.int64)
    for j in range(19):
        l = np.zeros(len(idx), np.uint32)
        for k in range(3): l |= bits[idx+17+3*j+k] << k
        l = np.where(j < ncode, l, 0)
        for L in range(1,8): hist[:,L] += (l==L)
    left = np.ones(len(idx), np.int64); bad = np.zeros(len(idx), bool)
    for L in range(1,8):
        left = 2*left - hist[:,L]; bad |= left<0
    bad |= left != 0
    s2 = idx[~bad]
    span=32768*8
    nch=(N+span-1)//span
    tot_scan=tot_s2=tot_rounds=tot_maxit=0
    for c in range(1,nch):
        b0=c*span; b1=min(b0+span,N)
        cand=s2[(s2>=b0)&(s2<b1)]
        found=None; rounds=0; maxit_sum=0
        for r0 in range(0,len(cand),64):
            rounds+=1; mx=0
            for p in cand[r0:r0+64]:
                ok,it=header_full(bits,int(p)); mx=max(mx,it)
                if ok and found is None: found=int(p)
            maxit_sum+=mx
            if found is not None: break
        scanned=(found if found is not None else b1)-b0
        tot_scan+=scanned; tot_rounds+=rounds; tot_maxit+=maxit_sum
        if c<6: print(c,'found',None if found is None else found-b0,'scanned',scanned,'s2 before',int(((cand<(found or b1))).sum()),'rounds',rounds,'maxit',maxit_sum)
    print('avg per chunk: scanned',tot_scan/(nch-1),'stage3 rounds',tot_rounds/(nch-1),'sum of max iterations',tot_maxit/(nch-1))
