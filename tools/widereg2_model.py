#!/usr/bin/env python3
"""Exact-integer model of the two-waves-per-gate FP64 transforms
(mkfhe_amd/csrc/mkacc_widereg2.hpp): the four register/lane layouts, the LDS
word map (injective, additive in every bit, and conflict-free: the 32 lanes of
every half-wave hit 32 distinct bank pairs in every layout), the per-lane twiddle
indexing of every pass, and the monomial exponent split -- the forward and
inverse transform pair run on (wave, lane, register) arrays and must equal the
oracle's NTT (reference order) -- and the two-buffer LDS schedule with a barrier only in
the cross-wave transposes is checked race-free over a sequence of gate-steps.
Test infrastructure: imports oracle/ only.
usage: python3 tools/widereg2_model.py      (about a minute)"""
import sys, numpy as np
import os
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'oracle'))
N=2048; Q=1125899906826241; PSI=1080667890455
def bit(p,k): return (p>>k)&1
# layouts: position p -> (w, l, r)
def A2(p): return (bit(p,6), p&63, p>>7)
def B2(p): return (bit(p,10), (p&7)|(bit(p,7)<<3)|(bit(p,8)<<4)|(bit(p,9)<<5), (p>>3)&15)
def C2(p): return (bit(p,10), bit(p,5)|(bit(p,6)<<1)|(bit(p,9)<<2)|(bit(p,7)<<3)|(bit(p,4)<<4)|(bit(p,8)<<5), p&15)
def D2(p): return (bit(p,10), (p&15)|(bit(p,8)<<4)|(bit(p,9)<<5), (p>>4)&15)
L={'A':A2,'B':B2,'C':C2,'D':D2}
inv={}
for n,f in L.items():
    m={}
    for p in range(N): m[f(p)]=p
    assert len(m)==N; inv[n]=m
def pad(p): return p + bit(p,5)*1 + bit(p,6)*2 + bit(p,7)*8 + bit(p,8)*16 + bit(p,9)*36 + bit(p,10)*64
assert len({pad(p) for p in range(N)})==N and max(pad(p) for p in range(N))==2174
# bank check, fixed (w, r): each 32-lane half distinct mod 32 (ds_read_b64 / ds_*_b32 lane
# groups) and, for the 8-byte layouts, each 16-lane group distinct mod 16 (ds_write_b64 and
# ds_read2/write2_b64 lane groups, banks (a/4) mod 32: MI355X_MICROARCH.md s LDS)
for n in L:
    for w in range(2):
        for r in range(16):
            for h in range(2):
                banks=[pad(inv[n][(w,l,r)])%32 for l in range(32*h,32*h+32)]
                assert len(set(banks))==32, (n,w,r,h)
            for q in range(4):
                banks=[pad(inv[n][(w,l,r)])%16 for l in range(16*q,16*q+16)]
                assert len(set(banks))==16, (n,w,r,q)
# additivity: pad(p) for layout = base(w,l) + off(r)
for n in L:
    for w in range(2):
        for l in range(64):
            b=pad(inv[n][(w,l,0)])
            for r in range(16):
                assert pad(inv[n][(w,l,r)]) - b == pad(inv[n][(0,0,r)]) - pad(inv[n][(0,0,0)]), (n,w,l,r)
print("layouts ok")
import pyoracle as O
O.build()
# reference tables
def brv(x,b): return int(format(x,'0%db'%b)[::-1],2)
tw=[pow(PSI, brv(k,11), Q) for k in range(N)]          # rootOfUnityTable: tw[k] = psi^brv11(k)
psii=pow(PSI, -1, Q); Ninv=pow(N,-1,Q)
pwi=[pow(psii, e, Q) for e in range(2*N)]
def regs_from(lay, vec):   # vec[p] -> X[w][l][r]
    X=[[[0]*16 for _ in range(64)] for _ in range(2)]
    f=L[lay]
    for p in range(N):
        w,l,r=f(p); X[w][l][r]=vec[p]
    return X
def vec_from(lay, X):
    v=[0]*N
    for (w,l,r),p in inv[lay].items(): v[p]=X[w][l][r]
    return v
def transpose(X, src, dst):
    return regs_from(dst, vec_from(src, X))
def pos(lay,w,l,r): return inv[lay][(w,l,r)]
# per-lane tables (value k for wave w lane l)
def FB(w,l,k):   # fwd B2 stage s=4..6, k = (2^(s-4)-1) + (r >> (8-s)); need r bits -> reconstruct p with those reg bits
    s = 4 if k==0 else (5 if k<3 else 6); m = k - ((1<<(s-4))-1)
    r = m << (8-s)                     # register bits above the operated one
    p = pos('B',w,l,r)
    return tw[(1<<s) + (p >> (11-s))]
def FC(w,l,k,CL='C'):
    s = 7 + (k+1).bit_length()-1; m = k - ((1<<(s-7))-1)
    r = m << (11-s)
    p = pos(CL,w,l,r)
    return tw[(1<<s) + (p >> (11-s))]
def ID(w,l,k):
    b = 4 + (k+1).bit_length()-1; H = 1<<(b-4); m = k-(H-1)
    p = pos('D',w,l,m)                 # register bits below the operated one = m
    t = p & ((1<<b)-1)
    return pwi[(t << (11-b)) % (2*N)]
def IA(w,l,k):
    b = 8 if k<2 else (9 if k<6 else 10); H = 1<<(b-7); m = k-(H-2)
    p = pos('A',w,l,m)
    t = p & ((1<<b)-1)
    return pwi[(t << (11-b)) % (2*N)]
def TW(w,l,k): return pwi[pos('A',w,l,k)] * Ninv % Q
def bf(a,b,wt): T=b*wt%Q; return (a+T)%Q, (a-T)%Q
def fwd(vec, CL='C'):
    X=regs_from('A',vec)
    for w in range(2):
        for l in range(64):
            x=X[w][l]
            for s in range(4):
                H=8>>s
                for r in range(16):
                    if r&H: continue
                    x[r],x[r+H]=bf(x[r],x[r+H],tw[(1<<s)+(r>>(4-s))])
    X=transpose(X,'A','B')
    for w in range(2):
        for l in range(64):
            x=X[w][l]
            for s in range(4,7):
                H=8>>(s-4)
                for r in range(16):
                    if r&H: continue
                    k=((1<<(s-4))-1)+(r>>(8-s))
                    x[r],x[r+H]=bf(x[r],x[r+H],FB(w,l,k))
    X=transpose(X,'B',CL)
    for w in range(2):
        for l in range(64):
            x=X[w][l]
            for s in range(7,11):
                H=8>>(s-7)
                for r in range(16):
                    if r&H: continue
                    k=((1<<(s-7))-1)+(r>>(11-s))
                    x[r],x[r+H]=bf(x[r],x[r+H],FC(w,l,k,CL))
    return vec_from(CL,X)
def inv_(vec, CL='C'):
    X=regs_from(CL,vec)
    for w in range(2):
        for l in range(64):
            x=X[w][l]
            for b in range(4):
                H=1<<b
                for r in range(16):
                    if r&H: continue
                    t=r&(H-1)
                    x[r],x[r+H]=bf(x[r],x[r+H],pwi[(t<<(11-b))])
    X=transpose(X,CL,'D')
    for w in range(2):
        for l in range(64):
            x=X[w][l]
            for b in range(4,8):
                H=1<<(b-4)
                for r in range(16):
                    if r&H: continue
                    x[r],x[r+H]=bf(x[r],x[r+H],ID(w,l,(H-1)+(r&(H-1))))
    X=transpose(X,'D','A')
    for w in range(2):
        for l in range(64):
            x=X[w][l]
            for b in range(8,11):
                H=1<<(b-7)
                for r in range(16):
                    if r&H: continue
                    x[r],x[r+H]=bf(x[r],x[r+H],IA(w,l,(H-2)+(r&(H-1))))
            for r in range(16): x[r]=x[r]*TW(w,l,r)%Q
    return vec_from('A',X)
a=[int(v) for v in O.fill_uniform(N,Q,5)]
e=fwd(a)
ref=[int(v) for v in O.ntt_forward(np.array(a,dtype=np.uint64),Q,PSI)]
assert e == ref, "forward transform"
print("forward transform ok")
b=inv_(ref)
assert b == a, "inverse transform"
print("inverse transform ok")
# mono: slot p (C2) exponent e*(2*brv11(p)+1) = e*(2*Lw+1) + ((e*brv4(r))<<8)
for p in range(N):
    w,l,r=C2(p)
    Lw = 32*bit(l,0)+16*bit(l,1)+2*bit(l,2)+8*bit(l,3)+64*bit(l,4)+4*bit(l,5)+w
    for e in (1,7,2047,4095):
        assert (e*(2*brv(p,11)+1))%(2*N) == (e*(2*Lw+1) + ((e*brv(r,4))<<8))%(2*N)
print("mono ok")
# ---- buffer schedule of widereg2::step_kernel (mkacc_layout2.hpp Bufs): two ping-pong
# buffers, a barrier only in the cross-wave transposes (LA <-> LB / LD), the local ones
# (LB -> LC, LC -> LD: w = p10 on both sides) in the buffer of the latest cross-wave one.
# Every pair of accesses by different waves to one LDS element, at least one a write,
# must be ordered the way the program means it: the earlier transpose's access (or, in
# one transpose, the write) in an earlier barrier epoch than the later one.
def addr_set(lay, w):
    return {pad(p) for p in range(N) if L[lay](p)[0] == w}
def schedule(ntrans):
    seq = []
    for t in ntrans:   # 'i' inverse (local C->D, cross D->A), 'f' forward (cross A->B, local B->C)
        seq += [('C', 'D', False), ('D', 'A', True)] if t == 'i' else [('A', 'B', True), ('B', 'C', False)]
    cb, ops, epoch = 0, {0: [], 1: []}, 0
    for ti, (src, dst, cross) in enumerate(seq):
        if cross:
            cb ^= 1
        for w in (0, 1):
            ops[w].append((ti, 0, 'W', cb, addr_set(src, w), epoch))
        if cross:
            epoch += 1
        for w in (0, 1):
            ops[w].append((ti, 1, 'R', cb, addr_set(dst, w), epoch))
    return ops
def check_schedule(ntrans):
    ops = schedule(ntrans)
    for a in ops[0]:
        for b in ops[1]:
            if a[3] != b[3] or 'W' not in (a[2], b[2]) or not (a[4] & b[4]):
                continue
            first, second = (a, b) if (a[0], a[1]) < (b[0], b[1]) else (b, a)
            assert first[5] < second[5], ("LDS race", first[:4], second[:4])
check_schedule('i' + 'f' * 4 + 'i' + 'f' * 4 + 'i' + 'f' * 4 + 'i' + 'f' * 4)   # two gates at k = 2, dg = 4
check_schedule('ififf')
print("buffer schedule ok")
