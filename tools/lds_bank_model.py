import numpy as np
# LDS bank-conflict model (MI355X_MICROARCH.md §LDS): ds_read_b64: groups 2x32 lanes, bank=(a/4)%64;
# ds_write_b64: groups 4x16 contiguous, bank=(a/4)%32.  extra cycles per group = max distinct addrs on a bank - 1.
def conflicts(addrs, kind):
    # addrs: byte addresses per lane (64), each an 8-B access (2 dwords)
    if kind=='r': groups=[range(0,32),range(32,64)]; nb=64
    else: groups=[range(0,16),range(16,32),range(32,48),range(48,64)]; nb=32
    extra=0
    for g in groups:
        banks={}
        for l in g:
            for d in (0,4):
                a=addrs[l]+d
                banks.setdefault((a//4)%nb,set()).add(a//4)
        extra+=max(len(v) for v in banks.values())-1
    return extra
def pad_default(e): return e + (e>>5)
def own8(t, pad): return [pad(8*t+i) for i in range(8)]
def chunk_group(t, LNG, i): return ((t>>6)<<(6+LNG)) + (i<<6) + (t&63)
def lds_chunk_addrs(t, LG, K, pad, LE=3):
    LGG=LG-K+1; g=1<<LGG; out=[]
    for i in range(1<<(LE-K)):
        q=chunk_group(t, LE-K, i)
        e0=((q>>LGG)<<(LG+1)) + (q&(g-1))
        out.append([pad(e0+j*g) for j in range(1<<K)])
    return out  # list over i of list over j
def flip_addrs(t,S,pad):
    g=1<<(S-1); LP=S-2
    base=(t>>LP)<<(S+1); r=t&((1<<LP)-1)
    return [pad(base+r+j*g) for j in range(4)]+[pad(base+g-1-r+j*g) for j in range(4)]
def head_conflicts(TLOG, pad):
    nt=1<<(TLOG-3); tot={'own':0,'flip':0,'chunk':0}
    waves=range(nt//64)
    for S in range(5,TLOG):
        for w in waves:
            ts=list(range(64*w,64*w+64))
            A=[own8(t,pad) for t in ts]
            for i in range(8):
                ad=[8*A[l][i] for l in range(64)]
                tot['own']+=conflicts(ad,'w')+conflicts(ad,'r')
            F=[flip_addrs(t,S,pad) for t in ts]
            for j in range(8):
                ad=[8*F[l][j] for l in range(64)]
                tot['flip']+=conflicts(ad,'w')+conflicts(ad,'r')
            LG=S-2
            while LG>=5:
                K=3 if LG-4>=3 else LG-4
                C=[lds_chunk_addrs(t,LG,K,pad) for t in ts]
                for i in range(len(C[0])):
                    for j in range(len(C[0][0])):
                        ad=[8*C[l][i][j] for l in range(64)]
                        tot['chunk']+=conflicts(ad,'w')+conflicts(ad,'r')
                LG-=K
    return {k:v/len(waves) for k,v in tot.items()}
if __name__=='__main__':
    print('default pad', head_conflicts(13, pad_default))

def conflicts2(addrs):
    # worst of both models: 16-lane groups mod 32 dwords and 32-lane groups mod 64 dwords
    return conflicts(addrs,'w')+conflicts(addrs,'r')
def all_patterns(TLOG):
    nt=1<<(TLOG-3); pats=[]
    ts=list(range(64))  # wave 0 (patterns repeat per wave up to base offsets)
    for S in range(5,TLOG):
        for i in range(8): pats.append(('own',[8*t+i for t in ts]))
        F=[None]*64
        for j in range(8): pats.append(('flip%d'%S,[ (lambda t: (lambda g,LP: ([((t>>LP)<<(S+1))+(t&((1<<LP)-1))+jj*g for jj in range(4)]+[((t>>LP)<<(S+1))+g-1-(t&((1<<LP)-1))+jj*g for jj in range(4)])[j])(1<<(S-1),S-2))(t) for t in ts]))
        LG=S-2
        while LG>=5:
            K=3 if LG-4>=3 else LG-4
            LGG=LG-K+1; g=1<<LGG
            for i in range(1<<(3-K)):
                for j in range(1<<K):
                    pats.append(('chunk',[ (((chunk_group(t,3-K,i)>>LGG)<<(LG+1)) + (chunk_group(t,3-K,i)&(g-1)) + j*g) for t in ts]))
            LG-=K
    # tail: strided write t + j*NT, chunks lds_chunks<TLOG-4>, own read
    NT=nt
    for j in range(8): pats.append(('tail_str',[t+j*NT for t in ts]))
    LG=TLOG-4
    while LG>=4:
        K=3 if LG-3>=3 else LG-3
        LGG=LG-K+1; g=1<<LGG
        for i in range(1<<(3-K)):
            for j in range(1<<K):
                pats.append(('tchunk',[ (((chunk_group(t,3-K,i)>>LGG)<<(LG+1)) + (chunk_group(t,3-K,i)&(g-1)) + j*g) for t in ts]))
        LG-=K
    return pats
def evaluate(TLOG, phys):
    tot={}
    for name,es in all_patterns(TLOG):
        c=conflicts2([8*phys(e) for e in es])
        k=name.rstrip('0123456789')
        tot[k]=tot.get(k,0)+c
    return tot
