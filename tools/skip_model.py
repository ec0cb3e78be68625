"""Model check of lcur_skip_ids (hocuspocus_amd/csrc/ygm_merge_big.hpp), tooling: the mask-based skip of an Item's
origin ids against sequential lib0 varuint reads (LCur::vu semantics: position, non-minimal flag, failure past the
update or 2^53) on random byte strings.  python tools/skip_model.py"""
import random
M=2**64-1
def top(h): return ((((h>>7)&0x0101010101010101)*0x0102040810204080)&M)>>56
def zb(x):
    t=((x&0x7F7F7F7F7F7F7F7F)+0x7F7F7F7F7F7F7F7F)&M
    return (~(t|x|0x7F7F7F7F7F7F7F7F))&M
def ctz(x):
    return (x&-x).bit_length()-1
def fast(b,pos,end,npair):
    if pos>=end: return None
    w=bytes(b[pos:pos+16]).ljust(16,b'\0')
    lo=int.from_bytes(w[:8],'little'); hi=int.from_bytes(w[8:],'little')
    T=top(~lo&0x8080808080808080 & M)|(top(~hi&0x8080808080808080&M)<<8)
    Z=top(zb(lo))|(top(zb(hi))<<8)
    t=T; es=[]
    for _ in range(4):
        es.append(ctz(t|0x80000000)); t&=t-1
    e1,e2,e3,e4=es
    e=e4 if npair==2 else e2
    lens=e1<7 and e2-e1<=7 and (npair!=2 or (e3-e2<=7 and e4-e3<=7))
    if not (e<16 and lens and pos+e<end): return None
    nm = 1 if (Z & ~(T<<1) & ~1 & ((2<<e)-1)) else 0
    return pos+e+1, nm
def slow(b,pos,end,npair):
    nm=0
    for _ in range(2*npair):
        k=0; num=0
        while True:
            if pos>=end: return 'fail'
            r=b[pos]; pos+=1
            num|=(r&127)<<(7*k)
            if r<128:
                if r==0 and k>0: nm=1
                break
            k+=1
        if num>2**53-1: return 'fail'
    return pos,nm
random.seed(1)
n=0
for it in range(300000):
    L=random.randrange(1,40)
    pool=[random.randrange(256) for _ in range(3)]+[0,0x80,0x81,1,0x7f]
    b=[random.choice(pool) if random.random()<0.5 else random.randrange(256) for _ in range(L+20)]
    end=random.randrange(0,L+1); pos=random.randrange(0,max(1,end+2))
    npair=random.choice([1,2])
    f=fast(b,pos,end,npair)
    if f is None: continue
    n+=1
    s=slow(b,pos,end,npair)
    assert s==f,(b,pos,end,npair,f,s)
print('ok', n)
