"""Host simulation behind the split-decode experiment (commit
4cb124d): how far past a
mid-string start bit a second decode chain needs to resynchronise with the
first, over the bench's synthetic strings (test-side oracle tables)."""
import os, sys
T = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests")
sys.path.insert(0, T)
import oracle_lib as O
import _paths, qhuff
codes = {}
for s in range(257):
    c,b = O.code_of(s); codes[(c,b)] = s
def boundaries(bits, start):
    out=[]; pos=start; 
    while True:
        c=0
        for L in range(1,31):
            if pos+L > len(bits): return out, None
            c = (c<<1) | bits[pos+L-1]
            if (c,L) in codes:
                sym=codes[(c,L)]
                pos += L; out.append(pos)
                if sym==256: return out, pos
                break
        else: return out, None
data, off = qhuff.synth_batch(3000, seed=5)
dist=[]
for i in range(3000):
    s=bytes(data[off[i]:off[i+1]]); hb=O.huffman_enc(s)
    bits=[(b>>(7-k))&1 for b in hb for k in range(8)]
    n=len(bits)
    if n < 200: continue
    h=(n>>1)&~7
    A,_=boundaries(bits,0); B,_=boundaries(bits,h)
    Bs=set(B)|{h}
    d=next((a-h for a in A if a>=h and a in Bs), None)
    dist.append(d)
import collections
print(len(dist), sorted(collections.Counter(min(x//8*8,200) if x is not None else -1 for x in dist).items()))
