"""LDS bank model of the C4 fan march line reads: a 32-lane
group = 4 lines (row +/-, column +/-) x 8 agents; agent a's line word at step k is
a*S + lx_a +/- k (rows) or C0 + a*S + ly_a +/- k (columns), u64 words, bank slot
w mod 32.  Prints the expected LDS cycles per group-instruction (1 = conflict
free) for the build's stride S = 8 TW + 1 = 49 and the best S / C0 found."""
import numpy as np
rng=np.random.default_rng(0)
def cycles(S, C0, trials=400, N=8):
    tot=0; cnt=0
    for _ in range(trials):
        lx=rng.integers(21,29,size=N); ly=rng.integers(21,29,size=N)
        for k in range(1,21):
            words=[]
            for m in range(4):
                for a in range(N):
                    if m==0: w=a*S+lx[a]+k
                    elif m==1: w=a*S+lx[a]-k
                    elif m==2: w=C0+a*S+ly[a]+k
                    else: w=C0+a*S+ly[a]-k
                    words.append(w)
            # group of 32 lanes: 4 lines x 8 agents
            slots={}
            for w in set(words):
                slots.setdefault(w%32,set()).add(w)
            tot+=max(len(v) for v in slots.values()); cnt+=1
    return tot/cnt
base=cycles(49, 0)
print('S=49 C0=0', base)
res=[]
for S in range(49,81):
    for C0 in range(0,32):
        res.append((cycles(S,C0,trials=60),S,C0))
res.sort()
print(res[:10])
for S in (49,):
    print([ (C0, round(cycles(S,C0,100),2)) for C0 in range(0,32,4)])
