import itertools
# lane groups of ds_read_b128
G=[list(range(0,4))+list(range(12,16))+list(range(20,28)),
   list(range(4,12))+list(range(16,20))+list(range(28,32)),
   list(range(32,36))+list(range(44,48))+list(range(52,60)),
   list(range(36,44))+list(range(48,52))+list(range(60,64))]
def conflicts(s, stride_chunks=4):
    worst=0
    for b in range(64):
        for g in G:
            quads={}
            for l in g:
                fr=l&15; fq=l>>4
                p=b+fr
                q=(p*stride_chunks + (fq ^ s(p)))%16
                quads[q]=quads.get(q,0)+1
            worst=max(worst,max(quads.values()))
    return worst
print("none", conflicts(lambda p:0))
best=[]
for perm in itertools.product(range(4),repeat=4):
    w=conflicts(lambda p:perm[(p>>2)&3])
    if w==1: best.append(perm)
print("g((p>>2)&3):",best[:5], len(best))
for perm in itertools.product(range(4),repeat=8):
    w=conflicts(lambda p:perm[(p>>2)&7])
    if w==1: print("g((p>>2)&7):",perm); break
else: print("none for &7")
