"""Model check of the BF tie sort used by the env kernels (vmp_kernels.hip
wave_aquicksort / aquicksort_lds): numpy's scalar introsort (aquicksort_ +
aheapsort_, npysort) restated serially, against the two transformations the
kernels make — (1) only partitions intersecting the needed position range are
sorted, (2) each Hoare partition is computed from the left/right stop lists
(A, B, K = #{A[k] < B[k]}, final stop min(A[K], B[K-1])) and small partitions
by a stable rank sort. Heavy ties, random ranges and forced depth-limit
heapsorts; positions lo..hi must equal the full serial sort's exactly."""
import numpy as np

def fless(a,b): return a<b
def heapsort(v,t,off,n):
    a=lambda i: t[off+i-1]
    def seta(i,x): t[off+i-1]=x
    l=n>>1
    while l>0:
        tmp=a(l); i=l; j=l<<1
        while j<=n:
            if j<n and fless(v[a(j)],v[a(j+1)]): j+=1
            if fless(v[tmp],v[a(j)]): seta(i,a(j)); i=j; j+=j
            else: break
        seta(i,tmp); l-=1
    while n>1:
        tmp=a(n); seta(n,a(1)); n-=1; i=1; j=2
        while j<=n:
            if j<n and fless(v[a(j)],v[a(j+1)]): j+=1
            if fless(v[tmp],v[a(j)]): seta(i,a(j)); i=j; j+=j
            else: break
        seta(i,tmp)
def serial(v,num,lo,hi,par=False,depthcap=None):
    t=list(range(num)); stack=[]; pl,pr=0,num-1
    cd=0;u=num
    while True:
        u>>=1
        if not u: break
        cd+=1
    cd*=2
    if depthcap is not None: cd=depthcap
    while True:
        skip=False
        if pr<lo or pl>hi: skip=True
        elif cd<0: heapsort(v,t,pl,pr-pl+1); skip=True
        if not skip:
            while pr-pl>15:
                pm=pl+((pr-pl)>>1)
                if fless(v[t[pm]],v[t[pl]]): t[pm],t[pl]=t[pl],t[pm]
                if fless(v[t[pr]],v[t[pm]]): t[pr],t[pm]=t[pm],t[pr]
                if fless(v[t[pm]],v[t[pl]]): t[pm],t[pl]=t[pl],t[pm]
                vp=v[t[pm]]; pj=pr-1
                t[pm],t[pj]=t[pj],t[pm]
                if not par:
                    pi=pl
                    while True:
                        pi+=1
                        while fless(v[t[pi]],vp): pi+=1
                        pj-=1
                        while fless(vp,v[t[pj]]): pj-=1
                        if pi>=pj: break
                        t[pi],t[pj]=t[pj],t[pi]
                else:
                    B=[q for q in range(pr-2,pl-1,-1) if not fless(vp,v[t[q]])]
                    A=[q for q in range(pl+1,pr) if not fless(v[t[q]],vp)]
                    K=sum(1 for k in range(min(len(A),len(B))) if A[k]<B[k])
                    for k in range(K): t[A[k]],t[B[k]]=t[B[k]],t[A[k]]
                    pi=A[K]
                    if K>0 and B[K-1]<pi: pi=B[K-1]
                pk=pr-1; t[pi],t[pk]=t[pk],t[pi]
                if pi-pl<pr-pi: stack.append((pi+1,pr,cd-1)); pr=pi-1
                else: stack.append((pl,pi-1,cd-1)); pl=pi+1
                cd-=1
                if pr<lo or pl>hi: skip=True; break
            if not skip:
                if par:
                    seg=t[pl:pr+1]; n=len(seg)
                    out=[None]*n
                    for i in range(n):
                        r=sum(1 for j in range(n) if fless(v[seg[j]],v[seg[i]]) or (j<i and not fless(v[seg[i]],v[seg[j]])))
                        out[r]=seg[i]
                    t[pl:pr+1]=out
                else:
                    for pi in range(pl+1,pr+1):
                        vi=t[pi]; vv=v[vi]; pj=pi; pk=pi-1
                        while pj>pl and fless(vv,v[t[pk]]): t[pj]=t[pk]; pj-=1; pk-=1
                        t[pj]=vi
        if not stack: break
        pl,pr,cd=stack.pop()
    return t


def test_parallel_partition_and_range_sort_equal_serial_introsort():
    rng = np.random.default_rng(1)
    for it in range(600):
        n = int(rng.integers(1, 300))
        nv = int(rng.integers(1, 30))
        v = list(rng.integers(0, nv, n).astype(np.float32))
        lo = int(rng.integers(0, n))
        hi = int(rng.integers(lo, n))
        dc = None if it % 5 else int(rng.integers(-1, 3))
        full = serial(v, n, 0, n - 1, depthcap=dc)
        assert sorted(full) == list(range(n))
        assert all(v[full[i]] <= v[full[i + 1]] for i in range(n - 1))
        for par in (False, True):
            r = serial(v, n, lo, hi, par, depthcap=dc)
            assert r[lo:hi + 1] == full[lo:hi + 1], (n, nv, lo, hi, par)
