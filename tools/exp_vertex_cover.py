"""Halo vertex cover: the push-pull greedy rule (distributed.py push_pull_plan) against a
minimum vertex cover (Konig: maximum bipartite matching, scipy) per peer pair, on a 1/10-scale
weak P=8 R-MAT (rank 0: 1M nodes).  CPU only.  Result: greedy is within 3.9 %."""
import sys, time
sys.path[:0]=['/root/repo']
import numpy as np, scipy.sparse as sp
from scipy.sparse.csgraph import maximum_bipartite_matching
from oracle.rmat import rmat_edges, scale_for
P=8; n_loc=1_000_000; N=P*n_loc; E=P*10_000_000
t=time.time()
s,d=[],[]
B=20_000_000
for e0 in range(0,E,B):
    ss,dd=rmat_edges(0, scale_for(N), N, e0, min(B,E-e0))
    m=dd<n_loc
    s.append(ss[m]); d.append(dd[m])
s=np.concatenate(s); d=np.concatenate(d)
print('gen',time.time()-t, len(s))
tot_greedy=tot_min=tot_pull=0
for peer in range(1,P):
    m=(s>=peer*n_loc)&(s<(peer+1)*n_loc)
    ps, pd = s[m]-peer*n_loc, d[m]
    # dedupe edges (multi-edges cover the same pair)
    key=np.unique(ps.astype(np.int64)*n_loc+pd)
    us,inv_s=np.unique(key//n_loc, return_inverse=True); ud,inv_d=np.unique(key%n_loc, return_inverse=True)
    cs=np.bincount(inv_s); cd=np.bincount(inv_d)
    push = cd[inv_d] > cs[inv_s]
    pulled=np.zeros(len(us),bool); pulled[inv_s[~push]]=True
    via_pull=pulled[inv_s]
    used=np.zeros(len(ud),bool); used[inv_d[~via_pull]]=True
    greedy=pulled.sum()+used.sum()
    A=sp.csr_matrix((np.ones(len(key),np.int8),(inv_s,inv_d)),shape=(len(us),len(ud)))
    mt=maximum_bipartite_matching(A, perm_type='column')
    mm=(mt>=0).sum()
    tot_greedy+=greedy; tot_min+=mm; tot_pull+=len(us)
    print(peer, 'pull-only',len(us),'greedy',greedy,'min cover',mm, flush=True)
print('total pull',tot_pull,'greedy',tot_greedy,'min',tot_min, 'saving %.1f%%'%(100*(1-tot_min/tot_greedy)))
