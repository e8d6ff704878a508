"""Emulation of the kernel's top-of-book slot cache rules (tools/experiments/top_of_book_cache.patch)
over the CPU oracle's book, one message at a time, on tests/streams.py::top_streams: at every
message start a valid cache must name the slot the reference formula (_get_top_*_order_idx)
picks.  Prints the first mismatch or "no mismatch".  Run from the repo root (test tooling; it
uses the oracle).  Set NO=16 in the environment for the 16-slot config."""
import os
import sys; sys.path[:0]=['tests','jaxmarl-hft_amd','.']
import numpy as np
from streams import top_streams, init_book_messages
from oracle import pyoracle as O
from hftlob.config import JAXLOB_Configuration
from hftlob.layout import pack_lob_cfg
MAXINT=2**31-1
_no = int(os.environ.get('NO', '100'))
cfg=JAXLOB_Configuration(nOrders=_no, nTrades=min(_no, 100) if _no > 16 else 8); lc=pack_lob_cfg(cfg); nO=cfg.nOrders
E=64
init=init_book_messages(E, seed=5); ea=np.full((E,nO,6),-1,np.int32); et=np.full((E,cfg.nTrades,8),-1,np.int32)
a0,b0,_,_,_=O.book_process(lc, init, ea, ea, et, save_best=False)
msgs=top_streams(E,400,11+nO)
def best(s, bid):
    p=s[:,0]
    if bid: return int(p.max())
    q=np.where(p==-1, MAXINT, p); m=int(q.min()); return -1 if m==MAXINT else m
QUIRK={}
def scan_top(s, bid):
    p=s[:,0]
    mp = int(p.max()) if bid else int(np.where(p==-1,MAXINT,p).min())
    t=np.where(p==mp, s[:,4], MAXINT); mts=t.min()
    n=np.where(t==mts, s[:,5], MAXINT); mtn=n.min()
    QUIRK['q'] = (mts==MAXINT) or (mtn==MAXINT)
    return int(np.nonzero(n==mtn)[0][0]), mp
for e in range(E):
    A=a0[e:e+1].copy(); B=b0[e:e+1].copy(); T=et[e:e+1].copy()
    cache={0:None,1:None}   # side -> (top, top_p, ts, tns)
    for k in range(msgs.shape[1]):
        for bid,S in ((0,A[0]),(1,B[0])):
            c=cache[bid]
            if c is not None and best(S,bid)!=-1:
                st,mp=scan_top(S,bid)
                if S[st,0]!=mp: st=-9
                if (st,mp)!=(c[0],c[1]):
                    print("MISMATCH env",e,"msg",k,"side","bid" if bid else "ask","cache",c,"scan",(st,mp,int(S[st,4]),int(S[st,5])), "prev msg", msgs[e,k-1].tolist()); sys.exit(0)
        preA,preB=A[0].copy(),B[0].copy()
        oa,ob,ot,_,_=O.book_process(lc, msgs[e:e+1,k:k+1], A, B, T)
        A,B,T=oa,ob,ot
        m=msgs[e,k]
        traded = (ot!=T).any() if False else None
        for bid,pre,post in ((0,preA,A[0]),(1,preB,B[0])):
            c=cache[bid]
            bp=best(pre,bid)
            changed=np.nonzero((pre!=post).any(1))[0]
            adds=[i for i in changed if (pre[i]==-1).all() and not (post[i]==-1).all()]
            clears=[i for i in changed if (post[i]==-1).all() and not (pre[i]==-1).all()]
            over=[i for i in changed if not (pre[i]==-1).all() and not (post[i]==-1).all() and (pre[i][[0,2,3,4,5]]!=post[i][[0,2,3,4,5]]).any()]
            qonly=[i for i in changed if i not in adds and i not in clears and i not in over]
            crossed = len(clears)+len(qonly)>0 and m[0] in (1,4)
            if over: c=None
            if c is not None and any(i==c[0] for i in clears): c=None
            if len(clears)>1 and c is not None:   # eviction: GPU keeps top if worst != top_p
                pass
            for i in adds:
                np_,t,tn=int(post[i,0]),int(post[i,4]),int(post[i,5])
                better = (np_>bp) if bid else (np_!=-1 and (bp==-1 or np_<bp))
                if better:
                    c=(i,np_,t,tn) if (t!=MAXINT and tn!=MAXINT) else None
                elif np_==bp and c is not None:
                    if (t,tn,i)<(c[2],c[3],c[0]):
                        c=(i,np_,t,tn) if tn!=MAXINT else None
            # a crossing message on this side: GPU sets the cache from its last scan
            if m[0] in (1,4) and (len(qonly)>0 or len(clears)>0) and best(post,bid)!=-1 and not adds:
                st,mp=scan_top(post,bid)
                c=(st,mp,int(post[st,4]),int(post[st,5])) if (post[st,4]!=MAXINT and post[st,5]!=MAXINT and post[st,0]==mp and not QUIRK['q']) else None
            cache[bid]=c
print("no mismatch")
