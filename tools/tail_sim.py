"""Tail scheduling study (tools, CPU): simulate the C4 shard's GPAD iterations in numpy fp32 (the
test as Algorithm 1, not bit-exact -- iteration counts within a few of the GPU's), then, at a
takeover iteration, the duo finisher as list scheduling on 512 slots: random order, perfect
longest-first (LPT), and orders by instance-state predictors (dual step |y - y_prev|, constraint
violations, ...), with their Spearman correlation to the remaining iterations.
  python3 tools/tail_sim.py 8192 [seed]
"""
import sys, time, numpy as np, heapq
import os
ROOT=os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0,ROOT); sys.path.insert(0,os.path.join(ROOT,'gpu-dualgradient-mpc_amd'))
import bench
from scipy.stats import spearmanr
B=int(sys.argv[1]); seed=int(sys.argv[2]) if len(sys.argv)>2 else 0
ML,G,L,M,g=bench.make_shard(200,200,B,seed*100000)
L=np.float32(L)
f=lambda a: np.ascontiguousarray(a,np.float32)
MLn=f(-ML); GL=f(G/L); pD=f(-g/L); gP=f(M); Gf=f(G); gf=f(g)
N=600
th=np.empty(N); be=np.empty(N); t,tm1,b=1.0,1.0,0.0
for v in range(N):
    tn=(np.sqrt(t**4+4*t**2)-t**2)/2; th[v]=t; be[v]=b; b=t*(1/tm1-1); tm1,t=t,tn
th=th.astype(np.float32); be=be.astype(np.float32)
tol=1e-4
y=np.zeros((B,200),np.float32); yp=y.copy(); z=np.zeros((B,200),np.float32)
done=np.zeros(B,bool); iters=np.full(B,N)
feats={}
prev=None
for v in range(N):
    w=y+be[v]*(y-yp)
    zh=w@MLn.T - gP
    z=(1-th[v])*z+th[v]*zh
    yn=np.maximum(w+zh@GL.T+pD,0)
    yp,y=y,yn
    if (v+1)%10==0:
        r=z@Gf.T-gf; rh=zh@Gf.T-gf
        vz=r.max(1); vh=rh.max(1); gap=-(w*rh).sum(1); wm=w.min(1)
        cA=vz<=tol; cB=(vh<=tol)&(wm>=0)&(gap<=tol)
        newly=(~done)&(cA|cB); iters[newly]=v+1; done|=newly
        cur=dict(vz=vz,vh=vh,dy=np.abs(y-yp).max(1),dy2=np.sqrt(((y-yp)**2).sum(1)),ny=np.sqrt((y*y).sum(1)))
        if v+1 in (260,270,280):
            feats[v+1]=dict(cur=cur,prev=prev,alive=~done.copy())
        prev=cur
        if done.all(): break
def sim(lens, slots, order, t_it=1.65):
    lens=lens[order]; h=[0.0]*slots; end=0
    for Lh in lens:
        t=heapq.heappop(h); t2=t+Lh*t_it; end=max(end,t2); heapq.heappush(h,t2)
    return end
for v0,F in feats.items():
    a=F['alive']; rem=(iters-v0)[a]; c=F['cur']; p=F['prev']
    cands={'dy':c['dy'],'dy2':c['dy2'],'vh':c['vh'],'vz':c['vz'],
           'dy_ratio':c['dy']/np.maximum(p['dy'],1e-30),'dy2/ny':c['dy2']/np.maximum(c['ny'],1e-30),
           'log(dy)/rate':np.log(np.maximum(c['dy'],1e-30)/1e-7)/np.maximum(np.log(np.maximum(p['dy'],1e-30)/np.maximum(c['dy'],1e-30)),0.01)}
    rng=np.random.default_rng(0)
    rnd=np.mean([sim(rem,512,rng.permutation(len(rem))) for _ in range(3)])
    best=sim(rem,512,np.argsort(-rem))
    s=[f'{k}: rho {spearmanr(v[a],rem).correlation:.2f} mk {sim(rem,512,np.argsort(-v[a])):.0f}' for k,v in cands.items()]
    print(v0, a.sum(), f'random {rnd:.0f} LPT {best:.0f} |', ' | '.join(s))
