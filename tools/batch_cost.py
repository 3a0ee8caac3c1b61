"""Offline batch-cost model for k_batch_rows (C4): reads the per-batch dump
written with SHDPE_DEBUG=1 SHDPE_DUMP_BATCHES=<file> (rows per batch, kernel
counters, hub offsets), correlates the relax / post cycles with the host-side
features the batch order can use, and replays the dynamic batch take (512
workgroups) for several orders to price the schedule tail.

usage: python tools/batch_cost.py <dump file>
"""
import sys
import numpy as np, heapq
b=open(sys.argv[1] if len(sys.argv) > 1 else 'gpurun_out/r03bd/c4_batches.bin','rb').read()
nB,LB=np.frombuffer(b[:8],np.int32)
o=8; order=np.frombuffer(b[o:o+4*nB*LB],np.int32).reshape(nB,LB); o+=4*nB*LB
dbg=np.frombuffer(b[o:o+4*nB*16],np.int32).reshape(nB,16).astype(np.float64); o+=4*nB*16
nOff=np.frombuffer(b[o:o+8],np.int64)[0]; o+=8
off=np.frombuffer(b[o:o+8*nOff],np.float64)
relax=dbg[:,5]*1024; post=(dbg[:,6]+dbg[:,7])*1024
offb=np.where(order>=0, off[np.maximum(order,0)], np.nan)
def makespan(costs,G=512):
    h=[0.0]*G; heapq.heapify(h)
    for c in costs:
        t=heapq.heappop(h); heapq.heappush(h,t+c)
    return max(h)
F={'mean':np.nanmean(offb,1),'max':np.nanmax(offb,1),'min':np.nanmin(offb,1),'sd':np.nanstd(offb,1),
   'med':np.nanmedian(offb,1),'q75':np.nanpercentile(offb,75,axis=1),'q25':np.nanpercentile(offb,25,axis=1)}
F['sumsq']=np.nanmean(offb**2,1)
for k,v in F.items(): print(k,'%.3f'%np.corrcoef(v,relax)[0,1])
X=np.column_stack([np.ones(nB)]+list(F.values()))
coef,*_=np.linalg.lstsq(X,relax,rcond=None)
pred=X@coef
print('linear fit corr %.3f'%np.corrcoef(pred,relax)[0,1])
for nm,key in [('cur(mean)',F['mean']),('fit',pred),('max',F['max']),('actual',relax)]:
    idx=np.argsort(-key,kind='stable')
    print(nm,'relax makespan %.1fM'%(makespan(relax[idx])/1e6))
# post: orderings
for nm,key in [('index',-np.arange(nB)),('procs',dbg[:,4]),('relax',relax),('phases',dbg[:,0]),('actual',post)]:
    idx=np.argsort(-key,kind='stable')
    print('post by',nm,'%.1fM'%(makespan(post[idx])/1e6))
for j in range(16):
    c=np.corrcoef(dbg[:,j],post)[0,1] if dbg[:,j].std()>0 else 0
    print('dbg',j,'corr post %.3f'%c, 'mean %.1f'%dbg[:,j].mean())
# 2-stream: relax jobs (index order) on 512 slots; a slot whose relax WG exits
# (no relax job left) runs post jobs in relax-completion order, waiting for
# the job's relax to finish
def combined(relax, post, G=512):
    h=[(0.0,i) for i in range(G)]; heapq.heapify(h)
    done=[]  # (finish time, batch)
    for b,c in enumerate(relax):
        t,i=heapq.heappop(h); done.append((t+c,b)); heapq.heappush(h,(t+c,i))
    done.sort()
    # slots free at their relax end
    free=sorted(t for t,i in h)
    hq=[(t,k) for k,t in enumerate(free)]; heapq.heapify(hq)
    end=0.0
    for fin,b in done:
        t,k=heapq.heappop(hq); s=max(t,fin); e=s+post[b]; end=max(end,e); heapq.heappush(hq,(e,k))
    return end
print('sequential %.1fM  combined %.1fM  lower bound %.1fM'%((makespan(relax)+makespan(post))/1e6, combined(relax,post)/1e6, (relax.sum()+post.sum())/512/1e6))
