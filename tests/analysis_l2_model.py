#!/usr/bin/env python3
"""LRU model of one XCD's 4 MB L2 under the C2 gather's line stream (DESIGN.md
section 5, "Why the L2 misses stay"): block walks (bands, resident counts) and
the camera-outer order.  CPU analysis over the oracle geometry; slow (minutes).

    python tests/analysis_l2_model.py band16 noband band4
    EXTRA=1 python tests/analysis_l2_model.py skip        # resident counts, super-bands
    CAMOUTER=1 DRIFT=16 python tests/analysis_l2_model.py skip
"""
import os, sys, collections
import numpy as np
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, 'faster-voxelpose_amd')]
from oracle import fvp_oracle as O
from fvp import geometry
from fvp.workloads import WORKLOADS
import warnings; warnings.filterwarnings('ignore')
wn='c2'
w=WORKLOADS[wn]; cams,seq=w.cameras(); cl=cams[seq]; cl=list(cl.values()) if isinstance(cl,dict) else cl
X,Y,Z=w.voxels_per_axis
grid=O.compute_grid(w.space_size,w.space_center,w.voxels_per_axis)
rt=geometry.resize_transform(w.ori_image_size,w.image_size)
Wd,Hd=w.heatmap_size
V=len(cl)
# per voxel, per camera: 4 tap lines (or -1)
lines=np.full((X*Y*Z,V,4),-1,np.int64)
img_lines=Hd*Wd*64//128
for ci,c in enumerate(cl):
    g=O.project_grid(grid,c,w.ori_image_size,w.image_size,w.heatmap_size,rt).astype(np.float64)
    ix=(g[:,0]+1)/2*(Wd-1); iy=(g[:,1]+1)/2*(Hd-1)
    x0=np.floor(ix).astype(np.int64); y0=np.floor(iy).astype(np.int64)
    k=0
    for dy in (0,1):
        for dx in (0,1):
            xx=x0+dx; yy=y0+dy; on=(xx>=0)&(xx<Wd)&(yy>=0)&(yy<Hd)
            lines[:,ci,k]=np.where(on, ci*img_lines+(yy*Wd+xx)//2, -1); k+=1
GRID_BASE=10**9
def block_cols(cb, cols, band, tx=1):
    ty=cols//tx
    if band>0:
        gpr=Y//ty; tb=band//tx; trows=(X+tx-1)//tx; per=tb*gpr
        bi=cb//per; r=cb-bi*per; rows=min(tb,trows-bi*tb); gc=r//rows; xr=r-gc*rows
        x0=(bi*tb+xr)*tx; y0=gc*ty; nc=min(tx,X-x0)*ty
        return [(x0+c//ty)*Y+y0+c%ty for c in range(nc)]
    c0=cb*cols; return list(range(c0,min(c0+cols,X*Y)))
def sim(order_blocks, cols, cap_lines=32768, resident=256, grid=True):
    # order_blocks: list of column lists in dispatch order
    cache=collections.OrderedDict(); hits=miss=0
    def acc(l):
        nonlocal hits,miss
        if l in cache: cache.move_to_end(l); hits+=1
        else:
            miss+=1; cache[l]=1
            if len(cache)>cap_lines: cache.popitem(last=False)
    queue=list(order_blocks); active=[]
    def start():
        b=queue.pop(0); cols_=b; T=len(cols_)*Z
        slots=[(cols_[s%len(cols_)], s//len(cols_)) for s in range(T)]  # layer-major
        return [slots,0]
    while queue and len(active)<resident: active.append(start())
    while active:
        nxt=[]
        for a in active:
            slots,p=a; part=slots[p*64:(p+1)*64]
            for (col,z) in part:
                n=col*Z+z
                if grid: acc(GRID_BASE+(n*48)//128)
            for ci in range(V):
                for (col,z) in part:
                    for l in lines[col*Z+z,ci]:
                        if l>=0: acc(int(l))
            a[1]+=1
            if a[1]*64<len(slots): nxt.append(a)
            elif queue: nxt.append(start())
        active=nxt
    return hits,miss
cols=8
variants=sys.argv[1:] or ['band16','band8','band4','band32','noband','band80']
for v in [x for x in variants if x!='skip']:
    band=0 if v=='noband' else int(v[4:])
    nb=(X*Y)//cols
    order=[block_cols(cb,cols,band) for cb in range(nb)]
    h,m=sim(order,cols)
    print(v,'hit %.3f'%(h/(h+m)),'miss',m, 'miss MB %.1f'%(m*128/1e6), flush=True)
if os.environ.get('EXTRA'):
    nb=(X*Y)//cols
    base=[block_cols(cb,cols,0) for cb in range(nb)]  # row-major: cb = xr*10+gc
    for res in (128,64):
        h,m=sim(base,cols,resident=res); print('row-major resident',res,'miss',m,flush=True)
    # half-width super bands: rows walked in bands of R with the y-range split in halves
    for R in (80,40,20):
        order=[]
        for bx in range(0,X,R):
            for half in (0,1):
                for xr in range(bx,min(X,bx+R)):
                    for gc in range(half*5,half*5+5): order.append(base[xr*10+gc])
        h,m=sim(order,cols); print('halves R',R,'miss',m,flush=True)
    order=[]
    for bx in range(0,X,20):
        for q in range(0,10,2):
            for xr in range(bx,min(X,bx+20)):
                for gc in (q,q+1): order.append(base[xr*10+gc])
    h,m=sim(order,cols); print('fifths R20','miss',m,flush=True)
if os.environ.get('CAMOUTER'):
    nblk=int(os.environ.get('NBLK','128')); drift=int(os.environ.get('DRIFT','0'))
    colsb=(X*Y)//nblk
    blocks=[list(range(b*colsb,(b+1)*colsb)) for b in range(nblk)]
    cache=collections.OrderedDict(); hits=miss=0
    def acc(l):
        global hits,miss
        if l in cache: cache.move_to_end(l); hits+=1
        else:
            miss+=1; cache[l]=1
            if len(cache)>32768: cache.popitem(last=False)
    # each block: slots layer-major over its columns; per camera all passes
    P=[(len(b)*Z+63)//64 for b in blocks]
    slots=[[(b[s%len(b)], s//len(b)) for s in range(len(b)*Z)] for b in blocks]
    # global time steps: block i at step t processes (camera, pass) = divmod(t - drift_i, P)
    rng=np.random.default_rng(0); off=rng.integers(0,drift+1,nblk) if drift else np.zeros(nblk,int)
    T=max(P)*V+drift
    for t in range(T):
        for i,b in enumerate(blocks):
            tt=t-off[i]
            if tt<0 or tt>=P[i]*V: continue
            ci,p=divmod(tt,P[i])
            part=slots[i][p*64:(p+1)*64]
            for (col,z) in part: acc(GRID_BASE+ci*10**7+((col*Z+z)*8)//128)
            for (col,z) in part:
                for l in lines[col*Z+z,ci]:
                    if l>=0: acc(int(l))
    print('camera-outer nblk',nblk,'drift',drift,'hit %.3f'%(hits/(hits+miss)),'miss',miss,flush=True)
