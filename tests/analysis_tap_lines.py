#!/usr/bin/env python3
"""Distinct 128-B lines per in-image tap and camera for a gather wave of 16 voxels
shaped tx x-rows x ty columns x tz z-layers (layer-major slots):
the L1 -> L2 traffic a wave arrangement implies.  CPU analysis over the oracle geometry.

    python tests/analysis_tap_lines.py c2            (c5: add a camera subsample, e.g. "c5 4")
"""
import os, sys
import numpy as np
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, 'faster-voxelpose_amd')]
from oracle import fvp_oracle as O
from fvp import geometry
from fvp.workloads import WORKLOADS
wn=sys.argv[1]
w=WORKLOADS[wn]; cams,seq=w.cameras(); cl=cams[seq]; cl=list(cl.values()) if isinstance(cl,dict) else cl
X,Y,Z=w.voxels_per_axis
sub=int(sys.argv[2]) if len(sys.argv)>2 else 1
grid=O.compute_grid(w.space_size,w.space_center,w.voxels_per_axis)
rt=geometry.resize_transform(w.ori_image_size,w.image_size)
Wd,Hd=w.heatmap_size
cl=cl[::sub]
proj=[]
for c in cl:
    g=O.project_grid(grid,c,w.ori_image_size,w.image_size,w.heatmap_size,rt).astype(np.float64)
    ix=(g[:,0]+1)/2*(Wd-1); iy=(g[:,1]+1)/2*(Hd-1)
    proj.append((np.floor(ix).astype(np.int64), np.floor(iy).astype(np.int64)))
V=np.arange(X*Y*Z).reshape(X,Y,Z)
def waves(tx,ty,tz):  # wave = tx x-rows * ty columns * tz z-layers (=16)
    assert tx*ty*tz==16
    return V.reshape(X//tx,tx,Y//ty,ty,Z//tz,tz).transpose(0,2,4,1,3,5).reshape(-1,16)
SHAPES=[(1,1,16),(1,8,2),(1,4,4),(1,2,8),(2,1,8),(2,4,2),(2,2,4),(4,4,1),(2,8,1),(4,2,2),(8,2,1),(4,1,4),(1,16,1),(16,1,1)]
pitch=128 if len(sys.argv)<=3 else int(sys.argv[3])
for (tx,ty,tz) in SHAPES:
    if X%tx or Y%ty or Z%tz: continue
    wv=waves(tx,ty,tz); lines=0; need=0
    for (x0,y0) in proj:
        X0=x0[wv]; Y0=y0[wv]; keys=[]; ons=[]
        for dy in (0,1):
            for dx in (0,1):
                xx=X0+dx; yy=Y0+dy
                on=(xx>=0)&(xx<Wd)&(yy>=0)&(yy<Hd)
                keys.append(np.where(on,(yy*Wd+xx)*64//pitch,-1)); ons.append(on)
        key=np.concatenate(keys,1)
        s=np.sort(key,axis=1); d=np.ones_like(s,dtype=bool); d[:,1:]=s[:,1:]!=s[:,:-1]; d&=s>=0
        lines+=d.sum(); need+=np.concatenate(ons,1).sum()
    print(wn, f'x{tx}y{ty}z{tz}', 'lines/tap %.3f'%(lines/need), flush=True)
