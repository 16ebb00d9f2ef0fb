#!/usr/bin/env python3
"""Tap sharing within a gather wave: for each camera and
each run of 16 consecutive voxels (one wave of voxelize_kernel, LPV = 4), the
fraction of distinct (row, x0) tap segments among the 2 per in-image
voxel-camera -- what deduplicating tap loads inside a wave could save.
Oracle geometry (CPU test tooling, kept under tests/ as the oracle's users are); C5 subsampled every 7th wave.

    python tests/analysis_tap_share.py c2 c4 c5
"""
import os, sys
import numpy as np
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, 'faster-voxelpose_amd')]
from oracle import fvp_oracle as O
from fvp import geometry
from fvp.workloads import WORKLOADS
def distinct(keys, valid):
    # keys [nw,k] int64, valid mask: count distinct valid keys per row
    k=np.where(valid, keys, np.iinfo(np.int64).max)
    s=np.sort(k,axis=1)
    d=np.ones_like(s,dtype=bool); d[:,1:]=s[:,1:]!=s[:,:-1]
    d&= s!=np.iinfo(np.int64).max
    return d.sum()
for wn in sys.argv[1:]:
    w=WORKLOADS[wn]; cams,seq=w.cameras(); cl=cams[seq]; cl=list(cl.values()) if isinstance(cl,dict) else cl
    grid=O.compute_grid(w.space_size,w.space_center,w.voxels_per_axis)
    sub = 7 if wn=='c5' else 1
    rt=geometry.resize_transform(w.ori_image_size,w.image_size)
    Wd,Hd=w.heatmap_size; N=grid.shape[0]; nw=N//16
    sel=np.arange(0,nw,sub)
    idx=(sel[:,None]*16+np.arange(16)[None]).ravel()
    g_=grid[idx]
    need=rows=act=0
    for c in cl:
        g=O.project_grid(g_,c,w.ori_image_size,w.image_size,w.heatmap_size,rt).astype(np.float64)
        ix=(g[:,0]+1)/2*(Wd-1); iy=(g[:,1]+1)/2*(Hd-1)
        x0=np.floor(ix).astype(np.int64); y0=np.floor(iy).astype(np.int64)
        on=((x0>=-1)&(x0<Wd)&(y0>=-1)&(y0<Hd)).reshape(-1,16)
        X0=x0.reshape(-1,16); Y0=y0.reshape(-1,16)
        k0=(Y0+2)*4096+X0+2; k1=(Y0+3)*4096+X0+2
        keys=np.concatenate([k0,k1],1); val=np.concatenate([on,on],1)
        rows+=distinct(keys,val); need+=2*on.sum(); act+=on.sum()
    print(wn,'distinct row segs / needed %.3f'%(rows/need),'active %.3f'%(act/(16*len(sel)*len(cl))), flush=True)
