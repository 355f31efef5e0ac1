#!/usr/bin/env python
"""Lane use of the render kernels under culling granularities (bench scene,
a sample of Gaussians, float64 EWA splats, T-termination ignored): the share
of SIMD lanes whose pixel passes alpha >= 1/255 when a wave evaluates an entry
for every 8x8 quadrant it reaches, vs 4x4 / 8x2 / 16x4 blocks.  Also the
rounds per (entry, tile) if each 16-lane group owned a fixed set of four 4x4
blocks of the tile (a colouring) and a wave evaluated one reached block per
group per round: max over the groups of its reached blocks, relative to the
8x8-quadrant count ("parity" is today's quadrant walk).
usage: S=int(__import__("os").environ.get("S","40000")) python tools/lane_use.py [P]"""
import math, sys, numpy as np, torch
sys.path.insert(0, __import__("os").path.join(__import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.abspath(__file__))), "wildgs-slam-blackwell_amd", "python"))
from wgsr.scene import make_scene
W,H=1920,1080
P=int(sys.argv[1]) if len(sys.argv)>1 else 1_000_000
S=int(__import__("os").environ.get("S","40000"))
sc=make_scene(P,W,H,3,seed=0)
idx=torch.randperm(P,generator=torch.Generator().manual_seed(1))[:S]
m=sc.means3D[idx].double().numpy(); s=sc.scales[idx].double().numpy(); q=sc.rotations[idx].double().numpy(); o=sc.opacities[idx,0].double().numpy()
fx=0.9*W; fy=fx; cx=W/2; cy=H/2
def rot(q):
    r,x,y,z=q[:,0],q[:,1],q[:,2],q[:,3]
    return np.stack([np.stack([1-2*(y*y+z*z),2*(x*y-r*z),2*(x*z+r*y)],-1),
                     np.stack([2*(x*y+r*z),1-2*(x*x+z*z),2*(y*z-r*x)],-1),
                     np.stack([2*(x*z-r*y),2*(y*z+r*x),1-2*(x*x+y*y)],-1)],-2)
R=rot(q); Sm=np.einsum('nij,nj->nij',R,s); cov3=np.einsum('nij,nkj->nik',Sm,Sm)
tx,ty,tz=m[:,0],m[:,1],m[:,2]
J=np.zeros((S,2,3)); J[:,0,0]=fx/tz; J[:,0,2]=-fx*tx/tz**2; J[:,1,1]=fy/tz; J[:,1,2]=-fy*ty/tz**2
c2=np.einsum('nij,njk,nlk->nil',J,cov3,J); c2[:,0,0]+=0.3; c2[:,1,1]+=0.3
det=c2[:,0,0]*c2[:,1,1]-c2[:,0,1]**2
con=np.stack([c2[:,1,1]/det,-c2[:,0,1]/det,c2[:,0,0]/det],-1)
mx=fx*tx/tz+cx-0.5; my=fy*ty/tz+cy-0.5
mid=0.5*(c2[:,0,0]+c2[:,1,1]); lam=mid+np.sqrt(np.maximum(0.1,mid*mid-det)); rad=np.ceil(3*np.sqrt(lam))
COL={'parity':lambda a,b:(a&1)+2*(b&1),'rows':lambda a,b:b,'diag':lambda a,b:(a+b)&3,'knight':lambda a,b:(a+2*b)&3}; EV={k:0 for k in COL}
ev8=0; lanes=0; ev4=0; ev82=0; ev168=0
for i in range(S):
    r=int(rad[i]); x0=max(0,int(mx[i]-r)); x1=min(W,int(mx[i]+r)+1); y0=max(0,int(my[i]-r)); y1=min(H,int(my[i]+r)+1)
    if x1<=x0 or y1<=y0: continue
    xs=np.arange(x0,x1); ys=np.arange(y0,y1)
    dx=mx[i]-xs[None,:]; dy=my[i]-ys[:,None]
    pw=-0.5*(con[i,0]*dx*dx+con[i,2]*dy*dy)-con[i,1]*dx*dy
    a=np.minimum(0.99,o[i]*np.exp(pw)); ok=(pw<=0)&(a>=1/255)
    if not ok.any(): continue
    yy,xx=np.nonzero(ok); X=xs[xx]; Y=ys[yy]
    lanes+=len(X)
    ev8+=len(set(zip(X//8,Y//8)));
    tiles={}
    for (a,b) in set(zip(X//4,Y//4)): tiles.setdefault((a//4,b//4),[]).append((a%4,b%4))
    for l in tiles.values():
        for nm,f in COL.items():
            c=[0]*4
            for (a,b) in l: c[f(a,b)]+=1
            EV[nm]+=max(c)
    ev4+=len(set(zip(X//4,Y//4))); ev82+=len(set(zip(X//8,Y//2))); ev168+=len(set(zip(X//16,Y//4)))
print(f"passing pixels {lanes}, 8x8 evals {ev8} util {lanes/(64*ev8):.3f}; 4x4 evals {ev4} util {lanes/(16*ev4):.3f} (lane-evals x{16*ev4/(64*ev8):.3f}); 8x2 util {lanes/(16*ev82):.3f} x{16*ev82/(64*ev8):.3f}; 16x4 util {lanes/(64*ev168):.3f} x{ev168/ev8:.3f}")
print("fixed-colouring rounds / 8x8 evals:", {k: round(v / ev8, 3) for k, v in EV.items()})
