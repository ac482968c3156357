#!/usr/bin/env python3
"""Round-5 estimate (CPU, numpy; not a test): how much of reverseRayTraceFast's idle lane time
could frustum culling before the march recover?  Rebuilds the bench's secondary volume with
the oracle (tests/golden/gen_march_digests.py), orders the occupied voxels along the same 3D
Morton curve as the GPU queue, and counts, per pose, the 64-item units whose voxels are partly
inside and partly outside the camera frustum (an approximate float projection: an estimate, not
the exact deproject test).  Result: 1.8 % of the units are mixed, holding
0.47M of the 22.0M rejected items -- frustum culling would not raise the lanes' occupancy."""
import sys, os, numpy as np, time
ROOT=os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0]=[ROOT,os.path.join(ROOT,'depth-map-fusion-utils_amd'),os.path.join(ROOT,'tests','golden')]
from gen_march_digests import build_volume
from dmf_amd import scene
t=time.time()
v,K,poses=build_volume(512,640,480,128,16)
occ=np.asarray(v.occupied_cells_,np.uint64)
V=len(occ); print('V',V, time.time()-t)
xid=(occ>>np.uint64(40)).astype(np.int64); yid=((occ>>np.uint64(20))&np.uint64(0xFFFFF)).astype(np.int64); zid=(occ&np.uint64(0xFFFFF)).astype(np.int64)
dl=1/512; cen=np.stack([xid*dl-0.5+dl/2, yid*dl-0.5+dl/2, zid*dl-0.5+dl/2],1)
def morton(x,y,z):
    def part(a):
        a=a.astype(np.uint64)&np.uint64(0x1fffff)
        a=(a|(a<<np.uint64(32)))&np.uint64(0x1f00000000ffff)
        a=(a|(a<<np.uint64(16)))&np.uint64(0x1f0000ff0000ff)
        a=(a|(a<<np.uint64(8)))&np.uint64(0x100f00f00f00f00f)
        a=(a|(a<<np.uint64(4)))&np.uint64(0x10c30c30c30c30c3)
        a=(a|(a<<np.uint64(2)))&np.uint64(0x1249249249249249)
        return a
    return part(x)|(part(y)<<np.uint64(1))|(part(z)<<np.uint64(2))
order=np.argsort(morton(xid,yid,zid),kind='stable')
c=cen[order]
Kf=np.asarray(K,np.float64).reshape(-1); fx,cx,fy,cy=Kf[0],Kf[2],Kf[4],Kf[5]
W,H=640,480
tot_units=0; mixed=0; rej_in_mixed=0; rej_total=0; valid_total=0
for p in range(128):
    T=poses[p].reshape(3,4).astype(np.float64); R=T[:,:3]; t=T[:,3]
    q=(c-t)@np.linalg.inv(R).T
    z=q[:,2]; 
    with np.errstate(divide='ignore',invalid='ignore'):
        col=fx*q[:,0]/z+cx; row=fy*q[:,1]/z+cy
    ok=(z>0)&(col>=0)&(col<W)&(row>=0)&(row<H)
    n=len(ok); nu=(n+63)//64
    pad=np.zeros(nu*64,bool); pad[:n]=ok
    u=pad.reshape(nu,64); cnt=u.sum(1)
    full=(cnt==64)|(cnt==0)
    tot_units+=nu; mixed+=(~full).sum(); rej_in_mixed+=(64-cnt[~full]).sum(); rej_total+=(n-ok.sum()); valid_total+=ok.sum()
print('units',tot_units,'mixed',mixed, 'frac mixed',mixed/tot_units,'rejected total',rej_total,'rejected in mixed',rej_in_mixed,'valid',valid_total)
