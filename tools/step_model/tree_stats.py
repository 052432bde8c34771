"""Tree statistics of the reference builder's BVH (BVH.hpp:92-173, the host library's
pinned build) for C2 and C3 and for C3 variants: leaf sizes, depth, and the SAH
interior / triangle cost (sum of node surface areas over the root's: the expected
node visits and triangle tests of a random line through the scene).  The C3-vs-C2
record of round 6; CPU only.

    python tools/step_model/tree_stats.py
"""
import os
import sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import numpy as np
from pnraytracing_amd import scenes as S
def sa(b):
    d=np.maximum(b[:,3:6]-b[:,0:3],0); return 2*(d[:,0]*d[:,1]+d[:,1]*d[:,2]+d[:,2]*d[:,0])
def report(name,cfg):
    N=cfg.packed.nodes; leaf=N[:,7]<0; s=sa(N[:,:6]); root=s[0]
    cnt=(N[:,9]-N[:,8])[leaf]
    # depth
    depth=np.zeros(len(N),int); 
    for i in range(len(N)):
        if not leaf[i]:
            depth[i+1]=depth[i]+1; depth[int(N[i,7])]=depth[i]+1
    # SAH cost: expected node tests (interior visits) + triangle tests for a random line through the root
    ci=s[~leaf].sum()/root; ct=(s[leaf]*cnt).sum()/root
    # triangle areas
    V=cfg.packed.vertices[:,:3]; T=cfg.packed.triangles[:,:3].astype(int)
    p=V[T]; ar=0.5*np.linalg.norm(np.cross(p[:,1]-p[:,0],p[:,2]-p[:,0]),axis=1)
    e=np.maximum.reduce([np.linalg.norm(p[:,1]-p[:,0],axis=1),np.linalg.norm(p[:,2]-p[:,1],axis=1),np.linalg.norm(p[:,0]-p[:,2],axis=1)])
    print(f"{name}: nodes {len(N)} interior {(~leaf).sum()} leaves {leaf.sum()} mean leaf {cnt.mean():.2f} max leaf {cnt.max()} "
          f"max depth {depth.max()} mean leaf depth {depth[leaf].mean():.1f}; SAH interior {ci:.2f} tri {ct:.2f}; "
          f"root SA {root:.1f}; tri longest edge median {np.median(e):.4f} p99 {np.percentile(e,99):.3f}, sliver (edge^2/area>50) {(e**2/np.maximum(ar,1e-30)>50).mean()*100:.1f}%")
    return N,leaf,s,depth
for nm,f in [("C2",S.bunny_c2),("C3",S.marry_c3)]:
    report(nm,f())
# C3 without boards / figure alone / figure at C2 tessellation
import pnraytracing_amd.host as H
def c3_variant(boards=True, nu=176, nv=144, scale=(0.75,1.5,0.6)):
    sb=H.SceneBuilder(); m=H.Material(baseColor=(0.65,0.65,0.65))
    fig=H.mesh_displaced_sphere(nu,nv,1.0,(0,0,0),0.05,0xA11CE)
    sb.add_model(fig,[H.translate(0.1,1.55,-0.5),H.scale(*scale)],m,"marry")
    S._cornell_walls(sb,m)
    if boards:
        board=H.mesh_quad(27.5)
        for k,(met,rough,z) in enumerate([(0.95,0.02,-2.2),(0.80,0.15,-1.4),(0.60,0.35,-0.6)]):
            sb.add_model(board,[H.translate(-1.6+1.6*k,0.6,z),H.rotate(50.0-15.0*k,1,0,0),H.scale(0.012,1.0,0.004)],m,f"b{k}")
    return S.SceneConfig("x",sb.build(),S._cornell_camera(64,64),64,64,1)
report("C3 no boards", c3_variant(False))
report("C3, figure at uniform scale 0.75 (no 2x vertical stretch)", c3_variant(True, scale=(0.75,0.75,0.75)))
