"""CPU estimate (not the renderer): how many of C2's kept burst children a
non-emissive sphere occludes, to decide whether a per-burst sphere occluder
(like pt_device.h Occl for planes) could pay.  Primary-ray diffuse hits on C2's
geometry, uniform hemisphere children; prints the fraction of kept children
(after the ground plane's occlusion) whose first hit is a sphere, the share the
burst's best single sphere takes, and that share where it exceeds 5 %.
Output of this script: profiles/round6/c2_occluder_sim.txt."""
import numpy as np, math
rng=np.random.default_rng(0)
# C2 geometry
sph=[]
for k in range(8):
    a=2*math.pi*k/8
    sph.append(((1.6*math.cos(a), -0.2+0.1*(k%3), -5+1.6*math.sin(a)), 0.45))
C=np.array([s[0] for s in sph]); R=np.array([s[1] for s in sph])
mats=["diffuse","mirror","glass","diffuse","diamond","mirror","glass","diffuse"]
W,H=1280,720; dist=2*min(W,H)
def first_hit(o,d):
    # returns t, kind ('sphere',i) or ('ground',) or ('sky',)
    best=(1e30,None)
    for i in range(8):
        oc=o-C[i]; b=np.dot(oc,d); c=np.dot(oc,oc)-R[i]**2; disc=b*b-c
        if disc>0:
            s=math.sqrt(disc); t0=-b-s; t1=-b+s
            t=t0 if t0>1e-4 else (t1 if t1>1e-4 else None)
            if t is not None and t<best[0]: best=(t,('s',i))
    if d[1]<0:
        t=(o[1]+0.7)/(-d[1])
        if t>1e-4 and t<best[0]: best=(t,('g',))
    return best
# sample primary rays -> diffuse hits (ground or diffuse spheres)
origins=[]
for _ in range(4000):
    px=rng.uniform(0,W); py=rng.uniform(0,H)
    d=np.array([(2*px/W-1)*W, (1-2*py/H)*H, -dist]); d/=np.linalg.norm(d)
    t,k=first_hit(np.zeros(3),d)
    if k is None: continue
    p=t*d
    if k[0]=='g': n=np.array([0,1.,0]); origins.append((p,n,'g'))
    elif mats[k[1]]=="diffuse": n=(p-C[k[1]])/R[k[1]]; origins.append((p,n,'s%d'%k[1]))
print("diffuse-burst origins:", len(origins))
tot_kept=0; sph_occ=0; top1=0; top1_sel=0; ground_occ=0
for (p,n,tag) in origins[:600]:
    # hemisphere directions (uniform in ball then normalized, accepted n.w>eps)
    v=rng.uniform(-1,1,(4000,3)); v=v[(v*v).sum(1)<1]; v=v[v@n>1e-4]
    d=v/np.linalg.norm(v,axis=1)[:,None]
    o=p+1e-4*n
    hits=np.zeros(len(d),int)-1; gocc=np.zeros(len(d),bool)
    for j,dd in enumerate(d):
        t,k=first_hit(o,dd)
        if k is None: continue
        if k[0]=='g': gocc[j]=True
        else: hits[j]=k[1]
    kept=~gocc
    tot_kept+=kept.sum(); ground_occ+=gocc.sum()
    sh=hits[kept]; sph_occ+=(sh>=0).sum()
    if (sh>=0).any():
        cnt=np.bincount(sh[sh>=0],minlength=8); b=cnt.max()
        top1+=b
        if b>=0.05*len(sh): top1_sel+=b
print("kept(after ground)",tot_kept,"sphere-occluded",sph_occ/tot_kept,"top1",top1/tot_kept,"top1>=5%",top1_sel/tot_kept,"ground-occluded frac of all", ground_occ/(ground_occ+tot_kept))
