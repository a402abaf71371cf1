import sys, torch
sys.path.insert(0, "/root/repo"); sys.path.insert(0, "/root/repo/tests")
import test_layers_gpu as T
from tensorflow_distributed_example_amd.ops import layer_ops as O
bf=torch.bfloat16; DEV="cuda"
B,H,W,C=2,112,112,64
R=B*H*W; Ho,Wo=56,56
(pt,pb),(pl,pr)=T._tf_same(H,3,2),T._tf_same(W,3,2)
g=O.ConvGeom(B,H,W,C,Ho,Wo,C,3,3,2,2,pt,pl)
y=T._r(R,C,seed=41,scale=2.0)+0.2
gamma=torch.rand(C,device=DEV)+0.5; beta=torch.randn(C,device=DEV)*0.3
stats=T._stats_buf(C); O.colstats(y,R,C,stats)
saved=torch.zeros(2*C,device=DEV); pooled=torch.zeros(B*Ho*Wo*C,device=DEV).to(bf); idx=torch.zeros(B*Ho*Wo*C,dtype=torch.uint8,device=DEV)
O.bn_relu_maxpool_fwd(y,R,C,pooled,idx,g,mode=1,stats=stats,saved=saved,gamma=gamma,beta=beta,eps=1e-5)
dpool=T._r(B*Ho*Wo*C,seed=42)
res=[]
for fused in (False,True):
    dst=torch.zeros(2*8*C,device=DEV); dx=torch.zeros(R,C,device=DEV).to(bf); dg=torch.zeros(C,device=DEV); db=torch.zeros(C,device=DEV)
    dout=torch.zeros(R,C,device=DEV).to(bf)
    if fused:
        O.bn_pool_bwd(dpool,idx,y,R,C,g,saved=saved,dstats=dst,dx=dx,gamma=gamma,beta=beta,relu=True,dgamma=dg,dbeta=db)
    else:
        O.maxpool_bwd(dpool,idx,dout,g)
        O.bn_bwd(dout,y,R,C,mode=1,saved=saved,gamma=gamma,beta=beta,relu=True,dstats=dst,dx=dx,dgamma=dg,dbeta=db)
    res.append((dx.float().cpu(),dg.cpu(),db.cpu(),dout.float().cpu()))
torch.cuda.synchronize()
# fp64 reference from the unfused dout
dout=res[0][3].double(); yd=y.double().cpu(); mu=saved[:C].double().cpu(); rs=saved[C:].double().cpu()
z=(yd-mu)*rs*gamma.double().cpu()+beta.double().cpu()
dz=dout*(z>0); xh=(yd-mu)*rs
sdz=dz.sum(0); sdx=(dz*xh).sum(0)
dxr=gamma.double().cpu()*rs*(dz-sdz/R-xh*sdx/R)
for name,(dx,dg,db,_) in zip(("unfused","fused"),res):
    print(name,"dx rel",T._rel(dx,dxr),"db rel",T._rel(db,sdz),"dg rel",T._rel(dg,sdx))
    print("  per-channel db err max", ((db.double()-sdz).abs()/(sdz.abs()+1e-3)).max().item())
print("sdz sample", sdz[:6].tolist()); print("fused db", res[1][2][:6].tolist()); print("unf db", res[0][2][:6].tolist())
