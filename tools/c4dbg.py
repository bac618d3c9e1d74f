import sys, numpy as np, torch, time
sys.path.insert(0,'distributed-drift-detection_amd')
from ddm_amd import kernels
S,L=1000000,4096
dev=torch.device('cuda',0)
err=torch.empty(S*L+16,dtype=torch.uint8,device=dev)
kernels.synth_bernoulli_streams(err,S,L,20261015)
nb=41
ev=torch.empty((S*nb,2),dtype=torch.int32,device=dev)
sc=torch.empty(kernels.scan_batches_scratch_size(S,L),dtype=torch.uint8,device=dev)
st=torch.from_numpy(kernels.fresh_states(S).view(np.uint8)).to(dev)
prm=kernels.params_struct()
kernels.scan_batches(err,S,L,prm,st,ev,sc)
torch.cuda.synchronize()
c=sc[:8].cpu().numpy().view(np.uint32)
print('list',c[0],'claimed',c[1])
need=sc[256:256+4*S].cpu().numpy().view(np.uint32)
print('need frac',need.mean())
fl=sc[256+4*S+4*S:256+8*S+64*S].cpu().numpy().reshape(S,64)[:,:41]
print('unchanged item frac',(fl&1==0).mean())
e=ev.cpu().numpy()
print('changes',(e[:,1]>=0).mean())
