import torch, sys
sys.path.insert(0, '.')
from mlmicroservicetemplate_amd import ops
import torch.nn.functional as F
DEV='cuda:0'
B,H,W,cin,cout=2,56,56,64,64
g=torch.Generator().manual_seed(1)
x=torch.randn(B,H,W,cin,generator=g).to(DEV).to(torch.bfloat16)
w=(torch.randn(cout,cin,3,3,generator=g)/(3*cin**0.5)).to(DEV).to(torch.bfloat16)
bias=(torch.randn(cout,generator=g)*0.1).to(DEV)
ref=F.conv2d(x.permute(0,3,1,2).float(), w.float(), padding=1)+bias.view(1,-1,1,1)
ref=torch.relu(ref).permute(0,2,3,1)
ws=torch.zeros(4*B*H*W*cout, device=DEV)
for sk in (1,2,2):
    out=torch.full((B,H,W,cout), 7.0, device=DEV, dtype=torch.bfloat16)
    ops.conv3x3_halo(x, ops.pack_conv_weight(w), bias, act=ops.ACT_RELU, variant=0, splitk=sk, workspace=ws, out=out)
    torch.cuda.synchronize()
    o=out.float()
    print(sk, 'untouched', (o==7.0).float().mean().item(), 'max', o.abs().max().item(), 'ref', ref.abs().max().item(),
          'err', ((o-ref).abs().max()/ref.abs().max()).item(), 'ws nonzero', (ws!=0).float().mean().item(), flush=True)
    s0=ws[:B*H*W*cout].view(B,H,W,cout); s1=ws[B*H*W*cout:2*B*H*W*cout].view(B,H,W,cout)
    pre=(F.conv2d(x.permute(0,3,1,2).float(), w.float(), padding=1)).permute(0,2,3,1)
    print('  slab sum vs conv', ((s0+s1-pre).abs().max()/pre.abs().max()).item(), 's0 max', s0.abs().max().item(), flush=True)
xs = x.permute(0,3,1,2).float(); wf = w.float()
p0 = F.conv2d(xs[:, :32], wf[:, :32], padding=1).permute(0,2,3,1)
p1 = F.conv2d(xs[:, 32:], wf[:, 32:], padding=1).permute(0,2,3,1)
def e(a, b): return round(((a-b).abs().max()/b.abs().max()).item(), 4)
print('s0~p0', e(s0,p0), 's0~p1', e(s0,p1), 's1~p0', e(s1,p0), 's1~p1', e(s1,p1), flush=True)
# per-tile check: which rows of s0 are right
rowerr = (s0-p0).abs().amax(dim=-1).reshape(-1)
bad = (rowerr > 0.05*p0.abs().max()).nonzero().flatten()
print('bad rows s0', bad.numel(), bad[:20].tolist(), flush=True)
colerr = (s0-p0).abs().reshape(-1, 64).amax(dim=0)
print('col err s0', [round(v,2) for v in colerr.tolist()], flush=True)
