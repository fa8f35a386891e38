import sys, torch
sys.path.insert(0, '.'); sys.path.insert(0, 'deep-learning-for-surgical-video-analysis_amd')
sys.path.insert(0, 'tests')
import torch.nn.functional as F
from test_temporal_train_gpu import _labels, CW
from oracle import inputs as I, mamba as OM
from models import mstcn
from svk import ops
cuda = torch.device('cuda', 0)
st = torch.load('dbg/nan_state.pt', weights_only=True)
sd, masks = st['sd'], st['masks']
m = mstcn.CausalMambaModel(4, 10, 64, 256, 14, True)
m.load_state_dict(sd)
m = m.to(cuda).eval()
T = 500
x = I.lfb(T, 256, 24)[0].contiguous()
ref = OM.causal_mamba(x.t().unsqueeze(0), sd, 10)
for groups in (512, 1):
    ops.MAMBA_GROUPS = groups
    with torch.no_grad():
        out = m(x.t().unsqueeze(0).to(cuda))
    torch.cuda.synchronize()
    print('groups', groups, 'finite', torch.isfinite(out).all().item(), 'maxdiff', (out.cpu().double() - ref).abs().max().item())
# block-level: scan kernel alone vs oracle selective_scan on block inputs from oracle
sd64 = {k: v.double() for k, v in sd.items()}
h = x.double().unsqueeze(0) @ sd64["in_proj.weight"].t() + sd64["in_proj.bias"]
for l in range(10):
    p = f"blocks.{l}."
    xz = h @ sd64[p + "in_proj.weight"].t()
    xi, z = xz.chunk(2, dim=-1)
    di = xi.shape[-1]
    xc = F.silu(F.conv1d(xi.transpose(1, 2), sd64[p + "conv1d.weight"], sd64[p + "conv1d.bias"], padding=3, groups=di)[..., :T]).transpose(1, 2)
    xdbl = xc @ sd64[p + "x_proj.weight"].t()
    R = 4
    dt, Bm, Cm = torch.split(xdbl, [R, 64, 64], dim=-1)
    delta = F.softplus(dt @ sd64[p + "dt_proj.weight"].t() + sd64[p + "dt_proj.bias"])
    A = -torch.exp(sd64[p + "A_log"])
    y = OM.selective_scan(xc, delta, A, Bm, Cm, sd64[p + "D"], z)
    for seg in (None, T):
        yk = ops.mamba_scan(xc[0].float().to(cuda).contiguous(), xdbl[0].float().to(cuda).contiguous(),
                            z[0].float().to(cuda).contiguous(), sd[p + "dt_proj.weight"].to(cuda), sd[p + "dt_proj.bias"].to(cuda),
                            (-torch.exp(sd[p + "A_log"])).to(cuda), sd[p + "D"].to(cuda), 1, T, seg_len=seg)
        torch.cuda.synchronize()
        err = (yk.cpu().double() - y[0]).abs().max().item()
        print(l, 'seg', seg, 'scan err', err, 'ymax', y.abs().max().item(), 'delta max', delta.max().item(), 'min', delta.min().item(), flush=True)
    h = h + y @ sd64[p + "out_proj.weight"].t()
