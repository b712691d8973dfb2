"""Diagnostic: per-quantity ulp differences of FusedAdam vs torch.optim.Adam after one step."""
import sys, os
sys.path[:0] = [os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "animating-gaussian-splats_amd")]
import numpy as np, torch, splat_adam
dev = torch.device("cuda:0")
g = torch.Generator().manual_seed(0)
P = 65539
x = torch.randn(P, 1, generator=g)
for steps in (1, 2, 6):
    pa, pb = torch.nn.Parameter(x.clone().to(dev)), torch.nn.Parameter(x.clone().to(dev))
    oa = torch.optim.Adam([{"params": [pa], "lr": 0.05}], lr=0.0, eps=1e-15)
    ob = splat_adam.FusedAdam([{"params": [pb], "lr": 0.05}], lr=0.0, eps=1e-15)
    gg = torch.Generator().manual_seed(1)
    for it in range(steps):
        gr = (0.01 * torch.randn(P, 1, generator=gg)).to(dev)
        pa.grad, pb.grad = gr.clone(), gr.clone()
        oa.step(); ob.step()
    def ulp(a, b):
        a = a.detach().cpu().numpy().view(np.int32).astype(np.int64); b = b.detach().cpu().numpy().view(np.int32).astype(np.int64)
        return np.abs(a - b)
    for nm, (a, b) in {"p": (pa, pb), "m": (oa.state[pa]["exp_avg"], ob.state[pb]["exp_avg"]),
                       "v": (oa.state[pa]["exp_avg_sq"], ob.state[pb]["exp_avg_sq"])}.items():
        u = ulp(a, b)
        print(steps, nm, "max ulp", u.max(), "n diff", (u > 0).sum(), "worst idx", u.argmax(), a.flatten()[u.argmax()].item(), b.flatten()[u.argmax()].item())
