import torch
torch.manual_seed(0)
x = torch.randn(64, 128256, device="cuda")
M = x.max(1, keepdim=True).values
n = (x > M - 12 * 0.2).sum(1)
print("cands per row: min", int(n.min()), "mean", float(n.float().mean()), "max", int(n.max()))
c = x.view(64, -1, 8192) if 128256 % 8192 == 0 else None
xs = torch.nn.functional.pad(x, (0, 16 * 8192 - 128256), value=-1e30).view(64, 16, 8192)
cm = xs.max(2, keepdim=True).values
nc = (xs > cm - 2.4).sum(2)
print("per-chunk (chunk-max relative): max", int(nc.max()), "mean", float(nc.float().mean()))
w = torch.exp((x - M) / 0.2); tot = w.sum(1)
cw = (w * (x > M - 2.4)).sum(1)
print("cand mass frac min", float((cw / tot).min()))
