"""Compare two lib_diff.py dumps: per tensor, the number of differing elements and the largest difference."""
import sys

import torch

a, b = (torch.load(f, weights_only=True) for f in sys.argv[1:3])
for k, (x, y) in enumerate(zip(a["imgs"], b["imgs"])):
    d = (x - y).abs()
    if d.max() > 0:
        print(f"img {k}: {(d > 0).sum().item()} differ, max {d.max().item():.3g}")
for k in a["grads"]:
    d = (a["grads"][k] - b["grads"][k]).abs()
    print(f"grad {k}: {(d > 0).sum().item()} of {d.numel()} differ, max {d.max().item():.3g} (scale {a['grads'][k].abs().max().item():.3g})")
