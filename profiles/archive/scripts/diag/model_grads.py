"""Locate where a model's GPU gradients first diverge from a float64 CPU run (module-output grads)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

import torch

from tutorial_torch_distributed_data_parallel_amd.models.registry import build_model

name = sys.argv[1] if len(sys.argv) > 1 else "resnet50"
hw = int(sys.argv[2]) if len(sys.argv) > 2 else 64
n = int(sys.argv[3]) if len(sys.argv) > 3 else 8
train_first = len(sys.argv) > 4 and sys.argv[4] == "train"
torch.manual_seed(0)
mc = build_model(name).double()
mg = build_model(name)
mg.load_state_dict(mc.state_dict())
mg.cuda()
x = torch.randn(n, 3, hw, hw, dtype=torch.float64)
if train_first:
    with torch.no_grad():
        mc.train()(x)
        mg.train()(x.float().cuda())
mc.eval()
mg.eval()
outs = {}


def reg(model, tag):
    for mn, mod in model.named_modules():
        if mn.count(".") > 1 or mn == "":
            continue

        def hk(mod, inp, out, mn=mn):
            outs[(tag, mn, "fwd")] = out.detach().double().cpu()
            out.register_hook(lambda g, mn=mn: outs.__setitem__((tag, mn, "grad"),
                                                                 g.detach().double().cpu()))
        mod.register_forward_hook(hk)


reg(mc, "c")
reg(mg, "g")
yc = mc(x)
yg = mg(x.float().cuda())
yc.square().sum().backward()
yg.square().sum().backward()
names = [mn for (t, mn, k) in outs if t == "c" and k == "fwd"]
for mn in names:
    line = f"{mn:24s}"
    for k in ("fwd", "grad"):
        a, b = outs.get(("g", mn, k)), outs.get(("c", mn, k))
        if a is None or b is None:
            line += f" {k} -"
            continue
        e = ((a - b).abs().max() / (b.abs().max() + 1e-30)).item()
        line += f" {k} {e:.2e}"
    print(line, flush=True)
