"""Backward of one ResNet block on GPU vs float64 CPU with identical inputs / upstream grads."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

import torch

from tutorial_torch_distributed_data_parallel_amd.models.registry import build_model

torch.manual_seed(0)
mc = build_model("resnet50").double()
mg = build_model("resnet50")
mg.load_state_dict(mc.state_dict())
mg.cuda()
x = torch.randn(8, 3, 64, 64, dtype=torch.float64)
with torch.no_grad():
    mc.train()(x)
    mg.train()(x.float().cuda())
mc.eval()
mg.eval()
cap = {}
h = mc.layer3[5].register_forward_hook(lambda m, i, o: cap.__setitem__("in", i[0].detach()))
mc(x)
h.remove()
xin = cap["in"]
torch.manual_seed(1)
up = torch.randn(8, 1024, 4, 4, dtype=torch.float64)
for blk_name in ("layer3.5", "layer3.4", "layer2.1", "layer4.1"):
    parts = blk_name.split(".")
    bc = getattr(mc, parts[0])[int(parts[1])]
    bg = getattr(mg, parts[0])[int(parts[1])]
    cin = bc.conv1.in_channels
    hw = {"layer2": 8, "layer3": 4, "layer4": 2}[parts[0]]
    torch.manual_seed(2)
    xi = torch.randn(8, cin, hw, hw, dtype=torch.float64).abs() if blk_name != "layer3.5" else xin
    outs = {}

    def reg(b, tag):
        hs = []
        for mn, mod in b.named_children():
            def hk(mod, inp, out, mn=mn):
                out.register_hook(lambda g, mn=mn: outs.__setitem__((tag, mn),
                                                                     g.detach().double().cpu()))
            hs.append(mod.register_forward_hook(hk))
        return hs
    hs = reg(bc, "c") + reg(bg, "g")
    a = xi.clone().requires_grad_()
    b = xi.float().cuda().requires_grad_()
    yc = bc(a)
    yg = bg(b)
    upc = torch.randn_like(yc)
    yc.backward(upc)
    yg.backward(upc.float().cuda())
    for hh in hs:
        hh.remove()
    print(blk_name, "fwd", ((yg.double().cpu() - yc).abs().max() / yc.abs().max()).item())
    mc_, mg_ = (yc > 0), (yg.double().cpu() > 0)
    print("  mask disagreements", (mc_ != mg_).sum().item(), "of", yc.numel(),
          "zeros cpu", (yc == 0).sum().item(), "zeros gpu", (yg == 0).sum().item())
    ta = torch.randn(8, 2048, 2, 2, device="cuda")
    tb = torch.randn(8, 2048, 2, 2, device="cuda")
    from tutorial_torch_distributed_data_parallel_amd import ops
    ta.requires_grad_(); tb.requires_grad_()
    ty = ops.add_relu(ta, tb)
    tdy = torch.randn_like(ty)
    ty.backward(tdy)
    print("  add_relu check", (ty - torch.relu(ta + tb)).abs().max().item(),
          (ta.grad - tdy * ((ta + tb) > 0)).abs().max().item(),
          (tb.grad - tdy * ((ta + tb) > 0)).abs().max().item())
    for (tag, mn) in sorted(outs):
        if tag != "c":
            continue
        gc, gg = outs[("c", mn)], outs[("g", mn)]
        print(f"  {mn:12s} grad {((gg - gc).abs().max() / gc.abs().max()).item():.2e}")
    print("  input grad", ((b.grad.double().cpu() - a.grad).abs().max() / a.grad.abs().max()).item(),
          flush=True)
