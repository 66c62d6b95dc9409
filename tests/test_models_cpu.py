"""Model topologies: parameter counts / state_dict keys of the torchvision models (CPU)."""
import torch

from tutorial_torch_distributed_data_parallel_amd.models.registry import build_model, input_shape


def test_alexnet_matches_reference_topology():
    m = build_model("alexnet")
    # torchvision AlexNet with classifier[6] = Linear(4096, 10) (REF/data_and_toy_model.py:43-44)
    assert sum(p.numel() for p in m.parameters()) == 57_044_810
    keys = list(m.state_dict().keys())
    assert keys[:2] == ["features.0.weight", "features.0.bias"]
    assert "classifier.6.weight" in keys and m.classifier[6].weight.shape == (10, 4096)
    y = m.eval()(torch.randn(1, 3, 224, 224))
    assert y.shape == (1, 10)


def test_resnet50_topology():
    m = build_model("resnet50")
    assert sum(p.numel() for p in m.parameters()) == 23_528_522  # torchvision resnet50, 10 classes
    assert len(list(m.parameters())) == 161
    sd = m.state_dict()
    assert "layer1.0.downsample.0.weight" in sd and "layer4.2.bn3.running_var" in sd
    assert m.layer2[0].conv2.stride == (2, 2)  # v1.5: stride on the 3x3
    y = m(torch.randn(2, 3, 64, 64))
    assert y.shape == (2, 10)
    y.sum().backward()


def test_input_shapes():
    assert input_shape("toy_mlp") == (9216,)
    assert input_shape("resnet50", 224) == (3, 224, 224)


def test_bottleneck_shared_input_grad_cpu():
    """The forked block input (ops/_grad.py fork / SharedGrad): gradients of its consumers meet
    in one buffer; equal to the plain block's autograd sum (with and without downsample)."""
    import copy

    import torch

    from tutorial_torch_distributed_data_parallel_amd.models.resnet import Bottleneck
    from tutorial_torch_distributed_data_parallel_amd.nn import BatchNorm2d, Conv2d

    torch.manual_seed(0)
    for inp, planes, stride, has_ds in [(32, 8, 1, False), (16, 8, 2, True), (16, 8, 1, True)]:
        ds = torch.nn.Sequential(Conv2d(inp, planes * 4, 1, stride=stride, bias=False),
                                 BatchNorm2d(planes * 4)) if has_ds else None
        a = Bottleneck(inp, planes, stride, ds).double()
        b = copy.deepcopy(a)
        b._fused_join = False
        x = torch.randn(2, inp, 8, 8, dtype=torch.float64)
        xa, xb = x.clone().requires_grad_(), x.clone().requires_grad_()
        ya, yb = a(xa), b(xb)
        g = torch.randn_like(ya)
        ya.backward(g)
        yb.backward(g)
        torch.testing.assert_close(ya, yb)
        torch.testing.assert_close(xa.grad, xb.grad)
        for (n, p), (_, q) in zip(a.named_parameters(), b.named_parameters()):
            torch.testing.assert_close(p.grad, q.grad, msg=lambda m: f"{n}: {m}")


def test_conv_plan_db_geometries():
    """ops/plan_db.py: the GEMM geometries of a pass mirror ops/conv.py (one for forward /
    weight gradient / stride-1 input gradient, one per stride phase otherwise), and the shipped
    table parses."""
    import json

    from tutorial_torch_distributed_data_parallel_amd.ops import plan_db

    g = plan_db.conv_geoms("fwd", (128, 3, 224, 224), (64, 3, 7, 7), (2, 2), (3, 3))
    assert g == [[128, 4, 224, 224, 64, 7, 7, 112, 112, 2, 2, 3, 3]]
    ph = plan_db.conv_geoms("dgrad", (128, 256, 28, 28), (256, 256, 3, 3), (2, 2), (1, 1))
    # 3x3 stride 2: phases (a, b) with Rp x Sp taps 1x1, 1x2, 2x1, 2x2 -- all 14x14 dx pixels
    assert sorted((p[5], p[6]) for p in ph) == [(1, 1), (1, 2), (2, 1), (2, 2)]
    assert all(p[2] == 14 and p[3] == 14 and p[7] == 14 and p[8] == 14 for p in ph)
    with open(plan_db.DEFAULT_DB) as f:
        table = json.load(f)
    for e in table["plans"]:
        assert e["pass"] in ("fwd", "dgrad", "wgrad") and e["fn"] in (1, 2) and e["splits"] >= 1
        assert e["us"] < e["us_heuristic"]

    class Rec:
        def __init__(self):
            self.n = 0

        def conv_plan_db_put(self, mode, geom, fn, splits):
            assert len(geom) == 13
            self.n += 1
    assert plan_db.register(Rec(), table["plans"]) >= len(table["plans"])
