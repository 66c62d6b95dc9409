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
