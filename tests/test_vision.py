"""ResNet family + vision kernels (Data GPU map_batches path). CPU tests check the
BN folding and the predictor; GPU tests compare the HIP kernels and the bf16
channels_last HIP-graph forward against plain fp32 PyTorch references."""
import numpy as np
import pytest
import torch

from cluster_anywhere_amd.models.resnet import ResNetPredictor, resnet
from cluster_anywhere_amd.ops.vision import add_relu_, image_normalize, image_normalize_ref


def test_resnet50_shape_params_flops():
    n = resnet("resnet50")
    assert sum(p.numel() for p in n.parameters()) == 25_557_032
    assert abs(n.flops_per_image(224) / 1e9 - 8.18) < 0.05
    x = torch.randn(2, 3, 64, 64)
    assert n.eval()(x).shape == (2, 1000)


def test_bn_folding_matches_reference():
    torch.manual_seed(0)
    n = resnet("resnet18").eval()
    # non-trivial running stats so the fold is exercised
    for m in n.modules():
        if isinstance(m, torch.nn.BatchNorm2d):
            m.running_mean.uniform_(-0.5, 0.5)
            m.running_var.uniform_(0.5, 2.0)
            m.weight.data.uniform_(0.5, 1.5)
            m.bias.data.uniform_(-0.2, 0.2)
    x = torch.randint(0, 256, (3, 64, 64, 3), dtype=torch.uint8)
    f = n.fuse_for_inference(torch.float32, "cpu")
    with torch.no_grad():
        ref = n(image_normalize_ref(x).contiguous())
        out = f.predict_uint8(x)
    torch.testing.assert_close(out, ref, rtol=1e-4, atol=1e-4)


@pytest.mark.parametrize("name", ["resnet18", "resnet50"])
def test_fused_random_matches_module_route(name):
    """FusedResNet.random (the GPU predictor's start-up path) builds the same fused
    network as resnet(name) + fuse_for_inference: conv shapes, strides, paddings,
    ReLU flags, shortcut placement, classifier shape, and weight scales of the same
    kaiming-normal init (the random streams differ)."""
    from cluster_anywhere_amd.models.resnet import FusedResNet

    torch.manual_seed(0)
    fr = FusedResNet.random(name, torch.float32, "cpu")
    ref = resnet(name).eval().fuse_for_inference(torch.float32, "cpu")

    def convs(f):
        out = [f.stem]
        for cs, down in f.blocks:
            out += cs + ([down] if down is not None else [])
        return out

    a, b = convs(fr), convs(ref)
    assert len(a) == len(b) and [d is None for _, d in fr.blocks] == [d is None for _, d in ref.blocks]
    for x, y in zip(a, b):
        assert (x.w.shape, x.b.shape, x.stride, x.pad, x.relu, x.ks) == (y.w.shape, y.b.shape, y.stride, y.pad, y.relu, y.ks)
        assert 0.85 < (x.w.float().std() / y.w.float().std()).item() < 1.15
        assert torch.count_nonzero(x.b) == 0
    assert fr.fc_w.shape == ref.fc_w.shape and fr.fc_b.shape == ref.fc_b.shape
    assert fr.fc_w.abs().max() <= 1.0 / fr.fc_w.shape[1] ** 0.5 + 1e-6
    x = torch.randint(0, 256, (2, 64, 64, 3), dtype=torch.uint8)
    assert fr.predict_uint8(x).shape == (2, 1000)


def test_predictor_cpu_batches():
    p = ResNetPredictor("resnet18", batch_size=4, hw=32, device="cpu")
    imgs = np.random.randint(0, 256, (10, 32, 32, 3), dtype=np.uint8)
    out = p(imgs)
    assert out.shape == (10,) and out.dtype == np.int64
    assert np.array_equal(out[:4], p(imgs[:4]))


C = pytest.mark.gpu


@C
@pytest.mark.parametrize("n", [1, 7, 64])
def test_image_normalize_gpu(n):
    x = torch.randint(0, 256, (n, 224, 224, 3), dtype=torch.uint8, device="cuda")
    out = image_normalize(x)
    ref = image_normalize_ref(x.cpu(), dtype=torch.float32)
    assert out.dtype == torch.bfloat16 and out.is_contiguous(memory_format=torch.channels_last)
    torch.testing.assert_close(out.float().cpu(), ref, rtol=8e-3, atol=8e-3)


@C
def test_image_normalize_tail_gpu():
    x = torch.randint(0, 256, (1, 5, 3, 3), dtype=torch.uint8, device="cuda")  # 45 bytes: tail only
    torch.testing.assert_close(image_normalize(x).float().cpu(), image_normalize_ref(x.cpu()), rtol=8e-3, atol=8e-3)


@C
def test_add_relu_gpu():
    y = torch.randn(4, 256, 14, 14, device="cuda").to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    r = torch.randn_like(y)
    ref = torch.relu(y.float() + r.float())
    add_relu_(y, r)
    torch.testing.assert_close(y.float(), ref, rtol=1e-2, atol=1e-2)


@C
def test_fused_resnet50_gpu_matches_fp32():
    torch.manual_seed(0)
    n = resnet("resnet50").eval()
    x = torch.randint(0, 256, (8, 224, 224, 3), dtype=torch.uint8)
    with torch.no_grad():
        ref = n(image_normalize_ref(x).contiguous())
    f = n.fuse_for_inference(torch.bfloat16, "cuda")
    out = f.predict_uint8(x.cuda()).float().cpu()
    # bf16 through 53 layers: compare relative to the logit scale
    err = (out - ref).abs().max() / ref.abs().max()
    assert err < 0.05, float(err)


@C
def test_fused_resnet_own_classifier_gemm():
    """At batch 256 the own-kernel forward runs the classifier on the MFMA GEMM with
    the padded weight: logits match the hipBLASLt F.linear of the same features."""
    torch.manual_seed(0)
    f = resnet("resnet50").eval().fuse_for_inference(torch.bfloat16, "cuda")
    if not f.own:
        pytest.skip("own-kernel path disabled")
    assert f.fc_wp is not None and f.fc_wp.shape[0] == 1024
    x = torch.randint(0, 256, (256, 64, 64, 3), dtype=torch.uint8, device="cuda")
    out = f.predict_uint8(x)
    assert out.shape == (256, 1000)
    feats = torch.randn(256, 2048, device="cuda").to(torch.bfloat16)
    from cluster_anywhere_amd.ops.gemm import linear_nt

    mine = linear_nt(feats, f.fc_wp, f.fc_bp)
    ref = feats.float() @ f.fc_w.float().t() + f.fc_b.float()
    torch.testing.assert_close(mine[:, :1000].float(), ref, rtol=2e-2, atol=2e-2)
    assert torch.isneginf(mine[:, 1000:].float()).all()
    assert torch.equal(out.argmax(1), out.float().argmax(1))


@C
def test_predictor_hip_graph_matches_eager():
    imgs = np.random.randint(0, 256, (300, 224, 224, 3), dtype=np.uint8)
    g = ResNetPredictor("resnet50", batch_size=128, use_graph=True, lazy_capture=False)
    lz = ResNetPredictor("resnet50", batch_size=128, use_graph=True, lazy_capture=True)
    e = ResNetPredictor("resnet50", batch_size=128, use_graph=False)
    assert g.graph is not None and lz.graph is None
    a, b = g(imgs), e(imgs)
    first = lz(imgs)  # lazy: the first call runs eagerly
    assert lz.graph is None
    second = lz(imgs)  # captured at the start of this call, then replayed per chunk
    assert lz.graph is not None
    assert a.shape == (300,)
    assert (a == b).mean() > 0.98 and (first == b).mean() > 0.98 and (second == b).mean() > 0.98


@C
@pytest.mark.parametrize("res,relu", [(False, True), (False, False), (True, True)])
def test_bias_act_gpu(res, relu):
    from cluster_anywhere_amd.ops.vision import bias_act_

    y = torch.randn(3, 64, 7, 9, device="cuda").to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    b = torch.randn(64, device="cuda").to(torch.bfloat16)
    r = torch.randn_like(y) if res else None
    ref = y.float() + b.float().view(1, -1, 1, 1) + (r.float() if res else 0)
    ref = ref.relu() if relu else ref
    bias_act_(y, b, r, relu)
    torch.testing.assert_close(y.float(), ref, rtol=1e-2, atol=1e-2)


def test_pixel_pair_stem_math_cpu():
    """The pixel-pair rewrite of the stem (CPU, fp32, torch conv): a 7x4 conv with
    stride (2, 1) over [N, H+6, (W+6)/2, 8] virtual pixels with conv_weight_pairs
    weights equals the 7x7 / stride-2 / pad-3 conv of the 3-channel image."""
    import torch.nn.functional as F

    from cluster_anywhere_amd.ops.vision import conv_weight_pairs

    torch.manual_seed(0)
    x = torch.randn(2, 3, 30, 42)
    w = torch.randn(16, 3, 7, 7)
    ref = F.conv2d(x, w, None, 2, 3)
    xp = F.pad(x.permute(0, 2, 3, 1), (0, 1, 3, 3, 3, 3))  # [N, H+6, W+6, 4]
    n, hp, wp, _ = xp.shape
    xv = xp.reshape(n, hp, wp // 2, 8).permute(0, 3, 1, 2)  # [N, 8, H+6, (W+6)/2]
    wv = conv_weight_pairs(w).reshape(16, 7, 4, 8).permute(0, 3, 1, 2)  # [Cout, 8, 7, 4]
    out = F.conv2d(xv, wv, None, (2, 1), 0)
    assert out.shape == ref.shape
    torch.testing.assert_close(out, ref, rtol=1e-4, atol=1e-4)
