"""Implicit-GEMM NHWC convolution (csrc/kernels/conv.hip) with the fused bias /
residual / ReLU epilogue, the pad-8 stem normalisation and the NHWC max pool,
each vs a plain fp32 PyTorch reference; and the own-conv ResNet-50 against the
MIOpen path."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


def _rel(a, b):
    return ((a.float() - b.float()).norm() / (b.float().norm() + 1e-12)).item()


# (N, H, W, Cin, Cout, ks, stride, pad, residual, relu, cin_real)
CASES = [
    (2, 17, 19, 64, 64, 3, 1, 1, False, True, 64),      # layer1 3x3, ragged M
    (3, 23, 23, 8, 64, 7, 2, 3, False, True, 3),        # stem (3 channels padded to 8)
    (2, 14, 14, 256, 128, 1, 1, 0, False, True, 256),   # 1x1 reduce
    (2, 14, 14, 128, 512, 1, 1, 0, True, True, 128),    # 1x1 expand + residual join
    (2, 15, 15, 256, 512, 1, 2, 0, False, False, 256),  # downsample 1x1 / 2
    (4, 16, 16, 128, 128, 3, 2, 1, False, True, 128),   # strided 3x3
    (1, 7, 7, 512, 2048, 1, 1, 0, True, True, 512),     # layer4 tail
]


@pytest.mark.parametrize("case", CASES)
@pytest.mark.parametrize("tile", [None, 2])
def test_conv2d_nhwc(case, tile):
    from cluster_anywhere_amd.ops.vision import conv2d_nhwc, conv2d_nhwc_ref, conv_weight_nhwc

    N, H, W, cin, cout, ks, s, p, res, relu, creal = case
    if tile == 2 and cout % 128:
        pytest.skip("128x128 tile needs Cout % 128")
    torch.manual_seed(0)
    x = torch.randn(N, H, W, cin, device="cuda").bfloat16()
    if creal < cin:
        x[..., creal:] = 0
    w4 = (torch.randn(cout, creal, ks, ks, device="cuda") / (creal * ks * ks) ** 0.5).bfloat16()
    b = (0.1 * torch.randn(cout, device="cuda")).bfloat16()
    Ho = (H + 2 * p - ks) // s + 1
    Wo = (W + 2 * p - ks) // s + 1
    r = torch.randn(N, Ho, Wo, cout, device="cuda").bfloat16() if res else None
    w2d = conv_weight_nhwc(w4.float(), cin).bfloat16()
    y = conv2d_nhwc(x, w2d, b, ks, s, p, relu, r, tile=tile)
    ref = conv2d_nhwc_ref(x[..., :creal], w4, b, s, p, relu, r)
    assert y.shape == ref.shape
    assert _rel(y, ref) < 1e-2
    assert (y.float() - ref).abs().max().item() < 0.1


def test_normalize_pad8_and_maxpool():
    from cluster_anywhere_amd.ops.vision import IMAGENET_MEAN, IMAGENET_STD, maxpool3s2_nhwc, normalize_pad8

    torch.manual_seed(1)
    u8 = torch.randint(0, 256, (3, 37, 29, 3), dtype=torch.uint8, device="cuda")
    x8 = normalize_pad8(u8)
    m = torch.tensor(IMAGENET_MEAN, device="cuda")
    sd = torch.tensor(IMAGENET_STD, device="cuda")
    ref = (u8.float() / 255 - m) / sd
    assert x8.shape == (3, 37, 29, 8)
    assert (x8[..., :3].float() - ref).abs().max().item() < 3e-2
    assert x8[..., 3:].abs().max().item() == 0
    z = torch.randn(2, 15, 13, 64, device="cuda").bfloat16()
    y = maxpool3s2_nhwc(z)
    yr = F.max_pool2d(z.permute(0, 3, 1, 2).float(), 3, 2, 1).permute(0, 2, 3, 1)
    assert torch.equal(y.float(), yr)


def test_resnet50_own_conv_matches_miopen():
    from cluster_anywhere_amd.models.resnet import resnet

    torch.manual_seed(2)
    with torch.device("cuda"):
        net = resnet("resnet50").eval()
    own = net.fuse_for_inference(torch.bfloat16, "cuda", own_conv=True)
    lib = net.fuse_for_inference(torch.bfloat16, "cuda", own_conv=False)
    u8 = torch.randint(0, 256, (8, 96, 96, 3), dtype=torch.uint8, device="cuda")
    a = own.predict_uint8(u8).float()
    b = lib.predict_uint8(u8).float()
    assert _rel(a, b) < 5e-2
    assert (a.argmax(1) == b.argmax(1)).float().mean().item() >= 0.75


def _pairs_ref(img, mean, std):
    """fp32 reference of normalize_pairs: [N,H,W,3] uint8 -> [N,H+6,(W+6)/2,8]."""
    x = img.float() / 255.0
    x = (x - torch.tensor(mean, device=img.device)) / torch.tensor(std, device=img.device)
    x = F.pad(x, (0, 1, 3, 3, 3, 3))  # channel 3 = 0, 3-pixel border
    n, hp, wp, _ = x.shape
    return x.reshape(n, hp, wp // 2, 8)


@pytest.mark.parametrize("shape", [(2, 224, 224), (3, 30, 42)])
def test_normalize_pairs(shape):
    from cluster_anywhere_amd.ops.vision import IMAGENET_MEAN, IMAGENET_STD, normalize_pairs

    n, h, w = shape
    img = torch.randint(0, 256, (n, h, w, 3), dtype=torch.uint8, device="cuda")
    out = normalize_pairs(img)
    ref = _pairs_ref(img, IMAGENET_MEAN, IMAGENET_STD)
    assert out.shape == ref.shape
    torch.testing.assert_close(out.float(), ref, rtol=1e-2, atol=1e-2)


@pytest.mark.parametrize("hw", [224, 64])
def test_pixel_pair_stem_matches_fp32_conv(hw):
    """The 7x7 / stride 2 / pad 3 stem as a 7x4 conv, stride (2, 1), over pixel pairs
    (conv_weight_pairs + normalize_pairs + conv2d_nhwc_ex) vs the fp32 reference conv
    of the real 3-channel input."""
    from cluster_anywhere_amd.ops.vision import (IMAGENET_MEAN, IMAGENET_STD, conv2d_nhwc_ex, conv2d_nhwc_ref,
                                                 conv_weight_pairs, normalize_pairs)

    torch.manual_seed(0)
    n = 2
    img = torch.randint(0, 256, (n, hw, hw, 3), dtype=torch.uint8, device="cuda")
    w4 = (torch.randn(64, 3, 7, 7, device="cuda") / 147 ** 0.5).bfloat16()
    b = (torch.randn(64, device="cuda") * 0.1).bfloat16()
    y = conv2d_nhwc_ex(normalize_pairs(img), conv_weight_pairs(w4.float()).bfloat16(), b, 7, 4, 2, 1, 0, 0, True)
    x = img.float() / 255.0
    x = ((x - torch.tensor(IMAGENET_MEAN, device="cuda")) / torch.tensor(IMAGENET_STD, device="cuda"))
    ref = conv2d_nhwc_ref(x.bfloat16(), w4, b, 2, 3, True)
    assert y.shape == ref.shape == (n, hw // 2, hw // 2, 64)
    assert _rel(y, ref) < 1e-2


def test_resnet_pixel_pair_stem_matches_pad8_stem():
    """Whole own-kernel ResNet-50 with the pixel-pair stem vs the 8-channel stem."""
    from cluster_anywhere_amd.models.resnet import resnet

    torch.manual_seed(0)
    f = resnet("resnet50").eval().fuse_for_inference(torch.bfloat16, "cuda")
    if f.stem_pair is None:
        pytest.skip("pixel-pair stem disabled")
    img = torch.randint(0, 256, (4, 224, 224, 3), dtype=torch.uint8, device="cuda")
    a = f.predict_uint8(img).float()
    keep = f.stem_pair
    f.stem_pair = None
    b = f.predict_uint8(img).float()
    f.stem_pair = keep
    assert _rel(a, b) < 2e-2
