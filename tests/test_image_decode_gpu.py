"""GPU image path, device half (ops.image_decode, csrc/image_decode.hip) against its NumPy
specification (ops/image_reference.py) and against the reference decode (PIL): a fixture batch of
JPEGs (several sizes / subsamplings / restart markers / grayscale / DCT-downscaled), raw RGB and
PIL-fallback containers decoded in ONE launch, plus the model-level check that the fused ResNet-50's
top-1 is unchanged vs PIL-decoded input."""
import numpy as np
import pytest
import torch

from test_image_decode import FIXTURES, jpeg, photo

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _fixture_batch():
    from mlmicroservicetemplate_amd.plugins.builtin import decode_image, image_container

    conts, refs, datas = [], [], []
    for i, (w, h, kw) in enumerate(FIXTURES):
        data = jpeg(photo(w, h, seed=i), **dict(kw))
        conts.append(image_container(data, "image/jpeg"))
        refs.append(decode_image(data, "image/jpeg"))
        datas.append(data)
    rgb = photo(224, 224, seed=99)
    conts.append(image_container(rgb.tobytes(), "application/octet-stream"))
    refs.append(rgb)
    prog = jpeg(photo(300, 300, seed=5), quality=90, progressive=True)  # PIL fallback, wrapped raw
    conts.append(image_container(prog, "image/jpeg"))
    refs.append(decode_image(prog, "image/jpeg"))
    return np.stack(conts), refs


def test_image_decode_matches_spec_and_pil():
    from mlmicroservicetemplate_amd import ops
    from mlmicroservicetemplate_amd.ops import image_reference as R

    conts, refs = _fixture_batch()
    err = torch.full((len(conts),), 7, dtype=torch.int32, device=DEV)
    out = ops.image_decode(torch.from_numpy(conts).to(DEV), err=err).cpu().numpy()
    assert err.tolist() == [0] * len(conts)
    for i, c in enumerate(conts):
        spec = R.decode_container(c)
        d = np.abs(out[i].astype(int) - spec.astype(int))
        assert d.max() <= 2 and d.mean() < 0.01, (i, d.max(), d.mean())  # fp64 IDCT: rounding ties only
        p = np.abs(out[i].astype(int) - refs[i].astype(int))
        assert p.mean() <= 2.0, (i, p.mean())


def test_image_decode_bad_container_is_black_and_flagged():
    from mlmicroservicetemplate_amd import ops

    conts, _ = _fixture_batch()
    bad = conts[:2].copy()
    bad[1, :4] = 0  # wrong magic
    err = torch.full((2,), 7, dtype=torch.int32, device=DEV)
    out = ops.image_decode(torch.from_numpy(bad).to(DEV), err=err).cpu().numpy()
    assert err.tolist() == [0, 1] and out[1].max() == 0 and out[0].max() > 0


def test_resnet_top1_unchanged_vs_pil_decode():
    from mlmicroservicetemplate_amd import ops
    from mlmicroservicetemplate_amd.models.resnet import ResNet50Fused, init_resnet50

    conts, refs = _fixture_batch()
    model = ResNet50Fused(init_resnet50(0), DEV, max_batch=16)
    gpu_imgs = ops.image_decode(torch.from_numpy(conts).to(DEV))
    pil_imgs = torch.from_numpy(np.stack(refs)).to(DEV)
    lg = model(gpu_imgs).float()
    lp = model(pil_imgs).float()
    top2 = lp.topk(2, dim=-1).values
    sure = (top2[:, 0] - top2[:, 1]) / lp.abs().max() > 1e-2
    assert torch.equal(lg.argmax(-1)[sure], lp.argmax(-1)[sure])
