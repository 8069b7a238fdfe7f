"""GPU image path, host half (frontend/csrc/jpeg_coefs.h) + its NumPy specification
(ops/image_reference.py) against the reference decode (plugins.builtin.decode_image = PIL /
libjpeg-turbo + Pillow bilinear, the reference contract of an uploaded image FILE,
reference src/model/model.py:16-23).  CPU only: the kernels are checked against the same
specification on the GPU in tests/test_image_decode_gpu.py.

Fixtures are synthetic (no network): smooth gradients + texture + mild noise, encoded by PIL at
several sizes, qualities, chroma subsamplings (4:2:0 / 4:2:2 / 4:4:4 / grayscale) and with restart
markers -- JPEG parameters a camera or browser would produce."""
import io

import numpy as np
import pytest
from PIL import Image

from mlmicroservicetemplate_amd.frontend.native import load_extension
from mlmicroservicetemplate_amd.ops import image_reference as R
from mlmicroservicetemplate_amd.plugins.builtin import decode_image, image_container


def photo(w, h, seed=0, noise=3.0):
    rng = np.random.default_rng(seed)
    x = np.linspace(0, 1, w)[None, :, None]
    y = np.linspace(0, 1, h)[:, None, None]
    base = rng.random((1, 1, 3)) * 150 + 40 * np.sin(6 * x + rng.random() * 3) * np.cos(4 * y) + 25 * np.sin(
        18 * x * y + rng.random((1, 1, 3)))
    img = base + rng.normal(0, noise, (h, w, 3)) + 60 * x
    return np.clip(img, 0, 255).astype(np.uint8)


def jpeg(img, **kw):
    b = io.BytesIO()
    mode = kw.pop("mode", None)
    im = Image.fromarray(img)
    if mode:
        im = im.convert(mode)
    im.save(b, "JPEG", **kw)
    return b.getvalue()


FIXTURES = [  # (w, h, save kwargs)
    (224, 224, dict(quality=90, subsampling=2)),
    (256, 256, dict(quality=90, subsampling=2)),
    (320, 240, dict(quality=85, subsampling=2)),
    (300, 260, dict(quality=88, subsampling=1)),
    (256, 300, dict(quality=80, subsampling=0)),
    (240, 320, dict(quality=92, subsampling=2, restart_marker_blocks=3)),
    (280, 280, dict(quality=90, mode="L")),
    (231, 229, dict(quality=75, subsampling=2)),  # not a multiple of the MCU
    (640, 480, dict(quality=85, subsampling=2)),  # PIL draft: DCT-domain 1/2
    (1024, 768, dict(quality=80, subsampling=2)),  # 1/2 (768 // 256 = 3)
]


@pytest.mark.parametrize("i", range(len(FIXTURES)))
def test_container_decode_matches_pil(i):
    w, h, kw = FIXTURES[i]
    data = jpeg(photo(w, h, seed=i), **dict(kw))
    c = load_extension().jpeg_container(data)
    assert isinstance(c, bytes), c
    assert len(c) == R.CONTAINER_BYTES
    hdr = R.parse_header(c)
    assert hdr["kind"] == 1 and not hdr["coarser"], hdr
    got = R.decode_container(c)
    ref = decode_image(data, "image/jpeg")
    d = np.abs(got.astype(int) - ref.astype(int))
    # full-scale decodes track libjpeg-turbo's integer IDCT to ~0.05 LSB; the DCT-downscaled ones
    # (reduced IDCT) within the 2-LSB bar
    assert d.mean() <= (0.1 if hdr["s"] == 8 else 2.0), (hdr, d.mean(), d.max())
    assert np.percentile(d, 99) <= (1 if hdr["s"] == 8 else 8)


def test_raw_and_fallbacks():
    ext = load_extension()
    rgb = photo(224, 224, seed=9)
    raw = image_container(rgb.tobytes(), "application/octet-stream")
    assert raw.dtype == np.uint8 and raw.size == R.CONTAINER_BYTES
    assert R.parse_header(raw)["kind"] == 0 and np.array_equal(R.decode_container(raw), rgb)
    prog = jpeg(photo(256, 256), quality=90, progressive=True)
    assert isinstance(ext.jpeg_container(prog), str)  # refused: progressive
    c = image_container(prog, "image/jpeg")  # -> PIL decode, wrapped raw
    assert R.parse_header(c)["kind"] == 0
    assert np.array_equal(R.decode_container(c), decode_image(prog, "image/jpeg"))
    png = io.BytesIO()
    Image.fromarray(rgb).save(png, "PNG")
    assert R.parse_header(image_container(png.getvalue(), "image/png"))["kind"] == 0


def test_corrupt_and_truncated_jpegs_never_crash():
    ext = load_extension()
    data = jpeg(photo(256, 256), quality=90, subsampling=2)
    rng = np.random.default_rng(0)
    for cut in (3, 20, len(data) // 3, len(data) - 10):
        r = ext.jpeg_container(data[:cut])
        assert isinstance(r, (bytes, str))
    for _ in range(50):
        b = bytearray(data)
        for j in rng.integers(2, len(b), 8):
            b[j] = int(rng.integers(0, 256))
        r = ext.jpeg_container(bytes(b))
        if isinstance(r, bytes):  # still parses: the container must be self-consistent
            hdr = R.parse_header(r)
            assert hdr["kind"] == 1 and hdr["nblocks"] * 4 <= R.PAYLOAD


def test_large_image_goes_coarser_but_fits():
    """A 1280 x 960 JPEG: its coefficients do not fit at PIL's scale, so the
    container holds a coarser DCT-domain downscale (flagged); a 12-MP image does not fit at all and
    takes the PIL path (image_container wraps PIL's decode)."""
    ext = load_extension()
    huge = jpeg(photo(4000, 3000, noise=2.0), quality=80, subsampling=2)
    assert isinstance(ext.jpeg_container(huge), str)
    assert R.parse_header(image_container(huge, "image/jpeg"))["kind"] == 0
    data = jpeg(photo(1280, 960, noise=3.0), quality=85, subsampling=2)
    c = ext.jpeg_container(data)
    assert isinstance(c, bytes), c
    hdr = R.parse_header(c)
    assert hdr["s"] < 8 and hdr["coarser"]
    out = R.decode_container(c)
    assert out.shape == (224, 224, 3)
    ref = decode_image(data, "image/jpeg")
    assert np.abs(out.astype(int) - ref.astype(int)).mean() < 8.0


def test_truncated_jpeg_is_refused_like_pil():
    """A JPEG cut inside its entropy-coded scan: the C++ decoder reports the overrun (it used to
    feed zero bits and return a grey-tailed container), so the upload takes the PIL path, which
    raises -- the same error the reference's PIL decode gives (no 200 with a made-up image)."""
    ext = load_extension()
    data = jpeg(photo(256, 256), quality=90, subsampling=2)
    for cut in (len(data) // 2, len(data) - 200):
        r = ext.jpeg_container(data[:cut])
        assert isinstance(r, str) and "truncated" in r, r
        with pytest.raises(Exception):
            decode_image(data[:cut], "image/jpeg")
        with pytest.raises(Exception):
            image_container(data[:cut], "image/jpeg")
    # restart markers: a cut in a later interval is caught at the next interval boundary / the end
    rst = jpeg(photo(256, 256, seed=4), quality=90, subsampling=2, restart_marker_blocks=4)
    r = ext.jpeg_container(rst[: len(rst) // 2])
    assert isinstance(r, str) and "truncated" in r, r
    # the untruncated files still decode
    assert isinstance(ext.jpeg_container(data), bytes) and isinstance(ext.jpeg_container(rst), bytes)


def test_extreme_aspect_ratio_takes_pil_path():
    """Resized width beyond the container header's 16-bit field (aspect > 256:1): refused by the
    C++ decoder (no uint16 wrap / zero width), decoded by PIL instead."""
    ext = load_extension()
    data = jpeg(photo(4096, 8, noise=1.0), quality=90)
    r = ext.jpeg_container(data)
    assert isinstance(r, str), "an aspect ratio of 512:1 must not produce a container"
    c = image_container(data, "image/jpeg")
    assert R.parse_header(c)["kind"] == 0
