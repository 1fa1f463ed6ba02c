"""JPEG reconstruction from coefficient blocks (csrc/jpeg_recon.h, run on the
GPU by csrc/jpeg.hip): the host threads only entropy-decode and ship the
crop's quantized DCT blocks.

Oracle: PIL's decoder (libjpeg-turbo with its defaults: islow IDCT, fancy
upsampling - what TF's decode_jpeg runs for the reference,
tcb/preprocessing.py:192-265).  The whole-image reconstruction must match it
bit for bit for every chroma layout the path takes (4:4:4, 4:2:2, 4:2:0,
grayscale) at any size and quality; the batch pipeline's resized crops must
match the host pipeline's bilinear formula applied to PIL's decode of the
crop; on the GPU the kernels must match the host reference exactly."""

import io
import struct

import numpy as np
import pytest

from kf_benchmarks_amd import runtime
from kf_benchmarks_amd.data import test_data

PIL = pytest.importorskip("PIL.Image")

needs_coef = pytest.mark.skipif(not runtime.coef_pipeline_available(),
                                reason="libjpeg with jpeg_read_coefficients not loadable")


def _jpeg(h, w, sub=2, q=90, gray=False, seed=0):
    rng = np.random.default_rng(seed)
    base = rng.normal(128, 60, (h // 4 + 2, w // 4 + 2, 3)).clip(0, 255).astype(np.uint8)
    img = PIL.fromarray(base).resize((w, h), PIL.BILINEAR)
    img = PIL.fromarray((np.asarray(img) + rng.normal(0, 12, (h, w, 3))).clip(0, 255)
                        .astype(np.uint8))
    if gray:
        img = img.convert("L")
    b = io.BytesIO()
    kw = dict(quality=q) if gray else dict(quality=q, subsampling=sub)
    img.save(b, "JPEG", **kw)
    return b.getvalue()


def _pil(data):
    return np.asarray(PIL.open(io.BytesIO(data)).convert("RGB"))


@needs_coef
@pytest.mark.parametrize("h,w", [(37, 53), (64, 64), (301, 451), (17, 9), (8, 200)])
@pytest.mark.parametrize("sub", [0, 1, 2, "gray"])
@pytest.mark.parametrize("q", [50, 90, 100])
def test_coefficient_reconstruction_matches_pil_bitwise(h, w, sub, q):
    data = _jpeg(h, w, 0 if sub == "gray" else sub, q, gray=sub == "gray", seed=h * w + q)
    got = runtime.jpeg_decode_coef(data)
    assert got is not None
    np.testing.assert_array_equal(got, _pil(data))


def _bilinear(src, oh, ow):
    """The host pipeline's resize (kfb_images.cpp resize_bilinear), float32."""
    sh, sw = src.shape[:2]
    fy, fx = np.float32(sh) / np.float32(oh), np.float32(sw) / np.float32(ow)
    out = np.empty((oh, ow, 3), np.uint8)
    for i in range(oh):
        sy = min(max((np.float32(i) + np.float32(0.5)) * fy - np.float32(0.5), np.float32(0)),
                 np.float32(sh - 1))
        y0 = int(sy)
        y1 = min(y0 + 1, sh - 1)
        ay = np.float32(sy - np.float32(y0))
        for j in range(ow):
            sx = min(max((np.float32(j) + np.float32(0.5)) * fx - np.float32(0.5),
                         np.float32(0)), np.float32(sw - 1))
            x0 = int(sx)
            x1 = min(x0 + 1, sw - 1)
            ax = np.float32(sx - np.float32(x0))
            for c in range(3):
                p00, p01 = np.float32(src[y0, x0, c]), np.float32(src[y0, x1, c])
                p10, p11 = np.float32(src[y1, x0, c]), np.float32(src[y1, x1, c])
                t = np.float32(p00 + ax * np.float32(p01 - p00))
                b = np.float32(p10 + ax * np.float32(p11 - p10))
                v = np.float32(t + ay * np.float32(b - t)) + np.float32(0.5)
                out[i, j, c] = int(min(np.float32(255), max(np.float32(0), v)))
    return out


class _Slot:
    def __init__(self, n, h, w, cap):
        import torch
        self.descs = torch.empty((n * runtime.jpeg_desc_bytes(),), dtype=torch.uint8)
        self.blocks = torch.empty((cap, 64), dtype=torch.int16)
        self.images = torch.zeros((n, h, w, 3), dtype=torch.uint8)
        self.params = torch.empty((n, 8), dtype=torch.float32)
        self.labels = torch.empty((n,), dtype=torch.int32)


def _records():
    recs, imgs = [], []
    for i, (h, w, sub) in enumerate([(120, 160, 2), (97, 75, 1), (64, 200, 0), (150, 150, 2),
                                     (33, 41, "gray"), (200, 90, 2)]):
        data = _jpeg(h, w, 0 if sub == "gray" else sub, 85, gray=sub == "gray", seed=i)
        recs.append(test_data.image_example("x%d.jpg" % i, data, i + 1, "n0", "x",
                                            [[0.1, 0.2, 0.9, 0.8]], h, w))
        imgs.append(_pil(data))
    return recs, imgs


def _crops(descs, n):
    words = struct.unpack("<%di" % (len(descs) // 4), bytes(descs))
    per = len(descs) // 4 // n
    return [(words[k * per], ) + tuple(words[k * per + 2:k * per + 6]) for k in range(n)]


@needs_coef
@pytest.mark.parametrize("cap", [1 << 16, 64])
def test_pipeline_crops_match_pil_reference(cap):
    """kfbrt_imgpipe_run_coef + the host reference of the device kernels:
    every resized crop equals the host bilinear of PIL's decode of that
    crop; with a tiny arena the images that do not fit are decoded on the
    host (MODE_HOST) and still come out."""
    recs, imgs = _records()
    n, oh, ow = len(recs), 40, 56
    slot = _Slot(n, oh, ow, cap)
    pipe = runtime.ImagePipe(3, oh, ow, True, False)
    try:
        nblocks, hosted, bad = pipe.run_coef(recs, np.arange(n, dtype=np.uint64) + 11, slot)
        nb2, _, _ = pipe.run_coef(recs, np.arange(n, dtype=np.uint64) + 11, _Slot(n, oh, ow, cap))
    finally:
        pipe.close()
    assert bad == 0 and nblocks == nb2 and 0 < nblocks <= cap
    assert (hosted == 0) == (cap == 1 << 16)
    assert slot.labels.tolist() == list(range(1, n + 1))
    out = np.empty((n, oh, ow, 3), np.uint8)
    runtime.jpeg_reconstruct(slot.descs.numpy(), n, slot.blocks[:nblocks].numpy(),
                             slot.images.numpy(), oh, ow, out)
    for k, (mode, cy, cx, ch, cw) in enumerate(_crops(slot.descs.numpy(), n)):
        if mode != 0:
            continue  # decoded on the host (libjpeg 9 path, its own crop draw)
        ref = _bilinear(imgs[k][cy:cy + ch, cx:cx + cw], oh, ow)
        np.testing.assert_array_equal(out[k], ref, err_msg="image %d" % k)
    prm = slot.params.numpy()
    assert set(np.unique(prm[:, 0])) <= {0.0, 1.0} and (prm[:, 6] == 1).all()


@needs_coef
@pytest.mark.gpu
def test_gpu_reconstruction_matches_host_reference(cuda):
    """csrc/jpeg.hip (IDCT kernel + reconstruct/resize kernel) against the
    host reference of the same code, bit for bit, including MODE_HOST
    images passed through."""
    import torch
    from kf_benchmarks_amd.ops import jpeg as J
    recs, _ = _records()
    recs = recs * 6  # 36 images
    n, oh, ow = len(recs), 64, 48
    for cap in (1 << 17, 600):
        slot = _Slot(n, oh, ow, cap)
        pipe = runtime.ImagePipe(4, oh, ow, False, False)
        try:
            nblocks, hosted, bad = pipe.run_coef(recs, np.arange(n, dtype=np.uint64), slot)
            crop_pixels = pipe.crop_pixels
        finally:
            pipe.close()
        assert bad == 0 and crop_pixels > 0
        ref = np.empty((n, oh, ow, 3), np.uint8)
        runtime.jpeg_reconstruct(slot.descs.numpy(), n, slot.blocks[:nblocks].numpy(),
                                 slot.images.numpy(), oh, ow, ref)
        # two-pass (each crop rebuilt once, then resized) and per-output-pixel
        for cp in (crop_pixels, -1):
            got = J.decode(slot.descs.to(cuda), slot.blocks[:nblocks].to(cuda),
                           slot.images.to(cuda) if hosted else None, n, oh, ow, cp)
            torch.cuda.synchronize()
            np.testing.assert_array_equal(got.cpu().numpy(), ref)
