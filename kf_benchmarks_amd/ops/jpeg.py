"""Device JPEG reconstruction for the train input pipeline (csrc/jpeg.hip).

The host threads of the native image pipeline only entropy-decode each
JPEG and ship the quantized coefficient blocks of its training crop
(``runtime.ImagePipe.run_coef``); :func:`decode` turns a batch of those into
the uint8 [n, H, W, 3] resized crops on the GPU - inverse DCT, chroma
upsampling, colour conversion and bilinear resize, bit-exact with a full
libjpeg-turbo decode followed by the host pipeline's resize - ready for
``nn.augment_u8``.  CPU tensors take the host reference of the same code
(csrc/jpeg_recon.h through the runtime library).

Reference: tf.image.decode_jpeg + crop + resize, tcb/preprocessing.py:192-265.
"""

from __future__ import annotations

import ctypes

import torch

from . import _native as N

N.register_optional("kfb_jpeg_desc_bytes", [], N.c_int)
N.register_optional("kfb_jpeg_decode", [N.P, N.I, N.P, N.L, N.P, N.P, N.P, N.I, N.I, N.P, N.P])


def decode(descs: torch.Tensor, blocks: torch.Tensor, host_images, n: int, height: int,
           width: int, crop_pixels: int = -1) -> torch.Tensor:
    """descs: uint8 [n * desc_bytes]; blocks: int16 [nblocks, 64];
    host_images: uint8 [n, H, W, 3] or None (images the host decoded
    itself) -> uint8 [n, height, width, 3] on the tensors' device."""
    if descs.device.type != "cuda":
        from .. import runtime
        out = torch.empty((n, height, width, 3), dtype=torch.uint8)
        runtime.jpeg_reconstruct(descs.numpy(), n, blocks.numpy(),
                                 None if host_images is None else host_images.numpy(),
                                 height, width, out.numpy())
        return out
    if blocks.dtype != torch.int16 or (blocks.numel() and blocks.shape[-1] != 64):
        raise ValueError("blocks must be int16 [nblocks, 64]")
    if descs.numel() != n * N.query("kfb_jpeg_desc_bytes"):
        raise ValueError("descriptor buffer does not match the batch size")
    nblocks = blocks.numel() // 64
    planes = torch.empty((max(nblocks, 1) * 64,), dtype=torch.uint8, device=descs.device)
    out = torch.empty((n, height, width, 3), dtype=torch.uint8, device=descs.device)
    # crop_pixels (kfbrt_imgpipe_run_coef's third count): each crop is rebuilt
    # once into this scratch, then resized; < 0: per output pixel
    crop = (torch.empty((max(crop_pixels, 1) * 3,), dtype=torch.uint8, device=descs.device)
            if crop_pixels >= 0 else None)
    N.call("kfb_jpeg_decode", descs.data_ptr(), n, blocks.data_ptr() if nblocks else None,
           nblocks, planes.data_ptr(), None if crop is None else crop.data_ptr(),
           None if host_images is None else host_images.contiguous().data_ptr(),
           height, width, out.data_ptr(), N.stream(descs.device))
    return out
