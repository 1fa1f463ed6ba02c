"""NHWC convolution autograd Function over the gfx950 implicit-GEMM kernels
(csrc/conv_igemm.hip).

forward : y  = igemm(x, W[Cout][KH*KW*Cin])
dgrad   : 1x1 stride 1  -> igemm(dY, W^T) (plain GEMM)
          1x1 stride s  -> dX = 0; igemm(dY, W^T) scattered to every s-th pixel
          general       -> transposed-gather igemm(dY, W permuted to [Cin][KH][KW][Cout])
wgrad   : split-M MFMA reduction into an fp32 [Cout][KH*KW*Cin] buffer, which
          is exactly the fp32 master weight layout.

Channel counts that are not multiples of 8 (the RGB stem, DenseNet growth
12) are zero-padded to the next multiple of 8 around the kernels.
"""

from __future__ import annotations

import os
import sys

import torch

from . import _native as N

_SIG = ([N.I, N.P, N.P, N.P] + [N.I] * 17 + [N.I, N.P, N.P, N.P, N.P, N.P, N.P]
        + [N.P, N.I] + [N.I, N.P]  # ... mcoef, bias, relu, algo, kshift
        + [N.P] * 9 + [N.c_float, N.c_float] + [N.P])  # BN finalize (BnFin), stream
N.register_optional("kfb_conv_igemm", _SIG)
N.register_optional("kfb_conv_igemm_fast", [N.I] * 4, N.c_int)
N.register_optional("kfb_conv_s3_applicable", [N.I] * 12, N.c_int)
N.register_optional("kfb_conv_s3_set_grid", [N.I], None)
N.register_optional("kfb_conv_s1_applicable", [N.I] * 12, N.c_int)
N.register_optional("kfb_conv_s1_set_grid", [N.I], None)
N.register_optional("kfb_conv_s1_dgrad_dual", [N.I, N.P, N.P, N.P] + [N.I] * 5 + [N.P] * 9)
N.register_optional("kfb_conv_s7_applicable", [N.I] * 12, N.c_int)
N.register_optional("kfb_set_deterministic", [N.I], None)

# igemm kernel choice (csrc/conv_igemm.hip): 1 = register-staged 128-tile
# igemm_k, 2 = LDS-DMA ring igemm_glds_k (FAST geometries only).
IG_CLASSIC, IG_GLDS, IG_CLASSIC_N64, IG_GLDS_N64, IG_ONEBUF, IG_ONEBUF_N64 = 1, 2, 3, 4, 5, 6
IG_TALL512, IG_TALL256, IG_SMALL, IG_GSHORT64, IG_GSHORT128 = 7, 8, 9, 10, 11
IG_GSHORT64_3, IG_GSHORT128_3 = 12, 13
# multi-tile workgroups (igemm_mt_k: the next tile's loads overlap this tile's
# output stores), forward-style epilogues only
IG_MULTI2, IG_MULTI4, IG_SMALL_MULTI4 = 14, 15, 16
# ... and the LDS-DMA 128x64 / 128x128 4-wave kernels with 2 tiles per workgroup
IG_GMULTI64, IG_GMULTI128 = 17, 18
# 8-wave LDS-DMA kernels with 128 x 64 wave tiles: 256 x 256 / 512 x 128 tiles
IG_GBIG256, IG_GBIG512 = 19, 20
IG_GENERIC = 21  # the generic (per-chunk division) loader, forced
# persistent 128 x 128 LDS-DMA tile, last partial round split along K (stream-K)
IG_SK128 = 22
# 256 x 256 LDS-DMA tile, 8-phase schedule with the two wave groups staggered
IG_G8P = 23
# register-staged 128x64 one- and two-stage kernels that load the dgrad-style
# epilogue operands (addend, mask, x_bn) before their K loop, behind the first
# K step's operand loads (offered with those operands; IG_ONEBUF_E = the
# 128x64 one-stage form too, 128x128 would spill)
IG_ONEBUF_E, IG_ONEBUF_N64_E, IG_CLASSIC_N64_E = 24, 25, 26
# 256x64 tile, four waves along M; only the weight tile goes through LDS, the
# pixel operand is loaded straight into MFMA B-fragment layout (igemm_db_k)
IG_DB = 27
# IG_GBIG256 / IG_GSHORT128 / IG_GSHORT64 on v_mfma_f32_32x32x16 (15% more
# sustained MFMA throughput than the 16x16x32 form, scripts/probes/mfma_rate.hip)
IG_GBIG256_32, IG_GSHORT128_32, IG_GSHORT64_32 = 28, 29, 30
# streaming 3x3 64-channel kernel (csrc/conv_stream.hip): persistent, weights
# resident in LDS, input read once through an LDS ring
IG_S3 = 31
# streaming 1x1 64 -> 256-channel kernel (csrc/conv_s1.hip): persistent,
# weights resident in LDS, every operand streamed through an LDS-DMA ring
IG_S1 = 32
# streaming stem conv over the pixel-pair view (csrc/conv_s7.hip): one image
# band per CU, input rows through an LDS ring, weights in VGPRs
IG_S7 = 33
# 224 x 256 tiles on the 8-wave LDS-DMA kernel (7 MFMA rows per wave): 224
# tiles instead of 196 for the 14x14 layers at batch 256 (M = 196 per image)
IG_GBIG224 = 34
# 448 x 128 tiles (waves 4 x 2 of 112 x 64) for the 128-channel layers
IG_GBIG448 = 35
IG_ALGOS = {"classic": IG_CLASSIC, "glds": IG_GLDS, "classic_n64": IG_CLASSIC_N64,
            "glds_n64": IG_GLDS_N64, "onebuf": IG_ONEBUF, "onebuf_n64": IG_ONEBUF_N64,
            "tall512": IG_TALL512, "tall256": IG_TALL256, "small": IG_SMALL,
            "gshort64": IG_GSHORT64, "gshort128": IG_GSHORT128, "gshort64_3": IG_GSHORT64_3,
            "gshort128_3": IG_GSHORT128_3, "multi2": IG_MULTI2, "multi4": IG_MULTI4,
            "small_multi4": IG_SMALL_MULTI4, "gmulti64": IG_GMULTI64,
            "gmulti128": IG_GMULTI128, "gbig256": IG_GBIG256, "gbig512": IG_GBIG512,
            "generic": IG_GENERIC, "sk128": IG_SK128, "g8p": IG_G8P, "onebuf_e": IG_ONEBUF_E,
            "onebuf_n64_e": IG_ONEBUF_N64_E, "classic_n64_e": IG_CLASSIC_N64_E, "db": IG_DB,
            "gbig256_32": IG_GBIG256_32, "gshort128_32": IG_GSHORT128_32,
            "gshort64_32": IG_GSHORT64_32, "s3": IG_S3, "s1": IG_S1,
            "s7": IG_S7, "gbig224": IG_GBIG224,
            "gbig448": IG_GBIG448}
_IG_FORCE = IG_ALGOS.get(os.environ.get("KFB_IGEMM_ALGO", ""))
_ig_tuned = {}
# Offered to the autotune only where they won (the lost forms stay
# selectable by name through KFB_IGEMM_ALGO, for the kernel tests):
#  * IG_SK128 (stream-K): slower than the one-tile kernels on every ResNet-50
#    bs256 geometry, neutral on the few-tile small-batch layers
#    (profiles/r7_stream_k.txt);
#  * IG_*_E (epilogue operands loaded before the K loop): 3 instead of 4
#    workgroups per CU lost 5-20% on every dgrad geometry
#    (profiles/r8_early_epilogue.txt);
#  * IG_DB (pixel operand straight into B fragments): 380-410 TF/s, 1.1-2x
#    slower than the chosen kernels (profiles/r8_direct_b.txt);
#  * IG_*_32 (32x32x16 MFMA forms): within -4..+1% (profiles/r8_mfma_forms.txt).
# largest K (= KH*KW*Cin) offered the multi-tile candidates (register-staged;
# the LDS-DMA form gets twice that)
_MULTI_K = 2304
# the streaming 3x3 kernels (IG_S3, the s3 weight gradient) off: the
# bitwise tape oracles run without them (tests/test_tape_gpu.py)
_NO_S3 = False
# the streaming 1x1 / stem kernels off (tests: their A/B against the
# one-tile kernels, e.g. tests/test_tape_gpu.py)
_NO_S1 = False
_NO_S7 = False
# The ReLU / bias backward of a conv without BN in the consuming conv's dgrad
# epilogue instead of its own pass: off (on VGG-16 it removes 1.05 ms/step of
# act_bwd_bias but the extra read of y slows the dgrad convs by 0.8 ms and the
# separate pass overlaps the weight-gradient side stream: 0.5 ms slower,
# profiles/r4_act_fuse_ab.txt); tests/test_conv_gpu.py switches it on
_ACT_FUSE = False
N.register_optional("kfb_conv_stats_spread", [], N.c_int)
N.register_optional("kfb_conv_wgrad", [N.I, N.P, N.P, N.P] + [N.I] * 12 + [N.I, N.I, N.P, N.L, N.P])
N.register_optional("kfb_conv_wgrad_splits", [N.I] * 8, N.c_int)

_WGRAD_TARGET_BLOCKS = int(os.environ.get("KFB_WGRAD_BLOCKS", "768"))


def supported(x, w, stride, pads) -> bool:
    return x.is_cuda and x.dtype in (torch.bfloat16, torch.float16) and x.dim() == 4


def _fuse_enabled():
    from .conv import FUSE_BN
    return FUSE_BN


def _pad8(n):
    return (n + 7) // 8 * 8


STATS_SPREAD = 32  # must match IG_SPREAD in csrc/conv_igemm.hip (checked at load)


class _StatsArena:
    """Per-step pool of zeroed fp32 partial-sum buffers: one memset per
    training step instead of one per BN (reset by Network.forward)."""

    def __init__(self):
        self.buf = {}
        self.off = {}
        self.need = {}

    def reset(self, device):
        key = str(torch.device(device))
        # high-water mark of the previous step (+25% headroom)
        need = self.need.get(key, 0)
        need = (need + need // 4 + 4095) // 4096 * 4096
        buf = self.buf.get(key)
        if buf is None or buf.numel() < need:
            self.buf[key] = buf = torch.zeros((max(need, 1 << 16),), dtype=torch.float32,
                                              device=device)
        elif buf.is_cuda:
            # the whole buffer (a few MB; native memset: part of a recorded
            # launch tape): a step of another network in this process, or a
            # tape's replays, may have used more of it than the last step
            N.zero_(buf)
        else:
            buf.zero_()
        self.off[key] = 0

    def snapshot(self):
        """The current buffers (a launch tape keeps them alive: its replays
        write them through raw pointers)."""
        return dict(self.buf)

    def forget_new(self, before):
        """Drop buffers allocated since ``before`` (a snapshot): ones made
        while a launch tape was recording live in the tape's private memory
        pool and must not outlive it."""
        for key, b in list(self.buf.items()):
            if before.get(key) is not b:
                del self.buf[key]
                self.off.pop(key, None)

    def take(self, n, device):
        key = str(torch.device(device))
        n = (n + 63) // 64 * 64
        buf = self.buf.get(key)
        off = self.off.get(key, 0)
        self.off[key] = off + n
        self.need[key] = max(self.need.get(key, 0), off + n)
        if buf is None or off + n > buf.numel():
            # grows at the next reset; this step falls back to a fresh buffer
            return torch.zeros((n,), dtype=torch.float32, device=device)
        return buf[off:off + n]


STATS_ARENA = _StatsArena()


_SPREAD_CHECKED = False


def stats_buffer(channels, device, shift=None):
    """Zeroed [2][STATS_SPREAD][C] fp32 buffer for fused BN partial sums.
    ``shift`` (fp32 [C], the consuming BN's stat_shift): the conv epilogue
    sums y - shift and (y - shift)^2, and the BN finalize undoes it; the
    buffer carries it (``_kfb_shift``) so producer and consumer agree.
    The zeroed 64 floats after it hold the arrival counter of the in-kernel
    BN finalize (``attach_bn_finalize``)."""
    global _SPREAD_CHECKED
    if not _SPREAD_CHECKED:
        lib_spread = N.query("kfb_conv_stats_spread")
        if lib_spread != STATS_SPREAD:
            raise N.NativeError("stats spread mismatch: library %d, Python %d"
                                % (lib_spread, STATS_SPREAD))
        _SPREAD_CHECKED = True
    full = STATS_ARENA.take(2 * STATS_SPREAD * channels + 64, device)
    buf = full[:2 * STATS_SPREAD * channels]
    buf._kfb_counter = full[2 * STATS_SPREAD * channels:]
    if shift is not None:
        buf._kfb_shift = shift
    return buf


# In-kernel BN finalize (attach_bn_finalize, attach_bn_grad_finalize):
# KFB_BN_FIN=1 in every igemm kernel, "persistent" (default) only in the
# persistent streaming kernels (forward statistics and the dgrad's backward
# partials), "grad" only the dgrad form there, 0 never.  Every workgroup of a kernel with the tail drains its stores
# before its arrival ticket; on the one-tile kernels (thousands of short
# workgroups) that drain costs more than the finalize launch it saves
# (ResNet-50 bs256: 19.64-19.70 vs 19.45-19.50 ms/step, gpurun_out/r9d),
# in a persistent kernel it is one drain per CU.
# Default "grad": ResNet-50 bs256 A/B (profiles/r10_bn_finalize_tails.txt):
# persistent 19.25-19.40, grad 18.84-19.02, off 18.87-18.88 ms/step - the
# forward tails cost more than the launches they replace (the last arriver's
# fold and parameter round trips are one serial post-step per kernel), the
# dgrad tails about break even and remove ~17 launches per step.
_BN_FIN_MODE = os.environ.get("KFB_BN_FIN", "grad")
_BN_FIN = _BN_FIN_MODE != "0"


def attach_bn_finalize(stats, gamma, beta, rm, rv, decay, eps, st, coef):
    """Asks the conv that fills ``stats`` to also run the consuming BN's
    finalize in its last workgroup (csrc/igemm_args.h BnFin): mean / invstd
    into ``st`` [2][C], scale / shift into ``coef`` [2][C], the running
    statistics and the statistics shift.  The BN forward then sees
    ``stats._kfb_finalized`` and skips its finalize launch."""
    if stats is None or not _BN_FIN or not stats.is_cuda:
        return
    stats._kfb_fin = (gamma, beta, rm, rv, float(decay), float(eps), st, coef)
    stats._kfb_finalized = False


def attach_bn_grad_finalize(parts, link, C, device):
    """Asks the dgrad that fills the BN backward partials ``parts`` (the
    last consumer of a BNLink) to also run the BN's backward finalize in
    its last workgroup (csrc/igemm_args.h BnGFin): dgamma / dbeta into the
    BN's gradient targets and the apply coefficients.  The BN backward then
    sees ``parts._kfb_gfinalized`` and only runs the apply pass."""
    if _BN_FIN_MODE not in ("persistent", "1", "grad") or link.gfin is None \
            or device.type != "cuda":
        return
    from .nn import _bn_grad_targets
    gamma, st, beta = link.gfin
    coef = torch.empty((3 * C,), dtype=torch.float32, device=device)
    targets = _bn_grad_targets(gamma, beta, C, device)
    direct, dgp, dbp, _ = targets
    parts._kfb_gfin = (parts._kfb_counter.data_ptr(), N.ptr(gamma), N.ptr(None), dgp, dbp,
                       coef[2 * C:].data_ptr(), st[1].data_ptr(), coef[:C].data_ptr(),
                       coef[C:2 * C].data_ptr(), 1.0 if direct else 0.0, 0.0)
    parts._kfb_gfin_out = (coef, targets)
    parts._kfb_gfinalized = False


def _fin_args(stats):
    fin = getattr(stats, "_kfb_fin", None) if stats is not None else None
    if fin is None:
        return (None,) * 9 + (0.0, 0.0)
    gamma, beta, rm, rv, decay, eps, st, coef = fin
    C = st.shape[-1]
    return (stats._kfb_counter.data_ptr(), N.ptr(gamma), N.ptr(beta), N.ptr(rm), N.ptr(rv),
            st[0].data_ptr(), st[1].data_ptr(), coef[:C].data_ptr(), coef[C:2 * C].data_ptr(),
            decay, eps)


def stats_shift(stats):
    """The statistics shift a stats buffer was filled with (None: none)."""
    return getattr(stats, "_kfb_shift", None) if stats is not None else None


def _igemm_call(algo, x, wmat, y, geo, stats=None, mask=None, xbn=None, mean=None, addend=None,
                mcoef=None, bias=None, relu=False):
    fin = (None,) * 9 + (0.0, 0.0)
    if (stats is not None and xbn is None and addend is None and geo[15] == 1
            and getattr(stats, "_kfb_fin", None) is not None
            and (_BN_FIN_MODE == "1" or (_BN_FIN_MODE != "grad" and algo in (IG_S3, IG_S1, IG_S7)))):
        fin = _fin_args(stats)
        stats._kfb_finalized = True
    elif (stats is not None and xbn is not None and geo[15] == 1 and algo in (IG_S3, IG_S1)
            and getattr(stats, "_kfb_gfin", None) is not None):
        # (the kfb_conv_igemm fin_* slots in their BnGFin meaning, in order:
        # counter, gamma, -, dgamma, dbeta, coefC, invstd, coefA, coefB,
        # accumulate, -; kernels without the tail launch the finalize after)
        fin = stats._kfb_gfin
        stats._kfb_gfinalized = True
    N.call("kfb_conv_igemm", N.dt(x), x.data_ptr(), wmat.data_ptr(), y.data_ptr(), *geo,
           N.ptr(stats), N.ptr(mask), N.ptr(xbn), N.ptr(mean), N.ptr(addend), N.ptr(mcoef),
           N.ptr(bias), int(relu), algo, N.ptr(stats_shift(stats)), *fin, N.stream(x.device))


# KFB_AUTOTUNE_LOG=1 prints every timed choice (tests/test_conv_gpu.py)
_TUNE_LOG = os.environ.get("KFB_AUTOTUNE_LOG", "0") == "1"
_ALGO_NAMES = {}


def _time_candidates(cands, run, rounds=2, reps=3, label=None, slack=0.0, cost=None):
    """The fastest candidate: each is warmed once, then timed ``reps``
    back-to-back calls per round over ``rounds`` interleaved rounds (min
    per candidate).  The device is synchronized first so no other stream's
    kernels (the weight-gradient side stream, the dgrad chain) share the
    chip while a candidate is timed - contended timings made the choice,
    and with it the step time, vary from run to run."""
    torch.cuda.synchronize()
    for c in cands:
        run(c)
    best_t = {c: float("inf") for c in cands}
    for _ in range(rounds):
        for c in cands:
            ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            ev0.record()
            for _ in range(reps):
                run(c)
            ev1.record()
            ev1.synchronize()
            best_t[c] = min(best_t[c], ev0.elapsed_time(ev1))
    best = min(best_t, key=best_t.get)
    if slack > 0 and cost is not None:
        # the cheapest candidate (e.g. fewest weight-gradient splits: fewer
        # slab bytes and reduce work beside the compute stream) among those
        # within ``slack`` of the fastest isolated time
        near = [c for c in cands if best_t[c] <= best_t[best] * (1.0 + slack)]
        best = min(near, key=lambda c: (cost(c), best_t[c]))
    if _TUNE_LOG and label is not None:
        if not _ALGO_NAMES:
            _ALGO_NAMES.update({v: k for k, v in IG_ALGOS.items()})
        ranked = sorted(best_t.items(), key=lambda kv: kv[1])
        print("[autotune] %s: %s" % (label, "  ".join(
            "%s %.1f" % (("s3w" if c >> 16 == 2 else "%s/%d" % (_WGRAD_NAMES[c >> 16], c & 0xFFFF))
                         if c >= (1 << 16)
                         else _ALGO_NAMES.get(c, c),
                         1e3 * t / reps) for c, t in ranked)),
            file=sys.stderr, flush=True)
    return best


def _igemm_algo(x, wmat, y, geo, fused=(None, None, None, None, None, None), bact=(None, False)):
    """Per-geometry kernel choice, timed once on the real operands with the
    real fused epilogue (the role cuDNN's algorithm autotune plays for the
    reference): all kernels but IG_SK128 run the same K order (stream-K adds
    fp32 partial sums of K ranges), so the choice changes the numerics by
    fp32 rounding at most.  ``fused`` = (stats, mask, xbn, mean, addend, mcoef); the
    timing runs write a scratch output and scratch statistics."""
    if _IG_FORCE is not None:
        return _IG_FORCE
    stats, mask, xbn, mean, addend, mcoef = fused
    # cached choice first: this runs on every conv call, and the candidate
    # list below costs a ctypes call (host time on the host-bound models)
    key = (str(x.device), x.dtype, stats is not None, mask is not None, xbn is not None,
           addend is not None, mcoef is not None, bact[0] is not None, int(bact[1])) + tuple(geo)
    best = _ig_tuned.get(key)
    if best is not None:
        return best
    C, KH, KW, ncol, trans = geo[3], geo[6], geo[7], geo[12], geo[17]
    fast = N.load().kfb_conv_igemm_fast(C, KH, KW, trans)
    # (IG_TALL512 is never the fastest on the ResNet-50 shapes: force-only)
    cands = (IG_CLASSIC, IG_GLDS, IG_ONEBUF, IG_TALL256) if fast else (IG_CLASSIC,)
    if fast:
        cands += (IG_SMALL, IG_GSHORT64, IG_GSHORT64_3)
        if ncol > 64:
            cands += (IG_GSHORT128, IG_GSHORT128_3)
    if fast and mask is None and xbn is None and addend is None \
            and KH * KW * C <= _MULTI_K and C % 64 == 0:
        # short-K layers: store-phase bound, the multi-tile overlap pays there
        cands += (IG_MULTI2, IG_MULTI4, IG_SMALL_MULTI4)
    if fast and KH * KW * C <= 2 * _MULTI_K and C % 64 == 0:
        cands += (IG_GMULTI64,) + ((IG_GMULTI128,) if ncol > 64 else ())
    if fast:
        # big tiles only where they give most CUs a workgroup: 196 256x256
        # tiles on 256 CUs (the 14x14 3x3 convs at batch 256) still beat 784
        # 128x128 tiles on 512 slots (71 vs 79 us, profiles/r7_stream_k.txt)
        M = geo[0] * geo[4] * geo[5]
        if ncol >= 256 and ((M + 255) // 256) * ((ncol + 255) // 256) >= 192:
            cands += (IG_GBIG256,) + ((IG_G8P,) if C % 64 == 0 else ())
            if ((M + 223) // 224) * ((ncol + 255) // 256) > \
                    ((M + 255) // 256) * ((ncol + 255) // 256):
                cands += (IG_GBIG224,)
        if 64 < ncol <= 256 and ((M + 511) // 512) * ((ncol + 127) // 128) >= 256:
            cands += (IG_GBIG512,)
        if 64 < ncol <= 256 and ((M + 447) // 448) * ((ncol + 127) // 128) >= 256:
            cands += (IG_GBIG448,)
    if fast and C % 64 != 0:
        # 8-channel geometry: the generic loader competes with the FAST ones
        cands += (IG_GENERIC,)
    if fast and not _NO_S3 and N.load().kfb_conv_s3_applicable(
            C, ncol, KH, KW, geo[8], geo[9], geo[10], geo[11], geo[1], geo[2], geo[4], geo[5]) \
            and geo[13] == geo[4] and geo[14] == geo[5] and geo[15] == 1 and geo[16] == ncol:
        cands += (IG_S3,)
    if fast and not _NO_S1 and mcoef is None and bact[0] is None and not (int(bact[1]) & 3) \
            and (mask is None or (xbn is not None and mask.dtype == torch.uint8)) \
            and N.load().kfb_conv_s1_applicable(
            C, ncol, KH, KW, geo[8], geo[9], geo[10], geo[11], geo[1], geo[2], geo[4], geo[5]) \
            and geo[13] == geo[4] and geo[14] == geo[5] and geo[15] == 1 and geo[16] == ncol:
        cands += (IG_S1,)
    if not _NO_S7 and xbn is None and addend is None and mask is None and bact[0] is None \
            and not (int(bact[1]) & 3) and not trans and N.load().kfb_conv_s7_applicable(
            C, ncol, KH, KW, geo[8], geo[9], geo[10], geo[11], geo[1], geo[2], geo[4], geo[5]) \
            and geo[13] == geo[4] and geo[14] == geo[5] and geo[15] == 1 and geo[16] == ncol:
        cands += (IG_S7,)
    if ncol > 64:  # 64-wide tiles: more workgroups for small-M layers
        cands += (IG_CLASSIC_N64, IG_GLDS_N64, IG_ONEBUF_N64) if fast else (IG_CLASSIC_N64,)
    if len(cands) == 1:
        _ig_tuned[key] = cands[0]
        return cands[0]
    if not _AUTOTUNE or torch.cuda.is_current_stream_capturing():
        return IG_GLDS if fast else IG_CLASSIC
    scratch = torch.empty_like(y)
    if addend is not None and addend.data_ptr() == y.data_ptr():
        addend = addend.clone()  # in-place accumulation target: time on a copy
    sstats = torch.zeros_like(stats) if stats is not None else None
    args = (x, wmat, scratch, geo, sstats, mask, xbn, mean, addend, mcoef) + tuple(bact)
    best = _time_candidates(cands, lambda algo: _igemm_call(algo, *args),
                            label="igemm %s%s" % (geo, " +bn" if xbn is not None else ""))
    _ig_tuned[key] = best
    return best


def _igemm(x, wmat, y, N_, H, W, C, OH, OW, KH, KW, sh, sw, pt, pl, ncol, YH, YW, ys, ldy,
           trans, stats=None, mask=None, xbn=None, mean=None, addend=None, mcoef=None,
           bias=None, relu=False, zfill=False, defer=False, dual=None):
    """``zfill``: stride-2 scatter whose epilogue also zeroes the unsampled
    pixels of each 2x2 block (the output needs no separate zero fill).
    ``defer`` (forward statistics): where the tuned kernel is the streaming
    1x1 one, sum the statistics without storing the output (its consumer
    recomputes it); returns True then."""
    geo = (N_, H, W, C, OH, OW, KH, KW, sh, sw, pt, pl, ncol, YH, YW, ys, ldy, int(trans))
    # a uint8 mask is the producer BN's ReLU bit mask (IgArgs::maskbits)
    mbits = mask is not None and mask.dtype == torch.uint8
    flags = int(bool(relu)) | (2 if zfill else 0) | (4 if mbits else 0)
    algo = _igemm_algo(x, wmat, y, geo, (stats, mask, xbn, mean, addend, mcoef), (bias, flags))
    if (dual is not None and algo == IG_S1 and mbits and xbn is not None and stats is not None
            and mcoef is None and bias is None and not trans and ys == 1 and YH == OH
            and getattr(stats, "_kfb_gfin", None) is None
            and 2 * max(x.numel(), y.numel()) < (1 << 31)):  # (the kernel's buffer ranges)
        # dual-BN data gradient: both BNs' backward partials in one pass
        xr, mean_r, parts_r = dual
        N.call("kfb_conv_s1_dgrad_dual", N.dt(x), x.data_ptr(), wmat.data_ptr(), y.data_ptr(),
               N_, H, W, C, ncol, stats.data_ptr(), mask.data_ptr(), xbn.data_ptr(),
               mean.data_ptr(), N.ptr(addend), xr.data_ptr(), mean_r.data_ptr(),
               parts_r.data_ptr(), N.stream(x.device))
        parts_r._kfb_dual_done = True
        return False
    deferred = (defer and algo == IG_S1 and stats is not None and xbn is None
                and addend is None and bias is None)
    if deferred:
        flags |= 8
    _igemm_call(algo, x, wmat, y, geo, stats, mask, xbn, mean, addend, mcoef, bias, flags)
    return deferred


# A residual BN's producing streaming 1x1 conv sums the statistics without
# storing its output; the BN's apply pass recomputes it (True; K > 1: only
# for convs with at most K input channels).  Off: it did not win in the
# network (profiles/r12_bn_recompute.txt); tests/test_bn_recompute_gpu.py
# switches it on against the exact oracle.
_RECOMPUTE = False


def conv_fwd(x, wl, stride, pads, stats=None, bias=None, relu=False):
    """x [N,H,W,C] (C%8==0), wl [Cout,KH,KW,C] compute dtype -> y [N,OH,OW,Cout].
    ``stats``: optional zeroed stats_buffer(Cout) receiving sum(y), sum(y^2).
    ``bias`` (fp32 [Cout], nullable) / ``relu``: y = act(conv + bias) in the
    epilogue (convs without BN; not combined with ``stats``)."""
    n, H, W, C = x.shape
    cout, KH, KW, _ = wl.shape
    sh, sw = stride
    pt, pb, pl, pr = pads
    OH = (H + pt + pb - KH) // sh + 1
    OW = (W + pl + pr - KW) // sw + 1
    y = torch.empty((n, OH, OW, cout), dtype=x.dtype, device=x.device)
    # a stats buffer marked by its consuming residual BN (models/builder.py):
    # the streaming 1x1 kernel leaves y unwritten; the BN's apply pass
    # recomputes it from (x, wl) and stores it (nn._BatchNormTrain)
    defer = (bool(_RECOMPUTE) and stats is not None and getattr(stats, "_kfb_defer", False)
             and (_RECOMPUTE is True or C <= _RECOMPUTE))
    if _igemm(x, wl, y, n, H, W, C, OH, OW, KH, KW, sh, sw, pt, pl, cout, OH, OW, 1, cout, False,
              stats, bias=bias, relu=relu, defer=defer):
        y._kfb_recompute = (x, wl)
    return y


def is_scatter_dgrad(w_shape, stride, pads):
    cout, KH, KW, _ = w_shape
    return KH == 1 and KW == 1 and pads[0] == 0 and pads[2] == 0 and stride != (1, 1)


def conv_dgrad(dy, wl, x_shape, stride, pads, fuse=None, addend=None, wt=None,
               addend_inplace=False, dual=None):
    """``fuse`` = (stats, mask, xbn, mean[, mcoef]): also apply the producer
    BN's ReLU mask (read from ``mask``, or recomputed from ``xbn`` with the BN's
    [scale | shift] ``mcoef``) to dX and accumulate its backward partial sums
    (see BNLink).
    ``addend``: gradient already produced by other consumers, added to dX
    (not combined with ``fuse`` on the strided-1x1 scatter path, where
    ``addend_inplace`` lets dX accumulate into the addend's own buffer).
    ``dual`` = (x_r, mean_r, parts_r): the producer is a dual-BN output
    relu(bn(x) + bn_r(x_r)) with the ReLU bit mask; where the streaming 1x1
    kernel runs it also sums bn_r's partial into the zeroed [32][C] parts_r
    and marks it ``_kfb_dual_done``."""
    n, H, W, C = x_shape
    # _igemm's fused operands: stats, mask, xbn, mean, addend, mcoef
    f5 = tuple(fuse) + (None,) * (5 - len(fuse)) if fuse is not None else (None,) * 5
    fz = f5[:4] + (addend, f5[4])
    cout, KH, KW, _ = wl.shape
    _, OH, OW, _ = dy.shape
    sh, sw = stride
    pt, pb, pl, pr = pads
    if KH == 1 and KW == 1 and pt == 0 and pl == 0:
        wt = _wrelayout(wl, False).view(C, cout) if wt is None else wt  # [Cin][Cout]
        if sh == 1 and sw == 1 and OH == H and OW == W:
            dx = torch.empty((n, H, W, C), dtype=dy.dtype, device=dy.device)
        elif addend is not None:
            # unsampled pixels keep the addend; sampled ones accumulate in place
            # (with ``fuse`` the caller guarantees the addend is zero at every
            # unsampled pixel, so the BN partials over sampled pixels are complete)
            dx = addend if addend_inplace else _copy(addend)
            fz = f5[:4] + (dx, f5[4])
        else:
            dx = None
        # GEMM over dY pixels (1x1, stride 1 in dY space), scattered by ys.
        ys = sh if sh == sw else None
        if ys is None:
            return None
        # stride 2 over an even grid: the epilogue zeroes the unsampled pixels
        zfill = dx is None and ys == 2 and H == 2 * OH and W == 2 * OW
        if dx is None:
            dx = (torch.empty if zfill else torch.zeros)((n, H, W, C), dtype=dy.dtype,
                                                         device=dy.device)
        _igemm(dy, wt, dx, n, OH, OW, cout, OH, OW, 1, 1, 1, 1, 0, 0, C, H, W, ys, C, False, *fz,
               zfill=zfill, dual=dual if ys == 1 and OH == H and OW == W else None)
        return dx
    if sh == 1 and sw == 1 and KH - 1 - pt >= 0 and KH - 1 - pb >= 0 \
            and KW - 1 - pl >= 0 and KW - 1 - pr >= 0:
        # stride-1 transposed conv == forward conv of dY with the spatially
        # flipped, channel-transposed kernel and complementary padding.
        wf = _wrelayout(wl, True) if wt is None else wt
        dx = torch.empty((n, H, W, C), dtype=dy.dtype, device=dy.device)
        _igemm(dy, wf, dx, n, OH, OW, cout, H, W, KH, KW, 1, 1, KH - 1 - pt, KW - 1 - pl, C,
               H, W, 1, C, False, *fz)
        return dx
    wd = _wrelayout(wl, False) if wt is None else wt  # [Cin][KH][KW][Cout]
    dx = torch.empty((n, H, W, C), dtype=dy.dtype, device=dy.device)
    _igemm(dy, wd, dx, n, OH, OW, cout, H, W, KH, KW, sh, sw, pt, pl, C, H, W, 1, C, True, *fz)
    return dx


def _wgrad_launch(dy, x, dw, geo, target):
    n, H, W, C, OH, OW, KH, KW, sh, sw, pt, pl, cout = geo
    slab, slab_elems = None, 0
    # split partial sums: a plain-store fp32 slab + one reduce launch (fp32
    # atomics into dW ran at ~1.3 TB/s at the memory side)
    splits = N.load().kfb_conv_wgrad_splits(n, OH, OW, KH, KW, C, cout, target)
    if splits > 1 or (target >> 16) == 2:  # (the streaming wgrad always folds slabs)
        slab_elems = splits * cout * KH * KW * C
        slab = torch.empty((slab_elems,), dtype=torch.float32, device=x.device)
    N.call("kfb_conv_wgrad", N.dt(x), dy.data_ptr(), x.data_ptr(), dw.data_ptr(), n, H, W, C, OH,
           OW, KH, KW, sh, sw, pt, pl, cout, target,
           slab.data_ptr() if slab is not None else None, slab_elems, N.stream(x.device))


# Launch-shape autotuning (the role cuDNN's algorithm autotune plays for the
# reference, TF_CUDNN_USE_AUTOTUNE): the first wgrad of each geometry times
# the candidate workgroup targets on the real operands and caches the best.
# KFB_CONV_AUTOTUNE=0 pins _WGRAD_TARGET_BLOCKS.
_AUTOTUNE = os.environ.get("KFB_CONV_AUTOTUNE", "1") != "0" and "KFB_WGRAD_BLOCKS" not in os.environ
_AUTOTUNE_WGRAD = _AUTOTUNE  # (separately switchable by the tests)
_WGRAD_CANDIDATES = (384, 512, 768, 1024)
# The autotune takes the smallest grid (fewest split-K slabs: fewer slab
# bytes and reduce work beside the compute stream) within this fraction of
# the fastest isolated time: in the network, 0.3 beat the fastest-isolated
# choice by 0.13 ms/step on interleaved runs, 0.15 by 0.08, 0.5 by 0.07,
# and capping the grid at 512 lost 0.25; a 256 grid offered as well lost
# 0.06, slack 0.4 0.06 (profiles/r13_wgrad_grid_ab.txt)
_WGRAD_SLACK = 0.3
# bit 16 of a candidate selects the LDS-DMA wgrad kernel (wgrad_glds_k: 128-wide
# output-channel tiles, operands < 2 GiB); KFB_WGRAD_ALGO=classic|glds pins one.
# (Its 2-stage ring of 64-row steps was measured against a 4-stage ring of
# 32-row steps and a 3-stage ring of 64-row steps at one workgroup per CU:
# neither won a single ResNet-50 geometry, profiles/r12_wgrad_rings.txt.)
_WGRAD_GLDS = 1 << 16
_WGRAD_NAMES = {1: "glds", 2: "s3w"}
_WGRAD_ALGO = os.environ.get("KFB_WGRAD_ALGO", "")
_wgrad_tuned = {}


_WGRAD_S3 = 2 << 16  # the streaming 3x3 64-channel wgrad (csrc/conv_stream.hip)


def _wgrad_candidates(geo):
    n, H, W, C, OH, OW, KH, KW, sh, sw, pt, pl, cout = geo
    if _WGRAD_ALGO == "s3":
        return (_WGRAD_S3,)
    s3 = ((_WGRAD_S3,) if not _NO_S3 and N.load().kfb_conv_s3_applicable(
        C, cout, KH, KW, sh, sw, pt, pl, H, W, OH, OW) else ())
    glds = tuple(t | _WGRAD_GLDS for t in _WGRAD_CANDIDATES) if cout > 64 else ()
    if _WGRAD_ALGO == "classic" or not glds:
        return _WGRAD_CANDIDATES + s3
    if _WGRAD_ALGO == "glds":
        return glds
    return _WGRAD_CANDIDATES + glds + s3


def _tune_wgrad(dy, x, dw, geo):
    key = (str(x.device), x.dtype) + geo
    best = _wgrad_tuned.get(key)
    if best is not None:
        return best
    if torch.cuda.is_current_stream_capturing():
        return _WGRAD_TARGET_BLOCKS
    scratch = torch.zeros_like(dw)
    best = _time_candidates(_wgrad_candidates(geo), lambda t: _wgrad_launch(dy, x, scratch, geo, t),
                            label="wgrad %s" % (geo,), slack=_WGRAD_SLACK,
                            cost=lambda t: t & 0xFFFF)
    _wgrad_tuned[key] = best
    return best


def conv_wgrad(dy, x, w_shape, stride, pads, out=None):
    """Accumulates dW into ``out`` (fp32 [Cout,KH,KW,C], e.g. the parameter's
    view of the zeroed flat gradient buffer) or into a fresh zeroed tensor."""
    cout, KH, KW, C = w_shape
    n, H, W, _ = x.shape
    _, OH, OW, _ = dy.shape
    sh, sw = stride
    pt, pb, pl, pr = pads
    if out is not None:
        dw = out
    elif x.is_cuda:
        dw = N.zero_(torch.empty((cout, KH, KW, C), dtype=torch.float32, device=x.device))
    else:
        dw = torch.zeros((cout, KH, KW, C), dtype=torch.float32, device=x.device)
    geo = (n, H, W, C, OH, OW, KH, KW, sh, sw, pt, pl, cout)
    target = _tune_wgrad(dy, x, dw, geo) if _AUTOTUNE_WGRAD else _WGRAD_TARGET_BLOCKS
    _wgrad_launch(dy, x, dw, geo, target)
    return dw


N.register_optional("kfb_pad_rkc", [N.I, N.P, N.P, N.I, N.L, N.I, N.I, N.I, N.P])
N.register_optional("kfb_unpad_accum_f32", [N.P, N.P, N.I, N.L, N.I, N.I, N.P])
N.register_optional("kfb_crop_rkc", [N.I, N.P, N.P, N.I, N.L, N.I, N.I, N.P])
N.register_optional("kfb_wrelayout", [N.I, N.P, N.P, N.I, N.I, N.I, N.I, N.I, N.P])


def _crop_channels(t, c):
    """[..., Cp] -> a new contiguous [..., c] holding the leading c channels
    (native on the GPU: recordable in a launch tape, unlike a slice copy)."""
    cp = t.shape[-1]
    if not t.is_cuda:
        return t[..., :c].contiguous()
    t = t.contiguous()
    out = torch.empty(tuple(t.shape[:-1]) + (c,), dtype=t.dtype, device=t.device)
    N.call("kfb_crop_rkc", N.dt(t), t.data_ptr(), out.data_ptr(), 1, t.numel() // cp, c, cp,
           N.stream(t.device))
    return out


def _copy(t):
    """Device copy of a contiguous tensor (native memcpy on the GPU)."""
    if not t.is_cuda:
        return t.clone()
    t = t.contiguous()
    out = torch.empty_like(t)
    N.call("kfb_memcpy_d2d", out.data_ptr(), t.data_ptr(), t.numel() * t.element_size(),
           N.stream(t.device))
    return out


def _wrelayout(wl, flip):
    """[Cout][KH][KW][Cin] -> [Cin][KH][KW][Cout], spatially flipped if
    ``flip`` (native on the GPU)."""
    cout, KH, KW, cin = wl.shape
    if not wl.is_cuda:
        w = wl.flip(1, 2) if flip else wl
        return w.permute(3, 1, 2, 0).contiguous()
    wl = wl.contiguous()
    out = torch.empty((cin, KH, KW, cout), dtype=wl.dtype, device=wl.device)
    N.call("kfb_wrelayout", N.dt(wl), wl.data_ptr(), out.data_ptr(), cout, KH, KW, cin, int(flip),
           N.stream(wl.device))
    return out


def _pad_rkc(t, R, K, C, Rp, Cp):
    """[R][K][C] -> zero-padded [Rp][K][Cp] (native: recordable in a launch tape)."""
    out = torch.empty((Rp * K * Cp,), dtype=t.dtype, device=t.device)
    N.call("kfb_pad_rkc", N.dt(t), t.contiguous().data_ptr(), out.data_ptr(), R, K, C, Rp, Cp,
           N.stream(t.device))
    return out


def _padded_input(x, cin_p):
    """Channel-padded copy of a few-channel network input (RGB 3 -> 8),
    made every step (no cross-step caching, also for the constant synthetic
    batch: the timed step does all of its work)."""
    if not x.is_cuda:
        return torch.nn.functional.pad(x, (0, cin_p - x.shape[-1]))
    n, H, W, C = x.shape
    return _pad_rkc(x, 1, n * H * W, C, 1, cin_p).view(n, H, W, cin_p)


def _padded_weight(wl, cout_p, cin_p):
    cout, KH, KW, cin = wl.shape
    return _pad_rkc(wl, cout, KH * KW, cin, cout_p, cin_p).view(cout_p, KH, KW, cin_p)


# Weight gradients on a side stream (KFB_WGRAD_STREAM=0: on the compute stream)
_WGRAD_SIDE = os.environ.get("KFB_WGRAD_STREAM", "1") != "0"
_SIDE_STREAMS = {}


# A layer's side-stream weight gradient is enqueued before its data gradient
# (both need only dy and x), so the side stream waits on the kernel that
# produced dy rather than on the data gradient and the two run side by side
# (ResNet-50 bs256: 18.36-18.41 vs 18.78-18.80 ms/step, 3 interleaved pairs,
# profiles/r12_side_stream_order.txt)


def wgrad_stream(device):
    """The side stream weight gradients run on for ``device`` (None when
    disabled or on the CPU)."""
    if not _WGRAD_SIDE or device.type != "cuda":
        return None
    idx = device.index if device.index is not None else torch.cuda.current_device()
    st = _SIDE_STREAMS.get(idx)
    if st is None:
        st = _SIDE_STREAMS[idx] = torch.cuda.Stream(device=idx)
    return st


_JOIN_QUEUED = set()


def _queue_join(device):
    """Once per backward pass: join the side stream when the autograd graph
    has finished, so every consumer of .grad (tests, optimizers) sees the
    weight gradients without knowing about the side stream."""
    idx = device.index
    if idx in _JOIN_QUEUED:
        return
    _JOIN_QUEUED.add(idx)

    def cb():
        _JOIN_QUEUED.discard(idx)
        join_wgrad_stream(torch.device("cuda", idx))
    torch.autograd.Variable._execution_engine.queue_callback(cb)


def join_wgrad_stream(device=None):
    """Makes the current stream wait for every weight gradient enqueued so
    far (before a gradient is read: all-reduce launch, optimizer step)."""
    if not _SIDE_STREAMS:
        return
    cur = torch.cuda.current_stream(device)
    st = _SIDE_STREAMS.get(cur.device.index)
    if st is not None and st != cur:
        N.stream_wait(cur.cuda_stream, st.cuda_stream, device_only=True)


N.register_optional("kfb_s2d_stem", [N.I, N.P, N.P] + [N.I] * 9 + [N.P])
# BN backward partials in the epilogue of strided-1x1 (scatter) dgrads whose
# pending gradient is sparse on the same grid (tests/test_model_gpu.py
# switches it off for its oracle)
_SCATTER_BN_FUSE = True


def use_s2d(x, wl_shape, stride, needs_dx, pads) -> bool:
    """Stride-2 conv over a <=4-channel input with a big kernel (the RGB
    stem) and no input gradient: run it as a 64-channel stride-1 conv over a
    space-to-depth repack (csrc/stem.hip)."""
    cout, KH, KW, cin = wl_shape
    if not (not needs_dx and tuple(stride) == (2, 2) and cin <= 4
            and KH <= 8 and KW <= 8 and KH * KW >= 25 and cout % 8 == 0
            and hasattr(N.load(), "kfb_s2d_stem")):
        return False
    OH, _, _, OW2 = s2d_geometry(x.shape, wl_shape, pads)
    row_bytes = x.shape[2] * cin * x.element_size()
    return (x.shape[0] * OH * OW2 * 64 < (1 << 31) and row_bytes % 4 == 0
            and row_bytes <= 4096 and x.data_ptr() % 4 == 0)


# "pairs": the stem as an 8x4-tap stride-(2,1) conv over a padded pixel-pair
# view of the image (csrc/stem.hip); "s2d": a 64-channel space-to-depth repack
_STEM_MODE = "pairs"
N.register_optional("kfb_stem_pad", [N.I, N.P, N.P] + [N.I] * 8 + [N.P])
N.register_optional("kfb_stem_weight", [N.I, N.P, N.P] + [N.I] * 4 + [N.P])
N.register_optional("kfb_stem_weight_grad", [N.P, N.P] + [N.I] * 4 + [N.P])


def stem_pairs_input(x, wl_shape, pads):
    """x [N,H,W,C<=4] -> the padded pair view [N, Hp, Wp/2, 8] (csrc/stem.hip)."""
    n, H, W, cin = x.shape
    OH, OW, _, _ = s2d_geometry(x.shape, wl_shape, pads)
    Hp = 2 * (OH - 1) + 8  # 8 tap rows at stride 2
    Wp = 2 * (OW + 3)      # 4 pair taps at stride 1
    xp = torch.empty((n, Hp, Wp // 2, 8), dtype=x.dtype, device=x.device)
    N.call("kfb_stem_pad", N.dt(x), x.data_ptr(), xp.data_ptr(), n, H, W, cin, Hp, Wp,
           pads[0], pads[2], N.stream(x.device))
    return xp


def stem_pairs_weight(wl):
    """[Cout,KH,KW,C] -> [Cout,8,4,8] (w2[n][kh][j][t*4+c] = w[n][kh][2j+t][c])."""
    cout, KH, KW, cin = wl.shape
    w2 = torch.empty((cout, 8, 4, 8), dtype=wl.dtype, device=wl.device)
    N.call("kfb_stem_weight", N.dt(wl), wl.data_ptr(), w2.data_ptr(), cout, KH, KW, cin,
           N.stream(wl.device))
    return w2


def s2d_geometry(x_shape, wl_shape, pads):
    n, H, W, _ = x_shape
    _, KH, KW, _ = wl_shape
    pt, pb, pl, pr = pads
    OH = (H + pt + pb - KH) // 2 + 1
    OW = (W + pl + pr - KW) // 2 + 1
    kw2 = (KW + 1) // 2
    return OH, OW, kw2, OW + kw2 - 1


def s2d_input(x, wl_shape, pads):
    """x [N,H,W,C<=4] -> X2 [N,OH,OW+KW2-1,64] (see csrc/stem.hip)."""
    n, H, W, cin = x.shape
    KH = wl_shape[1]
    OH, _, _, OW2 = s2d_geometry(x.shape, wl_shape, pads)
    x2 = torch.empty((n, OH, OW2, 64), dtype=x.dtype, device=x.device)
    N.call("kfb_s2d_stem", N.dt(x), x.data_ptr(), x2.data_ptr(), n, H, W, cin, OH, OW2, KH,
           pads[0], pads[2], N.stream(x.device))
    return x2


def s2d_weight(wl):
    """[Cout,KH,KW,C] -> [Cout,1,KW2,64] with channel = kh*8 + t*4 + c for
    tap column kw = 2*j + t (zeros where kh >= KH, kw >= KW, c >= C)."""
    cout, KH, KW, cin = wl.shape
    kw2 = (KW + 1) // 2
    wp = torch.nn.functional.pad(wl, (0, 4 - cin, 0, 2 * kw2 - KW, 0, 8 - KH))
    return wp.view(cout, 8, kw2, 2, 4).permute(0, 2, 1, 3, 4).reshape(cout, 1, kw2, 64)


def s2d_weight_grad(dw2, wl_shape):
    """Inverse of s2d_weight for the fp32 weight gradient."""
    cout, KH, KW, cin = wl_shape
    kw2 = dw2.shape[2]
    g = dw2.view(cout, kw2, 8, 2, 4).permute(0, 2, 1, 3, 4).reshape(cout, 8, 2 * kw2, 4)
    return g[:, :KH, :KW, :cin]


class _Conv2d(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, wl, stride, pads, stats, wt, bias=None, relu=False):
        x = x.contiguous()
        if wl is None or wl.dtype != x.dtype:
            wl = w.detach().to(x.dtype)
        cin = x.shape[-1]
        cout = wl.shape[0]
        ctx.s2d = None
        # bias + ReLU in the forward epilogue; their backward (ReLU mask and
        # bias column sums) runs as one pass at the top of this backward
        ctx.bact = bias is not None or relu
        ctx.out_link = None
        ctx.relu, ctx.bias = bool(relu), bias
        bd = bias.detach() if bias is not None else None
        if use_s2d(x, wl.shape, stride, ctx.needs_input_grad[0], pads) and \
                _STEM_MODE == "pairs" and wl.shape[2] <= 8 and x.dtype != torch.float32 \
                and hasattr(N.load(), "kfb_stem_pad"):
            xv = stem_pairs_input(x, wl.shape, pads)
            w2 = stem_pairs_weight(wl.contiguous())
            y = conv_fwd(xv, w2, (2, 1), (0, 0, 0, 0), stats, bd, relu)
            ctx.save_for_backward(xv, w2, y if relu else None)
            ctx.s2d = ("pairs",) + tuple(wl.shape)
            ctx.w = w
            _Conv2d._act_link(ctx, y, cout % 8 == 0)
            return y
        if use_s2d(x, wl.shape, stride, ctx.needs_input_grad[0], pads):
            x2 = s2d_input(x, wl.shape, pads)
            w2 = s2d_weight(wl).contiguous()
            y = conv_fwd(x2, w2, (1, 1), (0, 0, 0, 0), stats, bd, relu)
            ctx.save_for_backward(x2, w2, y if relu else None)
            ctx.s2d = tuple(wl.shape)
            ctx.w = w
            _Conv2d._act_link(ctx, y, cout % 8 == 0)
            return y
        cin_p, cout_p = _pad8(cin), _pad8(cout)
        xp, wp = x, wl
        if cin_p != cin:
            xp = _padded_input(x, cin_p)
        if cin_p != cin or cout_p != cout:
            wp = _padded_weight(wl.contiguous(), cout_p, cin_p)
        if cout_p != cout:
            stats = None
            if bd is not None:
                bd = (_pad_rkc(bd.contiguous(), 1, 1, cout, 1, cout_p) if bd.is_cuda
                      else torch.nn.functional.pad(bd, (0, cout_p - cout)))
        wp = wp.contiguous()
        y = conv_fwd(xp, wp, stride, pads, stats, bd, relu)
        if cout_p != cout:
            y = _crop_channels(y, cout)
        ctx.save_for_backward(xp, wp, y if relu else None)
        ctx.meta = (stride, pads, cin, cout, x.shape)
        ctx.x_needs_grad = ctx.needs_input_grad[0]
        ctx.w = w
        ctx.wt = wt if (cin_p == cin and cout_p == cout) else None
        ctx.link = getattr(x, "_kfb_bn_link", None)
        _Conv2d._act_link(ctx, y, cout_p == cout)
        return y

    @staticmethod
    def _act_link(ctx, y, aligned):
        if not (ctx.bact and aligned and _ACT_FUSE and _fuse_enabled()):
            return
        # bias (+ReLU) without BN: a conv consuming y applies the ReLU
        # mask and sums the bias gradient in its dgrad epilogue.  This is
        # the BNLink protocol with y standing in for x_bn (x_bn None: the
        # consumer passes its saved input, so the link holds no reference
        # to y), mean 0 and the mask recomputed as y * 1 + 0 > 0 (ReLU)
        # or y * 0 + 1 > 0 (bias only); the partials' first half is then
        # the bias gradient
        from .nn import BNLink
        mean, coef = _act_link_consts(y.shape[-1], ctx.relu, y.device)
        ctx.out_link = BNLink(None, mean, True, coef)
        y._kfb_bn_link = ctx.out_link

    @staticmethod
    def _side_wgrad(ctx, dy, xp, wp, stride, pads, cin, cout_p):
        """Weight gradient off the critical path, on the side stream: the
        dgrad chain continues on the compute stream while this runs beside
        it (backward of the small-grid stage-4/5 layers under-fills the
        chip).  Its inputs are kept alive for the side stream; gradient
        consumers join it (join_wgrad_stream).  False (nothing launched)
        where the gradient cannot go there."""
        w = ctx.w
        sink = getattr(w, "_kfb_grad_sink", None)
        if not (sink is not None and cout_p == ctx.meta[3] and wp.shape[-1] == cin
                and _fuse_enabled()):
            return False
        side = wgrad_stream(dy.device)
        if side is None:
            return False
        N.stream_wait(side.cuda_stream, N.stream(dy.device), device_only=True)
        _queue_join(dy.device)
        with torch.cuda.stream(side):
            conv_wgrad(dy, xp, wp.shape, stride, pads, out=sink)
            dy.record_stream(side)
            xp.record_stream(side)
            cb = getattr(w, "_kfb_ready_cb", None)
            if cb is not None:
                cb(w)
        return True

    @staticmethod
    def backward(ctx, dy):
        db = None
        if ctx.bact:
            ol = ctx.out_link
            if ol is not None and ol.partials is not None:
                # the consumer's dgrad epilogue already applied the ReLU mask
                # and summed the bias-gradient partials
                db = _bias_from_partials(ol.partials, ctx.bias, dy.shape[-1], dy.device)
                ol.partials = None
            else:
                dy, db = _bias_act_backward(dy, ctx.saved_tensors[2], ctx.relu, ctx.bias)
        if ctx.s2d is not None:
            return _Conv2d._backward_s2d(ctx, dy) + (db, None)
        xp, wp = ctx.saved_tensors[:2]
        stride, pads, cin, cout, x_shape = ctx.meta
        dy = dy.contiguous()
        cout_p = wp.shape[0]
        if cout_p != cout:
            rows = dy.numel() // cout
            dy = _pad_rkc(dy, 1, rows, cout, 1, cout_p).view(tuple(dy.shape[:-1]) + (cout_p,))
        dx = None
        # the side-stream weight gradient needs only dy and x: enqueued before
        # the data gradient, it may start beside it
        side_done = (ctx.needs_input_grad[1]
                     and _Conv2d._side_wgrad(ctx, dy, xp, wp, stride, pads, cin, cout_p))
        if ctx.x_needs_grad:
            link = ctx.link
            padded = wp.shape[-1] != cin
            if link is not None and link.fusable:
                if link.arrive():
                    link.take_pending_stream()
                    pend, owned = link.pending, link.pending_owned
                    link.pending = None
                    if padded:
                        dx = _crop_channels(conv_dgrad(dy, wp, xp.shape, stride, pads), cin)
                        if pend is not None:
                            if dx.is_cuda:
                                N.call("kfb_add", N.dt(dx), dx.data_ptr(), pend.contiguous().data_ptr(),
                                       dx.data_ptr(), dx.numel(), 0, N.stream(dx.device))
                            else:
                                dx = dx + pend
                    else:
                        fuse = None
                        scatter = is_scatter_dgrad(wp.shape, stride, pads)
                        # A strided-1x1 (scatter) dgrad writes only every s-th
                        # pixel, so it can finish the BN backward work only when
                        # the pending gradient is zero elsewhere too (every other
                        # contributor was a scatter of the same stride, as the
                        # projection shortcut + conv a of a ResNet v1 block).
                        sparse_ok = scatter and _SCATTER_BN_FUSE and stride[0] == stride[1] \
                            and link.pending_sparse == stride[0]
                        if link.accum:
                            pass  # accumulation-only link: pend as the addend, no BN work
                        elif not (pend is not None and scatter) or sparse_ok:
                            parts = stats_buffer(cin, dy.device)
                            # ReLU mask: recomputed from x_bn when the BN has no
                            # residual add (link.mcoef), else read from its output
                            rec = link.relu and link.mcoef is not None
                            xbn = link.x_bn if link.x_bn is not None else xp  # act link
                            # (y's ReLU bit mask when the BN apply wrote one)
                            mk = None
                            if link.relu and not rec:
                                mk = link.mbits if link.mbits is not None else xp
                            fuse = (parts, mk, xbn, link.mean, link.mcoef if rec else None)
                            attach_bn_grad_finalize(parts, link, cin, dy.device)
                        dual = None
                        if fuse is not None and link.dual is not None and not scatter \
                                and mk is not None and mk is link.mbits:
                            dual = link.dual + (STATS_ARENA.take(STATS_SPREAD * cin, dy.device),)
                        dx = conv_dgrad(dy, wp, xp.shape, stride, pads, fuse, addend=pend,
                                        wt=ctx.wt, addend_inplace=owned, dual=dual)
                        if fuse is not None:
                            link.partials = fuse[0]
                            if dual is not None and getattr(dual[2], "_kfb_dual_done", False):
                                link.partials_r = dual[2]
                else:
                    sparse = (stride[0] if not padded and stride[0] == stride[1]
                              and is_scatter_dgrad(wp.shape, stride, pads) else None)
                    g = None
                    if not padded and link.pending is not None:
                        # accumulate onto the pending gradient in the dgrad
                        # epilogue (one read of it) instead of a separate add
                        link.take_pending_stream()
                        g = conv_dgrad(dy, wp, xp.shape, stride, pads, addend=link.pending,
                                       wt=ctx.wt, addend_inplace=link.pending_owned)
                        if g is not None:
                            link.accumulated(g, sparse)
                    if g is None:
                        g = conv_dgrad(dy, wp, xp.shape, stride, pads, wt=ctx.wt)
                        link.deposit(_crop_channels(g, cin) if padded else g, sparse=sparse)
            else:
                dx = conv_dgrad(dy, wp, xp.shape, stride, pads, wt=ctx.wt)
                if dx is not None and padded:
                    dx = _crop_channels(dx, cin)
        dw = None
        if side_done:
            return dx, None, None, None, None, None, None, db, None
        if ctx.needs_input_grad[1]:
            w = ctx.w
            sink = getattr(w, "_kfb_grad_sink", None)
            direct = (sink is not None and cout_p == cout and wp.shape[-1] == cin
                      and _fuse_enabled())
            if _Conv2d._side_wgrad(ctx, dy, xp, wp, stride, pads, cin, cout_p):
                return dx, None, None, None, None, None, None, db, None
            padded_w = cout_p != cout or wp.shape[-1] != cin
            if padded_w and sink is not None and _fuse_enabled():
                # padded weight gradient, accumulated natively into the
                # parameter's gradient view (no slicing copy, no autograd add)
                full = torch.empty(tuple(wp.shape), dtype=torch.float32, device=dy.device)
                N.zero_(full)
                conv_wgrad(dy, xp, wp.shape, stride, pads, out=full)
                KH, KW = wp.shape[1], wp.shape[2]
                N.call("kfb_unpad_accum_f32", full.data_ptr(), sink.data_ptr(), cout, KH * KW,
                       cin, wp.shape[-1], N.stream(dy.device))
                cb = getattr(w, "_kfb_ready_cb", None)
                if cb is not None:
                    cb(w)
                return dx, None, None, None, None, None, None, db, None
            dw = conv_wgrad(dy, xp, wp.shape, stride, pads, out=sink if direct else None)
            if direct:
                cb = getattr(w, "_kfb_ready_cb", None)
                if cb is not None:
                    cb(w)
                dw = None
            elif dw.shape[0] != cout or dw.shape[-1] != cin:
                dw = dw[:cout, :, :, :cin].contiguous()
        return dx, dw, None, None, None, None, None, db, None


    @staticmethod
    def _backward_pairs(ctx, dy):
        xv, w2 = ctx.saved_tensors[:2]
        _, cout, KH, KW, cin = ctx.s2d
        if not ctx.needs_input_grad[1]:
            return None, None, None, None, None, None, None
        w = ctx.w
        sink = getattr(w, "_kfb_grad_sink", None)
        direct = sink is not None and _fuse_enabled()
        dw = sink if direct else torch.zeros((cout, KH, KW, cin), dtype=torch.float32,
                                             device=dy.device)
        scratch = torch.empty((cout, 8, 4, 8), dtype=torch.float32, device=dy.device)
        N.zero_(scratch)
        conv_wgrad(dy.contiguous(), xv, w2.shape, (2, 1), (0, 0, 0, 0), out=scratch)
        N.call("kfb_stem_weight_grad", scratch.data_ptr(), dw.data_ptr(), cout, KH, KW, cin,
               N.stream(dy.device))
        if direct:
            cb = getattr(w, "_kfb_ready_cb", None)
            if cb is not None:
                cb(w)
            dw = None
        return None, dw, None, None, None, None, None

    @staticmethod
    def _backward_s2d(ctx, dy):
        if ctx.s2d[0] == "pairs":
            return _Conv2d._backward_pairs(ctx, dy)
        x2, w2 = ctx.saved_tensors[:2]
        dw = None
        if ctx.needs_input_grad[1]:
            dw2 = conv_wgrad(dy.contiguous(), x2, w2.shape, (1, 1), (0, 0, 0, 0))
            dw = s2d_weight_grad(dw2, ctx.s2d)
            w = ctx.w
            sink = getattr(w, "_kfb_grad_sink", None)
            if sink is not None and _fuse_enabled():
                sink.add_(dw)
                cb = getattr(w, "_kfb_ready_cb", None)
                if cb is not None:
                    cb(w)
                dw = None
            else:
                dw = dw.contiguous()
        return None, dw, None, None, None, None, None


_act_consts = {}


def _act_link_consts(C, relu, dev):
    """(mean = 0, [scale | shift]) of an act link (see _Conv2d.forward)."""
    key = (C, relu, dev)
    if key not in _act_consts:
        coef = torch.zeros(2 * C, dtype=torch.float32, device=dev)
        coef[C if not relu else 0:C * (2 if not relu else 1)] = 1.0
        _act_consts[key] = (torch.zeros(C, dtype=torch.float32, device=dev), coef)
    return _act_consts[key]


def _bias_from_partials(parts, bias, C, dev):
    """Bias gradient = column sums of the [STATS_SPREAD][C] slab partials
    (first half of a stats buffer), into the flat-gradient view if any."""
    if bias is None:
        return None
    sink = getattr(bias, "_kfb_grad_sink", None)
    out = sink if sink is not None else torch.empty((C,), dtype=torch.float32, device=dev)
    N.call("kfb_slab_colsum", parts.data_ptr(), STATS_SPREAD, C, out.data_ptr(),
           int(sink is not None), N.stream(dev))
    if sink is not None:
        cb = getattr(bias, "_kfb_ready_cb", None)
        if cb is not None:
            cb(bias)
        return None
    return out


def _bias_act_backward(dy, y, relu, bias):
    """ReLU backward (mask from the saved output) and the bias gradient as
    one pass (kfb_act_bwd_bias); the bias gradient accumulates straight into
    the flat-gradient view when the bias has one."""
    dy = dy.contiguous()
    C = dy.shape[-1]
    rows = dy.numel() // C
    g = torch.empty_like(dy) if relu else dy
    pb = dbuf = None
    nslab = 1
    sink = getattr(bias, "_kfb_grad_sink", None) if bias is not None else None
    if bias is not None:
        nslab = N.query("kfb_colsum_num_slabs", rows, C)
        pb = torch.empty((nslab * C,), dtype=torch.float32, device=dy.device)
        dbuf = sink if sink is not None else torch.empty((C,), dtype=torch.float32,
                                                         device=dy.device)
    N.call("kfb_act_bwd_bias", N.dt(dy), dy.data_ptr(), N.ptr(y), g.data_ptr(), rows, C,
           int(relu), N.ptr(pb), nslab, N.ptr(dbuf), int(sink is not None), N.stream(dy.device))
    if sink is not None:
        cb = getattr(bias, "_kfb_ready_cb", None)
        if cb is not None:
            cb(bias)
        return g, None
    return g, dbuf


def conv2d(x, w, wl, stride, pads, stats=None, wt=None, bias=None, relu=False):
    return _Conv2d.apply(x, w, wl, tuple(stride), tuple(pads), stats, wt, bias, bool(relu))


N.register_optional("kfb_wtrans_item_bytes", [], N.c_int)
N.register_optional("kfb_weight_transforms", [N.I, N.P, N.P, N.P, N.I, N.P])

_ITEM = None


def _item_dtype():
    import numpy as np
    return np.dtype([("src", "<i8"), ("dst", "<i8"), ("cout", "<i4"), ("cin", "<i4"),
                     ("kh", "<i4"), ("kw", "<i4"), ("a", "<i4"), ("b", "<i4"),
                     ("flip", "<i4"), ("co0", "<i4"), ("ci0", "<i4"), ("pad", "<i4")])


class DgradWeights:
    """Keeps a dgrad-ready copy ([Cin][KH][KW][Cout], flipped for stride-1
    kernels) of every conv weight, refreshed by ONE batched launch
    (csrc/wtrans.hip) after each optimizer update instead of per-conv
    permute/flip copies in backward."""

    def __init__(self, net, flat):
        import numpy as np
        self.flat = flat
        lp = flat.lp
        base = lp.data_ptr()
        esz = lp.element_size()
        items, total, views = [], 0, []
        for layer in net.ordered_layers():
            wl = getattr(layer, "weight_lp", None)
            stride = getattr(layer, "stride", None)
            if wl is None or stride is None:
                continue
            cout, kh, kw, cin = wl.shape
            if cin % 8 or cout % 8:
                continue
            flip = int(tuple(stride) == (1, 1) and (kh, kw) != (1, 1))
            src = (wl.data_ptr() - base) // esz
            dst = total
            total += (wl.numel() + 63) // 64 * 64
            views.append((layer, dst, (cin, kh, kw, cout)))
            for a in range(kh):
                for b in range(kw):
                    for co0 in range(0, cout, 64):
                        for ci0 in range(0, cin, 64):
                            items.append((src, dst, cout, cin, kh, kw, a, b, flip, co0, ci0, 0))
        self.n = len(items)
        self.buf = torch.empty((max(total, 1),), dtype=lp.dtype, device=lp.device)
        for layer, off, shape in views:
            layer.weight_t = self.buf[off:off + int(np.prod(shape))].view(shape)
        arr = np.array(items, dtype=_item_dtype())
        assert arr.dtype.itemsize == N.query("kfb_wtrans_item_bytes")
        self.items = torch.from_numpy(arr.view(np.uint8).copy()).to(lp.device)
        self.run()

    def run(self):
        if self.n:
            lp = self.flat.lp
            N.call("kfb_weight_transforms", N.dt(lp), lp.data_ptr(), self.buf.data_ptr(),
                   self.items.data_ptr(), self.n, N.stream(lp.device))
