"""f2: from a particle table and MRC stacks to the device-resident image
batch the expectation consumes (Optimiser::initImg + initCTF + allocPreCal,
src/Optimiser.cpp:4608-5101, 8043-8171), over the C-ABI's preprocessing
kernels (csrc/preprocess.hip).

    t = io.read_thu("particles.thu")
    stack = ingest.Stack.from_thu(t, prefix, pixel_size=1.32, mask_radius_A=80, device=dev)
    dat, ctf, sig = stack.pixel_batch(px, sigRcp)   # image-major, for Expectation.run

stdN, the noise level statImg averages over the hemisphere's images, is a
hemisphere-wide all-reduce in the reference (MPI_Allreduce over _hemi);
``hemisphere_group`` (a torch.distributed group) makes it one here.
"""
import numpy as np
import torch

from . import io
from ._lib import check, lib
from .ops import _ptr, _req, _stream

EDGE_WIDTH_RL = 6          # include/Macro.h:99


def image_stats(img, centred, r_mask):
    """thx_img_stats on a device stack [n, N, N] float32 -> (normalised image
    in the reference's corner-origin layout, stats [n, 5])."""
    n, N, _ = img.shape
    _req(img, torch.float32, (n, N, N), "img")
    out = torch.empty_like(img)
    st = torch.empty(n, 5, dtype=torch.float32, device=img.device)
    check(lib().thx_img_stats(_ptr(img), int(bool(centred)), n, N, float(r_mask), _ptr(out),
                              _ptr(st), _stream(img.device)), "thx_img_stats")
    return out, st


def finish(img, r_mask, std_n, zero_mask=True, seed=1, keep_ori=True, edge=EDGE_WIDTH_RL):
    """thx_img_finish: mask, scale by 1 / stdN, forward FFT.  img is
    overwritten.  Returns (imgFT, oriFT or None), [n, N, N/2+1] complex64."""
    n, N, _ = img.shape
    _req(img, torch.float32, (n, N, N), "img")
    ft = torch.empty(n, N, N // 2 + 1, dtype=torch.complex64, device=img.device)
    ori = torch.empty_like(img) if keep_ori else None
    oft = torch.empty_like(ft) if keep_ori else None
    check(lib().thx_img_finish(_ptr(img), n, N, float(r_mask), float(edge), int(bool(zero_mask)),
                               float(std_n), int(seed), _ptr(ft), _ptr(ori), _ptr(oft),
                               _stream(img.device)), "thx_img_finish")
    return ft, oft


def remask(ft, r_mask, edge=EDGE_WIDTH_RL):
    """thx_remask in place (reMaskImg / ReMask)."""
    n, N, _ = ft.shape
    _req(ft, torch.complex64, (n, N, N // 2 + 1), "imgFT")
    rl = torch.empty(n, N, N, dtype=torch.float32, device=ft.device)
    check(lib().thx_remask(_ptr(ft), n, N, float(r_mask), float(edge), _ptr(rl), _stream(ft.device)),
          "thx_remask")
    return ft


def gather(ft, iPxl):
    """allocPreCal's datP [n, nPxl] from FT images and the pixel set's iPxl."""
    n, N, _ = ft.shape
    _req(ft, torch.complex64, (n, N, N // 2 + 1), "imgFT")
    ip = torch.as_tensor(np.ascontiguousarray(iPxl, np.int32), device=ft.device)
    out = torch.empty(n, len(ip), dtype=torch.complex64, device=ft.device)
    check(lib().thx_img_gather(_ptr(ft), n, N, _ptr(ip), len(ip), _ptr(out), _stream(ft.device)),
          "thx_img_gather")
    return out


def ctf_images(attr, N):
    """GCTFinit: [n, N, N/2+1] CTF over the whole half-complex grid."""
    n = attr.shape[0]
    _req(attr, torch.float32, (n, 8), "attr")
    out = torch.empty(n, N, N // 2 + 1, dtype=torch.float32, device=attr.device)
    check(lib().thx_ctf_image(_ptr(attr), n, N, _ptr(out), _stream(attr.device)), "thx_ctf_image")
    return out


class Stack:
    """A preprocessed particle stack on one device: imgFT (masked, the
    expectation's data), oriFT (unmasked, _imgOri), the CTF attributes, the
    noise level stdN and the per-image statistics."""

    def __init__(self, images, attr, pixel_size, mask_radius_A, device, centred=True,
                 zero_mask=True, hemisphere_group=None, seed=1, keep_ori=True):
        imgs = torch.as_tensor(np.ascontiguousarray(images, np.float32), device=device)
        self.N = imgs.shape[-1]
        self.pixel_size = pixel_size
        self.r_mask = mask_radius_A / pixel_size          # _para.maskRadius / _para.pixelSize
        norm, self.stats = image_stats(imgs, centred, self.r_mask)
        del imgs
        # statImg: stdN = mean over the hemisphere's images of bgStddev(0)
        s = torch.stack([self.stats[:, 2].double().sum(),
                         torch.tensor(float(self.stats.shape[0]), dtype=torch.float64,
                                      device=device)])
        if hemisphere_group is not None:
            import torch.distributed as dist
            st = s.cpu() if dist.get_backend(hemisphere_group) == "gloo" else s
            dist.all_reduce(st, group=hemisphere_group)
            s = st.to(device)
        self.std_n = float(s[0] / s[1])
        self.imgFT, self.oriFT = finish(norm, self.r_mask, self.std_n, zero_mask, seed, keep_ori)
        del norm
        self.attr = torch.as_tensor(np.ascontiguousarray(attr, np.float32), device=device)

    @classmethod
    def from_thu(cls, table, prefix, pixel_size, mask_radius_A, device, **kw):
        imgs = io.load_images(table, prefix)
        return cls(imgs, io.thu_ctf_attrs(table, pixel_size), pixel_size, mask_radius_A, device,
                   centred=True, **kw)

    def pixel_batch(self, px, sig_rcp=None):
        """(dat, ctf, sigRcp) image-major over pixel set px (ops.PixelSet):
        allocPreCal's gather, the CTF on the fly (thx_ctf), sigRcp = -1/2 per
        pixel unless given ([nPxl] per-shell values or [n, nPxl])."""
        from . import ops
        dat = gather(self.imgFT, px.iPxl)
        ctf = ops.ctf(self.attr, px)
        n = dat.shape[0]
        if sig_rcp is None:
            sig = torch.full((n, px.n), -0.5, dtype=torch.float32, device=dat.device)
        else:
            sig = torch.as_tensor(np.asarray(sig_rcp, np.float32), device=dat.device)
            sig = sig.expand(n, px.n).contiguous() if sig.dim() == 1 else sig.contiguous()
        return dat, ctf, sig
