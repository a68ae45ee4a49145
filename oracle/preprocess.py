"""numpy restatement of the image preprocessing (row f2), TEST INFRASTRUCTURE
ONLY (tests/), never imported by thunder_amd.  Parity status: "parity
unpinned" -- the reference ships no preprocessed fixtures; pinned here by
known answers (tests/test_ingest.py).

Follows, with the reference's compiled switches (OPTIMISER_MASK_IMG,
OPTIMISER_INIT_IMG_NORMALISE_OUT_MASK_REGION, include/Config.h:184, 190):
  ImageFile::readImage's centring (MESH_IMAGE_INDEX, include/Image/
    ImageFile.h:383-409): the stored image is rolled by -N/2 on both axes;
  substractBgImg (src/Optimiser.cpp:4928-4962) with bgMeanStddev
    (src/Image/ImageFunctions.cpp:607-620: pixels with i^2 + j^2 > r^2,
    GSL mean and sample sd);
  statImg's per-image terms (:4810-4905): bgStddev(0, img, r) (:585-596),
    stddev(0, img) (:543-547), regionMean(img, r, 0) (src/Functions/Mask.cpp:
    102-127);
  maskImg with zeroMask (:4964-4996) -> softMask(dst, src, r, ew, 0)
    (src/Functions/Mask.cpp:363-385), normaliseImg (:4998-5012), fwImg (FFTW
    r2c, unnormalised);
  reMaskImg (:6093-6150): backward FFT / N^2, x softMask(mask, r, ew)
    (Mask.cpp:333-350), forward.
"""
import numpy as np

EDGE_WIDTH_RL = 6


def rl_coords(N):
    """(i, j) of every stored pixel in the corner-origin layout (Image::iRL)."""
    k = np.arange(N)
    c = np.where(k < N // 2, k, k - N)
    j, i = np.meshgrid(c, c, indexing="ij")
    return i, j


def load(img_centred):
    """The reference's read: centred on disk -> corner origin."""
    N = img_centred.shape[-1]
    return np.roll(img_centred, (-(N // 2), -(N // 2)), axis=(-2, -1))


def stats_and_normalise(img, r):
    """img: [N, N] corner origin, float32 -> (normalised float32 image,
    [bgMean, bgSd, bgStddev(0) after, stddev(0) after, mean inside r after])."""
    N = img.shape[-1]
    i, j = rl_coords(N)
    q = i.astype(np.float64) ** 2 + j.astype(np.float64) ** 2
    bg = q > r * r
    x = img.astype(np.float64)[bg]
    mean = x.mean()
    sd = np.sqrt(((x - mean) ** 2).sum() / (x.size - 1))
    fm, fsd = np.float32(mean), np.float32(sd)
    out = ((img.astype(np.float32) - fm) / fsd).astype(np.float32)
    o = out.astype(np.float64)
    b0 = np.sqrt((o[bg] ** 2).sum() / (bg.sum() - 1))
    a0 = np.sqrt((o ** 2).sum() / (o.size - 1))
    inside = np.sqrt(q) < r
    cm = o[inside].mean()
    return out, np.array([fm, fsd, b0, a0, cm], np.float64)


def soft_mask_keep(N, r, ew=EDGE_WIDTH_RL):
    i, j = rl_coords(N)
    u = np.hypot(i, j).astype(np.float32).astype(np.float64)
    w = 0.5 - 0.5 * np.cos((u - r) / ew * np.pi)          # portion of background
    return np.where(u < r, 1.0, np.where(u > r + ew, 0.0, 1.0 - w))


def finish(img, r, std_n, ew=EDGE_WIDTH_RL):
    """zeroMask softMask + 1 / stdN + forward FFT -> (imgFT, oriFT)."""
    N = img.shape[-1]
    keep = soft_mask_keep(N, r, ew)
    m = img.astype(np.float64) * keep / std_n
    o = img.astype(np.float64) / std_n
    return np.fft.rfft2(m), np.fft.rfft2(o)


def remask(ft, N, r, ew=EDGE_WIDTH_RL):
    rl = np.fft.irfft2(ft, s=(N, N))          # numpy's inverse is FFTW's backward / N^2
    return np.fft.rfft2(rl * soft_mask_keep(N, r, ew))
