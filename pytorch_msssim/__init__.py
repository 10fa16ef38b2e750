"""Drop-in ``pytorch_msssim`` names backed by gsvc_amd.msssim (gfx950 kernels).

GSVC imports ``from pytorch_msssim import ms_ssim, ssim`` (utils.py:3,
train_video_Represent.py:11).  The package is unpinned (requirements.txt:5)
and not installed in this image; these are our kernels behind its public API
(ssim, ms_ssim, SSIM, MS_SSIM), CUDA (HIP) tensors only.  Parity against the
package itself is unpinned.
"""
from gsvc_amd.msssim import MS_SSIM, SSIM, ms_ssim, ssim  # noqa: F401

__all__ = ["ssim", "ms_ssim", "SSIM", "MS_SSIM"]
