"""Drop-in ``gsplat`` package backed by gsvc_amd (MI355X / gfx950).

Same public names as the reference's gsplat/gsplat/__init__.py:1-47, so GSVC's
imports (GaussianSplats_Represent.py:1-2) resolve here unchanged.
"""
from gsvc_amd import *  # noqa: F401,F403
from gsvc_amd import __all__, __version__  # noqa: F401
